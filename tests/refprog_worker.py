"""One PE of the reference's own test programs at 2, 3 and 4 PEs through the device exchange
(test_gpu_dist_reference_programs.py). Launched once per PE (RANK / WORLD_SIZE in the
environment, every PE on the box's one GPU, gloo host transport).

Each payload is the reference's SPMD program: every PE issues its own batch (the exchange is
collective, so every PE issues the same sequence of batch calls), then every PE reads the global
array and checks the payload's known answer:
  add_test.rs:88-160     PE p adds 10^(2p), pe_max_val times per element (shuffled batch)
                         -> sum_p 10^(2p) * pe_max_val (T-wrapping; f32: pe_max_val = 9);
                         :166-290 the same on the upper half sub-array (lower half stays 0)
  sub_test.rs:96-118     init 100 * num_pes, every PE subtracts 1 a hundred times -> 0
  mul_test.rs:99-117     init 1, every PE multiplies by 2 max_updates times -> 2^(mu * num_pes);
  div_test.rs:91-110     then divides back -> 1
  xor_test.rs:78-98 / or_test.rs   PE p sets bit p -> (1 << num_pes) - 1
  and_test.rs:80-100     init !0, PE p clears bit p -> !0 << num_pes
Failures are written to pe<rank>.npz (the parent asserts there are none).
"""
import os
import sys

import numpy as np
import faulthandler

# a PE stuck in a collective dumps where it is (and exits) before the parent's wait runs out
faulthandler.dump_traceback_later(int(os.environ.get("LMR_WORKER_DUMP_S", "150")), exit=True)

sys.path.insert(0, os.environ["LMR_ROOT"])
sys.path.insert(0, os.path.join(os.environ["LMR_ROOT"], "tests"))

import torch.distributed as dist  # noqa: E402

from _lamellar_bootstrap import load_package  # noqa: E402

lam = load_package()
from opgen import NP  # noqa: E402

DTS = ["u8", "u16", "u32", "u64", "i8", "i16", "i32", "i64", "f32", "f64"]
LENS = [19, 128]


def T(dt, v):
    return np.array([v]).astype(NP[dt])[0]


def wrap_mul(dt, a, b):
    return (np.array([a], dtype=NP[dt]) * np.array([b], dtype=NP[dt]))[0]


def close(vals, expect):
    """check_val!: ((val - max_val) as f64).abs() <= 0.0001, T-wrapping subtraction."""
    d = (vals - np.array([expect], dtype=vals.dtype)).astype(np.float64)
    return bool(np.all(np.abs(d) <= 1e-4))


def max_updates(dt, npes):
    """max_updates! (mul_test.rs:59-71): (128 - lz(T::MAX as u128 / npes) - 1) / npes."""
    tmax = {"u8": 2**8 - 1, "u16": 2**16 - 1, "u32": 2**32 - 1, "u64": 2**64 - 1, "i8": 2**7 - 1,
            "i16": 2**15 - 1, "i32": 2**31 - 1, "i64": 2**63 - 1,
            "f32": int(np.finfo(np.float32).max), "f64": 2**128 - 1}[dt]
    q = tmax // npes
    return (q.bit_length() - 1) // npes


def main():
    world = lam.LamellarWorldBuilder().build()
    me, npes = world.my_pe(), world.num_pes()
    dist_kind = int(os.environ["LMR_DIST"])
    fails = []
    checks = 0

    def check(ok, what):
        nonlocal checks
        checks += 1
        if not ok:
            fails.append(str(what))

    for dt in DTS:
        t = NP[dt]
        kinds = ["AtomicArray"] + (["LocalLockArray", "UnsafeArray"] if dt in ("u32", "f64") else [])
        for kind in kinds:
            for n in LENS:
                a = getattr(lam, kind)(world.team(), n, dist_kind, dt)
                rng = np.random.default_rng(n + 7 * me)
                # add
                pe_max_val = 9 if dt == "f32" else 50
                max_val = t(0)
                for pe in range(npes):
                    max_val = (np.array([max_val]) + np.array([wrap_mul(dt, T(dt, 10 ** (2 * pe)), T(dt, pe_max_val))])
                               ).astype(t)[0]
                a.fill(0)
                world.barrier()
                ind = np.tile(np.arange(n, dtype=np.uint64), pe_max_val)
                rng.shuffle(ind)
                a.batch_add(ind, T(dt, 10 ** (2 * me))).block()
                world.barrier()
                check(close(a.to_numpy().astype(t), max_val), (kind, dt, n, "add"))
                # add on the upper half sub-array
                a.fill(0)
                world.barrier()
                sub = a.sub_array(n // 2, n)
                sub.batch_add(np.tile(np.arange(sub.len(), dtype=np.uint64), pe_max_val), T(dt, 10 ** (2 * me))).block()
                world.barrier()
                got = a.to_numpy().astype(t)
                check(close(got[n // 2:], max_val) and np.all(got[:n // 2] == 0), (kind, dt, n, "sub-array add"))
                # sub
                a.fill(wrap_mul(dt, T(dt, 100), T(dt, npes)))
                world.barrier()
                a.batch_sub(np.tile(np.arange(n, dtype=np.uint64), 100), T(dt, 1)).block()
                world.barrier()
                check(close(a.to_numpy().astype(t), T(dt, 0)), (kind, dt, n, "sub"))
                # mul, div
                mu = max_updates(dt, npes)
                exp = np.array([2 ** (mu * npes)]).astype(t)[0] if not dt.startswith("f") else t(2.0 ** (mu * npes))
                a.fill(1)
                world.barrier()
                a.batch_mul(np.tile(np.arange(n, dtype=np.uint64), mu), T(dt, 2)).block()
                world.barrier()
                check(np.all(a.to_numpy().astype(t) == exp), (kind, dt, n, "mul"))
                a.batch_div(np.tile(np.arange(n, dtype=np.uint64), mu), T(dt, 2)).block()
                world.barrier()
                check(np.all(a.to_numpy().astype(t) == t(1)), (kind, dt, n, "div"))
                if dt.startswith("f") or kind != "AtomicArray":
                    continue
                # xor / or / and
                idx = np.arange(n, dtype=np.uint64)
                bit = T(dt, 1 << me)
                a.fill(0)
                world.barrier()
                a.batch_bit_xor(idx, bit).block()
                world.barrier()
                check(np.all(a.to_numpy().astype(t) == T(dt, (1 << npes) - 1)), (kind, dt, n, "xor"))
                a.fill(0)
                world.barrier()
                a.batch_bit_or(idx, bit).block()
                world.barrier()
                check(np.all(a.to_numpy().astype(t) == T(dt, (1 << npes) - 1)), (kind, dt, n, "or"))
                ones = t(~t(0))
                a.fill(ones)
                world.barrier()
                a.batch_bit_and(idx, t(~bit)).block()
                world.barrier()
                check(np.all(a.to_numpy().astype(t) == t(ones << t(npes))), (kind, dt, n, "and"))
    np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), fails=np.array(fails, dtype=object).astype(str),
             checks=np.array([checks]))
    world.barrier()
    if npes > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
