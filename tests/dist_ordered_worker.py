"""One PE of the multi-PE order-dependent exchange tests (test_gpu_dist_ordered.py).

Launched once per PE (RANK / WORLD_SIZE / LOCAL_RANK in the environment; every PE
shares the one GPU of the box). Runs swap, compare_exchange, compare_exchange_epsilon,
fetch_xor, fetch_mul, fetch_add on 16-bit and float elements, and the C5 mixed u32
sequence (bit_and, bit_or, bit_xor, swap, compare_exchange) through the real
lmr_batch_exchange, with indices that collide across PEs, and saves per case the
global array before and after, this PE's records and what came back. The parent
checks them with the oracle (tests/test_gpu_dist_ordered.py).

LMR_MODE=small runs instead one-AM batches (fewer than 1000 records per PE, indices
repeated within and across PEs): swap, store, compare_exchange, fetch_rem and f64
fetch_add, whose outcome the reference fixes per source (each destination's records in
input order, applied sequentially by the owner's AM); the parent replays them with the
oracle (test_gpu_dist_small.py).

LMR_XPORT=devptr replaces the transport by `DevPtrGlooTransport` below: a
host_buffers = 0 transport (the library hands it device pointers, exactly as it
hands them to RCCL) whose collectives run over gloo. It copies each PE's segment
at the offset the library gives, so the self-bypass gap in the receive layout
and the count-free pack's fixed send regions (non-prefix offsets) are exercised
the way the RCCL transport sees them.
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.environ["LMR_ROOT"])
sys.path.insert(0, os.path.join(os.environ["LMR_ROOT"], "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from _lamellar_bootstrap import load_package  # noqa: E402

lam = load_package()
from lamellar_runtime_amd import _capi  # noqa: E402

_H2D, _D2H = 1, 2


class DevPtrGlooTransport:
    """lmr_transport_t with host_buffers = 0 over a gloo group (test double of RCCL's
    calling convention: device pointers, per-PE byte counts and offsets)."""

    def __init__(self, num_pes, my_pe, group):
        self.num_pes, self.my_pe, self.group = num_pes, my_pe, group
        self.error = None
        self.gapped_send = 0        # calls whose send offsets were not prefix sums
        self.gapped_recv = 0
        self.calls = 0
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        self.hip = hip
        self._a2a = _capi.ALLTOALL_FN(self._alltoall)
        self._a2av = _capi.ALLTOALLV_FN(self._alltoallv)
        self.t = _capi.lmr_transport_t(num_pes, my_pe, 0, 1, None, self._a2a, self._a2av)   # flags: split headers

    @property
    def ptr(self):
        return ctypes.c_void_p(ctypes.addressof(self.t))

    def raise_pending(self):
        if self.error is not None:
            e, self.error = self.error, None
            raise e

    def _copy(self, dst, src, n, kind):
        if n and self.hip.hipMemcpy(dst, src, n, kind) != 0:
            raise RuntimeError("hipMemcpy failed")

    def _alltoall(self, _self, send, recv, nbytes, stream):
        try:
            self.calls += 1
            if self.hip.hipStreamSynchronize(stream) != 0:
                raise RuntimeError("hipStreamSynchronize failed")
            tot = int(nbytes) * self.num_pes
            s = torch.empty(tot, dtype=torch.uint8)
            r = torch.empty(tot, dtype=torch.uint8)
            self._copy(s.data_ptr(), send, tot, _D2H)
            dist.all_to_all_single(r, s, group=self.group)
            self._copy(recv, r.data_ptr(), tot, _H2D)
            return 0
        except Exception as e:  # noqa: BLE001
            self.error = e
            return 6

    def _alltoallv(self, _self, send, sb, so, recv, rb, ro, unit, stream):
        try:
            self.calls += 1
            n = self.num_pes
            sb, so, rb, ro = ([int(a[p]) for p in range(n)] for a in (sb, so, rb, ro))
            assert all(x % unit == 0 for x in sb + so + rb + ro), "splits not multiples of the unit"
            if any(sb[p] and so[p] != sum(sb[:p]) for p in range(n)):
                self.gapped_send += 1
            if any(rb[p] and ro[p] != sum(rb[:p]) for p in range(n)):
                self.gapped_recv += 1
            if self.hip.hipStreamSynchronize(stream) != 0:
                raise RuntimeError("hipStreamSynchronize failed")
            s = torch.empty(sum(sb), dtype=torch.uint8)
            r = torch.empty(sum(rb), dtype=torch.uint8)
            a = 0
            for p in range(n):
                self._copy(s.data_ptr() + a, send + so[p], sb[p], _D2H)
                a += sb[p]
            dist.all_to_all_single(r, s, output_split_sizes=rb, input_split_sizes=sb, group=self.group)
            a = 0
            for p in range(n):
                self._copy(recv + ro[p], r.data_ptr() + a, rb[p], _H2D)
                a += rb[p]
            return 0
        except Exception as e:  # noqa: BLE001
            self.error = e
            return 6


def main():
    from opgen import CODE, NP, ADD, CAS, CAS_EPS, FETCH_ADD, FETCH_MUL, FETCH_XOR, SWAP, AND, OR, XOR
    if os.environ.get("LMR_MODE") == "small":
        return main_small()
    world = lam.LamellarWorldBuilder().build()
    team = world.team()
    me, ws = world.my_pe(), world.num_pes()
    if os.environ.get("LMR_XPORT") == "devptr":
        team._transport = DevPtrGlooTransport(ws, me, team.group)
    dist_kind = int(os.environ["LMR_DIST"])
    n_len = int(os.environ["LMR_LEN"])
    nrec = int(os.environ["LMR_NREC"])
    rng = np.random.default_rng(4242 + 17 * me)
    shared = np.random.default_rng(99)              # the same on every PE: collisions across PEs
    hot = shared.choice(n_len, max(16, n_len // 16), replace=False).astype(np.uint64)
    hot_wide = shared.choice(n_len, max(16, n_len // 2), replace=False).astype(np.uint64)
    out = {}

    def case(name, cls, dt, op, fn, init, idx, vals, cur=None, eps=None):
        arr = cls(team, n_len, dist_kind, dt)
        t = NP[dt]
        mine = init(arr.num_elems_local(), t)
        arr.local_data().copy_(_storage(mine, arr))
        world.barrier()
        before = arr.to_numpy()
        h = fn(arr, idx, vals)
        r = h.block()
        world.barrier()
        after = arr.to_numpy()
        out[name + ":before"], out[name + ":after"] = before, after
        out[name + ":idx"], out[name + ":vals"] = idx, vals.astype(t)
        out[name + ":meta"] = np.array([op, CODE[dt], arr.kind])
        if r is not None:
            if hasattr(r, "numpy") and not isinstance(r, torch.Tensor):
                v, ok = r.numpy()
                out[name + ":res"], out[name + ":ok"] = v, ok.astype(np.uint8)
            else:
                out[name + ":res"] = r.cpu().numpy().view(t)
        if cur is not None:
            out[name + ":cur"] = np.array([cur], dtype=t)
        if eps is not None:
            out[name + ":eps"] = np.array([eps], dtype=t)

    def pick(pool, n):
        return pool[rng.integers(0, pool.size, n)].astype(np.uint64)

    u_any = lambda t: (lambda n, _t: rng.integers(0, np.iinfo(t).max, n, dtype=t, endpoint=True))  # noqa: E731

    # swap (u64): last writer wins; every old must chain
    case("swap_u64", lam.AtomicArray, "u64", SWAP, lambda a, i, v: a.batch_swap(i, v),
         u_any(np.uint64), pick(hot, nrec), rng.integers(0, 2**63, nrec, dtype=np.uint64))
    # compare_exchange (u32, current = 3): Ok flags travel back over the unit-1 all-to-all-v
    def few(t, k):
        return lambda n, _t: rng.integers(0, k, n).astype(t)
    v = rng.integers(0, 6, nrec).astype(np.uint32)
    case("cas_u32", lam.AtomicArray, "u32", CAS, lambda a, i, v: a.batch_compare_exchange(i, np.uint32(3), v),
         few(np.uint32, 6), pick(hot, nrec), v, cur=np.uint32(3))
    v = rng.integers(-3, 4, nrec).astype(np.int64)
    case("cas_i64", lam.AtomicArray, "i64", CAS, lambda a, i, v: a.batch_compare_exchange(i, np.int64(-1), v),
         lambda n, _t: rng.integers(-3, 4, n).astype(np.int64), pick(hot, nrec), v, cur=np.int64(-1))
    # compare_exchange_epsilon: NativeAtomic (Ok(new) on an exact match), GenericAtomic f64, LocalLock
    m = max(1, nrec // 8)
    v = rng.integers(0, 8, m).astype(np.int32)
    case("caseps_i32", lam.AtomicArray, "i32", CAS_EPS,
         lambda a, i, v: a.batch_compare_exchange_epsilon(i, np.int32(3), v, np.int32(2)),
         few(np.int32, 8), pick(hot_wide, m), v, cur=np.int32(3), eps=np.int32(2))
    v = rng.integers(0, 8, m).astype(np.float64)
    case("caseps_f64", lam.AtomicArray, "f64", CAS_EPS,
         lambda a, i, v: a.batch_compare_exchange_epsilon(i, 3.0, v, 0.5),
         lambda n, _t: rng.integers(0, 8, n).astype(np.float64), pick(hot_wide, m), v, cur=np.float64(3.0),
         eps=np.float64(0.5))
    v = rng.integers(0, 8, m).astype(np.uint16)
    case("caseps_ll_u16", lam.LocalLockArray, "u16", CAS_EPS,
         lambda a, i, v: a.batch_compare_exchange_epsilon(i, np.uint16(3), v, np.uint16(1)),
         few(np.uint16, 8), pick(hot_wide, m), v, cur=np.uint16(3), eps=np.uint16(1))
    # fetch_xor (u64), fetch_mul (u32, odd factors: no collapse to 0), fetch_add on i16 (32-bit
    # word CAS) and f32 (exact small integers)
    case("fxor_u64", lam.AtomicArray, "u64", FETCH_XOR, lambda a, i, v: a.batch_fetch_bit_xor(i, v),
         u_any(np.uint64), pick(hot, nrec), rng.integers(0, 2**63, nrec, dtype=np.uint64))
    case("fmul_u32", lam.AtomicArray, "u32", FETCH_MUL, lambda a, i, v: a.batch_fetch_mul(i, v),
         lambda n, _t: (rng.integers(0, 2**31, n) * 2 + 1).astype(np.uint32), pick(hot, nrec),
         (rng.integers(0, 500, nrec) * 2 + 1).astype(np.uint32))
    case("fadd_i16", lam.AtomicArray, "i16", FETCH_ADD, lambda a, i, v: a.batch_fetch_add(i, v),
         lambda n, _t: rng.integers(-2**15, 2**15, n).astype(np.int16),
         pick(hot, nrec), rng.integers(-2**15, 2**15, nrec).astype(np.int16))
    case("fadd_f32", lam.AtomicArray, "f32", FETCH_ADD, lambda a, i, v: a.batch_fetch_add(i, v),
         lambda n, _t: rng.integers(-1000, 1000, n).astype(np.float32), pick(hot, nrec),
         rng.integers(-64, 64, nrec).astype(np.float32))
    # C4's op: u64 batch_add (wrapping sums commute: the final array is bit-exact)
    case("add_u64", lam.AtomicArray, "u64", ADD, lambda a, i, v: a.batch_add(i, v),
         u_any(np.uint64), rng.integers(0, n_len, nrec).astype(np.uint64),
         rng.integers(0, 2**64, nrec, dtype=np.uint64))
    # C5's mixed u32 sequence on one array: bit_and, bit_or, bit_xor, swap, compare_exchange(0)
    c5 = lam.AtomicArray(team, n_len, dist_kind, "u32")
    c5.local_data().copy_(_storage(rng.integers(0, 4, c5.num_elems_local()), c5))
    world.barrier()
    for step, (op, fn) in enumerate(((AND, "batch_bit_and"), (OR, "batch_bit_or"), (XOR, "batch_bit_xor"),
                                     (SWAP, "batch_swap"), (CAS, "batch_compare_exchange"))):
        name = f"c5_{step}"
        before = c5.to_numpy()
        idx = rng.integers(0, n_len, nrec).astype(np.uint64)
        vals = rng.integers(0, 2**32, nrec, dtype=np.uint64).astype(np.uint32)
        if op == CAS:
            vals[rng.random(nrec) < 0.1] = 0
            r = c5.batch_compare_exchange(idx, np.uint32(0), vals).block()
            v, ok = r.numpy()
            out[name + ":res"], out[name + ":ok"] = v, ok.astype(np.uint8)
            out[name + ":cur"] = np.array([0], dtype=np.uint32)
        else:
            r = getattr(c5, fn)(idx, vals).block()
            if r is not None:
                out[name + ":res"] = r.cpu().numpy().view(np.uint32)
        world.barrier()
        out[name + ":before"], out[name + ":after"] = before, c5.to_numpy()
        out[name + ":idx"], out[name + ":vals"] = idx, vals
        out[name + ":meta"] = np.array([op, CODE["u32"], c5.kind])
        if step == 2:                        # zeros so that compare_exchange(0) succeeds somewhere
            c5.local_data()[: c5.num_elems_local() // 8] = 0
            world.barrier()
    tp = team._transport
    out["xport"] = np.array([getattr(tp, "gapped_send", -1), getattr(tp, "gapped_recv", -1),
                             getattr(tp, "calls", -1)])
    np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), **out)
    world.barrier()
    if ws > 1:
        dist.destroy_process_group()


def main_small():
    """One-AM batches: every PE issues fewer than 1000 records per batch over a small hot set
    that all PEs share, so elements are hit repeatedly by every source."""
    from opgen import CODE, NP, CAS, FETCH_ADD, FETCH_REM, STORE, SWAP
    world = lam.LamellarWorldBuilder().build()
    team = world.team()
    me, ws = world.my_pe(), world.num_pes()
    if os.environ.get("LMR_XPORT") == "devptr":
        team._transport = DevPtrGlooTransport(ws, me, team.group)
    dist_kind = int(os.environ["LMR_DIST"])
    n_len = int(os.environ["LMR_LEN"])
    nrec = int(os.environ["LMR_NREC"])
    assert nrec < 1000
    rng = np.random.default_rng(5151 + 31 * me)
    hot = np.random.default_rng(77).choice(n_len, 24, replace=False).astype(np.uint64)
    out = {}

    def case(name, cls, dt, op, fn, init, vals, cur=None):
        arr = cls(team, n_len, dist_kind, dt)
        t = NP[dt]
        arr.local_data().copy_(_storage(init(arr.num_elems_local()).astype(t), arr))
        world.barrier()
        before = arr.to_numpy()
        idx = hot[rng.integers(0, hot.size, nrec)]
        r = fn(arr, idx, vals).block()
        world.barrier()
        out[name + ":before"], out[name + ":after"] = before, arr.to_numpy()
        out[name + ":idx"], out[name + ":vals"] = idx, vals.astype(t)
        out[name + ":meta"] = np.array([op, CODE[dt], arr.kind])
        if r is not None:
            if hasattr(r, "numpy") and not isinstance(r, torch.Tensor):
                v, ok = r.numpy()
                out[name + ":res"], out[name + ":ok"] = v, ok.astype(np.uint8)
            else:
                out[name + ":res"] = r.cpu().numpy().view(t)
        if cur is not None:
            out[name + ":cur"] = np.array([cur], dtype=t)

    case("swap_u64", lam.AtomicArray, "u64", SWAP, lambda a, i, v: a.batch_swap(i, v),
         lambda n: rng.integers(0, 2**63, n, dtype=np.uint64), rng.integers(0, 2**63, nrec, dtype=np.uint64))
    case("store_u32", lam.AtomicArray, "u32", STORE, lambda a, i, v: a.batch_store(i, v),
         lambda n: rng.integers(0, 2**32, n, dtype=np.uint64), rng.integers(0, 2**32, nrec, dtype=np.uint64))
    case("cas_i64", lam.AtomicArray, "i64", CAS, lambda a, i, v: a.batch_compare_exchange(i, np.int64(1), v),
         lambda n: rng.integers(0, 3, n), rng.integers(0, 3, nrec).astype(np.int64), cur=np.int64(1))
    case("frem_u32", lam.AtomicArray, "u32", FETCH_REM, lambda a, i, v: a.batch_fetch_rem(i, v),
         lambda n: rng.integers(2**20, 2**32, n, dtype=np.uint64), rng.integers(2, 1000, nrec).astype(np.uint32))
    case("fadd_f64", lam.AtomicArray, "f64", FETCH_ADD, lambda a, i, v: a.batch_fetch_add(i, v),
         lambda n: rng.random(n) * 1e3, rng.random(nrec) * 10.0 - 5.0)
    np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), **out)
    world.barrier()
    if ws > 1:
        dist.destroy_process_group()


def _storage(mine, arr):
    """numpy values -> a tensor of the array's device storage dtype, same bits."""
    a = np.ascontiguousarray(np.asarray(mine).astype(arr.dtype.np))
    return torch.from_numpy(a.view(np.dtype(arr.dtype.torch_name))).to(arr.local_data().device)


if __name__ == "__main__":
    main()
