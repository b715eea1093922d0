"""Order-dependent ops through the device exchange (lmr_batch_exchange) at 1, 2, 4 and
8 PEs sharing the box's GPU, every pack / stage / apply / scatter a real HIP kernel.

The reference returns swap olds and compare_exchange Result<T,T>s to the issuing PE as
AM data (registered_active_message.rs:307-339 send_data_am, :530-554 exec_data_am) and
applies each record with one SeqCst RMW, a per-element mutex or a shard lock
(impl/src/array_ops.rs:327-545); it promises no order (operations/arithmetic.rs:57-58).
Its op tests run every op at 2, 3 and 4 PEs (lamellar_run.sh:31-40, tests/add.rs:24-47;
tests/array/atomic_ops/{swap,compare_exchange}_test.rs).

Checks, per case, over the records of every PE together (indices collide across PEs):
* add (C4's u64 batch_add) and and / or / xor (C5's first three batches): the final global
  array bit-exact against the oracle's sequential apply;
* swap, compare_exchange (Result values and Ok flags), compare_exchange_epsilon
  (NativeAtomic, GenericAtomic, LocalLock), fetch_xor, fetch_mul, fetch_add on i16 and
  f32: per element, the returned values / Ok flags and the final value form one serial
  order (oracle/linearize.c).

Transports: the gloo host transport (host_buffers = 1) at 2, 4 and 8 PEs; a device-
pointer transport over gloo (host_buffers = 0, tests/dist_ordered_worker.py), which is
handed the same non-prefix send offsets (count-free pack regions) and gapped receive
layouts (self-bypass) as the RCCL transport; and a 1-rank RCCL communicator
(LAMELLAR_FORCE_EXCHANGE=1), where the Ok flags cross RCCL in the unit-1 all-to-all-v.
Reduced C4/C5 shape: 2^18 records per PE and batch, chunks of 2^16 (4 per batch).
"""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from opgen import ADD, AND, NP, OR, XOR

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dist_ordered_worker.py")
pytestmark = pytest.mark.gpu

DTN = {0: "u8", 1: "u16", 2: "u32", 3: "u64", 4: "i8", 5: "i16", 6: "i32", 7: "i64", 8: "f32", 9: "f64"}
NREC = 1 << 18
LEN = (1 << 18) + 13
CHUNK = 1 << 16


def run_pes(ws, dist_kind, env_extra, outdir, port):
    env = dict(os.environ)
    env.update(LMR_ROOT=ROOT, LMR_OUT=outdir, LMR_DIST=str(dist_kind), LMR_LEN=str(LEN), LMR_NREC=str(NREC),
               LAMELLAR_EXCHANGE_CHUNK=str(CHUNK), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.update(env_extra)
    procs = [subprocess.Popen([sys.executable, "-u", WORKER],
                              env=dict(env, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK=str(r)))
             for r in range(ws)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * ws, rcs
    return [dict(np.load(os.path.join(outdir, f"pe{r}.npz"))) for r in range(ws)]


def check_cases(orc, pe):
    names = sorted({k.split(":")[0] for k in pe[0] if k.endswith(":meta")})
    assert len(names) == 16, names
    for name in names:
        op, code, kind = (int(x) for x in pe[0][name + ":meta"])
        t = NP[DTN[code]]
        before, after = pe[0][name + ":before"], pe[0][name + ":after"]
        for p in pe[1:]:                                   # the global view agrees on every PE
            assert np.array_equal(p[name + ":before"].view(np.uint8), before.view(np.uint8)), name
            assert np.array_equal(p[name + ":after"].view(np.uint8), after.view(np.uint8)), name
        idx = np.concatenate([p[name + ":idx"] for p in pe])
        vals = np.concatenate([p[name + ":vals"] for p in pe]).astype(t)
        if op in (ADD, AND, OR, XOR):
            ref = before.copy()
            L = orc.layout_new(ref.size, 1, 0, 0)
            st, _, _ = orc.batch_op(L, [ref], kind, code, t, op, idx, vals)
            assert st == 0
            assert np.array_equal(after, ref), name
            continue
        res = np.concatenate([p[name + ":res"] for p in pe]).astype(t)
        ok = np.concatenate([p[name + ":ok"] for p in pe]) if name + ":ok" in pe[0] else None
        cur = pe[0][name + ":cur"][0] if name + ":cur" in pe[0] else None
        eps = pe[0][name + ":eps"][0] if name + ":eps" in pe[0] else None
        if ok is not None:
            assert ok.any() and (~ok.astype(bool)).any(), (name, "expected successes and failures")
        st, bad = orc.check_linearizable(kind, code, t, op, before, after, idx, vals, res, ok, cur, eps)
        assert st == 0, (name, "status", st, "element", bad, "records", int((idx == bad).sum()))


@pytest.mark.parametrize("ws,dist_kind", [(2, 0), (3, 0), (4, 1), (8, 0), (8, 1)],
                         ids=["2pe-Block", "3pe-Block", "4pe-Cyclic", "8pe-Block", "8pe-Cyclic"])
def test_ordered_ops_gloo_host_transport(orc, ws, dist_kind):
    with tempfile.TemporaryDirectory() as d:
        pe = run_pes(ws, dist_kind, {"LAMELLAR_COMM_BACKEND": "gloo"}, d, 29300 + 10 * ws + dist_kind)
    check_cases(orc, pe)


@pytest.mark.parametrize("ws,dist_kind", [(2, 1), (4, 0)], ids=["2pe-Cyclic", "4pe-Block"])
def test_ordered_ops_device_pointer_transport(orc, ws, dist_kind):
    """host_buffers = 0: the callbacks get device pointers with RCCL's offsets (count-free
    send regions, the receive layout's self-bypass gap) and copy segment by segment."""
    with tempfile.TemporaryDirectory() as d:
        pe = run_pes(ws, dist_kind, {"LAMELLAR_COMM_BACKEND": "gloo", "LMR_XPORT": "devptr"}, d,
                     29400 + 10 * ws + dist_kind)
    check_cases(orc, pe)
    x = np.array([p["xport"] for p in pe])            # per PE: gapped sends, gapped receives, calls
    assert (x[:, 2] > 0).all()
    # (the last PE's receive layout has no gap after its own slot; with 2 PEs the last PE's
    # only send region starts at 0)
    assert x[:, 0].sum() > 0, "the count-free pack's fixed send regions were never handed over"
    assert x[:, 1].sum() > 0, "the self-bypass gap in the receive layout was never handed over"


def test_ordered_ops_rccl_one_rank(orc):
    """A 1-rank RCCL communicator with LAMELLAR_FORCE_EXCHANGE=1: records, results and
    Ok flags (unit 1) all cross RCCL's grouped send / recv."""
    with tempfile.TemporaryDirectory() as d:
        pe = run_pes(1, 0, {"LAMELLAR_COMM_BACKEND": "nccl", "LAMELLAR_FORCE_EXCHANGE": "1"}, d, 29390)
    check_cases(orc, pe)
