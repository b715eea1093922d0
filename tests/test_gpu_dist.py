"""Multi-PE path on the device (GPU box has one GPU):

* two PEs share the GPU, the exchange goes over gloo (LAMELLAR_COMM_BACKEND),
  every pack / apply / scatter is the real HIP kernel — checked against the
  oracle simulating both PEs;
* one PE with a 1-rank RCCL process group and LAMELLAR_FORCE_EXCHANGE=1: the
  exact torch.distributed "nccl" (RCCL) all-to-all calls the 8-GPU run makes.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

WORKER = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
world = lam.LamellarWorldBuilder().build()
me, ws = world.my_pe(), world.num_pes()
dist_kind = int(os.environ["LMR_DIST"])
rng = np.random.default_rng(500 + me)
n_len = 40009
out = {}
arr = lam.AtomicArray(world.team(), n_len, dist_kind, "u64")
gi = rng.integers(0, n_len, 200000).astype(np.uint64)
gv = rng.integers(0, 2**40, gi.size).astype(np.uint64)
arr.batch_add(gi, gv).block(); world.barrier()
out["after_add"] = arr.to_numpy()
# skewed: every record to the first quarter of the array (one PE under Block): the
# count-free pack's per-PE region overflows and the chunk is packed again, counted
si = rng.integers(0, n_len // 4, 150000).astype(np.uint64)
arr.batch_add(si, 3).block(); world.barrier()
arr.batch_sub(si, 3).block(); world.barrier()
out["after_skew"] = arr.to_numpy()
fi = rng.permutation(n_len)[:20000].astype(np.uint64)
olds = arr.batch_fetch_add(fi, 7).block(); world.barrier()
out["fetch_olds"] = olds.cpu().numpy().view(np.uint64)
out["after_fetch"] = arr.to_numpy()
arr.batch_add(5, np.arange(1, 11, dtype=np.uint64)).block(); world.barrier()
out["after_mvsi"] = arr.to_numpy()
f = lam.AtomicArray(world.team(), 3001, dist_kind, "f64")
fj = rng.integers(0, 3001, 50000).astype(np.uint64)
f.batch_add(fj, 1.0).block(); world.barrier()
out["f_after"] = f.to_numpy()
out["gi"], out["gv"], out["fi"], out["fj"] = gi, gv, fi, fj
out["self_bytes"] = np.array(getattr(world.team().transport(), "self_bytes", -1) if ws > 1 else -1)
np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), **out)
world.barrier()
'''


def _run(ws, env_extra, outdir, dist_kind):
    env = dict(os.environ)
    env.update(env_extra)
    env.update(LMR_ROOT=ROOT, LMR_OUT=outdir, LMR_DIST=str(dist_kind), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(29700 + dist_kind + 10 * ws + (os.getpid() % 100)))
    procs = []
    for r in range(ws):
        e = dict(env, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=e))
    rcs = [p.wait(timeout=300) for p in procs]
    assert rcs == [0] * ws, rcs


def _check(orc, outdir, ws, dist_kind):
    from simworld import SimArray
    pe = [dict(np.load(os.path.join(outdir, f"pe{r}.npz"))) for r in range(ws)]
    a = SimArray(orc, ws, 40009, dist_kind, "u64")
    for r in range(ws):
        assert a.op(0, pe[r]["gi"], pe[r]["gv"])[0] == 0
    exp = a.to_numpy()
    for r in range(ws):
        assert np.array_equal(pe[r]["after_add"], exp)
        assert np.array_equal(pe[r]["after_skew"], exp)       # +3 then -3 per skewed record
    cnt = np.zeros(exp.size, np.uint64)
    for r in range(ws):
        cnt[pe[r]["fi"].astype(np.int64)] += np.uint64(1)
    exp2 = exp + cnt * np.uint64(7)
    assert np.array_equal(pe[0]["after_fetch"], exp2)
    for r in range(ws):
        fi, olds = pe[r]["fi"].astype(np.int64), pe[r]["fetch_olds"]
        assert np.all((olds == exp[fi]) | (olds == exp[fi] + np.uint64(7)))
        if ws == 1:
            assert np.array_equal(olds, exp[fi])
    exp3 = exp2.copy()
    exp3[5] += np.uint64(55 * ws)
    assert np.array_equal(pe[-1]["after_mvsi"], exp3)
    fexp = np.zeros(3001)
    for r in range(ws):
        np.add.at(fexp, pe[r]["fj"].astype(np.int64), 1.0)
    assert np.array_equal(pe[0]["f_after"], fexp)
    if ws > 1:                        # a PE's own records never went through the transport
        via = os.environ.get("LAMELLAR_EXCHANGE_SELF", "") == "transport"
        for r in range(ws):
            assert (int(pe[r]["self_bytes"]) > 0) == via, (r, int(pe[r]["self_bytes"]))


@pytest.mark.parametrize("dist_kind", [0, 1], ids=["Block", "Cyclic"])
def test_two_pes_one_gpu_gloo_exchange(orc, dist_kind):
    with tempfile.TemporaryDirectory() as d:
        _run(2, {"LAMELLAR_COMM_BACKEND": "gloo"}, d, dist_kind)
        _check(orc, d, 2, dist_kind)


def test_peer_transport_falls_back_to_base(orc):
    """LAMELLAR_TRANSPORT=peer with shards of <= 128 tiles (counted owner sessions), fetch_add,
    MVSI and f64 batches: nothing here takes the push, every batch goes through the base
    transport's collectives under the peer transport's handshake."""
    with tempfile.TemporaryDirectory() as d:
        _run(2, {"LAMELLAR_COMM_BACKEND": "gloo", "LAMELLAR_TRANSPORT": "peer", "LAMELLAR_PEER_TIMEOUT": "60"}, d, 0)
        _check(orc, d, 2, 0)


@pytest.mark.parametrize("chunk", [None, 7000], ids=["one-chunk", "chunked"])
def test_rccl_exchange_calls_one_rank(orc, chunk):
    """chunked: LAMELLAR_EXCHANGE_CHUNK=7000 pipelines 29 chunks of the add and 3
    of the fetch_add over the pack / RCCL / apply streams."""
    env = {"LAMELLAR_FORCE_EXCHANGE": "1", "LAMELLAR_COMM_BACKEND": "nccl"}
    if chunk:
        env["LAMELLAR_EXCHANGE_CHUNK"] = str(chunk)
    with tempfile.TemporaryDirectory() as d:
        _run(1, env, d, 0)
        _check(orc, d, 1, 0)


def test_two_pes_one_gpu_gloo_chunked(orc):
    with tempfile.TemporaryDirectory() as d:
        _run(2, {"LAMELLAR_COMM_BACKEND": "gloo", "LAMELLAR_EXCHANGE_CHUNK": "9000"}, d, 1)
        _check(orc, d, 2, 1)


BIG_WORKER = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
world = lam.LamellarWorldBuilder().build()
me, ws = world.my_pe(), world.num_pes()
rng = np.random.default_rng(900 + me)
n_len = (1 << 21) + 9
arr = lam.AtomicArray(world.team(), n_len, lam.Distribution.Block, "u64")
gi = rng.integers(0, n_len, 1 << 20).astype(np.uint64)
gv = rng.integers(0, 2**40, gi.size).astype(np.uint64)
arr.batch_add(gi, gv).block(); world.barrier()
after_add = arr.to_numpy()
# conflict-free fetch_add across PEs: PE p takes the indices = p (mod ws)
perm = np.random.default_rng(7).permutation(n_len)
fi = perm[perm % ws == me][:300000].astype(np.uint64)
olds = arr.batch_fetch_add(fi, gv[:fi.size]).block(); world.barrier()
np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), after_add=after_add, gi=gi, gv=gv, fi=fi,
         olds=olds.cpu().numpy().view(np.uint64), after_fetch=arr.to_numpy())
world.barrier()
'''


@pytest.mark.parametrize("ws,backend", [(1, "nccl"), (2, "gloo")], ids=["rccl-1rank", "gloo-2pe"])
def test_staged_exchange_many_chunks(orc, ws, backend):
    """> 128 tiles per shard, 2^20 records per PE in chunks of 2^18: every chunk's
    received records are staged as regions (coarse + piece partition) and applied in
    one sweep; final state and fetch olds against the oracle."""
    env = dict(os.environ, LMR_ROOT=ROOT, LAMELLAR_COMM_BACKEND=backend, LAMELLAR_EXCHANGE_CHUNK=str(1 << 18),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29800 + ws + (os.getpid() % 100)))
    if ws == 1:
        env["LAMELLAR_FORCE_EXCHANGE"] = "1"
    with tempfile.TemporaryDirectory() as d:
        env["LMR_OUT"] = d
        procs = [subprocess.Popen([sys.executable, "-c", BIG_WORKER],
                                  env=dict(env, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK=str(r)))
                 for r in range(ws)]
        assert [p.wait(timeout=300) for p in procs] == [0] * ws
        pe = [dict(np.load(os.path.join(d, f"pe{r}.npz"))) for r in range(ws)]
    n_len = (1 << 21) + 9
    exp = np.zeros(n_len, dtype=np.uint64)
    for r in range(ws):
        np.add.at(exp, pe[r]["gi"].astype(np.int64), pe[r]["gv"])
    for r in range(ws):
        assert np.array_equal(pe[r]["after_add"], exp)
    exp2 = exp.copy()
    for r in range(ws):
        fi = pe[r]["fi"].astype(np.int64)
        assert np.array_equal(pe[r]["olds"], exp[fi])
        exp2[fi] += pe[r]["gv"][:fi.size]
    for r in range(ws):
        assert np.array_equal(pe[r]["after_fetch"], exp2)
