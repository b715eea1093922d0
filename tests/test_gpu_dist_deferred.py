"""Deferred exchange sessions (lmr_ctx_exchange_defer, on by default): a batch exchange of an op
that returns nothing leaves each PE's owner session open, so consecutive such batches on one
array share one shard sweep; another op, a barrier, wait_all or any read of the array applies it.
PEs share the GPU over gloo (host-buffer transport), or one rank drives the 1-rank RCCL
communicator (LAMELLAR_FORCE_EXCHANGE=1). Four spawned add batches are applied in fewer sweeps
than batches (the stage profile's tile sweeps), then a fetch_add batch (returning: applies the open
session first, its olds checked against the serial replay's per-element bounds), xor batches
deferred again and read by to_numpy; every state equals numpy's replay (wrapping u64). The same
program with LAMELLAR_EXCHANGE_DEFER=0 (one sweep per batch) gives the same arrays.
Reference: batches are asynchronous until wait_all / a barrier (src/array/operations.rs,
src/lamellar_world.rs wait_all)."""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

PER_PE = (1 << 21) + 3                # u64 elements per PE: > 128 tiles, a count-free owner session

WORKER = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
world = lam.LamellarWorldBuilder().build()
me, ws = world.my_pe(), world.num_pes()
n_len = int(os.environ["LMR_LEN"])
rng = np.random.default_rng(4100 + me)
arr = lam.AtomicArray(world.team(), n_len, lam.Distribution.Block, "u64")
k = world.team().kernels
k.reserve(1 << 23)                    # the owner sessions hold several batches
out = {}
adds = []
k.profile(True)
k.profile_read(reset=True)
for j in range(4):
    gi = rng.integers(0, n_len, 700000 - 1111 * me).astype(np.uint64)
    gv = rng.integers(0, 2**63, gi.size, dtype=np.uint64)
    adds.append((gi, gv))
    arr.batch_add(gi, gv).spawn()
world.wait_all()
st = k.profile_read(reset=True)
out["sweeps"] = np.array([st.get("tile_apply", (0, 0))[1]])
out["coarse"] = np.array([st.get("bin_scatter", (0, 0))[1]])
out["after_add"] = arr.to_numpy()
fi = rng.integers(0, n_len, 300000).astype(np.uint64)
fv = rng.integers(1, 1000, fi.size, dtype=np.uint64)
arr.batch_add(fi, fv).spawn()                    # deferred ...
olds = arr.batch_fetch_add(fi, fv).block()       # ... applied before the fetch_add exchange
out["olds"] = olds.cpu().numpy().view(np.uint64)
xi = rng.integers(0, n_len, 500000).astype(np.uint64)
xv = rng.integers(0, 2**63, xi.size, dtype=np.uint64)
arr.batch_bit_xor(xi, xv).spawn()
arr.batch_bit_xor(xi[::2].copy(), xv[::2].copy()).spawn()
world.barrier()
out["after_xor"] = arr.to_numpy()
for j, (gi, gv) in enumerate(adds):
    out[f"gi{j}"], out[f"gv{j}"] = gi, gv
out["fi"], out["fv"], out["xi"], out["xv"] = fi, fv, xi, xv
np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), **out)
world.barrier()
'''


def _run(ws, env_extra, outdir):
    env = dict(os.environ)
    env.update(env_extra)
    env.update(LMR_ROOT=ROOT, LMR_OUT=outdir, LMR_LEN=str(PER_PE * ws), LAMELLAR_EXCHANGE_CHUNK=str(1 << 18),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29400 + 11 * ws + (os.getpid() % 50)))
    procs = [subprocess.Popen([sys.executable, "-c", WORKER],
                              env=dict(env, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK=str(r)))
             for r in range(ws)]
    try:
        rcs = [p.wait(timeout=170) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0] * ws, rcs
    return [dict(np.load(os.path.join(outdir, f"pe{r}.npz"))) for r in range(ws)]


@pytest.mark.parametrize("ws,backend,defer,mode",
                         [(1, "nccl", "1", ""), (2, "gloo", "1", ""), (3, "gloo", "1", ""), (2, "gloo", "0", ""),
                          (1, "nccl", "1", "buckets"), (2, "gloo", "1", "buckets"), (3, "gloo", "1", "buckets"),
                          (2, "gloo", "0", "buckets")],
                         ids=["rccl-1rank", "gloo-2pe", "gloo-3pe", "gloo-2pe-nodefer", "buckets-1rank", "buckets-2pe",
                              "buckets-3pe", "buckets-2pe-nodefer"])
def test_deferred_exchange_sessions(ws, backend, defer, mode):
    """mode=buckets: the peer transport's bucketed push (LAMELLAR_EXCHANGE_BUCKETS=1): the owner's
    session is the bucketed one (fixed tile regions, no owner coarse pass: no bin_scatter launch
    in the add batches), left open across deferred batches the same way."""
    env = {"LAMELLAR_COMM_BACKEND": backend, "LAMELLAR_EXCHANGE_DEFER": defer}
    if mode == "buckets":
        env.update(LAMELLAR_TRANSPORT="peer", LAMELLAR_EXCHANGE_BUCKETS="1", LAMELLAR_PEER_TIMEOUT="60")
    if ws == 1:
        env["LAMELLAR_FORCE_EXCHANGE"] = "1"
    with tempfile.TemporaryDirectory() as d:
        pe = _run(ws, env, d)
    n_len = PER_PE * ws
    a = np.zeros(n_len, np.uint64)
    for j in range(4):
        for r in range(ws):
            np.add.at(a, pe[r][f"gi{j}"].astype(np.int64), pe[r][f"gv{j}"])
    for r in range(ws):
        assert np.array_equal(pe[r]["after_add"], a), r
    start = a.copy()
    for r in range(ws):
        np.add.at(a, pe[r]["fi"].astype(np.int64), pe[r]["fv"])        # the deferred add batches
    mid = a.copy()
    for r in range(ws):
        np.add.at(a, pe[r]["fi"].astype(np.int64), pe[r]["fv"])        # the fetch_add batches
    for r in range(ws):
        i = pe[r]["fi"].astype(np.int64)
        o = pe[r]["olds"]
        # every fetch_add saw every deferred add applied and at most the other fetch_adds
        assert np.all(o >= mid[i]) and np.all(o < a[i]), r
    for r in range(ws):
        np.bitwise_xor.at(a, pe[r]["xi"].astype(np.int64), pe[r]["xv"])
        np.bitwise_xor.at(a, pe[r]["xi"][::2].astype(np.int64), pe[r]["xv"][::2])
    for r in range(ws):
        assert np.array_equal(pe[r]["after_xor"], a), r
    sweeps = [int(pe[r]["sweeps"][0]) for r in range(ws)]
    if mode == "buckets":
        assert all(int(pe[r]["coarse"][0]) == 0 for r in range(ws)), [int(pe[r]["coarse"][0]) for r in range(ws)]
    if defer == "1":
        assert all(s < 4 for s in sweeps), sweeps          # four batches, fewer sweeps
    else:
        assert all(s == 4 for s in sweeps), sweeps
    del start


DROP_WORKER = r'''
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
world = lam.LamellarWorldBuilder().build()
n_len = int(os.environ["LMR_LEN"])
rng = np.random.default_rng(77)
k = world.team().kernels
k.reserve(1 << 22)
a = lam.AtomicArray(world.team(), n_len, lam.Distribution.Block, "u64")
ai = rng.integers(0, n_len, 600000).astype(np.uint64)
a.batch_add(ai, np.full(ai.size, 3, np.uint64)).spawn()      # left open: deferred exchange session
del a                                                      # dropped before anything applies it
b = lam.AtomicArray(world.team(), n_len, lam.Distribution.Block, "u64")
bi = rng.integers(0, n_len, 500000).astype(np.uint64)
b.batch_add(bi, np.full(bi.size, 5, np.uint64)).spawn()
world.wait_all()
ref = np.zeros(n_len, np.uint64)
np.add.at(ref, bi.astype(np.int64), np.uint64(5))
assert np.array_equal(b.to_numpy(), ref), "records of the dropped array reached the new one"
print("drop ok", flush=True)
world.barrier()
'''


def test_dropped_array_keeps_its_session():
    """An array dropped while its exchange session is open: the session holds its shard until
    the sweep runs, so a new array of the same size (which the caching allocator would place at
    the freed address, continuing the session) sees none of the dropped array's records.
    1-rank RCCL, forced exchange."""
    env = dict(os.environ, LMR_ROOT=ROOT, LMR_LEN=str(PER_PE), LAMELLAR_COMM_BACKEND="nccl",
               LAMELLAR_FORCE_EXCHANGE="1", LAMELLAR_EXCHANGE_CHUNK=str(1 << 18), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29500 + (os.getpid() % 50)))
    p = subprocess.run([sys.executable, "-c", DROP_WORKER], env=env, timeout=170,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert p.returncode == 0 and "drop ok" in p.stdout, p.stdout[-4000:]


CABI_WORKER = r'''
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
from lamellar_runtime_amd import _capi
world = lam.LamellarWorldBuilder().build()
n_len = int(os.environ["LMR_LEN"])
rng = np.random.default_rng(1234)
k = world.team().kernels
k.reserve(1 << 22)
lib = _capi.lib()
a = lam.AtomicArray(world.team(), n_len, lam.Distribution.Block, "u64")
ai = rng.integers(0, n_len, 600000).astype(np.uint64)
av = rng.integers(0, 2**63, ai.size, dtype=np.uint64)
a.batch_add(ai, av).spawn()                 # exchange left open: a deferred session in the workspace
assert k._xdeferred is not None
# a Rust caller on the raw ABI, with no Python flush in between: the staged-session calls are refused
# while the session is open ...
m = 1 << 20
b = torch.zeros(n_len, dtype=torch.int64, device=k.device)
bi = rng.integers(0, n_len, m).astype(np.uint64)
bv = rng.integers(0, 2**63, m, dtype=np.uint64)
ti = torch.from_numpy(bi.view(np.int64)).to(k.device)
tv = torch.from_numpy(bv.view(np.int64)).to(k.device)
d = k._desc(b, n_len, 1, lam.dtype_of("u64"), int(lam.ArrayOpCmd.Add))
assert lib.lmr_stage_begin(k.ctx, ctypes.byref(d)) == 1
assert lib.lmr_stage_finish(k.ctx, k.stream()) == 1
# ... and a tiled apply on another shard applies the open session first (stream order)
st = lib.lmr_apply_soa(k.ctx, ctypes.byref(d), ti.data_ptr(), 8, tv.data_ptr(), None, m, None, None, k.stream())
assert st == 0, st
k._xdeferred = None                         # (the apply above applied the open session)
assert lib.lmr_exchange_flush(k.ctx, k.stream()) == 0          # nothing left open: a no-op
assert lib.lmr_stage_begin(k.ctx, ctypes.byref(d)) == 0
assert lib.lmr_stage_finish(k.ctx, k.stream()) == 0
torch.cuda.synchronize()
assert k.errors() == 0
ra = np.zeros(n_len, np.uint64)
np.add.at(ra, ai.astype(np.int64), av)
rb = np.zeros(n_len, np.uint64)
np.add.at(rb, bi.astype(np.int64), bv)
assert np.array_equal(a.to_numpy(), ra), "the deferred exchange batch"
assert np.array_equal(b.cpu().numpy().view(np.uint64), rb), "the tiled apply on the other shard"
print("cabi ok", flush=True)
world.barrier()
'''


def test_deferred_session_protected_at_the_c_abi():
    """A deferred exchange session lives in the context's workspace: a tiled lmr_apply_soa on
    another shard, called through the raw C ABI with no flush in between (a Rust caller), applies
    the open session first in its stream order instead of reusing the workspace under it, and
    lmr_stage_begin is refused until lmr_exchange_flush. Both arrays equal numpy's replay.
    1-rank RCCL, forced exchange."""
    env = dict(os.environ, LMR_ROOT=ROOT, LMR_LEN=str(PER_PE), LAMELLAR_COMM_BACKEND="nccl",
               LAMELLAR_FORCE_EXCHANGE="1", LAMELLAR_EXCHANGE_CHUNK=str(1 << 18), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29550 + (os.getpid() % 50)))
    p = subprocess.run([sys.executable, "-c", CABI_WORKER], env=env, timeout=170,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    assert p.returncode == 0 and "cabi ok" in p.stdout, p.stdout[-4000:]
