"""The exchange's bucketed regions (lmr_bucket.hip) across element types and layouts: the sender
packs by (owner, owner bucket of 256 tiles) into the owners' bucket slices -- over the peer push,
or in its send buffer for the collective transport -- and the owner bins each chunk into its
session's fixed tile regions. The other bucketed tests use u64 Block arrays; here
1-, 2-, 4- and 8-byte elements (signed and unsigned), Block and Cyclic layouts, 2 and 3 PEs sharing
the GPU over gloo: array-valued add, xor, mul, and a skewed scalar add whose slices overflow (the overflow
round, applied with device atomics), every final state against numpy's serial replay (wrapping in
the element type: these ops commute, so any order gives the same array). The stage profile shows
the mode ran: no owner coarse pass in the add / xor / mul batches."""
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
dt = os.environ["LMR_DT"]
npt = np.dtype(lam.dtype_of(dt).np)
n_len = int(os.environ["LMR_LEN"])
dist = lam.Distribution.Block if os.environ["LMR_DIST"] == "block" else lam.Distribution.Cyclic
rng = np.random.default_rng(5100 + me)
arr = lam.AtomicArray(world.team(), n_len, dist, dt)
k = world.team().kernels
info = np.iinfo(npt)
def vals(n):
    return rng.integers(info.min, info.max, n, dtype=np.int64, endpoint=True).astype(npt)
out = {}
k.profile(True)
k.profile_read(reset=True)
gi = rng.integers(0, n_len, 400000 - 3331 * me).astype(np.uint64)
gv = vals(gi.size)
arr.batch_add(gi, gv).block(); world.barrier()
xi = rng.integers(0, n_len, 300000).astype(np.uint64)
xv = vals(xi.size)
arr.batch_bit_xor(xi, xv).block(); world.barrier()
mi = rng.integers(0, n_len, 200000).astype(np.uint64)
mv = vals(mi.size)
arr.batch_mul(mi, mv).block(); world.barrier()
st = k.profile_read(reset=True)
out["coarse"] = np.array([st.get("bin_scatter", (0, 0))[1]])
out["fine"] = np.array([st.get("fine_scatter", (0, 0))[1]])
# skewed: every record onto 4096 elements (one owner's first bucket), one scalar value
si = rng.integers(0, 4096, 300000).astype(np.uint64)
arr.batch_add(si, 3).block(); world.barrier()
out["final"] = arr.to_numpy()
out["gi"], out["gv"], out["xi"], out["xv"], out["si"] = gi, gv, xi, xv, si
out["mi"], out["mv"] = mi, mv
np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), **out)
world.barrier()
'''

# elements per 64 KiB tile
_TILE = {"i8": 65536, "u8": 65536, "i16": 32768, "u16": 32768, "u32": 16384, "i32": 16384, "i64": 8192, "u64": 8192}
_NP = {"i8": np.int8, "u8": np.uint8, "i16": np.int16, "u16": np.uint16, "u32": np.uint32, "i32": np.int32,
       "i64": np.int64, "u64": np.uint64}


def _run(ws, dt, dist, outdir, transport="peer"):
    per_pe = 129 * _TILE[dt] + 7          # > 128 tiles per PE: a count-free owner session
    env = dict(os.environ, LMR_ROOT=ROOT, LMR_OUT=outdir, LMR_LEN=str(per_pe * ws), LMR_DT=dt, LMR_DIST=dist,
               LAMELLAR_COMM_BACKEND="gloo", LAMELLAR_TRANSPORT=transport, LAMELLAR_EXCHANGE_BUCKETS="1",
               LAMELLAR_PEER_TIMEOUT="60", LAMELLAR_EXCHANGE_CHUNK=str(1 << 18),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + 13 * ws + (os.getpid() % 50)))
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
    return per_pe * ws, [dict(np.load(os.path.join(outdir, f"pe{r}.npz"))) for r in range(ws)]


@pytest.mark.parametrize("ws,dt,dist,transport",
                         [(2, "i8", "block", "peer"), (2, "u16", "cyclic", "peer"), (2, "u32", "block", "peer"),
                          (2, "i64", "cyclic", "peer"), (3, "u32", "cyclic", "peer"), (2, "i8", "cyclic", ""),
                          (3, "u32", "block", "")],
                         ids=["i8-block-2pe", "u16-cyclic-2pe", "u32-block-2pe", "i64-cyclic-2pe", "u32-cyclic-3pe",
                              "collective-i8-cyclic-2pe", "collective-u32-block-3pe"])
def test_bucketed_push_types_and_layouts(ws, dt, dist, transport):
    """transport "": the bucketed regions over the collective (host-buffer gloo) transport."""
    with tempfile.TemporaryDirectory() as d:
        n_len, pe = _run(ws, dt, dist, d, transport)
    t = _NP[dt]
    a = np.zeros(n_len, t)
    with np.errstate(over="ignore"):
        for r in range(ws):
            np.add.at(a, pe[r]["gi"].astype(np.int64), pe[r]["gv"].astype(t))
        for r in range(ws):
            np.bitwise_xor.at(a, pe[r]["xi"].astype(np.int64), pe[r]["xv"].astype(t))
        for r in range(ws):
            np.multiply.at(a, pe[r]["mi"].astype(np.int64), pe[r]["mv"].astype(t))
        for r in range(ws):
            np.add.at(a, pe[r]["si"].astype(np.int64), t(3))
    for r in range(ws):
        assert np.array_equal(pe[r]["final"].view(t), a), r
        assert int(pe[r]["coarse"][0]) == 0, ("owner coarse pass ran", r, int(pe[r]["coarse"][0]))
        assert int(pe[r]["fine"][0]) > 0, r
