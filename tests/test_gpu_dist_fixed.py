"""Fixed-region mode of lmr_batch_exchange (ops that return nothing, count-free pack and
count-free staging on every PE): each destination's fixed region goes whole, the owner stages
it with its record count read on the device from the chunk's header rows, and the host reads no
header after chunk 0. Records past a region (a skewed batch) travel in the overflow round after
the last chunk. PEs share the GPU over gloo (host-buffer transport), or one rank drives the
1-rank RCCL communicator (LAMELLAR_FORCE_EXCHANGE=1); shards of > 128 tiles per PE so the owner's
session is count-free. Every final state is checked against numpy's serial replay (wrapping
u64 sums commute), and LAMELLAR_EXCHANGE_FIXED=0 (the host reads every chunk's rows) must
give the same arrays."""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

PER_PE = (1 << 21) + 5           # u64 elements per PE: 257 tiles of 8192

WORKER = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
world = lam.LamellarWorldBuilder().build()
me, ws = world.my_pe(), world.num_pes()
n_len = int(os.environ["LMR_LEN"])
rng = np.random.default_rng(1300 + me)
arr = lam.AtomicArray(world.team(), n_len, lam.Distribution.Block, "u64")
out = {}
# ragged batches: each PE its own record count, several chunks (the last one partial)
n1 = (1 << 20) - 4321 * me
gi = rng.integers(0, n_len, n1).astype(np.uint64)
gv = rng.integers(0, 2**63, n1, dtype=np.uint64)
arr.batch_add(gi, gv).block(); world.barrier()
out["after_add"] = arr.to_numpy()
# skewed: every record into the first PE's first 2^20 elements -- its regions overflow, the
# rest go in the overflow round -- with one scalar value (no values on the wire)
si = rng.integers(0, 1 << 20, 600000).astype(np.uint64)
arr.batch_add(si, 3).block(); world.barrier()
out["after_skew_add"] = arr.to_numpy()
arr.batch_sub(si, 3).block(); world.barrier()
out["after_skew_sub"] = arr.to_numpy()
# xor with array values, then an empty batch on PE 0 only
xi = rng.integers(0, n_len, 300000).astype(np.uint64)
xv = rng.integers(0, 2**63, xi.size, dtype=np.uint64)
arr.batch_bit_xor(xi, xv).block(); world.barrier()
out["after_xor"] = arr.to_numpy()
ei = np.zeros(0, np.uint64) if me == 0 else rng.integers(0, n_len, 200000).astype(np.uint64)
arr.batch_add(ei, 1).block(); world.barrier()
out["after_empty"] = arr.to_numpy()
out["gi"], out["gv"], out["si"], out["xi"], out["xv"], out["ei"] = gi, gv, si, xi, xv, ei
tp = world.team().transport()
out["peer_stats"] = np.array(tp.stats() if hasattr(tp, "stats") else (-1, -1))
np.savez(os.path.join(os.environ["LMR_OUT"], f"pe{me}.npz"), **out)
world.barrier()
'''


def _run(ws, env_extra, outdir):
    env = dict(os.environ)
    env.update(env_extra)
    env.update(LMR_ROOT=ROOT, LMR_OUT=outdir, LMR_LEN=str(PER_PE * ws), LAMELLAR_EXCHANGE_CHUNK=str(1 << 18),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29900 + 7 * ws + (os.getpid() % 50)))
    procs = [subprocess.Popen([sys.executable, "-c", WORKER],
                              env=dict(env, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK=str(r)))
             for r in range(ws)]
    assert [p.wait(timeout=300) for p in procs] == [0] * ws
    return [dict(np.load(os.path.join(outdir, f"pe{r}.npz"))) for r in range(ws)]


def _expected(pe, n_len):
    ws = len(pe)
    a = np.zeros(n_len, np.uint64)
    for r in range(ws):
        np.add.at(a, pe[r]["gi"].astype(np.int64), pe[r]["gv"])
    steps = {"after_add": a.copy()}
    for r in range(ws):
        np.add.at(a, pe[r]["si"].astype(np.int64), np.uint64(3))
    steps["after_skew_add"] = a.copy()
    for r in range(ws):
        np.subtract.at(a, pe[r]["si"].astype(np.int64), np.uint64(3))
    steps["after_skew_sub"] = a.copy()
    for r in range(ws):
        np.bitwise_xor.at(a, pe[r]["xi"].astype(np.int64), pe[r]["xv"])
    steps["after_xor"] = a.copy()
    for r in range(ws):
        np.add.at(a, pe[r]["ei"].astype(np.int64), np.uint64(1))
    steps["after_empty"] = a.copy()
    return steps


@pytest.mark.parametrize("ws,backend,fixed,transport",
                         [(1, "nccl", "1", ""), (2, "gloo", "1", ""), (3, "gloo", "1", ""), (2, "gloo", "0", ""),
                          (1, "nccl", "1", "peer"), (2, "gloo", "1", "peer"), (3, "gloo", "1", "peer"),
                          (1, "nccl", "1", "peer-buckets"), (2, "gloo", "1", "peer-buckets"),
                          (3, "gloo", "1", "peer-buckets"), (1, "nccl", "1", "rb"), (2, "gloo", "1", "rb"),
                          (3, "gloo", "1", "rb")],
                         ids=["rccl-1rank", "gloo-2pe", "gloo-3pe", "gloo-2pe-hostcounts",
                              "peer-1rank", "peer-2pe", "peer-3pe", "buckets-1rank", "buckets-2pe", "buckets-3pe",
                              "rb-rccl-1rank", "rb-gloo-2pe", "rb-gloo-3pe"])
def test_fixed_region_exchange(ws, backend, fixed, transport):
    """transport=peer: lmr_transport_peer_create over the base transport -- every batch here is
    pushed (the sender's pack writes into the owners' IPC-mapped regions; counts and sequence
    numbers through the /dev/shm mailbox), the skewed batch's overflow round uses the base.
    peer-buckets: the push's bucketed mode (LAMELLAR_EXCHANGE_BUCKETS=1: the sender packs by
    (owner, owner bucket of 128 tiles) into bucket slices, the owner bins them straight into its
    session's tile regions); the skewed batch overflows its slices (overflow round, applied with
    device atomics). rb: the same bucketed regions over the collective transport (RCCL / gloo):
    sent whole by the all-to-all-v, binned by the owner without a coarse pass."""
    buckets = transport in ("peer-buckets", "rb")
    if transport == "peer-buckets":
        transport = "peer"
    elif transport == "rb":
        transport = ""
    env = {"LAMELLAR_COMM_BACKEND": backend, "LAMELLAR_EXCHANGE_FIXED": fixed, "LAMELLAR_TRANSPORT": transport,
           "LAMELLAR_PEER_TIMEOUT": "60", "LAMELLAR_EXCHANGE_BUCKETS": "1" if buckets else "0"}
    if ws == 1:
        env["LAMELLAR_FORCE_EXCHANGE"] = "1"
    with tempfile.TemporaryDirectory() as d:
        pe = _run(ws, env, d)
    exp = _expected(pe, PER_PE * ws)
    for key, want in exp.items():
        for r in range(ws):
            assert np.array_equal(pe[r][key], want), (key, r)
    if transport == "peer":
        for r in range(ws):
            batches, pushed = (int(v) for v in pe[r]["peer_stats"])
            assert batches == 5, batches                   # every batch handshaken
            assert pushed == 4 + 3 + 3 + 2 + 1, pushed     # and pushed, chunk by chunk (2^18-record chunks)
