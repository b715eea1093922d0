"""Debug driver: the test_gpu_dist WORKER steps with LAMELLAR_TRANSPORT=peer, printing each
step and dumping every thread's stack after 40 s (faulthandler)."""
import faulthandler
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
W = r'''
import faulthandler, os, sys, time
faulthandler.dump_traceback_later(30, exit=True)
import numpy as np
sys.path.insert(0, os.environ["LMR_ROOT"])
from _lamellar_bootstrap import load_package
lam = load_package()
world = lam.LamellarWorldBuilder().build()
me, ws = world.my_pe(), world.num_pes()
def say(*a): print(f"[pe{me} {time.time():.3f}]", *a, flush=True)
rng = np.random.default_rng(500 + me)
n_len = 40009
arr = lam.AtomicArray(world.team(), n_len, 0, "u64")
say("transport", type(world.team().transport()).__name__)
gi = rng.integers(0, n_len, 200000).astype(np.uint64)
gv = rng.integers(0, 2**40, gi.size).astype(np.uint64)
arr.batch_add(gi, gv).block(); say("add done"); world.barrier()
si = rng.integers(0, n_len // 4, 150000).astype(np.uint64)
arr.batch_add(si, 3).block(); say("skew add done"); world.barrier()
fi = rng.permutation(n_len)[:20000].astype(np.uint64)
olds = arr.batch_fetch_add(fi, 7).block(); say("fetch done"); world.barrier()
arr.batch_add(5, np.arange(1, 11, dtype=np.uint64)).block(); say("mvsi done"); world.barrier()
say("all done")
'''
for i, recs in enumerate(sys.argv[1:]):
    env = dict(os.environ, LMR_ROOT=ROOT, LAMELLAR_COMM_BACKEND="gloo", LAMELLAR_TRANSPORT="peer",
               LAMELLAR_PEER_TIMEOUT="15", LMR_PEER_DEBUG="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29655 + i),
               LAMELLAR_PEER_REGION_RECORDS=recs)
    procs = [subprocess.Popen([sys.executable, "-u", "-c", W], env=dict(env, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r)))
             for r in range(2)]
    print("region records", recs, "rcs", [p.wait(timeout=200) for p in procs], flush=True)
