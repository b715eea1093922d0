"""The reference's integration-test payloads at 2, 3 and 4 PEs through the device exchange.

tests/add.rs:24-47 (and every other op's .rs) runs each payload at 2, 3 and 4 PEs through
lamellar_run.sh. Here every PE is a process on the box's one GPU exchanging over gloo
(lmr_batch_exchange with real kernels), every PE issues its own part of the payload, and every
PE checks the payload's known answer on the global array (tests/refprog_worker.py): add (with
the sub-array form), sub, mul, div for every element type, xor / or / and for the integer ones;
AtomicArray for every type, LocalLockArray and UnsafeArray for u32 and f64; Block and Cyclic.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "refprog_worker.py")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ws,dist_kind", [(2, 0), (3, 1), (4, 0)], ids=["2pe-Block", "3pe-Cyclic", "4pe-Block"])
def test_reference_payloads_multi_pe(ws, dist_kind):
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, LMR_ROOT=ROOT, LMR_OUT=d, LMR_DIST=str(dist_kind), LAMELLAR_COMM_BACKEND="gloo",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + 10 * ws + dist_kind))
        procs = [subprocess.Popen([sys.executable, "-u", WORKER],
                                  env=dict(env, RANK=str(r), WORLD_SIZE=str(ws), LOCAL_RANK=str(r)))
                 for r in range(ws)]
        try:
            rcs = [p.wait(timeout=170) for p in procs]
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        assert rcs == [0] * ws, rcs
        for r in range(ws):
            z = np.load(os.path.join(d, f"pe{r}.npz"))
            assert int(z["checks"][0]) > 100
            assert z["fails"].size == 0, list(z["fails"])[:10]
