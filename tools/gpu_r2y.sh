#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_linearize.py -x -q --timeout 300 --timeout-method thread -k "dist or exchange or pe" > gpurun_out/r2y.log 2>&1 || { tail -40 gpurun_out/r2y.log; exit 1; }
LAMELLAR_EXCHANGE_SELF=transport timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/r2y.log 2>&1 || { tail -40 gpurun_out/r2y.log; exit 1; }
grep -E "passed|failed" gpurun_out/r2y.log
