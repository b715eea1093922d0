#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2u.log 2>&1 || { tail -30 gpurun_out/r2u.log; exit 1; }
LAMELLAR_FREE_PACK=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/r2u.log 2>&1 || { tail -30 gpurun_out/r2u.log; exit 1; }
grep passed gpurun_out/r2u.log
timeout -k 10 600 bash tools/ab_mix.sh c4 2 "cur|LAMELLAR_FREE_PACK=0" "cur|"
