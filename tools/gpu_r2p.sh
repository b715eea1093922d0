#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_linearize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2p.log 2>&1 || { tail -30 gpurun_out/r2p.log; exit 1; }
tail -2 gpurun_out/r2p.log
timeout -k 10 600 bash tools/ab_mix.sh c5 1 "cur|" && timeout -k 10 600 bash tools/ab_mix.sh c3 1 "cur|"
