#!/bin/bash
# window split: the new window test, then the parity + linearize suites it could disturb
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_window.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r2e_window.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2e_gpu.log 2>&1
rc=$?
tail -n 30 gpurun_out/r2e_window.log
tail -n 5 gpurun_out/r2e_gpu.log
exit $rc
