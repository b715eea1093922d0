#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_window.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r2j.log 2>&1
rc=$?
tail -40 gpurun_out/r2j.log
exit $rc
