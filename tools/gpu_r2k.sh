#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_programs.py tests/test_gpu_wire.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2k.log 2>&1
rc=$?
tail -15 gpurun_out/r2k.log
exit $rc
