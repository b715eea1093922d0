#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tools/gpu_steps.sh \
  "300|r2w_mixed.log|python -u -m pytest tests/test_gpu_stage_mixed.py -x -v --timeout 120 --timeout-method thread" || exit $?
grep -q "passed" gpurun_out/r2w_mixed.log && ! grep -q "failed" gpurun_out/r2w_mixed.log || { tail -40 gpurun_out/r2w_mixed.log; exit 1; }
timeout -k 10 600 bash tools/ab_mix.sh c5 2 "cur|LAMELLAR_DEFER=0" "cur|"
timeout -k 10 600 bash tools/ab_mix.sh c2 2 "cur|LAMELLAR_DEFER=0" "cur|"
