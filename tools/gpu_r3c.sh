#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3c; mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "400|$T/tests.log|python -u -m pytest tests/test_gpu_stage_mixed.py tests/test_gpu_linearize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || exit 1
tools/gpu_steps.sh \
  "400|$T/ab_c5_split.log|bash tools/ab_env.sh c5 2 LMR_CCOUNT_SPLIT=1 LMR_CCOUNT_SPLIT=2 LMR_CCOUNT_SPLIT=4 LMR_CCOUNT_SPLIT=8" \
  "400|$T/ab_c3_split.log|bash tools/ab_env.sh c3 2 LMR_CCOUNT_SPLIT=1 LMR_CCOUNT_SPLIT=4" \
  "400|$T/ab_c5_unpart.log|bash tools/ab_env.sh c5 2 LMR_UNPART_U=16 LMR_UNPART_U=8 LMR_UNPART_U=4 LMR_UNPART_SUB=4096 LMR_UNPART_SUB=16384" \
  "400|$T/ab_c3_unpart.log|bash tools/ab_env.sh c3 2 LMR_UNPART_U=4 LMR_UNPART_U=8 LMR_UNPART_SUB=2048 LMR_UNPART_SUB=8192"
