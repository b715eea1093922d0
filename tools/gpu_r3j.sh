#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3j; mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "500|$T/tests.log|python -u -m pytest tests/test_gpu_stage_mixed.py tests/test_gpu_linearize.py tests/test_gpu_dist_ordered.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || exit 1
tools/gpu_steps.sh \
  "400|$T/ab_c5.log|bash tools/ab_mix.sh c5 2 'tools/abl/r3f.so|' 'cur|' 'cur|LMR_UNPART_PIECES=0'" \
  "400|$T/ab_c3.log|bash tools/ab_mix.sh c3 2 'tools/abl/r3f.so|' 'cur|' 'cur|LMR_UNPART_PIECES=0'"
