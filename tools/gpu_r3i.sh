#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3i; mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "300|$T/tests_stage.log|python -u -m pytest tests/test_gpu_stage_mixed.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests_stage.log && ! grep -q "failed" gpurun_out/$T/tests_stage.log || exit 1
tools/gpu_steps.sh \
  "900|$T/tests.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
tools/gpu_steps.sh \
  "400|$T/ab_c5.log|bash tools/ab_mix.sh c5 2 'tools/abl/r3f.so|' 'cur|' 'cur|LMR_STAGE_LOCAL=0'" \
  "400|$T/ab_c3.log|bash tools/ab_mix.sh c3 2 'tools/abl/r3f.so|' 'cur|' 'cur|LMR_STAGE_LOCAL=0'"
