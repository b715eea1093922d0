#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3e; mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "300|$T/tests_stage.log|python -u -m pytest tests/test_gpu_stage_mixed.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests_stage.log && ! grep -q "failed" gpurun_out/$T/tests_stage.log || exit 1
tools/gpu_steps.sh \
  "900|$T/tests.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
tools/gpu_steps.sh \
  "400|$T/ab_c5.log|bash tools/ab_mix.sh c5 2 'tools/abl/base.so|LMR_CCOUNT_PRIV=0' 'cur|' 'cur|LMR_UNPART_U=8'" \
  "400|$T/ab_c3.log|bash tools/ab_mix.sh c3 2 'tools/abl/base.so|LMR_CCOUNT_PRIV=0' 'cur|' 'cur|LMR_UNPART_U=8'" \
  "400|$T/ab_c2.log|bash tools/ab_mix.sh c2 3 'tools/abl/base.so|' 'cur|'" \
  "400|$T/ab_c4.log|bash tools/ab_mix.sh c4 2 'tools/abl/base.so|' 'cur|'"
