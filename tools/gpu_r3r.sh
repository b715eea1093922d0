#!/bin/bash
# next7 (round-wise un-partition gathers, bucket counts derived from tile counts in k_ccount):
# the full -m gpu suite on that build, then same-box A/B on C5 and C3.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3r; mkdir -p gpurun_out/$T
L=tools/abl/next7.so; L4=tools/abl/next4.so
tools/gpu_steps.sh \
  "900|$T/tests.log|LAMELLAR_GPU_OPS_LIB=$PWD/$L python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || exit 1
tools/gpu_steps.sh \
  "300|$T/ab_c5.log|bash tools/ab_mix.sh c5 2 'tools/abl/r3f.so|' '$L|' '$L4|'" \
  "400|$T/ab_c3.log|bash tools/ab_mix.sh c3 2 'tools/abl/r3f.so|' '$L|' '$L|LMR_UNPART_ROUNDS=7' '$L|LMR_UNPART_ROUNDS=7 LMR_COARSE_RPT=8' '$L|LMR_COARSE_RPT=8'"
