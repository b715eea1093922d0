#!/bin/bash
# next8 (u16 round staging positions for the round-wise un-partition): staged-path GPU tests on
# that build, then same-box A/B against the in-tree build on C5 and C3.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3t; mkdir -p gpurun_out/$T
L=tools/abl/next8.so
tools/gpu_steps.sh \
  "600|$T/tests.log|LAMELLAR_GPU_OPS_LIB=$PWD/$L python -u -m pytest tests/test_gpu_stage_mixed.py tests/test_gpu_linearize.py tests/test_gpu_scan_sizes.py tests/test_gpu_dist_ordered.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || exit 1
tools/gpu_steps.sh \
  "300|$T/ab_c5.log|bash tools/ab_mix.sh c5 2 'cur|' '$L|'" \
  "300|$T/ab_c3.log|bash tools/ab_mix.sh c3 2 'cur|' '$L|'"
