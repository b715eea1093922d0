#!/bin/bash
# Round 3: the full -m gpu suite + smoke on the current build, then bench lines of every config.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r3
tools/gpu_steps.sh \
  "300|r3/check_stage.log|python -u -m pytest tests/test_gpu_stage_mixed.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/r3/check_stage.log && ! grep -q "failed" gpurun_out/r3/check_stage.log || exit 1
tools/gpu_steps.sh \
  "900|r3/check_gpu.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "200|r3/check_smoke.log|python -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
tools/round_measure.sh r3 1
