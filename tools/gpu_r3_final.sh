#!/bin/bash
# Round-3 check of the current build: the full -m gpu suite, smoke(), bench lines of every config
# and the default bench line (N = 1 with its CPU baselines).
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r3final}; O=gpurun_out/$T; mkdir -p $O
tools/gpu_steps.sh \
  "900|$T/tests.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "200|$T/smoke.log|python -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
grep -q " passed" $O/tests.log && ! grep -q "failed" $O/tests.log || exit 1
tools/round_measure.sh $T 1 || exit $?
tools/gpu_steps.sh "500|$T/default.log|python bench.py"
