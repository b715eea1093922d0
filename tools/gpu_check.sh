#!/bin/bash
# One GPU call's check of the current tree: the full -m gpu suite and smoke(), then
# optional same-box A/B lines (tools/ab_mix.sh) against tools/abl/base.so for the
# configs named as arguments (e.g. tools/gpu_check.sh c2 c5).
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tools/gpu_steps.sh \
  "900|check_gpu.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "200|check_smoke.log|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" || exit $?
grep -q " passed" gpurun_out/check_gpu.log && ! grep -q "failed" gpurun_out/check_gpu.log || { tail -30 gpurun_out/check_gpu.log; exit 1; }
for cfg in "$@"; do
  timeout -k 10 300 bash tools/ab_mix.sh $cfg 2 "tools/abl/base.so|" "cur|" || exit $?
done
