#!/bin/bash
# full -m gpu suite + smoke on the current tree
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tools/gpu_steps.sh \
  "900|r2v_gpu.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "200|r2v_smoke.log|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
