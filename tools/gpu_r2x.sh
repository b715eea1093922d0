#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tools/gpu_steps.sh \
  "900|r2x_gpu.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "200|r2x_smoke.log|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "200|r2x_c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r2x_c2.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline"
