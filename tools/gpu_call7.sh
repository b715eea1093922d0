#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r3b
tools/gpu_steps.sh \
  "200|r3b/c3.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r3b/c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r3b/c3b.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r3b/c5b.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "600|r3b/tests.log|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stage_mixed.py tests/test_gpu_linearize.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
