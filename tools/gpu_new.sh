#!/bin/bash
# Run the named -m gpu test files (default: the round-3 additions) and one default bench line.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
files=${FILES:-"tests/test_gpu_float_specials.py tests/test_gpu_dist_ordered.py"}
tools/gpu_steps.sh \
  "600|new_tests.log|python -u -m pytest $files -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "200|bench_default.log|python bench.py --steps 20 --warmup 5"
