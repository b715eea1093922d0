#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tools/gpu_steps.sh \
  "120|l2atomic.log|./tools/l2atomic" \
  "600|new_tests.log|python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_dist.py tests/test_gpu_dist_ordered.py tests/test_gpu_ordered.py tests/test_gpu_float_specials.py tests/test_gpu_host.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider"
