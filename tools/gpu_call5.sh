#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/c5x
tools/gpu_steps.sh \
  "200|c5x/pack_v1.log|LMR_PACK_V2=0 python tools/packbench.py --reps 10" \
  "200|c5x/pack_v2.log|python tools/packbench.py --reps 10" \
  "200|c5x/c4f_v1.log|LMR_PACK_V2=0 LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline" \
  "200|c5x/c4f_v2.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline" \
  "600|c5x/tests.log|python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_dist_ordered.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider"
