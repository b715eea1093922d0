#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r3e
steps=()
for i in 1 2 3; do
  steps+=("200|r3e/c2_i0_$i.log|LMR_IDX3=0 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-verify")
  steps+=("200|r3e/c2_i1_$i.log|LMR_IDX3=1 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline")
done
steps+=("600|r3e/tests.log|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stage_mixed.py tests/test_gpu_dist.py tests/test_gpu_window.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider")
tools/gpu_steps.sh "${steps[@]}"
