#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r3c
steps=()
for cfg in "4 65536" "2 32768" "2 16384" "1 16384" "1 8192" "4 65536"; do
  set -- $cfg
  steps+=("200|r3c/c3_$1_$2.log|LMR_DELTA_MUL=$1 LMR_DELTA_MIN=$2 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline")
done
tools/gpu_steps.sh "${steps[@]}"
