#!/bin/bash
# kernel traces of C3 and C5 (current build) + their bench lines
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
tools/gpu_steps.sh \
  "200|r3a/c3.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|r3a/c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "300|r3a/prof_c3.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-verify" \
  "300|r3a/prof_c5.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-verify"
