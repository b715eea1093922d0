#!/bin/bash
# Kernel traces of C3 and C5 on the final round-3 build (round-wise un-partition kernels).
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3u; O=gpurun_out/$T; mkdir -p $O
tools/gpu_steps.sh \
  "240|$T/prof_c3.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_c3/trace -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-verify" \
  "240|$T/prof_c5.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_c5/trace -o run -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-verify"
