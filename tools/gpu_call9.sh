#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
tools/gpu_steps.sh \
  "300|r3d/prof_c4f.log|rocprofv3 --kernel-trace -T --output-format csv -d $O/prof_c4f -o run -- python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-verify" 
