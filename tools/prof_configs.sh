#!/bin/bash
# rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the C3 and C5 bench lines
# (outputs under gpurun_out/<tag>/prof_<cfg>/); each GPU step under its own time limit.
tag=${1:-r2}
O=gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
steps=()
for cfg in c3 c5; do
  steps+=("300|$tag/prof_$cfg.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_$cfg/trace -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline")
  steps+=("300|$tag/pmc_fetch_$cfg.log|rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_fetch -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
  steps+=("300|$tag/pmc_write_$cfg.log|rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_write -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
done
tools/gpu_steps.sh "${steps[@]}"
