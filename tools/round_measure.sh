#!/bin/bash
# Round-end evidence (run from the repo root on the GPU box), in two GPU calls:
#   part 1: benches of every config;  part 2: the C2 rocprofv3 kernel trace, separate
#   FETCH_SIZE / WRITE_SIZE PMC passes, and the default bench line with its CPU baselines.
# Every GPU step has its own time limit; a fault / abort / timeout stops the sequence
# (tools/gpu_steps.sh).
# usage: tools/round_measure.sh <tag> <1|2>      (outputs under gpurun_out/<tag>/)
tag=${1:-r2}
part=${2:-1}
O=gpurun_out/$tag
mkdir -p $O
export TMPDIR=/tmp
if [ "$part" = 1 ]; then
tools/gpu_steps.sh \
  "200|$tag/c2.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|$tag/c3.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|$tag/c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|$tag/c2_direct.log|python bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline --strategy direct" \
  "200|$tag/c4_force.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline" \
  "300|$tag/e2e.log|python bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --e2e"
else
tools/gpu_steps.sh \
  "300|$tag/prof_c2.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_c2/trace -o run -- python3 bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline" \
  "300|$tag/pmc_fetch_c2.log|rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/prof_c2/pmc_fetch -o run -- python3 bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline --no-verify" \
  "300|$tag/pmc_write_c2.log|rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/prof_c2/pmc_write -o run -- python3 bench.py --config c2 --steps 5 --warmup 2 --no-cpu-baseline --no-verify" \
  "500|$tag/default.log|python bench.py"
fi
