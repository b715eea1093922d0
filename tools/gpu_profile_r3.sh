#!/bin/bash
# Round-3 evidence on the current build: bench lines of every config, kernel traces of C2/C3/C5
# and the C4 rehearsal, FETCH_SIZE / WRITE_SIZE passes of C2/C3/C5.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r3h}; O=gpurun_out/$T; mkdir -p $O
steps=()
for cfg in c2 c3 c5; do
  steps+=("200|$T/$cfg.log|python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline")
  steps+=("300|$T/prof_$cfg.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_$cfg/trace -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
  steps+=("300|$T/pmcf_$cfg.log|rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_fetch -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
  steps+=("300|$T/pmcw_$cfg.log|rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_write -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
done
steps+=("200|$T/c4.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline")
steps+=("300|$T/prof_c4.log|LAMELLAR_FORCE_EXCHANGE=1 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_c4/trace -o run -- python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
tools/gpu_steps.sh "${steps[@]}"
