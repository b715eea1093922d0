#!/bin/bash
# Round-3 evidence on the current build: bench lines of every config, kernel traces of C2/C3/C5
# and the C4 rehearsal, FETCH_SIZE / WRITE_SIZE passes of C2/C3/C5.
# usage: tools/gpu_profile_r3.sh <tag> [configs (default "c2 c3 c5 c4")]
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r3h}; O=gpurun_out/$T; mkdir -p $O
steps=()
CFGS=${2:-c2 c3 c5 c4}
for cfg in $CFGS; do
  [ "$cfg" = c4 ] && continue
  steps+=("200|$T/$cfg.log|python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline")
  steps+=("300|$T/prof_$cfg.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_$cfg/trace -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
  steps+=("300|$T/pmcf_$cfg.log|rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_fetch -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
  steps+=("300|$T/pmcw_$cfg.log|rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_write -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
done
if [[ " $CFGS " == *" c4 "* ]]; then
steps+=("200|$T/c4.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline")
steps+=("300|$T/prof_c4.log|LAMELLAR_FORCE_EXCHANGE=1 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_c4/trace -o run -- python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
fi
tools/gpu_steps.sh "${steps[@]}"
