#!/bin/bash
# One parametrised GPU-call recipe (run on the GPU box from the repo root). Every GPU step runs
# under its own time limit through tools/gpu_steps.sh; a fault / abort / timeout stops the call.
# usage: tools/gpu_round.sh <mode> <tag> [args...]      (outputs under gpurun_out/<tag>/)
#   check   <tag> [pytest selection]   the -m gpu suite (default: all of tests/) and smoke()
#   bench   <tag> <cfg>...             bench lines (c4 = one-rank rehearsal, forced exchange)
#   prof    <tag> <cfg>...             rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes
#   ab      <tag> <cfg> <reps> <spec>...  same-box A/B (tools/ab_mix.sh specs "<lib>|<env>[|<bench args>]")
#   default <tag>                      the default bench line (N = 1, with its CPU baselines)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mode=$1; T=$2; shift 2
O=gpurun_out/$T; mkdir -p $O
env_for() { [ "$1" = c4 ] && echo "LAMELLAR_FORCE_EXCHANGE=1 " || echo ""; }
case $mode in
check)
  sel=${*:-tests}
  tools/gpu_steps.sh \
    "1000|$T/tests.log|python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
    "200|$T/smoke.log|python -c 'import __graft_entry__ as g; g.smoke()'" || exit $?
  grep -q " passed" $O/tests.log && ! grep -q "failed" $O/tests.log || exit 1 ;;
bench)
  steps=()
  for cfg in "$@"; do
    n=20; [ "$cfg" = c4 ] && n=10
    steps+=("240|$T/$cfg.log|$(env_for $cfg)python bench.py --config $cfg --steps $n --warmup 5 --no-cpu-baseline")
  done
  tools/gpu_steps.sh "${steps[@]}" ;;
prof)
  steps=()
  for cfg in "$@"; do
    e=$(env_for $cfg); a="python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify"
    steps+=("300|$T/prof_$cfg.log|${e}rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_$cfg/trace -o run -- $a")
    [ "$cfg" = c4 ] && continue
    steps+=("300|$T/pmcf_$cfg.log|rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_fetch -o run -- $a")
    steps+=("300|$T/pmcw_$cfg.log|rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/prof_$cfg/pmc_write -o run -- $a")
  done
  tools/gpu_steps.sh "${steps[@]}" ;;
ab)
  cfg=$1; reps=$2; shift 2
  timeout -k 10 900 bash tools/ab_mix.sh $cfg $reps "$@" > $O/ab_$cfg.log 2>&1; rc=$?
  cat $O/ab_$cfg.log; exit $rc ;;
default)
  tools/gpu_steps.sh "500|$T/default.log|python bench.py" ;;
*) echo "unknown mode $mode"; exit 2 ;;
esac
