#!/bin/bash
# C5 on the wide (one-level) path: kernel trace, SQ stall counters, FETCH_SIZE and WRITE_SIZE
# passes (one counter group per run, each under its own time limit), plus producer-chunk variants.
# usage (GPU box): [NO_TRACE=1] tools/c5_wide_pmc.sh <tag>      outputs under gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp LMR_WIDE4=1
T=$1; O=gpurun_out/$T; mkdir -p $O
a="python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-verify"
K="--kernel-include-regex 'k_wide_stage|k_unpart_wide|k_wcount_stage|k_tile_owner'"
if [ -z "$NO_TRACE" ]; then
  tools/gpu_steps.sh "200|$T/trace.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- $a" || exit $?
fi
tools/gpu_steps.sh \
  "120|$T/sq.log|timeout -s KILL 110 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES -T --output-format csv -d $O/sq -o run -- $a" \
  "120|$T/fetch.log|timeout -s KILL 110 rocprofv3 $K --pmc FETCH_SIZE -T --output-format csv -d $O/fetch -o run -- $a" \
  "120|$T/write.log|timeout -s KILL 110 rocprofv3 $K --pmc WRITE_SIZE -T --output-format csv -d $O/write -o run -- $a" \
  "120|$T/chunk256k.log|LMR_WIDE_CHUNK=262144 python3 bench.py --config c5 --no-cpu-baseline" \
  "120|$T/chunk1m.log|LMR_WIDE_CHUNK=1048576 python3 bench.py --config c5 --no-cpu-baseline" \
  "120|$T/chunk4m.log|LMR_WIDE_CHUNK=4194304 python3 bench.py --config c5 --no-cpu-baseline" \
  "120|$T/chunk64k.log|python3 bench.py --config c5 --no-cpu-baseline"
