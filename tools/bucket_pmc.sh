#!/bin/bash
# tools/bucket_bench under rocprofv3: kernel trace, SQ stall counters, FETCH_SIZE and WRITE_SIZE
# (one counter group per run, each under its own time limit). Outputs under gpurun_out/<tag>/.
# usage (GPU box): tools/bucket_pmc.sh <tag>
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=$1; O=gpurun_out/$T; mkdir -p $O
K="--kernel-include-regex 'k_pack_bucket|k_fine_bucket|k_tile_owner'"
tools/gpu_steps.sh \
  "120|$T/run.log|timeout -k 10 100 tools/bucket_bench 6" \
  "120|$T/trace.log|timeout -k 10 100 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run -- tools/bucket_bench 4" \
  "90|$T/sq.log|timeout -s KILL 80 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -T --output-format csv -d $O/sq -o run -- tools/bucket_bench 2" \
  "90|$T/fetch.log|timeout -s KILL 80 rocprofv3 $K --pmc FETCH_SIZE -T --output-format csv -d $O/fetch -o run -- tools/bucket_bench 2" \
  "90|$T/write.log|timeout -s KILL 80 rocprofv3 $K --pmc WRITE_SIZE -T --output-format csv -d $O/write -o run -- tools/bucket_bench 2"
