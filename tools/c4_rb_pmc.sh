#!/bin/bash
# C4 one-rank RCCL rehearsal with bucketed regions (the default): kernel trace, then separate
# FETCH_SIZE and WRITE_SIZE passes (one counter group per run), each step under its own time limit.
# usage (GPU box): tools/c4_rb_pmc.sh <tag>      outputs under gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp LAMELLAR_FORCE_EXCHANGE=1
T=$1; O=gpurun_out/$T; mkdir -p $O
a="python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-verify"
tools/gpu_steps.sh \
  "300|$T/c4_trace.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/c4/trace -o run -- $a" \
  "120|$T/c4_fetch.log|timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/c4/pmc_fetch -o run -- $a" \
  "120|$T/c4_write.log|timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/c4/pmc_write -o run -- $a"
