#!/bin/bash
# rocprofv3 evidence for the bench's kernels (run on the GPU box from the repo root):
#   1) --kernel-trace --stats (per-kernel durations)
#   2) --pmc FETCH_SIZE and 3) --pmc WRITE_SIZE in separate passes (gfx950 TCC slots)
# usage: tools/profile.sh <outdir> [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/prof}; shift
ARGS=${@:---steps 5 --warmup 2 --no-cpu-baseline}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run \
    -- python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/pmc_fetch" -o run \
    -- python3 bench.py $ARGS --no-verify > "$OUT/bench_fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/pmc_write" -o run \
    -- python3 bench.py $ARGS --no-verify > "$OUT/bench_write.log" 2>&1 || exit $?
find "$OUT" -name "*.csv" | head -20
