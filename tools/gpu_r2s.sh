#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2s
LAMELLAR_FORCE_EXCHANGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r2s/prof_c4 -o run -- python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-verify > gpurun_out/r2s/prof_c4.log 2>&1
echo rc=$?
tail -c 600 gpurun_out/r2s/prof_c4.log
