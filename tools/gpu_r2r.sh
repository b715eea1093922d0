#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_linearize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2r_t.log 2>&1 || { tail -20 gpurun_out/r2r_t.log; exit 1; }
LMR_FINE_CONTIG=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_linearize.py -x -q --timeout 300 --timeout-method thread >> gpurun_out/r2r_t.log 2>&1 || { tail -20 gpurun_out/r2r_t.log; exit 1; }
grep passed gpurun_out/r2r_t.log
timeout -k 10 900 bash tools/ab_mix.sh c2 2 "tools/abl/base.so|" "cur|" "cur|LMR_FINE_CONTIG=1" && timeout -k 10 600 bash tools/ab_mix.sh c3 2 "tools/abl/base.so|" "cur|" "cur|LMR_FINE_CONTIG=1" && timeout -k 10 600 bash tools/ab_mix.sh c5 1 "cur|" "cur|LMR_FINE_CONTIG=1"
