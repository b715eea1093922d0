#!/bin/bash
# exchange behind the C ABI: multi-PE GPU tests, then the whole GPU suite, then a forced-exchange bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2d_dist.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2d_gpu.log 2>&1 &&
LAMELLAR_FORCE_EXCHANGE=1 LAMELLAR_COMM_BACKEND=nccl timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2d_bench_x.log 2>&1
rc=$?
tail -5 gpurun_out/r2d_dist.log gpurun_out/r2d_gpu.log
tail -c 1500 gpurun_out/r2d_bench_x.log
exit $rc
