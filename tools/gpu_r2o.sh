#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2o.log 2>&1 || { tail -30 gpurun_out/r2o.log; exit 1; }
tail -2 gpurun_out/r2o.log
timeout -k 10 600 bash tools/ab_mix.sh c5 2 "tools/abl/base.so|" "cur|"
