#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=r3d; mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "400|$T/tests.log|python -u -m pytest tests/test_gpu_stage_mixed.py tests/test_gpu_linearize.py tests/test_gpu_dist_ordered.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || exit 1
tools/gpu_steps.sh \
  "400|$T/ab_c5_priv.log|bash tools/ab_env.sh c5 2 LMR_CCOUNT_PRIV=0 LMR_CCOUNT_PRIV=1 'LMR_CCOUNT_PRIV=1 LMR_CCOUNT_SPLIT=1' 'LMR_CCOUNT_PRIV=1 LMR_UNPART_U=8'" \
  "400|$T/ab_c3_priv.log|bash tools/ab_env.sh c3 2 LMR_CCOUNT_PRIV=0 LMR_CCOUNT_PRIV=1" \
  "300|$T/pmc_fetch_c5.log|rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/$T/pmc_c5_fetch -o run -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-verify" \
  "300|$T/pmc_write_c5.log|rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/$T/pmc_c5_write -o run -- python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-verify"
