#!/bin/bash
# Round 3: staged/parity/linearize suites on the current build, then kernel traces of C2/C3/C5
# and their bench lines.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r3b}
mkdir -p gpurun_out/$T
tools/gpu_steps.sh \
  "600|$T/tests.log|python -u -m pytest tests/test_gpu_stage_mixed.py tests/test_gpu_parity.py tests/test_gpu_linearize.py tests/test_gpu_dist.py tests/test_gpu_dist_ordered.py tests/test_gpu_window.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit $?
grep -q " passed" gpurun_out/$T/tests.log && ! grep -q "failed" gpurun_out/$T/tests.log || exit 1
steps=()
for cfg in c5 c3 c2; do
  steps+=("200|$T/$cfg.log|python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline")
  steps+=("300|$T/prof_$cfg.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/$T/prof_$cfg -o run -- python3 bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-verify")
done
tools/gpu_steps.sh "${steps[@]}"
