# automatic piece-partition selection: parity + benches (GPU box, repo root)
mkdir -p gpurun_out/au && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/au/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/au/gpu_tests.log; tools/gpu_steps.sh \
  "200|au/c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|au/c5_seg.log|LMR_STAGED=0 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|au/c3.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|au/c3_st.log|LMR_STAGED=1 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|au/c2.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline"
