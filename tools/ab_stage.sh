# staged-path check: parity + multi-PE tests, C4 one-rank rehearsal, staged C2 (GPU box, repo root)
mkdir -p gpurun_out/st && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/st/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/st/gpu_tests.log; tools/gpu_steps.sh \
  "200|st/c4_force.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline" \
  "200|st/c2_staged.log|LMR_STAGED=1 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|st/c2_staged4.log|LMR_STAGED=1 LMR_STAGE_SPLIT=4 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|st/c2.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline"
