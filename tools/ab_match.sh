# A/B: LDS ranking by wave key matching (LMR_MATCH_RANK=1) vs per-record LDS atomics, plus
# the pack microbenchmark and the C4 one-rank rehearsal (GPU box, repo root; logs in gpurun_out/abm)
mkdir -p gpurun_out/abm && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abm/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/abm/gpu_tests.log; tools/gpu_steps.sh \
  "200|abm/packbench.log|python tools/packbench.py" \
  "200|abm/c2_a.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|abm/c2_m.log|LMR_MATCH_RANK=1 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|abm/c2_a2.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|abm/c2_m2.log|LMR_MATCH_RANK=1 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|abm/c5_a.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|abm/c5_m.log|LMR_MATCH_RANK=1 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|abm/c4_force.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline"
