# quick check after a kernel change: parity subset + C2/C3/C5 benches (GPU box, repo root)
mkdir -p gpurun_out/q && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/q/gpu_tests.log; tools/gpu_steps.sh \
  "200|q/c2.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|q/c3.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|q/c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|q/c4_force.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline" \
  "200|q/c4_force25.log|LAMELLAR_FORCE_EXCHANGE=1 LAMELLAR_EXCHANGE_CHUNK=33554432 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline"
