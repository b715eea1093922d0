# fine pass over merged segment ranges: full GPU suite + C2 / C3 benches (GPU box)
mkdir -p gpurun_out/mg && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mg/tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/mg/tests.log; tools/gpu_steps.sh \
  "200|mg/c2.log|python bench.py --config c2 --steps 20 --warmup 10 --no-cpu-baseline" \
  "200|mg/c3.log|python bench.py --config c3 --steps 20 --warmup 10 --no-cpu-baseline" \
  "200|mg/c2b.log|python bench.py --config c2 --steps 20 --warmup 10 --no-cpu-baseline"
