# check after the coarse-block default change: parity + all single-GPU configs (GPU box)
mkdir -p gpurun_out/g && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g/tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/g/tests.log; tools/gpu_steps.sh \
  "200|g/c2.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|g/c3.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|g/c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|g/c5_g256.log|LMR_BIN_BLOCKS=256 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|g/c4_force.log|LAMELLAR_FORCE_EXCHANGE=1 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline"
