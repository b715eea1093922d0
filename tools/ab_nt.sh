# A/B: 1024-thread partition blocks (one per CU) vs 512-thread blocks (two per CU), same box
mkdir -p gpurun_out/nt && export TMPDIR=/tmp && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "two_level or hot_tile or out_of_bounds" > gpurun_out/nt/tests.log 2>&1; echo "pytest(1024) rc=$?"; tail -1 gpurun_out/nt/tests.log; LMR_PART_NT=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "two_level or hot_tile or out_of_bounds" > gpurun_out/nt/tests512.log 2>&1; echo "pytest(512) rc=$?"; tail -1 gpurun_out/nt/tests512.log; tools/gpu_steps.sh \
  "200|nt/a1024.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|nt/a512.log|LMR_PART_NT=512 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|nt/a512f12.log|LMR_PART_NT=512 LMR_FINE_RPT=12 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|nt/b1024.log|python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|nt/b512.log|LMR_PART_NT=512 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|nt/b512f12.log|LMR_PART_NT=512 LMR_FINE_RPT=12 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|nt/c3_1024.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|nt/c3_512.log|LMR_PART_NT=512 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline"
