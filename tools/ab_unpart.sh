# slot-map un-partition vs position maps (LMR_SLOT_UNPARTITION=0): parity + C3 / C5 (GPU box, repo root)
mkdir -p gpurun_out/up && export TMPDIR=/tmp && timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_programs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/up/tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/up/tests.log; tools/gpu_steps.sh \
  "200|up/c3.log|python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|up/c3_old.log|LMR_SLOT_UNPARTITION=0 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|up/c5.log|python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|up/c5_seg.log|LMR_STAGED=0 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|up/c5_seg_old.log|LMR_STAGED=0 LMR_SLOT_UNPARTITION=0 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline"
