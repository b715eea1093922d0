# pack tests + microbenchmark (GPU box, repo root)
mkdir -p gpurun_out/pack && export TMPDIR=/tmp && timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pack" > gpurun_out/pack/tests.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pack/tests.log; tools/gpu_steps.sh \
  "200|pack/packbench.log|python tools/packbench.py"
