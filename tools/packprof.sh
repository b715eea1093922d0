# pack microbenchmark + its rocprofv3 kernel trace (GPU box, repo root)
mkdir -p gpurun_out/pack && export TMPDIR=/tmp && tools/gpu_steps.sh \
  "200|pack/packbench.log|python tools/packbench.py" \
  "300|pack/prof.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/pack/prof -o run -- python3 tools/packbench.py --reps 3"
