# C3 kernel trace + FETCH/WRITE PMC passes (GPU box, repo root)
mkdir -p gpurun_out/pc3 && export TMPDIR=/tmp && tools/gpu_steps.sh \
  "300|pc3/trace.log|rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/pc3/prof/trace -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline" \
  "300|pc3/fetch.log|rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pc3/prof/pmc_fetch -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-verify" \
  "300|pc3/write.log|rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d gpurun_out/pc3/prof/pmc_write -o run -- python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-verify"
