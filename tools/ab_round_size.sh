# A/B of the coarse / fine LDS round sizes (records per thread per round) on one GPU box.
# usage (GPU box): bash tools/ab_round_size.sh ; logs under gpurun_out/ab/
mkdir -p gpurun_out/ab && export TMPDIR=/tmp && tools/gpu_steps.sh \
  "200|ab/c2_r4a.log|LMR_COARSE_RPT=4 LMR_FINE_RPT=4 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c2_r8a.log|LMR_COARSE_RPT=8 LMR_FINE_RPT=8 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c2_r12a.log|LMR_COARSE_RPT=12 LMR_FINE_RPT=12 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c2_r4b.log|LMR_COARSE_RPT=4 LMR_FINE_RPT=4 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c2_r8b.log|LMR_COARSE_RPT=8 LMR_FINE_RPT=8 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c2_r12b.log|LMR_COARSE_RPT=12 LMR_FINE_RPT=12 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c2_c8f4.log|LMR_COARSE_RPT=8 LMR_FINE_RPT=4 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c2_c4f8.log|LMR_COARSE_RPT=4 LMR_FINE_RPT=8 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c5_r4.log|LMR_COARSE_RPT=4 LMR_FINE_RPT=4 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c5_r8.log|LMR_COARSE_RPT=8 LMR_FINE_RPT=8 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c3_r4.log|LMR_COARSE_RPT=4 LMR_FINE_RPT=4 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline" \
  "200|ab/c3_r8.log|LMR_COARSE_RPT=8 LMR_FINE_RPT=8 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline"
