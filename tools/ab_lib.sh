# Same-box A/B of two builds of the library: the current one and lamellar-runtime_amd/liblamellar_gpu_ops_prev.so
# (built from an earlier commit), alternating. usage: bash tools/ab_lib.sh <config> [reps]
cfg=${1:-c2}; reps=${2:-3}
mkdir -p gpurun_out/ablib && export TMPDIR=/tmp
for i in $(seq $reps); do
  for lib in cur prev; do
    if [ $lib = prev ]; then export LAMELLAR_GPU_OPS_LIB=$PWD/lamellar-runtime_amd/liblamellar_gpu_ops_prev.so; else unset LAMELLAR_GPU_OPS_LIB; fi
    timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 10 --no-cpu-baseline 2>/dev/null | grep '^{' | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$lib', round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in d['apply_pipeline']['stages'].items()})" || exit 1
  done
done
