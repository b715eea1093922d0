#!/bin/bash
# Same-box A/B of several builds of the library, alternating.
# usage: bash tools/ab_libs.sh <config> <reps> <lib> [<lib> ...]
#   <lib> = "cur" (lamellar-runtime_amd/liblamellar_gpu_ops.so) or a path to another build
cfg=$1; reps=$2; shift 2
mkdir -p gpurun_out/ablib && export TMPDIR=/tmp
extra=""; [ "$cfg" = c4 ] && extra="LAMELLAR_FORCE_EXCHANGE=1"
steps=20; [ "$cfg" = c4 ] && steps=10
for i in $(seq $reps); do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset LAMELLAR_GPU_OPS_LIB; else export LAMELLAR_GPU_OPS_LIB=$PWD/$lib; fi
    env $extra timeout -k 10 200 python bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{' | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d.get('apply_pipeline',{}).get('stages',{}); print('$cfg', '$(basename $lib)', round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in st.items()})" || exit 1
  done
done
