#!/bin/bash
# Same-box A/B over (library build, environment, bench arguments) triples, alternating.
# usage: bash tools/ab_mix.sh <config> <reps> "<lib>|<env settings>[|<bench args>]" ...
#   <lib> = cur (the in-tree build) or a path to another build; <env> and <bench args> may be empty
#   e.g. "cur|LMR_FREE_GROUP_BLOCKS=512|--reserve-log2 29"
cfg=$1; reps=$2; shift 2
export TMPDIR=/tmp
extra=""; [ "$cfg" = c4 ] && extra="LAMELLAR_FORCE_EXCHANGE=1"
steps=20; [ "$cfg" = c4 ] && steps=10
for i in $(seq $reps); do
  for spec in "$@"; do
    lib="${spec%%|*}"; rest="${spec#*|}"
    s="${rest%%|*}"; args=""; [ "$rest" != "$s" ] && args="${rest#*|}"
    if [ "$lib" = cur ]; then L=""; else L="LAMELLAR_GPU_OPS_LIB=$PWD/$lib"; fi
    env $extra $L $s timeout -k 10 200 python bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline $args 2>/dev/null | grep '^{' | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d.get('apply_pipeline',{}).get('stages',{}); print('$cfg', '$(basename $lib)', '[$s]', '[$args]', round(d['ms_per_step'],3), d.get('verified'), {k: round(v['ms_per_step'],3) for k,v in st.items()})" || exit 1
  done
done
