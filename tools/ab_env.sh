#!/bin/bash
# Same-box A/B of environment settings on one config, alternating.
# usage: bash tools/ab_env.sh <config> <reps> "<env settings A>" "<env settings B>" ...
#   e.g. bash tools/ab_env.sh c2 2 "LMR_FINE_RPT=8" "LMR_FINE_RPT=12"
# An empty setting string ("") runs the defaults. c4 runs with LAMELLAR_FORCE_EXCHANGE=1.
cfg=$1; reps=$2; shift 2
mkdir -p gpurun_out/abenv && export TMPDIR=/tmp
extra=""; [ "$cfg" = c4 ] && extra="LAMELLAR_FORCE_EXCHANGE=1"
steps=20; [ "$cfg" = c4 ] && steps=10
for i in $(seq $reps); do
  for s in "$@"; do
    env $extra $s timeout -k 10 200 python bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{' | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d.get('apply_pipeline',{}).get('stages',{}); print('$cfg', '[$s]', round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in st.items()})" || exit 1
  done
done
