#!/bin/bash
# C2 sweep over partition knobs: "crpt:frpt:bin_blocks:fine_blocks" per setting, repeated twice
cfg=${1:-c2}
list=${SWEEP:-"4:4:512:512 6:4:512:512 6:8:512:256 4:8:512:256 6:8:384:256 4:4:512:512"}
for spec in $list; do
  IFS=: read cr fr gb fb <<< "$spec"
  out=$(LMR_COARSE_RPT=$cr LMR_FINE_RPT=$fr LMR_BIN_BLOCKS=$gb LMR_FINE_BLOCKS=$fb \
        timeout -k 10 120 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{') || exit $?
  echo "$spec $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["verified"], {k: round(v["ms_per_step"],3) for k,v in d["apply_pipeline"]["stages"].items()})')"
done
