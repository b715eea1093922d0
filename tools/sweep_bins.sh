#!/bin/bash
# Sweep partition block counts on the C2 bench (tiled); one JSON summary line per setting.
for gb in 256 512 1024; do
  for fb in 256 512 2048; do
    out=$(LMR_BIN_BLOCKS=$gb LMR_FINE_BLOCKS=$fb timeout -k 10 120 python bench.py --steps 5 --warmup 2 --strategy tiled --no-cpu-baseline 2>/dev/null | grep '^{') || exit $?
    echo "$gb $fb $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), {k: round(v["ms_per_step"],3) for k,v in d["apply_pipeline"]["stages"].items()})')"
  done
done
