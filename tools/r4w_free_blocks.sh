# staged count-free pass: blocks per region, lone and grouped (same box, alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4w; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: round(v['ms_per_step'],3) for k,v in st.items()})"; }
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  run "c2 r28 b256" $B --config c2 || exit 1
  run "c2 r28 b128" LMR_FREE_BLOCKS=128 $B --config c2 || exit 1
  run "c2 r28 b64" LMR_FREE_BLOCKS=64 $B --config c2 || exit 1
  run "c2 r29 g256" LMR_FREE_GROUP_BLOCKS=256 $B --config c2 --reserve-log2 29 || exit 1
  run "c2 r29 g128" LMR_FREE_GROUP_BLOCKS=128 $B --config c2 --reserve-log2 29 || exit 1
  run "c4 b256" LAMELLAR_FORCE_EXCHANGE=1 $B --config c4 || exit 1
  run "c4 b128" LAMELLAR_FORCE_EXCHANGE=1 LMR_FREE_BLOCKS=128 $B --config c4 || exit 1
done > $O/runs.log 2>&1
cat $O/runs.log
