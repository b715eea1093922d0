# staged count-free pass: paired loads and grouped-launch blocks (same box, alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4v; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: round(v['ms_per_step'],3) for k,v in st.items()})"; }
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --config c2"
for i in 1 2 3; do
  run "c2 r28 pairs" $B || exit 1
  run "c2 r28 nopairs" LMR_FREE_STAGE_PAIRS=0 $B || exit 1
  run "c2 r29 g1024" $B --reserve-log2 29 || exit 1
  run "c2 r29 g512" LMR_FREE_GROUP_BLOCKS=512 $B --reserve-log2 29 || exit 1
  run "c2 r29 g256" LMR_FREE_GROUP_BLOCKS=256 $B --reserve-log2 29 || exit 1
done > $O/runs.log 2>&1
cat $O/runs.log
