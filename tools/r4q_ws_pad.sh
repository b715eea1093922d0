# workspace layout: record-array spacing and staggered padding (same box, alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4q; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: round(v['ms_per_step'],3) for k,v in st.items()})"; }
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  run "c3 base" $B --config c3 || exit 1
  run "c3 lay28" LMR_WS_LAYOUT_LOG2=28 $B --config c3 || exit 1
  run "c3 pad4K" LMR_WS_PAD_KB=4 $B --config c3 || exit 1
  run "c3 pad64K" LMR_WS_PAD_KB=64 $B --config c3 || exit 1
  run "c3 pad1028K" LMR_WS_PAD_KB=1028 $B --config c3 || exit 1
  run "c3 pad16M" LMR_WS_PAD_KB=16384 $B --config c3 || exit 1
  run "c2 base" $B --config c2 || exit 1
  run "c2 lay29" LMR_WS_LAYOUT_LOG2=29 $B --config c2 || exit 1
  run "c2 pad64K" LMR_WS_PAD_KB=64 $B --config c2 || exit 1
  run "c2 pad16M" LMR_WS_PAD_KB=16384 $B --config c2 || exit 1
done > $O/runs.log 2>&1
cat $O/runs.log
