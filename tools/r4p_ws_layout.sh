# workspace allocation size vs layout offset (same box, alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: round(v['ms_per_step'],3) for k,v in st.items()})"; }
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  run "c3 base" $B --config c3 || exit 1
  run "c3 extra12G" LMR_WS_EXTRA_MB=12288 $B --config c3 || exit 1
  run "c3 shift64K" LMR_WS_SHIFT_KB=64 $B --config c3 || exit 1
  run "c3 shift2M" LMR_WS_SHIFT_KB=2048 $B --config c3 || exit 1
  run "c3 shift1G" LMR_WS_SHIFT_KB=1048576 $B --config c3 || exit 1
  run "c3 reserve28" $B --config c3 --reserve-log2 28 || exit 1
  run "c2 base" $B --config c2 || exit 1
  run "c2 extra12G" LMR_WS_EXTRA_MB=12288 $B --config c2 || exit 1
  run "c2 shift1G" LMR_WS_SHIFT_KB=1048576 $B --config c2 || exit 1
done > $O/runs.log 2>&1
cat $O/runs.log
