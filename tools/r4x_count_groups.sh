# counted staged regions partitioned together: per-group block budget (same box, alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4x; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: round(v['ms_per_step'],3) for k,v in st.items()})"; }
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  run "c2 r28" $B --config c2 || exit 1
  run "c2 r29" $B --config c2 --reserve-log2 29 || exit 1
  for c in c3 c5; do
    run "$c r28" $B --config $c || exit 1
    run "$c r28 cg512" LMR_COUNT_GROUP_BLOCKS=512 $B --config $c || exit 1
    run "$c r28 cg256" LMR_COUNT_GROUP_BLOCKS=256 $B --config $c || exit 1
    run "$c r29 cg512" LMR_COUNT_GROUP_BLOCKS=512 $B --config $c --reserve-log2 29 || exit 1
    run "$c r29 cg256" LMR_COUNT_GROUP_BLOCKS=256 $B --config $c --reserve-log2 29 || exit 1
  done
done > $O/runs.log 2>&1
cat $O/runs.log
