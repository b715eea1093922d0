# deferred-session depth: workspace reservation 1x / 2^28 / 2^29 records (same box, alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4r; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: (round(v['ms_per_step'],3), round(v['launches_per_step'],2)) for k,v in st.items()})"; }
B="timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  for c in c3 c5 c2; do
    run "$c batch" $B --config $c || exit 1
    run "$c r28" $B --config $c --reserve-log2 28 || exit 1
    run "$c r29" $B --config $c --reserve-log2 29 || exit 1
  done
done > $O/runs.log 2>&1
cat $O/runs.log
