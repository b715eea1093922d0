# workspace-size sensitivity of C3 / C5 / C2 (same box, alternating)
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: round(v['ms_per_step'],3) for k,v in st.items()})"; }
for i in 1 2; do
  for r in 0 27 28; do
    a=""; [ $r != 0 ] && a="--reserve-log2 $r"
    run "c3 reserve=$r" timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline $a || exit 1
    run "c5 reserve=$r" timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline $a || exit 1
  done
  for r in 0 29; do
    a=""; [ $r != 0 ] && a="--reserve-log2 $r"
    run "c2 reserve=$r" timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline $a || exit 1
  done
done > $O/runs.log 2>&1
cat $O/runs.log
