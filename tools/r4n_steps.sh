cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
run() { tag=$1; shift; env "$@" 2>/dev/null | grep '^{' | python -c "import sys,json; d=json.loads(sys.stdin.read()); st=d['apply_pipeline']['stages']; print('$tag', round(d['ms_per_step'],3), d['verified'], {k: round(v['ms_per_step'],3) for k,v in st.items()})"; }
for i in 1 2; do
  run "c3 s10w3 dev" timeout -k 10 200 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  run "c3 s20w5 dev" timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  run "c3 s50w5 dev" timeout -k 10 200 python bench.py --config c3 --steps 50 --warmup 5 --no-cpu-baseline || exit 1
  run "c3 s20w5 sys" LMR_EVENT_SCOPE=system timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  run "c2 s20w5 dev" timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  run "c2 s20w5 sys" LMR_EVENT_SCOPE=system timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done > $O/runs.log 2>&1
cat $O/runs.log
