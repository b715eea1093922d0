set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2a/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/r2a/gputest.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py > gpurun_out/r2a/bench_default.log 2>&1; echo "bench rc=$?"
  tail -c 3000 gpurun_out/r2a/bench_default.log
fi
