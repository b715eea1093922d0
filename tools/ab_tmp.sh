cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
tools/gpu_steps.sh "900|check_gpu.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" || exit $?
grep -q " passed" gpurun_out/check_gpu.log && ! grep -q "failed" gpurun_out/check_gpu.log || { tail -30 gpurun_out/check_gpu.log; exit 1; }
for c in c2 c3 c5; do
timeout -k 10 400 bash tools/ab_mix.sh $c 2 "cur|" "cur|LMR_FINE_XCD=0" "cur|LMR_FINE_BLOCKS=1024" || exit $?
done
timeout -k 10 400 bash tools/ab_mix.sh c4 1 "cur|" "cur|LMR_FINE_XCD=0" || exit $?
