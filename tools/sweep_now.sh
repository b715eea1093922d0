# C2 / C3 sweep of partition block counts at the current round sizes (GPU box, repo root)
mkdir -p gpurun_out/sw && export TMPDIR=/tmp
for cfg in c2 c3; do
  SWEEP="12:8:512:512 12:8:256:256 12:8:512:256 12:8:256:512 8:8:256:256 12:8:384:256 12:8:512:512" timeout -k 10 600 bash tools/sweep_c2.sh $cfg > gpurun_out/sw/$cfg.txt 2>&1 || exit $?
  cat gpurun_out/sw/$cfg.txt
done
