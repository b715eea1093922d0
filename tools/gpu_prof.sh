#!/bin/bash
# bench + rocprofv3 kernel stats per config: tools/gpu_prof.sh <tag> <cfg>...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for cfg in "$@"; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_$cfg.json 2> $out/bench_$cfg.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/prof_$cfg -o run -- python3 bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-verify > $out/prof_$cfg.log 2>&1 || exit $?
done
for cfg in "$@"; do
  python3 - "$out/bench_$cfg.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "ms/step %.3f" % d["ms_per_step"], "verified", d["verified"])
for k, v in d["apply_pipeline"]["stages"].items():
    print("   %-16s %.3f ms  x%.1f  %s" % (k, v["ms_per_step"], v["launches_per_step"], ("%.0f GB/s" % v["achieved_GBps"]) if "achieved_GBps" in v else ""))
PY
done
