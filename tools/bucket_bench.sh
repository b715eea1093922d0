#!/bin/bash
# builds and runs tools/bucket_bench (the bucketed push's passes at the 8-GPU geometry, one GPU)
# usage: tools/bucket_bench.sh build | run [reps]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "$1" = build ]; then
  exec /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/bucket_bench tools/bucket_bench.hip \
    -Llamellar-runtime_amd -llamellar_gpu_ops -Wl,-rpath,'$ORIGIN/../lamellar-runtime_amd'
fi
tools/bucket_bench "${2:-10}"
