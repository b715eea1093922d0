# The peer transport's set-up at 8 ranks sharing cuda:0 (gloo base), each step timed (LMR_PEER_DEBUG=1).
mkdir -p gpurun_out/mr8 && export TMPDIR=/tmp LAMELLAR_COMM_BACKEND=gloo LAMELLAR_TRANSPORT=peer LAMELLAR_PEER_TIMEOUT=100 LMR_PEER_DEBUG=1 LMR_XDEBUG=1 && tools/gpu_steps.sh \
  "170|mr8/p8_debug.log|LAMELLAR_EXCHANGE_BUCKETS=0 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29942 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25"
