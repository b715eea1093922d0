# The peer push through the bench's N > 1 flow with more ranks than the tests use (4 and 8 ranks sharing
# cuda:0, gloo base): short peer timeouts so a wait that never completes ends in an error, not a hang.
mkdir -p gpurun_out/mr8 && export TMPDIR=/tmp LAMELLAR_COMM_BACKEND=gloo LAMELLAR_TRANSPORT=peer LAMELLAR_PEER_TIMEOUT=25 LMR_XDEBUG=1 && tools/gpu_steps.sh \
  "150|mr8/p4_buckets.log|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29931 bench.py --gpus 4 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "150|mr8/p8_plain.log|LAMELLAR_EXCHANGE_BUCKETS=0 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29932 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "150|mr8/p8_buckets.log|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29933 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25"
