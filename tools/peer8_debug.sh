# The peer transport's set-up with more ranks than the tests use, all sharing cuda:0 (gloo base), each
# set-up step timed (LMR_PEER_DEBUG=1): 8 ranks with fine-grained receive regions, then 6 and 5 ranks
# with the default (uncached) regions.
mkdir -p gpurun_out/mr8 && export TMPDIR=/tmp LAMELLAR_COMM_BACKEND=gloo LAMELLAR_TRANSPORT=peer LAMELLAR_PEER_TIMEOUT=40 LMR_PEER_DEBUG=1 LMR_XDEBUG=1 LAMELLAR_EXCHANGE_BUCKETS=0 && tools/gpu_steps.sh \
  "170|mr8/p8_fine.log|LMR_PEER_REGION_MEM=fine python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29951 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "170|mr8/p6.log|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 6 --master-addr 127.0.0.1 --master-port 29952 bench.py --gpus 6 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "170|mr8/p5.log|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 5 --master-addr 127.0.0.1 --master-port 29953 bench.py --gpus 5 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25"
