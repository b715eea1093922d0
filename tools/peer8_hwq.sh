# Eight ranks sharing cuda:0 (gloo base): C5 and C3 over the collective exchange, then the peer push with
# two hardware queues per process (GPU_MAX_HW_QUEUES=2; 6+ processes with the default 4 stall at set-up,
# profiles/r6/multirank/peer_ranks.txt), bucketed and plain.
mkdir -p gpurun_out/mr8 && export TMPDIR=/tmp LAMELLAR_COMM_BACKEND=gloo && tools/gpu_steps.sh \
  "200|mr8/c5_n8.log|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29961 bench.py --gpus 8 --config c5 --steps 3 --warmup 1 --records-log2 23 --elems-log2 22 --reserve-log2 25" \
  "200|mr8/c3_n8.log|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29962 bench.py --gpus 8 --config c3 --steps 3 --warmup 1 --records-log2 22 --elems-log2 20 --reserve-log2 25" \
  "170|mr8/p8_hwq2_buckets.log|LAMELLAR_TRANSPORT=peer LAMELLAR_PEER_TIMEOUT=40 LMR_PEER_DEBUG=1 GPU_MAX_HW_QUEUES=2 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29963 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "170|mr8/p8_hwq2_plain.log|LAMELLAR_TRANSPORT=peer LAMELLAR_PEER_TIMEOUT=40 LAMELLAR_EXCHANGE_BUCKETS=0 GPU_MAX_HW_QUEUES=2 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29964 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25"
