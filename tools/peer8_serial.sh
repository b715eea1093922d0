# The peer push at 8 ranks sharing cuda:0 (gloo base) with the set-up serialised through each PE's first
# kernel after its imports; LMR_PEER_DEBUG=1 times each set-up step.
mkdir -p gpurun_out/mr8 && export TMPDIR=/tmp LAMELLAR_COMM_BACKEND=gloo LAMELLAR_TRANSPORT=peer LAMELLAR_PEER_TIMEOUT=40 LMR_PEER_DEBUG=1 && tools/gpu_steps.sh \
  "120|mr8/p6_serial.log|LAMELLAR_EXCHANGE_BUCKETS=0 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 6 --master-addr 127.0.0.1 --master-port 29970 bench.py --gpus 6 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "120|mr8/p8_serial_buckets2.log|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29971 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "120|mr8/p8_serial_plain2.log|LAMELLAR_EXCHANGE_BUCKETS=0 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29972 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25"
