# The bench's N = 8 flow (torchrun, eight ranks) rehearsed on a one-GPU box: the eight ranks share
# cuda:0 and exchange over gloo (RCCL refuses two ranks on one GPU); small sizes, the timing is
# meaningless, the JSON line and its `verified` invariant are the check. The 8-PE geometry is what
# it exercises: 8 x C bucket keys per sender, eight sources per owner chunk, slice capacities and
# region sizes at eight PEs, over the collective exchange (bucketed regions, the default) and the
# peer push (IPC regions between the eight processes).
mkdir -p gpurun_out/mr8 && export TMPDIR=/tmp LAMELLAR_COMM_BACKEND=gloo && tools/gpu_steps.sh \
  "300|mr8/c4_n8.log|python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29921 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "300|mr8/c4_n8_peer.log|LAMELLAR_TRANSPORT=peer python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29922 bench.py --gpus 8 --steps 3 --warmup 1 --records-log2 22 --elems-log2 23 --reserve-log2 25" \
  "300|mr8/c5_n8.log|python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29923 bench.py --gpus 8 --config c5 --steps 3 --warmup 1 --records-log2 23 --elems-log2 22 --reserve-log2 25" \
  "300|mr8/c3_n8.log|python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29924 bench.py --gpus 8 --config c3 --steps 3 --warmup 1 --records-log2 22 --elems-log2 20 --reserve-log2 25"
