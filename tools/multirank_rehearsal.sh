# The bench's N > 1 flow (torchrun, one rank per PE) rehearsed on a one-GPU box: 2 and 4 ranks
# share cuda:0 and exchange over gloo (RCCL refuses two ranks on one GPU); small sizes, the
# timing is meaningless, the JSON line and its `verified` invariant are the check.
mkdir -p gpurun_out/mr && export TMPDIR=/tmp LAMELLAR_COMM_BACKEND=gloo && tools/gpu_steps.sh \
  "300|mr/c4_n2.log|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29911 bench.py --gpus 2 --steps 3 --warmup 1 --records-log2 22 --elems-log2 22 --reserve-log2 25" \
  "300|mr/c4_n4.log|python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29912 bench.py --gpus 4 --steps 3 --warmup 1 --records-log2 22 --elems-log2 22 --reserve-log2 25" \
  "300|mr/c3_n2.log|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29913 bench.py --gpus 2 --config c3 --steps 3 --warmup 1 --records-log2 22 --elems-log2 20 --reserve-log2 25" \
  "300|mr/c5_n4.log|python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29914 bench.py --gpus 4 --config c5 --steps 3 --warmup 1 --records-log2 24 --elems-log2 22 --reserve-log2 25"
