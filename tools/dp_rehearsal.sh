#!/bin/bash
# N>1 bench path (per-rank graphs + SUM all-reduce between them) rehearsed with 2 ranks sharing
# the box's one GPU over gloo.  The real N>1 runs use RCCL on an 8-GPU node (driver).
set -o pipefail
mkdir -p gpurun_out
export SNNFLOW_SHARE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --no-cpu-baseline --dist-backend gloo \
  > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { tail -30 gpurun_out/dp2.err; exit 3; }
cut -c1-400 gpurun_out/dp2.json
