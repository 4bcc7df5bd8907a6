#!/bin/bash
set -o pipefail
o=${1:-gpurun_out/dp}; mkdir -p $o
# 2-rank rehearsal of the DP bench path on the box's one GPU (gloo stages CUDA
# tensors through the host; timings say nothing about RCCL over xGMI)
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --full-stdout --gpus 2 --steps 5 --warmup 3 --dist-backend gloo --no-extras --no-cpu-baseline --no-iou > $o/dp_bench.json 2> $o/dp_bench.err; echo dp rc=$?
tail -c 1500 $o/dp_bench.json
