#!/bin/bash
# Round-6 experiment: the train step on a high-priority torch stream
# (UNET_MAIN_PRIORITY=-1; the plan's weight-gradient side stream keeps the
# lowest priority) against the default stream, A/B/A/B for fp32 and bf16, then
# a 2-rank gloo rehearsal of bench.py's multi-process path on one GPU.
set -e
O=gpurun_out/p1
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 5 --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --no-peaks"
for d in fp32 bf16; do
  for r in 0 1 2 3; do
    if [ $((r % 2)) -eq 1 ]; then P=-1; else P=; fi
    UNET_MAIN_PRIORITY=$P timeout -k 10 240 $B --dtype $d --detail-out $O/$d$r.json > $O/$d$r.log 2>&1
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --extra-dtypes= --no-extras \
  --no-cpu-baseline --no-iou --no-peaks --detail-out $O/dd.json > $O/dist.log 2>&1
