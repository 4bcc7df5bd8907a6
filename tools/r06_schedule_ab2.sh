#!/bin/bash
# Round-6 scheduling experiment 2 (fp32 bench, one box, runs in order):
# default vs the fused BN-backward apply + dY transform WITH the early U
# transforms on the side stream (UNET_BNB_FUSE=1 UNET_WGRAD_EARLY_U=1).
set -e
O=gpurun_out/s3
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 5 --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --no-peaks"
for r in 0 1 2 3 4 5; do
  F=$((r % 2))
  UNET_BNB_FUSE=$F UNET_WGRAD_EARLY_U=$F timeout -k 10 240 $B --detail-out $O/f$r.json > $O/f$r.log 2>&1
done
