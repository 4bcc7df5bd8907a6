#!/bin/bash
# Round-6 scheduling experiments on the fp32 bench (one box, runs in order):
#  e*: UNET_WGRAD_EARLY_U=0/1/0/1 -- the Winograd weight gradients' input
#      transform issued on the side stream before the wait for the layer's dY;
#  s*: UNET_CONCURRENT=0 with UNET_BNB_FUSE=0/1/0/1 -- the fused BN-backward
#      apply + dY transform with the weight gradients serialised.
set -e
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_bnb_fuse.py::test_wgrad_early_u_bit_identical" > $O/t.log 2>&1
B="python -u bench.py --steps 20 --warmup 5 --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --no-peaks"
for r in 0 1 2 3; do
  UNET_WGRAD_EARLY_U=$((r % 2)) timeout -k 10 240 $B --detail-out $O/e$r.json > $O/e$r.log 2>&1
done
for r in 0 1 2 3; do
  UNET_CONCURRENT=0 UNET_BNB_FUSE=$((r % 2)) timeout -k 10 240 $B --detail-out $O/s$r.json > $O/s$r.log 2>&1
done
