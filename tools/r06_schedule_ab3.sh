#!/bin/bash
# Round-6 scheduling experiment 3 (fp32 bench, one box, runs in order): the
# Winograd weight gradients' input transforms issued during the forward on the
# side stream (UNET_WGRAD_FWD_U=1) against the default schedule.
set -e
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_gpu_bnb_fuse.py::test_wgrad_fwd_u_bit_identical" > $O/t.log 2>&1
B="python -u bench.py --steps 20 --warmup 5 --extra-dtypes= --no-extras --no-cpu-baseline --no-iou --no-peaks"
for r in 0 1 2 3 4 5; do
  UNET_WGRAD_FWD_U=$((r % 2)) timeout -k 10 240 $B --detail-out $O/u$r.json > $O/u$r.log 2>&1
done
