"""Overlap-tile inference throughput (BASELINE.json configs[3]: a 1024 x 1024
image as 512 x 512 tiles, 16 tiles of 324 x 324 output) on the visible GPUs
(one replica per device, tiles dealt round-robin, no collectives).  Prints one
JSON line: images/s and tiles/s, mask output (scripts/predict.py:85-92).

    python tools/tile_bench.py [--size 1024] [--tile 512] [--batch 8] [--iters 10] [--devices 0]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--devices", default="0")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "bf16x3"])
    args = ap.parse_args()
    from unet_amd import UNet
    from unet_amd.tiling import TileFarm, TileGeometry
    torch.manual_seed(0)
    m = UNet(1, 2)
    m.precision = args.precision
    devs = [int(d) for d in args.devices.split(",")]
    farm = TileFarm(m, devices=devs, tile_in=args.tile, batch=args.batch)
    for r in farm.replicas:
        r.precision = args.precision
    img = torch.rand((1, args.size, args.size)) * 2 - 1
    for _ in range(2):
        farm.predict(img, return_mask=True)
    t0 = time.perf_counter()
    for _ in range(args.iters):
        mask = farm.predict(img, return_mask=True)
    dt = (time.perf_counter() - t0) / args.iters
    geo = TileGeometry(args.size, args.size, args.tile)
    print(json.dumps({"metric": "overlap-tile inference images/s (configs[3])", "value": round(1 / dt, 3),
                      "unit": "images/s", "ms_per_image": round(dt * 1e3, 2), "tiles_per_image": len(geo),
                      "tiles_per_s": round(len(geo) / dt, 1), "n_gpus": len(devs), "precision": args.precision,
                      "config": {"image": args.size, "tile_in": args.tile, "tile_out": geo.tile_out,
                                 "batch": args.batch}, "mask_shape": list(mask.shape)}))


if __name__ == "__main__":
    main()
