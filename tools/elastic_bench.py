"""Throughput of the GPU elastic-deformation pipeline (unet_elastic_deform) at
the training batch (8 x 512 x 512, alpha 2000, sigma 20: scripts/train.py:35-36)
next to the CPU restatement (oracle/elastic_oracle.py, NumPy) on a bounded
sample.  Prints one JSON line.

    python tools/elastic_bench.py [--batch 8] [--size 512] [--iters 50]

Per launch: two fp64 Gaussian passes (2r + 1 = 161 taps, one multiply and one
add per tap, no fma: the oracle's rounding) over 2 fields, then the warp.
Algorithmic work per sample: 4 * (2r + 1) * H * W fp64 multiply+add pairs;
HBM bytes per sample: noise 16 B/px read, two fp64 field pairs written and read
(4 x 16 B/px), image + labels read 3 B/px, x + target written 5 B/px.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X fp64 vector (fma) peak; the unfused mul+add pairs count 2 flops
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cpu-samples", type=int, default=3)
    args = ap.parse_args()
    from unet_amd.augment import ElasticDeform
    n, h = args.batch, args.size
    g = np.random.default_rng(0)
    images = torch.from_numpy(g.integers(0, 256, (n, h, h)).astype(np.uint8)).cuda()
    labels = torch.from_numpy(g.integers(0, 12, (n, h, h)).astype(np.uint16)).cuda()
    aug = ElasticDeform(2000.0, 20.0, noise="device", generator=torch.Generator(device="cuda").manual_seed(1))
    noise = aug.draw_noise(n, h, h, "cuda")
    for _ in range(3):
        aug(images, labels, noise=noise)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        aug(images, labels, noise=noise)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    # with the noise drawn on the device inside the timed region
    e0.record()
    for _ in range(args.iters):
        aug(images, labels)
    e1.record()
    torch.cuda.synchronize()
    ms_rng = e0.elapsed_time(e1) / args.iters

    r = int(4 * 20.0 + 0.5)
    px = n * h * h
    flops = 2.0 * 4 * (2 * r + 1) * px
    bytes_ = px * (16 + 4 * 16 + 3 + 5)

    from oracle import elastic_oracle as E
    t0 = time.perf_counter()
    for i in range(args.cpu_samples):
        im = images[i % n].cpu().numpy()
        lb = labels[i % n].cpu().numpy()
        nx, ny = E.noise_from_seed(i, (h, h))
        E.dataset_sample(im, lb, 2000.0, 20.0, nx, ny)
    cpu_s = (time.perf_counter() - t0) / args.cpu_samples

    print(json.dumps({
        "metric": "elastic-deformation samples/s (utils/augmentations.py:4-39 + dataset.py:84-111)",
        "value": round(n / (ms * 1e-3), 1), "unit": "samples/s", "ms_per_batch": round(ms, 4),
        "ms_per_batch_with_device_rng": round(ms_rng, 4),
        "config": {"batch": n, "size": h, "alpha": 2000, "sigma": 20, "radius": r},
        "roofline": {"bound": "fp64 valu", "achieved": round(flops / (ms * 1e-3) / 1e12, 2),
                     "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(flops / (ms * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS, 4),
                     "hbm_gbs": round(bytes_ / (ms * 1e-3) / 1e9, 1), "hbm_peak_gbs": HBM_PEAK_GBS},
        "cpu_baseline": {"value": round(1.0 / cpu_s, 2), "unit": "samples/s", "cores": 1, "kind": "port",
                         "sample": f"{args.cpu_samples} samples {h}x{h} through oracle/elastic_oracle.py "
                                   f"(NumPy fp64, {cpu_s * 1e3:.0f} ms each)"},
    }))


if __name__ == "__main__":
    main()
