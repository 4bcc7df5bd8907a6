"""Throughput of the widened §8f rows next to their CPU restatements, one JSON
line each: loss weight maps (unet_weight_map), instance masks (8-connected
labelling + small-object removal, unet_instance_masks) and the Rand index
(unet_rand_index), on the real HeLa masks tiled up to the training batch
(8 x 512 x 512 label maps / 324 x 324 predicted masks).

    python tools/aux_bench.py [--iters 50]

HBM bytes per launch (algorithmic): weight maps 2 B read + 4 B written per
pixel (+ a 2-B count pass); instance masks 1 B read, 4 x 4 B work arrays
written and read, 2 B written per pixel; Rand index 2 x 2 B read per pixel
(twice: presence marks, histogram).
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


def gpu_time(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def cpu_time(fn, reps):
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    from unet_amd.augment import weight_maps
    from unet_amd.postproc import instance_masks, rand_index
    from oracle import weightmap_oracle as W
    from oracle import postproc_oracle as P
    z = np.load(os.path.join(ROOT, "tests", "golden", "hela_real.npz"), allow_pickle=False)
    segs = np.concatenate([z["segs"]] * 3)[:8]            # (8, 512, 512) uint16
    masks = np.concatenate([z["masks"]] * 3)[:8]          # (8, 324, 324) uint8 0/255
    dsegs, dmasks = torch.from_numpy(segs).cuda(), torch.from_numpy(masks).cuda()
    gt = torch.from_numpy(z["segs"][0, 94:418, 94:418].astype(np.uint16)).cuda()
    pred = instance_masks(dmasks[0], 15)

    ms = gpu_time(lambda: weight_maps(dsegs), args.iters)
    cpu = cpu_time(lambda: W.calculate_weight_map(segs[0]), 3)
    px = segs.size
    print(json.dumps({"metric": "weight maps/s (scripts/preprocess_data.py:17-77)", "value": round(8 / (ms * 1e-3), 1),
                      "unit": "maps/s", "ms_per_batch": round(ms, 4), "config": {"batch": 8, "size": 512},
                      "roofline": {"bound": "hbm", "achieved_gbs": round(px * 8 / (ms * 1e-3) / 1e9, 1),
                                   "peak_gbs": 8000.0},
                      "cpu_baseline": {"value": round(1e3 / cpu, 1), "unit": "maps/s", "cores": 1, "kind": "port",
                                       "sample": "3 maps 512x512, oracle/weightmap_oracle.py"}}))
    ms = gpu_time(lambda: instance_masks(dmasks, 15), args.iters)
    cpu = cpu_time(lambda: P.get_instance_masks(masks[0], 15), 1)
    px = masks.size
    print(json.dumps({"metric": "instance masks/s (utils/metrics.py:42-72)", "value": round(8 / (ms * 1e-3), 1),
                      "unit": "masks/s", "ms_per_batch": round(ms, 4), "config": {"batch": 8, "size": 324},
                      "roofline": {"bound": "hbm/latency (union-find)",
                                   "achieved_gbs": round(px * 35 / (ms * 1e-3) / 1e9, 1), "peak_gbs": 8000.0},
                      "cpu_baseline": {"value": round(1e3 / cpu, 2), "unit": "masks/s", "cores": 1, "kind": "port",
                                       "sample": "1 mask 324x324, oracle/postproc_oracle.py (Python BFS)"}}))
    ms = gpu_time(lambda: rand_index(gt, pred), args.iters)
    cpu = cpu_time(lambda: P.rand_index(gt.cpu().numpy(), pred.cpu().numpy()), 3)
    print(json.dumps({"metric": "Rand index evaluations/s (utils/metrics.py:75-139)", "value": round(1 / (ms * 1e-3), 1),
                      "unit": "evals/s", "ms_per_eval": round(ms, 4), "config": {"size": 324},
                      "note": "includes one stream synchronisation (label counts size the table)",
                      "cpu_baseline": {"value": round(1e3 / cpu, 1), "unit": "evals/s", "cores": 1, "kind": "port",
                                       "sample": "3 evals 324x324, oracle/postproc_oracle.py (NumPy)"}}))


if __name__ == "__main__":
    main()
