"""Diagnostic: per-tensor gradient-norm error of one bf16 Trainer step at a
configured size against the reference's fp64 fixture and the bf16 oracle's
own gradients (tests/golden/train_n8_512{,_bf16}.npz), for the kernel mix the
environment selects (UNET_AUTOTUNE, UNET_TUNE_DB, UNET_BF16_NORM, ...).

    python tools/bf16_diag.py [--precision bf16] [--top 20]
Prints one line per tensor sorted by |gpu - bf16 oracle| / |bf16 oracle - ref|.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unet-segmentation_amd"), os.path.join(ROOT, "tests")]
from oracle import unet_oracle as O  # noqa: E402
from oracle import fixtures as F  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--fixture", default="train_n8_512")
    ap.add_argument("--small", default=None, help="n,h: fresh bf16 oracle (fp64 and fp32) at a small size instead")
    args = ap.parse_args()
    if args.small:
        return small(args)
    from test_gpu_fullsize import trainer_step
    z = np.load(os.path.join(G, f"{args.fixture}.npz"), allow_pickle=False)
    zb = np.load(os.path.join(G, f"{args.fixture}_bf16.npz"), allow_pickle=False)
    seed, n, h = int(z["x_seed"]), int(z["n"]), int(z["h"])
    c = int(z["c"]) if "c" in z.files else 1
    params = O.hash_init(c, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, c, h)
    lg, loss, grads, _ = trainer_step(params, x, tgt, wmap, args.precision, n_channels=c)
    print(f"env: " + " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("UNET_")))
    print(f"loss {loss:.6f} ref {float(z['loss']):.6f} bf16-oracle {float(zb['loss']):.6f}")
    rows = []
    for name, g in grads.items():
        if O.bn_cancelled(name):
            continue
        r, rb = float(z[f"gnorm/{name}"]), float(zb[f"gbf16norm/{name}"])
        gn = float(np.linalg.norm(g))
        floor = abs(rb - r)
        rows.append((abs(gn - rb) / max(floor, 1e-30), name, (gn - r) / r, (rb - r) / r, (gn - rb) / rb))
    rows.sort(reverse=True)
    print(f"{'tensor':58s} {'gpu-ref':>9s} {'bf-ref':>9s} {'gpu-bf':>9s} ratio")
    for ratio, name, a, b, d in rows[:args.top]:
        print(f"{name:58s} {a:+9.4f} {b:+9.4f} {d:+9.4f} {ratio:6.1f}")


def small(args):
    """GPU bf16 step vs the bf16 oracle in fp64, with the same oracle in fp32 as
    the rounding-boundary floor (tests/test_gpu_bf16.py's bar), per tensor."""
    from test_gpu_fullsize import trainer_step
    from test_gpu_bf16 import bf16_oracle_step
    n, h = (int(v) for v in args.small.split(","))
    params = O.hash_init(1, 2, seed=5, bn_random=True)
    x, tgt, wmap = F.make_inputs(5, n, 1, h)
    lg, loss, grads, _ = trainer_step(params, x, tgt, wmap, args.precision)
    rl, rloss, rg, _ = bf16_oracle_step(params, x, tgt, wmap)
    _, l32, g32, _ = bf16_oracle_step(params, x, tgt, wmap, np.float32)
    print(f"{n}x{h}: loss gpu {loss:.6f} oracle {rloss:.6f} oracle32 {l32:.6f}")
    rows = []
    for name, g in grads.items():
        if O.bn_cancelled(name):
            continue
        r = np.asarray(rg[name], np.float64)
        nr = max(np.linalg.norm(r), 1e-30)
        e = np.linalg.norm(g - r) / nr
        fl = np.linalg.norm(np.asarray(g32[name], np.float64) - r) / nr
        rows.append((e / max(fl, 1e-12), name, e, fl))
    rows.sort(reverse=True)
    for ratio, name, e, fl in rows[:args.top]:
        print(f"{name:58s} rel-L2 {e:.2e} floor32 {fl:.2e} ratio {ratio:6.1f}")


if __name__ == "__main__":
    main()
