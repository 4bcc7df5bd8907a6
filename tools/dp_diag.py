"""Data-parallel gradient diagnosis (GPU box): the two-rank Trainer of
tests/test_gpu_dp.py against its per-shard single-process reference, per
backward segment bucket and step, for the overlap schedules

    overlap + deferred join (default), overlap with a join at every segment
    end (UNET_DP_DEFER=0), and no overlap (one whole-backward all-reduce).

Every step's reference gradient is taken at the weights the ranks started
that step from.  A cross-segment race shows as one bucket far off while the
others agree at the weight-gradient kernels' atomic-order rounding.

    python tools/dp_diag.py [steps]
"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
for p in (ROOT, os.path.join(ROOT, "unet-segmentation_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import test_gpu_dp as T  # noqa: E402


def buckets():
    from unet_amd import _lib
    from unet_amd.plan import Plan
    from unet_amd.train import N_SEGMENTS
    from unet_amd import UNet
    from unet_amd.train import FlatParams
    m = UNet(1, 2)
    fp = FlatParams(m)
    pl = Plan(T.W.BATCH, 1, T.W.SIZE, T.W.SIZE, 2, "fp32")
    return [fp.range_for(*pl.segment_grads(s)) for s in range(N_SEGMENTS)]


def report(tag, ranks, sums, bk):
    for s in range(T.STEPS):
        g, ref = ranks[0][f"grad{s}"], sums[s]
        rel = np.linalg.norm(g - ref) / np.linalg.norm(ref)
        per = []
        for a, b in bk:
            d = np.linalg.norm(g[a:b] - ref[a:b]) / max(np.linalg.norm(ref[a:b]), 1e-30)
            per.append(f"{d:.1e}")
        print(f"{tag} step {s}: rel {rel:.2e} | buckets {' '.join(per)}", flush=True)


def main():
    T.STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    bk = buckets()
    print("buckets", bk, flush=True)
    with tempfile.TemporaryDirectory() as d:
        for tag, overlap, defer in (("defer", True, "1"), ("join-per-segment", True, "0"), ("no-overlap", False, "1")):
            os.environ["UNET_DP_DEFER"] = defer
            ranks = T.run_ranks(Path(d), overlap)
            ws = [ranks[0][f"w{s}"] for s in range(T.STEPS)]
            sums = T.single_process_reference(ws)
            report(tag, ranks, sums, bk)
            if tag == "defer":  # the reference against itself, same weights
                again = T.single_process_reference(ws)
                report("reference-vs-itself", [{f"grad{s}": again[s] for s in range(T.STEPS)}], sums, bk)


if __name__ == "__main__":
    main()
