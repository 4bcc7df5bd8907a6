"""Deterministic inputs shared by the fixture generator and the tests.

TEST INFRASTRUCTURE ONLY (see oracle/unet_oracle.py header).

Synthetic batch definition (SURVEY.md §8d "Synthetic inputs"):
* x ~ U[0,1) float32 (N,C,H,W) -- the range of ToTensor (utils/dataset.py:96)
* target ~ Bernoulli(0.4) int64 (N,Ho,Wo) -- mean foreground of man_seg000
* weight map = 10 + 1/freq(class) per image -- what scripts/preprocess_data.py
  actually produces (its line 47 leaves d1 = d2 = 0, so w = w_c + w0*exp(0) ...
  reduces to a per-class constant).
"""
from __future__ import annotations

import zlib

import numpy as np

from . import unet_oracle as O


def make_inputs(seed: int, n: int, c: int, h: int, w: int | None = None):
    w = h if w is None else w
    ho, wo = O.output_size(h), O.output_size(w)
    x = O.hash_uniform(seed, 1000, n * c * h * w).astype(np.float32).reshape(n, c, h, w)
    tgt = (O.hash_uniform(seed, 1001, n * ho * wo) < 0.4).astype(np.int64).reshape(n, ho, wo)
    wmap = class_weight_map(tgt)
    return x, tgt, wmap


def class_weight_map(tgt: np.ndarray) -> np.ndarray:
    """10 + 1/freq(class), per image (float32)."""
    out = np.empty(tgt.shape, np.float32)
    for i in range(tgt.shape[0]):
        t = tgt[i]
        f1 = max(t.mean(), 1e-6)
        f0 = max(1.0 - t.mean(), 1e-6)
        out[i] = np.where(t > 0, 10.0 + 1.0 / f1, 10.0 + 1.0 / f0)
    return out


def sample_indices(name: str, size: int, k: int = 32) -> np.ndarray:
    """Fixed per-parameter sample positions for gradient digests."""
    s = zlib.crc32(name.encode())
    u = O.hash_uniform(s, 77, k)
    return np.unique((u * size).astype(np.int64).clip(0, size - 1))


def elastic_synthetic_case():
    """Inputs of the synthetic elastic-deformation fixture
    (tests/golden/make_golden_elastic.py): a ragged 61 x 77 uint8 image and
    uint16 labels up to 300 (40 % background)."""
    g = np.random.default_rng(2024)
    img = g.integers(0, 256, (61, 77)).astype(np.uint8)
    lab = g.integers(0, 301, (61, 77)).astype(np.uint16)
    lab[g.random((61, 77)) < 0.4] = 0
    return img, lab


def weightmap_synthetic_cases():
    """Label maps of the synthetic weight-map fixtures
    (tests/golden/make_golden_weightmap.py): ragged multi-object, one object,
    empty, all foreground."""
    g = np.random.default_rng(77)
    multi = g.integers(0, 9, (45, 71)).astype(np.uint16)
    multi[g.random((45, 71)) < 0.5] = 0
    one = np.zeros((30, 30), np.uint16)
    one[5:12, 8:20] = 3
    empty = np.zeros((17, 23), np.uint16)
    full = np.full((9, 11), 5, np.uint16)
    return {"multi": multi, "one": one, "empty": empty, "full": full}


def plausible_running_stats(params, seed):
    """Replace the BatchNorm running statistics of a hash-initialised parameter
    set with plausible ones (mean ~ N(0, 0.2), var ~ 0.5 + U[0,1)), so that
    eval-mode forwards (tile farm fixtures) are not degenerate.  Deterministic
    (counter hash), shared by the fixture generator and the tests."""
    out = dict(params)
    for i, k in enumerate(sorted(params)):
        n = int(np.prod(params[k].shape))
        if k.endswith("running_mean"):
            out[k] = (0.2 * O.hash_normal(seed, 5000 + i, n)).astype(np.float32).reshape(params[k].shape)
        elif k.endswith("running_var"):
            out[k] = (0.5 + O.hash_uniform(seed, 5000 + i, n)).astype(np.float32).reshape(params[k].shape)
    return out
