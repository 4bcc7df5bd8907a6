"""CPU oracle for the per-pixel loss weight maps.

TEST INFRASTRUCTURE ONLY: only ``tests/`` import it, as the checker; the HIP
path (``csrc/weightmap.hip``) never falls back to it.

Restates scripts/preprocess_data.py:17-77 (``calculate_weight_map``, w0 = 10,
sigma = 5 at :14-15), the offline step whose ``weight_map_*.npy`` files
utils/dataset.py:85 loads (and casts to fp32 at :111):

* wc: 1 / (count / total) per class of ``labels > 0`` (fp64), 0 for an empty
  class, stored in an fp32 map (:25-37);
* separation term: per object ``min(edt(obj), edt(obj == 0))`` (:46-48), the two
  smallest over objects, ``w0 * exp(-(d1 + d2)^2 / (2 (sigma^2 + 1e-8)))``.
  ``distance_transform_edt(m)`` is 0 exactly where ``m`` is 0, so one of the two
  transforms is 0 at every pixel and their minimum is identically 0: d1 = d2 = 0
  for every mask (also the one- and no-object branches, :52-62), and the term
  is ``w0 * exp(-0.0) = w0`` exactly.  (The U-Net paper's border weighting is
  what the comments intend; the reference computes the constant, and so does
  this path.)
* weight = wc (fp32, widened) + w0 in fp64 (:72).

Pinned to the reference itself: ``tests/golden/make_golden_weightmap.py`` runs
the reference function on the committed HeLa label maps and synthetic masks and
checks it against the reference's own committed ``weight_map_00[0-2].npy``.
"""
import numpy as np


def calculate_weight_map(labels, w0=10.0, sigma=5.0):
    binary = (np.asarray(labels) > 0)
    fg = int(binary.sum())
    total = binary.size
    bg = total - fg
    wc_bg = 1.0 / (bg / total) if bg > 0 else 0.0
    wc_fg = 1.0 / (fg / total) if fg > 0 else 0.0
    wc = np.where(binary, np.float32(wc_fg), np.float32(wc_bg)).astype(np.float32)
    d = np.zeros(binary.shape, np.float64)  # d1 + d2, identically 0 (module docstring)
    exp_term = w0 * np.exp(-(d ** 2) / (2 * (sigma ** 2 + 1e-8)))
    return wc + exp_term


def training_weights(labels, w0=10.0, sigma=5.0):
    """utils/dataset.py:111: the fp32 tensor the loss sees."""
    return calculate_weight_map(labels, w0, sigma).astype(np.float32)
