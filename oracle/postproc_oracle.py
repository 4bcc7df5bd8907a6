"""CPU oracle for the segmentation post-processing.

TEST INFRASTRUCTURE ONLY: only ``tests/`` import it, as the checker; the HIP
path (``csrc/postproc.hip``) never falls back to it.

Restates utils/metrics.py:

* ``get_instance_masks`` (:42-72): ``skimage.measure.label(mask > 0,
  connectivity=2)`` -- 8-connected components numbered 1, 2, ... in raster
  order of each component's first pixel -- then
  ``skimage.morphology.remove_small_objects(labels, min_size=15)``, which zeroes
  every component with fewer than ``min_size`` pixels WITHOUT renumbering the
  others, and a uint16 cast.  scikit-image is not installed in this image (the
  reference module cannot be imported here), so the labelling is checked
  against ``scipy.ndimage.label`` with a 3x3 structure, which numbers components
  the same way, and -- the pin -- against the reference's OWN outputs: its 84
  committed ``01_RES/mask*.tif`` -> ``01_RES_INST/m*.tif`` pairs
  (scripts/predict.py:92-112 with min_size=15; tests/golden/hela_postproc.npz)
  are reproduced bit-exactly (tests/test_oracle_postproc.py); the small-object
  rule is skimage's published one (``component_sizes < min_size`` are removed).
* ``calculate_rand_index_and_error`` (:75-139): contingency table of the two
  labelings; a = sum n_ij (n_ij - 1) / 2, same_gt / same_pred the row / column
  analogues, b = total - same_gt - same_pred + a, RI = (a + b) / total with
  total = N (N - 1) / 2 -- all fp64, every intermediate an exact integer below
  2^53 for images up to ~94 Mpx, so the result does not depend on summation
  order.  Pinned by known answers only (parity unpinned against the reference
  for this function: its module needs scikit-image).
"""
from collections import deque

import numpy as np


def label8(mask):
    """8-connected components of mask > 0, numbered in raster order of their
    first pixel (BFS restatement)."""
    fg = np.asarray(mask) > 0
    h, w = fg.shape
    lab = np.zeros((h, w), np.int64)
    nxt = 0
    for y in range(h):
        for x in range(w):
            if fg[y, x] and lab[y, x] == 0:
                nxt += 1
                lab[y, x] = nxt
                q = deque([(y, x)])
                while q:
                    cy, cx = q.popleft()
                    for dy in (-1, 0, 1):
                        for dx in (-1, 0, 1):
                            yy, xx = cy + dy, cx + dx
                            if 0 <= yy < h and 0 <= xx < w and fg[yy, xx] and lab[yy, xx] == 0:
                                lab[yy, xx] = nxt
                                q.append((yy, xx))
    return lab


def remove_small_objects(lab, min_size):
    counts = np.bincount(lab.ravel())
    small = counts < min_size
    small[0] = False
    out = lab.copy()
    out[small[lab]] = 0
    return out


def get_instance_masks(binary_mask, min_size=15, labeler=label8):
    return remove_small_objects(labeler(binary_mask), min_size).astype(np.uint16)


def rand_index(gt, pred):
    """(rand index, rand error) of two instance labelings."""
    g = np.asarray(gt).ravel().astype(np.int64)
    p = np.asarray(pred).ravel().astype(np.int64)
    n = g.size
    if n < 2:
        return 1.0, 0.0
    total = n * (n - 1) / 2.0
    _, gi = np.unique(g, return_inverse=True)
    _, pi = np.unique(p, return_inverse=True)
    cont = np.zeros((gi.max() + 1, pi.max() + 1), np.int64)
    np.add.at(cont, (gi, pi), 1)
    a = np.sum(cont * (cont - 1) / 2)
    rows, cols = cont.sum(1), cont.sum(0)
    same_gt = np.sum(rows * (rows - 1) / 2)
    same_pred = np.sum(cols * (cols - 1) / 2)
    b = total - same_gt - same_pred + a
    ri = (a + b) / total
    return ri, 1.0 - ri
