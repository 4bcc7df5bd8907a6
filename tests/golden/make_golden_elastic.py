"""Golden fixtures of the elastic-deformation input pipeline, made by the
REFERENCE itself.

Runs only in the build container, where /root/reference exists: it imports the
reference's ``utils/augmentations.py`` (``elastic_deform_image_and_mask``, which
calls scipy.ndimage) and applies it, as ``utils/dataset.py:84-96`` does
(``alpha=2000, sigma=20`` from scripts/train.py:35-36, an int seed, then
``astype(np.uint8)`` of both outputs), to
* the three real DIC-C2DH-HeLa frames / label maps already committed in
  ``hela_real.npz`` (512 x 512), seeds 11, 12, 13;
* a synthetic ragged case (61 x 77, uint8 image, uint16 labels up to 300 --
  so the uint8 cast of a label wraps as in the reference), seed 7, and the same
  with sigma = 3 (a short kernel: out-of-range reflections everywhere).
Only the outputs are committed (``elastic.npz``, plain arrays); the inputs are
the committed frames or regenerated from a fixed numpy Generator seed.

Usage:  python tests/golden/make_golden_elastic.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
sys.path.insert(0, "/root/reference")

from oracle.fixtures import elastic_synthetic_case as synthetic_case  # noqa: E402
from utils.augmentations import elastic_deform_image_and_mask  # noqa: E402  (reference)


def main():
    z = np.load(os.path.join(HERE, "hela_real.npz"), allow_pickle=False)
    out = {}
    for i, seed in enumerate((11, 12, 13)):
        im, mk = elastic_deform_image_and_mask(z["images"][i], z["segs"][i], alpha=2000, sigma=20, random_state=seed)
        out[f"hela{i}_img"] = im.astype(np.uint8)
        out[f"hela{i}_mask"] = mk.astype(np.uint8)
        out[f"hela{i}_seed"] = np.int64(seed)
    img, lab = synthetic_case()
    for tag, sigma in (("syn", 20.0), ("syn_s3", 3.0)):
        im, mk = elastic_deform_image_and_mask(img, lab, alpha=2000, sigma=sigma, random_state=7)
        out[f"{tag}_img"] = im.astype(np.uint8)
        out[f"{tag}_mask"] = mk.astype(np.uint8)
        out[f"{tag}_sigma"] = np.float64(sigma)
    np.savez_compressed(os.path.join(HERE, "elastic.npz"), **out)
    print("wrote", os.path.join(HERE, "elastic.npz"), sorted(out))


if __name__ == "__main__":
    main()
