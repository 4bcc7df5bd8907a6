"""Golden weight maps made by the REFERENCE itself.

Runs only in the build container (/root/reference present): imports
``scripts/preprocess_data.py``'s ``calculate_weight_map`` (w0 = 10, sigma = 5 as
its :14-15) and applies it to the three committed HeLa label maps
(``hela_real.npz`` segs = 01_ST/SEG/man_seg000-002.tif) and the synthetic cases
of ``oracle.fixtures.weightmap_synthetic_cases``; also checks the HeLa results
against the reference's own committed ``01_ST/WEIGHT_MAPS/weight_map_00[0-2].npy``
(loaded with allow_pickle=False).  Writes ``weightmap.npz`` (fp64 maps).

Usage:  python tests/golden/make_golden_weightmap.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
sys.path.insert(0, os.path.join(REF, "scripts"))

from oracle.fixtures import weightmap_synthetic_cases  # noqa: E402
from preprocess_data import calculate_weight_map  # noqa: E402  (reference)


def main():
    z = np.load(os.path.join(HERE, "hela_real.npz"), allow_pickle=False)
    out = {}
    for i in range(3):
        wm = calculate_weight_map(z["segs"][i], 10, 5)
        committed = np.load(os.path.join(REF, "data/raw/train/DIC-C2DH-HeLa/01_ST/WEIGHT_MAPS",
                                         f"weight_map_{i:03d}.npy"), allow_pickle=False)
        assert wm.shape == committed.shape
        out[f"hela{i}"] = wm
        out[f"hela{i}_committed_maxdiff"] = np.float64(np.abs(wm - committed).max())
    for k, lab in weightmap_synthetic_cases().items():
        out[k] = calculate_weight_map(lab, 10, 5)
    np.savez_compressed(os.path.join(HERE, "weightmap.npz"), **out)
    print("wrote weightmap.npz;", {k: float(v) for k, v in out.items() if k.endswith("maxdiff")})


if __name__ == "__main__":
    main()
