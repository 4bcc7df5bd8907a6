"""CPU checks of the weight-map oracle (oracle/weightmap_oracle.py) against the
maps the reference's calculate_weight_map produced (tests/golden/weightmap.npz,
tests/golden/make_golden_weightmap.py) -- which in turn equal the reference's
own committed weight_map_00[0-2].npy (max difference recorded in the fixture)."""
import os

import numpy as np
import pytest

from oracle import weightmap_oracle as W
from oracle import fixtures as F

G = os.path.join(os.path.dirname(__file__), "golden")


def _z():
    return np.load(os.path.join(G, "weightmap.npz"), allow_pickle=False)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_hela_label_maps(i):
    z = _z()
    segs = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)["segs"]
    np.testing.assert_array_equal(W.calculate_weight_map(segs[i]), z[f"hela{i}"])
    assert float(z[f"hela{i}_committed_maxdiff"]) == 0.0  # reference function == its committed .npy


@pytest.mark.parametrize("case", ["multi", "one", "empty", "full"])
def test_synthetic_label_maps(case):
    z = _z()
    lab = F.weightmap_synthetic_cases()[case]
    np.testing.assert_array_equal(W.calculate_weight_map(lab), z[case])
