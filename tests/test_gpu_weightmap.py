"""GPU weight maps (unet_weight_map / unet_amd.augment.weight_maps) against the
reference's calculate_weight_map outputs (tests/golden/weightmap.npz): the fp64
map bit-exact, the fp32 training weights = its fp32 cast."""
import os

import numpy as np
import pytest

from oracle import weightmap_oracle as W
from oracle import fixtures as F

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def wm():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd.augment import weight_maps
    return weight_maps


def test_hela_batch(wm):
    z = np.load(os.path.join(G, "weightmap.npz"), allow_pickle=False)
    segs = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)["segs"]
    w32, w64 = wm(torch.from_numpy(segs).cuda(), fp64=True)
    for i in range(3):
        np.testing.assert_array_equal(w64[i].cpu().numpy(), z[f"hela{i}"])
        np.testing.assert_array_equal(w32[i].cpu().numpy(), z[f"hela{i}"].astype(np.float32))


@pytest.mark.parametrize("case", ["multi", "one", "empty", "full"])
def test_synthetic(wm, case):
    z = np.load(os.path.join(G, "weightmap.npz"), allow_pickle=False)
    lab = F.weightmap_synthetic_cases()[case]
    w32, w64 = wm(torch.from_numpy(lab[None]).cuda(), fp64=True)
    np.testing.assert_array_equal(w64[0].cpu().numpy(), z[case])


def test_ragged_batch_int_labels(wm):
    g = np.random.default_rng(3)
    lab = g.integers(0, 4, (5, 37, 301)).astype(np.int64)
    lab[2] = 0
    w32 = wm(torch.from_numpy(lab).cuda())
    for i in range(5):
        np.testing.assert_array_equal(w32[i].cpu().numpy(), W.training_weights(lab[i]))
