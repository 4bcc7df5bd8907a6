"""CPU checks of the elastic-deformation oracle (oracle/elastic_oracle.py): its
pieces against scipy.ndimage (the reference's dependency, called exactly as
utils/augmentations.py:25-37 calls it) and the whole function against the
fixtures the reference itself produced (tests/golden/make_golden_elastic.py)."""
import os

import numpy as np
import pytest

from oracle import elastic_oracle as E
from oracle import fixtures as F

G = os.path.join(os.path.dirname(__file__), "golden")
ndi = pytest.importorskip("scipy.ndimage")


@pytest.mark.parametrize("sigma", [20.0, 3.0, 0.7])
def test_gaussian_filter_matches_scipy(sigma):
    f = np.random.default_rng(1).random((70, 90)) * 2 - 1
    ref = ndi.gaussian_filter(f, sigma, mode="constant", cval=0)
    np.testing.assert_allclose(E.gaussian_filter_constant(f, sigma), ref, rtol=0, atol=1e-15)


@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("dtype", [np.uint8, np.uint16])
def test_map_coordinates_reflect_matches_scipy(order, dtype):
    """Far out-of-range coordinates (several reflections), exact integers and
    exact halves (the rounding boundaries of order 0)."""
    g = np.random.default_rng(2)
    hi = 255 if dtype == np.uint8 else 400
    img = g.integers(0, hi + 1, (37, 53)).astype(dtype)
    cy = g.uniform(-120, 160, 50000)
    cx = g.uniform(-150, 200, 50000)
    cy[:500] = g.integers(-80, 120, 500) + 0.5 * g.integers(0, 2, 500)
    cx[:500] = g.integers(-80, 120, 500) + 0.5 * g.integers(0, 2, 500)
    ref = ndi.map_coordinates(img, [cy, cx], order=order, mode="reflect")
    got = E.to_uint(E.map_coordinates_reflect(img, cy, cx, order), dtype)
    np.testing.assert_array_equal(got, ref)


def test_map_coordinates_single_row():
    img = np.arange(7, dtype=np.uint8)[None, :] * 30
    cy = np.array([-3.2, 0.0, 4.7])
    cx = np.array([-9.4, 2.5, 15.2])
    for order in (0, 1):
        ref = ndi.map_coordinates(img, [cy, cx], order=order, mode="reflect")
        np.testing.assert_array_equal(E.to_uint(E.map_coordinates_reflect(img, cy, cx, order), np.uint8), ref)


def _golden():
    return np.load(os.path.join(G, "elastic.npz"), allow_pickle=False)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_oracle_vs_reference_hela_frames(i):
    """Real 512x512 frames, alpha 2000 / sigma 20 (scripts/train.py:35-36),
    noise drawn like the reference (RandomState(seed), dx then dy)."""
    z = _golden()
    h = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)
    nx, ny = E.noise_from_seed(int(z[f"hela{i}_seed"]), (512, 512))
    img, msk = E.elastic_deform(h["images"][i], h["segs"][i], 2000.0, 20.0, nx, ny)
    np.testing.assert_array_equal(img.astype(np.uint8), z[f"hela{i}_img"])
    np.testing.assert_array_equal(msk.astype(np.uint8), z[f"hela{i}_mask"])


@pytest.mark.parametrize("tag", ["syn", "syn_s3"])
def test_oracle_vs_reference_synthetic(tag):
    """Ragged 61x77, labels > 255 (the reference's uint8 cast wraps them)."""
    z = _golden()
    img, lab = F.elastic_synthetic_case()
    nx, ny = E.noise_from_seed(7, img.shape)
    gi, gm = E.elastic_deform(img, lab, 2000.0, float(z[f"{tag}_sigma"]), nx, ny)
    np.testing.assert_array_equal(gi.astype(np.uint8), z[f"{tag}_img"])
    np.testing.assert_array_equal(gm.astype(np.uint8), z[f"{tag}_mask"])


def test_dataset_sample_tensors():
    """utils/dataset.py:98-111: ToTensor scaling and mask > 0."""
    img, lab = F.elastic_synthetic_case()
    nx, ny = E.noise_from_seed(7, img.shape)
    x, t = E.dataset_sample(img, lab, 2000.0, 20.0, nx, ny)
    z = _golden()
    assert x.dtype == np.float32 and t.dtype == np.uint8
    np.testing.assert_array_equal(x, z["syn_img"].astype(np.float32) / np.float32(255))
    np.testing.assert_array_equal(t, (z["syn_mask"] > 0).astype(np.uint8))
