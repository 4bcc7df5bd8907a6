"""CPU checks of the post-processing oracle (oracle/postproc_oracle.py):
8-connected labelling against scipy.ndimage.label (scikit-image, the
reference's dependency, is not installed; scipy numbers components the same
way), small-object removal, and the Rand index against brute-force pair
counting and known answers."""
import numpy as np
import pytest

from oracle import postproc_oracle as P

ndi = pytest.importorskip("scipy.ndimage")


@pytest.mark.parametrize("density,shape", [(0.3, (40, 57)), (0.55, (33, 20)), (0.8, (25, 64)), (0.0, (5, 5)),
                                           (1.0, (7, 9))])
def test_label8_matches_scipy(density, shape):
    m = np.random.default_rng(int(density * 100) + shape[0]).random(shape) < density
    ref, _ = ndi.label(m, structure=np.ones((3, 3), int))
    np.testing.assert_array_equal(P.label8(m), ref)


def test_remove_small_objects_keeps_numbering():
    m = np.zeros((10, 12), np.uint8)
    m[0:2, 0:2] = 1      # 4 px  -> label 1 (removed at min_size 5)
    m[5:9, 5:10] = 1     # 20 px -> label 2
    m[0, 11] = 1         # 1 px  -> label 3? raster order: (0,11) comes before (5,5)
    lab = P.label8(m)
    assert lab[0, 0] == 1 and lab[0, 11] == 2 and lab[5, 5] == 3
    out = P.get_instance_masks(m, min_size=5)
    assert out.dtype == np.uint16
    assert out[0, 0] == 0 and out[0, 11] == 0 and out[5, 5] == 3


def _brute_rand(g, p):
    g, p = g.ravel(), p.ravel()
    n = g.size
    agree = 0
    for i in range(n):
        for j in range(i + 1, n):
            agree += (g[i] == g[j]) == (p[i] == p[j])
    return agree / (n * (n - 1) / 2)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_rand_index_vs_pair_counting(seed):
    r = np.random.default_rng(seed)
    g = r.integers(0, 4, (6, 9))
    p = r.integers(0, 5, (6, 9))
    ri, re = P.rand_index(g, p)
    assert ri == pytest.approx(_brute_rand(g, p), abs=1e-15)
    assert re == 1.0 - ri


def test_rand_index_known_answers():
    g = np.array([[1, 1, 2, 2]])
    assert P.rand_index(g, g) == (1.0, 0.0)
    assert P.rand_index(g, g * 7 + 3) == (1.0, 0.0)   # relabelling does not matter
    # pairs: (0,1) same/same, (2,3) same/diff, others diff/diff except (1,2) diff/same
    assert P.rand_index(g, np.array([[5, 5, 5, 6]]))[0] == pytest.approx(3 / 6)
    assert P.rand_index(np.array([[3]]), np.array([[4]])) == (1.0, 0.0)


def test_oracle_instance_masks_vs_reference_committed_outputs():
    """The CC oracle reproduces the reference's committed 01_RES_INST labelings
    from its 01_RES masks (84 frames) -- pins the restatement to the
    reference's own outputs, not only to scipy.ndimage.label."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "hela_postproc.npz"), allow_pickle=False)
    t, h, w = (int(v) for v in z["mask_shape"])
    masks = (np.unpackbits(z["mask_bits"], axis=-1)[..., :w] * 255).astype(np.uint8)
    for i in range(t):
        np.testing.assert_array_equal(P.get_instance_masks(masks[i], int(z["min_size"])), z["labels"][i])
