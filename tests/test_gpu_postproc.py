"""GPU post-processing (unet_instance_masks / unet_rand_index, unet_amd.postproc)
against the oracle (oracle/postproc_oracle.py): labels bit-exact (numbering
included), Rand index bit-exact (exact integer pair counts)."""
import os

import numpy as np
import pytest

from oracle import postproc_oracle as P

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def pp():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd import postproc
    return postproc


def snake(h, w):
    """One long serpentine component (deep union-find chains) plus specks."""
    m = np.zeros((h, w), np.uint8)
    for y in range(0, h, 4):
        m[y, :] = 1
        if y + 2 < h:
            m[y + 1:y + 3, (w - 1) if (y // 4) % 2 == 0 else 0] = 1
    m[2, 3] = m[h - 2, w // 2] = 1
    return m


@pytest.mark.parametrize("case", ["random30", "random60", "snake", "empty", "full", "hela"])
@pytest.mark.parametrize("min_size", [1, 15])
def test_instance_masks_vs_oracle(pp, case, min_size):
    g = np.random.default_rng(9)
    if case.startswith("random"):
        m = (g.random((3, 97, 130)) < int(case[6:]) / 100).astype(np.uint8) * 255
    elif case == "snake":
        m = snake(64, 75)[None]
    elif case == "empty":
        m = np.zeros((2, 16, 16), np.uint8)
    elif case == "full":
        m = np.ones((2, 9, 31), np.uint8)
    else:  # the reference-run predicted masks of the real HeLa frames (0/255, 324 x 324)
        m = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)["masks"]
    got = pp.instance_masks(torch.from_numpy(m).cuda(), min_size=min_size).cpu().numpy()
    assert got.dtype == np.uint16
    for i in range(m.shape[0]):
        np.testing.assert_array_equal(got[i], P.get_instance_masks(m[i], min_size))


@pytest.mark.parametrize("seed", [0, 1])
def test_rand_index_vs_oracle(pp, seed):
    g = np.random.default_rng(seed)
    h = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)
    gt = h["segs"][seed, 94:418, 94:418].astype(np.uint16)        # 324 x 324 instance GT
    pred = P.get_instance_masks(h["masks"][seed], 15)
    assert pp.rand_index(torch.from_numpy(gt).cuda(), torch.from_numpy(pred).cuda()) == P.rand_index(gt, pred)
    a = g.integers(0, 3000, (61, 47)).astype(np.uint16)
    b = g.integers(0, 5, (61, 47)).astype(np.uint16)
    assert pp.rand_index(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()) == P.rand_index(a, b)
    assert pp.rand_index(torch.from_numpy(a).cuda(), torch.from_numpy(a).cuda()) == (1.0, 0.0)


def test_instance_masks_vs_reference_committed_outputs(pp):
    """get_instance_masks(min_size=15) (scripts/predict.py:92-112,
    utils/metrics.py:42-72) on the reference's own 84 predicted masks
    (01_RES/mask*.tif) must give its committed instance labelings
    (01_RES_INST/m*.tif) bit-exactly, numbering included
    (tests/golden/hela_postproc.npz)."""
    z = np.load(os.path.join(G, "hela_postproc.npz"), allow_pickle=False)
    t, h, w = (int(v) for v in z["mask_shape"])
    masks = (np.unpackbits(z["mask_bits"], axis=-1)[..., :w] * 255).astype(np.uint8)
    got = pp.instance_masks(torch.from_numpy(masks).cuda(), min_size=int(z["min_size"])).cpu().numpy()
    assert got.shape == (t, h, w)
    bad = [i for i in range(t) if not np.array_equal(got[i], z["labels"][i])]
    assert not bad, f"frames differing from the reference: {bad}"
