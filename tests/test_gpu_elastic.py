"""GPU elastic-deformation pipeline (unet_elastic_deform / unet_amd.augment)
against the reference's own outputs (tests/golden/elastic.npz, made by
importing utils/augmentations.py) and the oracle (oracle/elastic_oracle.py).

Bar: bit-exact.  Every rounding decision (bilinear value -> uint8, nearest
coordinate -> label) is taken in fp64 in the oracle's operation order, so the
deformed image, the target and x = image / 255 match exactly."""
import os

import numpy as np
import pytest

from oracle import elastic_oracle as E
from oracle import fixtures as F

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def aug():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd.augment import ElasticDeform
    return ElasticDeform


def run(aug_cls, images, labels, noise, sigma=20.0, alpha=2000.0):
    a = aug_cls(alpha=alpha, sigma=sigma)
    x, t, img = a(torch.from_numpy(np.ascontiguousarray(images)).cuda(),
                  torch.from_numpy(np.ascontiguousarray(labels)).cuda(),
                  noise=torch.from_numpy(np.ascontiguousarray(noise)).cuda(), return_image=True)
    torch.cuda.synchronize()
    return x.cpu().numpy()[:, 0], t.cpu().numpy()[:, 0], img.cpu().numpy()


def test_hela_frames_vs_reference(aug):
    """The three real 512x512 frames in ONE batched call, noise drawn like the
    reference (RandomState(seed).rand, dx then dy), alpha 2000 / sigma 20."""
    z = np.load(os.path.join(G, "elastic.npz"), allow_pickle=False)
    h = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)
    noise = np.stack([np.stack(E.noise_from_seed(int(z[f"hela{i}_seed"]), (512, 512))) for i in range(3)])
    x, t, img = run(aug, h["images"], h["segs"], noise)
    for i in range(3):
        np.testing.assert_array_equal(img[i], z[f"hela{i}_img"])
        np.testing.assert_array_equal(t[i], (z[f"hela{i}_mask"] > 0).astype(np.uint8))
        np.testing.assert_array_equal(x[i], z[f"hela{i}_img"].astype(np.float32) / np.float32(255))


@pytest.mark.parametrize("tag", ["syn", "syn_s3"])
def test_synthetic_vs_reference(aug, tag):
    """Ragged 61x77, labels above 255 (uint8 wrap), sigma 20 and 3."""
    z = np.load(os.path.join(G, "elastic.npz"), allow_pickle=False)
    img, lab = F.elastic_synthetic_case()
    noise = np.stack(E.noise_from_seed(7, img.shape))[None]
    x, t, gi = run(aug, img[None], lab[None], noise, sigma=float(z[f"{tag}_sigma"]))
    np.testing.assert_array_equal(gi[0], z[f"{tag}_img"])
    np.testing.assert_array_equal(t[0], (z[f"{tag}_mask"] > 0).astype(np.uint8))


@pytest.mark.parametrize("n,h,w,sigma,alpha", [(3, 100, 37, 5.0, 300.0), (2, 33, 128, 20.0, 2000.0),
                                               (1, 1, 64, 2.0, 50.0), (2, 257, 300, 11.3, 900.0)])
def test_batch_vs_oracle(aug, n, h, w, sigma, alpha):
    """Per-sample oracle vs one batched launch; single-row images, grids not
    multiples of the 64 / 256 tiles, non-integer sigma."""
    g = np.random.default_rng(n * 1000 + h)
    images = g.integers(0, 256, (n, h, w)).astype(np.uint8)
    labels = g.integers(0, 700, (n, h, w)).astype(np.uint16)
    noise = g.random((n, 2, h, w))
    x, t, gi = run(aug, images, labels, noise, sigma=sigma, alpha=alpha)
    for i in range(n):
        rx, rt = E.dataset_sample(images[i], labels[i], alpha, sigma, noise[i, 0], noise[i, 1])
        np.testing.assert_array_equal(x[i], rx)
        np.testing.assert_array_equal(t[i], rt)


def test_device_noise_matches_oracle_on_the_same_draw(aug):
    """noise="device" (torch.rand on the GPU): the outputs are the oracle's on
    the fields actually drawn."""
    from unet_amd.augment import ElasticDeform
    a = ElasticDeform(noise="device", generator=torch.Generator(device="cuda").manual_seed(3))
    g = np.random.default_rng(5)
    images = g.integers(0, 256, (2, 96, 80)).astype(np.uint8)
    labels = g.integers(0, 20, (2, 96, 80)).astype(np.uint16)
    noise = a.draw_noise(2, 96, 80, "cuda")
    x, t = a(torch.from_numpy(images).cuda(), torch.from_numpy(labels).cuda(), noise=noise)
    nz = noise.cpu().numpy()
    assert 0.45 < nz.mean() < 0.55
    for i in range(2):
        rx, rt = E.dataset_sample(images[i], labels[i], 2000.0, 20.0, nz[i, 0], nz[i, 1])
        np.testing.assert_array_equal(x[i, 0].cpu().numpy(), rx)
        np.testing.assert_array_equal(t[i, 0].cpu().numpy(), rt)


def test_errors(aug):
    a = aug(sigma=200.0)  # radius 800 > 160
    im = torch.zeros((1, 8, 8), dtype=torch.uint8, device="cuda")
    with pytest.raises(RuntimeError):
        a(im, torch.zeros((1, 8, 8), dtype=torch.int32, device="cuda"))
    with pytest.raises(ValueError):
        aug()(im.cpu(), torch.zeros((1, 8, 8), dtype=torch.int32))
