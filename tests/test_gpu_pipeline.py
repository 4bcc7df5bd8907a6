"""The reference's training loop end to end on the GPU (scripts/train.py:69-131
with augment=True): device-resident DIC-C2DH-HeLa 01 frames -> elastic warp
(utils/augmentations.py:4-39) -> ToTensor / mask > 0 (utils/dataset.py:84-111)
-> weight maps (scripts/preprocess_data.py:17-77) -> center-cropped views
(train.py:118-126) -> Trainer steps (unet_amd.pipeline.HeLaBatches).

Each link is checked on the data that actually flows through the chain: the
warp bit-exact against the reference's own outputs for the same seeds
(tests/golden/elastic.npz), the weight maps bit-exact against the oracle, the
first step's logits / loss against the NumPy fp64 oracle on those tensors,
and the Trainer's gradients against the autograd drop-in on the same batch."""
import os

import numpy as np
import pytest

from oracle import unet_oracle as O
from oracle import weightmap_oracle as WM

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def hela():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    zr = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)
    ze = np.load(os.path.join(G, "elastic.npz"), allow_pickle=False)
    return zr, ze


def _model(params):
    from unet_amd import UNet
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    return m.cuda().train()


def test_static_weights_are_the_preprocessed_maps(hela):
    """weights="static": the maps of the UNWARPED labels (what the reference's
    dataset loads from weight_map_*.npy), computed once on the device."""
    from unet_amd.pipeline import HeLaBatches
    zr, _ = hela
    imgs = torch.from_numpy(zr["images"]).cuda()
    labs = torch.from_numpy(zr["segs"].astype(np.int32)).cuda()
    data = HeLaBatches(imgs, labs, batch=2, out_hw=(324, 324), augment=False, shuffle=False)
    x, t, w = data.make_batch([2, 0])
    for j, i in enumerate([2, 0]):
        ref_w = WM.training_weights(zr["segs"][i])[94:418, 94:418]
        np.testing.assert_array_equal(w[j].cpu().numpy(), ref_w)
        np.testing.assert_array_equal(t[j].cpu().numpy(), (zr["segs"][i][94:418, 94:418] > 0).astype(np.int64))
        np.testing.assert_array_equal(x[j, 0].cpu().numpy(), zr["images"][i].astype(np.float32) / np.float32(255))
    assert t.dtype == torch.int64 and not t.is_contiguous() and not w.is_contiguous()   # views, as train.py
    # one epoch covers every frame once (DataLoader(shuffle=True) semantics)
    seen = []
    for xb, tb, wb in HeLaBatches(imgs, labs, batch=2, out_hw=(324, 324), augment=False, seed=3):
        seen.append(xb.shape[0])
    assert sum(seen) == 3 and seen == [2, 1]


@pytest.mark.parametrize("weights", ["warped", "static"])
def test_augmented_chain_into_trainer(hela, weights):
    from unet_amd import WeightedCrossEntropyLoss
    from unet_amd.pipeline import HeLaBatches
    from unet_amd.train import Trainer
    zr, ze = hela
    imgs = torch.from_numpy(zr["images"]).cuda()
    labs = torch.from_numpy(zr["segs"]).cuda()
    data = HeLaBatches(imgs, labs, batch=3, out_hw=(324, 324), augment=True, noise="numpy", weights=weights)
    seeds = [int(ze[f"hela{i}_seed"]) for i in range(3)]
    x, t, w = data.make_batch([0, 1, 2], seeds=seeds)
    torch.cuda.synchronize()
    # 1. the warp: the reference's own outputs for these seeds, bit-exact
    xn, tn, wn = x.cpu().numpy()[:, 0], t.cpu().numpy(), w.cpu().numpy()
    for i in range(3):
        np.testing.assert_array_equal(xn[i], ze[f"hela{i}_img"].astype(np.float32) / np.float32(255))
        np.testing.assert_array_equal(tn[i], (ze[f"hela{i}_mask"][94:418, 94:418] > 0).astype(np.int64))
        src = (ze[f"hela{i}_mask"] > 0) if weights == "warped" else zr["segs"][i]
        np.testing.assert_array_equal(wn[i], WM.training_weights(src)[94:418, 94:418])
    # 2. two train steps on the chain's tensors (cropped views straight from the pipeline)
    params = O.hash_init(1, 2, seed=11, bn_random=True)
    tr = Trainer(_model(params), 3, 512, 512, lr=1e-4, momentum=0.99)
    l0 = tr.forward_loss(x, t, w)
    tr.backward_and_reduce(x)
    torch.cuda.synchronize()
    lg = tr.logits.double().cpu().numpy()
    loss0 = float(l0.item())
    names = [k for k, _ in tr.model.named_parameters()]
    g_tr = {k: v.detach().clone() for k, v in zip(names, tr.flat.grad_views)}
    # the NumPy fp64 oracle forward + loss on exactly these inputs
    net = O.UNetOracle(params)
    rl, _, _ = net.forward(xn[:, None].astype(np.float64))
    rloss, _ = O.weighted_ce(rl, tn, wn.astype(np.float64))
    assert np.abs(lg - rl).max() <= 1e-3
    assert abs(loss0 - rloss) <= 1e-4 * abs(rloss)
    # the autograd drop-in on the same batch and weights
    a = _model(params)
    la = WeightedCrossEntropyLoss()(a(x), t, w)
    la.backward()
    assert abs(la.item() - loss0) <= 1e-5 * abs(loss0)
    for k in names:
        if O.bn_cancelled(k):
            continue
        ga = dict(a.named_parameters())[k].grad
        assert float((ga - g_tr[k]).abs().max()) <= 1e-4 * float(ga.abs().max()), k
    tr.optimizer_step()
    # the SGD step moved the loss on this batch down; then a step on a fresh
    # augmented batch (device noise) straight from the iterator
    assert float(tr.forward_loss(x, t, w).item()) < loss0
    data.noise = "device"
    data.aug.noise = "device"
    x2, t2, w2 = next(iter(data))
    assert x2.shape == (3, 1, 512, 512) and t2.shape == (3, 324, 324)
    assert np.isfinite(float(tr.step(x2, t2, w2).item()))
