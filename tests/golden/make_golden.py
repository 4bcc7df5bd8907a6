"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where /root/reference exists: it imports the
reference's ``models/unet_model.py`` (UNet) and ``utils/losses.py``
(WeightedCrossEntropyLoss) and runs them in float64 on torch CPU.  The outputs
are committed as small ``.npz`` files (plain arrays, loadable with
``allow_pickle=False``); the reference code itself never leaves this container.

Weights and inputs come from the build-defined counter hash in
``oracle/unet_oracle.py`` (hash_init / hash_uniform) so that the GPU tests can
regenerate them bit-identically without committing 124 MB of weights.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

from oracle import unet_oracle as O  # noqa: E402
from oracle import fixtures as F  # noqa: E402
from models.unet_model import UNet  # noqa: E402  (reference)
from utils.losses import WeightedCrossEntropyLoss  # noqa: E402  (reference)

torch.set_num_threads(os.cpu_count() or 8)
DT = torch.float64


def _t(a):
    return torch.from_numpy(np.array(a, copy=True)).to(DT)


def ref_model(params, n_channels=1, n_classes=2):
    m = UNet(n_channels, n_classes).to(DT)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}
    sd = {k: (v.to(DT) if v.is_floating_point() else v) for k, v in sd.items()}
    m.load_state_dict(sd)
    return m


def digest(name, g, out):
    g = np.asarray(g, np.float64).ravel()
    out[f"gnorm/{name}"] = np.array(np.linalg.norm(g))
    idx = F.sample_indices(name, g.size)
    out[f"gidx/{name}"] = idx
    out[f"gval/{name}"] = g[idx]


def whole_model_case(tag, n, h, n_channels=1, seed=1, steps=0):
    params = O.hash_init(n_channels, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, n_channels, h)
    m = ref_model(params, n_channels)
    m.train()
    crit = WeightedCrossEntropyLoss()
    xt = _t(x)
    out = {"x_seed": np.array(seed), "n": np.array(n), "h": np.array(h), "c": np.array(n_channels)}
    logits = m(xt)
    loss = crit(logits, torch.from_numpy(tgt), _t(wmap))
    loss.backward()
    out["logits"] = logits.detach().numpy()
    out["loss"] = np.array(loss.item())
    for name, p in m.named_parameters():
        digest(name, p.grad.numpy(), out)
    for name, b in m.named_buffers():
        if "running" in name:
            out[f"buf/{name}"] = b.detach().numpy().copy()
    # eval-mode forward with the updated running statistics (scripts/predict.py:70)
    m.eval()
    with torch.no_grad():
        out["logits_eval"] = m(xt).numpy()
    if steps:
        # scripts/train.py:25,97: lr 1e-4, momentum 0.99.  (lr 1e-2 was tried and is
        # chaotic: the reference's own fp32 runs on two CPU backends differ by 68 %
        # at step 4, so it cannot pin anything.)
        m.train()
        p0 = {k: v.detach().clone() for k, v in m.named_parameters()}
        opt = torch.optim.SGD(m.parameters(), lr=1e-4, momentum=0.99)
        losses = []
        for s in range(steps):
            opt.zero_grad()
            lo = crit(m(xt), torch.from_numpy(tgt), _t(wmap))
            lo.backward()
            opt.step()
            losses.append(lo.item())
        for k, v in m.named_parameters():
            out[f"dnorm/{k}"] = np.array(torch.linalg.norm(v.detach() - p0[k]).item())
        out["sgd_lr"] = np.array(1e-4)
        out["sgd_losses"] = np.array(losses)
        with torch.no_grad():
            m.eval()
            out["logits_after_sgd_eval"] = m(xt).numpy()
    path = os.path.join(HERE, f"model_{tag}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def forward_only_case(tag, n, h, n_channels=1, seed=3):
    params = O.hash_init(n_channels, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, n_channels, h)
    m = ref_model(params, n_channels)
    m.train()
    with torch.no_grad():
        logits = m(_t(x))
        loss = WeightedCrossEntropyLoss()(logits, torch.from_numpy(tgt), _t(wmap))
    out = {"x_seed": np.array(seed), "n": np.array(n), "h": np.array(h), "c": np.array(n_channels),
           "loss": np.array(loss.item()),
           # logits are large at 512^2: keep a strided sample + the mask digest
           "logits_sample": logits.numpy()[:, :, ::7, ::5].copy(),
           "mask": (logits[:, 1] > logits[:, 0]).numpy().astype(np.uint8),
           "margin": (logits[:, 1] - logits[:, 0]).abs().numpy().astype(np.float32)}
    path = os.path.join(HERE, f"fwd_{tag}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def op_cases():
    """Per-op fixtures from torch.nn itself (the reference's arithmetic)."""
    rng = np.random.default_rng(1234)
    out = {}
    # conv3x3 valid fwd/bwd (models/unet_model.py:11)
    x = rng.standard_normal((2, 5, 9, 11))
    w = rng.standard_normal((4, 5, 3, 3)) * 0.3
    b = rng.standard_normal(4)
    dy = rng.standard_normal((2, 4, 7, 9))
    conv = torch.nn.Conv2d(5, 4, 3, padding=0).to(DT)
    conv.weight.data = _t(w); conv.bias.data = _t(b)
    xt = _t(x).requires_grad_(True)
    y = conv(xt); y.backward(_t(dy))
    out.update({"conv.x": x, "conv.w": w, "conv.b": b, "conv.dy": dy, "conv.y": y.detach().numpy(),
                "conv.dx": xt.grad.numpy(), "conv.dw": conv.weight.grad.numpy(), "conv.db": conv.bias.grad.numpy()})
    # BatchNorm2d train fwd/bwd + running stats (models/unet_model.py:12)
    x = rng.standard_normal((2, 3, 5, 7)) * 2 + 1
    g = rng.uniform(0.5, 1.5, 3); bb = rng.standard_normal(3)
    dy = rng.standard_normal(x.shape)
    bn = torch.nn.BatchNorm2d(3).to(DT)
    bn.weight.data = _t(g); bn.bias.data = _t(bb)
    xt = _t(x).requires_grad_(True)
    y = bn(xt); y.backward(_t(dy))
    out.update({"bn.x": x, "bn.g": g, "bn.b": bb, "bn.dy": dy, "bn.y": y.detach().numpy(), "bn.dx": xt.grad.numpy(),
                "bn.dg": bn.weight.grad.numpy(), "bn.db": bn.bias.grad.numpy(),
                "bn.rm": bn.running_mean.numpy(), "bn.rv": bn.running_var.numpy()})
    bn.eval()
    with torch.no_grad():
        out["bn.y_eval"] = bn(_t(x)).numpy()
    # MaxPool2d(2), odd size + ties (models/unet_model.py:28)
    x = rng.integers(-2, 3, (2, 3, 7, 9)).astype(np.float64)
    x[0, 0, :2, :2] = 1.0  # all-equal window
    dy = rng.standard_normal((2, 3, 3, 4))
    xt = _t(x).requires_grad_(True)
    y = torch.nn.MaxPool2d(2)(xt); y.backward(_t(dy))
    out.update({"pool.x": x, "pool.dy": dy, "pool.y": y.detach().numpy(), "pool.dx": xt.grad.numpy()})
    # ConvTranspose2d(k=2, s=2) (models/unet_model.py:45)
    x = rng.standard_normal((2, 6, 4, 5))
    w = rng.standard_normal((6, 3, 2, 2)) * 0.3
    b = rng.standard_normal(3)
    dy = rng.standard_normal((2, 3, 8, 10))
    ct = torch.nn.ConvTranspose2d(6, 3, 2, stride=2).to(DT)
    ct.weight.data = _t(w); ct.bias.data = _t(b)
    xt = _t(x).requires_grad_(True)
    y = ct(xt); y.backward(_t(dy))
    out.update({"convT.x": x, "convT.w": w, "convT.b": b, "convT.dy": dy, "convT.y": y.detach().numpy(),
                "convT.dx": xt.grad.numpy(), "convT.dw": ct.weight.grad.numpy(), "convT.db": ct.bias.grad.numpy()})
    # WeightedCrossEntropyLoss (utils/losses.py:29-57)
    lg = rng.standard_normal((2, 2, 5, 6)) * 3
    t = rng.integers(0, 2, (2, 5, 6)).astype(np.int64)
    wm = rng.uniform(10, 13, (2, 5, 6))
    lt = _t(lg).requires_grad_(True)
    lo = WeightedCrossEntropyLoss()(lt, torch.from_numpy(t), _t(wm)); lo.backward()
    out.update({"wce.logits": lg, "wce.t": t, "wce.w": wm, "wce.loss": np.array(lo.item()), "wce.dlogits": lt.grad.numpy()})
    # SGD(momentum=0.99) three steps (scripts/train.py:97,131)
    p0 = rng.standard_normal(17); gs = rng.standard_normal((3, 17))
    pt = torch.nn.Parameter(_t(p0))
    opt = torch.optim.SGD([pt], lr=1e-4, momentum=0.99)
    traj = []
    for s in range(3):
        opt.zero_grad(); pt.grad = _t(gs[s]); opt.step(); traj.append(pt.detach().numpy().copy())
    out.update({"sgd.p0": p0, "sgd.g": gs, "sgd.traj": np.stack(traj)})
    # center crop offsets (models/unet_model.py:88-102) for the 512 path
    path = os.path.join(HERE, "ops.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def real_data_case(n_frames=3):
    """Real HeLa frames (data/raw/train/DIC-C2DH-HeLa/01, 01_ST/SEG) through the
    reference model with hash weights: masks + IoU (utils/metrics.py:6-37)."""
    from PIL import Image
    root = os.path.join(REF, "data/raw/train/DIC-C2DH-HeLa")
    params = O.hash_init(1, 2, seed=7, bn_random=True)
    m = ref_model(params)
    # put plausible running stats in place: one train-mode pass over the frames
    imgs, segs = [], []
    for i in range(n_frames):
        imgs.append(np.array(Image.open(os.path.join(root, "01", f"t{i:03d}.tif")).convert("L")))
        segs.append(np.array(Image.open(os.path.join(root, "01_ST", "SEG", f"man_seg{i:03d}.tif"))))
    imgs = np.stack(imgs)
    segs = np.stack(segs)
    x = imgs.astype(np.float64)[:, None] / 255.0            # ToTensor (dataset.py:96)
    xn = x * 2.0 - 1.0                                       # Normalize(0.5,0.5) (predict.py:50-54)
    # running stats := batch stats of these frames (momentum 1.0), so that the
    # eval-mode masks are not degenerate for hash-initialised weights
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.momentum = 1.0
    m.train()
    with torch.no_grad():
        m(_t(xn))
    m.eval()
    with torch.no_grad():
        logits = m(_t(xn)).numpy()
    masks = O.predict_mask(logits)
    oy = (512 - 324) // 2
    gt = segs[:, oy:oy + 324, oy:oy + 324]
    ious = np.array([O.calculate_iou(masks[i], gt[i]) for i in range(n_frames)])
    bufs = {f"buf/{k}": v.numpy().copy() for k, v in m.state_dict().items() if "running" in k}
    out = {"images": imgs.astype(np.uint8), "segs": segs.astype(np.uint16), "masks": masks,
           "margin": np.abs(logits[:, 1] - logits[:, 0]).astype(np.float32), "ious": ious,
           "seed": np.array(7), **bufs}
    path = os.path.join(HERE, "hela_real.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes", "IoUs", ious)


if __name__ == "__main__":
    which = sys.argv[1:] or ["ops", "m188", "m204", "f512", "f572", "hela"]
    if "ops" in which:
        op_cases()
    if "m188" in which:
        whole_model_case("n2_188", 2, 188, seed=1, steps=3)
    if "m204" in which:
        whole_model_case("n2_204", 2, 204, seed=2)
    if "f512" in which:
        forward_only_case("n1_512", 1, 512, seed=3)
    if "f572" in which:
        forward_only_case("n1_c3_572", 1, 572, n_channels=3, seed=4)
    if "hela" in which:
        real_data_case()
