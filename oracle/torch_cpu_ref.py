"""Torch-CPU restatement of the reference train step, for bench.py's
``cpu_baseline`` leg only.

TEST / MEASUREMENT INFRASTRUCTURE ONLY: bench.py times it on the GPU box's host
cores beside the HIP path; nothing in the product path imports it.  The
reference's own .py files never travel to the GPU box, so the
reference's CPU path is restated here with the same torch CPU kernels it runs
on (oneDNN conv2d / conv_transpose2d, native batch_norm, max_pool2d,
cross_entropy, autograd, torch.optim.SGD):

* forward = models/unet_model.py:105-146 (valid 3x3 convs, BatchNorm2d train,
  ReLU, MaxPool2d(2), ConvTranspose2d(k2, s2), center-crop + cat, 1x1 head);
* loss = utils/losses.py:49-57 (mean of weight_map * cross_entropy(reduction
  "none"));
* step = scripts/train.py:114-131 (zero_grad, forward, loss, backward,
  SGD(lr 1e-4, momentum 0.99).step()).

Written functionally over the reference's state_dict names (hash-initialised
weights, oracle/unet_oracle.hash_init), not as a copy of its module classes.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn.functional as F

from . import unet_oracle as O

_BLOCKS = ("inc", "down1", "down2", "down3", "down4")


def _crop(t, th, tw):
    h, w = t.shape[-2:]
    oy, ox = max(0, (h - th) // 2), max(0, (w - tw) // 2)
    return t[..., oy:oy + th, ox:ox + tw]


class TorchCpuUNet:
    """``dtype=torch.float64`` is the reference's own fp64 run (the golden
    fixtures' arithmetic: tests/golden/make_golden.py runs the reference module
    in float64 on the same torch CPU kernels); the GPU parity tests use it as the
    full-tensor oracle at 512^2, where a NumPy fp64 run would take minutes."""

    def __init__(self, params, n_channels=1, n_classes=2, dtype=torch.float32, training=True):
        # training=False: BatchNorm on the running statistics (model.eval(),
        # scripts/predict.py:70), differentiable like reference autograd's
        self.training = training
        self.p = {}
        for k, v in params.items():
            t = torch.from_numpy(np.array(v, copy=True))
            self.p[k] = t.to(dtype) if t.is_floating_point() else t
        for k, v in self.p.items():
            if v.is_floating_point() and not O.is_buffer(k):
                v.requires_grad_(True)

    def parameters(self):
        return [v for k, v in self.p.items() if v.requires_grad]

    def _dc(self, pre, x):
        for conv, bn in (("0", "1"), ("3", "4")):
            x = F.conv2d(x, self.p[f"{pre}{conv}.weight"], self.p[f"{pre}{conv}.bias"])
            b = f"{pre}{bn}"
            x = F.batch_norm(x, self.p[f"{b}.running_mean"], self.p[f"{b}.running_var"], self.p[f"{b}.weight"],
                             self.p[f"{b}.bias"], training=self.training, momentum=0.1, eps=1e-5)
            x = F.relu(x)
        return x

    def forward(self, x):
        skips = []
        for i, blk in enumerate(_BLOCKS):
            if i > 0:
                x = F.max_pool2d(x, 2)
            x = self._dc(O._dc_prefix(blk), x)
            skips.append(x)
        x = skips.pop()
        for k in range(1, 5):
            up = f"up{k}"
            x = F.conv_transpose2d(x, self.p[f"{up}.up.weight"], self.p[f"{up}.up.bias"], stride=2)
            s = skips.pop()
            x = torch.cat([_crop(s, x.shape[-2], x.shape[-1]), x], dim=1)
            x = self._dc(O._dc_prefix(up), x)
        return F.conv2d(x, self.p["outc.conv.weight"], self.p["outc.conv.bias"])


def weighted_ce(logits, target, weights):
    return (F.cross_entropy(logits, target, reduction="none") * weights).mean()


def train_steps_per_second(batch, size=512, seconds=10.0, max_steps=3, threads=None, seed=0):
    """Images/s of scripts/train.py steps (batch x 1 x size^2, fp32) on this
    host's cores; at least one step, then until `seconds` or `max_steps`."""
    if threads:
        torch.set_num_threads(threads)
    from . import fixtures as Fx
    params = O.hash_init(1, 2, seed=seed)
    net = TorchCpuUNet(params)
    x, t, w = Fx.make_inputs(seed, batch, 1, size)
    x, t, w = torch.from_numpy(x), torch.from_numpy(t), torch.from_numpy(w)
    opt = torch.optim.SGD(net.parameters(), lr=1e-4, momentum=0.99)
    steps, t0 = 0, time.perf_counter()
    while True:
        opt.zero_grad()
        loss = weighted_ce(net.forward(x), t, w)
        loss.backward()
        opt.step()
        steps += 1
        el = time.perf_counter() - t0
        if el > seconds or steps >= max_steps:
            break
    return batch * steps / el, steps, el


def train_step_times(batch, steps, size=512, seed=0):
    """Per-step wall times (s) of `steps` scripts/train.py steps at
    batch x 1 x size^2 on this host (the optimizer state carries over)."""
    from . import fixtures as Fx
    params = O.hash_init(1, 2, seed=seed)
    net = TorchCpuUNet(params)
    x, t, w = Fx.make_inputs(seed, batch, 1, size)
    x, t, w = torch.from_numpy(x), torch.from_numpy(t), torch.from_numpy(w)
    opt = torch.optim.SGD(net.parameters(), lr=1e-4, momentum=0.99)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        opt.zero_grad()
        loss = weighted_ce(net.forward(x), t, w)
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
    return batch, times
