"""GPU input pipeline: the reference's elastic augmentation for a whole batch.

``utils/augmentations.py:4-39`` (``elastic_deform_image_and_mask``) plus the
``utils/dataset.py:84-111`` steps around it (uint8 casts, ``ToTensor``,
``mask > 0``) as three HIP kernels behind ``unet_elastic_deform``
(include/unet_hip.h): two separable fp64 Gaussian passes over the uniform noise
fields and one warp.  The reference spends ~83 ms per 512x512 sample on one CPU
core; here a batch is a few launches on the training
stream.

Randomness: the reference draws ``RandomState(seed).rand(H, W)`` twice per
sample (dx, then dy) with a fresh random seed.  ``noise="numpy"`` reproduces
that draw on the host for given seeds (bit-identical outputs to the reference);
``noise="device"`` draws the same distribution with ``torch.rand`` on the GPU
(no host work; a different stream of numbers, as the reference's own seeds are
random anyway).

    aug = ElasticDeform(alpha=2000, sigma=20)        # scripts/train.py:35-36
    x, target = aug(images_u8, labels_u16)             # (N,1,H,W) fp32, (N,1,H,W) uint8
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


class ElasticDeform:
    def __init__(self, alpha: float = 2000.0, sigma: float = 20.0, noise: str = "device",
                 generator: torch.Generator | None = None):
        if noise not in ("device", "numpy"):
            raise ValueError("noise must be 'device' or 'numpy'")
        self.alpha, self.sigma, self.noise = float(alpha), float(sigma), noise
        self.generator = generator
        self.lib = _lib.load()
        self._ws = None

    def draw_noise(self, n, h, w, device, seeds=None):
        """(n, 2, h, w) fp64 uniform noise: per sample the reference's two
        RandomState(seed).rand(h, w) draws (noise="numpy"), or torch.rand."""
        if self.noise == "numpy":
            if seeds is None:
                seeds = np.random.randint(0, 2 ** 32 - 1, size=n, dtype=np.int64)
            buf = np.empty((n, 2, h, w), np.float64)
            for i, s in enumerate(seeds):
                rs = np.random.RandomState(int(s))
                buf[i, 0] = rs.rand(h, w)
                buf[i, 1] = rs.rand(h, w)
            return torch.from_numpy(buf).to(device, non_blocking=True)
        return torch.rand((n, 2, h, w), dtype=torch.float64, device=device, generator=self.generator)

    def __call__(self, images: torch.Tensor, labels: torch.Tensor, seeds=None, noise: torch.Tensor | None = None,
                 return_image: bool = False):
        """images (N, H, W) uint8, labels (N, H, W) uint16 (instance ids; the
        reference casts them to uint8 before `> 0`), both on the HIP device."""
        if images.device.type != "cuda" or labels.device.type != "cuda":
            raise ValueError("ElasticDeform runs on the HIP device only (no CPU fallback)")
        if images.dtype != torch.uint8 or images.dim() != 3:
            raise ValueError("images must be (N, H, W) uint8")
        if labels.shape != images.shape:
            raise ValueError("labels must match images")
        if labels.dtype != torch.uint16:  # same low 16 bits, reinterpreted
            labels = labels.to(torch.int32).to(torch.int16).view(torch.uint16)
        n, h, w = images.shape
        images, labels = images.contiguous(), labels.contiguous()
        if noise is None:
            noise = self.draw_noise(n, h, w, images.device, seeds)
        noise = noise.to(torch.float64).contiguous()
        if tuple(noise.shape) != (n, 2, h, w):
            raise ValueError(f"noise must be (N, 2, H, W) = {(n, 2, h, w)}")
        need = self.lib.unet_elastic_ws_bytes(n, h, w)
        if self._ws is None or self._ws.numel() < need or self._ws.device != images.device:
            self._ws = torch.empty(need, dtype=torch.uint8, device=images.device)
        x = torch.empty((n, 1, h, w), dtype=torch.float32, device=images.device)
        t = torch.empty((n, 1, h, w), dtype=torch.uint8, device=images.device)
        img = torch.empty((n, h, w), dtype=torch.uint8, device=images.device) if return_image else None
        _lib.check(self.lib.unet_elastic_deform(images.data_ptr(), labels.data_ptr(), n, h, w, noise.data_ptr(),
                                                ctypes.c_double(self.alpha), ctypes.c_double(self.sigma),
                                                x.data_ptr(), t.data_ptr(), img.data_ptr() if img is not None else None,
                                                self._ws.data_ptr(), _lib.stream_of()), "unet_elastic_deform")
        return (x, t, img) if return_image else (x, t)


def weight_maps(labels: torch.Tensor, w0: float = 10.0, sigma: float = 5.0, fp64: bool = False):
    """scripts/preprocess_data.py:17-77 on the device for a batch of label maps
    (N, H, W) (uint16 instance ids, or any integer type): the per-pixel loss
    weights (N, H, W) fp32 utils/dataset.py:111 feeds the loss, and with
    fp64=True also the fp64 map the reference saves as weight_map_*.npy."""
    lib = _lib.load()
    if labels.device.type != "cuda" or labels.dim() != 3:
        raise ValueError("labels must be an (N, H, W) tensor on the HIP device")
    if labels.dtype != torch.uint16:
        labels = labels.to(torch.int32).to(torch.int16).view(torch.uint16)
    labels = labels.contiguous()
    n, h, w = labels.shape
    out = torch.empty((n, h, w), dtype=torch.float32, device=labels.device)
    out64 = torch.empty((n, h, w), dtype=torch.float64, device=labels.device) if fp64 else None
    ws = torch.empty(lib.unet_weight_map_ws_bytes(n), dtype=torch.uint8, device=labels.device)
    _lib.check(lib.unet_weight_map(labels.data_ptr(), n, h, w, ctypes.c_double(w0), ctypes.c_double(sigma),
                                   out.data_ptr(), out64.data_ptr() if out64 is not None else None, ws.data_ptr(),
                                   _lib.stream_of()), "unet_weight_map")
    return (out, out64) if fp64 else out
