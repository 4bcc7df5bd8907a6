"""The reference's training data path on the GPU, end to end.

scripts/train.py:69-131 trains on ``HeLaDataset`` (utils/dataset.py:69-115):
per sample it decodes the frame and its instance label map, warps both with
``elastic_deform_image_and_mask`` (utils/augmentations.py:4-39, a fresh random
seed per sample), applies ToTensor (x = image / 255) and ``mask > 0``, and
loads the weight map that scripts/preprocess_data.py:17-77 computed offline
from the UNWARPED labels; the loop then center-crops targets and weights to the
logits' size as views (train.py:118-126) and takes one SGD step.

``HeLaBatches`` keeps the decoded frames and label maps resident in HBM and
produces each minibatch with three device launches (ElasticDeform: two
Gaussian passes + one warp, unet_amd.augment) and, for ``weights="warped"``,
one weight-map launch on the warped labels; ``weights="static"`` (the
reference's semantics) computes the maps of the unwarped labels once, on the
device, and gathers them per batch.  Shuffling and rank sharding follow
DataLoader(shuffle=True) / DistributedSampler (unet_amd.dist.ShardedIndices).

    data = HeLaBatches(images_u8, labels_u16, batch=4, out_hw=trainer.out_hw)
    for x, target, weight in data:              # target / weight: cropped views
        trainer.step(x, target, weight)
"""
from __future__ import annotations

import numpy as np
import torch

from .augment import ElasticDeform, weight_maps
from .dist import ShardedIndices


def center_crop_views(t, out_hw):
    """scripts/train.py:39-51 center_crop_tensor + squeeze(1): (N, 1, H, W) ->
    (N, oh, ow) strided view (no copy), offsets (H - oh) // 2."""
    h, w = t.shape[-2:]
    oh, ow = out_hw
    if oh > h or ow > w:
        raise ValueError(f"cannot crop {(h, w)} to {(oh, ow)}")
    hs, ws = (h - oh) // 2, (w - ow) // 2
    return t[:, :, hs:hs + oh, ws:ws + ow].squeeze(1)


class HeLaBatches:
    """Minibatches of (x (B,1,H,W) fp32, target (B,oh,ow) int64 view,
    weights (B,oh,ow) fp32 view) from device-resident frames.

    images: (N, H, W) uint8 frames; labels: (N, H, W) integer instance ids (the
    man_seg / ST label maps), both on one HIP device.  augment=False gives the
    reference's un-augmented path (x = image / 255, target = label > 0)."""

    def __init__(self, images, labels, batch, out_hw, augment=True, alpha=2000.0, sigma=20.0, noise="device",
                 weights="static", shuffle=True, seed=0, world=1, rank=0, drop_last=False, generator=None):
        if images.device.type != "cuda" or labels.device.type != "cuda":
            raise ValueError("HeLaBatches keeps its frames on the HIP device (no CPU fallback)")
        if images.dtype != torch.uint8 or images.dim() != 3 or tuple(labels.shape) != tuple(images.shape):
            raise ValueError("images must be (N, H, W) uint8 and labels the same shape")
        if weights not in ("static", "warped"):
            raise ValueError("weights must be 'static' (the reference's precomputed maps) or 'warped'")
        self.images = images.contiguous()
        if labels.dtype != torch.uint16:
            # instance ids are uint16 in the reference's man_seg*.tif files; a wider
            # label map must fit that range (65536 would wrap to 0 = background)
            if labels.numel():
                lo, hi = torch.aminmax(labels)
                if int(lo) < 0 or int(hi) > 65535:
                    raise ValueError(f"label ids must lie in [0, 65535] (uint16 instance ids), got [{int(lo)}, {int(hi)}]")
            labels = labels.to(torch.int32).to(torch.int16).view(torch.uint16)
        self.labels = labels.contiguous()
        self.batch, self.out_hw = int(batch), tuple(out_hw)
        self.augment, self.weights, self.drop_last = bool(augment), weights, bool(drop_last)
        self.aug = ElasticDeform(alpha=alpha, sigma=sigma, noise=noise, generator=generator) if augment else None
        self.sampler = ShardedIndices(images.shape[0], world, rank, shuffle=shuffle, seed=seed)
        # preprocess_data.py: maps of the unwarped labels, computed once (device)
        self.static_w = weight_maps(self.labels) if weights == "static" else None
        self._lut = None

    def set_epoch(self, epoch):
        self.sampler.set_epoch(epoch)

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch if self.drop_last else (n + self.batch - 1) // self.batch

    def make_batch(self, idx, seeds=None, noise=None):
        """One minibatch of the frames `idx` (list of ints).  `seeds` (numpy
        noise) or `noise` ((B, 2, H, W) fp64) fix the elastic fields."""
        dev = self.images.device
        sel = torch.as_tensor(np.asarray(idx, dtype=np.int64), device=dev)
        img, lab = self.images.index_select(0, sel), self.labels.index_select(0, sel)
        if self.augment:
            x, t8 = self.aug(img, lab, seeds=seeds, noise=noise)
        else:  # ToTensor + mask > 0 on the undeformed labels (dataset.py:96-104; no uint8 cast without the warp)
            # ToTensor's exact uint8 / 255 (a host-built table: the device's
            # scalar division rounds through a reciprocal)
            if self._lut is None:
                self._lut = (torch.arange(256, dtype=torch.float32) / 255.0).to(dev)
            x = self._lut[img.long()].unsqueeze(1)
            t8 = (lab.view(torch.int16) != 0).to(torch.uint8).unsqueeze(1)
        if self.weights == "static":
            w = self.static_w.index_select(0, sel)
        else:  # maps of the warped binary target (fixes the reference's unwarped maps)
            w = weight_maps(t8[:, 0].to(torch.int16).view(torch.uint16))
        target = center_crop_views(t8.to(torch.int64), self.out_hw)
        weight = center_crop_views(w.unsqueeze(1), self.out_hw)
        return x, target, weight

    def __iter__(self):
        order = self.sampler.indices()
        for b in range(len(self)):
            idx = order[b * self.batch:(b + 1) * self.batch]
            if not idx:
                return
            yield self.make_batch(idx)
