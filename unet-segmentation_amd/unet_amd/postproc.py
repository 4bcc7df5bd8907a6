"""Post-processing on the GPU (utils/metrics.py): instance labelling of
predicted masks and the Rand index, behind unet_instance_masks /
unet_rand_index (include/unet_hip.h).

    labels = instance_masks(mask_u8, min_size=15)   # get_instance_masks (:42-72), uint16
    ri, re = rand_index(gt_labels, labels)           # calculate_rand_index_and_error (:75-139)
"""
from __future__ import annotations

import torch

from . import _lib


def _u16(t):
    if t.dtype == torch.uint16:
        return t.contiguous()
    return t.to(torch.int32).to(torch.int16).view(torch.uint16).contiguous()


def instance_masks(mask: torch.Tensor, min_size: int = 15) -> torch.Tensor:
    """(N, H, W) or (H, W) mask on the HIP device, > 0 = foreground -> uint16
    labels: 8-connected components numbered in raster order of their first
    pixel, components under min_size pixels zeroed (not renumbered)."""
    if mask.device.type != "cuda":
        raise ValueError("instance_masks runs on the HIP device only (no CPU fallback)")
    squeeze = mask.dim() == 2
    m = mask[None] if squeeze else mask
    if m.dim() != 3:
        raise ValueError("mask must be (H, W) or (N, H, W)")
    m = (m > 0).to(torch.uint8).contiguous()
    n, h, w = m.shape
    lib = _lib.load()
    ws = torch.empty(lib.unet_instance_masks_ws_bytes(n, h, w), dtype=torch.uint8, device=m.device)
    out = torch.empty((n, h, w), dtype=torch.uint16, device=m.device)
    _lib.check(lib.unet_instance_masks(m.data_ptr(), n, h, w, int(min_size), out.data_ptr(), ws.data_ptr(),
                                       _lib.stream_of()), "unet_instance_masks")
    return out[0] if squeeze else out


def rand_index(gt: torch.Tensor, pred: torch.Tensor):
    """(Rand index, Rand error) of two (H, W) instance labelings on the device
    (labels < 65536)."""
    if gt.shape != pred.shape or gt.dim() != 2:
        raise ValueError("gt and pred must be (H, W) of the same shape")
    if gt.device.type != "cuda" or pred.device.type != "cuda":
        raise ValueError("rand_index runs on the HIP device only (no CPU fallback)")
    g, p = _u16(gt), _u16(pred)
    h, w = g.shape
    lib = _lib.load()
    ws = torch.empty(lib.unet_rand_index_ws_bytes(h, w), dtype=torch.uint8, device=g.device)
    out = torch.empty(2, dtype=torch.float64, device=g.device)
    _lib.check(lib.unet_rand_index(g.data_ptr(), p.data_ptr(), h, w, out.data_ptr(), ws.data_ptr(),
                                   _lib.stream_of()), "unet_rand_index")
    ri, re = out.tolist()
    return ri, re
