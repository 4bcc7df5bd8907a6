"""Cell tracking over instance labelings (scripts/track.py:103-275) on the
MI355X: the per-frame object overlaps come from one GPU pass
(unet_tracker_add_frame), the lineage logic runs in the library's native
host tracker.

    tr = Tracker(h, w)                 # IOU 0.3 / 0.1, <= 2 children (track.py:21-24)
    for frame, labels in enumerate(instance_label_maps):   # (h, w) uint16 on the device
        tr.add_frame(labels, frame)
    rows = tr.tracks()                 # (n, 4) int32: label start end parent
    track_sequence(instance_masks_dir, output_track_file)  # the reference's entry point
"""
from __future__ import annotations

import ctypes
import glob
import os

import numpy as np
import torch

from . import _lib
from .postproc import _u16


class Tracker:
    def __init__(self, height, width, iou_track=0.3, iou_division=0.1, max_children=2, device=None):
        self.lib = _lib.load()
        self.h, self.w = int(height), int(width)
        self.handle = self.lib.unet_tracker_create(self.h, self.w, float(iou_track), float(iou_division),
                                                   int(max_children))
        if not self.handle:
            raise ValueError(f"unet_tracker_create({height}, {width}, ...) rejected the arguments")
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.ws = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self.lib.unet_tracker_destroy(h)
            self.handle = None

    def add_frame(self, labels: torch.Tensor, frame: int):
        """One frame's instance labeling (h, w), integer labels < 65536, on the
        HIP device (0 = background)."""
        if labels.device.type != "cuda":
            raise ValueError("Tracker.add_frame runs on the HIP device only (no CPU fallback)")
        if tuple(labels.shape) != (self.h, self.w):
            raise ValueError(f"labels must be ({self.h}, {self.w}), got {tuple(labels.shape)}")
        if labels.dtype != torch.uint16 and labels.numel():
            # the device tables index labels as uint16: a wider label would wrap
            # (e.g. 65536 -> 0 = background, or merge with another object)
            lo, hi = torch.aminmax(labels)
            if int(lo) < 0 or int(hi) >= 65536:
                raise ValueError(f"labels must lie in [0, 65535], got [{int(lo)}, {int(hi)}]")
        lab = _u16(labels)
        if self.ws is None:
            self.ws = torch.empty(self.lib.unet_tracker_ws_bytes(self.h, self.w), dtype=torch.uint8,
                                  device=lab.device)
        _lib.check(self.lib.unet_tracker_add_frame(self.handle, lab.data_ptr(), int(frame), self.ws.data_ptr(),
                                                   _lib.stream_of(lab.device)), "unet_tracker_add_frame")

    def tracks(self) -> np.ndarray:
        n = self.lib.unet_tracker_num_tracks(self.handle)
        out = np.zeros((max(n, 0), 4), np.int32)
        _lib.check(0 if self.lib.unet_tracker_tracks(self.handle, out.ctypes.data_as(ctypes.c_void_p), n) == n
                   else -1, "unet_tracker_tracks")
        return out


def write_track_file(rows, path):
    """res_track.txt, one "label start end parent" line per track (track.py:265-272)."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        for r in rows:
            f.write(f"{int(r[0])} {int(r[1])} {int(r[2])} {int(r[3])}\n")


def track_sequence(instance_masks_dir, output_track_file, device=None):
    """scripts/track.py:103 track_sequence: reads mXXX.tif (sorted), tracks,
    writes output_track_file.  Returns the rows (None when no mask is found)."""
    from PIL import Image
    files = sorted(glob.glob(os.path.join(instance_masks_dir, "m*.tif")))
    if not files:
        print(f"Error: No instance masks (mXXX.tif) found in {instance_masks_dir}.")
        return None
    dev = torch.device("cuda") if device is None else torch.device(device)
    tr = None
    for path in files:
        frame = int(os.path.basename(path)[1:4])
        m = np.array(Image.open(path))
        if tr is None:
            tr = Tracker(m.shape[0], m.shape[1], device=dev)
        tr.add_frame(torch.from_numpy(m.astype(np.int32)).to(dev), frame)
    rows = tr.tracks()
    write_track_file(rows, output_track_file)
    return rows
