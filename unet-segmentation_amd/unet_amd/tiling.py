"""Overlap-tile inference (the U-Net paper's strategy; the reference only
computes its margin, scripts/predict1.py:35-49 -- the tiled script it mentions,
images/old readme unet.txt:79, is absent).

A valid U-Net maps a tile_in x tile_in tile to tile_out x tile_out with
tile_out = tile_in - 184 for clean sizes (models/unet_model.py:189), i.e. a
margin of 92-94 px per side.  The image is mirror-padded (reflect) by the
margin on the top/left and so that the bottom/right tiles are full; the output
tiles then tile the image exactly with no overlap, so stitching is a copy.

Tiles are farmed over GPUs with no collective: ``TileFarm`` runs one model
replica per device (one host thread each, HIP calls release the GIL) and deals
tiles round-robin; ``rank_share`` gives the tiles of one rank when each GPU is
driven by its own process.  On the device, ``unet_tile_gather`` reads each tile
batch straight from the unpadded image (mirror folded into the index),
each batch is an eval-mode forward (scripts/predict.py:70-82: BatchNorm with
running statistics), and ``unet_tile_scatter`` writes the tile logits -- or the
uint8 mask directly -- into the full image.
"""
from __future__ import annotations

import copy
import functools
import threading

import torch
import torch.nn.functional as F


def output_size(tile_in: int) -> int:
    """Spatial output of the valid U-Net for a square input (raises when the
    input cannot pass 4 valid down stages)."""
    s = tile_in - 4
    sizes = [s]
    for _ in range(4):
        s = s // 2 - 4
        if s < 1:
            raise ValueError(f"tile {tile_in} too small")
        sizes.append(s)
    u = sizes[-1]
    for k in range(4):
        u = 2 * u
        if sizes[3 - k] < u:
            raise ValueError(f"tile {tile_in}: skip smaller than the upsampled map")
        u -= 4
    return u


class TileGeometry:
    def __init__(self, height, width, tile_in=512):
        self.H, self.W, self.tile_in = height, width, tile_in
        self.tile_out = output_size(tile_in)
        self.margin = (tile_in - self.tile_out) // 2
        self.ny = -(-height // self.tile_out)
        self.nx = -(-width // self.tile_out)
        m, t = self.margin, self.tile_out
        # (top, bottom, left, right) mirror padding
        self.pads = (m, self.ny * t - height + (tile_in - t - m), m, self.nx * t - width + (tile_in - t - m))
        self.origins = [(ty * t, tx * t) for ty in range(self.ny) for tx in range(self.nx)]

    def __len__(self):
        return len(self.origins)


def mirror_index(n_out, start, n):
    """Indices of a whole-sample-symmetric extension (np.pad 'reflect',
    repeated for pads beyond the image; a length-1 axis repeats its sample):
    position start + i of the infinite mirrored axis, i < n_out."""
    i = torch.arange(start, start + n_out)
    if n == 1:
        return torch.zeros_like(i)
    p = 2 * n - 2
    i = torch.remainder(i, p)
    return torch.where(i < n, i, p - i)


def mirror_pad(img, pads):
    """Mirror padding of an (..., H, W) tensor on the host (the geometry
    reference of unet_tile_gather, which folds the same indices on the GPU)."""
    top, bottom, left, right = pads
    H, W = img.shape[-2:]
    iy = mirror_index(H + top + bottom, -top, H).to(img.device)
    ix = mirror_index(W + left + right, -left, W).to(img.device)
    return img.index_select(-2, iy).index_select(-1, ix)


def extract_tiles(padded, geo, indices):
    """Stack the input tiles (C, tile_in, tile_in) for the given tile indices."""
    ti = geo.tile_in
    return torch.stack([padded[:, y:y + ti, x:x + ti] for (y, x) in (geo.origins[i] for i in indices)])


def rank_share(geo, rank, world):
    """Tile indices processed by `rank` (round-robin deal, no collective)."""
    return list(range(rank, len(geo), world))


def stitch(results, geo, n_classes):
    """Assemble {index: (K, t, t)} tiles into (K, H, W) logits (host memory)."""
    t = geo.tile_out
    full = torch.empty((n_classes, geo.ny * t, geo.nx * t), dtype=torch.float32)
    for i, lg in results.items():
        y, x = geo.origins[i]
        full[:, y:y + t, x:x + t] = lg.detach().float().cpu()
    return full[:, :geo.H, :geo.W]


class TileFarm:
    """Overlap-tile inference of large images farmed over several GPUs of one
    process (one replica + one host thread per device, tiles dealt round-robin,
    no collectives).  On each device the tiles are gathered from the unpadded
    image with the mirror padding folded into the index (unet_tile_gather) and
    the tile logits are scattered into the device's full-image logits / mask
    (unet_tile_scatter): no padded copy, no per-tile host traffic."""

    def __init__(self, model, devices=None, tile_in=512, batch=4):
        if devices is None:
            devices = list(range(torch.cuda.device_count()))
        self.devices = [torch.device("cuda", d) if isinstance(d, int) else torch.device(d) for d in devices]
        self.tile_in, self.batch = tile_in, batch
        self.n_classes = model.n_classes
        self.replicas = []
        for d in self.devices:
            r = copy.deepcopy(model).to(d).eval()
            self.replicas.append(r)

    @torch.no_grad()
    def _run_device(self, k, image, geo, want_logits, want_mask):
        from . import _lib
        lib = _lib.load()
        dev, model = self.devices[k], self.replicas[k]
        world = len(self.devices)
        C, H, W = image.shape
        img = image.to(dev, torch.float32).contiguous()
        K = self.n_classes
        full = torch.zeros((K, H, W), dtype=torch.float32, device=dev) if want_logits else None
        mask = torch.zeros((H, W), dtype=torch.uint8, device=dev) if want_mask else None
        mine = rank_share(geo, k, world)
        ti, to, top, left = geo.tile_in, geo.tile_out, geo.pads[0], geo.pads[2]
        tiles = torch.empty((self.batch, C, ti, ti), dtype=torch.float32, device=dev)
        for s in range(0, len(mine), self.batch):
            nb = min(self.batch, len(mine) - s)
            st = _lib.stream_of(dev)
            _lib.check(lib.unet_tile_gather(img.data_ptr(), C, H, W, ti, to, top, left, geo.nx, mine[s], world, nb,
                                            tiles.data_ptr(), st), "unet_tile_gather")
            logits = model(tiles[:nb]).contiguous()
            _lib.check(lib.unet_tile_scatter(logits.data_ptr(), K, to, geo.nx, mine[s], world, nb, H, W,
                                             full.data_ptr() if full is not None else None,
                                             mask.data_ptr() if mask is not None else None, st), "unet_tile_scatter")
        return full, mask

    def predict(self, image, return_mask=False):
        """image: (C, H, W) or (H, W) float tensor (already normalised the way
        the model was trained, e.g. predict.py's Normalize(0.5, 0.5)).
        Returns (K, H, W) logits on the host, or with return_mask=True the
        (H, W) uint8 mask (255 * (l1 > l0), scripts/predict.py:85-92)."""
        if image.dim() == 2:
            image = image[None]
        C, H, W = image.shape
        geo = TileGeometry(H, W, self.tile_in)
        if return_mask and self.n_classes != 2:
            raise ValueError("the mask needs 2 classes")
        outs, errors = [None] * len(self.devices), []

        def work(k):
            try:
                with torch.cuda.device(self.devices[k]):
                    outs[k] = self._run_device(k, image, geo, not return_mask, return_mask)
                    torch.cuda.synchronize(self.devices[k])
            except Exception as e:  # surfaced below
                errors.append(e)

        threads = [threading.Thread(target=work, args=(k,)) for k in range(len(self.devices))]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        if errors:
            raise errors[0]
        # every pixel belongs to exactly one device's tiles; the others hold 0 there
        if return_mask:
            return functools.reduce(torch.maximum, [m.cpu() for _, m in outs])
        return functools.reduce(torch.add, [f.cpu() for f, _ in outs])


def mask_from_logits(logits):
    """scripts/predict.py:85-92: softmax(dim=0)[1] > 0.5  ==  logit1 > logit0 (uint8 0/255)."""
    return ((logits[1] > logits[0]).to(torch.uint8) * 255)
