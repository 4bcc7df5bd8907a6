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
driven by its own process.  Each tile batch is an eval-mode forward
(scripts/predict.py:70-82: BatchNorm with running statistics).
"""
from __future__ import annotations

import copy
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


def mirror_pad(img, pads):
    """Reflect padding of an (..., H, W) tensor; pads larger than the image are
    reflected repeatedly (np.pad(mode='reflect') semantics)."""
    top, bottom, left, right = pads
    out = img
    while top or bottom or left or right:
        H, W = out.shape[-2:]
        t, b = min(top, H - 1), min(bottom, H - 1)
        l, r = min(left, W - 1), min(right, W - 1)
        shp = out.shape
        o4 = out.reshape(-1, 1, H, W)
        o4 = F.pad(o4, (l, r, t, b), mode="reflect")
        out = o4.reshape(*shp[:-2], H + t + b, W + l + r)
        top, bottom, left, right = top - t, bottom - b, left - l, right - r
    return out


def extract_tiles(padded, geo, indices):
    """Stack the input tiles (C, tile_in, tile_in) for the given tile indices."""
    ti = geo.tile_in
    return torch.stack([padded[:, y:y + ti, x:x + ti] for (y, x) in (geo.origins[i] for i in indices)])


def rank_share(geo, rank, world):
    """Tile indices processed by `rank` (round-robin deal, no collective)."""
    return list(range(rank, len(geo), world))


@torch.no_grad()
def predict_tiles(model, padded, geo, indices, batch=4):
    """Eval forwards of the listed tiles; returns {index: logits (K, t, t)}."""
    out = {}
    dev = next(model.parameters()).device
    for s in range(0, len(indices), batch):
        idx = indices[s:s + batch]
        x = extract_tiles(padded, geo, idx).to(dev, torch.float32).contiguous()
        logits = model(x)
        for i, lg in zip(idx, logits):
            out[i] = lg
    return out


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
    no collectives)."""

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

    def predict(self, image):
        """image: (C, H, W) or (H, W) float tensor (already normalised the way
        the model was trained, e.g. predict.py's Normalize(0.5, 0.5)).
        Returns (K, H, W) logits on the host."""
        if image.dim() == 2:
            image = image[None]
        C, H, W = image.shape
        geo = TileGeometry(H, W, self.tile_in)
        padded = mirror_pad(image.float(), geo.pads)
        results, errors = {}, []
        lock = threading.Lock()

        def work(k):
            try:
                dev = self.devices[k]
                with torch.cuda.device(dev):
                    local = predict_tiles(self.replicas[k], padded.to(dev), geo,
                                          rank_share(geo, k, len(self.devices)), self.batch)
                    torch.cuda.synchronize(dev)
                with lock:
                    results.update(local)
            except Exception as e:  # surfaced below
                errors.append(e)

        threads = [threading.Thread(target=work, args=(k,)) for k in range(len(self.devices))]
        for th in threads:
            th.start()
        for th in threads:
            th.join()
        if errors:
            raise errors[0]
        return stitch(results, geo, self.n_classes)


def mask_from_logits(logits):
    """scripts/predict.py:85-92: softmax(dim=0)[1] > 0.5  ==  logit1 > logit0 (uint8 0/255)."""
    return ((logits[1] > logits[0]).to(torch.uint8) * 255)
