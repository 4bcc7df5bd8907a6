"""Golden fixtures for instance masks and cell tracking, taken from the
reference's OWN committed outputs (no reference code is copied):

* ``01_RES/mask*.tif`` (84 predicted binary masks, 324x324 uint8 0/255) and
  ``01_RES_INST/m*.tif`` (their instance labelings, uint16): the input and
  output of ``get_instance_masks(min_size=15)`` (scripts/predict.py:92-112,
  utils/metrics.py:42-72);
* ``01/res_track.txt`` (10,807 tracks "label start end parent"): the output of
  ``track_sequence`` (scripts/track.py:103-275) over those 84 instance masks.

With ``--verify-track`` it also imports the reference's scripts/track.py in this
container and re-runs ``track_sequence`` on ``01_RES_INST`` into /tmp, checking
that the committed res_track.txt is what the reference produces from the
committed masks (the pair is consistent, so it pins the restatement).

Usage:  python tests/golden/make_golden_postproc.py [--verify-track]
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
PRED = os.path.join(REF, "data/raw/processed/predictions/DIC-C2DH-HeLa")


def read_track_file(path):
    rows = [list(map(int, ln.split())) for ln in open(path) if ln.strip()]
    return np.array(rows, dtype=np.int32).reshape(-1, 4)


def main():
    from PIL import Image
    masks = sorted(glob.glob(os.path.join(PRED, "01_RES", "mask*.tif")))
    insts = sorted(glob.glob(os.path.join(PRED, "01_RES_INST", "m*.tif")))
    assert len(masks) == len(insts) == 84, (len(masks), len(insts))
    for a, b in zip(masks, insts):
        assert os.path.basename(a)[4:7] == os.path.basename(b)[1:4]
    M = np.stack([np.array(Image.open(f)) for f in masks])
    L = np.stack([np.array(Image.open(f)) for f in insts]).astype(np.uint16)
    frames = np.array([int(os.path.basename(f)[1:4]) for f in insts], np.int32)
    track = read_track_file(os.path.join(PRED, "01", "res_track.txt"))
    out = {"mask_bits": np.packbits(M > 0, axis=-1), "mask_shape": np.array(M.shape),
           "labels": L, "frames": frames, "res_track": track, "min_size": np.array(15)}
    path = os.path.join(HERE, "hela_postproc.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes;", len(track), "tracks")

    if "--verify-track" in sys.argv:
        sys.path.insert(0, os.path.join(REF, "scripts"))
        import track as ref_track  # noqa: E402  (reference)
        dst = "/tmp/ref_track_check/res_track.txt"
        ref_track.track_sequence(os.path.join(PRED, "01_RES_INST"), dst)
        again = read_track_file(dst)
        same = again.shape == track.shape and bool((again == track).all())
        print("reference re-run reproduces the committed res_track.txt:", same)
        if not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
