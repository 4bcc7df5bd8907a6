"""scripts/train.py on the MI355X path: the whole training loop with the data
path on the GPU (unet_amd.pipeline.HeLaBatches: device-resident frames, elastic
warp, weight maps, cropped views) and the fused Trainer step.

    python tools/train_hela.py --data /path/to/DIC-C2DH-HeLa --seq 01 --epochs 20
    python tools/train_hela.py --npz tests/golden/hela_real.npz --epochs 2 --batch 3

Like train.py:64-174: 90/10 random train/val split, batch 4, SGD(lr 1e-4,
momentum 0.99), kaiming fan_out init (train.py:54-61), elastic augmentation
(alpha 2000, sigma 20), weighted CE on cropped targets / weights; validation
with the unweighted CE (train.py:143-159 = WeightedCrossEntropyLoss with unit
weights), best-val checkpoint in the reference's state_dict schema.  Frames are
read from <data>/<seq>/t*.tif with labels from <data>/<seq>_ST/SEG/man_seg*.tif
(PIL on the host, once), or from an .npz holding `images` / `segs`.
Prints one JSON line per epoch.
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unet-segmentation_amd"))


def load_frames(args):
    if args.npz:
        z = np.load(args.npz, allow_pickle=False)
        return z["images"], z["segs"]
    from PIL import Image
    seq = os.path.join(args.data, args.seq)
    segs = sorted(glob.glob(os.path.join(args.data, f"{args.seq}_ST", "SEG", "man_seg*.tif")))
    imgs, labs = [], []
    for s in segs:
        t = os.path.basename(s)[len("man_seg"):-len(".tif")]
        f = os.path.join(seq, f"t{t}.tif")
        if os.path.exists(f):
            imgs.append(np.array(Image.open(f).convert("L")))
            labs.append(np.array(Image.open(s)).astype(np.uint16))
    if not imgs:
        raise SystemExit(f"no frame / label pairs under {args.data}/{args.seq}")
    return np.stack(imgs), np.stack(labs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=None)
    ap.add_argument("--seq", default="01")
    ap.add_argument("--npz", default=None)
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--val", type=float, default=0.1)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "bf16x3"])
    ap.add_argument("--weights", default="static", choices=["static", "warped"])
    ap.add_argument("--no-augment", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--checkpoint", default=None, help="save the best-val state_dict here")
    args = ap.parse_args()
    if not (args.data or args.npz):
        ap.error("--data or --npz")

    from unet_amd import UNet, WeightedCrossEntropyLoss
    from unet_amd.pipeline import HeLaBatches, center_crop_views
    from unet_amd.train import Trainer
    torch.manual_seed(args.seed)
    dev = torch.device("cuda", 0)
    images, labels = load_frames(args)
    n = images.shape[0]
    n_val = int(n * args.val)
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(args.seed)).numpy()
    tr_idx, va_idx = perm[n_val:], perm[:n_val]
    h, w = images.shape[1:]
    img_d = torch.from_numpy(images).to(dev)
    lab_d = torch.from_numpy(labels.astype(np.int32)).to(dev)

    model = UNet(1, 2)

    def init_weights(m):  # scripts/train.py:54-61
        if isinstance(m, torch.nn.Conv2d):
            torch.nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            if m.bias is not None:
                torch.nn.init.constant_(m.bias, 0)
        elif isinstance(m, torch.nn.BatchNorm2d):
            torch.nn.init.constant_(m.weight, 1)
            torch.nn.init.constant_(m.bias, 0)
    model.apply(init_weights)
    model = model.to(dev).train()
    bs = min(args.batch, len(tr_idx))
    trainer = Trainer(model, bs, h, w, lr=args.lr, momentum=0.99, precision=args.precision)
    sel = torch.as_tensor(tr_idx, device=dev)
    data = HeLaBatches(img_d.index_select(0, sel), lab_d.index_select(0, sel), bs, trainer.out_hw,
                       augment=not args.no_augment, weights=args.weights, seed=args.seed, drop_last=True)
    crit = WeightedCrossEntropyLoss()
    best = float("inf")
    for epoch in range(args.epochs):
        data.set_epoch(epoch)
        model.train()
        t0 = time.perf_counter()
        losses = [trainer.step(x, t, wt) for x, t, wt in data]
        trainer.check_targets()  # every step of the epoch, the last one included
        train_loss = float(torch.stack(losses).mean().item())
        dt = time.perf_counter() - t0
        val_loss = None
        if len(va_idx):
            model.eval()
            vl = []
            with torch.no_grad():
                for i in va_idx:
                    x = (img_d[i].to(torch.float32) / 255.0)[None, None]
                    out = model(x)
                    t = center_crop_views((lab_d[i] != 0).to(torch.int64)[None, None], out.shape[2:])
                    vl.append(crit(out, t, torch.ones_like(t, dtype=torch.float32)))
            val_loss = float(torch.stack(vl).mean().item())
            if args.checkpoint and val_loss < best:
                best = val_loss
                torch.save(model.state_dict(), args.checkpoint)
        print(json.dumps({"epoch": epoch + 1, "train_loss": round(train_loss, 6), "val_loss": val_loss,
                          "steps": len(losses), "images_per_s": round(len(losses) * bs / dt, 2),
                          "augment": not args.no_augment, "weights": args.weights,
                          "precision": args.precision}), flush=True)


if __name__ == "__main__":
    main()
