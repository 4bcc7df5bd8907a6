"""Per-tensor gradient error of one whole train step vs the fp64 oracle, next to
the fp32 oracle's own error (the noise floor), for the channel/class-count case
of tests/test_gpu_model.py (2 x 188, c input channels, k classes).  Used to see
which GEMM variants (UNET_WINO_* knobs) move which tensors.
    python tools/acc_probe.py C K [top] [tuning-db-out]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "unet-segmentation_amd"))
from oracle import unet_oracle as O  # noqa: E402
from oracle import fixtures as F  # noqa: E402


def main():
    c, k = int(sys.argv[1]), int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    from unet_amd import UNet, WeightedCrossEntropyLoss
    seed = 60 + 10 * c + k
    params = O.hash_init(c, k, seed=seed, bn_random=True)
    x, _, wmap = F.make_inputs(seed, 2, c, 188)
    ho = O.output_size(188)
    tgt = np.minimum((O.hash_uniform(seed, 1002, 2 * ho * ho) * k).astype(np.int64), k - 1).reshape(2, ho, ho)
    out = {}
    for dt in (np.float64, np.float32):
        net = O.UNetOracle(params, dtype=dt)
        rl, cache, _ = net.forward(x)
        _, rdl = O.weighted_ce(rl, tgt, wmap)
        out[dt] = net.backward(np.asarray(rdl, dt), cache)
    m = UNet(c, k)
    m.load_state_dict({kk: torch.from_numpy(np.asarray(v)) for kk, v in params.items()})
    m = m.cuda().train()
    loss = WeightedCrossEntropyLoss()(m(torch.from_numpy(x).cuda()), torch.from_numpy(tgt).cuda(),
                                      torch.from_numpy(wmap).cuda())
    loss.backward()
    rows = []
    for name, p in m.named_parameters():
        if O.bn_cancelled(name):
            continue
        r = np.asarray(out[np.float64][name], np.float64)
        nr = max(np.linalg.norm(r), 1e-30)
        e = np.linalg.norm(p.grad.double().cpu().numpy() - r) / nr
        fl = np.linalg.norm(np.asarray(out[np.float32][name], np.float64) - r) / nr
        rows.append((e, fl, name))
    for e, fl, name in sorted(rows, reverse=True)[:top]:
        print(f"{name:45s} err {e:.3e}  fp32-oracle floor {fl:.3e}")
    if len(sys.argv) > 4:
        from unet_amd import _lib
        _lib.load().unet_tuning_save(sys.argv[4].encode())


if __name__ == "__main__":
    main()
