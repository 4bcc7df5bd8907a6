"""Diagnostic: compare the Trainer fast path with the autograd drop-in path
step by step (gradients after backward, weights after SGD)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "unet-segmentation_amd")]
from oracle import unet_oracle as O  # noqa: E402
from oracle import fixtures as F  # noqa: E402
from unet_amd import UNet, WeightedCrossEntropyLoss  # noqa: E402
from unet_amd.train import Trainer  # noqa: E402


def mk(params):
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    return m.cuda()


params = O.hash_init(1, 2, seed=41, bn_random=True)
x, tgt, wmap = F.make_inputs(41, 2, 1, 204)
xd, td, wd = (torch.from_numpy(a).cuda() for a in (x, tgt, wmap))
a, b = mk(params), mk(params)
opt = torch.optim.SGD(a.parameters(), lr=1e-4, momentum=0.99)
crit = WeightedCrossEntropyLoss()
tr = Trainer(b, 2, 204, 204, lr=1e-4, momentum=0.99)
names = [n for n, _ in a.named_parameters()]
for step in range(3):
    opt.zero_grad()
    la = crit(a(xd), td, wd)
    la.backward()
    loss_b = tr.forward_loss(xd, td, wd)
    tr.backward_and_reduce(xd)
    torch.cuda.synchronize()
    ga = {n: p.grad.double().cpu().numpy() for n, p in a.named_parameters()}
    gb = {n: v.double().cpu().numpy() for n, v in zip(names, tr.flat.grad_views)}
    worst = sorted(((np.abs(ga[n] - gb[n]).max() / max(np.abs(ga[n]).max(), 1e-30), n) for n in names),
                   reverse=True)[:3]
    print(f"step {step} loss {la.item():.6f} vs {loss_b.item():.6f}; worst grad diffs {worst}")
    opt.step()
    tr.optimizer_step()
    torch.cuda.synchronize()
    sa, sb = a.state_dict(), b.state_dict()
    wd_ = sorted(((np.abs(sa[k].double().cpu().numpy() - sb[k].double().cpu().numpy()).max(), k) for k in sa),
                 reverse=True)[:3]
    print(f"   worst state diffs {wd_}")
