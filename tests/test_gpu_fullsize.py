"""Parity at the configured sizes, with the benchmarked kernel mix pinned.

The GEMM autotuner picks a kernel variant per shape by timing; ``bench.py``
writes its choices to ``profiles/tune_db.txt`` (``--tune-db-out``) and both the
bench and these tests load that file (``unet_tuning_load``), so the mix checked
here is the mix the bench line timed (shapes the file does not hold are tuned
live).

* configs[1] (fp32, 512^2): batch 2 against the reference's own fp64 arithmetic
  on EVERY logit (<= 1e-3 abs, argmax exact where the reference margin exceeds
  1e-3) and every gradient element (per-tensor rel-L2 <= max(1 %, 2 x the
  reference's own fp32-vs-fp64 rel-L2)), the fp64 run computed
  here by the torch-CPU restatement (oracle/torch_cpu_ref.py, first pinned to
  the reference-made digests of tests/golden/train_n2_512.npz).
* configs[2] per GPU (bf16, batch 8 x 512^2) and configs[4] (3-ch 572^2, bf16,
  fwd + bwd): the Trainer against the reference's fp64 fixtures at SURVEY.md
  §7's bf16 bar -- loss within 1 %, argmax agreement on the reference's sure
  pixels, gradient norms -- with floors calibrated from the bf16 arithmetic's
  own distance to the reference (UNetOracle(gemm="bf16"), every sum in fp64:
  tests/golden/train_*_bf16.npz), and against that bf16 oracle directly.
  models/unet_model.py:105-146, utils/losses.py:49-57, scripts/train.py:114-131.
"""
import os

import numpy as np
import pytest

from oracle import unet_oracle as O
from oracle import fixtures as F

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
# per-tensor cap of the bf16 sampled-entry rel-L2 against the bf16 oracle
SAMPLE_CAP = 0.5


@pytest.fixture(scope="module", autouse=True)
def _pinned(bench_tuning):
    """Every test of this module runs with the bench's tuning database loaded."""
    yield bench_tuning


def _bits(packed, w):
    return np.unpackbits(packed, axis=-1)[..., :w].astype(bool)


def make_model(params, n_channels=1, precision="fp32"):
    from unet_amd import UNet
    m = UNet(n_channels, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m.precision = precision
    return m.cuda()


def trainer_step(params, x, tgt, wmap, precision, n_channels=1):
    """One Trainer step without the optimizer: (logits, loss, {name: grad})."""
    from unet_amd.train import Trainer
    n, _, h, w = x.shape
    m = make_model(params, n_channels, precision)
    tr = Trainer(m, n, h, w, lr=1e-4, momentum=0.99, precision=precision)
    xd, td, wd = (torch.from_numpy(a).cuda() for a in (x, tgt, wmap))
    loss = tr.forward_loss(xd, td, wd)
    tr.backward_and_reduce(xd)
    torch.cuda.synchronize()
    names = [k for k, _ in m.named_parameters()]
    grads = {k: g.detach().double().cpu().numpy() for k, g in zip(names, tr.flat.grad_views)}
    return tr.logits.double().cpu().numpy(), float(loss.item()), grads, m


def flip_floors(zb, zf):
    """The rounding-boundary noise of the bf16 arithmetic at this size: the bf16
    oracle with every sum in fp32 (zf, tests/golden/make_golden.py bf16f32)
    against the same oracle in fp64 (zb).  A GPU run (fp32 sums in a different
    order) is one more sample of that noise: per tensor its own deviation, and
    per kind (BatchNorm parameters / everything else) the largest deviation of
    the kind -- measured 0.7-1.0 % median and 2.8-3.3 % max on the BatchNorm
    parameters (0.05-0.07 % / 0.3-0.7 % on the conv weights) at batch 8 x 512^2
    and 2 x 3 x 572^2."""
    per, kind = {}, {True: 0.0, False: 0.0}
    for k in zb.files:
        if not k.startswith("gbf16norm/"):
            continue
        name = k.split("/", 1)[1]
        if O.bn_cancelled(name):
            continue
        rb = float(zb[k])
        per[name] = abs(float(zf[k]) - rb)
        bn = O.is_bn_param(name)
        kind[bn] = max(kind[bn], per[name] / max(rb, 1e-30))
    return per, kind


def check_bf16_vs_reference(z, zb, lg, loss, grads, tag, zf=None):
    """SURVEY.md §7's bar for bf16 configs against the fp64 reference fixture z,
    floors from the bf16 oracle's own distance to it (zb) and from its
    rounding-boundary noise (zf: the same oracle in fp32 sums)."""
    flip, kind = flip_floors(zb, zf) if zf is not None else ({}, {True: 0.0, False: 0.0})
    ref_loss, bf_loss = float(z["loss"]), float(zb["loss"])
    wout = lg.shape[-1]
    lo = abs(loss - ref_loss) / abs(ref_loss)
    assert lo <= 1e-2, (tag, loss, ref_loss)
    sure = _bits(z["sure"], wout)
    ref_mask, bf_mask = _bits(z["mask"], wout), _bits(zb["mask"], wout)
    agree = float(((lg[:, 1] > lg[:, 0]) == ref_mask)[sure].mean())
    bf_agree = float((bf_mask == ref_mask)[sure].mean())   # what bf16 rounding itself costs
    assert agree >= bf_agree - 5e-3, (tag, agree, bf_agree)
    # argmax vs the bf16 oracle (same roundings, fp64 sums): the GPU's fp32 sums
    # move rare operands across a bf16 rounding boundary, nothing more
    agree_bf = float(((lg[:, 1] > lg[:, 0]) == bf_mask).mean())
    assert agree_bf >= 0.995, (tag, agree_bf)
    # element level against the bf16 oracle (same roundings, fp64 sums): the
    # logit sample within 3 x the rounding-boundary noise of the same oracle in
    # fp32 sums (zf), and the 32 sampled entries of every gradient (below)
    lt = np.abs(lg[:, :, ::7, ::5] - zb["logits_sample"]).max()
    if zf is not None:
        lflip = float(np.abs(zf["logits_sample"] - zb["logits_sample"]).max())
        assert lt <= 3 * lflip, (tag, lt, lflip)
    worst = worst_b = 0.0
    ratios, worst_s, worst_abs = [], (0.0, ""), (0.0, "")
    for name, g in grads.items():
        r = float(z[f"gnorm/{name}"])
        if O.bn_cancelled(name):
            wn = float(z[f"gnorm/{name.replace('.bias', '.weight')}"])
            assert np.abs(g).max() <= 5e-3 * wn, (tag, name)   # bf16 dgrad sums do not cancel exactly
            continue
        floor = abs(float(zb[f"gbf16norm/{name}"]) - r)
        # the GPU result carries its own bf16 rounding pattern (fp32 sums, tuned
        # tile mix) on top of the one the bf16 oracle measures: within 3 floors,
        # 3 x the tensor's rounding-boundary noise, and 1.5 x the largest such
        # noise of its kind (BatchNorm affine gradients are sums over 0.1-2 M
        # bf16-stored BN-input gradients with heavy cancellation)
        rb = float(zb[f"gbf16norm/{name}"])
        noise = max(3 * flip.get(name, 0.0), 1.5 * kind[O.is_bn_param(name)] * rb)
        rel = 2e-2 if O.is_bn_param(name) else 1e-2
        tol = max(rel * r, 3 * floor, noise)
        e = abs(np.linalg.norm(g) - r)
        worst = max(worst, e / tol)
        assert e <= tol, (tag, name, np.linalg.norm(g), r, floor)
        # against the bf16 oracle's own gradient (same roundings, fp64 sums): the
        # GPU's fp32 sums move operands across bf16 rounding boundaries, a
        # perturbation of the same kind as bf16's own -- within 3 % or 3 x it
        eb = abs(np.linalg.norm(g) - rb)
        tb = max(3e-2 * rb, 3 * floor, noise)
        worst_b = max(worst_b, eb / tb)
        assert eb <= tb, (tag, name, np.linalg.norm(g), rb)
        if zf is not None and f"gbf16val/{name}" in zb.files:
            # sampled entries (indices of the fp64 fixture) vs the bf16 oracle: a
            # bf16 rounding flip moves a BatchNorm channel's backward
            # coefficients and with them every entry of the channel coherently,
            # so single entries carry 10-80 % (median 27 %) rel-L2 of that noise
            # (zf vs zb); the GPU's sample is one more draw of it: within 3 x the
            # tensor's own noise (at least 5 %), and never above 0.5 (VERDICT
            # r04: the earlier cap of 1.2 sat close to an uncorrelated slice's
            # ~1.4; a sign-flipped slice reads ~2)
            idx = z[f"gidx/{name}"]
            vb, vf = zb[f"gbf16val/{name}"], zf[f"gbf16val/{name}"]
            nb = max(np.linalg.norm(vb), 1e-30)
            es, fs = np.linalg.norm(g.ravel()[idx] - vb) / nb, np.linalg.norm(vf - vb) / nb
            bar = min(SAMPLE_CAP, max(3 * fs, 0.05))
            ratios.append(es / max(fs, 0.05))
            if es / bar > worst_s[0]:
                worst_s = (es / bar, name)
            worst_abs = max(worst_abs, (es, name))
            assert es <= bar, (tag, name, es, fs)
    if ratios:
        # statistically the GPU is one more draw of the oracle's own boundary
        # noise: its typical sample error sits at ~1x that noise, not above 2x
        assert float(np.median(ratios)) <= 2.0, (tag, float(np.median(ratios)))
        print(f"{tag}: sampled gradient entries vs bf16 oracle: median err / own noise {np.median(ratios):.2f}, "
              f"worst err / bar {worst_s[0]:.2f} ({worst_s[1]}), largest sampled rel-L2 {worst_abs[0]:.3f} "
              f"({worst_abs[1]}; cap {SAMPLE_CAP})")
    print(f"{tag}: loss rel {lo:.2e} (bf16 oracle {abs(bf_loss - ref_loss) / abs(ref_loss):.2e}), "
          f"mask agreement {agree:.5f} (bf16 oracle {bf_agree:.5f}; vs bf16 oracle {agree_bf:.5f}), "
          f"logits vs bf16 oracle max {lt:.3f}, worst grad-norm err / tol {worst:.2f} (vs bf16 oracle {worst_b:.2f})")


def test_trainer_bf16_batch8_512_vs_reference():
    """configs[2] per GPU: Trainer(precision="bf16") at batch 8 x 512^2 -- the
    bench's bf16 workload, its tuned kernels -- against the reference's fp64
    fixture (tests/golden/train_n8_512.npz) at the bf16 bar."""
    z = np.load(os.path.join(G, "train_n8_512.npz"), allow_pickle=False)
    zb = np.load(os.path.join(G, "train_n8_512_bf16.npz"), allow_pickle=False)
    zf = np.load(os.path.join(G, "train_n8_512_bf16_f32.npz"), allow_pickle=False)
    seed, n, h = int(z["x_seed"]), int(z["n"]), int(z["h"])
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h)
    lg, loss, grads, m = trainer_step(params, x, tgt, wmap, "bf16")
    check_bf16_vs_reference(z, zb, lg, loss, grads, "bf16 8x512", zf)
    sd = m.state_dict()
    for k in zb.files:  # running statistics: the bf16 oracle's (same rounded conv outputs)
        if k.startswith("buf/"):
            np.testing.assert_allclose(sd[k[4:]].cpu().numpy(), zb[k], rtol=2e-3, atol=2e-3, err_msg=k)


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_c3_572_train_step_vs_reference(precision):
    """configs[4] shape: 3-channel 572x572 input (388x388 out), forward +
    weighted CE + backward, batch 2 (tests/golden/train_n2_c3_572.npz, the
    reference in fp64).  bf16: the bf16 bar above; fp32: the fp32 bar (logits
    <= 1e-3 abs, loss 1e-4, mask exact on sure pixels, gradient digests)."""
    z = np.load(os.path.join(G, "train_n2_c3_572.npz"), allow_pickle=False)
    seed, n, h, c = int(z["x_seed"]), int(z["n"]), int(z["h"]), int(z["c"])
    params = O.hash_init(c, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, c, h)
    lg, loss, grads, _ = trainer_step(params, x, tgt, wmap, precision, n_channels=c)
    assert lg.shape == (n, 2, 388, 388)
    if precision == "bf16":
        zb = np.load(os.path.join(G, "train_n2_c3_572_bf16.npz"), allow_pickle=False)
        zf = np.load(os.path.join(G, "train_n2_c3_572_bf16_f32.npz"), allow_pickle=False)
        check_bf16_vs_reference(z, zb, lg, loss, grads, "bf16 2x3x572", zf)
        return
    from test_gpu_model import check_full_size_outputs, check_grad_digests
    low = check_full_size_outputs(lg, loss, z, lg.shape[-1])
    check_grad_digests(list(grads.items()), z)
    print(f"fp32 2x3x572: {low} low-margin pixels")


def _torch_reference(params, x, tgt, wmap, dtype):
    """The reference's arithmetic on torch CPU (oracle/torch_cpu_ref.py)."""
    from oracle import torch_cpu_ref as R
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    net = R.TorchCpuUNet(params, dtype=dtype)
    lg = net.forward(torch.from_numpy(x).to(dtype))
    loss = R.weighted_ce(lg, torch.from_numpy(tgt), torch.from_numpy(wmap).to(dtype))
    loss.backward()
    grads = {k: v.grad.double().numpy() for k, v in net.p.items() if v.requires_grad}
    return lg.detach().double().numpy(), float(loss.item()), grads


@pytest.mark.parametrize("fixture,path", [("train_n2_512", "dropin"), ("train_n8_512", "trainer")])
def test_fp32_512_every_logit_and_gradient_vs_reference_fp64(fixture, path):
    """configs[1]'s image size, fp32: ALL logits and ALL 31 M gradient entries
    against the reference's arithmetic in fp64 -- at batch 2 through the
    autograd drop-in, and at the bench's own batch 8 through the bench's
    Trainer with its tuned batch-8 kernel mix.  The
    fp64 run is the torch-CPU restatement, checked first against the
    reference-made digests of the same step (train_n{2,8}_512.npz: logit
    sample, loss, gradient norms and sampled entries to 1e-9 relative); its
    fp32 twin gives each tensor's fp32 floor."""
    z = np.load(os.path.join(G, f"{fixture}.npz"), allow_pickle=False)
    seed, n, h = int(z["x_seed"]), int(z["n"]), int(z["h"])
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h)
    rl, rloss, rg = _torch_reference(params, x, tgt, wmap, torch.float64)
    # pin the fp64 oracle to the reference's own fixture
    assert np.abs(rl[:, :, ::7, ::5] - z["logits_sample"]).max() <= 1e-9
    assert abs(rloss - float(z["loss"])) <= 1e-12 * abs(rloss)
    for name, g in rg.items():
        if O.bn_cancelled(name):  # analytically zero: fp64 noise on both sides
            continue
        g = g.ravel()
        ref = float(z[f"gnorm/{name}"])
        assert abs(np.linalg.norm(g) - ref) <= 1e-9 * max(ref, 1e-30), name
        np.testing.assert_allclose(g[z[f"gidx/{name}"]], z[f"gval/{name}"], rtol=1e-8, atol=1e-14 * ref, err_msg=name)
    _, _, r32 = _torch_reference(params, x, tgt, wmap, torch.float32)

    if path == "trainer":
        lg, lossv, grads, _ = trainer_step(params, x, tgt, wmap, "fp32")
    else:
        from unet_amd import WeightedCrossEntropyLoss
        m = make_model(params)
        m.train()
        logits = m(torch.from_numpy(x).cuda())
        loss = WeightedCrossEntropyLoss()(logits, torch.from_numpy(tgt).cuda(), torch.from_numpy(wmap).cuda())
        loss.backward()
        lg, lossv = logits.detach().double().cpu().numpy(), loss.item()
        grads = {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}
    assert lg.shape == rl.shape
    lerr = np.abs(lg - rl).max()
    assert lerr <= 1e-3, lerr
    assert abs(lossv - rloss) <= 1e-4 * abs(rloss)
    sure = np.abs(rl[:, 1] - rl[:, 0]) > 1e-3
    np.testing.assert_array_equal((lg[:, 1] > lg[:, 0])[sure], (rl[:, 1] > rl[:, 0])[sure])
    worst, worst_name = 0.0, ""
    above, over_1pct = [], 0
    for name, g in grads.items():
        r = rg[name]
        g = g.reshape(r.shape)
        if O.bn_cancelled(name):
            assert np.abs(g).max() <= 1e-3 * np.abs(rg[name.replace(".bias", ".weight")]).max(), name
            continue
        nr = max(np.linalg.norm(r), 1e-30)
        e = np.linalg.norm(g - r) / nr
        floor = np.linalg.norm(r32[name] - r) / nr
        tol = max(1e-2, 2 * floor)
        if e / tol > worst:
            worst, worst_name = e / tol, name
        if tol > 1e-2:  # the bar rose above SURVEY §8c's 1 % with the reference's own fp32 floor
            above.append((name, e, floor, tol))
        over_1pct += e > 1e-2
        assert e <= tol, (name, e, floor)
    # every tensor whose bar exceeds 1 %: its error, the
    # reference's own fp32-vs-fp64 floor and the bar
    for name, e, floor, tol in sorted(above, key=lambda a: -a[3]):
        print(f"  bar > 1 %: {name}: rel-L2 {e:.4f}, reference fp32 floor {floor:.4f}, bar {tol:.4f} "
              f"({e / tol:.2f} of it)")
    print(f"512^2 batch {n} ({path}), every element: logits max |err| {lerr:.2e}, {int((~sure).sum())} low-margin "
          f"pixels, worst gradient rel-L2 / tol {worst:.2f} ({worst_name}); {len(above)} of {len(grads)} tensors "
          f"have a bar above 1 %, {over_1pct} have an error above 1 %")
