"""fp32 BatchNorm-backward apply fused with the F(6x6) weight gradient's dY
transform (k_bnb_wino6_dy, unet_set_tuning "bnb_fuse") against the two-pass
form it replaces (k_bnb_apply, then k_wino6_dy reading dYpad back).

BatchNorm2d backward of DoubleConv (reference models/unet_model.py:12,16):
dY = k0*dz + k1*(y - mean) + k2 per channel.  The fused pass forms dY with the
apply kernel's exact expression, stores it into the padded dY buffer the input
gradient reads (its zero border included) and transforms the register copy, so
a train step must be bit-identical with and without it.  The weight gradients
are forced to Winograd F(6x6) in slab mode (wgrad1074: no fp32 atomics), which
makes every tensor of the step run-to-run reproducible except the leaves whose
kernels keep atomics under the heuristic (the ConvTranspose2d weight gradients
and inc.c0's weight gradient): those are held to the run-to-run noise of a
repeated unfused step.  The fused pass is on by default, together with the
early input transforms of the Winograd weight gradients; the
oracle case checks a step under the tuned choices against fp64."""
import numpy as np
import pytest

from oracle import unet_oracle as O
from oracle import fixtures as F

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _atomic_leaf(name):
    return ".up.weight" in name or name == "inc.double_conv.0.weight"


def _step(params, x, tgt, wmap):
    from unet_amd import UNet, WeightedCrossEntropyLoss
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.cuda().train()
    logits = m(torch.from_numpy(x).cuda())
    loss = WeightedCrossEntropyLoss()(logits, torch.from_numpy(tgt).cuda(), torch.from_numpy(wmap).cuda())
    loss.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().cpu() for n, p in m.named_parameters()}
    bufs = {n: b.detach().cpu() for n, b in m.named_buffers()}
    return logits.detach().cpu(), loss.detach().cpu(), grads, bufs


@pytest.mark.parametrize("n,h,w,seed", [(2, 188, 188, 41), (1, 195, 195, 42), (1, 204, 252, 43)])
def test_fused_bnb_wino6_dy_bit_identical(n, h, w, seed):
    from unet_amd import _lib
    lib = _lib.load()
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h, w)
    runs, sites = [], []
    lib.unet_tuning_reset()
    lib.unet_set_tuning(b"autotune", 0)
    lib.unet_set_tuning(b"wgrad_variant", 1074)
    try:
        for fuse in (0, 0, 1):
            lib.unet_set_tuning(b"bnb_fuse", fuse)
            lib.unet_fused_bnb_sites(1)
            runs.append(_step(params, x, tgt, wmap))
            sites.append(lib.unet_fused_bnb_sites(1))
    finally:
        lib.unet_set_tuning(b"bnb_fuse", 1)
        lib.unet_set_tuning(b"wgrad_variant", -1)
        lib.unet_set_tuning(b"autotune", 1)
        lib.unet_tuning_reset()
    # the fused pass ran for every 3x3 layer after inc.c0 (17 layers), never when off
    assert sites[0] == 0 and sites[1] == 0 and sites[2] == 17, sites
    (l0, s0, g0, b0), (_, _, g0b, _), (l1, s1, g1, b1) = runs
    assert torch.equal(l0, l1) and torch.equal(s0, s1)
    for k in b0:
        assert torch.equal(b0[k], b1[k]), k
    exact = 0
    for k in g0:
        if _atomic_leaf(k):
            a, b, c = (t.double() for t in (g0[k], g0b[k], g1[k]))
            nrm = a.norm().item() + 1e-30
            noise, diff = (b - a).norm().item() / nrm, (c - a).norm().item() / nrm
            assert diff <= 2 * noise + 1e-6, (k, diff, noise)
        else:
            assert torch.equal(g0[k], g0b[k]), f"{k}: the unfused step is not reproducible"
            assert torch.equal(g0[k], g1[k]), f"{k}: fused and two-pass gradients differ"
            exact += 1
    print(f"{exact} gradient tensors bit-identical, fused sites {sites[2]}")


def test_fused_bnb_wino6_dy_vs_oracle():
    """The fused pass under the autotuner's own choices: a train step
    against the fp64 oracle at the fp32 bars of test_gpu_model.py (rel-L2 per
    gradient <= max(1e-2, 2 x the fp32 oracle's own error))."""
    from unet_amd import _lib
    import test_gpu_model as TM
    lib = _lib.load()
    lib.unet_set_tuning(b"bnb_fuse", 1)
    lib.unet_fused_bnb_sites(1)
    try:
        TM.test_train_step_vs_oracle(2, 188, 44, "fp32")
        used = lib.unet_fused_bnb_sites(1)
    finally:
        lib.unet_set_tuning(b"bnb_fuse", 1)
    print(f"fused sites under the tuned choices: {used}")


def _two_steps(params, x, tgt, wmap):
    """Two train steps of a fresh model: the first tunes / runs serially, the
    second runs the concurrent schedule (weight gradients on the side stream);
    returns the second step's outputs."""
    from unet_amd import UNet, WeightedCrossEntropyLoss
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m = m.cuda().train()
    xd, td, wd = (torch.from_numpy(a).cuda() for a in (x, tgt, wmap))
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        logits = m(xd)
        loss = WeightedCrossEntropyLoss()(logits, td, wd)
        loss.backward()
    torch.cuda.synchronize()
    return (logits.detach().cpu(), loss.detach().cpu(), {n: p.grad.detach().cpu() for n, p in m.named_parameters()})


@pytest.mark.parametrize("n,h,seed", [(2, 188, 45), (1, 195, 46)])
def test_wgrad_early_u_bit_identical(n, h, seed):
    """unet_set_tuning("wgrad_early_u", 1): the Winograd weight gradients' input
    transform U is issued on the side stream before the wait for the layer's dY
    (scheduling only: the same kernels on the same operands).  With F(6x6)
    forced in slab mode the concurrent step is bit-identical to the default
    schedule on every reproducible tensor."""
    from unet_amd import _lib
    lib = _lib.load()
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h)
    runs = []
    lib.unet_tuning_reset()
    lib.unet_set_tuning(b"autotune", 0)
    lib.unet_set_tuning(b"wgrad_variant", 1074)
    try:
        for early in (0, 0, 1):
            lib.unet_set_tuning(b"wgrad_early_u", early)
            runs.append(_two_steps(params, x, tgt, wmap))
    finally:
        lib.unet_set_tuning(b"wgrad_early_u", 1)
        lib.unet_set_tuning(b"wgrad_variant", -1)
        lib.unet_set_tuning(b"autotune", 1)
        lib.unet_tuning_reset()
    (l0, s0, g0), (_, _, g0b), (l1, s1, g1) = runs
    assert torch.equal(l0, l1) and torch.equal(s0, s1)
    for k in g0:
        if _atomic_leaf(k):
            a, b, c = (t.double() for t in (g0[k], g0b[k], g1[k]))
            nrm = a.norm().item() + 1e-30
            noise, diff = (b - a).norm().item() / nrm, (c - a).norm().item() / nrm
            assert diff <= 2 * noise + 1e-6, (k, diff, noise)
        else:
            assert torch.equal(g0[k], g0b[k]), f"{k}: the default step is not reproducible"
            assert torch.equal(g0[k], g1[k]), f"{k}: early-U and default gradients differ"


@pytest.mark.parametrize("n,h,seed", [(2, 188, 47), (1, 204, 48)])
def test_wgrad_fwd_u_bit_identical(n, h, seed):
    """unet_set_tuning("wgrad_fwd_u", 1) (read at plan creation): the Winograd
    weight gradients' input transform U is issued during the forward on the
    side stream, into a per-layer buffer the backward's point GEMMs read.  The
    second (concurrent) step is bit-identical to the default schedule on every
    reproducible tensor, with F(6x6) forced in slab mode."""
    from unet_amd import _lib
    lib = _lib.load()
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h)
    runs = []
    lib.unet_tuning_reset()
    lib.unet_set_tuning(b"autotune", 0)
    lib.unet_set_tuning(b"wgrad_variant", 1074)
    try:
        for fwd_u in (0, 0, 1):
            lib.unet_set_tuning(b"wgrad_fwd_u", fwd_u)
            runs.append(_two_steps(params, x, tgt, wmap))
    finally:
        lib.unet_set_tuning(b"wgrad_fwd_u", 0)
        lib.unet_set_tuning(b"wgrad_variant", -1)
        lib.unet_set_tuning(b"autotune", 1)
        lib.unet_tuning_reset()
    (l0, s0, g0), (_, _, g0b), (l1, s1, g1) = runs
    assert torch.equal(l0, l1) and torch.equal(s0, s1)
    for k in g0:
        if _atomic_leaf(k):
            a, b, c = (t.double() for t in (g0[k], g0b[k], g1[k]))
            nrm = a.norm().item() + 1e-30
            noise, diff = (b - a).norm().item() / nrm, (c - a).norm().item() / nrm
            assert diff <= 2 * noise + 1e-6, (k, diff, noise)
        else:
            assert torch.equal(g0[k], g0b[k]), f"{k}: the default step is not reproducible"
            assert torch.equal(g0[k], g1[k]), f"{k}: forward-U and default gradients differ"
