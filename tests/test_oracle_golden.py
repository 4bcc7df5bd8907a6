"""Pin the CPU oracle (oracle/unet_oracle.py) to the golden fixtures that
tests/golden/make_golden.py produced by running the reference itself."""
import os

import numpy as np
import pytest

from oracle import unet_oracle as O
from oracle import fixtures as F

G = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    p = os.path.join(G, name)
    if not os.path.exists(p):
        pytest.skip(f"fixture {name} missing")
    return np.load(p, allow_pickle=False)


def nhwc(a):
    return np.ascontiguousarray(np.transpose(a, (0, 2, 3, 1)))


def nchw(a):
    return np.transpose(a, (0, 3, 1, 2))


def test_conv_op():
    z = _load("ops.npz")
    y = O.conv_valid_fwd(nhwc(z["conv.x"]), z["conv.w"], z["conv.b"])
    np.testing.assert_allclose(nchw(y), z["conv.y"], rtol=1e-12, atol=1e-12)
    dx, dw, db = O.conv_valid_bwd(nhwc(z["conv.x"]), z["conv.w"], nhwc(z["conv.dy"]))
    np.testing.assert_allclose(nchw(dx), z["conv.dx"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(dw, z["conv.dw"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(db, z["conv.db"], rtol=1e-12, atol=1e-12)


def test_bn_op():
    z = _load("ops.npz")
    y, cache, mean, var_unb = O.bn_train_fwd(nhwc(z["bn.x"]), z["bn.g"], z["bn.b"])
    np.testing.assert_allclose(nchw(y), z["bn.y"], rtol=1e-12, atol=1e-12)
    rm, rv = O.bn_update_running(np.zeros(3), np.ones(3), mean, var_unb)
    np.testing.assert_allclose(rm, z["bn.rm"], rtol=1e-12)
    np.testing.assert_allclose(rv, z["bn.rv"], rtol=1e-12)
    dx, dg, db = O.bn_train_bwd(nhwc(z["bn.dy"]), cache, z["bn.g"])
    np.testing.assert_allclose(nchw(dx), z["bn.dx"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(dg, z["bn.dg"], rtol=1e-12)
    np.testing.assert_allclose(db, z["bn.db"], rtol=1e-12)
    ye = O.bn_eval_fwd(nhwc(z["bn.x"]), z["bn.g"], z["bn.b"], rm, rv)
    np.testing.assert_allclose(nchw(ye), z["bn.y_eval"], rtol=1e-12, atol=1e-12)


def test_maxpool_op_odd_and_ties():
    z = _load("ops.npz")
    y, arg = O.maxpool2_fwd(nhwc(z["pool.x"]))
    np.testing.assert_array_equal(nchw(y), z["pool.y"])
    dx = O.maxpool2_bwd(nhwc(z["pool.dy"]), arg, nhwc(z["pool.x"]).shape)
    np.testing.assert_array_equal(nchw(dx), z["pool.dx"])
    assert arg[0, 0, 0, 0] == 0  # all-equal window -> first element


def test_convT_op():
    z = _load("ops.npz")
    y = O.convT2_fwd(nhwc(z["convT.x"]), z["convT.w"], z["convT.b"])
    np.testing.assert_allclose(nchw(y), z["convT.y"], rtol=1e-12, atol=1e-12)
    dx, dw, db = O.convT2_bwd(nhwc(z["convT.x"]), z["convT.w"], nhwc(z["convT.dy"]))
    np.testing.assert_allclose(nchw(dx), z["convT.dx"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(dw, z["convT.dw"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(db, z["convT.db"], rtol=1e-12, atol=1e-12)


def test_weighted_ce_op():
    z = _load("ops.npz")
    loss, dl = O.weighted_ce(z["wce.logits"], z["wce.t"], z["wce.w"])
    np.testing.assert_allclose(loss, z["wce.loss"], rtol=1e-12)
    np.testing.assert_allclose(dl, z["wce.dlogits"], rtol=1e-10, atol=1e-14)


def test_sgd_op():
    z = _load("ops.npz")
    p, buf = z["sgd.p0"], None
    for s in range(3):
        p, buf = O.sgd_momentum_step(p, z["sgd.g"][s], buf)
        np.testing.assert_allclose(p, z["sgd.traj"][s], rtol=1e-13, atol=1e-15)


def test_output_size_rule():
    # models/unet_model.py:189-223 and SURVEY.md §0
    assert O.output_size(512) == 324
    assert O.output_size(572) == 388
    assert O.output_size(188) == 4
    assert O.output_size(204) == 20
    assert O.output_size(508) == 324


def test_param_schema_matches_reference_counts():
    shapes = O.param_shapes(1, 2)
    assert len(shapes) == 136
    n_params = sum(int(np.prod(s)) for k, s in shapes.items() if not O.is_buffer(k))
    assert n_params == 31_042_434
    assert sum(1 for k in shapes if not O.is_buffer(k)) == 82


@pytest.mark.parametrize("tag", ["n2_188", "n2_204", "n2_188x220", "n1_204x252"])
def test_whole_model_vs_reference(tag):
    """n2_188x220 / n1_204x252: H != W (the reference crops each axis on its
    own, models/unet_model.py:93-100)."""
    z = _load(f"model_{tag}.npz")
    seed, n, h, c = int(z["x_seed"]), int(z["n"]), int(z["h"]), int(z["c"])
    w = int(z["w"]) if "w" in z.files else h
    params = O.hash_init(c, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, c, h, w)
    assert z["logits"].shape[2:] == (O.output_size(h), O.output_size(w))
    net = O.UNetOracle(params)
    logits, cache, nb = net.forward(x)
    np.testing.assert_allclose(logits, z["logits"], rtol=1e-9, atol=1e-10)
    loss, dl = O.weighted_ce(logits, tgt, wmap)
    np.testing.assert_allclose(loss, z["loss"], rtol=1e-10)
    grads = net.backward(dl, cache)
    for name in O.param_shapes(c, 2):
        if O.is_buffer(name):
            continue
        g = grads[name].ravel()
        ref_norm = float(z[f"gnorm/{name}"])
        if O.bn_cancelled(name):
            # analytically zero (the bias precedes a train-mode BN): both are fp64 noise
            assert np.abs(g).max() < 1e-9 and ref_norm < 1e-9, name
            continue
        idx = z[f"gidx/{name}"]
        # fp64 both sides: BN-cancelled biases are ~1e-13 noise, compare absolutely
        scale = max(ref_norm, 1e-30)
        assert abs(np.linalg.norm(g) - ref_norm) <= 1e-7 * scale + 1e-12, name
        np.testing.assert_allclose(g[idx], z[f"gval/{name}"], rtol=1e-6, atol=1e-9 * scale + 1e-12, err_msg=name)
    for k, v in nb.items():
        if "running" in k:
            np.testing.assert_allclose(v, z[f"buf/{k}"], rtol=1e-9, atol=1e-12, err_msg=k)
    # eval forward with the updated running stats
    p2 = dict(params)
    for k, v in nb.items():
        p2[k] = v
    le, _, _ = O.UNetOracle(p2).forward(x, train=False)
    np.testing.assert_allclose(le, z["logits_eval"], rtol=1e-9, atol=1e-10)


def test_torch_cpu_restatement_fp64_vs_reference():
    """oracle/torch_cpu_ref.py in float64 (the full-tensor oracle of the 512^2
    GPU test and the CPU baseline's arithmetic) reproduces the reference's fp64
    fixture: logits, loss and every gradient digest."""
    import torch
    from oracle import torch_cpu_ref as R
    z = _load("model_n2_188.npz")
    seed, n, h = int(z["x_seed"]), int(z["n"]), int(z["h"])
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h)
    net = R.TorchCpuUNet(params, dtype=torch.float64)
    lg = net.forward(torch.from_numpy(x).double())
    loss = R.weighted_ce(lg, torch.from_numpy(tgt), torch.from_numpy(wmap).double())
    loss.backward()
    np.testing.assert_allclose(lg.detach().numpy(), z["logits"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(loss.item(), z["loss"], rtol=1e-12)
    for name, p in net.p.items():
        if not p.requires_grad:
            continue
        g = p.grad.numpy().ravel()
        ref = float(z[f"gnorm/{name}"])
        if O.bn_cancelled(name):  # analytically zero: fp64 noise on both sides
            assert np.abs(g).max() < 1e-9 and ref < 1e-9, name
            continue
        assert abs(np.linalg.norm(g) - ref) <= 1e-9 * max(ref, 1e-30) + 1e-13, name
        np.testing.assert_allclose(g[z[f"gidx/{name}"]], z[f"gval/{name}"], rtol=1e-8, atol=1e-12 * ref + 1e-14,
                                   err_msg=name)


def test_sgd_trajectory_vs_reference():
    z = _load("model_n2_188.npz")
    seed, n, h = int(z["x_seed"]), int(z["n"]), int(z["h"])
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h)
    p = {k: np.asarray(v, np.float64) for k, v in params.items()}
    bufs = {}
    lr = float(z["sgd_lr"])
    losses = []
    # the fixture was produced after one earlier train-mode forward (running stats moved once)
    _, _, nb = O.UNetOracle(p).forward(x)
    p.update(nb)
    for s in range(len(z["sgd_losses"])):
        net = O.UNetOracle(p)
        logits, cache, nb = net.forward(x)
        loss, dl = O.weighted_ce(logits, tgt, wmap)
        losses.append(loss)
        grads = net.backward(dl, cache)
        for k, g in grads.items():
            p[k], bufs[k] = O.sgd_momentum_step(p[k], g, bufs.get(k), lr=lr)
        p.update(nb)
    np.testing.assert_allclose(losses, z["sgd_losses"], rtol=1e-7)
    net = O.UNetOracle(p)
    le, _, _ = net.forward(x, train=False)
    np.testing.assert_allclose(le, z["logits_after_sgd_eval"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("tag", ["n1_512", "n1_c3_572"])
def test_forward_full_size_vs_reference(tag):
    z = _load(f"fwd_{tag}.npz")
    seed, n, h, c = int(z["x_seed"]), int(z["n"]), int(z["h"]), int(z["c"])
    params = O.hash_init(c, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, c, h)
    logits, _, _ = O.UNetOracle(params).forward(x)
    np.testing.assert_allclose(logits[:, :, ::7, ::5], z["logits_sample"], rtol=1e-8, atol=1e-9)
    loss, _ = O.weighted_ce(logits, tgt, wmap)
    np.testing.assert_allclose(loss, z["loss"], rtol=1e-10)
    np.testing.assert_array_equal(logits[:, 1] > logits[:, 0], z["mask"].astype(bool))


def test_hela_real_frames_iou_vs_reference():
    z = _load("hela_real.npz")
    params = O.hash_init(1, 2, seed=int(z["seed"]), bn_random=True)
    x = z["images"].astype(np.float64)[:, None] / 255.0 * 2.0 - 1.0
    _, _, nb = O.UNetOracle(params, bn_momentum=1.0).forward(x)
    for k, v in nb.items():
        if "running" in k:
            np.testing.assert_allclose(v, z[f"buf/{k}"], rtol=1e-8, atol=1e-10, err_msg=k)
    p2 = dict(params)
    p2.update(nb)
    logits, _, _ = O.UNetOracle(p2).forward(x, train=False)
    masks = O.predict_mask(logits)
    np.testing.assert_array_equal(masks, z["masks"])
    oy = (512 - 324) // 2
    gt = z["segs"][:, oy:oy + 324, oy:oy + 324]
    ious = [O.calculate_iou(masks[i], gt[i]) for i in range(len(masks))]
    np.testing.assert_allclose(ious, z["ious"], rtol=0, atol=1e-12)


def test_hela_gold_frames_vs_reference():
    """hela_gold.npz (the nine 01_GT/SEG frames through the reference's eval
    model): the oracle reproduces the reference's masks and IoUs on two of them
    (t002, t067; the GPU test checks all nine), with hela_real's running
    statistics (pinned above)."""
    zr, z = _load("hela_real.npz"), _load("hela_gold.npz")
    params = O.hash_init(1, 2, seed=int(z["seed"]), bn_random=True)
    for k in zr.files:
        if k.startswith("buf/"):
            params[k[4:]] = zr[k]
    pick = [0, len(z["frames"]) - 1]
    x = z["images"][pick].astype(np.float64)[:, None] / 255.0 * 2.0 - 1.0
    logits, _, _ = O.UNetOracle(params).forward(x, train=False)
    masks = O.predict_mask(logits)
    ref = np.unpackbits(z["masks"][pick], axis=-1)[..., :324]
    np.testing.assert_array_equal(masks > 0, ref > 0)
    gt = np.unpackbits(z["seg_fg"][pick], axis=-1)[..., :512][:, 94:418, 94:418]
    ious = [O.calculate_iou(masks[i], gt[i]) for i in range(len(pick))]
    np.testing.assert_allclose(ious, z["ious"][pick], rtol=0, atol=1e-12)


def test_iou_semantics():
    # utils/metrics.py:6-37
    assert O.calculate_iou(np.zeros((3, 3)), np.zeros((3, 3))) == 1.0
    a = np.array([[0, 255], [255, 0]])
    b = np.array([[0, 7], [0, 0]])
    assert O.calculate_iou(a, b) == 0.5


def test_overlap_tile_geometry():
    tile_out, pads, origins = O.overlap_tiles(1024, 1024, 512)
    assert tile_out == 324 and len(origins) == 16
    assert pads[0] == 94 and pads[2] == 94
    assert 94 + 4 * 324 + 94 == 1024 + pads[0] + pads[1]
