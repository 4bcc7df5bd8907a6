"""Op-level parity: every HIP kernel family vs the CPU oracle (float64), called
through the C-ABI (include/unet_hip.h).  Tolerances are fp32 accumulation
noise relative to the output scale."""
import ctypes

import numpy as np
import pytest

from oracle import unet_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd import _lib
    return _lib.load()


_KEEP = []


def dev(a, dtype=torch.float32):
    """Device copy that stays alive until the test ends (raw pointers are
    handed to the C-ABI, so the caching allocator must not recycle it)."""
    t = torch.from_numpy(np.ascontiguousarray(a)).to("cuda", dtype)
    _KEEP.append(t)
    return t


@pytest.fixture(autouse=True)
def _release():
    yield
    torch.cuda.synchronize()
    _KEEP.clear()


def host(t):
    return t.detach().double().cpu().numpy()


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def rel_err(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def ck(rc):
    from unet_amd import _lib
    _lib.check(rc, "op")


@pytest.fixture
def variant(request, lib):
    """Forced igemm tile for the per-op entry points (-1 = built-in choice;
    51-54 = the fp32 halo-tiled k_conv3_f32: 8x32, 16x16, 8x32 with 4 waves, 8x16)."""
    lib.unet_set_tuning(b"igemm_variant", request.param)
    yield request.param
    lib.unet_set_tuning(b"igemm_variant", -1)


HALO32 = [-1, 51, 52, 53, 54]


@pytest.mark.parametrize("variant", HALO32, indirect=True)
@pytest.mark.parametrize("n,h,w,ci,co,tf", [(2, 14, 13, 64, 128, False), (2, 11, 17, 64, 64, True),
                                              (1, 30, 29, 128, 256, True), (3, 7, 9, 32, 64, False),
                                              (1, 37, 70, 16, 64, True)])
def test_conv3x3_fwd(lib, n, h, w, ci, co, tf, variant):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((n, h, w, ci))
    wt = rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci)
    b = rng.standard_normal(co)
    sc = rng.uniform(-0.5, 1.5, ci) if tf else None
    sh = rng.standard_normal(ci) * 0.3 if tf else None
    xin = np.maximum(x * sc + sh, 0) if tf else x
    ref = O.conv_valid_fwd(xin, wt, b)
    y = torch.empty((n, h - 2, w - 2, co), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_fwd(dev(x).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), dev(b).data_ptr(), co,
                            dev(sc).data_ptr() if tf else None, dev(sh).data_ptr() if tf else None,
                            y.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(y), ref) < 2e-5


@pytest.mark.parametrize("variant", HALO32, indirect=True)
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 64, 64), (1, 9, 14, 128, 64), (2, 8, 8, 64, 256)])
def test_conv3x3_dgrad(lib, n, h, w, ci, co, variant):
    rng = np.random.default_rng(1)
    x = rng.standard_normal((n, h, w, ci))
    wt = rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci)
    dy = rng.standard_normal((n, h - 2, w - 2, co))
    ref, _, _ = O.conv_valid_bwd(x, wt, dy)
    dx = torch.empty((n, h, w, ci), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_dgrad(dev(dy).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), co, dx.data_ptr(),
                              ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(dx), ref) < 2e-5


def _conv_fwd(lib, x, wt, b, sc, sh):
    n, h, w, ci = x.shape
    co = wt.shape[0]
    y = torch.empty((n, h - 2, w - 2, co), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_fwd(dev(x).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), dev(b).data_ptr(), co,
                            dev(sc).data_ptr() if sc is not None else None,
                            dev(sh).data_ptr() if sh is not None else None, y.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    return host(y)


def _conv_dgrad(lib, dy, wt, h, w, ci):
    n = dy.shape[0]
    co = wt.shape[0]
    dx = torch.empty((n, h, w, ci), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_dgrad(dev(dy).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), co, dx.data_ptr(),
                              ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    return host(dx)


@pytest.mark.parametrize("n,h,w,ci,co,tf", [(2, 14, 13, 64, 64, False), (2, 11, 17, 64, 128, True),
                                              (1, 30, 29, 128, 64, True), (3, 7, 9, 16, 64, False),
                                              (1, 37, 70, 32, 192, True), (1, 6, 6, 48, 64, True)])
def test_wino4f64_pipelined_bitexact(lib, n, h, w, ci, co, tf):
    """Tile 76 (k_wino4f64p: tile 73's fused F(4x4) on a software-pipelined
    chunk loop, every load an LDS-DMA) keeps tile 73's operands, transforms and
    per-point accumulation order.  The two kernels are compiled separately, so
    the compiler's FMA contraction of the 4-5-term input-transform rows may
    differ (measured: last-bit differences on the outputs that read point rows
    0 and 5); a stale or torn operand would be off by O(1).  Forward (with and
    without the producer's BN+ReLU on load, ragged 4x4 tiles, tile counts not a
    multiple of 32, 1-6 input-channel chunks) and input gradient: within 8 fp32
    ulps of the output scale of tile 73, both at the oracle."""
    rng = np.random.default_rng(7)
    x = rng.standard_normal((n, h, w, ci))
    wt = rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci)
    b = rng.standard_normal(co)
    sc = rng.uniform(-0.5, 1.5, ci) if tf else None
    sh = rng.standard_normal(ci) * 0.3 if tf else None
    dy = rng.standard_normal((n, h - 2, w - 2, co))
    ref = O.conv_valid_fwd(np.maximum(x * sc + sh, 0) if tf else x, wt, b)
    rdx, _, _ = O.conv_valid_bwd(x, wt, dy)
    dg = ci % 64 == 0   # the dgrad entry point's channel rule
    outs = {}
    for v in (73, 76):
        lib.unet_set_tuning(b"igemm_variant", v)
        try:
            outs[v] = (_conv_fwd(lib, x, wt, b, sc, sh), _conv_dgrad(lib, dy, wt, h, w, ci) if dg else None)
        finally:
            lib.unet_set_tuning(b"igemm_variant", -1)
    ulp8 = 8 * 2.0 ** -23
    assert rel_err(outs[76][0], outs[73][0]) <= ulp8
    assert rel_err(outs[76][0], ref) < 2e-5
    if dg:
        assert rel_err(outs[76][1], outs[73][1]) <= ulp8
        assert rel_err(outs[76][1], rdx) < 2e-5
    print(f"76 vs 73: fwd {rel_err(outs[76][0], outs[73][0]):.1e}"
          + (f", dgrad {rel_err(outs[76][1], outs[73][1]):.1e}" if dg else ""))


@pytest.mark.parametrize("n,h,w,ci,co,tf", [(2, 14, 13, 64, 64, False), (2, 11, 17, 64, 128, True),
                                              (1, 30, 29, 128, 64, True), (3, 7, 9, 16, 64, False)])
def test_wino2_32col_vs_64col(lib, n, h, w, ci, co, tf):
    """Tile 77 (fused F(2x2) over 32 output columns, two workgroups per CU)
    against tile 75 (64 columns): same operands and per-point accumulation
    order, so within 8 fp32 ulps of the output scale (separately compiled
    FMA contraction), both at the oracle; forward with / without the
    producer's BN+ReLU, input gradient."""
    rng = np.random.default_rng(9)
    x = rng.standard_normal((n, h, w, ci))
    wt = rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci)
    b = rng.standard_normal(co)
    sc = rng.uniform(-0.5, 1.5, ci) if tf else None
    sh = rng.standard_normal(ci) * 0.3 if tf else None
    dy = rng.standard_normal((n, h - 2, w - 2, co))
    ref = O.conv_valid_fwd(np.maximum(x * sc + sh, 0) if tf else x, wt, b)
    rdx, _, _ = O.conv_valid_bwd(x, wt, dy)
    dg = ci % 64 == 0
    outs = {}
    for v in (75, 77):
        lib.unet_set_tuning(b"igemm_variant", v)
        try:
            outs[v] = (_conv_fwd(lib, x, wt, b, sc, sh), _conv_dgrad(lib, dy, wt, h, w, ci) if dg else None)
        finally:
            lib.unet_set_tuning(b"igemm_variant", -1)
    ulp8 = 8 * 2.0 ** -23
    assert rel_err(outs[77][0], outs[75][0]) <= ulp8
    assert rel_err(outs[77][0], ref) < 2e-5
    if dg:
        assert rel_err(outs[77][1], outs[75][1]) <= ulp8
        assert rel_err(outs[77][1], rdx) < 2e-5


@pytest.fixture
def wvariant(request, lib):
    """Forced weight-gradient tile (-1 = built-in; 22 / 23 = the fp32 halo-tiled
    all-taps k_wgrad3_f32, 8x16 / 4x32 pixel tiles)."""
    lib.unet_set_tuning(b"wgrad_variant", request.param)
    yield request.param
    lib.unet_set_tuning(b"wgrad_variant", -1)


@pytest.mark.parametrize("wvariant", [-1, 22, 23], indirect=True)
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 64, 64), (1, 40, 37, 128, 128), (2, 10, 9, 64, 128),
                                         (1, 7, 5, 64, 64), (2, 21, 44, 192, 128)])
def test_conv3x3_wgrad(lib, n, h, w, ci, co, wvariant):
    """Ragged pixel counts and grids that are not multiples of the halo tiles."""
    rng = np.random.default_rng(2)
    x = rng.standard_normal((n, h, w, ci))
    wt = rng.standard_normal((co, ci, 3, 3))
    dy = rng.standard_normal((n, h - 2, w - 2, co))
    _, rdw, rdb = O.conv_valid_bwd(x, wt, dy, need_dx=False)
    dw = torch.empty((co, ci, 3, 3), device="cuda")
    db = torch.empty(co, device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_wgrad(dev(x).data_ptr(), dev(dy).data_ptr(), n, h, w, ci, co, dw.data_ptr(),
                              db.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(dw), rdw) < 2e-5
    assert rel_err(host(db), rdb) < 2e-5


@pytest.mark.parametrize("n,h,w,ci,co", [(2, 5, 7, 128, 64), (1, 6, 6, 256, 128)])
def test_convT2_fwd_bwd(lib, n, h, w, ci, co):
    rng = np.random.default_rng(3)
    x = rng.standard_normal((n, h, w, ci))
    wt = rng.standard_normal((ci, co, 2, 2)) / np.sqrt(ci)
    b = rng.standard_normal(co)
    dy = rng.standard_normal((n, 2 * h, 2 * w, co))
    ref = O.convT2_fwd(x, wt, b)
    rdx, rdw, rdb = O.convT2_bwd(x, wt, dy)
    ws = torch.empty(lib.unet_conv_ws_bytes(n, 2 * h, 2 * w, ci, co), dtype=torch.uint8, device="cuda")
    y = torch.empty((n, 2 * h, 2 * w, co), device="cuda")
    xd, wd = dev(x), dev(wt)
    ck(lib.unet_convT2_fwd(xd.data_ptr(), n, h, w, ci, wd.data_ptr(), dev(b).data_ptr(), co, y.data_ptr(),
                           ws.data_ptr(), stream()))
    dx = torch.empty((n, h, w, ci), device="cuda")
    dw = torch.empty((ci, co, 2, 2), device="cuda")
    db = torch.empty(co, device="cuda")
    ck(lib.unet_convT2_bwd(xd.data_ptr(), dev(dy).data_ptr(), n, h, w, ci, wd.data_ptr(), co, dx.data_ptr(),
                           dw.data_ptr(), db.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(y), ref) < 2e-5
    assert rel_err(host(dx), rdx) < 2e-5
    assert rel_err(host(dw), rdw) < 2e-5
    assert rel_err(host(db), rdb) < 2e-5


def test_maxpool_odd_size_and_ties(lib):
    rng = np.random.default_rng(4)
    n, h, w, c = 2, 7, 9, 8
    x = rng.integers(-2, 3, (n, h, w, c)).astype(np.float64)
    x[0, :2, :2, :] = 1.0
    ref, arg = O.maxpool2_fwd(x)
    dy = rng.standard_normal(ref.shape)
    rdx = O.maxpool2_bwd(dy, arg, x.shape)
    y = torch.empty(ref.shape, device="cuda")
    a = torch.empty(ref.shape, dtype=torch.uint8, device="cuda")
    ck(lib.unet_maxpool2_fwd(dev(x).data_ptr(), n, h, w, c, y.data_ptr(), a.data_ptr(), stream()))
    dx = torch.empty(x.shape, device="cuda")
    ck(lib.unet_maxpool2_bwd(dev(dy).data_ptr(), a.data_ptr(), n, h, w, c, dx.data_ptr(), stream()))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(host(y), ref)
    np.testing.assert_array_equal(a.cpu().numpy(), arg)
    np.testing.assert_allclose(host(dx), rdx, rtol=1e-6, atol=1e-7)


def test_batchnorm_train_fwd_bwd(lib):
    rng = np.random.default_rng(5)
    n, h, w, c = 2, 5, 7, 64
    x = rng.standard_normal((n, h, w, c)) * 2 + 1
    g = rng.uniform(0.5, 1.5, c)
    b = rng.standard_normal(c)
    dy = rng.standard_normal(x.shape)
    ry, cache, mean, var_unb = O.bn_train_fwd(x, g, b)
    rm, rv = O.bn_update_running(np.zeros(c), np.ones(c), mean, var_unb)
    rdx, rdg, rdb = O.bn_train_bwd(dy, cache, g)
    xd = dev(x)
    y = torch.empty_like(xd)
    rmd = torch.zeros(c, device="cuda")
    rvd = torch.ones(c, device="cuda")
    sm = torch.empty(c, device="cuda")
    si = torch.empty(c, device="cuda")
    ws = torch.empty(lib.unet_bn_ws_bytes(c), dtype=torch.uint8, device="cuda")
    gd, bd = dev(g), dev(b)
    ck(lib.unet_bn_train_fwd(xd.data_ptr(), n, h, w, c, gd.data_ptr(), bd.data_ptr(), rmd.data_ptr(),
                             rvd.data_ptr(), y.data_ptr(), sm.data_ptr(), si.data_ptr(), ws.data_ptr(), stream()))
    dx = torch.empty_like(xd)
    dg = torch.empty(c, device="cuda")
    dbt = torch.empty(c, device="cuda")
    ck(lib.unet_bn_train_bwd(xd.data_ptr(), dev(dy).data_ptr(), n, h, w, c, gd.data_ptr(), sm.data_ptr(),
                             si.data_ptr(), dx.data_ptr(), dg.data_ptr(), dbt.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(y), ry) < 1e-5
    assert rel_err(host(rmd), rm) < 1e-5 and rel_err(host(rvd), rv) < 1e-5
    assert rel_err(host(dx), rdx) < 1e-4
    assert rel_err(host(dg), rdg) < 1e-5 and rel_err(host(dbt), rdb) < 1e-5


def test_weighted_ce_strided_targets(lib):
    from unet_amd import WeightedCrossEntropyLoss
    rng = np.random.default_rng(6)
    n, hh = 2, 30
    logits = rng.standard_normal((n, 2, 20, 20)) * 3
    t_full = rng.integers(0, 2, (n, 1, hh, hh))
    w_full = rng.uniform(10, 13, (n, 1, hh, hh))
    tc = O.center_crop_target(t_full, 20, 20)
    wc = O.center_crop_target(w_full, 20, 20)
    rloss, rdl = O.weighted_ce(logits, tc, wc)
    # scripts/train.py:118-126: center_crop_tensor(...).squeeze(1) -> non-contiguous views
    td = torch.from_numpy(t_full).cuda()[:, :, 5:25, 5:25].squeeze(1)
    wd = dev(w_full)[:, :, 5:25, 5:25].squeeze(1)
    assert not td.is_contiguous()
    ld = dev(logits).requires_grad_(True)
    loss = WeightedCrossEntropyLoss()(ld, td, wd)
    (loss * 2.0).backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - rloss) <= 1e-5 * abs(rloss)
    assert rel_err(host(ld.grad), 2.0 * rdl) < 1e-5


def test_sgd_momentum(lib):
    z = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "ops.npz"))
    p = dev(np.pad(z["sgd.p0"], (0, 3)))
    buf = torch.zeros_like(p)
    for s in range(3):
        g = dev(np.pad(z["sgd.g"][s], (0, 3)))
        ck(lib.unet_sgd_momentum(p.data_ptr(), g.data_ptr(), buf.data_ptr(), 17, ctypes.c_float(1e-4),
                                 ctypes.c_float(0.99), ctypes.c_float(1.0), int(s == 0), stream()))
        torch.cuda.synchronize()
        np.testing.assert_allclose(host(p)[:17], z["sgd.traj"][s], rtol=1e-6, atol=1e-7)


def test_mask_and_iou(lib):
    rng = np.random.default_rng(7)
    logits = rng.standard_normal((2, 2, 9, 11)).astype(np.float32)
    logits[0, 1, 0, 0] = logits[0, 0, 0, 0]  # tie -> background (p > 0.5 is strict)
    gt = (rng.uniform(size=(2, 9, 11)) < 0.4).astype(np.uint8) * 7
    ref = O.predict_mask(logits)
    m = torch.empty((2, 9, 11), dtype=torch.uint8, device="cuda")
    ck(lib.unet_mask_from_logits(dev(logits).data_ptr(), m.data_ptr(), 2, 9, 11, stream()))
    cnt = torch.zeros(2, dtype=torch.int64, device="cuda")
    gtd = torch.from_numpy(gt).cuda()
    ck(lib.unet_iou_counts(m.data_ptr(), gtd.data_ptr(), m.numel(), cnt.data_ptr(), stream()))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(m.cpu().numpy(), ref)
    c = cnt.cpu().numpy()
    assert abs(c[0] / c[1] - O.calculate_iou(ref, gt)) < 1e-12
