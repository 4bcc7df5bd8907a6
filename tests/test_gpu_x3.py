"""Split-operand GEMMs (UNET_PREC_BF16X3) per op on the GPU, through the C-ABI.

Each fp32 operand is split v = hi + lo (hi = bf16(v), lo = bf16(v - hi)) and a
product is taken as hi*hi' + hi*lo' + lo*hi' on v_mfma_f32_32x32x16_bf16 with
fp32 accumulation.  The oracle is the plain fp64 op (oracle/unet_oracle.py, no
rounding): the split arithmetic is held to fp32-class accuracy, 3e-5 of the
output scale per op (the dropped lo*lo' term and the split residual are each
<= 2^-16 relative per product), where bf16 operands miss by ~1e-3.  The
whole-network checks at the fp32 tolerances are test_gpu_model.py's, run for
both "fp32" and "bf16x3".
"""
import ctypes

import numpy as np
import pytest

from oracle import unet_oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
PREC_BF16X3 = 2
TOL = 3e-5


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd import _lib
    return _lib.load()


_KEEP = []


def dev(a):
    t = torch.from_numpy(np.ascontiguousarray(a)).to("cuda", torch.float32)
    _KEEP.append(t)
    return t


@pytest.fixture(autouse=True)
def _release():
    yield
    if torch.cuda.is_available():
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


def f32(a):
    return np.asarray(a, np.float32).astype(np.float64)


q = O.round_bf16


@pytest.fixture
def op_x3(lib):
    lib.unet_set_tuning(b"op_precision", PREC_BF16X3)
    yield lib
    lib.unet_set_tuning(b"op_precision", 0)
    lib.unet_set_tuning(b"igemm_variant", -1)
    lib.unet_set_tuning(b"wgrad_variant", -1)


# -1 = built-in choice, 21-26 = row-gather k_igemm_bf tiles, 31/33/35 =
# halo-tiled k_conv3_bf (8x32, 16x16, 8x16) -- the tiles with a split-operand
# kernel (a forced tile that does not fit the shape falls back to the built-in)
VARIANTS = [-1, 21, 22, 23, 24, 25, 26, 31, 33, 35]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("n,h,w,ci,co,tf", [(2, 14, 13, 64, 128, False), (2, 11, 17, 64, 64, True),
                                              (1, 30, 41, 128, 256, True), (3, 9, 9, 256, 64, False)])
def test_x3_conv3x3_fwd(op_x3, n, h, w, ci, co, tf, variant):
    lib = op_x3
    lib.unet_set_tuning(b"igemm_variant", variant)
    rng = np.random.default_rng(10)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci))
    b = f32(rng.standard_normal(co))
    sc = f32(rng.uniform(-0.5, 1.5, ci)) if tf else None
    sh = f32(rng.standard_normal(ci) * 0.3) if tf else None
    xin = np.maximum(f32(x * sc + sh), 0) if tf else x
    ref = O.conv_valid_fwd(xin, wt, b)
    y = torch.empty((n, h - 2, w - 2, co), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_fwd(dev(x).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), dev(b).data_ptr(), co,
                            dev(sc).data_ptr() if tf else None, dev(sh).data_ptr() if tf else None,
                            y.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    e = rel_err(host(y), ref)
    print(f"fwd err {e:.2e} (bf16 operands: {rel_err(O.conv_valid_fwd(q(xin), q(wt), b), ref):.2e})")
    assert e < TOL


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 64, 64), (1, 19, 40, 128, 64), (2, 8, 8, 64, 256)])
def test_x3_conv3x3_dgrad(op_x3, n, h, w, ci, co, variant):
    lib = op_x3
    lib.unet_set_tuning(b"igemm_variant", variant)
    rng = np.random.default_rng(11)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci))
    dy = f32(rng.standard_normal((n, h - 2, w - 2, co)))
    ref, _, _ = O.conv_valid_bwd(x, wt, dy)
    dx = torch.empty((n, h, w, ci), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_dgrad(dev(dy).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), co, dx.data_ptr(),
                              ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    e = rel_err(host(dx), ref)
    print(f"dgrad err {e:.2e}")
    assert e < TOL


@pytest.mark.parametrize("variant", [-1, 10, 12, 14, 20, 21])
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 64, 64), (1, 40, 37, 128, 128), (2, 10, 9, 64, 128),
                                         (1, 7, 5, 64, 64), (2, 21, 44, 192, 128)])
def test_x3_conv3x3_wgrad(op_x3, n, h, w, ci, co, variant):
    """10/12/14 = pixel-column tiles (k_wgrad_bf), 20/21 = halo-tiled all-taps
    (k_wgrad3_bf); ragged pixel counts and grids."""
    lib = op_x3
    lib.unet_set_tuning(b"wgrad_variant", variant)
    rng = np.random.default_rng(12)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((co, ci, 3, 3)))
    dy = f32(rng.standard_normal((n, h - 2, w - 2, co)))
    _, rdw, _ = O.conv_valid_bwd(x, wt, dy, need_dx=False)
    rdb = dy.reshape(-1, co).sum(0)
    dw = torch.empty((co, ci, 3, 3), device="cuda")
    db = torch.empty(co, device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_wgrad(dev(x).data_ptr(), dev(dy).data_ptr(), n, h, w, ci, co, dw.data_ptr(),
                              db.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    e = rel_err(host(dw), rdw)
    print(f"wgrad err {e:.2e}")
    assert e < TOL
    assert rel_err(host(db), rdb) < 2e-5


@pytest.mark.parametrize("n,h,w,ci,co", [(2, 5, 7, 128, 64), (1, 6, 6, 256, 128)])
def test_x3_convT2_fwd_bwd(op_x3, n, h, w, ci, co):
    lib = op_x3
    rng = np.random.default_rng(13)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((ci, co, 2, 2)) / np.sqrt(ci))
    b = f32(rng.standard_normal(co))
    dy = f32(rng.standard_normal((n, 2 * h, 2 * w, co)))
    ref = O.convT2_fwd(x, wt, b)
    rdx, rdw, _ = O.convT2_bwd(x, wt, dy)
    rdb = dy.reshape(-1, co).sum(0)
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
    errs = [rel_err(host(y), ref), rel_err(host(dx), rdx), rel_err(host(dw), rdw)]
    print("convT errs", ["%.2e" % e for e in errs])
    assert max(errs) < TOL
    assert rel_err(host(db), rdb) < 2e-5
