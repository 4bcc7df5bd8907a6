"""bf16-operand GEMM path (UNET_PREC_BF16; SURVEY.md §8a A1 "bf16-in/fp32-acc",
configs C3 / C5) on the GPU, through the C-ABI.

Oracle: UNetOracle(gemm="bf16") -- the same arithmetic as the HIP path (every
conv / convT / dgrad / wgrad operand rounded to bf16 after the producer's
BatchNorm+ReLU, exact accumulation, everything else unrounded).
* per op: the HIP kernels accumulate the same bf16 products in fp32, so they
  match to fp32 accumulation noise (rel <= 5e-5 of the output scale);
* whole network: the GPU's fp32 activations sit ~1e-7 away from the oracle's
  fp64 ones, so a rare operand lands on the other side of a bf16 rounding
  boundary and small-sample BatchNorm amplifies it.  The tolerance is
  self-calibrated like the fp32 tests: the same bf16 oracle run in plain fp32
  shows the size of that effect for each tensor.
* vs the fp32 reference: bf16 is a different arithmetic; the checks are the
  ones SURVEY.md §7 sets for it -- loss trajectory within 1 % and IoU on real
  HeLa frames.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import unet_oracle as O
from oracle import fixtures as F

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
G = os.path.join(os.path.dirname(__file__), "golden")
PREC_BF16 = 1


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd import _lib
    return _lib.load()


_KEEP = []


def dev(a, dtype=torch.float32):
    t = torch.from_numpy(np.ascontiguousarray(a)).to("cuda", dtype)
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


q = O.round_bf16


def f32(a):
    return np.asarray(a, np.float32).astype(np.float64)


@pytest.fixture
def op_bf16(lib):
    lib.unet_set_tuning(b"op_precision", PREC_BF16)
    yield lib
    lib.unet_set_tuning(b"op_precision", 0)
    lib.unet_set_tuning(b"igemm_variant", -1)
    lib.unet_set_tuning(b"wgrad_variant", -1)


# per-op GEMM tile: -1 = built-in choice (row-gather k_igemm_bf), 31-36 = the
# halo-tiled k_conv3_bf shapes (8x32, 16x16, 4x32/128, 8x16, 8x32/128), 41-44 =
# the persistent pipelined k_conv3p_bf (8x32 / 16x16, one or two rounds per CU)
HALO = [-1, 31, 32, 33, 34, 35, 36, 41, 42, 44]


# ------------------------------- per-op -------------------------------------
@pytest.mark.parametrize("variant", HALO)
@pytest.mark.parametrize("n,h,w,ci,co,tf", [(2, 14, 13, 64, 128, False), (2, 11, 17, 64, 64, True),
                                              (1, 30, 41, 128, 256, True), (3, 9, 9, 256, 64, False)])
def test_bf16_conv3x3_fwd(op_bf16, n, h, w, ci, co, tf, variant):
    """Grids smaller and larger than the halo tiles (overhanging tiles masked)."""
    lib = op_bf16
    lib.unet_set_tuning(b"igemm_variant", variant)
    rng = np.random.default_rng(10)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci))
    b = f32(rng.standard_normal(co))
    sc = f32(rng.uniform(-0.5, 1.5, ci)) if tf else None
    sh = f32(rng.standard_normal(ci) * 0.3) if tf else None
    # consumer transform in fp32 (one fma, then ReLU), then bf16
    xin = np.maximum(f32(x * sc + sh), 0) if tf else x
    ref = O.conv_valid_fwd(q(xin), q(wt), b)
    y = torch.empty((n, h - 2, w - 2, co), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_fwd(dev(x).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), dev(b).data_ptr(), co,
                            dev(sc).data_ptr() if tf else None, dev(sh).data_ptr() if tf else None,
                            y.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(y), ref) < 5e-5
    # and it is really bf16: the fp32 result is far further away than the noise
    assert rel_err(O.conv_valid_fwd(xin, wt, b), ref) > 1e-4


@pytest.mark.parametrize("variant", HALO)
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 64, 64), (1, 19, 40, 128, 64), (2, 8, 8, 64, 256)])
def test_bf16_conv3x3_dgrad(op_bf16, n, h, w, ci, co, variant):
    lib = op_bf16
    lib.unet_set_tuning(b"igemm_variant", variant)
    rng = np.random.default_rng(11)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci))
    dy = f32(rng.standard_normal((n, h - 2, w - 2, co)))
    ref, _, _ = O.conv_valid_bwd(x, q(wt), q(dy))
    dx = torch.empty((n, h, w, ci), device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_dgrad(dev(dy).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), co, dx.data_ptr(),
                              ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(dx), ref) < 5e-5


# k_conv3_dma (conv3_dma.hip): TH x 32 tiles, LDS-DMA weights, 2-stage ring;
# bf16-stored A only, so the per-op entry points run with op_a16 = 1 (x stored
# bf16 before its transform / padded dY bf16, as in a bf16 plan)
DMA = [63, 65, 66, 67, 68]


@pytest.mark.parametrize("variant", DMA + [31, 33, 81, 82, 83, 84, 88])
@pytest.mark.parametrize("n,h,w,ci,co,tf", [(2, 14, 13, 64, 128, False), (2, 11, 17, 64, 64, True),
                                              (1, 30, 41, 128, 256, True), (3, 9, 9, 256, 64, False),
                                              (1, 40, 70, 64, 64, True), (2, 21, 37, 192, 128, True)])
def test_bf16_conv3x3_fwd_a16(op_bf16, n, h, w, ci, co, tf, variant):
    """bf16-stored input (op_a16): the LDS-DMA halo kernels and the LDS-DMA ring
    (81-84), whose consumer BN+ReLU (tf) is applied to the raw halo in LDS, on
    ragged grids (chunks 32 / 64 channels: ci 192 runs three 64-channel chunks)."""
    if variant in (81, 84, 88) and ci % 64 or variant in (81, 83) and co % 128:
        pytest.skip("shape outside the ring tile's channel blocking")
    lib = op_bf16
    lib.unet_set_tuning(b"op_a16", 1)
    try:
        lib.unet_set_tuning(b"igemm_variant", variant)
        rng = np.random.default_rng(12)
        x = f32(rng.standard_normal((n, h, w, ci)))
        wt = f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci))
        b = f32(rng.standard_normal(co))
        sc = f32(rng.uniform(-0.5, 1.5, ci)) if tf else None
        sh = f32(rng.standard_normal(ci) * 0.3) if tf else None
        xq = f32(q(x))
        xin = np.maximum(f32(xq * sc + sh), 0) if tf else xq
        ref = O.conv_valid_fwd(q(xin), q(wt), b)
        y = torch.empty((n, h - 2, w - 2, co), device="cuda")
        ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
        ck(lib.unet_conv3x3_fwd(dev(x).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), dev(b).data_ptr(), co,
                                dev(sc).data_ptr() if tf else None, dev(sh).data_ptr() if tf else None,
                                y.data_ptr(), ws.data_ptr(), stream()))
        torch.cuda.synchronize()
        assert rel_err(host(y), ref) < 5e-5
    finally:
        lib.unet_set_tuning(b"op_a16", 0)


@pytest.mark.parametrize("pt,base", [(88, 84)])
@pytest.mark.parametrize("kind", ["fwd", "fwd_tf", "dgrad"])
def test_bf16_ring_persistent_bitexact(op_bf16, pt, base, kind):
    """The persistent ring tile (88: each workgroup walks pixel tiles with
    the next tile's halo and tap-0/1 weights in flight during this tile's last
    chunk and epilogue) against the one-tile-per-workgroup geometry it shares
    (84): the same arithmetic per tile, so bit-identical outputs, on a grid
    of 306 tiles -- more than the resident workgroups, so every one wraps; with
    the consumer BN+ReLU applied in LDS (fwd_tf: the next tile's halo is
    transformed at the current tile's last tap step) and as an input gradient."""
    lib = op_bf16
    n, h, w, ci, co = 2, 138, 290, 64, 128
    rng = np.random.default_rng(21)
    x = dev(f32(rng.standard_normal((n, h, w, ci))))
    wt = dev(f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci)))
    b = dev(f32(rng.standard_normal(co)))
    sc = dev(f32(rng.uniform(-0.5, 1.5, ci)))
    sh = dev(f32(rng.standard_normal(ci) * 0.3))
    dy = dev(f32(rng.standard_normal((n, h - 2, w - 2, co))))
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    lib.unet_set_tuning(b"op_a16", 1)
    outs = []
    try:
        for v in (base, pt):
            lib.unet_set_tuning(b"igemm_variant", v)
            if kind == "dgrad":
                out = torch.full((n, h, w, ci), float("nan"), device="cuda")
                ck(lib.unet_conv3x3_dgrad(dy.data_ptr(), n, h, w, ci, wt.data_ptr(), co, out.data_ptr(),
                                          ws.data_ptr(), stream()))
            else:
                tf = kind == "fwd_tf"
                out = torch.full((n, h - 2, w - 2, co), float("nan"), device="cuda")
                ck(lib.unet_conv3x3_fwd(x.data_ptr(), n, h, w, ci, wt.data_ptr(), b.data_ptr(), co,
                                        sc.data_ptr() if tf else None, sh.data_ptr() if tf else None,
                                        out.data_ptr(), ws.data_ptr(), stream()))
            torch.cuda.synchronize()
            outs.append(out)
    finally:
        lib.unet_set_tuning(b"op_a16", 0)
        lib.unet_set_tuning(b"igemm_variant", -1)
    assert torch.isfinite(outs[1]).all()
    assert torch.equal(outs[0], outs[1])


def _flat_tiling(n, hg, wg, bm=256, npx=400):
    """conv3_flat.hip's flat_map: ("cross" | "image" | None, tiles, worst
    halo run in pixels) of an (n, hg, wg) output grid."""
    hw, hin, win = hg * wg, hg + 2, wg + 2

    def qin(p):
        img, rem = divmod(p, hw)
        y, x = divmod(rem, wg)
        return (img * hin + y) * win + x

    def span(p0, c):
        return qin(p0 + c - 1) + 2 * win + 2 - qin(p0) + 1
    m = n * hw
    nt = (m + bm - 1) // bm
    worst = max(span(t * bm, min(bm, m - t * bm)) for t in range(nt))
    if worst <= npx:
        return "cross", nt, worst
    tpi = (hw + bm - 1) // bm
    worst = max(span(t * bm, min(bm, hw - t * bm)) for t in range(tpi))
    return ("image" if worst <= npx else None), n * tpi, worst


@pytest.mark.parametrize("kind", ["fwd", "fwd_tf", "dgrad"])
@pytest.mark.parametrize("n,h,w,ci,co", [(8, 26, 26, 128, 128), (2, 48, 48, 64, 128), (3, 30, 50, 64, 256),
                                         (1, 10, 9, 64, 128), (8, 28, 28, 64, 256)])
def test_bf16_flat_tile_bitexact_vs_ring(op_bf16, kind, n, h, w, ci, co):
    """The ring on flat pixel tiles (85, conv3_flat.hip: 256 consecutive
    output pixels per tile, fragments wrapping grid rows, tiles crossing image
    boundaries or per image) against the row-tiled ring of the same chunk / tap /
    k-step order (81): bit-identical outputs -- on grids narrower than a
    fragment (24, 26, 28), a 46-wide one, H != W with an odd batch, and a
    single tile with idle rows."""
    lib = op_bf16
    # the shapes are ones tile 85 takes (else the forced variant falls back)
    assert _flat_tiling(n, h - 2, w - 2)[0] and _flat_tiling(n, h, w)[0]
    rng = np.random.default_rng(h * 1000 + w)
    x = dev(f32(rng.standard_normal((n, h, w, ci))))
    wt = dev(f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci)))
    b = dev(f32(rng.standard_normal(co)))
    sc = dev(f32(rng.uniform(-0.5, 1.5, ci)))
    sh = dev(f32(rng.standard_normal(ci) * 0.3))
    dy = dev(f32(rng.standard_normal((n, h - 2, w - 2, co))))
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    lib.unet_set_tuning(b"op_a16", 1)
    outs = []
    try:
        for v in (81, 85):
            lib.unet_set_tuning(b"igemm_variant", v)
            if kind == "dgrad":
                out = torch.full((n, h, w, ci), float("nan"), device="cuda")
                ck(lib.unet_conv3x3_dgrad(dy.data_ptr(), n, h, w, ci, wt.data_ptr(), co, out.data_ptr(),
                                          ws.data_ptr(), stream()))
            else:
                tf = kind == "fwd_tf"
                out = torch.full((n, h - 2, w - 2, co), float("nan"), device="cuda")
                ck(lib.unet_conv3x3_fwd(x.data_ptr(), n, h, w, ci, wt.data_ptr(), b.data_ptr(), co,
                                        sc.data_ptr() if tf else None, sh.data_ptr() if tf else None,
                                        out.data_ptr(), ws.data_ptr(), stream()))
            torch.cuda.synchronize()
            outs.append(out)
    finally:
        lib.unet_set_tuning(b"op_a16", 0)
        lib.unet_set_tuning(b"igemm_variant", -1)
    assert torch.isfinite(outs[1]).all()
    assert torch.equal(outs[0], outs[1]), float((outs[0] - outs[1]).abs().max())


@pytest.mark.parametrize("kind", ["fwd", "fwd_tf", "dgrad"])
@pytest.mark.parametrize("n,h,w", [(2, 12, 11), (1, 40, 70), (8, 130, 131), (3, 9, 200)])
def test_bf16_conv3x3_c64_resident_weights(op_bf16, kind, n, h, w):
    """Tile 87 (conv3_c64.hip: 64 -> 64 channels, the weight slab resident in
    LDS, persistent workgroups walking double-buffered halo tiles) against the
    bf16-operand oracle: forward with and without the consumer BN+ReLU applied
    in LDS, and the input gradient; grids with fewer and with more tiles (680)
    than workgroups, ragged in both axes."""
    lib = op_bf16
    ci = co = 64
    lib.unet_set_tuning(b"op_a16", 1)
    try:
        lib.unet_set_tuning(b"igemm_variant", 87)
        rng = np.random.default_rng(h * 7 + w)
        x = f32(rng.standard_normal((n, h, w, ci)))
        wt = f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci))
        ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
        if kind == "dgrad":
            dy = f32(rng.standard_normal((n, h - 2, w - 2, co)))
            ref, _, _ = O.conv_valid_bwd(x, q(wt), q(dy))
            out = torch.full((n, h, w, ci), float("nan"), device="cuda")
            ck(lib.unet_conv3x3_dgrad(dev(dy).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), co, out.data_ptr(),
                                      ws.data_ptr(), stream()))
        else:
            tf = kind == "fwd_tf"
            b = f32(rng.standard_normal(co))
            sc = f32(rng.uniform(-0.5, 1.5, ci)) if tf else None
            sh = f32(rng.standard_normal(ci) * 0.3) if tf else None
            xq = f32(q(x))
            xin = np.maximum(f32(xq * sc + sh), 0) if tf else xq
            ref = O.conv_valid_fwd(q(xin), q(wt), b)
            out = torch.full((n, h - 2, w - 2, co), float("nan"), device="cuda")
            ck(lib.unet_conv3x3_fwd(dev(x).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), dev(b).data_ptr(), co,
                                    dev(sc).data_ptr() if tf else None, dev(sh).data_ptr() if tf else None,
                                    out.data_ptr(), ws.data_ptr(), stream()))
        torch.cuda.synchronize()
        assert rel_err(host(out), ref) < 5e-5
    finally:
        lib.unet_set_tuning(b"op_a16", 0)
        lib.unet_set_tuning(b"igemm_variant", -1)


@pytest.mark.parametrize("variant", DMA)
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 64, 64), (1, 19, 40, 128, 64), (2, 8, 8, 64, 256),
                                         (1, 36, 66, 64, 128)])
def test_bf16_conv3x3_dgrad_a16(op_bf16, n, h, w, ci, co, variant):
    lib = op_bf16
    lib.unet_set_tuning(b"op_a16", 1)
    try:
        lib.unet_set_tuning(b"igemm_variant", variant)
        rng = np.random.default_rng(13)
        x = f32(rng.standard_normal((n, h, w, ci)))
        wt = f32(rng.standard_normal((co, ci, 3, 3)) / np.sqrt(9 * ci))
        dy = f32(rng.standard_normal((n, h - 2, w - 2, co)))
        ref, _, _ = O.conv_valid_bwd(x, q(wt), q(dy))
        dx = torch.empty((n, h, w, ci), device="cuda")
        ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
        ck(lib.unet_conv3x3_dgrad(dev(dy).data_ptr(), n, h, w, ci, dev(wt).data_ptr(), co, dx.data_ptr(),
                                  ws.data_ptr(), stream()))
        torch.cuda.synchronize()
        assert rel_err(host(dx), ref) < 5e-5
    finally:
        lib.unet_set_tuning(b"op_a16", 0)


@pytest.mark.parametrize("variant", [-1, 10, 12, 20, 21])
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 64, 64), (1, 40, 37, 128, 128), (2, 10, 9, 64, 128),
                                         (1, 7, 5, 64, 64), (2, 21, 44, 192, 128)])
def test_bf16_conv3x3_wgrad(op_bf16, n, h, w, ci, co, variant):
    """Pixel counts that are not multiples of the K step and grids that are not
    multiples of the halo tiles (ragged tails); 10/12 = pixel-column tiles
    (k_wgrad_bf), 20/21 = halo-tiled all-taps kernel (k_wgrad3_bf, 8x16 / 4x32)."""
    lib = op_bf16
    lib.unet_set_tuning(b"wgrad_variant", variant)
    rng = np.random.default_rng(12)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((co, ci, 3, 3)))
    dy = f32(rng.standard_normal((n, h - 2, w - 2, co)))
    _, rdw, _ = O.conv_valid_bwd(q(x), wt, q(dy), need_dx=False)
    rdb = dy.reshape(-1, co).sum(0)
    dw = torch.empty((co, ci, 3, 3), device="cuda")
    db = torch.empty(co, device="cuda")
    ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
    ck(lib.unet_conv3x3_wgrad(dev(x).data_ptr(), dev(dy).data_ptr(), n, h, w, ci, co, dw.data_ptr(),
                              db.data_ptr(), ws.data_ptr(), stream()))
    torch.cuda.synchronize()
    assert rel_err(host(dw), rdw) < 5e-5
    assert rel_err(host(db), rdb) < 2e-5


@pytest.mark.parametrize("variant", [-1, 20, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33])
@pytest.mark.parametrize("n,h,w,ci,co", [(2, 12, 11, 128, 128), (1, 40, 37, 128, 128), (2, 21, 44, 256, 128),
                                         (1, 7, 5, 128, 64), (2, 30, 19, 64, 256), (1, 3, 3, 128, 128)])
def test_bf16_conv3x3_wgrad_bf16_storage(op_bf16, n, h, w, ci, co, variant):
    """bf16-stored dY (zero-bordered padded copy) and X (op_a16, as a bf16 plan
    stores them): the halo-tiled k_wgrad3_bf (20), the wide two-stage-ring
    k_wgrad3w_bf (24: 128 co x 64 ci, 25: 64 co x 128 ci per workgroup) and the
    LDS-DMA ring k_wgrad3_ring (26: 128 co x 64 ci with 4x16 pixel tiles, 27:
    the same with 8x8 tiles, 28: 64 x 64, 29: 64 co x 128 ci, 30 / 31: 64 x 64
    with 8x16 / 8x8 tiles, 32 / 33: the all-taps "slide" mapping at 128 x 64 /
    64 x 128) on ragged grids, including a grid smaller than one pixel tile."""
    need = {24: (128, 64), 25: (64, 128), 26: (128, 64), 27: (128, 64), 28: (64, 64), 29: (64, 128), 30: (64, 64),
            31: (64, 64), 32: (128, 64), 33: (64, 128)}
    if variant in need and (co % need[variant][0] or ci % need[variant][1]):
        pytest.skip("shape outside the tile's channel blocking")
    lib = op_bf16
    lib.unet_set_tuning(b"op_a16", 1)
    lib.unet_set_tuning(b"wgrad_variant", variant)
    try:
        rng = np.random.default_rng(14)
        x = f32(rng.standard_normal((n, h, w, ci)))
        dy = f32(rng.standard_normal((n, h - 2, w - 2, co)))
        _, rdw, _ = O.conv_valid_bwd(q(x), np.zeros((co, ci, 3, 3), np.float32), q(dy), need_dx=False)
        dw = torch.empty((co, ci, 3, 3), device="cuda")
        ws = torch.empty(lib.unet_conv_ws_bytes(n, h, w, ci, co), dtype=torch.uint8, device="cuda")
        ck(lib.unet_conv3x3_wgrad(dev(x).data_ptr(), dev(dy).data_ptr(), n, h, w, ci, co, dw.data_ptr(),
                                  None, ws.data_ptr(), stream()))
        torch.cuda.synchronize()
        assert rel_err(host(dw), rdw) < 5e-5
    finally:
        lib.unet_set_tuning(b"op_a16", 0)
        lib.unet_set_tuning(b"wgrad_variant", -1)


@pytest.mark.parametrize("n,h,w,ci,co", [(2, 5, 7, 128, 64), (1, 6, 6, 256, 128)])
def test_bf16_convT2_fwd_bwd(op_bf16, n, h, w, ci, co):
    lib = op_bf16
    rng = np.random.default_rng(13)
    x = f32(rng.standard_normal((n, h, w, ci)))
    wt = f32(rng.standard_normal((ci, co, 2, 2)) / np.sqrt(ci))
    b = f32(rng.standard_normal(co))
    dy = f32(rng.standard_normal((n, 2 * h, 2 * w, co)))
    ref = O.convT2_fwd(q(x), q(wt), b)
    rdx, rdw, _ = O.convT2_bwd(q(x), q(wt), q(dy))
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
    assert rel_err(host(y), ref) < 5e-5
    assert rel_err(host(dx), rdx) < 5e-5
    assert rel_err(host(dw), rdw) < 5e-5
    assert rel_err(host(db), rdb) < 2e-5


# ------------------------------ whole network --------------------------------
def make_model(params, precision="bf16", n_channels=1):
    from unet_amd import UNet
    m = UNet(n_channels, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    m.precision = precision
    return m.cuda()


def bf16_oracle_step(params, x, tgt, wmap, dtype=np.float64):
    net = O.UNetOracle(params, dtype=dtype, gemm="bf16")
    rl, cache, nb = net.forward(x)
    rloss, rdl = O.weighted_ce(rl, tgt, wmap)
    rg = net.backward(np.asarray(rdl, dtype), cache)
    return rl, rloss, rg, nb


def check_vs_bf16_oracle(m, params, x, tgt, wmap, tag=""):
    from unet_amd import WeightedCrossEntropyLoss
    rl, rloss, rg, _ = bf16_oracle_step(params, x, tgt, wmap)
    l32, loss32, g32, _ = bf16_oracle_step(params, x, tgt, wmap, np.float32)  # the rounding-boundary noise floor
    m.train()
    m.zero_grad()
    logits = m(torch.from_numpy(x).cuda())
    loss = WeightedCrossEntropyLoss()(logits, torch.from_numpy(tgt).cuda(), torch.from_numpy(wmap).cuda())
    loss.backward()
    torch.cuda.synchronize()
    lg = host(logits)
    scale = np.abs(rl).max()
    lerr, lfloor = np.abs(lg - rl).max() / scale, np.abs(l32 - rl).max() / scale
    # 3e-3 of the logit scale: under one bf16 ulp (2^-8) of the largest logit
    assert lerr <= max(3e-3, 4 * lfloor), (tag, lerr, lfloor)
    lo_err, lo_floor = abs(loss.item() - rloss) / abs(rloss), abs(loss32 - rloss) / abs(rloss)
    # the loss averages the logits: its noise is bounded by theirs
    assert lo_err <= max(1e-4, 4 * lo_floor, 0.5 * lfloor), (tag, lo_err, lo_floor)
    worst = 0.0
    for name, p in m.named_parameters():
        g = host(p.grad)
        r = np.asarray(rg[name], np.float64)
        if O.bn_cancelled(name):
            # analytically zero; with bf16 dgrad operands sum_p dY no longer
            # cancels exactly, so the residue is rounding noise of the size the
            # bf16 oracle itself shows (fp64 and fp32 runs)
            resid = max(np.abs(r).max(), np.abs(np.asarray(g32[name])).max())
            assert np.abs(g).max() <= 3 * resid + 1e-3 * np.abs(rg[name.replace(".bias", ".weight")]).max(), name
            continue
        nr = max(np.linalg.norm(r), 1e-30)
        e = np.linalg.norm(g - r) / nr
        floor = np.linalg.norm(np.asarray(g32[name], np.float64) - r) / nr
        tol = max(2e-2, 3 * floor)
        worst = max(worst, e / tol)
        assert e <= tol, (tag, name, e, floor)
    print(f"{tag}: logits {lerr:.2e} (floor {lfloor:.2e}), loss {lo_err:.2e} (floor {lo_floor:.2e}), "
          f"worst grad err / tol {worst:.2f}")


@pytest.mark.parametrize("n,h,w,seed", [(2, 188, 188, 11), (2, 204, 204, 12), (1, 220, 220, 13), (2, 188, 220, 41),
                                        (1, 204, 252, 42)])
def test_bf16_train_step_vs_bf16_oracle(lib, n, h, w, seed):
    """Square and H != W batches (the plan crops each axis on its own,
    models/unet_model.py:93-100)."""
    params = O.hash_init(1, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, 1, h, w)
    check_vs_bf16_oracle(make_model(params), params, x, tgt, wmap, f"{n}x{h}x{w}")


@pytest.fixture
def gemm_mode(request, lib):
    mode = request.param
    lib.unet_tuning_reset()
    for part in mode.split("+"):
        if part == "heuristic":
            lib.unet_set_tuning(b"autotune", 0)
        elif part == "norm":  # normalised bf16 operand copies (the ring tiles 81-84 need them)
            lib.unet_set_tuning(b"bf16_norm", 1)
        elif part.startswith("split"):
            lib.unet_set_tuning(b"force_split", int(part[5:]))
        elif part.startswith("tile"):
            lib.unet_set_tuning(b"force_tile", int(part[4:]))
        elif part.startswith("wtile"):  # every weight gradient that fits it (with "heuristic")
            lib.unet_set_tuning(b"wgrad_variant", int(part[5:]))
    yield mode
    lib.unet_set_tuning(b"wgrad_variant", -1)
    lib.unet_set_tuning(b"bf16_norm", 0)
    lib.unet_set_tuning(b"autotune", 1)
    lib.unet_set_tuning(b"force_split", 0)
    lib.unet_set_tuning(b"force_tile", 0)
    lib.unet_tuning_reset()


@pytest.mark.parametrize("gemm_mode", ["heuristic", "tile21", "tile22", "tile23", "tile24", "tile25", "tile26",
                                       "tile22+split3", "tile24+split8", "tile31", "tile32", "tile33", "tile34",
                                       "tile35", "tile36", "tile31+split2", "tile34+split3", "tile41", "tile42",
                                       "tile43", "tile44", "tile41+split3", "tile63", "tile65", "tile66",
                                       "tile67", "tile67+split3", "tile63+split2", "norm+tile81", "norm+tile82",
                                       "norm+tile83", "norm+tile84", "norm+tile81+split3", "norm+tile83+split2",
                                       "norm+tile31", "norm+heuristic", "tile81", "tile82", "tile83", "tile84",
                                       "tile88", "norm+tile88", "tile85", "norm+tile85", "tile85+split3", "tile86", "norm+tile86", "tile87", "norm+tile87",
                                       "norm+tile85+split2",
                                       "tile81+split3", "heuristic+wtile26", "heuristic+wtile27",
                                       "heuristic+wtile126", "heuristic+wtile130", "heuristic+wtile132",
                                       "heuristic+wtile110", "heuristic+wtile112",
                                       "heuristic+wtile28", "heuristic+wtile29", "heuristic+wtile30",
                                       "heuristic+wtile31", "heuristic+wtile32", "heuristic+wtile33",
                                       "norm+heuristic+wtile26", "tile91", "tile92", "tile93", "tile94",
                                       "tile95", "tile96", "tile97", "tile98", "tile99", "tile92+split2",
                                       "tile95+split3", "tile96+split2",
                                       "heuristic+wtile140", "heuristic+wtile141", "heuristic+wtile142",
                                       "heuristic+wtile143", "heuristic+wtile144", "heuristic+wtile40",
                                       "heuristic+wtile43"],
                         indirect=True)
def test_bf16_gemm_variants_vs_bf16_oracle(gemm_mode):
    """Every bf16 tile (21-26 row gather, 31-36 halo-tiled 3x3, 63-67 LDS-DMA
    halo, 81-84 LDS-DMA halo / weight rings -- the convT GEMMs fall back to the
    built-in tile there; 91-95 the convT forward / input-gradient K rings --
    the 3x3 GEMMs fall back there) and split-K on every conv / convT / dgrad
    GEMM of a train step; the weight gradients run the bf16 wgrad tiles
    (wtile140-144: the convT weight-gradient ring tiles 40-44 in slab mode on
    every convT layer they fit; wtile40 / 43: the same with fp32 atomics)."""
    params = O.hash_init(1, 2, seed=21, bn_random=True)
    x, tgt, wmap = F.make_inputs(21, 2, 1, 188)
    check_vs_bf16_oracle(make_model(params), params, x, tgt, wmap, gemm_mode)


@pytest.mark.parametrize("wtile", [140, 141, 142, 143, 144])
@pytest.mark.parametrize("n,h,w,seed", [(2, 204, 204, 22), (1, 220, 252, 23), (3, 196, 196, 24)])
def test_bf16_convT_wgrad_ring_vs_bf16_oracle(wtile, n, h, w, seed):
    """The convT weight-gradient ring (wgradT_ring.hip, tiles 40-44 in slab
    mode) on every convT layer of a whole train step where it fits, at sizes
    whose pixel counts leave ragged last stages and splits (the zeroed tail
    rows), an H != W batch and an odd batch."""
    from unet_amd import _lib
    lib = _lib.load()
    lib.unet_tuning_reset()
    lib.unet_set_tuning(b"autotune", 0)
    lib.unet_set_tuning(b"wgrad_variant", wtile)
    try:
        params = O.hash_init(1, 2, seed=seed, bn_random=True)
        x, tgt, wmap = F.make_inputs(seed, n, 1, h, w)
        check_vs_bf16_oracle(make_model(params), params, x, tgt, wmap, f"wtile{wtile} {n}x{h}x{w}")
    finally:
        lib.unet_set_tuning(b"wgrad_variant", -1)
        lib.unet_set_tuning(b"autotune", 1)
        lib.unet_tuning_reset()


def test_bf16_3ch_572_forward_vs_fp32_fixture(lib):
    """configs[4] shape (3-ch 572x572, 388x388 out): the bf16 forward against the
    reference's fp32 fixture -- the bf16 accuracy cost on the stress shape."""
    from unet_amd import WeightedCrossEntropyLoss
    z = np.load(os.path.join(G, "fwd_n1_c3_572.npz"), allow_pickle=False)
    seed, n, h, c = int(z["x_seed"]), int(z["n"]), int(z["h"]), int(z["c"])
    params = O.hash_init(c, 2, seed=seed, bn_random=True)
    x, tgt, wmap = F.make_inputs(seed, n, c, h)
    m = make_model(params, n_channels=c)
    with torch.no_grad():
        logits = m(torch.from_numpy(x).cuda())
        loss = WeightedCrossEntropyLoss()(logits, torch.from_numpy(tgt).cuda(), torch.from_numpy(wmap).cuda())
    lg = host(logits)
    ref = z["logits_sample"]
    got = lg[:, :, ::7, ::5]
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    lo = abs(loss.item() - float(z["loss"])) / abs(float(z["loss"]))
    agree = ((lg[:, 1] > lg[:, 0]) == z["mask"].astype(bool)).mean()
    print(f"3ch-572 bf16 vs fp32 reference: logits rel-L2 {rel:.2e}, loss rel {lo:.2e}, mask agreement {agree:.5f}")
    assert rel < 2e-2 and lo < 1e-2 and agree > 0.99


def test_autocast_bf16_selects_bf16_plan(lib):
    """torch.autocast('cuda', dtype=torch.bfloat16) around the drop-in UNet runs
    the bf16 GEMMs (the reference's convs would run in bf16 there)."""
    params = O.hash_init(1, 2, seed=5, bn_random=True)
    x = torch.from_numpy(F.make_inputs(5, 2, 1, 188)[0]).cuda()
    m = make_model(params, precision=None)
    m.eval()
    with torch.no_grad():
        ref32 = m(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            got = m(x)
        m.precision = "bf16"
        ref16 = m(x)
    assert got.dtype == torch.float32
    assert torch.equal(got, ref16)
    assert float((got - ref32).abs().max()) > 1e-5


def test_bf16_trainer_loss_trajectory_within_1pct_of_fp32(lib):
    """bf16 configs are judged by the loss trajectory (within 1 %)
    against the fp32 path; 30 train.py steps (SGD 0.99, lr 1e-4) at 2x204.
    This tiny problem is memorised within 30 steps (loss 44 -> 0.25), so the
    deviation is measured against the trajectory's scale (its first loss):
    relative to a loss that has collapsed to 0.5 % of it, rounding noise of
    either precision is not a trajectory difference."""
    from unet_amd.train import Trainer
    params = O.hash_init(1, 2, seed=7, bn_random=True)
    x, tgt, wmap = (torch.from_numpy(a).cuda() for a in F.make_inputs(7, 2, 1, 204))
    runs = {}
    for prec in ("fp32", "bf16"):
        m = make_model(params, precision=prec)
        tr = Trainer(m, 2, 204, 204, lr=1e-4, momentum=0.99, precision=prec)
        runs[prec] = [float(tr.step(x, tgt, wmap)) for _ in range(30)]
    a, b = np.array(runs["fp32"]), np.array(runs["bf16"])
    dev_ = np.abs(b - a) / a[0]
    print(f"loss fp32 {a[0]:.4f} -> {a[-1]:.4f}, bf16 {b[0]:.4f} -> {b[-1]:.4f}, "
          f"max |bf16 - fp32| / loss0 {dev_.max():.2e}, first-step rel {abs(b[0] - a[0]) / a[0]:.2e}")
    assert a[-1] < 0.1 * a[0] and b[-1] < 0.1 * b[0]
    assert dev_.max() <= 1e-2


def test_bf16_hela_real_frames_iou(lib):
    """Real DIC-C2DH-HeLa frames, eval mode (predict.py): IoU vs 01_ST/SEG of the
    bf16 path against the reference's (fp32) IoU on the same weights."""
    z = np.load(os.path.join(G, "hela_real.npz"), allow_pickle=False)
    params = O.hash_init(1, 2, seed=int(z["seed"]), bn_random=True)
    for k in z.files:
        if k.startswith("buf/"):
            params[k[4:]] = z[k].astype(np.float32)
    m = make_model(params)
    m.eval()
    x = (z["images"].astype(np.float32)[:, None] / 255.0) * 2.0 - 1.0
    with torch.no_grad():
        lg = host(m(torch.from_numpy(x).cuda()))
    mk = lg[:, 1] > lg[:, 0]
    oy = (512 - 324) // 2
    gt = z["segs"][:, oy:oy + 324, oy:oy + 324] > 0
    ious = np.array([O.calculate_iou(mk[i], gt[i]) for i in range(len(mk))])
    agree = (mk == (z["masks"] > 0)).mean()
    print(f"HeLa bf16: IoU {ious.round(4)} vs reference {np.asarray(z['ious']).round(4)}, mask agreement {agree:.5f}")
    np.testing.assert_allclose(ious, z["ious"], atol=1e-3)
