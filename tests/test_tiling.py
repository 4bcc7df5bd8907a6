"""Overlap-tile inference (unet_amd.tiling): geometry and stitching on CPU,
parity of the GPU tile farm against per-tile oracle eval forwards."""
import numpy as np
import pytest
import torch

from oracle import unet_oracle as O


def test_margin_rule_matches_predict1():
    from unet_amd.tiling import TileGeometry, output_size
    # scripts/predict1.py:45-46: margin = tile_in - tile_out = 188 for 512
    assert 512 - output_size(512) == 188
    g = TileGeometry(1024, 1024, 512)
    assert (g.tile_out, g.margin, len(g)) == (324, 94, 16)
    assert g.pads[0] == 94 and g.pads[2] == 94
    # padded image exactly covers all input tiles
    assert 1024 + g.pads[0] + g.pads[1] == (g.ny - 1) * g.tile_out + g.tile_in


@pytest.mark.parametrize("hw,tile", [((1024, 1024), 512), ((700, 333), 512), ((100, 90), 220), ((37, 41), 204)])
def test_tiles_stitch_back_to_the_image(hw, tile):
    from unet_amd.tiling import TileGeometry, mirror_pad, extract_tiles, stitch
    H, W = hw
    img = torch.arange(H * W, dtype=torch.float32).reshape(1, H, W)
    g = TileGeometry(H, W, tile)
    padded = mirror_pad(img, g.pads)
    np.testing.assert_array_equal(padded.numpy(), O.mirror_pad(img.numpy(), g.pads))
    tiles = extract_tiles(padded, g, list(range(len(g))))
    m, t = g.margin, g.tile_out
    # an "identity U-Net": the valid output of a tile is its centre
    res = {i: tiles[i][:, m:m + t, m:m + t] for i in range(len(g))}
    np.testing.assert_array_equal(stitch(res, g, 1).numpy(), img.numpy())


def test_rank_share_partitions_tiles():
    from unet_amd.tiling import TileGeometry, rank_share
    g = TileGeometry(1024, 1024, 512)
    for world in (1, 2, 8):
        got = sorted(i for r in range(world) for i in rank_share(g, r, world))
        assert got == list(range(len(g)))


@pytest.mark.gpu
def test_tile_farm_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd import UNet
    from unet_amd.tiling import TileFarm, TileGeometry, mask_from_logits
    params = O.hash_init(1, 2, seed=31, bn_random=True)
    rng = np.random.default_rng(0)
    for k in params:  # plausible running statistics
        if k.endswith("running_mean"):
            params[k] = (0.2 * rng.standard_normal(params[k].shape)).astype(np.float32)
        if k.endswith("running_var"):
            params[k] = (0.5 + rng.uniform(size=params[k].shape)).astype(np.float32)
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    H, W, tile = 100, 90, 220
    img = (rng.uniform(size=(H, W)) * 2 - 1).astype(np.float32)
    farm = TileFarm(m, devices=[0], tile_in=tile, batch=4)
    logits = farm.predict(torch.from_numpy(img)).numpy()
    # two replicas on the one device: the round-robin deal (stride 2) and the
    # merge; batch 3 runs other GEMM shapes, so equal to fp32 noise, not bits
    farm2 = TileFarm(m, devices=[0, 0], tile_in=tile, batch=3)
    np.testing.assert_allclose(farm2.predict(torch.from_numpy(img)).numpy(), logits, rtol=0, atol=1e-4)
    mask2 = farm2.predict(torch.from_numpy(img), return_mask=True).numpy()
    # oracle: mirror pad, eval forward per tile, stitch
    g = TileGeometry(H, W, tile)
    padded = O.mirror_pad(img[None], g.pads)
    net = O.UNetOracle(params)
    ref = np.zeros((2, g.ny * g.tile_out, g.nx * g.tile_out))
    for (y, x) in g.origins:
        lg, _, _ = net.forward(padded[None, :, y:y + tile, x:x + tile], train=False)
        ref[:, y:y + g.tile_out, x:x + g.tile_out] = lg[0]
    ref = ref[:, :H, :W]
    assert np.abs(logits - ref).max() <= 1e-3
    mk = mask_from_logits(torch.from_numpy(logits)).numpy()
    sure = np.abs(ref[1] - ref[0]) > 1e-3
    np.testing.assert_array_equal(mk[sure], ((ref[1] > ref[0]) * 255).astype(np.uint8)[sure])
    np.testing.assert_array_equal(mask2[sure], mk[sure])


@pytest.mark.gpu
@pytest.mark.parametrize("c,h,w,tile,world,rank", [(1, 100, 90, 220, 1, 0), (3, 5, 7, 220, 2, 1),
                                                   (2, 300, 41, 220, 3, 2), (1, 1, 9, 220, 1, 0)])
def test_tile_gather_scatter_kernels(c, h, w, tile, world, rank):
    """unet_tile_gather vs the oracle's mirror padding (pads far beyond the
    image: repeated reflection; single-row image), unet_tile_scatter vs a
    host stitch, for one rank of a round-robin deal."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes
    from unet_amd import _lib
    from unet_amd.tiling import TileGeometry, rank_share
    lib = _lib.load()
    g = TileGeometry(h, w, tile)
    img = np.random.default_rng(h * w).standard_normal((c, h, w)).astype(np.float32)
    padded = O.mirror_pad(img, g.pads)
    mine = rank_share(g, rank, world)
    if not mine:
        pytest.skip("no tile for this rank")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    dimg = torch.from_numpy(img).cuda()
    tiles = torch.empty((len(mine), c, tile, tile), device="cuda")
    _lib.check(lib.unet_tile_gather(dimg.data_ptr(), c, h, w, tile, g.tile_out, g.pads[0], g.pads[2], g.nx, mine[0],
                                    world, len(mine), tiles.data_ptr(), st), "gather")
    got = tiles.cpu().numpy()
    for b, t in enumerate(mine):
        y, x = g.origins[t]
        np.testing.assert_array_equal(got[b], padded[:, y:y + tile, x:x + tile])
    to = g.tile_out
    lt = np.random.default_rng(1).standard_normal((len(mine), 2, to, to)).astype(np.float32)
    full = torch.full((2, h, w), 7.0, device="cuda")
    mask = torch.full((h, w), 3, dtype=torch.uint8, device="cuda")
    _lib.check(lib.unet_tile_scatter(torch.from_numpy(lt).cuda().data_ptr(), 2, to, g.nx, mine[0], world, len(mine),
                                     h, w, full.data_ptr(), mask.data_ptr(), st), "scatter")
    ref = np.full((2, g.ny * to, g.nx * to), 7.0, np.float32)
    for b, t in enumerate(mine):
        y, x = g.origins[t]
        ref[:, y:y + to, x:x + to] = lt[b]
    ref = ref[:, :h, :w]
    np.testing.assert_array_equal(full.cpu().numpy(), ref)
    covered = ref[0] != 7.0
    mk = mask.cpu().numpy()
    np.testing.assert_array_equal(mk[covered], ((ref[1] > ref[0]) * 255).astype(np.uint8)[covered])
    assert (mk[~covered] == 3).all()


@pytest.mark.gpu
def test_tile_farm_1024_vs_reference_fixture():
    """configs[3] at its size: a 1024^2 image (2x2 stitch of DIC-C2DH-HeLa 01
    frames, Normalize(0.5, 0.5)), 512^2 tiles, 16 tiles dealt round-robin over
    two replicas (devices [0, 0]), batch 8 per forward, mask straight from the
    tile scatter -- against the reference UNet run per tile on numpy's own
    mirror padding (tests/golden/farm_1024.npz): mask bit-exact on every pixel
    whose reference margin exceeds 1e-3, logits within 1e-3."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import os
    from oracle import fixtures as F
    from unet_amd import UNet
    from unet_amd.plan import Plan
    from unet_amd.tiling import TileFarm, TileGeometry
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "farm_1024.npz"), allow_pickle=False)
    params = F.plausible_running_stats(O.hash_init(1, 2, seed=int(z["seed"]), bn_random=True), int(z["seed"]))
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    img = torch.from_numpy(z["image"].astype(np.float32) / 255.0 * 2.0 - 1.0)
    H, W = img.shape
    g = TileGeometry(H, W, int(z["tile_in"]))
    assert (len(g), g.tile_out, g.margin) == (16, 324, 94)
    farm = TileFarm(m, devices=[0, 0], tile_in=int(z["tile_in"]), batch=8)
    mask = farm.predict(img, return_mask=True).numpy()
    logits = farm.predict(img).numpy()
    sure = np.unpackbits(z["sure"], axis=-1)[..., :W].astype(bool)
    ref_mask = np.unpackbits(z["mask"], axis=-1)[..., :W].astype(bool)
    np.testing.assert_array_equal(mask[sure] > 0, ref_mask[sure])
    assert set(np.unique(mask)) <= {0, 255}
    assert np.abs(logits[:, ::7, ::5] - z["logits_sample"]).max() <= 1e-3
    # eval forwards run in the forward-only workspace prefix (no gradient buffers)
    p = Plan(8, 1, 512, 512, 2)
    assert p.forward_workspace_bytes < 0.5 * p.workspace_bytes
    print(f"1024^2 farm: {int((~sure).sum())} low-margin pixels of {sure.size}")
