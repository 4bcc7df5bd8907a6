"""CPU checks of the C-ABI library and the host-side plan logic (no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import unet_oracle as O

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _lib():
    from unet_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libunet_hip.so not built (run __graft_entry__.build())")
    return _lib


def test_library_exports_every_header_symbol():
    L = _lib()
    lib = L.load()
    header = open(os.path.join(ROOT, "include", "unet_hip.h")).read()
    header = re.sub(r"/\*.*?\*/", "", header, flags=re.S)
    names = set(re.findall(r"\b(unet_[A-Za-z0-9_]+)\s*\(", header))
    assert len(names) >= 25
    for n in sorted(names):
        assert hasattr(lib, n), f"missing export {n}"
    # and the binding declares exactly the header's functions
    assert names == set(L.SIGNATURES), names ^ set(L.SIGNATURES)
    assert b"gfx950" in lib.unet_version()


@pytest.mark.parametrize("h,out", [(512, 324), (572, 388), (188, 4), (204, 20), (508, 324)])
def test_plan_output_size_matches_reference_rule(h, out):
    from unet_amd.plan import Plan
    _lib()
    p = Plan(2, 1, h, h, 2)
    assert (p.out_h, p.out_w) == (out, out) == (O.output_size(h),) * 2
    assert p.workspace_bytes > 0


def test_tuning_db_roundtrip(tmp_path):
    """unet_tuning_load / _save (host-only: no GPU call): a database file is
    merged into the tuner's cache, reported, written back line for line."""
    L = _lib()
    lib = L.load()
    src = tmp_path / "tune.db"
    entries = {"igemm_bf16 M=8 N=64 K=576 Cg=64 taps=3x3 s=1 grid=4x4 epi=18": (31, 1),
               "wgrad Mo=64 No=576 P=16 Cg=64 taps=3x3 s=1 grid=4x4": (74, 504)}
    src.write_text("".join(f"{k}\t{t}\t{s}\n" for k, (t, s) in entries.items()) + "malformed line\n")
    lib.unet_tuning_reset()
    try:
        assert lib.unet_tuning_load(str(src).encode()) == 2
        n = lib.unet_tuning_report(None, 0)
        buf = ctypes.create_string_buffer(n)
        lib.unet_tuning_report(buf, n)
        assert buf.value.decode().count("tuning db") == 2, buf.value
        out = tmp_path / "out.db"
        assert lib.unet_tuning_save(str(out).encode()) == 2
        got = {}
        for line in out.read_text().splitlines():
            k, t, s = line.split("\t")
            got[k] = (int(t), int(s))
        assert got == entries
        assert lib.unet_tuning_load(str(tmp_path / "absent.db").encode()) < 0
    finally:
        lib.unet_tuning_reset()


def test_plan_rejects_too_small_input():
    from unet_amd.plan import Plan
    _lib()
    with pytest.raises(ValueError):
        Plan(1, 1, 100, 100, 2)


def test_plan_workspace_scales_with_batch():
    from unet_amd.plan import Plan
    _lib()
    a = Plan(1, 1, 512, 512, 2).workspace_bytes
    a2 = Plan(2, 1, 512, 512, 2).workspace_bytes
    b = Plan(8, 1, 512, 512, 2).workspace_bytes
    per_image = a2 - a               # activations scale with N, packed weights do not
    assert abs((b - a) - 7 * per_image) < 7 * 2**20
    assert b < 40 * 2**30  # fits easily in 288 GB HBM


def test_segments_cover_all_grads_once():
    from unet_amd.plan import Plan, N_GRADS, N_SEGMENTS
    _lib()
    p = Plan(1, 1, 188, 188, 2)
    seen = []
    for s in range(N_SEGMENTS):
        f, k = p.segment_grads(s)
        seen.extend(range(f, f + k))
    assert sorted(seen) == list(range(N_GRADS))


def test_module_state_dict_schema_matches_reference():
    import torch
    from unet_amd import UNet
    m = UNet(n_channels=1, n_classes=2)
    sd = m.state_dict()
    ref = O.param_shapes(1, 2)
    assert list(sd.keys()) == list(ref.keys())
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(ref[k]), k
    assert sum(p.numel() for p in m.parameters()) == 31_042_434
    names = [n for n, _ in m.named_parameters()]
    assert names == [k for k in ref if not O.is_buffer(k)]
    # scripts/train.py:54-61 init_weights works on the drop-in
    def init_weights(mod):
        if isinstance(mod, torch.nn.Conv2d):
            torch.nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
            if mod.bias is not None:
                torch.nn.init.constant_(mod.bias, 0)
        elif isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.constant_(mod.weight, 1)
            torch.nn.init.constant_(mod.bias, 0)
    m.apply(init_weights)
    assert float(m.inc.double_conv[0].bias.abs().sum()) == 0.0
    # the reference module path works too
    from models.unet_model import UNet as U2
    from utils.losses import WeightedCrossEntropyLoss  # noqa: F401
    assert U2 is UNet


def test_module_has_no_cpu_fallback():
    import torch
    from unet_amd import UNet, WeightedCrossEntropyLoss
    m = UNet(1, 2)
    with pytest.raises(RuntimeError, match="HIP device"):
        m(torch.zeros(1, 1, 188, 188))
    # the submodules' own forwards run on the per-op HIP blocks: no CPU path either
    with pytest.raises(RuntimeError, match="no CPU path"):
        m.inc(torch.zeros(1, 1, 188, 188))
    with pytest.raises(RuntimeError, match="no CPU path"):
        m.up1(torch.zeros(1, 1024, 4, 4), torch.zeros(1, 512, 8, 8))
    with pytest.raises(RuntimeError, match="no CPU path"):
        m.outc(torch.zeros(1, 64, 4, 4))
    with pytest.raises(RuntimeError):
        WeightedCrossEntropyLoss()(torch.zeros(1, 2, 4, 4), torch.zeros(1, 4, 4, dtype=torch.long),
                                   torch.ones(1, 4, 4))
    with pytest.raises(NotImplementedError):
        UNet(1, 2, bilinear=True)


def test_state_dict_roundtrip_with_reference_layout():
    import torch
    from unet_amd import UNet
    params = O.hash_init(1, 2, seed=5, bn_random=True)
    m = UNet(1, 2)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in params.items()})
    sd = m.state_dict()
    for k, v in params.items():
        np.testing.assert_array_equal(sd[k].numpy(), np.asarray(v))


def test_host_sanitizer_selftest():
    """The library's host logic under AddressSanitizer + UBSan
    (csrc/Makefile `sanitize`, built by __graft_entry__.build())."""
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "build", "asan", "host_selftest")
    if not os.path.exists(exe):
        pytest.skip("host_selftest not built (make -C unet-segmentation_amd/csrc sanitize)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_plan_takes_reference_channel_and_class_counts():
    """UNet(n_channels, n_classes) takes any counts in the reference
    (models/unet_model.py:66-85); the plan bounds both at 4096 only to keep
    its per-plan buffers in reason."""
    from unet_amd import UNet
    from unet_amd.plan import Plan
    _lib()
    for c, k in ((5, 5), (16, 32), (3, 9), (17, 2), (1, 33), (64, 150)):
        p = Plan(1, c, 188, 188, k)
        assert (p.out_h, p.out_w) == (4, 4)
        m = UNet(c, k)
        assert m.outc.conv.weight.shape == (k, 64, 1, 1) and m.inc.double_conv[0].weight.shape[1] == c
    for c, k in ((0, 2), (1, 0), (4097, 2), (1, 4097)):
        with pytest.raises(ValueError):
            Plan(1, c, 188, 188, k)
        with pytest.raises(ValueError):
            UNet(c, k)


def test_library_built_from_this_tree():
    """unet_version() carries the hash of the sources the .so was built from
    (csrc/Makefile SRC_HASH); it must equal the hash of the tree's sources."""
    L = _lib()
    ident = L.build_identity()
    assert ident["src_match"], ident



def test_pipeline_crop_views_and_cpu_rejection():
    """unet_amd.pipeline: train.py:39-51's center crop as a strided view (offset
    (H - oh) // 2, squeeze(1), no copy), and no CPU path for the frames."""
    import torch
    from unet_amd.pipeline import HeLaBatches, center_crop_views
    t = torch.arange(2 * 1 * 9 * 8).reshape(2, 1, 9, 8)
    v = center_crop_views(t, (4, 3))
    assert v.shape == (2, 4, 3) and v.data_ptr() == t[:, :, 2:6, 2:5].data_ptr()
    assert torch.equal(v, t[:, 0, 2:6, 2:5])
    with pytest.raises(ValueError):
        center_crop_views(t, (10, 3))
    with pytest.raises(ValueError):
        HeLaBatches(torch.zeros((2, 8, 8), dtype=torch.uint8), torch.zeros((2, 8, 8), dtype=torch.int32), 2, (4, 4))
