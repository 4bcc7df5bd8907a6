import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "unet-segmentation_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_runtest_makereport(item, call):
    """On a failing GPU test, keep the process's GEMM tuning state (the
    autotuner's per-shape choices are shared by every plan of the process) in
    $UNET_FAIL_TUNE_DIR, so the failing kernel mix can be replayed through
    UNET_TUNE_DB."""
    d = os.environ.get("UNET_FAIL_TUNE_DIR")
    if not d or call.when != "call" or call.excinfo is None or item.get_closest_marker("gpu") is None:
        return
    import pytest
    if call.excinfo.errisinstance(pytest.skip.Exception):
        return
    try:
        from unet_amd import _lib
        os.makedirs(d, exist_ok=True)
        name = "".join(ch if ch.isalnum() or ch in "-_" else "_" for ch in item.name)
        _lib.load().unet_tuning_save(os.path.join(d, f"{name}.db").encode())
    except Exception as e:  # debugging aid only
        print(f"tuning dump failed: {e}")
