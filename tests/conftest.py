import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(ROOT, "unet-segmentation_amd")
HERE = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, PKG, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)
# the GEMM choices bench.py timed (bench.py --tune-db-out); full-size tests load
# them so that they check the benchmarked kernel mix
TUNE_DB = os.path.join(ROOT, "profiles", "tune_db.txt")
# per test module that loaded the database: (module, entries, misses, missed keys),
# written to the terminal summary (fixture output is captured by pytest)
_TUNE_REPORT = []


@pytest.fixture(scope="module")
def bench_tuning(request):
    """Load profiles/tune_db.txt into the library's tuning cache (shapes it does
    not hold are tuned live); reset the cache afterwards."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd import _lib
    lib = _lib.load()
    lib.unet_tuning_reset()
    # UNET_TEST_TUNE_DB=<path> replays another database ('' = none: tune live)
    db = os.environ.get("UNET_TEST_TUNE_DB", TUNE_DB)
    n = lib.unet_tuning_load(db.encode()) if db and os.path.exists(db) else 0
    print(f"tuning database: {n} entries ({_lib.build_identity()})")
    yield n
    # GEMM shapes these tests met that the database did not hold (tuned live)
    live = [ln.split(" | ")[0] for ln in _lib.tuning_report().splitlines() if ln and "tuning db" not in ln]
    print(f"\ntuning database misses (shapes tuned live): {len(live)}" + "".join(f"\n  {k}" for k in live))
    print(f"slab-mode weight gradients that fell back to atomics: {_lib.slab_fallbacks(reset=True)}")
    _TUNE_REPORT.append((request.module.__name__, n, live))
    lib.unet_tuning_reset()


def pytest_terminal_summary(terminalreporter):
    for mod, n, live in _TUNE_REPORT:
        terminalreporter.write_line(f"{mod}: tuning database {n} entries, misses (shapes tuned live): {len(live)}")
        for k in live:
            terminalreporter.write_line(f"    {k}")


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
