"""Cell tracking (scripts/track.py:103-275) pinned to the reference's own
committed output: data/raw/processed/predictions/DIC-C2DH-HeLa/01/res_track.txt
(10,807 tracks) computed from 01_RES_INST/m000-m083.tif
(tests/golden/hela_postproc.npz; make_golden_postproc.py --verify-track re-ran
the reference's track_sequence on those masks and reproduced the file).

CPU: the oracle restatement and the library's native host tracker (fed the
oracle's overlap tables through unet_tracker_step_host) against the fixture,
and the library's linear sum assignment against scipy's on random, tied and
rectangular matrices.  GPU: the whole tracker (per-frame overlap tables on the
device) against the fixture, through the C ABI.
"""
import ctypes
import os
import zlib

import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment

from oracle import track_oracle as T

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def hela():
    return np.load(os.path.join(G, "hela_postproc.npz"), allow_pickle=False)


def test_oracle_reproduces_reference_res_track(hela):
    rows = T.track_masks(hela["labels"], hela["frames"])
    np.testing.assert_array_equal(rows, hela["res_track"])


def _lib():
    from unet_amd import _lib as L
    return L.load()


def _lsap(lib, cost):
    cost = np.ascontiguousarray(cost, np.float64)
    nr, nc = cost.shape
    k = min(nr, nc)
    r = np.zeros(k, np.int64)
    c = np.zeros(k, np.int64)
    rc = lib.unet_linear_sum_assignment(nr, nc, cost.ctypes.data_as(ctypes.c_void_p), r.ctypes.data_as(ctypes.c_void_p),
                                        c.ctypes.data_as(ctypes.c_void_p))
    return rc, r, c


@pytest.mark.parametrize("shape", [(1, 1), (3, 3), (5, 9), (9, 5), (40, 40), (37, 52), (60, 23), (0, 4)])
@pytest.mark.parametrize("kind", ["uniform", "ties", "track"])
def test_lsap_matches_scipy(shape, kind):
    """Same assignment as scipy (not just the same optimum): the reference's
    cost matrices are mostly the constant 1000, so tie-breaking matters."""
    lib = _lib()
    rng = np.random.default_rng(zlib.crc32(repr((shape, kind)).encode()))
    if kind == "uniform":
        cost = rng.uniform(size=shape)
    elif kind == "ties":
        cost = rng.integers(0, 4, size=shape).astype(np.float64)
    else:  # track.py:164-173 shape: 1000 except a sparse set of 1 - IoU
        cost = np.full(shape, 1000.0)
        m = rng.uniform(size=shape) < 0.08
        cost[m] = 1 - rng.uniform(0.01, 1.0, size=int(m.sum()))
    rc, r, c = _lsap(lib, cost)
    assert rc == 0
    sr, sc = linear_sum_assignment(cost)
    np.testing.assert_array_equal(r, sr)
    np.testing.assert_array_equal(c, sc)


def test_lsap_rejects_nan_and_infeasible():
    lib = _lib()
    assert _lsap(lib, np.array([[0.0, np.nan], [1.0, 2.0]]))[0] != 0
    assert _lsap(lib, np.array([[np.inf, np.inf], [1.0, 2.0]]))[0] != 0


def test_native_host_tracker_reproduces_reference(hela):
    """The library's tracker control flow (division rule, dict semantics of
    active_tracks_by_obj_label, output order) from host overlap tables."""
    lib = _lib()
    labels, frames = hela["labels"], hela["frames"]
    h, w = labels.shape[1:]
    tr = lib.unet_tracker_create(h, w, 0.3, 0.1, 2)
    assert tr
    try:
        prev = None
        for t in range(len(labels)):
            lab, area = T.frame_objects(labels[t])
            lab32 = np.ascontiguousarray(lab, np.int32)
            area64 = np.ascontiguousarray(area, np.int64)
            inter = None
            if prev is not None:
                inter = np.ascontiguousarray(T.overlap_table(labels[t - 1], prev, labels[t], lab), np.int64)
            rc = lib.unet_tracker_step_host(tr, int(frames[t]), len(lab32), lab32.ctypes.data_as(ctypes.c_void_p),
                                            area64.ctypes.data_as(ctypes.c_void_p),
                                            None if inter is None else inter.ctypes.data_as(ctypes.c_void_p))
            assert rc == 0
            prev = lab
        n = lib.unet_tracker_num_tracks(tr)
        out = np.zeros((n, 4), np.int32)
        assert lib.unet_tracker_tracks(tr, out.ctypes.data_as(ctypes.c_void_p), n) == n
    finally:
        lib.unet_tracker_destroy(tr)
    np.testing.assert_array_equal(out, hela["res_track"])


def test_host_tracker_rejects_unsorted_labels():
    lib = _lib()
    tr = lib.unet_tracker_create(4, 4, 0.3, 0.1, 2)
    try:
        lab = np.array([5, 3], np.int32)
        area = np.array([1, 1], np.int64)
        assert lib.unet_tracker_step_host(tr, 0, 2, lab.ctypes.data_as(ctypes.c_void_p),
                                          area.ctypes.data_as(ctypes.c_void_p), None) != 0
    finally:
        lib.unet_tracker_destroy(tr)
    assert not lib.unet_tracker_create(0, 4, 0.3, 0.1, 2)


@pytest.mark.gpu
def test_gpu_tracker_reproduces_reference(hela, tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd.track import Tracker, write_track_file
    labels, frames = hela["labels"], hela["frames"]
    dev = torch.from_numpy(labels.astype(np.int32)).cuda()
    tr = Tracker(labels.shape[1], labels.shape[2])
    for t in range(len(labels)):
        tr.add_frame(dev[t], int(frames[t]))
    rows = tr.tracks()
    np.testing.assert_array_equal(rows, hela["res_track"])
    # the writer's text equals the reference file's lines
    p = tmp_path / "res_track.txt"
    write_track_file(rows, str(p))
    lines = p.read_text().splitlines()
    assert len(lines) == 10807
    assert lines[:3] == ["1 0 0 -1", "2 0 0 -1", "3 0 0 -1"]


@pytest.mark.gpu
def test_gpu_tracker_edge_cases():
    """Empty frames, a frame with one object splitting into two (division),
    objects vanishing and reappearing (new tracks), labels up to 65535."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from unet_amd.track import Tracker
    h, w = 40, 50
    seq = np.zeros((6, h, w), np.int32)
    seq[0, 5:25, 5:25] = 7                  # one cell
    seq[1, 5:25, 5:25] = 9                  # moved label, same place -> linked
    seq[2, 5:25, 5:10] = 3                  # divides: two children, IoU 0.25 each
    seq[2, 5:25, 20:25] = 65535
    seq[3] = 0                              # empty frame
    seq[4, 30:35, 40:48] = 2                # new object
    seq[5, 30:35, 40:48] = 2
    seq[5, 0:3, 0:3] = 1
    ref = T.track_masks(seq, np.arange(6))
    tr = Tracker(h, w)
    d = torch.from_numpy(seq).cuda()
    for t in range(6):
        tr.add_frame(d[t], t)
    np.testing.assert_array_equal(tr.tracks(), ref)
    assert (ref[:, 3] > 0).sum() == 2       # the two children name their parent
