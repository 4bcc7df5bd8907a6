"""CPU restatement of the reference's cell tracker, scripts/track.py:103-275.

TEST INFRASTRUCTURE ONLY: the checker of the tracker in
unet-segmentation_amd/csrc/track.hip (unet_tracker_*); nothing in the product
path imports it.  Pinned by tests/test_track.py against the reference's own
committed output data/raw/processed/predictions/DIC-C2DH-HeLa/01/res_track.txt
computed from 01_RES_INST/m*.tif (tests/golden/hela_postproc.npz; the
generator re-ran the reference's track_sequence on those masks in the build
container and got the committed file back).

Differences from the reference are in representation only:
* object properties (get_mask_properties :39-70) are the sorted label list and
  per-label areas; calculate_mask_iou (:73-100) is intersection / union from a
  contingency table (np.bincount of (prev, curr) label pairs), the same integer
  counts, so the same fp64 quotient;
* the assignment is scipy.optimize.linear_sum_assignment, as in the reference
  (:6, :176), on the same cost matrix.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import linear_sum_assignment

IOU_THRESHOLD_TRACK = 0.3          # track.py:21
IOU_THRESHOLD_DIVISION = 0.1       # track.py:22
MAX_CHILD_CANDIDATES_FOR_DIVISION = 2  # track.py:24


def frame_objects(mask):
    """Ascending object labels (background 0 excluded) and their areas
    (get_mask_properties, track.py:52-69)."""
    labels, counts = np.unique(mask, return_counts=True)
    keep = labels != 0
    return labels[keep].astype(np.int64), counts[keep].astype(np.int64)


def overlap_table(prev_mask, prev_labels, curr_mask, curr_labels):
    """inter[i, j] = |prev object i AND curr object j| (pixel counts)."""
    ip = np.full(65536, -1, np.int64)
    ic = np.full(65536, -1, np.int64)
    ip[prev_labels] = np.arange(len(prev_labels))
    ic[curr_labels] = np.arange(len(curr_labels))
    a = ip[prev_mask.ravel().astype(np.int64)]
    b = ic[curr_mask.ravel().astype(np.int64)]
    both = (a >= 0) & (b >= 0)
    flat = a[both] * len(curr_labels) + b[both]
    return np.bincount(flat, minlength=len(prev_labels) * len(curr_labels)).reshape(len(prev_labels),
                                                                                   len(curr_labels))


class TrackOracle:
    """track_sequence's state (track.py:125-131) and frame step (:133-258)."""

    def __init__(self, iou_track=IOU_THRESHOLD_TRACK, iou_division=IOU_THRESHOLD_DIVISION,
                 max_children=MAX_CHILD_CANDIDATES_FOR_DIVISION):
        self.iou_track, self.iou_div, self.max_children = iou_track, iou_division, max_children
        self.tracks = {}   # id -> [label, start, end, parent]
        self.next_id = 1
        self.active = {}   # object label in the previous frame -> track id
        self.prev = None   # (labels, areas)
        self.first = True

    def _new(self, frame, parent=-1):
        tid = self.next_id
        self.tracks[tid] = [tid, frame, frame, parent]
        self.next_id += 1
        return tid

    def step(self, frame, labels, areas, inter):
        """labels/areas of the current frame; inter[i, j] against the previous."""
        labels = [int(v) for v in labels]
        if self.first:
            for lab in labels:
                self.active[lab] = self._new(frame)
            self.first = False
        else:
            plabels, pareas = self.prev
            plabels = [int(v) for v in plabels]
            npv, ncv = len(plabels), len(labels)

            def iou(i, j):
                it = int(inter[i, j])
                un = int(pareas[i]) + int(areas[j]) - it
                return 0.0 if un == 0 else it / un

            mp, mc = set(), set()
            if npv > 0 and ncv > 0:
                cost = np.ones((npv, ncv)) * 1000
                for i in range(npv):
                    for j in range(ncv):
                        v = iou(i, j)
                        if v > 0:
                            cost[i, j] = 1 - v
                rows, cols = linear_sum_assignment(cost)
                for i, j in zip(rows, cols):
                    pl, cl = plabels[i], labels[j]
                    v = 1 - cost[i, j]
                    if v >= self.iou_track and pl in self.active:
                        tid = self.active[pl]
                        self.tracks[tid][2] = frame
                        del self.active[pl]
                        self.active[cl] = tid
                        mp.add(i)
                        mc.add(j)
            up = [i for i in range(npv) if i not in mp]
            uc = [j for j in range(ncv) if j not in mc]
            for i in up:
                pl = plabels[i]
                if pl not in self.active:
                    continue
                kids = [j for j in uc if iou(i, j) >= self.iou_div]
                if 2 <= len(kids) <= self.max_children:
                    parent = self.active[pl]
                    self.tracks[parent][2] = frame - 1
                    del self.active[pl]
                    for j in kids:
                        self.active[labels[j]] = self._new(frame, parent)
                        mc.add(j)
            for j in range(ncv):
                if j not in mc:
                    self.active[labels[j]] = self._new(frame)
        self.prev = (np.asarray(labels, np.int64), np.asarray(areas, np.int64))

    def result(self):
        """(n, 4) int rows in the res_track.txt order (track.py:265-272)."""
        ids = sorted(self.tracks, key=lambda k: (self.tracks[k][1], self.tracks[k][0]))
        out = [[t[0], t[1], max(t[1], t[2]), t[3]] for t in (self.tracks[k] for k in ids)]
        return np.array(out, np.int64).reshape(-1, 4)


def track_masks(masks, frames=None):
    """Track a (T, H, W) stack of instance labelings; returns the res_track rows."""
    tr = TrackOracle()
    prev_mask = None
    for t, m in enumerate(masks):
        labels, areas = frame_objects(m)
        inter = None
        if prev_mask is not None:
            inter = overlap_table(prev_mask, tr.prev[0], m, labels)
        tr.step(int(frames[t]) if frames is not None else t, labels, areas, inter)
        prev_mask = m
    return tr.result()
