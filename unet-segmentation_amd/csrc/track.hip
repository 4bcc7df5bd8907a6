// Cell tracking (SURVEY.md §8f rank 4 remainder): scripts/track.py:103-275.
//
// Per frame the reference builds, for every (previous object, current object)
// pair, two full-frame boolean masks and counts their intersection and union
// (calculate_mask_iou, :73-100) -- O(objects^2 * pixels) host work.  Here one
// pass over the frame pair on the GPU gives the whole overlap table:
//   * label presence flags of both frames -> exclusive scans -> compact indices
//     (background forced to index 0, so objects are 1..n in ascending label
//     order = np.unique's order, get_mask_properties :52-54);
//   * a dense (n_prev + 1) x (n_curr + 1) histogram of (prev, curr) index
//     pairs: cell (i, j) = |prev object i AND curr object j|, row / column sums
//     = the object areas, so IoU = inter / (area_p + area_c - inter) exactly as
//     np.sum(and) / np.sum(or).
// The table (a few 10 KB) goes back to the host, where the tracker -- plain
// C++ below, a statement of track_sequence's control flow including its
// dictionary semantics -- runs the linear sum assignment and the division /
// new-object rules.  The assignment is a restatement of scipy's
// linear_sum_assignment (scipy 1.15.3, scipy/optimize/_lsap: Crouse's
// shortest augmenting path, "Implementing the 2-D rectangular assignment
// problem", IEEE TAES 2016) with the same tie-breaking, because the reference
// calls it on matrices full of equal 1000 entries.
//
// The augmenting_path / lsap functions below transcribe scipy's
// scipy/optimize/rectangular_lsap/rectangular_lsap.cpp, distributed under
// scipy's BSD 3-clause licence:
//
//   Copyright (c) 2001-2002 Enthought, Inc. 2003-2024, SciPy Developers.
//   All rights reserved.
//
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are
//   met:
//   1. Redistributions of source code must retain the above copyright notice,
//      this list of conditions and the following disclaimer.
//   2. Redistributions in binary form must reproduce the above copyright
//      notice, this list of conditions and the following disclaimer in the
//      documentation and/or other materials provided with the distribution.
//   3. Neither the name of the copyright holder nor the names of its
//      contributors may be used to endorse or promote products derived from
//      this software without specific prior written permission.
//
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS
//   IS" AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO,
//   THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR
//   PURPOSE ARE DISCLAIMED. IN NO EVENT SHALL THE COPYRIGHT HOLDER OR
//   CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL,
//   EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO,
//   PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS OF USE, DATA, OR
//   PROFITS; OR BUSINESS INTERRUPTION) HOWEVER CAUSED AND ON ANY THEORY OF
//   LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING
//   NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS
//   SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/unet_hip.h"
#include "unet_internal.h"

namespace {

constexpr int kLabels = 65536;
constexpr long long kMaxCells = 1ll << 24;

thread_local std::string g_track_err;

char* carve(char*& p, size_t bytes) {
  char* r = p;
  p += (bytes + 255) / 256 * 256;
  return r;
}

// ------------------------------- GPU part ------------------------------------
__global__ void k_tr_mark(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b, size_t n,
                          int* __restrict__ fa, int* __restrict__ fb) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i == 0) {  // background keeps compact index 0 whether or not it occurs
    fa[0] = 1;
    fb[0] = 1;
  }
  if (i >= n) return;
  if (a) fa[a[i]] = 1;
  fb[b[i]] = 1;
}

// compact index -> label value
__global__ void k_tr_list(const int* __restrict__ flag, const int* __restrict__ idx, int* __restrict__ list) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < kLabels && flag[l]) list[idx[l]] = l;
}

// table[(ia * nb) + ib] += 1 per pixel; a == nullptr: every pixel in row 0
__global__ void k_tr_hist(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b, size_t n,
                          const int* __restrict__ ia, const int* __restrict__ ib, int nb, unsigned* __restrict__ table) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = a ? ia[a[i]] : 0;
  atomicAdd(table + (size_t)r * nb + ib[b[i]], 1u);
}

size_t overlap_ws_bytes(int h, int w) {
  size_t scan = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const int*)nullptr, (int*)nullptr, kLabels + 1) != hipSuccess)
    return 0;
  return 4 * ((size_t)(kLabels + 1) * 4 + 256) + 2 * ((size_t)kLabels * 4 + 256) + (size_t)kMaxCells * 4 + 256 +
         scan + 256 + (size_t)h * w * 2 + 256;
}

// Overlap table of frames (a, b) (a may be null = no previous frame).  Host
// outputs: label lists (without background) and the (na+1) x (nb+1) table.
hipError_t overlap(const uint16_t* a, const uint16_t* b, int h, int w, void* ws, hipStream_t s,
                   std::vector<int>& la, std::vector<int>& lb, std::vector<unsigned>& table) {
  const size_t n = (size_t)h * w;
  char* c = reinterpret_cast<char*>(ws);
  int* fa = reinterpret_cast<int*>(carve(c, (kLabels + 1) * 4));
  int* fb = reinterpret_cast<int*>(carve(c, (kLabels + 1) * 4));
  int* ia = reinterpret_cast<int*>(carve(c, (kLabels + 1) * 4));
  int* ib = reinterpret_cast<int*>(carve(c, (kLabels + 1) * 4));
  int* lista = reinterpret_cast<int*>(carve(c, kLabels * 4));
  int* listb = reinterpret_cast<int*>(carve(c, kLabels * 4));
  unsigned* tab = reinterpret_cast<unsigned*>(carve(c, (size_t)kMaxCells * 4));
  size_t scan = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan, fa, ia, kLabels + 1, s);
  if (e != hipSuccess) return e;
  void* tmp = carve(c, scan);
  if ((e = hipMemsetAsync(fa, 0, (kLabels + 1) * 4, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(fb, 0, (kLabels + 1) * 4, s)) != hipSuccess) return e;
  const unsigned g = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_tr_mark, dim3(g), dim3(256), 0, s, a, b, n, fa, fb);
  if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, scan, fa, ia, kLabels + 1, s)) != hipSuccess) return e;
  if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, scan, fb, ib, kLabels + 1, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_tr_list, dim3(kLabels / 256), dim3(256), 0, s, fa, ia, lista);
  hipLaunchKernelGGL(k_tr_list, dim3(kLabels / 256), dim3(256), 0, s, fb, ib, listb);
  int cnt[2];
  if ((e = hipMemcpyAsync(&cnt[0], ia + kLabels, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(&cnt[1], ib + kLabels, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  const long long cells = (long long)cnt[0] * cnt[1];
  if (cells > kMaxCells) return hipErrorInvalidValue;
  if ((e = hipMemsetAsync(tab, 0, (size_t)cells * 4, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_tr_hist, dim3(g), dim3(256), 0, s, a, b, n, ia, ib, cnt[1], tab);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  table.resize((size_t)cells);
  std::vector<int> l0(cnt[0]), l1(cnt[1]);
  if ((e = hipMemcpyAsync(table.data(), tab, (size_t)cells * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(l0.data(), lista, (size_t)cnt[0] * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipMemcpyAsync(l1.data(), listb, (size_t)cnt[1] * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
  la.assign(l0.begin() + 1, l0.end());
  lb.assign(l1.begin() + 1, l1.end());
  return hipSuccess;
}

// --------------------------- linear sum assignment ---------------------------
// Shortest augmenting path (Crouse 2016) as scipy implements it: columns are
// scanned from a "remaining" list filled in reverse order, ties go to a column
// that ends the path; a tall matrix is solved transposed and the result sorted
// by row.  Returns 0, or -1 for an infeasible / invalid matrix.
long long augmenting_path(long long nc, const double* cost, std::vector<double>& u, std::vector<double>& v,
                          std::vector<long long>& path, std::vector<long long>& row4col,
                          std::vector<double>& spc, long long i, std::vector<char>& SR, std::vector<char>& SC,
                          std::vector<long long>& remaining, double* p_min) {
  double minVal = 0;
  long long num_remaining = nc;
  for (long long it = 0; it < nc; ++it) remaining[it] = nc - it - 1;
  std::fill(SR.begin(), SR.end(), 0);
  std::fill(SC.begin(), SC.end(), 0);
  std::fill(spc.begin(), spc.end(), INFINITY);
  long long sink = -1;
  while (sink == -1) {
    long long index = -1;
    double lowest = INFINITY;
    SR[i] = 1;
    for (long long it = 0; it < num_remaining; ++it) {
      const long long j = remaining[it];
      const double r = minVal + cost[i * nc + j] - u[i] - v[j];
      if (r < spc[j]) {
        path[j] = i;
        spc[j] = r;
      }
      if (spc[j] < lowest || (spc[j] == lowest && row4col[j] == -1)) {
        lowest = spc[j];
        index = it;
      }
    }
    minVal = lowest;
    if (minVal == INFINITY) return -1;
    const long long j = remaining[index];
    if (row4col[j] == -1)
      sink = j;
    else
      i = row4col[j];
    SC[j] = 1;
    remaining[index] = remaining[--num_remaining];
  }
  *p_min = minVal;
  return sink;
}

int lsap(long long nr, long long nc, const double* cost_in, int64_t* a, int64_t* b) {
  if (nr == 0 || nc == 0) return 0;
  const bool transpose = nc < nr;
  std::vector<double> temp;
  const double* cost = cost_in;
  if (transpose) {
    temp.resize((size_t)(nr * nc));
    for (long long i = 0; i < nr; ++i)
      for (long long j = 0; j < nc; ++j) temp[j * nr + i] = cost_in[i * nc + j];
    std::swap(nr, nc);
    cost = temp.data();
  }
  for (long long i = 0; i < nr * nc; ++i)
    if (cost[i] != cost[i] || cost[i] == -INFINITY) return -1;
  std::vector<double> u(nr, 0), v(nc, 0), spc(nc);
  std::vector<long long> path(nc, -1), col4row(nr, -1), row4col(nc, -1), remaining(nc);
  std::vector<char> SR(nr), SC(nc);
  for (long long cur = 0; cur < nr; ++cur) {
    double minVal;
    const long long sink = augmenting_path(nc, cost, u, v, path, row4col, spc, cur, SR, SC, remaining, &minVal);
    if (sink < 0) return -1;
    u[cur] += minVal;
    for (long long i = 0; i < nr; ++i)
      if (SR[i] && i != cur) u[i] += minVal - spc[col4row[i]];
    for (long long j = 0; j < nc; ++j)
      if (SC[j]) v[j] -= minVal - spc[j];
    long long j = sink;
    while (true) {
      const long long i = path[j];
      row4col[j] = i;
      std::swap(col4row[i], j);
      if (i == cur) break;
    }
  }
  if (transpose) {
    std::vector<long long> order(nr);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](long long x, long long y) { return col4row[x] < col4row[y]; });
    for (long long k = 0; k < nr; ++k) {
      a[k] = col4row[order[k]];
      b[k] = order[k];
    }
  } else {
    for (long long i = 0; i < nr; ++i) {
      a[i] = i;
      b[i] = col4row[i];
    }
  }
  return 0;
}

}  // namespace

// ------------------------------- host tracker --------------------------------
struct unet_tracker {
  int h = 0, w = 0;
  double iou_track = 0.3, iou_div = 0.1;
  int max_children = 2;
  struct Track {
    int label, start, end, parent;
  };
  std::vector<Track> tracks;        // track id = index + 1 (next_track_id, :126)
  std::vector<int> active;          // active_tracks_by_obj_label: label -> track id, -1 = absent (:131)
  std::vector<int> prev_labels;     // prev_frame_properties keys (ascending)
  std::vector<long long> prev_area;
  bool first = true;
  bool has_prev_dev = false;        // the device copy of the previous frame is valid
  unet_tracker() : active(kLabels, -1) {}

  int new_track(int frame, int parent) {
    tracks.push_back({(int)tracks.size() + 1, frame, frame, parent});
    return (int)tracks.size();
  }

  // one iteration of track_sequence's frame loop (:133-258) from the overlap
  // table inter[i * nc + j] of previous object i and current object j
  int step(int frame, const std::vector<int>& cur, const std::vector<long long>& area,
           const std::vector<long long>& inter) {
    const long long np = (long long)prev_labels.size(), nc = (long long)cur.size();
    if (first) {
      for (int lab : cur) active[lab] = new_track(frame, -1);
      first = false;
    } else {
      auto iou_of = [&](long long i, long long j) -> double {
        const long long it = inter[i * nc + j];
        const long long un = prev_area[i] + area[j] - it;
        return un == 0 ? 0.0 : (double)it / (double)un;
      };
      std::vector<char> mp(np, 0), mc(nc, 0);
      if (np > 0 && nc > 0) {
        std::vector<double> cost((size_t)(np * nc), 1000.0);
        for (long long i = 0; i < np; ++i)
          for (long long j = 0; j < nc; ++j) {
            const double iou = iou_of(i, j);
            if (iou > 0) cost[i * nc + j] = 1 - iou;
          }
        const long long k = std::min(np, nc);
        std::vector<int64_t> ri(k), ci(k);
        if (lsap(np, nc, cost.data(), ri.data(), ci.data()) != 0) return -EINVAL;
        for (long long q = 0; q < k; ++q) {
          const long long i = ri[q], j = ci[q];
          const int pl = prev_labels[i], cl = cur[j];
          const double iou = 1 - cost[i * nc + j];
          if (iou >= iou_track && active[pl] >= 0) {
            const int tid = active[pl];
            tracks[tid - 1].end = frame;
            active[pl] = -1;
            active[cl] = tid;
            mp[i] = 1;
            mc[j] = 1;
          }
        }
      }
      // division (:204-243): the unmatched lists are taken once, before any
      // division is recorded
      std::vector<long long> up, uc;
      for (long long i = 0; i < np; ++i)
        if (!mp[i]) up.push_back(i);
      for (long long j = 0; j < nc; ++j)
        if (!mc[j]) uc.push_back(j);
      for (long long i : up) {
        const int pl = prev_labels[i];
        if (active[pl] < 0) continue;
        std::vector<long long> kids;
        for (long long j : uc)
          if (iou_of(i, j) >= iou_div) kids.push_back(j);
        if ((int)kids.size() >= 2 && (int)kids.size() <= max_children) {
          const int parent = active[pl];
          tracks[parent - 1].end = frame - 1;
          active[pl] = -1;
          for (long long j : kids) {
            active[cur[j]] = new_track(frame, parent);
            mc[j] = 1;
          }
        }
      }
      for (long long j = 0; j < nc; ++j)  // new objects (:248-254)
        if (!mc[j]) active[cur[j]] = new_track(frame, -1);
    }
    prev_labels = cur;
    prev_area = area;
    return 0;
  }
};

extern "C" {

int unet_linear_sum_assignment(long long nr, long long nc, const double* cost, int64_t* row_ind, int64_t* col_ind) {
  if (nr < 0 || nc < 0 || ((nr > 0 && nc > 0) && (!cost || !row_ind || !col_ind))) return -EINVAL;
  return lsap(nr, nc, cost, row_ind, col_ind) == 0 ? 0 : -EINVAL;
}

unet_tracker* unet_tracker_create(int h, int w, double iou_track, double iou_division, int max_children) {
  if (h < 1 || w < 1 || max_children < 1) return nullptr;
  auto* t = new unet_tracker();
  t->h = h;
  t->w = w;
  t->iou_track = iou_track;
  t->iou_div = iou_division;
  t->max_children = max_children;
  return t;
}

void unet_tracker_destroy(unet_tracker* t) { delete t; }

size_t unet_tracker_ws_bytes(int h, int w) { return h > 0 && w > 0 ? overlap_ws_bytes(h, w) : 0; }

int unet_tracker_step_host(unet_tracker* t, int frame, int n_curr, const int32_t* labels, const int64_t* areas,
                           const int64_t* inter) {
  if (!t || n_curr < 0 || (n_curr > 0 && (!labels || !areas))) return -EINVAL;
  const long long np = (long long)t->prev_labels.size();
  if (np > 0 && n_curr > 0 && !inter && !t->first) return -EINVAL;
  std::vector<int> cur(labels, labels + n_curr);
  for (int k = 0; k < n_curr; ++k)
    if (cur[k] <= 0 || cur[k] >= kLabels || (k > 0 && cur[k] <= cur[k - 1])) return -EINVAL;
  std::vector<long long> area(areas, areas + n_curr);
  std::vector<long long> it;
  if (!t->first && np > 0 && n_curr > 0) it.assign(inter, inter + np * n_curr);
  return t->step(frame, cur, area, it);
}

int unet_tracker_add_frame(unet_tracker* t, const uint16_t* labels, int frame, void* ws, unet_stream_t stream) {
  if (!t || !labels || !ws) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t n = (size_t)t->h * t->w;
  // the previous frame's copy sits at the end of the workspace
  char* base = reinterpret_cast<char*>(ws);
  uint16_t* prev = reinterpret_cast<uint16_t*>(base + overlap_ws_bytes(t->h, t->w) - ((n * 2 + 255) / 256 * 256));
  std::vector<int> la, lb;
  std::vector<unsigned> tab;
  hipError_t e = overlap(t->has_prev_dev ? prev : nullptr, labels, t->h, t->w, ws, s, la, lb, tab);
  if (e != hipSuccess) {
    g_track_err = std::string("unet_tracker_add_frame: ") + hipGetErrorString(e);
    return e == hipErrorInvalidValue ? -EINVAL : -EIO;
  }
  const long long nb = (long long)lb.size() + 1, na = (long long)la.size() + 1;
  std::vector<long long> area(nb - 1, 0), inter;
  for (long long r = 0; r < na; ++r)
    for (long long j = 1; j < nb; ++j) area[j - 1] += tab[r * nb + j];
  if (t->has_prev_dev) {
    // the previous objects must be the ones the tracker holds (same frame)
    if (la != t->prev_labels) return -EINVAL;
    inter.resize((size_t)((na - 1) * (nb - 1)));
    for (long long i = 1; i < na; ++i)
      for (long long j = 1; j < nb; ++j) inter[(i - 1) * (nb - 1) + (j - 1)] = tab[i * nb + j];
  }
  const int rc = t->step(frame, lb, area, inter);
  if (rc) return rc;
  if ((e = hipMemcpyAsync(prev, labels, n * 2, hipMemcpyDeviceToDevice, s)) != hipSuccess) return -EIO;
  t->has_prev_dev = true;
  return 0;
}

int unet_tracker_num_tracks(const unet_tracker* t) { return t ? (int)t->tracks.size() : -EINVAL; }

int unet_tracker_tracks(const unet_tracker* t, int32_t* out, int cap) {
  if (!t || (cap > 0 && !out)) return -EINVAL;
  // output order and clamping of the res_track.txt writer (:265-272)
  std::vector<int> order(t->tracks.size());
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int x, int y) {
    const auto &a = t->tracks[x], &b = t->tracks[y];
    return a.start != b.start ? a.start < b.start : a.label < b.label;
  });
  const int k = std::min(cap, (int)order.size());
  for (int q = 0; q < k; ++q) {
    const auto& tr = t->tracks[order[q]];
    out[4 * q + 0] = tr.label;
    out[4 * q + 1] = tr.start;
    out[4 * q + 2] = std::max(tr.start, tr.end);
    out[4 * q + 3] = tr.parent;
  }
  return (int)order.size();
}

}  // extern "C"
