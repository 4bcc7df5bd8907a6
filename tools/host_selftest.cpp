// Host-side self test of libunet_hip's pure-host logic, built with
// AddressSanitizer + UndefinedBehaviorSanitizer (csrc/Makefile target
// `sanitize`, host-only objects: no device code, no HIP call is made).
// Covers: plan shape / workspace layout arithmetic over many input sizes, the
// segment table, argument validation of the C ABI, the linear sum assignment
// (random, tied, rectangular, degenerate matrices; checked for a valid
// assignment and against brute force on small ones), the tracker's host step
// on a synthetic sequence, the tuning report.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <algorithm>
#include <vector>

#include "../include/unet_hip.h"

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

static unsigned long long rng_state = 0x9E3779B97F4A7C15ull;
static double urand() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (double)(rng_state >> 11) * (1.0 / 9007199254740992.0);
}

static void test_plans() {
  const int sizes[] = {188, 195, 198, 204, 220, 252, 300, 508, 512, 572, 700};
  for (int prec = 0; prec < 3; ++prec)
    for (int h : sizes)
      for (int n : {1, 2, 8})
        for (int c : {1, 3}) {
          unet_plan* p = unet_plan_create_ex(n, c, h, h + 4 * (n == 2), 2, prec);
          if (!p) continue;  // sizes the valid U-Net cannot take
          int oh = 0, ow = 0;
          CHECK(unet_plan_out_hw(p, &oh, &ow) == 0 && oh > 0 && ow > 0);
          const size_t full = unet_plan_workspace_bytes(p), fwd = unet_plan_forward_workspace_bytes(p);
          CHECK(fwd > 0 && fwd < full && full % 256 == 0);
          CHECK(unet_plan_precision(p) == prec);
          int total = 0;
          for (int s = 0; s < unet_plan_num_segments(p); ++s) {
            int f = -1, k = -1;
            CHECK(unet_plan_segment_grads(p, s, &f, &k) == 0 && f >= 0 && k > 0 && f + k <= 82);
            total += k;
          }
          CHECK(total == 82);
          CHECK(unet_plan_segment_grads(p, 9, nullptr, nullptr) != 0);
          unet_plan_destroy(p);
        }
  CHECK(unet_plan_create(1, 1, 100, 100, 2) == nullptr);  // too small
  CHECK(unet_plan_create(1, 4097, 512, 512, 2) == nullptr);  // c_in > 4096 (kMaxInChannels)
  CHECK(unet_plan_create(1, 1, 512, 512, 4097) == nullptr);  // n_classes > 4096 (kMaxClassCount)
  CHECK(unet_plan_create(1, 0, 512, 512, 2) == nullptr);
  CHECK(unet_plan_create(1, 1, 512, 512, 0) == nullptr);
  if (unet_plan* q = unet_plan_create(1, 5, 188, 188, 5)) {  // 5 channels / 5 classes take a plan
    CHECK(unet_plan_num_params(q) == 136);
    unet_plan_destroy(q);
  } else {
    CHECK(false);
  }
  CHECK(unet_plan_create_ex(1, 1, 512, 512, 2, 7) == nullptr);
  CHECK(unet_plan_forward(nullptr, nullptr, nullptr, nullptr, nullptr, 1, nullptr) != 0);
  CHECK(unet_plan_backward(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 9, nullptr) != 0);
  unet_plan_destroy(nullptr);
}

static double assignment_cost(const std::vector<double>& c, int nc, const std::vector<int64_t>& r,
                              const std::vector<int64_t>& q) {
  double s = 0;
  for (size_t i = 0; i < r.size(); ++i) s += c[r[i] * nc + q[i]];
  return s;
}

static void test_lsap() {
  for (int trial = 0; trial < 300; ++trial) {
    const int nr = 1 + (int)(urand() * 9), nc = 1 + (int)(urand() * 9);
    const int kind = trial % 3;
    std::vector<double> c((size_t)nr * nc);
    for (auto& v : c) v = kind == 0 ? urand() : kind == 1 ? (double)(int)(urand() * 3) : (urand() < 0.1 ? urand() : 1000.0);
    const int k = std::min(nr, nc);
    std::vector<int64_t> r(k), q(k);
    CHECK(unet_linear_sum_assignment(nr, nc, c.data(), r.data(), q.data()) == 0);
    std::vector<char> ur(nr, 0), uc(nc, 0);
    for (int i = 0; i < k; ++i) {
      CHECK(r[i] >= 0 && r[i] < nr && q[i] >= 0 && q[i] < nc);
      CHECK(!ur[r[i]] && !uc[q[i]]);
      ur[r[i]] = uc[q[i]] = 1;
      if (i) CHECK(r[i] > r[i - 1]);
    }
    // brute force over injections of the smaller side (sizes <= 9)
    const bool rows_small = nr <= nc;
    const int a = rows_small ? nr : nc, b = rows_small ? nc : nr;
    std::vector<int> perm(b);
    std::iota(perm.begin(), perm.end(), 0);
    double best = INFINITY;
    if (b <= 7) {
      do {
        double s = 0;
        for (int i = 0; i < a; ++i) s += rows_small ? c[(size_t)i * nc + perm[i]] : c[(size_t)perm[i] * nc + i];
        best = std::min(best, s);
      } while (std::next_permutation(perm.begin(), perm.end()));
      CHECK(std::fabs(assignment_cost(c, nc, r, q) - best) <= 1e-9 * std::max(1.0, std::fabs(best)));
    }
  }
  std::vector<double> bad = {0.0, NAN, 1.0, 2.0};
  std::vector<int64_t> r(2), q(2);
  CHECK(unet_linear_sum_assignment(2, 2, bad.data(), r.data(), q.data()) != 0);
  CHECK(unet_linear_sum_assignment(0, 3, nullptr, nullptr, nullptr) == 0);
  CHECK(unet_linear_sum_assignment(-1, 3, nullptr, nullptr, nullptr) != 0);
}

static void test_tracker() {
  unet_tracker* t = unet_tracker_create(8, 8, 0.3, 0.1, 2);
  CHECK(t != nullptr);
  // frame 0: objects 3, 9; frame 1: 3 continues, 9 splits into 4 and 5; frame 2: empty
  const int32_t l0[] = {3, 9};
  const int64_t a0[] = {10, 20};
  CHECK(unet_tracker_step_host(t, 0, 2, l0, a0, nullptr) == 0);
  const int32_t l1[] = {3, 4, 5};
  const int64_t a1[] = {10, 6, 6};
  const int64_t i1[] = {10, 0, 0, 0, 5, 5};  // 2 x 3
  CHECK(unet_tracker_step_host(t, 1, 3, l1, a1, i1) == 0);
  CHECK(unet_tracker_step_host(t, 2, 0, nullptr, nullptr, nullptr) == 0);
  const int n = unet_tracker_num_tracks(t);
  CHECK(n == 4);
  std::vector<int32_t> rows(4 * (size_t)n);
  CHECK(unet_tracker_tracks(t, rows.data(), n) == n);
  // track 1 (label 3) 0..1, track 2 (label 9) ends at 0, children 3 and 4 at 1 with parent 2
  CHECK(rows[0] == 1 && rows[1] == 0 && rows[2] == 1 && rows[3] == -1);
  CHECK(rows[4] == 2 && rows[5] == 0 && rows[6] == 0 && rows[7] == -1);
  CHECK(rows[8] == 3 && rows[11] == 2 && rows[12] == 4 && rows[15] == 2);
  const int32_t unsorted[] = {5, 2};
  CHECK(unet_tracker_step_host(t, 3, 2, unsorted, a0, nullptr) != 0);
  CHECK(unet_tracker_tracks(t, nullptr, 0) == n);
  unet_tracker_destroy(t);
  CHECK(unet_tracker_create(0, 8, 0.3, 0.1, 2) == nullptr);
  unet_tracker_destroy(nullptr);
}

static void test_misc() {
  CHECK(std::strlen(unet_version()) > 0);
  const size_t need = unet_tuning_report(nullptr, 0);
  std::vector<char> buf(need + 1);
  CHECK(unet_tuning_report(buf.data(), buf.size()) == need);
  CHECK(unet_tuning_reset() == 0);
  CHECK(unet_set_tuning("no_such_key", 1) != 0);
}

int main() {
  test_plans();
  test_lsap();
  test_tracker();
  test_misc();
  if (fails) {
    std::fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  std::printf("host_selftest: all checks passed\n");
  return 0;
}
