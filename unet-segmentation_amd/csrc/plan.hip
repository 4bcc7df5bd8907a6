// Network plan: the U-Net of models/unet_model.py:66-146 (bilinear=False) as a
// fixed schedule of HIP launches over one caller-provided workspace, plus the
// C-ABI declared in include/unet_hip.h.
//
// Forward (train):  conv outputs are stored RAW (pre-BN); each consumer applies
// the BatchNorm+ReLU of its producer while loading (scale/shift per channel),
// so no normalised activation is ever materialised except the 2x2-pooled
// tensors (pool needs relu(bn(.)) before the max: gamma may be negative).
// Backward: dz (grad after ReLU mask) -> BN-bwd stats -> dY into a zero-bordered
// padded buffer -> weight grad (pixel-reduction GEMM) and input grad (implicit
// GEMM with the flipped kernel) whose epilogue applies the next ReLU mask and
// collects the next BN-bwd statistics.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <array>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/unet_hip.h"
#include "unet_internal.h"

using namespace unet;

namespace unet {
extern int g_wino_max, g_wino_dgrad_max, g_wino_wgrad_max, g_wino4_fwd_min_cg, g_wino4_fwd_small_cg;  // igemm.hip (Winograd tile caps)
size_t conv3_flat_sk_slab_bytes(const IgemmArgs& a);  // conv3_flat.hip (tile 86: stream-K partial slots)
// unet_set_tuning("autotune", v) or UNET_AUTOTUNE (default on)
int g_autotune = getenv("UNET_AUTOTUNE") ? atoi(getenv("UNET_AUTOTUNE")) : 1;
// unet_set_tuning("concurrent", v) or UNET_CONCURRENT (default on): weight
// gradients on a side stream
int g_concurrent = getenv("UNET_CONCURRENT") ? atoi(getenv("UNET_CONCURRENT")) : 1;
// unet_set_tuning("bf16_norm", v) or UNET_BF16_NORM (default off): bf16 plans
// materialise relu(bn(y)) once per element (the normalised copy every GEMM
// consumer stages as a plain operand); 2: only the encoder outputs, whose copy
// the max-pool writes while it reads them anyway (no extra pass: the skip
// operand of the up blocks' first convs and their weight gradients becomes a
// plain LDS-DMA-able copy); off: consumers transform on load.
// Read at plan creation (workspace layout).
int g_bf16_norm = getenv("UNET_BF16_NORM") ? atoi(getenv("UNET_BF16_NORM")) : 0;
// unet_set_tuning("bn_fold", v) or UNET_BN_FOLD (default on): eval forwards
// fold each BatchNorm into its conv (scale into the packed weights, scale *
// bias + shift as the bias) and store relu(conv') in the epilogue, so every
// consumer reads a plain operand
int g_bn_fold = getenv("UNET_BN_FOLD") ? atoi(getenv("UNET_BN_FOLD")) : 1;
// unet_set_tuning("force_split", k) / ("force_tile", id): every igemm site
// runs split-K k and/or tile id where they apply (tests)
int g_force_split = 0;
int g_force_tile = 0;
// unet_set_tuning("deterministic", 1) or UNET_DETERMINISTIC=1 (default off):
// every weight gradient runs a variant without fp32 atomics (slab partials
// summed in a fixed order, or one split storing straight into the gradient),
// and inc.c0's slab reduction sums every slab in one pass, so two runs of a
// step give bit-identical results whatever the stream timing (the analogue of
// torch.use_deterministic_algorithms).  The autotuner then times only those
// variants (their own tuning keys); a site with none counts in
// unet_nondeterministic_sites().
int g_deterministic = getenv("UNET_DETERMINISTIC") ? atoi(getenv("UNET_DETERMINISTIC")) : 0;
std::atomic<long long> g_nondet_sites{0};
// unet_set_tuning("bnb_fuse", v) or UNET_BNB_FUSE (default on): fp32 plans form
// dY of a layer whose weight gradient runs Winograd F(6x6) in one pass with
// that weight gradient's dY transform (k_bnb_wino6_dy) instead of k_bnb_apply
// + k_wino6_dy (bit-identical results).  Measured with the early U transforms
// below (both on by default): 25.60 vs 25.74 ms per fp32 step (three A/B pairs,
// one box); alone it is 0.2 ms SLOWER, because the dY transform leaves the side
// stream for the main stream's critical path and the side stream idles while
// the main stream runs the fused pass.  Its per-layer Vd buffers
// are allocated by plans created while it is on.
int g_bnb_fuse = getenv("UNET_BNB_FUSE") ? atoi(getenv("UNET_BNB_FUSE")) : 1;
std::atomic<long long> g_fused_bnb_sites{0};
// unet_set_tuning("wgrad_early_u", v) or UNET_WGRAD_EARLY_U (default on): with
// the side stream, a Winograd weight gradient's input transform U (forward
// tensors only) is issued on the side stream before it waits for the layer's
// dY, so it runs beside the main stream's BN-backward finalize / apply (or
// fused pass) of that layer instead of after it
int g_wgrad_early_u = getenv("UNET_WGRAD_EARLY_U") ? atoi(getenv("UNET_WGRAD_EARLY_U")) : 1;
// unet_set_tuning("wgrad_fwd_u", v) or UNET_WGRAD_FWD_U (default off): fp32
// training plans issue each Winograd weight gradient's input transform U
// during the FORWARD, on the side stream (idle there), into a per-layer buffer
// the backward's point GEMMs read; read for the workspace layout at plan creation
int g_wgrad_fwd_u = getenv("UNET_WGRAD_FWD_U") ? atoi(getenv("UNET_WGRAD_FWD_U")) : 0;
}  // namespace unet

namespace {

thread_local std::string g_err;
void set_err(const std::string& s) { g_err = s; }

constexpr float kEps = 1e-5f, kMom = 0.1f;

struct Buf {
  size_t off = 0, bytes = 0;
};

struct Alloc {
  size_t top = 0;
  Buf take(size_t bytes) {
    Buf b;
    b.off = top;
    b.bytes = bytes;
    top += (bytes + 255) / 256 * 256;
    return b;
  }
};

struct Conv {
  int ci = 0, co = 0, hi = 0, wi = 0, ho = 0, wo = 0;
  int pw = 0, gw = 0;  // param / grad table base (conv w, b, bn w, bn b, rm, rv, nbt)
  Buf y, mean, invstd, scale, shift, wf, wd, dwp, dz, dyp, coef, stats, bstats;
  Buf vdw;  // fp32 plans: the F(6x6) weight gradient's dY transform (k_bnb_wino6_dy), one per layer
  Buf uws;  // fp32 plans with wgrad_fwd_u: this layer's Winograd weight-gradient scratch (U | Vd | Mw)
  bool u_fwd = false;  // U of this step already issued by the forward (side stream)
  Buf a;  // bf16 plans: relu(bn(y)) in bf16, the operand its GEMM consumers read
};
struct ConvT {
  int ci = 0, co = 0, h = 0, w = 0;  // input grid (h, w) -> output (2h, 2w)
  int pw = 0, gw = 0;
  Buf u, wf, wd, dwp, du, colsum;
};
struct Pool {
  int c = 0, h = 0, w = 0;  // input grid
  Buf p, arg, dp;
};
struct Skip {
  int c = 0, th = 0, tw = 0, oy = 0, ox = 0;  // crop of encoder output
  Buf d;                                      // compact gradient of the cropped region
};

double conv_flops(const Conv& c, int n) { return 2.0 * n * c.ho * c.wo * (double)c.co * c.ci * 9; }

}  // namespace

struct unet_plan {
  int n = 0, cin = 0, h = 0, w = 0, ncls = 0, ho = 0, wo = 0;
  int prec = UNET_PREC_FP32;  // GEMM operand precision (include/unet_hip.h)
  // every packed GEMM weight matrix (conv wf/wd, convT wf/wd) lies in one
  // contiguous fp32 region; with bf16 GEMMs its RNE copy is `pack16` (same
  // element offsets), refreshed by one conversion launch per forward
  Buf pack_region, pack16;
  Conv L[18];
  ConvT T[4];
  Pool P[4];
  Skip S[4];
  Buf stat_region, dwp_region, head_acc, wce_acc, first_slabs;
  Buf fold0w;         // inc.c0 weights with its BatchNorm folded in (eval)
  bool fold = false;  // this forward folds BatchNorm into the convs (eval + g_bn_fold)
  // weight-gradient GEMMs run on a side stream beside the dY -> dX chain of the
  // backward (joined at the end of every backward call)
  hipStream_t side = nullptr;
  hipEvent_t ev_dy[18] = {}, ev_du[4] = {}, ev_join = nullptr;
  hipEvent_t ev_bwd0 = nullptr;  // main stream at a backward call's start (early U transforms wait on it)
  hipEvent_t ev_fwdu = nullptr;  // main stream before a forward layer whose U the side stream computes
  // per backward segment: recorded on the side stream after the segment's
  // weight gradients (UNET_BWD_DEFER_JOIN calls), waited on by the caller's
  // collective stream (unet_plan_wait_segment)
  hipEvent_t ev_seg[9] = {};
  bool seg_on_side[9] = {};
  bool side_pending = false;  // side-stream work not yet joined into a caller stream
  int bwd_full = 0;  // completed whole backward passes (the first one tunes, serially)
  Buf slab;          // split-K partial tiles (igemm sites the tuner splits)
  Buf wino;          // Winograd F(2x2, 3x3) / F(4x4, 3x3) scratch (fp32 plans; U, M, V of one GEMM)
  Buf wino_w;        // the weight-gradient twin (U, Vd, Mw; backward part of the workspace)
  Buf wslab;         // split partials of the slab-mode weight gradients (side stream)
  Buf tune_scratch;  // atomic targets of the autotuner's trial launches
  size_t ws_bytes = 0;
  size_t fwd_ws_bytes = 0;  // prefix of the workspace a forward uses (no backward buffers)
  // timing
  bool timing = false;
  struct Ev {
    hipEvent_t a, b;
    int cls;
    double flops, bytes, xflops;
    int site;  // GEMM launch site (site_name), -1 = none
  };
  std::vector<Ev> evs;
  // per GEMM launch site of the last timed step: ms, direct flops, MFMA flops
  std::map<int, std::array<double, 3>> sites, sites_last;
  // MFMA flops the chosen GEMM variants execute (Winograd: its point GEMMs),
  // summed on the host as launches are enqueued; Timer intervals take deltas
  double xfl = 0;
  double t_ms[UNET_KC_COUNT] = {0}, t_fl[UNET_KC_COUNT] = {0}, t_by[UNET_KC_COUNT] = {0};
  double t_xf[UNET_KC_COUNT] = {0}, t_xf_last[UNET_KC_COUNT] = {0};
  int t_n[UNET_KC_COUNT] = {0};
};

namespace {

// ---------------- parameter table layout (reference state_dict order) -----
int block_pbase(int b) { return b <= 4 ? 14 * b : 70 + 16 * (b - 5) + 2; }
int block_gbase(int b) { return b <= 4 ? 8 * b : 40 + 10 * (b - 5) + 2; }

template <typename T>
T* P(void* const* tab, int i) { return reinterpret_cast<T*>(tab[i]); }

struct Ctx {
  unet_plan* p;
  char* ws;
  hipStream_t s;
  float* f(const Buf& b) const { return reinterpret_cast<float*>(ws + b.off); }
  double* d(const Buf& b) const { return reinterpret_cast<double*>(ws + b.off); }
  uint8_t* u8(const Buf& b) const { return reinterpret_cast<uint8_t*>(ws + b.off); }
};

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e_ = (x);                                        \
    if (e_ != hipSuccess) {                                     \
      set_err(std::string(#x) + ": " + hipGetErrorString(e_));  \
      return -EIO;                                              \
    }                                                           \
  } while (0)

// the 1024-channel bottleneck set of SURVEY.md §8d: down4.c0, down4.c1, up1.c0
// (and up1.convT, ConvT index 0)
inline bool bottleneck_conv(int l) { return l == 8 || l == 9 || l == 10; }

// GEMM launch-site ids of the per-site timing report (unet_plan_timing_sites):
// kind 0 = forward, 1 = input gradient, 2 = weight gradient
inline int site_conv(int l, int kind) { return l * 4 + kind; }
inline int site_convT(int k, int kind) { return 100 + k * 4 + kind; }
std::string site_name(int site) {
  static const char* kinds[3] = {"fwd", "dgrad", "wgrad"};
  if (site >= 100) return "up" + std::to_string((site - 100) / 4 + 1) + ".convT " + kinds[site % 4];
  const int l = site / 4;
  std::string layer = l < 2 ? "inc" : l < 10 ? "down" + std::to_string(l / 2) : "up" + std::to_string((l - 10) / 2 + 1);
  return layer + ".c" + std::to_string(l % 2) + " " + kinds[site % 4];
}

struct Timer {
  unet_plan* p;
  hipStream_t s;
  hipEvent_t a{}, b{};
  bool ok = false;
  int cls;
  double fl, by, x0;
  int site;
  Timer(unet_plan* p_, hipStream_t s_, int c, double f, double by_, bool on = true, int site_ = -1)
      : p(p_), s(s_), cls(c), fl(f), by(by_), x0(p_->xfl), site(site_) {
    // timing is best effort (bench / tools only): a failed event leaves the
    // interval out of the report instead of failing the plan call
    if (p->timing && on) {
      ok = hipEventCreate(&a) == hipSuccess;
      if (ok && hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        ok = false;
      }
      if (ok) ok = hipEventRecord(a, s) == hipSuccess;
    }
  }
  ~Timer() {
    if (p->timing && ok) {
      if (hipEventRecord(b, s) == hipSuccess) {
        p->evs.push_back({a, b, cls, fl, by, p->xfl - x0, site});
      } else {
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
      }
    }
  }
};


// ---------------- GEMM variant autotuner ------------------------------------
// Every implicit-GEMM launch site is resolved to a (tile, split) variant by
// timing the applicable candidates once, on the live operands, the first time
// its GEMM shape is met (the way MIOpen's find step picks a conv solver).
// Choices are cached process-wide per shape key, so plans of equal shapes (the
// Trainer and a drop-in module, DP replicas in one process) run identical
// kernels.  Trial launches redirect their atomic accumulators to scratch; their
// plain stores are overwritten by the real launch that follows.
std::mutex g_tune_mu;
std::map<std::string, GemmChoice> g_tuned;
std::map<std::string, std::string> g_tune_log;

// Tuning database (the analogue of MIOpen's perf-db): one "key<TAB>tile<TAB>split"
// line per tuned GEMM shape.  With UNET_TUNE_DB=<path> the first lookup loads
// the file and every newly tuned shape is appended to it, so a later process
// (a profiler pass, a restarted job) replays the same kernel choices instead of
// re-timing them under different conditions.  Callers hold g_tune_mu.
int tune_db_read(const char* path, bool overwrite) {
  FILE* f = fopen(path, "r");
  if (!f) return -errno;
  char line[512];
  int n = 0;
  while (fgets(line, sizeof line, f)) {
    char* t1 = strchr(line, '\t');
    if (!t1) continue;
    *t1 = 0;
    int tile = 0, split = 0;
    if (sscanf(t1 + 1, "%d\t%d", &tile, &split) != 2) continue;
    const std::string key(line);
    if (!overwrite && g_tuned.count(key)) continue;
    g_tuned[key] = GemmChoice{tile, split};
    g_tune_log[key] = key + " | tuning db: tile " + std::to_string(tile) + " split " + std::to_string(split);
    ++n;
  }
  fclose(f);
  return n;
}

const char* tune_db_path() {
  static const char* p = getenv("UNET_TUNE_DB");
  return p && *p ? p : nullptr;
}

void tune_db_load_once() {
  static bool done = false;
  if (done) return;
  done = true;
  if (const char* p = tune_db_path()) (void)tune_db_read(p, false);
}

void tune_db_append(const std::string& key, const GemmChoice& g) {
  const char* p = tune_db_path();
  if (!p) return;
  if (FILE* f = fopen(p, "a")) {
    fprintf(f, "%s\t%d\t%d\n", key.c_str(), g.tile, g.split);
    fclose(f);
  }
}

int env_autotune() { return unet::g_autotune; }

constexpr size_t kSlabBudget = 256ull << 20;  // split-K partials (fp32)

// Version of the GEMM variant tables (tile ids and their kernels): part of every
// tuning key, so a database written by a build with another tile set is never
// replayed (its lines simply miss).  Bump whenever a tile id changes meaning.
constexpr int kTileTableVersion = 14;

std::string igemm_key(const IgemmArgs& a) {
  char b[240], small[16] = "";
  if (unet::g_wino4_fwd_small_cg) snprintf(small, sizeof small, "/s%d", unet::g_wino4_fwd_small_cg);
  const Epilogue& e = a.e;
  const int epi = (e.shuffle_co ? 1 : 0) | (e.stats ? 2 : 0) | (e.yref ? 4 : 0) | (e.colsum1 ? 8 : 0) |
                  (a.a.s[0].scale ? 16 : 0) | (a.a.c_split != a.a.Cg ? 32 : 0) | (e.relu ? 64 : 0) |
                  // a forward without statistics or ReLU (unfolded eval): the
                  // only forward the other bits do not already tell apart
                  (a.fwd && !e.stats && !e.relu ? 128 : 0);
  // the Winograd caps decide which candidates exist: a choice tuned under other
  // caps is a different key
  snprintf(b, sizeof b, "igemm%s M=%d N=%d K=%d Cg=%d taps=%dx%d s=%d grid=%dx%d epi=%d wino=%d/%d/%d%s tt=%d",
           a.bl ? "_bf16x3" : a.bh ? "_bf16" : "", a.M,
           a.N, a.K, a.a.Cg, a.a.taps_h, a.a.taps_w, a.a.stride, a.a.Hg, a.a.Wg, epi, unet::g_wino_max,
           unet::g_wino_dgrad_max, unet::g_wino4_fwd_min_cg, small, kTileTableVersion);
  return b;
}

std::string wgrad_key(const WgradArgs& a) {
  char b[240];
  snprintf(b, sizeof b, "wgrad%s Mo=%d No=%d P=%d Cg=%d taps=%dx%d s=%d grid=%dx%d wino=%d%s tt=%d",
           a.split ? "_bf16x3" : a.bf16 ? "_bf16" : "", a.Mo,
           a.No, a.P, a.gb.Cg, a.gb.taps_h, a.gb.taps_w, a.gb.stride, a.gb.Hg, a.gb.Wg, unet::g_wino_wgrad_max,
           unet::g_deterministic ? " det" : "", kTileTableVersion);
  return b;
}

// a weight-gradient variant that adds no fp32 atomics: slab modes (ring per_cu
// codes 11 / 12, pixel-column codes 101-104, Winograd codes >= 1000: split
// partials by plain stores, summed by k_wr_reduce in a fixed order; one split
// stores straight into the gradient).  A slab launch whose partials exceed
// the plan's slab falls back to atomics and counts in unet_slab_fallbacks().
bool wgrad_choice_deterministic(const GemmChoice& g) {
  if (g.tile == 71 || g.tile == 74) return g.split >= 1000;
  if (g.tile >= 26 && g.tile <= 33) return g.split >= 10;
  if (g.tile >= 40 && g.tile <= 44) return g.split >= 10;
  if (g.tile >= 0 && g.tile <= 14) return g.split >= 100;
  return false;
}

// UNET_TUNE_SKIP="73,74": tile ids the autotuner never tries (A/B experiments
// on accuracy or speed; igemm and wgrad ids alike)
bool tune_skipped(int tile) {
  static const std::vector<int> skip = [] {
    std::vector<int> v;
    if (const char* e = getenv("UNET_TUNE_SKIP"))
      for (const char* q = e; *q;) {
        char* end = nullptr;
        const long t = strtol(q, &end, 10);
        if (end == q) { ++q; continue; }
        v.push_back((int)t);
        q = end;
      }
    return v;
  }();
  for (int t : skip)
    if (t == tile) return true;
  return false;
}

std::vector<GemmChoice> igemm_candidates(const IgemmArgs& a, size_t slab_bytes) {
  std::vector<GemmChoice> v;
  const long long cus = num_cus();
  for (int t : {4, 1, 2, 8, 6, 3, 9, 7, 11, 12, 13, 14, 51, 52, 53, 54, 21, 22, 23, 24, 25, 26, 31, 32, 33, 34, 35,
                36, 41, 42, 43, 44, 63, 65, 66, 67, 68, 81, 82, 83, 84, 85, 70, 71, 72, 73,
                74, 75, 76, 77, 88, 91, 92, 93, 94, 95, 96, 97, 98, 99}) {  // fits() filters by precision and gather
    if (!igemm_tile_fits(a, t) || tune_skipped(t)) continue;
    // (86, the stream-K form of 85, and 87, the resident-weight 64-channel
    // kernel, are forced only: measured slower on the shapes they target --
    // DESIGN.md §13)
    if (t == 86 && conv3_flat_sk_slab_bytes(a) > slab_bytes) continue;  // stream-K partial slots
    v.push_back({t, 1});
    if (t == 70 || t == 71 || t == 74)  // Winograd: no K split; the tile of its batched point GEMMs
      for (int inner : {1, 2, 3, 4, 6, 7, 8, 9}) v.push_back({t, 100 + inner});
    // Winograd (70-77) and the persistent ring 88 take no K split; the LDS-DMA
    // rings 81-84 (3x3) and 91-99 (convT) do (the 24-48^2
    // bottleneck grids give them 144-192 workgroups for 256 CUs)
    if ((t >= 70 && t <= 77) || t == 88 || t == 86 || t == 87) continue;
    const long long cnt = igemm_tile_count(a, t);
    const long long slots = (long long)igemm_tile_slots(t) * cus;
    if (cnt >= 4 * slots || a.N % 64 != 0) continue;  // enough workgroup rounds already
    for (int ks : {2, 3, 4, 6, 8}) {
      if (igemm_slab_bytes(a, ks) > slab_bytes || a.K / ks < 256 || cnt * ks > 8 * slots) break;
      v.push_back({t, ks});
    }
  }
  return v;
}

std::vector<GemmChoice> wgrad_candidates(const WgradArgs& a) {
  std::vector<GemmChoice> v;
  for (int t : {0, 1, 2, 3, 4, 10, 11, 12, 13, 14, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 40, 41, 42, 43, 44,
                71, 74}) {  // fits() filters by precision
    if (!wgrad_tile_fits(a, t) || tune_skipped(t)) continue;
    if (t >= 40 && t <= 44) {  // convT LDS-DMA ring (one resident workgroup per CU): slab mode only
      for (int per_cu : {11, 12}) v.push_back({t, per_cu});
      continue;
    }
    if (t == 71 || t == 74) {  // Winograd: point-GEMM tile (k_wgrad 0-4) x workgroups per CU
      // (each pixel split adds a full points x Co x Ci slab by fp32 atomics:
      // 1-2 per CU cut that traffic on the deep, few-tile layers); + 1000:
      // slab mode (plain-store partials, no accumulator memset)
      for (int inner : {0, 1, 2, 3, 4})
        for (int per_cu : {1, 2, 4, 8, 16}) v.push_back({t, per_cu + 100 * (inner + 1)});
      if (a.slab)
        for (int inner : {0, 3, 4})
          for (int per_cu : {1, 2, 4}) v.push_back({t, 1000 + per_cu + 100 * (inner + 1)});
      continue;
    }
    if (t >= 24 && t <= 33) {  // wide halo-tiled / LDS-DMA ring: one resident workgroup per CU
      for (int per_cu : {1, 2}) v.push_back({t, per_cu});
      // ring (26-33) in slab mode: split partials by plain stores + one
      // reduction pass instead of per-element fp32 atomics
      if (t >= 26 && a.slab)
        for (int per_cu : {11, 12}) v.push_back({t, per_cu});
      continue;
    }
    if (t >= 20) {  // halo-tiled: workgroups per CU (2 resident)
      for (int per_cu : {1, 2, 4, 8}) v.push_back({t, per_cu});
      continue;
    }
    // pixel-split column tiles: fewer splits trade fill for fewer fp32
    // atomics per output (the short-pixel convT weight gradients); codes
    // 101-104: the same splits in slab mode (plain-store partials + reduction)
    for (int per_cu : {1, 2, 4, 8, 16}) v.push_back({t, per_cu});
    if (a.slab && a.batch == 1)
      for (int per_cu : {101, 102, 104}) v.push_back({t, per_cu});
  }
  return v;
}

// min over 2 timed runs after 1 warm-up; < 0 if the launch failed
template <typename F>
float time_launch(hipStream_t s, F&& launch) {
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return -1.f;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return -1.f;
  }
  float best = -1.f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0, s);
    if (launch() != hipSuccess) {
      (void)hipGetLastError();
      best = -1.f;
      break;
    }
    (void)hipEventRecord(e1, s);
    if (hipEventSynchronize(e1) != hipSuccess) {
      best = -1.f;
      break;
    }
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r > 0 && (best < 0.f || ms < best)) best = ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

GemmChoice choose_igemm(const Ctx& c, const IgemmArgs& a) {
  if (unet::g_force_split > 1 || unet::g_force_tile > 0) {
    const int ks = unet::g_force_split > 1 ? unet::g_force_split : 1;
    if (igemm_slab_bytes(a, ks) > c.p->slab.bytes) return GemmChoice{};
    if (unet::g_force_tile > 0) {
      if (igemm_tile_fits(a, unet::g_force_tile) &&
          (unet::g_force_tile != 86 || (ks == 1 && conv3_flat_sk_slab_bytes(a) <= c.p->slab.bytes)))
        return GemmChoice{unet::g_force_tile, ks};
    }
    for (int t : {4, 1, 2, 8, 21, 22, 24, 23})
      if (igemm_tile_fits(a, t)) return GemmChoice{t, ks};
    return GemmChoice{};
  }
  if (!env_autotune()) return GemmChoice{};
  const std::string key = igemm_key(a);
  std::lock_guard<std::mutex> lk(g_tune_mu);
  tune_db_load_once();
  auto it = g_tuned.find(key);
  if (it != g_tuned.end()) {
    // a cached / database choice must still apply to this build and plan (a
    // database from another tile set, or a split whose partials no longer fit
    // the slab): otherwise it is dropped and the shape re-tuned
    const GemmChoice g = it->second;
    const bool slab_ok = g.tile == 86 ? conv3_flat_sk_slab_bytes(a) <= c.p->slab.bytes
                                      : g.tile >= 70 || igemm_slab_bytes(a, g.split) <= c.p->slab.bytes;  // Winograd: split = inner tile
    if (g.tile < 0 || (igemm_tile_fits(a, g.tile) && slab_ok)) return g;
    g_tuned.erase(it);
    g_tune_log.erase(key);
  }
  if (capturing(c.s)) return GemmChoice{};  // hipGraph capture: replay the tuned choice, never time
  IgemmArgs t = a;
  double* scr = c.d(c.p->tune_scratch);
  if (t.e.stats) t.e.stats = scr;
  if (t.e.bstats) t.e.bstats = scr;
  if (t.e.colsum1) t.e.colsum1 = scr;
  const float th = time_launch(c.s, [&] { return launch_igemm(t, c.s); });
  GemmChoice best{};
  float tb = th;
  std::string log = key + " | heuristic " + std::to_string(th * 1e3f) + " us";
  static const bool verbose = getenv("UNET_TUNE_VERBOSE") != nullptr;
  std::string all;
  for (const GemmChoice& g : igemm_candidates(a, c.p->slab.bytes)) {
    const float tm = time_launch(c.s, [&] { return launch_igemm_v(t, c.s, g); });
    if (verbose)
      all += " " + std::to_string(g.tile) + (g.split > 1 ? "s" + std::to_string(g.split) : "") + ":" +
             std::to_string((int)(tm * 1e3f));
    if (tm > 0.f && (tb < 0.f || tm < tb)) {
      tb = tm;
      best = g;
    }
  }
  log += " | best tile " + std::to_string(best.tile) + " split " + std::to_string(best.split) + " " +
         std::to_string(tb * 1e3f) + " us" + (verbose ? " |" + all : "");
  g_tuned[key] = best;
  g_tune_log[key] = log;
  tune_db_append(key, best);
  return best;
}

GemmChoice choose_wgrad(const Ctx& c, const WgradArgs& a) {
  const bool det = unet::g_deterministic != 0;
  if (!env_autotune() && !det) return GemmChoice{};
  if (det && !env_autotune()) {  // untimed: the first atomic-free candidate
    for (const GemmChoice& g : wgrad_candidates(a))
      if (wgrad_choice_deterministic(g)) return g;
    return GemmChoice{};
  }
  const std::string key = wgrad_key(a);
  std::lock_guard<std::mutex> lk(g_tune_mu);
  tune_db_load_once();
  auto it = g_tuned.find(key);
  if (it != g_tuned.end()) {
    const GemmChoice g = it->second;
    if (g.tile < 0 || wgrad_tile_fits(a, g.tile)) return g;
    g_tuned.erase(it);  // not applicable to this build: re-tune
    g_tune_log.erase(key);
  }
  if (capturing(c.s)) return GemmChoice{};
  WgradArgs t = a;
  t.out = c.f(c.p->tune_scratch);
  // deterministic mode: the heuristic (atomics) is no candidate
  const float th = det ? -1.f : time_launch(c.s, [&] { return launch_wgrad(t, c.s); });
  GemmChoice best{};
  float tb = th;
  std::string log = key + " | heuristic " + std::to_string(th * 1e3f) + " us";
  static const bool verbose = getenv("UNET_TUNE_VERBOSE") != nullptr;
  std::string all;
  for (const GemmChoice& g : wgrad_candidates(a)) {
    if (det && !wgrad_choice_deterministic(g)) continue;
    const float tm = time_launch(c.s, [&] { return launch_wgrad_v(t, c.s, g); });
    if (verbose) all += " " + std::to_string(g.tile) + "/" + std::to_string(g.split) + ":" + std::to_string((int)(tm * 1e3f));
    if (tm > 0.f && (tb < 0.f || tm < tb)) {
      tb = tm;
      best = g;
    }
  }
  log += " | best tile " + std::to_string(best.tile) + " per_cu " + std::to_string(best.split) + " " +
         std::to_string(tb * 1e3f) + " us" + (verbose ? " |" + all : "");
  g_tuned[key] = best;
  g_tune_log[key] = log;
  tune_db_append(key, best);
  return best;
}

hipError_t run_igemm(const Ctx& c, IgemmArgs a) {
  a.slab = c.f(c.p->slab);
  if (c.p->wino.bytes) {  // fp32 plans: the Winograd candidate's scratch
    a.wino_ws = c.f(c.p->wino);
    a.wino_ws_bytes = c.p->wino.bytes;
  }
  if (c.p->prec != UNET_PREC_FP32) {  // B -> its bf16 copy (and lo plane) at the same element offset
    const char* b = reinterpret_cast<const char*>(a.b);
    const char* base = c.ws + c.p->pack_region.off;
    if (b < base || b >= base + c.p->pack_region.bytes) return hipErrorInvalidValue;
    const size_t el = (b - base) / sizeof(float);
    const uint16_t* hi = reinterpret_cast<const uint16_t*>(c.ws + c.p->pack16.off);
    a.bh = hi + el;
    if (c.p->prec == UNET_PREC_BF16X3) a.bl = hi + c.p->pack_region.bytes / 4 + el;
    a.b = nullptr;
  }
  const GemmChoice ch = choose_igemm(c, a);
  if (c.p->timing) c.p->xfl += igemm_exec_flops(a, ch);
  return launch_igemm_v(a, c.s, ch);
}

void prep_wgrad(const Ctx& c, WgradArgs& a) {
  a.bf16 = c.p->prec != UNET_PREC_FP32;
  a.split = c.p->prec == UNET_PREC_BF16X3;
  if (c.p->wino_w.bytes && !a.wino_ws) {  // fp32 training plans: the Winograd weight-gradient scratch
    a.wino_ws = c.f(c.p->wino_w);           // (side stream; a layer's own with wgrad_fwd_u)
    a.wino_ws_bytes = c.p->wino_w.bytes;
  }
  if (c.p->wslab.bytes) {  // partial planes of the slab-mode weight gradients (side stream)
    a.slab = c.f(c.p->wslab);
    a.slab_bytes = c.p->wslab.bytes;
  }
}

hipError_t run_wgrad(const Ctx& c, WgradArgs a) {
  prep_wgrad(c, a);
  const GemmChoice ch = choose_wgrad(c, a);
  if (unet::g_deterministic && !wgrad_choice_deterministic(ch)) ++unet::g_nondet_sites;
  if (c.p->timing) c.p->xfl += wgrad_exec_flops(a, ch);
  return launch_wgrad_v(a, c.s, ch);
}

Src src_of(const Ctx& c, const Conv& L, bool transform) {
  Src s;
  s.ptr = c.f(L.y);
  s.H = L.ho;
  s.W = L.wo;
  s.C = L.co;
  s.h16 = c.p->prec == UNET_PREC_BF16;  // raw conv outputs of a bf16 plan are stored bf16
  if (transform && !c.p->fold) {  // folded eval: y is already relu(bn(conv))
    s.scale = c.f(L.scale);
    s.shift = c.f(L.shift);
  }
  return s;
}

// Layer l's output as its GEMM consumers read it: relu(bn(y)).  bf16 plans
// read the normalised bf16 copy (written once per element after the layer's
// statistics are final: k_bn_relu_bf, or the max-pool for encoder outputs), so
// their staging is a plain copy; fp32 plans apply BN+ReLU on load.
Src src_in(const Ctx& c, int l) {
  const Conv& L = c.p->L[l];
  if (!L.a.bytes || c.p->fold) return src_of(c, L, true);
  Src s;
  s.ptr = c.f(L.a);
  s.H = L.ho;
  s.W = L.wo;
  s.C = L.co;
  s.h16 = 1;
  return s;
}

// Gather describing the input of conv layer l (1..17), as rows over its OUTPUT grid
// with 3x3 taps (forward A operand and wgrad B operand).
Gather input_gather(const Ctx& c, int l) {
  unet_plan* p = c.p;
  const Conv& L = p->L[l];
  Gather g;
  g.taps_h = g.taps_w = 3;
  g.stride = 1;
  g.Hg = L.ho;
  g.Wg = L.wo;
  g.nimg = p->n;
  if (l % 2 == 1) {  // second conv of a DoubleConv: input = relu(bn(y[l-1]))
    g.s[0] = src_in(c, l - 1);
    g.Cg = g.c_split = L.ci;
  } else if (l <= 8) {  // first conv of down block: pooled tensor
    const Pool& pl = p->P[l / 2 - 1];
    Src s;
    s.ptr = c.f(pl.p);
    s.H = pl.h / 2;
    s.W = pl.w / 2;
    s.C = pl.c;
    s.h16 = p->prec == UNET_PREC_BF16;
    g.s[0] = s;
    g.Cg = g.c_split = L.ci;
  } else {  // first conv of up block: cat([crop(skip), up], 1)
    const int k = (l - 10) / 2;
    const Skip& sk = p->S[k];
    const int enc = 7 - 2 * k;
    Src a = src_in(c, enc);
    a.oy = sk.oy;
    a.ox = sk.ox;
    Src b;
    b.ptr = c.f(p->T[k].u);
    b.H = 2 * p->T[k].h;
    b.W = 2 * p->T[k].w;
    b.C = p->T[k].co;
    b.h16 = p->prec == UNET_PREC_BF16;
    g.s[0] = a;
    g.s[1] = b;
    g.c_split = sk.c;
    g.Cg = sk.c + p->T[k].co;
  }
  if (g.s[1].ptr == nullptr) g.s[1] = g.s[0];
  return g;
}

hipError_t ensure_side_stream(unet_plan* p);

// Weight gradient of 3x3 layer l >= 1: dW(l) = dY(l)^T x im2col(input of l),
// dY read from the interior of the padded buffer
WgradArgs conv_wgrad_args(const Ctx& c, int l) {
  const Conv& L = c.p->L[l];
  Src dy;
  dy.ptr = c.f(L.dyp);
  dy.H = L.ho + 4;
  dy.W = L.wo + 4;
  dy.C = L.co;
  dy.oy = dy.ox = 2;
  dy.h16 = c.p->prec == UNET_PREC_BF16;
  WgradArgs w;
  w.ga.s[0] = dy;
  w.ga.s[1] = dy;
  w.ga.Cg = w.ga.c_split = L.co;
  w.ga.Hg = L.ho;
  w.ga.Wg = L.wo;
  w.ga.nimg = c.p->n;
  w.gb = input_gather(c, l);
  w.Mo = L.co;
  w.No = 9 * L.ci;
  w.P = c.p->n * L.ho * L.wo;
  w.out = c.f(L.dwp);
  return w;
}

int run_forward(unet_plan* p, void* const* prm, const float* x, float* logits, char* ws, int train, hipStream_t s) {
  Ctx c{p, ws, s};
  const int n = p->n;
  // One memset for every accumulator of this forward AND of the backward that
  // follows it (BN stats, BN-bwd stats, convT bias sums, head/loss sums, and in
  // train mode the packed weight-gradient region, laid out right after).
  CK(hipMemsetAsync(ws + p->stat_region.off, 0, p->stat_region.bytes + (train ? p->dwp_region.bytes : 0), s));
  p->fold = !train && unet::g_bn_fold;
  // ---- repack weights (per call: the optimizer moves them every step) ----
  {
    Timer t(p, s, UNET_KC_ELEMWISE, 0, 0);
    PackJobs jobs{};
    for (int l = 1; l < 18; ++l) {
      Conv& L = p->L[l];
      jobs.j[jobs.n++] = PackJob{P<float>(prm, L.pw), c.f(L.wf), train ? c.f(L.wd) : nullptr, L.co, L.ci, 0};
    }
    for (int k = 0; k < 4; ++k) {
      ConvT& T = p->T[k];
      jobs.j[jobs.n++] = PackJob{P<float>(prm, T.pw), c.f(T.wf), c.f(T.wd), T.co, T.ci, 1};
    }
    CK(launch_pack_all(jobs, s));
    if (!train) {  // BatchNorm from the running statistics (scripts/predict.py:70 model.eval())
      for (int l = 0; l < 18; ++l) {
        Conv& L = p->L[l];
        CK(launch_bn_eval_prepare(L.co, P<float>(prm, L.pw + 2), P<float>(prm, L.pw + 3), P<float>(prm, L.pw + 4),
                                  P<float>(prm, L.pw + 5), c.f(L.scale), c.f(L.shift), kEps, s));
      }
    }
    if (p->fold) {  // bn(conv(x)) = conv'(x): scale into the weights, folded bias into L.coef
      const Conv& L0 = p->L[0];
      CK(launch_fold_bn(P<float>(prm, L0.pw), 9LL * L0.ci, L0.co, c.f(L0.scale), c.f(L0.shift),
                        P<float>(prm, L0.pw + 1), c.f(p->fold0w), c.f(L0.coef), s));
      for (int l = 1; l < 18; ++l) {
        Conv& L = p->L[l];
        CK(launch_fold_bn(c.f(L.wf), 9LL * L.ci, L.co, c.f(L.scale), c.f(L.shift), P<float>(prm, L.pw + 1),
                          c.f(L.wf), c.f(L.coef), s));
      }
    }
    if (p->prec != UNET_PREC_FP32) {
      uint16_t* hi = reinterpret_cast<uint16_t*>(c.u8(p->pack16));
      const size_t ne = p->pack_region.bytes / 4;
      CK(launch_f2bf(c.f(p->pack_region), hi, ne, s, p->prec == UNET_PREC_BF16X3 ? hi + ne : nullptr));
    }
  }
  auto finalize = [&](int l) -> int {
    if (!train) return 0;
    Conv& L = p->L[l];
    CK(launch_bn_finalize(c.d(L.stats), L.co, (double)n * L.ho * L.wo, P<float>(prm, L.pw + 2),
                          P<float>(prm, L.pw + 3), P<float>(prm, L.pw + 4), P<float>(prm, L.pw + 5),
                          P<int64_t>(prm, L.pw + 6), c.f(L.mean), c.f(L.invstd), c.f(L.scale), c.f(L.shift), kMom,
                          kEps, s));
    return 0;
  };
  // bf16 plans: the normalised copy of layer l's output (encoder outputs get it
  // from their max-pool, which reads every element with the transform anyway)
  auto normalise = [&](int l) -> int {
    Conv& L = p->L[l];
    if (!L.a.bytes || p->fold || (l <= 7 && l % 2 == 1)) return 0;
    Timer t(p, s, UNET_KC_ELEMWISE, 0, 4.0 * n * L.ho * L.wo * L.co);
    CK(launch_bn_relu_bf(reinterpret_cast<const uint16_t*>(c.f(L.y)), c.f(L.scale), c.f(L.shift),
                         (long long)n * L.ho * L.wo, L.co, reinterpret_cast<uint16_t*>(c.f(L.a)), s));
    return 0;
  };
  // ---- inc.c0 ----
  {
    Conv& L = p->L[0];
    Timer t(p, s, UNET_KC_STAGE1, conv_flops(L, n),
            4.0 * n * (double)p->cin * p->h * p->w +
                (p->prec == UNET_PREC_BF16 ? 2.0 : 4.0) * n * (double)L.ho * L.wo * L.co);
    CK(launch_conv_first_fwd(x, n, p->cin, p->h, p->w, p->fold ? c.f(p->fold0w) : P<float>(prm, L.pw),
                             p->fold ? c.f(L.coef) : P<float>(prm, L.pw + 1), L.co, c.f(L.y),
                             train ? c.d(L.stats) : nullptr, s, p->prec == UNET_PREC_BF16, p->fold));
  }
  if (int r = finalize(0)) return r;
  if (int r = normalise(0)) return r;
  for (int l = 1; l < 18; ++l) {
    Conv& L = p->L[l];
    if (l >= 10 && l % 2 == 0) {  // ConvTranspose2d of up block k, input = y[l-1]
      const int k = (l - 10) / 2;
      ConvT& T = p->T[k];
      IgemmArgs a;
      a.a.s[0] = src_in(c, l - 1);
      a.a.s[1] = a.a.s[0];
      a.a.Cg = a.a.c_split = T.ci;
      a.a.Hg = T.h;
      a.a.Wg = T.w;
      a.a.nimg = n;
      a.b = c.f(T.wf);
      a.M = n * T.h * T.w;
      a.N = 4 * T.co;
      a.K = T.ci;
      a.e.bias = P<float>(prm, T.pw + 1);  // bias[co], col = ab*Co + co
      a.e.shuffle_co = T.co;
      a.e.d[0] = Dst{c.f(T.u), 2 * T.h, 2 * T.w, T.co, 0, 0, p->prec == UNET_PREC_BF16};
      Timer t(p, s, UNET_KC_CONV_FWD, 2.0 * a.M * a.N * a.K, 0, true, site_convT(k, 0));
      Timer tb(p, s, UNET_KC_BOTTLENECK, 2.0 * a.M * a.N * a.K, 0, k == 0);
      CK(run_igemm(c, a));
    }
    L.u_fwd = false;
    if (train && unet::g_wgrad_fwd_u && L.uws.bytes && unet::g_concurrent && !p->timing && p->bwd_full > 0) {
      // this layer's weight-gradient input transform U on the (idle) side
      // stream, beside the forward GEMMs: its inputs are final at this point
      CK(ensure_side_stream(p));
      Ctx cs{p, ws, p->side};
      WgradArgs q = conv_wgrad_args(c, l);
      prep_wgrad(cs, q);
      const int mt = wgrad_winograd_mt(q, choose_wgrad(cs, q));
      q.wino_ws = c.f(L.uws);
      q.wino_ws_bytes = L.uws.bytes;
      if (mt && wino_wgrad_applies(q, mt)) {
        CK(hipEventRecord(p->ev_fwdu, s));
        CK(hipStreamWaitEvent(p->side, p->ev_fwdu, 0));
        CK(launch_wino_wgrad_u(q, p->side, mt));
        L.u_fwd = true;
      }
    }
    IgemmArgs a;
    a.a = input_gather(c, l);
    a.b = c.f(L.wf);
    a.M = n * L.ho * L.wo;
    a.N = L.co;
    a.K = 9 * L.ci;
    a.e.bias = p->fold ? c.f(L.coef) : P<float>(prm, L.pw + 1);
    a.e.relu = p->fold;
    a.fwd = 1;
    a.e.d[0] = Dst{c.f(L.y), L.ho, L.wo, L.co, 0, 0, p->prec == UNET_PREC_BF16};
    a.e.stats = train ? c.d(L.stats) : nullptr;
    {
      Timer t(p, s, UNET_KC_CONV_FWD, conv_flops(L, n), 0, true, site_conv(l, 0));
      Timer tb(p, s, UNET_KC_BOTTLENECK, conv_flops(L, n), 0, bottleneck_conv(l));
      CK(run_igemm(c, a));
    }
    if (int r = finalize(l)) return r;
    if (int r = normalise(l)) return r;
    if (l <= 7 && l % 2 == 1) {  // encoder output -> MaxPool2d(2)
      Pool& pl = p->P[l / 2];
      Timer t(p, s, UNET_KC_ELEMWISE, 0, 4.0 * n * pl.h * pl.w * pl.c * 1.25);
      CK(launch_maxpool_fwd(src_of(c, L, true), n, pl.h, pl.w, c.f(pl.p), c.u8(pl.arg), s, p->prec == UNET_PREC_BF16,
                            L.a.bytes && !p->fold ? reinterpret_cast<uint16_t*>(c.f(L.a)) : nullptr));
    }
  }
  {
    Conv& L = p->L[17];
    Timer t(p, s, UNET_KC_ELEMWISE, 0, 4.0 * n * L.ho * L.wo * (L.co + p->ncls));
    CK(launch_head_fwd(src_of(c, L, true), n, L.ho, L.wo, L.co, P<float>(prm, 134), P<float>(prm, 135), p->ncls,
                       logits, s));
  }
  return 0;
}

// segment id of each backward step (for DP overlap): 0 = head+up4 ... 3 = up1,
// 4 = down4 ... 7 = down1, 8 = inc.
int seg_of_layer(int l) {
  if (l >= 10) return (17 - l) / 2;  // 17,16 -> 0 ; 11,10 -> 3
  return 4 + (9 - l) / 2;            // 9,8 -> 4 ; 1,0 -> 8
}

hipError_t ensure_side_stream(unet_plan* p) {
  if (p->side) return hipSuccess;
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  e = hipStreamCreateWithPriority(&p->side, hipStreamNonBlocking, least);
  if (e != hipSuccess) return e;
  for (auto& ev : p->ev_dy)
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
  for (auto& ev : p->ev_du)
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
  for (auto& ev : p->ev_seg)
    if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return e;
  if ((e = hipEventCreateWithFlags(&p->ev_bwd0, hipEventDisableTiming)) != hipSuccess) return e;
  if ((e = hipEventCreateWithFlags(&p->ev_fwdu, hipEventDisableTiming)) != hipSuccess) return e;
  return hipEventCreateWithFlags(&p->ev_join, hipEventDisableTiming);
}

int run_backward(unet_plan* p, void* const* prm, void* const* grd, const float* x, const float* dlogits, char* ws,
                 int seg_b, int seg_e, hipStream_t s, int flags) {
  Ctx c{p, ws, s};
  const int n = p->n;
  // bf16 plans store the activation gradients between GEMMs in bf16 (as
  // autocast does): the BN-input gradients dz, the pooled-map gradient and the
  // skip gradient; their BN-backward statistics are those of the rounded values
  const int g16 = p->prec == UNET_PREC_BF16;
  // Weight gradients of layer l need only dY(l) and forward tensors: they go to
  // the side stream once the plan is tuned (timing runs stay serial so that
  // per-kernel event times stay clean).  Under hipGraph capture the side stream
  // joins the capture through the fork / join events.
  const bool conc = unet::g_concurrent && !p->timing && p->bwd_full > 0;
  if (conc) CK(ensure_side_stream(p));
  Ctx cw{p, ws, conc ? p->side : s};
  const hipStream_t sw = cw.s;
  auto in_seg = [&](int sg) { return sg >= seg_b && sg < seg_e; };
  if (conc && unet::g_wgrad_early_u) {
    // early U transforms read this step's forward tensors: the side stream
    // starts after everything the main stream has queued so far
    CK(hipEventRecord(p->ev_bwd0, s));
    CK(hipStreamWaitEvent(sw, p->ev_bwd0, 0));
  }
  if (seg_b == 0) {
    // accumulators (bstats, colsums, packed weight grads) were zeroed by the
    // train-mode forward that filled this workspace
    Conv& L = p->L[17];
    Timer t(p, s, UNET_KC_ELEMWISE, 0, 4.0 * n * L.ho * L.wo * (2 * L.co + p->ncls));
    CK(launch_head_bwd(src_of(c, L, true), dlogits, n, L.ho, L.wo, L.co, P<float>(prm, 134), p->ncls, c.f(L.y),
                       c.f(L.mean), c.f(L.invstd), c.f(L.dz), c.d(L.bstats), P<float>(grd, 80), P<float>(grd, 81),
                       c.d(p->head_acc), s, g16));
  }
  for (int l = 17; l >= 0; --l) {
    if (!in_seg(seg_of_layer(l))) continue;
    Conv& L = p->L[l];
    const double M = (double)n * L.ho * L.wo;
    const int dy16 = p->prec == UNET_PREC_BF16 && l > 0;
    if (l == 0) {
      // stage 1 backward: BN0 backward fused into inc.c0's weight
      // gradient -- reads dz0, y0 and x once, dY(0) is never materialised
      {
        Timer t(p, s, UNET_KC_STAGE1, 0, 0);
        CK(launch_bnb_finalize(c.d(L.bstats), L.co, M, P<float>(prm, L.pw + 2), c.f(L.mean), c.f(L.invstd),
                               P<float>(grd, L.gw + 2), P<float>(grd, L.gw + 3), P<float>(grd, L.gw + 1),
                               c.f(L.coef), s));
      }
      if (conc) {
        CK(hipEventRecord(p->ev_dy[l], s));
        CK(hipStreamWaitEvent(sw, p->ev_dy[l], 0));
      }
      Timer t(p, sw, UNET_KC_STAGE1, 2.0 * M * L.co * L.ci * 9,
              4.0 * n * ((double)p->cin * p->h * p->w) +
                  (p->prec == UNET_PREC_BF16 ? 6.0 : 8.0) * n * (double)L.ho * L.wo * L.co);
      CK(launch_conv_first_wgrad_bn(x, n, p->cin, p->h, p->w, c.f(L.dz), c.f(L.y), p->prec == UNET_PREC_BF16,
                                    c.f(L.coef), L.co, P<float>(grd, L.gw), c.f(p->first_slabs), sw, g16));
      continue;
    }
    CK(launch_bnb_finalize(c.d(L.bstats), L.co, M, P<float>(prm, L.pw + 2), c.f(L.mean), c.f(L.invstd),
                           P<float>(grd, L.gw + 2), P<float>(grd, L.gw + 3), P<float>(grd, L.gw + 1), c.f(L.coef), s));
    WgradArgs w = conv_wgrad_args(c, l);  // weight gradient dW(l) = dY(l)^T x im2col(input of l)
    const Src dy = w.ga.s[0];             // dY interior of the padded buffer
    if (L.u_fwd && conc) {  // U issued by this step's forward on the side stream (FIFO before this wgrad)
      w.wino_ws = c.f(L.uws);
      w.wino_ws_bytes = L.uws.bytes;
      w.u_ready = 1;
    }
    L.u_fwd = false;
    // fp32: when this weight gradient runs Winograd F(6x6), dY and its transform
    // Vd come out of one pass over dz and y (k_bnb_wino6_dy)
    bool fused_vd = false;
    const bool early_u = conc && unet::g_wgrad_early_u && !w.u_ready;
    if (p->prec == UNET_PREC_FP32 && ((unet::g_bnb_fuse && L.vdw.bytes) || early_u)) {
      WgradArgs q = w;
      prep_wgrad(cw, q);
      const int wmt = wgrad_winograd_mt(q, choose_wgrad(cw, q));
      fused_vd = unet::g_bnb_fuse && wmt == 6 && L.vdw.bytes >= bnb_wino6_vd_bytes(n, L.ho, L.wo, L.co);
      if (early_u && wmt) {  // side stream, FIFO after the previous layer's point GEMMs
        CK(launch_wino_wgrad_u(q, sw, wmt));
        w.u_ready = 1;
      }
    }
    if (fused_vd) {
      Timer t(p, s, UNET_KC_ELEMWISE, 0,
              4.0 * n * ((double)(L.ho + 4) * (L.wo + 4) + 2.0 * L.ho * L.wo) * L.co +
                  4.0 * 64.0 * n * ((L.ho + 5) / 6) * ((L.wo + 5) / 6) * L.co);
      CK(launch_bnb_wino6_dy(c.f(L.dz), c.f(L.y), c.f(L.coef), n, L.ho, L.wo, L.co, c.f(L.dyp), c.f(L.vdw), s));
      w.vd_pre = c.f(L.vdw);
      ++unet::g_fused_bnb_sites;
    } else {
      Timer t(p, s, UNET_KC_ELEMWISE, 0, (g16 ? 2.0 : 4.0) * n * ((double)(L.ho + 4) * (L.wo + 4) + 2.0 * L.ho * L.wo) * L.co);
      // bf16 plans store dY(l > 0) in bf16: it only feeds bf16 GEMMs (inc.c0's
      // fp32 direct weight-gradient kernel reads dY(0))
      CK(launch_bnb_apply(c.f(L.dz), c.f(L.y), c.f(L.coef), n, L.ho, L.wo, L.co, c.f(L.dyp), 2, s, dy16,
                          p->prec == UNET_PREC_BF16, g16));
    }
    if (conc) {
      CK(hipEventRecord(p->ev_dy[l], s));
      CK(hipStreamWaitEvent(sw, p->ev_dy[l], 0));
    }
    {
      Timer t(p, sw, UNET_KC_CONV_WGRAD, conv_flops(L, n), 0, true, site_conv(l, 2));
      Timer tb(p, sw, UNET_KC_BOTTLENECK, conv_flops(L, n), 0, bottleneck_conv(l));
      CK(run_wgrad(cw, w));
    }
    CK(launch_permute_last2(c.f(L.dwp), L.co, 9, L.ci, P<float>(grd, L.gw), sw));
    // input gradient
    IgemmArgs a;
    a.a.s[0] = dy;
    a.a.s[0].oy = a.a.s[0].ox = 0;  // padded coordinates: rows index the input grid
    a.a.s[1] = a.a.s[0];
    a.a.Cg = a.a.c_split = L.co;
    a.a.taps_h = a.a.taps_w = 3;
    a.a.Hg = L.hi;
    a.a.Wg = L.wi;
    a.a.nimg = n;
    a.b = c.f(L.wd);
    a.M = n * L.hi * L.wi;
    a.N = L.ci;
    a.K = 9 * L.co;
    if (l % 2 == 1) {  // -> dz of layer l-1 (masked + BN-bwd stats)
      Conv& Q = p->L[l - 1];
      a.e.d[0] = Dst{c.f(Q.dz), Q.ho, Q.wo, Q.co, 0, 0, g16};
      a.e.yref = c.f(Q.y);
      a.e.yref_h16 = p->prec == UNET_PREC_BF16;
      a.e.bn_scale = c.f(Q.scale);
      a.e.bn_shift = c.f(Q.shift);
      a.e.bn_mean = c.f(Q.mean);
      a.e.bn_invstd = c.f(Q.invstd);
      a.e.bstats = c.d(Q.bstats);
      Timer t(p, s, UNET_KC_CONV_DGRAD, conv_flops(L, n), 0, true, site_conv(l, 1));
      Timer tb(p, s, UNET_KC_BOTTLENECK, conv_flops(L, n), 0, bottleneck_conv(l));
      CK(run_igemm(c, a));
    } else if (l <= 8) {  // -> gradient of the pooled tensor, then pool backward
      const int k = l / 2 - 1;
      Pool& pl = p->P[k];
      a.e.d[0] = Dst{c.f(pl.dp), pl.h / 2, pl.w / 2, pl.c, 0, 0, g16};
      {
        Timer t(p, s, UNET_KC_CONV_DGRAD, conv_flops(L, n), 0, true, site_conv(l, 1));
        Timer tb(p, s, UNET_KC_BOTTLENECK, conv_flops(L, n), 0, bottleneck_conv(l));
        CK(run_igemm(c, a));
      }
      Conv& Q = p->L[l - 1];  // encoder output feeding this pool (and a skip)
      const Skip& sk = p->S[3 - k];
      Timer t(p, s, UNET_KC_ELEMWISE, 0, (g16 ? 2.0 : 4.0) * n * (double)Q.ho * Q.wo * Q.co * 2.6);
      CK(launch_maxpool_bwd_fused(c.f(pl.dp), c.u8(pl.arg), c.f(sk.d), sk.oy, sk.ox, sk.th, sk.tw, c.f(Q.y),
                                  c.f(Q.scale), c.f(Q.shift), c.f(Q.mean), c.f(Q.invstd), n, Q.ho, Q.wo, Q.co,
                                  c.f(Q.dz), c.d(Q.bstats), s, p->prec == UNET_PREC_BF16, g16));
    } else {  // first conv of up block: split into skip grad and upsampled grad
      const int k = (l - 10) / 2;
      ConvT& T = p->T[k];
      Skip& sk = p->S[k];
      a.e.d[0] = Dst{c.f(sk.d), sk.th, sk.tw, sk.c, 0, 0, g16};
      a.e.d[1] = Dst{c.f(T.du), 2 * T.h, 2 * T.w, T.co, 0, 0, p->prec == UNET_PREC_BF16};
      a.e.n_split = sk.c;
      a.e.colsum1 = c.d(T.colsum);
      {
        Timer t(p, s, UNET_KC_CONV_DGRAD, conv_flops(L, n), 0, true, site_conv(l, 1));
        Timer tb(p, s, UNET_KC_BOTTLENECK, conv_flops(L, n), 0, bottleneck_conv(l));
        CK(run_igemm(c, a));
      }
      CK(launch_colsum(c.d(T.colsum), kStatGroups, T.co, P<float>(grd, T.gw + 1), s));
      if (conc) {  // du (the dgrad's second destination) feeds the convT weight grad
        CK(hipEventRecord(p->ev_du[k], s));
        CK(hipStreamWaitEvent(sw, p->ev_du[k], 0));
      }
      // ConvTranspose2d weight grad: C[ci][ab*Co+co] = sum_p z[p][ci] * du[2p+ab][co]
      Conv& Q = p->L[l - 1];
      {
        WgradArgs w;
        w.ga.s[0] = src_in(c, l - 1);
        w.ga.s[1] = w.ga.s[0];
        w.ga.Cg = w.ga.c_split = T.ci;
        w.ga.Hg = T.h;
        w.ga.Wg = T.w;
        w.ga.nimg = n;
        Src du;
        du.ptr = c.f(T.du);
        du.H = 2 * T.h;
        du.W = 2 * T.w;
        du.C = T.co;
        du.h16 = p->prec == UNET_PREC_BF16;
        w.gb.s[0] = du;
        w.gb.s[1] = du;
        w.gb.Cg = w.gb.c_split = T.co;
        w.gb.taps_h = w.gb.taps_w = 2;
        w.gb.stride = 2;
        w.gb.Hg = T.h;
        w.gb.Wg = T.w;
        w.gb.nimg = n;
        w.Mo = T.ci;
        w.No = 4 * T.co;
        w.P = n * T.h * T.w;
        w.out = c.f(T.dwp);
        Timer t(p, sw, UNET_KC_CONV_WGRAD, 2.0 * w.P * (double)w.Mo * w.No, 0, true, site_convT(k, 2));
        Timer tb(p, sw, UNET_KC_BOTTLENECK, 2.0 * w.P * (double)w.Mo * w.No, 0, k == 0);
        CK(run_wgrad(cw, w));
      }
      CK(launch_permute_last2(c.f(T.dwp), T.ci, 4, T.co, P<float>(grd, T.gw), sw));
      // ConvTranspose2d input grad -> dz of layer l-1
      IgemmArgs b;
      Src du;
      du.ptr = c.f(T.du);
      du.H = 2 * T.h;
      du.W = 2 * T.w;
      du.C = T.co;
      du.h16 = p->prec == UNET_PREC_BF16;
      b.a.s[0] = du;
      b.a.s[1] = du;
      b.a.Cg = b.a.c_split = T.co;
      b.a.taps_h = b.a.taps_w = 2;
      b.a.stride = 2;
      b.a.Hg = T.h;
      b.a.Wg = T.w;
      b.a.nimg = n;
      b.b = c.f(T.wd);
      b.M = n * T.h * T.w;
      b.N = T.ci;
      b.K = 4 * T.co;
      b.e.d[0] = Dst{c.f(Q.dz), Q.ho, Q.wo, Q.co, 0, 0, g16};
      b.e.yref = c.f(Q.y);
      b.e.yref_h16 = p->prec == UNET_PREC_BF16;
      b.e.bn_scale = c.f(Q.scale);
      b.e.bn_shift = c.f(Q.shift);
      b.e.bn_mean = c.f(Q.mean);
      b.e.bn_invstd = c.f(Q.invstd);
      b.e.bstats = c.d(Q.bstats);
      Timer t(p, s, UNET_KC_CONV_DGRAD, 2.0 * b.M * (double)b.N * b.K, 0, true, site_convT(k, 1));
      Timer tb(p, s, UNET_KC_BOTTLENECK, 2.0 * b.M * (double)b.N * b.K, 0, k == 0);
      CK(run_igemm(c, b));
    }
  }
  for (int sg = seg_b; sg < seg_e; ++sg) p->seg_on_side[sg] = conc;
  if (conc) {
    if (flags & UNET_BWD_DEFER_JOIN) {
      // data-parallel schedule: the caller's next segment (dgrad chain) does not
      // wait for this segment's weight gradients; its all-reduce waits on this
      // event (unet_plan_wait_segment) and unet_plan_join() ends the backward
      for (int sg = seg_b; sg < seg_e; ++sg) CK(hipEventRecord(p->ev_seg[sg], sw));
      p->side_pending = true;
    } else {
      CK(hipEventRecord(p->ev_join, sw));
      CK(hipStreamWaitEvent(s, p->ev_join, 0));
      p->side_pending = false;
    }
  }
  if (seg_e == 9) ++p->bwd_full;
  return 0;
}

}  // namespace

// =========================== C-ABI =======================================
extern "C" {

#ifndef UNET_SRC_HASH
#define UNET_SRC_HASH "unknown"
#endif
// the hash of the sources this library was built from (csrc/Makefile: sha256
// over $(SRCS), the internal headers and include/unet_hip.h, first 16 hex
// digits), so a run's record names the code it ran
#ifdef UNET_ABLATIONS
#define UNET_BUILD_KIND " ablations"
#else
#define UNET_BUILD_KIND ""
#endif
const char* unet_version(void) { return "unet_hip 0.4 gfx950 fp32/bf16/bf16x3-mfma src " UNET_SRC_HASH UNET_BUILD_KIND; }
const char* unet_last_error(void) { return g_err.c_str(); }

unet_plan* unet_plan_create(int n, int c_in, int h, int w, int n_classes) {
  return unet_plan_create_ex(n, c_in, h, w, n_classes, UNET_PREC_FP32);
}

int unet_plan_precision(const unet_plan* p) { return p ? p->prec : -EINVAL; }

unet_plan* unet_plan_create_ex(int n, int c_in, int h, int w, int n_classes, int prec) {
  // models/unet_model.py:66 takes any channel / class count; the bounds here
  // only keep the per-plan buffers (logits, head accumulators) within reason
  if (n < 1 || c_in < 1 || c_in > kMaxInChannels || n_classes < 1 || n_classes > kMaxClassCount) {
    set_err("unet_plan_create: need n>=1, 1<=c_in<=4096, 1<=n_classes<=4096");
    return nullptr;
  }
  if (prec != UNET_PREC_FP32 && prec != UNET_PREC_BF16 && prec != UNET_PREC_BF16X3) {
    set_err("unet_plan_create_ex: precision must be UNET_PREC_FP32, UNET_PREC_BF16 or UNET_PREC_BF16X3");
    return nullptr;
  }
  auto* p = new unet_plan();
  p->prec = prec;
  p->n = n;
  p->cin = c_in;
  p->h = h;
  p->w = w;
  p->ncls = n_classes;
  const int chans[5] = {64, 128, 256, 512, 1024};
  Alloc al;
  auto fsz = [&](long long elems) { return (size_t)elems * 4; };
  // encoder shapes (models/unet_model.py:106-110)
  int hh = h, ww = w;
  int cprev = c_in;
  for (int b = 0; b < 5; ++b) {
    if (b > 0) {
      Pool& pl = p->P[b - 1];
      pl.c = chans[b - 1];
      pl.h = hh;
      pl.w = ww;
      hh /= 2;
      ww /= 2;
    }
    for (int j = 0; j < 2; ++j) {
      Conv& L = p->L[2 * b + j];
      L.ci = j == 0 ? cprev : chans[b];
      L.co = chans[b];
      L.hi = hh;
      L.wi = ww;
      hh -= 2;
      ww -= 2;
      L.ho = hh;
      L.wo = ww;
      if (L.ho < 1 || L.wo < 1) {
        set_err("input too small for the valid U-Net");
        delete p;
        return nullptr;
      }
    }
    cprev = chans[b];
  }
  // decoder (models/unet_model.py:129-143)
  for (int k = 0; k < 4; ++k) {
    ConvT& T = p->T[k];
    const Conv& prev = p->L[9 + 2 * k];
    T.ci = prev.co;
    T.co = prev.co / 2;
    T.h = prev.ho;
    T.w = prev.wo;
    const Conv& enc = p->L[7 - 2 * k];
    Skip& sk = p->S[k];
    sk.c = enc.co;
    sk.th = 2 * T.h;
    sk.tw = 2 * T.w;
    if (enc.ho < sk.th || enc.wo < sk.tw) {
      set_err("skip connection smaller than the upsampled map (input size not supported by the valid U-Net)");
      delete p;
      return nullptr;
    }
    sk.oy = (enc.ho - sk.th) / 2;  // UNet._center_crop, models/unet_model.py:97-100
    sk.ox = (enc.wo - sk.tw) / 2;
    int hh2 = sk.th, ww2 = sk.tw;
    for (int j = 0; j < 2; ++j) {
      Conv& L = p->L[10 + 2 * k + j];
      L.ci = j == 0 ? sk.c + T.co : T.co;
      L.co = T.co;
      L.hi = hh2;
      L.wi = ww2;
      hh2 -= 2;
      ww2 -= 2;
      L.ho = hh2;
      L.wo = ww2;
      if (L.ho < 1 || L.wo < 1) {
        set_err("input too small for the valid U-Net");
        delete p;
        return nullptr;
      }
    }
  }
  p->ho = p->L[17].ho;
  p->wo = p->L[17].wo;
  // parameter table indices
  for (int l = 0; l < 18; ++l) {
    const int b = l / 2, j = l % 2;
    p->L[l].pw = block_pbase(b) + 7 * j;
    p->L[l].gw = block_gbase(b) + 4 * j;
  }
  for (int k = 0; k < 4; ++k) {
    p->T[k].pw = 70 + 16 * k;
    p->T[k].gw = 40 + 10 * k;
  }
  // ---- workspace ----
  // stat region first (zeroed per forward/backward)
  const size_t stat_start = al.top;
  for (int l = 0; l < 18; ++l) {
    Conv& L = p->L[l];
    L.stats = al.take(sizeof(double) * kStatGroups * L.co * 2);
    L.bstats = al.take(sizeof(double) * kStatGroups * L.co * 2);
  }
  for (int k = 0; k < 4; ++k)  // colsum groups + (tail) expanded bias table
    p->T[k].colsum = al.take(sizeof(double) * kStatGroups * p->T[k].co);
  p->head_acc = al.take(sizeof(double) * (64 * (size_t)n_classes + n_classes));  // head dW, db
  p->wce_acc = al.take(64);
  p->first_slabs = al.take(conv_first_wgrad_ws_bytes(c_in));
  p->stat_region.off = stat_start;
  p->stat_region.bytes = al.top - stat_start;
  const size_t dwp_start = al.top;
  for (int l = 1; l < 18; ++l) p->L[l].dwp = al.take(fsz(9LL * p->L[l].co * p->L[l].ci));
  for (int k = 0; k < 4; ++k) p->T[k].dwp = al.take(fsz(4LL * p->T[k].co * p->T[k].ci));
  p->dwp_region.off = dwp_start;
  p->dwp_region.bytes = al.top - dwp_start;
  {
    // split-K partials: the budget, or the largest 8-way split of any conv GEMM if smaller
    size_t mx = 0, wmax = (size_t)kStatGroups * 1024 * 2 * sizeof(double);
    for (int l = 1; l < 18; ++l) {
      const Conv& L = p->L[l];
      mx = std::max(mx, 8 * (size_t)n * L.ho * L.wo * L.co * sizeof(float));
      mx = std::max(mx, 8 * (size_t)n * L.hi * L.wi * L.ci * sizeof(float));
      wmax = std::max(wmax, (size_t)9 * L.co * L.ci * sizeof(float));
    }
    p->slab = al.take(std::min(mx, kSlabBudget));
    p->tune_scratch = al.take(wmax);
    if (prec == UNET_PREC_FP32) {
      // Winograd candidates: every 3x3 GEMM after inc.c0 (forward: Cg = ci,
      // N = co over the output grid; input gradient: Cg = co, N = ci over the
      // input grid); the autotuner decides per shape
      size_t wmx = 0;
      for (int l = 1; l < 18; ++l) {
        const Conv& L = p->L[l];
        wmx = std::max(wmx, wino_ws_bytes_grid(n, L.ho, L.wo, L.ci, L.co));
        wmx = std::max(wmx, wino_ws_bytes_grid(n, L.hi, L.wi, L.co, L.ci));
      }
      p->wino = al.take(wmx);
    }
  }
  {
    const size_t pack_start = al.top;
    for (int l = 1; l < 18; ++l) {
      Conv& L = p->L[l];
      L.wf = al.take(fsz(9LL * L.co * L.ci));
      L.wd = al.take(fsz(9LL * L.co * L.ci));
    }
    for (int k = 0; k < 4; ++k) {
      ConvT& T = p->T[k];
      T.wf = al.take(fsz(4LL * T.co * T.ci));
      T.wd = al.take(fsz(4LL * T.co * T.ci));
    }
    p->pack_region.off = pack_start;
    p->pack_region.bytes = al.top - pack_start;
    if (prec != UNET_PREC_FP32)  // hi plane (+ lo plane for split operands)
      p->pack16 = al.take(p->pack_region.bytes / 2 * (prec == UNET_PREC_BF16X3 ? 2 : 1));
  }
  // everything a forward touches (train or eval) ...
  p->fold0w = al.take(fsz(64LL * c_in * 9));
  for (int l = 0; l < 18; ++l) {
    Conv& L = p->L[l];
    const long long pix = (long long)n * L.ho * L.wo;
    L.y = al.take(fsz(pix * L.co));
    L.mean = al.take(fsz(L.co));
    L.invstd = al.take(fsz(L.co));
    L.scale = al.take(fsz(L.co));
    L.shift = al.take(fsz(L.co));
    L.coef = al.take(fsz(4LL * L.co));
    if (prec == UNET_PREC_BF16 &&
        ((unet::g_bf16_norm == 1 && l < 17) || (unet::g_bf16_norm == 2 && l <= 7 && l % 2 == 1)))
      L.a = al.take((size_t)pix * L.co * 2);  // head reads y17 itself
  }
  for (int k = 0; k < 4; ++k) {
    ConvT& T = p->T[k];
    T.u = al.take(fsz((long long)n * 4 * T.h * T.w * T.co));
  }
  for (int k = 0; k < 4; ++k) {
    Pool& pl = p->P[k];
    const long long pp = (long long)n * (pl.h / 2) * (pl.w / 2) * pl.c;
    pl.p = al.take(fsz(pp));
    pl.arg = al.take((size_t)pp);
  }
  p->fwd_ws_bytes = al.top;
  // ... then the gradient buffers only a backward writes (about 2/3 of a
  // train workspace): a forward that no backward follows -- eval, predict.py,
  // the tile farm, no_grad validation -- needs only the prefix
  for (int l = 0; l < 18; ++l) {
    Conv& L = p->L[l];
    const long long pix = (long long)n * L.ho * L.wo;
    L.dz = al.take(fsz(pix * L.co));
    if (l > 0)  // dY(0) is formed inside inc.c0's weight-gradient kernel
      L.dyp = al.take(fsz((long long)n * (L.ho + 4) * (L.wo + 4) * L.co));
  }
  for (int k = 0; k < 4; ++k) {
    ConvT& T = p->T[k];
    T.du = al.take(fsz((long long)n * 4 * T.h * T.w * T.co));
    Skip& sk = p->S[k];
    sk.d = al.take(fsz((long long)n * sk.th * sk.tw * sk.c));
  }
  for (int k = 0; k < 4; ++k) {
    Pool& pl = p->P[k];
    pl.dp = al.take(fsz((long long)n * (pl.h / 2) * (pl.w / 2) * pl.c));
  }
  if (prec == UNET_PREC_FP32) {
    // Winograd weight-gradient candidate (wgrad tile 71): its own scratch, as the
    // weight gradients run on the side stream next to the dgrad GEMMs
    size_t wmx = 0;
    for (int l = 1; l < 18; ++l) {
      const Conv& L = p->L[l];
      wmx = std::max(wmx, wino_ws_bytes_grid(n, L.ho, L.wo, L.ci, L.co));
    }
    p->wino_w = al.take(wmx);
    // k_bnb_wino6_dy's Vd planes (bnb_fuse on at plan creation): one buffer
    // per layer, so that the main stream's next layers never overwrite a plane
    // the side stream's point GEMMs still read (64/36 of the layer's dY: 4.2 GB
    // at 8 x 512^2)
    for (int l = 1; l < 18 && unet::g_bnb_fuse; ++l) {
      Conv& L = p->L[l];
      if (L.co % 64 == 0) L.vdw = al.take(bnb_wino6_vd_bytes(n, L.ho, L.wo, L.co));
    }
    for (int l = 1; l < 18 && unet::g_wgrad_fwd_u; ++l) {
      Conv& L = p->L[l];
      L.uws = al.take(wino_ws_bytes_grid(n, L.ho, L.wo, L.ci, L.co));
    }
  }
  // slab-mode weight gradients (ring tiles 26-33 with per_cu codes 11 / 12,
  // pixel-column tiles with codes 101-104): one [Mo][No] fp32 plane per pixel
  // split instead of fp32 atomics; sized for 2 per CU x the largest ring
  // channel block (128 x 9 x 64); a launch that needs more uses the atomics
  p->wslab = al.take((size_t)2 * num_cus() * 128 * 9 * 64 * sizeof(float));
  p->ws_bytes = al.top;
  return p;
}

void unet_plan_destroy(unet_plan* p) {
  if (!p) return;
  if (p->side) {
    (void)hipStreamSynchronize(p->side);
    for (auto ev : p->ev_dy) (void)hipEventDestroy(ev);
    for (auto ev : p->ev_du) (void)hipEventDestroy(ev);
    for (auto ev : p->ev_seg) (void)hipEventDestroy(ev);
    (void)hipEventDestroy(p->ev_join);
    (void)hipEventDestroy(p->ev_bwd0);
    (void)hipEventDestroy(p->ev_fwdu);
    (void)hipStreamDestroy(p->side);
  }
  for (auto& e : p->evs) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  delete p;
}

int unet_plan_out_hw(const unet_plan* p, int* oh, int* ow) {
  if (!p) return -EINVAL;
  if (oh) *oh = p->ho;
  if (ow) *ow = p->wo;
  return 0;
}
size_t unet_plan_workspace_bytes(const unet_plan* p) { return p ? p->ws_bytes : 0; }
size_t unet_plan_forward_workspace_bytes(const unet_plan* p) { return p ? p->fwd_ws_bytes : 0; }
int unet_plan_num_params(const unet_plan*) { return 136; }
int unet_plan_num_grads(const unet_plan*) { return 82; }
int unet_plan_num_segments(const unet_plan*) { return 9; }
int unet_plan_segment_grads(const unet_plan*, int seg, int* first, int* cnt) {
  // grad table: inc 0-7, down1..4 8-39, up1..4 40-79, outc 80-81
  int f, k;
  if (seg == 0) { f = 70; k = 12; }            // head + up4
  else if (seg <= 3) { f = 70 - 10 * seg; k = 10; }  // up3, up2, up1
  else if (seg <= 8) { f = 8 * (8 - seg); k = 8; }   // down4 .. inc
  else return -EINVAL;
  if (first) *first = f;
  if (cnt) *cnt = k;
  return 0;
}

int unet_plan_forward(unet_plan* p, void* const* prm, const float* x, float* logits, void* ws, int train,
                      unet_stream_t stream) {
  if (!p || !prm || !x || !logits || !ws) {
    set_err("unet_plan_forward: null argument");
    return -EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(ws) & 255) {
    set_err("unet_plan_forward: workspace must be 256-byte aligned");
    return -EINVAL;
  }
  return run_forward(p, prm, x, logits, reinterpret_cast<char*>(ws), train, reinterpret_cast<hipStream_t>(stream));
}

int unet_plan_backward(unet_plan* p, void* const* prm, void* const* grd, const float* x, const float* dlogits,
                       void* ws, int sb, int se, unet_stream_t stream) {
  if (!p || !prm || !grd || !x || !dlogits || !ws || sb < 0 || se > 9 || sb >= se) {
    set_err("unet_plan_backward: bad argument");
    return -EINVAL;
  }
  return run_backward(p, prm, grd, x, dlogits, reinterpret_cast<char*>(ws), sb, se,
                      reinterpret_cast<hipStream_t>(stream), 0);
}

int unet_plan_backward_ex(unet_plan* p, void* const* prm, void* const* grd, const float* x, const float* dlogits,
                          void* ws, int sb, int se, int flags, unet_stream_t stream) {
  if (!p || !prm || !grd || !x || !dlogits || !ws || sb < 0 || se > 9 || sb >= se || (flags & ~UNET_BWD_DEFER_JOIN)) {
    set_err("unet_plan_backward_ex: bad argument");
    return -EINVAL;
  }
  return run_backward(p, prm, grd, x, dlogits, reinterpret_cast<char*>(ws), sb, se,
                      reinterpret_cast<hipStream_t>(stream), flags);
}

size_t unet_plan_input_grad_scratch_bytes(const unet_plan* p) {
  return p ? (size_t)p->n * p->L[0].ho * p->L[0].wo * p->L[0].co * sizeof(float) : 0;
}

// The gradient of the network input (the reference's x.grad when x requires
// grad, models/unet_model.py:105 under autograd).  The training backward never
// forms it -- inc.c0's BatchNorm backward is fused into its weight gradient and
// dY(0) is not materialised -- so after the backward segment holding inc.c0
// this call materialises dY(0) = k0 dz0 + k1 (y0 - mean) + k2 into `scratch`
// (fp32, unet_plan_input_grad_scratch_bytes) and correlates it with inc.c0's
// weights into dx (NCHW fp32, overwritten).
int unet_plan_input_grad(unet_plan* p, void* const* prm, float* dx, void* ws, void* scratch, unet_stream_t stream) {
  if (!p || !prm || !dx || !ws || !scratch) {
    set_err("unet_plan_input_grad: bad argument");
    return -EINVAL;
  }
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  Ctx c{p, reinterpret_cast<char*>(ws), s};
  const Conv& L = p->L[0];
  const int g16 = p->prec == UNET_PREC_BF16;
  float* dy0 = reinterpret_cast<float*>(scratch);
  CK(launch_bnb_apply(c.f(L.dz), c.f(L.y), c.f(L.coef), p->n, L.ho, L.wo, L.co, dy0, 0, s, 0,
                      p->prec == UNET_PREC_BF16, g16));
  CK(launch_conv_first_dgrad(dy0, p->n, p->cin, p->h, p->w, P<float>(prm, L.pw), dx, s));
  return 0;
}

int unet_plan_wait_segment(unet_plan* p, int seg, unet_stream_t stream) {
  if (!p || seg < 0 || seg >= 9) {
    set_err("unet_plan_wait_segment: bad argument");
    return -EINVAL;
  }
  // the segment ran without the side stream (tuning pass, timing, serial mode):
  // its weight gradients are on the caller's stream already
  if (!p->seg_on_side[seg] || !p->side) return 0;
  CK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), p->ev_seg[seg], 0));
  return 0;
}

int unet_plan_join(unet_plan* p, unet_stream_t stream) {
  if (!p) {
    set_err("unet_plan_join: null plan");
    return -EINVAL;
  }
  if (!p->side || !p->side_pending) return 0;
  CK(hipEventRecord(p->ev_join, p->side));
  CK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), p->ev_join, 0));
  p->side_pending = false;
  return 0;
}

size_t unet_tuning_report(char* buf, size_t len) {
  std::string r;
  {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    for (const auto& kv : g_tune_log) r += kv.second + "\n";
  }
  if (buf && len > 0) {
    const size_t k = std::min(len - 1, r.size());
    memcpy(buf, r.data(), k);
    buf[k] = 0;
  }
  return r.size() + 1;
}

long long unet_nondeterministic_sites(int reset) {
  return reset ? g_nondet_sites.exchange(0) : g_nondet_sites.load();
}

long long unet_fused_bnb_sites(int reset) {
  return reset ? unet::g_fused_bnb_sites.exchange(0) : unet::g_fused_bnb_sites.load();
}
long long unet_slab_fallbacks(int reset) {
  return reset ? g_slab_fallbacks.exchange(0) : g_slab_fallbacks.load();
}

int unet_tuning_reset(void) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  g_tuned.clear();
  g_tune_log.clear();
  return 0;
}

int unet_tuning_save(const char* path) {
  if (!path) return -EINVAL;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  FILE* f = fopen(path, "w");
  if (!f) return -errno;
  for (const auto& kv : g_tuned) fprintf(f, "%s\t%d\t%d\n", kv.first.c_str(), kv.second.tile, kv.second.split);
  fclose(f);
  return (int)g_tuned.size();
}

int unet_tuning_load(const char* path) {
  if (!path) return -EINVAL;
  std::lock_guard<std::mutex> lk(g_tune_mu);
  return tune_db_read(path, true);
}

int unet_plan_set_timing(unet_plan* p, int enable) {
  if (!p) return -EINVAL;
  p->timing = enable != 0;
  return 0;
}

int unet_plan_timing(const unet_plan* pc, double* ms, double* fl, double* by, int* cnt) {
  auto* p = const_cast<unet_plan*>(pc);
  if (!p) return -EINVAL;
  int rc = 0;
  for (auto& e : p->evs) {
    float t = 0;
    if (hipEventSynchronize(e.b) != hipSuccess || hipEventElapsedTime(&t, e.a, e.b) != hipSuccess) {
      set_err("unet_plan_timing: event query failed");
      rc = -EIO;
    } else {
      p->t_ms[e.cls] += t;
      p->t_fl[e.cls] += e.flops;
      p->t_by[e.cls] += e.bytes;
      p->t_xf[e.cls] += e.xflops;
      p->t_n[e.cls] += 1;
      if (e.site >= 0) {
        auto& v = p->sites[e.site];
        v[0] += t;
        v[1] += e.flops;
        v[2] += e.xflops;
      }
    }
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  p->evs.clear();
  for (int i = 0; i < UNET_KC_COUNT; ++i) {
    if (ms) ms[i] = p->t_ms[i];
    if (fl) fl[i] = p->t_fl[i];
    if (by) by[i] = p->t_by[i];
    if (cnt) cnt[i] = p->t_n[i];
    p->t_xf_last[i] = p->t_xf[i];
    p->t_ms[i] = p->t_fl[i] = p->t_by[i] = p->t_xf[i] = 0;
    p->t_n[i] = 0;
  }
  p->sites_last.swap(p->sites);
  p->sites.clear();
  return rc;
}

size_t unet_plan_timing_sites(const unet_plan* p, char* buf, size_t cap) {
  if (!p) return 0;
  std::string out;
  for (const auto& kv : p->sites_last) {
    char line[160];
    snprintf(line, sizeof line, "%s\t%.4f\t%.6e\t%.6e\n", site_name(kv.first).c_str(), kv.second[0], kv.second[1],
             kv.second[2]);
    out += line;
  }
  if (buf && cap) {
    const size_t m = out.size() < cap - 1 ? out.size() : cap - 1;
    memcpy(buf, out.data(), m);
    buf[m] = 0;
  }
  return out.size() + 1;
}

int unet_plan_timing_mfma_flops(const unet_plan* p, double* xfl) {
  if (!p || !xfl) return -EINVAL;
  for (int i = 0; i < UNET_KC_COUNT; ++i) xfl[i] = p->t_xf_last[i];
  return 0;
}

}  // extern "C"
