// Per-op C-ABI entry points (include/unet_hip.h): single reference ops on
// caller buffers, built from the same kernels the network plan schedules.
// They exist for op-level parity tests and for callers that compose their own
// graph; the training path uses unet_plan_*.
#include <algorithm>
#include <cerrno>
#include <string>

#include "../../include/unet_hip.h"
#include "unet_internal.h"

using namespace unet;

namespace unet {
extern int g_tune_igemm, g_tune_wgrad, g_autotune, g_force_split, g_force_tile, g_concurrent, g_wino_max,
    g_wino_dgrad_max, g_wino_wgrad_max, g_bf16_norm, g_bn_fold, g_wino4_fwd_min_cg, g_wino4_fwd_small_cg,
    g_maxpool_vec8, g_wgrad_fwd_u;
hipError_t launch_fill(float* p, size_t n, float v, hipStream_t s);
hipError_t launch_pair_sum(const double* st, int g, int c, float* out, hipStream_t s);
}  // namespace unet

namespace {
thread_local std::string g_op_err;
inline size_t al256(size_t b) { return (b + 255) / 256 * 256; }
// unet_set_tuning("op_precision", UNET_PREC_*): GEMM arithmetic of the per-op
// entry points (the plan has its own, unet_plan_create_ex)
int g_op_prec = UNET_PREC_FP32;
// unet_set_tuning("op_a16", 1): with op_precision UNET_PREC_BF16 the 3x3
// conv entry points store their A operand in bf16 first, as a bf16 plan does
// (raw conv outputs and padded dY are bf16 there): the conv forward rounds x to
// bf16 before its BN+ReLU transform, the input gradient stores the padded dY
// bf16.  Lets op-level tests and tools run the plan's exact GEMM configuration.
int g_op_a16 = 0;

// bf16 / split per-op GEMMs: round the packed fp32 B (n elements) into
// `scratch` (4n bytes: hi plane, then the lo plane of split operands) and point
// the GEMM at it
hipError_t op_b_to_bf16(IgemmArgs& a, size_t n, void* scratch, hipStream_t s) {
  if (g_op_prec == UNET_PREC_FP32) return hipSuccess;
  uint16_t* bh = reinterpret_cast<uint16_t*>(scratch);
  uint16_t* bl = g_op_prec == UNET_PREC_BF16X3 ? bh + n : nullptr;
  hipError_t e = launch_f2bf(a.b, bh, n, s, bl);
  a.bh = bh;
  a.bl = bl;
  a.b = nullptr;
  return e;
}
}  // namespace

namespace {
// dz = dy where the (ReLU) output y > 0, else 0 (torch's threshold_backward on
// the output, nn.ReLU(inplace=True) of models/unet_model.py:13, 17)
__global__ void k_relu_mask(const float* __restrict__ dy, const float* __restrict__ y, long long n4,
                            float* __restrict__ dz) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const float4 g = reinterpret_cast<const float4*>(dy)[i], v = reinterpret_cast<const float4*>(y)[i];
    reinterpret_cast<float4*>(dz)[i] =
        make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f, v.w > 0.f ? g.w : 0.f);
  }
}

// eval-mode BatchNorm statistics: the running ones (invstd as k_bn_eval_prepare)
__global__ void k_bn_eval_stats(int C, const float* rm, const float* rv, float eps, float* mean, float* invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
}
}  // namespace

#define OPCK(x)                                                           \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) return e_ == hipErrorInvalidValue ? -EINVAL : -EIO; \
  } while (0)

extern "C" {

// transformed weights of the fused Winograd tiles (72, 73, 75, 76) for forced
// per-op GEMMs (tests: unet_set_tuning("igemm_variant", t)); the built-in
// choice of the per-op entry points never takes a Winograd tile
static size_t op_wino_bytes(int ci, int co) { return al256(sizeof(float) * 36 * (size_t)ci * co); }
static void op_set_wino(IgemmArgs& a, void* ws, size_t ws_bytes, int ci, int co) {
  a.wino_ws = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + ws_bytes - op_wino_bytes(ci, co));
  a.wino_ws_bytes = op_wino_bytes(ci, co);
}

size_t unet_conv_ws_bytes(int n, int h, int w, int ci, int co) {
  const size_t wb = al256(sizeof(float) * 9 * (size_t)ci * co);
  const size_t pad = al256(sizeof(float) * (size_t)n * (h + 2) * (w + 2) * co);  // (h-2+4)
  const size_t misc = al256(sizeof(float) * 4 * co) + al256(sizeof(double) * kStatGroups * 2 * co);
  const size_t x16 = al256(sizeof(uint16_t) * (size_t)n * h * w * ci);  // op_a16: bf16 copy of x
  return 2 * wb + pad + misc + x16 + op_wino_bytes(ci, co);
}

int unet_conv3x3_fwd(const float* x, int n, int h, int w, int ci, const float* wt, const float* bias, int co,
                     const float* xs, const float* xb, float* y, void* ws, unet_stream_t st) {
  if (ci % 16 || co % 64 || h < 3 || w < 3) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  float* wf = reinterpret_cast<float*>(ws);
  OPCK(launch_pack_conv(wt, co, ci, 3, 3, wf, nullptr, s));
  IgemmArgs a;
  Src x0;
  x0.ptr = x;
  x0.H = h;
  x0.W = w;
  x0.C = ci;
  x0.scale = xs;
  x0.shift = xb;
  if (g_op_prec == UNET_PREC_BF16 && g_op_a16) {
    const size_t wb = al256(sizeof(float) * 9 * (size_t)ci * co);
    const size_t off = 2 * wb + al256(sizeof(float) * (size_t)n * (h + 2) * (w + 2) * co) +
                       al256(sizeof(float) * 4 * co) + al256(sizeof(double) * kStatGroups * 2 * co);
    uint16_t* x16 = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(ws) + off);
    OPCK(launch_f2bf(x, x16, (size_t)n * h * w * ci, s));
    x0.ptr = reinterpret_cast<const float*>(x16);
    x0.h16 = 1;
  }
  a.a.s[0] = a.a.s[1] = x0;
  a.a.Cg = a.a.c_split = ci;
  a.a.taps_h = a.a.taps_w = 3;
  a.a.Hg = h - 2;
  a.a.Wg = w - 2;
  a.a.nimg = n;
  a.b = wf;
  a.M = n * (h - 2) * (w - 2);
  a.N = co;
  a.K = 9 * ci;
  a.e.bias = bias;
  a.e.d[0] = Dst{y, h - 2, w - 2, co, 0, 0};
  op_set_wino(a, ws, unet_conv_ws_bytes(n, h, w, ci, co), ci, co);
  OPCK(op_b_to_bf16(a, 9 * (size_t)ci * co, reinterpret_cast<char*>(ws) + al256(sizeof(float) * 9 * (size_t)ci * co),
                    s));
  OPCK(launch_igemm(a, s));
  return 0;
}

int unet_conv3x3_dgrad(const float* dy, int n, int h, int w, int ci, const float* wt, int co, float* dx, void* ws,
                       unet_stream_t st) {
  if (ci % 64 || co % 16 || h < 3 || w < 3) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  const size_t wb = al256(sizeof(float) * 9 * (size_t)ci * co);
  float* wf = reinterpret_cast<float*>(p);
  float* wd = reinterpret_cast<float*>(p + wb);
  float* dyp = reinterpret_cast<float*>(p + 2 * wb);
  float* coef = reinterpret_cast<float*>(p + 2 * wb + al256(sizeof(float) * (size_t)n * (h + 2) * (w + 2) * co));
  OPCK(launch_pack_conv(wt, co, ci, 3, 3, wf, wd, s));
  // zero-bordered copy of dy: dYpad = 1*dy + 0*(y-0) + 0
  OPCK(launch_fill(coef, co, 1.f, s));
  OPCK(launch_fill(coef + co, 3 * (size_t)co, 0.f, s));
  const int dy16 = g_op_prec == UNET_PREC_BF16 && g_op_a16;
  OPCK(launch_bnb_apply(dy, dy, coef, n, h - 2, w - 2, co, dyp, 2, s, dy16, 0));
  IgemmArgs a;
  Src d;
  d.ptr = dyp;
  d.h16 = dy16;
  d.H = h + 2;
  d.W = w + 2;
  d.C = co;
  a.a.s[0] = a.a.s[1] = d;
  a.a.Cg = a.a.c_split = co;
  a.a.taps_h = a.a.taps_w = 3;
  a.a.Hg = h;
  a.a.Wg = w;
  a.a.nimg = n;
  a.b = wd;
  a.M = n * h * w;
  a.N = ci;
  a.K = 9 * co;
  a.e.d[0] = Dst{dx, h, w, ci, 0, 0};
  op_set_wino(a, ws, unet_conv_ws_bytes(n, h, w, ci, co), ci, co);
  OPCK(op_b_to_bf16(a, 9 * (size_t)ci * co, wf, s));
  OPCK(launch_igemm(a, s));
  return 0;
}

int unet_conv3x3_wgrad(const float* x, const float* dy, int n, int h, int w, int ci, int co, float* dw, float* db,
                       void* ws, unet_stream_t st) {
  if (ci % 64 || co % 64 || h < 3 || w < 3) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  const size_t wb = al256(sizeof(float) * 9 * (size_t)ci * co);
  float* dwp = reinterpret_cast<float*>(p);
  double* st2 = reinterpret_cast<double*>(p + 2 * wb + al256(sizeof(float) * (size_t)n * (h + 2) * (w + 2) * co) +
                                          al256(sizeof(float) * 4 * co));
  OPCK(hipMemsetAsync(dwp, 0, sizeof(float) * 9 * (size_t)ci * co, s));
  WgradArgs a;
  Src d;
  d.ptr = dy;
  d.H = h - 2;
  d.W = w - 2;
  d.C = co;
  a.ga.s[0] = a.ga.s[1] = d;
  a.ga.Cg = a.ga.c_split = co;
  a.ga.Hg = h - 2;
  a.ga.Wg = w - 2;
  a.ga.nimg = n;
  Src xs;
  xs.ptr = x;
  xs.H = h;
  xs.W = w;
  xs.C = ci;
  a.gb.s[0] = a.gb.s[1] = xs;
  a.gb.Cg = a.gb.c_split = ci;
  a.gb.taps_h = a.gb.taps_w = 3;
  a.gb.Hg = h - 2;
  a.gb.Wg = w - 2;
  a.gb.nimg = n;
  a.Mo = co;
  a.No = 9 * ci;
  a.P = n * (h - 2) * (w - 2);
  a.out = dwp;
  a.bf16 = g_op_prec != UNET_PREC_FP32;
  a.split = g_op_prec == UNET_PREC_BF16X3;
  if (g_op_prec == UNET_PREC_BF16 && g_op_a16) {  // bf16-stored dY and X, as in a bf16 plan
    // dY as the plan keeps it: a zero-bordered padded bf16 copy (border 2),
    // written by the BN-backward apply with identity coefficients
    uint16_t* dy16 = reinterpret_cast<uint16_t*>(p + 2 * wb);
    float* coef = reinterpret_cast<float*>(p + 2 * wb + al256(sizeof(float) * (size_t)n * (h + 2) * (w + 2) * co));
    uint16_t* x16 = reinterpret_cast<uint16_t*>(p + 2 * wb + al256(sizeof(float) * (size_t)n * (h + 2) * (w + 2) * co) +
                                                al256(sizeof(float) * 4 * co) +
                                                al256(sizeof(double) * kStatGroups * 2 * co));
    OPCK(launch_fill(coef, co, 1.f, s));
    OPCK(launch_fill(coef + co, 3 * (size_t)co, 0.f, s));
    OPCK(launch_bnb_apply(dy, dy, coef, n, h - 2, w - 2, co, reinterpret_cast<float*>(dy16), 2, s, 1, 0));
    OPCK(launch_f2bf(x, x16, (size_t)n * h * w * ci, s));
    a.ga.s[0].ptr = a.ga.s[1].ptr = reinterpret_cast<const float*>(dy16);
    a.ga.s[0].H = a.ga.s[1].H = h + 2;
    a.ga.s[0].W = a.ga.s[1].W = w + 2;
    a.ga.s[0].oy = a.ga.s[1].oy = a.ga.s[0].ox = a.ga.s[1].ox = 2;
    a.ga.s[0].h16 = a.ga.s[1].h16 = 1;
    a.gb.s[0].ptr = a.gb.s[1].ptr = reinterpret_cast<const float*>(x16);
    a.gb.s[0].h16 = a.gb.s[1].h16 = 1;
  }
  OPCK(launch_wgrad(a, s));
  OPCK(launch_permute_last2(dwp, co, 9, ci, dw, s));
  if (db) {
    OPCK(hipMemsetAsync(st2, 0, sizeof(double) * kStatGroups * 2 * co, s));
    OPCK(launch_channel_stats(dy, (size_t)n * (h - 2) * (w - 2), co, st2, s));
    OPCK(launch_pair_sum(st2, kStatGroups, co, db, s));
  }
  return 0;
}

int unet_convT2_fwd(const float* x, int n, int h, int w, int ci, const float* wt, const float* bias, int co, float* y,
                    void* ws, unet_stream_t st) {
  if (ci % 16 || co % 16) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  float* wf = reinterpret_cast<float*>(p);
  float* wd = reinterpret_cast<float*>(p + al256(sizeof(float) * 4 * (size_t)ci * co));
  OPCK(launch_pack_convT(wt, ci, co, wf, wd, s));
  IgemmArgs a;
  Src x0;
  x0.ptr = x;
  x0.H = h;
  x0.W = w;
  x0.C = ci;
  a.a.s[0] = a.a.s[1] = x0;
  a.a.Cg = a.a.c_split = ci;
  a.a.Hg = h;
  a.a.Wg = w;
  a.a.nimg = n;
  a.b = wf;
  a.M = n * h * w;
  a.N = 4 * co;
  a.K = ci;
  a.e.bias = bias;
  a.e.shuffle_co = co;
  a.e.d[0] = Dst{y, 2 * h, 2 * w, co, 0, 0};
  OPCK(op_b_to_bf16(a, 4 * (size_t)ci * co, p + 2 * al256(sizeof(float) * 4 * (size_t)ci * co), s));
  OPCK(launch_igemm(a, s));
  return 0;
}

int unet_convT2_bwd(const float* x, const float* dy, int n, int h, int w, int ci, const float* wt, int co, float* dx,
                    float* dw, float* db, void* ws, unet_stream_t st) {
  if (ci % 64 || co % 64) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  const size_t wb = al256(sizeof(float) * 4 * (size_t)ci * co);
  float* wf = reinterpret_cast<float*>(p);
  float* wd = reinterpret_cast<float*>(p + wb);
  float* dwp = reinterpret_cast<float*>(p + 2 * wb);
  double* st2 = reinterpret_cast<double*>(p + 3 * wb);
  OPCK(launch_pack_convT(wt, ci, co, wf, wd, s));
  Src d;
  d.ptr = dy;
  d.H = 2 * h;
  d.W = 2 * w;
  d.C = co;
  IgemmArgs a;
  a.a.s[0] = a.a.s[1] = d;
  a.a.Cg = a.a.c_split = co;
  a.a.taps_h = a.a.taps_w = 2;
  a.a.stride = 2;
  a.a.Hg = h;
  a.a.Wg = w;
  a.a.nimg = n;
  a.b = wd;
  a.M = n * h * w;
  a.N = ci;
  a.K = 4 * co;
  a.e.d[0] = Dst{dx, h, w, ci, 0, 0};
  OPCK(op_b_to_bf16(a, 4 * (size_t)ci * co, wf, s));  // wf (4n bytes) is not read again
  OPCK(launch_igemm(a, s));
  OPCK(hipMemsetAsync(dwp, 0, sizeof(float) * 4 * (size_t)ci * co, s));
  WgradArgs g;
  Src x0;
  x0.ptr = x;
  x0.H = h;
  x0.W = w;
  x0.C = ci;
  g.ga.s[0] = g.ga.s[1] = x0;
  g.ga.Cg = g.ga.c_split = ci;
  g.ga.Hg = h;
  g.ga.Wg = w;
  g.ga.nimg = n;
  g.gb.s[0] = g.gb.s[1] = d;
  g.gb.Cg = g.gb.c_split = co;
  g.gb.taps_h = g.gb.taps_w = 2;
  g.gb.stride = 2;
  g.gb.Hg = h;
  g.gb.Wg = w;
  g.gb.nimg = n;
  g.Mo = ci;
  g.No = 4 * co;
  g.P = n * h * w;
  g.out = dwp;
  g.bf16 = g_op_prec != UNET_PREC_FP32;
  g.split = g_op_prec == UNET_PREC_BF16X3;
  OPCK(launch_wgrad(g, s));
  OPCK(launch_permute_last2(dwp, ci, 4, co, dw, s));
  OPCK(hipMemsetAsync(st2, 0, sizeof(double) * kStatGroups * 2 * co, s));
  OPCK(launch_channel_stats(dy, (size_t)n * 4 * h * w, co, st2, s));
  OPCK(launch_pair_sum(st2, kStatGroups, co, db, s));
  return 0;
}

int unet_maxpool2_fwd(const float* x, int n, int h, int w, int c, float* y, uint8_t* arg, unet_stream_t st) {
  Src s0;
  s0.ptr = x;
  s0.H = h;
  s0.W = w;
  s0.C = c;
  OPCK(launch_maxpool_fwd(s0, n, h, w, y, arg, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_maxpool2_bwd(const float* dy, const uint8_t* arg, int n, int h, int w, int c, float* dx, unet_stream_t st) {
  OPCK(launch_maxpool_bwd_fused(dy, arg, nullptr, 0, 0, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, n, h, w, c,
                                dx, nullptr, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

size_t unet_bn_ws_bytes(int c) { return al256(sizeof(double) * kStatGroups * 2 * c) + 8 * al256(sizeof(float) * c); }

int unet_bn_train_fwd(const float* x, int n, int h, int w, int c, const float* gamma, const float* beta, float* rm,
                      float* rv, float* y, float* save_mean, float* save_invstd, void* ws, unet_stream_t st) {
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  double* stats = reinterpret_cast<double*>(p);
  float* scale = reinterpret_cast<float*>(p + al256(sizeof(double) * kStatGroups * 2 * c));
  float* shift = scale + al256(sizeof(float) * c) / 4;
  const size_t pix = (size_t)n * h * w;
  OPCK(hipMemsetAsync(stats, 0, sizeof(double) * kStatGroups * 2 * c, s));
  OPCK(launch_channel_stats(x, pix, c, stats, s));
  OPCK(launch_bn_finalize(stats, c, (double)pix, gamma, beta, rm, rv, nullptr, save_mean, save_invstd, scale, shift,
                          0.1f, 1e-5f, s));
  OPCK(launch_affine_relu(x, pix, c, scale, shift, 0, y, s));
  return 0;
}

int unet_bn_train_bwd(const float* x, const float* dy, int n, int h, int w, int c, const float* gamma,
                      const float* mean, const float* invstd, float* dx, float* dgamma, float* dbeta, void* ws,
                      unet_stream_t st) {
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  double* stats = reinterpret_cast<double*>(p);
  float* coef = reinterpret_cast<float*>(p + al256(sizeof(double) * kStatGroups * 2 * c));
  const size_t pix = (size_t)n * h * w;
  OPCK(hipMemsetAsync(stats, 0, sizeof(double) * kStatGroups * 2 * c, s));
  OPCK(launch_bn_bwd_stats(dy, x, mean, invstd, pix, c, stats, s));
  OPCK(launch_bnb_finalize(stats, c, (double)pix, gamma, mean, invstd, dgamma, dbeta, nullptr, coef, s));
  OPCK(launch_bnb_apply(dy, x, coef, n, h, w, c, dx, 0, s));
  return 0;
}

size_t unet_bn_relu_ws_bytes(int n, int h, int w, int c) {
  return unet_bn_ws_bytes(c) + al256(sizeof(float) * (size_t)n * h * w * c);
}

int unet_bn_relu_fwd(const float* x, int n, int h, int w, int c, const float* gamma, const float* beta, float* rm,
                     float* rv, int64_t* nbt, float momentum, float eps, int training, int relu, float* y,
                     float* save_mean, float* save_invstd, void* ws, unet_stream_t st) {
  if (!x || !y || !gamma || !beta || !save_mean || !save_invstd || c < 4 || c % 4 || 256 % (c / 4) || n < 1) return -EINVAL;
  if (!training && (!rm || !rv)) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  double* stats = reinterpret_cast<double*>(p);
  float* scale = reinterpret_cast<float*>(p + al256(sizeof(double) * kStatGroups * 2 * c));
  float* shift = scale + al256(sizeof(float) * c) / 4;
  const size_t pix = (size_t)n * h * w;
  if (training) {
    OPCK(hipMemsetAsync(stats, 0, sizeof(double) * kStatGroups * 2 * c, s));
    OPCK(launch_channel_stats(x, pix, c, stats, s));
    OPCK(launch_bn_finalize(stats, c, (double)pix, gamma, beta, rm, rv, nbt, save_mean, save_invstd, scale, shift,
                            momentum, eps, s));
  } else {
    OPCK(launch_bn_eval_prepare(c, gamma, beta, rm, rv, scale, shift, eps, s));
    hipLaunchKernelGGL(k_bn_eval_stats, dim3((c + 255) / 256), dim3(256), 0, s, c, rm, rv, eps, save_mean,
                       save_invstd);
    OPCK(hipGetLastError());
  }
  OPCK(launch_affine_relu(x, pix, c, scale, shift, relu, y, s));
  return 0;
}

int unet_bn_relu_bwd(const float* x, const float* y, const float* dy, int n, int h, int w, int c, const float* gamma,
                     const float* save_mean, const float* save_invstd, int training, int relu, float* dx,
                     float* dgamma, float* dbeta, void* ws, unet_stream_t st) {
  if (!x || !dy || !dx || !gamma || c < 4 || c % 4 || 256 % (c / 4) || n < 1 || (relu && !y)) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  double* stats = reinterpret_cast<double*>(p);
  float* coef = reinterpret_cast<float*>(p + al256(sizeof(double) * kStatGroups * 2 * c));
  float* dz = reinterpret_cast<float*>(p + unet_bn_ws_bytes(c));
  const size_t pix = (size_t)n * h * w;
  const float* g = dy;
  if (relu) {
    const long long n4 = (long long)(pix * c / 4);
    hipLaunchKernelGGL(k_relu_mask, dim3((unsigned)std::min<long long>((n4 + 255) / 256, 8192)), dim3(256), 0, s, dy,
                       y, n4, dz);
    OPCK(hipGetLastError());
    g = dz;
  }
  OPCK(hipMemsetAsync(stats, 0, sizeof(double) * kStatGroups * 2 * c, s));
  OPCK(launch_bn_bwd_stats(g, x, save_mean, save_invstd, pix, c, stats, s));
  OPCK(launch_bnb_finalize(stats, c, (double)pix, gamma, save_mean, save_invstd, dgamma, dbeta, nullptr, coef, s,
                           training ? 0 : 1));
  OPCK(launch_bnb_apply(g, x, coef, n, h, w, c, dx, 0, s));
  return 0;
}

size_t unet_conv_first_ws_bytes(int n, int ci, int h, int w) {
  (void)n; (void)h; (void)w;
  return conv_first_wgrad_ws_bytes(ci) + al256(sizeof(double) * kStatGroups * 2 * 64);
}

int unet_conv_first_fwd(const float* x, int n, int ci, int h, int w, const float* wt, const float* bias, float* y,
                        unet_stream_t st) {
  if (!x || !wt || !bias || !y || n < 1 || ci < 1 || h < 3 || w < 3) return -EINVAL;
  OPCK(launch_conv_first_fwd(x, n, ci, h, w, wt, bias, 64, y, nullptr, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_conv_first_bwd(const float* x, const float* dy, int n, int ci, int h, int w, const float* wt, float* dx,
                        float* dw, float* db, void* ws, unet_stream_t st) {
  if (!x || !dy || !wt || !dw || !db || !ws || n < 1 || ci < 1 || h < 3 || w < 3) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  char* p = reinterpret_cast<char*>(ws);
  float* slabs = reinterpret_cast<float*>(p);
  double* st2 = reinterpret_cast<double*>(p + conv_first_wgrad_ws_bytes(ci));
  Src d;
  d.ptr = dy;
  d.H = h - 2;
  d.W = w - 2;
  d.C = 64;
  OPCK(launch_conv_first_wgrad(x, n, ci, h, w, d, 64, dw, slabs, s));
  OPCK(hipMemsetAsync(st2, 0, sizeof(double) * kStatGroups * 2 * 64, s));
  OPCK(launch_channel_stats(dy, (size_t)n * (h - 2) * (w - 2), 64, st2, s));
  OPCK(launch_pair_sum(st2, kStatGroups, 64, db, s));
  if (dx) OPCK(launch_conv_first_dgrad(dy, n, ci, h, w, wt, dx, s));
  return 0;
}

size_t unet_conv1x1_ws_bytes(int k) { return al256(sizeof(double) * ((size_t)k * 64 + k)); }

int unet_conv1x1_fwd(const float* x, int n, int h, int w, int c, const float* wt, const float* bias, int k,
                     float* logits, unet_stream_t st) {
  if (!x || !wt || !bias || !logits || c != 64 || k < 1 || n < 1) return -EINVAL;
  Src s0;
  s0.ptr = x;
  s0.H = h;
  s0.W = w;
  s0.C = 64;
  OPCK(launch_head_fwd(s0, n, h, w, 64, wt, bias, k, logits, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_conv1x1_bwd(const float* x, const float* dl, int n, int h, int w, int c, const float* wt, int k, float* dx,
                     float* dw, float* db, void* ws, unet_stream_t st) {
  if (!x || !dl || !wt || !dw || !db || !ws || c != 64 || k < 1 || n < 1) return -EINVAL;
  OPCK(launch_head_bwd_plain(x, dl, n, h, w, wt, k, dx, dw, db, reinterpret_cast<double*>(ws),
                             reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_wce_fwd_bwd(const float* logits, const int64_t* t, const float* wm, int n, int k, int h, int w,
                     const int64_t* ts, const int64_t* wsd, float* loss, float* dl, float gscale, void* ws,
                     unet_stream_t st) {
  if (!ts || !wsd || k < 1) return -EINVAL;
  OPCK(launch_wce(logits, t, wm, n, k, h, w, ts, wsd, loss, dl, gscale, reinterpret_cast<double*>(ws),
                  reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_scale_by_device_scalar(float* x, size_t n, const float* g, unet_stream_t st) {
  OPCK(launch_scale_by_dev(x, x, n, g, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_scale_by_device_scalar_out(const float* x, float* y, size_t n, const float* g, unet_stream_t st) {
  OPCK(launch_scale_by_dev(x, y, n, g, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_sgd_momentum(float* p, const float* g, float* buf, size_t n, float lr, float mom, float gscale, int first,
                      unet_stream_t st) {
  OPCK(launch_sgd(p, g, buf, n, lr, mom, gscale, first, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_iou_counts(const uint8_t* a, const uint8_t* b, size_t n, unsigned long long* out, unet_stream_t st) {
  OPCK(launch_iou(a, b, n, out, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_set_tuning(const char* key, int value) {
  if (!key) return -EINVAL;
  const std::string k(key);
  if (k == "igemm_variant") g_tune_igemm = value;
  else if (k == "wgrad_variant") g_tune_wgrad = value;
  else if (k == "autotune") g_autotune = value;
  else if (k == "force_split") g_force_split = value;
  else if (k == "force_tile") g_force_tile = value;
  else if (k == "concurrent") g_concurrent = value;
  else if (k == "wino_max") g_wino_max = value;
  else if (k == "bf16_norm") g_bf16_norm = value;
  else if (k == "bn_fold") g_bn_fold = value != 0;
  else if (k == "wino_dgrad_max") g_wino_dgrad_max = value;
  else if (k == "wino_wgrad_max") g_wino_wgrad_max = value;
  else if (k == "wino4_fwd_min_cg") g_wino4_fwd_min_cg = value;
  else if (k == "wino4_fwd_small_cg") g_wino4_fwd_small_cg = value;
  else if (k == "op_a16") g_op_a16 = value != 0;
  else if (k == "maxpool_vec8") g_maxpool_vec8 = value;
  else if (k == "bnb_fuse") g_bnb_fuse = value;
  else if (k == "wgrad_early_u") g_wgrad_early_u = value;
  else if (k == "wgrad_fwd_u") g_wgrad_fwd_u = value;
  else if (k == "deterministic") g_deterministic = value != 0;  // 0: bf16 plans pool with the 4-channel kernel (A/B tests)
  else if (k == "op_precision") {
    if (value != UNET_PREC_FP32 && value != UNET_PREC_BF16 && value != UNET_PREC_BF16X3) return -EINVAL;
    g_op_prec = value;
  } else return -EINVAL;
  return 0;
}

int unet_tile_gather(const float* image, int c, int h, int w, int tile_in, int tile_out, int top, int left, int nx,
                     int first, int stride, int ntiles, float* tiles, unet_stream_t st) {
  if (!image || !tiles) return -EINVAL;
  OPCK(launch_tile_gather(image, c, h, w, tile_in, tile_out, top, left, nx, first, stride, ntiles, tiles,
                          reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_tile_scatter(const float* tile_logits, int k, int tile_out, int nx, int first, int stride, int ntiles, int h,
                      int w, float* logits, uint8_t* mask, unet_stream_t st) {
  if (!tile_logits) return -EINVAL;
  OPCK(launch_tile_scatter(tile_logits, k, tile_out, nx, first, stride, ntiles, h, w, logits, mask,
                           reinterpret_cast<hipStream_t>(st)));
  return 0;
}

size_t unet_instance_masks_ws_bytes(int n, int h, int w) {
  return n > 0 && h > 0 && w > 0 ? instance_masks_ws_bytes(n, h, w) : 0;
}

int unet_instance_masks(const uint8_t* mask, int n, int h, int w, int min_size, uint16_t* labels, void* ws,
                        unet_stream_t st) {
  if (!mask || !labels || !ws) return -EINVAL;
  OPCK(launch_instance_masks(mask, n, h, w, min_size, labels, ws, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

size_t unet_rand_index_ws_bytes(int h, int w) { return h > 0 && w > 0 ? rand_index_ws_bytes(h, w) : 0; }

int unet_rand_index(const uint16_t* gt, const uint16_t* pred, int h, int w, double* out, void* ws,
                    unet_stream_t st) {
  if (!gt || !pred || !out || !ws) return -EINVAL;
  OPCK(launch_rand_index(gt, pred, h, w, out, ws, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

size_t unet_weight_map_ws_bytes(int n) { return n > 0 ? weight_map_ws_bytes(n) : 0; }

int unet_weight_map(const uint16_t* labels, int n, int h, int w, double w0, double sigma, float* weights,
                    double* weights64, void* ws, unet_stream_t st) {
  if (!labels || !weights || !ws || (reinterpret_cast<uintptr_t>(ws) & 7)) return -EINVAL;
  OPCK(launch_weight_map(labels, n, h, w, w0, sigma, weights, weights64, ws, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

size_t unet_elastic_ws_bytes(int n, int h, int w) { return n > 0 && h > 0 && w > 0 ? elastic_ws_bytes(n, h, w) : 0; }

int unet_elastic_deform(const uint8_t* image, const uint16_t* labels, int n, int h, int w, const double* noise,
                        double alpha, double sigma, float* x_out, uint8_t* target_out, uint8_t* image_out, void* ws,
                        unet_stream_t st) {
  if (!image || !labels || !noise || !x_out || !target_out || !ws || (reinterpret_cast<uintptr_t>(ws) & 7)) return -EINVAL;
  OPCK(launch_elastic(image, labels, n, h, w, noise, alpha, sigma, x_out, target_out, image_out, ws,
                      reinterpret_cast<hipStream_t>(st)));
  return 0;
}

int unet_mask_from_logits(const float* logits, uint8_t* mask, int n, int h, int w, unet_stream_t st) {
  OPCK(launch_mask(logits, mask, n, h, w, reinterpret_cast<hipStream_t>(st)));
  return 0;
}

}  // extern "C"
