// Winograd F(2x2, 3x3) for the fp32 3x3 valid convolutions (forward and input
// gradient) of the deep, wide layers -- igemm tile id 70, an autotuner
// candidate beside the direct implicit GEMMs (the plan times both on the live
// operands and keeps the faster per GEMM shape).
//
// Direct: 9 * Ci MACs per output element.  Winograd F(2x2, 3x3) (Lavin & Gray,
// "Fast Algorithms for Convolutional Neural Networks", 2016): per 2x2 output
// tile and channel pair, 16 MACs instead of 36 -- 2.25x fewer MFMA flops:
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A,  d = 4x4 input patch, g = 3x3 kernel
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
//   G   = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1]
//   A^T = [1 1 1 0; 0 1 -1 -1]
// Four launches (the input / output transforms are HBM-bound, the GEMMs run on
// the f32 MFMA through the igemm machinery):
//  1. k_wino_w:   V[p][n][c]  = (G g_{n,c} G^T)_p from the packed B [N][9][Cg];
//  2. k_wino_in:  U[p][t][c]  = (B^T d_{t,c} B)_p over the gather (two sources,
//                 crop origin, the producer's BatchNorm+ReLU applied on load);
//  3. 16 GEMMs:   M[p] (T x N) = U[p] (T x Cg) . V[p]^T;
//  4. k_wino_out: the 2x2 outputs A^T M_t A + bias and the full epilogue
//                 (linear destinations: BN statistics, ReLU mask + BN-backward
//                 statistics, concat split + column sums).
// Transform arithmetic is exact in the +-1, 1/2 coefficients; the fp32
// rounding of the 16-term products differs from the direct sum's, at the same
// order (tests/test_gpu_ops.py, tests/test_gpu_model.py force tile 70).
#include <algorithm>
#include <cstdlib>

#include "gemm_common.h"
#include "ring_common.h"

namespace unet {

// ---- 1. weight transform: V[p][n][c] from B[n][tap][c] (tap = 3 ky + kx) ----
__global__ void k_wino_w(const float* __restrict__ b, int N, int Cg, float* __restrict__ v) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)N * Cg) return;
  const int n = (int)(i / Cg), c = (int)(i - (long long)n * Cg);
  float g[3][3];
#pragma unroll
  for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = b[((size_t)n * 9 + t) * Cg + c];
  float tg[4][3];  // G g
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    tg[0][k] = g[0][k];
    tg[1][k] = 0.5f * (g[0][k] + g[1][k] + g[2][k]);
    tg[2][k] = 0.5f * (g[0][k] - g[1][k] + g[2][k]);
    tg[3][k] = g[2][k];
  }
  const size_t plane = (size_t)N * Cg, o = (size_t)n * Cg + c;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v[(r * 4 + 0) * plane + o] = tg[r][0];
    v[(r * 4 + 1) * plane + o] = 0.5f * (tg[r][0] + tg[r][1] + tg[r][2]);
    v[(r * 4 + 2) * plane + o] = 0.5f * (tg[r][0] - tg[r][1] + tg[r][2]);
    v[(r * 4 + 3) * plane + o] = tg[r][2];
  }
}

// ---- 2. input transform --------------------------------------------------
// Thread = (tile, 4 channels).  The gather's output grid is (Hg, Wg); its 3x3
// valid window needs input rows / columns 0 .. Hg+1 / Wg+1; tile (ty, tx)
// reads rows 2ty .. 2ty+3 (the last row of an odd grid's last tile only feeds
// the dropped output row: read as 0).
__global__ __launch_bounds__(256) void k_wino_in(Gather g, int Th, int Tw, long long T, float* __restrict__ u) {
  const int C4 = g.Cg / 4;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= T * C4) return;
  const long long t = i / C4;
  const int c = (int)(i - t * C4) * 4;
  const int tx = (int)(t % Tw);
  const long long r = t / Tw;
  const int ty = (int)(r % Th), n = (int)(r / Th);
  const bool second = c >= g.c_split;
  const Src s = pick_src(g, second);
  const int cl = second ? c - g.c_split : c;
  float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
  if (s.scale) {
    sc = ld4(s.scale + cl);
    sh = ld4(s.shift + cl);
  }
  float4 d[4][4];
#pragma unroll
  for (int yy = 0; yy < 4; ++yy)
#pragma unroll
    for (int xx = 0; xx < 4; ++xx) {
      const int y = 2 * ty + yy, x = 2 * tx + xx;
      const bool in = y < g.Hg + 2 && x < g.Wg + 2;  // unconditional load, clamped address
      float4 v = ld4(s.ptr + ((size_t)(n * s.H + (in ? y : 0) + s.oy) * s.W + (in ? x : 0) + s.ox) * s.C + cl);
      if (s.scale) v = affine_relu4(v, sc, sh);
      d[yy][xx] = in ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  // B^T d (rows), then (.) B (columns)
  float4 e[4][4];
#pragma unroll
  for (int xx = 0; xx < 4; ++xx) {
    e[0][xx] = d[0][xx] - d[2][xx];
    e[1][xx] = d[1][xx] + d[2][xx];
    e[2][xx] = d[2][xx] - d[1][xx];
    e[3][xx] = d[1][xx] - d[3][xx];
  }
  const size_t plane = (size_t)T * g.Cg, o = (size_t)t * g.Cg + c;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    st4(u + (a * 4 + 0) * plane + o, e[a][0] - e[a][2]);
    st4(u + (a * 4 + 1) * plane + o, e[a][1] + e[a][2]);
    st4(u + (a * 4 + 2) * plane + o, e[a][2] - e[a][1]);
    st4(u + (a * 4 + 3) * plane + o, e[a][1] - e[a][3]);
  }
}

// ---- 4. output transform + epilogue ---------------------------------------
// Block = (up to 64 four-channel groups) x (tile lanes); each thread walks
// tiles with a grid stride, keeps its channels' statistics in registers, and
// the block adds them with one fp64 atomic per column into a spread group.
__global__ __launch_bounds__(256) void k_wino_out(const float* __restrict__ m, long long T, int Th, int Tw, int N,
                                                  Gather g, Epilogue e) {
  const int C4 = N / 4;
  const int cgs = C4 < 64 ? C4 : 64;      // channel groups per block
  const int lanes = 256 / cgs;             // tile lanes per block
  const int cg = blockIdx.y * cgs + (int)(threadIdx.x % cgs);
  const int tl = threadIdx.x / cgs;
  const bool active = cg < C4 && tl < lanes;
  const int col = cg * 4;
  const bool second = col >= e.n_split;
  float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
  const int dC = second ? e.d[1].C : e.d[0].C;
  const int dcol = second ? col - e.n_split : col;
  const bool bwd_mask = e.yref != nullptr && !second;
  float4 bias = make_float4(0.f, 0.f, 0.f, 0.f), bsc, bsh, bmu, bis;
  if (active && e.bias) bias = ld4(e.bias + col);
  if (active && bwd_mask) {
    bsc = ld4(e.bn_scale + col); bsh = ld4(e.bn_shift + col);
    bmu = ld4(e.bn_mean + col); bis = ld4(e.bn_invstd + col);
  }
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  const size_t plane = (size_t)T * N;
  if (active) {
    for (long long t = blockIdx.x * (long long)lanes + tl; t < T; t += (long long)gridDim.x * lanes) {
      float4 q[16];
#pragma unroll
      for (int p = 0; p < 16; ++p) q[p] = ld4(m + p * plane + (size_t)t * N + col);
      // A^T q (rows of the 4x4), then (.) A (columns)
      float4 w[2][4];
#pragma unroll
      for (int xx = 0; xx < 4; ++xx) {
        w[0][xx] = q[xx] + q[4 + xx] + q[8 + xx];
        w[1][xx] = q[4 + xx] - q[8 + xx] - q[12 + xx];
      }
      const int tx = (int)(t % Tw);
      const long long r = t / Tw;
      const int ty = (int)(r % Th), n = (int)(r / Th);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int y = 2 * ty + a, x = 2 * tx + bb;
          if (y >= g.Hg || x >= g.Wg) continue;
          float4 v = bb == 0 ? w[a][0] + w[a][1] + w[a][2] : w[a][1] - w[a][2] - w[a][3];
          v = v + bias;
          const size_t idx = ((size_t)(n * g.Hg + y) * g.Wg + x) * dC + dcol;
          if (bwd_mask) {
            const float4 yv = ld4(e.yref + idx);
            v.x = fmaf(yv.x, bsc.x, bsh.x) > 0.f ? v.x : 0.f;
            v.y = fmaf(yv.y, bsc.y, bsh.y) > 0.f ? v.y : 0.f;
            v.z = fmaf(yv.z, bsc.z, bsh.z) > 0.f ? v.z : 0.f;
            v.w = fmaf(yv.w, bsc.w, bsh.w) > 0.f ? v.w : 0.f;
            s1 = s1 + v;
            s2.x += v.x * ((yv.x - bmu.x) * bis.x);
            s2.y += v.y * ((yv.y - bmu.y) * bis.y);
            s2.z += v.z * ((yv.z - bmu.z) * bis.z);
            s2.w += v.w * ((yv.w - bmu.w) * bis.w);
          } else if (e.stats) {
            s1 = s1 + v;
            s2 = s2 + v * v;
          } else if (second && e.colsum1) {
            s1 = s1 + v;
          }
          if (e.relu) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          st4(dptr + idx, v);
        }
    }
  }
  const bool want = e.stats || e.yref || e.colsum1;
  if (!want) return;
  __shared__ float red[256][8];
  red[threadIdx.x][0] = s1.x; red[threadIdx.x][1] = s1.y; red[threadIdx.x][2] = s1.z; red[threadIdx.x][3] = s1.w;
  red[threadIdx.x][4] = s2.x; red[threadIdx.x][5] = s2.y; red[threadIdx.x][6] = s2.z; red[threadIdx.x][7] = s2.w;
  __syncthreads();
  if (threadIdx.x < cgs && cg < C4) {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int l = 0; l < lanes; ++l)
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += red[l * cgs + threadIdx.x][k];
    const int grp = blockIdx.x % kStatGroups;
    const int nsplit = e.n_split < N ? e.n_split : N;
    if (col < nsplit) {
      double* st = e.yref ? e.bstats : e.stats;
      if (st)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          atomicAdd(st + ((size_t)grp * nsplit + col + k) * 2 + 0, (double)a[k]);
          atomicAdd(st + ((size_t)grp * nsplit + col + k) * 2 + 1, (double)a[4 + k]);
        }
    } else if (e.colsum1) {
      const int n2 = N - nsplit;
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(e.colsum1 + (size_t)grp * n2 + (col - nsplit + k), (double)a[k]);
    }
  }
}

// ---------------------------------------------------------------------------
// F(4x4, 3x3) (tile 71): 6x6 input patches, 36 points, 4x4 outputs -- 4x fewer
// MACs than direct and 2.25 points per output pixel instead of 4 (less
// transform traffic).  Interpolation points 0, 1, -1, 2, -1/2, inf (Toom-Cook,
// G carrying the Lagrange denominators).  Against Lavin & Gray's 0, +-1, +-2,
// inf the fp32 output error is ~1.6x smaller (NumPy emulation, post-ReLU
// inputs, 64-256 channels: 6.3e-7 vs 1.06e-6 ... 1.9e-6 vs 3.1e-6 rel-RMS):
// that rounding reaches every gradient through the BatchNorm statistics of the
// forward GEMMs.
//   B^T = [1 3/2 -2 -3/2 1 0; 0 -1 -5/2 -1/2 1 0; 0 1 1/2 -5/2 1 0;
//          0 -1/2 -1 1/2 1 0; 0 2 -1 -2 1 0; 0 1 3/2 -2 -3/2 1]
//   G   = [1 0 0; -1/3 -1/3 -1/3; 1/3 -1/3 1/3; 1/15 2/15 4/15;
//          -16/15 8/15 -4/15; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -1/2 0; 0 1 1 4 1/4 0; 0 1 -1 8 -1/8 1]
// (every coefficient but 1/3 and 1/15 is exact in fp32).  One channel per
// thread (36 values in registers), coalesced across channels.
// ---------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ void bt6v(const T (&d)[6], T (&r)[6]) {
  r[0] = d[0] + 1.5f * (d[1] - d[3]) - 2.f * d[2] + d[4];
  r[1] = d[4] - d[1] - 2.5f * d[2] - 0.5f * d[3];
  r[2] = d[1] + 0.5f * d[2] - 2.5f * d[3] + d[4];
  r[3] = 0.5f * (d[3] - d[1]) - d[2] + d[4];
  r[4] = 2.f * (d[1] - d[3]) - d[2] + d[4];
  r[5] = d[1] + 1.5f * (d[2] - d[4]) - 2.f * d[3] + d[5];
}
__device__ __forceinline__ void bt6(const float (&d)[6], float (&r)[6]) { bt6v(d, r); }
__device__ __forceinline__ void g6(const float (&g)[3], float (&r)[6]) {
  r[0] = g[0];
  r[1] = -(g[0] + g[1] + g[2]) * (1.f / 3.f);
  r[2] = (g[0] - g[1] + g[2]) * (1.f / 3.f);
  r[3] = (g[0] + 2.f * g[1] + 4.f * g[2]) * (1.f / 15.f);
  r[4] = (8.f * g[1] - 16.f * g[0] - 4.f * g[2]) * (1.f / 15.f);
  r[5] = g[2];
}
__device__ __forceinline__ void at4(const float (&m)[6], float (&o)[4]) {
  o[0] = m[0] + m[1] + m[2] + m[3] + m[4];
  o[1] = m[1] - m[2] + 2.f * m[3] - 0.5f * m[4];
  o[2] = m[1] + m[2] + 4.f * m[3] + 0.25f * m[4];
  o[3] = m[1] - m[2] + 8.f * m[3] - 0.125f * m[4] + m[5];
}

__global__ void k_wino4_w(const float* __restrict__ b, int N, int Cg, float* __restrict__ v) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)N * Cg) return;
  const int n = (int)(i / Cg), c = (int)(i - (long long)n * Cg);
  float tg[6][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float col[3] = {b[((size_t)n * 9 + 0 + k) * Cg + c], b[((size_t)n * 9 + 3 + k) * Cg + c],
                    b[((size_t)n * 9 + 6 + k) * Cg + c]};
    float r[6];
    g6(col, r);
#pragma unroll
    for (int a = 0; a < 6; ++a) tg[a][k] = r[a];
  }
  const size_t plane = (size_t)N * Cg, o = (size_t)n * Cg + c;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float r[6];
    g6(tg[a], r);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) v[(a * 6 + bb) * plane + o] = r[bb];
  }
}

// Thread = (tile, V consecutive channels): V-wide loads and stores (V = 4 when
// the channel count allows), 32-bit byte offsets from the source base.
template <int V>
__global__ __launch_bounds__(256) void k_wino4_in(Gather g, int Th, int Tw, long long T, float* __restrict__ u) {
  typedef float vec __attribute__((ext_vector_type(V)));
  const int CV = g.Cg / V;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= T * CV) return;
  const long long t = i / CV;
  const int c = (int)(i - t * CV) * V;
  const int tx = (int)(t % Tw);
  const long long r = t / Tw;
  const int ty = (int)(r % Th), n = (int)(r / Th);
  const bool second = c >= g.c_split;
  const Src s = pick_src(g, second);
  const int cl = second ? c - g.c_split : c;
  vec sc, sh;
  if (s.scale) {
    sc = *reinterpret_cast<const vec*>(s.scale + cl);
    sh = *reinterpret_cast<const vec*>(s.shift + cl);
  }
  const int vr = min(6, g.Hg + 2 - 4 * ty), vc = min(6, g.Wg + 2 - 4 * tx);  // in-window rows / columns
  const char* base = reinterpret_cast<const char*>(s.ptr) +
                     ((size_t)(n * s.H + 4 * ty + s.oy) * s.W + 4 * tx + s.ox) * s.C * 4 + (size_t)cl * 4;
  const unsigned rs = (unsigned)s.W * s.C * 4u, cs = (unsigned)s.C * 4u;
  // all 36 loads first (unconditional, clamped address), then the BatchNorm
  // branch once: a load consumed inside a branch region is waited for at the
  // region's boundary, which serialised the 36 loads
  vec raw[6][6];
#pragma unroll
  for (int xx = 0; xx < 6; ++xx)
#pragma unroll
    for (int yy = 0; yy < 6; ++yy) {
      const bool in = yy < vr && xx < vc;
      raw[yy][xx] = *reinterpret_cast<const vec*>(base + (in ? yy * rs + xx * cs : 0u));
    }
  if (s.scale) {
#pragma unroll
    for (int xx = 0; xx < 6; ++xx)
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int k = 0; k < V; ++k) raw[yy][xx][k] = fmaxf(fmaf(raw[yy][xx][k], sc[k], sh[k]), 0.f);
  }
  vec e[6][6];  // B^T d (rows), per column
#pragma unroll
  for (int xx = 0; xx < 6; ++xx) {
    vec d[6];
#pragma unroll
    for (int yy = 0; yy < 6; ++yy) d[yy] = (yy < vr && xx < vc) ? raw[yy][xx] : (vec)0.f;
    vec r[6];
    bt6v(d, r);
#pragma unroll
    for (int a = 0; a < 6; ++a) e[a][xx] = r[a];
  }
  const size_t plane = (size_t)T * g.Cg, o = (size_t)t * g.Cg + c;
  char* ub = reinterpret_cast<char*>(u + o);
  const unsigned pbytes = (unsigned)(plane * 4);
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    vec rr[6];
    bt6v(e[a], rr);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) *reinterpret_cast<vec*>(ub + (unsigned)(a * 6 + bb) * pbytes) = rr[bb];
  }
}

static int wino4_in_vec() {
  static const int v = getenv("UNET_WINO_IN_VEC") ? atoi(getenv("UNET_WINO_IN_VEC")) : 2;
  return v;
}

static void launch_wino4_in(const Gather& g, int Th, int Tw, long long T, float* U, hipStream_t s) {
  int V = wino4_in_vec();
  while (V > 1 && (g.Cg % V || g.c_split % V)) V >>= 1;
  const long long n = T * (g.Cg / V);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (V == 4) hipLaunchKernelGGL(k_wino4_in<4>, grid, dim3(256), 0, s, g, Th, Tw, T, U);
  else if (V == 2) hipLaunchKernelGGL(k_wino4_in<2>, grid, dim3(256), 0, s, g, Th, Tw, T, U);
  else hipLaunchKernelGGL(k_wino4_in<1>, grid, dim3(256), 0, s, g, Th, Tw, T, U);
}

// The 4x4 ReLU-mask operands of output tile (n, ty, tx), column dcol, issued as
// 16 independent loads (coordinates past the grid clamped to its last row /
// column: those outputs are not stored).
__device__ __forceinline__ void wf_yref4(const float* __restrict__ yref, const Gather& g, int n, int ty, int tx, int dC,
                                         int dcol, float (&yv)[4][4]) {
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int y = min(4 * ty + a, g.Hg - 1);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const int x = min(4 * tx + bb, g.Wg - 1);
      yv[a][bb] = yref[((size_t)(n * g.Hg + y) * g.Wg + x) * dC + dcol];
    }
  }
}

// Block = 64 channels x 4 tile lanes; grid-stride over tiles.
__global__ __launch_bounds__(256) void k_wino4_out(const float* __restrict__ m, long long T, int Th, int Tw, int N,
                                                   Gather g, Epilogue e) {
  const int col = blockIdx.y * 64 + (int)(threadIdx.x & 63);
  const int tl = threadIdx.x >> 6;
  const bool active = col < N;
  const bool second = col >= e.n_split;
  float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
  const int dC = second ? e.d[1].C : e.d[0].C;
  const int dcol = second ? col - e.n_split : col;
  const bool bwd_mask = e.yref != nullptr && !second;
  float bias = 0.f, bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
  if (active && e.bias) bias = e.bias[col];
  if (active && bwd_mask) { bsc = e.bn_scale[col]; bsh = e.bn_shift[col]; bmu = e.bn_mean[col]; bis = e.bn_invstd[col]; }
  float s1 = 0.f, s2 = 0.f;
  const size_t plane = (size_t)T * N;
  if (active) {
    const unsigned pb = (unsigned)(plane * 4);  // bytes per point plane (36 planes < 4 GB: wino_applies)
    for (long long t = blockIdx.x * 4ll + tl; t < T; t += (long long)gridDim.x * 4) {
      const char* mb = reinterpret_cast<const char*>(m + (size_t)t * N + col);
      float w[4][6];  // A^T q (rows), per column
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) {
        float q[6];
#pragma unroll
        for (int yy = 0; yy < 6; ++yy)
          q[yy] = *reinterpret_cast<const float*>(mb + (unsigned)(yy * 6 + xx) * pb);  // 32-bit offsets
        float o[4];
        at4(q, o);
#pragma unroll
        for (int a = 0; a < 4; ++a) w[a][xx] = o[a];
      }
      const int tx = (int)(t % Tw);
      const long long r = t / Tw;
      const int ty = (int)(r % Th), n = (int)(r / Th);
      // ReLU-mask operands of the 16 outputs loaded before the first store
      // (wf_yref4: the stores may alias yref for the compiler)
      float yv[4][4];
      if (bwd_mask) wf_yref4(e.yref, g, n, ty, tx, dC, dcol, yv);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        float o[4];
        at4(w[a], o);
        const int y = 4 * ty + a;
        if (y >= g.Hg) continue;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const int x = 4 * tx + bb;
          if (x >= g.Wg) continue;
          float v = o[bb] + bias;
          const size_t idx = ((size_t)(n * g.Hg + y) * g.Wg + x) * dC + dcol;
          if (bwd_mask) {
            v = fmaf(yv[a][bb], bsc, bsh) > 0.f ? v : 0.f;
            s1 += v;
            s2 += v * ((yv[a][bb] - bmu) * bis);
          } else if (e.stats) {
            s1 += v;
            s2 += v * v;
          } else if (second && e.colsum1) {
            s1 += v;
          }
          if (e.relu) v = fmaxf(v, 0.f);
        dptr[idx] = v;
        }
      }
    }
  }
  const bool want = e.stats || e.yref || e.colsum1;
  if (!want) return;
  __shared__ float red[2][256];
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (threadIdx.x < 64 && active) {
    const float a = red[0][threadIdx.x] + red[0][threadIdx.x + 64] + red[0][threadIdx.x + 128] + red[0][threadIdx.x + 192];
    const float b2 = red[1][threadIdx.x] + red[1][threadIdx.x + 64] + red[1][threadIdx.x + 128] + red[1][threadIdx.x + 192];
    const int grp = blockIdx.x % kStatGroups;
    const int nsplit = e.n_split < N ? e.n_split : N;
    if (col < nsplit) {
      double* st = e.yref ? e.bstats : e.stats;
      if (st) {
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 0, (double)a);
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 1, (double)b2);
      }
    } else if (e.colsum1) {
      atomicAdd(e.colsum1 + (size_t)grp * (N - nsplit) + (col - nsplit), (double)a);
    }
  }
}

// ---------------------------------------------------------------------------
// F(6x6, 3x3) (tile 74): 8x8 input patches, 64 points, 6x6 outputs -- 1.78
// point products per output instead of 2.25 (F4) and 1.78 U / M values per
// pixel instead of 2.25, at ~2.5x F4's fp32 rounding (interpolation points
// 0, +-1, +-2, +-1/2, inf; Lavin & Gray 2016; the matrices were checked
// against direct correlation to 3e-14 in fp64 before use).
// ---------------------------------------------------------------------------
template <int R, int C>
__device__ __forceinline__ void mat_apply(const float (&m)[R][C], const float (&in)[C], float (&out)[R]) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float acc = 0.f;
    bool first = true;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float k = m[r][c];
      if (k == 0.f) continue;  // compile-time after unrolling: zero terms vanish
      const float t = k == 1.f ? in[c] : k == -1.f ? -in[c] : k * in[c];
      acc = first ? t : acc + t;
      first = false;
    }
    out[r] = acc;
  }
}

__device__ __forceinline__ void bt8(const float (&d)[8], float (&r)[8]) {
  constexpr float B[8][8] = {{1, 0, -5.25f, 0, 5.25f, 0, -1, 0},
                             {0, 1, 1, -4.25f, -4.25f, 1, 1, 0},
                             {0, -1, 1, 4.25f, -4.25f, -1, 1, 0},
                             {0, 0.5f, 0.25f, -2.5f, -1.25f, 2, 1, 0},
                             {0, -0.5f, 0.25f, 2.5f, -1.25f, -2, 1, 0},
                             {0, 2, 4, -2.5f, -5, 0.5f, 1, 0},
                             {0, -2, 4, 2.5f, -5, -0.5f, 1, 0},
                             {0, -1, 0, 5.25f, 0, -5.25f, 0, 1}};
  mat_apply(B, d, r);
}
__device__ __forceinline__ void g8(const float (&g)[3], float (&r)[8]) {
  constexpr float G[8][3] = {{1, 0, 0},
                             {-2.f / 9, -2.f / 9, -2.f / 9},
                             {-2.f / 9, 2.f / 9, -2.f / 9},
                             {1.f / 90, 1.f / 45, 2.f / 45},
                             {1.f / 90, -1.f / 45, 2.f / 45},
                             {32.f / 45, 16.f / 45, 8.f / 45},
                             {32.f / 45, -16.f / 45, 8.f / 45},
                             {0, 0, 1}};
  mat_apply(G, g, r);
}
__device__ __forceinline__ void at6(const float (&m)[8], float (&o)[6]) {
  constexpr float A[6][8] = {{1, 1, 1, 1, 1, 1, 1, 0},
                             {0, 1, -1, 2, -2, 0.5f, -0.5f, 0},
                             {0, 1, 1, 4, 4, 0.25f, 0.25f, 0},
                             {0, 1, -1, 8, -8, 0.125f, -0.125f, 0},
                             {0, 1, 1, 16, 16, 0.0625f, 0.0625f, 0},
                             {0, 1, -1, 32, -32, 0.03125f, -0.03125f, 1}};
  mat_apply(A, m, o);
}

__global__ void k_wino6_w(const float* __restrict__ b, int N, int Cg, float* __restrict__ v) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)N * Cg) return;
  const int n = (int)(i / Cg), c = (int)(i - (long long)n * Cg);
  float tg[8][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float col[3] = {b[((size_t)n * 9 + 0 + k) * Cg + c], b[((size_t)n * 9 + 3 + k) * Cg + c],
                    b[((size_t)n * 9 + 6 + k) * Cg + c]};
    float r[8];
    g8(col, r);
#pragma unroll
    for (int a = 0; a < 8; ++a) tg[a][k] = r[a];
  }
  const size_t plane = (size_t)N * Cg, o = (size_t)n * Cg + c;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    float r[8];
    g8(tg[a], r);
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) v[(a * 8 + bb) * plane + o] = r[bb];
  }
}

// Thread = (tile, V channels); 8x8 patch with clamped unconditional loads
template <int V>
__global__ __launch_bounds__(256) void k_wino6_in(Gather g, int Th, int Tw, long long T, float* __restrict__ u) {
  typedef float vec __attribute__((ext_vector_type(V)));
  const int CV = g.Cg / V;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= T * CV) return;
  const long long t = i / CV;
  const int c = (int)(i - t * CV) * V;
  const int tx = (int)(t % Tw);
  const long long r = t / Tw;
  const int ty = (int)(r % Th), n = (int)(r / Th);
  const bool second = c >= g.c_split;
  const Src s = pick_src(g, second);
  const int cl = second ? c - g.c_split : c;
  // producer BatchNorm + ReLU as max(fma(x, sc, sh), lo), identity without one:
  // branch-free, so the 64 loads are not serialised at branch boundaries
  vec sc = (vec)1.f, sh = (vec)0.f;
  float lo = -INFINITY;
  if (s.scale) {
    sc = *reinterpret_cast<const vec*>(s.scale + cl);
    sh = *reinterpret_cast<const vec*>(s.shift + cl);
    lo = 0.f;
  }
  const int vr = min(8, g.Hg + 2 - 6 * ty), vc = min(8, g.Wg + 2 - 6 * tx);
  const char* base = reinterpret_cast<const char*>(s.ptr) +
                     (((size_t)(n * s.H + 6 * ty + s.oy) * s.W + 6 * tx + s.ox) * s.C + cl) * 4;
  const unsigned rs = (unsigned)s.W * s.C * 4u, cs = (unsigned)s.C * 4u;
  float e[V][8][8];
#pragma unroll
  for (int xx = 0; xx < 8; ++xx) {
    float d[V][8];
#pragma unroll
    for (int yy = 0; yy < 8; ++yy) {
      const bool in = yy < vr && xx < vc;
      vec v = *reinterpret_cast<const vec*>(base + (in ? yy * rs + xx * cs : 0u));
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const float x = fmaxf(fmaf(v[k], sc[k], sh[k]), lo);
        d[k][yy] = in ? x : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float rr[8];
      bt8(d[k], rr);
#pragma unroll
      for (int a = 0; a < 8; ++a) e[k][a][xx] = rr[a];
    }
  }
  const size_t plane = (size_t)T * g.Cg, o = (size_t)t * g.Cg + c;
  char* ub = reinterpret_cast<char*>(u + o);
  const unsigned pbytes = (unsigned)(plane * 4);
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    float rr[V][8];
#pragma unroll
    for (int k = 0; k < V; ++k) bt8(e[k][a], rr[k]);
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) {
      vec o4;
#pragma unroll
      for (int k = 0; k < V; ++k) o4[k] = rr[k][bb];
      *reinterpret_cast<vec*>(ub + (unsigned)(a * 8 + bb) * pbytes) = o4;
    }
  }
}

static void launch_wino6_in(const Gather& g, int Th, int Tw, long long T, float* U, hipStream_t s) {
  int V = wino4_in_vec();
  while (V > 1 && (g.Cg % V || g.c_split % V)) V >>= 1;
  const long long n = T * (g.Cg / V);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (V >= 2) hipLaunchKernelGGL(k_wino6_in<2>, grid, dim3(256), 0, s, g, Th, Tw, T, U);
  else hipLaunchKernelGGL(k_wino6_in<1>, grid, dim3(256), 0, s, g, Th, Tw, T, U);
}

// Block = 64 channels x 4 tile lanes; grid-stride over tiles (k_wino4_out's epilogue)
__global__ __launch_bounds__(256) void k_wino6_out(const float* __restrict__ m, long long T, int Th, int Tw, int N,
                                                   Gather g, Epilogue e) {
  const int col = blockIdx.y * 64 + (int)(threadIdx.x & 63);
  const int tl = threadIdx.x >> 6;
  const bool active = col < N;
  const bool second = col >= e.n_split;
  float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
  const int dC = second ? e.d[1].C : e.d[0].C;
  const int dcol = second ? col - e.n_split : col;
  const bool bwd_mask = e.yref != nullptr && !second;
  float bias = 0.f, bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
  if (active && e.bias) bias = e.bias[col];
  if (active && bwd_mask) { bsc = e.bn_scale[col]; bsh = e.bn_shift[col]; bmu = e.bn_mean[col]; bis = e.bn_invstd[col]; }
  float s1 = 0.f, s2 = 0.f;
  const size_t plane = (size_t)T * N;
  if (active) {
    const unsigned pb = (unsigned)(plane * 4);  // bytes per point plane (64 planes < 4 GB: wino_applies)
    for (long long t = blockIdx.x * 4ll + tl; t < T; t += (long long)gridDim.x * 4) {
      const char* mb = reinterpret_cast<const char*>(m + (size_t)t * N + col);
      float w[6][8];
#pragma unroll
      for (int xx = 0; xx < 8; ++xx) {
        float q[8];
#pragma unroll
        for (int yy = 0; yy < 8; ++yy)
          q[yy] = *reinterpret_cast<const float*>(mb + (unsigned)(yy * 8 + xx) * pb);  // 32-bit offsets
        float o[6];
        at6(q, o);
#pragma unroll
        for (int a = 0; a < 6; ++a) w[a][xx] = o[a];
      }
      const int tx = (int)(t % Tw);
      const long long r = t / Tw;
      const int ty = (int)(r % Th), n = (int)(r / Th);
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        float o[6];
        at6(w[a], o);
        const int y = 6 * ty + a;
        if (y >= g.Hg) continue;
#pragma unroll
        for (int bb = 0; bb < 6; ++bb) {
          const int x = 6 * tx + bb;
          if (x >= g.Wg) continue;
          float v = o[bb] + bias;
          const size_t idx = ((size_t)(n * g.Hg + y) * g.Wg + x) * dC + dcol;
          if (bwd_mask) {
            const float yv = e.yref[idx];
            v = fmaf(yv, bsc, bsh) > 0.f ? v : 0.f;
            s1 += v;
            s2 += v * ((yv - bmu) * bis);
          } else if (e.stats) {
            s1 += v;
            s2 += v * v;
          } else if (second && e.colsum1) {
            s1 += v;
          }
          if (e.relu) v = fmaxf(v, 0.f);
          dptr[idx] = v;
        }
      }
    }
  }
  const bool want = e.stats || e.yref || e.colsum1;
  if (!want) return;
  __shared__ float red[2][256];
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (threadIdx.x < 64 && active) {
    const float a = red[0][threadIdx.x] + red[0][threadIdx.x + 64] + red[0][threadIdx.x + 128] + red[0][threadIdx.x + 192];
    const float b2 = red[1][threadIdx.x] + red[1][threadIdx.x + 64] + red[1][threadIdx.x + 128] + red[1][threadIdx.x + 192];
    const int grp = blockIdx.x % kStatGroups;
    const int nsplit = e.n_split < N ? e.n_split : N;
    if (col < nsplit) {
      double* st = e.yref ? e.bstats : e.stats;
      if (st) {
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 0, (double)a);
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 1, (double)b2);
      }
    } else if (e.colsum1) {
      atomicAdd(e.colsum1 + (size_t)grp * (N - nsplit) + (col - nsplit), (double)a);
    }
  }
}

// workspace of the Winograd path for one GEMM (U, M, V; 256-B aligned pieces):
// P points over T output tiles
static size_t wino_bytes(int P, long long T, int Cg, int N) {
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  return al((size_t)P * T * Cg * 4) + al((size_t)P * T * N * 4) + al((size_t)P * N * Cg * 4);
}
size_t wino_ws_bytes(long long T, int Cg, int N) { return wino_bytes(16, T, Cg, N); }
// the larger of F(2x2) and F(4x4) for an (H, W) output grid of nimg images
size_t wino_ws_bytes_grid(int nimg, int H, int W, int Cg, int N) {
  const long long t2 = (long long)nimg * ((H + 1) / 2) * ((W + 1) / 2);
  const long long t4 = (long long)nimg * ((H + 3) / 4) * ((W + 3) / 4);
  const long long t6 = (long long)nimg * ((H + 5) / 6) * ((W + 5) / 6);
  const size_t a = wino_bytes(16, t2, Cg, N), b = wino_bytes(36, t4, Cg, N), c = wino_bytes(64, t6, Cg, N);
  return std::max(a, std::max(b, c));
}

bool wino_applies(const IgemmArgs& a, int mt) {
  const Gather& g = a.a;
  if (a.b == nullptr || a.bh != nullptr || g.taps_h != 3 || g.taps_w != 3 || g.stride != 1 || a.K != 9 * g.Cg ||
      g.Cg % 4 || g.c_split % 4 || a.N % 64 || g.s[0].h16 || g.s[1].h16 || a.e.shuffle_co)
    return false;
  for (int k = 0; k < 2; ++k) {
    const Dst& d = a.e.d[k];
    if (k == 1 && a.e.n_split >= a.N) break;
    if (d.h16 || d.oy || d.ox || d.H != g.Hg || d.W != g.Wg || d.C % 4) return false;
  }
  if (a.e.yref_h16 || a.e.n_split % 4) return false;
  const long long T = (long long)g.nimg * ((g.Hg + mt - 1) / mt) * ((g.Wg + mt - 1) / mt);
  // the transforms address U / M with 32-bit byte offsets
  if ((long long)(mt + 2) * (mt + 2) * T * std::max(g.Cg, a.N) * 4 >= (1ll << 32)) return false;
  return a.wino_ws != nullptr && wino_bytes((mt + 2) * (mt + 2), T, g.Cg, a.N) <= a.wino_ws_bytes;
}

hipError_t launch_wino(const IgemmArgs& a, hipStream_t s, int mt) {
  if (!wino_applies(a, mt)) return hipErrorInvalidValue;
  const Gather& g = a.a;
  const int P = (mt + 2) * (mt + 2);
  const int Th = (g.Hg + mt - 1) / mt, Tw = (g.Wg + mt - 1) / mt;
  const long long T = (long long)g.nimg * Th * Tw;
  char* w = reinterpret_cast<char*>(a.wino_ws);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  float* U = reinterpret_cast<float*>(w);
  float* Mm = reinterpret_cast<float*>(w + al((size_t)P * T * g.Cg * 4));
  float* V = reinterpret_cast<float*>(w + al((size_t)P * T * g.Cg * 4) + al((size_t)P * T * a.N * 4));
  const long long nw = (long long)a.N * g.Cg;
  if (mt == 2) {
    hipLaunchKernelGGL(k_wino_w, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
    const long long ni = T * (g.Cg / 4);
    hipLaunchKernelGGL(k_wino_in, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, s, g, Th, Tw, T, U);
  } else if (mt == 4) {
    hipLaunchKernelGGL(k_wino4_w, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
    launch_wino4_in(g, Th, Tw, T, U, s);
  } else {
    hipLaunchKernelGGL(k_wino6_w, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
    launch_wino6_in(g, Th, Tw, T, U, s);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  {
    // the P point GEMMs as one batched launch over a 1 x P*T row grid:
    // M[p] = U[p] (T x Cg) . V[p]^T, V[p] = [N][Cg]
    IgemmArgs q;
    Src u;
    u.ptr = U;
    u.H = 1;
    u.W = (int)(P * T);
    u.C = g.Cg;
    q.a.s[0] = q.a.s[1] = u;
    q.a.Cg = q.a.c_split = g.Cg;
    q.a.taps_h = q.a.taps_w = 1;
    q.a.Hg = 1;
    q.a.Wg = (int)(P * T);
    q.a.nimg = 1;
    q.b = V;
    q.M = (int)(P * T);
    q.N = a.N;
    q.K = g.Cg;
    q.e.d[0] = Dst{Mm, 1, (int)(P * T), a.N, 0, 0};
    q.batch = P;
    q.batch_rows = (int)T;
    q.batch_b = (long long)a.N * g.Cg;
    // 256 x 128 tiles when they give two rounds of workgroups, else 128 x 128
    // (register-staged k_igemm: the batched launch form)
    int tile = a.wino_choice.tile;  // autotuned (GemmChoice split 100 + tile), else the heuristic
    if (tile <= 0 || !igemm_tile_fits(q, tile)) {
      const long long t256 = ((T + 255) / 256) * (a.N / 128) * P;
      tile = (a.N % 128 == 0 && t256 >= 2 * num_cus()) ? 4 : (a.N % 128 == 0 ? 1 : 8);
    }
    if ((e = launch_igemm_v(q, s, GemmChoice{tile, 1})) != hipSuccess) return e;
  }
  if (mt == 2) {
    const int C4 = a.N / 4, cgs = C4 < 64 ? C4 : 64, lanes = 256 / cgs;
    long long gx = (T + lanes * 4 - 1) / (lanes * 4);  // ~4 tiles per thread: statistics kept in registers
    if (gx > 65535) gx = 65535;
    dim3 grid((unsigned)gx, (unsigned)((C4 + cgs - 1) / cgs));
    hipLaunchKernelGGL(k_wino_out, grid, dim3(256), 0, s, Mm, T, Th, Tw, a.N, g, a.e);
  } else {
    long long gx = (T + 15) / 16;  // 4 tile lanes x ~4 tiles per thread
    if (gx > 65535) gx = 65535;
    dim3 grid((unsigned)gx, (unsigned)((a.N + 63) / 64));
    if (mt == 4) hipLaunchKernelGGL(k_wino4_out, grid, dim3(256), 0, s, Mm, T, Th, Tw, a.N, g, a.e);
    else hipLaunchKernelGGL(k_wino6_out, grid, dim3(256), 0, s, Mm, T, Th, Tw, a.N, g, a.e);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused F(4x4, 3x3) (tile 72): one kernel per GEMM, no U / M in HBM.
// A workgroup (8 waves) owns 32 output tiles (4x4 pixels each, linear tile
// order) x 32 output channels and loops over the input channels in chunks of 16:
//   * thread (tile = tid / 16, channel = tid % 16) loads its 6x6 input patch
//     into registers (prefetched one chunk ahead), applies the producer's
//     BatchNorm + ReLU, computes B^T d B and writes the 36 points to LDS
//     U[p][tile][16];
//   * the pre-transformed weights V (k_wino4f_w, layout [Cg/16][36][N][16]) are
//     staged the same way into V[p][n][16];
//   * wave w multiplies the 16-tile half w & 1 for points 9 (w >> 1) .. +8 and
//     both 16-channel halves with v_mfma_f32_16x16x4_f32: per point one
//     ds_read_b128 of U, two of V, eight MFMAs (lane quarter q takes channels
//     4q .. 4q+3 as its k: any order works as long as A and B agree);
//   * the 36 accumulators of every (tile, channel) leave through LDS
//     ([36][32][32], reusing the staging space) and each thread applies
//     A^T M A and the epilogue of k_wino4_out to the 16 pixels of two pairs.
// LDS rows are 16 floats (64 B) with 16-B piece q stored at q ^ (2 * ((row >> 3)
// & 1)): the ds_read_b128 lane groups then hit 64 distinct banks.  147 KB of
// LDS, one workgroup (2 waves per SIMD) per CU.
// ---------------------------------------------------------------------------
template <int CK>
__global__ void k_wino4f_w(const float* __restrict__ b, int N, int Cg, float* __restrict__ v) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)N * Cg) return;
  const int n = (int)(i / Cg), c = (int)(i - (long long)n * Cg);
  float tg[6][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float col[3] = {b[((size_t)n * 9 + 0 + k) * Cg + c], b[((size_t)n * 9 + 3 + k) * Cg + c],
                    b[((size_t)n * 9 + 6 + k) * Cg + c]};
    float r[6];
    g6(col, r);
#pragma unroll
    for (int a = 0; a < 6; ++a) tg[a][k] = r[a];
  }
  const size_t base = (size_t)(c / CK) * 36 * N;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float r[6];
    g6(tg[a], r);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) v[(base + (size_t)(a * 6 + bb) * N + n) * CK + (c % CK)] = r[bb];
  }
}

// float offset of 16-B piece q of LDS row `row` (16 floats per row)
__device__ __forceinline__ int wf_off(int row, int q) { return row * 16 + ((q ^ (((row >> 3) & 1) << 1)) << 2); }

// Output stage of the fused kernels (512 threads): X = LDS [36][32 tiles][32
// channels] holds the point accumulators; thread = channel oc of tiles ot and
// ot + 16 applies A^T M A and the epilogue of k_wino4_out to their 16 pixels.
__device__ __forceinline__ void wf_output(float* lds, int tid, long long t0, int n0, long long T, int Th, int Tw,
                                          int N, const Gather& g, const Epilogue& e) {
  const float* X = lds;
  const int oc = tid & 31;
  const int col = n0 + oc;
  const bool second = col >= e.n_split;
  float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
  const int dC = second ? e.d[1].C : e.d[0].C;
  const int dcol = second ? col - e.n_split : col;
  const bool bwd_mask = e.yref != nullptr && !second;
  const float bias = e.bias ? e.bias[col] : 0.f;
  float bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
  if (bwd_mask) { bsc = e.bn_scale[col]; bsh = e.bn_shift[col]; bmu = e.bn_mean[col]; bis = e.bn_invstd[col]; }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ot = (tid >> 5) + 16 * k;
    const long long tt = t0 + ot;
    if (tt >= T) continue;
    float w[4][6];
#pragma unroll
    for (int xx = 0; xx < 6; ++xx) {
      float m[6];
#pragma unroll
      for (int yy = 0; yy < 6; ++yy) m[yy] = X[(yy * 6 + xx) * 1024 + ot * 32 + oc];
      float o[4];
      at4(m, o);
#pragma unroll
      for (int a = 0; a < 4; ++a) w[a][xx] = o[a];
    }
    const int ox = (int)(tt % Tw);
    const long long r = tt / Tw;
    const int oy = (int)(r % Th), on = (int)(r / Th);
    float yv[4][4];
    if (bwd_mask) wf_yref4(e.yref, g, on, oy, ox, dC, dcol, yv);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float o[4];
      at4(w[a], o);
      const int y = 4 * oy + a;
      if (y >= g.Hg) continue;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int x = 4 * ox + bb;
        if (x >= g.Wg) continue;
        float v = o[bb] + bias;
        const size_t idx = ((size_t)(on * g.Hg + y) * g.Wg + x) * dC + dcol;
        if (bwd_mask) {
          v = fmaf(yv[a][bb], bsc, bsh) > 0.f ? v : 0.f;
          s1 += v;
          s2 += v * ((yv[a][bb] - bmu) * bis);
        } else if (e.stats) {
          s1 += v;
          s2 += v * v;
        } else if (second && e.colsum1) {
          s1 += v;
        }
        if (e.relu) v = fmaxf(v, 0.f);
        dptr[idx] = v;
      }
    }
  }
  const bool want = e.stats || e.yref || e.colsum1;
  if (!want) return;
  __syncthreads();
  float* red = lds;  // [2][16][32]
  red[tid] = s1;
  red[512 + tid] = s2;
  __syncthreads();
  if (tid < 32) {
    float a = 0.f, b2 = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      a += red[q * 32 + tid];
      b2 += red[512 + q * 32 + tid];
    }
    const int grp = blockIdx.x % kStatGroups;
    const int nsplit = e.n_split < N ? e.n_split : N;
    if (col < nsplit) {
      double* st = e.yref ? e.bstats : e.stats;
      if (st) {
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 0, (double)a);
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 1, (double)b2);
      }
    } else if (e.colsum1) {
      atomicAdd(e.colsum1 + (size_t)grp * (N - nsplit) + (col - nsplit), (double)a);
    }
  }
}

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ABL: ablation switches for timing experiments only (UNET_WF_ABL; results are
// wrong with any bit set): 1 = no input transform / BatchNorm, 2 = no MFMA,
// 4 = no global loads in the chunk loop
template <int ABL>
__global__ __launch_bounds__(512, 1) void k_wino4f(Gather g, const float* __restrict__ V, int N, long long T,
                                                   int Th, int Tw, int NB, Epilogue e) {
  constexpr int PS = 32 * 16;  // floats per point plane of U / V
  __shared__ __attribute__((aligned(16))) float lds[2 * 36 * PS];
  float* Us = lds;
  float* Vs = lds + 36 * PS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long bid = blockIdx.x;
  const long long G = gridDim.x;
  if ((G & 7) == 0) bid = (bid & 7) * (G >> 3) + (bid >> 3);  // an XCD's workgroups share tiles
  const int nb = (int)(bid % NB);
  const long long t0 = (bid / NB) * 32;
  const int n0 = nb * 32;

  // ---- loader role: (tile lt, channel lc of the chunk) ----
  const int lt = tid >> 4, lc = tid & 15;
  const long long t = t0 + lt;
  int img = 0, ty = 0, tx = 0;
  if (t < T) {
    tx = (int)(t % Tw);
    const long long r = t / Tw;
    ty = (int)(r % Th);
    img = (int)(r / Th);
  }
  // patch rows / columns inside the (Hg+2) x (Wg+2) input window (all of them
  // except in the last tile row / column)
  const int vrows = t < T ? min(6, g.Hg + 2 - 4 * ty) : 0;
  const int vcols = t < T ? min(6, g.Wg + 2 - 4 * tx) : 0;
  const bool full = vrows == 6 && vcols == 6;
  const bool wfull = __all(full);
  const int uoff = wf_off(lt, lc >> 2) + (lc & 3);
  float raw[36];
  float4 vr[9];
  const int nk = g.Cg >> 4;
  auto load = [&](int kc) {
    // chunks never straddle the concat split (c_split % 16 == 0): uniform source
    const bool second = kc * 16 >= g.c_split;
    const float* sp = second ? g.s[1].ptr : g.s[0].ptr;
    const int sH = second ? g.s[1].H : g.s[0].H, sW = second ? g.s[1].W : g.s[0].W;
    const int sC = second ? g.s[1].C : g.s[0].C;
    const int soy = second ? g.s[1].oy : g.s[0].oy, sox = second ? g.s[1].ox : g.s[0].ox;
    const int cl = kc * 16 - (second ? g.c_split : 0) + lc;
    // unsigned 32-bit byte offsets from a uniform base (sources are below 4 GB,
    // wino_fused_applies): one v_add per load, SGPR-base addressing
    const char* sb = reinterpret_cast<const char*>(sp);
    const unsigned o0 = ((unsigned)((img * sH + 4 * ty + soy) * sW + 4 * tx + sox) * sC + cl) * 4u;
    const unsigned rs = (unsigned)sW * sC * 4u, cs = (unsigned)sC * 4u;
    if (wfull) {  // wave-uniform: no edge tile in this wave
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int xx = 0; xx < 6; ++xx)
          raw[yy * 6 + xx] = *reinterpret_cast<const float*>(sb + (o0 + (yy * rs + xx * cs)));
    } else {
      // edge tiles: rows / columns past the window re-read the last in-window
      // one (branch-free clamp; zeroed in commit)
      const unsigned lr = (unsigned)max(vrows - 1, 0), lcn = (unsigned)max(vcols - 1, 0);
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int xx = 0; xx < 6; ++xx)
          raw[yy * 6 + xx] = *reinterpret_cast<const float*>(
              sb + (o0 + (min((unsigned)yy, lr) * rs + min((unsigned)xx, lcn) * cs)));
    }
    const char* vb = reinterpret_cast<const char*>(V + ((size_t)kc * 36 * N + n0) * 16);
    const unsigned vo = ((unsigned)(tid >> 7) * N * 16u + ((tid >> 2) & 31) * 16u + (tid & 3) * 4u) * 4u;
    const unsigned vstep = 4u * N * 16u * 4u;  // 4 points per 512 float4
#pragma unroll
    for (int j = 0; j < 9; ++j) vr[j] = *reinterpret_cast<const float4*>(vb + (vo + j * vstep));
  };
  auto commit = [&](int kc) {
    const bool second = kc * 16 >= g.c_split;
    const float* scp = second ? g.s[1].scale : g.s[0].scale;
    const float* shp = second ? g.s[1].shift : g.s[0].shift;
    const int cl = kc * 16 - (second ? g.c_split : 0) + lc;
    if constexpr (ABL & 1) {
#pragma unroll
      for (int q = 0; q < 36; ++q) Us[q * PS + uoff] = raw[q];
    } else {
    if (scp) {
      const float sc = scp[cl], sh = shp[cl];
#pragma unroll
      for (int q = 0; q < 36; ++q) raw[q] = fmaxf(fmaf(raw[q], sc, sh), 0.f);
    }
    if (!wfull) {
#pragma unroll
      for (int q = 0; q < 36; ++q) raw[q] = (q / 6 < vrows && q % 6 < vcols) ? raw[q] : 0.f;
    }
#pragma unroll
    for (int xx = 0; xx < 6; ++xx) {  // columns in place: raw[a][xx] = (B^T d)[a][xx]
      float d[6];
#pragma unroll
      for (int yy = 0; yy < 6; ++yy) d[yy] = raw[yy * 6 + xx];
      float rr[6];
      bt6(d, rr);
#pragma unroll
      for (int a = 0; a < 6; ++a) raw[a * 6 + xx] = rr[a];
    }
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      float d[6];
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) d[xx] = raw[a * 6 + xx];
      float rr[6];
      bt6(d, rr);
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) Us[(a * 6 + bb) * PS + uoff] = rr[bb];
    }
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int q = tid + 512 * j;
      const int p = q >> 7, n = (q >> 2) & 31, piece = q & 3;
      st4(Vs + p * PS + wf_off(n, piece), vr[j]);
    }
  };

  // ---- MFMA role: tile half th, points 9 pg .. 9 pg + 8, both channel halves ----
  const int th = wave & 1, pg = wave >> 1;
  const int mi = lane & 15, mq = lane >> 4;
  const int aoff = wf_off(16 * th + mi, mq);
  const int boff0 = wf_off(mi, mq), boff1 = wf_off(16 + mi, mq);
  floatx4 acc[9][2];
#pragma unroll
  for (int j = 0; j < 9; ++j)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) acc[j][hh] = (floatx4){0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int kc = 0; kc < nk; ++kc) {
    commit(kc);
    __syncthreads();
    if (!(ABL & 4) && kc + 1 < nk) load(kc + 1);
    if constexpr (!(ABL & 2))
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int p = pg * 9 + j;
      const float4 a = ld4(Us + p * PS + aoff);
      const float4 b0 = ld4(Vs + p * PS + boff0);
      const float4 b1 = ld4(Vs + p * PS + boff1);
      acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b0.x, acc[j][0], 0, 0, 0);
      acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b1.x, acc[j][1], 0, 0, 0);
      acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b0.y, acc[j][0], 0, 0, 0);
      acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b1.y, acc[j][1], 0, 0, 0);
      acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b0.z, acc[j][0], 0, 0, 0);
      acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b1.z, acc[j][1], 0, 0, 0);
      acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b0.w, acc[j][0], 0, 0, 0);
      acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b1.w, acc[j][1], 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- accumulators -> LDS X[36][32 tiles][32 channels] ----
  // 16x16 accumulator: lane l holds column l & 15, rows 4 (l >> 4) + r
  float* X = lds;
#pragma unroll
  for (int j = 0; j < 9; ++j)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        X[(pg * 9 + j) * 1024 + (16 * th + 4 * mq + r) * 32 + 16 * hh + mi] = acc[j][hh][r];
  __syncthreads();

  wf_output(lds, tid, t0, n0, T, Th, Tw, N, g, e);
}

bool wino_fused_applies(const IgemmArgs& a) {
  constexpr int ck = 16;
  const Gather& g = a.a;
  if (a.b == nullptr || a.bh != nullptr || a.batch != 1) return false;
  if (g.taps_h != 3 || g.taps_w != 3 || g.stride != 1 || a.K != 9 * g.Cg || g.Cg % ck != 0 ||
      g.c_split % ck != 0 || a.N % 32 != 0)
    return false;
  if (g.s[0].h16 || g.s[1].h16 || a.e.shuffle_co || a.e.d[0].h16 || a.e.d[1].h16 || a.e.yref_h16) return false;
  if (a.e.d[0].oy || a.e.d[0].ox || a.e.d[0].H != g.Hg || a.e.d[0].W != g.Wg) return false;
  if (a.e.n_split < a.N && (a.e.d[1].oy || a.e.d[1].ox || a.e.d[1].H != g.Hg || a.e.d[1].W != g.Wg)) return false;
  for (int k = 0; k < 2; ++k)  // 32-bit byte offsets into the sources
    if ((long long)g.nimg * g.s[k].H * g.s[k].W * g.s[k].C * 4 >= (1ll << 32)) return false;
  const long long T = (long long)g.nimg * ((g.Hg + 3) / 4) * ((g.Wg + 3) / 4);
  if ((T + 31) / 32 * (a.N / 32) > 0x7fffffffLL) return false;
  return a.wino_ws != nullptr && (size_t)36 * a.N * g.Cg * 4 <= a.wino_ws_bytes;
}

hipError_t launch_wino_fused(const IgemmArgs& a, hipStream_t s) {
  if (!wino_fused_applies(a)) return hipErrorInvalidValue;
  const Gather& g = a.a;
  const int Th = (g.Hg + 3) / 4, Tw = (g.Wg + 3) / 4;
  const long long T = (long long)g.nimg * Th * Tw;
  float* V = reinterpret_cast<float*>(a.wino_ws);
  const long long nw = (long long)a.N * g.Cg;
  const int NB = a.N / 32;
  const long long G = (T + 31) / 32 * NB;
  hipLaunchKernelGGL(k_wino4f_w<16>, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
  static const int abl = ablation_env("UNET_WF_ABL");
  switch (abl) {
    case 1: hipLaunchKernelGGL(k_wino4f<1>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e); break;
    case 2: hipLaunchKernelGGL(k_wino4f<2>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e); break;
    case 4: hipLaunchKernelGGL(k_wino4f<4>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e); break;
    case 6: hipLaunchKernelGGL(k_wino4f<6>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e); break;
    default: hipLaunchKernelGGL(k_wino4f<0>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused F(4x4, 3x3), 64 output channels (tile 73).  k_wino4f's input transform
// (and the loads + BatchNorm in front of it) is done once per 32 tiles x 32
// output channels; f32 MFMA and that VALU work share the SIMD, so the kernel
// runs at their sum.  Here a workgroup owns 32 tiles x 64 output channels and
// walks the input channels in chunks of 8, which halves the transform work per
// MFMA at the same LDS (U 32 tiles x 8 + V 64 outputs x 8 per point) and the
// same 72 MFMAs per wave and chunk:
//   * 256 patches (32 tiles x 8 channels) per chunk, two threads per patch:
//     lanes of 16-lane row 2r take the patch's columns 0..2, row 2r + 1 its
//     columns 3..5 (same tile / channel by lane & 15).  Each transforms its
//     three columns (B^T d), then v_permlane16_swap exchanges the halves so
//     that the even row holds rows 0..2 and the odd row rows 3..5 of all six
//     columns (no lane-dependent selects), and each applies the row transform
//     to its three rows: 18 loads, 6 bt6 and 9 swaps per thread and chunk;
//   * V (k_wino4f_w8, layout [Cg/8][36][N][8], 8-float rows pre-swizzled) is
//     copied row for row: 9 float4 per thread;
//   * LDS rows are 8 floats; slot s (2 floats) of row r holds channels (q, q+4)
//     with s = q ^ ((r >> 2) & 3) (wf8_slot), so the operand reads of a
//     16x16x4 MFMA (lane quarter q: k = q in step 0, q + 4 in step 1) are
//     conflict-free;
//   * wave w: tile half w & 1, points 9 (w >> 1) .. +8, the four 16-channel
//     output blocks: per point one U read, four V reads, eight MFMAs;
//   * the accumulators leave in two 32-channel passes through wf_output.
// ---------------------------------------------------------------------------
// slot of channel pair (q, q + 4) in an 8-float row: XOR by row bits 2-3, so
// that 16 consecutive rows hit 16 distinct 8-byte bank pairs both mod 64 banks
// (ds_read_b64) and mod 32 (the ds_read2_b64 / ds_read2st64_b64 the compiler
// merges two points' reads into; the bit-3-only swizzle was 2-way conflicted
// there: 3e8 conflict cycles per step, profiles/r03_pmc_summary_fp32.txt)
__device__ __forceinline__ int wf8_slot(int row, int q) { return (q ^ ((row >> 2) & 3)) << 1; }

__global__ void k_wino4f_w8(const float* __restrict__ b, int N, int Cg, float* __restrict__ v) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)N * Cg) return;
  const int n = (int)(i / Cg), c = (int)(i - (long long)n * Cg);
  float tg[6][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float col[3] = {b[((size_t)n * 9 + 0 + k) * Cg + c], b[((size_t)n * 9 + 3 + k) * Cg + c],
                    b[((size_t)n * 9 + 6 + k) * Cg + c]};
    float r[6];
    g6(col, r);
#pragma unroll
    for (int a = 0; a < 6; ++a) tg[a][k] = r[a];
  }
  const size_t base = (size_t)(c >> 3) * 36 * N;
  const int pos = wf8_slot(n, c & 3) + ((c >> 2) & 1);  // n & 63 and n agree on bits 2-3
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float r[6];
    g6(tg[a], r);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) v[(base + (size_t)(a * 6 + bb) * N + n) * 8 + pos] = r[bb];
  }
}

// ABL: timing ablations (UNET_WF64_ABL; results wrong with any bit set): 1 = no
// BatchNorm / transform arithmetic, 2 = no MFMA, 4 = no operand loads after the
// first chunk, 8 = no output stage, 16 = no wait for the chunk's V DMAs
// One output element of the register-output fused kernels: the dgrad ReLU
// mask + BN-backward statistics (bwd_mask) or the forward sums (s1 = sum v,
// s2 = sum v^2; the caller reduces s1 only where it wants a column sum), then
// the optional ReLU.  Branch-free in the per-wave flags.
__device__ __forceinline__ float wf_epi(float v, float yv, float sc, float sh, float mu, float is, bool bwd_mask,
                                        bool relu, float& s1, float& s2) {
  v = (bwd_mask && !(fmaf(yv, sc, sh) > 0.f)) ? 0.f : v;
  s1 += v;
  s2 += v * (bwd_mask ? (yv - mu) * is : v);
  return relu ? fmaxf(v, 0.f) : v;
}

// The output stage of the 64-channel fused F(4x4) kernels (tiles 73, 76):
// lane (mi, mq) of wave (th, cb) holds all 36 points of channels n0 + 16 cb +
// 4 mq .. +3 of tile t0 + 16 th + mi; A^T M A from registers, the epilogue
// (bias, dgrad ReLU mask + BN-backward statistics or forward sums), 16-B
// stores.  `lds` is free (every wave past the chunk loop's last barrier).
__device__ __forceinline__ void wf64_output(const floatx4 (&acc)[36], const Gather& g, const Epilogue& e, int N,
                                            long long T, int Th, int Tw, long long t0, int n0, int th, int cb,
                                            int mi, int mq, int lane, int wave, float* lds) {
  const long long tt = t0 + 16 * th + mi;
  const int col0 = n0 + 16 * cb + 4 * mq;
  const bool second = col0 >= e.n_split;  // uniform per 16-channel block (n_split % 16 == 0)
  float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
  const int dC = second ? e.d[1].C : e.d[0].C;
  const int dcol = second ? col0 - e.n_split : col0;
  const bool bwd_mask = e.yref != nullptr && !second;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (tt < T) {
    const int ox = (int)(tt % Tw);
    const long long rq = tt / Tw;
    const int oy = (int)(rq % Th), on = (int)(rq / Th);
    float o[4][4][4];  // [channel][row][col]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float w[4][6];
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) {
        float m[6];
#pragma unroll
        for (int yy = 0; yy < 6; ++yy) m[yy] = acc[yy * 6 + xx][r];
        float t4[4];
        at4(m, t4);
#pragma unroll
        for (int a = 0; a < 4; ++a) w[a][xx] = t4[a];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) at4(w[a], o[r][a]);
    }
    const float4 bias = e.bias ? ld4(e.bias + col0) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 bsc = make_float4(0.f, 0.f, 0.f, 0.f), bsh = bsc, bmu = bsc, bis = bsc;
    if (bwd_mask) { bsc = ld4(e.bn_scale + col0); bsh = ld4(e.bn_shift + col0); bmu = ld4(e.bn_mean + col0); bis = ld4(e.bn_invstd + col0); }
    const float bsv[4] = {bias.x, bias.y, bias.z, bias.w};
    const float scv[4] = {bsc.x, bsc.y, bsc.z, bsc.w}, shv[4] = {bsh.x, bsh.y, bsh.z, bsh.w};
    const float muv[4] = {bmu.x, bmu.y, bmu.z, bmu.w}, isv[4] = {bis.x, bis.y, bis.z, bis.w};
    // The dgrad's mask operand y (16 B per pixel and lane) comes in by LDS-DMA,
    // 8 pixels at a time into this wave's 8 KB of the (now idle) LDS, one wait
    // per 8: register loads here made the compiler chain load -> wait -> store
    // per pixel (the in-order vmcnt counts the stores), with nothing else on the
    // CU to hide it (round 4: ~0.9 ms of the fp32 step, UNET_WF64_ABL=8).
    const unsigned long long ybase = uniform_u64(e.yref);  // kernel argument: SGPRs (unused unless bwd_mask)
    const unsigned ylds = (unsigned)(size_t)(lds_u8_t*)lds + (unsigned)wave * 8192u;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (bwd_mask) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int y = min(4 * oy + 2 * h + (q >> 2), g.Hg - 1), x = min(4 * ox + (q & 3), g.Wg - 1);
          dma_sv((((unsigned)(on * g.Hg + y) * g.Wg + x) * dC + dcol) * 4u, ybase, ylds + q * 1024u);
        }
      }
      // vmcnt(0) as a builtin, not asm: it retires the DMAs and, visibly to the
      // compiler's wait-count tracking, the coefficient loads above, so no
      // per-pixel branch join leaves them pending (it then re-waited, stores
      // included, before every pixel)
      __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int a = 2 * h + (q >> 2), bb = q & 3;
        const int y = 4 * oy + a, x = 4 * ox + bb;
        if (y >= g.Hg || x >= g.Wg) continue;
        const float4 yq = bwd_mask ? *reinterpret_cast<const float4*>(lds + wave * 2048 + q * 256 + lane * 4)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        const float yv[4] = {yq.x, yq.y, yq.z, yq.w};
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = wf_epi(o[r][a][bb] + bsv[r], yv[r], scv[r], shv[r], muv[r], isv[r],
                                                   bwd_mask, e.relu, s1[r], s2[r]);
        st4(dptr + ((size_t)(on * g.Hg + y) * g.Wg + x) * dC + dcol, make_float4(v[0], v[1], v[2], v[3]));
      }
    }
  }
  const bool want = e.stats || e.yref || e.colsum1;
  if (!want) return;
  // the 16 lanes of a quarter hold the same 4 channels (other tiles)
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o2 = 1; o2 < 16; o2 <<= 1) {
      s1[r] += __shfl_xor(s1[r], o2);
      s2[r] += __shfl_xor(s2[r], o2);
    }
  if (mi == 0) {
    const int grp = blockIdx.x % kStatGroups;
    const int nsplit = e.n_split < N ? e.n_split : N;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = col0 + r;
      if (col < nsplit) {
        double* st = e.yref ? e.bstats : e.stats;
        if (st) {
          atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 0, (double)s1[r]);
          atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 1, (double)s2[r]);
        }
      } else if (e.colsum1) {
        atomicAdd(e.colsum1 + (size_t)grp * (N - nsplit) + (col - nsplit), (double)s1[r]);
      }
    }
  }
}

template <int ABL>
__global__ __launch_bounds__(512, 1) void k_wino4f64(Gather g, const float* __restrict__ V, int N, long long T,
                                                     int Th, int Tw, int NB, Epilogue e) {
  constexpr int PU = 32 * 8 + 8;  // U point plane (+8: the two lane rows of a patch store 18 planes apart)
  constexpr int PV = 64 * 8;      // V point plane
  __shared__ __attribute__((aligned(16))) float lds[36 * PU + 36 * PV];  // U, V
  float* Us = lds;
  float* Vs = lds + 36 * PU;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long bid = blockIdx.x;
  const long long G = gridDim.x;
  if ((G & 7) == 0) bid = (bid & 7) * (G >> 3) + (bid >> 3);  // an XCD's workgroups share tiles
  const int nb = (int)(bid % NB);
  const long long t0 = (bid / NB) * 32;
  const int n0 = nb * 64;

  // ---- loader role: patch (tile lt, channel lc), column half hf ----
  const int hf = (lane >> 4) & 1;
  const int pt = wave * 32 + (lane & 15) + ((lane >> 5) << 4);
  const int lt = pt >> 3, lc = pt & 7;
  const long long t = t0 + lt;
  int img = 0, ty = 0, tx = 0;
  if (t < T) {
    tx = (int)(t % Tw);
    const long long r = t / Tw;
    ty = (int)(r % Th);
    img = (int)(r / Th);
  }
  const int vrows = t < T ? min(6, g.Hg + 2 - 4 * ty) : 0;
  const int vcols = t < T ? min(6, g.Wg + 2 - 4 * tx) : 0;
  const bool wfull = __all(vrows == 6 && vcols == 6);
  // this thread's three output rows 3 hf .. 3 hf + 2 of the transformed patch
  float* const ubase = Us + (3 * hf) * 6 * PU + lt * 8 + wf8_slot(lt, lc & 3) + (lc >> 2);
  float raw[18];  // [row 0..5][column 3 hf + 0..2]
  float sc = 1.f, sh = 0.f;  // the chunk's producer BN+ReLU (loaded with raw)
  const int nk = g.Cg >> 3;
  // V (the chunk's 36 x 64 x 8 transformed weights, 2 KB contiguous per point
  // in k_wino4f_w8's layout) goes global -> LDS by DMA, 9 x 1 KB per wave,
  // during the input transform (round 4; through registers it held 36 VGPRs of
  // a kernel at the 256 limit)
  const unsigned long long vbase = uniform_u64(V);
  const unsigned vlds = (unsigned)(size_t)(lds_u8_t*)lds + (unsigned)(36 * PU * 4);
  auto load = [&](int kc) {
    const bool second = kc * 8 >= g.c_split;  // c_split % 8 == 0: uniform source
    const float* sp = second ? g.s[1].ptr : g.s[0].ptr;
    const int sH = second ? g.s[1].H : g.s[0].H, sW = second ? g.s[1].W : g.s[0].W;
    const int sC = second ? g.s[1].C : g.s[0].C;
    const int soy = second ? g.s[1].oy : g.s[0].oy, sox = second ? g.s[1].ox : g.s[0].ox;
    const int cl = kc * 8 - (second ? g.c_split : 0) + lc;
    const float* scp = second ? g.s[1].scale : g.s[0].scale;
    if (scp) {
      sc = scp[cl];
      sh = (second ? g.s[1].shift : g.s[0].shift)[cl];
    }
    const char* sb = reinterpret_cast<const char*>(sp);
    const unsigned o0 = ((unsigned)((img * sH + 4 * ty + soy) * sW + 4 * tx + sox) * sC + cl) * 4u;
    const unsigned rs = (unsigned)sW * sC * 4u, cs = (unsigned)sC * 4u;
    if (wfull) {
      const unsigned oh = o0 + 3u * hf * cs;
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int xx = 0; xx < 3; ++xx)
          raw[yy * 3 + xx] = *reinterpret_cast<const float*>(sb + (oh + (yy * rs + xx * cs)));
    } else {  // clamp to the last in-window row / column (zeroed in commit)
      const unsigned lr = (unsigned)max(vrows - 1, 0), lcn = (unsigned)max(vcols - 1, 0);
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int xx = 0; xx < 3; ++xx)
          raw[yy * 3 + xx] = *reinterpret_cast<const float*>(
              sb + (o0 + (min((unsigned)yy, lr) * rs + min((unsigned)(3 * hf + xx), lcn) * cs)));
    }
  };
  auto commit = [&](int kc) {
    const bool second = kc * 8 >= g.c_split;
    const float* scp = second ? g.s[1].scale : g.s[0].scale;
    // raw(kc) and its BN coefficients (issued a whole MFMA phase ago): retired
    // by a wait the compiler sees, so nothing it tracks is pending behind the
    // V DMAs queued next (in-order vmcnt: a later wait would cover them)
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int pc = wave + 8 * j;  // 1-KB piece: point pc >> 1, half pc & 1
      dma_sv((unsigned)((((size_t)kc * 36 + (pc >> 1)) * N + n0) * 32) + (unsigned)((pc & 1) * 1024 + lane * 16),
             vbase, vlds + (unsigned)((pc >> 1) * PV * 4 + (pc & 1) * 1024));
    }
    if constexpr (ABL & 1) {
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int bb = 0; bb < 6; ++bb) ubase[(a * 6 + bb) * PU] = raw[a * 6 + bb];
    } else {
    if (scp) {
#pragma unroll
      for (int q = 0; q < 18; ++q) raw[q] = fmaxf(fmaf(raw[q], sc, sh), 0.f);
    }
    if (!wfull) {
#pragma unroll
      for (int q = 0; q < 18; ++q) raw[q] = (q / 3 < vrows && 3 * hf + q % 3 < vcols) ? raw[q] : 0.f;
    }
#pragma unroll
    for (int xx = 0; xx < 3; ++xx) {  // columns in place: raw[a][xx] = (B^T d)[a][3 hf + xx]
      float d[6];
#pragma unroll
      for (int yy = 0; yy < 6; ++yy) d[yy] = raw[yy * 3 + xx];
      float rr[6];
      bt6(d, rr);
#pragma unroll
      for (int a = 0; a < 6; ++a) raw[a * 3 + xx] = rr[a];
    }
    // X = rows 0..2, Y = rows 3..5 of this thread's columns; the swap trades
    // the odd lane row's X for the even lane row's Y: the even row then holds
    // rows 0..2 x columns (0..2 in X, 3..5 in Y), the odd row rows 3..5 alike
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(raw[k]), __float_as_uint(raw[9 + k]),
                                                       false, false);
      raw[k] = __uint_as_float(sw[0]);
      raw[9 + k] = __uint_as_float(sw[1]);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float d[6] = {raw[a * 3 + 0], raw[a * 3 + 1], raw[a * 3 + 2],
                          raw[9 + a * 3 + 0], raw[9 + a * 3 + 1], raw[9 + a * 3 + 2]};
      float rr[6];
      bt6(d, rr);
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) ubase[(a * 6 + bb) * PU] = rr[bb];
    }
    }
    if constexpr (!(ABL & 16)) vm_wait<0>();  // V(kc) landed (the DMAs are asm: invisible to the compiler's counts)
  };

  // ---- MFMA role: wave = (tile half th, 16-channel block cb), all 36 points ----
  // C_p = V_p^T U_p (channels as MFMA rows, tiles as columns): lane (mi, mq)
  // holds every point of channels 4 mq .. 4 mq + 3 of tile mi, applies A^T M A
  // from registers and stores 4 channels per pixel with one 16-B store (the
  // LDS output stage and its 64 scalar stores per lane are gone).
  const int th = wave & 1, cb = wave >> 1;
  const int mi = lane & 15, mq = lane >> 4;
  const int aoff = (16 * th + mi) * 8 + wf8_slot(16 * th + mi, mq);
  const int boff = (16 * cb + mi) * 8 + wf8_slot(mi, mq);  // rows 16 cb + mi and mi agree on bits 2-3
  floatx4 acc[36];
#pragma unroll
  for (int p = 0; p < 36; ++p) acc[p] = (floatx4){0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int kc = 0; kc < nk; ++kc) {
    commit(kc);
    __syncthreads();
    if (!(ABL & 4) && kc + 1 < nk) load(kc + 1);
    if constexpr (!(ABL & 2))
#pragma unroll
    for (int p = 0; p < 36; ++p) {
      const float2 a = *reinterpret_cast<const float2*>(Us + p * PU + aoff);
      const float2 b = *reinterpret_cast<const float2*>(Vs + p * PV + boff);
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.x, a.x, acc[p], 0, 0, 0);
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.y, a.y, acc[p], 0, 0, 0);
    }
    __syncthreads();
  }
  if constexpr (ABL & 8) {  // every accumulator stays live (the MFMAs are kept)
    float sum = 0.f;
#pragma unroll
    for (int p = 0; p < 36; ++p) sum += acc[p][0] + acc[p][1] + acc[p][2] + acc[p][3];
    if (sum == 1.2345f) e.d[0].ptr[tid] = sum;
    return;
  }

  wf64_output(acc, g, e, N, T, Th, Tw, t0, n0, th, cb, mi, mq, lane, wave, lds);
}

bool wino_fused64_applies(const IgemmArgs& a) {
  // Cg, c_split % 16 == 0 imply % 8; the mask operand's LDS-DMA takes 32-bit byte offsets
  return wino_fused_applies(a) && a.N % 64 == 0 &&
         (a.e.yref == nullptr || (long long)a.a.nimg * a.a.Hg * a.a.Wg * a.e.d[0].C * 4 < (1ll << 32));
}

hipError_t launch_wino_fused64(const IgemmArgs& a, hipStream_t s) {
  if (!wino_fused64_applies(a)) return hipErrorInvalidValue;
  const Gather& g = a.a;
  const int Th = (g.Hg + 3) / 4, Tw = (g.Wg + 3) / 4;
  const long long T = (long long)g.nimg * Th * Tw;
  float* V = reinterpret_cast<float*>(a.wino_ws);
  const long long nw = (long long)a.N * g.Cg;
  const int NB = a.N / 64;
  const long long G = (T + 31) / 32 * NB;
  hipLaunchKernelGGL(k_wino4f_w8, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
  static const int abl = ablation_env("UNET_WF64_ABL");
  switch (abl) {
#define WF64(A) \
  case A: hipLaunchKernelGGL(k_wino4f64<A>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e); break;
    WF64(1) WF64(2) WF64(4) WF64(8) WF64(6) WF64(3) WF64(16) WF64(20) WF64(18) WF64(7) WF64(15)
#undef WF64
    default: hipLaunchKernelGGL(k_wino4f64<0>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e);
  }
  return hipGetLastError();
}



// ---------------------------------------------------------------------------
// k_wino4f64p: tile 76 = tile 73's arithmetic (the same operands, the same
// per-point accumulation order: bit-identical outputs) on a software-pipelined
// chunk loop.  Round-5 ablations of tile 73 (fp32 bench, 12 launch sites,
// profiles/r05_wino4f64_ablation.txt): without its MFMAs the two GEMM classes
// lose 2.18 ms, without the patch loads 0.67 ms, without the transform
// arithmetic 0.12 ms, without all of those and the output stage 4.07 of the
// kernel's ~5.7 ms.  Tile 73 fills its LDS between two barriers while no MFMA
// runs: V (74 KB per chunk from L2) is DMA'd during the transform, the patch
// loads are retired by a full vmcnt, so the L2 -> LDS transfer of every chunk
// is serialised with its MFMAs.  Here every global -> LDS transfer is an
// LDS-DMA retired by counted vmcnt waits (no compiler-tracked load in the loop):
//   * the 18 patch values of a thread land in a per-wave raw area (dword DMA,
//     lane-contiguous rows) one chunk ahead; the BatchNorm scale / shift of
//     every input channel sits in an LDS table;
//   * V is split into half A (points 0-15, 32 KB) and half B (points 16-35,
//     40 KB), each refilled for the next chunk as soon as the MFMAs of its
//     points are done: 4 + 5 pieces of 1 KB per wave and chunk;
//   * per chunk: commit (raw -> BN+ReLU -> B^T d B -> U), barrier, MFMAs of
//     points 0-15, barrier, V(next) half A, MFMAs of points 16-35, barrier,
//     V(next) half B.
// Per wave and chunk the DMAs are issued in the order raw(k+1) [18], VA(k+1)
// [4], VB(k+1) [5], so the waits are constant: raw(k) before the commit
// (vmcnt 9), VA(k) before the first barrier (23), VB(k) before the second (18).
// The last chunk re-issues its own transfers (same counts; never read).
// LDS: U 38 KB + V 72 KB + raw 36 KB + BN table 8 KB = 153 KB, one workgroup
// per CU as tile 73.
// ---------------------------------------------------------------------------
constexpr int kWf64pMaxCg = 1024;

__global__ __launch_bounds__(512, 1) void k_wino4f64p(Gather g, const float* __restrict__ V, int N, long long T,
                                                      int Th, int Tw, int NB, Epilogue e) {
  constexpr int PU = 32 * 8 + 8, PV = 64 * 8;
  constexpr int PA = 16;  // points of V half A
  constexpr int U_F = 36 * PU, VA_F = PA * PV, VB_F = (36 - PA) * PV, RAW_F = 8 * 18 * 64;
  __shared__ __attribute__((aligned(16))) float lds[U_F + VA_F + VB_F + RAW_F + 2 * kWf64pMaxCg];
  float* Us = lds;
  float* VAs = lds + U_F;
  float* VBs = VAs + VA_F;
  float* raws = VBs + VB_F;
  float* ss = raws + RAW_F;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long bid = blockIdx.x;
  const long long G = gridDim.x;
  if ((G & 7) == 0) bid = (bid & 7) * (G >> 3) + (bid >> 3);  // an XCD's workgroups share tiles
  const int nb = (int)(bid % NB);
  const long long t0 = (bid / NB) * 32;
  const int n0 = nb * 64;
  const int Cg = g.Cg, nk = Cg >> 3;

  // ---- loader role: patch (tile lt, channel lc), column half hf (tile 73) ----
  const int hf = (lane >> 4) & 1;
  const int pt = wave * 32 + (lane & 15) + ((lane >> 5) << 4);
  const int lt = pt >> 3, lc = pt & 7;
  const long long t = t0 + lt;
  int img = 0, ty = 0, tx = 0;
  if (t < T) {
    tx = (int)(t % Tw);
    const long long r = t / Tw;
    ty = (int)(r % Th);
    img = (int)(r / Th);
  }
  const int vrows = t < T ? min(6, g.Hg + 2 - 4 * ty) : 0;
  const int vcols = t < T ? min(6, g.Wg + 2 - 4 * tx) : 0;
  const bool wfull = __all(vrows == 6 && vcols == 6);
  float* const ubase = Us + (3 * hf) * 6 * PU + lt * 8 + wf8_slot(lt, lc & 3) + (lc >> 2);

  // the consumer BatchNorm+ReLU table (scale | shift) of the concatenated channels
  const bool tf0 = g.s[0].scale != nullptr, tf1 = g.c_split < Cg && g.s[1].scale != nullptr;
  if (tf0 || tf1) {
    for (int c = tid; c < Cg; c += 512) {
      const bool sec = c >= g.c_split;
      const float* scp = sec ? g.s[1].scale : g.s[0].scale;
      const float* shp = sec ? g.s[1].shift : g.s[0].shift;
      const int cl = sec ? c - g.c_split : c;
      ss[c] = scp ? scp[cl] : 1.f;
      ss[kWf64pMaxCg + c] = scp ? shp[cl] : 0.f;
    }
  }

  const unsigned raw_lds = (unsigned)(size_t)(lds_u8_t*)raws + (unsigned)wave * (18u * 256u);
  auto issue_raw = [&](int kc) {  // 18 dword DMAs: raw[yy][xx] -> raw area row yy * 3 + xx
    const bool second = kc * 8 >= g.c_split;  // c_split % 8 == 0: uniform source
    const unsigned long long sb = uniform_u64(second ? g.s[1].ptr : g.s[0].ptr);
    const int sH = second ? g.s[1].H : g.s[0].H, sW = second ? g.s[1].W : g.s[0].W;
    const int sC = second ? g.s[1].C : g.s[0].C;
    const int soy = second ? g.s[1].oy : g.s[0].oy, sox = second ? g.s[1].ox : g.s[0].ox;
    const int cl = kc * 8 - (second ? g.c_split : 0) + lc;
    const unsigned o0 = ((unsigned)((img * sH + 4 * ty + soy) * sW + 4 * tx + sox) * sC + cl) * 4u;
    const unsigned rs = (unsigned)sW * sC * 4u, cs = (unsigned)sC * 4u;
    if (wfull) {
      const unsigned oh = o0 + 3u * hf * cs;
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int xx = 0; xx < 3; ++xx) dma4_sv(oh + (yy * rs + xx * cs), sb, raw_lds + (yy * 3 + xx) * 256u);
    } else {  // clamp to the last in-window row / column (zeroed in commit)
      const unsigned lr = (unsigned)max(vrows - 1, 0), lcn = (unsigned)max(vcols - 1, 0);
#pragma unroll
      for (int yy = 0; yy < 6; ++yy)
#pragma unroll
        for (int xx = 0; xx < 3; ++xx)
          dma4_sv(o0 + (min((unsigned)yy, lr) * rs + min((unsigned)(3 * hf + xx), lcn) * cs), sb,
                  raw_lds + (yy * 3 + xx) * 256u);
    }
  };
  // V (k_wino4f_w8 layout [Cg/8][36][N][8]: 2 KB per point for 64 columns):
  // half A = points 0-15 as 32 pieces of 1 KB, 4 per wave; half B = points
  // 16-35, 40 pieces, 5 per wave
  const unsigned long long vbase = uniform_u64(V);
  const unsigned va_lds = (unsigned)(size_t)(lds_u8_t*)VAs, vb_lds = (unsigned)(size_t)(lds_u8_t*)VBs;
  auto issue_v = [&](int kc, int half) {
    const int np = half ? 5 : 4, p0 = half ? PA : 0;
    const unsigned dst = half ? vb_lds : va_lds;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (j < np) {
        const int pc = wave + 8 * j;  // piece: point p0 + (pc >> 1), 1-KB half pc & 1
        dma_sv((unsigned)((((size_t)kc * 36 + p0 + (pc >> 1)) * N + n0) * 32) + (unsigned)((pc & 1) * 1024 + lane * 16),
               vbase, dst + (unsigned)((pc >> 1) * PV * 4 + (pc & 1) * 1024));
      }
    }
  };
  auto commit = [&](int kc) {
    vm_wait<9>();  // raw(kc) landed (VA(kc), VB(kc) may still be in flight)
    float raw[18];
#pragma unroll
    for (int q = 0; q < 18; ++q) raw[q] = raws[wave * (18 * 64) + q * 64 + lane];
    lgkm_wait0();  // the raw area is read before its refill is issued
    issue_raw(kc + 1 < nk ? kc + 1 : kc);
    const bool second = kc * 8 >= g.c_split;
    const bool tf = second ? tf1 : tf0;
    if (tf) {
      const float sc = ss[kc * 8 + lc], sh = ss[kWf64pMaxCg + kc * 8 + lc];
#pragma unroll
      for (int q = 0; q < 18; ++q) raw[q] = fmaxf(fmaf(raw[q], sc, sh), 0.f);
    }
    if (!wfull) {
#pragma unroll
      for (int q = 0; q < 18; ++q) raw[q] = (q / 3 < vrows && 3 * hf + q % 3 < vcols) ? raw[q] : 0.f;
    }
#pragma unroll
    for (int xx = 0; xx < 3; ++xx) {  // columns in place: raw[a][xx] = (B^T d)[a][3 hf + xx]
      float d[6];
#pragma unroll
      for (int yy = 0; yy < 6; ++yy) d[yy] = raw[yy * 3 + xx];
      float rr[6];
      bt6(d, rr);
#pragma unroll
      for (int a = 0; a < 6; ++a) raw[a * 3 + xx] = rr[a];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(raw[k]), __float_as_uint(raw[9 + k]),
                                                       false, false);
      raw[k] = __uint_as_float(sw[0]);
      raw[9 + k] = __uint_as_float(sw[1]);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float d[6] = {raw[a * 3 + 0], raw[a * 3 + 1], raw[a * 3 + 2],
                          raw[9 + a * 3 + 0], raw[9 + a * 3 + 1], raw[9 + a * 3 + 2]};
      float rr[6];
      bt6(d, rr);
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) ubase[(a * 6 + bb) * PU] = rr[bb];
    }
  };

  // ---- MFMA role: wave = (tile half th, 16-channel block cb), all 36 points (tile 73) ----
  const int th = wave & 1, cb = wave >> 1;
  const int mi = lane & 15, mq = lane >> 4;
  const int aoff = (16 * th + mi) * 8 + wf8_slot(16 * th + mi, mq);
  const int boff = (16 * cb + mi) * 8 + wf8_slot(mi, mq);
  floatx4 acc[36];
#pragma unroll
  for (int p = 0; p < 36; ++p) acc[p] = (floatx4){0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // BN table
  issue_raw(0);
  issue_v(0, 0);
  issue_v(0, 1);
  for (int kc = 0; kc < nk; ++kc) {
    const int kn = kc + 1 < nk ? kc + 1 : kc;
    commit(kc);
    vm_wait<23>();  // VA(kc) landed (VB(kc) and raw(kc + 1) may be in flight)
    lgkm_wait0();   // U stores
    raw_barrier();
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const float2 a = *reinterpret_cast<const float2*>(Us + p * PU + aoff);
      const float2 b = *reinterpret_cast<const float2*>(VAs + p * PV + boff);
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.x, a.x, acc[p], 0, 0, 0);
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.y, a.y, acc[p], 0, 0, 0);
    }
    vm_wait<18>();  // VB(kc) landed (raw(kc + 1) may be in flight)
    lgkm_wait0();
    raw_barrier();  // every wave is past its half-A reads
    issue_v(kn, 0);
#pragma unroll
    for (int p = PA; p < 36; ++p) {
      const float2 a = *reinterpret_cast<const float2*>(Us + p * PU + aoff);
      const float2 b = *reinterpret_cast<const float2*>(VBs + (p - PA) * PV + boff);
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.x, a.x, acc[p], 0, 0, 0);
      acc[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.y, a.y, acc[p], 0, 0, 0);
    }
    lgkm_wait0();
    raw_barrier();  // every wave is past its U and half-B reads
    issue_v(kn, 1);
  }
  vm_wait<0>();  // the last chunk's re-issued transfers, before the output stage reuses the LDS
  __syncthreads();
  wf64_output(acc, g, e, N, T, Th, Tw, t0, n0, th, cb, mi, mq, lane, wave, lds);
}

bool wino_fused64p_applies(const IgemmArgs& a) { return wino_fused64_applies(a) && a.a.Cg <= kWf64pMaxCg; }

hipError_t launch_wino_fused64p(const IgemmArgs& a, hipStream_t s) {
  if (!wino_fused64p_applies(a)) return hipErrorInvalidValue;
  const Gather& g = a.a;
  const int Th = (g.Hg + 3) / 4, Tw = (g.Wg + 3) / 4;
  const long long T = (long long)g.nimg * Th * Tw;
  float* V = reinterpret_cast<float*>(a.wino_ws);
  const long long nw = (long long)a.N * g.Cg;
  const int NB = a.N / 64;
  const long long G = (T + 31) / 32 * NB;
  hipLaunchKernelGGL(k_wino4f_w8, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
  hipLaunchKernelGGL(k_wino4f64p, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_wino2f64: fused Winograd F(2x2, 3x3), 64 output channels x 64 tiles per
// workgroup (igemm tile 75, round 4).  The 64-channel forwards (inc.c1, up4.c1)
// ran direct (k_conv3_f32, ~73 % MFMA busy, 1.9 ms of the fp32 step) because
// F(4x4)'s rounding on them sits at the every-element parity bar;
// F(2x2)'s transforms are exact in their +-1 / 1/2 coefficients and its error
// is the direct sum's order (r03 sweep: 0.56 of the bar with F(2x2) forwards),
// at 16 point products per 2x2 outputs = 4/9 of the direct MFMA work.
// Structure of k_wino4f64 with 4x4 patches:
//   * per 8-channel chunk a thread owns one (tile, channel) patch: 16 loads
//     (the next chunk's issued before this chunk's MFMAs), the producer's
//     BN+ReLU, B^T d B (24 adds), 16 points into U[p][tile][8] in LDS; V (the
//     chunk's 16 x 64 x 8 transformed weights, k_wino2f_w8) goes through
//     registers into LDS too;
//   * wave w: tile quarter w & 3, output-channel half w >> 2 (two 16-channel
//     blocks): per point one U read, two V reads, four v_mfma_f32_16x16x4_f32;
//     lane (mi, mq) ends with all 16 points of channels 4 mq .. +3 of tile mi
//     for each block: A^T M A and the epilogue from registers, 16-B stores.
// ---------------------------------------------------------------------------
__global__ void k_wino2f_w8(const float* __restrict__ b, int N, int Cg, float* __restrict__ v) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)N * Cg) return;
  const int n = (int)(i / Cg), c = (int)(i - (long long)n * Cg);
  float g[3][3];
#pragma unroll
  for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = b[((size_t)n * 9 + t) * Cg + c];
  float tg[4][3];  // G g (k_wino_w's G)
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    tg[0][k] = g[0][k];
    tg[1][k] = 0.5f * (g[0][k] + g[1][k] + g[2][k]);
    tg[2][k] = 0.5f * (g[0][k] - g[1][k] + g[2][k]);
    tg[3][k] = g[2][k];
  }
  const size_t base = (size_t)(c >> 3) * 16 * N;
  const int pos = wf8_slot(n, c & 3) + ((c >> 2) & 1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float w4[4] = {tg[r][0], 0.5f * (tg[r][0] + tg[r][1] + tg[r][2]), 0.5f * (tg[r][0] - tg[r][1] + tg[r][2]),
                         tg[r][2]};
#pragma unroll
    for (int q = 0; q < 4; ++q) v[(base + (size_t)(r * 4 + q) * N + n) * 8 + pos] = w4[q];
  }
}

// NC: output columns per workgroup.  64 (tile 75): one workgroup per CU (128
// accumulator VGPRs per lane).  32 (tile 77, round 5): half the accumulators
// and V, two workgroups per CU, so one workgroup's loads, transforms and
// epilogue overlap the other's MFMAs (tile 75 waits 45 % of its wave cycles,
// profiles/r05_pmc_summary_fp32.txt); the input transform is then done per
// 32 output columns -- cheap in F(2x2) (24 adds per patch).
template <int NC>
__global__ __launch_bounds__(512, NC == 32 ? 2 : 1) void k_wino2f64(Gather g, const float* __restrict__ V, int N,
                                                                   long long T, int Th, int Tw, int NB, Epilogue e) {
  constexpr int TT = 64;      // tiles per workgroup
  constexpr int PU = TT * 8;  // U point plane
  constexpr int PV = NC * 8;  // V point plane
  constexpr int NJ = NC / 32;  // 16-column blocks per wave
  __shared__ __attribute__((aligned(16))) float lds[16 * PU + 16 * PV];
  float* Us = lds;
  float* Vs = lds + 16 * PU;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long bid = blockIdx.x;
  const long long G = gridDim.x;
  if ((G & 7) == 0) bid = (bid & 7) * (G >> 3) + (bid >> 3);  // an XCD's workgroups share tiles
  const int nb = (int)(bid % NB);
  const long long t0 = (bid / NB) * TT;
  const int n0 = nb * NC;

  // ---- loader role: patch (tile lt, channel lc) ----
  const int lt = tid >> 3, lc = tid & 7;
  const long long t = t0 + lt;
  int img = 0, ty = 0, tx = 0;
  if (t < T) {
    tx = (int)(t % Tw);
    const long long r = t / Tw;
    ty = (int)(r % Th);
    img = (int)(r / Th);
  }
  // rows / columns of the 4x4 patch inside the gather's input grid (Hg+2, Wg+2)
  const int vrows = t < T ? min(4, g.Hg + 2 - 2 * ty) : 0;
  const int vcols = t < T ? min(4, g.Wg + 2 - 2 * tx) : 0;
  const bool wfull = __all(vrows == 4 && vcols == 4);
  float* const ubase = Us + lt * 8 + wf8_slot(lt, lc & 3) + (lc >> 2);
  float raw[16];
  float sc = 1.f, sh = 0.f;  // the chunk's producer BN+ReLU (loaded with raw)
  const int nk = g.Cg >> 3;
  // V (16 points x NC / 32 KB per chunk) by LDS-DMA during the input transform,
  // 4 (NC 64) or 2 (NC 32) x 1 KB per wave (as k_wino4f64)
  const unsigned long long vbase = uniform_u64(V);
  const unsigned vlds = (unsigned)(size_t)(lds_u8_t*)lds + (unsigned)(16 * PU * 4);
  auto load = [&](int kc) {
    const bool second = kc * 8 >= g.c_split;  // c_split % 8 == 0: uniform source
    const float* sp = second ? g.s[1].ptr : g.s[0].ptr;
    const int sH = second ? g.s[1].H : g.s[0].H, sW = second ? g.s[1].W : g.s[0].W;
    const int sC = second ? g.s[1].C : g.s[0].C;
    const int soy = second ? g.s[1].oy : g.s[0].oy, sox = second ? g.s[1].ox : g.s[0].ox;
    const int cl = kc * 8 - (second ? g.c_split : 0) + lc;
    const float* scp = second ? g.s[1].scale : g.s[0].scale;
    if (scp) {
      sc = scp[cl];
      sh = (second ? g.s[1].shift : g.s[0].shift)[cl];
    }
    const char* sb = reinterpret_cast<const char*>(sp);
    const unsigned o0 = ((unsigned)((img * sH + 2 * ty + soy) * sW + 2 * tx + sox) * sC + cl) * 4u;
    const unsigned rs = (unsigned)sW * sC * 4u, cs = (unsigned)sC * 4u;
    if (wfull) {
#pragma unroll
      for (int yy = 0; yy < 4; ++yy)
#pragma unroll
        for (int xx = 0; xx < 4; ++xx)
          raw[yy * 4 + xx] = *reinterpret_cast<const float*>(sb + (o0 + (yy * rs + xx * cs)));
    } else {  // clamp to the last in-window row / column (zeroed in commit)
      const unsigned lr = (unsigned)max(vrows - 1, 0), lcn = (unsigned)max(vcols - 1, 0);
#pragma unroll
      for (int yy = 0; yy < 4; ++yy)
#pragma unroll
        for (int xx = 0; xx < 4; ++xx)
          raw[yy * 4 + xx] = *reinterpret_cast<const float*>(
              sb + (o0 + (min((unsigned)yy, lr) * rs + min((unsigned)xx, lcn) * cs)));
    }
  };
  auto commit = [&](int kc) {
    const bool second = kc * 8 >= g.c_split;
    const float* scp = second ? g.s[1].scale : g.s[0].scale;
    __builtin_amdgcn_s_waitcnt(0x0F70);  // raw(kc), sc, sh: retired visibly before the DMAs queue
#pragma unroll
    for (int j = 0; j < 2 * NJ; ++j) {
      const int pc = wave + 8 * j;  // 1-KB piece: point pc / NJ, part pc % NJ
      dma_sv((unsigned)((((size_t)kc * 16 + pc / NJ) * N + n0) * 32) + (unsigned)((pc % NJ) * 1024 + lane * 16),
             vbase, vlds + (unsigned)((pc / NJ) * PV * 4 + (pc % NJ) * 1024));
    }
    if (scp) {
#pragma unroll
      for (int q = 0; q < 16; ++q) raw[q] = fmaxf(fmaf(raw[q], sc, sh), 0.f);
    }
    if (!wfull) {
#pragma unroll
      for (int q = 0; q < 16; ++q) raw[q] = (q / 4 < vrows && q % 4 < vcols) ? raw[q] : 0.f;
    }
    // B^T d (rows), then (.) B (columns): k_wino_in's transform
    float ev[4][4];
#pragma unroll
    for (int xx = 0; xx < 4; ++xx) {
      ev[0][xx] = raw[0 * 4 + xx] - raw[2 * 4 + xx];
      ev[1][xx] = raw[1 * 4 + xx] + raw[2 * 4 + xx];
      ev[2][xx] = raw[2 * 4 + xx] - raw[1 * 4 + xx];
      ev[3][xx] = raw[1 * 4 + xx] - raw[3 * 4 + xx];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      ubase[(a * 4 + 0) * PU] = ev[a][0] - ev[a][2];
      ubase[(a * 4 + 1) * PU] = ev[a][1] + ev[a][2];
      ubase[(a * 4 + 2) * PU] = ev[a][2] - ev[a][1];
      ubase[(a * 4 + 3) * PU] = ev[a][1] - ev[a][3];
    }
    vm_wait<0>();  // V(kc) landed
  };

  // ---- MFMA role: wave = (tile quarter th, channel half ch), all 16 points ----
  const int th = wave & 3, ch = wave >> 2;
  const int mi = lane & 15, mq = lane >> 4;
  const int aoff = (16 * th + mi) * 8 + wf8_slot(16 * th + mi, mq);
  const int boff = (16 * NJ * ch + mi) * 8 + wf8_slot(mi, mq);  // rows 16 (NJ ch + j) + mi and mi agree on bits 2-3
  floatx4 acc[16][NJ];
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[p][j] = (floatx4){0.f, 0.f, 0.f, 0.f};
  load(0);
  for (int kc = 0; kc < nk; ++kc) {
    commit(kc);
    __syncthreads();
    if (kc + 1 < nk) load(kc + 1);
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const float2 a = *reinterpret_cast<const float2*>(Us + p * PU + aoff);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float2 b = *reinterpret_cast<const float2*>(Vs + p * PV + boff + 16 * j * 8);
        acc[p][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.x, a.x, acc[p][j], 0, 0, 0);
        acc[p][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b.y, a.y, acc[p][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- output: tile 16 th + mi, channels n0 + 16 (NJ ch + j) + 4 mq + (0..3) ----
  const long long tt = t0 + 16 * th + mi;
  const bool want = e.stats || e.yref || e.colsum1;
  const int nsplit = e.n_split < N ? e.n_split : N;
  const int grp = blockIdx.x % kStatGroups;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col0 = n0 + 16 * NJ * ch + 16 * j + 4 * mq;
    const bool second = col0 >= e.n_split;  // uniform per 16-channel block (n_split % 16 == 0)
    float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
    const int dC = second ? e.d[1].C : e.d[0].C;
    const int dcol = second ? col0 - e.n_split : col0;
    const bool bwd_mask = e.yref != nullptr && !second;
    const float4 bias = e.bias ? ld4(e.bias + col0) : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 bsc = make_float4(0.f, 0.f, 0.f, 0.f), bsh = bsc, bmu = bsc, bis = bsc;
    if (bwd_mask) { bsc = ld4(e.bn_scale + col0); bsh = ld4(e.bn_shift + col0); bmu = ld4(e.bn_mean + col0); bis = ld4(e.bn_invstd + col0); }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    if (tt < T) {
      const int ox = (int)(tt % Tw);
      const long long rq = tt / Tw;
      const int oy = (int)(rq % Th), on = (int)(rq / Th);
      float4 y4[4];  // mask operands first, one wait (k_wino4f64)
      if (bwd_mask) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) {
            const int y = min(2 * oy + a, g.Hg - 1), x = min(2 * ox + bb, g.Wg - 1);
            y4[a * 2 + bb] = ld4(e.yref + ((size_t)(on * g.Hg + y) * g.Wg + x) * dC + dcol);
          }
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) once: see k_wino4f64's epilogue
      float o[4][2][2];  // [channel][row][col] = A^T M A
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float w[2][4];
#pragma unroll
        for (int xx = 0; xx < 4; ++xx) {
          const float m0 = acc[0 * 4 + xx][j][r], m1 = acc[1 * 4 + xx][j][r];
          const float m2 = acc[2 * 4 + xx][j][r], m3 = acc[3 * 4 + xx][j][r];
          w[0][xx] = m0 + m1 + m2;
          w[1][xx] = m1 - m2 - m3;
        }
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          o[r][a][0] = w[a][0] + w[a][1] + w[a][2];
          o[r][a][1] = w[a][1] - w[a][2] - w[a][3];
        }
      }
      const float bsv[4] = {bias.x, bias.y, bias.z, bias.w};
      const float scv[4] = {bsc.x, bsc.y, bsc.z, bsc.w}, shv[4] = {bsh.x, bsh.y, bsh.z, bsh.w};
      const float muv[4] = {bmu.x, bmu.y, bmu.z, bmu.w}, isv[4] = {bis.x, bis.y, bis.z, bis.w};
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int y = 2 * oy + a;
        if (y >= g.Hg) continue;
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int x = 2 * ox + bb;
          if (x >= g.Wg) continue;
          const size_t idx = ((size_t)(on * g.Hg + y) * g.Wg + x) * dC + dcol;
          const float4 yq = bwd_mask ? y4[a * 2 + bb] : make_float4(0.f, 0.f, 0.f, 0.f);
          const float yv[4] = {yq.x, yq.y, yq.z, yq.w};
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = wf_epi(o[r][a][bb] + bsv[r], yv[r], scv[r], shv[r], muv[r], isv[r],
                                                     bwd_mask, e.relu, s1[r], s2[r]);
          st4(dptr + idx, make_float4(v[0], v[1], v[2], v[3]));
        }
      }
    }
    if (!want) continue;
    // the 16 lanes of a quarter hold the same 4 channels (other tiles)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o2 = 1; o2 < 16; o2 <<= 1) {
        s1[r] += __shfl_xor(s1[r], o2);
        s2[r] += __shfl_xor(s2[r], o2);
      }
    if (mi == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = col0 + r;
        if (col < nsplit) {
          double* st = e.yref ? e.bstats : e.stats;
          if (st) {
            atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 0, (double)s1[r]);
            atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 1, (double)s2[r]);
          }
        } else if (e.colsum1) {
          atomicAdd(e.colsum1 + (size_t)grp * (N - nsplit) + (col - nsplit), (double)s1[r]);
        }
      }
    }
  }
}

bool wino_fused2_applies(const IgemmArgs& a, int nc) {
  const Gather& g = a.a;
  if (a.b == nullptr || a.bh != nullptr || a.batch != 1) return false;
  if (g.taps_h != 3 || g.taps_w != 3 || g.stride != 1 || a.K != 9 * g.Cg || g.Cg % 8 != 0 || g.c_split % 8 != 0 ||
      a.N % nc != 0 || (a.e.n_split < a.N && a.e.n_split % 16 != 0))
    return false;
  if (g.s[0].h16 || g.s[1].h16 || a.e.shuffle_co || a.e.d[0].h16 || a.e.d[1].h16 || a.e.yref_h16) return false;
  if (a.e.d[0].oy || a.e.d[0].ox || a.e.d[0].H != g.Hg || a.e.d[0].W != g.Wg) return false;
  if (a.e.n_split < a.N && (a.e.d[1].oy || a.e.d[1].ox || a.e.d[1].H != g.Hg || a.e.d[1].W != g.Wg)) return false;
  for (int k = 0; k < 2; ++k)  // 32-bit byte offsets into the sources
    if ((long long)g.nimg * g.s[k].H * g.s[k].W * g.s[k].C * 4 >= (1ll << 32)) return false;
  const long long T = (long long)g.nimg * ((g.Hg + 1) / 2) * ((g.Wg + 1) / 2);
  if ((T + 63) / 64 * (a.N / nc) > 0x7fffffffLL) return false;
  return a.wino_ws != nullptr && (size_t)16 * a.N * g.Cg * 4 <= a.wino_ws_bytes;
}

hipError_t launch_wino_fused2(const IgemmArgs& a, hipStream_t s, int nc) {
  if ((nc != 64 && nc != 32) || !wino_fused2_applies(a, nc)) return hipErrorInvalidValue;
  const Gather& g = a.a;
  const int Th = (g.Hg + 1) / 2, Tw = (g.Wg + 1) / 2;
  const long long T = (long long)g.nimg * Th * Tw;
  float* V = reinterpret_cast<float*>(a.wino_ws);
  const long long nw = (long long)a.N * g.Cg;
  const int NB = a.N / nc;
  const long long G = (T + 63) / 64 * NB;
  hipLaunchKernelGGL(k_wino2f_w8, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
  if (nc == 64)
    hipLaunchKernelGGL(k_wino2f64<64>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e);
  else
    hipLaunchKernelGGL(k_wino2f64<32>, dim3((unsigned)G), dim3(512), 0, s, g, (const float*)V, a.N, T, Th, Tw, NB, a.e);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Weight gradient, F(4x4, 3x3) (wgrad tile 71).  The forward bilinear form
// sum_p (A y)_p (G g)_p (B^T d)_p gives, differentiated by g,
//   dW = G^T [ sum_tiles (A dY A^T) . (B^T X B) ] G,
// so per output tile of dY (4x4) and its 6x6 input patch the reduction over
// tiles is 36 independent GEMMs  Mw[p][co][ci] = sum_t Vd[p][t][co] U[p][t][ci]
// (k_wgrad batched over p, pixel split over t): 36/16 MACs per output pixel
// instead of 9.  U is the forward's input transform (same gather, BN + ReLU on
// load), Vd the dY transform below, dW[co][tap][ci] = G^T Mw[co][ci] G.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void a6(const float (&y)[4], float (&r)[6]) {  // A = (A^T)^T
  r[0] = y[0];
  r[1] = y[0] + y[1] + y[2] + y[3];
  r[2] = y[0] - y[1] + y[2] - y[3];
  r[3] = y[0] + 2.f * y[1] + 4.f * y[2] + 8.f * y[3];
  r[4] = y[0] - 0.5f * y[1] + 0.25f * y[2] - 0.125f * y[3];
  r[5] = y[3];
}
__device__ __forceinline__ void gt3(const float (&m)[6], float (&r)[3]) {  // G^T
  r[0] = m[0] + (m[2] - m[1]) * (1.f / 3.f) + (m[3] - 16.f * m[4]) * (1.f / 15.f);
  r[1] = -(m[1] + m[2]) * (1.f / 3.f) + (2.f * m[3] + 8.f * m[4]) * (1.f / 15.f);
  r[2] = (m[2] - m[1]) * (1.f / 3.f) + (4.f * m[3] - 4.f * m[4]) * (1.f / 15.f) + m[5];
}

// Vd[p][t][co], one (tile, channel) per thread; dY outside the Hg x Wg grid is 0
__global__ __launch_bounds__(256) void k_wino4_dy(Src dy, int Hg, int Wg, int Th, int Tw, long long T, int Co,
                                                  float* __restrict__ vd) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= T * Co) return;
  const long long t = i / Co;
  const int c = (int)(i - t * Co);
  const int tx = (int)(t % Tw);
  const long long r = t / Tw;
  const int ty = (int)(r % Th), n = (int)(r / Th);
  float e[6][4];
#pragma unroll
  for (int xx = 0; xx < 4; ++xx) {
    float d[4];
#pragma unroll
    for (int yy = 0; yy < 4; ++yy) {
      const int y = 4 * ty + yy, x = 4 * tx + xx;
      const bool in = y < Hg && x < Wg;
      const float v = dy.ptr[((size_t)(n * dy.H + (in ? y : 0) + dy.oy) * dy.W + (in ? x : 0) + dy.ox) * dy.C + c];
      d[yy] = in ? v : 0.f;
    }
    float rr[6];
    a6(d, rr);
#pragma unroll
    for (int a = 0; a < 6; ++a) e[a][xx] = rr[a];
  }
  const size_t plane = (size_t)T * Co, o = (size_t)t * Co + c;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float rr[6];
    a6(e[a], rr);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) vd[(a * 6 + bb) * plane + o] = rr[bb];
  }
}

// out[co][ky*3+kx][ci] = (G^T Mw[.][co][ci] G)[ky][kx]; the only writer of out
__global__ __launch_bounds__(256) void k_wino4_wout(const float* __restrict__ mw, int Co, int Ci,
                                                    float* __restrict__ out) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)Co * Ci) return;
  const int co = (int)(i / Ci), ci = (int)(i - (long long)co * Ci);
  const size_t plane = (size_t)Co * Ci;
  float w[3][6];
#pragma unroll
  for (int bb = 0; bb < 6; ++bb) {
    float m[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) m[a] = mw[(a * 6 + bb) * plane + i];
    float r[3];
    gt3(m, r);
#pragma unroll
    for (int k = 0; k < 3; ++k) w[k][bb] = r[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float r[3];
    gt3(w[k], r);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) out[((size_t)co * 9 + k * 3 + kx) * Ci + ci] = r[kx];
  }
}

// F(6x6) weight-gradient transforms (wgrad tile 74): Vd = A dY A^T with
// A = (A^T of at6)^T (8x6), dW = G^T Mw G with G of g8 (8x3)
__device__ __forceinline__ void a8(const float (&y)[6], float (&r)[8]) {
  constexpr float A[8][6] = {{1, 0, 0, 0, 0, 0},
                             {1, 1, 1, 1, 1, 1},
                             {1, -1, 1, -1, 1, -1},
                             {1, 2, 4, 8, 16, 32},
                             {1, -2, 4, -8, 16, -32},
                             {1, 0.5f, 0.25f, 0.125f, 0.0625f, 0.03125f},
                             {1, -0.5f, 0.25f, -0.125f, 0.0625f, -0.03125f},
                             {0, 0, 0, 0, 0, 1}};
  mat_apply(A, y, r);
}
__device__ __forceinline__ void gt8(const float (&m)[8], float (&r)[3]) {
  constexpr float GT[3][8] = {{1, -2.f / 9, -2.f / 9, 1.f / 90, 1.f / 90, 32.f / 45, 32.f / 45, 0},
                              {0, -2.f / 9, 2.f / 9, 1.f / 45, -1.f / 45, 16.f / 45, -16.f / 45, 0},
                              {0, -2.f / 9, -2.f / 9, 2.f / 45, 2.f / 45, 8.f / 45, 8.f / 45, 1}};
  mat_apply(GT, m, r);
}

// Thread = (tile, V output channels): 6x6 dY patch by clamped unconditional
// vector loads from a per-thread base (32-bit offsets), 64 points out as V-wide
// stores (32-bit plane offsets: wino_wgrad_applies)
template <int V>
__global__ __launch_bounds__(256) void k_wino6_dy(Src dy, int Hg, int Wg, int Th, int Tw, long long T, int Co,
                                                  float* __restrict__ vd) {
  typedef float vec __attribute__((ext_vector_type(V)));
  const int CV = Co / V;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= T * CV) return;
  const long long t = i / CV;
  const int c = (int)(i - t * CV) * V;
  const int tx = (int)(t % Tw);
  const long long r = t / Tw;
  const int ty = (int)(r % Th), n = (int)(r / Th);
  const int vr = min(6, Hg - 6 * ty), vc = min(6, Wg - 6 * tx);
  const char* base = reinterpret_cast<const char*>(dy.ptr) +
                     (((size_t)(n * dy.H + 6 * ty + dy.oy) * dy.W + 6 * tx + dy.ox) * dy.C + c) * 4;
  const unsigned rs = (unsigned)dy.W * dy.C * 4u, cs = (unsigned)dy.C * 4u;
  float e[V][8][6];
#pragma unroll
  for (int xx = 0; xx < 6; ++xx) {
    float d[V][6];
#pragma unroll
    for (int yy = 0; yy < 6; ++yy) {
      const bool in = yy < vr && xx < vc;
      const vec v = *reinterpret_cast<const vec*>(base + (in ? yy * rs + xx * cs : 0u));
#pragma unroll
      for (int k = 0; k < V; ++k) d[k][yy] = in ? v[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float rr[8];
      a8(d[k], rr);
#pragma unroll
      for (int a = 0; a < 8; ++a) e[k][a][xx] = rr[a];
    }
  }
  char* ob = reinterpret_cast<char*>(vd + (size_t)t * Co + c);
  const unsigned pbytes = (unsigned)((size_t)T * Co * 4);
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    float rr[V][8];
#pragma unroll
    for (int k = 0; k < V; ++k) a8(e[k][a], rr[k]);
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) {
      vec o;
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = rr[k][bb];
      *reinterpret_cast<vec*>(ob + (unsigned)(a * 8 + bb) * pbytes) = o;
    }
  }
}

// BatchNorm-backward apply fused with k_wino6_dy (fp32 plans whose weight
// gradient runs F(6x6), wgrad tile 74).  The unfused pair streams dY three
// times: k_bnb_apply reads dz and y and writes dYpad, k_wino6_dy reads dYpad
// back.  Here a thread owns one 6x6 dY tile x V channels (the tiles partition
// the grid, so every dY element has one owner): it forms
// dY = k0*dz + k1*(y - mean) + k2 with k_bnb_apply's exact expression, stores
// it into dYpad for the input gradient, writes its tile's share of dYpad's
// zero border, and transforms the values still in registers into Vd
// (k_wino6_dy's arithmetic and layout) -- dY is never read back.  BN backward:
// models/unet_model.py:12,16 (nn.BatchNorm2d in DoubleConv).
template <int V>
__global__ __launch_bounds__(256) void k_bnb_wino6_dy(const float* __restrict__ dz, const float* __restrict__ yr,
                                                      const float* __restrict__ coef, int Ho, int Wo, int Co, int Th,
                                                      int Tw, long long T, float* __restrict__ dyp,
                                                      float* __restrict__ vd) {
  typedef float vec __attribute__((ext_vector_type(V)));
  const int CV = Co / V;
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= T * CV) return;
  const long long t = i / CV;
  const int c = (int)(i - t * CV) * V;
  const int tx = (int)(t % Tw);
  const long long r = t / Tw;
  const int ty = (int)(r % Th), n = (int)(r / Th);
  const int vr = min(6, Ho - 6 * ty), vc = min(6, Wo - 6 * tx);
  const vec k0 = *reinterpret_cast<const vec*>(coef + c), k1 = *reinterpret_cast<const vec*>(coef + Co + c);
  const vec k2 = *reinterpret_cast<const vec*>(coef + 2 * Co + c), mu = *reinterpret_cast<const vec*>(coef + 3 * Co + c);
  const int Wp = Wo + 4;
  const size_t src0 = ((size_t)(n * Ho + 6 * ty) * Wo + 6 * tx) * Co + c;
  const size_t dst0 = ((size_t)(n * (Ho + 4) + 6 * ty + 2) * Wp + 6 * tx + 2) * Co + c;
  float e[V][8][6];
#pragma unroll
  for (int xx = 0; xx < 6; ++xx) {
    float d[V][6];
#pragma unroll
    for (int yy = 0; yy < 6; ++yy) {
      vec o;
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = 0.f;
      if (yy < vr && xx < vc) {
        const size_t so = src0 + ((size_t)yy * Wo + xx) * Co;
        const vec dv = *reinterpret_cast<const vec*>(dz + so), yv = *reinterpret_cast<const vec*>(yr + so);
#pragma unroll
        for (int k = 0; k < V; ++k) o[k] = fmaf(k0[k], dv[k], fmaf(k1[k], yv[k] - mu[k], k2[k]));
        *reinterpret_cast<vec*>(dyp + dst0 + ((size_t)yy * Wp + xx) * Co) = o;
      }
#pragma unroll
      for (int k = 0; k < V; ++k) d[k][yy] = o[k];
    }
#pragma unroll
    for (int k = 0; k < V; ++k) {
      float rr[8];
      a8(d[k], rr);
#pragma unroll
      for (int a = 0; a < 8; ++a) e[k][a][xx] = rr[a];
    }
  }
  float* ob = vd + (size_t)t * Co + c;
  const size_t plane = (size_t)T * Co;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    float rr[V][8];
#pragma unroll
    for (int k = 0; k < V; ++k) a8(e[k][a], rr[k]);
#pragma unroll
    for (int bb = 0; bb < 8; ++bb) {
      vec o;
#pragma unroll
      for (int k = 0; k < V; ++k) o[k] = rr[k][bb];
      *reinterpret_cast<vec*>(ob + (size_t)(a * 8 + bb) * plane) = o;
    }
  }
  // the zero border of dYpad (2 rows / columns each side): the first / last
  // tile row owns the top / bottom rows over its tiles' column span (the outer
  // tiles' spans run into the corners), the first / last tile column the left
  // / right columns beside its tile's rows
  if (ty == 0 || ty == Th - 1 || tx == 0 || tx == Tw - 1) {
    vec z;
#pragma unroll
    for (int k = 0; k < V; ++k) z[k] = 0.f;
    float* pb = dyp + (size_t)n * (Ho + 4) * Wp * Co + c;
    const int x0 = tx == 0 ? 0 : 6 * tx + 2, x1 = tx == Tw - 1 ? Wo + 4 : 6 * tx + 8;
    auto zero = [&](int py, int px) { *reinterpret_cast<vec*>(pb + ((size_t)py * Wp + px) * Co) = z; };
    if (ty == 0)
      for (int py = 0; py < 2; ++py)
        for (int px = x0; px < x1; ++px) zero(py, px);
    if (ty == Th - 1)
      for (int py = Ho + 2; py < Ho + 4; ++py)
        for (int px = x0; px < x1; ++px) zero(py, px);
    for (int py = 6 * ty + 2; py < 6 * ty + 2 + vr; ++py) {
      if (tx == 0) { zero(py, 0); zero(py, 1); }
      if (tx == Tw - 1) { zero(py, Wo + 2); zero(py, Wo + 3); }
    }
  }
}

size_t bnb_wino6_vd_bytes(int n, int h, int w, int c) {
  return (size_t)64 * n * ((h + 5) / 6) * ((w + 5) / 6) * c * sizeof(float);
}

hipError_t launch_bnb_wino6_dy(const float* dz, const float* y, const float* coef, int n, int h, int w, int c,
                               float* dypad, float* vd, hipStream_t s) {
  if (c % 64 != 0 || n < 1 || h < 1 || w < 1) return hipErrorInvalidValue;  // wino_wgrad_applies: Co % 64 == 0
  const int Th = (h + 5) / 6, Tw = (w + 5) / 6;
  const long long T = (long long)n * Th * Tw, nd = T * (c / 2);
  hipLaunchKernelGGL(k_bnb_wino6_dy<2>, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, dz, y, coef, h, w, c,
                     Th, Tw, T, dypad, vd);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_wino6_wout(const float* __restrict__ mw, int Co, int Ci,
                                                    float* __restrict__ out) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= (long long)Co * Ci) return;
  const int co = (int)(i / Ci), ci = (int)(i - (long long)co * Ci);
  const size_t plane = (size_t)Co * Ci;
  float w[3][8];
#pragma unroll
  for (int bb = 0; bb < 8; ++bb) {
    float m[8];
#pragma unroll
    for (int a = 0; a < 8; ++a) m[a] = mw[(a * 8 + bb) * plane + i];
    float r[3];
    gt8(m, r);
#pragma unroll
    for (int k = 0; k < 3; ++k) w[k][bb] = r[k];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float r[3];
    gt8(w[k], r);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) out[((size_t)co * 9 + k * 3 + kx) * Ci + ci] = r[kx];
  }
}

static long long wino_wgrad_tiles(const WgradArgs& a, int mt) {
  return (long long)a.gb.nimg * ((a.gb.Hg + mt - 1) / mt) * ((a.gb.Wg + mt - 1) / mt);
}

bool wino_wgrad_applies(const WgradArgs& a, int mt) {
  const Gather& ga = a.ga;
  const Gather& gb = a.gb;
  if (a.bf16 || a.batch != 1 || a.wino_ws == nullptr) return false;
  if (ga.taps_h != 1 || ga.taps_w != 1 || ga.stride != 1 || ga.c_split != ga.Cg || ga.s[0].h16 || ga.s[0].scale)
    return false;
  if (gb.taps_h != 3 || gb.taps_w != 3 || gb.stride != 1 || gb.s[0].h16 || gb.s[1].h16) return false;
  if (ga.Hg != gb.Hg || ga.Wg != gb.Wg || ga.nimg != gb.nimg || a.P != gb.nimg * gb.Hg * gb.Wg) return false;
  if (a.Mo != ga.Cg || a.No != 9 * gb.Cg || a.Mo % 64 != 0 || gb.Cg % 64 != 0 || gb.c_split % 4 != 0) return false;
  const long long T = wino_wgrad_tiles(a, mt);
  if ((long long)(mt + 2) * (mt + 2) * T * std::max(gb.Cg, a.Mo) * 4 >= (1ll << 32)) return false;  // 32-bit offsets
  return wino_bytes((mt + 2) * (mt + 2), T, gb.Cg, a.Mo) <= a.wino_ws_bytes;
}

// The input transform U = B^T X B alone (into the head of a.wino_ws, where
// launch_wino_wgrad with u_ready reads it): it needs only forward tensors, so
// the plan can issue it before the layer's dY exists (UNET_WGRAD_EARLY_U)
hipError_t launch_wino_wgrad_u(const WgradArgs& a, hipStream_t s, int mt) {
  if ((mt != 4 && mt != 6) || !wino_wgrad_applies(a, mt)) return hipErrorInvalidValue;
  const Gather& gb = a.gb;
  const int Th = (gb.Hg + mt - 1) / mt, Tw = (gb.Wg + mt - 1) / mt;
  const long long T = wino_wgrad_tiles(a, mt);
  if (mt == 4) launch_wino4_in(gb, Th, Tw, T, a.wino_ws, s);
  else launch_wino6_in(gb, Th, Tw, T, a.wino_ws, s);
  return hipGetLastError();
}

// mt = 4 (wgrad tile 71) or 6 (tile 74).  per_cu: workgroups per CU of the point
// GEMMs' pixel split, + 100 * (1 + k_wgrad tile id) to force their tile
// (autotuner candidates)
hipError_t launch_wino_wgrad(const WgradArgs& a, hipStream_t s, int per_cu, int mt) {
  // code = [1000: slab mode] + [100 * (point-GEMM tile + 1)] + workgroups per CU
  const bool slab = per_cu >= 1000;
  per_cu %= 1000;
  const int forced = per_cu >= 100 ? per_cu / 100 - 1 : -1;
  per_cu %= 100;
  if (per_cu <= 0) per_cu = 8;
  if ((mt != 4 && mt != 6) || !wino_wgrad_applies(a, mt)) return hipErrorInvalidValue;
  const Gather& gb = a.gb;
  const int P = (mt + 2) * (mt + 2);
  const int Th = (gb.Hg + mt - 1) / mt, Tw = (gb.Wg + mt - 1) / mt;
  const long long T = wino_wgrad_tiles(a, mt);
  const int Ci = gb.Cg, Co = a.Mo;
  if (P * T > 0x7fffffffLL) return hipErrorInvalidValue;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  char* w = reinterpret_cast<char*>(a.wino_ws);
  float* U = reinterpret_cast<float*>(w);
  float* Vd = reinterpret_cast<float*>(w + al((size_t)P * T * Ci * 4));
  float* Mw = reinterpret_cast<float*>(w + al((size_t)P * T * Ci * 4) + al((size_t)P * T * Co * 4));
  const long long nd = T * Co;
  if (mt == 4) {
    if (!a.u_ready) launch_wino4_in(gb, Th, Tw, T, U, s);
    hipLaunchKernelGGL(k_wino4_dy, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, a.ga.s[0], gb.Hg, gb.Wg, Th,
                       Tw, T, Co, Vd);
  } else {
    if (!a.u_ready) launch_wino6_in(gb, Th, Tw, T, U, s);
    if (a.vd_pre)  // written by k_bnb_wino6_dy beside dYpad (same tiles, same layout)
      Vd = const_cast<float*>(a.vd_pre);
    else
      hipLaunchKernelGGL(k_wino6_dy<2>, dim3((unsigned)((nd / 2 + 255) / 256)), dim3(256), 0, s, a.ga.s[0], gb.Hg,
                         gb.Wg, Th, Tw, T, Co, Vd);  // Co % 64 == 0 (wino_wgrad_applies)
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  {
    // the P point GEMMs Mw[p] = Vd[p]^T U[p] as one batched k_wgrad launch
    WgradArgs q;
    Src v;
    v.ptr = Vd;
    v.H = 1;
    v.W = (int)T;
    v.C = Co;
    q.ga.s[0] = q.ga.s[1] = v;
    q.ga.Cg = q.ga.c_split = Co;
    q.ga.Hg = 1;
    q.ga.Wg = (int)T;
    q.ga.nimg = 1;
    Src u = v;
    u.ptr = U;
    u.C = Ci;
    q.gb.s[0] = q.gb.s[1] = u;
    q.gb.Cg = q.gb.c_split = Ci;
    q.gb.Hg = 1;
    q.gb.Wg = (int)T;
    q.gb.nimg = 1;
    q.Mo = Co;
    q.No = Ci;
    q.P = (int)T;
    q.out = Mw;
    q.batch = P;
    q.batch_a = T * Co;
    q.batch_b = T * Ci;
    q.batch_out = (long long)Co * Ci;
    int tile = (Co % 128 == 0 && Ci % 128 == 0) ? 0 : (Ci % 128 == 0 ? 3 : 4);
    if (forced >= 0 && wgrad_tile_fits(q, forced)) tile = forced;
    // slab mode (plain-store partials, every Mw element assigned) needs no
    // zeroed accumulator; the atomics do (0.8 GB of memsets per fp32 step)
    q.slab = a.slab;
    q.slab_bytes = a.slab_bytes;
    int pps = 0;
    const bool use_slab = slab && wgrad_slab_fits(q, wgrad_splits(q, tile, per_cu, pps));
    if (slab && !use_slab) ++g_slab_fallbacks;
    if (!use_slab && (e = hipMemsetAsync(Mw, 0, (size_t)P * Co * Ci * 4, s)) != hipSuccess) return e;
    if ((e = launch_wgrad_v(q, s, GemmChoice{tile, use_slab ? per_cu + 100 : per_cu})) != hipSuccess) return e;
  }
  const long long no = (long long)Co * Ci;
  if (mt == 4)
    hipLaunchKernelGGL(k_wino4_wout, dim3((unsigned)((no + 255) / 256)), dim3(256), 0, s, Mw, Co, Ci, a.out);
  else
    hipLaunchKernelGGL(k_wino6_wout, dim3((unsigned)((no + 255) / 256)), dim3(256), 0, s, Mw, Co, Ci, a.out);
  return hipGetLastError();
}

}  // namespace unet
