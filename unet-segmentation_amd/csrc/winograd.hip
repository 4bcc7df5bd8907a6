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
#include "gemm_common.h"

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
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (y < g.Hg + 2 && x < g.Wg + 2) {
        v = ld4(s.ptr + ((size_t)(n * s.H + y + s.oy) * s.W + x + s.ox) * s.C + cl);
        if (s.scale) v = affine_relu4(v, sc, sh);
      }
      d[yy][xx] = v;
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
// transform traffic).  Interpolation points 0, +-1, +-2, inf (Lavin & Gray):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0;
//          0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6;
//          1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// One channel per thread (36 values in registers), coalesced across channels.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void bt6(const float (&d)[6], float (&r)[6]) {
  r[0] = 4.f * d[0] - 5.f * d[2] + d[4];
  r[1] = -4.f * d[1] - 4.f * d[2] + d[3] + d[4];
  r[2] = 4.f * d[1] - 4.f * d[2] - d[3] + d[4];
  r[3] = -2.f * d[1] - d[2] + 2.f * d[3] + d[4];
  r[4] = 2.f * d[1] - d[2] - 2.f * d[3] + d[4];
  r[5] = 4.f * d[1] - 5.f * d[3] + d[5];
}
__device__ __forceinline__ void g6(const float (&g)[3], float (&r)[6]) {
  r[0] = 0.25f * g[0];
  r[1] = -(g[0] + g[1] + g[2]) * (1.f / 6.f);
  r[2] = -(g[0] - g[1] + g[2]) * (1.f / 6.f);
  r[3] = g[0] * (1.f / 24.f) + g[1] * (1.f / 12.f) + g[2] * (1.f / 6.f);
  r[4] = g[0] * (1.f / 24.f) - g[1] * (1.f / 12.f) + g[2] * (1.f / 6.f);
  r[5] = g[2];
}
__device__ __forceinline__ void at4(const float (&m)[6], float (&o)[4]) {
  o[0] = m[0] + m[1] + m[2] + m[3] + m[4];
  o[1] = m[1] - m[2] + 2.f * (m[3] - m[4]);
  o[2] = m[1] + m[2] + 4.f * (m[3] + m[4]);
  o[3] = m[1] - m[2] + 8.f * (m[3] - m[4]) + m[5];
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

__global__ __launch_bounds__(256) void k_wino4_in(Gather g, int Th, int Tw, long long T, float* __restrict__ u) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= T * g.Cg) return;
  const long long t = i / g.Cg;
  const int c = (int)(i - t * g.Cg);
  const int tx = (int)(t % Tw);
  const long long r = t / Tw;
  const int ty = (int)(r % Th), n = (int)(r / Th);
  const bool second = c >= g.c_split;
  const Src s = pick_src(g, second);
  const int cl = second ? c - g.c_split : c;
  float sc = 1.f, sh = 0.f;
  if (s.scale) {
    sc = s.scale[cl];
    sh = s.shift[cl];
  }
  float e[6][6];  // B^T d (rows), per column
#pragma unroll
  for (int xx = 0; xx < 6; ++xx) {
    float d[6];
#pragma unroll
    for (int yy = 0; yy < 6; ++yy) {
      const int y = 4 * ty + yy, x = 4 * tx + xx;
      float v = 0.f;
      if (y < g.Hg + 2 && x < g.Wg + 2) {
        v = s.ptr[((size_t)(n * s.H + y + s.oy) * s.W + x + s.ox) * s.C + cl];
        if (s.scale) v = fmaxf(fmaf(v, sc, sh), 0.f);
      }
      d[yy] = v;
    }
    float rr[6];
    bt6(d, rr);
#pragma unroll
    for (int a = 0; a < 6; ++a) e[a][xx] = rr[a];
  }
  const size_t plane = (size_t)T * g.Cg, o = (size_t)t * g.Cg + c;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    float rr[6];
    bt6(e[a], rr);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb) u[(a * 6 + bb) * plane + o] = rr[bb];
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
    for (long long t = blockIdx.x * 4ll + tl; t < T; t += (long long)gridDim.x * 4) {
      float w[4][6];  // A^T q (rows), per column
#pragma unroll
      for (int xx = 0; xx < 6; ++xx) {
        float q[6];
#pragma unroll
        for (int yy = 0; yy < 6; ++yy) q[yy] = m[(yy * 6 + xx) * plane + (size_t)t * N + col];
        float o[4];
        at4(q, o);
#pragma unroll
        for (int a = 0; a < 4; ++a) w[a][xx] = o[a];
      }
      const int tx = (int)(t % Tw);
      const long long r = t / Tw;
      const int ty = (int)(r % Th), n = (int)(r / Th);
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
  const size_t a = wino_bytes(16, t2, Cg, N), b = wino_bytes(36, t4, Cg, N);
  return a > b ? a : b;
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
  } else {
    hipLaunchKernelGGL(k_wino4_w, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
    const long long ni = T * g.Cg;
    hipLaunchKernelGGL(k_wino4_in, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, s, g, Th, Tw, T, U);
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
    int tile = a.wino_choice.tile;
    if (tile != 1 && tile != 3 && tile != 4) {
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
    hipLaunchKernelGGL(k_wino4_out, grid, dim3(256), 0, s, Mm, T, Th, Tw, a.N, g, a.e);
  }
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
__device__ __forceinline__ void a6(const float (&y)[4], float (&r)[6]) {
  r[0] = y[0];
  r[1] = y[0] + y[1] + y[2] + y[3];
  r[2] = y[0] - y[1] + y[2] - y[3];
  r[3] = y[0] + 2.f * y[1] + 4.f * y[2] + 8.f * y[3];
  r[4] = y[0] - 2.f * y[1] + 4.f * y[2] - 8.f * y[3];
  r[5] = y[3];
}
__device__ __forceinline__ void gt3(const float (&m)[6], float (&r)[3]) {
  r[0] = 0.25f * m[0] - (m[1] + m[2]) * (1.f / 6.f) + (m[3] + m[4]) * (1.f / 24.f);
  r[1] = (m[2] - m[1]) * (1.f / 6.f) + (m[3] - m[4]) * (1.f / 12.f);
  r[2] = (m[3] + m[4] - m[1] - m[2]) * (1.f / 6.f) + m[5];
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
      d[yy] = (y < Hg && x < Wg) ? dy.ptr[((size_t)(n * dy.H + y + dy.oy) * dy.W + x + dy.ox) * dy.C + c] : 0.f;
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

static long long wino_wgrad_tiles(const WgradArgs& a) {
  return (long long)a.gb.nimg * ((a.gb.Hg + 3) / 4) * ((a.gb.Wg + 3) / 4);
}

bool wino_wgrad_applies(const WgradArgs& a) {
  const Gather& ga = a.ga;
  const Gather& gb = a.gb;
  if (a.bf16 || a.batch != 1 || a.wino_ws == nullptr) return false;
  if (ga.taps_h != 1 || ga.taps_w != 1 || ga.stride != 1 || ga.c_split != ga.Cg || ga.s[0].h16 || ga.s[0].scale)
    return false;
  if (gb.taps_h != 3 || gb.taps_w != 3 || gb.stride != 1 || gb.s[0].h16 || gb.s[1].h16) return false;
  if (ga.Hg != gb.Hg || ga.Wg != gb.Wg || ga.nimg != gb.nimg || a.P != gb.nimg * gb.Hg * gb.Wg) return false;
  if (a.Mo != ga.Cg || a.No != 9 * gb.Cg || a.Mo % 64 != 0 || gb.Cg % 64 != 0 || gb.c_split % 4 != 0) return false;
  return wino_bytes(36, wino_wgrad_tiles(a), gb.Cg, a.Mo) <= a.wino_ws_bytes;
}

hipError_t launch_wino_wgrad(const WgradArgs& a, hipStream_t s, int per_cu) {
  if (!wino_wgrad_applies(a)) return hipErrorInvalidValue;
  const Gather& gb = a.gb;
  const int Th = (gb.Hg + 3) / 4, Tw = (gb.Wg + 3) / 4;
  const long long T = wino_wgrad_tiles(a);
  const int Ci = gb.Cg, Co = a.Mo;
  if (36 * T > 0x7fffffffLL) return hipErrorInvalidValue;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  char* w = reinterpret_cast<char*>(a.wino_ws);
  float* U = reinterpret_cast<float*>(w);
  float* Vd = reinterpret_cast<float*>(w + al((size_t)36 * T * Ci * 4));
  float* Mw = reinterpret_cast<float*>(w + al((size_t)36 * T * Ci * 4) + al((size_t)36 * T * Co * 4));
  const long long ni = T * Ci, nd = T * Co;
  hipLaunchKernelGGL(k_wino4_in, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, s, gb, Th, Tw, T, U);
  hipLaunchKernelGGL(k_wino4_dy, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, a.ga.s[0], gb.Hg, gb.Wg, Th,
                     Tw, T, Co, Vd);
  hipError_t e = hipMemsetAsync(Mw, 0, (size_t)36 * Co * Ci * 4, s);
  if (e != hipSuccess) return e;
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    // the 36 point GEMMs Mw[p] = Vd[p]^T U[p] as one batched k_wgrad launch
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
    q.batch = 36;
    q.batch_a = T * Co;
    q.batch_b = T * Ci;
    q.batch_out = (long long)Co * Ci;
    const int tile = (Co % 128 == 0 && Ci % 128 == 0) ? 0 : (Ci % 128 == 0 ? 3 : 4);
    if ((e = launch_wgrad_v(q, s, GemmChoice{tile, per_cu})) != hipSuccess) return e;
  }
  const long long no = (long long)Co * Ci;
  hipLaunchKernelGGL(k_wino4_wout, dim3((unsigned)((no + 255) / 256)), dim3(256), 0, s, Mw, Co, Ci, a.out);
  return hipGetLastError();
}

}  // namespace unet
