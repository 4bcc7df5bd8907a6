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

// workspace of the Winograd path for one GEMM (U, M, V; 256-B aligned pieces)
size_t wino_ws_bytes(long long T, int Cg, int N) {
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  return al(16 * (size_t)T * Cg * 4) + al(16 * (size_t)T * N * 4) + al(16 * (size_t)N * Cg * 4);
}

bool wino_applies(const IgemmArgs& a) {
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
  const long long T = (long long)g.nimg * ((g.Hg + 1) / 2) * ((g.Wg + 1) / 2);
  return a.wino_ws != nullptr && wino_ws_bytes(T, g.Cg, a.N) <= a.wino_ws_bytes;
}

hipError_t launch_wino(const IgemmArgs& a, hipStream_t s) {
  if (!wino_applies(a)) return hipErrorInvalidValue;
  const Gather& g = a.a;
  const int Th = (g.Hg + 1) / 2, Tw = (g.Wg + 1) / 2;
  const long long T = (long long)g.nimg * Th * Tw;
  char* w = reinterpret_cast<char*>(a.wino_ws);
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  float* U = reinterpret_cast<float*>(w);
  float* Mm = reinterpret_cast<float*>(w + al(16 * (size_t)T * g.Cg * 4));
  float* V = reinterpret_cast<float*>(w + al(16 * (size_t)T * g.Cg * 4) + al(16 * (size_t)T * a.N * 4));
  const long long nw = (long long)a.N * g.Cg;
  hipLaunchKernelGGL(k_wino_w, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, a.b, a.N, g.Cg, V);
  const long long ni = T * (g.Cg / 4);
  hipLaunchKernelGGL(k_wino_in, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, s, g, Th, Tw, T, U);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  {
    // the 16 point GEMMs as one batched launch over a 1 x 16T row grid:
    // M[p] = U[p] (T x Cg) . V[p]^T, V[p] = [N][Cg]
    IgemmArgs q;
    Src u;
    u.ptr = U;
    u.H = 1;
    u.W = (int)(16 * T);
    u.C = g.Cg;
    q.a.s[0] = q.a.s[1] = u;
    q.a.Cg = q.a.c_split = g.Cg;
    q.a.taps_h = q.a.taps_w = 1;
    q.a.Hg = 1;
    q.a.Wg = (int)(16 * T);
    q.a.nimg = 1;
    q.b = V;
    q.M = (int)(16 * T);
    q.N = a.N;
    q.K = g.Cg;
    q.e.d[0] = Dst{Mm, 1, (int)(16 * T), a.N, 0, 0};
    q.batch = 16;
    q.batch_rows = (int)T;
    q.batch_b = (long long)a.N * g.Cg;
    // 256 x 128 tiles when they give two rounds of workgroups, else 128 x 128
    // (register-staged k_igemm: the batched launch form)
    int tile = a.wino_choice.tile;
    if (tile != 1 && tile != 3 && tile != 4) {
      const long long t256 = ((T + 255) / 256) * (a.N / 128) * 16;
      tile = (a.N % 128 == 0 && t256 >= 2 * num_cus()) ? 4 : (a.N % 128 == 0 ? 1 : 8);
    }
    if ((e = launch_igemm_v(q, s, GemmChoice{tile, 1})) != hipSuccess) return e;
  }
  const int C4 = a.N / 4, cgs = C4 < 64 ? C4 : 64, lanes = 256 / cgs;
  long long gx = (T + lanes * 4 - 1) / (lanes * 4);  // ~4 tiles per thread: statistics kept in registers
  if (gx > 65535) gx = 65535;
  dim3 grid((unsigned)gx, (unsigned)((C4 + cgs - 1) / cgs));
  hipLaunchKernelGGL(k_wino_out, grid, dim3(256), 0, s, Mm, T, Th, Tw, a.N, g, a.e);
  return hipGetLastError();
}

}  // namespace unet
