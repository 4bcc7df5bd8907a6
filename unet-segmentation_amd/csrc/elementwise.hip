// Memory-bound kernels of the U-Net hot path (gfx950): the first conv (Ci<=4,
// HBM-bound), BatchNorm finalize/apply passes, 2x2 max-pool with argmax, the
// 1x1 head, the fused weighted cross-entropy, SGD-momentum and weight repacks.
// All NHWC activations are touched as float4 (16 B per lane) so every wave
// instruction moves 1 KiB of contiguous bytes where the layout allows it.
#include "gemm_common.h"

namespace unet {

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
static inline int grid_cap(long long work, int per_block, int cap = 4096) {
  long long g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g < cap ? g : cap);
}

// Per-channel reduction of (a, b) pairs accumulated by threads that own channel
// group tid % CG (4 channels each).  One fp64 atomic per channel per block.
__device__ void reduce_pairs_to_global(const float (&a)[4], const float (&b)[4], int CG, int C,
                                       double* dst /* [C][2] of this group */) {
  __shared__ float red[256][9];
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) { red[tid][k] = a[k]; red[tid][4 + k] = b[k]; }
  __syncthreads();
  if (tid < CG) {
    float sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
    for (int r = tid; r < 256; r += CG) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { sa[k] += red[r][k]; sb[k] += red[r][4 + k]; }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      atomicAdd(dst + (size_t)(tid * 4 + k) * 2 + 0, (double)sa[k]);
      atomicAdd(dst + (size_t)(tid * 4 + k) * 2 + 1, (double)sb[k]);
    }
  }
}

// ---------------------------------------------------------------------------
// inc.c0 forward (models/unet_model.py:11 with in_channels = n_channels <= 4):
// direct 3x3 valid conv from the NCHW network input, 64 output channels NHWC,
// + conv bias, + BatchNorm batch statistics (sum, sumsq) of the output.
// Block = one output row segment of 64 pixels; thread = (channel, pixel phase).
// ---------------------------------------------------------------------------
template <int CI, int H16>  // H16: y stored bf16 (statistics of the rounded values)
__global__ __launch_bounds__(256) void k_conv_first_fwd(const float* __restrict__ x, int h, int w,
                                                        const float* __restrict__ wt,
                                                        const float* __restrict__ bias, float* __restrict__ y,
                                                        double* __restrict__ stats, int relu) {
  const int ho = h - 2, wo = w - 2;
  const int x0 = blockIdx.x * 64, row = blockIdx.y, n = blockIdx.z;
  __shared__ float tile[CI][3][66];
  const int tid = threadIdx.x;
  for (int i = tid; i < CI * 3 * 66; i += 256) {
    const int ci = i / 198, rem = i - ci * 198, r = rem / 66, cx = rem - r * 66;
    const int gx = min(x0 + cx, w - 1);
    tile[ci][r][cx] = x[((size_t)(n * CI + ci) * h + row + r) * w + gx];
  }
  const int c = tid & 63, q = tid >> 6;
  float wr[CI * 9];
#pragma unroll
  for (int k = 0; k < CI * 9; ++k) wr[k] = wt[c * CI * 9 + k];
  const float b = bias[c];
  __syncthreads();
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {
    const int px = q + 4 * j;
    const int gx = x0 + px;
    float acc = b;
#pragma unroll
    for (int ci = 0; ci < CI; ++ci)
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc = fmaf(tile[ci][ky][px + kx], wr[(ci * 3 + ky) * 3 + kx], acc);
    if (relu) acc = fmaxf(acc, 0.f);  // eval with BatchNorm folded into wt / bias
    if (gx < wo) {
      const size_t yi = ((size_t)(n * ho + row) * wo + gx) * 64 + c;
      if (H16) {
        acc = round_bf(acc);
        reinterpret_cast<uint16_t*>(y)[yi] = bf16_of(acc);
      } else {
        y[yi] = acc;
      }
      s1 += acc;
      s2 += acc * acc;
    }
  }
  if (stats == nullptr) return;  // eval mode: no batch statistics
  __shared__ float red[4][2][64];
  red[q][0][c] = s1;
  red[q][1][c] = s2;
  __syncthreads();
  if (tid < 64) {
    const float a = red[0][0][tid] + red[1][0][tid] + red[2][0][tid] + red[3][0][tid];
    const float bb = red[0][1][tid] + red[1][1][tid] + red[2][1][tid] + red[3][1][tid];
    const int grp = (blockIdx.x + blockIdx.y * gridDim.x) % kStatGroups;
    atomicAdd(stats + ((size_t)grp * 64 + tid) * 2 + 0, (double)a);
    atomicAdd(stats + ((size_t)grp * 64 + tid) * 2 + 1, (double)bb);
  }
}

// inc.c0 weight gradient: dW[co][ci][ky][kx] = sum_p dY[p][co] * x[ci][p+(ky,kx)].
// HBM-bound reduction over every output pixel (dY is 64 ch x 510^2 x N floats).
// Work item = a strip of RB rows x 64 columns; thread = (4-channel group,
// pixel slot): 16 lanes read one pixel's 64 channels as float4 (a wave moves
// 1 KiB of contiguous dY per load), 8 loads in flight per thread; the x strip
// is staged in LDS.  Per-thread register sums, one fp32 atomic per weight per
// workgroup at the end.
// FUSED: dY is not read from a padded buffer but formed on the fly from the
// BN0 backward -- dY = k0*dz + k1*(y - mean) + k2 with the per-channel
// coefficients of k_bnb_finalize (coef[4][64]) -- from dz (dy.ptr, the
// unpadded (ho, wo) grid) and the saved raw conv output y (Y16: bf16).  inc.c0
// has no input gradient, so dY(0) is consumed only here and is never written
// (SURVEY.md §8d's fused stage-1 backward: read dz, y, x once).  Z16: dz stored
// bf16 (bf16 plans).
template <int CI, int FUSED = 0, int Y16 = 0, int Z16 = 0>
__global__ __launch_bounds__(256) void k_conv_first_wgrad(const float* __restrict__ x, int nimg, int h, int w,
                                                          Src dy, float* __restrict__ dw, int ci_tot, int ci_off,
                                                          const float* __restrict__ yr = nullptr,
                                                          const float* __restrict__ coef = nullptr) {
  constexpr int RB = 4, PX = 64, TW = PX + 2;
  const int ho = h - 2, wo = w - 2;
  const int nseg = (wo + PX - 1) / PX, nstrip = (ho + RB - 1) / RB;
  const long long items = (long long)nimg * nstrip * nseg;
  __shared__ float tile[CI][RB + 2][TW];
  const int tid = threadIdx.x, cg = tid & 15, slot = tid >> 4;  // 16 channel groups x 16 pixel slots
  float4 k0, k1, k2, mu;
  if (FUSED) {
    k0 = ld4(coef + cg * 4);
    k1 = ld4(coef + 64 + cg * 4);
    k2 = ld4(coef + 128 + cg * 4);
    mu = ld4(coef + 192 + cg * 4);
  }
  float acc[4][CI * 9];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int k = 0; k < CI * 9; ++k) acc[c][k] = 0.f;
  for (long long it = blockIdx.x; it < items; it += gridDim.x) {
    const int seg = (int)(it % nseg);
    const long long t2 = it / nseg;
    const int strip = (int)(t2 % nstrip), n = (int)(t2 / nstrip);
    const int x0 = seg * PX, r0 = strip * RB;
    __syncthreads();
    for (int i = tid; i < CI * (RB + 2) * TW; i += 256) {
      const int ci = i / ((RB + 2) * TW), rem = i - ci * (RB + 2) * TW, r = rem / TW, cx = rem - r * TW;
      const int gx = min(x0 + cx, w - 1), gy = min(r0 + r, h - 1);
      tile[ci][r][cx] = x[((size_t)(n * ci_tot + ci_off + ci) * h + gy) * w + gx];
    }
    __syncthreads();
    // RB*PX = 256 pixels, 16 per slot, in two batches of 8 loads
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      float4 g[8];
      int pr[8], pc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int pix = slot + 16 * (8 * b + j);  // 0..255
        pr[j] = pix / PX;
        pc[j] = pix - pr[j] * PX;
        const bool ok = (r0 + pr[j] < ho) && (x0 + pc[j] < wo);
        const int yy = min(r0 + pr[j], ho - 1), xx = min(x0 + pc[j], wo - 1);
        const size_t off = ((size_t)(n * dy.H + yy + dy.oy) * dy.W + xx + dy.ox) * dy.C + cg * 4;
        if (Z16)
          g[j] = bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(dy.ptr) + off));
        else
          g[j] = *reinterpret_cast<const float4*>(dy.ptr + off);
        if (FUSED) {
          const float4 d = g[j];
          const float4 yv = Y16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(yr) + off))
                                : ld4(yr + off);
          g[j].x = fmaf(k0.x, d.x, fmaf(k1.x, yv.x - mu.x, k2.x));
          g[j].y = fmaf(k0.y, d.y, fmaf(k1.y, yv.y - mu.y, k2.y));
          g[j].z = fmaf(k0.z, d.z, fmaf(k1.z, yv.z - mu.z, k2.z));
          g[j].w = fmaf(k0.w, d.w, fmaf(k1.w, yv.w - mu.w, k2.w));
        }
        if (!ok) g[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int ci = 0; ci < CI; ++ci)
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const float xv = tile[ci][pr[j] + ky][pc[j] + kx];
              const int k = (ci * 3 + ky) * 3 + kx;
              acc[0][k] = fmaf(g[j].x, xv, acc[0][k]);
              acc[1][k] = fmaf(g[j].y, xv, acc[1][k]);
              acc[2][k] = fmaf(g[j].z, xv, acc[2][k]);
              acc[3][k] = fmaf(g[j].w, xv, acc[3][k]);
            }
      }
    }
  }
  // reduce the 16 pixel slots that share a channel group, one weight index at a
  // time through a small LDS buffer, then write this workgroup's partial slab
  // (no atomics: 2048 workgroups adding into the same 576 words serialise at
  // the memory side; k_reduce_slabs sums the slabs)
  __shared__ float red[16][65];
  float* slab = dw + (size_t)blockIdx.x * CI * 9 * 64;
#pragma unroll
  for (int k = 0; k < CI * 9; ++k) {
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) red[slot][cg * 4 + c] = acc[c][k];
    __syncthreads();
    if (tid < 64) {
      float v = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) v += red[s2][tid];
      slab[(size_t)tid * CI * 9 + k] = v;
    }
  }
}

// out[i] += sum_{b in chunk} slabs[b][i]: block (word group of 64, chunk of
// 64 slabs); 4 waves each sum 16 slabs of the same 64 words (256-B coalesced
// rows), then one atomic per word per block (out zeroed by the launcher).
// Destination word of slab word w: (w / rowlen) * rowstride + rowoff + w % rowlen
// (an input-channel group of a Ci > 4 first conv lands in its columns of
// dW[co][ci][3][3]).
__global__ __launch_bounds__(256) void k_reduce_slabs(const float* __restrict__ slabs, int nslab, int n,
                                                      float* __restrict__ out, int rowlen, int rowstride,
                                                      int rowoff, int chunk) {
  const int w = blockIdx.x * 64 + (threadIdx.x & 63);
  const int b0 = blockIdx.y * chunk;
  const int b1 = min(nslab, b0 + chunk);
  float s = 0.f;
  if (w < n)
    for (int b = b0 + (threadIdx.x >> 6); b < b1; b += 4) s += slabs[(size_t)b * n + w];
  __shared__ float red[4][64];
  red[threadIdx.x >> 6][threadIdx.x & 63] = s;
  __syncthreads();
  if (threadIdx.x < 64 && w < n)
    atomicAdd(out + (w / rowlen) * rowstride + rowoff + w % rowlen,
              red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// n_channels > 4 (models/unet_model.py:66 takes any count): the same direct
// conv with the input-channel count at run time, staged through LDS in chunks
// of kFirstChunk channels (tile + 64 x chunk x 9 weights), the 16 pixel
// accumulators of a thread carried across chunks.  Not on the benchmarked path.
constexpr int kFirstChunk = 16;
template <int H16>
__global__ __launch_bounds__(256) void k_conv_first_fwd_gen(const float* __restrict__ x, int ci_n, int h, int w,
                                                            const float* __restrict__ wt,
                                                            const float* __restrict__ bias, float* __restrict__ y,
                                                            double* __restrict__ stats, int relu) {
  const int ho = h - 2, wo = w - 2;
  const int x0 = blockIdx.x * 64, row = blockIdx.y, n = blockIdx.z;
  __shared__ float tile[kFirstChunk][3][66];
  __shared__ float wl[kFirstChunk * 9][64];
  const int tid = threadIdx.x;
  const int c = tid & 63, q = tid >> 6;
  float acc[16];
  const float b = bias[c];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = b;
  for (int c0 = 0; c0 < ci_n; c0 += kFirstChunk) {
    const int cn = min(kFirstChunk, ci_n - c0);
    __syncthreads();
    for (int i = tid; i < cn * 3 * 66; i += 256) {
      const int ci = i / 198, rem = i - ci * 198, r = rem / 66, cx = rem - r * 66;
      const int gx = min(x0 + cx, w - 1);
      tile[ci][r][cx] = x[((size_t)(n * ci_n + c0 + ci) * h + row + r) * w + gx];
    }
    for (int i = tid; i < cn * 9 * 64; i += 256) {
      const int cc = i / (cn * 9), k = i - cc * (cn * 9);
      wl[k][cc] = wt[(size_t)cc * ci_n * 9 + c0 * 9 + k];
    }
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      const int px = q + 4 * j;
      float a = acc[j];
      for (int ci = 0; ci < cn; ++ci)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) a = fmaf(tile[ci][ky][px + kx], wl[(ci * 3 + ky) * 3 + kx][c], a);
      acc[j] = a;
    }
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int gx = x0 + q + 4 * j;
    float a = acc[j];
    if (relu) a = fmaxf(a, 0.f);  // eval with BatchNorm folded into wt / bias
    if (gx < wo) {
      const size_t yi = ((size_t)(n * ho + row) * wo + gx) * 64 + c;
      if (H16) {
        a = round_bf(a);
        reinterpret_cast<uint16_t*>(y)[yi] = bf16_of(a);
      } else {
        y[yi] = a;
      }
      s1 += a;
      s2 += a * a;
    }
  }
  if (stats == nullptr) return;
  __shared__ float red[4][2][64];
  red[q][0][c] = s1;
  red[q][1][c] = s2;
  __syncthreads();
  if (tid < 64) {
    const float a = red[0][0][tid] + red[1][0][tid] + red[2][0][tid] + red[3][0][tid];
    const float bb = red[0][1][tid] + red[1][1][tid] + red[2][1][tid] + red[3][1][tid];
    const int grp = (blockIdx.x + blockIdx.y * gridDim.x) % kStatGroups;
    atomicAdd(stats + ((size_t)grp * 64 + tid) * 2 + 0, (double)a);
    atomicAdd(stats + ((size_t)grp * 64 + tid) * 2 + 1, (double)bb);
  }
}

template <int H16>
static void conv_first_go(dim3 grid, int ci, const float* x, int h, int w, const float* wt, const float* bias, float* y,
                          double* stats, int relu, hipStream_t s) {
  if (ci > 4) {
    hipLaunchKernelGGL((k_conv_first_fwd_gen<H16>), grid, dim3(256), 0, s, x, ci, h, w, wt, bias, y, stats, relu);
    return;
  }
  switch (ci) {
    case 1: hipLaunchKernelGGL((k_conv_first_fwd<1, H16>), grid, dim3(256), 0, s, x, h, w, wt, bias, y, stats, relu); break;
    case 2: hipLaunchKernelGGL((k_conv_first_fwd<2, H16>), grid, dim3(256), 0, s, x, h, w, wt, bias, y, stats, relu); break;
    case 3: hipLaunchKernelGGL((k_conv_first_fwd<3, H16>), grid, dim3(256), 0, s, x, h, w, wt, bias, y, stats, relu); break;
    default: hipLaunchKernelGGL((k_conv_first_fwd<4, H16>), grid, dim3(256), 0, s, x, h, w, wt, bias, y, stats, relu); break;
  }
}

hipError_t launch_conv_first_fwd(const float* x, int n, int ci, int h, int w, const float* wt,
                                 const float* bias, int co, float* y, double* stats, hipStream_t s, int out_h16,
                                 int relu) {
  if (co != 64 || ci < 1 || h < 3 || w < 3) return hipErrorInvalidValue;
  dim3 grid(cdiv(w - 2, 64), h - 2, n);
  if (out_h16) conv_first_go<1>(grid, ci, x, h, w, wt, bias, y, stats, relu, s);
  else conv_first_go<0>(grid, ci, x, h, w, wt, bias, y, stats, relu, s);
  return hipGetLastError();
}

// inc.c0 input gradient (the per-op path, unet_conv_first_bwd; the network
// never needs it): dx[n][ci][y][x] = sum_{co, ky, kx} dY[n][y-ky][x-kx][co] *
// W[co][ci][ky][kx] over the valid output positions.  Thread = one input pixel
// of one channel; 64-channel dY rows read as float4.
__global__ __launch_bounds__(256) void k_conv_first_dgrad(const float* __restrict__ dy, int n, int ci_n, int h,
                                                          int w, const float* __restrict__ wt,
                                                          float* __restrict__ dx) {
  const int ho = h - 2, wo = w - 2;
  const long long total = (long long)n * ci_n * h * w;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % w);
    long long t = i / w;
    const int yy = (int)(t % h);
    t /= h;
    const int ci = (int)(t % ci_n), nn = (int)(t / ci_n);
    float acc = 0.f;
    for (int ky = 0; ky < 3; ++ky) {
      const int oy = yy - ky;
      if (oy < 0 || oy >= ho) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int ox = xx - kx;
        if (ox < 0 || ox >= wo) continue;
        const float* g = dy + ((size_t)(nn * ho + oy) * wo + ox) * 64;
        const float* wk = wt + (size_t)ci * 9 + ky * 3 + kx;
        for (int co = 0; co < 64; co += 4) {
          const float4 gv = ld4(g + co);
          acc = fmaf(gv.x, wk[(size_t)(co + 0) * ci_n * 9], acc);
          acc = fmaf(gv.y, wk[(size_t)(co + 1) * ci_n * 9], acc);
          acc = fmaf(gv.z, wk[(size_t)(co + 2) * ci_n * 9], acc);
          acc = fmaf(gv.w, wk[(size_t)(co + 3) * ci_n * 9], acc);
        }
      }
    }
    dx[i] = acc;
  }
}

hipError_t launch_conv_first_dgrad(const float* dy, int n, int ci, int h, int w, const float* wt, float* dx,
                                   hipStream_t s) {
  if (ci < 1 || h < 3 || w < 3) return hipErrorInvalidValue;
  const long long total = (long long)n * ci * h * w;
  hipLaunchKernelGGL(k_conv_first_dgrad, dim3(grid_cap(total, 256, 8192)), dim3(256), 0, s, dy, n, ci, h, w, wt, dx);
  return hipGetLastError();
}

// BatchNorm folded into a conv for eval (scripts/predict.py:70 model.eval()):
// row r of the weight matrix w[rows][K] times scale[r] (into wout, may alias w)
// and bias_out[r] = scale[r] * bias[r] + shift[r], scale / shift from the
// running statistics (k_bn_eval_prepare): bn(conv(x)) = conv'(x).
__global__ void k_fold_bn(const float* __restrict__ w, long long K, int rows, const float* __restrict__ scale,
                          const float* __restrict__ shift, const float* __restrict__ bias, float* __restrict__ wout,
                          float* __restrict__ bias_out) {
  const long long n = (long long)rows * K;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / K);
    wout[i] = w[i] * scale[r];
    if (i - (long long)r * K == 0) bias_out[r] = fmaf(scale[r], bias[r], shift[r]);
  }
}

hipError_t launch_fold_bn(const float* w, long long K, int rows, const float* scale, const float* shift,
                          const float* bias, float* wout, float* bias_out, hipStream_t s) {
  const long long n = (long long)rows * K;
  hipLaunchKernelGGL(k_fold_bn, dim3(grid_cap(n, 256, 8192)), dim3(256), 0, s, w, K, rows, scale, shift, bias, wout,
                     bias_out);
  return hipGetLastError();
}

// slabs of one pass of <= 4 input channels (passes reuse the region in stream order)
size_t conv_first_wgrad_ws_bytes(int ci) { return sizeof(float) * (size_t)kFirstWgradSlabs * (ci < 4 ? ci : 4) * 9 * 64; }

// sum the pass's slabs into its columns [ci_off * 9, (ci_off + cp) * 9) of dW[64][ci_tot * 9]
static hipError_t reduce_first_slabs(int cp, int ci_tot, int ci_off, int grid, float* dw, const float* slabs,
                                     hipStream_t s) {
  const int nw = cp * 9 * 64;
  // deterministic mode: one block per word group sums every slab (a single
  // atomic per word onto the zeroed output: order-free); else 64-slab chunks
  const int chunk = g_deterministic ? grid : 64;
  hipLaunchKernelGGL(k_reduce_slabs, dim3(cdiv(nw, 64), cdiv(grid, chunk)), dim3(256), 0, s, slabs, grid, nw, dw,
                     cp * 9, ci_tot * 9, ci_off * 9, chunk);
  return hipGetLastError();
}

// One launch per group of <= 4 input channels (models/unet_model.py:66 takes
// any n_channels; the register accumulators hold 4 x 9 x 4 weights per thread).
template <int FUSED, int Y16, int Z16 = 0>
static hipError_t first_wgrad_run(int ci, const float* x, int n, int h, int w, const Src& dy, float* dw, float* slabs,
                                  const float* y, const float* coef, hipStream_t s) {
  const long long items = (long long)n * cdiv(h - 2, 4) * cdiv(w - 2, 64);
  const int grid = (int)(items < kFirstWgradSlabs ? items : kFirstWgradSlabs);
  hipError_t e = hipMemsetAsync(dw, 0, sizeof(float) * (size_t)ci * 9 * 64, s);
  if (e != hipSuccess) return e;
  for (int c0 = 0; c0 < ci; c0 += 4) {
    const int cp = ci - c0 < 4 ? ci - c0 : 4;
    switch (cp) {
      case 1: hipLaunchKernelGGL((k_conv_first_wgrad<1, FUSED, Y16, Z16>), dim3(grid), dim3(256), 0, s, x, n, h, w, dy, slabs, ci, c0, y, coef); break;
      case 2: hipLaunchKernelGGL((k_conv_first_wgrad<2, FUSED, Y16, Z16>), dim3(grid), dim3(256), 0, s, x, n, h, w, dy, slabs, ci, c0, y, coef); break;
      case 3: hipLaunchKernelGGL((k_conv_first_wgrad<3, FUSED, Y16, Z16>), dim3(grid), dim3(256), 0, s, x, n, h, w, dy, slabs, ci, c0, y, coef); break;
      default: hipLaunchKernelGGL((k_conv_first_wgrad<4, FUSED, Y16, Z16>), dim3(grid), dim3(256), 0, s, x, n, h, w, dy, slabs, ci, c0, y, coef); break;
    }
    if ((e = reduce_first_slabs(cp, ci, c0, grid, dw, slabs, s)) != hipSuccess) return e;
  }
  return hipGetLastError();
}

hipError_t launch_conv_first_wgrad(const float* x, int n, int ci, int h, int w, const Src& dy, int co,
                                   float* dw, float* slabs, hipStream_t s) {
  if (co != 64 || ci < 1) return hipErrorInvalidValue;
  return first_wgrad_run<0, 0>(ci, x, n, h, w, dy, dw, slabs, nullptr, nullptr, s);
}

// inc.c0 weight gradient straight from the BN0 backward (dz, saved y, coef):
// no padded dY(0) is written or read.
hipError_t launch_conv_first_wgrad_bn(const float* x, int n, int ci, int h, int w, const float* dz, const float* y,
                                      int y_h16, const float* coef, int co, float* dw, float* slabs, hipStream_t s,
                                      int dz_h16) {
  if (co != 64 || ci < 1) return hipErrorInvalidValue;
  Src d;
  d.ptr = dz;
  d.H = h - 2;
  d.W = w - 2;
  d.C = 64;
  if (y_h16 && dz_h16) return first_wgrad_run<1, 1, 1>(ci, x, n, h, w, d, dw, slabs, y, coef, s);
  if (y_h16) return first_wgrad_run<1, 1>(ci, x, n, h, w, d, dw, slabs, y, coef, s);
  return first_wgrad_run<1, 0>(ci, x, n, h, w, d, dw, slabs, y, coef, s);
}

// ---------------------------------------------------------------------------
// BatchNorm2d (train) finalize: grouped fp64 (sum, sumsq) -> batch mean, biased
// variance, invstd; consumer transform scale = gamma*invstd, shift = beta -
// mean*scale; running stats: momentum 0.1, unbiased variance; nbt += 1.
// ---------------------------------------------------------------------------
// Sum the kStatGroups group partials of (a, b) for 64 channels per block: the
// 4 waves each take a quarter of the groups, then combine through LDS.
// Returns true for the 64 threads that hold a channel's totals.
__device__ __forceinline__ bool group_sum(const double* __restrict__ st, int C, double& s1, double& s2, int& c) {
  __shared__ double red[4][64][2];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  c = blockIdx.x * 64 + lane;
  double a = 0, b = 0;
  if (c < C) {
#pragma unroll 4
    for (int g = q; g < kStatGroups; g += 4) {
      a += st[((size_t)g * C + c) * 2 + 0];
      b += st[((size_t)g * C + c) * 2 + 1];
    }
  }
  red[q][lane][0] = a;
  red[q][lane][1] = b;
  __syncthreads();
  if (q != 0 || c >= C) return false;
  s1 = red[0][lane][0] + red[1][lane][0] + red[2][lane][0] + red[3][lane][0];
  s2 = red[0][lane][1] + red[1][lane][1] + red[2][lane][1] + red[3][lane][1];
  return true;
}

__global__ __launch_bounds__(256) void k_bn_finalize(const double* __restrict__ st, int C, double count,
                                                     const float* gamma, const float* beta, float* rmean,
                                                     float* rvar, int64_t* nbt, float* mean, float* invstd,
                                                     float* scale, float* shift, float mom, float eps) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  double s1, s2;
  int c;
  if (!group_sum(st, C, s1, s2, c)) return;
  const double mu = s1 / count;
  double var = s2 / count - mu * mu;
  if (var < 0) var = 0;
  const double is = 1.0 / sqrt(var + (double)eps);
  const double sc = (double)gamma[c] * is;
  mean[c] = (float)mu;
  invstd[c] = (float)is;
  scale[c] = (float)sc;
  shift[c] = (float)((double)beta[c] - mu * sc);
  if (rmean) rmean[c] = (float)((1.0 - mom) * rmean[c] + mom * mu);
  if (rvar) rvar[c] = (float)((1.0 - mom) * rvar[c] + mom * var * count / (count > 1 ? count - 1 : 1));
}

__global__ void k_bn_eval_prepare(int C, const float* gamma, const float* beta, const float* rm,
                                  const float* rv, float* scale, float* shift, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double is = 1.0 / sqrt((double)rv[c] + (double)eps);
  const double sc = (double)gamma[c] * is;
  scale[c] = (float)sc;
  shift[c] = (float)((double)beta[c] - (double)rm[c] * sc);
}

// BN backward finalize.  With B1 = sum dz', B2 = sum dz'*xhat (dz' = dL/dz after
// the ReLU mask):  dbeta = B1, dgamma = B2 and
//   dY = gamma*invstd*(dz' - B1/M - xhat*B2/M)
//      = k0*dz' + k1*(y - mean) + k2,  k0 = g*is, k1 = -g*is^2*B2/M, k2 = -g*is*B1/M.
// The conv bias that precedes the BN gets sum_p dY = k0*B1 + k2*M (+ k1*0),
// which is zero up to rounding (BN-cancelled biases).
// eval != 0: BatchNorm in eval mode (running statistics are constants): dY =
// gamma*invstd*dz', k1 = k2 = 0.
__global__ __launch_bounds__(256) void k_bnb_finalize(const double* __restrict__ st, int C, double M,
                                                      const float* gamma, const float* mean, const float* invstd,
                                                      float* dgamma, float* dbeta, float* dbias, float* coef,
                                                      int eval) {
  double b1, b2;
  int c;
  if (!group_sum(st, C, b1, b2, c)) return;
  const double gi = (double)gamma[c] * (double)invstd[c];
  const double k0 = gi, k1 = eval ? 0.0 : -gi * (double)invstd[c] * b2 / M, k2 = eval ? 0.0 : -gi * b1 / M;
  if (dgamma) dgamma[c] = (float)b2;
  if (dbeta) dbeta[c] = (float)b1;
  if (dbias) dbias[c] = (float)(k0 * b1 + k2 * M);
  coef[c] = (float)k0;
  coef[C + c] = (float)k1;
  coef[2 * C + c] = (float)k2;
  coef[3 * C + c] = mean[c];
}

// dYpad[n][y+pad][x+pad][c] = k0*dz + k1*(y - mean) + k2 ; border written as 0.
// H16: dYpad stored bf16 (it is only ever a bf16 GEMM operand then).
template <int H16, int Y16, int Z16 = 0>  // H16: dYpad stored bf16; Y16: y stored bf16; Z16: dz stored bf16
__global__ void k_bnb_apply(const float* __restrict__ dz, const float* __restrict__ yr,
                            const float* __restrict__ coef, int n, int h, int w, int C,
                            float* __restrict__ dyp, int pad) {
  // grid: x over one padded row's (pixel, 4-channel group) pairs, y over padded
  // rows; one division per row instead of per element
  const int C4 = C / 4;
  const int hp = h + 2 * pad, wp = w + 2 * pad, rowlen = wp * C4;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= rowlen) return;
  const int xp = j / C4, c4 = j - xp * C4, xx = xp - pad;
  float4 k0, k1, k2, mu;
  const bool colin = xx >= 0 && xx < w;
  if (colin) {
    k0 = ld4(coef + c4 * 4); k1 = ld4(coef + C + c4 * 4); k2 = ld4(coef + 2 * C + c4 * 4);
    mu = ld4(coef + 3 * C + c4 * 4);
  }
  for (int r = blockIdx.y; r < n * hp; r += gridDim.y) {
    const int nn = r / hp, yy = r - nn * hp - pad;
    float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
    if (colin && yy >= 0 && yy < h) {
      const size_t src = (((size_t)nn * h + yy) * w + xx) * C + c4 * 4;
      const float4 d = Z16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(dz) + src))
                           : ld4(dz + src);
      const float4 yv = Y16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(yr) + src))
                            : ld4(yr + src);
      out.x = fmaf(k0.x, d.x, fmaf(k1.x, yv.x - mu.x, k2.x));
      out.y = fmaf(k0.y, d.y, fmaf(k1.y, yv.y - mu.y, k2.y));
      out.z = fmaf(k0.z, d.z, fmaf(k1.z, yv.z - mu.z, k2.z));
      out.w = fmaf(k0.w, d.w, fmaf(k1.w, yv.w - mu.w, k2.w));
    }
    const size_t i = (size_t)r * rowlen + j;
    if (H16)
      reinterpret_cast<uint2*>(dyp)[i] = make_uint2(bf16pack(out.x, out.y), bf16pack(out.z, out.w));
    else
      st4(dyp + i * 4, out);
  }
}

// All-bf16 twin of k_bnb_apply (bf16 plans: dz, y and dYpad bf16): 8 channels
// (16 B) per lane and two padded rows per loop trip, both rows' loads issued
// before either is used.
__global__ void k_bnb_apply_bf8(const uint16_t* __restrict__ dz, const uint16_t* __restrict__ yr,
                                const float* __restrict__ coef, int n, int h, int w, int C,
                                uint16_t* __restrict__ dyp, int pad) {
  const int C8 = C / 8;
  const int hp = h + 2 * pad, wp = w + 2 * pad, rowlen = wp * C8;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= rowlen) return;
  const int xp = j / C8, c8 = j - xp * C8, xx = xp - pad;
  const bool colin = xx >= 0 && xx < w;
  float4 k0[2], k1[2], k2[2], mu[2];
  if (colin) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int c = c8 * 8 + 4 * hh;
      k0[hh] = ld4(coef + c); k1[hh] = ld4(coef + C + c); k2[hh] = ld4(coef + 2 * C + c);
      mu[hh] = ld4(coef + 3 * C + c);
    }
  }
  const int rows = n * hp;
  for (int r0 = blockIdx.y; r0 < rows; r0 += 2 * gridDim.y) {
    uint4 d[2], yv[2];
    bool in[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      // (predicated loads: a branch-free clamped form measured slower here,
      // 0.61 -> 0.67 ms per step, as did one for the fp32 twin)
      const int r = r0 + u * gridDim.y;
      const int nn = r / hp, yy = r - nn * hp - pad;
      in[u] = r < rows && colin && yy >= 0 && yy < h;
      d[u] = yv[u] = make_uint4(0u, 0u, 0u, 0u);
      if (in[u]) {
        const size_t src = ((((size_t)nn * h + yy) * w + xx) * C + c8 * 8) / 8;
        d[u] = reinterpret_cast<const uint4*>(dz)[src];
        yv[u] = reinterpret_cast<const uint4*>(yr)[src];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = r0 + u * gridDim.y;
      if (r >= rows) continue;
      uint4 o = make_uint4(0u, 0u, 0u, 0u);
      if (in[u]) {
        float4 res[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const float4 dd = bf16x4_to_f4(hh ? make_uint2(d[u].z, d[u].w) : make_uint2(d[u].x, d[u].y));
          const float4 y4 = bf16x4_to_f4(hh ? make_uint2(yv[u].z, yv[u].w) : make_uint2(yv[u].x, yv[u].y));
          res[hh].x = fmaf(k0[hh].x, dd.x, fmaf(k1[hh].x, y4.x - mu[hh].x, k2[hh].x));
          res[hh].y = fmaf(k0[hh].y, dd.y, fmaf(k1[hh].y, y4.y - mu[hh].y, k2[hh].y));
          res[hh].z = fmaf(k0[hh].z, dd.z, fmaf(k1[hh].z, y4.z - mu[hh].z, k2[hh].z));
          res[hh].w = fmaf(k0[hh].w, dd.w, fmaf(k1[hh].w, y4.w - mu[hh].w, k2[hh].w));
        }
        o = bf16pack8(res[0], res[1]);
      }
      reinterpret_cast<uint4*>(dyp)[(size_t)r * rowlen + j] = o;
    }
  }
}

hipError_t launch_bn_finalize(const double* stats, int c, double count, const float* gamma, const float* beta,
                              float* rmean, float* rvar, int64_t* nbt, float* mean, float* invstd, float* scale,
                              float* shift, float momentum, float eps, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_finalize, dim3(cdiv(c, 64)), dim3(256), 0, s, stats, c, count, gamma, beta, rmean, rvar,
                     nbt, mean, invstd, scale, shift, momentum, eps);
  return hipGetLastError();
}
hipError_t launch_bn_eval_prepare(int c, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                  float* scale, float* shift, float eps, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_eval_prepare, dim3(cdiv(c, 256)), dim3(256), 0, s, c, gamma, beta, rmean, rvar, scale, shift,
                     eps);
  return hipGetLastError();
}
hipError_t launch_bnb_finalize(const double* bstats, int c, double count, const float* gamma, const float* mean,
                               const float* invstd, float* dgamma, float* dbeta, float* dbias, float* coef,
                               hipStream_t s, int eval) {
  hipLaunchKernelGGL(k_bnb_finalize, dim3(cdiv(c, 64)), dim3(256), 0, s, bstats, c, count, gamma, mean, invstd,
                     dgamma, dbeta, dbias, coef, eval);
  return hipGetLastError();
}
hipError_t launch_bnb_apply(const float* dz, const float* y, const float* coef, int n, int h, int w, int c,
                            float* dypad, int pad, hipStream_t s, int out_h16, int y_h16, int dz_h16) {
  if (c % 4) return hipErrorInvalidValue;
  const long long rowlen = (long long)(w + 2 * pad) * (c / 4), rows = (long long)n * (h + 2 * pad);
  if (rows >= (1LL << 31) || rowlen >= (1LL << 31)) return hipErrorInvalidValue;
  const int gx = (int)((rowlen + 255) / 256);
  // ~4 rows per block keeps the row loop short while filling the chip
  const dim3 grid(gx, (unsigned)std::max<long long>(1, std::min<long long>(rows, std::max<long long>(1, 32768 / gx))));
  if (dz_h16) {  // bf16 plans: dz and y bf16; dYpad bf16 (fp32 only for the input gradient's dY(0))
    if (!y_h16) return hipErrorInvalidValue;
    if (!out_h16) {
      hipLaunchKernelGGL((k_bnb_apply<0, 1, 1>), grid, dim3(256), 0, s, dz, y, coef, n, h, w, c, dypad, pad);
      return hipGetLastError();
    }
    if (c % 8 == 0) {
      const long long rl8 = (long long)(w + 2 * pad) * (c / 8);
      const int gx8 = (int)((rl8 + 255) / 256);
      const dim3 g8(gx8, (unsigned)std::max<long long>(1, std::min<long long>(rows, std::max<long long>(1, 32768 / gx8))));
      hipLaunchKernelGGL(k_bnb_apply_bf8, g8, dim3(256), 0, s, reinterpret_cast<const uint16_t*>(dz),
                         reinterpret_cast<const uint16_t*>(y), coef, n, h, w, c, reinterpret_cast<uint16_t*>(dypad), pad);
      return hipGetLastError();
    }
    hipLaunchKernelGGL((k_bnb_apply<1, 1, 1>), grid, dim3(256), 0, s, dz, y, coef, n, h, w, c, dypad, pad);
    return hipGetLastError();
  }
  switch (out_h16 * 2 + y_h16) {
    case 0: hipLaunchKernelGGL((k_bnb_apply<0, 0>), grid, dim3(256), 0, s, dz, y, coef, n, h, w, c, dypad, pad); break;
    case 1: hipLaunchKernelGGL((k_bnb_apply<0, 1>), grid, dim3(256), 0, s, dz, y, coef, n, h, w, c, dypad, pad); break;
    case 2: hipLaunchKernelGGL((k_bnb_apply<1, 0>), grid, dim3(256), 0, s, dz, y, coef, n, h, w, c, dypad, pad); break;
    default: hipLaunchKernelGGL((k_bnb_apply<1, 1>), grid, dim3(256), 0, s, dz, y, coef, n, h, w, c, dypad, pad); break;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// MaxPool2d(2) forward (models/unet_model.py:28) of relu(bn(y)): floor mode,
// scan order (0,0),(0,1),(1,0),(1,1) with strict '>' so the FIRST max wins.
// ---------------------------------------------------------------------------
// anorm (optional, bf16 plans): the normalised input relu(bn(y)) of every
// window element, bf16 at its NHWC position -- the encoder output's skip view
// for the up block's concat (a row / column that floor mode drops is never
// inside that center crop).
template <int H16, int Y16>  // H16: pooled map stored bf16 (a GEMM operand only); Y16: input y stored bf16
__global__ void k_maxpool_fwd(Src s, int n, int h, int w, float* __restrict__ y, uint8_t* __restrict__ arg,
                              uint16_t* __restrict__ anorm) {
  const int C = s.C, C4 = C / 4, ho = h / 2, wo = w / 2;
  const long long total = (long long)n * ho * wo * C4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  // U items per loop trip, every window load issued before any use
  // (latency-bound otherwise: one HBM round trip per trip)
  constexpr int U = 4;
  for (long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x; i0 < total; i0 += U * stride) {
    float4 v[U][4];
    size_t sb0[U];  // window corner; element k at + ((k >> 1) W + (k & 1)) C
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = min(i0 + u * stride, total - 1);  // tail items recompute the last one (not stored)
      const int c4 = (int)(i % C4);
      long long p = i / C4;
      const int xo = (int)(p % wo);
      p /= wo;
      const int yo = (int)(p % ho);
      const int nn = (int)(p / ho);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int yy = 2 * yo + (k >> 1), xx = 2 * xo + (k & 1);
        const size_t si = ((size_t)(nn * s.H + yy + s.oy) * s.W + xx + s.ox) * C + c4 * 4;
        if (k == 0) sb0[u] = si;
        v[u][k] = Y16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(s.ptr) + si))
                      : ld4(s.ptr + si);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i >= total) continue;
      const int c4 = (int)(i % C4);
      if (s.scale) {
        const float4 a = ld4(s.scale + c4 * 4), b = ld4(s.shift + c4 * 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float4& t = v[u][k];
          t.x = fmaxf(fmaf(t.x, a.x, b.x), 0.f);
          t.y = fmaxf(fmaf(t.y, a.y, b.y), 0.f);
          t.z = fmaxf(fmaf(t.z, a.z, b.z), 0.f);
          t.w = fmaxf(fmaf(t.w, a.w, b.w), 0.f);
        }
      }
      if (anorm) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          *reinterpret_cast<uint2*>(anorm + sb0[u] + ((size_t)(k >> 1) * s.W + (k & 1)) * C) =
              make_uint2(bf16pack(v[u][k].x, v[u][k].y), bf16pack(v[u][k].z, v[u][k].w));
      }
      float4 best = v[u][0];
      uchar4 am = make_uchar4(0, 0, 0, 0);
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        if (v[u][k].x > best.x) { best.x = v[u][k].x; am.x = k; }
        if (v[u][k].y > best.y) { best.y = v[u][k].y; am.y = k; }
        if (v[u][k].z > best.z) { best.z = v[u][k].z; am.z = k; }
        if (v[u][k].w > best.w) { best.w = v[u][k].w; am.w = k; }
      }
      if (H16)
        reinterpret_cast<uint2*>(y)[i] = make_uint2(bf16pack(best.x, best.y), bf16pack(best.z, best.w));
      else
        st4(y + i * 4, best);
      *reinterpret_cast<uchar4*>(arg + i * 4) = am;
    }
  }
}

// bf16 in / bf16 out twin of k_maxpool_fwd<1, 1>: 8 channels (16 B) per lane
// instead of 4 (8 B), the same fmaf / fmaxf / strict '>' / RNE per element, so
// the pooled map, argmax bytes and normalised copy are bit-identical to it
__global__ __launch_bounds__(256) void k_maxpool_fwd_bf8(Src s, int n, int h, int w, uint16_t* __restrict__ y,
                                                         uint8_t* __restrict__ arg, uint16_t* __restrict__ anorm) {
  const int C = s.C, C8 = C / 8, ho = h / 2, wo = w / 2;
  const long long total = (long long)n * ho * wo * C8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const uint16_t* src = reinterpret_cast<const uint16_t*>(s.ptr);
  constexpr int U = 2;  // items per trip, every window load issued before any use
  for (long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x; i0 < total; i0 += U * stride) {
    uint4 raw[U][4];
    size_t sb0[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = min(i0 + u * stride, total - 1);  // tail items recompute the last one (not stored)
      const int c8 = (int)(i % C8);
      long long p = i / C8;
      const int xo = (int)(p % wo);
      p /= wo;
      const int yo = (int)(p % ho);
      const int nn = (int)(p / ho);
      sb0[u] = ((size_t)(nn * s.H + 2 * yo + s.oy) * s.W + 2 * xo + s.ox) * C + c8 * 8;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        raw[u][k] = *reinterpret_cast<const uint4*>(src + sb0[u] + ((size_t)(k >> 1) * s.W + (k & 1)) * C);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i >= total) continue;
      const int c = (int)(i % C8) * 8;
      float4 v[4][2];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k][0] = bf16x4_to_f4(make_uint2(raw[u][k].x, raw[u][k].y));
        v[k][1] = bf16x4_to_f4(make_uint2(raw[u][k].z, raw[u][k].w));
      }
      if (s.scale) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const float4 a = ld4(s.scale + c + 4 * hh), b = ld4(s.shift + c + 4 * hh);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float4& t = v[k][hh];
            t.x = fmaxf(fmaf(t.x, a.x, b.x), 0.f);
            t.y = fmaxf(fmaf(t.y, a.y, b.y), 0.f);
            t.z = fmaxf(fmaf(t.z, a.z, b.z), 0.f);
            t.w = fmaxf(fmaf(t.w, a.w, b.w), 0.f);
          }
        }
      }
      if (anorm) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          *reinterpret_cast<uint4*>(anorm + sb0[u] + ((size_t)(k >> 1) * s.W + (k & 1)) * C) =
              bf16pack8(v[k][0], v[k][1]);
      }
      float4 best[2];
      uchar4 am[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        best[hh] = v[0][hh];
        am[hh] = make_uchar4(0, 0, 0, 0);
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          if (v[k][hh].x > best[hh].x) { best[hh].x = v[k][hh].x; am[hh].x = k; }
          if (v[k][hh].y > best[hh].y) { best[hh].y = v[k][hh].y; am[hh].y = k; }
          if (v[k][hh].z > best[hh].z) { best[hh].z = v[k][hh].z; am[hh].z = k; }
          if (v[k][hh].w > best[hh].w) { best[hh].w = v[k][hh].w; am[hh].w = k; }
        }
      }
      reinterpret_cast<uint4*>(y)[i] = bf16pack8(best[0], best[1]);
      uint2 ab;
      ab.x = (unsigned)am[0].x | ((unsigned)am[0].y << 8) | ((unsigned)am[0].z << 16) | ((unsigned)am[0].w << 24);
      ab.y = (unsigned)am[1].x | ((unsigned)am[1].y << 8) | ((unsigned)am[1].z << 16) | ((unsigned)am[1].w << 24);
      reinterpret_cast<uint2*>(arg)[i] = ab;
    }
  }
}

// unet_set_tuning("maxpool_vec8", 0): the 4-channel forward (A/B tests).  An
// 8-channel twin of k_maxpool_bwd_fused<1, 1> was measured too: with its
// statistics partials kept bit-identical (128-lane blocks on the same grid) it
// ran no faster (118 vs 115 us per launch), so the backward keeps 4 channels.
int g_maxpool_vec8 = 1;

hipError_t launch_maxpool_fwd(const Src& s, int n, int h, int w, float* y, uint8_t* arg, hipStream_t st,
                              int out_h16, uint16_t* anorm) {
  if (s.C % 4 || (anorm && (s.oy || s.ox))) return hipErrorInvalidValue;
  if (g_maxpool_vec8 && out_h16 && s.h16 && s.C % 8 == 0) {
    const long long work8 = (long long)n * (h / 2) * (w / 2) * (s.C / 8);
    hipLaunchKernelGGL(k_maxpool_fwd_bf8, dim3(grid_cap(work8, 256, 8192)), dim3(256), 0, st, s, n, h, w,
                       reinterpret_cast<uint16_t*>(y), arg, anorm);
    return hipGetLastError();
  }
  const long long work = (long long)n * (h / 2) * (w / 2) * (s.C / 4);
  const dim3 grid(grid_cap(work, 256, 8192));
  switch (out_h16 * 2 + (s.h16 ? 1 : 0)) {
    case 0: hipLaunchKernelGGL((k_maxpool_fwd<0, 0>), grid, dim3(256), 0, st, s, n, h, w, y, arg, anorm); break;
    case 1: hipLaunchKernelGGL((k_maxpool_fwd<0, 1>), grid, dim3(256), 0, st, s, n, h, w, y, arg, anorm); break;
    case 2: hipLaunchKernelGGL((k_maxpool_fwd<1, 0>), grid, dim3(256), 0, st, s, n, h, w, y, arg, anorm); break;
    default: hipLaunchKernelGGL((k_maxpool_fwd<1, 1>), grid, dim3(256), 0, st, s, n, h, w, y, arg, anorm); break;
  }
  return hipGetLastError();
}

// a = bf16(relu(y * scale + shift)) over an NHWC bf16 tensor (8 channels = 16 B
// per lane-step): the normalised copy a bf16 plan's GEMMs read as a plain
// operand (BatchNorm + ReLU of the producer applied once per element instead
// of in every consumer's staging path; the same fmaf / max / RNE, so the
// operand bits are those of the on-load transform).
__global__ __launch_bounds__(256) void k_bn_relu_bf(const uint16_t* __restrict__ y, const float* __restrict__ scale,
                                                    const float* __restrict__ shift, long long n8, int c8,
                                                    uint16_t* __restrict__ a) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % c8) * 8;
    const uint4 u = reinterpret_cast<const uint4*>(y)[i];
    const float4 r0 = affine_relu4(bf16x4_to_f4(make_uint2(u.x, u.y)), ld4(scale + c), ld4(shift + c));
    const float4 r1 = affine_relu4(bf16x4_to_f4(make_uint2(u.z, u.w)), ld4(scale + c + 4), ld4(shift + c + 4));
    reinterpret_cast<uint4*>(a)[i] = bf16pack8(r0, r1);
  }
}

hipError_t launch_bn_relu_bf(const uint16_t* y, const float* scale, const float* shift, long long pixels, int c,
                             uint16_t* a, hipStream_t s) {
  if (c % 8) return hipErrorInvalidValue;
  const long long n8 = pixels * (c / 8);
  hipLaunchKernelGGL(k_bn_relu_bf, dim3(grid_cap(n8, 256, 8192)), dim3(256), 0, s, y, scale, shift, n8, c / 8, a);
  return hipGetLastError();
}

// Maxpool backward fused with the skip-gradient add (the encoder output feeds
// both the pool and the center-cropped concat, models/unet_model.py:107,130-142),
// the ReLU mask and the BN-backward statistics of that layer.
// G16: the gradients (dpool, dskip in; dz out) stored bf16 (bf16 plans; dz is
// rounded before its BN-backward statistics)
template <int Y16, int G16 = 0>  // y stored bf16
__global__ __launch_bounds__(256) void k_maxpool_bwd_fused(const float* __restrict__ dpool,
                                                           const uint8_t* __restrict__ arg,
                                                           const float* __restrict__ dskip, int soy, int sox,
                                                           int sh, int sw, const float* __restrict__ yr,
                                                           const float* scale, const float* shift,
                                                           const float* mean, const float* invstd, int n, int h,
                                                           int w, int C, float* __restrict__ dz,
                                                           double* __restrict__ bstats) {
  const int C4 = C / 4;            // channel groups; C4 divides 256 (C <= 1024, power of 2)
  const int tid = threadIdx.x;
  const int cg = tid % C4;
  const int ppb = 256 / C4;        // pixels of one row per block
  const int ho = h / 2, wo = w / 2;
  float sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
  const int c = cg * 4;
  float4 sc = make_float4(0, 0, 0, 0), sf = sc, mu = sc, is = sc;
  if (scale) { sc = ld4(scale + c); sf = ld4(shift + c); mu = ld4(mean + c); is = ld4(invstd + c); }
  // grid: x over ppb-pixel segments of a row, y over row pairs (the two input
  // rows of one pooled row; an odd last row is alone): the pooled gradient and
  // argmax are read once for both rows, and both rows' loads are in flight
  // together.  The row-pair index is the only division.
  const int xx = blockIdx.x * ppb + tid / C4;
  const int hq = (h + 1) / 2;
  // U row pairs per loop trip, all their loads issued before any use: the
  // kernel is latency-bound (one HBM round trip per trip), not bandwidth-bound
  constexpr int U = 4;
  if (xx < w) {
    const int xo = xx >> 1;
    const bool in_skip_x = dskip && xx >= sox && xx < sox + sw;
    const int nq = n * hq;
    const int qe = nq, qs = gridDim.y;  // row pairs strided over the grid's y (a contiguous run per block measured the same)
    for (int q0 = blockIdx.y; q0 < qe; q0 += U * qs) {
      // Branch-free loads from clamped addresses, validity applied afterwards:
      // a load inside a conditional region gets its own s_waitcnt at the
      // region's end, which serialised every load of the trip.
      uchar4 a[U];
      float4 g[U], d[U][2], yv[U][2];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = min(q0 + u * qs, qe - 1);
        const int nn = q / hq, yo = q - nn * hq;
        const bool pin = yo < ho && xo < wo;
        const size_t pi = (((size_t)nn * ho + min(yo, ho - 1)) * wo + min(xo, wo - 1)) * C + c;
        const uchar4 av = *reinterpret_cast<const uchar4*>(arg + pi);
        const float4 gv = G16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(dpool) + pi))
                              : ld4(dpool + pi);
        a[u] = pin ? av : make_uchar4(255, 255, 255, 255);
        g[u] = pin ? gv : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int yy = min(2 * yo + k, h - 1);
          const bool sin = in_skip_x && yy >= soy && yy < soy + sh;
          const int sy = min(max(yy - soy, 0), sh - 1), sx = in_skip_x ? xx - sox : 0;
          // absent operands read element 0 of the pooled gradient instead (no branch)
          const float* dsp = dskip ? dskip : dpool;
          const size_t si = dskip ? (((size_t)nn * sh + sy) * sw + sx) * C + c : 0;
          const float4 dv = G16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(dsp) + si))
                                : ld4(dsp + si);
          d[u][k] = sin ? dv : make_float4(0.f, 0.f, 0.f, 0.f);
          const float* yp = scale ? yr : dpool;
          const size_t oi = scale ? (((size_t)nn * h + yy) * w + xx) * C + c : 0;
          const bool y16 = scale ? Y16 != 0 : G16 != 0;
          yv[u][k] = y16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(yp) + oi))
                         : ld4(yp + oi);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int q = q0 + u * qs;
        if (q >= qe) continue;
        const int nn = q / hq, yo = q - nn * hq;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int yy = 2 * yo + k;
          if (yy >= h) continue;
          const int sel = k * 2 + (xx & 1);  // window position of this pixel (argmax byte 255: not pooled)
          float4 dd = d[u][k];
          dd.x += (a[u].x == sel) ? g[u].x : 0.f;
          dd.y += (a[u].y == sel) ? g[u].y : 0.f;
          dd.z += (a[u].z == sel) ? g[u].z : 0.f;
          dd.w += (a[u].w == sel) ? g[u].w : 0.f;
          if (G16) {
            dd.x = round_bf(dd.x);
            dd.y = round_bf(dd.y);
            dd.z = round_bf(dd.z);
            dd.w = round_bf(dd.w);
          }
          if (scale) {
            const float4 y4 = yv[u][k];
            dd.x = (fmaf(y4.x, sc.x, sf.x) > 0.f) ? dd.x : 0.f;
            dd.y = (fmaf(y4.y, sc.y, sf.y) > 0.f) ? dd.y : 0.f;
            dd.z = (fmaf(y4.z, sc.z, sf.z) > 0.f) ? dd.z : 0.f;
            dd.w = (fmaf(y4.w, sc.w, sf.w) > 0.f) ? dd.w : 0.f;
            sa[0] += dd.x; sa[1] += dd.y; sa[2] += dd.z; sa[3] += dd.w;
            sb[0] += dd.x * (y4.x - mu.x) * is.x;
            sb[1] += dd.y * (y4.y - mu.y) * is.y;
            sb[2] += dd.z * (y4.z - mu.z) * is.z;
            sb[3] += dd.w * (y4.w - mu.w) * is.w;
          }
          const size_t oi = (((size_t)nn * h + yy) * w + xx) * C + c;
          if (G16)
            reinterpret_cast<uint2*>(dz)[oi / 4] = make_uint2(bf16pack(dd.x, dd.y), bf16pack(dd.z, dd.w));
          else
            st4(dz + oi, dd);
        }
      }
    }
  }
  // every thread of the block takes part in the reduction (out-of-row lanes add zeros)
  if (bstats)
    reduce_pairs_to_global(sa, sb, C4, C,
                           bstats + (size_t)((blockIdx.y * gridDim.x + blockIdx.x) % kStatGroups) * C * 2);
}

hipError_t launch_maxpool_bwd_fused(const float* dpool, const uint8_t* arg, const float* dskip, int soy, int sox,
                                    int sh, int sw, const float* y, const float* scale, const float* shift,
                                    const float* mean, const float* invstd, int n, int h, int w, int c, float* dz,
                                    double* bstats, hipStream_t s, int y_h16, int g_h16) {
  if (c < 4 || c % 4 || (256 % (c / 4)) != 0) return hipErrorInvalidValue;
  const long long rows = (long long)n * ((h + 1) / 2);  // row pairs
  if ((long long)n * h * w >= (1LL << 31)) return hipErrorInvalidValue;
  const int ppb = 256 / (c / 4);
  const int gx = (w + ppb - 1) / ppb;
  // ~1024 blocks in all (per step at 512^2 x 8 with the branch-free batched
  // loads, bf16: 1024 blocks 0.32 ms; 512 and 4096 and a contiguous run of row
  // pairs per block measured slower or the same; before, each predicated load
  // waited out its own round trip: 0.51-0.56 ms)
  const dim3 grid(gx, (unsigned)std::max<long long>(1, std::min<long long>(rows, std::max(1, 1024 / gx))));
  if (g_h16) {
    if (!y_h16) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_maxpool_bwd_fused<1, 1>), grid, dim3(256), 0, s, dpool, arg, dskip, soy, sox, sh, sw, y, scale,
                       shift, mean, invstd, n, h, w, c, dz, bstats);
  } else if (y_h16)
    hipLaunchKernelGGL(k_maxpool_bwd_fused<1>, grid, dim3(256), 0, s, dpool, arg, dskip, soy, sox, sh, sw, y, scale,
                       shift, mean, invstd, n, h, w, c, dz, bstats);
  else
    hipLaunchKernelGGL(k_maxpool_bwd_fused<0>, grid, dim3(256), 0, s, dpool, arg, dskip, soy, sox, sh, sw, y, scale,
                       shift, mean, invstd, n, h, w, c, dz, bstats);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// OutConv 1x1 head (models/unet_model.py:56-63): logits[n][k][y][x] =
// b[k] + sum_c W[k][c] * relu(bn(y))[c].  16 lanes per pixel (C = 64).
// ---------------------------------------------------------------------------
// K: class capacity of the instantiation, kn <= K the model's classes (the
// first 4 counts have their own instantiations; 5-8, 9-16 share one).  A pass
// writes classes koff .. koff + kn - 1 of ktot (more than 16 classes: one pass
// per 16, a lane per class in the 16-lane pixel group).
template <int K>
__global__ __launch_bounds__(256) void k_head_fwd(Src s, int n, int h, int w, const float* __restrict__ wt,
                                                  const float* __restrict__ bias, float* __restrict__ logits, int kn,
                                                  int koff, int ktot) {
  const int tid = threadIdx.x, sub = tid & 15;
  const long long pixels = (long long)n * h * w;
  const int c = sub * 4;
  float4 wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = k < kn ? ld4(wt + (koff + k) * 64 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sc = make_float4(1, 1, 1, 1), sf = make_float4(0, 0, 0, 0);
  if (s.scale) { sc = ld4(s.scale + c); sf = ld4(s.shift + c); }
  for (long long p = (long long)blockIdx.x * 16 + (tid >> 4); p < pixels; p += (long long)gridDim.x * 16) {
    const int xx = (int)(p % w);
    const long long t = p / w;
    const int yy = (int)(t % h);
    const int nn = (int)(t / h);
    const size_t si = ((size_t)(nn * s.H + yy + s.oy) * s.W + xx + s.ox) * 64 + c;
    float4 v = s.h16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(s.ptr) + si))
                     : ld4(s.ptr + si);
    if (s.scale) {
      v.x = fmaxf(fmaf(v.x, sc.x, sf.x), 0.f);
      v.y = fmaxf(fmaf(v.y, sc.y, sf.y), 0.f);
      v.z = fmaxf(fmaf(v.z, sc.z, sf.z), 0.f);
      v.w = fmaxf(fmaf(v.w, sc.w, sf.w), 0.f);
    }
    float acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      acc[k] = v.x * wk[k].x + v.y * wk[k].y + v.z * wk[k].z + v.w * wk[k].w;
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) acc[k] += __shfl_xor(acc[k], o);
    }
    if (sub < kn) {
      float val = acc[0];
#pragma unroll
      for (int k = 1; k < K; ++k)
        if (sub == k) val = acc[k];
      logits[(((size_t)nn * ktot + koff + sub) * h + yy) * w + xx] = val + bias[koff + sub];
    }
  }
}

// head backward: dz = W^T dl masked by ReLU'(bn(y)) (+ BN-bwd stats), dW, db.
// Classes koff .. koff + kn - 1 of ktot; DZ = 0 (more than kMaxClasses classes):
// only this class slice's dW / db, dz comes from k_head_bwd_dz.  TF = 0 (the
// per-op 1x1 conv, unet_conv1x1_bwd): the input is read as is -- no BN+ReLU
// transform, no mask, no statistics.
template <int K, int Y16, int DZ = 1, int TF = 1>  // class capacity (kn <= K, as k_head_fwd); Y16: y stored bf16
__global__ __launch_bounds__(256) void k_head_bwd(Src s, const float* __restrict__ dl, int n, int h, int w,
                                                  const float* __restrict__ wt, const float* __restrict__ mean,
                                                  const float* __restrict__ invstd, float* __restrict__ dz,
                                                  double* __restrict__ bstats, double* __restrict__ acc_out,
                                                  int dz16, int kn, int koff, int ktot) {
  const int tid = threadIdx.x, sub = tid & 15;
  const int pixels = n * h * w;  // < 2^31 (launch_head_bwd)
  const int c = sub * 4;
  float4 wk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) wk[k] = k < kn ? ld4(wt + (koff + k) * 64 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 one = make_float4(1.f, 1.f, 1.f, 1.f), zero = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 sc = TF ? ld4(s.scale + c) : one, sf = TF ? ld4(s.shift + c) : zero;
  const float4 mu = TF ? ld4(mean + c) : zero, is = TF ? ld4(invstd + c) : one;
  float dwa[K][4], dba[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    dba[k] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) dwa[k][j] = 0.f;
  }
  float sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
  const int hw = h * w;
  // U pixels per loop trip, every load issued (branch-free, clamped) before any
  // use: the loop was one or two HBM round trips per pixel
  constexpr int U = 4;
  const int stride = gridDim.x * 16;
  for (int p0 = blockIdx.x * 16 + (tid >> 4); p0 < pixels; p0 += U * stride) {
    float4 yv[U];
    float g[U][K];
    int rr[U], nnu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = min(p0 + u * stride, pixels - 1);
      const int nn = p / hw, r = p - nn * hw;
      const int y = r / w, x = r - y * w;
      nnu[u] = nn;
      rr[u] = r;
      const size_t ii = ((size_t)(nn * s.H + y + s.oy) * s.W + x + s.ox) * 64 + c;
      yv[u] = Y16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(s.ptr) + ii))
                  : ld4(s.ptr + ii);
#pragma unroll
      for (int k = 0; k < K; ++k) g[u][k] = dl[((size_t)nn * ktot + koff + min(k, kn - 1)) * hw + r];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = p0 + u * stride;
      if (p >= pixels) continue;
#pragma unroll
      for (int k = 0; k < K; ++k) g[u][k] = k < kn ? g[u][k] : 0.f;
      const float zx = TF ? fmaf(yv[u].x, sc.x, sf.x) : yv[u].x, zy = TF ? fmaf(yv[u].y, sc.y, sf.y) : yv[u].y,
                  zz = TF ? fmaf(yv[u].z, sc.z, sf.z) : yv[u].z, zw = TF ? fmaf(yv[u].w, sc.w, sf.w) : yv[u].w;
      const float ax = TF ? fmaxf(zx, 0.f) : zx, ay = TF ? fmaxf(zy, 0.f) : zy, az = TF ? fmaxf(zz, 0.f) : zz,
                  aw = TF ? fmaxf(zw, 0.f) : zw;
      float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        d.x = fmaf(wk[k].x, g[u][k], d.x);
        d.y = fmaf(wk[k].y, g[u][k], d.y);
        d.z = fmaf(wk[k].z, g[u][k], d.z);
        d.w = fmaf(wk[k].w, g[u][k], d.w);
        dwa[k][0] += g[u][k] * ax;
        dwa[k][1] += g[u][k] * ay;
        dwa[k][2] += g[u][k] * az;
        dwa[k][3] += g[u][k] * aw;
        dba[k] += g[u][k];
      }
      if (!DZ) continue;
      if (!TF) {
        st4(dz + (size_t)p * 64 + c, d);
        continue;
      }
      d.x = zx > 0.f ? d.x : 0.f;
      d.y = zy > 0.f ? d.y : 0.f;
      d.z = zz > 0.f ? d.z : 0.f;
      d.w = zw > 0.f ? d.w : 0.f;
      if (dz16) {  // bf16 plans store dz bf16: statistics of the rounded values
        d.x = round_bf(d.x);
        d.y = round_bf(d.y);
        d.z = round_bf(d.z);
        d.w = round_bf(d.w);
      }
      sa[0] += d.x; sa[1] += d.y; sa[2] += d.z; sa[3] += d.w;
      sb[0] += d.x * (yv[u].x - mu.x) * is.x;
      sb[1] += d.y * (yv[u].y - mu.y) * is.y;
      sb[2] += d.z * (yv[u].z - mu.z) * is.z;
      sb[3] += d.w * (yv[u].w - mu.w) * is.w;
      if (dz16)
        reinterpret_cast<uint2*>(dz)[((size_t)p * 64 + c) / 4] = make_uint2(bf16pack(d.x, d.y), bf16pack(d.z, d.w));
      else
        st4(dz + (size_t)p * 64 + c, d);
    }
  }
  if (DZ && TF) reduce_pairs_to_global(sa, sb, 16, 64, bstats + (size_t)(blockIdx.x % kStatGroups) * 64 * 2);
  __syncthreads();
  __shared__ float red[256][4];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k >= kn) continue;  // uniform
#pragma unroll
    for (int j = 0; j < 4; ++j) red[tid][j] = dwa[k][j];
    __syncthreads();
    if (tid < 16) {
      float t[4] = {0, 0, 0, 0};
      for (int rr = tid; rr < 256; rr += 16)
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] += red[rr][j];
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(acc_out + (koff + k) * 64 + tid * 4 + j, (double)t[j]);
    }
    __syncthreads();
    red[tid][0] = (sub == 0) ? dba[k] : 0.f;
    __syncthreads();
    if (tid == 0) {
      float t = 0.f;
      for (int rr = 0; rr < 256; rr += 16) t += red[rr][0];
      atomicAdd(acc_out + ktot * 64 + koff + k, (double)t);
    }
    __syncthreads();
  }
}

// head backward input gradient for more than kMaxClasses classes: the class
// loop at run time, W rows read through the cache (same arithmetic order as
// k_head_bwd's d: fmaf over k ascending); ReLU mask, bf16 rounding and the
// BN-backward statistics as there.
template <int Y16, int TF = 1>
__global__ __launch_bounds__(256) void k_head_bwd_dz(Src s, const float* __restrict__ dl, int n, int h, int w,
                                                     const float* __restrict__ wt, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd, float* __restrict__ dz,
                                                     double* __restrict__ bstats, int dz16, int kn) {
  const int tid = threadIdx.x, sub = tid & 15;
  const int pixels = n * h * w;
  const int c = sub * 4;
  const float4 one = make_float4(1.f, 1.f, 1.f, 1.f), zero = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 sc = TF ? ld4(s.scale + c) : one, sf = TF ? ld4(s.shift + c) : zero;
  const float4 mu = TF ? ld4(mean + c) : zero, is = TF ? ld4(invstd + c) : one;
  float sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
  const int hw = h * w;
  for (int p = blockIdx.x * 16 + (tid >> 4); p < pixels; p += gridDim.x * 16) {
    const int nn = p / hw, r = p - nn * hw;
    const int y = r / w, x = r - y * w;
    const size_t ii = ((size_t)(nn * s.H + y + s.oy) * s.W + x + s.ox) * 64 + c;
    const float4 yv = Y16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(s.ptr) + ii))
                          : ld4(s.ptr + ii);
    float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < kn; ++k) {
      const float g = dl[((size_t)nn * kn + k) * hw + r];
      const float4 wk = ld4(wt + k * 64 + c);
      d.x = fmaf(wk.x, g, d.x);
      d.y = fmaf(wk.y, g, d.y);
      d.z = fmaf(wk.z, g, d.z);
      d.w = fmaf(wk.w, g, d.w);
    }
    if (!TF) {
      st4(dz + (size_t)p * 64 + c, d);
      continue;
    }
    const float zx = fmaf(yv.x, sc.x, sf.x), zy = fmaf(yv.y, sc.y, sf.y), zz = fmaf(yv.z, sc.z, sf.z),
                zw = fmaf(yv.w, sc.w, sf.w);
    d.x = zx > 0.f ? d.x : 0.f;
    d.y = zy > 0.f ? d.y : 0.f;
    d.z = zz > 0.f ? d.z : 0.f;
    d.w = zw > 0.f ? d.w : 0.f;
    if (dz16) {
      d.x = round_bf(d.x);
      d.y = round_bf(d.y);
      d.z = round_bf(d.z);
      d.w = round_bf(d.w);
    }
    sa[0] += d.x; sa[1] += d.y; sa[2] += d.z; sa[3] += d.w;
    sb[0] += d.x * (yv.x - mu.x) * is.x;
    sb[1] += d.y * (yv.y - mu.y) * is.y;
    sb[2] += d.z * (yv.z - mu.z) * is.z;
    sb[3] += d.w * (yv.w - mu.w) * is.w;
    if (dz16)
      reinterpret_cast<uint2*>(dz)[((size_t)p * 64 + c) / 4] = make_uint2(bf16pack(d.x, d.y), bf16pack(d.z, d.w));
    else
      st4(dz + (size_t)p * 64 + c, d);
  }
  if (TF) reduce_pairs_to_global(sa, sb, 16, 64, bstats + (size_t)(blockIdx.x % kStatGroups) * 64 * 2);
}

__global__ void k_d2f(const double* __restrict__ a, int n, float* __restrict__ o) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = (float)a[i];
}

// largest class count of the register-blocked head backward and loss (K values
// per thread); models/unet_model.py:66 takes any count: above it the head
// backward runs k_head_bwd_dz + class slices of k_head_bwd<32, *, 0>, the loss
// k_wce_gen (run-time class loop)
constexpr int kMaxClasses = 32;
static int class_capacity(int k) { return k <= 4 ? k : k <= 8 ? 8 : k <= 16 ? 16 : 32; }

hipError_t launch_head_fwd(const Src& s, int n, int h, int w, int c, const float* wt, const float* bias, int k,
                           float* logits, hipStream_t st) {
  if (c != 64 || k < 1) return hipErrorInvalidValue;
  const long long pixels = (long long)n * h * w;
  dim3 grid(grid_cap(pixels, 16 * 4, 8192));
  for (int k0 = 0; k0 < k; k0 += 16) {
    const int kn = k - k0 < 16 ? k - k0 : 16;
    switch (class_capacity(kn)) {
      case 1: hipLaunchKernelGGL(k_head_fwd<1>, grid, dim3(256), 0, st, s, n, h, w, wt, bias, logits, kn, k0, k); break;
      case 2: hipLaunchKernelGGL(k_head_fwd<2>, grid, dim3(256), 0, st, s, n, h, w, wt, bias, logits, kn, k0, k); break;
      case 3: hipLaunchKernelGGL(k_head_fwd<3>, grid, dim3(256), 0, st, s, n, h, w, wt, bias, logits, kn, k0, k); break;
      case 4: hipLaunchKernelGGL(k_head_fwd<4>, grid, dim3(256), 0, st, s, n, h, w, wt, bias, logits, kn, k0, k); break;
      case 8: hipLaunchKernelGGL(k_head_fwd<8>, grid, dim3(256), 0, st, s, n, h, w, wt, bias, logits, kn, k0, k); break;
      default: hipLaunchKernelGGL(k_head_fwd<16>, grid, dim3(256), 0, st, s, n, h, w, wt, bias, logits, kn, k0, k); break;
    }
  }
  return hipGetLastError();
}

hipError_t launch_head_bwd(const Src& s, const float* dl, int n, int h, int w, int c, const float* wt, int k,
                           const float* yraw, const float* mean, const float* invstd, float* dz, double* bstats,
                           float* dw, float* db, double* acc, hipStream_t st, int dz_h16) {
  (void)yraw;
  if (c != 64 || k < 1) return hipErrorInvalidValue;
  const long long pixels = (long long)n * h * w;
  // 512 blocks: the per-block fp64 atomics (BN statistics, dW, db) bound this
  // kernel at larger grids (measured: 256 blocks 199 us, 512 146 us, 2048 236 us)
  dim3 grid(grid_cap(pixels, 16 * 8, 512));
  hipError_t me = hipMemsetAsync(acc, 0, sizeof(double) * (k * 64 + k), st);
  if (me != hipSuccess) return me;
  if (pixels >= (1LL << 31)) return hipErrorInvalidValue;
  if (k > kMaxClasses) {
    if (s.h16)
      hipLaunchKernelGGL((k_head_bwd_dz<1>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, mean, invstd, dz, bstats,
                         dz_h16, k);
    else
      hipLaunchKernelGGL((k_head_bwd_dz<0>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, mean, invstd, dz, bstats,
                         dz_h16, k);
    for (int k0 = 0; k0 < k; k0 += kMaxClasses) {
      const int kn = k - k0 < kMaxClasses ? k - k0 : kMaxClasses;
      if (s.h16)
        hipLaunchKernelGGL((k_head_bwd<kMaxClasses, 1, 0>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, mean, invstd,
                           dz, bstats, acc, dz_h16, kn, k0, k);
      else
        hipLaunchKernelGGL((k_head_bwd<kMaxClasses, 0, 0>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, mean, invstd,
                           dz, bstats, acc, dz_h16, kn, k0, k);
    }
    hipLaunchKernelGGL(k_d2f, dim3(cdiv(k * 64, 256)), dim3(256), 0, st, acc, k * 64, dw);
    hipLaunchKernelGGL(k_d2f, dim3(cdiv(k, 256)), dim3(256), 0, st, acc + k * 64, k, db);
    return hipGetLastError();
  }
#define HEAD_BWD(KK)                                                                                            \
  do {                                                                                                          \
    if (s.h16)                                                                                                  \
      hipLaunchKernelGGL((k_head_bwd<KK, 1>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, mean, invstd, dz, bstats, \
                         acc, dz_h16, k, 0, k);                                                                 \
    else                                                                                                        \
      hipLaunchKernelGGL((k_head_bwd<KK, 0>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, mean, invstd, dz, bstats, \
                         acc, dz_h16, k, 0, k);                                                                 \
  } while (0)
  switch (class_capacity(k)) {
    case 1: HEAD_BWD(1); break;
    case 2: HEAD_BWD(2); break;
    case 3: HEAD_BWD(3); break;
    case 4: HEAD_BWD(4); break;
    case 8: HEAD_BWD(8); break;
    case 16: HEAD_BWD(16); break;
    default: HEAD_BWD(32); break;
  }
#undef HEAD_BWD
  hipLaunchKernelGGL(k_d2f, dim3(cdiv(k * 64, 256)), dim3(256), 0, st, acc, k * 64, dw);
  hipLaunchKernelGGL(k_d2f, dim3(1), dim3(64), 0, st, acc + k * 64, k, db);
  return hipGetLastError();
}

// 1x1 conv backward on a plain (already activated) fp32 NHWC input, any class
// count (the per-op unet_conv1x1_bwd): dx = W^T dl, dW, db (acc: k*64 + k doubles)
hipError_t launch_head_bwd_plain(const float* x, const float* dl, int n, int h, int w, const float* wt, int k,
                                 float* dx, float* dw, float* db, double* acc, hipStream_t st) {
  if (k < 1) return hipErrorInvalidValue;
  const long long pixels = (long long)n * h * w;
  if (pixels >= (1LL << 31)) return hipErrorInvalidValue;
  Src s;
  s.ptr = x;
  s.H = h;
  s.W = w;
  s.C = 64;
  dim3 grid(grid_cap(pixels, 16 * 8, 512));
  hipError_t me = hipMemsetAsync(acc, 0, sizeof(double) * (k * 64 + k), st);
  if (me != hipSuccess) return me;
  if (dx)
    hipLaunchKernelGGL((k_head_bwd_dz<0, 0>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, nullptr, nullptr, dx,
                       nullptr, 0, k);
  for (int k0 = 0; k0 < k; k0 += kMaxClasses) {
    const int kn = k - k0 < kMaxClasses ? k - k0 : kMaxClasses;
    hipLaunchKernelGGL((k_head_bwd<kMaxClasses, 0, 0, 0>), grid, dim3(256), 0, st, s, dl, n, h, w, wt, nullptr,
                       nullptr, nullptr, nullptr, acc, 0, kn, k0, k);
  }
  hipLaunchKernelGGL(k_d2f, dim3(cdiv(k * 64, 256)), dim3(256), 0, st, acc, k * 64, dw);
  hipLaunchKernelGGL(k_d2f, dim3(cdiv(k, 256)), dim3(256), 0, st, acc + k * 64, k, db);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// WeightedCrossEntropyLoss (utils/losses.py:29-57), forward and backward fused:
// loss = mean(w * (logsumexp(l) - l[t]));  dl = w*(softmax - onehot)/count.
// targets/weights through element strides (the caller's cropped views).
// ---------------------------------------------------------------------------
// K: class capacity, kn <= K classes.  A label outside [0, kn) other than
// ignore_index (-100) contributes nothing and raises a flag: acc[1] = 1,
// acc[2] = the label (torch's nn.CrossEntropyLoss raises "Target t is out of
// bounds"; the host reads the flag at its next synchronisation point instead of
// synchronising every step).
template <int K>
__global__ __launch_bounds__(256) void k_wce(const float* __restrict__ lg, const int64_t* __restrict__ t,
                                             const float* __restrict__ wm, int n, int h, int w, int64_t ts0,
                                             int64_t ts1, int64_t ts2, int64_t ws0, int64_t ws1, int64_t ws2,
                                             float* __restrict__ dl, float gscale, double* __restrict__ acc, int kn) {
  const long long hw = (long long)h * w, total = (long long)n * hw;
  const double inv = 1.0 / (double)total;
  float local = 0.f;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < total;
       p += (long long)gridDim.x * blockDim.x) {
    const int nn = (int)(p / hw);
    const long long r = p - nn * hw;
    const int yy = (int)(r / w), xx = (int)(r % w);
    float l[K];
#pragma unroll
    for (int k = 0; k < K; ++k) l[k] = k < kn ? lg[((size_t)nn * kn + k) * hw + r] : -INFINITY;
    const int64_t tg = t[nn * ts0 + yy * ts1 + xx * ts2];
    const float wt = wm[nn * ws0 + yy * ws1 + xx * ws2];
    float mx = l[0];
#pragma unroll
    for (int k = 1; k < K; ++k) mx = fmaxf(mx, l[k]);
    float se = 0.f, e[K];
#pragma unroll
    for (int k = 0; k < K; ++k) { e[k] = k < kn ? __expf(l[k] - mx) : 0.f; se += e[k]; }
    const float lse = mx + __logf(se);
    const bool valid = (tg >= 0 && tg < kn);   // ignore_index (-100) -> 0 loss, 0 grad
    if (!valid && tg != -100) {
      acc[1] = 1.0;
      acc[2] = (double)tg;
    }
    float lt = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k == tg) lt = l[k];
    if (valid) local += wt * (lse - lt);
    const float sc = valid ? (float)((double)wt * inv) * gscale : 0.f;
    const float rs = 1.f / se;
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k < kn) dl[((size_t)nn * kn + k) * hw + r] = sc * (e[k] * rs - (k == tg ? 1.f : 0.f));
  }
  for (int o = 32; o >= 1; o >>= 1) local += __shfl_xor(local, o);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = local;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(acc, (double)(red[0] + red[1] + red[2] + red[3]));
}

// more than kMaxClasses classes: the same arithmetic with the class loop at run
// time (the logits of a pixel are read twice: max / sum, then the gradient)
__global__ __launch_bounds__(256) void k_wce_gen(const float* __restrict__ lg, const int64_t* __restrict__ t,
                                                 const float* __restrict__ wm, int n, int h, int w, int64_t ts0,
                                                 int64_t ts1, int64_t ts2, int64_t ws0, int64_t ws1, int64_t ws2,
                                                 float* __restrict__ dl, float gscale, double* __restrict__ acc,
                                                 int kn) {
  const long long hw = (long long)h * w, total = (long long)n * hw;
  const double inv = 1.0 / (double)total;
  float local = 0.f;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < total;
       p += (long long)gridDim.x * blockDim.x) {
    const int nn = (int)(p / hw);
    const long long r = p - nn * hw;
    const int yy = (int)(r / w), xx = (int)(r % w);
    const float* l = lg + (size_t)nn * kn * hw + r;
    const int64_t tg = t[nn * ts0 + yy * ts1 + xx * ts2];
    const float wt = wm[nn * ws0 + yy * ws1 + xx * ws2];
    float mx = l[0];
    for (int k = 1; k < kn; ++k) mx = fmaxf(mx, l[(size_t)k * hw]);
    float se = 0.f, lt = 0.f;
    for (int k = 0; k < kn; ++k) {
      const float v = l[(size_t)k * hw];
      se += __expf(v - mx);
      if (k == tg) lt = v;
    }
    const float lse = mx + __logf(se);
    const bool valid = (tg >= 0 && tg < kn);
    if (!valid && tg != -100) {
      acc[1] = 1.0;
      acc[2] = (double)tg;
    }
    if (valid) local += wt * (lse - lt);
    const float sc = valid ? (float)((double)wt * inv) * gscale : 0.f;
    const float rs = 1.f / se;
    for (int k = 0; k < kn; ++k)
      dl[((size_t)nn * kn + k) * hw + r] = sc * (__expf(l[(size_t)k * hw] - mx) * rs - (k == tg ? 1.f : 0.f));
  }
  for (int o = 32; o >= 1; o >>= 1) local += __shfl_xor(local, o);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = local;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(acc, (double)(red[0] + red[1] + red[2] + red[3]));
}

__global__ void k_wce_final(const double* acc, double count, float* loss) { *loss = (float)(acc[0] / count); }

// Clears the sum, the bad-label flag and the bad label.  A kernel rather than a
// hipMemsetAsync, so that a captured step (Trainer(graph=True)) holds a kernel
// node ordered on the same queue as k_wce, not a memset node.
__global__ void k_wce_init(double* acc) {
  if (threadIdx.x < 3) acc[threadIdx.x] = 0.0;
}

hipError_t launch_wce(const float* logits, const int64_t* t, const float* wm, int n, int k, int h, int w,
                      const int64_t* ts, const int64_t* wsd, float* loss, float* dlogits, float gscale, double* acc,
                      hipStream_t s) {
  if (k < 1) return hipErrorInvalidValue;
  const long long total = (long long)n * h * w;
  dim3 grid(grid_cap(total, 256 * 4, 2048));
  hipLaunchKernelGGL(k_wce_init, dim3(1), dim3(64), 0, s, acc);
  if (k > kMaxClasses)
    hipLaunchKernelGGL(k_wce_gen, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1],
                       wsd[2], dlogits, gscale, acc, k);
  else
  switch (class_capacity(k)) {
    case 1: hipLaunchKernelGGL(k_wce<1>, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1], wsd[2], dlogits, gscale, acc, k); break;
    case 2: hipLaunchKernelGGL(k_wce<2>, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1], wsd[2], dlogits, gscale, acc, k); break;
    case 3: hipLaunchKernelGGL(k_wce<3>, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1], wsd[2], dlogits, gscale, acc, k); break;
    case 4: hipLaunchKernelGGL(k_wce<4>, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1], wsd[2], dlogits, gscale, acc, k); break;
    case 8: hipLaunchKernelGGL(k_wce<8>, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1], wsd[2], dlogits, gscale, acc, k); break;
    case 16: hipLaunchKernelGGL(k_wce<16>, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1], wsd[2], dlogits, gscale, acc, k); break;
    default: hipLaunchKernelGGL(k_wce<32>, grid, dim3(256), 0, s, logits, t, wm, n, h, w, ts[0], ts[1], ts[2], wsd[0], wsd[1], wsd[2], dlogits, gscale, acc, k); break;
  }
  hipLaunchKernelGGL(k_wce_final, dim3(1), dim3(1), 0, s, acc, (double)total, loss);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// torch.optim.SGD(momentum, dampening=0, nesterov=False, weight_decay=0) step.
// ---------------------------------------------------------------------------
__global__ void k_sgd(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ b, size_t n, float lr,
                      float mom, float gs, int first) {
  const size_t n4 = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 gv = ld4(g + 4 * i), pv = ld4(p + 4 * i), bv;
    gv.x *= gs; gv.y *= gs; gv.z *= gs; gv.w *= gs;
    if (first) {
      bv = gv;
    } else {
      bv = ld4(b + 4 * i);
      bv.x = fmaf(mom, bv.x, gv.x);
      bv.y = fmaf(mom, bv.y, gv.y);
      bv.z = fmaf(mom, bv.z, gv.z);
      bv.w = fmaf(mom, bv.w, gv.w);
    }
    pv.x = fmaf(-lr, bv.x, pv.x);
    pv.y = fmaf(-lr, bv.y, pv.y);
    pv.z = fmaf(-lr, bv.z, pv.z);
    pv.w = fmaf(-lr, bv.w, pv.w);
    st4(b + 4 * i, bv);
    st4(p + 4 * i, pv);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const size_t i = n4 * 4 + threadIdx.x;
    const float bv = first ? g[i] * gs : fmaf(mom, b[i], g[i] * gs);
    b[i] = bv;
    p[i] = fmaf(-lr, bv, p[i]);
  }
}

hipError_t launch_sgd(float* p, const float* g, float* buf, size_t n, float lr, float mom, float gs, int first,
                      hipStream_t s) {
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(buf)) & 15)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_sgd, dim3(grid_cap((long long)(n / 4 + 1), 256, 4096)), dim3(256), 0, s, p, g, buf, n, lr, mom,
                     gs, first);
  return hipGetLastError();
}

__global__ void k_scale_dev(const float* x, float* y, size_t n, const float* g) {
  const float s = *g;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = x[i] * s;
}
hipError_t launch_scale_by_dev(const float* x, float* y, size_t n, const float* g, hipStream_t s) {
  hipLaunchKernelGGL(k_scale_dev, dim3(grid_cap((long long)n, 256, 4096)), dim3(256), 0, s, x, y, n, g);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Weight repacks (per step; weights change every optimizer step).
//   conv fwd  B[co][t*Ci+ci]  = W[co][ci][t]
//   conv dgrad B[ci][t'*Co+co] = W[co][ci][T-1-t']   (flipped, transposed)
//   convT fwd  B[ab*Co+co][ci] = W[ci][co][ab]
//   convT dgrad B[ci][ab*Co+co] = W[ci][co][ab]
// ---------------------------------------------------------------------------
// out[a][c][b] = in[a][b][c], 32x32 (b, c) tiles through LDS so both the reads
// (rows of c) and the writes (rows of b) are contiguous.  grid = (ceil(C/32),
// ceil(B/32), A).
__global__ __launch_bounds__(256) void k_permute_last2(const float* __restrict__ in, int A, int B, int C,
                                                       float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int c0 = blockIdx.x * 32, b0 = blockIdx.y * 32;
  const size_t a = blockIdx.z;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int b = b0 + k, c = c0 + tx;
    if (b < B && c < C) tile[k][tx] = in[(a * B + b) * C + c];
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, b = b0 + tx;
    if (b < B && c < C) out[(a * C + c) * B + b] = tile[tx][k];
  }
}

// out[r2(s)][r] = in[r][s] for a [R][S] matrix with S = T*Cb, s = t*Cb + cb,
// r2 = cb*T + (flip ? T-1-t : t).  32x32 tiles through LDS.
__global__ void k_transpose_taps(const float* __restrict__ in, int R, int T, int Cb, int flip,
                                 float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int S = T * Cb;
  const int s0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, s = s0 + tx;
    tile[k][tx] = (r < R && s < S) ? in[(size_t)r * S + s] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int s = s0 + k, r = r0 + tx;
    if (s < S && r < R) {
      const int t = s / Cb, cb = s - t * Cb;
      const int r2 = cb * T + (flip ? T - 1 - t : t);
      out[(size_t)r2 * R + r] = tile[tx][k];
    }
  }
}

// Small inner dim C (taps, packing OIHW -> [co][tap][ci]): thread per (a, b)
// reads its C contiguous words, lanes write consecutive b (coalesced).
__global__ void k_permute_small_c(const float* __restrict__ in, long long AB, int B, int C, float* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < AB; i += (long long)gridDim.x * blockDim.x) {
    const long long a = i / B;
    const int b = (int)(i - a * B);
    const float* src = in + i * C;
    float* dst = out + a * (long long)C * B + b;
    for (int c = 0; c < C; ++c) dst[(long long)c * B] = src[c];
  }
}
// Small middle dim B (taps, unpacking [co][tap][ci] -> OIHW): thread per (a, c)
// reads lanes-consecutive c for every b, writes its B contiguous words.
__global__ void k_permute_small_b(const float* __restrict__ in, long long AC, int B, int C, float* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < AC; i += (long long)gridDim.x * blockDim.x) {
    const long long a = i / C;
    const int c = (int)(i - a * C);
    const float* src = in + a * (long long)B * C + c;
    float* dst = out + i * B;
    for (int b = 0; b < B; ++b) dst[b] = src[(long long)b * C];
  }
}

// out[a][c][b] = in[a][b][c] with one block per a: the B x C slab is read and
// written contiguously (coalesced both ways) through LDS, rows padded to C + 1
// words so the transposed reads spread over the banks.  Used when one of B, C is
// a tap count (<= 16) and the slab fits 64 KiB.
__global__ __launch_bounds__(256) void k_permute_slab(const float* __restrict__ in, int B, int C,
                                                      float* __restrict__ out) {
  extern __shared__ float slab[];
  const size_t base = (size_t)blockIdx.x * B * C;
  const int BC = B * C;
  for (int i = threadIdx.x; i < BC; i += 256) {
    const int b = i / C, c = i - b * C;
    slab[b * (C + 1) + c] = in[base + i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < BC; i += 256) {
    const int c = i / B, b = i - c * B;
    out[base + i] = slab[b * (C + 1) + c];
  }
}

hipError_t launch_permute_last2(const float* in, int A, int B, int C, float* out, hipStream_t s) {
  if (A <= 0 || B <= 0 || C <= 0) return hipErrorInvalidValue;
  const size_t slab_bytes = sizeof(float) * (size_t)B * (C + 1);
  if ((B <= 16 || C <= 16) && slab_bytes <= 65536 && A <= 0x7fffffff) {
    hipLaunchKernelGGL(k_permute_slab, dim3(A), dim3(256), slab_bytes, s, in, B, C, out);
  } else if (C <= 16) {
    const long long ab = (long long)A * B;
    hipLaunchKernelGGL(k_permute_small_c, dim3(grid_cap(ab, 256, 8192)), dim3(256), 0, s, in, ab, B, C, out);
  } else if (B <= 16) {
    const long long ac = (long long)A * C;
    hipLaunchKernelGGL(k_permute_small_b, dim3(grid_cap(ac, 256, 8192)), dim3(256), 0, s, in, ac, B, C, out);
  } else {
    if (A > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_permute_last2, dim3(cdiv(C, 32), cdiv(B, 32), A), dim3(256), 0, s, in, A, B, C, out);
  }
  return hipGetLastError();
}

hipError_t launch_pack_conv(const float* w, int co, int ci, int kh, int kw, float* wf, float* wd, hipStream_t s) {
  const int T = kh * kw;
  hipError_t e = launch_permute_last2(w, co, ci, T, wf, s);  // [co][T][ci]
  if (e != hipSuccess || !wd) return e;
  // wf viewed as [co][T*ci]: out row = ci*T + (T-1-t), col = co
  dim3 grid(cdiv((long long)T * ci, 32), cdiv(co, 32));
  hipLaunchKernelGGL(k_transpose_taps, grid, dim3(256), 0, s, wf, co, T, ci, 1, wd);
  return hipGetLastError();
}

hipError_t launch_pack_convT(const float* w, int ci, int co, float* wf, float* wd, hipStream_t s) {
  // wd[ci][ab][co] = W[ci][co][ab]
  hipError_t e = launch_permute_last2(w, ci, co, 4, wd, s);
  if (e != hipSuccess) return e;
  // wf[ab*co + c][ci] = wd[ci][ab*co + c]: plain transpose (T=1)
  dim3 grid(cdiv(4LL * co, 32), cdiv(ci, 32));
  hipLaunchKernelGGL(k_transpose_taps, grid, dim3(256), 0, s, wd, ci, 1, 4 * co, 0, wf);
  return hipGetLastError();
}

// Every per-step weight repack of a forward in ONE launch (round 4; it was 2
// launches per layer, 42 small-grid kernels in front of every forward): block =
// (job, 32 x 32 channel tile).  Conv jobs: W[co][ci][9] (OIHW) -> wf[co][t][ci]
// (forward B operand) and wd[ci*9 + 8-t][co] (input-gradient B operand, taps
// flipped); convT jobs: W[ci][co][4] -> wd[ci][ab][co] and wf[ab*co + c][ci].
// The tile goes through LDS (rows padded by one word: conflict-free transposed
// reads), every global access is a 128-B run.
__global__ __launch_bounds__(256) void k_pack_all(const PackJobs jobs) {
  __shared__ float t[32 * 289];
  int j = 0;
  while (j + 1 < jobs.n && (int)blockIdx.x >= jobs.first[j + 1]) ++j;
  const PackJob& J = jobs.j[j];
  const int b = blockIdx.x - jobs.first[j];
  const int tid = threadIdx.x;
  if (J.kind == 0) {  // conv 3x3
    const int CI = J.ci, CO = J.co, nct = CI / 32;
    const int co0 = (b / nct) * 32, ci0 = (b % nct) * 32;
    for (int i = tid; i < 32 * 288; i += 256) {
      const int r = i / 288, q = i - r * 288;  // q = ci_l * 9 + tap
      t[r * 289 + q] = J.w[((size_t)(co0 + r) * CI + ci0) * 9 + q];
    }
    __syncthreads();
    for (int i = tid; i < 32 * 9 * 32; i += 256) {  // wf: ci fastest
      const int c = i & 31, rt = i >> 5, r = rt / 9, tp = rt - r * 9;
      J.wf[((size_t)(co0 + r) * 9 + tp) * CI + ci0 + c] = t[r * 289 + c * 9 + tp];
    }
    if (J.wd)
      for (int i = tid; i < 32 * 9 * 32; i += 256) {  // wd: co fastest
        const int r = i & 31, ct = i >> 5, c = ct / 9, tp = ct - c * 9;
        J.wd[((size_t)(ci0 + c) * 9 + 8 - tp) * CO + co0 + r] = t[r * 289 + c * 9 + tp];
      }
  } else {  // convT 2x2 stride 2
    const int CI = J.ci, CO = J.co, nct = CO / 32;
    const int ci0 = (b / nct) * 32, co0 = (b % nct) * 32;
    for (int i = tid; i < 32 * 128; i += 256) {
      const int r = i >> 7, q = i & 127;  // q = co_l * 4 + ab
      t[r * 129 + q] = J.w[((size_t)(ci0 + r) * CO + co0) * 4 + q];
    }
    __syncthreads();
    for (int i = tid; i < 32 * 4 * 32; i += 256) {  // wd[ci][ab][co]: co fastest
      const int c = i & 31, ra = i >> 5, r = ra >> 2, ab = ra & 3;
      J.wd[((size_t)(ci0 + r) * 4 + ab) * CO + co0 + c] = t[r * 129 + c * 4 + ab];
    }
    for (int i = tid; i < 32 * 4 * 32; i += 256) {  // wf[ab*CO + co][ci]: ci fastest
      const int r = i & 31, ac = i >> 5, ab = ac >> 5, c = ac & 31;
      J.wf[((size_t)ab * CO + co0 + c) * CI + ci0 + r] = t[r * 129 + c * 4 + ab];
    }
  }
}

hipError_t launch_pack_all(PackJobs jobs, hipStream_t s) {
  if (jobs.n <= 0 || jobs.n > kPackJobsMax) return hipErrorInvalidValue;  // before touching j[] / first[]
  int blocks = 0;
  for (int j = 0; j < jobs.n; ++j) {
    const PackJob& J = jobs.j[j];
    if (J.ci % 32 || J.co % 32 || !J.w || !J.wf || (J.kind == 1 && !J.wd)) return hipErrorInvalidValue;
    jobs.first[j] = blocks;
    blocks += (J.ci / 32) * (J.co / 32);
  }
  jobs.first[jobs.n] = blocks;
  hipLaunchKernelGGL(k_pack_all, dim3(blocks), dim3(256), 0, s, jobs);
  return hipGetLastError();
}

__global__ void k_fill(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
hipError_t launch_fill(float* p, size_t n, float v, hipStream_t s) {
  hipLaunchKernelGGL(k_fill, dim3(grid_cap((long long)n, 256, 1024)), dim3(256), 0, s, p, n, v);
  return hipGetLastError();
}
// out[c] = sum_g st[g][c][0]  (first member of grouped (a, b) pairs)
__global__ void k_pair_sum(const double* __restrict__ st, int G, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0;
  for (int g = 0; g < G; ++g) s += st[((size_t)g * C + c) * 2];
  out[c] = (float)s;
}
hipError_t launch_pair_sum(const double* st, int g, int c, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_pair_sum, dim3(cdiv(c, 256)), dim3(256), 0, s, st, g, c, out);
  return hipGetLastError();
}

// 64 channels per block, the 4 waves each over a quarter of the groups (as
// group_sum): one thread per channel walking all G rows was a 16 us latency
// chain per convT bias gradient
__global__ __launch_bounds__(256) void k_colsum(const double* __restrict__ g, int G, int C,
                                                float* __restrict__ out) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6, c = blockIdx.x * 64 + lane;
  double s = 0;
  if (c < C) {
#pragma unroll 4
    for (int i = q; i < G; i += 4) s += g[(size_t)i * C + c];
  }
  red[q][lane] = s;
  __syncthreads();
  if (q == 0 && c < C) out[c] = (float)(red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}
hipError_t launch_colsum(const double* groups, int g, int c, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_colsum, dim3(cdiv(c, 64)), dim3(256), 0, s, groups, g, c, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// predict.py:85-92 mask and metrics.py:6-37 IoU counts.
// ---------------------------------------------------------------------------
__global__ void k_mask(const float* __restrict__ lg, uint8_t* __restrict__ m, int n, long long hw) {
  const long long total = n * hw;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long nn = i / hw, r = i - nn * hw;
    m[i] = (lg[(nn * 2 + 1) * hw + r] > lg[(nn * 2) * hw + r]) ? 255 : 0;
  }
}
hipError_t launch_mask(const float* logits, uint8_t* mask, int n, int h, int w, hipStream_t s) {
  hipLaunchKernelGGL(k_mask, dim3(grid_cap((long long)n * h * w, 256, 4096)), dim3(256), 0, s, logits, mask, n,
                     (long long)h * w);
  return hipGetLastError();
}
__global__ void k_iou(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, size_t n,
                      unsigned long long* out) {
  unsigned long long inter = 0, uni = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const bool p = a[i] > 0, g = b[i] > 0;
    inter += (p && g);
    uni += (p || g);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    inter += __shfl_xor(inter, o);
    uni += __shfl_xor(uni, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out, inter);
    atomicAdd(out + 1, uni);
  }
}
hipError_t launch_iou(const uint8_t* a, const uint8_t* b, size_t n, unsigned long long* out, hipStream_t s) {
  hipError_t me = hipMemsetAsync(out, 0, 2 * sizeof(unsigned long long), s);
  if (me != hipSuccess) return me;
  hipLaunchKernelGGL(k_iou, dim3(grid_cap((long long)n, 256, 1024)), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Generic per-channel helpers for the per-op BatchNorm API.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_channel_stats(const float* __restrict__ x, long long pixels, int C,
                                                       double* __restrict__ st) {
  const int C4 = C / 4, tid = threadIdx.x, cg = tid % C4, ppb = 256 / C4;
  float sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
  for (long long p = (long long)blockIdx.x * ppb + tid / C4; p < pixels; p += (long long)gridDim.x * ppb) {
    const float4 v = ld4(x + p * C + cg * 4);
    sa[0] += v.x; sa[1] += v.y; sa[2] += v.z; sa[3] += v.w;
    sb[0] += v.x * v.x; sb[1] += v.y * v.y; sb[2] += v.z * v.z; sb[3] += v.w * v.w;
  }
  reduce_pairs_to_global(sa, sb, C4, C, st + (size_t)(blockIdx.x % kStatGroups) * C * 2);
}
__global__ __launch_bounds__(256) void k_bn_bwd_stats(const float* __restrict__ dy, const float* __restrict__ x,
                                                      const float* mean, const float* invstd, long long pixels,
                                                      int C, double* __restrict__ st) {
  const int C4 = C / 4, tid = threadIdx.x, cg = tid % C4, ppb = 256 / C4;
  const float4 mu = ld4(mean + cg * 4), is = ld4(invstd + cg * 4);
  float sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
  for (long long p = (long long)blockIdx.x * ppb + tid / C4; p < pixels; p += (long long)gridDim.x * ppb) {
    const float4 d = ld4(dy + p * C + cg * 4), v = ld4(x + p * C + cg * 4);
    sa[0] += d.x; sa[1] += d.y; sa[2] += d.z; sa[3] += d.w;
    sb[0] += d.x * (v.x - mu.x) * is.x;
    sb[1] += d.y * (v.y - mu.y) * is.y;
    sb[2] += d.z * (v.z - mu.z) * is.z;
    sb[3] += d.w * (v.w - mu.w) * is.w;
  }
  reduce_pairs_to_global(sa, sb, C4, C, st + (size_t)(blockIdx.x % kStatGroups) * C * 2);
}
__global__ void k_affine_relu(const float* __restrict__ x, long long total4, int C, const float* sc, const float* sh,
                              int relu, float* __restrict__ y) {
  const int C4 = C / 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total4;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    float4 v = ld4(x + i * 4);
    const float4 a = ld4(sc + c), b = ld4(sh + c);
    v.x = fmaf(v.x, a.x, b.x); v.y = fmaf(v.y, a.y, b.y); v.z = fmaf(v.z, a.z, b.z); v.w = fmaf(v.w, a.w, b.w);
    if (relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
    st4(y + i * 4, v);
  }
}

hipError_t launch_channel_stats(const float* x, size_t pixels, int c, double* stats, hipStream_t s) {
  if (c < 4 || c % 4 || 256 % (c / 4)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_channel_stats, dim3(grid_cap((long long)pixels, 256 / (c / 4) * 4, 2048)), dim3(256), 0, s, x,
                     (long long)pixels, c, stats);
  return hipGetLastError();
}
hipError_t launch_bn_bwd_stats(const float* dy, const float* x, const float* mean, const float* invstd, size_t pixels,
                               int c, double* bstats, hipStream_t s) {
  if (c < 4 || c % 4 || 256 % (c / 4)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_bwd_stats, dim3(grid_cap((long long)pixels, 256 / (c / 4) * 4, 2048)), dim3(256), 0, s, dy,
                     x, mean, invstd, (long long)pixels, c, bstats);
  return hipGetLastError();
}
hipError_t launch_affine_relu(const float* x, size_t pixels, int c, const float* scale, const float* shift, int relu,
                              float* y, hipStream_t s) {
  if (c % 4) return hipErrorInvalidValue;
  const long long t4 = (long long)pixels * (c / 4);
  hipLaunchKernelGGL(k_affine_relu, dim3(grid_cap(t4, 256, 8192)), dim3(256), 0, s, x, t4, c, scale, shift, relu, y);
  return hipGetLastError();
}

}  // namespace unet
