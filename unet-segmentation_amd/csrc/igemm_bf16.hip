// bf16-operand implicit-GEMM kernels for gfx950 (MI355X): the same GEMMs as
// igemm.hip -- 3x3 valid conv forward and input gradient, ConvTranspose2d k2s2
// forward and input gradient, every weight gradient -- with both operands
// rounded to bf16 and fp32 accumulation on v_mfma_f32_32x32x16_bf16 (16x the
// f32 MFMA rate).  This is the "bf16-in / fp32-acc" arithmetic of SURVEY.md §8a
// A1 for configs C3/C5.  Activations stay fp32 in HBM: the raw conv outputs that
// feed the BatchNorm statistics, the BN/ReLU/pool/head/loss kernels and the
// optimizer are unchanged; operands are rounded (RNE) when they are staged into
// LDS, after the consumer-side BatchNorm+ReLU of the producer.  Weights arrive
// packed in bf16 (launch_f2bf over the plan's packed-weight region).
//
// LDS image of both kernels: per operand one [rows][32 k + 8 pad] bf16 tile
// (80-B rows).  The MFMA fragment of 16-k step s is one ds_read_b128 per lane
// (row l&31, k = 16s + 8(l>>5) .. +7), conflict-free over the ds_read_b128
// lane groups ({0-3,12-15,20-27}: rows*20 dwords land on 16 distinct bank
// quads).  Two stages double-buffer the K loop; the next stage's global loads
// are issued before the current stage's MFMAs and converted/stored after them.
#include "gemm_common.h"

namespace unet {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kBfBK = 32;   // k per LDS stage (two 16-k MFMA steps)
constexpr int kBfLdr = 40;  // bf16 elements per LDS row (32 + 8 pad)

// One 16-k MFMA step of a wave's TM x TN block of 32x32 tiles; A rows
// arow + 32i and B rows brow + 32j of the stage, k offset koff.
template <int TM, int TN>
__device__ __forceinline__ void bf_mfma_step(floatx16 (&acc)[TM][TN], const unsigned short* As,
                                             const unsigned short* Bs, int arow, int brow, int koff) {
  bf16x8_t fa[TM], fb[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const bf16x8_t*>(As + (arow + 32 * i) * kBfLdr + koff);
#pragma unroll
  for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const bf16x8_t*>(Bs + (brow + 32 * j) * kBfLdr + koff);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
}

constexpr int igemm_bf_minw(int BM, int BN, int WM, int WN) {
  int blocks = 163840 / (2 * (BM + BN) * kBfLdr * 2);
  if (blocks > 8) blocks = 8;
  const int w = blocks * WM * WN * 64 / 256;
  return w < 1 ? 1 : (w > 2 ? 2 : w);  // <= 2 waves/SIMD: up to 256 registers, no spills
}

// ---------------------------------------------------------------------------
// k_igemm_bf: C[m][n] = sum_k bf16(A[m][k]) * Bh[n][k];  A gathered from fp32
// NHWC sources (crop origin, two-source concat, stride-2 convT taps, consumer
// BN+ReLU), Bh packed bf16 [N][K].  Staging: each lane owns 8 consecutive k
// (32 B of fp32 A, 16 B of bf16 B) of one row per pass.
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, igemm_bf_minw(BM, BN, WM, WN)) void k_igemm_bf(const IgemmArgs args) {
  constexpr int NT = WM * WN * 64, BK = kBfBK, LDR = kBfLdr;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int RPP = NT / 4;  // staged rows per pass (4 lanes x 8 k per row)
  constexpr int AV = BM / RPP, BV = BN / RPP;
  constexpr int STAGE = (BM + BN) * LDR;
  static_assert(TM >= 1 && TN >= 1 && AV >= 1 && BV >= 1 && BM % RPP == 0 && BN % RPP == 0, "tile");
  static_assert(WM * 3 * BN * 4 <= 2 * STAGE * 2, "epilogue reduction must fit the LDS ring");
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const Gather& g = args.a;
  const int M = args.M, K = args.K;
  const int chunk = tid & 3, row0 = tid >> 2;

  // per staged A row: pixel base in each source grid (before the tap offset)
  int rb0[AV], rb1[AV];
  const int HWg = g.Hg * g.Wg;
#pragma unroll
  for (int q = 0; q < AV; ++q) {
    int m = m0 + row0 + RPP * q;
    m = m < M ? m : M - 1;
    const int n = m / HWg, r = m - n * HWg;
    int y = r / g.Wg, x = r - y * g.Wg;
    y *= g.stride;
    x *= g.stride;
    rb0[q] = (n * g.s[0].H + y + g.s[0].oy) * g.s[0].W + x + g.s[0].ox;
    rb1[q] = (n * g.s[1].H + y + g.s[1].oy) * g.s[1].W + x + g.s[1].ox;
  }
  const uint16_t* bptr[BV];
#pragma unroll
  for (int q = 0; q < BV; ++q) bptr[q] = args.bh + (size_t)(n0 + row0 + RPP * q) * K + chunk * 8;

  // K range of this workgroup (split-K slices chunks over blockIdx.z)
  const int nk_all = K / BK;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = blockIdx.z * per;
    kc1 = min(nk_all, kc0 + per);
  }
  // K iterator: chunk -> (tap_y, tap_x, c0); a chunk never straddles a tap or
  // the concat split (Cg and c_split are multiples of 32)
  int it_ty, it_tx, it_c;
  {
    const int cpt = g.Cg / BK;
    const int tap = kc0 / cpt;
    it_c = (kc0 - tap * cpt) * BK;
    it_ty = tap / g.taps_w;
    it_tx = tap - it_ty * g.taps_w;
  }

  float4 ra[AV][2];
  uint4 rb[BV];
  float4 sc0, sc1, sh0, sh1;
  bool tf = false;
  auto issue = [&](int k0) {
    const bool second = it_c >= g.c_split;
    const Src& s = second ? g.s[1] : g.s[0];
    const int c = (second ? it_c - g.c_split : it_c) + chunk * 8;
    const int toff = it_ty * s.W + it_tx;
#pragma unroll
    for (int q = 0; q < AV; ++q) {
      const float* p = s.ptr + (size_t)((second ? rb1[q] : rb0[q]) + toff) * s.C + c;
      ra[q][0] = ld4(p);
      ra[q][1] = ld4(p + 4);
    }
#pragma unroll
    for (int q = 0; q < BV; ++q) rb[q] = *reinterpret_cast<const uint4*>(bptr[q] + k0);
    tf = s.scale != nullptr;
    if (tf) {
      sc0 = ld4(s.scale + c);
      sc1 = ld4(s.scale + c + 4);
      sh0 = ld4(s.shift + c);
      sh1 = ld4(s.shift + c + 4);
    }
    it_c += BK;
    if (it_c == g.Cg) {
      it_c = 0;
      if (++it_tx == g.taps_w) { it_tx = 0; ++it_ty; }
    }
  };
  auto commit = [&](int buf) {
    unsigned short* As = lds + buf * STAGE;
    unsigned short* Bs = As + BM * LDR;
#pragma unroll
    for (int q = 0; q < AV; ++q) {
      float4 v0 = ra[q][0], v1 = ra[q][1];
      if (tf) {
        v0 = affine_relu4(v0, sc0, sh0);
        v1 = affine_relu4(v1, sc1, sh1);
      }
      *reinterpret_cast<uint4*>(As + (row0 + RPP * q) * LDR + chunk * 8) = bf16pack8(v0, v1);
    }
#pragma unroll
    for (int q = 0; q < BV; ++q) *reinterpret_cast<uint4*>(Bs + (row0 + RPP * q) * LDR + chunk * 8) = rb[q];
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int h = lane >> 5, li = lane & 31;
  auto compute = [&](int buf) {
    const unsigned short* As = lds + buf * STAGE;
    const unsigned short* Bs = As + BM * LDR;
#pragma unroll
    for (int s = 0; s < 2; ++s) bf_mfma_step<TM, TN>(acc, As, Bs, wm * TM * 32 + li, wn * TN * 32 + li, 16 * s + 8 * h);
  };

  if (kc0 < kc1) {
    issue(kc0 * BK);
    commit(0);
    __syncthreads();
  }
  for (int kc = kc0; kc < kc1; ++kc) {
    const int cur = (kc - kc0) & 1;
    const bool more = kc + 1 < kc1;
    if (more) issue((kc + 1) * BK);
    compute(cur);
    if (more) commit(cur ^ 1);
    __syncthreads();
  }
  // the ring is free (barrier above): reuse it as the epilogue's reduction buffer
  igemm_finish<BM, BN, WM, WN, NT>(args, acc, m0, n0, wm, wn, tid, reinterpret_cast<float*>(lds));
}

// ---------------------------------------------------------------------------
// k_wgrad_bf: C[i][j] = sum_p bf16(A_p[i]) * bf16(B_p[j]) over the pixels p of
// this workgroup's slice (blockIdx.z), fp32 atomics into out[Mo][No].
// A_p = channels of ga.s[0] (dY, or the BN+ReLU'd convT input), B_p = the
// (tap, channel) gather of gb.  The pixel index is the MFMA k: a staging unit
// (lane) loads one channel quad at 8 consecutive pixels (8 float4, coalesced
// across lanes of neighbouring quads) and transposes it in registers into 4
// LDS rows x 8 k (four ds_write_b128), so the LDS image is the k-contiguous
// [rows][k] layout of k_igemm_bf and the fragment reads are identical.
// Units: (channel quad, 8-pixel group) with the group fastest across lanes
// (keeps the four 16-B stores of 8 consecutive lanes on distinct bank quads).
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, 2) void k_wgrad_bf(const WgradArgs args) {
  constexpr int NT = WM * WN * 64, BK = kBfBK, LDR = kBfLdr;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int UA = BM, UB = BN;  // units: 4 pixel groups x (rows / 4) quads
  constexpr int UPT = (UA + UB + NT - 1) / NT;
  constexpr int STAGE = (BM + BN) * LDR;
  static_assert(TM >= 1 && TN >= 1 && BM % 64 == 0, "tile");
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int i0 = blockIdx.x * BM, j0 = blockIdx.y * BN;
  const int pbeg = blockIdx.z * args.pix_per_split;
  const int pend = min(args.P, pbeg + args.pix_per_split);
  const int nk = (pend - pbeg + BK - 1) / BK;
  if (nk <= 0) return;

  // per-unit constants (unit u: A if u < UA, else B; wave-uniform split since UA % 64 == 0)
  bool act[UPT], isb[UPT], tf[UPT];
  int grp[UPT], lrow[UPT], C[UPT], H[UPT], W[UPT], oy[UPT], ox[UPT], stride[UPT], Hg[UPT], Wg[UPT];
  const float* base[UPT];
  float4 sc[UPT], sh[UPT];
  PixIt it[UPT];
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int u = tid + k * NT;
    act[k] = u < UA + UB;
    isb[k] = u >= UA;
    const int uu = isb[k] ? u - UA : u;
    grp[k] = uu & 3;
    const int quad = uu >> 2;
    const Gather& gg = isb[k] ? args.gb : args.ga;
    int c, ty = 0, tx = 0;
    const Src* s;
    if (isb[k]) {
      const int bj = j0 + quad * 4;
      const int tap = bj / gg.Cg;
      const int c0 = bj - tap * gg.Cg;
      const bool second = c0 >= gg.c_split;
      s = second ? &gg.s[1] : &gg.s[0];
      c = second ? c0 - gg.c_split : c0;
      ty = tap / gg.taps_w;
      tx = tap - ty * gg.taps_w;
      lrow[k] = BM + quad * 4;
    } else {
      s = &gg.s[0];
      c = i0 + quad * 4;
      lrow[k] = quad * 4;
    }
    if (!act[k]) { s = &args.ga.s[0]; c = 0; }
    base[k] = s->ptr + c;
    C[k] = s->C;
    H[k] = s->H;
    W[k] = s->W;
    oy[k] = s->oy + ty;
    ox[k] = s->ox + tx;
    stride[k] = gg.stride;
    Hg[k] = gg.Hg;
    Wg[k] = gg.Wg;
    tf[k] = s->scale != nullptr && act[k];
    sc[k] = make_float4(1.f, 1.f, 1.f, 1.f);
    sh[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tf[k]) {
      sc[k] = ld4(s->scale + c);
      sh[k] = ld4(s->shift + c);
    }
    it[k].init(min(pbeg + grp[k] * 8, args.P - 1), Hg[k], Wg[k]);
  }

  float4 v[UPT][8];
  unsigned valid[UPT];
  auto issue = [&](int p0) {  // p0 = first pixel of the stage
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      valid[k] = 0;
      PixIt q = it[k];
      const int pb = p0 + grp[k] * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = act[k] && pb + j < pend;
        const int pix = (q.n * H[k] + q.y * stride[k] + oy[k]) * W[k] + q.x * stride[k] + ox[k];
        v[k][j] = ok ? ld4(base[k] + (size_t)pix * C[k]) : make_float4(0.f, 0.f, 0.f, 0.f);
        valid[k] |= ok ? (1u << j) : 0u;
        if (pb + j + 1 < pend) q.next(Hg[k], Wg[k]);
      }
      if (pb + BK < pend) it[k].advance(BK, Hg[k], Wg[k]);
    }
  };
  auto commit = [&](int buf) {
    unsigned short* S = lds + buf * STAGE;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      if (!act[k]) continue;
      if (tf[k]) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float4 t = affine_relu4(v[k][j], sc[k], sh[k]);
          v[k][j] = (valid[k] >> j) & 1 ? t : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      unsigned short* dst = S + lrow[k] * LDR + grp[k] * 8;
      *reinterpret_cast<uint4*>(dst + 0 * LDR) =
          make_uint4(bf16pack(v[k][0].x, v[k][1].x), bf16pack(v[k][2].x, v[k][3].x), bf16pack(v[k][4].x, v[k][5].x),
                     bf16pack(v[k][6].x, v[k][7].x));
      *reinterpret_cast<uint4*>(dst + 1 * LDR) =
          make_uint4(bf16pack(v[k][0].y, v[k][1].y), bf16pack(v[k][2].y, v[k][3].y), bf16pack(v[k][4].y, v[k][5].y),
                     bf16pack(v[k][6].y, v[k][7].y));
      *reinterpret_cast<uint4*>(dst + 2 * LDR) =
          make_uint4(bf16pack(v[k][0].z, v[k][1].z), bf16pack(v[k][2].z, v[k][3].z), bf16pack(v[k][4].z, v[k][5].z),
                     bf16pack(v[k][6].z, v[k][7].z));
      *reinterpret_cast<uint4*>(dst + 3 * LDR) =
          make_uint4(bf16pack(v[k][0].w, v[k][1].w), bf16pack(v[k][2].w, v[k][3].w), bf16pack(v[k][4].w, v[k][5].w),
                     bf16pack(v[k][6].w, v[k][7].w));
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int h = lane >> 5, li = lane & 31;
  issue(pbeg);
  commit(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    const bool more = kc + 1 < nk;
    if (more) issue(pbeg + (kc + 1) * BK);
    const unsigned short* As = lds + cur * STAGE;
    const unsigned short* Bs = As + BM * LDR;
#pragma unroll
    for (int s = 0; s < 2; ++s) bf_mfma_step<TM, TN>(acc, As, Bs, wm * TM * 32 + li, wn * TN * 32 + li, 16 * s + 8 * h);
    if (more) commit(cur ^ 1);
    __syncthreads();
  }
  // accumulate the tile into out (fp32 atomics; the output is small next to the reduction)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = j0 + wn * TN * 32 + j * 32 + li;
        atomicAdd(args.out + (size_t)row * args.No + col, acc[i][j][r]);
      }
}

// ---------------------------------------------------------------------------
// fp32 -> bf16 (RNE) of the packed weight region, 4 elements per lane-step
// ---------------------------------------------------------------------------
__global__ void k_f2bf(const float* __restrict__ in, uint16_t* __restrict__ out, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = ld4(in + 4 * i);
    *reinterpret_cast<uint2*>(out + 4 * i) = make_uint2(bf16pack(v.x, v.y), bf16pack(v.z, v.w));
  }
}

hipError_t launch_f2bf(const float* in, uint16_t* out, size_t n, hipStream_t s) {
  if (n % 4 || (reinterpret_cast<uintptr_t>(in) & 15) || (reinterpret_cast<uintptr_t>(out) & 7))
    return hipErrorInvalidValue;
  const size_t n4 = n / 4;
  size_t grid = (n4 + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_f2bf, dim3((unsigned)grid), dim3(256), 0, s, in, out, n4);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launchers (tile ids: igemm.hip tile_info 21-26, wgrad_tile 10-14)
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN>
static hipError_t go_bf(const IgemmArgs& a, hipStream_t s) {
  if (a.bh == nullptr || a.N % BN != 0 || a.K % kBfBK != 0 || a.a.Cg % kBfBK != 0 || a.a.c_split % kBfBK != 0)
    return hipErrorInvalidValue;
  dim3 grid((a.M + BM - 1) / BM, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  hipLaunchKernelGGL((k_igemm_bf<BM, BN, WM, WN>), grid, dim3(WM * WN * 64), 0, s, a);
  return hipGetLastError();
}

hipError_t go_igemm_bf16(const IgemmArgs& a, hipStream_t s, int tile) {
  switch (tile) {
    case 21: return go_bf<256, 128, 4, 2>(a, s);
    case 22: return go_bf<128, 128, 2, 2>(a, s);
    case 23: return go_bf<128, 64, 2, 2>(a, s);
    case 24: return go_bf<64, 128, 2, 2>(a, s);
    case 25: return go_bf<256, 64, 4, 1>(a, s);
    case 26: return go_bf<128, 256, 2, 4>(a, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t go_wgrad_bf16(const WgradArgs& a, hipStream_t s, int tile, dim3 grid) {
  if (!a.bf16 || a.pix_per_split % kBfBK != 0) return hipErrorInvalidValue;
  switch (tile) {
    case 10: hipLaunchKernelGGL((k_wgrad_bf<128, 128, 2, 2>), grid, dim3(256), 0, s, a); break;
    case 11: hipLaunchKernelGGL((k_wgrad_bf<128, 192, 2, 2>), grid, dim3(256), 0, s, a); break;
    case 12: hipLaunchKernelGGL((k_wgrad_bf<64, 128, 2, 2>), grid, dim3(256), 0, s, a); break;
    case 13: hipLaunchKernelGGL((k_wgrad_bf<64, 64, 2, 2>), grid, dim3(256), 0, s, a); break;
    case 14: hipLaunchKernelGGL((k_wgrad_bf<256, 128, 4, 2>), grid, dim3(512), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace unet
