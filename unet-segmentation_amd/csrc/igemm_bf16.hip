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
#include <cerrno>

#include "gemm_common.h"

namespace unet {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
// 16-B staging register (an array of the HIP uint4 struct is not promoted to
// registers; one of ext_vector_type is)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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

// 8 staged channels of an A operand -> 8 bf16 for LDS.  fp32 storage: r0, r1
// hold the values; bf16 storage: r0 holds the raw 16 bytes (copied as is, or
// widened, BN+ReLU-transformed and re-rounded when the source has a transform).
__device__ __forceinline__ uint4 stage8(float4 r0, float4 r1, bool h16, bool tf, float4 sc0, float4 sc1, float4 sh0,
                                       float4 sh1) {
  if (h16) {
    const uint4 u = __builtin_bit_cast(uint4, r0);
    if (!tf) return u;
    r0 = bf16x4_to_f4(make_uint2(u.x, u.y));
    r1 = bf16x4_to_f4(make_uint2(u.z, u.w));
  }
  if (tf) {
    r0 = affine_relu4(r0, sc0, sh0);
    r1 = affine_relu4(r1, sc1, sh1);
  }
  return bf16pack8(r0, r1);
}

// Split operands (UNET_PREC_BF16X3): v = hi + lo + O(2^-16 |v|) with
// hi = bf16(v), lo = bf16(v - hi); a product is taken as hi*hi' + hi*lo' + lo*hi'
// (three bf16 MFMAs, fp32 accumulation).  lo halves of the pair (a, b) whose
// packed hi halves are `hi`:
__device__ __forceinline__ unsigned bf16pack_lo(float a, float b, unsigned hi) {
  return bf16pack(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u));
}
__device__ __forceinline__ uint4 bf16pack8_lo(float4 a, float4 b, uint4 hi) {
  return make_uint4(bf16pack_lo(a.x, a.y, hi.x), bf16pack_lo(a.z, a.w, hi.y), bf16pack_lo(b.x, b.y, hi.z),
                    bf16pack_lo(b.z, b.w, hi.w));
}
// stage8 with the lo half: returns hi, writes lo (0 for raw bf16 data)
__device__ __forceinline__ uint4 stage8x(float4 r0, float4 r1, bool h16, bool tf, float4 sc0, float4 sc1, float4 sh0,
                                        float4 sh1, uint4& lo) {
  if (h16) {
    const uint4 u = __builtin_bit_cast(uint4, r0);
    lo = make_uint4(0u, 0u, 0u, 0u);
    if (!tf) return u;
    r0 = bf16x4_to_f4(make_uint2(u.x, u.y));
    r1 = bf16x4_to_f4(make_uint2(u.z, u.w));
  }
  if (tf) {
    r0 = affine_relu4(r0, sc0, sh0);
    r1 = affine_relu4(r1, sc1, sh1);
  }
  const uint4 hi = bf16pack8(r0, r1);
  lo = bf16pack8_lo(r0, r1, hi);
  return hi;
}

// One 16-k step of split operands: hi/lo planes of A (As, Al) and B (Bs, Bl)
template <int TM, int TN>
__device__ __forceinline__ void bf_mfma_step_x3(floatx16 (&acc)[TM][TN], const unsigned short* As,
                                                const unsigned short* Al, const unsigned short* Bs,
                                                const unsigned short* Bl, int arow, int brow, int koff) {
  bf16x8_t fa[TM], fal[TM], fb[TN], fbl[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    fa[i] = *reinterpret_cast<const bf16x8_t*>(As + (arow + 32 * i) * kBfLdr + koff);
    fal[i] = *reinterpret_cast<const bf16x8_t*>(Al + (arow + 32 * i) * kBfLdr + koff);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    fb[j] = *reinterpret_cast<const bf16x8_t*>(Bs + (brow + 32 * j) * kBfLdr + koff);
    fbl[j] = *reinterpret_cast<const bf16x8_t*>(Bl + (brow + 32 * j) * kBfLdr + koff);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fal[i], fb[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fbl[j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
}

constexpr int igemm_bf_minw(int BM, int BN, int WM, int WN, int planes = 1) {
  int blocks = 163840 / (2 * (BM + BN) * kBfLdr * 2 * planes);
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
// SPLIT: operands as hi/lo bf16 pairs (UNET_PREC_BF16X3), B's lo plane in args.bl;
// a stage then holds [A hi][B hi][A lo][B lo].  LDS is dynamic (igemm_bf_smem).
template <int BM, int BN, int SPLIT>
constexpr size_t igemm_bf_smem() {
  return (size_t)2 * (BM + BN) * kBfLdr * 2 * (SPLIT ? 2 : 1);
}

template <int BM, int BN, int WM, int WN, int SPLIT>
__global__ __launch_bounds__(WM * WN * 64, igemm_bf_minw(BM, BN, WM, WN, SPLIT ? 2 : 1)) void k_igemm_bf(
    const IgemmArgs args) {
  constexpr int NT = WM * WN * 64, BK = kBfBK, LDR = kBfLdr;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int RPP = NT / 4;  // staged rows per pass (4 lanes x 8 k per row)
  constexpr int AV = BM / RPP, BV = BN / RPP;
  constexpr int PLANE = (BM + BN) * LDR, STAGE = PLANE * (SPLIT ? 2 : 1);
  static_assert(TM >= 1 && TN >= 1 && AV >= 1 && BV >= 1 && BM % RPP == 0 && BN % RPP == 0, "tile");
  static_assert(WM * 3 * BN * 4 <= 2 * STAGE * 2, "epilogue reduction must fit the LDS ring");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];

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
  int bptr[BV];  // element offsets into args.bh / args.bl
#pragma unroll
  for (int q = 0; q < BV; ++q) bptr[q] = (n0 + row0 + RPP * q) * K + chunk * 8;

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

  float4 ra0[AV], ra1[AV];  // two 1-D arrays: a [N][2] array of vectors is not promoted to registers
  u32x4 rb[BV], rbl[SPLIT ? BV : 1];
  float4 sc0, sc1, sh0, sh1;
  bool tf = false, h16 = false;
  auto issue = [&](int k0) {
    const bool second = it_c >= g.c_split;
    const Src s = pick_src(g, second);
    const int c = (second ? it_c - g.c_split : it_c) + chunk * 8;
    const int toff = it_ty * s.W + it_tx;
    h16 = s.h16 != 0;
#pragma unroll
    for (int q = 0; q < AV; ++q) {
      const size_t e = (size_t)((second ? rb1[q] : rb0[q]) + toff) * s.C + c;
      if (h16) {  // stored bf16: 8 channels = 16 B, staged as is
        ra0[q] = __builtin_bit_cast(float4, *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(s.ptr) + e));
      } else {
        ra0[q] = ld4(s.ptr + e);
        ra1[q] = ld4(s.ptr + e + 4);
      }
    }
#pragma unroll
    for (int q = 0; q < BV; ++q) {
      rb[q] = *reinterpret_cast<const u32x4*>(args.bh + bptr[q] + k0);
      if constexpr (SPLIT) rbl[q] = *reinterpret_cast<const u32x4*>(args.bl + bptr[q] + k0);
    }
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
      unsigned short* d = As + (row0 + RPP * q) * LDR + chunk * 8;
      if constexpr (SPLIT) {
        uint4 lo;
        *reinterpret_cast<uint4*>(d) = stage8x(ra0[q], ra1[q], h16, tf, sc0, sc1, sh0, sh1, lo);
        *reinterpret_cast<uint4*>(d + PLANE) = lo;
      } else {
        *reinterpret_cast<uint4*>(d) = stage8(ra0[q], ra1[q], h16, tf, sc0, sc1, sh0, sh1);
      }
    }
#pragma unroll
    for (int q = 0; q < BV; ++q) {
      unsigned short* d = Bs + (row0 + RPP * q) * LDR + chunk * 8;
      *reinterpret_cast<u32x4*>(d) = rb[q];
      if constexpr (SPLIT) *reinterpret_cast<u32x4*>(d + PLANE) = rbl[q];
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
  auto compute = [&](int buf) {
    const unsigned short* As = lds + buf * STAGE;
    const unsigned short* Bs = As + BM * LDR;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (SPLIT)
        bf_mfma_step_x3<TM, TN>(acc, As, As + PLANE, Bs, Bs + PLANE, wm * TM * 32 + li, wn * TN * 32 + li,
                                16 * s + 8 * h);
      else
        bf_mfma_step<TM, TN>(acc, As, Bs, wm * TM * 32 + li, wn * TN * 32 + li, 16 * s + 8 * h);
    }
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
// k_conv3_bf: halo-tiled 3x3 stride-1 implicit GEMM (conv forward and conv
// input gradient), bf16 operands.  A workgroup owns a TH x TW spatial tile of
// one image's output grid and BN output columns.  Per 32-channel chunk it
// stages the (TH+2) x (TW+2) input halo ONCE (BN+ReLU applied, rounded to bf16)
// and the chunk's weights for all 9 taps; the 9 taps then read shifted pixel
// windows of the same LDS halo.  Against the pixel-row gather of k_igemm_bf
// (every A element fetched 9 times from L2) the A traffic drops to the halo
// overhead ((TH+2)(TW+2)/(TH TW), 1.33 at 8x32): the row-gather kernels are
// bound by that L2 traffic on the wide layers ("LDS-stage input
// tiles with a 2-px halo").
// LDS: halo [(TH+2)(TW+2)][40] bf16, weights [9][BN][40] bf16, BN scale/shift
// [2][Cg] fp32; one buffer, the next chunk in registers while this one computes.
// MFMA rows = output pixels in row-major tile order (32 per fragment), so a
// fragment lane reads LDS pixel (ry + ty)(TW+2) + rx + tx: one ds_read_b128.
// ---------------------------------------------------------------------------
// SPLIT (UNET_PREC_BF16X3): halo and weights as hi/lo planes, [A hi][B hi][A lo][B lo].
template <int TH, int TW, int BN, int SPLIT = 0>
constexpr size_t conv3_bf_smem(int cg) {
  return (size_t)((TH + 2) * (TW + 2) + 9 * BN) * kBfLdr * 2 * (SPLIT ? 2 : 1) + (size_t)2 * cg * 4;
}

// Phase timestamps of k_conv3_bf for a diagnosis build only (-DUNET_PHASE_PROBE,
// tools/phase_probe.sh): s_memrealtime (100 MHz) of workgroup (x, 0, 0) at its
// phase boundaries plus its hardware id, read back by unet_phase_probe_read.
#ifdef UNET_PHASE_PROBE
__device__ unsigned long long g_phase_probe[1 << 17];
#define UNET_PROBE(k)                                                                         \
  do {                                                                                        \
    if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && blockIdx.x < (1 << 14))      \
      g_phase_probe[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                 \
  } while (0)
#define UNET_PROBE_ID()                                                                       \
  do {                                                                                        \
    if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && blockIdx.x < (1 << 14))      \
      g_phase_probe[blockIdx.x * 8 + 7] = ((unsigned long long)__builtin_amdgcn_s_getreg(63508) << 32) | \
                                          (unsigned)__builtin_amdgcn_s_getreg(63492);          \
  } while (0)
#else
#define UNET_PROBE(k) do {} while (0)
#define UNET_PROBE_ID() do {} while (0)
#endif

// A16: every A source is stored bf16 (the usual case in a bf16 plan): no fp32
// staging registers, no per-source storage branch.
template <int TH, int TW, int BN, int WM, int WN, int MINW, int SPLIT, int A16>
__global__ __launch_bounds__(WM * WN * 64, MINW) void k_conv3_bf(const IgemmArgs args) {
  constexpr int NT = WM * WN * 64, BM = TH * TW, LDR = kBfLdr;
  constexpr int HW2 = TW + 2, PH = (TH + 2) * HW2;  // halo pixels
  constexpr int FM = BM / 32, TM = FM / WM, TN = BN / (WN * 32);
  constexpr int UA = PH * 4, UB = 9 * BN * 4;  // 16-B staging units (8 channels / 8 k each)
  constexpr int NA = (UA + NT - 1) / NT, NB = (UB + NT - 1) / NT;
  constexpr int A_ELEMS = PH * LDR, B_ELEMS = 9 * BN * LDR;
  static_assert(BM % 32 == 0 && FM % WM == 0 && TM >= 1 && TN >= 1, "tile");
  static_assert(WM * 3 * BN * 4 <= A_ELEMS * 2, "epilogue reduction must fit the halo buffer");
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  constexpr int PLANE = A_ELEMS + B_ELEMS;  // offset of the lo plane
  unsigned short* As = smem;
  unsigned short* Bs = smem + A_ELEMS;
  float* ssc = reinterpret_cast<float*>(smem + PLANE * (SPLIT ? 2 : 1));  // [2][Cg]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const Gather& g = args.a;
  const int Cg = g.Cg, K = args.K, Hg = g.Hg, Wg = g.Wg;
  const int tiles_x = (Wg + TW - 1) / TW, tiles_y = (Hg + TH - 1) / TH;
  int t = blockIdx.x;
  const int x0 = (t % tiles_x) * TW;
  t /= tiles_x;
  const int y0 = (t % tiles_y) * TH;
  const int n = t / tiles_y;
  const int n0 = blockIdx.y * BN;

  // consumer BN+ReLU parameters of the concatenated channel range
  const bool any_tf = g.s[0].scale != nullptr || (g.c_split < Cg && g.s[1].scale != nullptr);
  if (any_tf) {
    for (int c = tid; c < Cg; c += NT) {
      const bool sec = c >= g.c_split;
      const Src sr = pick_src(g, sec);
      const int cl = sec ? c - g.c_split : c;
      ssc[c] = sr.scale ? sr.scale[cl] : 1.f;
      ssc[Cg + c] = sr.scale ? sr.shift[cl] : 0.f;
    }
  }

  // staging units: A = (halo pixel, 8-channel piece), B = (tap, row, 8-k piece)
  int pi0[NA], pi1[NA];
  int bsrc[NB];  // element offsets into args.bh (32-bit: one VGPR, scalar base)
  // staging rows pair 4 apart in each block of 8 (stage_row8: conflict-free
  // ds_write_b128 groups at 80-B rows); the halo's last partial block as is
  auto arow = [&](int u) {
    const int q = u >> 2;
    return (q | 7) < PH ? stage_row8(q) : q;
  };
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    const int u = min(tid + k * NT, UA - 1);
    const int ph = arow(u);
    const int hy = ph / HW2, hx = ph - (ph / HW2) * HW2;
    const int yy = min(y0 + hy, Hg + 1), xx = min(x0 + hx, Wg + 1);  // overhang: any in-range pixel
    pi0[k] = (n * g.s[0].H + yy + g.s[0].oy) * g.s[0].W + xx + g.s[0].ox;
    pi1[k] = (n * g.s[1].H + yy + g.s[1].oy) * g.s[1].W + xx + g.s[1].ox;
  }
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int u = min(tid + k * NT, UB - 1);
    const int br = stage_row8(u >> 2);  // 9 x BN rows: whole blocks of 8
    const int r = br % BN, tap = br / BN;
    bsrc[k] = (n0 + r) * K + tap * Cg + (u & 3) * 8;
  }

  const int nk_all = Cg / 32;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = blockIdx.z * per;
    kc1 = min(nk_all, kc0 + per);
  }

  float4 ra0[NA], ra1[A16 ? 1 : NA];  // two 1-D arrays: a [N][2] array of vectors is not promoted to registers
  u32x4 rb[NB], rbl[SPLIT ? NB : 1];
  auto issue = [&](int kc) {
    const int c0 = kc * 32;
    const bool second = c0 >= g.c_split;
    const Src s = pick_src(g, second);
    const int cl = (second ? c0 - g.c_split : c0) + (tid & 3) * 8;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      if (tid + k * NT < UA) {
        const size_t e = (size_t)(second ? pi1[k] : pi0[k]) * s.C + cl;
        if (A16 || s.h16) {  // stored bf16: staged as is
          ra0[k] = __builtin_bit_cast(float4, *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(s.ptr) + e));
        } else if constexpr (!A16) {
          ra0[k] = ld4(s.ptr + e);
          ra1[k] = ld4(s.ptr + e + 4);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (tid + k * NT < UB) {
        rb[k] = *reinterpret_cast<const u32x4*>(args.bh + bsrc[k] + c0);
        if constexpr (SPLIT) rbl[k] = *reinterpret_cast<const u32x4*>(args.bl + bsrc[k] + c0);
      }
  };
  auto commit = [&](int kc) {
    const int c = kc * 32 + (tid & 3) * 8;
    const Src sc_src = pick_src(g, c >= g.c_split);
    const bool tf = sc_src.scale != nullptr, h16 = A16 || sc_src.h16 != 0;
    float4 sc0, sc1, sh0, sh1;
    if (tf) {
      sc0 = ld4(ssc + c);
      sc1 = ld4(ssc + c + 4);
      sh0 = ld4(ssc + Cg + c);
      sh1 = ld4(ssc + Cg + c + 4);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      if (u < UA) {
        unsigned short* d = As + arow(u) * LDR + (u & 3) * 8;
        const float4 r1 = ra1[A16 ? 0 : k];
        if constexpr (SPLIT) {
          uint4 lo;
          *reinterpret_cast<uint4*>(d) = stage8x(ra0[k], r1, h16, tf, sc0, sc1, sh0, sh1, lo);
          *reinterpret_cast<uint4*>(d + PLANE) = lo;
        } else {
          *reinterpret_cast<uint4*>(d) = stage8(ra0[k], r1, h16, tf, sc0, sc1, sh0, sh1);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = tid + k * NT;
      if (u < UB) {
        unsigned short* d = Bs + stage_row8(u >> 2) * LDR + (u & 3) * 8;
        *reinterpret_cast<u32x4*>(d) = rb[k];
        if constexpr (SPLIT) *reinterpret_cast<u32x4*>(d + PLANE) = rbl[k];
      }
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
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = (wm * TM + i) * 32 + li;
    int ty, tx;
    halo_pix<TH, TW>(p, ty, tx);
    abase[i] = ty * HW2 + tx;
  }
  // 18 (tap, 16-k) steps; the fragments of step t+1 are read while step t's
  // MFMAs issue (register double buffer), so each wave keeps one step of LDS
  // reads in flight instead of waiting on every read
  auto compute_pipe = [&] {
    bf16x8_t fa[2][TM], fb[2][TN];
    auto load = [&](int step, int buf) {
      const int tap = step >> 1, s = step & 1;
      const int off = (tap / 3) * HW2 + tap % 3;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[buf][i] = *reinterpret_cast<const bf16x8_t*>(As + (abase[i] + off) * LDR + 16 * s + 8 * h);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[buf][j] = *reinterpret_cast<const bf16x8_t*>(Bs + (tap * BN + wn * TN * 32 + j * 32 + li) * LDR + 16 * s + 8 * h);
    };
    load(0, 0);
#pragma unroll
    for (int step = 0; step < 18; ++step) {
      if (step + 1 < 18) load(step + 1, (step + 1) & 1);
      // keep the scheduler from sinking the next step's reads below this step's
      // MFMAs (it otherwise re-serialises read -> wait -> MFMA)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[step & 1][i], fb[step & 1][j], acc[i][j], 0, 0, 0);
    }
  };
  auto compute = [&] {
    if constexpr (!SPLIT) {
      compute_pipe();
      return;
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int off = (tap / 3) * HW2 + tap % 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8_t fa[TM], fb[TN], fal[SPLIT ? TM : 1], fbl[SPLIT ? TN : 1];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const unsigned short* p = As + (abase[i] + off) * LDR + 16 * s + 8 * h;
          fa[i] = *reinterpret_cast<const bf16x8_t*>(p);
          if constexpr (SPLIT) fal[i] = *reinterpret_cast<const bf16x8_t*>(p + PLANE);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const unsigned short* p = Bs + (tap * BN + wn * TN * 32 + j * 32 + li) * LDR + 16 * s + 8 * h;
          fb[j] = *reinterpret_cast<const bf16x8_t*>(p);
          if constexpr (SPLIT) fbl[j] = *reinterpret_cast<const bf16x8_t*>(p + PLANE);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if constexpr (SPLIT) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fal[i], fb[j], acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fbl[j], acc[i][j], 0, 0, 0);
            }
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
          }
      }
    }
  };

  UNET_PROBE_ID();
  UNET_PROBE(0);
  if (any_tf) __syncthreads();  // scale/shift table before the first commit
  if (kc0 < kc1) {
    issue(kc0);
    commit(kc0);
  }
  __syncthreads();
  UNET_PROBE(1);
  for (int kc = kc0; kc < kc1; ++kc) {
    const bool more = kc + 1 < kc1;
    if (more) issue(kc + 1);
    compute();
    __syncthreads();
    if (kc - kc0 < 2) UNET_PROBE(2 + 2 * (kc - kc0));
    if (more) {
      commit(kc + 1);
      __syncthreads();
      if (kc - kc0 < 1) UNET_PROBE(3);
    }
  }
  UNET_PROBE(5);
  if constexpr (TN == 2 && !SPLIT && NT / 64 * 4096 + WM * 3 * BN * 4 <= (A_ELEMS + B_ELEMS) * 2) {
    // LDS-staged epilogue: the waves' 4-KB staging tiles, then the statistics buffer
    igemm_finish<BM, BN, WM, WN, NT>(args, acc, 0, n0, wm, wn, tid,
                                     reinterpret_cast<float*>(smem + NT / 64 * 2048),
                                     HaloRows<TW, TH>{n, y0, x0, Hg, Wg}, smem);
  } else {
    igemm_finish<BM, BN, WM, WN, NT>(args, acc, 0, n0, wm, wn, tid, reinterpret_cast<float*>(smem),
                                     HaloRows<TW, TH>{n, y0, x0, Hg, Wg});
  }
  UNET_PROBE(6);
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
// AH / BH: storage of the A / B sources (0 fp32, 1 bf16, 2 per unit -- the
// concat gather of an up block's first conv mixes an fp32 skip and a bf16
// upsampled map); compile-time so that the staging loads carry no branches.
// SPLIT (UNET_PREC_BF16X3, fp32 sources only): hi/lo planes per stage, dynamic LDS.
template <int BM, int BN, int SPLIT>
constexpr size_t wgrad_bf_smem() {
  return (size_t)2 * (BM + BN) * kBfLdr * 2 * (SPLIT ? 2 : 1);
}

template <int BM, int BN, int WM, int WN, int AH, int BH, int SPLIT>
__global__ __launch_bounds__(WM * WN * 64, 2) void k_wgrad_bf(const WgradArgs args) {
  constexpr int NT = WM * WN * 64, BK = kBfBK, LDR = kBfLdr;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int UA = BM, UB = BN;  // units: 4 pixel groups x (rows / 4) quads
  constexpr int UPT = (UA + UB + NT - 1) / NT;
  constexpr int PLANE = (BM + BN) * LDR, STAGE = PLANE * (SPLIT ? 2 : 1);
  static_assert(TM >= 1 && TN >= 1 && BM % 64 == 0, "tile");
  static_assert(!SPLIT || (AH == 0 && BH == 0), "split operands come from fp32 storage");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int i0 = blockIdx.x * BM, j0 = blockIdx.y * BN;
  const int pbeg = blockIdx.z * args.pix_per_split;
  const int pend = min(args.P, pbeg + args.pix_per_split);
  const int nk = (pend - pbeg + BK - 1) / BK;
  if (nk <= 0) return;

  // per-unit constants (unit u: A if u < UA, else B; wave-uniform split since UA % 64 == 0)
  bool act[UPT], isb[UPT], tf[UPT], h16[UPT];
  int grp[UPT], lrow[UPT], C[UPT], H_[UPT], W[UPT], oy[UPT], ox[UPT], stride[UPT], Hg[UPT], Wg[UPT];
  const float* base[UPT];      // fp32 storage
  const uint16_t* baseh[UPT];  // bf16 storage
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
    baseh[k] = reinterpret_cast<const uint16_t*>(s->ptr) + c;
    C[k] = s->C;
    H_[k] = s->H;
    W[k] = s->W;
    oy[k] = s->oy + ty;
    ox[k] = s->ox + tx;
    stride[k] = gg.stride;
    Hg[k] = gg.Hg;
    Wg[k] = gg.Wg;
    tf[k] = s->scale != nullptr && act[k];
    h16[k] = isb[k] ? (BH == 2 ? s->h16 != 0 : BH == 1) : AH == 1;
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
  // one unit's 8 pixel loads; H = storage of its source (0 fp32, 1 bf16, 2 per
  // unit).  Unconditional: the iterator never leaves the grid, so the address
  // is valid past `pend` too; invalid pixels are zeroed in commit.  bf16 data
  // stays raw (bits in .x/.y) until commit, so no load is waited for here.
  auto load_unit = [&](auto hc, int k, int pb) {
    constexpr int H = decltype(hc)::value;
    valid[k] = 0;
    PixIt q = it[k];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = act[k] && pb + j < pend;
      const int pix = (q.n * H_[k] + q.y * stride[k] + oy[k]) * W[k] + q.x * stride[k] + ox[k];
      const size_t e = (size_t)pix * C[k];
      const bool half = H == 1 || (H == 2 && h16[k]);
      if (half) {
        const uint2 r = *reinterpret_cast<const uint2*>(baseh[k] + e);
        v[k][j] = make_float4(__uint_as_float(r.x), __uint_as_float(r.y), 0.f, 0.f);
      } else {
        v[k][j] = ld4(base[k] + e);
      }
      valid[k] |= ok ? (1u << j) : 0u;
      if (pb + j + 1 < pend) q.next(Hg[k], Wg[k]);
    }
    if (pb + BK < pend) it[k].advance(BK, Hg[k], Wg[k]);
  };
  auto issue = [&](int p0) {  // p0 = first pixel of the stage
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int pb = p0 + grp[k] * 8;
      if (isb[k])  // wave-uniform: a wave stages A units or B units
        load_unit(std::integral_constant<int, BH>{}, k, pb);
      else
        load_unit(std::integral_constant<int, AH>{}, k, pb);
    }
  };
  auto commit = [&](int buf) {
    unsigned short* S = lds + buf * STAGE;
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      if (!act[k]) continue;
      const bool wide = isb[k] ? (BH == 2 ? h16[k] : BH == 1) : AH == 1;
      if (wide) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = bf16x4_to_f4(make_uint2(__float_as_uint(v[k][j].x), __float_as_uint(v[k][j].y)));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 t = tf[k] ? affine_relu4(v[k][j], sc[k], sh[k]) : v[k][j];
        v[k][j] = (valid[k] >> j) & 1 ? t : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      unsigned short* dst = S + lrow[k] * LDR + grp[k] * 8;
      // row r of the unit's 4: component r of the 8 pixels
      auto put_row = [&](unsigned short* d, float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                         float a7) {
        const uint4 hi = make_uint4(bf16pack(a0, a1), bf16pack(a2, a3), bf16pack(a4, a5), bf16pack(a6, a7));
        *reinterpret_cast<uint4*>(d) = hi;
        if constexpr (SPLIT)
          *reinterpret_cast<uint4*>(d + PLANE) = make_uint4(bf16pack_lo(a0, a1, hi.x), bf16pack_lo(a2, a3, hi.y),
                                                            bf16pack_lo(a4, a5, hi.z), bf16pack_lo(a6, a7, hi.w));
      };
      put_row(dst + 0 * LDR, v[k][0].x, v[k][1].x, v[k][2].x, v[k][3].x, v[k][4].x, v[k][5].x, v[k][6].x, v[k][7].x);
      put_row(dst + 1 * LDR, v[k][0].y, v[k][1].y, v[k][2].y, v[k][3].y, v[k][4].y, v[k][5].y, v[k][6].y, v[k][7].y);
      put_row(dst + 2 * LDR, v[k][0].z, v[k][1].z, v[k][2].z, v[k][3].z, v[k][4].z, v[k][5].z, v[k][6].z, v[k][7].z);
      put_row(dst + 3 * LDR, v[k][0].w, v[k][1].w, v[k][2].w, v[k][3].w, v[k][4].w, v[k][5].w, v[k][6].w, v[k][7].w);
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
    for (int s = 0; s < 2; ++s) {
      if constexpr (SPLIT)
        bf_mfma_step_x3<TM, TN>(acc, As, As + PLANE, Bs, Bs + PLANE, wm * TM * 32 + li, wn * TN * 32 + li,
                                16 * s + 8 * h);
      else
        bf_mfma_step<TM, TN>(acc, As, Bs, wm * TM * 32 + li, wn * TN * 32 + li, 16 * s + 8 * h);
    }
    if (more) commit(cur ^ 1);
    __syncthreads();
  }
  // accumulate the tile into out (fp32 atomics; the output is small next to the
  // reduction), or (slab mode) store this split's partial for launch_slab_reduce
  float* const plane = args.slab ? args.slab + (size_t)blockIdx.z * args.Mo * args.No : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = j0 + wn * TN * 32 + j * 32 + li;
        if (plane) plane[(size_t)row * args.No + col] = acc[i][j][r];
        else atomicAdd(args.out + (size_t)row * args.No + col, acc[i][j][r]);
      }
}

// ---------------------------------------------------------------------------
// k_conv3p_bf: the halo-tiled 3x3 GEMM of k_conv3_bf as a persistent, software-
// pipelined loop.  A workgroup owns one 64-column block (blockIdx.y) and walks
// (tile, 32-channel chunk) stages of its tiles (tile = blockIdx.x + i*gridDim.x,
// chunks of its split-K slice blockIdx.z).  Two LDS stage buffers: while stage
// s computes from one, stage s+1 (loaded into registers during stage s-1) is
// committed into the other and stage s+2's loads are issued -- one barrier per
// stage, load latency hidden behind a whole stage of MFMAs, no pipeline drain
// at tile boundaries (the epilogue of a finished tile runs between stages).
// LDS rows are 64 B (32 bf16) without padding; the 16-B chunk c of row r sits
// at slot c ^ ((r >> 2) & 3), which keeps every ds_read_b128 group of 16 lanes
// (16 consecutive rows from any start) on distinct bank quads.
// 8 waves (WM = 8 along the tile's 32-pixel fragments, TN = 2), BN = 64.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int c3p_off(int row, int chunk) { return row * 32 + ((chunk ^ ((row >> 2) & 3)) << 3); }

template <int TH, int TW>
constexpr size_t conv3p_smem(int cg) {
  return (size_t)2 * ((TH + 2) * (TW + 2) + 9 * 64) * 64 + (size_t)2 * cg * 4 + (size_t)8 * 3 * 64 * 4;
}

template <int TH, int TW>
__global__ __launch_bounds__(512, 2) void k_conv3p_bf(const IgemmArgs args) {
  constexpr int NT = 512, BN = 64, WM = 8, WN = 1, BM = TH * TW;
  constexpr int HW2 = TW + 2, PH = (TH + 2) * HW2;
  constexpr int FM = BM / 32, TM = FM / WM, TN = BN / 32;
  constexpr int UA = PH * 4, UB = 9 * BN * 4;  // 16-B staging units
  constexpr int NA = (UA + NT - 1) / NT, NB = (UB + NT - 1) / NT;
  constexpr int A_EL = PH * 32, B_EL = 9 * BN * 32, ST_EL = A_EL + B_EL;  // bf16 elements
  static_assert(BM % 32 == 0 && FM % WM == 0 && TM >= 1, "tile");
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  float* ssc = reinterpret_cast<float*>(smem + 2 * ST_EL);  // [2][Cg]
  const Gather& g = args.a;
  const int Cg = g.Cg, K = args.K, Hg = g.Hg, Wg = g.Wg;
  float* red = ssc + 2 * Cg;  // epilogue reduction [WM*3][BN]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int n0 = blockIdx.y * BN;
  const int tiles_x = (Wg + TW - 1) / TW, tiles_y = (Hg + TH - 1) / TH;
  const int tiles = g.nimg * tiles_x * tiles_y;

  const bool any_tf = g.s[0].scale != nullptr || (g.c_split < Cg && g.s[1].scale != nullptr);
  if (any_tf) {
    for (int c = tid; c < Cg; c += NT) {
      const bool sec = c >= g.c_split;
      const Src sr = pick_src(g, sec);
      const int cl = sec ? c - g.c_split : c;
      ssc[c] = sr.scale ? sr.scale[cl] : 1.f;
      ssc[Cg + c] = sr.scale ? sr.shift[cl] : 0.f;
    }
  }

  // K slice of this workgroup (split-K over blockIdx.z) and its stage list
  const int nk_all = Cg / 32;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = blockIdx.z * per;
    kc1 = min(nk_all, kc0 + per);
  }
  const int nk = kc1 - kc0;
  const int my_tiles = (tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int S = nk > 0 ? my_tiles * nk : 0;

  // B staging units (tap, row, piece) are the same for every stage but the chunk
  int bsrc[NB];  // element offsets into args.bh (32-bit: one VGPR, scalar base)
  int boff[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int u = min(tid + k * NT, UB - 1);
    const int r = (u >> 2) % BN, tap = (u >> 2) / BN;
    bsrc[k] = (n0 + r) * K + tap * Cg + (u & 3) * 8;
    boff[k] = A_EL + c3p_off(u >> 2, u & 3);
  }

  float4 ra0[NA], ra1[NA];  // two 1-D arrays: a [N][2] array of vectors is not promoted to registers
  u32x4 rb[NB];
  auto tile_of = [&](int s, int& n, int& y0, int& x0) {
    int t = (int)blockIdx.x + (s / nk) * (int)gridDim.x;
    x0 = (t % tiles_x) * TW;
    t /= tiles_x;
    y0 = (t % tiles_y) * TH;
    n = t / tiles_y;
  };
  auto issue = [&](int s) {
    int n, y0, x0;
    tile_of(s, n, y0, x0);
    const int c0 = (kc0 + s % nk) * 32;
    const bool second = c0 >= g.c_split;
    const Src src = pick_src(g, second);
    const int cl = (second ? c0 - g.c_split : c0) + (tid & 3) * 8;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = min(tid + k * NT, UA - 1);
      const int ph = u >> 2;
      const int yy = min(y0 + ph / HW2, Hg + 1), xx = min(x0 + ph % HW2, Wg + 1);  // overhang: any in-range pixel
      const size_t e = (size_t)((n * src.H + yy + src.oy) * src.W + xx + src.ox) * src.C + cl;
      if (src.h16) {
        ra0[k] = __builtin_bit_cast(float4, *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(src.ptr) + e));
      } else {
        ra0[k] = ld4(src.ptr + e);
        ra1[k] = ld4(src.ptr + e + 4);
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) rb[k] = *reinterpret_cast<const u32x4*>(args.bh + bsrc[k] + c0);
  };
  auto commit = [&](int s, int buf) {
    unsigned short* st = smem + buf * ST_EL;
    const int c = (kc0 + s % nk) * 32 + (tid & 3) * 8;
    const Src src = pick_src(g, c >= g.c_split);
    const bool tf = src.scale != nullptr, h16 = src.h16 != 0;
    float4 sc0, sc1, sh0, sh1;
    if (tf) {
      sc0 = ld4(ssc + c);
      sc1 = ld4(ssc + c + 4);
      sh0 = ld4(ssc + Cg + c);
      sh1 = ld4(ssc + Cg + c + 4);
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      if (u < UA)
        *reinterpret_cast<uint4*>(st + c3p_off(u >> 2, u & 3)) = stage8(ra0[k], ra1[k], h16, tf, sc0, sc1, sh0, sh1);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (tid + k * NT < UB) *reinterpret_cast<u32x4*>(st + boff[k]) = rb[k];
  };

  floatx16 acc[TM][TN];
  auto zero_acc = [&] {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };
  zero_acc();

  const int h = lane >> 5, li = lane & 31;
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = (wm * TM + i) * 32 + li;
    abase[i] = (p / TW) * HW2 + p % TW;
  }
  auto compute = [&](int buf) {
    const unsigned short* st = smem + buf * ST_EL;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int off = (tap / 3) * HW2 + tap % 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int ch = 2 * s + h;
        bf16x8_t fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[i] = *reinterpret_cast<const bf16x8_t*>(st + c3p_off(abase[i] + off, ch));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const bf16x8_t*>(st + A_EL + c3p_off(tap * BN + wn * TN * 32 + j * 32 + li, ch));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  if (any_tf) __syncthreads();  // scale/shift table before the first commit
  if (S > 0) {
    issue(0);
    commit(0, 0);
    if (S > 1) issue(1);
  }
  __syncthreads();
  for (int s = 0; s < S; ++s) {
    if (s + 1 < S) {
      commit(s + 1, (s + 1) & 1);  // buffer of stage s-1: free since the last barrier
      if (s + 2 < S) issue(s + 2);
    }
    compute(s & 1);
    if (s % nk == nk - 1) {  // tile finished: epilogue (its own LDS reduction buffer)
      int n, y0, x0;
      tile_of(s, n, y0, x0);
      igemm_finish<BM, BN, WM, WN, NT>(args, acc, 0, n0, wm, wn, tid, red, HaloRows<TW>{n, y0, x0, Hg, Wg});
      zero_acc();
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// k_wgrad3_bf: halo-tiled weight gradient of a 3x3 stride-1 conv, all 9 taps in
// one workgroup.  dW[co][tap][ci] = sum_p dY[p][co] * X[p + tap][ci].  A
// workgroup owns 64 output channels (co) x 64 input channels (ci) x 9 taps and
// walks TH x TW output-pixel tiles (strided over blockIdx.z): per tile it stages
// the dY tile once and the (TH+2) x (TW+2) X halo once (consumer BN+ReLU,
// bf16), and every tap reads a shifted pixel window of that halo.  Against the
// (tap, channel)-column gather of k_wgrad_bf (X fetched once per tap, dY once
// per 64/128-column block) the operand traffic drops to ~1.4x the tensors.
// The MFMA k is the pixel; both LDS images are [pixel][64 channels] bf16
// (128-B rows, 16-B chunks swizzled by c ^ (((row >> 1) & 1) << 2)) and the
// operands come out transposed with ds_read_b64_tr_b16 (T10): a 16-lane group
// reads 4 pixels x 16 channels and lane i receives channel i of the 4 pixels,
// which is the 32x32x16 operand layout (row = channel, k = pixel).  Any 4
// consecutive rows are conflict-free under that swizzle, so the shifted tap
// windows need no realignment.
// Waves (8): co tile w & 1, ci tile (w >> 1) & 1, tap group w >> 2 (taps 0-4 or
// 5-8): one accumulator per tap of the group.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 lds_bf16x4_t;

__device__ __forceinline__ bf16x4_t tr_read(const unsigned char* p) {
  auto q = (__attribute__((address_space(3))) lds_bf16x4_t*)(const_cast<unsigned char*>(p));
  return __builtin_bit_cast(bf16x4_t, __builtin_amdgcn_ds_read_tr16_b64_v4bf16(q));
}
__device__ __forceinline__ int wg3_swz(int row, int chunk) { return chunk ^ (((row >> 1) & 1) << 2); }

// SPLIT (UNET_PREC_BF16X3): dY tile and X halo as hi/lo planes ([A][B] hi, then lo).
template <int TH, int TW, int SPLIT = 0>
constexpr size_t wgrad3_smem() {
  return (size_t)(TH * TW + (TH + 2) * (TW + 2)) * 128 * (SPLIT ? 2 : 1) + 2 * 64 * 4;
}

template <int TH, int TW, int D16, int SPLIT>
__global__ __launch_bounds__(512, 2) void k_wgrad3_bf(const WgradArgs args) {
  constexpr int NT = 512, BC = 64, ROWB = 128, NTAP = 5;
  constexpr int PT = TH * TW, HW2 = TW + 2, PH = (TH + 2) * HW2;
  constexpr int UA = PT * 8, UB = PH * 8;  // 16-B units: (pixel, 8-channel chunk)
  constexpr int NA = (UA + NT - 1) / NT, NB = (UB + NT - 1) / NT;
  static_assert(TW % 16 == 0 && UA % NT == 0, "a 16-pixel k-step stays inside one tile row");
  extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
  static_assert(!SPLIT || !D16, "split operands come from fp32 storage");
  constexpr int PLANE = (PT + PH) * ROWB;                        // bytes, offset of the lo plane
  unsigned char* Ad = wsm;                                       // dY tile [PT][64]
  unsigned char* Bx = wsm + PT * ROWB;                           // X halo [PH][64]
  float* ssc = reinterpret_cast<float*>(wsm + PLANE * (SPLIT ? 2 : 1));  // [2][64]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Gather& gb = args.gb;
  const Src& ds = args.ga.s[0];
  const int i0 = blockIdx.x * 64;  // co block
  const int cb = blockIdx.y * BC;  // ci block (gather channel index)
  const int Hg = gb.Hg, Wg = gb.Wg, Ci = gb.Cg;
  const bool second = cb >= gb.c_split;  // a 64-channel block never straddles the concat split
  const Src& xs = second ? gb.s[1] : gb.s[0];
  const int xc = second ? cb - gb.c_split : cb;
  const bool xtf = xs.scale != nullptr, x16 = xs.h16 != 0;
  if (xtf) {
    for (int c = tid; c < BC; c += NT) {
      ssc[c] = xs.scale[xc + c];
      ssc[BC + c] = xs.shift[xc + c];
    }
  }
  const int tiles_x = (Wg + TW - 1) / TW, tiles_y = (Hg + TH - 1) / TH;
  const int tiles = gb.nimg * tiles_x * tiles_y;

  // staging registers: dY (bf16 raw, or fp32 pairs), X (bf16 raw bits in [0], or an fp32 pair)
  uint4 rdh[NA];
  float4 rdf[D16 ? 1 : NA][2];
  float4 rx[NB][2];
  unsigned dvalid = 0;
  auto issue = [&](int t) {
    const int x0 = (t % tiles_x) * TW;
    const int r = t / tiles_x;
    const int y0 = (r % tiles_y) * TH, n = r / tiles_y;
    dvalid = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      const int p = u >> 3, ch = u & 7;
      const int y = y0 + p / TW, x = x0 + p % TW;
      dvalid |= (y < Hg && x < Wg) ? (1u << k) : 0u;
      const int yy = min(y, Hg - 1), xx = min(x, Wg - 1);
      const size_t e = (size_t)((n * ds.H + yy + ds.oy) * ds.W + xx + ds.ox) * ds.C + i0 + ch * 8;
      if constexpr (D16) {
        rdh[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(ds.ptr) + e);
      } else {
        rdf[k][0] = ld4(ds.ptr + e);
        rdf[k][1] = ld4(ds.ptr + e + 4);
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = min(tid + k * NT, UB - 1);
      const int hp = u >> 3, ch = u & 7;
      const int yy = min(y0 + hp / HW2, Hg + 1), xx = min(x0 + hp % HW2, Wg + 1);
      const size_t e = (size_t)((n * xs.H + yy + xs.oy) * xs.W + xx + xs.ox) * xs.C + xc + ch * 8;
      if (x16) {
        rx[k][0] = __builtin_bit_cast(float4, *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(xs.ptr) + e));
      } else {
        rx[k][0] = ld4(xs.ptr + e);
        rx[k][1] = ld4(xs.ptr + e + 4);
      }
    }
  };
  auto commit = [&] {
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      const int p = u >> 3, ch = u & 7;
      uint4 o, ol = make_uint4(0u, 0u, 0u, 0u);
      if constexpr (D16) o = rdh[k];
      else o = bf16pack8(rdf[k][0], rdf[k][1]);
      if constexpr (SPLIT) ol = bf16pack8_lo(rdf[k][0], rdf[k][1], o);
      if (!((dvalid >> k) & 1)) o = ol = make_uint4(0u, 0u, 0u, 0u);  // pixels past the grid add nothing
      unsigned char* d = Ad + p * ROWB + wg3_swz(p, ch) * 16;
      *reinterpret_cast<uint4*>(d) = o;
      if constexpr (SPLIT) *reinterpret_cast<uint4*>(d + PLANE) = ol;
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = tid + k * NT;
      if (u < UB) {
        const int hp = u >> 3, ch = u & 7;
        float4 sc0 = make_float4(1.f, 1.f, 1.f, 1.f), sc1 = sc0, sh0 = make_float4(0.f, 0.f, 0.f, 0.f), sh1 = sh0;
        if (xtf) {
          sc0 = ld4(ssc + ch * 8);
          sc1 = ld4(ssc + ch * 8 + 4);
          sh0 = ld4(ssc + BC + ch * 8);
          sh1 = ld4(ssc + BC + ch * 8 + 4);
        }
        unsigned char* d = Bx + hp * ROWB + wg3_swz(hp, ch) * 16;
        if constexpr (SPLIT) {
          uint4 lo;
          *reinterpret_cast<uint4*>(d) = stage8x(rx[k][0], rx[k][1], x16, xtf, sc0, sc1, sh0, sh1, lo);
          *reinterpret_cast<uint4*>(d + PLANE) = lo;
        } else {
          *reinterpret_cast<uint4*>(d) = stage8(rx[k][0], rx[k][1], x16, xtf, sc0, sc1, sh0, sh1);
        }
      }
    }
  };

  floatx16 acc[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // transposed-read lane roles: group g16 = lane >> 4 reads channel half (g16 & 1)
  // of k half (g16 >> 1); lane 4q + p of the group addresses pixel row q, channels 4p..4p+3
  const int g16 = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int hk = g16 >> 1;
  const int ct = wave & 1, it_ = (wave >> 1) & 1, tap0 = (wave >> 2) * NTAP;
  const int ntap = wave >> 2 ? 9 - NTAP : NTAP;  // wave-uniform
  const int colA = ct * 32 + (g16 & 1) * 16 + pp * 4, colB = it_ * 32 + (g16 & 1) * 16 + pp * 4;
  const int cA = colA >> 3, bA = (colA & 7) * 2, cB = colB >> 3, bB = (colB & 7) * 2;
  auto compute = [&] {
#pragma unroll 2
    for (int ks = 0; ks < PT / 16; ++ks) {
      const int prow = (ks * 16) / TW, px0 = (ks * 16) % TW;
      // 8 pixels (k) of one lane: rows r and r + 4 of the transposed read
      auto frag = [&](const unsigned char* base, int r, int cc, int bo) {
        const bf16x4_t a = tr_read(base + r * ROWB + wg3_swz(r, cc) * 16 + bo);
        const bf16x4_t b = tr_read(base + (r + 4) * ROWB + wg3_swz(r + 4, cc) * 16 + bo);
        return (bf16x8_t)__builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      const int pa = ks * 16 + 8 * hk + q;
      const bf16x8_t fa = frag(Ad, pa, cA, bA);
      bf16x8_t fal;
      if constexpr (SPLIT) fal = frag(Ad + PLANE, pa, cA, bA);
#pragma unroll
      for (int j = 0; j < NTAP; ++j) {
        if (j < ntap) {
          const int tap = tap0 + j;
          const int hb = (prow + tap / 3) * HW2 + px0 + tap % 3 + 8 * hk + q;
          const bf16x8_t fb = frag(Bx, hb, cB, bB);
          if constexpr (SPLIT) {
            const bf16x8_t fbl = frag(Bx + PLANE, hb, cB, bB);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fal, fb, acc[j], 0, 0, 0);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fbl, acc[j], 0, 0, 0);
          }
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[j], 0, 0, 0);
        }
      }
    }
  };

  if (xtf) __syncthreads();  // scale/shift table before the first commit
  int t = blockIdx.z;
  if (t < tiles) {
    issue(t);
    commit();
  }
  __syncthreads();
  for (; t < tiles; t += gridDim.z) {
    const bool more = t + (int)gridDim.z < tiles;
    if (more && !(args.abl & 4)) issue(t + gridDim.z);
    if (!(args.abl & 2)) compute();
    __syncthreads();
    if (more) {
      commit();
      __syncthreads();
    }
  }
  // accumulate into out[co][tap * Ci + ci] (fp32 atomics, one per element per workgroup)
  const int h = lane >> 5, li = lane & 31;
#pragma unroll
  for (int j = 0; j < NTAP; ++j) {
    if (j < ntap) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = (tap0 + j) * Ci + cb + it_ * 32 + li;
        if (args.abl & 1) args.out[(size_t)row * args.No + col] = acc[j][r];
        else atomicAdd(args.out + (size_t)row * args.No + col, acc[j][r]);
      }
    }
  }
}

// dynamic LDS above the 64 KiB default needs the attribute once per kernel
static hipError_t allow_smem(const void* fn, size_t bytes, bool& done) {
  if (done) return hipSuccess;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) done = true;
  return e;
}
constexpr size_t kLdsBytes = 160 * 1024;

template <int TH, int TW, int D16, int SPLIT>
static hipError_t go_wgrad3(const WgradArgs& a, hipStream_t s, int per_cu) {
  static bool attr = false;
  const size_t smem = wgrad3_smem<TH, TW, SPLIT>();
  hipError_t e = allow_smem(reinterpret_cast<const void*>(&k_wgrad3_bf<TH, TW, D16, SPLIT>), smem, attr);
  if (e != hipSuccess) return e;
  const int tiles = a.gb.nimg * ((a.gb.Hg + TH - 1) / TH) * ((a.gb.Wg + TW - 1) / TW);
  const int blocks = (a.Mo / 64) * (a.gb.Cg / 64);
  int splits = (per_cu * num_cus() + blocks - 1) / blocks;
  splits = splits < 1 ? 1 : (splits > tiles ? tiles : splits);
  dim3 grid(a.Mo / 64, a.gb.Cg / 64, splits);
  static const int abl = ablation_env("UNET_WG_ABL");
  WgradArgs b = a;
  b.abl = abl;
  hipLaunchKernelGGL((k_wgrad3_bf<TH, TW, D16, SPLIT>), grid, dim3(512), smem, s, b);
  return hipGetLastError();
}

// halo-tiled 3x3 weight gradient (tiles 20: 8x16, 21: 4x32 output pixels per step)
bool wgrad3_fits(const WgradArgs& a) {
  const Gather& g = a.gb;
  return a.bf16 && g.taps_h == 3 && g.taps_w == 3 && g.stride == 1 && a.No == 9 * g.Cg && a.Mo % 64 == 0 &&
         g.Cg % 64 == 0 && (g.c_split % 64 == 0 || g.c_split >= g.Cg) && a.ga.Cg == a.Mo && a.ga.taps_h == 1 &&
         a.ga.taps_w == 1 && g.Hg == a.ga.Hg && g.Wg == a.ga.Wg && g.nimg == a.ga.nimg &&
         !(a.split && a.ga.s[0].h16);
}

hipError_t go_wgrad3_bf16(const WgradArgs& a, hipStream_t s, int tile, int per_cu) {
  if (!wgrad3_fits(a)) return hipErrorInvalidValue;
  const bool d16 = a.ga.s[0].h16 != 0;
  if (a.split) {
    switch (tile) {
      case 20: return go_wgrad3<8, 16, 0, 1>(a, s, per_cu);
      case 21: return go_wgrad3<4, 32, 0, 1>(a, s, per_cu);
      default: return hipErrorInvalidValue;
    }
  }
  switch (tile * 2 + (d16 ? 1 : 0)) {
    case 40: return go_wgrad3<8, 16, 0, 0>(a, s, per_cu);
    case 41: return go_wgrad3<8, 16, 1, 0>(a, s, per_cu);
    case 42: return go_wgrad3<4, 32, 0, 0>(a, s, per_cu);
    case 43: return go_wgrad3<4, 32, 1, 0>(a, s, per_cu);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// k_wgrad3w_bf: k_wgrad3_bf with a wider workgroup tile and a two-stage ring
// (wgrad tiles 24: 128 co x 64 ci, 25: 64 co x 128 ci; bf16-stored dY and X).
// k_wgrad3_bf's waves hold 32 co x 32 ci x 5 taps: per 16-pixel k step 12
// transposed LDS reads feed 5 MFMAs, which saturates the LDS (~150 B/clk per CU
// at full MFMA rate against 128) -- and with one staging buffer the next
// tile's loads land before a ~1 us compute phase is over, so the barrier-bound
// loop exposes their latency (measured: without its MFMAs the kernel still
// takes ~70 % of its time).  Here a wave holds 64 co x 32 ci x 5 taps (160
// accumulator registers, one workgroup of 8 waves per CU): 14 transposed reads
// feed 10 MFMAs (~90 B/clk), and tile t+1 is loaded while tile t is multiplied
// and committed into the other buffer: one barrier per tile.
// LDS rows: [pixel][channels] bf16, 128 B (64 channels; 16-B chunk c stored at
// c ^ (((row >> 1) & 1) << 2), as k_wgrad3_bf) or 256 B (128 channels; the
// 64-B segment s of row r at s ^ (r & 3)): the 4 rows x 64 B a 32-lane half of
// a transposed read covers fall in 4 distinct 64-B bank groups either way.
// ---------------------------------------------------------------------------
template <int RB>  // row bytes 128 or 256
__device__ __forceinline__ int wgw_chunk(int row, int c) {
  if constexpr (RB == 128) return c ^ (((row >> 1) & 1) << 2);
  else return (((c >> 2) ^ (row & 3)) << 2) | (c & 3);
}

template <int BCO, int BCI>
constexpr size_t wgrad3w_smem() {
  return 2 * (size_t)(128 * BCO + 180 * BCI) * 2 + 2 * BCI * 4;  // 2 stages of (dY 8x16 px, X 10x18 halo) + scale/shift
}

template <int BCO, int BCI>
__global__ __launch_bounds__(512, 1) void k_wgrad3w_bf(const WgradArgs args, int gx, int gy) {
  constexpr int NT = 512, TH = 8, TW = 16, NTAP = 5;
  constexpr int PT = TH * TW, HW2 = TW + 2, PH = (TH + 2) * HW2;
  constexpr int RA = BCO * 2, RBX = BCI * 2;                // LDS row bytes
  constexpr int CA = BCO / 8, CB = BCI / 8;                 // 16-B chunks per row
  constexpr int UA = PT * CA, UB = PH * CB;                 // 16-B staging units per tile
  constexpr int NA = UA / NT, NB = (UB + NT - 1) / NT;
  constexpr int WCO = BCO / 64, WCI = BCI / 32;
  static_assert(UA % NT == 0 && WCO * WCI * 2 == 8, "8 waves: co groups x ci groups x 2 tap groups");
  constexpr int STAGE = PT * RA + PH * RBX;
  extern __shared__ __attribute__((aligned(16))) unsigned char wsm[];
  float* ssc = reinterpret_cast<float*>(wsm + 2 * STAGE);  // [2][BCI]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // workgroups of one pixel-tile set (same z) share the dY / X tiles: keep
  // them on one XCD (consecutive dispatch ids go round-robin over the 8 XCDs)
  long long bid = blockIdx.x;
  const long long G = gridDim.x;
  if ((G & 7) == 0) bid = (bid & 7) * (G >> 3) + (bid >> 3);
  const int bx = (int)(bid % gx), by = (int)((bid / gx) % gy), bz = (int)(bid / ((long long)gx * gy));
  const int splits = (int)(G / ((long long)gx * gy));
  const Gather& gb = args.gb;
  const Src& ds = args.ga.s[0];
  const int i0 = bx * BCO, cb = by * BCI;
  const int Hg = gb.Hg, Wg = gb.Wg, Ci = gb.Cg;
  const bool second = cb >= gb.c_split;  // a BCI-channel block never straddles the concat split
  const Src& xs = second ? gb.s[1] : gb.s[0];
  const int xc = second ? cb - gb.c_split : cb;
  const bool xtf = xs.scale != nullptr;
  if (xtf)
    for (int c = tid; c < BCI; c += NT) {
      ssc[c] = xs.scale[xc + c];
      ssc[BCI + c] = xs.shift[xc + c];
    }
  const int tiles_x = (Wg + TW - 1) / TW, tiles_y = (Hg + TH - 1) / TH;
  const int tiles = gb.nimg * tiles_x * tiles_y;

  uint4 ra[NA], rx[NB];
  unsigned dvalid = 0;
  auto issue = [&](int t) {
    const int x0 = (t % tiles_x) * TW;
    const int r = t / tiles_x;
    const int y0 = (r % tiles_y) * TH, n = r / tiles_y;
    dvalid = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      const int p = u / CA, ch = u % CA;
      const int y = y0 + p / TW, x = x0 + p % TW;
      dvalid |= (y < Hg && x < Wg) ? (1u << k) : 0u;
      const int yy = min(y, Hg - 1), xx = min(x, Wg - 1);
      const size_t e = (size_t)((n * ds.H + yy + ds.oy) * ds.W + xx + ds.ox) * ds.C + i0 + ch * 8;
      ra[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(ds.ptr) + e);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = min(tid + k * NT, UB - 1);
      const int hp = u / CB, ch = u % CB;
      const int yy = min(y0 + hp / HW2, Hg + 1), xx = min(x0 + hp % HW2, Wg + 1);
      const size_t e = (size_t)((n * xs.H + yy + xs.oy) * xs.W + xx + xs.ox) * xs.C + xc + ch * 8;
      rx[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(xs.ptr) + e);
    }
  };
  auto commit = [&](int b) {
    unsigned char* Ad = wsm + b * STAGE;
    unsigned char* Bx = Ad + PT * RA;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      const int p = u / CA, ch = u % CA;
      const uint4 o = ((dvalid >> k) & 1) ? ra[k] : make_uint4(0u, 0u, 0u, 0u);  // pixels past the grid add nothing
      *reinterpret_cast<uint4*>(Ad + p * RA + wgw_chunk<RA>(p, ch) * 16) = o;
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = tid + k * NT;
      if (u < UB) {
        const int hp = u / CB, ch = u % CB;
        uint4 o = rx[k];
        if (xtf) {
          const float4 r0 = affine_relu4(bf16x4_to_f4(make_uint2(o.x, o.y)), ld4(ssc + ch * 8), ld4(ssc + BCI + ch * 8));
          const float4 r1 =
              affine_relu4(bf16x4_to_f4(make_uint2(o.z, o.w)), ld4(ssc + ch * 8 + 4), ld4(ssc + BCI + ch * 8 + 4));
          o = bf16pack8(r0, r1);
        }
        *reinterpret_cast<uint4*>(Bx + hp * RBX + wgw_chunk<RBX>(hp, ch) * 16) = o;
      }
    }
  };

  floatx16 acc[2][NTAP];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int t = 0; t < NTAP; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][t][r] = 0.f;

  // transposed-read lane roles (k_wgrad3_bf): group g16 = lane >> 4 reads channel
  // half (g16 & 1) of k half (g16 >> 1); lane 4q + p of the group addresses
  // pixel row q, channels 4p .. 4p+3
  const int g16 = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int hk = g16 >> 1;
  const int wco = wave % WCO, wci = (wave / WCO) % WCI, tg = wave / (WCO * WCI);
  const int tap0 = tg * NTAP, ntap = tg ? 9 - NTAP : NTAP;  // wave-uniform
  const int colA = wco * 64 + (g16 & 1) * 16 + pp * 4, colB = wci * 32 + (g16 & 1) * 16 + pp * 4;
  auto compute = [&](int b) {
    const unsigned char* Ad = wsm + b * STAGE;
    const unsigned char* Bx = Ad + PT * RA;
#pragma unroll 2
    for (int ks = 0; ks < PT / 16; ++ks) {
      auto frag = [&](const unsigned char* base, int rb, int r, int col) {
        const int c = col >> 3, bo = (col & 7) * 2;
        const bf16x4_t lo = tr_read(base + r * rb + (rb == 128 ? wgw_chunk<128>(r, c) : wgw_chunk<256>(r, c)) * 16 + bo);
        const bf16x4_t hi =
            tr_read(base + (r + 4) * rb + (rb == 128 ? wgw_chunk<128>(r + 4, c) : wgw_chunk<256>(r + 4, c)) * 16 + bo);
        return (bf16x8_t)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      };
      const int pa = ks * 16 + 8 * hk + q;
      const bf16x8_t fa0 = frag(Ad, RA, pa, colA), fa1 = frag(Ad, RA, pa, colA + 32);
      const int prow = ks, px0 = 0;  // TW = 16: one tile row per k step
#pragma unroll
      for (int j = 0; j < NTAP; ++j) {
        if (j < ntap) {
          const int tap = tap0 + j;
          const int hb = (prow + tap / 3) * HW2 + px0 + tap % 3 + 8 * hk + q;
          const bf16x8_t fb = frag(Bx, RBX, hb, colB);
          acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0, fb, acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1, fb, acc[1][j], 0, 0, 0);
        }
      }
    }
  };

  if (xtf) __syncthreads();  // scale/shift table before the first commit
  int t = bz, b = 0;
  if (t < tiles) {
    issue(t);
    commit(0);
  }
  __syncthreads();
  for (; t < tiles; t += splits) {
    const bool more = t + splits < tiles;
    if (more && !(args.abl & 4)) issue(t + splits);
    if (!(args.abl & 2)) compute(b);
    if (more) commit(b ^ 1);  // its last reader (compute of the previous tile) passed the last barrier
    __syncthreads();
    b ^= 1;
  }
  // accumulate into out[co][tap * Ci + ci] (fp32 atomics, one per element per workgroup)
  const int h = lane >> 5, li = lane & 31;
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int j = 0; j < NTAP; ++j) {
      if (j < ntap) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = i0 + wco * 64 + 32 * f + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int col = (tap0 + j) * Ci + cb + wci * 32 + li;
          if (args.abl & 1) args.out[(size_t)row * args.No + col] = acc[f][j][r];
          else atomicAdd(args.out + (size_t)row * args.No + col, acc[f][j][r]);
        }
      }
    }
}

bool wgrad3w_fits(const WgradArgs& a, int tile) {
  const int bco = tile == 24 ? 128 : 64, bci = tile == 24 ? 64 : 128;
  const Gather& g = a.gb;
  const bool two = g.c_split < g.Cg;
  return (tile == 24 || tile == 25) && wgrad3_fits(a) && !a.split && a.ga.s[0].h16 && g.s[0].h16 &&
         (!two || g.s[1].h16) && a.Mo % bco == 0 && g.Cg % bci == 0 && (!two || g.c_split % bci == 0);
}

template <int BCO, int BCI>
static hipError_t go_wgrad3w(const WgradArgs& a, hipStream_t s, int per_cu) {
  static bool attr = false;
  const size_t smem = wgrad3w_smem<BCO, BCI>();
  hipError_t e = allow_smem(reinterpret_cast<const void*>(&k_wgrad3w_bf<BCO, BCI>), smem, attr);
  if (e != hipSuccess) return e;
  const int tiles = a.gb.nimg * ((a.gb.Hg + 7) / 8) * ((a.gb.Wg + 15) / 16);
  const int gx = a.Mo / BCO, gy = a.gb.Cg / BCI, blocks = gx * gy;
  int splits = (per_cu * num_cus() + blocks - 1) / blocks;
  splits = splits < 1 ? 1 : (splits > tiles ? tiles : splits);
  static const int abl = ablation_env("UNET_WG_ABL");
  WgradArgs b = a;
  b.abl = abl;
  hipLaunchKernelGGL((k_wgrad3w_bf<BCO, BCI>), dim3((unsigned)(blocks * splits)), dim3(512), smem, s, b, gx, gy);
  return hipGetLastError();
}

hipError_t go_wgrad3w_bf16(const WgradArgs& a, hipStream_t s, int tile, int per_cu) {
  if (!wgrad3w_fits(a, tile)) return hipErrorInvalidValue;
  return tile == 24 ? go_wgrad3w<128, 64>(a, s, per_cu) : go_wgrad3w<64, 128>(a, s, per_cu);
}

// ---------------------------------------------------------------------------
// fp32 -> bf16 (RNE) of the packed weight region, 4 elements per lane-step;
// with `lo` also the residual plane bf16(v - bf16(v)) of split operands
// ---------------------------------------------------------------------------
__global__ void k_f2bf(const float* __restrict__ in, uint16_t* __restrict__ out, uint16_t* __restrict__ lo,
                       size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = ld4(in + 4 * i);
    const uint2 h = make_uint2(bf16pack(v.x, v.y), bf16pack(v.z, v.w));
    *reinterpret_cast<uint2*>(out + 4 * i) = h;
    if (lo) *reinterpret_cast<uint2*>(lo + 4 * i) = make_uint2(bf16pack_lo(v.x, v.y, h.x), bf16pack_lo(v.z, v.w, h.y));
  }
}

hipError_t launch_f2bf(const float* in, uint16_t* out, size_t n, hipStream_t s, uint16_t* lo) {
  if (n % 4 || (reinterpret_cast<uintptr_t>(in) & 15) || (reinterpret_cast<uintptr_t>(out) & 7) ||
      (reinterpret_cast<uintptr_t>(lo) & 7))
    return hipErrorInvalidValue;
  const size_t n4 = n / 4;
  size_t grid = (n4 + 255) / 256;
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_f2bf, dim3((unsigned)grid), dim3(256), 0, s, in, out, lo, n4);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launchers (tile ids: igemm.hip tile_info 21-26, 31-36, 41-44; wgrad_tile
// 10-14, 20-21).  Split operands (a.bl / a.split) select the SPLIT kernels.
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, int SPLIT>
static hipError_t go_bf_t(const IgemmArgs& a, hipStream_t s) {
  static bool attr = false;
  const size_t smem = igemm_bf_smem<BM, BN, SPLIT>();
  hipError_t e = allow_smem(reinterpret_cast<const void*>(&k_igemm_bf<BM, BN, WM, WN, SPLIT>), smem, attr);
  if (e != hipSuccess) return e;
  dim3 grid((a.M + BM - 1) / BM, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  hipLaunchKernelGGL((k_igemm_bf<BM, BN, WM, WN, SPLIT>), grid, dim3(WM * WN * 64), smem, s, a);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN>
static hipError_t go_bf(const IgemmArgs& a, hipStream_t s) {
  if (a.bh == nullptr || a.N % BN != 0 || a.K % kBfBK != 0 || a.a.Cg % kBfBK != 0 || a.a.c_split % kBfBK != 0)
    return hipErrorInvalidValue;
  return a.bl ? go_bf_t<BM, BN, WM, WN, 1>(a, s) : go_bf_t<BM, BN, WM, WN, 0>(a, s);
}

template <int TH, int TW, int BN, int WM, int WN, int MINW, int SPLIT, int A16>
static hipError_t go_halo_t(const IgemmArgs& a, hipStream_t s) {
  static bool attr = false;
  hipError_t e = allow_smem(reinterpret_cast<const void*>(&k_conv3_bf<TH, TW, BN, WM, WN, MINW, SPLIT, A16>),
                            conv3_bf_smem<TH, TW, BN, SPLIT>(1024), attr);
  if (e != hipSuccess) return e;
  const long long tiles = (long long)a.a.nimg * ((a.a.Hg + TH - 1) / TH) * ((a.a.Wg + TW - 1) / TW);
  dim3 grid((unsigned)tiles, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  const size_t smem = conv3_bf_smem<TH, TW, BN, SPLIT>(a.a.Cg);
  hipLaunchKernelGGL((k_conv3_bf<TH, TW, BN, WM, WN, MINW, SPLIT, A16>), grid, dim3(WM * WN * 64), smem, s, a);
  return hipGetLastError();
}

// split variants run at <= 2 waves/SIMD (their LDS holds one workgroup per CU)
template <int TH, int TW, int BN, int WM, int WN, int MINW>
static hipError_t go_halo(const IgemmArgs& a, hipStream_t s) {
  if (a.bh == nullptr || a.N % BN != 0 || a.a.Cg % 32 != 0 || a.a.c_split % 32 != 0 || a.a.taps_h != 3 ||
      a.a.taps_w != 3 || a.a.stride != 1 || a.K != 9 * a.a.Cg || a.a.Cg > 1024)
    return hipErrorInvalidValue;
  if (a.bl) {
    // the lo fragments double the operand registers: at most 2 accumulator tiles per wave
    constexpr int TM = TH * TW / 32 / WM, TN = BN / (WN * 32);
    if constexpr (conv3_bf_smem<TH, TW, BN, 1>(1024) <= kLdsBytes && TM * TN <= 2)
      return go_halo_t<TH, TW, BN, WM, WN, (MINW < 2 ? MINW : 2), 1, 0>(a, s);
    return hipErrorInvalidValue;
  }
  const bool a16 = a.a.s[0].h16 && (a.a.c_split >= a.a.Cg || a.a.s[1].h16);
  return a16 ? go_halo_t<TH, TW, BN, WM, WN, MINW, 0, 1>(a, s) : go_halo_t<TH, TW, BN, WM, WN, MINW, 0, 0>(a, s);
}


template <int TH, int TW>
static hipError_t go_halo_p(const IgemmArgs& a, hipStream_t s, int waves_of_cus) {
  if (a.bh == nullptr || a.bl != nullptr || a.N % 64 != 0 || a.a.Cg % 32 != 0 || a.a.c_split % 32 != 0 ||
      a.a.taps_h != 3 || a.a.taps_w != 3 || a.a.stride != 1 || a.K != 9 * a.a.Cg || a.a.Cg > 1024)
    return hipErrorInvalidValue;
  static bool attr = false;
  hipError_t e = allow_smem(reinterpret_cast<const void*>(&k_conv3p_bf<TH, TW>), conv3p_smem<TH, TW>(1024), attr);
  if (e != hipSuccess) return e;
  const long long tiles = (long long)a.a.nimg * ((a.a.Hg + TH - 1) / TH) * ((a.a.Wg + TW - 1) / TW);
  const int ks = a.ksplit > 1 ? a.ksplit : 1;
  const long long cols = (long long)(a.N / 64) * ks;
  long long gx = ((long long)waves_of_cus * num_cus() + cols - 1) / cols;  // one resident workgroup per CU
  gx = gx < 1 ? 1 : (gx > tiles ? tiles : gx);
  dim3 grid((unsigned)gx, a.N / 64, ks);
  const size_t smem = conv3p_smem<TH, TW>(a.a.Cg);
  hipLaunchKernelGGL((k_conv3p_bf<TH, TW>), grid, dim3(512), smem, s, a);
  return hipGetLastError();
}

// halo tile shapes: id -> (TH, TW, BN); see go_igemm_bf16
bool halo_tile_shape(int tile, int& th, int& tw, int& bn) {
  switch (tile) {
    case 31: th = 8; tw = 32; bn = 64; return true;
    case 32: th = 8; tw = 32; bn = 64; return true;
    case 33: th = 16; tw = 16; bn = 64; return true;
    case 34: th = 4; tw = 32; bn = 128; return true;
    case 35: th = 8; tw = 16; bn = 64; return true;
    case 36: th = 8; tw = 32; bn = 128; return true;
    case 41: case 43: th = 8; tw = 32; bn = 64; return true;
    case 42: case 44: th = 16; tw = 16; bn = 64; return true;
    // fp32 k_conv3_f32 (igemm.hip)
    case 51: case 53: th = 8; tw = 32; bn = 64; return true;
    case 52: th = 16; tw = 16; bn = 64; return true;
    case 54: th = 8; tw = 16; bn = 64; return true;
    default: return false;
  }
}

// tiles with a split-operand kernel (the LDS of 34/36 and the persistent
// kernel's double buffer do not hold the lo planes; 32's 4 accumulator tiles
// per wave would spill)
bool bf16_tile_splits(int tile) { return (tile >= 21 && tile <= 26) || tile == 31 || tile == 33 || tile == 35; }

hipError_t go_igemm_bf16(const IgemmArgs& a, hipStream_t s, int tile) {
  if (a.bl && !bf16_tile_splits(tile)) return hipErrorInvalidValue;
  switch (tile) {
    case 31: return go_halo<8, 32, 64, 8, 1, 4>(a, s);
    case 32: return go_halo<8, 32, 64, 4, 1, 2>(a, s);
    case 33: return go_halo<16, 16, 64, 8, 1, 4>(a, s);
    case 34: return go_halo<4, 32, 128, 4, 2, 2>(a, s);
    case 35: return go_halo<8, 16, 64, 4, 1, 2>(a, s);
    case 36: return go_halo<8, 32, 128, 4, 2, 2>(a, s);
    // persistent pipelined (k_conv3p_bf): 1 or 2 rounds of workgroups per CU
    case 41: return go_halo_p<8, 32>(a, s, 1);
    case 42: return go_halo_p<16, 16>(a, s, 1);
    case 43: return go_halo_p<8, 32>(a, s, 2);
    case 44: return go_halo_p<16, 16>(a, s, 2);
    case 21: return go_bf<256, 128, 4, 2>(a, s);
    case 22: return go_bf<128, 128, 2, 2>(a, s);
    case 23: return go_bf<128, 64, 2, 2>(a, s);
    case 24: return go_bf<64, 128, 2, 2>(a, s);
    case 25: return go_bf<256, 64, 4, 1>(a, s);
    case 26: return go_bf<128, 256, 2, 4>(a, s);
    default: return hipErrorInvalidValue;
  }
}

template <int BM, int BN, int WM, int WN, int AH, int BH, int SPLIT>
static hipError_t go_wgrad_bf_t(const WgradArgs& a, hipStream_t s, dim3 grid) {
  static bool attr = false;
  const size_t smem = wgrad_bf_smem<BM, BN, SPLIT>();
  hipError_t e = allow_smem(reinterpret_cast<const void*>(&k_wgrad_bf<BM, BN, WM, WN, AH, BH, SPLIT>), smem, attr);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_wgrad_bf<BM, BN, WM, WN, AH, BH, SPLIT>), grid, dim3(WM * WN * 64), smem, s, a);
  return hipGetLastError();
}

template <int AH, int BH, int SPLIT>
static hipError_t wgrad_bf_tile(const WgradArgs& a, hipStream_t s, int tile, dim3 grid) {
  switch (tile) {
    case 10: return go_wgrad_bf_t<128, 128, 2, 2, AH, BH, SPLIT>(a, s, grid);
    case 11: return go_wgrad_bf_t<128, 192, 2, 2, AH, BH, SPLIT>(a, s, grid);
    case 12: return go_wgrad_bf_t<64, 128, 2, 2, AH, BH, SPLIT>(a, s, grid);
    case 13: return go_wgrad_bf_t<64, 64, 2, 2, AH, BH, SPLIT>(a, s, grid);
    case 14: return go_wgrad_bf_t<256, 128, 4, 2, AH, BH, SPLIT>(a, s, grid);
    default: return hipErrorInvalidValue;
  }
}

hipError_t go_wgrad_bf16(const WgradArgs& a, hipStream_t s, int tile, dim3 grid) {
  if (!a.bf16 || a.pix_per_split % kBfBK != 0) return hipErrorInvalidValue;
  const int ah = a.ga.s[0].h16;
  const bool two = a.gb.c_split < a.gb.Cg;
  const int bh = two && a.gb.s[0].h16 != a.gb.s[1].h16 ? 2 : a.gb.s[0].h16;
  if (a.split) return ah == 0 && bh == 0 ? wgrad_bf_tile<0, 0, 1>(a, s, tile, grid) : hipErrorInvalidValue;
  switch (ah * 3 + bh) {
    case 0: return wgrad_bf_tile<0, 0, 0>(a, s, tile, grid);
    case 1: return wgrad_bf_tile<0, 1, 0>(a, s, tile, grid);
    case 2: return wgrad_bf_tile<0, 2, 0>(a, s, tile, grid);
    case 3: return wgrad_bf_tile<1, 0, 0>(a, s, tile, grid);
    case 4: return wgrad_bf_tile<1, 1, 0>(a, s, tile, grid);
    default: return wgrad_bf_tile<1, 2, 0>(a, s, tile, grid);
  }
}

}  // namespace unet

#ifdef UNET_PHASE_PROBE
extern "C" int unet_phase_probe_read(void* host, size_t bytes) {
  if (bytes > sizeof(unet::g_phase_probe)) return -EINVAL;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(unet::g_phase_probe), bytes) == hipSuccess ? 0 : -EIO;
}
extern "C" int unet_phase_probe_clear() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(unet::g_phase_probe)) != hipSuccess) return -EIO;
  return hipMemset(p, 0, sizeof(unet::g_phase_probe)) == hipSuccess ? 0 : -EIO;
}
#endif
