// k_conv3_dma: bf16 3x3 stride-1 implicit GEMM (conv forward and conv input
// gradient) with a double-buffered LDS ring and the weights staged by LDS-DMA.
//
// The round-1 halo kernel (k_conv3_bf, igemm_bf16.hip) spent ~50 % of its wave
// cycles parked (PMC, profiles/r01_pmc_summary_bf16.txt): one LDS buffer, two
// barriers per 32-channel chunk, every staged byte -- the 9-tap weight slab
// (3-4x the halo's bytes) included -- moved global -> VGPR -> ds_write by the
// computing waves, and 16x16 tiles whose fragment rows straddle two tile rows
// (LDS bank conflicts).  Here:
//  * tiles are TH x 32 output pixels: an MFMA fragment (32 lanes) is exactly one
//    tile row, so the 16-B piece swizzle below is conflict-free for every tap
//    offset (the fragment rows are 32 consecutive LDS rows from any base);
//  * the weight slab of a chunk, [9 taps][BN][CH] bf16, goes global -> LDS by
//    global_load_lds_dwordx4 (no VGPRs, no VALU, no ds_write);
//  * the input halo [(TH+2) x 34][CH] bf16 is staged through registers when the
//    producer's BatchNorm+ReLU must be applied (forward: the consumer-side
//    transform of the raw conv output, once per halo element), or by LDS-DMA
//    too when the source needs no transform (ADMA: the padded dY of the input
//    gradient, pooled maps, transposed-conv outputs);
//  * two ring stages: chunk k+1 is loaded while chunk k computes, one barrier
//    per chunk.
// LDS row layout: row r = CH bf16 (CH/8 pieces of 16 B); piece q is stored at
// slot q ^ f(r), f(r) = (r >> 2) & 3 for CH = 32 and (r >> 3) & 1 for CH = 16.
// Over the two ds_read_b128 lane groups of a fragment read (rows base + {0-3,
// 12-15, 20-27} and base + {4-11, 16-19, 28-31}) the rows that share a bank
// residue differ in f, for any base: no conflicts.
// bf16 sources only (the bf16 plan stores every A source bf16); fp32-source
// and split-operand GEMMs stay on k_conv3_bf.
#include "gemm_common.h"

namespace unet {

typedef __bf16 bf16x8d_t __attribute__((ext_vector_type(8)));
typedef unsigned u32x4d __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) unsigned short lds_u16_t;

// One global_load_lds_dwordx4: 16 B per lane from `src` into LDS at the
// wave-uniform `dst` + lane * 16 (see k_igemm_g: inline asm so that hipcc does
// not drain it before unrelated ds_reads; the caller retires it by vmcnt).
__device__ __forceinline__ void dma16(const void* src, unsigned short* dst) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_u16_t*)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}

// s_waitcnt vmcnt(n), expcnt / lgkmcnt unconstrained (gfx9 encoding)
#define UNET_DMA_WAIT(n) __builtin_amdgcn_s_waitcnt(((n)&15) | (7 << 4) | (15 << 8) | ((((n) >> 4) & 3) << 14))

template <int CH>
__device__ __forceinline__ int piece_swz(int r) {
  if constexpr (CH == 32) return (r >> 2) & 3;
  else return (r >> 3) & 1;
}

// A region of a stage: whole 64-piece DMA instructions (the last one's extra
// lanes land in the padding, never in the B region)
template <int TH, int CH>
constexpr int conv3_dma_a_elems() {
  return (((TH + 2) * 34 * (CH / 8) + 63) / 64) * 512;
}
template <int TH, int BN, int CH>
constexpr int conv3_dma_stage_bytes() {
  return (conv3_dma_a_elems<TH, CH>() + 9 * BN * CH) * 2;
}
template <int TH, int BN, int CH>
constexpr size_t conv3_dma_smem(int cg) {
  return (size_t)2 * conv3_dma_stage_bytes<TH, BN, CH>() + (size_t)2 * cg * 4;
}

template <int TH, int BN, int CH, int WM, int WN, int MINW, int ADMA>
__global__ __launch_bounds__(WM * WN * 64, MINW) void k_conv3_dma(const IgemmArgs args) {
  constexpr int TW = 32, HW2 = TW + 2, PH = (TH + 2) * HW2, BM = TH * TW;
  constexpr int NT = WM * WN * 64, NW = WM * WN, PPR = CH / 8;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int PA = PH * PPR, PB = 9 * BN * PPR;         // 16-B pieces per stage
  constexpr int IA = (PA + 63) / 64, IB = PB / 64;        // DMA instructions per stage
  constexpr int IAW = (IA + NW - 1) / NW, IBW = (IB + NW - 1) / NW;  // per wave (duplicates pad)
  constexpr int NA = (PA + NT - 1) / NT;                  // register-staged pieces per thread
  constexpr int SA = conv3_dma_a_elems<TH, CH>(), STAGE = SA + 9 * BN * CH;  // bf16 elements
  static_assert(TM >= 1 && TN >= 1 && BM % (WM * 32) == 0 && BN % (WN * 32) == 0, "tile");
  static_assert(PB % 64 == 0 && (CH == 16 || CH == 32), "stage");
  static_assert(WM * 3 * BN * 4 <= 2 * STAGE * 2, "epilogue reduction must fit the ring");
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  float* ssc = reinterpret_cast<float*>(smem + 2 * STAGE);  // [2][Cg] (transform)

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

  const bool any_tf = !ADMA && (g.s[0].scale != nullptr || (g.c_split < Cg && g.s[1].scale != nullptr));
  if (any_tf) {
    for (int c = tid; c < Cg; c += NT) {
      const bool sec = c >= g.c_split;
      const Src sr = pick_src(g, sec);
      const int cl = sec ? c - g.c_split : c;
      ssc[c] = sr.scale ? sr.scale[cl] : 1.f;
      ssc[Cg + c] = sr.scale ? sr.shift[cl] : 0.f;
    }
  }

  // ---- producer geometry (chunk independent) ----
  // halo row r -> pixel index in each source grid (overhang clamped to any
  // in-range pixel: it only feeds outputs past the grid, masked at the end)
  auto halo_src = [&](int r, int& p0, int& p1) {
    const int hy = r / HW2, hx = r - (r / HW2) * HW2;
    const int yy = min(y0 + hy, Hg + 1), xx = min(x0 + hx, Wg + 1);
    p0 = (n * g.s[0].H + yy + g.s[0].oy) * g.s[0].W + xx + g.s[0].ox;
    p1 = (n * g.s[1].H + yy + g.s[1].oy) * g.s[1].W + xx + g.s[1].ox;
  };
  // B pieces: DMA instruction i = wave + NW * k (clamped: padding duplicates
  // re-load the last instruction's bytes into the same LDS words)
  int boff[IBW];
#pragma unroll
  for (int k = 0; k < IBW; ++k) {
    const int i = min(wave + NW * k, IB - 1);
    const int P = i * 64 + lane, row = P / PPR, slot = P % PPR;
    const int q = slot ^ piece_swz<CH>(row);
    const int tap = row / BN, co = row - tap * BN;
    boff[k] = (n0 + co) * K + tap * Cg + q * 8;
  }
  // A pieces: DMA (ADMA) or register staging
  int a0[ADMA ? IAW : NA], a1[ADMA ? IAW : NA], aq[ADMA ? IAW : NA];
  if constexpr (ADMA) {
#pragma unroll
    for (int k = 0; k < IAW; ++k) {
      const int i = min(wave + NW * k, IA - 1);
      const int P = min(i * 64 + lane, PA - 1), row = P / PPR, slot = P % PPR;
      aq[k] = (slot ^ piece_swz<CH>(row)) * 8;
      halo_src(row, a0[k], a1[k]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int P = min(tid + k * NT, PA - 1), row = P / PPR;
      aq[k] = (P % PPR) * 8;  // logical piece (channel offset); the LDS slot is swizzled at commit
      halo_src(row, a0[k], a1[k]);
    }
  }

  const int nk_all = Cg / CH;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = blockIdx.z * per;
    kc1 = min(nk_all, kc0 + per);
  }

  u32x4d ra[ADMA ? 1 : NA];
  // issue chunk kc into stage st: A (register loads or DMA) first, then B DMA
  auto issue = [&](int kc, int st) {
    const int c0 = kc * CH;
    const bool second = c0 >= g.c_split;
    const Src s = pick_src(g, second);
    const int cl = second ? c0 - g.c_split : c0;
    const uint16_t* ap = reinterpret_cast<const uint16_t*>(s.ptr);
    unsigned short* As = smem + st * STAGE;
    if constexpr (ADMA) {
#pragma unroll
      for (int k = 0; k < IAW; ++k) {
        const int i = min(wave + NW * k, IA - 1);
        dma16(ap + (size_t)(second ? a1[k] : a0[k]) * s.C + cl + aq[k], As + i * 512);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NA; ++k)
        if (tid + k * NT < PA)
          ra[k] = *reinterpret_cast<const u32x4d*>(ap + (size_t)(second ? a1[k] : a0[k]) * s.C + cl + aq[k]);
    }
    unsigned short* Bs = As + SA;
#pragma unroll
    for (int k = 0; k < IBW; ++k) {
      const int i = min(wave + NW * k, IB - 1);
      dma16(args.bh + boff[k] + c0, Bs + i * 512);
    }
  };
  // register-staged A: BN+ReLU of the producer (when it has one), round, store
  auto commit = [&](int kc, int st) {
    if constexpr (!ADMA) {
      unsigned short* As = smem + st * STAGE;
      const int c0 = kc * CH;
      const bool tf = pick_src(g, c0 >= g.c_split).scale != nullptr;
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        const int P = tid + k * NT;
        if (P < PA) {
          const int row = P / PPR, q = P % PPR;
          uint4 v = __builtin_bit_cast(uint4, ra[k]);
          if (tf) {
            const int c = c0 + q * 8;
            const float4 sc0 = ld4(ssc + c), sc1 = ld4(ssc + c + 4);
            const float4 sh0 = ld4(ssc + Cg + c), sh1 = ld4(ssc + Cg + c + 4);
            const float4 r0 = affine_relu4(bf16x4_to_f4(make_uint2(v.x, v.y)), sc0, sh0);
            const float4 r1 = affine_relu4(bf16x4_to_f4(make_uint2(v.z, v.w)), sc1, sh1);
            v = bf16pack8(r0, r1);
          }
          *reinterpret_cast<uint4*>(As + row * CH + ((q ^ piece_swz<CH>(row)) * 8)) = v;
        }
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
  // fragment i of this wave = tile row (wm * TM + i): 32 consecutive halo rows
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) abase[i] = (wm * TM + i) * HW2 + li;
  int bbase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bbase[j] = wn * TN * 32 + j * 32 + li;

  // 9 x CH/16 (tap, 16-k) steps, fragments of step t+1 read while step t's
  // MFMAs issue (register double buffer)
  constexpr int KS = CH / 16, NSTEP = 9 * KS;
  auto compute = [&](int st) {
    const unsigned short* As = smem + st * STAGE;
    const unsigned short* Bs = As + SA;
    bf16x8d_t fa[2][TM], fb[2][TN];
    auto load = [&](int step, int buf) {
      const int tap = step / KS, s = step % KS;
      const int off = (tap / 3) * HW2 + tap % 3;
      const int q = 2 * s + h;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = abase[i] + off;
        fa[buf][i] = *reinterpret_cast<const bf16x8d_t*>(As + r * CH + ((q ^ piece_swz<CH>(r)) * 8));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = tap * BN + bbase[j];
        fb[buf][j] = *reinterpret_cast<const bf16x8d_t*>(Bs + r * CH + ((q ^ piece_swz<CH>(r)) * 8));
      }
    };
    load(0, 0);
#pragma unroll
    for (int step = 0; step < NSTEP; ++step) {
      if (step + 1 < NSTEP) load(step + 1, (step + 1) & 1);
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

  if (any_tf) __syncthreads();  // scale/shift table before the first commit
  if (kc0 < kc1) {
    issue(kc0, 0);
    if constexpr (!ADMA) {
      UNET_DMA_WAIT(IBW);  // this wave's A loads (issued before its B pieces) landed
      commit(kc0, 0);
    }
    UNET_DMA_WAIT(0);
  }
  __syncthreads();
  int st = 0;
  for (int kc = kc0; kc < kc1; ++kc) {
    const bool more = kc + 1 < kc1;
    if (more) issue(kc + 1, st ^ 1);
    compute(st);
    if (more) {
      if constexpr (!ADMA) {
        UNET_DMA_WAIT(IBW);
        commit(kc + 1, st ^ 1);
      }
      UNET_DMA_WAIT(0);
      __syncthreads();  // stage st^1 complete for every wave; stage st free
    }
    st ^= 1;
  }
  __syncthreads();  // the ring is reused as the epilogue's reduction buffer
  igemm_finish<BM, BN, WM, WN, NT>(args, acc, 0, n0, wm, wn, tid, reinterpret_cast<float*>(smem),
                                   HaloRows<TW, TH>{n, y0, x0, Hg, Wg});
}

template <int TH, int BN, int CH, int WM, int WN, int MINW, int ADMA>
static hipError_t go_conv3_dma_t(const IgemmArgs& a, hipStream_t s) {
  static bool attr = false;
  const size_t full = conv3_dma_smem<TH, BN, CH>(ADMA ? 0 : 1024);
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3_dma<TH, BN, CH, WM, WN, MINW, ADMA>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)full);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const long long tiles = (long long)a.a.nimg * ((a.a.Hg + TH - 1) / TH) * ((a.a.Wg + 31) / 32);
  dim3 grid((unsigned)tiles, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  const size_t smem = conv3_dma_smem<TH, BN, CH>(ADMA ? 0 : a.a.Cg);
  hipLaunchKernelGGL((k_conv3_dma<TH, BN, CH, WM, WN, MINW, ADMA>), grid, dim3(WM * WN * 64), smem, s, a);
  return hipGetLastError();
}

// A needs no transform (and is bf16): DMA staging; else register staging
template <int TH, int BN, int CH, int WM, int WN, int MINW>
static hipError_t go_conv3_dma(const IgemmArgs& a, hipStream_t s) {
  const Gather& g = a.a;
  const bool two = g.c_split < g.Cg;
  if (a.bh == nullptr || a.bl != nullptr || a.N % BN != 0 || g.Cg % CH != 0 || g.c_split % CH != 0 ||
      g.taps_h != 3 || g.taps_w != 3 || g.stride != 1 || a.K != 9 * g.Cg || g.Cg > 1024 || !g.s[0].h16 ||
      (two && !g.s[1].h16))
    return hipErrorInvalidValue;
  const bool tf = g.s[0].scale != nullptr || (two && g.s[1].scale != nullptr);
  return tf ? go_conv3_dma_t<TH, BN, CH, WM, WN, MINW, 0>(a, s) : go_conv3_dma_t<TH, BN, CH, WM, WN, MINW, 1>(a, s);
}

// tile ids 63, 65-68 (igemm.hip tile_info): (TH, BN, CH, waves).  Measured and
// dropped (profiles/r02_conv_dma_variants.txt): one-wave-per-SIMD shapes
// (8x32/128 and 8x32/64 with 32-channel chunks at 4 waves) and 16x32/128 at 8
// waves (spills in the register-staged form) ran 1.3-3x slower than k_conv3_bf.
bool conv3_dma_tile_shape(int tile, int& th, int& bn, int& ch) {
  switch (tile) {
    case 63: th = 8; bn = 64; ch = 16; return true;
    case 65: th = 16; bn = 64; ch = 16; return true;
    case 66: th = 16; bn = 64; ch = 32; return true;
    case 67: th = 8; bn = 64; ch = 16; return true;
    case 68: th = 8; bn = 128; ch = 16; return true;
    default: return false;
  }
}

hipError_t go_conv3_dma_tile(const IgemmArgs& a, hipStream_t s, int tile) {
  switch (tile) {
    case 63: return go_conv3_dma<8, 64, 16, 4, 1, 2>(a, s);   // 4 waves, TM 2 x TN 2; 59 KB, 2 WG/CU
    case 65: return go_conv3_dma<16, 64, 16, 4, 2, 2>(a, s);  // 8 waves, TM 4 x TN 1; 84 KB
    case 66: return go_conv3_dma<16, 64, 32, 4, 2, 2>(a, s);  // 8 waves, TM 4 x TN 1; 160 KB
    case 67: return go_conv3_dma<8, 64, 16, 8, 1, 4>(a, s);   // 8 waves, TM 1 x TN 2; 59 KB: 2 WG/CU, 4 waves/SIMD
    case 68: return go_conv3_dma<8, 128, 16, 4, 2, 2>(a, s);  // 8 waves, TM 2 x TN 2 (64x64 per wave); 96 KB
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
