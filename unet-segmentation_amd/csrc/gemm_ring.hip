// k_gemm_ring: bf16 implicit GEMM of the ConvTranspose2d(k=2, s=2) layers
// (models/unet_model.py:45) with every operand byte staged by LDS-DMA through
// a ring of K stages -- the convT forward (1x1 gather of the previous conv's
// output, pixel-shuffle epilogue) and the convT input gradient (2x2 stride-2
// gather of the upsampled map's gradient, ReLU-mask + BatchNorm-backward
// epilogue of the layer before).
//
// The register-staged row-gather tiles (k_igemm_bf) ran these at 0.1 of the
// bf16 MFMA peak (9.9 % MFMA busy, 0.6-0.8 ms per bf16 step):
// 32-k stages, 4 MFMAs per wave between barriers, every byte through VGPRs.
// Here a workgroup owns BM pixel rows x BN columns and walks K in BK-k stages
// (BK = 32 or 64):
//  * stage s of A (BM rows x 2 BK bytes) and of B (BN rows) go global -> LDS
//    by global_load_lds_dwordx4 from an SGPR base (advanced per stage on the
//    scalar unit) plus per-lane 32-bit offsets computed once, NSTG-1 stages
//    ahead, retired by counted vmcnt waits; one raw s_barrier per stage;
//  * the gather is folded into the SGPR base: a stage lies inside one tap
//    (channel counts are multiples of 64), and a tap moves every row's source
//    pixel by the same (ty * W + tx) * C elements;
//  * 16-B pieces are XOR-swizzled by the row's position in its 256-B bank row
//    on the DMA source and on the fragment read: every ds_read_b128 lane group
//    hits 16 distinct bank quads;
//  * XTF: a source with a consumer transform (relu(bn(y)) of the producer) is
//    DMA'd raw and rewritten in place once per stage, one stage ahead of its
//    MFMAs;
//  * each wave computes (TM x 32) x (TN x 32) with v_mfma_f32_32x32x16_bf16;
//    the stage's DMAs are issued one per k-step between the MFMAs;
//  * the epilogue is the shared one (igemm_finish: pixel shuffle + bias, ReLU
//    mask + BN-backward statistics, split-K partials).
#include <algorithm>

#include "gemm_common.h"
#include "ring_common.h"

namespace unet {

namespace {
typedef __bf16 bf16x8g_t __attribute__((ext_vector_type(8)));
}  // namespace

// LDS-staged pixel-shuffle epilogue of the convT forward (bf16 destination,
// 64 columns per wave inside one sub-pixel ab): a 32-row fragment x 64 columns
// passes through the wave's 4 KB of LDS ([row][64] bf16, 128-B rows) and leaves
// by four 16-B stores per lane -- each row's 64 channels are 128 contiguous
// bytes at output pixel (2y + a, 2x + b) -- instead of 32 2-B stores per lane
// and fragment (epi_shuffle; round 5's phase probe put that per-element form at
// a quarter of a small-K workgroup's time, profiles/r05_conv3_bf_phases.txt).
// Same values (bias, optional ReLU, RNE to bf16) as epi_shuffle.  Returns false
// (nothing stored) when the launch's epilogue is not of that form (a split-K
// slice stores its raw partial through igemm_finish instead).
template <int TM, int TN, int WM, int WN>
__device__ __forceinline__ bool epi_shuffle_staged(const IgemmArgs& args, const floatx16 (&acc)[TM][TN], int m0, int n0,
                                                   int wm, int wn, int tid, unsigned short* stage) {
  static_assert(TN == 2, "64 columns per wave");
  const Epilogue& e = args.e;
  const Gather& g = args.a;
  const Dst& d = e.d[0];
  const int Co = e.shuffle_co, N = args.N;
  if (!(args.ksplit <= 1 && Co > 0 && Co % 64 == 0 && e.n_split >= N && !e.stats && !e.yref && !e.colsum1 && d.h16 &&
        d.C == Co &&
        d.oy == 0 && d.ox == 0 && d.H == 2 * g.Hg && d.W == 2 * g.Wg &&
        (reinterpret_cast<size_t>(d.ptr) & 15) == 0 && (size_t)args.M * 4 * (size_t)Co * 2 < (1ull << 32)))
    return false;
  const int lane = tid & 63, h = lane >> 5, li = lane & 31;
  unsigned short* wl = stage + (tid >> 6) * (32 * 64);
  const int col0 = n0 + wn * 64;
  const int ab = col0 / Co, co0 = col0 - ab * Co;  // one sub-pixel per 64-column block (Co % 64 == 0)
  const unsigned W2 = (unsigned)d.W, H2 = (unsigned)d.H;
  const int Hg = g.Hg, Wg = g.Wg, M = args.M;
  float bias[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bias[j] = e.bias ? e.bias[co0 + j * 32 + li] : 0.f;
  uint16_t* const dst = reinterpret_cast<uint16_t*>(d.ptr);
  const int rq = lane >> 3, cq = (lane & 7) * 8;  // this lane's rows rq + 8q and 8 channels of the readback
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = m0 + (wm * TM + i) * 32;
    const int lim = M - mb;
    if (lim <= 0) continue;  // wave-uniform
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
        float v = acc[i][j][r] + bias[j];
        if (e.relu) v = fmaxf(v, 0.f);
        wl[k * 64 + j * 32 + li] = (unsigned short)bf16_of(v);
      }
    __builtin_amdgcn_sched_barrier(0);
    // the output pixel of row mb + rq, then + 8 per q
    int m = mb + rq;
    int n = m / (Hg * Wg);
    int rr = m - n * Hg * Wg;
    int y = rr / Wg, x = rr - y * Wg;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = rq + 8 * q;
      const uint4 val = *reinterpret_cast<const uint4*>(wl + k * 64 + cq);
      if (k < lim) {
        const unsigned pix = ((unsigned)n * H2 + 2u * y + (ab >> 1)) * W2 + 2u * x + (ab & 1);
        *reinterpret_cast<uint4*>(dst + (size_t)pix * Co + co0 + cq) = val;
      }
      x += 8;  // next row of this lane
      while (x >= Wg) {
        x -= Wg;
        if (++y == Hg) {
          y = 0;
          ++n;
        }
      }
    }
    lgkm_wait0();  // this fragment's LDS reads retired before the next one overwrites the tile
  }
  return true;
}

template <int BM, int BN, int BK, int NSTG>
struct GemmRingGeo {
  static constexpr int RB = BK * 2, CPR = RB / 16, RPB = 256 / RB;  // row bytes, 16-B pieces per row, rows per bank row
  static constexpr int ASZ = BM * RB, BSZ = BN * RB, SSZ = ASZ + BSZ;
  static constexpr size_t smem = (size_t)NSTG * SSZ;
};

// TAPS2: the 2x2 stride-2 gather of a convT input gradient (else 1x1)
template <int BM, int BN, int WM, int WN, int BK, int NSTG, int XTF, int TAPS2>
__global__ __launch_bounds__(WM * WN * 64, 1) void k_gemm_ring(const IgemmArgs args) {
  using G = GemmRingGeo<BM, BN, BK, NSTG>;
  constexpr int RB = G::RB, CPR = G::CPR, RPB = G::RPB;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int DA = BM * RB / 1024 / NW, DB = BN * RB / 1024 / NW, D = DA + DB;  // DMAs per wave per stage
  constexpr int KS = BK / 16;
  constexpr int P = NSTG - 1;  // stages in flight ahead of the one computed
  static_assert(TM >= 1 && TN >= 1 && DA >= 1 && DB >= 1 && (BM * RB / 1024) % NW == 0 &&
                (BN * RB / 1024) % NW == 0, "tile");
  static_assert(BK == 32 || BK == 64, "stage depth");
  static_assert(NSTG >= 3 && NSTG <= 8, "ring depth");
  static_assert(!XTF || NSTG >= 3, "the transform runs one stage ahead");
  static_assert(WM * 3 * BN * 4 <= (int)G::smem, "epilogue reduction must fit the LDS image");
  static_assert(D * (P - (XTF ? 1 : 0)) < 64, "vmcnt");
  extern __shared__ __attribute__((aligned(1024))) unsigned char lds[];
  const unsigned lds0 = (unsigned)(size_t)(lds_u8_t*)lds;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const Gather& g = args.a;
  const Src& s0 = g.s[0];
  const int K = args.K, Cg = g.Cg, M = args.M;
  int bx, by, bz;  // grid position in XCD-aware order
  xcd_block(bx, by, bz);
  const int m0 = bx * BM, n0 = by * BN;
  const int HWg = g.Hg * g.Wg;

  // XTF: BN scale / shift of the source channels, after the ring
  float* xts = reinterpret_cast<float*>(lds + G::smem);
  if constexpr (XTF) {
    for (int c = tid; c < Cg; c += NT) {
      xts[c] = s0.scale[c];
      xts[Cg + c] = s0.shift[c];
    }
  }

  // ---- per-lane DMA source offsets (bytes) ----
  unsigned aoff[DA], boff[DB];
#pragma unroll
  for (int u = 0; u < DA; ++u) {
    const int p = (wave + NW * u) * 64 + lane;  // 16-B piece of the A stage
    const int r = p / CPR, q = (p % CPR) ^ ((r / RPB) % CPR);
    const int m = min(m0 + r, M - 1);  // rows past M: any valid row, never stored
    const int n = m / HWg, rr = m - n * HWg, y = rr / g.Wg, x = rr - y * g.Wg;
    const int sy = TAPS2 ? 2 * y : y, sx = TAPS2 ? 2 * x : x;
    aoff[u] = (unsigned)((((n * s0.H + sy + s0.oy) * s0.W + sx + s0.ox) * s0.C) * 2 + q * 16);
  }
#pragma unroll
  for (int u = 0; u < DB; ++u) {
    const int p = (wave + NW * u) * 64 + lane;
    const int r = p / CPR, q = (p % CPR) ^ ((r / RPB) % CPR);
    boff[u] = (unsigned)((n0 + r) * K * 2 + q * 16);
  }
  // ---- fragment read bases (bytes); k-step and stage are immediates on top ----
  const int hh = lane >> 5, ll = lane & 31;
  unsigned fa[KS], fb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int ra = wm * TM * 32 + ll, rb = wn * TN * 32 + ll;
    fa[s] = (unsigned)(ra * RB + 16 * ((2 * s + hh) ^ ((ra / RPB) % CPR)));
    fb[s] = (unsigned)(G::ASZ + rb * RB + 16 * ((2 * s + hh) ^ ((rb / RPB) % CPR)));
  }

  const int nk_all = K / BK;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = bz * per;
    kc1 = min(nk_all, kc0 + per);
  }
  const int nk = kc1 - kc0;

  // the A source address of stage kc: k0 = kc * BK lies in tap k0 / Cg
  auto a_base = [&](int kc) {
    const int k0 = kc * BK;
    const int tap = TAPS2 ? k0 / Cg : 0, c0 = TAPS2 ? k0 - tap * Cg : k0;
    const int ty = tap >> 1, tx = tap & 1;
    return uniform_u64(reinterpret_cast<const uint16_t*>(s0.ptr) + ((size_t)(ty * s0.W + tx) * s0.C + c0));
  };
  auto b_base = [&](int kc) { return uniform_u64(args.bh + (size_t)kc * BK); };
  // DMA u (0 .. D-1) of stage kc into ring slot `slot`
  auto issue1 = [&](int kc, int slot, int u) {
    if (u < DA) dma_sv(aoff[u], a_base(kc), lds0 + slot * G::SSZ + (wave + NW * u) * 1024);
    else dma_sv(boff[u - DA], b_base(kc), lds0 + slot * G::SSZ + G::ASZ + (wave + NW * (u - DA)) * 1024);
  };
  // relu(bn(.)) of stage kc's A pieces in slot `slot`, in place
  auto transform = [&](int kc, int slot) {
    unsigned char* ab = lds + slot * G::SSZ;
    const int c0 = kc * BK;
#pragma unroll
    for (int k = 0; k < (BM * CPR + NT - 1) / NT; ++k) {
      const int p = tid + NT * k;
      if (p < BM * CPR) {
        const int r = p / CPR, q = (p % CPR) ^ ((r / RPB) % CPR);
        const float* sc = xts + c0 + q * 8;
        const float* sh = xts + Cg + c0 + q * 8;
        uint4* pv = reinterpret_cast<uint4*>(ab + p * 16);
        const uint4 u = *pv;
        *pv = bf16pack8(affine_relu4(bf16x4_to_f4(make_uint2(u.x, u.y)), ld4(sc), ld4(sh)),
                        affine_relu4(bf16x4_to_f4(make_uint2(u.z, u.w)), ld4(sc + 4), ld4(sh + 4)));
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

  const bool xtf = XTF && s0.scale != nullptr;
  if (nk > 0) {
    // prologue: stages 0 .. P-1 (clamped: past the last stage the last one is
    // re-issued into a slot no MFMA reads, so every step retires D DMAs)
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int u = 0; u < D; ++u) issue1(kc0 + min(j, nk - 1), j, u);
    if constexpr (XTF) {
      vm_wait<D * (P - 1)>();
      __syncthreads();  // stage 0 and the BN table visible to every wave
      if (xtf) transform(kc0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  for (int i = 0; i < nk; ++i) {
    // stage i (XTF: and i+1) landed for this wave; the barrier makes every
    // wave's pieces (and the transform of stage i) visible and frees slot i-1
    if constexpr (XTF) vm_wait<D * (P - 2)>();
    else vm_wait<D * (P - 1)>();
    raw_barrier();
    const int slot = i % NSTG, nslot = (i + P) % NSTG;
    const int kn = kc0 + min(i + P, nk - 1);
    if constexpr (XTF) {
      if (xtf && i + 1 < nk) {
        transform(kc0 + i + 1, (i + 1) % NSTG);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    const unsigned sb = slot * G::SSZ;
    bf16x8g_t va[2][TM], vb[2][TN];
    auto rd = [&](int s, int b) {
#pragma unroll
      for (int t = 0; t < TM; ++t) va[b][t] = *reinterpret_cast<const bf16x8g_t*>(lds + sb + fa[s] + t * 32 * RB);
#pragma unroll
      for (int t = 0; t < TN; ++t) vb[b][t] = *reinterpret_cast<const bf16x8g_t*>(lds + sb + fb[s] + t * 32 * RB);
    };
    rd(0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 1 < KS) rd(s + 1, (s + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[s & 1][a], vb[s & 1][b], acc[a][b], 0, 0, 0);
      // this stage's DMAs, spread over the k-steps
#pragma unroll
      for (int u = 0; u < D; ++u)
        if (u * KS / D == s) issue1(kn, nslot, u);
    }
  }
  vm_wait<0>();
  __syncthreads();
  // the whole LDS image is free: the waves' 4-KB staging tiles first, the
  // statistics buffer after them
  constexpr bool kStage = TN == 2 && (size_t)NW * 4096 + (size_t)WM * 3 * BN * 4 <= G::smem;
  unsigned short* stage = kStage ? reinterpret_cast<unsigned short*>(lds) : nullptr;
  float* red = reinterpret_cast<float*>(lds + (kStage ? NW * 4096 : 0));
  if constexpr (kStage) {
    if (epi_shuffle_staged<TM, TN, WM, WN>(args, acc, m0, n0, wm, wn, tid, stage)) return;
  }
  igemm_finish<BM, BN, WM, WN, NT, LinearRows, 1>(args, acc, m0, n0, wm, wn, tid, red, LinearRows{0, 0}, stage, bz);
}

// ---------------------------------------------------------------------------
// tile ids (igemm.hip tile_info 91-99)
// ---------------------------------------------------------------------------
bool gemm_ring_tile_shape(int tile, int& bm, int& bn) {
  switch (tile) {
    case 91: bm = 128; bn = 128; return true;  // 4 waves (2 x 2), BK 64, 4 stages: 128 KB
    case 92: bm = 256; bn = 128; return true;  // 8 waves (4 x 2), BK 64, 3 stages: 144 KB
    case 93: bm = 128; bn = 256; return true;  // 8 waves (2 x 4), BK 64, 3 stages: 144 KB
    case 94: bm = 128; bn = 128; return true;  // 8 waves (2 x 4), BK 64, 4 stages: 128 KB
    case 95: bm = 64; bn = 128; return true;   // 4 waves (1 x 4), BK 64, 4 stages: 96 KB
    case 96: bm = 256; bn = 256; return true;  // 8 waves (2 x 4, 128 x 64 each), BK 32, 4 stages: 128 KB
    case 97: bm = 256; bn = 128; return true;  // 8 waves (4 x 2), BK 32, 6 stages: 144 KB
    case 98: bm = 128; bn = 256; return true;  // 8 waves (2 x 4), BK 32, 6 stages: 144 KB
    case 99: bm = 128; bn = 128; return true;  // 4 waves (2 x 2), BK 32, 8 stages: 128 KB
    default: return false;
  }
}

// convT forward (1x1 gather, K = Cg) or convT input gradient (2x2 stride-2
// gather, K = 4 Cg), bf16 sources and packed bf16 B, channel counts multiples
// of 64, one source (no concat)
bool gemm_ring_fits(const IgemmArgs& a, int tile) {
  int bm, bn;
  if (!gemm_ring_tile_shape(tile, bm, bn)) return false;
  const Gather& g = a.a;
  const bool t1 = g.taps_h == 1 && g.taps_w == 1 && g.stride == 1 && a.K == g.Cg;
  const bool t2 = g.taps_h == 2 && g.taps_w == 2 && g.stride == 2 && a.K == 4 * g.Cg && g.s[0].scale == nullptr;
  const double bytes = (double)g.nimg * g.s[0].H * g.s[0].W * g.s[0].C * 2;
  return (t1 || t2) && a.bh != nullptr && a.bl == nullptr && g.s[0].h16 && g.c_split >= g.Cg && g.Cg % 64 == 0 &&
         g.Cg <= 2048 && a.N % bn == 0 && a.batch <= 1 && bytes < 4294967296.0 &&
         (double)a.N * a.K * 2 < 4294967296.0;
}

template <int BM, int BN, int WM, int WN, int BK, int NSTG>
static hipError_t go_gemm_ring(const IgemmArgs& a, hipStream_t s) {
  using G = GemmRingGeo<BM, BN, BK, NSTG>;
  const bool t2 = a.a.taps_h == 2, xtf = a.a.s[0].scale != nullptr;
  const int v = (t2 ? 2 : 0) | (xtf ? 1 : 0);
  static bool attr[4] = {false, false, false, false};
  const void* fns[4] = {reinterpret_cast<const void*>(&k_gemm_ring<BM, BN, WM, WN, BK, NSTG, 0, 0>),
                        reinterpret_cast<const void*>(&k_gemm_ring<BM, BN, WM, WN, BK, NSTG, 1, 0>),
                        reinterpret_cast<const void*>(&k_gemm_ring<BM, BN, WM, WN, BK, NSTG, 0, 1>),
                        reinterpret_cast<const void*>(&k_gemm_ring<BM, BN, WM, WN, BK, NSTG, 1, 1>)};
  if (v == 3) return hipErrorInvalidValue;  // the input-gradient gather has no transform
  const size_t smem = G::smem + (xtf ? 8 * (size_t)a.a.Cg : 0);
  if (!attr[v]) {
    hipError_t e = hipFuncSetAttribute(fns[v], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr[v] = true;
  }
  dim3 grid((a.M + BM - 1) / BM, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  switch (v) {
    case 0: hipLaunchKernelGGL((k_gemm_ring<BM, BN, WM, WN, BK, NSTG, 0, 0>), grid, dim3(WM * WN * 64), smem, s, a); break;
    case 1: hipLaunchKernelGGL((k_gemm_ring<BM, BN, WM, WN, BK, NSTG, 1, 0>), grid, dim3(WM * WN * 64), smem, s, a); break;
    default: hipLaunchKernelGGL((k_gemm_ring<BM, BN, WM, WN, BK, NSTG, 0, 1>), grid, dim3(WM * WN * 64), smem, s, a); break;
  }
  return hipGetLastError();
}

hipError_t go_gemm_ring_tile(const IgemmArgs& a, hipStream_t s, int tile) {
  if (!gemm_ring_fits(a, tile)) return hipErrorInvalidValue;
  switch (tile) {
    case 91: return go_gemm_ring<128, 128, 2, 2, 64, 4>(a, s);
    case 92: return go_gemm_ring<256, 128, 4, 2, 64, 3>(a, s);
    case 93: return go_gemm_ring<128, 256, 2, 4, 64, 3>(a, s);
    case 94: return go_gemm_ring<128, 128, 2, 4, 64, 4>(a, s);
    case 95: return go_gemm_ring<64, 128, 1, 4, 64, 4>(a, s);
    case 96: return go_gemm_ring<256, 256, 2, 4, 32, 4>(a, s);
    case 97: return go_gemm_ring<256, 128, 4, 2, 32, 6>(a, s);
    case 98: return go_gemm_ring<128, 256, 2, 4, 32, 6>(a, s);
    default: return go_gemm_ring<128, 128, 2, 2, 32, 8>(a, s);
  }
}

}  // namespace unet
