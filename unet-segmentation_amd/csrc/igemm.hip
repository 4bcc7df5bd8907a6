// Implicit-GEMM convolution kernels for gfx950 (MI355X), fp32 in / fp32 accumulate
// on the matrix cores (v_mfma_f32_32x32x2_f32: exact f32 fma chain, 64 FLOP/clk/SIMD).
//
// One kernel family serves every dense op of the U-Net hot path
// (models/unet_model.py): 3x3 valid conv forward (nn.Conv2d, :11/:15), its input
// gradient (full correlation with the flipped kernel over a zero-padded dY), the
// ConvTranspose2d k2s2 forward (:45, a GEMM + pixel-shuffle store) and its input
// gradient (a 4-tap stride-2 gather).  The weight gradient of all of them is the
// second kernel (k_wgrad): a pixel-reduction GEMM split over workgroups.
//
// Operand staging: A rows are pixels gathered from NHWC tensors (16 channels =
// 64 contiguous bytes per row per K-step), with the consumer-side BatchNorm+ReLU
// transform and the skip/upsample channel concat folded into the gather.
// LDS tiles are [rows][16+4] floats (80-B row stride: ds_read_b128 conflict-free),
// double buffered.  The next K-step's global loads are issued before the MFMA
// block and consumed (transform + ds_write) after it, so each wave's HBM/L2
// latency hides under its own 32 MFMAs (2048 cycles) plus its SIMD partners'.
#include <cstdio>
#include <cstdlib>

#include "gemm_common.h"
#include "ring_common.h"

namespace unet {
// convT weight gradient on an LDS-DMA ring of pixel stages (wgradT_ring.hip,
// wgrad tiles 40-43)
bool wgradT_ring_fits(const WgradArgs& a, int tile);
hipError_t go_wgradT_ring(const WgradArgs& a, hipStream_t s, int tile, int per_cu);
// conv3_flat.hip (tile 85: the ring on flat pixel tiles)
bool conv3_flat_fits(const IgemmArgs& a, int tile);
long long conv3_flat_tiles(const IgemmArgs& a, int tile);
hipError_t go_conv3_flat_tile(const IgemmArgs& a, hipStream_t s, int tile);
// conv3_c64.hip (tile 87: 64 -> 64 channels, resident weights, persistent)
bool conv3_c64_fits(const IgemmArgs& a);
long long conv3_c64_tiles(const IgemmArgs& a);
hipError_t go_conv3_c64(const IgemmArgs& a, hipStream_t s);

// Occupancy the register allocator must preserve: as many workgroups as the
// LDS footprint admits per CU (without it hipcc moves the accumulators to
// AGPRs and drops a wave per SIMD).
constexpr int igemm_minw(int BM, int BN, int WM, int WN, int BK) {
  const int lds = 2 * (BM + BN) * (BK + 4) * 4 + WM * 3 * BN * 4;
  int blocks = 163840 / lds;
  if (blocks > 8) blocks = 8;
  int w = blocks * WM * WN * 64 / 256;
  // 8-wave tiles: at most 2 waves/SIMD (256 registers).  At 4 the 256x128 tile
  // spilled 52 VGPRs to scratch inside the LDS-DMA pipeline and lost parity.
  if (WM * WN >= 8 && w > 2) w = 2;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// ABL: ablation switches for tools/igemm_bench.cpp only (0 in the library):
// 1 no global loads, 2 no in-loop barrier, 4 no BN transform, 8 no LDS
// fragment reads, 16 no LDS stores, 32 BN transform with constant scale/shift
// (no scale/shift loads), 64 no A loads, 128 no B loads, 256 A loads from
// contiguous addresses, 512 global loads for the first two K-steps only (the
// LDS keeps real, non-zero data: MFMA power and clock stay representative).
// Results are meaningless when set.
// PF: K-steps of operands in flight in registers (1 or 2).
template <int BM, int BN, int WM, int WN, int BK, int ABL = 0, int PF = 1>
__global__ __launch_bounds__(WM * WN * 64, igemm_minw(BM, BN, WM, WN, BK)) void k_igemm(const IgemmArgs args) {
  constexpr int NT = WM * WN * 64;
  constexpr int LDK = BK + 4;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int C4 = BK / 4;           // float4 per staged row
  constexpr int RPP = NT / C4;         // rows per staging pass
  constexpr int AV = BM / RPP, BV = BN / RPP;
  constexpr int KH = BK / 2, KF = KH / 4;
  static_assert(TM >= 1 && TN >= 1 && AV >= 1 && BV >= 1 && BM % RPP == 0 && BN % RPP == 0, "tile");
  __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * LDK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // batched dense GEMMs (Winograd points): rows of batch z are z*batch_rows ..
  int bx, by, bz;  // XCD-aware grid order: an XCD's run shares the B panels (and a batch entry) in its L2
  xcd_block(bx, by, bz);
  const int zb = args.batch > 1 ? bz : 0;
  const int m0 = zb * args.batch_rows + bx * BM, n0 = by * BN;
  const Gather& g = args.a;
  const int M = args.batch > 1 ? (zb + 1) * args.batch_rows : args.M, K = args.K;
  // staging row of this thread.  With BK = 16 a row is 4 x 16 B and the 8 lanes
  // of a ds_write_b128 group store two rows; rows r and r + 1 (80-B stride) share
  // 2 of the 32 bank quads (mod-32 banking of stores), r and r + 4 share none:
  // pair rows 4 apart within each block of 8 (the fragment reads are unchanged)
  const int col4 = tid % C4, row0 = C4 == 4 ? stage_row8(tid / C4) : tid / C4;

  // Per staged A row: pixel base in each source grid (before the tap offset).
  int rb0[AV], rb1[AV];
  const int HWg = g.Hg * g.Wg;
#pragma unroll
  for (int q = 0; q < AV; ++q) {
    int m = m0 + row0 + RPP * q;
    m = m < M ? m : M - 1;
    int n = m / HWg, r = m - n * HWg;
    int y = r / g.Wg, x = r - y * g.Wg;
    y *= g.stride;
    x *= g.stride;
    rb0[q] = (n * g.s[0].H + y + g.s[0].oy) * g.s[0].W + x + g.s[0].ox;
    rb1[q] = (n * g.s[1].H + y + g.s[1].oy) * g.s[1].W + x + g.s[1].ox;
  }
  const float* bptr[BV];
#pragma unroll
  for (int q = 0; q < BV; ++q)
    bptr[q] = args.b + (size_t)zb * args.batch_b + (size_t)(n0 + row0 + RPP * q) * K + col4 * 4;

  // K range of this workgroup (split-K slices chunks over blockIdx.z)
  const int nk_all = K / BK;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1 && args.batch <= 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = bz * per;
    kc1 = min(nk_all, kc0 + per);
  }
  // K iterator (uniform): chunk -> (tap_y, tap_x, c0).  A chunk never straddles
  // a tap or the concat split (Cg and c_split are multiples of BK).
  int it_ty = 0, it_tx = 0, it_c = 0;
  {
    const int cpt = g.Cg / BK;
    const int tap = kc0 / cpt;
    it_c = (kc0 - tap * cpt) * BK;
    it_ty = tap / g.taps_w;
    it_tx = tap - it_ty * g.taps_w;
  }
  // One K-step of staged operands in registers (PF of them in flight).
  struct Stage {
    float4 ra[AV], rb[BV], sc, sh;
    bool tf;
  };
  Stage S0, S1;
  if (ABL & (1 | 64 | 128)) {
#pragma unroll
    for (int q = 0; q < AV; ++q) S0.ra[q] = S1.ra[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < BV; ++q) S0.rb[q] = S1.rb[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    S0.sc = S0.sh = S1.sc = S1.sh = S0.ra[0];
  }
  int nissued = 0;
  auto issue = [&](Stage& st, int k0) {
    const bool second = it_c >= g.c_split;
    const Src& s = second ? g.s[1] : g.s[0];
    const int c = (second ? it_c - g.c_split : it_c) + col4 * 4;
    const int toff = it_ty * s.W + it_tx;
    if (!(ABL & 1) && (!(ABL & 512) || nissued++ < 2)) {
      if (ABL & 256) {  // contiguous 1 KiB per wave-instruction (layout experiment)
#pragma unroll
        for (int q = 0; q < AV; ++q)
          st.ra[q] = ld4(s.ptr + (((size_t)(m0 + RPP * q) * BK + k0 * 64) % ((size_t)s.C * s.H * s.W)) + tid * 4);
      } else if (!(ABL & 64)) {
#pragma unroll
        for (int q = 0; q < AV; ++q) st.ra[q] = ld4(s.ptr + (size_t)((second ? rb1[q] : rb0[q]) + toff) * s.C + c);
      }
      if (!(ABL & 128)) {
#pragma unroll
        for (int q = 0; q < BV; ++q) st.rb[q] = ld4(bptr[q] + k0);
      }
    }
    st.tf = !(ABL & 4) && s.scale != nullptr;
    if (ABL & 32) {
      st.sc = make_float4(1.f, 1.f, 1.f, 1.f);
      st.sh = make_float4(0.f, 0.f, 0.f, 0.f);
    } else if (st.tf && !(ABL & 1)) {
      st.sc = ld4(s.scale + c);
      st.sh = ld4(s.shift + c);
    }
    it_c += BK;
    if (it_c == g.Cg) {
      it_c = 0;
      if (++it_tx == g.taps_w) { it_tx = 0; ++it_ty; }
    }
  };
  auto commit = [&](Stage& st, int buf) {
    if (ABL & 16) return;
    float* As = lds + buf * (BM + BN) * LDK;
    float* Bs = As + BM * LDK;
    if (st.tf) {
#pragma unroll
      for (int q = 0; q < AV; ++q) st.ra[q] = affine_relu4(st.ra[q], st.sc, st.sh);
    }
#pragma unroll
    for (int q = 0; q < AV; ++q) st4(As + (row0 + RPP * q) * LDK + col4 * 4, st.ra[q]);
#pragma unroll
    for (int q = 0; q < BV; ++q) st4(Bs + (row0 + RPP * q) * LDK + col4 * 4, st.rb[q]);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int h = lane >> 5, li = lane & 31;
  auto compute = [&](int buf, int kc) {
    const float* As = lds + buf * (BM + BN) * LDK;
    const float* Bs = As + BM * LDK;
    float4 fa[TM][KF], fb[TN][KF];
    if (ABL & 8) {
      const float v = (float)(lane + kc);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int f = 0; f < KF; ++f) fa[i][f] = make_float4(v, v + i, v + f, v);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int f = 0; f < KF; ++f) fb[j][f] = make_float4(v, v + j, v + f, v);
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* p = As + (wm * TM * 32 + i * 32 + li) * LDK + h * KH;
#pragma unroll
        for (int f = 0; f < KF; ++f) fa[i][f] = ld4(p + 4 * f);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* p = Bs + (wn * TN * 32 + j * 32 + li) * LDK + h * KH;
#pragma unroll
        for (int f = 0; f < KF; ++f) fb[j][f] = ld4(p + 4 * f);
      }
    }
#pragma unroll
    for (int s = 0; s < KH; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(getc(fa[i][s >> 2], s & 3), getc(fb[j][s >> 2], s & 3),
                                                           acc[i][j], 0, 0, 0);
  };
  auto barrier = [&] {
    if (!(ABL & 2)) __syncthreads();
  };

  if constexpr (PF == 1) {
    // one K-step in flight: loads for kc+1 issued before kc's MFMAs, stored after
    if (kc0 < kc1) {
      issue(S0, kc0 * BK);
      commit(S0, 0);
      barrier();
    }
    for (int kc = kc0; kc < kc1; ++kc) {
      const int cur = (kc - kc0) & 1;
      const bool more = kc + 1 < kc1;
      if (more) issue(S0, (kc + 1) * BK);
      compute(cur, kc);
      if (more) commit(S0, cur ^ 1);
      barrier();
    }
  } else {
    // two K-steps in flight (register sets S0/S1 alternate; loop unrolled by 2)
    if (kc0 < kc1) {
      issue(S0, kc0 * BK);
      commit(S0, 0);
      if (kc0 + 1 < kc1) issue(S1, (kc0 + 1) * BK);
      barrier();
    }
    for (int kc = kc0; kc < kc1; kc += 2) {
      if (kc + 2 < kc1) issue(S0, (kc + 2) * BK);
      compute(0, kc);
      if (kc + 1 < kc1) commit(S1, 1);
      barrier();
      if (kc + 1 >= kc1) break;
      if (kc + 3 < kc1) issue(S1, (kc + 3) * BK);
      compute(1, kc + 1);
      if (kc + 2 < kc1) commit(S0, 0);
      barrier();
    }
  }

  __shared__ float red[WM * 3 * BN];
  igemm_finish<BM, BN, WM, WN, NT>(args, acc, m0, n0, wm, wn, tid, red, LinearRows{m0, M}, nullptr, bz);
}


// ---------------------------------------------------------------------------
// k_igemm_g: the same implicit GEMM with LDS-DMA staging.  Every K-step's A
// and B tiles go global -> LDS by global_load_lds_dwordx4 (no staging VGPRs,
// no ds_write), through a 3-slot LDS ring: the loads of step k+2 are in flight
// while step k computes.  LDS rows are 16 floats (64 B) unpadded; the 16-B
// chunk c of row r sits at slot c ^ ((r >> 2) & 3) (the source address carries
// the permutation, the fragment read applies it), which keeps every
// ds_read_b128 lane group on distinct bank quads.  The consumer-side BN+ReLU
// of the A operand is applied to the fragments after the LDS read, with
// scale/shift preloaded into LDS once per workgroup.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) float lds_float_t;

// One global_load_lds_dwordx4: 16 B per lane from `src` into LDS at the
// wave-uniform `dst` + lane*16.  Inline asm, so that hipcc neither waits for it
// before unrelated ds_reads (it cannot tell ring slots apart) nor counts it:
// the caller retires it with an explicit vmcnt.
__device__ __forceinline__ void glds16(const float* src, float* dst) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_float_t*)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds)
               : "memory");
}

constexpr int igemm_g_lds_floats(int BM, int BN) { return 3 * (BM + BN) * 16; }
constexpr int igemm_g_minw(int BM, int BN, int WM, int WN) {
  int blocks = 163840 / (igemm_g_lds_floats(BM, BN) * 4 + 2048);
  if (blocks > 8) blocks = 8;
  int w = blocks * WM * WN * 64 / 256;
  // 8-wave tiles: at most 2 waves/SIMD (256 registers).  At 4 the 256x128 tile
  // spilled 52 VGPRs to scratch inside the LDS-DMA pipeline and lost parity.
  if (WM * WN >= 8 && w > 2) w = 2;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

// s_waitcnt vmcnt(n) leaving expcnt/lgkmcnt unconstrained (gfx9 encoding)
#define UNET_WAIT_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n)&15) | (7 << 4) | (15 << 8) | ((((n) >> 4) & 3) << 14))

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, igemm_g_minw(BM, BN, WM, WN)) void k_igemm_g(const IgemmArgs args) {
  constexpr int NT = WM * WN * 64, NW = WM * WN, BK = 16, NS = 3;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int PA = BM / (16 * NW), PB = BN / (16 * NW);  // 1-KiB pieces per wave per step
  static_assert(PA >= 1 && PB >= 1 && BM % (16 * NW) == 0 && BN % (16 * NW) == 0, "tile");
  extern __shared__ __attribute__((aligned(16))) float dl[];
  float* ssc = dl + NS * STAGE;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int bx, by, bz;  // XCD-aware grid order
  xcd_block(bx, by, bz);
  const int m0 = bx * BM, n0 = by * BN;
  const Gather& g = args.a;
  const int M = args.M, K = args.K, Cg = g.Cg;
  const int lrow = lane >> 2, lslot = lane & 3;

  // per-lane source rows of this wave's pieces (row r of the tile = piece*16 + lrow)
  int rb0[PA], rb1[PA], ca[PA];
  const int HWg = g.Hg * g.Wg;
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int r = (wave * PA + p) * 16 + lrow;
    int m = m0 + r;
    m = m < M ? m : M - 1;
    const int n = m / HWg, rr = m - n * HWg;
    int y = rr / g.Wg, x = rr - y * g.Wg;
    y *= g.stride;
    x *= g.stride;
    rb0[p] = (n * g.s[0].H + y + g.s[0].oy) * g.s[0].W + x + g.s[0].ox;
    rb1[p] = (n * g.s[1].H + y + g.s[1].oy) * g.s[1].W + x + g.s[1].ox;
    ca[p] = (lslot ^ ((r >> 2) & 3)) * 4;
  }
  const float* bptr[PB];
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int r = (wave * PB + p) * 16 + lrow;
    bptr[p] = args.b + (size_t)(n0 + r) * K + (lslot ^ ((r >> 2) & 3)) * 4;
  }
  // consumer BN+ReLU parameters of the concatenated channel range
  const bool any_tf = g.s[0].scale != nullptr || (g.c_split < Cg && g.s[1].scale != nullptr);
  if (any_tf) {
    for (int c = tid; c < Cg; c += NT) {
      const bool sec = c >= g.c_split;
      const Src& sr = sec ? g.s[1] : g.s[0];
      const int cl = sec ? c - g.c_split : c;
      ssc[c] = sr.scale ? sr.scale[cl] : 1.f;
      ssc[Cg + c] = sr.scale ? sr.shift[cl] : 0.f;
    }
    __syncthreads();
  }

  const int nk_all = K / BK;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = bz * per;
    kc1 = min(nk_all, kc0 + per);
  }
  // producer-side K iterator (issue runs two steps ahead of compute)
  int it_ty, it_tx, it_c;
  {
    const int cpt = Cg / BK;
    const int tap = kc0 / cpt;
    it_c = (kc0 - tap * cpt) * BK;
    it_ty = tap / g.taps_w;
    it_tx = tap - it_ty * g.taps_w;
  }
  int cc = it_c;  // consumer-side channel offset of the step being computed

  auto issue = [&](int slot, int k0) {
    const bool second = it_c >= g.c_split;
    const Src& s = second ? g.s[1] : g.s[0];
    const int c = second ? it_c - g.c_split : it_c;
    const int toff = it_ty * s.W + it_tx;
    float* As = dl + slot * STAGE;
    float* Bs = As + BM * BK;
#pragma unroll
    for (int p = 0; p < PA; ++p)
      glds16(s.ptr + (size_t)((second ? rb1[p] : rb0[p]) + toff) * s.C + c + ca[p], As + (wave * PA + p) * 16 * BK);
#pragma unroll
    for (int p = 0; p < PB; ++p) glds16(bptr[p] + k0, Bs + (wave * PB + p) * 16 * BK);
    it_c += BK;
    if (it_c == Cg) {
      it_c = 0;
      if (++it_tx == g.taps_w) { it_tx = 0; ++it_ty; }
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
  const int sw = (li >> 2) & 3;  // row swizzle of this lane's fragment rows (row bases are multiples of 32)
  auto compute = [&](int slot) {
    const float* As = dl + slot * STAGE;
    const float* Bs = As + BM * BK;
    float4 fa[TM][2], fb[TN][2];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* pr = As + (wm * TM * 32 + i * 32 + li) * BK;
#pragma unroll
      for (int f = 0; f < 2; ++f) fa[i][f] = ld4(pr + (((2 * h + f) ^ sw) << 2));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float* pr = Bs + (wn * TN * 32 + j * 32 + li) * BK;
#pragma unroll
      for (int f = 0; f < 2; ++f) fb[j][f] = ld4(pr + (((2 * h + f) ^ sw) << 2));
    }
    const bool tf = cc < g.c_split ? g.s[0].scale != nullptr : g.s[1].scale != nullptr;
    if (tf) {
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const float4 sc = ld4(ssc + cc + 8 * h + 4 * f), sh = ld4(ssc + Cg + cc + 8 * h + 4 * f);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i][f] = affine_relu4(fa[i][f], sc, sh);
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(getc(fa[i][s >> 2], s & 3), getc(fb[j][s >> 2], s & 3),
                                                           acc[i][j], 0, 0, 0);
    cc += BK;
    if (cc == Cg) cc = 0;
  };

  if (kc0 < kc1) issue(0, kc0 * BK);
  if (kc0 + 1 < kc1) issue(1, (kc0 + 1) * BK);
  int slot = 0;
  for (int kc = kc0; kc < kc1; ++kc) {
    // this wave's loads of step kc have landed (step kc+1's may still fly) ...
    if (kc + 1 < kc1) UNET_WAIT_VMCNT(PA + PB);
    else UNET_WAIT_VMCNT(0);
    // ... and every wave's (also: every wave is done reading the slot refilled next)
    __builtin_amdgcn_s_barrier();
    if (kc + 2 < kc1) issue(slot == 0 ? 2 : slot - 1, (kc + 2) * BK);
    compute(slot);
    slot = slot == 2 ? 0 : slot + 1;
  }
  __syncthreads();  // the ring is reused as the epilogue's reduction buffer
  igemm_finish<BM, BN, WM, WN, NT>(args, acc, m0, n0, wm, wn, tid, dl, LinearRows{0, 0}, nullptr, bz);
}

template <int BM, int BN>
constexpr size_t igemm_g_smem(int cg) {
  return (size_t)igemm_g_lds_floats(BM, BN) * 4 + (size_t)2 * cg * 4;
}

// ---------------------------------------------------------------------------
// k_conv3_f32: halo-tiled 3x3 stride-1 implicit GEMM in fp32 (conv forward and
// conv input gradient), the fp32 twin of k_conv3_bf (igemm_bf16.hip).  A
// workgroup owns a TH x TW tile of one image's output grid and BN output
// columns; per 16-channel chunk it stages the (TH+2) x (TW+2) input halo once
// (consumer BN+ReLU applied) and the chunk's weights for all 9 taps, and each
// tap reads a shifted window of the same halo.  Against k_igemm's pixel-row
// gather (one barrier and one staging pass per 16-k step, A fetched once per
// tap) a chunk carries 9 taps x 8 MFMA k-steps between its two barriers.
// LDS rows: 16 floats + 4 pad (80 B, ds_read_b128 conflict-free); fragment
// k-order as k_igemm (lane half h holds k = 8h .. 8h+7, MFMA s pairs k = s and
// 8 + s in both operands).  BN scale/shift are read per staged unit from global
// (L1/L2 hits), so the LDS holds only the operands: 8x32 x BN64 = 73 KiB, two
// workgroups per CU.
// ---------------------------------------------------------------------------
template <int TH, int TW, int BN>
constexpr size_t conv3_f32_smem() {
  return (size_t)((TH + 2) * (TW + 2) + 9 * BN) * 20 * 4;
}

template <int TH, int TW, int BN, int WM, int WN, int MINW>
__global__ __launch_bounds__(WM * WN * 64, MINW) void k_conv3_f32(const IgemmArgs args) {
  constexpr int NT = WM * WN * 64, BM = TH * TW, LDR = 20;
  constexpr int HW2 = TW + 2, PH = (TH + 2) * HW2;
  constexpr int FM = BM / 32, TM = FM / WM, TN = BN / (WN * 32);
  constexpr int UA = PH * 4, UB = 9 * BN * 4;  // 16-B staging units (4 channels / 4 k each)
  constexpr int NA = (UA + NT - 1) / NT, NB = (UB + NT - 1) / NT;
  constexpr int A_EL = PH * LDR;
  static_assert(BM % 32 == 0 && FM % WM == 0 && TM >= 1 && TN >= 1, "tile");
  static_assert(WM * 3 * BN <= A_EL, "epilogue reduction must fit the halo buffer");
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  float* As = hsm;
  float* Bs = hsm + A_EL;

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

  // staging units: A = (halo pixel, 4-channel piece), B = (tap, row, 4-k piece)
  int pi0[NA], pi1[NA];
#pragma unroll
  for (int k = 0; k < NA; ++k) {
    const int u = min(tid + k * NT, UA - 1);
    const int ph = u >> 2;
    const int hy = ph / HW2, hx = ph - hy * HW2;
    const int yy = min(y0 + hy, Hg + 1), xx = min(x0 + hx, Wg + 1);  // overhang: any in-range pixel
    pi0[k] = (n * g.s[0].H + yy + g.s[0].oy) * g.s[0].W + xx + g.s[0].ox;
    pi1[k] = (n * g.s[1].H + yy + g.s[1].oy) * g.s[1].W + xx + g.s[1].ox;
  }
  int bsrc[NB];  // element offsets into args.b
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int u = min(tid + k * NT, UB - 1);
    const int r = (u >> 2) % BN, tap = (u >> 2) / BN;
    bsrc[k] = (n0 + r) * K + tap * Cg + (u & 3) * 4;
  }

  const int nk_all = Cg / 16;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = blockIdx.z * per;
    kc1 = min(nk_all, kc0 + per);
  }

  float4 ra[NA], rb[NB], sc, sh;
  bool tf = false;
  auto issue = [&](int kc) {
    const int c0 = kc * 16;
    const bool second = c0 >= g.c_split;
    const Src s = pick_src(g, second);
    const int cl = (second ? c0 - g.c_split : c0) + (tid & 3) * 4;
#pragma unroll
    for (int k = 0; k < NA; ++k)
      if (tid + k * NT < UA) ra[k] = ld4(s.ptr + (size_t)(second ? pi1[k] : pi0[k]) * s.C + cl);
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (tid + k * NT < UB) rb[k] = ld4(args.b + bsrc[k] + c0);
    tf = s.scale != nullptr;
    if (tf) {  // the unit's 4 channels are the same for every A unit of this lane
      sc = ld4(s.scale + cl);
      sh = ld4(s.shift + cl);
    }
  };
  auto commit = [&] {
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      if (u < UA) st4(As + (u >> 2) * LDR + (u & 3) * 4, tf ? affine_relu4(ra[k], sc, sh) : ra[k]);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = tid + k * NT;
      if (u < UB) st4(Bs + (u >> 2) * LDR + (u & 3) * 4, rb[k]);
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
  auto compute = [&] {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int off = (tap / 3) * HW2 + tap % 3;
      float4 fa[TM][2], fb[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* p = As + (abase[i] + off) * LDR + 8 * h;
        fa[i][0] = ld4(p);
        fa[i][1] = ld4(p + 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* p = Bs + (tap * BN + wn * TN * 32 + j * 32 + li) * LDR + 8 * h;
        fb[j][0] = ld4(p);
        fb[j][1] = ld4(p + 4);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(getc(fa[i][s >> 2], s & 3), getc(fb[j][s >> 2], s & 3),
                                                             acc[i][j], 0, 0, 0);
    }
  };

  if (kc0 < kc1) {
    issue(kc0);
    commit();
  }
  __syncthreads();
  for (int kc = kc0; kc < kc1; ++kc) {
    const bool more = kc + 1 < kc1;
    if (more) issue(kc + 1);
    compute();
    __syncthreads();
    if (more) {
      commit();
      __syncthreads();
    }
  }
  igemm_finish<BM, BN, WM, WN, NT>(args, acc, 0, n0, wm, wn, tid, hsm, HaloRows<TW, TH>{n, y0, x0, Hg, Wg});
}

// ---------------------------------------------------------------------------
// k_wgrad3_f32: halo-tiled weight gradient of a 3x3 stride-1 conv in fp32, the
// fp32 twin of k_wgrad3_bf.  dW[co][tap][ci] = sum_p dY[p][co] * X[p + tap][ci]
// for a 64 (co) x 64 (ci) block and all 9 taps per workgroup, walking TH x TW
// output-pixel tiles strided over blockIdx.z; per tile the dY tile and the
// (TH+2) x (TW+2) X halo are staged once (X with the consumer BN+ReLU) and every
// tap reads a shifted pixel window of the halo.  The MFMA k is the pixel: in
// v_mfma_f32_32x32x2_f32 lane half h holds pixel 2s + h of k-step s, so each
// operand is one ds_read_b32 per lane from the natural [pixel][64 ch] image
// (256-B rows).  Rows of odd pixels store their two 32-channel halves swapped,
// so the two lane halves (adjacent pixels) always sit in opposite bank halves:
// conflict-free for every tap shift.  LDS (8x16 tile): (128 + 180) x 256 B =
// 77 KiB, two workgroups per CU.  Waves (8): co tile w & 1, ci tile (w >> 1) & 1,
// tap group w >> 2 (taps 0-4 / 5-8), one accumulator per tap.
// ---------------------------------------------------------------------------
template <int TH, int TW>
constexpr size_t wgrad3_f32_smem() {
  return (size_t)(TH * TW + (TH + 2) * (TW + 2)) * 256 + 2 * 64 * 4;
}
__device__ __forceinline__ int w3f_idx(int p, int c) { return p * 64 + (c ^ ((p & 1) << 5)); }

template <int TH, int TW>
__global__ __launch_bounds__(512, 2) void k_wgrad3_f32(const WgradArgs args) {
  constexpr int NT = 512, BC = 64, NTAP = 5;
  constexpr int PT = TH * TW, HW2 = TW + 2, PH = (TH + 2) * HW2;
  constexpr int UA = PT * 16, UB = PH * 16;  // 16-B units: (pixel, 4-channel piece)
  constexpr int NA = (UA + NT - 1) / NT, NB = (UB + NT - 1) / NT;
  static_assert(TW % 2 == 0 && UA % NT == 0 && NA <= 32, "a k-step's pixel pair stays inside one tile row");
  extern __shared__ __attribute__((aligned(16))) float wsf[];
  float* Ad = wsf;                   // dY tile [PT][64]
  float* Bx = wsf + PT * 64;         // X halo [PH][64]
  float* ssc = wsf + (PT + PH) * 64;  // [2][64]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const Gather& gb = args.gb;
  const Src& ds = args.ga.s[0];
  const int i0 = blockIdx.x * 64;  // co block
  const int cb = blockIdx.y * BC;  // ci block (gather channel index)
  const int Hg = gb.Hg, Wg = gb.Wg, Ci = gb.Cg;
  const bool second = cb >= gb.c_split;  // a 64-channel block never straddles the concat split
  const Src xs = pick_src(gb, second);
  const int xc = second ? cb - gb.c_split : cb;
  const bool xtf = xs.scale != nullptr;
  if (xtf) {
    for (int c = tid; c < BC; c += NT) {
      ssc[c] = xs.scale[xc + c];
      ssc[BC + c] = xs.shift[xc + c];
    }
  }
  const int tiles_x = (Wg + TW - 1) / TW, tiles_y = (Hg + TH - 1) / TH;
  const int tiles = gb.nimg * tiles_x * tiles_y;

  float4 rd[NA], rx[NB];
  unsigned dvalid = 0;
  auto issue = [&](int t) {
    const int x0 = (t % tiles_x) * TW;
    const int r = t / tiles_x;
    const int y0 = (r % tiles_y) * TH, n = r / tiles_y;
    dvalid = 0;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      const int p = u >> 4, ch = u & 15;
      const int y = y0 + p / TW, x = x0 + p % TW;
      dvalid |= (y < Hg && x < Wg) ? (1u << k) : 0u;
      const int yy = min(y, Hg - 1), xx = min(x, Wg - 1);
      rd[k] = ld4(ds.ptr + (size_t)((n * ds.H + yy + ds.oy) * ds.W + xx + ds.ox) * ds.C + i0 + ch * 4);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = min(tid + k * NT, UB - 1);
      const int hp = u >> 4, ch = u & 15;
      const int yy = min(y0 + hp / HW2, Hg + 1), xx = min(x0 + hp % HW2, Wg + 1);
      rx[k] = ld4(xs.ptr + (size_t)((n * xs.H + yy + xs.oy) * xs.W + xx + xs.ox) * xs.C + xc + ch * 4);
    }
  };
  auto commit = [&] {
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int u = tid + k * NT;
      const int p = u >> 4, ch = u & 15;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      st4(Ad + w3f_idx(p, ch * 4), (dvalid >> k) & 1 ? rd[k] : z);  // pixels past the grid add nothing
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int u = tid + k * NT;
      if (u < UB) {
        const int hp = u >> 4, ch = u & 15;
        float4 v = rx[k];
        if (xtf) v = affine_relu4(v, ld4(ssc + ch * 4), ld4(ssc + BC + ch * 4));
        st4(Bx + w3f_idx(hp, ch * 4), v);
      }
    }
  };

  floatx16 acc[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  const int h = lane >> 5, li = lane & 31;
  const int ct = wave & 1, it_ = (wave >> 1) & 1, tap0 = (wave >> 2) * NTAP;
  const int ntap = wave >> 2 ? 9 - NTAP : NTAP;  // wave-uniform
  const int ca = ct * 32 + li, cbb = it_ * 32 + li;
  auto compute = [&] {
#pragma unroll 4
    for (int ks = 0; ks < PT / 2; ++ks) {
      const int p = 2 * ks + h;  // this lane's pixel (k)
      const int prow = p / TW, px = p % TW;
      const float a = Ad[w3f_idx(p, ca)];
#pragma unroll
      for (int j = 0; j < NTAP; ++j) {
        if (j < ntap) {
          const int tap = tap0 + j;
          const int hb = (prow + tap / 3) * HW2 + px + tap % 3;
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bx[w3f_idx(hb, cbb)], acc[j], 0, 0, 0);
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
    if (more) issue(t + gridDim.z);
    compute();
    __syncthreads();
    if (more) {
      commit();
      __syncthreads();
    }
  }
  // accumulate into out[co][tap * Ci + ci] (fp32 atomics, one per element per workgroup)
#pragma unroll
  for (int j = 0; j < NTAP; ++j) {
    if (j < ntap) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = (tap0 + j) * Ci + cb + it_ * 32 + li;
        atomicAdd(args.out + (size_t)row * args.No + col, acc[j][r]);
      }
    }
  }
}

static bool wgrad3_f32_fits(const WgradArgs& a) {
  const Gather& g = a.gb;
  return !a.bf16 && g.taps_h == 3 && g.taps_w == 3 && g.stride == 1 && a.No == 9 * g.Cg && a.Mo % 64 == 0 &&
         g.Cg % 64 == 0 && (g.c_split % 64 == 0 || g.c_split >= g.Cg) && a.ga.Cg == a.Mo && a.ga.taps_h == 1 &&
         a.ga.taps_w == 1 && g.Hg == a.ga.Hg && g.Wg == a.ga.Wg && g.nimg == a.ga.nimg && a.ga.s[0].h16 == 0 &&
         g.s[0].h16 == 0 && g.s[1].h16 == 0;
}

template <int TH, int TW>
static hipError_t go_wgrad3_f32(const WgradArgs& a, hipStream_t s, int per_cu) {
  constexpr size_t smem = wgrad3_f32_smem<TH, TW>();
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wgrad3_f32<TH, TW>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int tiles = a.gb.nimg * ((a.gb.Hg + TH - 1) / TH) * ((a.gb.Wg + TW - 1) / TW);
  const int blocks = (a.Mo / 64) * (a.gb.Cg / 64);
  int splits = (per_cu * num_cus() + blocks - 1) / blocks;
  splits = splits < 1 ? 1 : (splits > tiles ? tiles : splits);
  dim3 grid(a.Mo / 64, a.gb.Cg / 64, splits);
  hipLaunchKernelGGL((k_wgrad3_f32<TH, TW>), grid, dim3(512), smem, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_splitk_epi: out = sum_z slab[z] + the k_igemm epilogue (bias, pixel-shuffle
// or cropped destination, ReLU-mask + BN-bwd stats, BN stats, concat colsum).
// 256 threads = 16 column quads x 16 row lanes over a 128-row x 64-column
// block; every Dst channel count, n_split and shuffle_co is a multiple of 4, so
// a column quad maps to 4 contiguous destination floats.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_splitk_epi(const IgemmArgs args) {
  const int tid = threadIdx.x, cq = tid & 15, rl = tid >> 4;
  const int col = blockIdx.y * 64 + cq * 4;
  const int mbeg = blockIdx.x * 128, mend = min(args.M, mbeg + 128);
  const Epilogue& e = args.e;
  const Gather& g = args.a;
  const int M = args.M, N = args.N, HWg = g.Hg * g.Wg;
  const bool second = col >= e.n_split;
  const Dst& d = second ? e.d[1] : e.d[0];
  const int dcol = second ? col - e.n_split : col;
  float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e.bias) bias = ld4(e.bias + (e.shuffle_co ? col % e.shuffle_co : col));
  const bool bwd_mask = (e.yref != nullptr) && !second;
  float4 bsc = bias, bsh = bias, bmu = bias, bis = bias;
  if (bwd_mask) {
    bsc = ld4(e.bn_scale + col);
    bsh = ld4(e.bn_shift + col);
    bmu = ld4(e.bn_mean + col);
    bis = ld4(e.bn_invstd + col);
  }
  const bool linear = !e.shuffle_co && d.oy == 0 && d.ox == 0 && d.H == g.Hg && d.W == g.Wg;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  for (int m = mbeg + rl; m < mend; m += 16) {
    float4 v = bias;
    for (int z = 0; z < args.ksplit; ++z) {
      const float4 p = ld4(args.slab + ((size_t)z * M + m) * N + col);
      v.x += p.x;
      v.y += p.y;
      v.z += p.z;
      v.w += p.w;
    }
    size_t idx;
    if (linear) {
      idx = (size_t)m * d.C + dcol;
    } else {
      const int n = m / HWg, rr = m - n * HWg;
      const int y = rr / g.Wg, x = rr - y * g.Wg;
      if (e.shuffle_co) {
        const int ab = dcol / e.shuffle_co, co = dcol - ab * e.shuffle_co;
        idx = ((size_t)(n * d.H + 2 * y + (ab >> 1) + d.oy) * d.W + 2 * x + (ab & 1) + d.ox) * d.C + co;
      } else {
        idx = ((size_t)(n * d.H + y + d.oy) * d.W + x + d.ox) * d.C + dcol;
      }
    }
    float vv[4] = {v.x, v.y, v.z, v.w};
    if (d.h16 && (e.stats || bwd_mask)) {  // bf16-stored output: statistics of the rounded values
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = round_bf(vv[q]);
    }
    if (bwd_mask) {
      const float4 y4 = e.yref_h16 ? bf16x4_to_f4(*reinterpret_cast<const uint2*>(
                                         reinterpret_cast<const uint16_t*>(e.yref) + idx))
                                   : ld4(e.yref + idx);
      const float yv[4] = {y4.x, y4.y, y4.z, y4.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float sc = getc(bsc, q), sh = getc(bsh, q), mu = getc(bmu, q), is = getc(bis, q);
        vv[q] = (fmaf(yv[q], sc, sh) > 0.f) ? vv[q] : 0.f;
        s1[q] += vv[q];
        s2[q] += vv[q] * ((yv[q] - mu) * is);
      }
    } else if (e.stats || (second && e.colsum1)) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s1[q] += vv[q];
        s2[q] += vv[q] * vv[q];
      }
    }
    if (e.relu) {
#pragma unroll
      for (int q = 0; q < 4; ++q) vv[q] = fmaxf(vv[q], 0.f);
    }
    if (d.h16)
      *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(d.ptr) + idx) =
          make_uint2(bf16pack(vv[0], vv[1]), bf16pack(vv[2], vv[3]));
    else
      st4(d.ptr + idx, make_float4(vv[0], vv[1], vv[2], vv[3]));
  }
  const bool want = (e.stats != nullptr) || (e.yref != nullptr) || (e.colsum1 != nullptr);
  if (!want) return;
  __shared__ float red[2][16][65];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red[0][rl][cq * 4 + q] = s1[q];
    red[1][rl][cq * 4 + q] = s2[q];
  }
  __syncthreads();
  if (tid < 64) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      a += red[0][r][tid];
      b += red[1][r][tid];
    }
    const int c = blockIdx.y * 64 + tid;
    const int grp = blockIdx.x % kStatGroups;
    const int nsplit = min(e.n_split, N);
    if (c < nsplit) {
      double* st = e.yref ? e.bstats : e.stats;
      if (st) {
        atomicAdd(st + ((size_t)grp * nsplit + c) * 2 + 0, (double)a);
        atomicAdd(st + ((size_t)grp * nsplit + c) * 2 + 1, (double)b);
      }
    } else if (e.colsum1) {
      atomicAdd(e.colsum1 + (size_t)grp * (N - nsplit) + (c - nsplit), (double)a);
    }
  }
}

// ---------------------------------------------------------------------------
// k_wgrad: C[i][j] = sum_p A_p[i] * B_p[j], p = pixels (split over blockIdx.z).
// LDS tiles are [16 pixels][BM] and [16 pixels][BN] (channel contiguous).
// Each thread owns fixed columns (channel slice of A; (tap, channel) of B) and
// walks its staged pixel rows incrementally (no divisions in the loop).
// ---------------------------------------------------------------------------

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256, 2) void k_wgrad(const WgradArgs args) {
  constexpr int BK = 16;
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  constexpr int AR = BM / 4, BR = BN / 4;            // float4 per staged pixel row
  constexpr int ASTEP = 256 / AR, BSTEP = 256 / BR;  // rows covered per pass
  constexpr int AP = (BK + ASTEP - 1) / ASTEP, BP = (BK + BSTEP - 1) / BSTEP;
  static_assert(AR <= 256 && BR <= 256, "tile widths");
  __shared__ __attribute__((aligned(16))) float lds[2 * BK * (BM + BN)];
  // threads beyond the last full pass of a row group stage nothing (BN = 192: 240 of 256)
  const bool aact = threadIdx.x < ASTEP * AR, bact = threadIdx.x < BSTEP * BR;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  int bx, by, bz;  // XCD-aware grid order: an XCD's run shares a pixel split's panels in its L2
  xcd_block(bx, by, bz);
  const int i0 = bx * BM, j0 = by * BN;
  const int nz = gridDim.z / args.batch;  // pixel splits per batch entry
  const int zb = bz / nz;
  const int pbeg = (bz - zb * nz) * args.pix_per_split;
  const int pend = min(args.P, pbeg + args.pix_per_split);
  const Gather& ga = args.ga;
  const Gather& gb = args.gb;

  // A: fixed channel slice of the (single) source of ga.
  const int acol4 = tid % AR, arow = tid / AR;
  const int ac = i0 + acol4 * 4;
  const Src& as = ga.s[0];
  const float* const aptr = as.ptr + zb * args.batch_a;
  // B: fixed (tap, channel) per thread.
  const int bcol4 = tid % BR, brow = tid / BR;
  const int bj = j0 + bcol4 * 4;
  const int btap = bj / gb.Cg;
  const int bc0 = bj - btap * gb.Cg;
  const bool bsecond = bc0 >= gb.c_split;
  const Src& bs = bsecond ? gb.s[1] : gb.s[0];
  const int bc = bsecond ? bc0 - gb.c_split : bc0;
  const int bty = btap / gb.taps_w, btx = btap - bty * gb.taps_w;
  const float* const bptr = bs.ptr + zb * args.batch_b;

  float4 asc = make_float4(0, 0, 0, 0), ash = asc, bsc = asc, bsh = asc;
  if (as.scale) { asc = ld4(as.scale + ac); ash = ld4(as.shift + ac); }
  if (bs.scale) { bsc = ld4(bs.scale + bc); bsh = ld4(bs.shift + bc); }

  PixIt ait[AP], bit[BP];
  bool ain[AP], bin[BP];
#pragma unroll
  for (int q = 0; q < AP; ++q) ait[q].init(min(pbeg + arow + ASTEP * q, args.P - 1), ga.Hg, ga.Wg);
#pragma unroll
  for (int q = 0; q < BP; ++q) bit[q].init(min(pbeg + brow + BSTEP * q, args.P - 1), gb.Hg, gb.Wg);

  float4 ra[AP], rb[BP];
  auto issue = [&](int p0) {
#pragma unroll
    for (int q = 0; q < AP; ++q) {
      const int p = p0 + arow + ASTEP * q;
      ain[q] = p < pend && (arow + ASTEP * q) < BK;
      const int pix = (ait[q].n * as.H + ait[q].y * ga.stride + as.oy) * as.W + ait[q].x * ga.stride + as.ox;
      ra[q] = ld4(aptr + (size_t)pix * as.C + ac);
      if (p + BK < pend) ait[q].advance(BK, ga.Hg, ga.Wg);
    }
#pragma unroll
    for (int q = 0; q < BP; ++q) {
      const int p = p0 + brow + BSTEP * q;
      bin[q] = p < pend && (brow + BSTEP * q) < BK;
      const int pix = (bit[q].n * bs.H + bit[q].y * gb.stride + bty + bs.oy) * bs.W + bit[q].x * gb.stride + btx +
                      bs.ox;
      rb[q] = ld4(bptr + (size_t)pix * bs.C + bc);
      if (p + BK < pend) bit[q].advance(BK, gb.Hg, gb.Wg);
    }
  };
  auto commit = [&](int buf) {
    float* As = lds + buf * BK * (BM + BN);
    float* Bs = As + BK * BM;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < AP; ++q) {
      float4 v = as.scale ? affine_relu4(ra[q], asc, ash) : ra[q];
      if (aact && arow + ASTEP * q < BK) st4(As + (arow + ASTEP * q) * BM + acol4 * 4, ain[q] ? v : z);
    }
#pragma unroll
    for (int q = 0; q < BP; ++q) {
      float4 v = bs.scale ? affine_relu4(rb[q], bsc, bsh) : rb[q];
      if (bact && brow + BSTEP * q < BK) st4(Bs + (brow + BSTEP * q) * BN + bcol4 * 4, bin[q] ? v : z);
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
  const int nk = (pend - pbeg + BK - 1) / BK;
  if (nk <= 0) return;
  issue(pbeg);
  commit(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    const bool more = kc + 1 < nk;
    if (more) issue(pbeg + (kc + 1) * BK);
    const float* As = lds + cur * BK * (BM + BN);
    const float* Bs = As + BK * BM;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[(h * 8 + s) * BM + wm * TM * 32 + i * 32 + li];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[(h * 8 + s) * BN + wn * TN * 32 + j * 32 + li];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) commit(cur ^ 1);
    __syncthreads();
  }
  // accumulate the tile into out (fp32 atomics; the output is small next to the
  // reduction), or (slab mode, batch 1) store this split's partial for
  // launch_slab_reduce
  float* const plane = args.slab ? args.slab + (size_t)bz * args.Mo * args.No : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = j0 + wn * TN * 32 + j * 32 + li;
        if (plane) plane[(size_t)row * args.No + col] = acc[i][j][r];
        else atomicAdd(args.out + zb * args.batch_out + (size_t)row * args.No + col, acc[i][j][r]);
      }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static int g_num_cus = 0;
int num_cus() {
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                hipSuccess && n > 0)
      g_num_cus = n;
    else
      g_num_cus = 256;
  }
  return g_num_cus;
}

int ablation_env(const char* name) {
  const char* v = getenv(name);
  if (!v || !*v) return 0;
#ifdef UNET_ABLATIONS
  return atoi(v);
#else
  fprintf(stderr, "unet_hip: %s=%s ignored (timing ablations need a build with -DUNET_ABLATIONS: make ABLATIONS=1)\n",
          name, v);
  return 0;
#endif
}

static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
}
// unet_set_tuning("igemm_variant", v) or UNET_IGEMM_VARIANT; -1 = heuristic
int g_tune_igemm = env_int("UNET_IGEMM_VARIANT", -1);
int g_tune_wgrad = env_int("UNET_WGRAD_VARIANT", -1);
std::atomic<long long> g_slab_fallbacks{0};
// unet_set_tuning("wino_max", m) or UNET_WINO_MAX: largest Winograd output tile
// the fp32 forward / input-gradient candidates may use (6 = F(6x6) and below,
// 4 = up to F(4x4), 2, 0 = none); "wino_wgrad_max" / UNET_WINO_WGRAD_MAX the
// same for the weight gradients.  F(6x6)'s rounding (~2.5x F(4x4)'s) feeds the
// BatchNorm-normalised dX chain in forward / input gradients and moved small
// (188-198 px) whole-step parity past its tolerances, so those default to
// F(4x4); a weight gradient's rounding stays in that one tensor.
int g_wino_max = env_int("UNET_WINO_MAX", 4);
int g_wino_dgrad_max = env_int("UNET_WINO_DGRAD_MAX", 4);  // input gradients (no forward BN statistics)
int g_wino_wgrad_max = env_int("UNET_WINO_WGRAD_MAX", 6);
// "wino4_fwd_min_cg" / UNET_WINO4_FWD_MIN_CG: forward (BN-statistics) GEMMs use
// F(4x4) only from this many input channels on.  The forward's rounding feeds
// the BatchNorm statistics and from there every gradient.  With Lavin's points
// F(4x4) on every forward put the 512^2 every-element gradient check at
// 1.00-1.07 % of its 1 % bar (direct GEMMs: 0.72 %), >= 128 channels 1.03 %,
// >= 256 0.81 %.  With the better-conditioned points (winograd.hip, round 3):
// every forward 0.97-0.98 (and the 3-step SGD trajectory at 1.02 % in one of two
// tunings), >= 128 channels 0.85 -- the default (profiles/r03_wino_fwd_sweep.txt;
// fp32 bench 301 / 292 / 278 img/s for 0 / 128 / 256)
int g_wino4_fwd_min_cg = env_int("UNET_WINO4_FWD_MIN_CG", 128);
// ... and also up to this many ("wino4_fwd_small_cg" / UNET_WINO4_FWD_SMALL_CG)
int g_wino4_fwd_small_cg = env_int("UNET_WINO4_FWD_SMALL_CG", 0);
static int wino_tile_m(int tile) {
  return tile == 70 || tile == 75 || tile == 77 ? 2 : tile == 71 || tile == 72 || tile == 73 || tile == 76 ? 4 : tile == 74 ? 6 : 0;
}

// igemm tile table: id -> (BM, BN, waves M x N, BK), resident workgroups per CU
// (min of the LDS and VGPR limits of the built kernels).
struct TileInfo {
  int bm, bn, bk, slots;
};
static TileInfo tile_info(int id) {
  switch (id) {
    case 1: return {128, 128, 16, 3};
    case 2: return {64, 128, 16, 4};
    case 3: return {128, 128, 32, 2};
    case 4: return {256, 128, 16, 2};
    case 6: return {256, 64, 16, 2};
    case 7: return {256, 64, 32, 1};
    case 8: return {128, 64, 16, 4};
    case 9: return {64, 128, 32, 2};
    // LDS-DMA staged (k_igemm_g)
    case 11: return {256, 128, 16, 2};
    case 12: return {128, 128, 16, 3};
    case 13: return {64, 128, 16, 4};
    case 14: return {128, 64, 16, 4};
    // bf16 operands, register staged (k_igemm_bf, igemm_bf16.hip)
    case 21: return {256, 128, 32, 2};
    case 22: return {128, 128, 32, 3};
    case 23: return {128, 64, 32, 4};
    case 24: return {64, 128, 32, 4};
    case 25: return {256, 64, 32, 2};
    case 26: return {128, 256, 32, 2};
    // bf16 halo-tiled 3x3 (k_conv3_bf): bm = pixels per tile, bk = one
    // 32-channel chunk x 9 taps (the split-K unit)
    case 31: return {256, 64, 288, 2};
    case 32: return {256, 64, 288, 2};
    case 33: return {256, 64, 288, 2};
    case 34: return {128, 128, 288, 1};
    case 35: return {128, 64, 288, 2};
    case 36: return {256, 128, 288, 1};
    case 41: case 42: case 43: case 44: return {256, 64, 288, 1};  // persistent k_conv3p_bf
    // bf16 halo-tiled 3x3 with LDS-DMA weights and a 2-stage ring (k_conv3_dma,
    // conv3_dma.hip): bk = one channel chunk (16 or 32) x 9 taps
    case 63: return {256, 64, 144, 2};
    case 65: return {512, 64, 144, 1};
    case 66: return {512, 64, 288, 1};
    case 67: return {256, 64, 144, 2};
    case 68: return {256, 128, 144, 1};
    // bf16 3x3 with LDS-DMA halo and weight rings (k_conv3_ring, conv3_ring.hip):
    // bk = one 64- or 32-channel chunk x 9 taps (the split-K unit)
    case 81: return {256, 128, 576, 1};
    case 82: return {256, 64, 288, 2};
    case 83: return {128, 128, 288, 3};
    case 84: return {256, 64, 576, 1};
    // the ring on flat tiles of 256 consecutive pixels (k_conv3_flat, conv3_flat.hip)
    case 85: return {256, 128, 576, 1};
    // 85 stream-K: one workgroup per CU, equal runs of (tile, column block, chunk) units
    case 86: return {256, 128, 576, 1};
    // 64 -> 64 channels with the weights resident in LDS (k_conv3_c64, conv3_c64.hip): persistent
    case 87: return {256, 64, 576, 1};
    // 84 persistent (k_conv3_ring PT): whole K per workgroup
    case 88: return {256, 64, 576, 1};
    // bf16 convT forward / input gradient on LDS-DMA K rings (k_gemm_ring,
    // gemm_ring.hip): 64-k stages
    case 91: return {128, 128, 64, 1};
    case 92: return {256, 128, 64, 1};
    case 93: return {128, 256, 64, 1};
    case 94: return {128, 128, 64, 1};
    case 95: return {64, 128, 64, 1};
    case 96: return {256, 256, 32, 1};
    case 97: return {256, 128, 32, 1};
    case 98: return {128, 256, 32, 1};
    case 99: return {128, 128, 32, 1};
    // Winograd F(2x2, 3x3) (winograd.hip): no K split
    case 70: case 71: case 74: return {256, 64, 9, 2};
    case 72: return {32, 32, 16, 1};
    case 73: case 76: return {32, 64, 8, 1};
    case 75: return {64, 64, 8, 1};
    case 77: return {64, 32, 8, 2};
    // fp32 halo-tiled 3x3 (k_conv3_f32): bk = one 16-channel chunk x 9 taps
    case 51: return {256, 64, 144, 2};
    case 52: return {256, 64, 144, 2};
    case 53: return {256, 64, 144, 2};
    case 54: return {128, 64, 144, 2};
    default: return {0, 0, 0, 0};
  }
}

static bool is_halo_tile(int tile) { return (tile >= 31 && tile <= 36) || (tile >= 41 && tile <= 44); }
static bool is_dma_tile(int tile) { return tile == 63 || (tile >= 65 && tile <= 68); }
static bool is_ring_tile(int tile) { return (tile >= 81 && tile <= 84) || tile == 88; }
static bool is_gemm_ring_tile(int tile) { return tile >= 91 && tile <= 99; }
static bool is_bf16_tile(int tile) {
  return (tile >= 21 && tile <= 26) || is_halo_tile(tile) || is_dma_tile(tile) || is_ring_tile(tile) || tile == 85 || tile == 86 || tile == 87 ||
         is_gemm_ring_tile(tile);
}
static bool is_halo32_tile(int tile) { return tile >= 51 && tile <= 54; }

// A tile applies when the shape divides and the packed B operand is in the
// tile's precision (fp32 `b` for tiles 1-14, bf16 `bh` for 21-26).
bool igemm_tile_fits(const IgemmArgs& a, int tile) {
  // every 3x3 forward conv feeds a BatchNorm (stats); the input gradients do
  // not.  An eval forward is held to the forward caps too, so eval logits see
  // the same arithmetic as the training forward's parity checks;
  // run_forward marks every 3x3 forward conv explicitly (IgemmArgs::fwd,
  // ADVICE r04) rather than the caps being inferred from the epilogue
  const bool fwd = a.fwd != 0;
  if (wino_tile_m(tile) > (fwd ? g_wino_max : g_wino_dgrad_max)) return false;
  if (fwd && wino_tile_m(tile) >= 4 && a.a.Cg < g_wino4_fwd_min_cg && a.a.Cg > g_wino4_fwd_small_cg)
    return false;
  const TileInfo t = tile_info(tile);
  const bool prec_ok = is_bf16_tile(tile) ? a.bh != nullptr && (a.bl == nullptr || bf16_tile_splits(tile))
                                           : a.b != nullptr;
  if (is_halo_tile(tile))  // 3x3 stride-1 gathers only (conv fwd / dgrad), K = 9 x Cg
    return prec_ok && a.N % t.bn == 0 && a.a.taps_h == 3 && a.a.taps_w == 3 && a.a.stride == 1 &&
           a.K == 9 * a.a.Cg && a.a.Cg % 32 == 0 && a.a.c_split % 32 == 0 && a.a.Cg <= 1024;
  if (is_ring_tile(tile)) return conv3_ring_fits(a, tile);
  if (tile == 85 || tile == 86) return conv3_flat_fits(a, tile);
  if (tile == 87) return conv3_c64_fits(a);
  if (is_gemm_ring_tile(tile)) return gemm_ring_fits(a, tile);
  if (tile == 70 || tile == 71 || tile == 74) return wino_applies(a, tile == 70 ? 2 : tile == 71 ? 4 : 6);
  if (tile == 72) return wino_fused_applies(a);
  if (tile == 73) return wino_fused64_applies(a);
  if (tile == 76) return wino_fused64p_applies(a);
  if (tile == 75) return wino_fused2_applies(a, 64);
  if (tile == 77) return wino_fused2_applies(a, 32);
  if (is_dma_tile(tile)) {  // bf16-stored A sources, no split operands
    const int ch = tile_info(tile).bk / 9;
    const bool two = a.a.c_split < a.a.Cg;
    return a.bh != nullptr && a.bl == nullptr && a.N % t.bn == 0 && a.a.taps_h == 3 && a.a.taps_w == 3 &&
           a.a.stride == 1 && a.K == 9 * a.a.Cg && a.a.Cg % ch == 0 && a.a.c_split % ch == 0 && a.a.Cg <= 1024 &&
           a.a.s[0].h16 && (!two || a.a.s[1].h16);
  }
  if (is_halo32_tile(tile))
    return prec_ok && a.N % t.bn == 0 && a.a.taps_h == 3 && a.a.taps_w == 3 && a.a.stride == 1 &&
           a.K == 9 * a.a.Cg && a.a.Cg % 16 == 0 && a.a.c_split % 16 == 0;
  return t.bm > 0 && prec_ok && a.N % t.bn == 0 && a.K % t.bk == 0 && a.a.Cg % t.bk == 0 &&
         a.a.c_split % t.bk == 0;
}
long long igemm_tile_count(const IgemmArgs& a, int tile) {
  const TileInfo t = tile_info(tile);
  if (t.bm == 0) return 0;
  int th, tw, bn, ch;
  if (tile == 85 || tile == 86) return conv3_flat_tiles(a, tile);
  if (tile == 87) return conv3_c64_tiles(a);
  if (halo_tile_shape(tile, th, tw, bn))
    return (long long)a.a.nimg * ((a.a.Hg + th - 1) / th) * ((a.a.Wg + tw - 1) / tw) * (a.N / bn);
  if (conv3_dma_tile_shape(tile, th, bn, ch) || conv3_ring_tile_shape(tile, th, bn, ch))
    return (long long)a.a.nimg * ((a.a.Hg + th - 1) / th) * ((a.a.Wg + 31) / 32) * (a.N / bn);
  return (long long)((a.M + t.bm - 1) / t.bm) * (a.N / t.bn);
}
int igemm_tile_slots(int tile) { return tile_info(tile).slots; }
size_t igemm_slab_bytes(const IgemmArgs& a, int ksplit) {
  return ksplit > 1 ? (size_t)ksplit * a.M * a.N * sizeof(float) : 0;
}

template <int BM, int BN, int WM, int WN, int BK>
static hipError_t go_igemm(const IgemmArgs& a, hipStream_t s) {
  if (a.N % BN != 0 || a.K % BK != 0 || a.a.Cg % BK != 0 || a.a.c_split % BK != 0) return hipErrorInvalidValue;
  if (a.batch > 1) {
    if (a.ksplit > 1 || a.batch_rows < 1) return hipErrorInvalidValue;
    dim3 grid((a.batch_rows + BM - 1) / BM, a.N / BN, a.batch);
    hipLaunchKernelGGL((k_igemm<BM, BN, WM, WN, BK>), grid, dim3(WM * WN * 64), 0, s, a);
    return hipGetLastError();
  }
  dim3 grid((a.M + BM - 1) / BM, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  hipLaunchKernelGGL((k_igemm<BM, BN, WM, WN, BK>), grid, dim3(WM * WN * 64), 0, s, a);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN>
static hipError_t go_igemm_g(const IgemmArgs& a, hipStream_t s) {
  if (a.N % BN != 0 || a.K % 16 != 0 || a.a.Cg % 16 != 0 || a.a.c_split % 16 != 0) return hipErrorInvalidValue;
  static bool attr = false;
  const size_t full = igemm_g_smem<BM, BN>(1024);
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_igemm_g<BM, BN, WM, WN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)full);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const bool tf = a.a.s[0].scale != nullptr || (a.a.c_split < a.a.Cg && a.a.s[1].scale != nullptr);
  if (tf && a.a.Cg > 1024) return hipErrorInvalidValue;
  const size_t smem = igemm_g_smem<BM, BN>(tf ? a.a.Cg : 0);
  dim3 grid((a.M + BM - 1) / BM, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  hipLaunchKernelGGL((k_igemm_g<BM, BN, WM, WN>), grid, dim3(WM * WN * 64), smem, s, a);
  return hipGetLastError();
}

template <int TH, int TW, int BN, int WM, int WN, int MINW>
static hipError_t go_halo32(const IgemmArgs& a, hipStream_t s) {
  if (a.b == nullptr || a.N % BN != 0 || a.a.Cg % 16 != 0 || a.a.c_split % 16 != 0 || a.a.taps_h != 3 ||
      a.a.taps_w != 3 || a.a.stride != 1 || a.K != 9 * a.a.Cg)
    return hipErrorInvalidValue;
  constexpr size_t smem = conv3_f32_smem<TH, TW, BN>();
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv3_f32<TH, TW, BN, WM, WN, MINW>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const long long tiles = (long long)a.a.nimg * ((a.a.Hg + TH - 1) / TH) * ((a.a.Wg + TW - 1) / TW);
  dim3 grid((unsigned)tiles, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  hipLaunchKernelGGL((k_conv3_f32<TH, TW, BN, WM, WN, MINW>), grid, dim3(WM * WN * 64), smem, s, a);
  return hipGetLastError();
}

static hipError_t go_tile(const IgemmArgs& a, hipStream_t s, int tile) {
  switch (tile) {
    case 1: return go_igemm<128, 128, 2, 2, 16>(a, s);
    case 2: return go_igemm<64, 128, 2, 2, 16>(a, s);
    case 3: return go_igemm<128, 128, 2, 2, 32>(a, s);
    case 4: return go_igemm<256, 128, 4, 2, 16>(a, s);
    case 6: return go_igemm<256, 64, 4, 1, 16>(a, s);
    case 7: return go_igemm<256, 64, 4, 1, 32>(a, s);
    case 8: return go_igemm<128, 64, 2, 2, 16>(a, s);
    case 9: return go_igemm<64, 128, 2, 2, 32>(a, s);
    case 11: return go_igemm_g<256, 128, 4, 2>(a, s);
    case 12: return go_igemm_g<128, 128, 2, 2>(a, s);
    case 13: return go_igemm_g<64, 128, 2, 2>(a, s);
    case 14: return go_igemm_g<128, 64, 2, 2>(a, s);
    case 21: case 22: case 23: case 24: case 25: case 26:
    case 31: case 32: case 33: case 34: case 35: case 36:
    case 41: case 42: case 43: case 44: return go_igemm_bf16(a, s, tile);
    case 63: case 65: case 66: case 67: case 68: return go_conv3_dma_tile(a, s, tile);
    case 81: case 82: case 83: case 84: case 88: return go_conv3_ring_tile(a, s, tile);
    case 85: case 86: return go_conv3_flat_tile(a, s, tile);
    case 87: return go_conv3_c64(a, s);
    case 91: case 92: case 93: case 94: case 95: case 96: case 97: case 98: case 99:
      return go_gemm_ring_tile(a, s, tile);
    case 70: return launch_wino(a, s, 2);
    case 71: return launch_wino(a, s, 4);
    case 74: return launch_wino(a, s, 6);
    case 72: return launch_wino_fused(a, s);
    case 73: return launch_wino_fused64(a, s);
    case 76: return launch_wino_fused64p(a, s);
    case 75: return launch_wino_fused2(a, s, 64);
    case 77: return launch_wino_fused2(a, s, 32);
    case 51: return go_halo32<8, 32, 64, 8, 1, 4>(a, s);
    case 52: return go_halo32<16, 16, 64, 8, 1, 4>(a, s);
    case 53: return go_halo32<8, 32, 64, 4, 1, 2>(a, s);
    case 54: return go_halo32<8, 16, 64, 4, 1, 2>(a, s);
    default: return hipErrorInvalidValue;
  }
}

static bool igemm_args_ok(const IgemmArgs& a) {
  return a.M > 0 && a.N > 0 && a.K > 0 && (a.K % 16) == 0 && (a.a.Cg % 16) == 0 && (a.a.c_split % 16) == 0;
}

// Built-in tile choice (used when no tuned choice exists), measured per U-Net
// layer shape on MI355X (profiles/r01_tuning.txt):
//  N = 64 (Co or Ci = 64): 128x64, 5 waves/SIMD            (+19 % on inc.c1 dgrad)
//  N >= 256, >= 1.5 x CUs 256x128 tiles: 8-wave 256x128    (+5..10 % on down1-3, up2)
//  N = 128 with large M: 128x128
//  otherwise (bottleneck, M <= ~20k pixels): 64x128 to fill the CUs
static int heuristic_tile(const IgemmArgs& a) {
  if (g_tune_igemm > 0 && igemm_tile_fits(a, g_tune_igemm)) return g_tune_igemm;
  const long long cus = num_cus();
  if (a.bh != nullptr) {  // bf16 operands: same shape rules over the bf16 tiles
    if (a.K % 32 || a.a.Cg % 32 || a.a.c_split % 32) return -1;
    if (a.N % 128 == 0) {
      const long long t256 = ((a.M + 255) / 256) * (long long)(a.N / 128);
      const long long t128 = ((a.M + 127) / 128) * (long long)(a.N / 128);
      if (a.N >= 256 && t256 >= 3 * cus / 2) return 21;
      if (t128 >= 2 * cus) return 22;
      return 24;
    }
    return a.N % 64 == 0 ? 23 : -1;
  }
  if (a.N % 128 == 0) {
    const long long t256 = ((a.M + 255) / 256) * (long long)(a.N / 128);
    const long long t128 = ((a.M + 127) / 128) * (long long)(a.N / 128);
    if (a.N >= 256 && t256 >= 3 * cus / 2) return 4;
    if (t128 >= 4 * cus) return 1;
    return 2;
  }
  if (a.N % 64 == 0) return 8;
  return -1;
}

hipError_t launch_igemm(const IgemmArgs& a0, hipStream_t s) {
  if (!igemm_args_ok(a0)) return hipErrorInvalidValue;
  IgemmArgs a = a0;
  a.ksplit = 1;
  return go_tile(a, s, heuristic_tile(a));
}

hipError_t launch_igemm_v(const IgemmArgs& a0, hipStream_t s, GemmChoice c) {
  if (c.tile < 0) return launch_igemm(a0, s);
  if (!igemm_args_ok(a0) || !igemm_tile_fits(a0, c.tile)) return hipErrorInvalidValue;
  IgemmArgs a = a0;
  const int nk = a.K / tile_info(c.tile).bk;
  const bool wino = c.tile >= 70 && c.tile <= 77;
  if ((c.tile == 70 || c.tile == 71 || c.tile == 74) && c.split >= 100) a.wino_choice.tile = c.split - 100;  // point GEMMs
  int ks = c.split < 1 || wino ? 1 : (c.split > nk ? nk : c.split);
  if (ks > 1) {  // no empty slice: ks = ceil(nk / ceil(nk / ks))
    const int per = (nk + ks - 1) / ks;
    ks = (nk + per - 1) / per;
  }
  a.ksplit = ks;
  if (ks > 1 && (a.slab == nullptr || a.N % 64 != 0)) return hipErrorInvalidValue;
  hipError_t e = go_tile(a, s, c.tile);
  if (e != hipSuccess || ks == 1) return e;
  dim3 grid((a.M + 127) / 128, a.N / 64);
  hipLaunchKernelGGL(k_splitk_epi, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// wgrad tile table: id -> (BM, BN); 0-4 fp32 (k_wgrad), 10-14 bf16 (k_wgrad_bf)
static void wgrad_tile(int id, int& bm, int& bn) {
  static const int t[5][2] = {{128, 128}, {128, 192}, {64, 192}, {64, 128}, {64, 64}};
  static const int tb[5][2] = {{128, 128}, {128, 192}, {64, 128}, {64, 64}, {256, 128}};
  bm = bn = 0;
  if (id >= 0 && id < 5) { bm = t[id][0]; bn = t[id][1]; }
  if (id >= 10 && id < 15) { bm = tb[id - 10][0]; bn = tb[id - 10][1]; }
}
bool wgrad_tile_fits(const WgradArgs& a, int tile) {
  if (wino_tile_m(tile) > g_wino_wgrad_max) return false;
  // the Winograd weight gradients assign G^T Mw G to out: no accumulation
  if (tile == 71 || tile == 74) return !a.accumulate && wino_wgrad_applies(a, tile == 71 ? 4 : 6);
  if (a.batch > 1 && (tile < 0 || tile > 4)) return false;  // batched: fp32 pixel-column tiles only
  if (tile == 20 || tile == 21) return wgrad3_fits(a);  // halo-tiled 3x3, all taps
  if (tile == 22 || tile == 23) return wgrad3_f32_fits(a);  // fp32 twin
  if (tile == 24 || tile == 25) return wgrad3w_fits(a, tile);  // wide halo-tiled 3x3, two-stage ring
  if (tile >= 26 && tile <= 33) return wgrad3_ring_fits(a, tile);  // LDS-DMA ring of pixel tiles
  if (tile >= 40 && tile <= 44) return wgradT_ring_fits(a, tile);  // convT: LDS-DMA ring of pixel stages
  int bm, bn;
  wgrad_tile(tile, bm, bn);
  return bm > 0 && (tile >= 10) == (a.bf16 != 0) && a.Mo % bm == 0 && a.No % bn == 0;
}

hipError_t launch_wgrad_v(const WgradArgs& a0, hipStream_t s, GemmChoice c) {
  WgradArgs a = a0;
  if (a.Mo % 64 != 0 || a.P <= 0 || a.gb.Cg % 4 != 0 || a.gb.c_split % 4 != 0 || a.ga.Cg % 4 != 0)
    return hipErrorInvalidValue;
  int tile = c.tile;
  if (tile < 0 && a.bf16) {
    if (g_tune_wgrad >= 10 && wgrad_tile_fits(a, g_tune_wgrad)) tile = g_tune_wgrad;  // forced (tests)
    else if (g_tune_wgrad >= 126 && g_tune_wgrad <= 133 && wgrad_tile_fits(a, g_tune_wgrad - 100)) {
      tile = g_tune_wgrad - 100;  // forced ring tile in slab mode (tests)
      c.split = 11;
    } else if (g_tune_wgrad >= 110 && g_tune_wgrad <= 114 && wgrad_tile_fits(a, g_tune_wgrad - 100)) {
      c.tile = tile = g_tune_wgrad - 100;  // forced pixel-column tile in slab mode, 2 per CU (tests)
      c.split = 102;
    } else if (g_tune_wgrad >= 140 && g_tune_wgrad <= 144 && wgrad_tile_fits(a, g_tune_wgrad - 100)) {
      tile = g_tune_wgrad - 100;  // forced convT ring tile in slab mode, 1 per CU (tests)
      c.split = 11;
    }
    else if (wgrad3_fits(a)) tile = 20;
    else if (a.Mo % 128 == 0 && a.No % 128 == 0) tile = 10;
    else if (a.No % 128 == 0) tile = 12;
    else tile = 13;
  } else if (tile < 0) {
    if ((g_tune_wgrad == 22 || g_tune_wgrad == 23 || g_tune_wgrad == 71 || g_tune_wgrad == 74) &&
        wgrad_tile_fits(a, g_tune_wgrad))
      tile = g_tune_wgrad;  // forced fp32 halo tile (tests)
    else if ((g_tune_wgrad == 1071 || g_tune_wgrad == 1074) && wgrad_tile_fits(a, g_tune_wgrad - 1000)) {
      tile = g_tune_wgrad - 1000;  // forced Winograd weight gradient in slab mode (tests; no Mw memset)
      c.split = 1000;
    } else if (g_tune_wgrad >= 100 && g_tune_wgrad <= 104 && wgrad_tile_fits(a, g_tune_wgrad - 100)) {
      c.tile = tile = g_tune_wgrad - 100;  // forced fp32 pixel-column tile in slab mode, 2 per CU (tests)
      c.split = 102;
    } else if (g_tune_wgrad == 1) tile = 4;  // force the small tile (A/B tests)
    else if (a.Mo % 128 == 0 && a.No % 128 == 0) tile = 0;
    else if (a.Mo % 128 == 0 && a.No % 192 == 0) tile = 1;
    else if (a.No % 192 == 0) tile = 2;
    else if (a.No % 128 == 0) tile = 3;
    else tile = 4;
  }
  if (!wgrad_tile_fits(a, tile)) return hipErrorInvalidValue;
  if (tile == 71 || tile == 74) return launch_wino_wgrad(a, s, c.split, tile == 71 ? 4 : 6);
  if (tile == 20 || tile == 21) return go_wgrad3_bf16(a, s, tile, c.split > 0 ? c.split : 4);
  if (tile == 22) return go_wgrad3_f32<8, 16>(a, s, c.split > 0 ? c.split : 4);
  if (tile == 24 || tile == 25) return go_wgrad3w_bf16(a, s, tile, c.split > 0 ? c.split : 1);
  if (tile >= 26 && tile <= 33) return go_wgrad3_ring(a, s, tile, c.split > 0 ? c.split : 1);
  if (tile >= 40 && tile <= 44) return go_wgradT_ring(a, s, tile, c.split > 0 ? c.split : 1);
  if (tile == 23) return go_wgrad3_f32<4, 32>(a, s, c.split > 0 ? c.split : 4);
  int bm, bn;
  wgrad_tile(tile, bm, bn);
  // split the pixel reduction so that the grid has ~`per_cu` workgroups per CU;
  // codes >= 100: slab mode (plain-store split partials + one reduction pass)
  const bool slab_mode = c.tile >= 0 && c.split >= 100;
  if (slab_mode) c.split -= 100;
  const int per_cu = c.tile >= 0 ? (c.split > 0 ? c.split : 8) : (g_tune_wgrad >= 2 ? g_tune_wgrad : 8);
  int pps = 0;
  const int splits = wgrad_splits(a, tile, per_cu, pps);
  a.pix_per_split = pps;
  const size_t plane = (size_t)a.Mo * a.No;
  // slab mode: one split writes its planes straight into out (plain stores),
  // more go through the slab and an assigning reduction; either way every
  // output element is written, so out needs no zeroing
  if (!(slab_mode && wgrad_slab_fits(a, splits))) {
    if (slab_mode) ++g_slab_fallbacks;  // split partials exceed the plan's wslab: atomics instead
    a.slab = nullptr;
  }
  else if (splits == 1) a.slab = a.out;
  dim3 grid(a.Mo / bm, a.No / bn, splits * a.batch);
  hipError_t e = hipSuccess;
  if (tile >= 10) {
    e = go_wgrad_bf16(a, s, tile, grid);
  } else {
    switch (tile) {
      case 0: hipLaunchKernelGGL((k_wgrad<128, 128, 2, 2>), grid, dim3(256), 0, s, a); break;
      case 1: hipLaunchKernelGGL((k_wgrad<128, 192, 2, 2>), grid, dim3(256), 0, s, a); break;
      case 2: hipLaunchKernelGGL((k_wgrad<64, 192, 2, 2>), grid, dim3(256), 0, s, a); break;
      case 3: hipLaunchKernelGGL((k_wgrad<64, 128, 2, 2>), grid, dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL((k_wgrad<64, 64, 2, 2>), grid, dim3(256), 0, s, a); break;
    }
    e = hipGetLastError();
  }
  if (e != hipSuccess || !a.slab || a.slab == a.out) return e;
  return launch_slab_reduce(a.slab, splits, a.batch, plane, a.batch_out, a.out, s);
}

int wgrad_splits(const WgradArgs& a, int tile, int per_cu, int& pps) {
  int bm, bn;
  wgrad_tile(tile, bm, bn);
  const int tiles = (a.Mo / bm) * (a.No / bn) * a.batch;
  const int target = per_cu * num_cus();
  int splits = (target + tiles - 1) / tiles;
  const int max_splits = (a.P + 255) / 256;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  pps = (a.P + splits - 1) / splits;
  const int kq = tile >= 10 ? 32 : 16;  // pixels per K-step
  pps = (pps + kq - 1) / kq * kq;
  return (a.P + pps - 1) / pps;
}

bool wgrad_slab_fits(const WgradArgs& a, int splits) {
  const size_t plane = (size_t)a.Mo * a.No;
  if (!a.slab || a.accumulate || plane % 4 != 0 || (a.batch > 1 && a.batch_out != (long long)plane)) return false;
  return splits == 1 || (size_t)splits * a.batch * plane * sizeof(float) <= a.slab_bytes;
}

hipError_t launch_wgrad(const WgradArgs& a, hipStream_t s) { return launch_wgrad_v(a, s, GemmChoice{}); }

// The Winograd tile (mt = 4 / 6) launch_wgrad_v(a, s, c) runs for an fp32
// launch, 0 if it runs another kernel (the same resolution of forced and
// heuristic tiles as launch_wgrad_v)
int wgrad_winograd_mt(const WgradArgs& a, GemmChoice c) {
  if (a.bf16) return 0;
  int tile = c.tile;
  if (tile < 0) {
    if ((g_tune_wgrad == 71 || g_tune_wgrad == 74) && wgrad_tile_fits(a, g_tune_wgrad)) tile = g_tune_wgrad;
    else if ((g_tune_wgrad == 1071 || g_tune_wgrad == 1074) && wgrad_tile_fits(a, g_tune_wgrad - 1000))
      tile = g_tune_wgrad - 1000;
  }
  if ((tile == 71 || tile == 74) && wgrad_tile_fits(a, tile)) return tile == 71 ? 4 : 6;
  return 0;
}

double igemm_exec_flops(const IgemmArgs& a, GemmChoice c) {
  int t = c.tile;
  if (t < 0 && g_tune_igemm >= 70 && g_tune_igemm <= 77 && igemm_tile_fits(a, g_tune_igemm)) t = g_tune_igemm;
  if (t >= 70 && t <= 77) {
    const int mt = t == 70 || t == 75 || t == 77 ? 2 : t == 74 ? 6 : 4;
    const Gather& g = a.a;
    const double T = (double)g.nimg * ((g.Hg + mt - 1) / mt) * ((g.Wg + mt - 1) / mt);
    return 2.0 * (mt + 2) * (mt + 2) * T * g.Cg * a.N;
  }
  return 2.0 * a.M * (double)a.N * a.K;
}

double wgrad_exec_flops(const WgradArgs& a, GemmChoice c) {
  int t = c.tile;
  if (t < 0 && !a.bf16 && (g_tune_wgrad == 71 || g_tune_wgrad == 74) && wgrad_tile_fits(a, g_tune_wgrad))
    t = g_tune_wgrad;
  if (t < 0 && !a.bf16 && (g_tune_wgrad == 1071 || g_tune_wgrad == 1074) && wgrad_tile_fits(a, g_tune_wgrad - 1000))
    t = g_tune_wgrad - 1000;
  if (t == 71 || t == 74) {
    const int mt = t == 71 ? 4 : 6;
    const double T = (double)a.gb.nimg * ((a.gb.Hg + mt - 1) / mt) * ((a.gb.Wg + mt - 1) / mt);
    return 2.0 * (mt + 2) * (mt + 2) * T * a.Mo * a.gb.Cg;
  }
  return 2.0 * a.P * (double)a.Mo * a.No;
}

}  // namespace unet
