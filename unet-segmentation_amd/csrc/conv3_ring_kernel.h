// conv3_ring_kernel.h -- k_conv3_ring and its launcher template, shared by
// conv3_ring.hip (tiles 81-84) and conv3_ring_pt.hip (the persistent 88:
// a translation unit of their own so the two compile in parallel).
//
// k_conv3_ring: bf16 3x3 stride-1 implicit GEMM (conv forward and conv input
// gradient) with every operand byte staged by LDS-DMA through rings.
//
// Round-2's halo kernels ran at ~28 % MFMA busy: per 32-channel chunk they
// re-staged the whole 9-tap weight slab and the BN+ReLU-transformed halo
// through VGPRs, two barriers per chunk, 1.5 fragment reads per MFMA (32x64
// wave tiles), 15 VALU per MFMA on the 64-channel layers
// (profiles/r02_halo_bf16_instmix.txt).  Here the A operand is a plain bf16
// tensor (the plan's normalised copy relu(bn(y)), the padded dY, the pooled
// map, the convT output -- no transform on load) and:
//  * a workgroup owns TH x 32 output pixels x BN columns; per CK-channel chunk
//    it keeps the (TH+2) x 34 input halo resident in one of two halo slots
//    (the next chunk's halo is DMA'd in 1/NW pieces during this chunk's first
//    taps) and streams the weights tap by tap through a 3-slot ring (one
//    BN x CK slab per tap, prefetched two taps ahead);
//  * one barrier per tap step, counted `s_waitcnt vmcnt` (never 0 in the
//    loop), raw s_barrier: the next slabs stay in flight across it;
//  * DMA addresses are an SGPR base (advanced per step on the scalar unit) plus
//    per-lane 32-bit offsets computed once: no VALU per staged byte;
//  * fragment read addresses are per-lane registers computed once (per tap
//    column and k-step) plus compile-time immediates (tap row, fragment, ring
//    slot): no address VALU in the MFMA loop either;
//  * 16-B pieces are XOR-swizzled inside each pixel / weight row by the row's
//    position in its 256-B bank row, on the DMA's global source address and
//    on the fragment read, so every ds_read_b128 lane group hits distinct
//    bank quads for any tap offset (halo rows use a 36-pixel pitch so the
//    swizzle depends on the pixel's column only).
//  * XTF (round 4): a source with a consumer transform (relu(bn(y)) of the
//    producer, bf16 raw conv output) is DMA'd raw and transformed in LDS, in
//    place, once per chunk: at the chunk's last tap step every piece of the
//    next chunk's halo has landed (issued >= 2 steps earlier, retired by the
//    counted vmcnt + barrier), the waves rewrite it (BN scale / shift of its
//    channels from an LDS table), and the next chunk's first barrier releases
//    it to the MFMAs -- so every forward conv of a bf16 plan runs on the ring
//    without a normalised copy of its input.
// MFMA: v_mfma_f32_32x32x16_bf16, fp32 accumulation; each wave computes
// (TM x 32) pixels x (TN x 32) columns.  The epilogue is the shared one
// (igemm_finish: bias, BN statistics / ReLU mask + BN-backward statistics,
// concat split, split-K partials).
#pragma once
#include <algorithm>

#include "gemm_common.h"
#include "ring_common.h"

namespace unet {

typedef __bf16 bf16x8r_t __attribute__((ext_vector_type(8)));
template <int TH, int BN, int CK>
struct RingGeo {
  static constexpr int TW = 32, HP = 36, RB = CK * 2, KS = CK / 16;
  static constexpr int RPB = 256 / RB, CPR = RB / 16;  // pixel rows per 256-B bank row, 16-B pieces per row
  static constexpr int WSZ = BN * RB;                  // weight slot: one tap x CK channels x BN columns
  static constexpr int PH = (TH + 2) * HP;             // halo pixel rows (36-pixel pitch)
  static constexpr int IH = (PH * RB + 1023) / 1024;   // halo DMA instructions per chunk
  static constexpr int HSZ = IH * 1024;
  static constexpr int H0 = 3 * WSZ;                   // LDS: 3 weight slots, then 2 halo slots
  // + 1 KB junk target: the tap steps past the halo's last piece re-issue a
  // DMA only to keep the per-step vmcnt arithmetic uniform; landing in a halo
  // slot it would overwrite bytes transformed in place meanwhile (XTF)
  static constexpr size_t JNK = (size_t)H0 + 2 * HSZ;
  static constexpr size_t smem = JNK + 1024;
};

template <int TH, int BN, int WM, int WN, int CK, int TWO, int MINW, int XTF, int PT>
__global__ __launch_bounds__(WM * WN * 64, MINW) void k_conv3_ring(const IgemmArgs args) {
  using G = RingGeo<TH, BN, CK>;
  constexpr int HP = G::HP, RB = G::RB, KS = G::KS, RPB = G::RPB, CPR = G::CPR;
  constexpr int WSZ = G::WSZ, IH = G::IH, HSZ = G::HSZ, H0 = G::H0, PH = G::PH;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int TM = TH / WM, TN = BN / (WN * 32);
  constexpr int IW = WSZ / 1024, IWW = IW / NW;  // weight DMAs per tap step: total, per wave
  constexpr int NHS = (IH + NW - 1) / NW;        // halo DMAs per wave per chunk (one per tap step)
  constexpr int D = IWW + 1;                     // DMAs per wave per tap step
  static_assert(TH % WM == 0 && TM >= 1 && TN >= 1 && IW % NW == 0 && IWW >= 1, "tile");
  static_assert(NHS <= 7, "the next chunk's halo must be issued >= 2 tap steps before it is read");
  static_assert(HSZ + (TM + 1) * HP * RB < 65536, "halo fragment offsets must fit the ds_read immediate");
  static_assert(WM * 3 * BN * 4 <= (int)G::smem, "epilogue reduction must fit the LDS image");
  static_assert(!PT || WM * 3 * BN * 4 <= HSZ, "a persistent tile's epilogue scratch is one halo slot");
  extern __shared__ __attribute__((aligned(1024))) unsigned char lds[];
  const unsigned lds0 = (unsigned)(size_t)(lds_u8_t*)lds;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const Gather& g = args.a;
  const int Cg = g.Cg, K = args.K, Hg = g.Hg, Wg = g.Wg;
  int bx, by, bz;  // grid position in XCD-aware order (the column blocks' weights stay in one L2)
  xcd_block(bx, by, bz);
  const int tiles_x = (Wg + 31) / 32, tiles_y = (Hg + TH - 1) / TH;
  const long long ntiles = (long long)g.nimg * tiles_y * tiles_x;
  auto coords = [&](long long t, int& n_, int& y0_, int& x0_) {
    x0_ = (int)(t % tiles_x) * 32;
    t /= tiles_x;
    y0_ = (int)(t % tiles_y) * TH;
    n_ = (int)(t / tiles_y);
  };
  // PT (persistent, tile 88): the workgroup walks tiles blockIdx.x,
  // + gridDim.x, ...; the next tile's first halo and tap-0/1 weights are DMA'd
  // during this tile's last chunk exactly like a next chunk's, so its
  // prologue latency hides under this tile's MFMAs and epilogue
  long long tile = bx;
  int n, y0, x0;
  coords(tile, n, y0, x0);
  const int n0 = by * BN;

  // XTF: BN scale / shift of source 0 (the only source that can carry a
  // transform: a skip or a previous conv output; the convT output never does)
  // in LDS after the ring: [2][C of source 0]
  const int xtc = TWO ? g.c_split : Cg;
  float* xts = reinterpret_cast<float*>(lds + G::smem);
  const bool xtf0 = XTF && g.s[0].scale != nullptr;
  if constexpr (XTF) {
    if (xtf0)
      for (int c = tid; c < xtc; c += NT) {
        xts[c] = g.s[0].scale[c];
        xts[xtc + c] = g.s[0].shift[c];
      }
  }

  // ---- per-lane DMA offsets (bytes) ----
  // (PT: recomputed per tile from an opaque copy of the lane id, so they are
  // not held live across the epilogue -- the persistent form spilled otherwise)
  unsigned woff[IWW];
  auto weight_offsets = [&](int wv, int ln) {
#pragma unroll
    for (int u = 0; u < IWW; ++u) {
      const int b = (wv + NW * u) * 1024 + ln * 16;
      const int row = b / RB, pc = (b % RB) / 16;
      const int q = pc ^ ((row / RPB) % CPR);
      woff[u] = (unsigned)(((n0 + row) * K + q * 8) * 2);
    }
  };
  unsigned hoff0[NHS], hoff1[TWO ? NHS : 1];
  auto halo_offsets = [&](int n_, int y0_, int x0_, unsigned (&o0)[NHS], unsigned (&o1)[TWO ? NHS : 1]) {
#pragma unroll
    for (int k = 0; k < NHS; ++k) {
      const int p = min(k * NW + wave, IH - 1);
      const int b = p * 1024 + lane * 16;
      const int r = min(b / RB, PH - 1), pc = (b % RB) / 16;
      const int hy = r / HP, hx = r % HP;
      const int q = pc ^ ((hx / RPB) % CPR);
      // halo pixels past the input grid (and the 2 pitch-pad columns) read any
      // in-range pixel: they only feed outputs past the grid, never stored
      const int yy = min(y0_ + hy, Hg + 1), xx = min(x0_ + min(hx, 33), Wg + 1);
      const Src& s0 = g.s[0];
      o0[k] = (unsigned)((((n_ * s0.H + yy + s0.oy) * s0.W + xx + s0.ox) * s0.C) * 2 + q * 16);
      if constexpr (TWO) {
        const Src& s1 = g.s[1];
        o1[k] = (unsigned)((((n_ * s1.H + yy + s1.oy) * s1.W + xx + s1.ox) * s1.C) * 2 + q * 16);
      }
    }
  };
  halo_offsets(n, y0, x0, hoff0, hoff1);
  // the next tile's (PT): selected element-wise into the issue (no arrays of
  // register arrays: a runtime pick between two would go to scratch)
  unsigned hnext0[PT ? NHS : 1], hnext1[(PT && TWO) ? NHS : 1];
  bool wrap = false;  // PT: this tile's last chunk hands over to the next tile
  // ---- per-lane fragment read bases (bytes); tap row, fragment and ring
  // slot are compile-time immediates on top ----
  unsigned xa[3][KS], yb[KS];
  auto frag_offsets = [&](int wmv, int wnv, int ln) {
    const int hh = ln >> 5, ll = ln & 31;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int hx = kx + ll;
        xa[kx][s] = (unsigned)(H0 + (wmv * TM * HP + hx) * RB + 16 * ((2 * s + hh) ^ ((hx / RPB) % CPR)));
      }
#pragma unroll
    for (int s = 0; s < KS; ++s)
      yb[s] = (unsigned)((wnv * TN * 32 + ll) * RB + 16 * ((2 * s + hh) ^ ((ll / RPB) % CPR)));
  };
  auto lane_state = [&]() {
    int tv = tid;
    if constexpr (PT) asm volatile("" : "+v"(tv));
    const int wv = tv >> 6, ln = tv & 63;
    weight_offsets(wv, ln);
    frag_offsets(wv / WN, wv % WN, ln);
  };
  lane_state();

  const int nk_all = Cg / CK;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = bz * per;
    kc1 = min(nk_all, kc0 + per);
  }

  // weights of (chunk c, tap t) -> ring slot t % 3 (9 taps per chunk: the slot
  // pattern repeats every chunk)
  auto issue_w = [&](int c, int t, int slot) {
    const unsigned long long base = uniform_u64(args.bh + (size_t)t * Cg + (size_t)c * CK);
#pragma unroll
    for (int u = 0; u < IWW; ++u) dma_sv(woff[u], base, lds0 + slot * WSZ + (wave + NW * u) * 1024);
  };
  auto issue_w1 = [&](int c, int t, int slot, int u) {
    const unsigned long long base = uniform_u64(args.bh + (size_t)t * Cg + (size_t)c * CK);
    dma_sv(woff[u], base, lds0 + slot * WSZ + (wave + NW * u) * 1024);
  };
  // halo piece k of chunk c -> halo slot hs (hs < 0: the junk KB); nt: of the
  // next tile (PT)
  auto issue_h = [&](int c, int k, int hs, bool nt) {
    const int c0 = c * CK;
    const bool second = TWO && c0 >= g.c_split;
    const Src& s = second ? g.s[1] : g.s[0];
    const int cl = second ? c0 - g.c_split : c0;
    const unsigned long long base = uniform_u64(reinterpret_cast<const uint16_t*>(s.ptr) + cl);
    unsigned off = second ? hoff1[TWO ? k : 0] : hoff0[k];
    if constexpr (PT) {
      const unsigned offn = second ? hnext1[TWO ? k : 0] : hnext0[k];
      off = nt ? offn : off;
    }
    dma_sv(off, base, hs < 0 ? lds0 + (unsigned)G::JNK : lds0 + H0 + hs * HSZ + min(k * NW + wave, IH - 1) * 1024);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // one tap step: KS k-steps of TM x TN MFMAs; the next k-step's fragments are
  // read while this one's MFMAs issue
  auto tap_mfma = [&](auto HSc, auto Tc, auto&& after) {
    constexpr int hs = decltype(HSc)::value, t = decltype(Tc)::value;
    constexpr int ky = t / 3, kx = t % 3, ws = t % 3;
    bf16x8r_t fa[2][TM], fb[2][TN];
    auto rd = [&](auto Sc, int b) {
      constexpr int s = decltype(Sc)::value;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[b][i] = *reinterpret_cast<const bf16x8r_t*>(lds + xa[kx][s] + (hs * HSZ + (i + ky) * HP * RB));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[b][j] = *reinterpret_cast<const bf16x8r_t*>(lds + yb[s] + (ws * WSZ + j * 32 * RB));
    };
    rd(std::integral_constant<int, 0>{}, 0);
    auto step = [&](auto Sc) {
      constexpr int s = decltype(Sc)::value;
      if constexpr (s + 1 < KS) rd(std::integral_constant<int, s + 1>{}, (s + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s & 1][i], fb[s & 1][j], acc[i][j], 0, 0, 0);
      after(s);
    };
    step(std::integral_constant<int, 0>{});
    if constexpr (KS > 1) step(std::integral_constant<int, 1>{});
    if constexpr (KS > 2) step(std::integral_constant<int, 2>{});
    if constexpr (KS > 3) step(std::integral_constant<int, 3>{});
  };

  // XTF: relu(bn(.)) of chunk c's raw halo in slot hs, in place (every piece
  // landed and visible: called after a barrier that follows their vmcnt)
  auto transform_h = [&](int c, int hs) {
    const int c0 = c * CK;
    if (!xtf0 || (TWO && c0 >= g.c_split)) return;  // the plain source needs nothing
    unsigned char* hb = lds + H0 + hs * HSZ;
    constexpr int PCS = PH * CPR;  // 16-B pieces of the halo rows
#pragma unroll
    for (int k = 0; k < (PCS + NT - 1) / NT; ++k) {
      const int p = tid + NT * k;
      if (p < PCS) {
        const int r = p / CPR, hx = r % HP;
        const int q = (p % CPR) ^ ((hx / RPB) % CPR);  // logical 8-channel group of the piece
        const float* sc = xts + c0 + q * 8;
        const float* sh = xts + xtc + c0 + q * 8;
        uint4* pv = reinterpret_cast<uint4*>(hb + p * 16);
        const uint4 u = *pv;
        *pv = bf16pack8(affine_relu4(bf16x4_to_f4(make_uint2(u.x, u.y)), ld4(sc), ld4(sh)),
                        affine_relu4(bf16x4_to_f4(make_uint2(u.z, u.w)), ld4(sc + 4), ld4(sh + 4)));
      }
    }
  };

  // one chunk: 9 tap steps; step (c, t): wait for this wave's DMAs of step
  // (c, t) - 2 and older, barrier (everyone's landed, everyone done reading
  // the slot refilled next), issue the weights of step (c, t) + 2 and a piece
  // of chunk c+1's halo, compute
  bool after_epi = false;  // PT: the first tap step after an epilogue (its wait was taken before it)
  auto chunk = [&](auto HSc, int c) {
    constexpr int hs = decltype(HSc)::value;
    const bool wr = PT && wrap && c == kc1 - 1;  // the next "chunk" is the next tile's first
    // past the last chunk: identical bytes rewritten, never read
    const int cn = wr ? kc0 : min(c + 1, kc1 - 1);
    auto tap = [&](auto Tc) {
      constexpr int t = decltype(Tc)::value;
      if (t != 0 || !after_epi) vm_wait<D>();
      raw_barrier();
      if constexpr (t == 0) after_epi = false;
      const bool nx = t + 2 >= 9;
      int cw = nx ? c + 1 : c, tw = nx ? t - 7 : t + 2;
      if (cw >= kc1) {
        if (wr) cw = kc0;  // the next tile's taps 0 / 1
        else { cw = kc1 - 1; tw = 8; }  // tail: reload the last slab into a free slot
      }
      if constexpr (XTF && t == 8) {
        if (cn != c || wr) transform_h(cn, hs ^ 1);
      }
      // this step's D DMAs go out one per k-step between the MFMAs (all at
      // once after the barrier they put every wave of the CU in its DMA phase
      // together): the weights of step + 2, then a piece of the next chunk's
      // halo to the other slot (past the last chunk the re-issued bytes land
      // there too: never read), or -- once the halo's pieces are out -- a
      // dummy piece to the junk KB (keeps D DMAs per step for the vmcnt count
      // without touching a halo that may be transformed in place)
      auto after = [&](int k) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          if (u == k || (k == KS - 1 && u > k)) {
            if (u < IWW) issue_w1(cw, tw, (t + 2) % 3, u);
            else issue_h(cn, t < NHS ? t : NHS - 1, t < NHS ? hs ^ 1 : -1, wr);
          }
        }
      };
      tap_mfma(HSc, Tc, after);
    };
    tap(std::integral_constant<int, 0>{});
    tap(std::integral_constant<int, 1>{});
    tap(std::integral_constant<int, 2>{});
    tap(std::integral_constant<int, 3>{});
    tap(std::integral_constant<int, 4>{});
    tap(std::integral_constant<int, 5>{});
    tap(std::integral_constant<int, 6>{});
    tap(std::integral_constant<int, 7>{});
    tap(std::integral_constant<int, 8>{});
  };

  if (kc0 < kc1) {
    // prologue: chunk kc0's halo, the weights of its taps 0 and 1
#pragma unroll
    for (int k = 0; k < NHS; ++k) issue_h(kc0, k, 0, false);
    issue_w(kc0, 0, 0);
    issue_w(kc0, 1, 1);
    vm_wait<0>();
    if constexpr (XTF) {
      __syncthreads();  // the halo (and the BN table) visible to every wave
      transform_h(kc0, 0);
    }
    raw_barrier();
  }
  int par = 0;  // halo slot parity: alternates per chunk across tiles
  for (;;) {
    if (PT && after_epi) {  // the new tile's lane state (dead across the epilogue)
      lane_state();
      halo_offsets(n, y0, x0, hoff0, hoff1);
    }
    int nn = 0, ny0 = 0, nx0 = 0;
    const long long tnext = tile + gridDim.x;
    if constexpr (PT) {
      wrap = kc0 < kc1 && tnext < ntiles;
      if (wrap) {
        coords(tnext, nn, ny0, nx0);
        halo_offsets(nn, ny0, nx0, hnext0, hnext1);
      }
    }
    for (int c = kc0; c < kc1; ++c, ++par) {
      if (par & 1) chunk(std::integral_constant<int, 1>{}, c);
      else chunk(std::integral_constant<int, 0>{}, c);
    }
    // One epilogue call site (an empty split-K slice writes its zero partial).
    // PT with a next tile: its halo and tap-0/1 weights are in flight; this
    // wave's DMAs of tap step 7 and older retire here (so the next tile's tap
    // 0 takes no wait), every wave gets past the last tap's MFMAs, and the halo
    // slot just read serves as the epilogue's scratch (the in-flight DMAs
    // target the other halo slot, weight slots 0 / 1 and the junk KB).
    // Otherwise every DMA lands and the whole LDS image is free.
    float* red = reinterpret_cast<float*>(lds);
    // LDS-staged bf16 stores (epi_lds) when the whole image is free: the waves'
    // 4-KB staging tiles first, the statistics buffer after them
    constexpr bool kStage = TN == 2 && (size_t)NW * 4096 + (size_t)WM * 3 * BN * 4 <= G::smem;
    unsigned short* stage = nullptr;
    if (PT && wrap) {
      vm_wait<D>();
      raw_barrier();
      red = reinterpret_cast<float*>(lds + H0 + ((par - 1) & 1) * HSZ);
    } else {
      vm_wait<0>();
      __syncthreads();
      if constexpr (kStage) {
        stage = reinterpret_cast<unsigned short*>(lds);
        red = reinterpret_cast<float*>(lds + NW * 4096);
      }
    }
    igemm_finish<TH * 32, BN, WM, WN, NT, HaloRows<32, TH>, 1>(args, acc, 0, n0, wm, wn, tid, red,
                                                                HaloRows<32, TH>{n, y0, x0, Hg, Wg}, stage, bz);
    if (!PT || !wrap) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    tile = tnext;
    n = nn; y0 = ny0; x0 = nx0;
    after_epi = true;
  }
}

// the LDS image of a launch: the ring, plus the BN table of source 0 (XTF)
template <int TH, int BN, int CK>
static size_t ring_smem(const IgemmArgs& a, bool xtf) {
  const Gather& g = a.a;
  return RingGeo<TH, BN, CK>::smem + (xtf ? 8 * (size_t)(g.c_split < g.Cg ? g.c_split : g.Cg) : 0);
}

static int ring_num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <int TH, int BN, int WM, int WN, int CK, int MINW, int PT>
static hipError_t go_ring(const IgemmArgs& a, hipStream_t s) {
  const Gather& g = a.a;
  const bool two = g.c_split < g.Cg, xtf = g.s[0].scale != nullptr;
  const int v = (two ? 1 : 0) | (xtf ? 2 : 0);
  static bool attr[4] = {false, false, false, false};
  const void* fns[4] = {reinterpret_cast<const void*>(&k_conv3_ring<TH, BN, WM, WN, CK, 0, MINW, 0, PT>),
                        reinterpret_cast<const void*>(&k_conv3_ring<TH, BN, WM, WN, CK, 1, MINW, 0, PT>),
                        reinterpret_cast<const void*>(&k_conv3_ring<TH, BN, WM, WN, CK, 0, MINW, 1, PT>),
                        reinterpret_cast<const void*>(&k_conv3_ring<TH, BN, WM, WN, CK, 1, MINW, 1, PT>)};
  const size_t smem = ring_smem<TH, BN, CK>(a, xtf);
  if (!attr[v]) {  // the largest image any launch of this variant can ask for
    hipError_t e = hipFuncSetAttribute(fns[v], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr[v] = true;
  }
  const long long tiles = (long long)g.nimg * ((g.Hg + TH - 1) / TH) * ((g.Wg + 31) / 32);
  long long gx = tiles;
  if (PT) {  // resident workgroups only: every CU's slots once (column blocks share them)
    const long long per_cu = std::max<long long>(1, std::min<long long>(MINW, (160 * 1024) / (long long)smem));
    gx = std::min(tiles, std::max<long long>(1, ring_num_cus() * per_cu / (a.N / BN)));
  }
  dim3 grid((unsigned)gx, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  switch (v) {
    case 0: hipLaunchKernelGGL((k_conv3_ring<TH, BN, WM, WN, CK, 0, MINW, 0, PT>), grid, dim3(WM * WN * 64), smem, s, a); break;
    case 1: hipLaunchKernelGGL((k_conv3_ring<TH, BN, WM, WN, CK, 1, MINW, 0, PT>), grid, dim3(WM * WN * 64), smem, s, a); break;
    case 2: hipLaunchKernelGGL((k_conv3_ring<TH, BN, WM, WN, CK, 0, MINW, 1, PT>), grid, dim3(WM * WN * 64), smem, s, a); break;
    default: hipLaunchKernelGGL((k_conv3_ring<TH, BN, WM, WN, CK, 1, MINW, 1, PT>), grid, dim3(WM * WN * 64), smem, s, a); break;
  }
  return hipGetLastError();
}

}  // namespace unet
