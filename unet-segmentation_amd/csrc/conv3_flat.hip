// k_conv3_flat (tile 85): the LDS-DMA ring 3x3 conv (conv3_ring_kernel.h) on
// flat pixel tiles.
//
// k_conv3_ring owns TH x 32 output pixels: one 32-wide MFMA fragment per tile
// row.  On the 24-48-pixel grids of the 1024-channel bottleneck (down4, up1:
// models/unet_model.py:95-104) a row of 24, 26, 44 or 46 pixels leaves 19-31 %
// of every fragment's rows past the grid, and the row tiles of a 26-row map
// another 19 % -- a third of the MFMA work of the step's most expensive convs
// fed nothing.  Here a tile is BM = TH x 32 CONSECUTIVE output
// pixels of the flattened (image, row, column) grid, so fragments wrap grid rows
// and the only idle rows are the last tile's:
//  * the input of a valid 3x3 conv over consecutive output pixels is a
//    contiguous run of the virtual input grid (image, Hg + 2, Wg + 2) -- at most
//    NPX pixels, held in a halo slot at a 128-B (CK = 64) pitch, 16-B pieces
//    XOR-swizzled by the halo pixel's index (consecutive output pixels hit
//    distinct bank quads except across a row wrap);
//  * each DMA piece maps its virtual pixel to the stored tensor through the
//    source's own geometry (crop origin, concat split), once per tile;
//  * a lane's fragment row is its output pixel's halo index plus the tap's
//    uniform offset ky (Wg + 2) + kx: a handful of VALU per fragment and tap
//    (the ring's tap rows were compile-time immediates);
//  * tiles run across image boundaries when the run stays within NPX (the two
//    boundary rows join the halo), else per image (FlatMap::tpi).
// Everything else -- 3-slot weight ring, double-buffered halo, counted vmcnt,
// raw barriers, XTF in LDS, the shared epilogue on linear rows -- is the ring's.
#include <algorithm>
#include <atomic>

#include "gemm_common.h"
#include "ring_common.h"

namespace unet {

typedef __bf16 bf16x8f_t __attribute__((ext_vector_type(8)));

// tiles_per_image 0: tiles cross images (tile t = pixels t*BM ..); else tile t
// = image t / tpi, pixels (t % tpi) * BM .. of that image.  Stream-K (tile 86):
// U = ntiles x (N / BN) x nk work units (tile, column block, K chunk) dealt in
// equal contiguous runs over the grid; token: this launch's flag value.
struct FlatMap {
  int tpi, Hin, Win, Qmax;
  int ntiles, nk, U;
  unsigned token;
};

template <int TH, int BN, int CK, int NPX>
struct FlatGeo {
  static constexpr int RB = CK * 2, KS = CK / 16;
  static constexpr int RPB = 256 / RB, CPR = RB / 16;  // halo pixels per 256-B bank row, 16-B pieces per pixel
  static constexpr int SH = RPB == 2 ? 1 : RPB == 4 ? 2 : 3;
  static constexpr int WSZ = BN * RB;
  static constexpr int IH = (NPX * RB + 1023) / 1024;  // halo DMA instructions per chunk
  static constexpr int HSZ = IH * 1024;
  static constexpr int H0 = 3 * WSZ;
  static constexpr size_t JNK = (size_t)H0 + 2 * HSZ;
  static constexpr size_t smem = JNK + 1024;
};

// stream-K: at most kSkSeg workgroups share one (tile, column block); the
// non-first ones leave fp32 partial tiles in slots of the split-K slab
constexpr int kSkSeg = 4;

// SK (stream-K, tile 86): each workgroup walks its run of work units; a run
// that starts inside a (tile, column block) leaves its partial tile in the slab
// and raises that segment's flag; the workgroup holding the block's first
// chunk -- it reaches the block at the end of its run, after the later
// segments' workgroups (which start with them) -- adds those partials and runs
// the epilogue.  Owners wait only on higher-numbered workgroups whose partial
// is their first work: no cycle.  Spins are bounded.
template <int TH, int BN, int WM, int WN, int CK, int NPX, int TWO, int MINW, int XTF, int SK>
__global__ __launch_bounds__(WM * WN * 64, MINW) void k_conv3_flat(const IgemmArgs args, const FlatMap fm) {
  using G = FlatGeo<TH, BN, CK, NPX>;
  constexpr int RB = G::RB, KS = G::KS, CPR = G::CPR, SH = G::SH;
  constexpr int WSZ = G::WSZ, IH = G::IH, HSZ = G::HSZ, H0 = G::H0;
  constexpr int NW = WM * WN, NT = NW * 64, BM = TH * 32;
  constexpr int TM = TH / WM, TN = BN / (WN * 32);
  constexpr int IW = WSZ / 1024, IWW = IW / NW;
  constexpr int NHS = (IH + NW - 1) / NW;
  constexpr int D = IWW + 1;
  static_assert(TH % WM == 0 && TM >= 1 && TN >= 1 && IW % NW == 0 && IWW >= 1, "tile");
  static_assert(NHS <= 7, "the next chunk's halo must be issued >= 2 tap steps before it is read");
  static_assert(WM * 3 * BN * 4 <= (int)G::smem, "epilogue reduction must fit the LDS image");
  extern __shared__ __attribute__((aligned(1024))) unsigned char lds[];
  const unsigned lds0 = (unsigned)(size_t)(lds_u8_t*)lds;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const Gather& g = args.a;
  const int Cg = g.Cg, K = args.K, Wg = g.Wg, HW = g.Hg * g.Wg;
  const int Hin = fm.Hin, Win = fm.Win, HWin = Hin * Win;

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
  // the work of this workgroup
  int bx = 0, by = 0, bz = 0;
  int wgi = 0, base = 1, rem = 0, u = 0, ue = 0;
  if constexpr (SK) {
    const unsigned ng = gridDim.x, bid = blockIdx.x;
    // XCD-aware: each XCD runs a contiguous stretch of the unit order
    wgi = (ng & 7u) == 0 ? (int)((bid & 7u) * (ng >> 3) + (bid >> 3)) : (int)bid;
    base = fm.U / (int)ng;
    rem = fm.U - base * (int)ng;
    u = wgi * base + min(wgi, rem);
    ue = u + base + (wgi < rem ? 1 : 0);
  } else {
    xcd_block(bx, by, bz);
  }
  // the workgroup whose run holds unit v
  auto owner_of = [&](int v) {
    const int b1 = base + 1;
    return v < rem * b1 ? v / b1 : rem + (v - rem * b1) / base;
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (;;) {
    int tile, nb, kc0, kc1;
    if constexpr (SK) {
      if (u >= ue) break;
      const int tb = u / fm.nk;
      kc0 = u - tb * fm.nk;
      kc1 = min(fm.nk, kc0 + (ue - u));
      tile = tb % fm.ntiles;
      nb = tb / fm.ntiles;
    } else {
      tile = bx;
      nb = by;
      kc0 = 0;
      kc1 = Cg / CK;
      if (args.ksplit > 1) {
        const int per = (kc1 + args.ksplit - 1) / args.ksplit;
        kc0 = bz * per;
        kc1 = min(Cg / CK, kc0 + per);
      }
    }
    int P0, cnt;
    if (fm.tpi > 0) {
      const int img = tile / fm.tpi, lt = tile - img * fm.tpi;
      P0 = img * HW + lt * BM;
      cnt = min(BM, HW - lt * BM);
    } else {
      P0 = tile * BM;
      cnt = min(BM, args.M - P0);
    }
    // virtual input pixel of output pixel P's tap (0, 0)
    auto qin = [&](int P) {
      const int img = P / HW, rem_ = P - img * HW, y = rem_ / Wg, x = rem_ - y * Wg;
      return (img * Hin + y) * Win + x;
    };
    const int Q0 = qin(P0);
    const int n0 = nb * BN;
    // lane-derived state, recomputed per segment from an opaque copy of the
    // thread id (stream-K: not held live across the epilogue)
    int tv = tid;
    if constexpr (SK) asm volatile("" : "+v"(tv));
    const int lane_ = tv & 63, wave_ = tv >> 6, ll_ = lane_ & 31, hh_ = lane_ >> 5;
    const int wm_ = wave_ / WN, wn_ = wave_ % WN;
    unsigned yb[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      yb[s] = (unsigned)((wn_ * TN * 32 + ll_) * RB + 16 * ((2 * s + hh_) ^ ((ll_ / G::RPB) % CPR)));

    // ---- per-lane DMA offsets (bytes) ----
    unsigned woff[IWW];
#pragma unroll
    for (int q8 = 0; q8 < IWW; ++q8) {
      const int b = (wave_ + NW * q8) * 1024 + lane_ * 16;
      const int row = b / RB, pc = (b % RB) / 16;
      const int q = pc ^ ((row / G::RPB) % CPR);
      woff[q8] = (unsigned)(((n0 + row) * K + q * 8) * 2);
    }
    unsigned hoff0[NHS], hoff1[TWO ? NHS : 1];
#pragma unroll
    for (int k = 0; k < NHS; ++k) {
      const int p = min(k * NW + wave_, IH - 1);
      const int b = p * 1024 + lane_ * 16;
      const int r = min(b / RB, NPX - 1), pc = (b % RB) / 16;
      const int q = pc ^ ((r >> SH) & (CPR - 1));
      // halo pixels past the grid's last input pixel read that pixel: they only
      // feed rows past the tile's count, never stored
      const int Q = min(Q0 + r, fm.Qmax);
      const int img = Q / HWin, rq_ = Q - img * HWin, yy = rq_ / Win, xx = rq_ - yy * Win;
      const Src& s0 = g.s[0];
      hoff0[k] = (unsigned)((((img * s0.H + yy + s0.oy) * s0.W + xx + s0.ox) * s0.C) * 2 + q * 16);
      if constexpr (TWO) {
        const Src& s1 = g.s[1];
        hoff1[k] = (unsigned)((((img * s1.H + yy + s1.oy) * s1.W + xx + s1.ox) * s1.C) * 2 + q * 16);
      }
    }
    // ---- per-lane fragment rows: the halo index of each fragment's output
    // pixel (rows past the count repeat the last pixel) ----
    int rq[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) rq[i] = qin(P0 + min((wm_ * TM + i) * 32 + ll_, cnt - 1)) - Q0;

    auto issue_w = [&](int c, int t, int slot) {
      const unsigned long long bs = uniform_u64(args.bh + (size_t)t * Cg + (size_t)c * CK);
#pragma unroll
      for (int q8 = 0; q8 < IWW; ++q8) dma_sv(woff[q8], bs, lds0 + slot * WSZ + (wave + NW * q8) * 1024);
    };
    auto issue_w1 = [&](int c, int t, int slot, int q8) {
      const unsigned long long bs = uniform_u64(args.bh + (size_t)t * Cg + (size_t)c * CK);
      dma_sv(woff[q8], bs, lds0 + slot * WSZ + (wave + NW * q8) * 1024);
    };
    auto issue_h = [&](int c, int k, int hs) {
      const int c0 = c * CK;
      const bool second = TWO && c0 >= g.c_split;
      const Src& sr = second ? g.s[1] : g.s[0];
      const int cl = second ? c0 - g.c_split : c0;
      const unsigned long long bs = uniform_u64(reinterpret_cast<const uint16_t*>(sr.ptr) + cl);
      const unsigned off = second ? hoff1[TWO ? k : 0] : hoff0[k];
      dma_sv(off, bs, hs < 0 ? lds0 + (unsigned)G::JNK : lds0 + H0 + hs * HSZ + min(k * NW + wave, IH - 1) * 1024);
    };

    // one tap step: the fragment rows moved by the tap's offset, then KS
    // k-steps of TM x TN MFMAs (the next k-step's fragments read during this one's)
    auto tap_mfma = [&](auto HSc, auto Tc, auto&& after) {
      constexpr int hs = decltype(HSc)::value, t = decltype(Tc)::value;
      constexpr int ky = t / 3, kx = t % 3, ws = t % 3;
      const int dlt = ky * Win + kx;
      unsigned fab[TM];
      int hv[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        // opaque per tap: the rows of all 18 (slot, tap) steps hoisted out of
        // the chunk loop would not fit the register file
        int rv = rq[i];
        asm volatile("" : "+v"(rv));
        const int r = rv + dlt;
        fab[i] = (unsigned)(H0 + hs * HSZ + r * RB);
        hv[i] = hh_ ^ ((r >> SH) & (CPR - 1));
      }
      bf16x8f_t fa[2][TM], fb[2][TN];
      auto rd = [&](auto Sc, int b) {
        constexpr int s = decltype(Sc)::value;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[b][i] = *reinterpret_cast<const bf16x8f_t*>(lds + fab[i] + (((2 * s) ^ hv[i]) << 4));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[b][j] = *reinterpret_cast<const bf16x8f_t*>(lds + yb[s] + (ws * WSZ + j * 32 * RB));
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

    // XTF: relu(bn(.)) of chunk c's raw halo in slot hs, in place
    auto transform_h = [&](int c, int hs) {
      const int c0 = c * CK;
      if (!xtf0 || (TWO && c0 >= g.c_split)) return;
      unsigned char* hb = lds + H0 + hs * HSZ;
      constexpr int PCS = NPX * CPR;
#pragma unroll
      for (int k = 0; k < (PCS + NT - 1) / NT; ++k) {
        const int p = tid + NT * k;
        if (p < PCS) {
          const int r = p / CPR;
          const int q = (p % CPR) ^ ((r >> SH) & (CPR - 1));
          const float* sc = xts + c0 + q * 8;
          const float* sh = xts + xtc + c0 + q * 8;
          uint4* pv = reinterpret_cast<uint4*>(hb + p * 16);
          const uint4 v = *pv;
          *pv = bf16pack8(affine_relu4(bf16x4_to_f4(make_uint2(v.x, v.y)), ld4(sc), ld4(sh)),
                          affine_relu4(bf16x4_to_f4(make_uint2(v.z, v.w)), ld4(sc + 4), ld4(sh + 4)));
        }
      }
    };

    // one chunk: 9 tap steps (the ring's schedule: wait for this wave's DMAs of
    // step - 2, barrier, issue the weights of step + 2 and a piece of the next
    // chunk's halo between the k-steps, compute)
    auto chunk = [&](auto HSc, int c) {
      constexpr int hs = decltype(HSc)::value;
      const int cn = min(c + 1, kc1 - 1);
      auto tap = [&](auto Tc) {
        constexpr int t = decltype(Tc)::value;
        vm_wait<D>();
        raw_barrier();
        const bool nx = t + 2 >= 9;
        int cw = nx ? c + 1 : c, tw = nx ? t - 7 : t + 2;
        if (cw >= kc1) { cw = kc1 - 1; tw = 8; }
        if constexpr (XTF && t == 8) {
          if (cn != c) transform_h(cn, hs ^ 1);
        }
        auto after = [&](int k) {
#pragma unroll
          for (int q8 = 0; q8 < D; ++q8) {
            if (q8 == k || (k == KS - 1 && q8 > k)) {
              if (q8 < IWW) issue_w1(cw, tw, (t + 2) % 3, q8);
              else issue_h(cn, t < NHS ? t : NHS - 1, t < NHS ? hs ^ 1 : -1);
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
#pragma unroll
      for (int k = 0; k < NHS; ++k) issue_h(kc0, k, 0);
      issue_w(kc0, 0, 0);
      issue_w(kc0, 1, 1);
      vm_wait<0>();
      if constexpr (XTF) {
        __syncthreads();
        transform_h(kc0, 0);
      }
      raw_barrier();
    }
    for (int c = kc0; c < kc1; ++c) {
      if ((c - kc0) & 1) chunk(std::integral_constant<int, 1>{}, c);
      else chunk(std::integral_constant<int, 0>{}, c);
    }
    vm_wait<0>();
    __syncthreads();

    if constexpr (SK) {
      const int tb = tile + nb * fm.ntiles;
      const int ntb = fm.ntiles * (args.N / BN);
      float4* const part = reinterpret_cast<float4*>(args.slab);
      unsigned* const flags = reinterpret_cast<unsigned*>(args.slab + (size_t)ntb * (kSkSeg - 1) * BM * BN);
      // partial slot layout: the accumulator registers in lane order (16-B stores)
      auto slot_at = [&](int sl, int i, int j, int r4) {
        return part + (size_t)sl * (BM * BN / 4) + ((size_t)((wave * TM + i) * TN + j) * 4 + r4) * 64 + lane;
      };
      if (kc0 > 0) {  // a later segment: leave the partial, raise its flag
        const int sl = tb * (kSkSeg - 1) + (wgi - owner_of(tb * fm.nk)) - 1;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
              *slot_at(sl, i, j, r4) = make_float4(acc[i][j][4 * r4], acc[i][j][4 * r4 + 1], acc[i][j][4 * r4 + 2],
                                                   acc[i][j][4 * r4 + 3]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(flags + sl, fm.token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        u += kc1 - kc0;
        continue;
      }
      // the first segment: add the later segments' partials
      const int nseg = owner_of((tb + 1) * fm.nk - 1) - wgi + 1;
      for (int sg = 1; sg < nseg; ++sg) {
        const int sl = tb * (kSkSeg - 1) + sg - 1;
        if (tid == 0) {
          for (int spin = 0; spin < (1 << 24); ++spin) {
            if (__hip_atomic_load(flags + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == fm.token) break;
            __builtin_amdgcn_s_sleep(4);
          }
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
              const float4 v = *slot_at(sl, i, j, r4);
              acc[i][j][4 * r4] += v.x;
              acc[i][j][4 * r4 + 1] += v.y;
              acc[i][j][4 * r4 + 2] += v.z;
              acc[i][j][4 * r4 + 3] += v.w;
            }
        if (tid == 0) __hip_atomic_store(flags + sl, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }

    float* red = reinterpret_cast<float*>(lds);
    constexpr bool kStage = TN == 2 && (size_t)NW * 4096 + (size_t)WM * 3 * BN * 4 <= G::smem;
    unsigned short* stage = nullptr;
    if constexpr (kStage) {
      stage = reinterpret_cast<unsigned short*>(lds);
      red = reinterpret_cast<float*>(lds + NW * 4096);
    }
    igemm_finish<BM, BN, WM, WN, NT, LinearRows, 1>(args, acc, P0, n0, wm, wn, tid, red, LinearRows{P0, P0 + cnt},
                                                    stage, bz);
    if constexpr (!SK) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    u += kc1 - kc0;
    __syncthreads();  // the epilogue's LDS before the next segment's prologue DMA
  }
}

namespace {

constexpr int kFlatTH = 8, kFlatBN = 128, kFlatCK = 64, kFlatNPX = 400;

// the flat tiling of a launch: across images when every tile's input run fits
// NPX halo pixels, else per image; false when neither does
bool flat_map(const Gather& g, long long M, int BM, int npx, FlatMap& fm, long long& ntiles) {
  const long long Hg = g.Hg, Wg = g.Wg, HW = Hg * Wg, Hin = Hg + 2, Win = Wg + 2;
  if (HW <= 0 || g.nimg <= 0 || (long long)g.nimg * Hin * Win >= (1LL << 31)) return false;
  auto qin = [&](long long P) {
    const long long img = P / HW, rem = P - img * HW, y = rem / Wg, x = rem - y * Wg;
    return (img * Hin + y) * Win + x;
  };
  auto span = [&](long long P0, long long cnt) { return qin(P0 + cnt - 1) + 2 * Win + 2 - qin(P0) + 1; };
  fm = FlatMap{};
  fm.Hin = (int)Hin;
  fm.Win = (int)Win;
  fm.Qmax = (int)(g.nimg * Hin * Win - 1);
  long long worst = 0;
  const long long nt = (M + BM - 1) / BM;
  for (long long t = 0; t < nt; ++t) worst = std::max(worst, span(t * BM, std::min<long long>(BM, M - t * BM)));
  if (worst <= npx) {
    fm.tpi = 0;
    ntiles = nt;
  } else {
    const long long tpi = (HW + BM - 1) / BM;
    worst = 0;
    for (long long t = 0; t < tpi; ++t) worst = std::max(worst, span(t * BM, std::min<long long>(BM, HW - t * BM)));
    if (worst > npx) return false;
    fm.tpi = (int)tpi;
    ntiles = g.nimg * tpi;
  }
  fm.ntiles = (int)ntiles;
  return true;
}

size_t flat_smem(const IgemmArgs& a, bool xtf) {
  const Gather& g = a.a;
  return FlatGeo<kFlatTH, kFlatBN, kFlatCK, kFlatNPX>::smem +
         (xtf ? 8 * (size_t)(g.c_split < g.Cg ? g.c_split : g.Cg) : 0);
}

size_t src_bytes(const Src& s, int nimg) { return (size_t)nimg * s.H * s.W * s.C * 2; }

int flat_num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

// stream-K deal (tile 86): one workgroup per CU, every (tile, column block)
// shared by at most kSkSeg of them; false when the launch has fewer units than
// workgroups or a block would need more segments
bool sk_deal(const IgemmArgs& a, FlatMap& fm, int& grid) {
  long long nt = 0;
  if (!flat_map(a.a, a.M, kFlatTH * 32, kFlatNPX, fm, nt)) return false;
  const long long nk = a.a.Cg / kFlatCK, U = nt * (a.N / kFlatBN) * nk;
  const long long G = flat_num_cus();
  if (U < G || U >= (1LL << 31)) return false;
  const long long base = U / G, rem = U % G;
  auto owner = [&](long long v) { return v < rem * (base + 1) ? v / (base + 1) : rem + (v - rem * (base + 1)) / base; };
  for (long long tb = 0; tb < U / nk; ++tb)
    if (owner((tb + 1) * nk - 1) - owner(tb * nk) + 1 > kSkSeg) return false;
  fm.nk = (int)nk;
  fm.U = (int)U;
  grid = (int)G;
  return true;
}

}  // namespace

size_t conv3_flat_sk_slab_bytes(const IgemmArgs& a) {
  FlatMap fm;
  long long nt = 0;
  if (!flat_map(a.a, a.M, kFlatTH * 32, kFlatNPX, fm, nt)) return ~(size_t)0;
  const size_t ntb = (size_t)nt * (a.N / kFlatBN);
  return ntb * (kSkSeg - 1) * ((size_t)kFlatTH * 32 * kFlatBN * 4 + 4);
}

bool conv3_flat_fits(const IgemmArgs& a, int tile) {
  if (tile != 85 && tile != 86) return false;
  const Gather& g = a.a;
  const bool two = g.c_split < g.Cg, xtf = g.s[0].scale != nullptr;
  FlatMap fm;
  long long nt;
  int grid;
  const bool base = a.bh != nullptr && a.bl == nullptr && a.N % kFlatBN == 0 && g.taps_h == 3 && g.taps_w == 3 &&
                    g.stride == 1 && a.K == 9 * g.Cg && g.Cg % kFlatCK == 0 && g.c_split % kFlatCK == 0 &&
                    g.s[0].h16 && (!two || (g.s[1].h16 && g.s[1].scale == nullptr)) &&
                    (!xtf || g.s[0].shift != nullptr) && flat_smem(a, xtf) <= 160 * 1024 &&
                    src_bytes(g.s[0], g.nimg) < (1ull << 32) && (!two || src_bytes(g.s[1], g.nimg) < (1ull << 32)) &&
                    (size_t)a.N * a.K * 2 < (1ull << 32) && flat_map(g, a.M, kFlatTH * 32, kFlatNPX, fm, nt);
  if (!base) return false;
  // stream-K: its partial slots live in the split-K slab (the plan checks the size)
  return tile == 85 || (a.slab != nullptr && a.ksplit <= 1 && sk_deal(a, fm, grid));
}

long long conv3_flat_tiles(const IgemmArgs& a, int tile) {
  FlatMap fm;
  long long nt = 0;
  if (!flat_map(a.a, a.M, kFlatTH * 32, kFlatNPX, fm, nt)) return 0;
  if (tile == 86) return flat_num_cus();
  return nt * (a.N / kFlatBN);
}

hipError_t go_conv3_flat_tile(const IgemmArgs& a, hipStream_t s, int tile) {
  if (!conv3_flat_fits(a, tile)) return hipErrorInvalidValue;
  constexpr int TH = kFlatTH, BN = kFlatBN, CK = kFlatCK, NPX = kFlatNPX, WM = 4, WN = 2, MINW = 2;
  const Gather& g = a.a;
  FlatMap fm;
  long long nt;
  flat_map(g, a.M, TH * 32, NPX, fm, nt);
  const bool sk = tile == 86;
  int skg = 0;
  if (sk) {
    if (!sk_deal(a, fm, skg)) return hipErrorInvalidValue;
    static std::atomic<unsigned> tokens{0x5A17C0DEu};
    unsigned t = tokens.fetch_add(2u);
    fm.token = t ? t : 1u;  // never 0: a consumed flag is cleared to 0
  }
  const bool two = g.c_split < g.Cg, xtf = g.s[0].scale != nullptr;
  const int v = (two ? 1 : 0) | (xtf ? 2 : 0) | (sk ? 4 : 0);
  static bool attr[8] = {false, false, false, false, false, false, false, false};
#define FLAT_K(T2, X, S) k_conv3_flat<TH, BN, WM, WN, CK, NPX, T2, MINW, X, S>
  const void* fns[8] = {reinterpret_cast<const void*>(&FLAT_K(0, 0, 0)), reinterpret_cast<const void*>(&FLAT_K(1, 0, 0)),
                        reinterpret_cast<const void*>(&FLAT_K(0, 1, 0)), reinterpret_cast<const void*>(&FLAT_K(1, 1, 0)),
                        reinterpret_cast<const void*>(&FLAT_K(0, 0, 1)), reinterpret_cast<const void*>(&FLAT_K(1, 0, 1)),
                        reinterpret_cast<const void*>(&FLAT_K(0, 1, 1)), reinterpret_cast<const void*>(&FLAT_K(1, 1, 1))};
  if (!attr[v]) {
    hipError_t e = hipFuncSetAttribute(fns[v], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr[v] = true;
  }
  const size_t smem = flat_smem(a, xtf);
  const dim3 grid = sk ? dim3((unsigned)skg, 1, 1) : dim3((unsigned)nt, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  const dim3 block(WM * WN * 64);
  switch (v) {
    case 0: hipLaunchKernelGGL((FLAT_K(0, 0, 0)), grid, block, smem, s, a, fm); break;
    case 1: hipLaunchKernelGGL((FLAT_K(1, 0, 0)), grid, block, smem, s, a, fm); break;
    case 2: hipLaunchKernelGGL((FLAT_K(0, 1, 0)), grid, block, smem, s, a, fm); break;
    case 3: hipLaunchKernelGGL((FLAT_K(1, 1, 0)), grid, block, smem, s, a, fm); break;
    case 4: hipLaunchKernelGGL((FLAT_K(0, 0, 1)), grid, block, smem, s, a, fm); break;
    case 5: hipLaunchKernelGGL((FLAT_K(1, 0, 1)), grid, block, smem, s, a, fm); break;
    case 6: hipLaunchKernelGGL((FLAT_K(0, 1, 1)), grid, block, smem, s, a, fm); break;
    default: hipLaunchKernelGGL((FLAT_K(1, 1, 1)), grid, block, smem, s, a, fm); break;
  }
#undef FLAT_K
  return hipGetLastError();
}

}  // namespace unet
