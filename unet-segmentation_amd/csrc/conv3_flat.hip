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

#include "gemm_common.h"
#include "ring_common.h"

namespace unet {

typedef __bf16 bf16x8f_t __attribute__((ext_vector_type(8)));

// tiles_per_image 0: tiles cross images (tile t = pixels t*BM ..); else tile t
// = image t / tpi, pixels (t % tpi) * BM .. of that image
struct FlatMap {
  int tpi, Hin, Win, Qmax;
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

template <int TH, int BN, int WM, int WN, int CK, int NPX, int TWO, int MINW, int XTF>
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
  int bx, by, bz;
  xcd_block(bx, by, bz);
  int P0, cnt;
  if (fm.tpi > 0) {
    const int img = bx / fm.tpi, lt = bx - img * fm.tpi;
    P0 = img * HW + lt * BM;
    cnt = min(BM, HW - lt * BM);
  } else {
    P0 = bx * BM;
    cnt = min(BM, args.M - P0);
  }
  // virtual input pixel of output pixel P's tap (0, 0)
  auto qin = [&](int P) {
    const int img = P / HW, rem = P - img * HW, y = rem / Wg, x = rem - y * Wg;
    return (img * Hin + y) * Win + x;
  };
  const int Q0 = qin(P0);
  const int n0 = by * BN;

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
  unsigned woff[IWW];
#pragma unroll
  for (int u = 0; u < IWW; ++u) {
    const int b = (wave + NW * u) * 1024 + lane * 16;
    const int row = b / RB, pc = (b % RB) / 16;
    const int q = pc ^ ((row / G::RPB) % CPR);
    woff[u] = (unsigned)(((n0 + row) * K + q * 8) * 2);
  }
  unsigned hoff0[NHS], hoff1[TWO ? NHS : 1];
#pragma unroll
  for (int k = 0; k < NHS; ++k) {
    const int p = min(k * NW + wave, IH - 1);
    const int b = p * 1024 + lane * 16;
    const int r = min(b / RB, NPX - 1), pc = (b % RB) / 16;
    const int q = pc ^ ((r >> SH) & (CPR - 1));
    // halo pixels past the grid's last input pixel read that pixel: they only
    // feed rows past the tile's count, never stored
    const int Q = min(Q0 + r, fm.Qmax);
    const int img = Q / HWin, rem = Q - img * HWin, yy = rem / Win, xx = rem - yy * Win;
    const Src& s0 = g.s[0];
    hoff0[k] = (unsigned)((((img * s0.H + yy + s0.oy) * s0.W + xx + s0.ox) * s0.C) * 2 + q * 16);
    if constexpr (TWO) {
      const Src& s1 = g.s[1];
      hoff1[k] = (unsigned)((((img * s1.H + yy + s1.oy) * s1.W + xx + s1.ox) * s1.C) * 2 + q * 16);
    }
  }
  // ---- per-lane fragment rows: the halo index of each fragment's output pixel
  // (rows past the count repeat the last pixel) ----
  const int hh = lane >> 5, ll = lane & 31;
  int rq[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) rq[i] = qin(P0 + min((wm * TM + i) * 32 + ll, cnt - 1)) - Q0;
  unsigned yb[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    yb[s] = (unsigned)((wn * TN * 32 + ll) * RB + 16 * ((2 * s + hh) ^ ((ll / G::RPB) % CPR)));

  const int nk_all = Cg / CK;
  int kc0 = 0, kc1 = nk_all;
  if (args.ksplit > 1) {
    const int per = (nk_all + args.ksplit - 1) / args.ksplit;
    kc0 = bz * per;
    kc1 = min(nk_all, kc0 + per);
  }

  auto issue_w = [&](int c, int t, int slot) {
    const unsigned long long base = uniform_u64(args.bh + (size_t)t * Cg + (size_t)c * CK);
#pragma unroll
    for (int u = 0; u < IWW; ++u) dma_sv(woff[u], base, lds0 + slot * WSZ + (wave + NW * u) * 1024);
  };
  auto issue_w1 = [&](int c, int t, int slot, int u) {
    const unsigned long long base = uniform_u64(args.bh + (size_t)t * Cg + (size_t)c * CK);
    dma_sv(woff[u], base, lds0 + slot * WSZ + (wave + NW * u) * 1024);
  };
  auto issue_h = [&](int c, int k, int hs) {
    const int c0 = c * CK;
    const bool second = TWO && c0 >= g.c_split;
    const Src& s = second ? g.s[1] : g.s[0];
    const int cl = second ? c0 - g.c_split : c0;
    const unsigned long long base = uniform_u64(reinterpret_cast<const uint16_t*>(s.ptr) + cl);
    const unsigned off = second ? hoff1[TWO ? k : 0] : hoff0[k];
    dma_sv(off, base, hs < 0 ? lds0 + (unsigned)G::JNK : lds0 + H0 + hs * HSZ + min(k * NW + wave, IH - 1) * 1024);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // one tap step: the fragment rows moved by the tap's offset, then KS k-steps
  // of TM x TN MFMAs (the next k-step's fragments read during this one's)
  auto tap_mfma = [&](auto HSc, auto Tc, auto&& after) {
    constexpr int hs = decltype(HSc)::value, t = decltype(Tc)::value;
    constexpr int ky = t / 3, kx = t % 3, ws = t % 3;
    const int dlt = ky * Win + kx;
    unsigned fab[TM];
    int hv[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // opaque per tap: the rows of all 18 (slot, tap) steps hoisted out of the
      // chunk loop would not fit the register file
      int rv = rq[i];
      asm volatile("" : "+v"(rv));
      const int r = rv + dlt;
      fab[i] = (unsigned)(H0 + hs * HSZ + r * RB);
      hv[i] = hh ^ ((r >> SH) & (CPR - 1));
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
        const uint4 u = *pv;
        *pv = bf16pack8(affine_relu4(bf16x4_to_f4(make_uint2(u.x, u.y)), ld4(sc), ld4(sh)),
                        affine_relu4(bf16x4_to_f4(make_uint2(u.z, u.w)), ld4(sc + 4), ld4(sh + 4)));
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
        for (int u = 0; u < D; ++u) {
          if (u == k || (k == KS - 1 && u > k)) {
            if (u < IWW) issue_w1(cw, tw, (t + 2) % 3, u);
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
  float* red = reinterpret_cast<float*>(lds);
  constexpr bool kStage = TN == 2 && (size_t)NW * 4096 + (size_t)WM * 3 * BN * 4 <= G::smem;
  unsigned short* stage = nullptr;
  if constexpr (kStage) {
    stage = reinterpret_cast<unsigned short*>(lds);
    red = reinterpret_cast<float*>(lds + NW * 4096);
  }
  igemm_finish<BM, BN, WM, WN, NT, LinearRows, 1>(args, acc, P0, n0, wm, wn, tid, red, LinearRows{P0, P0 + cnt},
                                                  stage, bz);
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
  fm.Hin = (int)Hin;
  fm.Win = (int)Win;
  fm.Qmax = (int)(g.nimg * Hin * Win - 1);
  long long worst = 0;
  const long long nt = (M + BM - 1) / BM;
  for (long long t = 0; t < nt; ++t) worst = std::max(worst, span(t * BM, std::min<long long>(BM, M - t * BM)));
  if (worst <= npx) {
    fm.tpi = 0;
    ntiles = nt;
    return true;
  }
  const long long tpi = (HW + BM - 1) / BM;
  worst = 0;
  for (long long t = 0; t < tpi; ++t) worst = std::max(worst, span(t * BM, std::min<long long>(BM, HW - t * BM)));
  if (worst > npx) return false;
  fm.tpi = (int)tpi;
  ntiles = g.nimg * tpi;
  return true;
}

size_t flat_smem(const IgemmArgs& a, bool xtf) {
  const Gather& g = a.a;
  return FlatGeo<kFlatTH, kFlatBN, kFlatCK, kFlatNPX>::smem +
         (xtf ? 8 * (size_t)(g.c_split < g.Cg ? g.c_split : g.Cg) : 0);
}

size_t src_bytes(const Src& s, int nimg) { return (size_t)nimg * s.H * s.W * s.C * 2; }

}  // namespace

bool conv3_flat_fits(const IgemmArgs& a, int tile) {
  if (tile != 85) return false;
  const Gather& g = a.a;
  const bool two = g.c_split < g.Cg, xtf = g.s[0].scale != nullptr;
  FlatMap fm;
  long long nt;
  return a.bh != nullptr && a.bl == nullptr && a.N % kFlatBN == 0 && g.taps_h == 3 && g.taps_w == 3 &&
         g.stride == 1 && a.K == 9 * g.Cg && g.Cg % kFlatCK == 0 && g.c_split % kFlatCK == 0 && g.s[0].h16 &&
         (!two || (g.s[1].h16 && g.s[1].scale == nullptr)) && (!xtf || g.s[0].shift != nullptr) &&
         flat_smem(a, xtf) <= 160 * 1024 && src_bytes(g.s[0], g.nimg) < (1ull << 32) &&
         (!two || src_bytes(g.s[1], g.nimg) < (1ull << 32)) && (size_t)a.N * a.K * 2 < (1ull << 32) &&
         flat_map(g, a.M, kFlatTH * 32, kFlatNPX, fm, nt);
}

long long conv3_flat_tiles(const IgemmArgs& a) {
  FlatMap fm;
  long long nt = 0;
  if (!flat_map(a.a, a.M, kFlatTH * 32, kFlatNPX, fm, nt)) return 0;
  return nt * (a.N / kFlatBN);
}

hipError_t go_conv3_flat_tile(const IgemmArgs& a, hipStream_t s, int tile) {
  if (!conv3_flat_fits(a, tile)) return hipErrorInvalidValue;
  constexpr int TH = kFlatTH, BN = kFlatBN, CK = kFlatCK, NPX = kFlatNPX, WM = 4, WN = 2, MINW = 2;
  const Gather& g = a.a;
  FlatMap fm;
  long long nt;
  flat_map(g, a.M, TH * 32, NPX, fm, nt);
  const bool two = g.c_split < g.Cg, xtf = g.s[0].scale != nullptr;
  const int v = (two ? 1 : 0) | (xtf ? 2 : 0);
  static bool attr[4] = {false, false, false, false};
  const void* fns[4] = {reinterpret_cast<const void*>(&k_conv3_flat<TH, BN, WM, WN, CK, NPX, 0, MINW, 0>),
                        reinterpret_cast<const void*>(&k_conv3_flat<TH, BN, WM, WN, CK, NPX, 1, MINW, 0>),
                        reinterpret_cast<const void*>(&k_conv3_flat<TH, BN, WM, WN, CK, NPX, 0, MINW, 1>),
                        reinterpret_cast<const void*>(&k_conv3_flat<TH, BN, WM, WN, CK, NPX, 1, MINW, 1>)};
  if (!attr[v]) {
    hipError_t e = hipFuncSetAttribute(fns[v], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr[v] = true;
  }
  const size_t smem = flat_smem(a, xtf);
  dim3 grid((unsigned)nt, a.N / BN, a.ksplit > 1 ? a.ksplit : 1);
  switch (v) {
    case 0: hipLaunchKernelGGL((k_conv3_flat<TH, BN, WM, WN, CK, NPX, 0, MINW, 0>), grid, dim3(WM * WN * 64), smem, s, a, fm); break;
    case 1: hipLaunchKernelGGL((k_conv3_flat<TH, BN, WM, WN, CK, NPX, 1, MINW, 0>), grid, dim3(WM * WN * 64), smem, s, a, fm); break;
    case 2: hipLaunchKernelGGL((k_conv3_flat<TH, BN, WM, WN, CK, NPX, 0, MINW, 1>), grid, dim3(WM * WN * 64), smem, s, a, fm); break;
    default: hipLaunchKernelGGL((k_conv3_flat<TH, BN, WM, WN, CK, NPX, 1, MINW, 1>), grid, dim3(WM * WN * 64), smem, s, a, fm); break;
  }
  return hipGetLastError();
}

}  // namespace unet
