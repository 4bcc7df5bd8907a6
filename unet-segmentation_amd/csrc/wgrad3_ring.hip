// k_wgrad3_ring: bf16 weight gradient of a 3x3 stride-1 conv,
//   dW[co][tap][ci] = sum_p dY[p][co] * X[p + tap][ci]      (fp32 accumulation)
// with every operand byte staged by LDS-DMA through a 4-slot ring of pixel
// tiles (the structure of k_conv3_ring carried over to the
// weight gradient).
//
// k_wgrad3_bf (igemm_bf16.hip) stages each pixel tile through VGPRs (per-lane
// address arithmetic, BN+ReLU and packing per staged element, two barriers per
// tile, one staging buffer) and ran at ~27 % MFMA busy.  Here:
//  * a workgroup owns BCO output channels (co) x BCI input channels (ci) x all
//    9 taps and walks TH x TW output-pixel tiles (tile z, z + gz, ... of the
//    pixel split blockIdx.z); per tile the dY tile [TH*TW][BCO] and the X halo
//    [(TH+2)(TW+2)][BCI] are DMA'd (global_load_lds_dwordx4) straight into one
//    ring slot, three tiles ahead of the one being multiplied: one barrier per
//    tile, counted vmcnt (never 0 in the loop);
//  * dY pixels past the output grid read a zero pixel of the padded dY buffer's
//    border (so they add nothing), X halo pixels past the input grid read a
//    clamped in-range pixel (they only meet those zero dY pixels);
//  * an X source with a consumer transform (relu(bn(y)) of the producer, bf16
//    storage) is transformed in LDS, in place, one tile ahead (after its DMA
//    landed, before the barrier that releases it to the MFMAs);
//  * the MFMA k is the pixel: both LDS images are [pixel][channels] rows and
//    the operands come out transposed with ds_read_b64_tr_b16, as in
//    k_wgrad3_bf; 16-B chunks are XOR-swizzled inside a row (by row bits 1 for
//    128-B rows, by row & 3 on 64-B segments for 256-B rows) on the DMA source
//    address, so every transposed read of 4 consecutive pixel rows is
//    conflict-free at any tap offset;
//  * every LDS read address is a per-lane register computed once plus a
//    compile-time immediate (slot, k-step, tap): no address VALU in the loop.
// Waves (8), two mappings:
//  * TMC >= 1 (tap groups): tap group tg = wave >> 2 (taps 0-4 / 5-8; the two
//    waves sharing a SIMD get one group each), then NCI ci tiles x NCO co groups
//    of TMC 32-channel co tiles; a wave holds TMC x 5 (or 4) 32x32 accumulators;
//  * TMC == 0 ("slide", TW = 16): a wave owns one 32 co x 32 ci block and all 9
//    taps (9 accumulators).  A k-step is one tile row, so the B fragment of tap
//    (ky, kx) at k-step ks is the halo row ks + ky: each halo row's fragment is
//    read once per kx and feeds the three (ks, ky) pairs that meet it -- per
//    tile 2 TH + 6 (TH + 2) transposed reads for 9 TH MFMAs (1.2 per MFMA at
//    TH = 4, against 2.3 with tap groups, whose LDS issue stalls bound them).
// Each wave adds its accumulators into the packed weight gradient
// out[co][tap * Ci + ci] with fp32 atomics once.
#include "gemm_common.h"
#include "ring_common.h"

#include <algorithm>

namespace unet {

typedef __bf16 bf16x8w_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4w_t __attribute__((ext_vector_type(4)));
typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 lds_bf16x4w_t;

__device__ __forceinline__ bf16x4w_t tr_read4(unsigned addr) {
  auto q = (__attribute__((address_space(3))) lds_bf16x4w_t*)(size_t)addr;
  return __builtin_bit_cast(bf16x4w_t, __builtin_amdgcn_ds_read_tr16_b64_v4bf16(q));
}

// LDS position of logical 16-B chunk c in pixel row `row` (an involution in c)
template <int RB>
__host__ __device__ constexpr int rswz(int row, int c) {
  if constexpr (RB == 128) return c ^ (((row >> 1) & 1) << 2);
  else return (((c >> 2) ^ (row & 3)) << 2) | (c & 3);
}

template <int TH, int TW, int BCO, int BCI>
struct WRGeo {
  static constexpr int RA = BCO * 2, RX = BCI * 2, HW2 = TW + 2;
  static constexpr int PT = TH * TW, PH = (TH + 2) * HW2;
  static constexpr int NDA = PT * RA / 1024;             // dY DMA instructions per tile
  static constexpr int NDX = (PH * RX + 1023) / 1024;    // X halo DMA instructions per tile
  static constexpr int ASZ = NDA * 1024, SSZ = ASZ + NDX * 1024;
  static constexpr int NS = 4;                           // ring slots
  static constexpr size_t smem = (size_t)NS * SSZ + 2 * BCI * 4;
};

// compile-time part of a pixel's tile coordinates for k-step ks, lane row
// offset r4 (0 / 4): tile row py_c and column px_c (the lane adds its own)
template <int TW>
__host__ __device__ constexpr int wr_pyc(int ks) { return TW == 16 ? ks : TW == 8 ? 2 * ks : ks >> 1; }
template <int TW>
__host__ __device__ constexpr int wr_pxc(int ks, int r4) { return TW == 32 ? 16 * (ks & 1) + r4 : r4; }

template <int TH, int TW, int BCO, int BCI, int TMC, int XTF>
__global__ __launch_bounds__(512, 1) void k_wgrad3_ring(const WgradArgs args, int cblk0) {
  using G = WRGeo<TH, TW, BCO, BCI>;
  constexpr int RA = G::RA, RX = G::RX, HW2 = G::HW2, PT = G::PT, PH = G::PH;
  constexpr int NDA = G::NDA, NDX = G::NDX, ASZ = G::ASZ, SSZ = G::SSZ, NS = G::NS;
  constexpr bool SLIDE = TMC == 0;
  constexpr int TMC1 = SLIDE ? 1 : TMC, NACC = SLIDE ? 9 : 5;
  constexpr int NCI = BCI / 32, NCO = BCO / (32 * TMC1);
  static_assert(NCI * NCO * (SLIDE ? 1 : 2) == 8, "8 waves: (2 tap groups x) ci tiles x co groups");
  static_assert(!SLIDE || TW == 16, "slide mode: one tile row per k-step");
  static_assert(TW == 8 || TW == 16 || TW == 32, "tile width");
  static_assert(NDA % 8 == 0, "dY DMA instructions spread evenly over the waves");
  constexpr int DA = NDA / 8, DX = (NDX + 7) / 8, D = DA + DX;  // DMAs per wave per tile
  constexpr int KS = PT / 16;                                    // 16-pixel k-steps per tile
  constexpr int RPA = 1024 / RA, RPX = 1024 / RX;                // pixel rows per DMA instruction
  constexpr int LPA = RA / 16, LPX = RX / 16;                    // lanes per pixel row
  extern __shared__ __attribute__((aligned(1024))) unsigned char lds[];
  const unsigned lds0 = (unsigned)(size_t)(lds_u8_t*)lds;
  float* ssc = reinterpret_cast<float*>(lds + NS * SSZ);  // [2][BCI]: BN scale, shift of X

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tg = SLIDE ? 0 : wave >> 2, wr = SLIDE ? wave : wave & 3, ct = wr % NCI, cg = wr / NCI;
  int bx, by, bz;  // grid position in XCD-aware order (a pixel split's operand slices stay in one L2)
  xcd_block(bx, by, bz);
  const int i0 = bx * BCO, cb = (by + cblk0) * BCI;
  const Gather& gb = args.gb;
  const Src& ds = args.ga.s[0];
  const int Hg = gb.Hg, Wg = gb.Wg, Ci = gb.Cg;
  // X source of this ci block (a block never straddles the concat split), picked
  // field by field (a run-time index into the argument array goes to scratch)
  const bool second = cb >= gb.c_split;
  const uint16_t* xptr = reinterpret_cast<const uint16_t*>(second ? gb.s[1].ptr : gb.s[0].ptr);
  const int xH = second ? gb.s[1].H : gb.s[0].H, xW = second ? gb.s[1].W : gb.s[0].W;
  const int xC = second ? gb.s[1].C : gb.s[0].C;
  const int xoy = second ? gb.s[1].oy : gb.s[0].oy, xox = second ? gb.s[1].ox : gb.s[0].ox;
  const int xc = second ? cb - gb.c_split : cb;
  if constexpr (XTF) {
    const float* sc = second ? gb.s[1].scale : gb.s[0].scale;
    const float* sh = second ? gb.s[1].shift : gb.s[0].shift;
    for (int c = tid; c < BCI; c += 512) {
      ssc[c] = sc[xc + c];
      ssc[BCI + c] = sh[xc + c];
    }
  }
  const int tiles_x = (Wg + TW - 1) / TW, tiles_y = (Hg + TH - 1) / TH;
  const int tiles = gb.nimg * tiles_x * tiles_y;
  const int z = bz, gz = gridDim.z;
  const int cnt = z < tiles ? (tiles - z + gz - 1) / gz : 0;
  if (cnt == 0) return;

  // ---- per-lane DMA constants ----
  const unsigned long long abase = uniform_u64(ds.ptr), xbase = uniform_u64(xptr);
  const int dH = ds.H, dW = ds.W, dC = ds.C;
  int a_ty[DA], a_tx[DA];
  unsigned a_rel[DA], a_zero[DA];
#pragma unroll
  for (int u = 0; u < DA; ++u) {
    const int row = (wave + 8 * u) * RPA + lane / LPA;
    const int c = rswz<RA>(row, lane % LPA);
    a_ty[u] = row / TW;
    a_tx[u] = row % TW;
    a_rel[u] = (unsigned)(((a_ty[u] + ds.oy) * dW + a_tx[u] + ds.ox) * dC + i0 + c * 8);
    a_zero[u] = (unsigned)(i0 + c * 8);  // pixel (0, 0) of the padded buffer: zero border
  }
  int x_hy[DX], x_hx[DX], x_c[DX];
#pragma unroll
  for (int u = 0; u < DX; ++u) {
    const int j = min(wave + 8 * u, NDX - 1);
    const int hp = min(j * RPX + lane / LPX, PH - 1);
    x_c[u] = xc + rswz<RX>(hp, lane % LPX) * 8;
    x_hy[u] = hp / HW2;
    x_hx[u] = hp % HW2;
  }
  // local tile i (tile z + i * gz; past the end: the last one again, so every
  // wave always has D DMAs per tile in flight) -> ring slot i % NS
  struct TileRef {
    unsigned slot, zrow;
    int arow, y0, x0, n;
  };
  auto tile_ref = [&](int i) {
    const int t = z + min(i, cnt - 1) * gz;
    const int tx0 = t % tiles_x, r = t / tiles_x;
    TileRef T;
    T.y0 = (r % tiles_y) * TH;
    T.x0 = tx0 * TW;
    T.n = r / tiles_y;
    T.slot = lds0 + (unsigned)((i % NS) * SSZ);
    T.arow = (T.n * dH + T.y0) * dW + T.x0;  // + the lane's pixel and the origin in a_rel
    T.zrow = (unsigned)(T.n * dH * dW * dC);
    return T;
  };
  // DMA u (0 .. D-1: the dY pieces, then the X halo pieces) of tile T
  auto dma_piece = [&](const TileRef& T, int u) {
    if (u < DA) {
      const bool ok = a_ty[u] < Hg - T.y0 && a_tx[u] < Wg - T.x0;
      // select by mask: a plain ?: between the two lane arrays was turned into
      // a select of their addresses (the arrays then live in scratch)
      const unsigned v = (unsigned)(T.arow * dC) + a_rel[u], zv = T.zrow + a_zero[u];
      const unsigned off = zv ^ ((v ^ zv) & (0u - (unsigned)ok));
      dma_sv(off * 2u, abase, T.slot + (wave + 8 * u) * 1024);
    } else {
      const int k = u - DA;
      const int yy = min(T.y0 + x_hy[k], Hg + 1), xx = min(T.x0 + x_hx[k], Wg + 1);
      const unsigned off = (unsigned)(((T.n * xH + yy + xoy) * xW + xx + xox) * xC + x_c[k]);
      dma_sv(off * 2u, xbase, T.slot + ASZ + min(wave + 8 * k, NDX - 1) * 1024);
    }
  };
  auto issue = [&](int i) {
    const TileRef T = tile_ref(i);
#pragma unroll
    for (int u = 0; u < D; ++u) dma_piece(T, u);
  };

  // ---- in-LDS BN+ReLU of a slot's X halo (XTF) ----
  constexpr int XP = PH * RX / 16, NXP = (XP + 511) / 512;  // 16-B pieces, per thread
  float4 tsc0, tsc1, tsh0, tsh1;
  if constexpr (XTF) {
    __syncthreads();  // scale / shift table
    // a thread's pieces tid + 512k keep their logical chunk (the swizzle bits of
    // their rows agree), so its 8 channels' coefficients are loaded once
    const int row = tid / LPX, c = rswz<RX>(row, tid % LPX);
    tsc0 = ld4(ssc + c * 8);
    tsc1 = ld4(ssc + c * 8 + 4);
    tsh0 = ld4(ssc + BCI + c * 8);
    tsh1 = ld4(ssc + BCI + c * 8 + 4);
  }
  auto transform = [&](int i) {
    unsigned char* xs = lds + (i % NS) * SSZ + ASZ;
#pragma unroll
    for (int k = 0; k < NXP; ++k) {
      const int p = tid + 512 * k;
      if (p < XP) {
        uint4* q = reinterpret_cast<uint4*>(xs + p * 16);
        const uint4 u = *q;
        // bf16 -> fp32 (exact), relu(v * scale + shift), RNE back to bf16: the
        // consumer transform of the register-staged kernels (stage8)
        *q = bf16pack8(affine_relu4(bf16x4_to_f4(make_uint2(u.x, u.y)), tsc0, tsh0),
                       affine_relu4(bf16x4_to_f4(make_uint2(u.z, u.w)), tsc1, tsh1));
      }
    }
  };

  // ---- per-lane LDS read offsets (bytes within a slot) ----
  const int g16 = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3, hk = g16 >> 1, half = g16 & 1;
  unsigned aoff[TMC1];
#pragma unroll
  for (int i = 0; i < TMC1; ++i) {
    const int col = cg * 32 * TMC1 + i * 32 + half * 16 + pp * 4;
    const int rowl = 8 * hk + q;
    aoff[i] = (unsigned)(rowl * RA + rswz<RA>(rowl, col >> 3) * 16 + (col & 7) * 2);
  }
  const int pyl = TW == 8 ? hk : 0, pxl = TW == 8 ? q : 8 * hk + q;
  const unsigned boff = (unsigned)(ASZ + (HW2 * pyl + pxl) * RX);
  unsigned sw[2][3];
  {
    const int col = ct * 32 + half * 16 + pp * 4;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        // a row congruent (mod 4) to every halo row this lane reads at parity p, tap column kx
        const int rrep = 2 * ((p + pyl) & 1) + kx + pxl;
        sw[p][kx] = (unsigned)(rswz<RX>(rrep, col >> 3) * 16 + (col & 7) * 2);
      }
  }

  floatx16 acc[TMC1][NACC];
#pragma unroll
  for (int i = 0; i < TMC1; ++i)
#pragma unroll
    for (int j = 0; j < NACC; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // one tile from slot S, taps TG*5 .. : KS k-steps of TMC x NT MFMAs; the
  // fragments of k-step ks + 1 are read (into the other register buffer)
  // before k-step ks's MFMAs issue, so LDS latency hides behind them
  auto compute = [&](auto Sc, auto TGc, auto&& after) {
    constexpr int S = decltype(Sc)::value, TG = decltype(TGc)::value;
    constexpr int T0 = TG * 5, NT = TG ? 4 : 5;
    const unsigned sbase = lds0 + S * SSZ;
    bf16x8w_t fa[2][TMC1], fb[2][NT];  // TMC == 1 only (below)
    auto rd = [&](auto KSc) {
      constexpr int ks = decltype(KSc)::value, b = ks & 1;
#pragma unroll
      for (int i = 0; i < TMC1; ++i) {
        const bf16x4w_t a0 = tr_read4(sbase + aoff[i] + (16 * ks) * RA);
        const bf16x4w_t a1 = tr_read4(sbase + aoff[i] + (16 * ks + 4) * RA);
        fa[b][i] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int tap = T0 + j, ky = tap / 3, kx = tap % 3;
        const int pyc = wr_pyc<TW>(ks) + ky;
        const unsigned b0 = sbase + boff + sw[pyc & 1][kx] + (HW2 * pyc + wr_pxc<TW>(ks, 0) + kx) * RX;
        const unsigned b1 = sbase + boff + sw[pyc & 1][kx] + (HW2 * pyc + wr_pxc<TW>(ks, 4) + kx) * RX;
        fb[b][j] = __builtin_shufflevector(tr_read4(b0), tr_read4(b1), 0, 1, 2, 3, 4, 5, 6, 7);
      }
    };
    auto mm = [&](auto KSc) {
      constexpr int ks = decltype(KSc)::value, b = ks & 1;
      if constexpr (ks + 1 < KS) rd(std::integral_constant<int, ks + 1>{});
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < TMC1; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[b][i], fb[b][j], acc[i][j], 0, 0, 0);
      after(ks);
    };
    if constexpr (TMC > 1) {
      // two co tiles per wave: no register room for a second fragment buffer;
      // each tap's B fragment is read right before its two MFMAs
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8w_t a[TMC];
#pragma unroll
        for (int i = 0; i < TMC; ++i)
          a[i] = __builtin_shufflevector(tr_read4(sbase + aoff[i] + (16 * ks) * RA),
                                         tr_read4(sbase + aoff[i] + (16 * ks + 4) * RA), 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int tap = T0 + j, ky = tap / 3, kx = tap % 3;
          const int pyc = wr_pyc<TW>(ks) + ky;
          const unsigned b0 = sbase + boff + sw[pyc & 1][kx] + (HW2 * pyc + wr_pxc<TW>(ks, 0) + kx) * RX;
          const unsigned b1 = sbase + boff + sw[pyc & 1][kx] + (HW2 * pyc + wr_pxc<TW>(ks, 4) + kx) * RX;
          const bf16x8w_t b = __builtin_shufflevector(tr_read4(b0), tr_read4(b1), 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
          for (int i = 0; i < TMC; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b, acc[i][j], 0, 0, 0);
        }
        after(ks);
      }
      return;
    }
    rd(std::integral_constant<int, 0>{});
    mm(std::integral_constant<int, 0>{});
    if constexpr (KS > 1) mm(std::integral_constant<int, 1>{});
    if constexpr (KS > 2) mm(std::integral_constant<int, 2>{});
    if constexpr (KS > 3) mm(std::integral_constant<int, 3>{});
    if constexpr (KS > 4) mm(std::integral_constant<int, 4>{});
    if constexpr (KS > 5) mm(std::integral_constant<int, 5>{});
    if constexpr (KS > 6) mm(std::integral_constant<int, 6>{});
    if constexpr (KS > 7) mm(std::integral_constant<int, 7>{});
    static_assert(KS <= 8, "k-steps per tile");
  };

  // slide mode: one tile from slot S, all 9 taps; A fragments of the TH
  // k-steps (tile rows) are read once, then per tap column kx the halo rows
  // r = 0 .. TH+1 in order, each feeding MFMAs (ks = r - ky, ky) for ky = 0..2;
  // the next row's fragment is read before the current row's MFMAs issue
  auto compute_slide = [&](auto Sc, auto&& after) {
    constexpr int S = decltype(Sc)::value;
    const unsigned sbase = lds0 + S * SSZ;
    bf16x8w_t fa[TH];
#pragma unroll
    for (int ks = 0; ks < TH; ++ks)
      fa[ks] = __builtin_shufflevector(tr_read4(sbase + aoff[0] + (16 * ks) * RA),
                                       tr_read4(sbase + aoff[0] + (16 * ks + 4) * RA), 0, 1, 2, 3, 4, 5, 6, 7);
    auto rdb = [&](int kx, int r) {
      const unsigned b0 = sbase + boff + sw[r & 1][kx] + (HW2 * r + kx) * RX;
      const unsigned b1 = sbase + boff + sw[r & 1][kx] + (HW2 * r + 4 + kx) * RX;
      return (bf16x8w_t)__builtin_shufflevector(tr_read4(b0), tr_read4(b1), 0, 1, 2, 3, 4, 5, 6, 7);
    };
    bf16x8w_t b = rdb(0, 0);
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int r = 0; r < TH + 2; ++r) {
        bf16x8w_t bn = b;
        if (r + 1 < TH + 2) bn = rdb(kx, r + 1);
        else if (kx < 2) bn = rdb(kx + 1, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int ks = r - ky;
          if (ks >= 0 && ks < TH)
            acc[0][ky * 3 + kx] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks], b, acc[0][ky * 3 + kx], 0, 0, 0);
        }
        after(kx * (TH + 2) + r);
        b = bn;
      }
  };

  // ring step for local tile i in slot S: wait for this wave's DMAs of the tile
  // the step needs (XTF: tile i + 1, to transform it; else tile i), barrier
  // (everyone's landed; everyone is done with tile i - 1, whose slot is
  // refilled next), issue tile i + 3, transform tile i + 1, multiply tile i
  auto step = [&](auto Sc, int i) {
    if constexpr (XTF) vm_wait<D>();
    else vm_wait<2 * D>();
    raw_barrier();
    if constexpr (XTF) {
      if (i + 1 < cnt) transform(i + 1);
    }
    // tile i + 3's DMAs go out one per k-step between the MFMAs (issued all at
    // once after the barrier they held every wave of the CU in its DMA phase
    // together, with the matrix pipes idle)
    const TileRef T = tile_ref(i + 3);
    constexpr int KLAST = SLIDE ? 3 * (TH + 2) - 1 : KS - 1;  // index of the last k-step callback
    auto after = [&](int k) {
      if (k < D) dma_piece(T, k);
      if (k == KLAST)  // fewer k-steps than DMAs: the rest after the last one
#pragma unroll
        for (int u = KLAST + 1; u < D; ++u) dma_piece(T, u);
    };
    if constexpr (SLIDE) compute_slide(Sc, after);
    else if (tg == 0) compute(Sc, std::integral_constant<int, 0>{}, after);
    else compute(Sc, std::integral_constant<int, 1>{}, after);
  };

  issue(0);
  issue(1);
  issue(2);
  if constexpr (XTF) {
    vm_wait<2 * D>();
    raw_barrier();
    transform(0);
  }
  for (int i = 0; i < cnt; i += NS) {
    step(std::integral_constant<int, 0>{}, i);
    if (i + 1 < cnt) step(std::integral_constant<int, 1>{}, i + 1);
    if (i + 2 < cnt) step(std::integral_constant<int, 2>{}, i + 2);
    if (i + 3 < cnt) step(std::integral_constant<int, 3>{}, i + 3);
  }
  vm_wait<0>();  // the tail's re-issued DMAs land before the workgroup exits

  // accumulate into out[co][tap * Ci + ci]: fp32 atomics, one per element per
  // workgroup, or (slab mode) this split's partial into its slab plane with
  // plain stores, summed into out by k_wr_reduce
  const int h = lane >> 5, li = lane & 31;
  const int t0 = tg * 5, nt = SLIDE ? 9 : tg ? 4 : 5;
  float* const plane = args.slab ? args.slab + (size_t)bz * args.Mo * args.No : nullptr;
#pragma unroll
  for (int i = 0; i < TMC1; ++i)
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      if (j < nt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = i0 + cg * 32 * TMC1 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int col = (t0 + j) * Ci + cb + ct * 32 + li;
          if (plane) plane[(size_t)row * args.No + col] = acc[i][j][r];
          else atomicAdd(args.out + (size_t)row * args.No + col, acc[i][j][r]);
        }
      }
    }
}

// out[b][e] = sum over the splits of slab[b * splits + z][e] (slab-mode weight
// gradients: every element of every plane is written by the splits, so the
// sum is assigned -- out needs no zeroing)
// The planes of a small layer are few float4s but many (a 64 x 576 plane over
// 512 splits: 9216 float4s): the 2^ls threads of an element each take every
// 2^ls-th split with 8 independent loads in flight, then combine through LDS,
// so such a plane still spreads over hundreds of workgroups instead of 36
// workgroups of 512-deep load chains.
__global__ __launch_bounds__(256) void k_wr_reduce(const float* __restrict__ slab, int splits, int batch,
                                                   long long n4, long long out4, int ls, float* __restrict__ out) {
  __shared__ float4 red[256];
  const int E = 256 >> ls, el = threadIdx.x & (E - 1), sl = threadIdx.x >> (8 - ls), S = 1 << ls;
  const long long total = (long long)batch * n4;
  for (long long i0 = (long long)blockIdx.x * E; i0 < total; i0 += (long long)gridDim.x * E) {
    const long long i = i0 + el;
    float4 acc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < total) {
      const long long b = i / n4, e = i - b * n4;
      const float4* src = reinterpret_cast<const float4*>(slab) + (size_t)b * splits * n4 + e;
      int z = sl;
      for (; z + 7 * S < splits; z += 8 * S) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(z + u * S) * n4];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
        }
      }
      for (; z < splits; z += S) {
        const float4 v = src[(size_t)z * n4];
        acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
      }
#pragma unroll
      for (int u = 1; u < 8; ++u) {
        acc[0].x += acc[u].x; acc[0].y += acc[u].y; acc[0].z += acc[u].z; acc[0].w += acc[u].w;
      }
    }
    red[threadIdx.x] = acc[0];
    __syncthreads();
    if (sl == 0 && i < total) {
      float4 t = red[el];
      for (int q = 1; q < S; ++q) {
        const float4 v = red[q * E + el];
        t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
      }
      const long long b = i / n4, e = i - b * n4;
      reinterpret_cast<float4*>(out)[b * out4 + e] = t;
    }
    __syncthreads();
  }
}

hipError_t launch_slab_reduce(const float* slab, int splits, int batch, size_t plane, long long batch_out, float* out,
                              hipStream_t s) {
  if (plane % 4 != 0 || splits < 1 || batch < 1 || (batch > 1 && batch_out % 4 != 0)) return hipErrorInvalidValue;
  const long long n4 = (long long)(plane / 4), tot = n4 * batch;
  // split slices per element: enough threads for ~2 workgroups of 256 per CU,
  // at least 8 splits per thread, at most 16 slices
  int ls = 0;
  while (ls < 4 && (tot << ls) < 2ll * 256 * num_cus() && (splits >> (ls + 1)) >= 8) ++ls;
  const long long E = 256 >> ls;
  hipLaunchKernelGGL(k_wr_reduce, dim3((unsigned)std::min<long long>((tot + E - 1) / E, 8192)), dim3(256), 0, s,
                     slab, splits, batch, n4, batch > 1 ? batch_out / 4 : n4, ls, out);
  return hipGetLastError();
}

// wgrad tiles 26-29 (igemm.hip wgrad_tile_fits / launch_wgrad_v):
//   26: 128 co x 64 ci, 4 x 16 px tiles   27: 128 co x 64 ci, 8 x 8 px tiles
//   28:  64 co x 64 ci, 4 x 16 px tiles   29:  64 co x 128 ci, 4 x 16 px tiles
//   30:  64 co x 64 ci, 8 x 16 px tiles   31:  64 co x 64 ci, 8 x 8 px tiles
//   32: slide, 128 co x 64 ci, 4 x 16 px  33: slide, 64 co x 128 ci, 4 x 16 px
bool wgrad3_ring_fits(const WgradArgs& a, int tile) {
  const Gather& g = a.gb;
  const int bco = tile == 26 || tile == 27 || tile == 32 ? 128 : 64, bci = tile == 29 || tile == 33 ? 128 : 64;
  if (tile < 26 || tile > 33 || !a.bf16 || a.split) return false;
  const Src& d = a.ga.s[0];
  const bool two = g.c_split < g.Cg;
  // dY: the zero-bordered padded buffer (bf16); X sources bf16, with or without
  // a consumer transform (all of a block's channels from one source)
  // 32-bit DMA offsets: every operand tensor below 4 GiB
  const double dy_bytes = 2.0 * g.nimg * d.H * d.W * d.C;
  const double x_bytes = 2.0 * g.nimg * std::max(g.s[0].H * g.s[0].W * g.s[0].C, two ? g.s[1].H * g.s[1].W * g.s[1].C : 0);
  return g.taps_h == 3 && g.taps_w == 3 && g.stride == 1 && a.No == 9 * g.Cg && a.Mo % bco == 0 &&
         g.Cg % bci == 0 && (!two || g.c_split % bci == 0) && a.ga.Cg == a.Mo && a.ga.taps_h == 1 &&
         a.ga.taps_w == 1 && g.Hg == a.ga.Hg && g.Wg == a.ga.Wg && g.nimg == a.ga.nimg && d.h16 && d.oy == 2 &&
         d.ox == 2 && d.scale == nullptr && g.s[0].h16 && (!two || g.s[1].h16) && dy_bytes < 4294967296.0 &&
         x_bytes < 4294967296.0;
}

template <int TH, int TW, int BCO, int BCI, int TMC>
static hipError_t go_wr(const WgradArgs& a0, hipStream_t s, int per_cu) {
  using Gm = WRGeo<TH, TW, BCO, BCI>;
  static bool attr[2] = {false, false};
  const Gather& g = a0.gb;
  // per_cu >= 10: slab mode (per_cu - 10 workgroups per CU), when the plan's
  // slab holds every split's plane (else the atomics)
  const bool slab_mode = per_cu >= 10;
  if (slab_mode) per_cu -= 10;
  const int tiles = g.nimg * ((g.Hg + TH - 1) / TH) * ((g.Wg + TW - 1) / TW);
  const int blocks = (a0.Mo / BCO) * (g.Cg / BCI);
  int splits = (per_cu * num_cus() + blocks - 1) / blocks;
  splits = splits < 1 ? 1 : (splits > tiles ? tiles : splits);
  WgradArgs a = a0;
  const size_t plane = (size_t)a.Mo * a.No;
  const bool use_slab = slab_mode && a.slab && !a.accumulate && (size_t)splits * plane * sizeof(float) <= a.slab_bytes &&
                        splits > 1 && plane % 4 == 0;
  // (a single split adds each element once onto the zeroed gradient: order-free)
  if (slab_mode && splits > 1 && !use_slab) ++g_slab_fallbacks;
  if (!use_slab) a.slab = nullptr;
  const dim3 grid(a.Mo / BCO, g.Cg / BCI, splits);
  // X transform per launch: the sources of the two concat halves may differ
  // (relu(bn(skip)) vs the plain convT output), so a block picks its kernel by
  // its own source; launch both halves separately when they differ
  const bool t0 = g.s[0].scale != nullptr, two = g.c_split < g.Cg;
  const bool t1 = two && g.s[1].scale != nullptr;
  auto launch = [&](bool tf, int cblk0, dim3 gr) -> hipError_t {
    const void* fn = tf ? reinterpret_cast<const void*>(&k_wgrad3_ring<TH, TW, BCO, BCI, TMC, 1>)
                        : reinterpret_cast<const void*>(&k_wgrad3_ring<TH, TW, BCO, BCI, TMC, 0>);
    if (!attr[tf]) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)Gm::smem);
      if (e != hipSuccess) return e;
      attr[tf] = true;
    }
    if (tf) hipLaunchKernelGGL((k_wgrad3_ring<TH, TW, BCO, BCI, TMC, 1>), gr, dim3(512), Gm::smem, s, a, cblk0);
    else hipLaunchKernelGGL((k_wgrad3_ring<TH, TW, BCO, BCI, TMC, 0>), gr, dim3(512), Gm::smem, s, a, cblk0);
    return hipGetLastError();
  };
  hipError_t e;
  if (!two || t0 == t1) {
    e = launch(t0, 0, grid);
  } else {
    // concat with one transformed half (relu(bn(skip)) and the plain convT
    // output): the column blocks of each source as a launch of its own
    const int nb0 = g.c_split / BCI;
    e = launch(t0, 0, dim3(a.Mo / BCO, nb0, splits));
    if (e == hipSuccess) e = launch(t1, nb0, dim3(a.Mo / BCO, g.Cg / BCI - nb0, splits));
  }
  if (e != hipSuccess || !a.slab) return e;
  return launch_slab_reduce(a.slab, splits, 1, plane, 0, a.out, s);
}

hipError_t go_wgrad3_ring(const WgradArgs& a, hipStream_t s, int tile, int per_cu) {
  if (!wgrad3_ring_fits(a, tile)) return hipErrorInvalidValue;
  switch (tile) {
    case 26: return go_wr<4, 16, 128, 64, 2>(a, s, per_cu);
    case 27: return go_wr<8, 8, 128, 64, 2>(a, s, per_cu);
    case 28: return go_wr<4, 16, 64, 64, 1>(a, s, per_cu);
    case 29: return go_wr<4, 16, 64, 128, 2>(a, s, per_cu);
    case 30: return go_wr<8, 16, 64, 64, 1>(a, s, per_cu);
    case 31: return go_wr<8, 8, 64, 64, 1>(a, s, per_cu);
    case 32: return go_wr<4, 16, 128, 64, 0>(a, s, per_cu);
    case 33: return go_wr<4, 16, 64, 128, 0>(a, s, per_cu);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
