// k_wgradT_ring: bf16 weight gradient of the ConvTranspose2d(k=2, s=2) layers
// (models/unet_model.py:45), wgrad tiles 40-44:
//   C[ci][ab * Co + co] = sum_p X[p][ci] * dY[2p + ab][co]      (fp32 accumulation)
// over the input pixels p = (n, y, x) of the convT, with dY the gradient of its
// 2h x 2w output (sub-pixel ab = (a, b) at (2y + a, 2x + b)) and X the convT
// input as its consumers read it (relu(bn(y)) of the previous conv, applied in
// LDS).
//
// the register-staged pixel-column kernel k_wgrad_bf ran
// these at 9 % MFMA busy (up1's 19.3 GF in 80-97 us): per 32-pixel stage every
// lane loaded 8-B pieces of 8 pixels, transposed them in registers and wrote
// four 16-B LDS rows, two barriers per stage.  Here the structure of the bf16
// ring kernels carries over:
//  * a workgroup owns a BMO (ci) x BNO ((ab, co)) output block and walks its
//    pixel split in BK-pixel stages through an NS-slot LDS ring; each stage is
//    [BK pixel rows][BMO ci] of X and [BK pixel rows][BNO columns] of dY, both
//    copied global -> LDS by global_load_lds_dwordx4 (16-B pieces, NS - 1
//    stages in flight, counted vmcnt, one raw barrier per stage);
//  * the pixel is the MFMA k: both images are read transposed with
//    ds_read_b64_tr_b16 (two 4-pixel reads per 32x32x16 fragment, as
//    k_wgrad3_ring), 16-B chunks XOR-swizzled by row & 3 on 64-B segments
//    (rswz) on the DMA source address, so each 32-lane read group covers the 64
//    banks once;
//  * per lane the DMA source offsets are affine in the pixel (whole-grid
//    sources): a stage adds a constant for X and, for dY at (n, 2y + a, 2x + b),
//    tracks x = p mod w by one conditional subtraction -- a few VALU per piece,
//    no division or loop;
//  * X's BatchNorm + ReLU is applied in place one stage ahead of its MFMAs
//    (XTF); pixels past the split's end read a clamped valid pixel and their X
//    rows are zeroed in the same pass, so they add nothing;
//  * the splits of one pixel range sit on one XCD when the split count is a
//    multiple of 8 (its slice of X and dY then stays in that XCD's L2 for every
//    output block that reads it);
//  * each split stores its BMO x BNO partial with plain 128-B row stores into
//    the plan's weight-gradient slab; k_wr_reduce assigns their sum (one split:
//    straight into the gradient).  No fp32 atomics: deterministic.
#include "gemm_common.h"
#include "ring_common.h"

#include <algorithm>

namespace unet {

namespace {
typedef __bf16 bf16x8t_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4t_t __attribute__((ext_vector_type(4)));
typedef __attribute__((__vector_size__(4 * sizeof(__bf16)))) __bf16 lds_bf16x4t_t;

__device__ __forceinline__ bf16x4t_t tr4(unsigned addr) {
  auto q = (__attribute__((address_space(3))) lds_bf16x4t_t*)(size_t)addr;
  return __builtin_bit_cast(bf16x4t_t, __builtin_amdgcn_ds_read_tr16_b64_v4bf16(q));
}

// LDS position of logical 16-B chunk c in pixel row `row` (an involution in c):
// 64-B segments XOR row & 3 (rows of >= 256 B), 16-B chunks XOR (row >> 1) & 1
// ... for 128-B rows (as rswz in wgrad3_ring.hip)
template <int R>
__host__ __device__ constexpr int tswz(int row, int c) {
  if constexpr (R == 128) return c ^ (((row >> 1) & 1) << 2);
  else return (((c >> 2) ^ (row & 3)) << 2) | (c & 3);
}

}  // namespace

template <int BMO, int BNO, int BK, int NS>
struct WTGeo {
  static constexpr int RA = BMO * 2, RB = BNO * 2;
  static constexpr int ASZ = BK * RA, BSZ = BK * RB, SSZ = ASZ + BSZ;
  static constexpr size_t smem = (size_t)NS * SSZ + 2 * BMO * 4;  // ring + the X block's BN scale / shift
};

template <int BMO, int BNO, int WM, int WN, int BK, int NS, int XTF>
__global__ __launch_bounds__(WM * WN * 64, 1) void k_wgradT_ring(const WgradArgs args, int tiles_m, int tiles_n,
                                                                  int splits, int xcd_map) {
  using G = WTGeo<BMO, BNO, BK, NS>;
  constexpr int RA = G::RA, RB = G::RB, ASZ = G::ASZ, SSZ = G::SSZ;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int TM = BMO / (WM * 32), TN = BNO / (WN * 32);
  constexpr int NDA = G::ASZ / 1024, NDB = G::BSZ / 1024;  // DMA wave-instructions per stage
  constexpr int DA = NDA / NW, DB = NDB / NW, D = DA + DB;    // per wave
  constexpr int KS = BK / 16;                                  // 16-pixel k-steps per stage
  constexpr int P = NS - 1;                                    // stages in flight
  static_assert(TM >= 1 && TN >= 1 && NDA % NW == 0 && NDB % NW == 0 && DA >= 1 && DB >= 1, "tile");
  static_assert(NS >= 3 && D * P < 64, "ring depth / vmcnt");
  static_assert(RA >= 128 && RB >= 128, "rows of at least 128 B");
  extern __shared__ __attribute__((aligned(1024))) unsigned char lds[];
  const unsigned lds0 = (unsigned)(size_t)(lds_u8_t*)lds;
  float* ssc = reinterpret_cast<float*>(lds + (size_t)NS * SSZ);  // [2][BMO]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // workgroup -> (pixel split z, column block j, row block i).  Workgroups
  // are dealt to the 8 XCDs round robin (L % 8); with xcd_map each XCD takes a
  // contiguous run of the (z slowest, j, i fastest) enumeration instead, so it
  // holds one or two splits' slices of X and dY in its own L2 and every output
  // block it computes re-reads them from there (up1: 4.7 MB per XCD, each byte
  // fetched beyond L2 once or twice, against eight times for dY in the plain
  // order)
  const int tiles = tiles_m * tiles_n;
  int e = blockIdx.x;
  if (xcd_map) {
    const int per = (int)(gridDim.x >> 3);
    e = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  }
  const int z = e / tiles, t = e % tiles;
  const int i0 = (t % tiles_m) * BMO, j0 = (t / tiles_m) * BNO;
  const int pbeg = z * args.pix_per_split;
  const int pend = min(args.P, pbeg + args.pix_per_split);
  const int nk = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;

  const Gather& ga = args.ga;  // X: taps 1, channels = Mo
  const Gather& gb = args.gb;  // dY: 2 x 2 stride-2 taps, channels Co
  const Src& xs = ga.s[0];
  const Src& ds = gb.s[0];
  const int Wg = ga.Wg, Co = gb.Cg;
  const bool xtf = XTF && xs.scale != nullptr;
  if constexpr (XTF) {
    if (xtf)
      for (int c = tid; c < BMO; c += NT) {
        ssc[c] = xs.scale[i0 + c];
        ssc[BMO + c] = xs.shift[i0 + c];
      }
  }

  // ---- per-lane DMA pieces ----
  // Both sources are whole grids without an origin (fits(): X on the h x w
  // convT input grid, dY on its 2h x 2w output), so a piece's byte offset is
  // affine in its pixel p = (n*h + y)*w + x, up to dY's column term:
  //   X:  (p*C + ci) * 2
  //   dY: ((4p - 2x)*Co + ab_off + co) * 2      (ab_off = (a*2w + b)*Co)
  // and a stage advances p by BK: X adds a constant, dY tracks x = p mod w by
  // one conditional subtraction (BK mod w precomputed).  Pieces past the last
  // pixel are clamped to a valid address (their X rows are zeroed in LDS).
  const unsigned long long xbase = uniform_u64(xs.ptr), dbase = uniform_u64(ds.ptr);
  const int Cx = xs.C;
  const int rbk = BK % Wg;
  const unsigned xlast = (unsigned)((size_t)(args.P - 1) * Cx * 2);                   // + the piece's channel bytes
  const unsigned dlast = (unsigned)(((size_t)ga.nimg * ds.H * ds.W * Co - 8) * 2);  // last 16-B piece of dY
  unsigned axo[DA], acb[DA];  // X: byte offset of the piece's pixel row, its channel bytes
  int bpix[DB], bx[DB];       // dY: the piece's pixel and its x
  unsigned bcb[DB];           // dY: (ab_off + co) * 2
#pragma unroll
  for (int u = 0; u < DA; ++u) {
    const int b = (wave + NW * u) * 1024 + lane * 16;
    const int row = b / RA;
    acb[u] = (unsigned)((i0 + tswz<RA>(row, (b % RA) / 16) * 8) * 2);
    axo[u] = (unsigned)((size_t)(pbeg + row) * Cx * 2);
  }
#pragma unroll
  for (int u = 0; u < DB; ++u) {
    const int b = (wave + NW * u) * 1024 + lane * 16;
    const int row = b / RB;
    const int col = j0 + tswz<RB>(row, (b % RB) / 16) * 8;
    const int ab = col / Co;
    bcb[u] = (unsigned)((((ab >> 1) * ds.W + (ab & 1)) * Co + (col - ab * Co)) * 2);
    bpix[u] = pbeg + row;
    bx[u] = bpix[u] % Wg;
  }

  // DMA u (0 .. D-1: X pieces, then dY pieces) of the next stage to issue, into
  // ring slot `slot`; then advances that piece by BK pixels
  auto issue1 = [&](int slot, int u) {
    if (u < DA) {
      dma_sv(min(axo[u], xlast) + acb[u], xbase, lds0 + slot * SSZ + (wave + NW * u) * 1024);
      axo[u] += (unsigned)(BK * Cx * 2);
    } else {
      const int k = u - DA;
      const unsigned off = (unsigned)(4 * bpix[k] - 2 * bx[k]) * (unsigned)(Co * 2) + bcb[k];
      dma_sv(min(off, dlast), dbase, lds0 + slot * SSZ + ASZ + (wave + NW * k) * 1024);
      bpix[k] += BK;
      bx[k] += rbk;
      bx[k] -= bx[k] >= Wg ? Wg : 0;
    }
  };

  // in-LDS pass over stage `st` (pixels pb ..): X's relu(bn(.)) (XTF) and
  // zeroed rows for pixels >= pend
  auto fix_stage = [&](int slot, int pb) {
    const bool tail = pb + BK > pend;
    if (!xtf && !tail) return;
    unsigned char* as = lds + slot * SSZ;
    constexpr int PCS = ASZ / 16;
#pragma unroll
    for (int k = 0; k < (PCS + NT - 1) / NT; ++k) {
      const int p = tid + NT * k;
      if (p < PCS) {
        const int row = p / (RA / 16);
        uint4* pv = reinterpret_cast<uint4*>(as + p * 16);
        if (pb + row >= pend) {
          *pv = make_uint4(0u, 0u, 0u, 0u);
        } else if (xtf) {
          const int c = tswz<RA>(row, p % (RA / 16)) * 8;  // logical channel group of the piece
          const uint4 v = *pv;
          *pv = bf16pack8(affine_relu4(bf16x4_to_f4(make_uint2(v.x, v.y)), ld4(ssc + c), ld4(ssc + BMO + c)),
                          affine_relu4(bf16x4_to_f4(make_uint2(v.z, v.w)), ld4(ssc + c + 4), ld4(ssc + BMO + c + 4)));
        }
      }
    }
  };

  // ---- per-lane transposed-read offsets (bytes within a stage) ----
  const int g16 = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3, hk = g16 >> 1, half = g16 & 1;
  const int rowl = 8 * hk + q4;
  unsigned aoff[TM], boff[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int col = wm * TM * 32 + i * 32 + half * 16 + pp * 4;
    aoff[i] = (unsigned)(rowl * RA + tswz<RA>(rowl, col >> 3) * 16 + (col & 7) * 2);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * TN * 32 + j * 32 + half * 16 + pp * 4;
    boff[j] = (unsigned)(ASZ + rowl * RB + tswz<RB>(rowl, col >> 3) * 16 + (col & 7) * 2);
  }

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    // prologue: stages 0 .. P-1 (past the last stage the last one is re-issued
    // into a slot no MFMA reads, so every step retires D DMAs)
#pragma unroll
    for (int j = 0; j < P; ++j)
#pragma unroll
      for (int u = 0; u < D; ++u) issue1(j, u);
    vm_wait<D * (P - 1)>();
    __syncthreads();  // stage 0 and the BN table visible to every wave
    fix_stage(0, pbeg);
    lgkm_wait0();     // its rewritten pieces land before the first barrier releases them
  }
  // ring step for stage i in slot S (compile-time: the LDS read addresses are a
  // per-lane base plus immediates):
  // stage i + 1 landed for this wave (stage i was fixed before the barrier);
  // the barrier publishes every wave's pieces and the fix of stage i, and
  // frees slot i - 1 for the refill below
  auto step = [&](auto Sc, int i) {
    constexpr int S = decltype(Sc)::value, S1 = (S + 1) % NS, SN = (S + P) % NS;
    vm_wait<D * (P - 2)>();
    raw_barrier();
    if (i + 1 < nk) {
      fix_stage(S1, pbeg + (i + 1) * BK);
      lgkm_wait0();  // (the fixed stage i + 1 is read only after the next barrier)
    }
    unsigned ra[TM], rb[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) ra[t] = lds0 + S * SSZ + aoff[t];
#pragma unroll
    for (int t = 0; t < TN; ++t) rb[t] = lds0 + S * SSZ + boff[t];
    bf16x8t_t fa[2][TM], fb[2][TN];
    auto rd = [&](int ks, int b) {
#pragma unroll
      for (int t = 0; t < TM; ++t)
        fa[b][t] = __builtin_shufflevector(tr4(ra[t] + (16 * ks) * RA), tr4(ra[t] + (16 * ks + 4) * RA), 0, 1, 2, 3,
                                           4, 5, 6, 7);
#pragma unroll
      for (int t = 0; t < TN; ++t)
        fb[b][t] = __builtin_shufflevector(tr4(rb[t] + (16 * ks) * RB), tr4(rb[t] + (16 * ks + 4) * RB), 0, 1, 2, 3,
                                           4, 5, 6, 7);
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) rd(ks + 1, (ks + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ks & 1][a], fb[ks & 1][b], acc[a][b], 0, 0, 0);
      // the stage P ahead, its DMAs spread over the k-steps
#pragma unroll
      for (int u = 0; u < D; ++u)
        if (u * KS / D == ks) issue1(SN, u);
    }
  };
  static_assert(NS <= 6, "ring steps unrolled below");
  for (int i = 0; i < nk; i += NS) {
    step(std::integral_constant<int, 0>{}, i);
    if (i + 1 < nk) step(std::integral_constant<int, 1>{}, i + 1);
    if (i + 2 < nk) step(std::integral_constant<int, 2 % NS>{}, i + 2);
    if constexpr (NS > 3) {
      if (i + 3 < nk) step(std::integral_constant<int, 3 % NS>{}, i + 3);
    }
    if constexpr (NS > 4) {
      if (i + 4 < nk) step(std::integral_constant<int, 4 % NS>{}, i + 4);
    }
    if constexpr (NS > 5) {
      if (i + 5 < nk) step(std::integral_constant<int, 5 % NS>{}, i + 5);
    }
  }
  vm_wait<0>();  // the tail's re-issued DMAs land before the workgroup exits

  // this split's partial: plain stores into its slab plane (or straight into
  // the gradient for a single split); fp32 atomics only without a slab
  const int h = lane >> 5, li = lane & 31;
  float* const plane = args.slab ? args.slab + (size_t)z * args.Mo * args.No : nullptr;
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
// tile ids (igemm.hip wgrad_tile_fits / launch_wgrad_v): BMO x BNO, BK pixels
// per stage, NS stages
//   40: 128 x 256, 8 waves (2 x 4, 64 x 64 each), BK 32, 6 stages: 144 KB
//   41: 256 x 256, 8 waves (4 x 2, 64 x 128 each), BK 32, 4 stages: 128 KB
//   42: 256 x 128, 8 waves (4 x 2, 64 x 64 each), BK 32, 6 stages: 144 KB
//   43: 128 x 128, 8 waves (2 x 4, 64 x 32 each), BK 64, 4 stages: 128 KB
//   44: 128 x 256, 8 waves (2 x 4, 64 x 64 each), BK 64, 3 stages: 144 KB
// per_cu codes: >= 10 slab mode (per_cu - 10 workgroups per CU), else atomics
// ---------------------------------------------------------------------------
static bool wgradT_shape(int tile, int& bmo, int& bno) {
  switch (tile) {
    case 40: bmo = 128; bno = 256; return true;
    case 41: bmo = 256; bno = 256; return true;
    case 42: bmo = 256; bno = 128; return true;
    case 43: bmo = 128; bno = 128; return true;
    case 44: bmo = 128; bno = 256; return true;
    default: return false;
  }
}

bool wgradT_ring_fits(const WgradArgs& a, int tile) {
  int bmo, bno;
  if (!wgradT_shape(tile, bmo, bno) || !a.bf16 || a.split || a.batch > 1) return false;
  const Gather& ga = a.ga;
  const Gather& gb = a.gb;
  const Src& xs = ga.s[0];
  const Src& ds = gb.s[0];
  const double xb = 2.0 * ga.nimg * xs.H * xs.W * xs.C, db = 2.0 * gb.nimg * ds.H * ds.W * ds.C;
  return ga.taps_h == 1 && ga.taps_w == 1 && ga.stride == 1 && ga.c_split >= ga.Cg && ga.Cg == a.Mo &&
         gb.taps_h == 2 && gb.taps_w == 2 && gb.stride == 2 && gb.c_split >= gb.Cg && a.No == 4 * gb.Cg &&
         gb.Cg % 8 == 0 && a.Mo % bmo == 0 && a.No % bno == 0 && ga.Hg == gb.Hg && ga.Wg == gb.Wg &&
         ga.nimg == gb.nimg && a.P == ga.nimg * ga.Hg * ga.Wg && xs.h16 && ds.h16 && ds.scale == nullptr &&
         (xs.scale == nullptr || xs.shift != nullptr) && xb < 4294967296.0 && db < 4294967296.0 && a.P > 0 &&
         // whole grids without an origin (the plan's convT input and output gradient)
         xs.oy == 0 && xs.ox == 0 && xs.H == ga.Hg && xs.W == ga.Wg && xs.C == a.Mo && ds.oy == 0 && ds.ox == 0 &&
         ds.H == 2 * gb.Hg && ds.W == 2 * gb.Wg && ds.C == gb.Cg;
}

template <int BMO, int BNO, int WM, int WN, int BK, int NS>
static hipError_t go_wt(const WgradArgs& a0, hipStream_t s, int per_cu) {
  using G = WTGeo<BMO, BNO, BK, NS>;
  static bool attr[2] = {false, false};
  const bool slab_mode = per_cu >= 10;
  if (slab_mode) per_cu -= 10;
  if (per_cu < 1) per_cu = 1;
  const int tm = a0.Mo / BMO, tn = a0.No / BNO, tiles = tm * tn;
  int splits = (per_cu * num_cus() + tiles - 1) / tiles;
  const int max_splits = (a0.P + BK - 1) / BK;
  splits = std::max(1, std::min(splits, max_splits));
  WgradArgs a = a0;
  int pps = (a.P + splits - 1) / splits;
  pps = (pps + BK - 1) / BK * BK;
  splits = (a.P + pps - 1) / pps;
  a.pix_per_split = pps;
  const size_t plane = (size_t)a.Mo * a.No;
  const bool use_slab = slab_mode && a.slab && !a.accumulate && (size_t)splits * plane * sizeof(float) <= a.slab_bytes &&
                        splits > 1 && plane % 4 == 0;
  if (slab_mode && splits > 1 && !use_slab) ++g_slab_fallbacks;
  // one split: the partial is the gradient (plain stores); else the slab or,
  // without one, fp32 atomics into the zeroed gradient
  a.slab = use_slab ? a.slab : (splits == 1 && !a.accumulate ? a.out : nullptr);
  const int xcd_map = (tiles * splits) % 8 == 0;
  const bool tf = a.ga.s[0].scale != nullptr;
  const void* fn = tf ? reinterpret_cast<const void*>(&k_wgradT_ring<BMO, BNO, WM, WN, BK, NS, 1>)
                      : reinterpret_cast<const void*>(&k_wgradT_ring<BMO, BNO, WM, WN, BK, NS, 0>);
  if (!attr[tf]) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::smem);
    if (e != hipSuccess) return e;
    attr[tf] = true;
  }
  const dim3 grid((unsigned)(tiles * splits));
  if (tf)
    hipLaunchKernelGGL((k_wgradT_ring<BMO, BNO, WM, WN, BK, NS, 1>), grid, dim3(WM * WN * 64), G::smem, s, a, tm, tn,
                       splits, xcd_map);
  else
    hipLaunchKernelGGL((k_wgradT_ring<BMO, BNO, WM, WN, BK, NS, 0>), grid, dim3(WM * WN * 64), G::smem, s, a, tm, tn,
                       splits, xcd_map);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !use_slab) return e;
  return launch_slab_reduce(a.slab, splits, 1, plane, 0, a.out, s);
}

hipError_t go_wgradT_ring(const WgradArgs& a, hipStream_t s, int tile, int per_cu) {
  if (!wgradT_ring_fits(a, tile)) return hipErrorInvalidValue;
  switch (tile) {
    case 40: return go_wt<128, 256, 2, 4, 32, 6>(a, s, per_cu);
    case 41: return go_wt<256, 256, 4, 2, 32, 4>(a, s, per_cu);
    case 42: return go_wt<256, 128, 4, 2, 32, 6>(a, s, per_cu);
    case 43: return go_wt<128, 128, 2, 4, 64, 4>(a, s, per_cu);
    case 44: return go_wt<128, 256, 2, 4, 64, 3>(a, s, per_cu);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
