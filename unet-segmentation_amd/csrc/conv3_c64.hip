// k_conv3_c64 (tile 87): bf16 3x3 conv forward / input gradient of the
// full-resolution 64 -> 64-channel layers (inc.c1 and up4.c1, forward and
// input gradient: models/unet_model.py:11-17 at 508-510^2 and 324-326^2) with
// the whole weight slab resident in LDS.
//
// On these shapes (K = 576, N = 64, 2-8 M pixels) every ring / halo kernel ran
// at 0.25-0.35 of the MFMA peak (profiles/r06_pmc_summary_bf16.txt: 34 %
// busy): with one 64-channel chunk per tile, the ring re-streams the 72 KB
// weight slab tap by tap for every 256-pixel tile (a barrier per tap), and the
// halo kernels re-stage it through VGPRs.  Here:
//  * a persistent workgroup (4 waves, one per SIMD) DMAs the 9 x 64 x 64 bf16
//    weights into LDS once and walks pixel tiles t = blockIdx.x, + gridDim.x, ..;
//  * per tile the (TH + 2) x 34 input halo is DMA'd into one of two halo
//    buffers while the MFMAs of the previous tile run from the other: one
//    barrier per tile, none per tap;
//  * each wave owns two tile rows x all 64 columns; the three tap rows of a tap
//    column share halo rows (tile row i at tap row ky reads halo row i + ky), so
//    a k-step reads 4 A and 6 B fragments for 12 MFMAs (0.83 reads per MFMA);
//  * the producer's BN+ReLU (XTF) is applied to the landed halo in place, the
//    epilogue (the shared igemm_finish: bias, BN statistics / ReLU mask + BN
//    backward statistics) uses the consumed halo buffer as its scratch.
// LDS: weights 72 KB + 2 x 43 KB halo (34-pixel pitch) + the BN table.
#include <algorithm>

#include "gemm_common.h"
#include "ring_common.h"

namespace unet {

namespace {
typedef __bf16 bf16x8c_t __attribute__((ext_vector_type(8)));

constexpr int kTH = 8, kHP = 34, kRB = 128, kCPR = 8, kRPB = 2, kKS = 4, kNW = 4;
constexpr int kPH = (kTH + 2) * kHP;              // halo pixels
constexpr int kIH = (kPH * kRB + 1023) / 1024;    // halo DMA instructions per tile
constexpr int kHSZ = kIH * 1024;
constexpr int kWB = 9 * 64 * kRB;                 // resident weights: [tap][co][64 ch]
constexpr int kNHS = (kIH + kNW - 1) / kNW;       // halo DMAs per wave per tile
constexpr int kIWW = kWB / 1024 / kNW;            // weight DMAs per wave (once)
constexpr size_t kSmem = (size_t)kWB + 2 * kHSZ;  // + the BN table (XTF)
}  // namespace

template <int XTF>
__global__ __launch_bounds__(256, 1) void k_conv3_c64(const IgemmArgs args) {
  constexpr int TM = 2, TN = 2, NT = kNW * 64;
  extern __shared__ __attribute__((aligned(1024))) unsigned char lds[];
  const unsigned lds0 = (unsigned)(size_t)(lds_u8_t*)lds;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hh = lane >> 5, ll = lane & 31;
  const Gather& g = args.a;
  const Src& s0 = g.s[0];
  const int Hg = g.Hg, Wg = g.Wg;
  const int tiles_x = (Wg + 31) / 32, tiles_y = (Hg + kTH - 1) / kTH;
  const int ntiles = g.nimg * tiles_y * tiles_x;

  float* xts = reinterpret_cast<float*>(lds + kSmem);
  const bool xtf0 = XTF && s0.scale != nullptr;
  if constexpr (XTF) {
    if (xtf0 && tid < 64) {
      xts[tid] = s0.scale[tid];
      xts[64 + tid] = s0.shift[tid];
    }
  }

  // ---- resident weights: piece p of the image = (tap, co, physical chunk) ----
  {
    const unsigned long long wb = uniform_u64(args.bh);
#pragma unroll
    for (int u = 0; u < kIWW; ++u) {
      const int b = (wave + kNW * u) * 1024 + lane * 16;
      const int row = b / kRB, pc = (b % kRB) / 16;  // row = tap * 64 + co
      const int t = row >> 6, co = row & 63;
      const int q = pc ^ ((co / kRPB) % kCPR);
      dma_sv((unsigned)((co * 576 + t * 64 + q * 8) * 2), wb, lds0 + (wave + kNW * u) * 1024);
    }
  }

  auto coords = [&](int t, int& n, int& y0, int& x0) {
    x0 = (t % tiles_x) * 32;
    t /= tiles_x;
    y0 = (t % tiles_y) * kTH;
    n = t / tiles_y;
  };
  const unsigned long long sbase = uniform_u64(s0.ptr);
  // the halo DMAs of tile t into buffer hb (offsets recomputed per tile)
  auto issue_halo = [&](int t, int hb) {
    int n, y0, x0;
    coords(t, n, y0, x0);
#pragma unroll
    for (int k = 0; k < kNHS; ++k) {
      const int p = min(k * kNW + wave, kIH - 1);
      const int b = p * 1024 + lane * 16;
      const int r = min(b / kRB, kPH - 1), pc = (b % kRB) / 16;
      const int hy = r / kHP, hx = r % kHP;
      const int q = pc ^ ((hx / kRPB) % kCPR);
      // halo pixels past the input grid read an in-range pixel: they only feed
      // outputs past the grid, never stored
      const int yy = min(y0 + hy, Hg + 1), xx = min(x0 + hx, Wg + 1);
      const unsigned off = (unsigned)((((n * s0.H + yy + s0.oy) * s0.W + xx + s0.ox) * s0.C) * 2 + q * 16);
      dma_sv(off, sbase, lds0 + kWB + hb * kHSZ + p * 1024);
    }
  };
  // XTF: relu(bn(.)) of buffer hb's halo, in place
  auto transform = [&](int hb) {
    unsigned char* h = lds + kWB + hb * kHSZ;
    constexpr int PCS = kPH * kCPR;
    for (int p = tid; p < PCS; p += NT) {
      const int r = p / kCPR, hx = r % kHP;
      const int q = (p % kCPR) ^ ((hx / kRPB) % kCPR);
      const float* sc = xts + q * 8;
      const float* sh = xts + 64 + q * 8;
      uint4* pv = reinterpret_cast<uint4*>(h + p * 16);
      const uint4 v = *pv;
      *pv = bf16pack8(affine_relu4(bf16x4_to_f4(make_uint2(v.x, v.y)), ld4(sc), ld4(sh)),
                      affine_relu4(bf16x4_to_f4(make_uint2(v.z, v.w)), ld4(sc + 4), ld4(sh + 4)));
    }
  };

  // per-lane fragment bases (bytes): A per (buffer, tap column, k-step) at this
  // wave's first halo row; B per k-step (taps 0-6 / 7-8 from two bases so the
  // immediates stay below 64 KB)
  unsigned xa[2][3][kKS], yb[2][kKS];
#pragma unroll
  for (int hb = 0; hb < 2; ++hb)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int s = 0; s < kKS; ++s) {
        const int hx = kx + ll;
        xa[hb][kx][s] = (unsigned)(kWB + hb * kHSZ + (2 * wave * kHP + hx) * kRB +
                                   16 * ((2 * s + hh) ^ ((hx / kRPB) % kCPR)));
      }
#pragma unroll
  for (int s = 0; s < kKS; ++s) {
    yb[0][s] = (unsigned)(ll * kRB + 16 * ((2 * s + hh) ^ ((ll / kRPB) % kCPR)));
    yb[1][s] = yb[0][s] + 7 * 64 * kRB;
  }

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // the MFMAs of one tile from buffer HB: per tap column kx and k-step s, halo
  // rows 2w .. 2w + 3 (A) and the three tap rows' weights (B)
  auto compute = [&](auto HBc) {
    constexpr int hb = decltype(HBc)::value;
    bf16x8c_t fa[2][4], fb[2][3][TN];
    auto rd = [&](auto KXc, auto Sc, int b) {
      constexpr int kx = decltype(KXc)::value, s = decltype(Sc)::value;
#pragma unroll
      for (int m = 0; m < 4; ++m)
        fa[b][m] = *reinterpret_cast<const bf16x8c_t*>(lds + xa[hb][kx][s] + m * kHP * kRB);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int t = ky * 3 + kx;
          const unsigned a = t < 7 ? yb[0][s] + (t * 64 + j * 32) * kRB : yb[1][s] + ((t - 7) * 64 + j * 32) * kRB;
          fb[b][ky][j] = *reinterpret_cast<const bf16x8c_t*>(lds + a);
        }
      }
    };
    rd(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, 0);
    auto step = [&](auto KXc, auto Sc) {
      constexpr int kx = decltype(KXc)::value, s = decltype(Sc)::value;
      constexpr int cur = (kx * kKS + s) & 1;
      if constexpr (s + 1 < kKS) rd(KXc, std::integral_constant<int, s + 1>{}, cur ^ 1);
      else if constexpr (kx + 1 < 3) rd(std::integral_constant<int, kx + 1>{}, std::integral_constant<int, 0>{}, cur ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cur][i + ky], fb[cur][ky][j], acc[i][j], 0, 0, 0);
    };
    auto kcol = [&](auto KXc) {
      step(KXc, std::integral_constant<int, 0>{});
      step(KXc, std::integral_constant<int, 1>{});
      step(KXc, std::integral_constant<int, 2>{});
      step(KXc, std::integral_constant<int, 3>{});
    };
    kcol(std::integral_constant<int, 0>{});
    kcol(std::integral_constant<int, 1>{});
    kcol(std::integral_constant<int, 2>{});
  };

  int tile = blockIdx.x;
  if (tile < ntiles) issue_halo(tile, 0);
  vm_wait<0>();
  __syncthreads();  // weights, the first halo and the BN table visible
  if constexpr (XTF) {
    if (xtf0 && tile < ntiles) transform(0);
    __syncthreads();
  }
  // one tile per trip; two trips per loop iteration so the buffer is a constant
  auto trip = [&](auto HBc) -> bool {
    constexpr int hb = decltype(HBc)::value;
    if (tile >= ntiles) return false;
    const int next = tile + (int)gridDim.x;
    if (next < ntiles) issue_halo(next, hb ^ 1);  // lands during this tile's MFMAs
    compute(HBc);
    vm_wait<0>();
    __syncthreads();  // buffer hb consumed by every wave; the next halo landed and visible
    if constexpr (XTF) {
      if (xtf0 && next < ntiles) transform(hb ^ 1);
    }
    int n, y0, x0;
    coords(tile, n, y0, x0);
    unsigned short* stage = reinterpret_cast<unsigned short*>(lds + kWB + hb * kHSZ);
    float* red = reinterpret_cast<float*>(lds + kWB + hb * kHSZ + kNW * 4096);
    igemm_finish<kTH * 32, 64, kNW, 1, NT, HaloRows<32, kTH>, 1>(args, acc, 0, 0, wave, 0, tid, red,
                                                                 HaloRows<32, kTH>{n, y0, x0, Hg, Wg}, stage);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __syncthreads();  // the epilogue's scratch (buffer hb) before the next halo DMA into it; the transform
    tile = next;
    return true;
  };
  for (;;) {
    if (!trip(std::integral_constant<int, 0>{})) break;
    if (!trip(std::integral_constant<int, 1>{})) break;
  }
}

namespace {
size_t c64_smem(const IgemmArgs& a) { return kSmem + (a.a.s[0].scale ? 2 * 64 * sizeof(float) : 0); }
int c64_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}
}  // namespace

// 64 -> 64 channels, one bf16 source (no concat), packed bf16 B, whole K per
// workgroup, 32-bit source offsets
bool conv3_c64_fits(const IgemmArgs& a) {
  const Gather& g = a.a;
  const Src& s = g.s[0];
  return a.bh != nullptr && a.bl == nullptr && a.N == 64 && g.Cg == 64 && g.c_split >= g.Cg && g.taps_h == 3 &&
         g.taps_w == 3 && g.stride == 1 && a.K == 576 && s.h16 && (s.scale == nullptr || s.shift != nullptr) &&
         a.ksplit <= 1 && (size_t)g.nimg * s.H * s.W * s.C * 2 < (1ull << 32) && c64_smem(a) <= 160 * 1024;
}

long long conv3_c64_tiles(const IgemmArgs& a) {
  const Gather& g = a.a;
  return (long long)g.nimg * ((g.Hg + kTH - 1) / kTH) * ((g.Wg + 31) / 32);
}

hipError_t go_conv3_c64(const IgemmArgs& a, hipStream_t s) {
  if (!conv3_c64_fits(a)) return hipErrorInvalidValue;
  const bool xtf = a.a.s[0].scale != nullptr;
  static bool attr[2] = {false, false};
  const void* fn = xtf ? reinterpret_cast<const void*>(&k_conv3_c64<1>) : reinterpret_cast<const void*>(&k_conv3_c64<0>);
  if (!attr[xtf]) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr[xtf] = true;
  }
  const long long tiles = conv3_c64_tiles(a);
  const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(tiles, c64_cus()));
  if (xtf) hipLaunchKernelGGL((k_conv3_c64<1>), dim3(grid), dim3(256), c64_smem(a), s, a);
  else hipLaunchKernelGGL((k_conv3_c64<0>), dim3(grid), dim3(256), c64_smem(a), s, a);
  return hipGetLastError();
}

}  // namespace unet
