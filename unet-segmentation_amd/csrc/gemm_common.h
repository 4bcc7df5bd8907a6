// Device helpers shared by the fp32 (igemm.hip) and bf16 (igemm_bf16.hip)
// implicit-GEMM kernel families: vector load/store, the consumer-side
// BatchNorm+ReLU transform, bf16 packing, the pixel iterator of the
// weight-gradient GEMMs and the common epilogue of every forward /
// input-gradient GEMM tile.
//
// Accumulator layout (identical for v_mfma_f32_32x32x2_f32 and
// v_mfma_f32_32x32x16_bf16 on gfx950): lane l holds column l&31 of a 32x32 tile,
// register r holds row (r&3) + 8*(r>>2) + 4*(l>>5).
#pragma once
#include <type_traits>

#include "ring_common.h"
#include "unet_internal.h"

namespace unet {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float floatx2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

__device__ __forceinline__ float4 affine_relu4(float4 v, float4 a, float4 b) {
  v.x = fmaxf(fmaf(v.x, a.x, b.x), 0.f);
  v.y = fmaxf(fmaf(v.y, a.y, b.y), 0.f);
  v.z = fmaxf(fmaf(v.z, a.z, b.z), 0.f);
  v.w = fmaxf(fmaf(v.w, a.w, b.w), 0.f);
  return v;
}

__device__ __forceinline__ float getc(const float4& v, int c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}

// two fp32 -> two bf16 (round to nearest even, v_cvt_pk_bf16_f32), low half = a
__device__ __forceinline__ unsigned bf16pack(float a, float b) {
  const bf16x2_t v = __builtin_convertvector((floatx2_t){a, b}, bf16x2_t);
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ uint4 bf16pack8(float4 a, float4 b) {
  return make_uint4(bf16pack(a.x, a.y), bf16pack(a.z, a.w), bf16pack(b.x, b.y), bf16pack(b.z, b.w));
}
__device__ __forceinline__ uint16_t bf16_of(float v) { return (uint16_t)(bf16pack(v, 0.f) & 0xffffu); }
// v rounded to the nearest bf16, as fp32
__device__ __forceinline__ float round_bf(float v) { return __uint_as_float((unsigned)bf16_of(v) << 16); }
// element idx of an fp32 or bf16 tensor
__device__ __forceinline__ float ld_elem(const float* p, size_t idx, int h16) {
  return h16 ? __uint_as_float((unsigned)reinterpret_cast<const uint16_t*>(p)[idx] << 16) : p[idx];
}
// 4 bf16 (uint2) -> 4 fp32 (exact)
__device__ __forceinline__ float4 bf16x4_to_f4(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
// g.s[second], picked field by field: a reference into the kernel-argument
// array selected at run time makes the compiler copy the array to scratch
__device__ __forceinline__ Src pick_src(const Gather& g, bool second) {
  Src r;
  r.ptr = second ? g.s[1].ptr : g.s[0].ptr;
  r.H = second ? g.s[1].H : g.s[0].H;
  r.W = second ? g.s[1].W : g.s[0].W;
  r.C = second ? g.s[1].C : g.s[0].C;
  r.oy = second ? g.s[1].oy : g.s[0].oy;
  r.ox = second ? g.s[1].ox : g.s[0].ox;
  r.scale = second ? g.s[1].scale : g.s[0].scale;
  r.shift = second ? g.s[1].shift : g.s[0].shift;
  r.h16 = second ? g.s[1].h16 : g.s[0].h16;
  return r;
}
// store one element of a Dst (fp32 or bf16 storage)
__device__ __forceinline__ void dst_store(const Dst& d, size_t idx, float v) {
  if (d.h16)
    reinterpret_cast<uint16_t*>(d.ptr)[idx] = bf16_of(v);
  else
    d.ptr[idx] = v;
}

// Pixel iterator over an (nimg, Hg, Wg) grid (weight-gradient GEMMs walk their
// staged pixel rows incrementally, no divisions in the loop).
struct PixIt {
  int n, y, x;
  __device__ __forceinline__ void init(int p, int Hg, int Wg) {
    const int hw = Hg * Wg;
    n = p / hw;
    const int r = p - n * hw;
    y = r / Wg;
    x = r - y * Wg;
  }
  __device__ __forceinline__ void advance(int d, int Hg, int Wg) {
    x += d;
    while (x >= Wg) {
      x -= Wg;
      if (++y == Hg) { y = 0; ++n; }
    }
  }
  __device__ __forceinline__ void next(int Hg, int Wg) {
    if (++x == Wg) {
      x = 0;
      if (++y == Hg) { y = 0; ++n; }
    }
  }
};

// Tile row -> output row m of the GEMM.  LinearRows: rows m0.. of a
// pixel-linear tile.  HaloRows: a TH x TW spatial tile of image n at (y0, x0)
// in row-major order (the halo-tiled 3x3 kernels); rows outside the grid are
// not stored.
struct LinearRows {
  int m0, M;
  __device__ __forceinline__ bool map(int row, int& m) const {
    m = m0 + row;
    return m < M;
  }
  // fragment block fr (tile rows fr*32 ..): the row of accumulator register r
  // of a lane in half h is mb + k_r (k_r = (r & 3) + 8 (r >> 2)), valid iff
  // k_r < lim
  __device__ __forceinline__ void block(int fr, int h, int& mb, int& lim) const {
    mb = m0 + fr * 32 + 4 * h;
    lim = M - mb;
  }
  __device__ __forceinline__ bool full(int fr) const { return M - (m0 + fr * 32) >= 32; }
};
// Tile pixel of GEMM row p (32 rows per MFMA fragment).  Row-major, except in
// 16 x 16 tiles read from 80-B LDS rows: there fragment f holds tile rows f and
// f + 8 (lanes 0-15 / 16-31), 144 halo pixels apart -- a multiple of 16 bank
// quads, like the two halves of a 32-wide row -- instead of rows f, f + 1 (18
// pixels apart), whose ds_read_b128 lane groups collide on two bank quads.
template <int TH, int TW>
__device__ __forceinline__ void halo_pix(int p, int& ty, int& tx) {
  if constexpr (TH == 16 && TW == 16) {
    const int f = p >> 5, l = p & 31;
    ty = f + 8 * (l >> 4);
    tx = l & 15;
  } else {
    ty = p / TW;
    tx = p % TW;
  }
}

template <int TW, int TH = 0>
struct HaloRows {
  int n, y0, x0, Hg, Wg;
  __device__ __forceinline__ bool map(int row, int& m) const {
    int ty, tx;
    halo_pix<TH, TW>(row, ty, tx);
    const int y = y0 + ty, x = x0 + tx;
    m = (n * Hg + y) * Wg + x;
    return y < Hg && x < Wg;
  }
  // 32-wide tiles: fragment block fr is tile row fr (see LinearRows::block)
  __device__ __forceinline__ void block(int fr, int h, int& mb, int& lim) const {
    const int y = y0 + fr;
    mb = (n * Hg + y) * Wg + x0 + 4 * h;
    lim = y < Hg ? Wg - x0 - 4 * h : 0;
  }
  // every row of fragment block fr lies inside the grid (wave-uniform)
  __device__ __forceinline__ bool full(int fr) const { return y0 + fr < Hg && Wg - x0 >= 32; }
};

template <class R>
struct fast_rows : std::false_type {};
template <>
struct fast_rows<LinearRows> : std::true_type {};
template <int TH>
struct fast_rows<HaloRows<32, TH>> : std::true_type {};

// Row permutation inside blocks of 8 (q -> 0, 4, 1, 5, 2, 6, 3, 7): staging
// loops whose 8-lane ds_write_b128 groups cover two 4-piece rows then pair rows
// 4 apart -- conflict-free for 80-B rows under the stores' mod-32 banking.
__device__ __forceinline__ int stage_row8(int q) { return (q & ~7) | ((q & 1) << 2) | ((q >> 1) & 3); }

// Column statistics of an epilogue (BN sums, BN-backward sums, concat column
// sums): wave halves, then waves of a column block through LDS, then one fp64
// atomic per column per workgroup into a spread group.
template <int BN, int WM, int WN, int NT, int TN>
__device__ __forceinline__ void igemm_finish_stats(const Epilogue& e, float (&s1)[TN], float (&s2)[TN],
                                                   float (&t1)[TN], int n0, int wn, int N, int tid, float* red) {
  const int lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int wm = (tid >> 6) / WN;
  const bool want_stats = (e.stats != nullptr) || (e.yref != nullptr) || (e.colsum1 != nullptr);
  if (!want_stats) return;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    s1[j] += __shfl_xor(s1[j], 32);
    s2[j] += __shfl_xor(s2[j], 32);
    t1[j] += __shfl_xor(t1[j], 32);
  }
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int lc = wn * TN * 32 + j * 32 + li;
      red[(wm * 3 + 0) * BN + lc] = s1[j];
      red[(wm * 3 + 1) * BN + lc] = s2[j];
      red[(wm * 3 + 2) * BN + lc] = t1[j];
    }
  }
  __syncthreads();
  const int grp = blockIdx.x % kStatGroups;
  const int nsplit = min(e.n_split, N);
  for (int lc = tid; lc < BN; lc += NT) {
    float a = 0.f, b = 0.f, c = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) { a += red[(w * 3 + 0) * BN + lc]; b += red[(w * 3 + 1) * BN + lc]; c += red[(w * 3 + 2) * BN + lc]; }
    const int col = n0 + lc;
    if (col < nsplit) {
      double* st = e.yref ? e.bstats : e.stats;
      if (st) {
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 0, (double)a);
        atomicAdd(st + ((size_t)grp * nsplit + col) * 2 + 1, (double)b);
      }
    } else if (e.colsum1) {
      const int n2 = N - nsplit;
      atomicAdd(e.colsum1 + (size_t)grp * n2 + (col - nsplit), (double)c);
    }
  }
}


// Fast-path epilogue, specialised at compile time on what the GEMM's epilogue
// does -- KIND 0: plain store (+ concat column sums of the second destination),
// 1: forward BatchNorm statistics, 2: ReLU mask of the producer + BN-backward
// statistics, 3: ReLU (eval with BatchNorm folded in) -- and on the storage (H16: bf16 destination, YH16: bf16 yref).
// Row bases per fragment block; fragments whose 32 rows all lie inside the grid
// (the wave-uniform common case) store without per-element guards.  A bf16
// value is converted once: its bits are stored and its rounded value feeds the
// statistics (the values the consumers read).
template <int TM, int TN, int KIND, int H16, int YH16, class RowMap>
__device__ __forceinline__ void epi_fast(const Epilogue& e, const floatx16 (&acc)[TM][TN], const RowMap& rows,
                                         const Gather& g, int n0, int wm, int wn, int h, int li, float (&s1)[TN],
                                         float (&s2)[TN], float (&t1)[TN]) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * TN * 32 + j * 32 + li;
    const float bias = e.bias ? e.bias[col] : 0.f;
    const bool second = col >= e.n_split;  // uniform per 32-column block (n_split % 32 == 0)
    float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
    const int dC = second ? e.d[1].C : e.d[0].C;
    const int dcol = second ? col - e.n_split : col;
    const bool csum = second && e.colsum1 != nullptr;
    float bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
    if constexpr (KIND == 2) {
      bsc = e.bn_scale[col];
      bsh = e.bn_shift[col];
      bmu = e.bn_mean[col];
      bis = e.bn_invstd[col];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      int mb, lim;
      rows.block(wm * TM + i, h, mb, lim);
      const unsigned ib = (unsigned)mb * (unsigned)dC + (unsigned)dcol;
      float yv[KIND == 2 ? 16 : 1];
      if constexpr (KIND == 2) {
        // the mask operand of all 16 rows before the first store (the
        // destination may alias yref as far as the compiler knows); rows past
        // the grid re-load the last valid row
        if (lim > 0) {
          const int kmax = lim - 1;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const unsigned idx = ib + (unsigned)(min((r & 3) + 8 * (r >> 2), kmax) * dC);
            yv[r] = YH16 ? __uint_as_float((unsigned)reinterpret_cast<const uint16_t*>(e.yref)[idx] << 16)
                         : e.yref[idx];
          }
        }
      }
      auto one = [&](int r) {
        const int k = (r & 3) + 8 * (r >> 2);
        const unsigned idx = ib + (unsigned)(k * dC);
        float v = acc[i][j][r] + bias;
        if constexpr (KIND == 3) v = fmaxf(v, 0.f);
        unsigned bits = 0;
        if constexpr (H16) {
          bits = bf16_of(v);
          if constexpr (KIND == 1 || KIND == 2) v = __uint_as_float(bits << 16);  // statistics of the stored value
        }
        if constexpr (KIND == 2) {
          const bool on = fmaf(yv[r], bsc, bsh) > 0.f;
          v = on ? v : 0.f;
          if constexpr (H16) bits = on ? bits : 0u;
          s1[j] += v;
          s2[j] += v * ((yv[r] - bmu) * bis);
        } else if constexpr (KIND == 1) {
          s1[j] += v;
          s2[j] += v * v;
        } else {
          if (csum) t1[j] += v;
        }
        if constexpr (H16)
          reinterpret_cast<uint16_t*>(dptr)[idx] = (uint16_t)bits;
        else
          dptr[idx] = v;
      };
      if (rows.full(wm * TM + i)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) one(r);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if ((r & 3) + 8 * (r >> 2) < lim) one(r);
      }
    }
  }
}

// LDS-staged form of epi_fast for a bf16 destination and 64 columns per wave
// (TN = 2), round 5.  The per-element path moves one 2-B element per lane and
// memory instruction (32 stores, and for the input gradient 32 mask loads, per
// lane and fragment); k_conv3_bf's phase probe (tools/phase_probe.py,
// profiles/r05_conv3_bf_phases.txt) put that epilogue at 3.2 of the 12.9 us of
// an inc.c1 workgroup.  Here a fragment's 32 rows x 64 columns pass through the
// wave's 4 KB of LDS ([row][64] bf16, 128-B rows): the mask operand comes in by
// four 1-KB LDS-DMAs, every lane reads and rewrites its 2-B elements in place
// (column-contiguous 32-lane groups: no bank conflict), and the tile leaves by
// four 16-B stores per lane (ds_read_b128 lane groups on 16 distinct bank
// quads at 128-B rows).  Same values, statistics and rows as epi_fast.
template <int TM, int TN, int KIND, class RowMap>
__device__ __forceinline__ void epi_lds(const Epilogue& e, const floatx16 (&acc)[TM][TN], const RowMap& rows, int n0,
                                        int wm, int wn, int h, int li, int lane, float (&s1)[TN], float (&s2)[TN],
                                        unsigned short* wl) {
  static_assert(TN == 2, "64 columns per wave: 128-B LDS rows");
  constexpr int ROW = TN * 32;  // bf16 per LDS row
  const Dst& d = e.d[0];
  const unsigned dC = (unsigned)d.C;
  const int col0 = n0 + wn * TN * 32;
  float bias[TN], bsc[TN], bsh[TN], bmu[TN], bis[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + j * 32 + li;
    bias[j] = e.bias ? e.bias[col] : 0.f;
    bsc[j] = bsh[j] = bmu[j] = bis[j] = 0.f;
    if constexpr (KIND == 2) {
      bsc[j] = e.bn_scale[col];
      bsh[j] = e.bn_shift[col];
      bmu[j] = e.bn_mean[col];
      bis[j] = e.bn_invstd[col];
    }
  }
  const unsigned wl_lds = (unsigned)(size_t)(lds_u8_t*)wl;
  unsigned long long ybase = 0;
  if constexpr (KIND == 2) ybase = uniform_u64(e.yref);
  uint16_t* const dst = reinterpret_cast<uint16_t*>(d.ptr);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int mb, lim;
    rows.block(wm * TM + i, 0, mb, lim);
    if (lim <= 0) continue;  // wave-uniform
    const int kmax = (lim < 32 ? lim : 32) - 1;
    if constexpr (KIND == 2) {  // mask operand rows: 8 rows x 128 B per DMA (rows past the grid re-read the last)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = min((lane >> 3) + 8 * q, kmax);
        dma_sv(((unsigned)(mb + k) * dC + (unsigned)col0) * 2u + (unsigned)(lane & 7) * 16u, ybase,
               wl_lds + (unsigned)q * 1024u);
      }
      vm_wait<0>();
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      // one 32-column block at a time: the scheduler may not hoist the next
      // block's mask reads (16 more live VGPRs at the 128-register budget)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = (r & 3) + 8 * (r >> 2) + 4 * h;
        unsigned short* el = wl + k * ROW + j * 32 + li;
        float v = acc[i][j][r] + bias[j];
        if constexpr (KIND == 3) v = fmaxf(v, 0.f);
        unsigned bits = bf16_of(v);
        if constexpr (KIND == 1 || KIND == 2) v = __uint_as_float(bits << 16);  // statistics of the stored value
        const bool in = k < lim;
        if constexpr (KIND == 2) {
          const float yv = __uint_as_float((unsigned)*el << 16);
          const bool on = fmaf(yv, bsc[j], bsh[j]) > 0.f;
          v = on ? v : 0.f;
          bits = on ? bits : 0u;
          if (in) {
            s1[j] += v;
            s2[j] += v * ((yv - bmu[j]) * bis[j]);
          }
        } else if constexpr (KIND == 1) {
          if (in) {
            s1[j] += v;
            s2[j] += v * v;
          }
        }
        *el = (unsigned short)bits;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = (lane >> 3) + 8 * q;
      const uint4 val = *reinterpret_cast<const uint4*>(wl + k * ROW + (lane & 7) * 8);
      if (k < lim) *reinterpret_cast<uint4*>(dst + (size_t)(mb + k) * dC + col0 + (lane & 7) * 8) = val;
    }
    lgkm_wait0();  // this fragment's LDS reads retired before the next one's mask DMA lands there
  }
}

// Pixel-shuffle epilogue of the ConvTranspose2d(k2, s2) GEMM (rows = input
// pixels of the linear grid, column ab * Co + co -> output pixel (2y + a, 2x + b),
// channel co): the destination base of each accumulator row is computed once
// per fragment row (one pixel decomposition per block, then increments) and a
// 32-column block is one (a, b) sub-pixel, so an element costs an add and its
// store.  (The generic path decomposes every element's pixel: two integer
// divisions per element dominated the convT forward.)
template <int TM, int TN, int H16>
__device__ __forceinline__ void epi_shuffle(const Epilogue& e, const floatx16 (&acc)[TM][TN], const LinearRows& rows,
                                            const Gather& g, int n0, int wm, int wn, int h, int li) {
  const Dst& d = e.d[0];
  const unsigned Co = (unsigned)e.shuffle_co, W2 = (unsigned)d.W, H2 = (unsigned)d.H;
  const int Wg = g.Wg, Hg = g.Hg;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int mb, lim;
    rows.block(wm * TM + i, h, mb, lim);
    if (lim <= 0) continue;
    int nn = mb / (Hg * Wg);
    const int rr = mb - nn * Hg * Wg;
    int y = rr / Wg, x = rr - y * Wg;
    unsigned base[16];
    int kprev = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = (r & 3) + 8 * (r >> 2);
      x += k - kprev;
      kprev = k;
      while (x >= Wg) {  // at most (27 / Wg) + 1 wraps
        x -= Wg;
        if (++y == Hg) {
          y = 0;
          ++nn;
        }
      }
      base[r] = (((unsigned)nn * H2 + 2u * y) * W2 + 2u * x) * Co;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * TN * 32 + j * 32 + li;
      const unsigned ab = (unsigned)col / Co, co = (unsigned)col - ab * Co;  // ab uniform per 32 columns
      const unsigned off = ((ab >> 1) * W2 + (ab & 1)) * Co + co;
      const float bias = e.bias ? e.bias[co] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if ((r & 3) + 8 * (r >> 2) >= lim) continue;
        float v = acc[i][j][r] + bias;
        if (e.relu) v = fmaxf(v, 0.f);
        if constexpr (H16)
          reinterpret_cast<uint16_t*>(d.ptr)[base[r] + off] = (uint16_t)bf16_of(v);
        else
          d.ptr[base[r] + off] = v;
      }
    }
  }
}

// Split-K partial store or the full epilogue of an implicit-GEMM tile: bias,
// destination mapping (linear / pixel shuffle / cropped), ReLU mask + BN-bwd
// statistics, BN statistics, concat column sums.  `red` is WM*3*BN floats of
// LDS that no wave reads or writes any more (a barrier precedes its use).
// `stage` (optional): NT / 64 x 4 KB of LDS, disjoint from `red`, that no wave
// reads or writes any more -- enables epi_lds for bf16 destinations at TN = 2.
// KSTAGE2: also stage the input gradient's masked form (KIND 2; callers with the
// register budget for it -- k_conv3_bf's 128 VGPRs spilled).
// kz: this workgroup's K slice (split-K partial plane), when its grid position
// is remapped (xcd_block); < 0: blockIdx.z.
template <int BM, int BN, int WM, int WN, int NT, class RowMap = LinearRows, int KSTAGE2 = 0>
__device__ __forceinline__ void igemm_finish(const IgemmArgs& args, floatx16 (&acc)[BM / (WM * 32)][BN / (WN * 32)],
                                             int m0, int n0, int wm, int wn, int tid, float* red,
                                             RowMap rows = RowMap{0, 0}, unsigned short* stage = nullptr,
                                             int kz = -1) {
  if constexpr (std::is_same<RowMap, LinearRows>::value) {
    if (rows.M == 0) rows = LinearRows{m0, args.M};  // callers may pass a batched bound
  }
  constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
  const Gather& g = args.a;
  const int M = args.M;
  const int lane = tid & 63, h = lane >> 5, li = lane & 31;
  const int HWg = g.Hg * g.Wg;
  const int N = args.N;
  if (args.ksplit > 1) {  // raw partial tile; k_splitk_epi finishes
    float* sl = args.slab + (size_t)(kz >= 0 ? kz : (int)blockIdx.z) * M * N;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * TN * 32 + j * 32 + li;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int m;
          if (rows.map(wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, m)) sl[(size_t)m * N + col] = acc[i][j][r];
        }
    }
    return;
  }

  // ------------------------------ epilogue ---------------------------------
  const Epilogue& e = args.e;
  float s1[TN], s2[TN], t1[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) { s1[j] = 0.f; s2[j] = 0.f; t1[j] = 0.f; }

  // Fast path (the common case: every 3x3 conv forward / input gradient of the
  // plan): destinations laid out on the gather grid itself, no pixel shuffle.
  // Row bases come per fragment block, a register's element offset is the base
  // plus a compile-time multiple of the (uniform) channel count: a handful of
  // VALU per element instead of a per-element pixel decomposition -- the
  // epilogue is a large share of the small-K (64 / 128-channel) GEMMs.
  if constexpr (std::is_same<RowMap, LinearRows>::value) {
    const Dst& d = e.d[0];
    if (e.shuffle_co && e.shuffle_co % 32 == 0 && e.n_split >= N && !e.stats && !e.yref && !e.colsum1 &&
        d.C == e.shuffle_co && d.oy == 0 && d.ox == 0 && d.H == 2 * g.Hg && d.W == 2 * g.Wg &&
        (size_t)args.M * 4 * d.C < (1ull << 32)) {
      if (d.h16) epi_shuffle<TM, TN, 1>(e, acc, rows, g, n0, wm, wn, h, li);
      else epi_shuffle<TM, TN, 0>(e, acc, rows, g, n0, wm, wn, h, li);
      return;
    }
  }
  if constexpr (fast_rows<RowMap>::value) {
    auto lin = [&](const Dst& d) { return d.oy == 0 && d.ox == 0 && d.H == g.Hg && d.W == g.Wg; };
    const bool two = e.n_split < N;
    if (!e.shuffle_co && lin(e.d[0]) && (!two || (lin(e.d[1]) && e.d[1].h16 == e.d[0].h16)) &&
        !(e.stats && (two || e.yref)) && !(e.yref && two) && !(e.relu && (two || e.stats || e.yref))) {
      const int kind = e.yref ? 2 : e.stats ? 1 : e.relu ? 3 : 0;
      const int h16 = e.d[0].h16, yh16 = e.yref_h16;
      if constexpr (TN == 2) {
        // LDS-staged path: bf16 destination (and bf16 mask operand), one destination,
        // 16-B aligned rows, 32-bit byte offsets for the mask DMA
        // (the input gradient's mask form, KIND 2, only with KSTAGE2: in
        // k_conv3_bf its staging spilled at the 128-VGPR budget and ran slower)
        if (stage && h16 && !two && (kind != 2 || (KSTAGE2 && yh16)) && e.d[0].C % 8 == 0 &&
            ((reinterpret_cast<size_t>(e.d[0].ptr) | (kind == 2 ? reinterpret_cast<size_t>(e.yref) : 0)) & 15) == 0 &&
            (size_t)args.M * e.d[0].C * 2 < (1ull << 32)) {
          unsigned short* wl = stage + (tid >> 6) * (32 * 64);
          switch (kind) {
            case 0: epi_lds<TM, TN, 0>(e, acc, rows, n0, wm, wn, h, li, lane, s1, s2, wl); break;
            case 1: epi_lds<TM, TN, 1>(e, acc, rows, n0, wm, wn, h, li, lane, s1, s2, wl); break;
            case 2:
              if constexpr (KSTAGE2) epi_lds<TM, TN, 2>(e, acc, rows, n0, wm, wn, h, li, lane, s1, s2, wl);
              break;
            default: epi_lds<TM, TN, 3>(e, acc, rows, n0, wm, wn, h, li, lane, s1, s2, wl); break;
          }
          igemm_finish_stats<BN, WM, WN, NT>(e, s1, s2, t1, n0, wn, N, tid, red);
          return;
        }
      }
      const int sel = kind * 4 + h16 * 2 + (kind == 2 ? yh16 : 0);
      switch (sel) {
        case 0: epi_fast<TM, TN, 0, 0, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 2: epi_fast<TM, TN, 0, 1, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 4: epi_fast<TM, TN, 1, 0, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 6: epi_fast<TM, TN, 1, 1, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 8: epi_fast<TM, TN, 2, 0, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 9: epi_fast<TM, TN, 2, 0, 1>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 10: epi_fast<TM, TN, 2, 1, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 11: epi_fast<TM, TN, 2, 1, 1>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        case 12: epi_fast<TM, TN, 3, 0, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
        default: epi_fast<TM, TN, 3, 1, 0>(e, acc, rows, g, n0, wm, wn, h, li, s1, s2, t1); break;
      }
      igemm_finish_stats<BN, WM, WN, NT>(e, s1, s2, t1, n0, wn, N, tid, red);
      return;
    }
    if (!e.shuffle_co && lin(e.d[0]) && (e.n_split >= N || lin(e.d[1]))) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * TN * 32 + j * 32 + li;
        const float bias = e.bias ? e.bias[col] : 0.f;
        const bool second = col >= e.n_split;  // uniform per 32-column block (n_split % 32 == 0)
        float* dptr = second ? e.d[1].ptr : e.d[0].ptr;
        const int dC = second ? e.d[1].C : e.d[0].C;
        const int dh16 = second ? e.d[1].h16 : e.d[0].h16;
        const int dcol = second ? col - e.n_split : col;
        const bool bwd_mask = (e.yref != nullptr) && !second;
        float bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
        if (bwd_mask) { bsc = e.bn_scale[col]; bsh = e.bn_shift[col]; bmu = e.bn_mean[col]; bis = e.bn_invstd[col]; }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          int mb, lim;
          rows.block(wm * TM + i, h, mb, lim);
          const unsigned ib = (unsigned)mb * (unsigned)dC + (unsigned)dcol;
          // The ReLU-mask operand of all 16 rows is loaded before the first
          // store: the destination may alias yref as far as the compiler knows,
          // so loads interleaved with the stores each waited out a full memory
          // latency (16 serialised round trips per fragment).  Rows past the
          // grid re-load the last valid row.
          float yv[16];
          if (bwd_mask && lim > 0) {
            const int kmax = lim - 1;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int k = min((r & 3) + 8 * (r >> 2), kmax);
              const unsigned idx = ib + (unsigned)(k * dC);
              yv[r] = e.yref_h16 ? __uint_as_float((unsigned)reinterpret_cast<const uint16_t*>(e.yref)[idx] << 16)
                                 : e.yref[idx];
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int k = (r & 3) + 8 * (r >> 2);
            if (k >= lim) continue;
            const unsigned idx = ib + (unsigned)(k * dC);
            float v = acc[i][j][r] + bias;
            // a bf16-stored conv output / BN-input gradient: the statistics are
            // those of the rounded values its consumers read
            if (dh16 && (e.stats || bwd_mask)) v = round_bf(v);
            if (bwd_mask) {
              v = (fmaf(yv[r], bsc, bsh) > 0.f) ? v : 0.f;
              s1[j] += v;
              s2[j] += v * ((yv[r] - bmu) * bis);
            } else if (e.stats) {
              s1[j] += v;
              s2[j] += v * v;
            } else if (second && e.colsum1) {
              t1[j] += v;
            }
            if (e.relu) v = fmaxf(v, 0.f);
            if (dh16)
              reinterpret_cast<uint16_t*>(dptr)[idx] = bf16_of(v);
            else
              dptr[idx] = v;
          }
        }
      }
      igemm_finish_stats<BN, WM, WN, NT>(e, s1, s2, t1, n0, wn, N, tid, red);
      return;
    }
  }

#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * TN * 32 + j * 32 + li;
    const float bias = e.bias ? e.bias[e.shuffle_co ? col % e.shuffle_co : col] : 0.f;
    const bool second = col >= e.n_split;
    const Dst& d = second ? e.d[1] : e.d[0];
    const int dcol = second ? col - e.n_split : col;
    float bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
    const bool bwd_mask = (e.yref != nullptr) && !second;
    if (bwd_mask) { bsc = e.bn_scale[col]; bsh = e.bn_shift[col]; bmu = e.bn_mean[col]; bis = e.bn_invstd[col]; }
    const bool linear = !e.shuffle_co && d.oy == 0 && d.ox == 0 && d.H == g.Hg && d.W == g.Wg;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        int m;
        if (!rows.map(row, m)) continue;
        float v = acc[i][j][r] + bias;
        // a bf16-stored conv output: its BatchNorm statistics are those of the
        // rounded values the consumers will normalise
        if (d.h16 && (e.stats || bwd_mask)) v = round_bf(v);
        size_t idx;
        if (linear) {
          idx = (size_t)m * d.C + dcol;
        } else if (e.shuffle_co) {
          const int ab = dcol / e.shuffle_co, co = dcol - ab * e.shuffle_co;
          const int n = m / HWg, rr = m - n * HWg;
          const int y = rr / g.Wg, x = rr - y * g.Wg;
          idx = ((size_t)(n * d.H + 2 * y + (ab >> 1) + d.oy) * d.W + 2 * x + (ab & 1) + d.ox) * d.C + co;
        } else {
          const int n = m / HWg, rr = m - n * HWg;
          const int y = rr / g.Wg, x = rr - y * g.Wg;
          idx = ((size_t)(n * d.H + y + d.oy) * d.W + x + d.ox) * d.C + dcol;
        }
        if (bwd_mask) {
          const float yv = ld_elem(e.yref, idx, e.yref_h16);
          v = (fmaf(yv, bsc, bsh) > 0.f) ? v : 0.f;
          s1[j] += v;
          s2[j] += v * ((yv - bmu) * bis);
        } else if (e.stats) {
          s1[j] += v;
          s2[j] += v * v;
        } else if (second && e.colsum1) {
          t1[j] += v;
        }
        if (e.relu) v = fmaxf(v, 0.f);
        dst_store(d, idx, v);
      }
    }
  }
  igemm_finish_stats<BN, WM, WN, NT>(e, s1, s2, t1, n0, wn, N, tid, red);
}

}  // namespace unet
