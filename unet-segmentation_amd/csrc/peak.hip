// Ceilings measured on the box the bench runs on (roofline
// fractions "against peaks measured on that box"), for bench.py's untimed
// tail.  Not on the training path.
//   kind 0: dense bf16 MFMA, v_mfma_f32_32x32x16_bf16 (the bf16 plans' MFMA)
//   kind 1: f32 MFMA, v_mfma_f32_16x16x4_f32 (the fp32 plans' Winograd MFMA)
//   kind 2: HBM, a float4 streaming copy of 2 x 1 GiB (read + write bytes)
//   kind 3: HBM, a read-only stream of 2 GiB
// Each probe runs a few launch shapes (MFMA: 1 and 2 waves per SIMD with
// independent accumulator chains per wave, enough in flight to cover the MFMA
// dependency latency; copy: 1 or 4 loads in flight per thread, grid-strided or
// one contiguous non-temporal chunk per workgroup, two grids),
// times `reps` launches of each with hipEvents on `stream` after a warm-up
// launch and reports the best: TFLOP/s for the MFMA kinds, GB/s for the copy.
#include <cerrno>

#include "../../include/unet_hip.h"
#include "unet_internal.h"

namespace {
typedef __bf16 pk_bf16x8_t __attribute__((ext_vector_type(8)));
typedef float pk_floatx16 __attribute__((ext_vector_type(16)));
typedef float pk_floatx4 __attribute__((ext_vector_type(4)));

constexpr int kChains = 4;

__global__ __launch_bounds__(256) void k_peak_bf16(int iters, float* out, int store) {
  pk_bf16x8_t a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (float)((threadIdx.x + i) & 7));
    b[i] = (__bf16)(0.002f * (float)((threadIdx.x * 3 + i) & 7));
  }
  pk_floatx16 acc[kChains];
  for (int c = 0; c < kChains; ++c)
    for (int j = 0; j < 16; ++j) acc[c][j] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
  }
  if (store) {
    float s = 0.f;
    for (int c = 0; c < kChains; ++c)
      for (int j = 0; j < 16; ++j) s += acc[c][j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

__global__ __launch_bounds__(256) void k_peak_f32(int iters, float* out, int store) {
  const float a = 0.001f * (float)(threadIdx.x & 7), b = 0.002f * (float)((threadIdx.x * 3) & 7);
  pk_floatx4 acc[kChains * 2];
  for (int c = 0; c < kChains * 2; ++c)
    for (int j = 0; j < 4; ++j) acc[c][j] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains * 2; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  }
  if (store) {
    float s = 0.f;
    for (int c = 0; c < kChains * 2; ++c)
      for (int j = 0; j < 4; ++j) s += acc[c][j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

__global__ __launch_bounds__(256) void k_peak_f32_32(int iters, float* out, int store) {
  const float a = 0.001f * (float)(threadIdx.x & 7), b = 0.002f * (float)((threadIdx.x * 3) & 7);
  pk_floatx16 acc[kChains];
  for (int c = 0; c < kChains; ++c)
    for (int j = 0; j < 16; ++j) acc[c][j] = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  }
  if (store) {
    float s = 0.f;
    for (int c = 0; c < kChains; ++c)
      for (int j = 0; j < 16; ++j) s += acc[c][j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

// U float4 loads in flight per thread before their stores
template <int U>
__global__ __launch_bounds__(256) void k_peak_copy(const float4* __restrict__ src, float4* __restrict__ dst, size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += U * stride) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * stride < n4 ? src[i + u * stride] : make_float4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n4) dst[i + u * stride] = v[u];
  }
}
// each workgroup streams one contiguous chunk, 4 x 16 B per thread in flight,
// non-temporal loads and stores (no cache allocation for streamed lines)
__global__ __launch_bounds__(256) void k_peak_copy_nt(const float4* __restrict__ src, float4* __restrict__ dst,
                                                      size_t n4) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t b = blockIdx.x * per, e = b + per < n4 ? b + per : n4;
  for (size_t i = b + threadIdx.x; i < e; i += 4 * 256) {
    const pk_floatx4* s4 = reinterpret_cast<const pk_floatx4*>(src);
    pk_floatx4* d4 = reinterpret_cast<pk_floatx4*>(dst);
    pk_floatx4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < e) v[u] = __builtin_nontemporal_load(s4 + i + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < e) __builtin_nontemporal_store(v[u], d4 + i + u * 256);
  }
}
// read-only stream: each workgroup sums one contiguous chunk (non-temporal
// loads, 4 x 16 B per thread in flight), one float per thread written
__global__ __launch_bounds__(256) void k_peak_read(const float4* __restrict__ src, size_t n4, float* out) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t b = blockIdx.x * per, e = b + per < n4 ? b + per : n4;
  const pk_floatx4* s4 = reinterpret_cast<const pk_floatx4*>(src);
  pk_floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (size_t i = b + threadIdx.x; i < e; i += 4 * 256) {
    pk_floatx4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i + u * 256 < e ? __builtin_nontemporal_load(s4 + i + u * 256) : acc * 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}
}  // namespace

extern "C" int unet_peak_probe(int kind, int reps, double* result, unet_stream_t st) {
  if (!result || kind < 0 || kind > 3 || reps < 1) return -EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(st);
  const int cus = unet::num_cus();
  float* out = nullptr;
  void* big = nullptr;
  const size_t copy_bytes = (size_t)1 << 30;
  if (hipMalloc(&out, sizeof(float) * cus * 32 * 256) != hipSuccess) return -ENOMEM;
  if (kind >= 2 && hipMalloc(&big, 2 * copy_bytes) != hipSuccess) {
    (void)hipFree(out);
    return -ENOMEM;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 1 << 15;
  double best = 0.0;
  int rc = 0;
  // variants: MFMA kinds at 1 and 2 waves per SIMD (kind 1 also with the
  // 32x32x2 form); the copy with 1 and 4 loads in flight per thread and two grids
  for (int v = 0; v < 6 && rc == 0; ++v) {
    if ((kind == 0 && v >= 2) || (kind == 1 && v >= 4) || (kind == 3 && v >= 2)) break;
    const int blocks = cus * (v & 1 ? 2 : 1);  // 4 waves per block: 1 or 2 per SIMD
    for (int r = 0; r <= reps; ++r) {  // launch 0 warms up
      (void)hipEventRecord(e0, s);
      if (kind == 0) {
        hipLaunchKernelGGL(k_peak_bf16, dim3(blocks), dim3(256), 0, s, iters, out, 0);
      } else if (kind == 1) {
        if (v < 2) hipLaunchKernelGGL(k_peak_f32, dim3(blocks), dim3(256), 0, s, iters, out, 0);
        else hipLaunchKernelGGL(k_peak_f32_32, dim3(blocks), dim3(256), 0, s, iters, out, 0);
      } else if (kind == 3) {
        hipLaunchKernelGGL(k_peak_read, dim3(cus * (v & 1 ? 32 : 8)), dim3(256), 0, s,
                           reinterpret_cast<const float4*>(big), 2 * copy_bytes / 16, out);
      } else {
        const float4* src = reinterpret_cast<const float4*>(big);
        float4* dst = reinterpret_cast<float4*>(static_cast<char*>(big) + copy_bytes);
        const dim3 g(cus * (v & 1 ? 32 : 8));
        if (v < 2) hipLaunchKernelGGL(k_peak_copy<1>, g, dim3(256), 0, s, src, dst, copy_bytes / 16);
        else if (v < 4) hipLaunchKernelGGL(k_peak_copy<4>, g, dim3(256), 0, s, src, dst, copy_bytes / 16);
        else hipLaunchKernelGGL(k_peak_copy_nt, g, dim3(256), 0, s, src, dst, copy_bytes / 16);
      }
      (void)hipEventRecord(e1, s);
      if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess) {
        rc = -EIO;
        break;
      }
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r == 0 || ms <= 0.f) continue;
      const double waves = (double)blocks * 4;
      double val;
      if (kind == 0) val = waves * iters * kChains * (2.0 * 32 * 32 * 16) / (ms * 1e-3) / 1e12;
      else if (kind == 1 && v < 2) val = waves * iters * kChains * 2 * (2.0 * 16 * 16 * 4) / (ms * 1e-3) / 1e12;
      else if (kind == 1) val = waves * iters * kChains * (2.0 * 32 * 32 * 2) / (ms * 1e-3) / 1e12;
      else val = 2.0 * copy_bytes / (ms * 1e-3) / 1e9;  // copy: 1 GiB each way; read: 2 GiB
      if (val > best) best = val;
    }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(out);
  if (big) (void)hipFree(big);
  *result = best;
  return rc;
}
