// Per-pixel loss weight maps: scripts/preprocess_data.py
// :17-77 (calculate_weight_map) for a batch of label maps, on the device.
// weight = fp32(wc[class]) + w0 * exp(-(d1 + d2)^2 / (2 (sigma^2 + 1e-8))), with
// wc = 1 / (count / total) of the pixel's class (fp64, 0 for an empty class)
// and d1 = d2 = 0: the reference's per-object distance, min(edt(obj),
// edt(obj == 0)), is identically zero (each transform is 0 where its mask is
// 0, and one of the two masks is 0 at every pixel), so the separation term is
// exactly w0 (oracle/weightmap_oracle.py states the argument; the fixtures made
// by the reference pin it).  Two launches: a per-sample foreground count
// (wave reduction + one 64-bit atomic per workgroup) and the map.
#include <cmath>
#include <cstdint>

#include "unet_internal.h"

#pragma clang fp contract(off)

namespace unet {

__global__ __launch_bounds__(256) void k_wm_count(const uint16_t* __restrict__ lab, size_t hw,
                                                  unsigned long long* __restrict__ cnt) {
  const int s = blockIdx.y;
  const uint16_t* l = lab + (size_t)s * hw;
  unsigned c = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < hw; i += (size_t)gridDim.x * blockDim.x)
    c += l[i] != 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  __shared__ unsigned part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(cnt + s, (unsigned long long)(part[0] + part[1] + part[2] + part[3]));
}

__global__ __launch_bounds__(256) void k_wm_apply(const uint16_t* __restrict__ lab, int n, size_t hw,
                                                  const unsigned long long* __restrict__ cnt, double w0,
                                                  double sigma, float* __restrict__ out, double* __restrict__ out64) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)n * hw) return;
  const int s = (int)(i / hw);
  const double total = (double)hw, fg = (double)cnt[s], bg = total - fg;
  const bool is_fg = lab[i] != 0;
  const double wc = is_fg ? (fg > 0 ? 1.0 / (fg / total) : 0.0) : (bg > 0 ? 1.0 / (bg / total) : 0.0);
  const double d = 0.0;  // d1 + d2
  const double term = w0 * exp(-(d * d) / (2 * (sigma * sigma + 1e-8)));
  const double v = (double)(float)wc + term;
  out[i] = (float)v;
  if (out64) out64[i] = v;
}

size_t weight_map_ws_bytes(int n) { return (size_t)n * sizeof(unsigned long long); }

hipError_t launch_weight_map(const uint16_t* lab, int n, int h, int w, double w0, double sigma, float* out,
                             double* out64, void* ws, hipStream_t s) {
  if (n < 1 || h < 1 || w < 1) return hipErrorInvalidValue;
  auto* cnt = reinterpret_cast<unsigned long long*>(ws);
  hipError_t e = hipMemsetAsync(cnt, 0, weight_map_ws_bytes(n), s);
  if (e != hipSuccess) return e;
  const size_t hw = (size_t)h * w;
  unsigned gx = (unsigned)((hw + 255) / 256);
  if (gx > 256) gx = 256;
  hipLaunchKernelGGL(k_wm_count, dim3(gx, n), dim3(256), 0, s, lab, hw, cnt);
  const size_t total = (size_t)n * hw;
  hipLaunchKernelGGL(k_wm_apply, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, lab, n, hw, cnt, w0, sigma,
                     out, out64);
  return hipGetLastError();
}

}  // namespace unet
