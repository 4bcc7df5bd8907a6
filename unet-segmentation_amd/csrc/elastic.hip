// Elastic-deformation input pipeline on the GPU:
// utils/augmentations.py:4-39 (elastic_deform_image_and_mask) and the
// utils/dataset.py:84-111 steps around it (uint8 casts, ToTensor, mask > 0),
// for a batch of N samples in one stream.
//
//   noise (N, 2, H, W) fp64 uniform [0, 1): field 0 -> dx, field 1 -> dy
//   k_gauss_v:  t = sum_j w[j] (2 u[y + j - r][x] - 1)      (axis 0, zeros outside)
//   k_gauss_h:  d = alpha * sum_j w[j] t[y][x + j - r]       (axis 1, zeros outside)
//   k_warp:     (cy, cx) = (y + dy, x + dx); image bilinear, labels nearest,
//               half-sample-symmetric ("reflect") extension; integer outputs
//               rounded half up and clamped (scipy.ndimage's conversion)
//   x = uint8(image') / 255 (fp32), target = uint8(label') > 0
//
// Everything that decides a rounding is fp64 in the same operation order as
// oracle/elastic_oracle.py (sequential tap sums, no fma contraction), so the
// outputs are bit-identical to the oracle -- and, through it, to the reference
// (tests/golden/elastic.npz) -- except for interpolated values within ~1e-13 of
// a rounding boundary.  The filters run from LDS tiles (fp64 VALU bound: 2 x
// (2r + 1) multiply-adds per field per pixel); the warp is a gather from the
// L2-resident uint8 / uint16 planes.
#include <cmath>
#include <cstdint>

#include "unet_internal.h"

#pragma clang fp contract(off)

namespace unet {

constexpr int kGaussMaxTaps = 321;  // r <= 160
__constant__ double c_gauss_w[kGaussMaxTaps];

// axis 0: a workgroup = 64 columns x TY output rows of one field; LDS holds
// rows [y0 - r, y0 + TY + r) of the 64 columns (2u - 1, zeros outside)
template <int TY>
__global__ __launch_bounds__(256) void k_gauss_v(const double* __restrict__ u, double* __restrict__ t, int h, int w,
                                                 int r) {
  extern __shared__ double gl[];
  const int fld = blockIdx.z;  // n * 2 + field
  const int x0 = blockIdx.x * 64, y0 = blockIdx.y * TY;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const double* src = u + (size_t)fld * h * w;
  const int rows = TY + 2 * r;
  const int x = x0 + tx;
  for (int i = ty; i < rows; i += 4) {
    const int y = y0 - r + i;
    gl[i * 64 + tx] = (y >= 0 && y < h && x < w) ? src[(size_t)y * w + x] * 2 - 1 : 0.0;
  }
  __syncthreads();
  if (x >= w) return;
  const int taps = 2 * r + 1;
  for (int k = ty; k < TY; k += 4) {
    const int y = y0 + k;
    if (y >= h) break;
    double s = 0.0;
    for (int j = 0; j < taps; ++j) s = s + c_gauss_w[j] * gl[(k + j) * 64 + tx];
    t[(size_t)fld * h * w + (size_t)y * w + x] = s;
  }
}

// axis 1: a workgroup = 4 rows x 256 output columns; LDS rows hold columns
// [x0 - r, x0 + 256 + r) (zeros outside); output scaled by alpha
__global__ __launch_bounds__(256) void k_gauss_h(const double* __restrict__ t, double* __restrict__ d, int h, int w,
                                                 int r, double alpha) {
  extern __shared__ double gl[];
  const int fld = blockIdx.z;
  const int x0 = blockIdx.x * 256, y0 = blockIdx.y * 4;
  const int cols = 256 + 2 * r;
  const double* src = t + (size_t)fld * h * w;
  for (int i = threadIdx.x; i < 4 * cols; i += 256) {
    const int ry = i / cols, cx = i - ry * cols;
    const int y = y0 + ry, x = x0 - r + cx;
    gl[i] = (y < h && x >= 0 && x < w) ? src[(size_t)y * w + x] : 0.0;
  }
  __syncthreads();
  const int ry = threadIdx.x >> 6, lx = threadIdx.x & 63;
  const int y = y0 + ry;
  if (y >= h) return;
  const int taps = 2 * r + 1;
  for (int q = 0; q < 4; ++q) {
    const int c = lx + 64 * q, x = x0 + c;
    if (x >= w) break;
    double s = 0.0;
    for (int j = 0; j < taps; ++j) s = s + c_gauss_w[j] * gl[ry * cols + c + j];
    d[(size_t)fld * h * w + (size_t)y * w + x] = s * alpha;
  }
}

// half-sample-symmetric fold of a coordinate into [-0.5, n - 0.5] (numpy's mod)
__device__ __forceinline__ double reflect_coord(double c, int n) {
  if (n == 1) return 0.0;
  const double p = 2.0 * n;
  double m = fmod(c + 0.5, p);
  if (m != 0.0 && m < 0.0) m += p;
  if (m >= n) m = p - m;
  return m - 0.5;
}
__device__ __forceinline__ int reflect_index(int i, int n) {
  if (i < 0) i = -i - 1;
  if (i >= n) i = 2 * n - i - 1;
  return i;
}
__device__ __forceinline__ unsigned to_uint(double v, double hi) {
  v = floor(fmax(v, 0.0) + 0.5);
  return (unsigned)(v > hi ? hi : v);
}

__global__ __launch_bounds__(256) void k_warp(const uint8_t* __restrict__ img, const uint16_t* __restrict__ lab,
                                              const double* __restrict__ d, int n, int h, int w,
                                              float* __restrict__ xo, uint8_t* __restrict__ to,
                                              uint8_t* __restrict__ io) {
  const size_t hw = (size_t)h * w;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= (size_t)n * hw) return;
  const int s = (int)(i / hw);
  const int p = (int)(i - (size_t)s * hw);
  const int y = p / w, x = p - (p / w) * w;
  const double dx = d[(size_t)(2 * s) * hw + p], dy = d[(size_t)(2 * s + 1) * hw + p];
  const double cy = reflect_coord((double)y + dy, h), cx = reflect_coord((double)x + dx, w);
  const uint8_t* im = img + (size_t)s * hw;
  const uint16_t* lb = lab + (size_t)s * hw;
  // order 1 (image)
  const double fy = floor(cy), fx = floor(cx);
  const double ty = cy - fy, tx = cx - fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int ya = reflect_index(y0, h), yb = reflect_index(y0 + 1, h);
  const int xa = reflect_index(x0, w), xb = reflect_index(x0 + 1, w);
  const double v = (1 - ty) * ((1 - tx) * (double)im[ya * w + xa] + tx * (double)im[ya * w + xb]) +
                   ty * ((1 - tx) * (double)im[yb * w + xa] + tx * (double)im[yb * w + xb]);
  const unsigned iv = to_uint(v, 255.0);
  // order 0 (labels): nearest, round half up; the uint16 -> uint8 cast wraps
  const int ny = reflect_index((int)floor(cy + 0.5), h), nx = reflect_index((int)floor(cx + 0.5), w);
  const unsigned lv = lb[ny * w + nx] & 0xffu;
  xo[i] = (float)iv / 255.0f;
  to[i] = lv != 0 ? 1 : 0;
  if (io) io[i] = (uint8_t)iv;
}

static int gauss_radius(double sigma) { return (int)(4.0 * sigma + 0.5); }

size_t elastic_ws_bytes(int n, int h, int w) { return (size_t)2 * (2 * (size_t)n * h * w) * sizeof(double); }

hipError_t launch_elastic(const uint8_t* img, const uint16_t* lab, int n, int h, int w, const double* noise,
                          double alpha, double sigma, float* x_out, uint8_t* t_out, uint8_t* img_out, void* ws,
                          hipStream_t s) {
  const int r = gauss_radius(sigma);
  if (n < 1 || h < 1 || w < 1 || !(sigma > 0) || r < 0 || 2 * r + 1 > kGaussMaxTaps) return hipErrorInvalidValue;
  // kernel weights exactly as oracle/elastic_oracle.py gaussian_kernel (fp64, normalised by the sum)
  double wts[kGaussMaxTaps];
  double sum = 0.0;
  for (int j = -r; j <= r; ++j) {
    const double x = (double)j;
    wts[j + r] = std::exp(-0.5 / (sigma * sigma) * x * x);
  }
  for (int j = 0; j <= 2 * r; ++j) sum += wts[j];
  for (int j = 0; j <= 2 * r; ++j) wts[j] /= sum;
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_gauss_w), wts, sizeof(double) * (2 * r + 1), 0,
                                        hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  double* tmp = reinterpret_cast<double*>(ws);
  double* disp = tmp + (size_t)2 * n * h * w;
  constexpr int TY = 64;
  const size_t lv = (size_t)(TY + 2 * r) * 64 * sizeof(double), lh = (size_t)4 * (256 + 2 * r) * sizeof(double);
  static bool attr = false;
  if (!attr) {
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gauss_v<TY>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (lv > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_gauss_v<TY>), dim3((w + 63) / 64, (h + TY - 1) / TY, 2 * n), dim3(256), lv, s, noise, tmp, h,
                     w, r);
  hipLaunchKernelGGL(k_gauss_h, dim3((w + 255) / 256, (h + 3) / 4, 2 * n), dim3(256), lh, s, tmp, disp, h, w, r,
                     alpha);
  const size_t total = (size_t)n * h * w;
  hipLaunchKernelGGL(k_warp, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, img, lab, disp, n, h, w, x_out,
                     t_out, img_out);
  return hipGetLastError();
}

}  // namespace unet
