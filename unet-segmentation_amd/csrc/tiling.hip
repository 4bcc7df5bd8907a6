// Overlap-tile inference data movement (the strategy of
// scripts/predict1.py:35-49's margin rule): tiles are gathered straight from
// the unpadded image with the mirror ("reflect", edge not repeated, repeated
// for pads beyond the image as np.pad / F.pad iterated) folded into the index,
// and the tile outputs are scattered back into the full-image logits and / or
// the uint8 mask (scripts/predict.py:85-92: softmax[1] > 0.5 == l1 > l0 ->
// 255), so neither the padded image nor the stitched logits need a host pass.
#include <cstdint>

#include "unet_internal.h"

namespace unet {

// whole-sample symmetric index fold (period 2n - 2)
__device__ __forceinline__ int mirror(int i, int n) {
  if (n == 1) return 0;
  const int p = 2 * n - 2;
  i %= p;
  if (i < 0) i += p;
  return i < n ? i : p - i;
}

// tiles[b][c][i][j] = image[c][mirror(oy + i)][mirror(ox + j)], tile t = first + b * stride,
// origin (oy, ox) = ((t / nx) * tile_out - top, (t % nx) * tile_out - left)
__global__ __launch_bounds__(256) void k_tile_gather(const float* __restrict__ img, int c, int h, int w, int ti,
                                                     int to, int top, int left, int nx, int first, int stride,
                                                     int ntiles, float* __restrict__ tiles) {
  const size_t per = (size_t)c * ti * ti;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= per * ntiles) return;
  const int b = (int)(i / per);
  int r = (int)(i - (size_t)b * per);
  const int ch = r / (ti * ti);
  r -= ch * ti * ti;
  const int y = r / ti, x = r - (r / ti) * ti;
  const int t = first + b * stride;
  const int oy = (t / nx) * to - top, ox = (t % nx) * to - left;
  tiles[i] = img[((size_t)ch * h + mirror(oy + y, h)) * w + mirror(ox + x, w)];
}

// tile logits (ntiles, k, to, to) -> full logits (k, h, w) and / or the mask
// (h, w) uint8 = 255 * (l1 > l0) (k == 2); pixels past the image are dropped
__global__ __launch_bounds__(256) void k_tile_scatter(const float* __restrict__ lt, int k, int to, int nx, int first,
                                                      int stride, int ntiles, int h, int w, float* __restrict__ full,
                                                      uint8_t* __restrict__ mask) {
  const size_t per = (size_t)to * to;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= per * ntiles) return;
  const int b = (int)(i / per);
  const int r = (int)(i - (size_t)b * per);
  const int y = r / to, x = r - (r / to) * to;
  const int t = first + b * stride;
  const int gy = (t / nx) * to + y, gx = (t % nx) * to + x;
  if (gy >= h || gx >= w) return;
  const float* src = lt + (size_t)b * k * per + r;
  if (full)
    for (int q = 0; q < k; ++q) full[((size_t)q * h + gy) * w + gx] = src[(size_t)q * per];
  if (mask) mask[(size_t)gy * w + gx] = src[per] > src[0] ? 255 : 0;
}

hipError_t launch_tile_gather(const float* img, int c, int h, int w, int ti, int to, int top, int left, int nx,
                              int first, int stride, int ntiles, float* tiles, hipStream_t s) {
  if (c < 1 || h < 1 || w < 1 || ti < 1 || to < 1 || to > ti || nx < 1 || first < 0 || stride < 1 || ntiles < 1)
    return hipErrorInvalidValue;
  const size_t total = (size_t)c * ti * ti * ntiles;
  hipLaunchKernelGGL(k_tile_gather, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, img, c, h, w, ti, to, top,
                     left, nx, first, stride, ntiles, tiles);
  return hipGetLastError();
}

hipError_t launch_tile_scatter(const float* lt, int k, int to, int nx, int first, int stride, int ntiles, int h,
                               int w, float* full, uint8_t* mask, hipStream_t s) {
  if (k < 1 || to < 1 || nx < 1 || first < 0 || stride < 1 || ntiles < 1 || h < 1 || w < 1 || (mask && k != 2) ||
      (!full && !mask))
    return hipErrorInvalidValue;
  const size_t total = (size_t)to * to * ntiles;
  hipLaunchKernelGGL(k_tile_scatter, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, lt, k, to, nx, first,
                     stride, ntiles, h, w, full, mask);
  return hipGetLastError();
}

}  // namespace unet
