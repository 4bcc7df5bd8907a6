// Ring tiles 83, 84 and the persistent 88 (k_conv3_ring PT = 1, the geometry
// of 84: each workgroup walks pixel tiles with the next tile's halo and first
// weights in flight during this tile's last chunk and epilogue), a second
// translation unit so the ring instantiations compile in two halves in
// parallel.  (A persistent 82 geometry spilled 200-500 B per lane around its
// epilogue and ran 1.2-1.4x slower than 82; measured 88 vs 84: 7-11 % faster on
// the 64-128-channel layers, tools/conv_bench.py --a16.)
#include "conv3_ring_kernel.h"
#include "unet_internal.h"

namespace unet {

hipError_t go_conv3_ring_pt(const IgemmArgs& a, hipStream_t s, int tile) {
  switch (tile) {
    case 83: return go_ring<4, 128, 2, 2, 32, 2, 0>(a, s);
    case 84: return go_ring<8, 64, 8, 1, 64, 2, 0>(a, s);
    case 88: return go_ring<8, 64, 8, 1, 64, 2, 1>(a, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
