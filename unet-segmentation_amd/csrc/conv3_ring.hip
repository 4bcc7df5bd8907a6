// k_conv3_ring tiles 81, 82 and the ring tile table (kernel:
// conv3_ring_kernel.h; tiles 83, 84 and the persistent 88 are instantiated in
// conv3_ring_pt.hip, a second translation unit that compiles in parallel).
#include "conv3_ring_kernel.h"

namespace unet {

// tile ids (igemm.hip tile_info 81-84; 88 the geometry of 84, persistent):
// TH x 32 pixels x BN columns, CK-channel chunks
bool conv3_ring_tile_shape(int tile, int& th, int& bn, int& ck) {
  if (tile == 88) tile -= 4;
  switch (tile) {
    case 81: th = 8; bn = 128; ck = 64; return true;  // 8 waves (4 x 2), 64 x 64 per wave; 138 KB, 1 WG/CU
    case 82: th = 8; bn = 64; ck = 32; return true;   // 4 waves (4 x 1), 64 x 64 per wave; 57 KB, 2 WG/CU
    case 83: th = 4; bn = 128; ck = 32; return true;  // 4 waves (2 x 2), 64 x 64 per wave; 51 KB, 3 WG/CU
    case 84: th = 8; bn = 64; ck = 64; return true;   // 8 waves (8 x 1), 32 x 64 per wave; 114 KB, 1 WG/CU
    default: return false;
  }
}

// A sources bf16 (the plan's raw conv outputs with their consumer transform,
// normalised copies, padded dY, pooled maps, convT outputs); a transform only
// on source 0 (the second source of a concat is the convT output); no split
// operands; the BN table must fit the LDS beside the ring; the persistent
// tiles take the whole K per workgroup
bool conv3_ring_fits(const IgemmArgs& a, int tile) {
  int th, bn, ck;
  if (!conv3_ring_tile_shape(tile, th, bn, ck)) return false;
  const Gather& g = a.a;
  const bool two = g.c_split < g.Cg, xtf = g.s[0].scale != nullptr;
  size_t smem = 0;
  switch (tile) {
    case 81: smem = ring_smem<8, 128, 64>(a, xtf); break;
    case 82: smem = ring_smem<8, 64, 32>(a, xtf); break;
    case 83: smem = ring_smem<4, 128, 32>(a, xtf); break;
    default: smem = ring_smem<8, 64, 64>(a, xtf); break;
  }
  if (tile == 88 && a.ksplit > 1) return false;
  return a.bh != nullptr && a.bl == nullptr && a.N % bn == 0 && g.taps_h == 3 && g.taps_w == 3 && g.stride == 1 &&
         a.K == 9 * g.Cg && g.Cg % ck == 0 && g.c_split % ck == 0 && g.s[0].h16 &&
         (!two || (g.s[1].h16 && g.s[1].scale == nullptr)) && (!xtf || g.s[0].shift != nullptr) &&
         smem <= 160 * 1024;
}

hipError_t go_conv3_ring_tile(const IgemmArgs& a, hipStream_t s, int tile) {
  if (!conv3_ring_fits(a, tile)) return hipErrorInvalidValue;
  switch (tile) {
    case 81: return go_ring<8, 128, 4, 2, 64, 2, 0>(a, s);
    case 82: return go_ring<8, 64, 4, 1, 32, 2, 0>(a, s);
    case 83: case 84: case 88: return go_conv3_ring_pt(a, s, tile);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet

