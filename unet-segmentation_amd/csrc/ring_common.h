// LDS-DMA ring helpers shared by the ring kernels (conv3_ring.hip,
// wgrad3_ring.hip): one global_load_lds_dwordx4 per wave from an SGPR base and
// per-lane 32-bit offsets, counted vmcnt waits and a raw s_barrier that leaves
// the DMAs of later ring slots in flight.
#pragma once
#include <hip/hip_runtime.h>

namespace unet {

typedef __attribute__((address_space(3))) unsigned char lds_u8_t;

// one global_load_lds_dwordx4: 16 B per lane from sbase + voff into LDS at the
// wave-uniform byte address `lds` + lane * 16 (M0); the caller retires it with
// a counted vmcnt.  Inline asm: hipcc does not track it (see conv3_dma.hip).
__device__ __forceinline__ void dma_sv(unsigned voff, unsigned long long sbase, unsigned lds_addr) {
  // wave-uniform by construction (wave index, slot, piece); readfirstlane puts it in an SGPR
  const unsigned lds = __builtin_amdgcn_readfirstlane(lds_addr);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

// one global_load_lds_dword: 4 B per lane from sbase + voff into LDS at the
// wave-uniform byte address `lds` + lane * 4 (M0); retired by a counted vmcnt
__device__ __forceinline__ void dma4_sv(unsigned voff, unsigned long long sbase, unsigned lds_addr) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(lds_addr);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

// XCD-aware workgroup order (cdna_hip_programming.md T1): workgroups are dealt
// round robin over the 8 XCDs (linear id = x + gx (y + gy z)); remapped, each
// XCD runs one contiguous run of that order, so the column blocks it computes
// -- the weight slabs every pixel tile of a block re-reads -- and the split's
// operand slices stay in its own 4 MB L2 instead of being fetched from the
// Infinity Cache by all eight.  Identity when the grid does not split evenly.
// Speed only: every (bx, by, bz) is still visited exactly once.
__device__ __forceinline__ void xcd_block(int& bx, int& by, int& bz) {
  const unsigned gx = gridDim.x, gy = gridDim.y, total = gx * gy * gridDim.z;
  unsigned bid = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if ((total & 7u) == 0) bid = (bid & 7u) * (total >> 3) + (bid >> 3);
  bx = (int)(bid % gx);
  bid /= gx;
  by = (int)(bid % gy);
  bz = (int)(bid / gy);
}

__device__ __forceinline__ unsigned long long uniform_u64(const void* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }
// s_waitcnt lgkmcnt(0) as asm: LDS reads issued before it cannot sink below it
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

}  // namespace unet
