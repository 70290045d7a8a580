// CU-mask construction for spatial compute partitioning on MI355X.
//
// The reference limits SMs *temporally* (token bucket). On
// MI355X the hardware offers per-queue CU masks (hsa_amd_queue_cu_set_mask,
// hsa_ext_amd.h:1359), which partition the chip spatially with zero per-launch cost.
//
// Physical mask bit b is mapped by KFD to XCC (b % num_xcc); the XCC-local index
// l = b / num_xcc then goes round-robin over that XCC's shader engines: SE = l % num_se,
// and it is the (l / num_se)-th active CU of that SE (measured on box with a
// HW_ID-recording kernel, profiles/cu_mask_calibration.md).
//
// The *logical* CU index used by ranges below is SE-major inside each XCC: logical L
// -> XCC L % num_xcc, rank r = L / num_xcc, SE = r / cus_per_se, k = r % cus_per_se,
// physical bit = (k * num_se + SE) * num_xcc + XCC. A contiguous logical range of
// 256/N CUs is then "the same whole shader engine(s) on every XCC" for N <= 4 tenants
// (half an SE for N = 8), so co-resident vGPUs do not share an SE's workgroup
// dispatcher. num_se = 1 reproduces the plain interleaved layout.
// Workgroups of a dispatch are dealt round-robin over all 8 XCCs regardless of the
// mask, so a mask must give every XCC the same number of CUs or the slowest XCC
// bounds the kernel - and an XCC with no CU falls back to "all CUs". Masks built
// here are therefore contiguous logical ranges whose length is a multiple of
// num_xcc; disjoint ranges give co-resident vGPUs disjoint physical CUs.
#pragma once

#include <cstdint>

#include "vgpu/config.h"

namespace vgpu {

struct CuMask {
  uint32_t words[kCuMaskWords] = {0};
  int nbits = 0;  // width of the mask (cu_count)
  int count() const;
  bool test(int i) const { return (words[i >> 5] >> (i & 31)) & 1u; }
  void set(int i) { words[i >> 5] |= 1u << (i & 31); }
  bool empty() const { return count() == 0; }
};

// Number of CUs granted for `pct` percent of `cu_count`, rounded down to a multiple
// of `num_xcc` (at least num_xcc). pct <= 0 or >= 100 -> cu_count.
int cu_share_count(int cu_count, int num_xcc, int pct);

// Mask for logical range [begin, end). begin/end are snapped to multiples of num_xcc.
CuMask cu_mask_range(int cu_count, int num_xcc, int begin, int end, int num_se = 1);

// Mask for a vGPU: explicit range if given (begin >= 0), else the first
// cu_share_count() CUs.
CuMask cu_mask_for(int cu_count, int num_xcc, int pct, int range_begin, int range_end, int num_se = 1);

// Physical mask bit of logical CU index L (layout described above).
int cu_logical_to_bit(int cu_count, int num_xcc, int num_se, int L);

// The logical range of vGPU `slot` among `split` equal tenants of one GPU; the
// remainder (in units of num_xcc) goes to the lowest slots. Used by the plugin to
// hand disjoint ranges to co-resident containers.
void cu_partition_range(int cu_count, int num_xcc, int split, int slot, int* begin, int* end);

// True when every XCC gets the same non-zero number of CUs.
bool cu_mask_balanced(const CuMask& m, int num_xcc);

// a & b, rebalanced: if the intersection is unbalanced or empty, returns `b`
// (the vGPU mask wins over a user mask that would escape or hang the partition).
CuMask cu_mask_intersect(const CuMask& user, const CuMask& vgpu, int num_xcc);

}  // namespace vgpu
