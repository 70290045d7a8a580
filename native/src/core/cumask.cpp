#include "vgpu/cumask.h"

#include <algorithm>

namespace vgpu {

int CuMask::count() const {
  int c = 0;
  for (int w = 0; w < kCuMaskWords; w++) c += __builtin_popcount(words[w]);
  return c;
}

int cu_share_count(int cu_count, int num_xcc, int pct) {
  if (cu_count <= 0) return 0;
  if (num_xcc <= 0) num_xcc = 1;
  if (pct <= 0 || pct >= 100) return cu_count;
  int n = (int)((int64_t)cu_count * pct / 100);
  n = n / num_xcc * num_xcc;
  if (n < num_xcc) n = num_xcc;
  return std::min(n, cu_count);
}

int cu_logical_to_bit(int cu_count, int num_xcc, int num_se, int L) {
  if (num_xcc <= 0) num_xcc = 1;
  const int per_xcc = cu_count / num_xcc;
  if (num_se <= 1 || per_xcc % num_se) return L;  // no (or irregular) SE structure: identity
  const int per_se = per_xcc / num_se;
  const int xcc = L % num_xcc, r = L / num_xcc;
  const int se = r / per_se, k = r % per_se;
  return (k * num_se + se) * num_xcc + xcc;
}

CuMask cu_mask_range(int cu_count, int num_xcc, int begin, int end, int num_se) {
  CuMask m;
  if (num_xcc <= 0) num_xcc = 1;
  cu_count = std::min(cu_count, kMaxCUs);
  m.nbits = cu_count;
  begin = std::max(0, begin / num_xcc * num_xcc);
  end = std::min(cu_count, (end + num_xcc - 1) / num_xcc * num_xcc);
  for (int i = begin; i < end; i++) m.set(cu_logical_to_bit(cu_count, num_xcc, num_se, i));
  return m;
}

CuMask cu_mask_for(int cu_count, int num_xcc, int pct, int range_begin, int range_end, int num_se) {
  if (range_begin >= 0 && range_end > range_begin)
    return cu_mask_range(cu_count, num_xcc, range_begin, range_end, num_se);
  return cu_mask_range(cu_count, num_xcc, 0, cu_share_count(cu_count, num_xcc, pct), num_se);
}

void cu_partition_range(int cu_count, int num_xcc, int split, int slot, int* begin, int* end) {
  if (num_xcc <= 0) num_xcc = 1;
  if (split <= 1) {
    *begin = 0;
    *end = cu_count;
    return;
  }
  int units = cu_count / num_xcc;  // allocation unit = one CU on every XCC
  int base = units / split, rem = units % split;
  if (base == 0) {  // more tenants than units: tenants share units round-robin
    int u = slot % units;
    *begin = u * num_xcc;
    *end = *begin + num_xcc;
    return;
  }
  int start = slot * base + std::min(slot, rem);
  int len = base + (slot < rem ? 1 : 0);
  *begin = start * num_xcc;
  *end = (start + len) * num_xcc;
}

bool cu_mask_balanced(const CuMask& m, int num_xcc) {
  if (num_xcc <= 0) num_xcc = 1;
  int per[16] = {0};
  for (int i = 0; i < m.nbits; i++)
    if (m.test(i)) per[i % num_xcc]++;
  for (int x = 0; x < num_xcc; x++)
    if (per[x] == 0 || per[x] != per[0]) return false;
  return true;
}

CuMask cu_mask_intersect(const CuMask& user, const CuMask& vgpu, int num_xcc) {
  CuMask r;
  r.nbits = vgpu.nbits;
  for (int w = 0; w < kCuMaskWords; w++) r.words[w] = user.words[w] & vgpu.words[w];
  if (r.empty() || !cu_mask_balanced(r, num_xcc)) return vgpu;
  return r;
}

}  // namespace vgpu
