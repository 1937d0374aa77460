// oracle_voxel.h — TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// pcl::VoxelGrid<PointXYZI>::applyFilter as PCL 1.10 states it (PCL is not in /root/reference
// and not in this image; the algorithm is restated from its published source), with
// downsample_all_data_ = true and min_points_per_voxel_ = 0, the configuration of every
// downSizeFilter* in the reference (FA:1268-1270; MO:92-104, 1157-1167, 1225-1267):
//   * min / max over x, y, z (getMinMax3D);
//   * the (max - min) * inv + 1 product check: over INT32_MAX the filter warns and returns the
//     input unchanged;
//   * min_b = floor(min * inv), div = max_b - min_b + 1, idx = i0 + i1 * div0 + i2 * div0 * div1
//     with i_a = int(floor(p_a * inv) - float(min_b_a));
//   * std::sort of (idx, point index) by idx alone, then one centroid per run of equal idx:
//     x, y, z, intensity summed in float in the sorted order and divided by the run length.
// `stable` = true replaces std::sort with std::stable_sort: the run is then summed in input order,
// which is what the device VoxelGrid does (llsr_map.hip), so that variant is bit-exact against it;
// the std::sort variant (the PCL statement) differs only in the within-voxel summation order.
#ifndef LLSR_ORACLE_VOXEL_H_
#define LLSR_ORACLE_VOXEL_H_
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

namespace oracle_voxel {

// in: n points as x, y, z, intensity; out: the centroids, same layout.
inline void voxel_grid(const float* in, size_t n, float leaf, std::vector<float>& out, bool stable = false) {
  out.clear();
  if (n == 0) return;
  const float inv = 1.0f / leaf;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (size_t k = 0; k < n; ++k)
    for (int a = 0; a < 3; ++a) {
      mn[a] = std::min(mn[a], in[4 * k + a]);
      mx[a] = std::max(mx[a], in[4 * k + a]);
    }
  const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1, dy = (int64_t)((mx[1] - mn[1]) * inv) + 1,
                dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
  if (dx * dy * dz > (int64_t)INT32_MAX) {
    out.assign(in, in + 4 * n);
    return;
  }
  int minb[3], maxb[3], div[3];
  for (int a = 0; a < 3; ++a) {
    minb[a] = (int)std::floor(mn[a] * inv);
    maxb[a] = (int)std::floor(mx[a] * inv);
    div[a] = maxb[a] - minb[a] + 1;
  }
  const int mul1 = div[0], mul2 = div[0] * div[1];
  struct Idx { unsigned idx; unsigned cloud; };
  std::vector<Idx> iv;
  iv.reserve(n);
  for (size_t k = 0; k < n; ++k) {
    const int i0 = (int)(std::floor(in[4 * k] * inv) - (float)minb[0]);
    const int i1 = (int)(std::floor(in[4 * k + 1] * inv) - (float)minb[1]);
    const int i2 = (int)(std::floor(in[4 * k + 2] * inv) - (float)minb[2]);
    iv.push_back({(unsigned)(i0 + i1 * mul1 + i2 * mul2), (unsigned)k});
  }
  auto less = [](const Idx& a, const Idx& b) { return a.idx < b.idx; };
  if (stable)
    std::stable_sort(iv.begin(), iv.end(), less);
  else
    std::sort(iv.begin(), iv.end(), less);
  size_t k = 0;
  while (k < iv.size()) {
    size_t e = k + 1;
    while (e < iv.size() && iv[e].idx == iv[k].idx) ++e;
    float s[4] = {0, 0, 0, 0};
    for (size_t q = k; q < e; ++q)
      for (int a = 0; a < 4; ++a) s[a] += in[4 * iv[q].cloud + a];
    const float cnt = (float)(e - k);
    for (int a = 0; a < 4; ++a) out.push_back(s[a] / cnt);
    k = e;
  }
}

}  // namespace oracle_voxel

#endif  // LLSR_ORACLE_VOXEL_H_
