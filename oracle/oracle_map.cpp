// oracle_map.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Scalar CPU restatement of MapOptimization's local-map assembly, both branches of
// extractSurroundingKeyFrames (MO:1096-1232):
//   * the keyframe store of saveKeyFramesAndFactor (MO:1686-1752): key pose x, y, z, roll, pitch,
//     yaw (cloudKeyPoses3D / 6D, intensity = keyframe index) + the corner / surf / outlier clouds;
//   * extractSurroundingKeyFrames (MO:1151-1231): radiusSearch of the key poses around the robot
//     position (MO:1155-1159; nanoflann RadiusResultSet keeps d^2 < float(r * r), nanoflann_pcl.h:
//     155-175, the distance being ((0 + dx^2) + dy^2) + dz^2 of L2_Simple_Adaptor), VoxelGrid 1.0 of
//     those poses (MO:1166-1167), the surroundingExistingKeyPosesID list kept in the reference's
//     erase / append order (MO:1169-1222), transformPointCloud (MO:671-701) of every listed keyframe
//     and the concatenation + VoxelGrid 0.2 / 0.4 (MO:1224-1231);
//   * with enable_loop_closure (the VLP-32c / HDL-64E blocks, CFG:91, 159), MO:1099-1151 as written:
//     three deques of clouds transformed when pushed (recent{Corner,Surf,Outlier}CloudKeyFrames),
//     rebuilt from the newest keyframe backwards while shorter than surrounding_keyframe_search_num,
//     else pop-front / push-back of the newest when latestFrameID changed.
// The radius search is brute force here: the result SET is what matters, because the VoxelGrid of
// the selected poses only keeps the integer mean of their indices (exact in float for any summation
// order below 2^24). The _ref build (-DLLSR_ORACLE_NANOFLANN) also exports ref_keypose_radius over
// the reference's own nanoflann.hpp, the cross-check of that set (tests/test_map_oracle.py).
// sin / cos are the host glibc float functions the reference calls on the float pose fields.
#include <algorithm>
#include <array>
#include <deque>
#include <cmath>
#include <cstring>
#include <vector>

#include "../include/llsr.h"
#include "oracle.h"
#include "oracle_voxel.h"
#ifdef LLSR_ORACLE_NANOFLANN
#include "nanoflann.hpp"
#endif

#ifndef LLSR_ORACLE_NANOFLANN
namespace {

// transformPointCloud(cloudIn, transformIn) (MO:671-701): x, y, z, intensity in, rotated by yaw,
// roll, pitch and translated, in the reference's float expression order.
void transform_cloud(const std::vector<float>& in, const float* t, std::vector<float>& out) {
  const float x = t[0], y = t[1], z = t[2], roll = t[3], pitch = t[4], yaw = t[5];
  const size_t n = in.size() / 4;
  for (size_t k = 0; k < n; ++k) {
    const float* p = &in[4 * k];
    const float x1 = std::cos(yaw) * p[0] - std::sin(yaw) * p[1];
    const float y1 = std::sin(yaw) * p[0] + std::cos(yaw) * p[1];
    const float z1 = p[2];
    const float x2 = x1;
    const float y2 = std::cos(roll) * y1 - std::sin(roll) * z1;
    const float z2 = std::sin(roll) * y1 + std::cos(roll) * z1;
    out.push_back(std::cos(pitch) * x2 + std::sin(pitch) * z2 + x);
    out.push_back(y2 + y);
    out.push_back(-std::sin(pitch) * x2 + std::cos(pitch) * z2 + z);
    out.push_back(p[3]);
  }
}

}  // namespace
#endif

struct oracle_map {
  float radius, kp_leaf, corner_leaf, surf_leaf;
  int loop_closure = 0, search_num = 50;                   // _loop_closure_enabled, _surrounding_keyframe_search_num
  std::vector<std::array<float, 6>> pose;                  // x, y, z, roll, pitch, yaw
  std::vector<std::vector<float>> corner, surf, outlier;   // per keyframe, x y z i
  std::vector<int> existing;                               // surroundingExistingKeyPosesID
  // loop-closure branch (mapOptimization.h:139-142): transformed clouds + their keyframe indices
  std::deque<std::vector<float>> recent_corner, recent_surf, recent_outlier;
  std::deque<int> recent_id;
  int latestFrameID = 0;                                    // MO:301
};

#ifdef LLSR_ORACLE_NANOFLANN
namespace {
struct PoseAdaptor {
  const float* p = nullptr;
  size_t n = 0;
  size_t kdtree_get_point_count() const { return n; }
  float kdtree_get_pt(const size_t idx, int dim) const { return p[4 * idx + dim]; }
  template <class BBOX> bool kdtree_get_bbox(BBOX&) const { return false; }
};
using PoseTree = nanoflann::KDTreeSingleIndexAdaptor<nanoflann::SO3_Adaptor<float, PoseAdaptor>, PoseAdaptor, 3, int>;
}  // namespace
#endif

extern "C" {

int64_t oracle_voxel_grid(const float* in, int64_t n, float leaf, int32_t stable, float* out) {
  if (n < 0 || (n > 0 && (!in || !out)) || !(leaf > 0)) return -1;
  std::vector<float> o;
  oracle_voxel::voxel_grid(in, (size_t)n, leaf, o, stable != 0);
  if (!o.empty()) std::memcpy(out, o.data(), o.size() * sizeof(float));
  return (int64_t)(o.size() / 4);
}

// Indices (ascending) of the K key poses (x, y, z, intensity) with d^2 < float(radius^2).
int32_t oracle_keypose_radius(const float* poses4, int32_t K, const float* pos, float radius, int32_t* out) {
  const float r2 = (float)((double)radius * (double)radius);
  int32_t n = 0;
  for (int k = 0; k < K; ++k) {
    float d = 0;
    for (int a = 0; a < 3; ++a) {
      const float df = pos[a] - poses4[4 * k + a];
      d += df * df;
    }
    if (d < r2) out[n++] = k;
  }
  return n;
}

#ifdef LLSR_ORACLE_NANOFLANN

// KdTreeFLANN::radiusSearch (nanoflann_pcl.h:155-175) over the reference's kd-tree; ascending index.
int32_t ref_keypose_radius(const float* poses4, int32_t K, const float* pos, float radius, int32_t* out) {
  if (K <= 0) return 0;
  PoseAdaptor ad;
  ad.p = poses4;
  ad.n = (size_t)K;
  PoseTree tree(3, ad);
  tree.buildIndex();
  std::vector<std::pair<int, float>> res;
  nanoflann::RadiusResultSet<float, int> rs(static_cast<float>((double)radius * (double)radius), res);
  tree.findNeighbors(rs, pos, nanoflann::SearchParams());
  std::vector<int> idx;
  for (auto& r : res) idx.push_back(r.first);
  std::sort(idx.begin(), idx.end());
  for (size_t k = 0; k < idx.size(); ++k) out[k] = idx[k];
  return (int32_t)idx.size();
}
#endif

#ifndef LLSR_ORACLE_NANOFLANN
oracle_map* oracle_map_create(float radius, float keypose_leaf, float corner_leaf, float surf_leaf,
                              int32_t loop_closure, int32_t search_num) {
  oracle_map* m = new oracle_map();
  m->loop_closure = loop_closure;
  m->search_num = search_num;
  m->radius = radius;
  m->kp_leaf = keypose_leaf;
  m->corner_leaf = corner_leaf;
  m->surf_leaf = surf_leaf;
  return m;
}

void oracle_map_destroy(oracle_map* m) { delete m; }

// transformPointCloud (MO:671-701) of n points by a key pose (x, y, z, roll, pitch, yaw).
void oracle_transform_cloud(const float* pose6, const float* in, int64_t n, float* out) {
  std::vector<float> src(in, in + 4 * (size_t)n), dst;
  transform_cloud(src, pose6, dst);
  if (!dst.empty()) std::memcpy(out, dst.data(), dst.size() * sizeof(float));
}

int32_t oracle_map_add_keyframe(oracle_map* m, const float* pose6, const float* c, int32_t nc, const float* s,
                                int32_t ns, const float* o, int32_t no) {
  if (!m || !pose6 || nc < 0 || ns < 0 || no < 0) return LLSR_EINVAL;
  std::array<float, 6> p;
  std::memcpy(p.data(), pose6, sizeof p);
  m->pose.push_back(p);
  m->corner.emplace_back(c, c + 4 * (size_t)nc);
  m->surf.emplace_back(s, s + 4 * (size_t)ns);
  m->outlier.emplace_back(o, o + 4 * (size_t)no);
  return (int32_t)m->pose.size() - 1;
}

// extractSurroundingKeyFrames (MO:1151-1231). Outputs: the two downsampled local maps (capacity =
// the raw map sizes, which raw_counts[0..1] report), the keyframe id list after the update,
// raw_counts = {corner map, surf map, selected poses, downsampled poses}.
int32_t oracle_map_extract(oracle_map* m, const float* pos, int32_t stable, float* corner_out, int64_t cap_c,
                           int64_t* n_corner, float* surf_out, int64_t cap_s, int64_t* n_surf, int32_t* ids,
                           int32_t cap_ids, int32_t* n_ids, int64_t* raw_counts) {
  if (!m || !pos || !n_corner || !n_surf || !n_ids || !raw_counts) return LLSR_EINVAL;
  *n_corner = *n_surf = 0;
  *n_ids = 0;
  for (int k = 0; k < 4; ++k) raw_counts[k] = 0;
  const int K = (int)m->pose.size();
  if (K == 0) return LLSR_OK;  // MO:1097
  if (m->loop_closure) {
    std::vector<float> cm, sm;
    if ((int)m->recent_corner.size() < m->search_num) {  // MO:1101-1123
      m->recent_corner.clear();
      m->recent_surf.clear();
      m->recent_outlier.clear();
      m->recent_id.clear();
      const int numPoses = K;
      for (int i = numPoses - 1; i >= 0; --i) {
        const int thisKeyInd = i;  // (int)cloudKeyPoses3D->points[i].intensity, = i (MO:1695-1697)
        std::vector<float> c, s, o;
        transform_cloud(m->corner[thisKeyInd], m->pose[thisKeyInd].data(), c);
        transform_cloud(m->surf[thisKeyInd], m->pose[thisKeyInd].data(), s);
        transform_cloud(m->outlier[thisKeyInd], m->pose[thisKeyInd].data(), o);
        m->recent_corner.push_front(c);
        m->recent_surf.push_front(s);
        m->recent_outlier.push_front(o);
        m->recent_id.push_front(thisKeyInd);
        if ((int)m->recent_corner.size() >= m->search_num) break;
      }
    } else if (m->latestFrameID != K - 1) {  // MO:1124-1144
      m->recent_corner.pop_front();
      m->recent_surf.pop_front();
      m->recent_outlier.pop_front();
      m->recent_id.pop_front();
      m->latestFrameID = K - 1;
      std::vector<float> c, s, o;
      transform_cloud(m->corner[m->latestFrameID], m->pose[m->latestFrameID].data(), c);
      transform_cloud(m->surf[m->latestFrameID], m->pose[m->latestFrameID].data(), s);
      transform_cloud(m->outlier[m->latestFrameID], m->pose[m->latestFrameID].data(), o);
      m->recent_corner.push_back(c);
      m->recent_surf.push_back(s);
      m->recent_outlier.push_back(o);
      m->recent_id.push_back(m->latestFrameID);
    }
    for (size_t i = 0; i < m->recent_corner.size(); ++i) {  // MO:1147-1151
      cm.insert(cm.end(), m->recent_corner[i].begin(), m->recent_corner[i].end());
      sm.insert(sm.end(), m->recent_surf[i].begin(), m->recent_surf[i].end());
      sm.insert(sm.end(), m->recent_outlier[i].begin(), m->recent_outlier[i].end());
    }
    raw_counts[0] = (int64_t)(cm.size() / 4);
    raw_counts[1] = (int64_t)(sm.size() / 4);
    std::vector<float> cds, sds;
    oracle_voxel::voxel_grid(cm.data(), cm.size() / 4, m->corner_leaf, cds, stable != 0);
    oracle_voxel::voxel_grid(sm.data(), sm.size() / 4, m->surf_leaf, sds, stable != 0);
    *n_corner = (int64_t)(cds.size() / 4);
    *n_surf = (int64_t)(sds.size() / 4);
    *n_ids = (int32_t)m->recent_id.size();
    if (*n_corner > cap_c || *n_surf > cap_s || *n_ids > cap_ids) return LLSR_ERANGE;
    if (!cds.empty()) std::memcpy(corner_out, cds.data(), cds.size() * sizeof(float));
    if (!sds.empty()) std::memcpy(surf_out, sds.data(), sds.size() * sizeof(float));
    for (int k = 0; k < *n_ids; ++k) ids[k] = m->recent_id[k];
    return LLSR_OK;
  }
  std::vector<float> p4(4 * (size_t)K);
  for (int k = 0; k < K; ++k) {
    for (int a = 0; a < 3; ++a) p4[4 * k + a] = m->pose[k][a];
    p4[4 * k + 3] = (float)k;
  }
  std::vector<int32_t> sel(K);
  const int ns = oracle_keypose_radius(p4.data(), K, pos, m->radius, sel.data());
  std::vector<float> sp;
  for (int k = 0; k < ns; ++k) sp.insert(sp.end(), &p4[4 * sel[k]], &p4[4 * sel[k]] + 4);
  std::vector<float> ds;
  oracle_voxel::voxel_grid(sp.data(), (size_t)ns, m->kp_leaf, ds, stable != 0);
  const int nds = (int)(ds.size() / 4);
  raw_counts[2] = ns;
  raw_counts[3] = nds;
  // MO:1169-1189: drop listed keyframes no downsampled pose names
  for (size_t i = 0; i < m->existing.size(); ++i) {
    bool found = false;
    for (int j = 0; j < nds; ++j)
      if (m->existing[i] == (int)ds[4 * j + 3]) { found = true; break; }
    if (!found) { m->existing.erase(m->existing.begin() + i); --i; }
  }
  // MO:1190-1222: append the new ones in downsampled order
  for (int j = 0; j < nds; ++j) {
    const int id = (int)ds[4 * j + 3];
    if (std::find(m->existing.begin(), m->existing.end(), id) == m->existing.end()) m->existing.push_back(id);
  }
  std::vector<float> cm, sm;
  for (int id : m->existing) {
    transform_cloud(m->corner[id], m->pose[id].data(), cm);
    transform_cloud(m->surf[id], m->pose[id].data(), sm);
    transform_cloud(m->outlier[id], m->pose[id].data(), sm);
  }
  raw_counts[0] = (int64_t)(cm.size() / 4);
  raw_counts[1] = (int64_t)(sm.size() / 4);
  std::vector<float> cds, sds;
  oracle_voxel::voxel_grid(cm.data(), cm.size() / 4, m->corner_leaf, cds, stable != 0);
  oracle_voxel::voxel_grid(sm.data(), sm.size() / 4, m->surf_leaf, sds, stable != 0);
  *n_corner = (int64_t)(cds.size() / 4);
  *n_surf = (int64_t)(sds.size() / 4);
  *n_ids = (int32_t)m->existing.size();
  if (*n_corner > cap_c || *n_surf > cap_s || *n_ids > cap_ids) return LLSR_ERANGE;
  if (!cds.empty()) std::memcpy(corner_out, cds.data(), cds.size() * sizeof(float));
  if (!sds.empty()) std::memcpy(surf_out, sds.data(), sds.size() * sizeof(float));
  for (int k = 0; k < *n_ids; ++k) ids[k] = m->existing[k];
  return LLSR_OK;
}
#endif

}  // extern "C"
