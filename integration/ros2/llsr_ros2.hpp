// llsr_ros2.hpp — the node-side half of the drop-in: what the reference's ROS2 nodes call in place
// of their per-scan arithmetic, over the C-ABI of include/llsr.h. Header-only C++11, templated on
// the message and cloud types so the same code builds against ROS2 + PCL (cloud_msgs::msg::CloudInfo,
// pcl::PointCloud<pcl::PointXYZI>) and, in tests/test_ros2_adapter.py, against plain structs with
// the same field names (no ROS here). INTEGRATION.md §2 shows the four member bodies that call it.
//
// Seams (reference file:line):
//   ImageProjection::cloudHandler            imageProjection.cpp:189-222 -> Projection::run
//   FeatureAssociation feature stage         featureAssociation.cpp:2769-2775 (+ 1310-1314 shadow points)
//                                                                         -> Projection::features
//   FeatureAssociation::updateTransformation featureAssociation.cpp:2505-2535 -> update_transformation
//   MapOptimization::scan2MapOptimization    mapOptmization.cpp:1572-1610 -> scan2map_optimization
#pragma once
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "llsr.h"

namespace llsr_ros2 {

inline void check(int32_t rc, llsr_handle* h, const char* what) {
  if (rc != LLSR_OK)
    throw std::runtime_error(std::string("llsr: ") + what + ": " + (h ? llsr_last_error(h) : "no handle"));
}

// PCL PointXYZI is 32 bytes (x, y, z, pad, intensity, pad...): the ABI takes packed float4 rows.
template <class Cloud>
void repack_xyzi(const Cloud& c, std::vector<float>& out) {
  const size_t n = c.points.size();
  out.resize(4 * n);
  for (size_t i = 0; i < n; ++i) {
    const auto& p = c.points[i];
    out[4 * i] = p.x;
    out[4 * i + 1] = p.y;
    out[4 * i + 2] = p.z;
    out[4 * i + 3] = p.intensity;
  }
}

template <class Cloud>
void unpack_xyzi(const float* xyzi, int32_t n, Cloud& c) {
  c.points.resize((size_t)n);
  for (int32_t i = 0; i < n; ++i) {
    auto& p = c.points[(size_t)i];
    p.x = xyzi[4 * i];
    p.y = xyzi[4 * i + 1];
    p.z = xyzi[4 * i + 2];
    p.intensity = xyzi[4 * i + 3];
  }
  c.width = (uint32_t)n;
  c.height = 1;
}

// rows `ind` of a float4 array, in list order (cornerPointsSharp / LessSharp, surfPointsFlat)
template <class Cloud>
void gather_xyzi(const float* xyzi, const int32_t* ind, int32_t n, Cloud& c) {
  c.points.resize((size_t)n);
  for (int32_t k = 0; k < n; ++k) {
    const float* r = xyzi + 4 * (size_t)ind[k];
    auto& p = c.points[(size_t)k];
    p.x = r[0];
    p.y = r[1];
    p.z = r[2];
    p.intensity = r[3];
  }
  c.width = (uint32_t)n;
  c.height = 1;
}

// CloudInfo as IP:791-832 fills _seg_msg (header left to the caller: IP:199)
template <class CloudInfo>
void cloud_info(const llsr_scan_out& o, int32_t rings, CloudInfo& msg) {
  const size_t S = (size_t)o.n_segmented;
  msg.start_ring_index.assign(o.start_ring_index, o.start_ring_index + rings);
  msg.end_ring_index.assign(o.end_ring_index, o.end_ring_index + rings);
  msg.start_orientation = o.orientation[0];
  msg.end_orientation = o.orientation[1];
  msg.orientation_diff = o.orientation[2];
  msg.segmented_cloud_ground_flag.resize(S);
  msg.segmented_cloud_col_ind.resize(S);
  msg.segmented_cloud_range.resize(S);
  for (size_t k = 0; k < S; ++k) {
    msg.segmented_cloud_ground_flag[k] = o.seg_ground_flag[k] != 0;
    msg.segmented_cloud_col_ind[k] = o.seg_col_ind[k];
    msg.segmented_cloud_range[k] = o.seg_range[k];
  }
}

// ProjectionOut (UT:63-72) as publishClouds hands it to the FA channel (IP:933-1000): the
// segmented and outlier clouds, seg_msg, and the two intensity vectors (double, as declared)
template <class ProjOut, class Cloud>
void projection_out(const llsr_scan_out& o, int32_t rings, ProjOut& po, Cloud& segmented_cloud, Cloud& outlier_cloud) {
  unpack_xyzi(o.seg_xyzi, o.n_segmented, segmented_cloud);
  unpack_xyzi(o.outlier_xyzi, o.n_outlier, outlier_cloud);
  cloud_info(o, rings, po.seg_msg);
  po.segmentedCloud_Intensity.assign(o.seg_intensity, o.seg_intensity + o.n_segmented);
  po.outlierCloud_Intensity.assign(o.outlier_intensity, o.outlier_intensity + o.n_outlier);
}

// The FA feature stage's clouds (FA:2769-2775): segmentedCloud after adjustDistortion (LOAM
// frame), cornerPointsSharp / LessSharp and surfPointsFlat as gathers of it, the `ns` shadow points
// (GenerateShadowPoint, FA:412-450) appended to surfPointsFlat as FA:1310-1314 does, and
// surfPointsLessFlat as the per-ring VoxelGrid output
template <class Cloud>
void features(const llsr_scan_out& o, const float* shadow, int32_t ns, Cloud& segmented_cloud, Cloud& corner_sharp,
              Cloud& corner_less_sharp, Cloud& surf_flat, Cloud& surf_less_flat) {
  unpack_xyzi(o.loam_xyzi, o.n_segmented, segmented_cloud);
  gather_xyzi(o.loam_xyzi, o.sharp_ind, o.n_sharp, corner_sharp);
  gather_xyzi(o.loam_xyzi, o.less_sharp_ind, o.n_less_sharp, corner_less_sharp);
  gather_xyzi(o.loam_xyzi, o.flat_ind, o.n_flat, surf_flat);
  const size_t f = surf_flat.points.size();
  surf_flat.points.resize(f + (size_t)ns);
  for (int32_t k = 0; k < ns; ++k) {
    auto& p = surf_flat.points[f + (size_t)k];
    p.x = shadow[4 * k];
    p.y = shadow[4 * k + 1];
    p.z = shadow[4 * k + 2];
    p.intensity = shadow[4 * k + 3];
  }
  surf_flat.width = (uint32_t)surf_flat.points.size();
  surf_flat.height = 1;
  unpack_xyzi(o.less_flat_xyzi, o.n_less_flat, surf_less_flat);
}

// One handle and its host output buffers (capacity H*W per array, llsr_query_sizes), for the
// single-scan call shape the nodes use; one per pipeline thread, as the reference runs one thread
// per node.
class Projection {
 public:
  // max_points: raw points per scan the handle accepts (0: twice the range image)
  explicit Projection(int32_t lidar, int32_t device = 0, int32_t max_points = 0) {
    llsr_config cfg;
    check(llsr_config_default(&cfg, lidar), nullptr, "llsr_config_default");
    if (llsr_abi_version() != LLSR_ABI_VERSION) throw std::runtime_error("llsr: library ABI version differs from llsr.h");
    if (max_points < 1) max_points = 2 * cfg.num_vertical_scans * cfg.num_horizontal_scans;
    llsr_handle* h = nullptr;
    const int32_t rc = llsr_create(&cfg, device, 1, max_points, &h);
    if (rc != LLSR_OK || !h) throw std::runtime_error("llsr: llsr_create failed (no HIP device?)");
    h_ = h;
    llsr_sizes sz;
    check(llsr_query_sizes(h_, &sz), h_, "llsr_query_sizes");
    rings_ = sz.rings;
    cells_ = (size_t)sz.cells;
    start_.resize((size_t)rings_);
    end_.resize((size_t)rings_);
    seg_.resize(4 * cells_);
    loam_.resize(4 * cells_);
    lflat_.resize(4 * cells_);
    out_.resize(4 * cells_);
    gflag_.resize(cells_);
    col_.resize(cells_);
    rng_.resize(cells_);
    sint_.resize(cells_);
    oint_.resize(cells_);
    edge_.resize(cells_);
    sharp_.resize(cells_);
    flat_.resize(cells_);
    shadow_.resize(4 * (size_t)sz.shadow_points);
    check(llsr_shadow_points(shadow_.data()), h_, "llsr_shadow_points");
  }
  ~Projection() {
    if (h_) llsr_destroy(h_);
  }
  Projection(const Projection&) = delete;
  Projection& operator=(const Projection&) = delete;

  llsr_handle* handle() const { return h_; }
  const llsr_scan_out& out() const { return o_; }

  // cloudHandler from fromROSMsg on (IP:196-207): NaN removal, findStartEndAngle,
  // projectPointCloud, groundRemovalOurs, cloudSegmentation, then the FA feature stage of the
  // same scan (the handle keeps FA's carry-over arrays, FA:167-198)
  template <class Cloud>
  void run(const Cloud& laser_cloud_in) {
    repack_xyzi(laser_cloud_in, xyzi_);
    o_ = llsr_scan_out();
    o_.start_ring_index = start_.data();
    o_.end_ring_index = end_.data();
    o_.seg_xyzi = seg_.data();
    o_.seg_ground_flag = gflag_.data();
    o_.seg_col_ind = col_.data();
    o_.seg_range = rng_.data();
    o_.seg_intensity = sint_.data();
    o_.outlier_xyzi = out_.data();
    o_.outlier_intensity = oint_.data();
    o_.loam_xyzi = loam_.data();
    o_.less_sharp_ind = edge_.data();
    o_.sharp_ind = sharp_.data();
    o_.flat_ind = flat_.data();
    o_.less_flat_xyzi = lflat_.data();
    check(llsr_process_scan(h_, xyzi_.data(), (int32_t)(xyzi_.size() / 4), &o_), h_, "llsr_process_scan");
  }

  // the marshalling below, on this handle's last scan
  template <class CloudInfo>
  void cloud_info(CloudInfo& msg) const { llsr_ros2::cloud_info(o_, rings_, msg); }
  template <class ProjOut, class Cloud>
  void projection_out(ProjOut& po, Cloud& segmented_cloud, Cloud& outlier_cloud) const {
    llsr_ros2::projection_out(o_, rings_, po, segmented_cloud, outlier_cloud);
  }
  template <class Cloud>
  void features(Cloud& segmented_cloud, Cloud& corner_sharp, Cloud& corner_less_sharp, Cloud& surf_flat,
                Cloud& surf_less_flat) const {
    llsr_ros2::features(o_, shadow_.data(), (int32_t)(shadow_.size() / 4), segmented_cloud, corner_sharp,
                        corner_less_sharp, surf_flat, surf_less_flat);
  }

 private:
  llsr_handle* h_ = nullptr;
  int32_t rings_ = 0;
  size_t cells_ = 0;
  llsr_scan_out o_ = llsr_scan_out();
  std::vector<float> xyzi_, seg_, loam_, lflat_, out_, rng_, sint_, oint_, shadow_;
  std::vector<int32_t> start_, end_, edge_, sharp_, flat_;
  std::vector<uint8_t> gflag_;
  std::vector<uint32_t> col_;
};

// updateTransformation (FA:2505-2535) with its member state: transformCur[6] and isDegenerate in
// and out; returns the report (corner_iterations = iterCount2, the odometry_itertimes entry)
template <class Cloud>
llsr_s2s_report update_transformation(llsr_handle* h, const Cloud& corner_sharp, const Cloud& surf_flat,
                                      const Cloud& corner_last, const Cloud& surf_last, float transform_cur[6],
                                      bool& is_degenerate) {
  std::vector<float> a, b, c, d;
  repack_xyzi(corner_sharp, a);
  repack_xyzi(surf_flat, b);
  repack_xyzi(corner_last, c);
  repack_xyzi(surf_last, d);
  int32_t deg = is_degenerate ? 1 : 0;
  llsr_s2s_report rep;
  check(llsr_scan2scan(h, a.data(), (int32_t)(a.size() / 4), b.data(), (int32_t)(b.size() / 4), c.data(),
                       (int32_t)(c.size() / 4), d.data(), (int32_t)(d.size() / 4), transform_cur, &deg, &rep),
        h, "llsr_scan2scan");
  is_degenerate = deg != 0;
  return rep;
}

// scan2MapOptimization (MO:1572-1610) once its guard (MO:1573: corner map > 10, surf map > 100)
// holds: kd-tree builds, corner / surf optimisation and LMOptimization on transformTobeMapped;
// the report's iterations feed MapIterTimes (MO:1587-1588), min_lambda / cf_mean localInfo
template <class Cloud>
llsr_lm_report scan2map_optimization(llsr_handle* h, const Cloud& corner_scan_ds, const Cloud& surf_total_last_ds,
                                     const Cloud& corner_from_map_ds, const Cloud& surf_from_map_ds,
                                     float transform_tobe_mapped[6]) {
  std::vector<float> a, b, c, d;
  repack_xyzi(corner_scan_ds, a);
  repack_xyzi(surf_total_last_ds, b);
  repack_xyzi(corner_from_map_ds, c);
  repack_xyzi(surf_from_map_ds, d);
  llsr_lm_report rep;
  check(llsr_scan2map(h, a.data(), (int32_t)(a.size() / 4), b.data(), (int32_t)(b.size() / 4), c.data(),
                      (int32_t)(c.size() / 4), d.data(), (int32_t)(d.size() / 4), transform_tobe_mapped, &rep),
        h, "llsr_scan2map");
  return rep;
}

}  // namespace llsr_ros2
