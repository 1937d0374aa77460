// llsr_ros2.hpp — the node-side half of the drop-in: what the reference's ROS2 nodes call in place
// of their per-scan arithmetic, over the C-ABI of include/llsr.h. Header-only C++11, templated on
// the message and cloud types so the same code builds against ROS2 + PCL (cloud_msgs::msg::CloudInfo,
// pcl::PointCloud<pcl::PointXYZI>) and, in tests/test_ros2_adapter.py, against plain structs with
// the same field names (no ROS here). INTEGRATION.md §2 shows the four member bodies that call it.
//
// Seams (reference file:line):
//   ImageProjection::cloudHandler            imageProjection.cpp:189-222 -> Projection::run
//   FeatureAssociation feature stage         featureAssociation.cpp:2769-2775 (+ 1310-1314 shadow points)
//                                            -> Projection::handoff (on the IP thread, into ProjectionOut)
//   runFeatureAssociation after the features featureAssociation.cpp:2777-2796, 2291-2315, 2660-2712
//                                            -> Odometry::step (on the FA thread, its own handle)
//   FeatureAssociation::updateTransformation featureAssociation.cpp:2505-2535 -> update_transformation
//   MapOptimization::scan2MapOptimization    mapOptmization.cpp:1572-1610 -> scan2map_optimization
//
// Threads. The reference runs IP, FA and MO on their own executor threads joined by one-slot
// Channels (main.cpp:10-11, channel.h:24-54); IP's blocking send waits only until FA has *taken*
// the previous scan, so IP's next cloudHandler overlaps FA's work on the last one. A handle is
// single-threaded and its host buffers are overwritten by the next scan, so nothing that FA uses
// may point into the IP node's Projection: the feature stage keeps FA's carry-over state
// (FA:167-198) in the IP handle and runs with the rest of the scan on the IP thread, and
// Projection::handoff copies its clouds into the ProjectionOut that crosses the channel
// (FeatureClouds below). FA's Odometry and MO's scan-to-map each own another handle.
#pragma once
#include <stdint.h>

#include <stdexcept>
#include <string>
#include <utility>
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

// The feature clouds of one scan as runFeatureAssociation holds them after extractFeaturesOurs
// (FA:2769-2775): computed on the IP thread and carried to FA inside ProjectionOut. A maintainer
// adds the member `llsr_ros2::FeatureClouds<pcl::PointCloud<PointType>> features;` to ProjectionOut
// (UT:63-72). Values, not pointers into a handle's buffers: the IP thread's next scan cannot touch
// them once they are in the channel.
template <class Cloud>
struct FeatureClouds {
  Cloud segmented;          // segmentedCloud after adjustDistortion (LOAM frame)
  Cloud corner_sharp;       // cornerPointsSharp
  Cloud corner_less_sharp;  // cornerPointsLessSharp
  Cloud surf_flat;          // surfPointsFlat + the shadow points (FA:1310-1314)
  Cloud surf_less_flat;     // surfPointsLessFlat (per-ring VoxelGrid)
};

// TransformToEnd (FA:1414-1490) of every point of `in` into `out` (may be the same cloud)
template <class Cloud>
void transform_to_end(const float transform_cur[6], const Cloud& in, Cloud& out) {
  std::vector<float> a;
  repack_xyzi(in, a);
  const int32_t n = (int32_t)(a.size() / 4);
  check(llsr_transform_to_end(transform_cur, a.data(), n, a.data()), nullptr, "llsr_transform_to_end");
  unpack_xyzi(a.data(), n, out);
}

template <class Cloud>
void append_xyzi(const float* xyzi, int32_t n, Cloud& c) {
  const size_t f = c.points.size();
  c.points.resize(f + (size_t)n);
  for (int32_t k = 0; k < n; ++k) {
    auto& p = c.points[f + (size_t)k];
    p.x = xyzi[4 * k];
    p.y = xyzi[4 * k + 1];
    p.z = xyzi[4 * k + 2];
    p.intensity = xyzi[4 * k + 3];
  }
  c.width = (uint32_t)c.points.size();
  c.height = 1;
}

// An llsr handle owned by one node thread (FA's scan-to-scan, MO's scan-to-map): one scan slot,
// the LMs' buffers grow on first use. mode: LLSR_MODE_FAITHFUL / LLSR_MODE_LM_APPLIED (MO:1539-1545)
class Handle {
 public:
  explicit Handle(int32_t lidar, int32_t device = 0, int32_t mode = LLSR_MODE_LM_APPLIED) {
    llsr_config cfg;
    check(llsr_config_default(&cfg, lidar), nullptr, "llsr_config_default");
    if (llsr_abi_version() != LLSR_ABI_VERSION) throw std::runtime_error("llsr: library ABI version differs from llsr.h");
    cfg.mode = mode;
    llsr_handle* h = nullptr;
    const int32_t rc = llsr_create(&cfg, device, 1, cfg.num_vertical_scans * cfg.num_horizontal_scans, &h);
    if (rc != LLSR_OK || !h) throw std::runtime_error("llsr: llsr_create failed (no HIP device?)");
    h_ = h;
  }
  ~Handle() {
    if (h_) llsr_destroy(h_);
  }
  Handle(const Handle&) = delete;
  Handle& operator=(const Handle&) = delete;
  llsr_handle* get() const { return h_; }

 private:
  llsr_handle* h_ = nullptr;
};

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
  // publishClouds' ProjectionOut (IP:933-1000) with this scan's feature clouds in po.features, built
  // on the IP thread before Channel::send; po.segmented_cloud / outlier_cloud must be allocated
  template <class ProjOut>
  void handoff(ProjOut& po) const {
    projection_out(po, *po.segmented_cloud, *po.outlier_cloud);
    features(po.features.segmented, po.features.corner_sharp, po.features.corner_less_sharp, po.features.surf_flat,
             po.features.surf_less_flat);
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

// runFeatureAssociation from `if (!systemInitedLM)` on (FA:2777-2796) for the FA node's thread, on
// its own handle and its own clouds: checkSystemInitialization (FA:2291-2315) on the first scan,
// then updateTransformation (FA:2505-2535), integrateTransformation (FA:2537-2568) and
// publishCloudsLast (FA:2660-2712: TransformToEnd of the less-sharp / less-flat clouds, which
// become the last clouds + the shadow points, and of the sharp / flat clouds, MO's scan clouds).
// updateInitialGuess (FA:2790) and publishOdometry stay node code; without an IMU, transformCur
// carries over as the next LM's initial guess (LLSR_MODE_LM_APPLIED semantics).
template <class Cloud>
class Odometry {
 public:
  explicit Odometry(int32_t lidar, int32_t device = 0) : h_(lidar, device) {
    shadow_.resize(4 * 160);
    check(llsr_shadow_points(shadow_.data()), nullptr, "llsr_shadow_points");
  }
  llsr_handle* handle() const { return h_.get(); }

  // one scan's features (moved from the channel's ProjectionOut); false on the initialisation scan
  bool step(FeatureClouds<Cloud>& f) {
    if (!inited_) {
      corner_last = std::move(f.corner_less_sharp);
      surf_last = std::move(f.surf_less_flat);
      append_xyzi(shadow_.data(), (int32_t)(shadow_.size() / 4), surf_last);
      inited_ = true;
      return false;
    }
    report = update_transformation(h_.get(), f.corner_sharp, f.surf_flat, corner_last, surf_last, transform_cur,
                                   is_degenerate);
    check(llsr_integrate_transformation(transform_sum, transform_cur), nullptr, "llsr_integrate_transformation");
    transform_to_end(transform_cur, f.corner_less_sharp, corner_last);
    transform_to_end(transform_cur, f.surf_less_flat, surf_last);
    append_xyzi(shadow_.data(), (int32_t)(shadow_.size() / 4), surf_last);
    transform_to_end(transform_cur, f.corner_sharp, corner_scan);
    transform_to_end(transform_cur, f.surf_flat, surf_scan);
    return true;
  }

  // FA's member state after the last step
  float transform_cur[6] = {0, 0, 0, 0, 0, 0};
  float transform_sum[6] = {0, 0, 0, 0, 0, 0};
  bool is_degenerate = false;
  llsr_s2s_report report = llsr_s2s_report();
  Cloud corner_last, surf_last;   // laserCloudCornerLast / laserCloudSurfLast
  Cloud corner_scan, surf_scan;   // laserCloudCornerScan / laserCloudSurfScan (AssociationOut)

 private:
  Handle h_;
  bool inited_ = false;
  std::vector<float> shadow_;
};

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
