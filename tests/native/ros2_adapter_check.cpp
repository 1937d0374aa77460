// Builds integration/ros2/llsr_ros2.hpp against plain structs carrying the field names of the ROS2
// / PCL types the reference's nodes use (cloud_msgs/msg/CloudInfo.msg, ProjectionOut of
// utility.h:63-72, pcl::PointCloud<pcl::PointXYZI>): no ROS in this image, so these structs stand in
// for the message types only to compile and run the adapter's code.
//
//   marshal          (CPU): a hand-made llsr_scan_out -> CloudInfo / ProjectionOut / feature clouds,
//                    every field checked; prints "ok"
//   node <lidar> <in.bin> <out.bin>  (GPU): llsr_ros2::Projection on one scan (float4 rows), then
//                    the marshalled CloudInfo arrays and feature clouds written for the test to
//                    compare with the ctypes pipeline's outputs
//   drive <lidar> <frames.bin> <map.bin> <out.bin>  (GPU): the reference's thread layout
//                    (main.cpp:10-11): an IP thread (Projection::run + handoff, blocking one-slot
//                    send), an FA thread (Odometry::step on its own handle: updateTransformation,
//                    integrateTransformation, publishCloudsLast) and an MO thread
//                    (scan2map_optimization on a third handle, non-blocking send as
//                    association_out_channel(false)); every frame's features, poses and clouds
//                    written for the test to compare with the oracle
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../integration/ros2/llsr_ros2.hpp"

namespace mock {
struct PointXYZI {
  float x, y, z, pad0, intensity, pad1, pad2, pad3;  // PCL's 32-byte layout
};
struct Cloud {
  std::vector<PointXYZI> points;
  uint32_t width = 0, height = 0;
};
struct Header {
  int32_t sec = 0;
};
struct CloudInfo {  // cloud_msgs/msg/CloudInfo.msg
  Header header;
  std::vector<int32_t> start_ring_index, end_ring_index;
  float start_orientation = 0, end_orientation = 0, orientation_diff = 0;
  std::vector<bool> segmented_cloud_ground_flag;
  std::vector<uint32_t> segmented_cloud_col_ind;
  std::vector<float> segmented_cloud_range;
};
struct ProjectionOut {  // utility.h:63-72, with the member INTEGRATION.md §2 adds
  std::shared_ptr<Cloud> segmented_cloud, outlier_cloud;
  CloudInfo seg_msg;
  std::vector<double> outlierCloud_Intensity, segmentedCloud_Intensity;
  llsr_ros2::FeatureClouds<Cloud> features;
};
struct AssociationOut {  // utility.h:75-83 (the odometry message left out: not compared here)
  Header header;
  std::shared_ptr<Cloud> cloud_corner_last, cloud_surf_last, cloud_corner_scan, cloud_surf_scan;
  float transform_sum[6];
};

// One writer, one reader, one slot: send waits for an empty slot when blocking and otherwise
// overwrites; receive waits for an item and empties the slot (the semantics of channel.h:24-54).
template <class T>
class Channel {
 public:
  explicit Channel(bool blocking_send) : blocking_(blocking_send) {}
  void send(T&& v) {
    std::unique_lock<std::mutex> lk(m_);
    if (blocking_) cv_.wait(lk, [this] { return !full_; });
    slot_ = std::move(v);
    full_ = true;
    cv_.notify_all();
  }
  void receive(T& v) {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [this] { return full_; });
    v = std::move(slot_);
    full_ = false;
    cv_.notify_all();
  }

 private:
  bool blocking_;
  bool full_ = false;
  T slot_;
  std::mutex m_;
  std::condition_variable cv_;
};
}  // namespace mock

static int fails = 0;
#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                \
    }                                                         \
  } while (0)

static bool same_pt(const mock::PointXYZI& p, const float* r) {
  return p.x == r[0] && p.y == r[1] && p.z == r[2] && p.intensity == r[3];
}

static int marshal() {
  const int H = 3, S = 7, O = 2, L = 3;
  int32_t start[H] = {4, 6, 9}, end[H] = {0, 1, 2};
  std::vector<float> seg(4 * S), loam(4 * S), outl(4 * O), lflat(4 * L), rng(S), sint(S), oint(O);
  for (int i = 0; i < 4 * S; ++i) { seg[i] = 0.5f * i; loam[i] = -0.25f * i; }
  for (int i = 0; i < 4 * O; ++i) outl[i] = 100.f + i;
  for (int i = 0; i < 4 * L; ++i) lflat[i] = 7.f - i;
  for (int i = 0; i < S; ++i) { rng[i] = 3.f + i; sint[i] = 1.0001f * i; }
  for (int i = 0; i < O; ++i) oint[i] = 2.5f * i;
  uint8_t gflag[S] = {1, 0, 0, 1, 0, 1, 0};
  uint32_t col[S] = {5, 10, 15, 20, 25, 30, 35};
  int32_t sharp[2] = {3, 1}, edge[3] = {1, 3, 6}, flat[2] = {0, 5};
  llsr_scan_out o;
  memset(&o, 0, sizeof o);
  o.orientation[0] = -3.1f; o.orientation[1] = 3.2f; o.orientation[2] = 6.3f;
  o.start_ring_index = start; o.end_ring_index = end;
  o.n_segmented = S; o.seg_xyzi = seg.data(); o.seg_ground_flag = gflag; o.seg_col_ind = col;
  o.seg_range = rng.data(); o.seg_intensity = sint.data();
  o.n_outlier = O; o.outlier_xyzi = outl.data(); o.outlier_intensity = oint.data();
  o.loam_xyzi = loam.data();
  o.n_sharp = 2; o.sharp_ind = sharp; o.n_less_sharp = 3; o.less_sharp_ind = edge;
  o.n_flat = 2; o.flat_ind = flat; o.n_less_flat = L; o.less_flat_xyzi = lflat.data();

  mock::ProjectionOut po;
  po.segmented_cloud = std::make_shared<mock::Cloud>();
  po.outlier_cloud = std::make_shared<mock::Cloud>();
  llsr_ros2::projection_out(o, H, po, *po.segmented_cloud, *po.outlier_cloud);
  const mock::CloudInfo& m = po.seg_msg;
  CHECK(m.start_ring_index == std::vector<int32_t>(start, start + H));
  CHECK(m.end_ring_index == std::vector<int32_t>(end, end + H));
  CHECK(m.start_orientation == -3.1f && m.end_orientation == 3.2f && m.orientation_diff == 6.3f);
  CHECK((int)m.segmented_cloud_ground_flag.size() == S && (int)m.segmented_cloud_col_ind.size() == S &&
        (int)m.segmented_cloud_range.size() == S);
  for (int k = 0; k < S; ++k) {
    CHECK(m.segmented_cloud_ground_flag[k] == (gflag[k] != 0));
    CHECK(m.segmented_cloud_col_ind[k] == col[k]);
    CHECK(m.segmented_cloud_range[k] == rng[k]);
    CHECK(po.segmentedCloud_Intensity[k] == (double)sint[k]);
    CHECK(same_pt(po.segmented_cloud->points[k], &seg[4 * k]));
  }
  CHECK(po.segmented_cloud->width == (uint32_t)S && po.segmented_cloud->height == 1);
  CHECK((int)po.outlier_cloud->points.size() == O && (int)po.outlierCloud_Intensity.size() == O);
  for (int k = 0; k < O; ++k) {
    CHECK(same_pt(po.outlier_cloud->points[k], &outl[4 * k]));
    CHECK(po.outlierCloud_Intensity[k] == (double)oint[k]);
  }

  const float shadow[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  mock::Cloud segc, cs, cls, sf, slf;
  llsr_ros2::features(o, shadow, 2, segc, cs, cls, sf, slf);
  CHECK((int)segc.points.size() == S);
  for (int k = 0; k < S; ++k) CHECK(same_pt(segc.points[k], &loam[4 * k]));
  CHECK(cs.points.size() == 2 && same_pt(cs.points[0], &loam[12]) && same_pt(cs.points[1], &loam[4]));
  CHECK(cls.points.size() == 3 && same_pt(cls.points[2], &loam[24]));
  CHECK(sf.points.size() == 4 && same_pt(sf.points[0], &loam[0]) && same_pt(sf.points[1], &loam[20]));
  CHECK(same_pt(sf.points[2], shadow) && same_pt(sf.points[3], shadow + 4) && sf.width == 4);
  CHECK((int)slf.points.size() == L && same_pt(slf.points[1], &lflat[4]));

  std::vector<float> packed;
  llsr_ros2::repack_xyzi(sf, packed);
  CHECK(packed.size() == 16 && packed[4] == loam[20] && packed[15] == 8.f);
  if (!fails) printf("ok\n");
  return fails ? 1 : 0;
}

#ifdef LLSR_ADAPTER_NODE
// the GPU half: the node-side class end to end
static int node(int lidar, const char* in, const char* out) {
  FILE* f = fopen(in, "rb");
  if (!f) return 2;
  std::vector<float> rows;
  float buf[4];
  while (fread(buf, sizeof(float), 4, f) == 4) rows.insert(rows.end(), buf, buf + 4);
  fclose(f);
  mock::Cloud in_cloud;
  llsr_ros2::unpack_xyzi(rows.data(), (int32_t)(rows.size() / 4), in_cloud);
  llsr_ros2::Projection proj(lidar, 0);
  proj.run(in_cloud);
  mock::ProjectionOut po;
  po.segmented_cloud = std::make_shared<mock::Cloud>();
  po.outlier_cloud = std::make_shared<mock::Cloud>();
  proj.projection_out(po, *po.segmented_cloud, *po.outlier_cloud);
  mock::Cloud segc, cs, cls, sf, slf;
  proj.features(segc, cs, cls, sf, slf);
  FILE* g = fopen(out, "wb");
  if (!g) return 2;
  auto put_i = [&](int32_t v) { fwrite(&v, 4, 1, g); };
  auto put_cloud = [&](const mock::Cloud& c) {
    put_i((int32_t)c.points.size());
    for (const auto& p : c.points) {
      const float r[4] = {p.x, p.y, p.z, p.intensity};
      fwrite(r, 4, 4, g);
    }
  };
  const mock::CloudInfo& m = po.seg_msg;
  put_i((int32_t)m.start_ring_index.size());
  fwrite(m.start_ring_index.data(), 4, m.start_ring_index.size(), g);
  fwrite(m.end_ring_index.data(), 4, m.end_ring_index.size(), g);
  const float orient[3] = {m.start_orientation, m.end_orientation, m.orientation_diff};
  fwrite(orient, 4, 3, g);
  put_i((int32_t)m.segmented_cloud_range.size());
  for (bool b : m.segmented_cloud_ground_flag) { const uint8_t v = b ? 1 : 0; fwrite(&v, 1, 1, g); }
  fwrite(m.segmented_cloud_col_ind.data(), 4, m.segmented_cloud_col_ind.size(), g);
  fwrite(m.segmented_cloud_range.data(), 4, m.segmented_cloud_range.size(), g);
  put_cloud(*po.segmented_cloud);
  put_cloud(*po.outlier_cloud);
  put_cloud(segc);
  put_cloud(cs);
  put_cloud(cls);
  put_cloud(sf);
  put_cloud(slf);
  fclose(g);
  return 0;
}
#endif

#ifdef LLSR_ADAPTER_NODE
static bool read_cloud(FILE* f, mock::Cloud& c) {
  int32_t n = 0;
  if (fread(&n, 4, 1, f) != 1 || n < 0) return false;
  std::vector<float> rows(4 * (size_t)n);
  if (n && fread(rows.data(), 4, rows.size(), f) != rows.size()) return false;
  llsr_ros2::unpack_xyzi(rows.data(), n, c);
  return true;
}

static void put_cloud(FILE* g, const mock::Cloud& c) {
  const int32_t n = (int32_t)c.points.size();
  fwrite(&n, 4, 1, g);
  for (const auto& p : c.points) {
    const float r[4] = {p.x, p.y, p.z, p.intensity};
    fwrite(r, 4, 4, g);
  }
}

// per FA frame: what FA received and what Odometry::step left
struct FaRecord {
  int32_t seq = -1, lm = 0;
  mock::Cloud sharp, less_sharp, flat, less_flat;
  float tcur[6], tsum[6];
  int32_t degenerate = 0;
  llsr_s2s_report rep = llsr_s2s_report();
  mock::Cloud corner_last, surf_last, corner_scan, surf_scan;
};
struct MoRecord {
  int32_t seq = -1;
  float pose[6];
  llsr_lm_report rep;
};

static int drive(int lidar, const char* frames_path, const char* map_path, const char* out) {
  FILE* f = fopen(frames_path, "rb");
  if (!f) return 2;
  int32_t F = 0;
  if (fread(&F, 4, 1, f) != 1 || F < 1) return 2;
  std::vector<mock::Cloud> frames((size_t)F);
  for (auto& c : frames)
    if (!read_cloud(f, c)) return 2;
  fclose(f);
  mock::Cloud corner_map, surf_map;
  float pose0[6];
  FILE* m = fopen(map_path, "rb");
  if (!m || !read_cloud(m, corner_map) || !read_cloud(m, surf_map) || fread(pose0, 4, 6, m) != 6) return 2;
  fclose(m);

  mock::Channel<mock::ProjectionOut> ip_to_fa(true);    // projection_out_channel(true)
  mock::Channel<mock::AssociationOut> fa_to_mo(false);  // association_out_channel(false)
  std::vector<FaRecord> fa_rec;
  std::vector<MoRecord> mo_rec;
  std::string err;
  std::mutex err_m;
  auto guard = [&](const char* who, const std::exception& e) {
    std::lock_guard<std::mutex> lk(err_m);
    err += std::string(who) + ": " + e.what() + "\n";
  };

  std::thread ip([&] {  // ImageProjection::cloudHandler per message, then publishClouds' send
    try {
      llsr_ros2::Projection proj(lidar, 0);
      for (int32_t k = 0; k <= F; ++k) {
        mock::ProjectionOut po;
        po.seg_msg.header.sec = k < F ? k : -1;  // -1: end of the drive
        if (k < F) {
          proj.run(frames[(size_t)k]);
          po.segmented_cloud = std::make_shared<mock::Cloud>();
          po.outlier_cloud = std::make_shared<mock::Cloud>();
          proj.handoff(po);
          po.seg_msg.header.sec = k;
        }
        ip_to_fa.send(std::move(po));
      }
    } catch (const std::exception& e) {
      guard("ip", e);
      mock::ProjectionOut end;
      end.seg_msg.header.sec = -1;
      ip_to_fa.send(std::move(end));
    }
  });
  std::thread fa([&] {  // runFeatureAssociation's loop (FA:2742-2853) on its own handle
    bool dead = false;
    try {
      llsr_ros2::Odometry<mock::Cloud> odo(lidar, 0);
      while (true) {
        mock::ProjectionOut po;
        ip_to_fa.receive(po);
        if (po.seg_msg.header.sec < 0) break;
        if (dead) continue;
        FaRecord r;
        r.seq = po.seg_msg.header.sec;
        r.sharp = po.features.corner_sharp;
        r.less_sharp = po.features.corner_less_sharp;
        r.flat = po.features.surf_flat;
        r.less_flat = po.features.surf_less_flat;
        r.lm = odo.step(po.features) ? 1 : 0;
        for (int i = 0; i < 6; ++i) {
          r.tcur[i] = odo.transform_cur[i];
          r.tsum[i] = odo.transform_sum[i];
        }
        r.degenerate = odo.is_degenerate ? 1 : 0;
        r.rep = odo.report;
        r.corner_last = odo.corner_last;
        r.surf_last = odo.surf_last;
        if (r.lm) {
          r.corner_scan = odo.corner_scan;
          r.surf_scan = odo.surf_scan;
          mock::AssociationOut ao;  // _output_channel.send (FA:2822-2852), mapping_frequency_divider 1
          ao.header.sec = r.seq;
          ao.cloud_corner_last = std::make_shared<mock::Cloud>(odo.corner_last);
          ao.cloud_surf_last = std::make_shared<mock::Cloud>(odo.surf_last);
          ao.cloud_corner_scan = std::make_shared<mock::Cloud>(odo.corner_scan);
          ao.cloud_surf_scan = std::make_shared<mock::Cloud>(odo.surf_scan);
          for (int i = 0; i < 6; ++i) ao.transform_sum[i] = odo.transform_sum[i];
          fa_to_mo.send(std::move(ao));
        }
        fa_rec.push_back(std::move(r));
      }
    } catch (const std::exception& e) {
      guard("fa", e);
      dead = true;
      mock::ProjectionOut po;  // drain so that IP's blocking send returns
      do ip_to_fa.receive(po); while (po.seg_msg.header.sec >= 0);
    }
    mock::AssociationOut end;
    end.header.sec = -1;
    fa_to_mo.send(std::move(end));
  });
  std::thread mo([&] {  // MapOptimization's loop: scan2MapOptimization on a third handle
    try {
      llsr_ros2::Handle h(lidar, 0, LLSR_MODE_LM_APPLIED);
      while (true) {
        mock::AssociationOut ao;
        fa_to_mo.receive(ao);
        if (ao.header.sec < 0) break;
        MoRecord r;
        r.seq = ao.header.sec;
        for (int i = 0; i < 6; ++i) r.pose[i] = pose0[i];
        r.rep = llsr_ros2::scan2map_optimization(h.get(), *ao.cloud_corner_scan, *ao.cloud_surf_scan, corner_map,
                                                 surf_map, r.pose);
        mo_rec.push_back(r);
      }
    } catch (const std::exception& e) {
      guard("mo", e);
      mock::AssociationOut ao;
      do fa_to_mo.receive(ao); while (ao.header.sec >= 0);
    }
  });
  ip.join();
  fa.join();
  mo.join();
  if (!err.empty()) {
    fprintf(stderr, "%s", err.c_str());
    return 1;
  }
  FILE* g = fopen(out, "wb");
  if (!g) return 2;
  const int32_t nf = (int32_t)fa_rec.size(), nm = (int32_t)mo_rec.size();
  fwrite(&nf, 4, 1, g);
  for (const auto& r : fa_rec) {
    const int32_t hdr[9] = {r.seq, r.lm, r.degenerate, r.rep.surf_iterations, r.rep.corner_iterations,
                            r.rep.n_surf_corr, r.rep.n_corner_corr, r.rep.degenerate, r.rep.skipped};
    fwrite(hdr, 4, 9, g);
    fwrite(r.tcur, 4, 6, g);
    fwrite(r.tsum, 4, 6, g);
    for (const mock::Cloud* c : {&r.sharp, &r.less_sharp, &r.flat, &r.less_flat, &r.corner_last, &r.surf_last,
                                 &r.corner_scan, &r.surf_scan})
      put_cloud(g, *c);
  }
  fwrite(&nm, 4, 1, g);
  for (const auto& r : mo_rec) {
    fwrite(&r.seq, 4, 1, g);
    fwrite(r.pose, 4, 6, g);
    fwrite(&r.rep.iterations, 4, 1, g);
  }
  fclose(g);
  return 0;
}
#endif

int main(int argc, char** argv) {
  if (argc >= 2 && !strcmp(argv[1], "marshal")) return marshal();
#ifdef LLSR_ADAPTER_NODE
  if (argc >= 5 && !strcmp(argv[1], "node")) return node(atoi(argv[2]), argv[3], argv[4]);
  if (argc >= 6 && !strcmp(argv[1], "drive")) return drive(atoi(argv[2]), argv[3], argv[4], argv[5]);
#endif
  fprintf(stderr, "usage: %s marshal | node <lidar> <in.bin> <out.bin> | drive <lidar> <frames.bin> <map.bin> <out.bin>\n",
          argv[0]);
  return 2;
}
