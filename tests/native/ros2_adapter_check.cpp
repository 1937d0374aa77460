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
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
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
struct ProjectionOut {  // utility.h:63-72
  std::shared_ptr<Cloud> segmented_cloud, outlier_cloud;
  CloudInfo seg_msg;
  std::vector<double> outlierCloud_Intensity, segmentedCloud_Intensity;
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

int main(int argc, char** argv) {
  if (argc >= 2 && !strcmp(argv[1], "marshal")) return marshal();
#ifdef LLSR_ADAPTER_NODE
  if (argc >= 5 && !strcmp(argv[1], "node")) return node(atoi(argv[2]), argv[3], argv[4]);
#endif
  fprintf(stderr, "usage: %s marshal | node <lidar> <in.bin> <out.bin>\n", argv[0]);
  return 2;
}
