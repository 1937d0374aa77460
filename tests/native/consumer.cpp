// consumer.cpp — TEST HARNESS: a C++ caller of the drop-in boundary, built against include/llsr.h
// and linked with libllsr.so exactly as INTEGRATION.md §2 tells a maintainer to (one TU, the
// header, -lllsr). It follows ImageProjection::cloudHandler's replacement: the scan arrives as
// PCL PointXYZI records (32 bytes: x y z _ intensity _ _ _, pcl/point_types.h layout), is repacked
// to float4, handed to llsr_process_scan, and the outputs that fill CloudInfo / ProjectionOut and
// the FA feature clouds are written to a file the test compares with the ctypes path.
//
// usage: consumer <scans.bin> <out.bin>
//   scans.bin: int32 n_scans, then per scan int32 n + n x float32[4] (x, y, z, intensity)
//   out.bin:   per scan int32[8] counts {n_points, S, O, M, Ms, F, L, H}, float32[3] orientation,
//              int32[H] start_ring, int32[H] end_ring, float32[4S] seg_xyzi, uint8[S] ground flag,
//              uint32[S] col_ind, float32[S] range, float32[4O] outlier_xyzi, float32[4S] loam_xyzi,
//              int32[M] less_sharp_ind, int32[Ms] sharp_ind, int32[F] flat_ind, float32[4L] less_flat
#include <cstdint>
#include <cstdio>
#include <vector>

#include "llsr.h"

namespace {
struct PointXYZI {  // pcl::PointXYZI memory layout (PCL_ADD_POINT4D + intensity, 16-byte aligned)
  float x, y, z, pad0;
  float intensity, pad1, pad2, pad3;
};

template <class T>
void put(FILE* f, const T* p, size_t n) {
  if (n) fwrite(p, sizeof(T), n, f);
}
}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s scans.bin out.bin\n", argv[0]);
    return 2;
  }
  FILE* in = fopen(argv[1], "rb");
  FILE* out = fopen(argv[2], "wb");
  if (!in || !out) return 2;
  int32_t n_scans = 0;
  if (fread(&n_scans, 4, 1, in) != 1) return 2;

  llsr_config cfg;
  if (llsr_config_default(&cfg, LLSR_LIDAR_VLP16) != LLSR_OK) return 3;
  llsr_handle* h = nullptr;
  int32_t rc = llsr_create(&cfg, 0, 1, 40000, &h);
  if (rc != LLSR_OK) {
    fprintf(stderr, "llsr_create: %d\n", rc);
    return 4;
  }
  llsr_sizes sz;
  llsr_query_sizes(h, &sz);
  const size_t HW = (size_t)sz.cells, H = (size_t)sz.rings;
  // reusable buffers, sized once from llsr_query_sizes (the node's members in INTEGRATION.md)
  std::vector<int32_t> start(H), end(H), edge(HW), sharp(HW), flat(HW);
  std::vector<float> seg(4 * HW), rng(HW), sint(HW), outl(4 * HW), oint(HW), loam(4 * HW), lflat(4 * HW);
  std::vector<uint8_t> gflag(HW);
  std::vector<uint32_t> col(HW);
  std::vector<PointXYZI> cloud;
  std::vector<float> xyzi;

  for (int s = 0; s < n_scans; ++s) {
    int32_t n = 0;
    if (fread(&n, 4, 1, in) != 1) return 2;
    // pcl::fromROSMsg(*msg, *_laser_cloud_in) stand-in: the PCL cloud the callback holds
    cloud.assign((size_t)n, PointXYZI{});
    for (int i = 0; i < n; ++i) {
      float p[4];
      if (fread(p, 4, 4, in) != 4) return 2;
      cloud[i].x = p[0]; cloud[i].y = p[1]; cloud[i].z = p[2]; cloud[i].intensity = p[3];
    }
    // repack the 32-byte PCL points to float4, NaNs kept (the ABI removes them)
    xyzi.resize(4 * (size_t)n);
    for (int i = 0; i < n; ++i) {
      const PointXYZI& p = cloud[i];
      xyzi[4 * i] = p.x; xyzi[4 * i + 1] = p.y; xyzi[4 * i + 2] = p.z; xyzi[4 * i + 3] = p.intensity;
    }
    llsr_scan_out o{};
    o.start_ring_index = start.data(); o.end_ring_index = end.data();
    o.seg_xyzi = seg.data(); o.seg_ground_flag = gflag.data(); o.seg_col_ind = col.data();
    o.seg_range = rng.data(); o.seg_intensity = sint.data();
    o.outlier_xyzi = outl.data(); o.outlier_intensity = oint.data();
    o.loam_xyzi = loam.data(); o.less_sharp_ind = edge.data(); o.sharp_ind = sharp.data();
    o.flat_ind = flat.data(); o.less_flat_xyzi = lflat.data();
    rc = llsr_process_scan(h, xyzi.data(), n, &o);
    if (rc != LLSR_OK) {
      fprintf(stderr, "llsr_process_scan: %d %s\n", rc, llsr_last_error(h));
      return 5;
    }
    const int32_t counts[8] = {o.n_points, o.n_segmented, o.n_outlier, o.n_less_sharp,
                               o.n_sharp,  o.n_flat,      o.n_less_flat, (int32_t)H};
    put(out, counts, 8);
    put(out, o.orientation, 3);
    put(out, start.data(), H);
    put(out, end.data(), H);
    const size_t S = (size_t)o.n_segmented, O = (size_t)o.n_outlier;
    put(out, seg.data(), 4 * S);
    put(out, gflag.data(), S);
    put(out, col.data(), S);
    put(out, rng.data(), S);
    put(out, outl.data(), 4 * O);
    put(out, loam.data(), 4 * S);
    put(out, edge.data(), (size_t)o.n_less_sharp);
    put(out, sharp.data(), (size_t)o.n_sharp);
    put(out, flat.data(), (size_t)o.n_flat);
    put(out, lflat.data(), 4 * (size_t)o.n_less_flat);
  }
  llsr_destroy(h);
  fclose(out);
  fclose(in);
  return 0;
}
