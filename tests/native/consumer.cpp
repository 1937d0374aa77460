// consumer.cpp — TEST HARNESS: a C++ caller of the drop-in boundary, built against include/llsr.h
// and linked with libllsr.so exactly as INTEGRATION.md §2 tells a maintainer to (one TU, the
// header, -lllsr), making the calls INTEGRATION.md §2 shows the ROS nodes making. Each mode writes
// its outputs to a file that tests/test_gpu_consumer.py compares with the oracle (and, for ipfa,
// with the ctypes path too).
//
// usage: consumer <mode> <in.bin> <out.bin>
//   ipfa     ImageProjection::cloudHandler's replacement: the scan arrives as PCL PointXYZI records
//            (32 bytes: x y z _ intensity _ _ _, pcl/point_types.h layout), is repacked to float4
//            and handed to llsr_process_scan; the outputs that fill CloudInfo / ProjectionOut and
//            the FA feature clouds are written out.
//              in:  int32 n_scans, then per scan int32 n + n x float32[4] (x, y, z, intensity)
//              out: per scan int32[8] counts {n_points, S, O, M, Ms, F, L, H}, float32[3]
//                   orientation, int32[H] start_ring, int32[H] end_ring, float32[4S] seg_xyzi,
//                   uint8[S] ground flag, uint32[S] col_ind, float32[S] range, float32[4O]
//                   outlier_xyzi, float32[4S] loam_xyzi, int32[M] less_sharp_ind, int32[Ms]
//                   sharp_ind, int32[F] flat_ind, float32[4L] less_flat
//   s2s      FeatureAssociation::updateTransformation's replacement (llsr_scan2scan) on a sequence
//            of problems; transformCur / isDegenerate are the node's members, carried from one
//            problem to the next as in the reference.
//              in:  int32 P, float32[6] transformCur, int32 isDegenerate, then per problem
//                   int32[4] sizes + the float4 clouds cornerPointsSharp, surfPointsFlat,
//                   laserCloudCornerLast, laserCloudSurfLast
//              out: per problem float32[6] transformCur, int32 isDegenerate, llsr_s2s_report
//   s2m      MapOptimization::scan2MapOptimization's replacement (llsr_scan2map)
//              in:  int32 P, then per problem int32[4] sizes + the float4 clouds CornerScanDS,
//                   SurfTotalLastDS, CornerFromMapDS, SurfFromMapDS, float32[6] transformTobeMapped
//              out: per problem float32[6] transformTobeMapped, llsr_lm_report
//   mapping  the whole chain for one drive through the device-resident entry points
//            (llsr_mapping_init / _batch / _fetch / _keyposes), scans uploaded with hipMemcpy
//              in:  int32 mo_mode, int32 n_scans, then per scan int32 n + float4 points
//              out: per scan llsr_mapping_slot, then int32 K + float32[6K] key poses
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
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

template <class T>
bool get(FILE* f, T* p, size_t n) {
  return n == 0 || fread(p, sizeof(T), n, f) == n;
}

bool get_cloud(FILE* f, std::vector<float>& c, int32_t n) {
  if (n < 0) return false;
  c.resize(4 * (size_t)n);
  return get(f, c.data(), c.size());
}

const float* ptr(const std::vector<float>& c) { return c.empty() ? nullptr : c.data(); }

// FeatureAssociation::updateTransformation: the node's transformCur and
// isDegenerate members go in and come back through the call
int run_s2s(FILE* in, FILE* out) {
  int32_t P = 0, deg = 0;
  float tcur[6];
  if (!get(in, &P, 1) || !get(in, tcur, 6) || !get(in, &deg, 1)) return 2;
  llsr_config cfg;
  llsr_config_default(&cfg, LLSR_LIDAR_VLP16);
  cfg.mode = LLSR_MODE_LM_APPLIED;
  llsr_handle* h = nullptr;
  if (llsr_create(&cfg, 0, 1, 1, &h) != LLSR_OK) return 4;
  std::vector<float> c[4];
  for (int p = 0; p < P; ++p) {
    int32_t n[4];
    if (!get(in, n, 4)) return 2;
    for (int k = 0; k < 4; ++k)
      if (!get_cloud(in, c[k], n[k])) return 2;
    llsr_s2s_report rep;
    const int32_t rc = llsr_scan2scan(h, ptr(c[0]), n[0], ptr(c[1]), n[1], ptr(c[2]), n[2], ptr(c[3]), n[3], tcur,
                                      &deg, &rep);
    if (rc != LLSR_OK) {
      fprintf(stderr, "llsr_scan2scan: %d %s\n", rc, llsr_last_error(h));
      return 5;
    }
    put(out, tcur, 6);
    put(out, &deg, 1);
    put(out, &rep, 1);
  }
  llsr_destroy(h);
  return 0;
}

// MapOptimization::scan2MapOptimization: transformTobeMapped in / out
int run_s2m(FILE* in, FILE* out) {
  int32_t P = 0;
  if (!get(in, &P, 1)) return 2;
  llsr_config cfg;
  llsr_config_default(&cfg, LLSR_LIDAR_VLP16);
  cfg.mode = LLSR_MODE_LM_APPLIED;
  llsr_handle* h = nullptr;
  if (llsr_create(&cfg, 0, 1, 1, &h) != LLSR_OK) return 4;
  std::vector<float> c[4];
  for (int p = 0; p < P; ++p) {
    int32_t n[4];
    float pose[6];
    if (!get(in, n, 4)) return 2;
    for (int k = 0; k < 4; ++k)
      if (!get_cloud(in, c[k], n[k])) return 2;
    if (!get(in, pose, 6)) return 2;
    llsr_lm_report rep;
    const int32_t rc = llsr_scan2map(h, ptr(c[0]), n[0], ptr(c[1]), n[1], ptr(c[2]), n[2], ptr(c[3]), n[3], pose, &rep);
    if (rc != LLSR_OK) {
      fprintf(stderr, "llsr_scan2map: %d %s\n", rc, llsr_last_error(h));
      return 5;
    }
    put(out, pose, 6);
    put(out, &rep, 1);
  }
  llsr_destroy(h);
  return 0;
}

// The mapping chain of one drive: scans uploaded to HBM (what a node holding the decoded cloud on
// the device would pass), one llsr_mapping_batch per scan, the slot state and key poses read back
int run_mapping(FILE* in, FILE* out) {
  int32_t mo_mode = 0, n_scans = 0;
  if (!get(in, &mo_mode, 1) || !get(in, &n_scans, 1)) return 2;
  llsr_config cfg;
  llsr_config_default(&cfg, LLSR_LIDAR_VLP16);
  cfg.mode = LLSR_MODE_LM_APPLIED;  // the odometry's mode; mo_mode is MapOptimization's
  llsr_handle* h = nullptr;
  if (llsr_create(&cfg, 0, 1, 40000, &h) != LLSR_OK) return 4;
  if (llsr_mapping_init(h, mo_mode, nullptr) != LLSR_OK) {
    fprintf(stderr, "llsr_mapping_init: %s\n", llsr_last_error(h));
    return 5;
  }
  float* d_pts = nullptr;
  int64_t* d_off = nullptr;
  if (hipMalloc(&d_pts, 40000 * 16) != hipSuccess || hipMalloc(&d_off, 2 * sizeof(int64_t)) != hipSuccess) return 4;
  std::vector<float> c;
  for (int s = 0; s < n_scans; ++s) {
    int32_t n = 0;
    if (!get(in, &n, 1) || n > 40000 || !get_cloud(in, c, n)) return 2;
    const int64_t off[2] = {0, n};
    if (hipMemcpy(d_pts, c.data(), c.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_off, off, sizeof off, hipMemcpyHostToDevice) != hipSuccess)
      return 4;
    int32_t rc = llsr_mapping_batch(h, d_pts, d_off, 1, nullptr);
    llsr_mapping_slot slot;
    if (rc == LLSR_OK) rc = llsr_mapping_fetch(h, 0, &slot);
    if (rc != LLSR_OK) {
      fprintf(stderr, "llsr_mapping: %d %s\n", rc, llsr_last_error(h));
      return 5;
    }
    put(out, &slot, 1);
  }
  const int32_t K = llsr_mapping_keyposes(h, 0, nullptr, 0);
  std::vector<float> kp(6 * (size_t)(K > 0 ? K : 1));
  llsr_mapping_keyposes(h, 0, kp.data(), K);
  put(out, &K, 1);
  put(out, kp.data(), 6 * (size_t)K);
  (void)hipFree(d_pts);
  (void)hipFree(d_off);
  llsr_destroy(h);
  return 0;
}
}  // namespace

int run_ipfa(FILE* in, FILE* out);

int main(int argc, char** argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: %s ipfa|s2s|s2m|mapping in.bin out.bin\n", argv[0]);
    return 2;
  }
  if (llsr_abi_version() != LLSR_ABI_VERSION) {  // built against another header
    fprintf(stderr, "libllsr ABI %d, header %d\n", (int)llsr_abi_version(), LLSR_ABI_VERSION);
    return 5;
  }
  const std::string mode = argv[1];
  FILE* in = fopen(argv[2], "rb");
  FILE* out = fopen(argv[3], "wb");
  if (!in || !out) return 2;
  int rc = 2;
  if (mode == "ipfa") rc = run_ipfa(in, out);
  else if (mode == "s2s") rc = run_s2s(in, out);
  else if (mode == "s2m") rc = run_s2m(in, out);
  else if (mode == "mapping") rc = run_mapping(in, out);
  fclose(out);
  fclose(in);
  return rc;
}

// ImageProjection::cloudHandler + the FA feature stage
int run_ipfa(FILE* in, FILE* out) {
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
  return 0;
}
