// llsr_input.hip — the input wire formats in front of ImageProjection:
//
//   * sensor_msgs/PointCloud2 -> PointXYZI, as pcl::fromROSMsg<PointXYZI> does it (IP:196) for a
//     batch of messages already in HBM: k_decode_pc2, one lane per point, gathers the x / y / z /
//     intensity fields at their byte offsets (row_step / point_step addressing of organized and
//     unorganized clouds, unaligned fields by bytes) into the float4 layout llsr_process_batch
//     reads. PCL maps a field only when its name, datatype (FLOAT32) and count (1) match; an
//     unmapped field keeps PointXYZI's default (0). NaN points are kept: removeNaNFromPointCloud
//     (IP:198) runs inside llsr_process_batch.
//   * KITTI velodyne .bin (offlineKittiService IP:224-248, KittiLoader imageProjection.h:127-200):
//     float32 x, y, z, reflectance records; the reference reads at most 1,000,000 floats per file
//     and keeps floor(floats_read / 4) points. llsr_kitti_load reads B frames into pinned memory and
//     uploads them with one copy, packed with the offsets llsr_process_batch takes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../include/llsr.h"

namespace {

struct Pc2Msg {            // device copy of one message's addressing
  long long data_off;      // first byte of the message in the packed byte buffer
  long long out_off;       // first output point
  int width, row_step;
};
struct Pc2Fields {
  int point_step;
  int off[4];              // byte offset of x, y, z, intensity; -1 = not mapped
  int aligned;             // every mapped field 4-byte aligned in every point
};

__device__ __forceinline__ float load_f32(const unsigned char* p, bool aligned) {
  if (aligned) return *reinterpret_cast<const float*>(p);
  const unsigned u = (unsigned)p[0] | ((unsigned)p[1] << 8) | ((unsigned)p[2] << 16) | ((unsigned)p[3] << 24);
  return __uint_as_float(u);
}

__global__ __launch_bounds__(256) void k_decode_pc2(const unsigned char* data, const Pc2Msg* msgs, int B,
                                                    Pc2Fields f, long long N, float4* out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  int lo = 0, hi = B - 1;  // last message with out_off <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (msgs[mid].out_off <= i) lo = mid;
    else hi = mid - 1;
  }
  const Pc2Msg m = msgs[lo];
  const long long k = i - m.out_off;
  const long long row = k / m.width, col = k - row * m.width;
  const unsigned char* p = data + m.data_off + row * m.row_step + col * f.point_step;
  const bool al = f.aligned != 0;
  float v[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) v[a] = f.off[a] >= 0 ? load_f32(p + f.off[a], al) : 0.0f;
  out[i] = make_float4(v[0], v[1], v[2], v[3]);
}

}  // namespace

extern "C" int32_t llsr_decode_pointcloud2(const llsr_pc2_layout* lay, const uint8_t* d_data,
                                           const llsr_pc2_msg* msgs, int32_t B, float* d_out, int64_t* out_off,
                                           int64_t* d_out_off, void* hip_stream) {
  if (!lay || !msgs || !out_off || B < 1 || lay->point_step <= 0 || lay->num_fields < 0 ||
      lay->num_fields > LLSR_PC2_MAX_FIELDS)
    return LLSR_EINVAL;
  // createMapping (PCL 1.10 conversions.h): x, y, z, intensity by name + FLOAT32 + count 1
  static const char* kNames[4] = {"x", "y", "z", "intensity"};
  Pc2Fields f{};
  f.point_step = lay->point_step;
  bool aligned = lay->point_step % 4 == 0;
  for (int a = 0; a < 4; ++a) {
    f.off[a] = -1;
    for (int k = 0; k < lay->num_fields; ++k) {
      const llsr_pc2_field& fd = lay->fields[k];
      if (std::strncmp(fd.name, kNames[a], sizeof fd.name) == 0 && fd.datatype == LLSR_PC2_FLOAT32 &&
          fd.count == 1) {
        if (fd.offset < 0 || fd.offset + 4 > lay->point_step) return LLSR_EINVAL;
        f.off[a] = fd.offset;
        aligned = aligned && fd.offset % 4 == 0;
        break;
      }
    }
  }
  std::vector<Pc2Msg> hm(B);
  long long N = 0;
  for (int b = 0; b < B; ++b) {
    const llsr_pc2_msg& m = msgs[b];
    if (m.width < 0 || m.height < 0 || m.data_offset < 0) return LLSR_EINVAL;
    if (m.height > 1 && m.row_step < (long long)m.width * lay->point_step) return LLSR_EINVAL;
    hm[b] = {m.data_offset, N, m.width > 0 ? m.width : 1, m.row_step};
    aligned = aligned && m.data_offset % 4 == 0 && (m.height <= 1 || m.row_step % 4 == 0);
    out_off[b] = N;
    N += (long long)m.width * m.height;
  }
  out_off[B] = N;
  f.aligned = aligned;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  if (N > 0 && (!d_data || !d_out)) return LLSR_EINVAL;
  Pc2Msg* dm = nullptr;
  const size_t tb = B * sizeof(Pc2Msg);
  if (hipMallocAsync(reinterpret_cast<void**>(&dm), tb, s) != hipSuccess) return LLSR_ENOMEM;
  hipError_t e = hipMemcpyAsync(dm, hm.data(), tb, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && N > 0)
    k_decode_pc2<<<(unsigned)((N + 255) / 256), 256, 0, s>>>(d_data, dm, B, f, N, reinterpret_cast<float4*>(d_out));
  if (e == hipSuccess) e = hipGetLastError();
  if (e == hipSuccess && d_out_off)
    e = hipMemcpyAsync(d_out_off, out_off, (B + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s);
  // the host tables are pageable: wait until the copies have consumed them before returning
  if (e == hipSuccess) e = hipFreeAsync(dm, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return e == hipSuccess ? LLSR_OK : LLSR_EIO;
}

// ---- KITTI velodyne .bin ----

static std::string kitti_name(const char* dir, int idx) {
  char buf[32];
  std::snprintf(buf, sizeof buf, "/%06d.bin", idx);
  return std::string(dir) + buf;
}

extern "C" int32_t llsr_kitti_count(const char* velodyne_dir) {
  if (!velodyne_dir) return LLSR_EINVAL;
  int n = 0;
  struct stat st;
  while (stat(kitti_name(velodyne_dir, n).c_str(), &st) == 0) ++n;  // KittiLoader (imageProjection.h:131-136)
  return n;
}

extern "C" int32_t llsr_kitti_read(const char* path, float* xyzi, int32_t cap, int32_t* n) {
  if (!path || !n || cap < 0) return LLSR_EINVAL;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return LLSR_EIO;
  std::vector<float> buf(LLSR_KITTI_MAX_FLOATS);
  const size_t got = std::fread(buf.data(), sizeof(float), buf.size(), fp);  // IP:236
  std::fclose(fp);
  const int32_t np = (int32_t)(got / 4);
  *n = np;
  if (np > cap) return LLSR_ERANGE;
  if (np && xyzi) std::memcpy(xyzi, buf.data(), (size_t)np * 4 * sizeof(float));
  return LLSR_OK;
}

extern "C" int32_t llsr_kitti_load(const char* velodyne_dir, int32_t first, int32_t B, float* d_xyzi,
                                   int64_t cap_points, int64_t* off, int64_t* d_off, void* hip_stream) {
  if (!velodyne_dir || !off || B < 1 || first < 0 || cap_points < 0) return LLSR_EINVAL;
  std::vector<std::vector<float>> frames(B);
  long long N = 0;
  for (int b = 0; b < B; ++b) {
    frames[b].resize(LLSR_KITTI_MAX_FLOATS);
    FILE* fp = std::fopen(kitti_name(velodyne_dir, first + b).c_str(), "rb");
    if (!fp) return LLSR_EIO;
    const size_t got = std::fread(frames[b].data(), sizeof(float), frames[b].size(), fp);
    std::fclose(fp);
    frames[b].resize((got / 4) * 4);
    off[b] = N;
    N += (long long)(got / 4);
  }
  off[B] = N;
  if (N > cap_points) return LLSR_ERANGE;
  if (N > 0 && !d_xyzi) return LLSR_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  float* pinned = nullptr;
  if (N > 0 && hipHostMalloc(reinterpret_cast<void**>(&pinned), (size_t)N * 4 * sizeof(float)) != hipSuccess)
    return LLSR_ENOMEM;
  for (int b = 0; b < B; ++b)
    if (!frames[b].empty()) std::memcpy(pinned + 4 * off[b], frames[b].data(), frames[b].size() * sizeof(float));
  hipError_t e = hipSuccess;
  if (N > 0) e = hipMemcpyAsync(d_xyzi, pinned, (size_t)N * 4 * sizeof(float), hipMemcpyHostToDevice, s);
  if (e == hipSuccess && d_off) e = hipMemcpyAsync(d_off, off, (B + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (pinned) (void)hipHostFree(pinned);
  return e == hipSuccess ? LLSR_OK : LLSR_EIO;
}
