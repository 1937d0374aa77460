// llsr_capi.hip — host side of the C-ABI (include/llsr.h): handle lifetime, the HBM buffer
// pool, the per-batch launch sequence and result fetch. No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/llsr.h"
#include "llsr_device.h"
#include "llsr_libm.h"
#include "llsr_grid.h"
#include "llsr_mapping.h"
#include "llsr_mo.h"
#include "llsr_odo.h"
#include "llsr_s2s.h"

namespace llsr {
__global__ void k_project(DevCfg, const float4*, const int64_t*, DevBufs);
__global__ void k_gather_column(DevCfg, const float4*, const int64_t*, DevBufs);
__global__ void k_project_fused(DevCfg, const float4*, const int64_t*, DevBufs);
__global__ void k_ground_add(DevCfg, DevBufs);
__global__ void k_ground_elev_ransac(DevCfg, DevBufs);
template <bool kLds> __global__ void k_label(DevCfg, DevBufs);
__global__ void k_segment(DevCfg, const float4*, const int64_t*, DevBufs);
void launch_fa_points(const DevCfg&, const DevBufs&, int, hipStream_t);
__global__ void k_select_ring(DevCfg, DevBufs);
__global__ void k_vox_pcl(DevCfg, DevBufs);
__global__ void k_debug_exact_sort(const float*, int, int*, long long*);
__global__ void k_debug_exact_sort32(const uint32_t*, int, int*);
__global__ void k_debug_half_passed(const float*, int, uint8_t*);
__global__ void k_fa_concat(DevCfg, DevBufs);
__global__ void k_dbscan_adj(DevCfg, DevBufs, const float4* __restrict__);
__global__ void k_vis_clouds(DevCfg, DevBufs, int, float4*, int*);
template <int kDbL> __global__ void k_dbscan_merge(DevCfg, DevBufs);

__global__ void k_init_counts(int* counts, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int* c = counts + b * kCnt;
  for (int k = 0; k < kCnt; ++k) c[k] = 0;
  c[C_FIRST] = INT_MAX;
  c[C_LAST] = -1;
}
}  // namespace llsr

using namespace llsr;

namespace {
const char* kKernelNames[] = {"init",          "k_project",    "k_gather_column", "k_ground_add",
                              "k_ground_elev_ransac", "k_label", "k_segment",      "k_fa_points",
                              "k_select_ring", "k_vox_pcl", "k_fa_concat", "k_dbscan_adj", "k_dbscan_merge"};
constexpr int kNumKernels = 13;
}  // namespace

struct llsr_handle {
  llsr_config cfg;
  DevCfg dc;
  int device = 0;
  int max_batch = 0, max_points = 0;
  DevBufs d{};
  void* pool = nullptr;
  size_t pool_bytes = 0;
  float4* d_in = nullptr;      // single-scan staging
  float4* d_vis = nullptr;     // llsr_fetch_vis_clouds: 6 x HW points + 4 counts (on first use)
  int64_t* d_off = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t last_stream = nullptr;  // compared, never used: the caller may destroy its streams
  hipEvent_t last_done = nullptr;  // recorded after each batch: the next one (any stream) waits on it
  // Handle-owned completion events of the last work enqueued on a caller's stream, per kind
  // (feature batches / odometry / mapping, scan-to-scan, scan-to-map): buffer re-allocation and
  // llsr_destroy wait on these, so a stream the caller destroyed since is never touched.
  hipEvent_t s2s_done = nullptr, mo_done = nullptr;
  bool last_rec = false, s2s_rec = false, mo_rec = false;
  int last_B = 0;
  const float4* last_pts = nullptr;  // inputs of the last batch (diagnostic re-launches only)
  const int64_t* last_off = nullptr;
  bool profiling = false;
  bool debug_sync = false;  // LLSR_DEBUG_SYNC=1: wait after every feature-batch kernel, name a failing one
  // Event sets for up to kRing in-flight profiled batches; retired sets are summed into ksum.
  static constexpr int kRing = 64;
  hipEvent_t ev[kRing][kNumKernels + 1] = {};
  int ring_head = 0, ring_used = 0;
  double ksum[kNumKernels] = {};
  long long kbatches = 0;
  // scan-to-map (llsr_scan2map_*): buffers sized by llsr_scan2map_reserve
  struct {
    int P = 0, qc = 0, qs = 0, mc = 0, ms = 0, log2T_c = 0, log2T_s = 0, blocks_c = 0, blocks = 0;
    void* pool = nullptr;
    S2MArgs a{};
    int* host_flags = nullptr;   // pinned: n_active, error
    void* stage = nullptr;       // single-problem staging (llsr_scan2map)
    size_t stage_bytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipEvent_t p0 = nullptr, p1 = nullptr, p2 = nullptr;  // profiling: start, grid built, LM done
    llsr_s2m_stats stats{};
    S2MArgs sh{};                // the open split-correspondence batch (llsr_scan2map_shard_*)
    bool sh_live = false;
  } mo;
  // scan-to-scan (llsr_scan2scan_*)
  struct {
    int P = 0, ms = 0, f = 0, nc = 0, ns = 0;
    void* pool = nullptr;
    S2SArgs a{};
    int* host_flag = nullptr;
    void* stage = nullptr;
    size_t stage_bytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipEvent_t p0 = nullptr, p1 = nullptr, p2 = nullptr;  // profiling: start, grids built, LM done
    llsr_s2s_stats stats{};
    int last_variant = 0;  // kLdsRows of the last k_s2s_lm instantiation launched (diagnostics)
  } s2s;
  // end-to-end odometry (llsr_odometry_*): per-slot FA state + packed clouds, allocated lazily
  struct {
    void* pool = nullptr;
    int B = 0;                    // slots
    size_t cap = 0;               // points per packed buffer (B * (H*W + 160))
    float* tcur = nullptr;        // [B][6]
    float* tsum = nullptr;        // [B][6]
    int* deg = nullptr;           // [B] isDegenerate
    int* inited = nullptr;        // [B]
    int* frames = nullptr;        // [B]
    float4* shadow = nullptr;     // [160]
    float4 *sharp = nullptr, *flat = nullptr, *scan_c = nullptr, *scan_s = nullptr;
    float4 *last_c[2] = {nullptr, nullptr}, *last_s[2] = {nullptr, nullptr};
    int64_t* off = nullptr;       // device [6][B+1]: sharp, flat, last_c[0], last_c[1], last_s[0], last_s[1]
    int64_t* h_off = nullptr;     // pinned host copy
    int* h_counts = nullptr;      // pinned [B][kCnt]
    llsr_s2s_report* report = nullptr;  // [B]
    int cur = 0;                  // last_c/s[cur] hold the current last clouds
  } odo;
  // mapping chain (llsr_mapping_*): MapOptimization's members per slot + the batch buffers
  struct MapSlot {
    llsr_mapping::MoPoses pose;
    llsr_map* map = nullptr;           // keyframe store (cornerCloudKeyFrames etc., cloudKeyPoses6D)
    float robot[3] = {0, 0, 0};        // currentRobotPosPoint
    int frames = 0, mo_frames = 0, lm_ran = 0, n_cq = 0, n_sq = 0;
    int cycle = 0;                     // FeatureAssociation's _cycle_count (FA:2818-2821)
    llsr_lm_report lm{};
    llsr_map_report mrep{};
    std::vector<float> keyposes;       // [keyframes][6]
  };
  struct {
    bool live = false;
    int mode = LLSR_MODE_LM_APPLIED;   // MapOptimization's LM mode
    llsr_map_config mcfg{};
    llsr_map* vg = nullptr;            // VoxelGrid engine of the batched downsample
    std::vector<MapSlot> slot;
    float4 *outl = nullptr, *ds = nullptr, *tot = nullptr, *cmap = nullptr;  // cmap: empty-map base
    size_t cap_outl = 0, cap_ds = 0, cap_tot = 0, cap_cmap = 0;
    void* small = nullptr;             // device: pose [B][6], report [B], deg [B], matP [B][36], off [5][B+1],
                                       // and the deg / matP of the frame before (rollback)
    void* hsmall = nullptr;            // pinned host mirror
    float* d_pose = nullptr; llsr_lm_report* d_rep = nullptr; int* d_deg = nullptr; float* d_matP = nullptr;
    int* d_deg_bak = nullptr; float* d_matP_bak = nullptr;
    int64_t* d_off = nullptr;
    float* h_pose = nullptr; llsr_lm_report* h_rep = nullptr; int64_t* h_off = nullptr; int* h_frames = nullptr;
    float* h_tsum = nullptr;
  } mp;
  std::string err;
};

// The fused projection keeps the winning raw index per cell in LDS (k_project_fused).
static int fused_lds(const DevCfg& c) { return c.HW * (int)sizeof(int); }
// k_label<true>'s dynamic LDS: the parent word and the edge-bit byte of every cell (HW <= 32000:
// <= 160000 B)
static int label_lds(const DevCfg& c) { return c.HW * (int)(sizeof(int) + 1); }

static int label_band_lds(const DevCfg& c) { return c.lbl_band * c.W * (int)sizeof(int); }
static bool use_fused(const llsr_handle* h) { return h->dc.ccl_lds != 0; }

// k_segment / k_ground_elev_ransac (any multiple of 64 up to 1024 threads): 512 for range images
// that fit LDS (VLP-16: three / two scans per CU instead of one; r06_v40, 0.289 -> 0.282 and
// 0.180 -> 0.167 ms per 1024 scans), 1024 for the larger ones (HDL-64E: 512 was slower)
static int per_scan_threads(const DevCfg& c) { return c.ccl_lds ? 512 : 1024; }

// the PCL-order less-flat VoxelGrid of every pending ring
static void launch_vox_pcl(const DevCfg& c, const DevBufs& d, int B, hipStream_t s) {
  k_vox_pcl<<<dim3(c.H, B), 256, 0, s>>>(c, d);
}

static int32_t fail(llsr_handle* h, int32_t code, const std::string& msg) {
  if (h) h->err = msg;
  return code;
}

#define HIP_OK(h, expr)                                                                  \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(h, LLSR_EIO, std::string(#expr ": ") + hipGetErrorString(e_));         \
  } while (0)

extern "C" int32_t llsr_abi_version(void) { return LLSR_ABI_VERSION; }

extern "C" int32_t llsr_config_default(llsr_config* c, int32_t lidar) {
  if (!c) return LLSR_EINVAL;
  std::memset(c, 0, sizeof *c);
  if (lidar == LLSR_LIDAR_VLP16) {  // loam_config.yaml:1-67
    c->num_vertical_scans = 16; c->num_horizontal_scans = 1800;
    c->vertical_angle_bottom = -15.0f; c->vertical_angle_top = 15.0f;
    c->ground_scan_index = 7; c->use_kitti = 0;
    c->DBFr = 5.0f; c->RatioXY = 0.5f; c->RatioZ = 2.5f;
    c->edge_threshold = 0.03f; c->surf_threshold = 0.03f; c->nearest_feature_search_distance = 5.0f;
  } else if (lidar == LLSR_LIDAR_HDL64E) {  // loam_config.yaml:137-203
    c->num_vertical_scans = 64; c->num_horizontal_scans = 1800;
    c->vertical_angle_bottom = -24.8f; c->vertical_angle_top = 2.0f;
    c->ground_scan_index = 50; c->use_kitti = 1;
    c->DBFr = 7.5f; c->RatioXY = 0.3f; c->RatioZ = 5.0f;
    c->edge_threshold = 0.005f; c->surf_threshold = 0.005f; c->nearest_feature_search_distance = 25.0f;
  } else {
    return LLSR_EINVAL;
  }
  c->sensor_mount_angle = 0.0f;
  c->use_vlp32c = 0;
  c->segment_theta = 60.0f; c->segment_valid_point_num = 5; c->segment_valid_line_num = 3;
  c->scan_period = 0.1f;
  c->mapping_frequency_divider = 1;
  c->iterCountThres = 200; c->step_size = 1.0f; c->stop_thres = 0.05f;
  c->mode = LLSR_MODE_FAITHFUL;
  return LLSR_OK;
}

// Host-side constants with the reference's exact conversions (IP:117-121, 849; FA:152-154).
static void make_devcfg(const llsr_config& c, DevCfg& d) {
  const double kDegToRad = M_PI / 180.0;
  d.H = c.num_vertical_scans;
  d.W = c.num_horizontal_scans;
  d.HW = d.H * d.W;
  d.ip_resX = (float)((M_PI * 2) / d.W);
  d.ip_resY = (float)(kDegToRad * (c.vertical_angle_top - c.vertical_angle_bottom) / float(d.H - 1));
  d.ip_angBottom = (float)(-(c.vertical_angle_bottom - 0.1) * kDegToRad);
  const float segTheta = (float)(c.segment_theta * kDegToRad);
  d.segThr = std::tan(segTheta);
  d.sinX = std::sin(d.ip_resX); d.cosX = std::cos(d.ip_resX);
  d.sinY = std::sin(d.ip_resY); d.cosY = std::cos(d.ip_resY);
  d.use_kitti = c.use_kitti;
  d.gsi = c.ground_scan_index;
  d.pointNum = c.segment_valid_point_num;
  d.lineNum = c.segment_valid_line_num;
  d.scan_period = c.scan_period;
  d.edge_thr = c.edge_threshold;
  d.surf_thr = c.surf_threshold;
  const float fa_resX = (float)((M_PI * 2) / d.W);
  d.fa_resY = (float)(kDegToRad * (c.vertical_angle_top - c.vertical_angle_bottom) / float(d.H - 1));
  d.sinResX = std::sin(fa_resX);
  d.RatioXY = c.RatioXY;
  d.RatioZ = c.RatioZ;
  d.DBFr = c.DBFr;
  d.gnd_cos[0] = llsr_libm::ground_cos_threshold(12.5f);
  d.gnd_cos[1] = llsr_libm::ground_cos_threshold(60.0f);
  d.gnd_cos[2] = llsr_libm::ground_cos_threshold(25.0f);
  d.ccl_lds = (d.H <= 16 && d.HW <= 32000) ? 1 : 0;
  // 72 KB bands: two labelling workgroups per CU (a 512-scan HDL-64E batch runs in one round)
  // (at most 16 rows: a band root's LDS word keeps its members' rows in 16 bits)
  d.lbl_band = std::max(1, std::min(std::min(d.H, 16), 18432 / std::max(1, d.W)));
  d.exact_vg = 1;  // LLSR_VOXEL_ORDER_PCL: the reference's summation order
  d.dbg_phase = 1 << 30;
}

template <class T>
static T* carve(char*& p, size_t n) {
  T* r = reinterpret_cast<T*>(p);
  p += (n * sizeof(T) + 255) & ~size_t(255);
  return r;
}

static void mapping_free(llsr_handle* h);

// Wait for every stream this handle has launched work on (before its buffers are re-allocated):
// stream-scoped, so other handles' streams on the device keep running.
static hipError_t sync_handle_streams(llsr_handle* h);

// boost::mt19937 seeded with 12345 (PCL 1.10 SampleConsensusModel's rng_alg_, IP:716-721), state
// after the seeding recurrence and the first twist: every scan's RANSAC starts its draws here, so
// the device loads 624 words instead of running 1248 serial steps on one lane per scan.
static void mt_first_state(uint32_t* m) {
  m[0] = 12345u;
  for (int k = 1; k < 624; ++k) m[k] = 1812433253u * (m[k - 1] ^ (m[k - 1] >> 30)) + (uint32_t)k;
  for (int k = 0; k < 624; ++k) {
    const uint32_t y = (m[k] & 0x80000000u) | (m[(k + 1) % 624] & 0x7fffffffu);
    m[k] = m[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
}

static size_t layout(DevBufs& d, char* p0, int B, int H, int HW) {
  char* p = p0;
  const size_t n = (size_t)B * HW;
  d.counts = carve<int>(p, (size_t)B * kCnt);
  d.orient = carve<float>(p, (size_t)B * 4);
  d.cell_pt = carve<int>(p, n);
  d.range = carve<float>(p, n);
  d.full = carve<float4>(p, n);
  d.ground = carve<int8_t>(p, n);
  d.label = carve<int>(p, n);
  d.near_pts = carve<float4>(p, n);
  d.shuf = carve<int>(p, n);
  d.ccl_a = carve<int>(p, n);
  d.ccl_b = carve<unsigned long long>(p, n);
  d.start_ring = carve<int>(p, (size_t)B * H);
  d.end_ring = carve<int>(p, (size_t)B * H);
  d.seg = carve<float4>(p, n);
  d.seg_ground = carve<uint8_t>(p, n);
  d.seg_col = carve<uint32_t>(p, n);
  d.seg_range = carve<float>(p, n);
  d.seg_int = carve<float>(p, n);
  d.outl = carve<float4>(p, n);
  d.outl_int = carve<float>(p, n);
  d.loam = carve<float4>(p, n);
  d.curv = carve<float>(p, n);
  d.picked = carve<uint8_t>(p, n);
  d.clabel = carve<int8_t>(p, n);
  d.ring_cnt = carve<int>(p, (size_t)B * 3 * H);
  d.edge_tmp = carve<int>(p, n);
  d.flat_tmp = carve<int>(p, n);
  d.lflat_tmp = carve<float4>(p, n);
  d.less_sharp = carve<int>(p, n);
  d.cluster = carve<int>(p, n);
  d.sharp = carve<int>(p, n);
  d.flat = carve<int>(p, n);
  d.lflat = carve<float4>(p, n);
  d.db_pts = carve<float4>(p, n);
  d.db_kz = carve<float>(p, n);
  d.db_adj = carve<uint32_t>(p, (size_t)B * kAdjCap * kAdjWords);
  d.mt0 = carve<uint32_t>(p, 624);
  d.phantom = carve<int>(p, (size_t)B);
  d.seg_zero = carve<int>(p, (size_t)B);
  return (size_t)(p - p0);
}

extern "C" int32_t llsr_create(const llsr_config* cfg, int32_t hip_device, int32_t max_batch,
                               int32_t max_points, llsr_handle** out) {
  if (!cfg || !out || max_batch < 1 || max_points < 1) return LLSR_EINVAL;
  *out = nullptr;
  if (cfg->use_vlp32c) return LLSR_ENOSYS;
  if (cfg->num_vertical_scans < 2 || cfg->num_vertical_scans > 64 || cfg->num_horizontal_scans < 16 ||
      cfg->num_horizontal_scans > 2048)
    return LLSR_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= hip_device || hip_device < 0) return LLSR_ENODEV;
  llsr_handle* h = new (std::nothrow) llsr_handle();
  if (!h) return LLSR_ENOMEM;
  h->cfg = *cfg;
  h->device = hip_device;
  h->max_batch = max_batch;
  h->max_points = max_points;
  make_devcfg(*cfg, h->dc);
  if (hipSetDevice(hip_device) != hipSuccess) { delete h; return LLSR_ENODEV; }
  DevBufs probe{};
  const size_t bytes = layout(probe, nullptr, max_batch, h->dc.H, h->dc.HW) + 4096;
  if (hipMalloc(&h->pool, bytes) != hipSuccess) { delete h; return LLSR_ENOMEM; }
  h->pool_bytes = bytes;
  layout(h->d, (char*)h->pool, max_batch, h->dc.H, h->dc.HW);
  {
    uint32_t mt0[624];
    mt_first_state(mt0);
    if (hipMemcpy(h->d.mt0, mt0, sizeof(mt0), hipMemcpyHostToDevice) != hipSuccess) {
      llsr_destroy(h);
      return LLSR_ENODEV;
    }
  }
  if (hipMalloc(&h->d_in, sizeof(float4) * (size_t)max_points) != hipSuccess ||
      hipMalloc(&h->d_off, sizeof(int64_t) * 2) != hipSuccess ||
      hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    llsr_destroy(h);
    return LLSR_ENOMEM;
  }
  {
    const char* ds = std::getenv("LLSR_DEBUG_SYNC");
    h->debug_sync = ds && ds[0] == '1';
  }
  for (auto& set : h->ev)
    for (auto& e : set)
      if (hipEventCreate(&e) != hipSuccess) { llsr_destroy(h); return LLSR_ENODEV; }
  if (hipEventCreateWithFlags(&h->last_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->s2s_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->mo_done, hipEventDisableTiming) != hipSuccess) {
    llsr_destroy(h);
    return LLSR_ENODEV;
  }
  if (!h->dc.ccl_lds &&
      hipFuncSetAttribute((const void*)k_label<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          label_band_lds(h->dc)) != hipSuccess) {
    llsr_destroy(h);
    return LLSR_ENODEV;
  }
  if (h->dc.ccl_lds) {
    if (hipFuncSetAttribute((const void*)k_label<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            label_lds(h->dc)) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_project_fused, hipFuncAttributeMaxDynamicSharedMemorySize,
                            fused_lds(h->dc)) != hipSuccess) {
      llsr_destroy(h);
      return LLSR_ENODEV;
    }
  }
  int32_t rc = llsr_reset_state(h);
  if (rc != LLSR_OK) { llsr_destroy(h); return rc; }
  *out = h;
  return LLSR_OK;
}

extern "C" void llsr_destroy(llsr_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)sync_handle_streams(h);
  for (auto& set : h->ev)
    for (auto& e : set)
      if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {h->last_done, h->s2s_done, h->mo_done})
    if (e) (void)hipEventDestroy(e);
  if (h->pool) (void)hipFree(h->pool);
  if (h->d_vis) (void)hipFree(h->d_vis);
  if (h->mo.pool) (void)hipFree(h->mo.pool);
  if (h->s2s.pool) (void)hipFree(h->s2s.pool);
  if (h->s2s.stage) (void)hipFree(h->s2s.stage);
  if (h->s2s.host_flag) (void)hipHostFree(h->s2s.host_flag);
  if (h->s2s.e0) (void)hipEventDestroy(h->s2s.e0);
  if (h->s2s.e1) (void)hipEventDestroy(h->s2s.e1);
  for (hipEvent_t e : {h->s2s.p0, h->s2s.p1, h->s2s.p2})
    if (e) (void)hipEventDestroy(e);
  if (h->odo.pool) (void)hipFree(h->odo.pool);
  if (h->odo.h_off) (void)hipHostFree(h->odo.h_off);
  if (h->odo.h_counts) (void)hipHostFree(h->odo.h_counts);
  if (h->mo.stage) (void)hipFree(h->mo.stage);
  if (h->mo.host_flags) (void)hipHostFree(h->mo.host_flags);
  if (h->mo.e0) (void)hipEventDestroy(h->mo.e0);
  if (h->mo.e1) (void)hipEventDestroy(h->mo.e1);
  for (hipEvent_t e : {h->mo.p0, h->mo.p1, h->mo.p2})
    if (e) (void)hipEventDestroy(e);
  mapping_free(h);
  for (void* p : {(void*)h->mp.outl, (void*)h->mp.ds, (void*)h->mp.tot, (void*)h->mp.cmap})
    if (p) (void)hipFree(p);
  if (h->d_in) (void)hipFree(h->d_in);
  if (h->d_off) (void)hipFree(h->d_off);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

static hipError_t sync_handle_streams(llsr_handle* h) {
  if (h->stream) {
    const hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return e;
  }
  const std::pair<hipEvent_t, bool> evs[] = {{h->last_done, h->last_rec}, {h->s2s_done, h->s2s_rec},
                                             {h->mo_done, h->mo_rec}};
  for (const auto& ev : evs) {
    if (!ev.first || !ev.second) continue;
    const hipError_t e = hipEventSynchronize(ev.first);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

extern "C" int32_t llsr_get_config(const llsr_handle* h, llsr_config* cfg) {
  if (!h || !cfg) return LLSR_EINVAL;
  *cfg = h->cfg;
  return LLSR_OK;
}

extern "C" const char* llsr_last_error(const llsr_handle* h) { return h ? h->err.c_str() : "null handle"; }

extern "C" int32_t llsr_query_sizes(const llsr_handle* h, llsr_sizes* s) {
  if (!h || !s) return LLSR_EINVAL;
  s->cells = h->dc.HW;
  s->rings = h->dc.H;
  s->max_points = h->max_points;
  s->shadow_points = 160;
  return LLSR_OK;
}

extern "C" int32_t llsr_set_voxel_order(llsr_handle* h, int32_t order) {
  if (!h) return LLSR_EINVAL;
  if (order != LLSR_VOXEL_ORDER_INPUT && order != LLSR_VOXEL_ORDER_PCL) return fail(h, LLSR_EINVAL, "voxel order");
  h->dc.exact_vg = order == LLSR_VOXEL_ORDER_PCL ? 1 : 0;
  return LLSR_OK;
}

extern "C" int32_t llsr_reset_state(llsr_handle* h) {
  if (!h) return LLSR_EINVAL;
  HIP_OK(h, hipSetDevice(h->device));
  const size_t n = (size_t)h->max_batch * h->dc.HW;
  HIP_OK(h, hipMemsetAsync(h->d.picked, 0, n, h->stream));
  HIP_OK(h, hipMemsetAsync(h->d.clabel, 0, n, h->stream));
  HIP_OK(h, hipMemsetAsync(h->d.phantom, 0, sizeof(int) * (size_t)h->max_batch, h->stream));
  HIP_OK(h, hipMemsetD32Async(h->d.seg_zero, h->dc.HW, (size_t)h->max_batch, h->stream));
  HIP_OK(h, hipStreamSynchronize(h->stream));
  return LLSR_OK;
}

// Retire the oldest profiled batch: wait for its last event and add its kernel intervals.
static void retire_oldest(llsr_handle* h) {
  const int slot = (h->ring_head - h->ring_used + llsr_handle::kRing) % llsr_handle::kRing;
  (void)hipEventSynchronize(h->ev[slot][kNumKernels]);
  for (int k = 0; k < kNumKernels; ++k) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->ev[slot][k], h->ev[slot][k + 1]) == hipSuccess) h->ksum[k] += ms;
  }
  h->kbatches += 1;
  h->ring_used -= 1;
}

extern "C" int32_t llsr_set_profiling(llsr_handle* h, int32_t enable) {
  if (!h) return LLSR_EINVAL;
  while (h->ring_used > 0) retire_oldest(h);
  for (double& v : h->ksum) v = 0.0;
  h->kbatches = 0;
  h->mo.stats = llsr_s2m_stats{};
  h->s2s.stats = llsr_s2s_stats{};
  h->profiling = enable != 0;
  return LLSR_OK;
}

extern "C" int32_t llsr_process_batch(llsr_handle* h, const float* d_xyzi, const int64_t* d_offsets,
                                      int32_t B, void* hip_stream) {
  if (!h || !d_xyzi || !d_offsets) return fail(h, LLSR_EINVAL, "null argument");
  if (B < 1 || B > h->max_batch) return fail(h, LLSR_ERANGE, "batch size outside [1, max_batch]");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  // the slot buffers and the FA carry-over state are shared by every batch of this handle: a
  // batch on another stream than the previous one starts after it
  if (h->last_stream && h->last_stream != s) HIP_OK(h, hipStreamWaitEvent(s, h->last_done, 0));
  const DevCfg& c = h->dc;
  const float4* pts = reinterpret_cast<const float4*>(d_xyzi);
  int k = 0;
  if (h->profiling && h->ring_used == llsr_handle::kRing) retire_oldest(h);
  hipEvent_t* evs = h->ev[h->ring_head];
  auto mark = [&]() {
    if (h->profiling) (void)hipEventRecord(evs[k], s);
    if (h->debug_sync) {  // diagnostics: the kernel that faults is the last one named
      const hipError_t e = hipStreamSynchronize(s);
      std::fprintf(stderr, "llsr debug: after %s: %s\n", k < kNumKernels ? kKernelNames[k] : "?", hipGetErrorString(e));
    }
    ++k;
  };
  mark();
  const bool fused = use_fused(h);
  if (!fused) HIP_OK(h, hipMemsetAsync(h->d.ccl_a, 0xFF, sizeof(int) * (size_t)B * c.HW, s));
  k_init_counts<<<(B + 255) / 256, 256, 0, s>>>(h->d.counts, B);
  mark();
  if (fused) {  // fused projection + column ground pass with the cell table in LDS
    k_project_fused<<<B, 1024, fused_lds(c), s>>>(c, pts, d_offsets, h->d);
    mark();
    mark();
  } else {
    // grid-stride kernels: ~16k workgroups in all, at least 4 per scan
    const int gx = std::max(1, std::min((h->max_points + 255) / 256, std::max(4, 16384 / B)));
    k_project<<<dim3(gx, B), 256, 0, s>>>(c, pts, d_offsets, h->d);
    mark();
    k_gather_column<<<dim3((c.W + 63) / 64, B), 64, sizeof(int) * 64 * (c.H + 1), s>>>(c, pts, d_offsets, h->d);
    mark();
  }
  k_ground_add<<<dim3((c.H + 3) / 4, B), 256, 0, s>>>(c, h->d);
  mark();
  k_ground_elev_ransac<<<B, per_scan_threads(c), 0, s>>>(c, h->d);
  mark();
  if (c.ccl_lds)
    k_label<true><<<B, 1024, label_lds(c), s>>>(c, h->d);
  else
    k_label<false><<<B, 1024, label_band_lds(c), s>>>(c, h->d);
  mark();
  k_segment<<<B, per_scan_threads(c), 0, s>>>(c, pts, d_offsets, h->d);
  mark();
  launch_fa_points(c, h->d, B, s);
  mark();
  k_select_ring<<<dim3(c.H, B), 256, 0, s>>>(c, h->d);
  mark();
  if (c.exact_vg) launch_vox_pcl(c, h->d, B, s);  // the PCL-order VoxelGrid
  mark();
  k_fa_concat<<<B, 256, 0, s>>>(c, h->d);
  mark();
  k_dbscan_adj<<<dim3(32, B), 256, 0, s>>>(c, h->d, h->d.db_pts);
  mark();
  if (c.HW <= 32768) k_dbscan_merge<1024><<<B, 64, 0, s>>>(c, h->d);
  else k_dbscan_merge<2048><<<B, 64, 0, s>>>(c, h->d);
  mark();
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipEventRecord(h->last_done, s));
  h->last_rec = true;
  if (h->profiling) {
    h->ring_head = (h->ring_head + 1) % llsr_handle::kRing;
    h->ring_used += 1;
  }
  h->last_stream = s;
  h->last_B = B;
  h->last_pts = pts;
  h->last_off = d_offsets;
  return LLSR_OK;
}

static int32_t sync_last(llsr_handle* h) {
  HIP_OK(h, hipSetDevice(h->device));
  if (h->last_rec) HIP_OK(h, hipEventSynchronize(h->last_done));
  else HIP_OK(h, hipStreamSynchronize(h->stream));
  return LLSR_OK;
}

extern "C" int32_t llsr_kernel_times_ms(llsr_handle* h, float* out, int32_t cap) {
  if (!h || !out) return LLSR_EINVAL;
  HIP_OK(h, hipSetDevice(h->device));
  while (h->ring_used > 0) retire_oldest(h);
  if (h->kbatches == 0) return 0;
  int n = 0;
  for (int k = 0; k < kNumKernels && n < cap; ++k, ++n) out[n] = (float)(h->ksum[k] / (double)h->kbatches);
  return n;
}

// Diagnostics (not part of the ABI header): the device's exact libstdc++ std::sort (the per-ring
// curvature sort's tie path and the PCL-order VoxelGrid, llsr_isort.h block_introsort) on n <= 2048 host values; out[k] = the
// input position at sorted position k. For tests/test_gpu_features_ties.py.
extern "C" int32_t llsr_debug_exact_sort(const float* vals, int32_t n, int32_t* out) {
  if (!vals || !out || n < 0 || n > 2048) return LLSR_EINVAL;
  if (n == 0) return LLSR_OK;
  float* dv = nullptr;
  int* di = nullptr;
  if (hipMalloc(&dv, sizeof(float) * n) != hipSuccess) return LLSR_ENODEV;
  if (hipMalloc(&di, sizeof(int) * n) != hipSuccess) { (void)hipFree(dv); return LLSR_ENODEV; }
  int32_t rc = LLSR_OK;
  if (hipMemcpy(dv, vals, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess) rc = LLSR_EIO;
  if (rc == LLSR_OK) {
    k_debug_exact_sort<<<1, 256>>>(dv, n, di, nullptr);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, di, sizeof(int) * n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LLSR_EIO;
  }
  (void)hipFree(dv);
  (void)hipFree(di);
  return rc;
}

// Diagnostics (not part of the ABI header): the PCL-order VoxelGrid's exact sort of 32-bit keys
// (VoxLess32: voxel rank << 11 | position) on n <= 2048 host ranks < 2^21, as k_vox_pcl runs it
// (block_introsort); out[k] = the input position at sorted position k. For
// tests/test_gpu_features_ties.py.
extern "C" int32_t llsr_debug_exact_sort32(const uint32_t* ranks, int32_t n, int32_t* out) {
  if (!ranks || !out || n < 0 || n > 2048) return LLSR_EINVAL;
  for (int32_t t = 0; t < n; ++t)
    if (ranks[t] >= (1u << 21)) return LLSR_EINVAL;
  if (n == 0) return LLSR_OK;
  uint32_t* dv = nullptr;
  int* di = nullptr;
  if (hipMalloc(&dv, sizeof(uint32_t) * n) != hipSuccess) return LLSR_ENODEV;
  if (hipMalloc(&di, sizeof(int) * n) != hipSuccess) { (void)hipFree(dv); return LLSR_ENODEV; }
  int32_t rc = LLSR_OK;
  if (hipMemcpy(dv, ranks, sizeof(uint32_t) * n, hipMemcpyHostToDevice) != hipSuccess) rc = LLSR_EIO;
  if (rc == LLSR_OK) {
    k_debug_exact_sort32<<<1, 256>>>(dv, n, di);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, di, sizeof(int) * n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LLSR_EIO;
  }
  (void)hipFree(dv);
  (void)hipFree(di);
  return rc;
}

// Diagnostics (not part of the ABI header): adjustDistortion's halfPassed test (FA:578-586) as
// k_segment evaluates it, for n (y, x, start) triples: out[3 i] = the certified fast test's code
// (0 fails, 1 passes, 2 undecided), out[3 i + 1] = its decision with the exact fallback, out[3 i + 2] =
// the exact libm test.
extern "C" int32_t llsr_debug_half_passed(const float* yxs, int32_t n, uint8_t* out) {
  if (!yxs || !out || n < 0 || n > (1 << 24)) return LLSR_EINVAL;
  if (n == 0) return LLSR_OK;
  float* dv = nullptr;
  uint8_t* dout = nullptr;
  if (hipMalloc(&dv, sizeof(float) * 3 * (size_t)n) != hipSuccess) return LLSR_ENODEV;
  if (hipMalloc(&dout, 3 * (size_t)n) != hipSuccess) { (void)hipFree(dv); return LLSR_ENODEV; }
  int32_t rc = LLSR_OK;
  if (hipMemcpy(dv, yxs, sizeof(float) * 3 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess) rc = LLSR_EIO;
  if (rc == LLSR_OK) {
    k_debug_half_passed<<<(n + 255) / 256, 256>>>(dv, n, dout);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, dout, 3 * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = LLSR_EIO;
  }
  (void)hipFree(dv);
  (void)hipFree(dout);
  return rc;
}

// Diagnostics (not part of the ABI header): mean device ms of one block_introsort of vals[0, n)
// by one 256-thread workgroup (k_debug_exact_sort), over `reps` launches.
extern "C" float llsr_debug_exact_sort_ms(const float* vals, int32_t n, int32_t reps) {
  if (!vals || n < 1 || n > 2048 || reps < 1) return -1.f;
  float* dv = nullptr;
  int* di = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float ms = -1.f;
  if (hipMalloc(&dv, sizeof(float) * n) == hipSuccess && hipMalloc(&di, sizeof(int) * n) == hipSuccess &&
      hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
      hipMemcpy(dv, vals, sizeof(float) * n, hipMemcpyHostToDevice) == hipSuccess) {
    k_debug_exact_sort<<<1, 256>>>(dv, n, di, nullptr);
    (void)hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; ++r) k_debug_exact_sort<<<1, 256>>>(dv, n, di, nullptr);
    (void)hipEventRecord(e1, nullptr);
    if (hipEventSynchronize(e1) == hipSuccess && hipEventElapsedTime(&ms, e0, e1) == hipSuccess) ms /= reps;
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (dv) (void)hipFree(dv);
  if (di) (void)hipFree(di);
  return ms;
}

// Diagnostics (not part of the ABI header): one block_introsort of vals[0, n) with clock stamps:
// cycles[0] = core clocks of the sort, cycles[1] = the block-wide part, cycles[2 + 4 w + 0..3] =
// wave w's clocks in partitions, small sorts, heap sorts, and waiting at the end (18 values used).
extern "C" int32_t llsr_debug_exact_sort_phases(const float* vals, int32_t n, long long* cycles) {
  if (!vals || !cycles || n < 1 || n > 2048) return LLSR_EINVAL;
  float* dv = nullptr;
  int* di = nullptr;
  long long* dp = nullptr;
  int32_t rc = LLSR_OK;
  if (hipMalloc(&dv, sizeof(float) * n) != hipSuccess || hipMalloc(&di, sizeof(int) * n) != hipSuccess ||
      hipMalloc(&dp, 21 * sizeof(long long)) != hipSuccess || hipMemset(dp, 0, 21 * sizeof(long long)) != hipSuccess)
    rc = LLSR_ENODEV;
  if (rc == LLSR_OK && hipMemcpy(dv, vals, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess) rc = LLSR_EIO;
  if (rc == LLSR_OK) {
    for (int r = 0; r < 3; ++r) k_debug_exact_sort<<<1, 256>>>(dv, n, di, dp);  // warm: the last run counts
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(cycles, dp, 21 * sizeof(long long), hipMemcpyDeviceToHost) != hipSuccess)
      rc = LLSR_EIO;
  }
  if (dv) (void)hipFree(dv);
  if (di) (void)hipFree(di);
  if (dp) (void)hipFree(dp);
  return rc;
}

// After diagnostic launches of the selection stage that stop early: the whole stage once more with
// the handle's configuration, so every ring's less-flat count is final again (k_select_ring leaves
// a pending ring's count negative until the PCL-order VoxelGrid writes it; a later k_fa_concat
// builds its ring offsets from these counts).
static void restore_selection(llsr_handle* h, int B, hipStream_t s) {
  const DevCfg& c = h->dc;
  launch_fa_points(c, h->d, B, s);
  k_select_ring<<<dim3(c.H, B), 256, 0, s>>>(c, h->d);
  if (c.exact_vg) launch_vox_pcl(c, h->d, B, s);
  (void)hipStreamSynchronize(s);
}

// Diagnostics (not part of the ABI header): re-launch kernel k on the last batch's buffers with
// an early exit at `phase`, `reps` times; returns the mean device ms per launch (< 0 on error).
// Used to attribute a kernel's time to its phases; results of such launches are meaningless.
extern "C" float llsr_debug_phase_ms(llsr_handle* h, int32_t k, int32_t phase, int32_t reps) {
  if (!h || h->last_B < 1 || reps < 1) return -1.f;
  if (hipSetDevice(h->device) != hipSuccess) return -1.f;
  hipStream_t s = h->stream;
  DevCfg c = h->dc;
  c.dbg_phase = phase;
  const int B = h->last_B;
  hipEvent_t e0 = h->ev[0][0], e1 = h->ev[0][1];
  if (sync_last(h) != LLSR_OK) return -1.f;
  if (k == 9) {  // k_vox_pcl needs the keys k_select_ring leaves: both re-run before each launch
    float tot = 0.f;
    for (int r = 0; r < reps; ++r) {
      launch_fa_points(h->dc, h->d, B, s);
      k_select_ring<<<dim3(c.H, B), 256, 0, s>>>(h->dc, h->d);
      (void)hipEventRecord(e0, s);
      launch_vox_pcl(c, h->d, B, s);
      (void)hipEventRecord(e1, s);
      float ms = 0.f;
      if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return -1.f;
      tot += ms;
    }
    restore_selection(h, B, s);
    return tot / reps;
  }
  if (k == 8) {
    // k_select_ring consumes the picked / label state k_fa_points leaves (and overwrites it):
    // k_fa_points restores it before every timed launch, so each phase sees the batch's real work
    float tot = 0.f;
    for (int r = 0; r < reps; ++r) {
      launch_fa_points(h->dc, h->d, B, s);
      (void)hipEventRecord(e0, s);
      k_select_ring<<<dim3(c.H, B), 256, 0, s>>>(c, h->d);
      (void)hipEventRecord(e1, s);
      float ms = 0.f;
      if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return -1.f;
      tot += ms;
    }
    restore_selection(h, B, s);
    return tot / reps;
  }
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) {
    switch (k) {
      case 8: k_select_ring<<<dim3(c.H, B), 256, 0, s>>>(c, h->d); break;
      case 10: k_fa_concat<<<B, 256, 0, s>>>(c, h->d); break;
      case 11: k_dbscan_adj<<<dim3(32, B), 256, 0, s>>>(c, h->d, h->d.db_pts); break;
      case 12:
        if (c.HW <= 32768) k_dbscan_merge<1024><<<B, 64, 0, s>>>(c, h->d);
        else k_dbscan_merge<2048><<<B, 64, 0, s>>>(c, h->d);
        break;
      case 7: launch_fa_points(c, h->d, B, s); break;
      case 6: k_segment<<<B, per_scan_threads(c), 0, s>>>(c, h->last_pts, h->last_off, h->d); break;
      case 5:
        if (c.ccl_lds) k_label<true><<<B, 1024, label_lds(c), s>>>(c, h->d);
        else k_label<false><<<B, 1024, label_band_lds(c), s>>>(c, h->d);
        break;
      case 4: k_ground_elev_ransac<<<B, per_scan_threads(c), 0, s>>>(c, h->d); break;
      case 3: k_ground_add<<<dim3((c.H + 3) / 4, B), 256, 0, s>>>(c, h->d); break;
      case 1:
        if (!use_fused(h)) return -2.f;
        k_project_fused<<<B, 1024, fused_lds(c), s>>>(c, h->last_pts, h->last_off, h->d);
        break;
      default: return -2.f;
    }
  }
  (void)hipEventRecord(e1, s);
  if (hipEventSynchronize(e1) != hipSuccess) return -1.f;
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

extern "C" const char* llsr_kernel_name(int32_t k) {
  return (k >= 0 && k < kNumKernels) ? kKernelNames[k] : "";
}

extern "C" int32_t llsr_batch_counts(llsr_handle* h, int32_t* out) {
  if (!h || !out) return LLSR_EINVAL;
  int32_t rc = sync_last(h);
  if (rc) return rc;
  std::vector<int> cnt((size_t)h->last_B * kCnt);
  HIP_OK(h, hipMemcpy(cnt.data(), h->d.counts, cnt.size() * sizeof(int), hipMemcpyDeviceToHost));
  const int idx[8] = {C_NPTS, C_S, C_O, C_M, C_SHARP, C_F, C_L, C_K};
  for (int b = 0; b < h->last_B; ++b)
    for (int q = 0; q < 8; ++q) out[b * 8 + q] = cnt[(size_t)b * kCnt + idx[q]];
  return LLSR_OK;
}

template <class T>
static hipError_t d2h(void* dst, const T* src, size_t n) {
  if (!dst || n == 0) return hipSuccess;
  return hipMemcpy(dst, src, n * sizeof(T), hipMemcpyDeviceToHost);
}

extern "C" int32_t llsr_fetch_scan(llsr_handle* h, int32_t b, llsr_scan_out* o) {
  if (!h || !o) return LLSR_EINVAL;
  if (b < 0 || b >= h->last_B) return fail(h, LLSR_ERANGE, "slot outside last batch");
  int32_t rc = sync_last(h);
  if (rc) return rc;
  const DevCfg& c = h->dc;
  const size_t base = (size_t)b * c.HW;
  int cnt[kCnt];
  HIP_OK(h, d2h(cnt, h->d.counts + b * kCnt, kCnt));
  float ori[4];
  HIP_OK(h, d2h(ori, h->d.orient + b * 4, 4));
  o->n_points = cnt[C_NPTS];
  std::memcpy(o->orientation, ori, sizeof(float) * 3);
  const int S = cnt[C_S], O = cnt[C_O], M = cnt[C_M];
  o->n_segmented = S;
  o->n_outlier = O;
  o->n_near = cnt[C_K];
  o->n_ransac_inliers = cnt[C_INL];
  o->ransac_iterations = cnt[C_RIT];
  o->n_less_sharp = M;
  o->n_sharp = cnt[C_SHARP];
  o->n_flat = cnt[C_F];
  o->n_less_flat = cnt[C_L];
  HIP_OK(h, d2h(o->range_image, h->d.range + base, c.HW));
  HIP_OK(h, d2h(o->cell_point, h->d.cell_pt + base, c.HW));
  HIP_OK(h, d2h(o->ground_image, h->d.ground + base, c.HW));
  HIP_OK(h, d2h(o->label_image, h->d.label + base, c.HW));
  HIP_OK(h, d2h(o->start_ring_index, h->d.start_ring + (size_t)b * c.H, c.H));
  HIP_OK(h, d2h(o->end_ring_index, h->d.end_ring + (size_t)b * c.H, c.H));
  HIP_OK(h, d2h(o->seg_xyzi, (const float*)(h->d.seg + base), 4 * (size_t)S));
  HIP_OK(h, d2h(o->seg_ground_flag, h->d.seg_ground + base, S));
  HIP_OK(h, d2h(o->seg_col_ind, h->d.seg_col + base, S));
  HIP_OK(h, d2h(o->seg_range, h->d.seg_range + base, S));
  HIP_OK(h, d2h(o->seg_intensity, h->d.seg_int + base, S));
  HIP_OK(h, d2h(o->outlier_xyzi, (const float*)(h->d.outl + base), 4 * (size_t)O));
  HIP_OK(h, d2h(o->outlier_intensity, h->d.outl_int + base, O));
  HIP_OK(h, d2h(o->loam_xyzi, (const float*)(h->d.loam + base), 4 * (size_t)S));
  HIP_OK(h, d2h(o->curvature, h->d.curv + base, S));
  HIP_OK(h, d2h(o->picked, h->d.picked + base, S));
  HIP_OK(h, d2h(o->label, h->d.clabel + base, S));
  HIP_OK(h, d2h(o->less_sharp_ind, h->d.less_sharp + base, M));
  HIP_OK(h, d2h(o->dbscan_cluster, h->d.cluster + base, M));
  HIP_OK(h, d2h(o->sharp_ind, h->d.sharp + base, o->n_sharp));
  HIP_OK(h, d2h(o->flat_ind, h->d.flat + base, o->n_flat));
  HIP_OK(h, d2h(o->less_flat_xyzi, (const float*)(h->d.lflat + base), 4 * (size_t)o->n_less_flat));
  return LLSR_OK;
}

extern "C" int32_t llsr_fetch_vis_clouds(llsr_handle* h, int32_t b, llsr_vis_out* o) {
  if (!h || !o) return LLSR_EINVAL;
  if (b < 0 || b >= h->last_B) return fail(h, LLSR_ERANGE, "slot outside last batch");
  int32_t rc = sync_last(h);
  if (rc) return rc;
  const DevCfg& c = h->dc;
  const size_t HW = (size_t)c.HW;
  if (!h->d_vis) HIP_OK(h, hipMalloc(&h->d_vis, sizeof(float4) * (6 * HW + 1)));
  int* d_cnt = reinterpret_cast<int*>(h->d_vis + 6 * HW);
  k_vis_clouds<<<1, 1024, 0, h->stream>>>(c, h->d, b, h->d_vis, d_cnt);
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipStreamSynchronize(h->stream));
  int cnt[4];
  HIP_OK(h, d2h(cnt, d_cnt, 4));
  o->n_ground = cnt[0];
  o->n_nonground = cnt[1];
  o->n_unknownground = cnt[2];
  o->n_segmented_pure = cnt[3];
  float* dst[6] = {o->full_cloud, o->full_info_cloud, o->ground_cloud, o->nonground_cloud, o->unknownground_cloud,
                   o->segmented_cloud_pure};
  const size_t n[6] = {HW, HW, (size_t)cnt[0], (size_t)cnt[1], (size_t)cnt[2], (size_t)cnt[3]};
  for (int k = 0; k < 6; ++k)
    if (dst[k] && n[k]) HIP_OK(h, d2h(dst[k], (const float*)(h->d_vis + k * HW), 4 * n[k]));
  return LLSR_OK;
}

extern "C" int32_t llsr_process_scan(llsr_handle* h, const float* xyzi, int32_t n, llsr_scan_out* out) {
  if (!h || !out || n < 0 || (n > 0 && !xyzi)) return fail(h, LLSR_EINVAL, "bad argument");
  if (n > h->max_points) return fail(h, LLSR_ERANGE, "scan larger than max_points");
  HIP_OK(h, hipSetDevice(h->device));
  const int64_t off[2] = {0, n};
  HIP_OK(h, hipStreamSynchronize(h->stream));
  if (n > 0) HIP_OK(h, hipMemcpy(h->d_in, xyzi, sizeof(float4) * (size_t)n, hipMemcpyHostToDevice));
  HIP_OK(h, hipMemcpy(h->d_off, off, sizeof off, hipMemcpyHostToDevice));
  int32_t rc = llsr_process_batch(h, (const float*)h->d_in, h->d_off, 1, h->stream);
  if (rc) return rc;
  return llsr_fetch_scan(h, 0, out);
}

// ---------------------------------------------------------------------------------------------
// Scan-to-map (MapOptimization::scan2MapOptimization, MO:1572-1610): see llsr_mo.hip.

extern "C" int32_t llsr_scan2map_reserve(llsr_handle* h, int32_t P, int32_t mc, int32_t ms, int32_t qc,
                                         int32_t qs) {
  if (!h) return LLSR_EINVAL;
  if (P < 1 || mc < 0 || ms < 0 || qc < 0 || qs < 0 || mc > (1 << 26) || ms > (1 << 26) ||
      qc > (1 << 20) || qs > (1 << 20))  // the solving block keeps the per-block row prefix in LDS
    return fail(h, LLSR_EINVAL, "scan2map capacities out of range");
  HIP_OK(h, hipSetDevice(h->device));
  auto& m = h->mo;
  if (m.pool && P <= m.P && mc <= m.mc && ms <= m.ms && qc <= m.qc && qs <= m.qs) return LLSR_OK;
  if (m.pool) {
    HIP_OK(h, sync_handle_streams(h));
    HIP_OK(h, hipFree(m.pool));
    m.pool = nullptr;
  }
  m.sh_live = false;
  m.P = P; m.mc = mc; m.ms = ms; m.qc = qc; m.qs = qs;
  m.log2T_c = grid_log2_table(mc);
  m.log2T_s = grid_log2_table(ms);
  m.blocks_c = (qc + 255) / 256;
  m.blocks = m.blocks_c + (qs + 255) / 256;
  if (m.blocks == 0) m.blocks = 1;  // one (empty) block still runs each iteration's solve
  const size_t Tc = (size_t)1 << m.log2T_c, Ts = (size_t)1 << m.log2T_s;
  // Eigen's GEMM depth blocks of up to qc + qs rows: kc >= 344 once k exceeds max_kc = 680
  // (llsr_eigen::gemm_kc), so at most ceil(N / 344) blocks; k_s2m_solve keeps 64 in LDS
  const long long n_rows = (long long)qc + qs;
  const int spill_cap = std::max(0, (int)((n_rows + 343) / 344) - 64);
  const size_t bytes = sizeof(S2MProb) * P + sizeof(CellSlot) * P * (Tc + Ts) +
                       sizeof(float4) * P * ((size_t)mc + ms) + sizeof(int2) * P * ((size_t)mc + ms) +
                       sizeof(int) * 2 * P +
                       sizeof(float4) * 2 * 256 * (size_t)P * m.blocks + sizeof(int) * (size_t)P * m.blocks +
                       sizeof(float) * 29 * (size_t)P * spill_cap + 4096 + 11 * 256;
  if (hipMalloc(&m.pool, bytes) != hipSuccess) {
    m.pool = nullptr;
    m.P = 0;
    return fail(h, LLSR_ENOMEM, "scan2map buffers");
  }
  char* q = (char*)m.pool;
  S2MArgs& a = m.a;
  a = S2MArgs{};
  a.prob = carve<S2MProb>(q, P);
  CellGrid& gc = a.grids.g[0];
  CellGrid& gs = a.grids.g[1];
  gc.tab = carve<CellSlot>(q, P * Tc);
  gs.tab = carve<CellSlot>(q, P * Ts);
  gc.sorted = carve<float4>(q, (size_t)P * mc);
  gs.sorted = carve<float4>(q, (size_t)P * ms);
  gc.where = carve<int2>(q, (size_t)P * mc);
  gs.where = carve<int2>(q, (size_t)P * ms);
  gc.cursor = carve<int>(q, (size_t)P);
  gs.cursor = carve<int>(q, (size_t)P);
  gc.cap = mc; gs.cap = ms;
  gc.log2T = m.log2T_c; gs.log2T = m.log2T_s;
  a.rows = carve<float4>(q, 2 * 256 * (size_t)P * m.blocks);
  a.solve_rows = (kSolveLds - 4 * ((m.blocks + 4) & ~3)) / 32;
  if (a.solve_rows < 256)
    return fail(h, LLSR_EINVAL, "scan2map: too many query blocks for the solve kernel's LDS");
  if (hipFuncSetAttribute((const void*)k_s2m_solve, hipFuncAttributeMaxDynamicSharedMemorySize, kSolveLds) !=
      hipSuccess)
    return fail(h, LLSR_ENODEV, "k_s2m_solve LDS attribute");
  a.bcnt = carve<int>(q, (size_t)P * m.blocks);
  a.blk_spill = carve<float>(q, 29 * (size_t)P * spill_cap);
  a.spill_cap = spill_cap;
  a.n_active = carve<int>(q, 2);
  a.error = a.n_active + 1;
  a.cap_qc = qc; a.cap_qs = qs; a.cap_mc = mc; a.cap_ms = ms;
  a.blocks_c = m.blocks_c;
  a.blocks = m.blocks;
  if (!m.host_flags && hipHostMalloc((void**)&m.host_flags, 2 * sizeof(int)) != hipSuccess) {
    m.host_flags = nullptr;
    return fail(h, LLSR_ENOMEM, "pinned flags");
  }
  if (!m.e0 && (hipEventCreate(&m.e0) != hipSuccess || hipEventCreate(&m.e1) != hipSuccess ||
                 hipEventCreate(&m.p0) != hipSuccess || hipEventCreate(&m.p1) != hipSuccess ||
                 hipEventCreate(&m.p2) != hipSuccess))
    return fail(h, LLSR_ENODEV, "events");
  return LLSR_OK;
}

// Options of the internal scan-to-map entry (the mapping chain): the MO mode and the optimiser's
// cross-frame members; the public entries use the handle's mode and a fresh optimiser.
struct S2MOpts {
  int mode = -1;  // -1: h->cfg.mode
  const int* deg_in = nullptr;
  const float* matP_in = nullptr;
  int* deg_out = nullptr;
  float* matP_out = nullptr;
};

// Validate a scan-to-map batch and enqueue the per-problem setup and both cell-grid builds.
static int32_t s2m_prepare(llsr_handle* h, const llsr_s2m_batch* b, hipStream_t s, S2MArgs& a,
                           const S2MOpts& opt = S2MOpts{}) {
  auto& m = h->mo;
  if (!m.pool) return fail(h, LLSR_EINVAL, "llsr_scan2map_reserve not called");
  const int P = b->n_problems;
  if (P < 1 || P > m.P) return fail(h, LLSR_ERANGE, "n_problems outside [1, reserved]");
  if (!b->corner_q_off || !b->surf_q_off || !b->corner_map_off || !b->surf_map_off || !b->pose || !b->report)
    return fail(h, LLSR_EINVAL, "null batch array");
  a = m.a;
  a.P = P;
  a.applied = (opt.mode >= 0 ? opt.mode : h->cfg.mode) == LLSR_MODE_LM_APPLIED;
  a.deg_in = opt.deg_in; a.matP_in = opt.matP_in;
  a.deg_out = opt.deg_out; a.matP_out = opt.matP_out;
  a.iter_max = h->cfg.iterCountThres;
#ifdef LLSR_S2S_PROF
  {  // diagnostics build only: k_s2m_solve stops after stage LLSR_S2M_DBG (scripts/)
    const char* dbg = std::getenv("LLSR_S2M_DBG");
    a.dbg = dbg ? std::atoi(dbg) : 0;
  }
#else
  a.dbg = 0;
#endif
  a.step_size = h->cfg.step_size;
  a.stop_thres = h->cfg.stop_thres;
  a.cq = b->corner_q; a.cq_off = b->corner_q_off;
  a.sq = b->surf_q; a.sq_off = b->surf_q_off;
  a.cm = b->corner_map; a.cm_off = b->corner_map_off;
  a.sm = b->surf_map; a.sm_off = b->surf_map_off;
  a.pose = b->pose;
  a.report = b->report;
  a.rank = 0;
  a.world = 1;
  a.ne = nullptr;
  HIP_OK(h, hipMemsetAsync(a.n_active, 0, 2 * sizeof(int), s));
  a.grids.P = P;
  a.grids.g[0].src = reinterpret_cast<const float4*>(b->corner_map);
  a.grids.g[0].off = b->corner_map_off;
  a.grids.g[1].src = reinterpret_cast<const float4*>(b->surf_map);
  a.grids.g[1].off = b->surf_map_off;
  k_s2m_setup<<<(P + 63) / 64, 64, 0, s>>>(a);
  grid_build(a.grids, s);
  HIP_OK(h, hipGetLastError());
  return LLSR_OK;
}

static int32_t s2m_batch(llsr_handle* h, const llsr_s2m_batch* b, hipStream_t s, const S2MOpts& opt) {
  auto& m = h->mo;
  if (h->profiling && m.pool) HIP_OK(h, hipEventRecord(m.p0, s));
  S2MArgs a{};
  m.sh_live = false;  // one scan-to-map batch per handle at a time: this one replaces a shard batch
  // the scan-to-map buffers are the handle's: start after its previous scan-to-map work (any stream)
  if (h->mo_rec) HIP_OK(h, hipStreamWaitEvent(s, h->mo_done, 0));
  int32_t rc = s2m_prepare(h, b, s, a, opt);
  h->mo_rec = true;
  HIP_OK(h, hipEventRecord(h->mo_done, s));
  if (rc != LLSR_OK) return rc;
  const int P = a.P;
  if (h->profiling) HIP_OK(h, hipEventRecord(m.p1, s));
  // LM iterations; the host reads the active count every `poll` launch pairs (converged problems
  // leave their workgroups at the first instruction, so launches past convergence cost little):
  // 4 for lm_applied's few iterations, 16 for faithful's 200 (13 host round trips instead of 50)
  const int poll = a.iter_max >= 64 ? 16 : 4;
  int launches = 0;
  for (int it = 0; it < a.iter_max;) {
    const int n = (a.iter_max - it) < poll ? (a.iter_max - it) : poll;
    for (int k = 0; k < n; ++k) {
      k_s2m_iter<<<8 * ((P + 7) / 8) * m.blocks, 256, 0, s>>>(a);  // XCD-aware (llsr_mo.hip)
      k_s2m_solve<<<P, 256, kSolveLds, s>>>(a);
    }
    it += n;
    launches += n;
    HIP_OK(h, hipGetLastError());
    HIP_OK(h, hipMemcpyAsync(m.host_flags, a.n_active, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_OK(h, hipStreamSynchronize(s));
    if (m.host_flags[1]) return fail(h, LLSR_ERANGE, "a scan2map cloud exceeds the reserved capacity or has bad offsets");
    if (m.host_flags[0] == 0) break;
  }
  if (h->profiling) HIP_OK(h, hipEventRecord(m.p2, s));
  k_s2m_finish<<<(P + 63) / 64, 64, 0, s>>>(a);
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipEventRecord(h->mo_done, s));
  if (h->profiling) {
    float g = 0.f, it = 0.f;
    HIP_OK(h, hipEventSynchronize(m.p2));
    HIP_OK(h, hipEventElapsedTime(&g, m.p0, m.p1));
    HIP_OK(h, hipEventElapsedTime(&it, m.p1, m.p2));
    m.stats.batches += 1;
    m.stats.iteration_launches += launches;
    m.stats.grid_ms += g;
    m.stats.iterate_ms += it;
  }
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2map_batch(llsr_handle* h, const llsr_s2m_batch* b, void* hip_stream) {
  if (!h || !b) return fail(h, LLSR_EINVAL, "null argument");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  return s2m_batch(h, b, s, S2MOpts{});
}

// ---- split-correspondence scan-to-map (llsr_scan2map_shard_*): the LM loop is the caller's,
// so the per-problem normal equations can be all-reduced across GPUs between the Jacobian build
// (llsr_scan2map_shard_partial) and the solve (llsr_scan2map_shard_step).

extern "C" int32_t llsr_scan2map_shard_begin(llsr_handle* h, const llsr_s2m_batch* b, void* hip_stream) {
  if (!h || !b) return fail(h, LLSR_EINVAL, "null argument");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  auto& m = h->mo;
  m.sh_live = false;
  if (h->mo_rec) HIP_OK(h, hipStreamWaitEvent(s, h->mo_done, 0));
  int32_t rc = s2m_prepare(h, b, s, m.sh);
  h->mo_rec = true;
  HIP_OK(h, hipEventRecord(h->mo_done, s));
  if (rc != LLSR_OK) return rc;
  m.sh_live = true;
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2map_shard_partial(llsr_handle* h, int32_t rank, int32_t world, int64_t* d_ne,
                                               void* hip_stream) {
  if (!h || !d_ne) return fail(h, LLSR_EINVAL, "null argument");
  auto& m = h->mo;
  if (!m.sh_live) return fail(h, LLSR_EINVAL, "llsr_scan2map_shard_begin not called");
  if (world < 1 || rank < 0 || rank >= world) return fail(h, LLSR_EINVAL, "rank outside [0, world)");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  S2MArgs a = m.sh;
  a.rank = rank;
  a.world = world;
  a.ne = reinterpret_cast<long long*>(d_ne);
  HIP_OK(h, hipStreamWaitEvent(s, h->mo_done, 0));
  HIP_OK(h, hipMemsetAsync(d_ne, 0, sizeof(int64_t) * LLSR_NE_WORDS * (size_t)a.P, s));
  const int bs = m.blocks - m.blocks_c;
  const int nb = (m.blocks_c + world - 1) / world + (bs + world - 1) / world;
  if (nb > 0) k_s2m_iter_fx<<<8 * ((a.P + 7) / 8) * nb, 256, 0, s>>>(a, nb);  // XCD-aware (llsr_mo.hip)
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipEventRecord(h->mo_done, s));
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2map_shard_step(llsr_handle* h, const int64_t* d_ne, int32_t* n_active,
                                            void* hip_stream) {
  if (!h || !d_ne) return fail(h, LLSR_EINVAL, "null argument");
  auto& m = h->mo;
  if (!m.sh_live) return fail(h, LLSR_EINVAL, "llsr_scan2map_shard_begin not called");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  S2MArgs a = m.sh;
  a.ne = const_cast<long long*>(reinterpret_cast<const long long*>(d_ne));
  HIP_OK(h, hipStreamWaitEvent(s, h->mo_done, 0));
  k_s2m_solve_fx<<<(a.P + 63) / 64, 64, 0, s>>>(a);
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipEventRecord(h->mo_done, s));
  if (n_active) {
    HIP_OK(h, hipMemcpyAsync(m.host_flags, a.n_active, 2 * sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_OK(h, hipStreamSynchronize(s));
    if (m.host_flags[1] & 1) return fail(h, LLSR_ERANGE, "a scan2map cloud exceeds the reserved capacity or has bad offsets");
    if (m.host_flags[1] & 2)
      return fail(h, LLSR_ERANGE, "a normal-equation term is non-finite or outside the fixed-point range (|v| >= 2^32)");
    *n_active = m.host_flags[0];
  }
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2map_shard_end(llsr_handle* h, void* hip_stream) {
  if (!h) return LLSR_EINVAL;
  auto& m = h->mo;
  if (!m.sh_live) return fail(h, LLSR_EINVAL, "llsr_scan2map_shard_begin not called");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  HIP_OK(h, hipStreamWaitEvent(s, h->mo_done, 0));
  k_s2m_finish<<<(m.sh.P + 63) / 64, 64, 0, s>>>(m.sh);
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipEventRecord(h->mo_done, s));
  m.sh_live = false;
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2map_stats(llsr_handle* h, llsr_s2m_stats* out) {
  if (!h || !out) return LLSR_EINVAL;
  *out = h->mo.stats;
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2map(llsr_handle* h, const float* cq, int32_t Qc, const float* sq, int32_t Qs,
                                 const float* cm, int32_t Mc, const float* sm, int32_t Ms, float* pose,
                                 llsr_lm_report* rep) {
  if (!h || !pose || !rep || Qc < 0 || Qs < 0 || Mc < 0 || Ms < 0) return fail(h, LLSR_EINVAL, "bad argument");
  if ((Qc && !cq) || (Qs && !sq) || (Mc && !cm) || (Ms && !sm)) return fail(h, LLSR_EINVAL, "null cloud");
  auto& m = h->mo;
  const int P = m.pool ? m.P : 1;
  int32_t rc = llsr_scan2map_reserve(h, P, Mc > m.mc ? Mc : m.mc, Ms > m.ms ? Ms : m.ms,
                                     Qc > m.qc ? Qc : m.qc, Qs > m.qs ? Qs : m.qs);
  if (rc != LLSR_OK) return rc;
  const size_t npts = (size_t)Qc + Qs + Mc + Ms;
  const size_t need = sizeof(float4) * npts + 8 * sizeof(int64_t) + 6 * sizeof(float) + sizeof(llsr_lm_report) +
                      8 * 256;  // carve() pads each of the 7 pieces to 256 B
  if (need > m.stage_bytes) {
    if (m.stage) HIP_OK(h, hipFree(m.stage));
    m.stage = nullptr;
    if (hipMalloc(&m.stage, need) != hipSuccess) { m.stage_bytes = 0; return fail(h, LLSR_ENOMEM, "staging"); }
    m.stage_bytes = need;
  }
  char* q = (char*)m.stage;
  float4* d_cq = carve<float4>(q, Qc);
  float4* d_sq = carve<float4>(q, Qs);
  float4* d_cm = carve<float4>(q, Mc);
  float4* d_sm = carve<float4>(q, Ms);
  int64_t* d_off = carve<int64_t>(q, 8);
  float* d_pose = carve<float>(q, 6);
  llsr_lm_report* d_rep = carve<llsr_lm_report>(q, 1);
  hipStream_t s = h->stream;
  HIP_OK(h, hipSetDevice(h->device));
  if (Qc) HIP_OK(h, hipMemcpyAsync(d_cq, cq, sizeof(float4) * Qc, hipMemcpyHostToDevice, s));
  if (Qs) HIP_OK(h, hipMemcpyAsync(d_sq, sq, sizeof(float4) * Qs, hipMemcpyHostToDevice, s));
  if (Mc) HIP_OK(h, hipMemcpyAsync(d_cm, cm, sizeof(float4) * Mc, hipMemcpyHostToDevice, s));
  if (Ms) HIP_OK(h, hipMemcpyAsync(d_sm, sm, sizeof(float4) * Ms, hipMemcpyHostToDevice, s));
  const int64_t offs[8] = {0, Qc, 0, Qs, 0, Mc, 0, Ms};
  HIP_OK(h, hipMemcpyAsync(d_off, offs, sizeof offs, hipMemcpyHostToDevice, s));
  HIP_OK(h, hipMemcpyAsync(d_pose, pose, 6 * sizeof(float), hipMemcpyHostToDevice, s));
  llsr_s2m_batch b{};
  b.n_problems = 1;
  b.corner_q = (const float*)d_cq; b.corner_q_off = d_off;
  b.surf_q = (const float*)d_sq; b.surf_q_off = d_off + 2;
  b.corner_map = (const float*)d_cm; b.corner_map_off = d_off + 4;
  b.surf_map = (const float*)d_sm; b.surf_map_off = d_off + 6;
  b.pose = d_pose;
  b.report = d_rep;
  HIP_OK(h, hipEventRecord(m.e0, s));
  rc = llsr_scan2map_batch(h, &b, s);
  if (rc != LLSR_OK) return rc;
  HIP_OK(h, hipEventRecord(m.e1, s));
  HIP_OK(h, hipMemcpyAsync(rep, d_rep, sizeof *rep, hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipMemcpyAsync(pose, d_pose, 6 * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipStreamSynchronize(s));
  float ms_ = 0.f;
  HIP_OK(h, hipEventElapsedTime(&ms_, m.e0, m.e1));
  rep->ms = ms_;
  return LLSR_OK;
}

// ---------------------------------------------------------------------------------------------
// Scan-to-scan (FeatureAssociation::updateTransformation, FA:2505-2535): see llsr_fa_lm.hip.

extern "C" int32_t llsr_shadow_points(float* out) {
  // GenerateShadowPoint (FA:412-439) with lidar_to_body_centor = (0.008, 0, -0.035) (FA:300),
  // row_size 16, col_size 10 (FA:301); computed on the host with the same libm as the reference.
  if (!out) return LLSR_EINVAL;
  const double c0 = 0.008, c1 = 0.0, c2 = -0.035;
  const int row_size = 16, col_size = 10;
  const double row_angle = (std::atan2(0.120, 0.05) * 2) / (row_size - 1);
  const double col_angle = (std::atan2(0.077, 0.05) * 2) / (col_size - 1);
  int k = 0;
  for (int row = 0; row < row_size; row++) {
    const float row_x = (float)(0.05 * std::tan((((row_size - 1.0) / 2.0) * row_angle) - (row * row_angle)));
    for (int col = 0; col < col_size; col++) {
      const float col_y = (float)(0.05 * std::tan((((col_size - 1.0) / 2.0) * col_angle) - (col * col_angle)));
      out[4 * k + 0] = (float)(col_y + c1);
      out[4 * k + 1] = (float)(-(0.035f + 0.05f) + c2);
      out[4 * k + 2] = (float)(row_x + c0);
      out[4 * k + 3] = (float)((double)((float)row + (float)17) + (double)(float)col / 10000.0);
      ++k;
    }
  }
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2scan_reserve(llsr_handle* h, int32_t P, int32_t ms, int32_t f, int32_t nc, int32_t ns) {
  if (!h) return LLSR_EINVAL;
  if (P < 1 || ms < 0 || f < 0 || nc < 0 || ns < 0 || ms > (1 << 24) || f > (1 << 24) || nc > (1 << 24) || ns > (1 << 24))
    return fail(h, LLSR_EINVAL, "scan2scan capacities out of range");
  HIP_OK(h, hipSetDevice(h->device));
  auto& m = h->s2s;
  if (m.pool && P <= m.P && ms <= m.ms && f <= m.f && nc <= m.nc && ns <= m.ns) return LLSR_OK;
  if (m.pool) {
    HIP_OK(h, sync_handle_streams(h));
    HIP_OK(h, hipFree(m.pool));
    m.pool = nullptr;
  }
  m.P = P; m.ms = ms; m.f = f; m.nc = nc; m.ns = ns;
  const int lc = grid_log2_table(nc), ls = grid_log2_table(ns);
  const size_t Tc = (size_t)1 << lc, Ts = (size_t)1 << ls;
  const size_t capq = (size_t)(ms > f ? ms : f) + 1;
  const size_t bytes = sizeof(CellSlot) * P * (Tc + Ts) + (sizeof(float4) + sizeof(int2)) * P * ((size_t)nc + ns) +
                       sizeof(int) * 2 * P + (5 * sizeof(int) + sizeof(float4) + 1) * P * capq +
                       sizeof(float4) * 2 * P * (((size_t)ns + 7) / 8 + ((size_t)ns + 63) / 64) +
                       sizeof(float) * 8 * P + 64 + 16 * 256;
  if (hipMalloc(&m.pool, bytes) != hipSuccess) {
    m.pool = nullptr;
    m.P = 0;
    return fail(h, LLSR_ENOMEM, "scan2scan buffers");
  }
  char* q = (char*)m.pool;
  S2SArgs& a = m.a;
  a = S2SArgs{};
  CellGrid& gc = a.grids.g[0];
  CellGrid& gs = a.grids.g[1];
  gc.tab = carve<CellSlot>(q, P * Tc);
  gs.tab = carve<CellSlot>(q, P * Ts);
  gc.sorted = carve<float4>(q, (size_t)P * nc);
  gs.sorted = carve<float4>(q, (size_t)P * ns);
  gc.where = carve<int2>(q, (size_t)P * nc);
  gs.where = carve<int2>(q, (size_t)P * ns);
  gc.cursor = carve<int>(q, (size_t)P);
  gs.cursor = carve<int>(q, (size_t)P);
  gc.cap = nc; gs.cap = ns;
  gc.log2T = lc; gs.log2T = ls;
  a.idx = carve<int>(q, 5 * (size_t)P * capq);  // kIx ints per query (llsr_fa_lm.hip)
  a.rows = carve<float4>(q, (size_t)P * capq);
  a.valid = carve<uint8_t>(q, (size_t)P * capq);
  a.error = carve<int>(q, 1);
  a.sbox = carve<float4>(q, 2 * (size_t)P * (((size_t)ns + 7) / 8));
  a.sbox2 = carve<float4>(q, 2 * (size_t)P * (((size_t)ns + 63) / 64));
  a.prof = carve<float>(q, 8 * (size_t)P);

  a.cap_sharp = ms;
  a.cap_flat = f;
  if (!m.host_flag && hipHostMalloc((void**)&m.host_flag, sizeof(int)) != hipSuccess) {
    m.host_flag = nullptr;
    return fail(h, LLSR_ENOMEM, "pinned flag");
  }
  if (!m.e0 && (hipEventCreate(&m.e0) != hipSuccess || hipEventCreate(&m.e1) != hipSuccess))
    return fail(h, LLSR_ENODEV, "events");
  HIP_OK(h, hipMemset(a.error, 0, sizeof(int)));
  return LLSR_OK;
}

// hint_q / hint_nc: this launch's largest query count and corner-last cloud when the caller knows
// them (the odometry chain), else 0 = the reserved capacities; they pick the LM instantiation only
static int32_t s2s_launch(llsr_handle* h, const llsr_s2s_batch* b, void* hip_stream, int hint_q, int hint_nc) {
  if (!h || !b) return fail(h, LLSR_EINVAL, "null argument");
  auto& m = h->s2s;
  if (!m.pool) return fail(h, LLSR_EINVAL, "llsr_scan2scan_reserve not called");
  const int P = b->n_problems;
  if (P < 1 || P > m.P) return fail(h, LLSR_ERANGE, "n_problems outside [1, reserved]");
  if (!b->sharp_off || !b->flat_off || !b->corner_last_off || !b->surf_last_off || !b->transform_cur ||
      !b->is_degenerate || !b->report)
    return fail(h, LLSR_EINVAL, "null batch array");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  S2SArgs a = m.a;
  a.P = P;
  a.dist_sqr = h->cfg.nearest_feature_search_distance * h->cfg.nearest_feature_search_distance;  // FA:152
  a.sharp = reinterpret_cast<const float4*>(b->sharp); a.sharp_off = b->sharp_off;
  a.flat = reinterpret_cast<const float4*>(b->flat); a.flat_off = b->flat_off;
  a.grids.P = P;
  a.grids.g[0].src = reinterpret_cast<const float4*>(b->corner_last);
  a.grids.g[0].off = b->corner_last_off;
  a.grids.g[1].src = reinterpret_cast<const float4*>(b->surf_last);
  a.grids.g[1].off = b->surf_last_off;
  a.tcur = b->transform_cur;
  a.degen = b->is_degenerate;
  a.report = b->report;
  if (h->profiling && !m.p0 &&
      (hipEventCreate(&m.p0) != hipSuccess || hipEventCreate(&m.p1) != hipSuccess || hipEventCreate(&m.p2) != hipSuccess))
    return fail(h, LLSR_ENODEV, "events");
  if (h->s2s_rec) HIP_OK(h, hipStreamWaitEvent(s, h->s2s_done, 0));  // shared buffers: after the last batch
  if (h->profiling) HIP_OK(h, hipEventRecord(m.p0, s));
  grid_build(a.grids, s);
  {
    const int nb = (m.ns + 7) / 8;
    if (nb > 0) k_s2s_boxes<<<dim3((nb + 255) / 256, P), 256, 0, s>>>(a);
  }
  if (h->profiling) HIP_OK(h, hipEventRecord(m.p1, s));
  // the small-LDS instantiation (4 workgroups per CU instead of 2) when every problem's queries
  // and corner-last cloud fit it (reserved capacities are the batch maxima)
  // bounds: this launch's largest clouds when the caller knows them (the odometry chain), else
  // the reserved capacities
  const int bq = hint_q > 0 ? hint_q : std::max(m.ms, m.f);
  const int bnc = hint_nc > 0 ? hint_nc : m.nc;
  if (bq <= 1024 && bnc <= 1024) {
    s2s_lm_launch<1024, 1024, 256>(P, s, a);
    m.last_variant = 1024;
  } else if (bq <= 2560 && bnc <= 1536) {
    s2s_lm_launch<2560, 1536, 512>(P, s, a);
    m.last_variant = 2560;
  } else {
    s2s_lm_launch<2048, 2048, 512>(P, s, a);
    m.last_variant = 2048;
  }
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipEventRecord(h->s2s_done, s));
  h->s2s_rec = true;
  if (h->profiling) {
    float g = 0.f, lm = 0.f;
    HIP_OK(h, hipEventRecord(m.p2, s));
    HIP_OK(h, hipEventSynchronize(m.p2));
    HIP_OK(h, hipEventElapsedTime(&g, m.p0, m.p1));
    HIP_OK(h, hipEventElapsedTime(&lm, m.p1, m.p2));
    m.stats.batches += 1;
    m.stats.grid_ms += g;
    m.stats.lm_ms += lm;
  }
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2scan_batch(llsr_handle* h, const llsr_s2s_batch* b, void* hip_stream) {
  return s2s_launch(h, b, hip_stream, 0, 0);
}

// Diagnostics (not part of the ABI header): the LDS rows (1024, 2560 or 2048) of the k_s2s_lm
// instantiation the last scan-to-scan launch of this handle used, 0 before any; the two large ones
// run the whole-wave surf walks (tests/test_gpu_fa_lm.py asserts which one a test exercised).
extern "C" int32_t llsr_debug_s2s_variant(llsr_handle* h) { return h ? h->s2s.last_variant : -1; }

// Diagnostics (not part of the ABI header): the diagnostics build's per-problem phase ticks of the
// last scan-to-scan launch (k_s2s_lm, LLSR_S2S_PROF: knn surf / corner, A rows, B sums, C solve,
// corner / surf walks, whole kernel, 100 MHz; [7] the shell fallback queries), [P][8] into out.
// Synchronises. The product build leaves the buffer unwritten.
extern "C" int32_t llsr_debug_s2s_prof(llsr_handle* h, float* out, int32_t cap) {
  if (!h || !out || cap < 0) return LLSR_EINVAL;
  auto& m = h->s2s;
  if (!m.pool) return fail(h, LLSR_EINVAL, "no scan-to-scan batch");
  HIP_OK(h, hipSetDevice(h->device));
  HIP_OK(h, sync_handle_streams(h));
  const int n = cap < m.P ? cap : m.P;
  HIP_OK(h, hipMemcpy(out, m.a.prof, sizeof(float) * 8 * (size_t)n, hipMemcpyDeviceToHost));
  return n;
}

extern "C" int32_t llsr_scan2scan_stats(llsr_handle* h, llsr_s2s_stats* out) {
  if (!h || !out) return LLSR_EINVAL;
  *out = h->s2s.stats;
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2scan_check(llsr_handle* h) {
  if (!h) return LLSR_EINVAL;
  auto& m = h->s2s;
  if (!m.pool) return LLSR_OK;
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = h->stream;  // the handle's stream, after the last scan-to-scan batch
  if (h->s2s_rec) HIP_OK(h, hipStreamWaitEvent(s, h->s2s_done, 0));
  HIP_OK(h, hipMemcpyAsync(m.host_flag, m.a.error, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipStreamSynchronize(s));
  if (*m.host_flag) {
    HIP_OK(h, hipMemsetAsync(m.a.error, 0, sizeof(int), s));
    HIP_OK(h, hipStreamSynchronize(s));
    return fail(h, LLSR_ERANGE, "a scan2scan cloud exceeds the reserved capacity or has bad offsets");
  }
  return LLSR_OK;
}

extern "C" int32_t llsr_scan2scan(llsr_handle* h, const float* sharp, int32_t Ms, const float* flat, int32_t F,
                                  const float* cl, int32_t Nc, const float* sl, int32_t Ns, float* tcur,
                                  int32_t* degen, llsr_s2s_report* rep) {
  if (!h || !tcur || !degen || !rep || Ms < 0 || F < 0 || Nc < 0 || Ns < 0) return fail(h, LLSR_EINVAL, "bad argument");
  if ((Ms && !sharp) || (F && !flat) || (Nc && !cl) || (Ns && !sl)) return fail(h, LLSR_EINVAL, "null cloud");
  auto& m = h->s2s;
  const int P = m.pool ? m.P : 1;
  int32_t rc = llsr_scan2scan_reserve(h, P, Ms > m.ms ? Ms : m.ms, F > m.f ? F : m.f, Nc > m.nc ? Nc : m.nc,
                                      Ns > m.ns ? Ns : m.ns);
  if (rc != LLSR_OK) return rc;
  const size_t npts = (size_t)Ms + F + Nc + Ns;
  const size_t need = sizeof(float4) * npts + 8 * sizeof(int64_t) + 6 * sizeof(float) + sizeof(int) +
                      sizeof(llsr_s2s_report) + 9 * 256;
  if (need > m.stage_bytes) {
    if (m.stage) HIP_OK(h, hipFree(m.stage));
    m.stage = nullptr;
    if (hipMalloc(&m.stage, need) != hipSuccess) { m.stage_bytes = 0; return fail(h, LLSR_ENOMEM, "staging"); }
    m.stage_bytes = need;
  }
  char* q = (char*)m.stage;
  float4* d_sh = carve<float4>(q, Ms);
  float4* d_fl = carve<float4>(q, F);
  float4* d_cl = carve<float4>(q, Nc);
  float4* d_sl = carve<float4>(q, Ns);
  int64_t* d_off = carve<int64_t>(q, 8);
  float* d_t = carve<float>(q, 6);
  int* d_deg = carve<int>(q, 1);
  llsr_s2s_report* d_rep = carve<llsr_s2s_report>(q, 1);
  hipStream_t s = h->stream;
  HIP_OK(h, hipSetDevice(h->device));
  if (Ms) HIP_OK(h, hipMemcpyAsync(d_sh, sharp, sizeof(float4) * Ms, hipMemcpyHostToDevice, s));
  if (F) HIP_OK(h, hipMemcpyAsync(d_fl, flat, sizeof(float4) * F, hipMemcpyHostToDevice, s));
  if (Nc) HIP_OK(h, hipMemcpyAsync(d_cl, cl, sizeof(float4) * Nc, hipMemcpyHostToDevice, s));
  if (Ns) HIP_OK(h, hipMemcpyAsync(d_sl, sl, sizeof(float4) * Ns, hipMemcpyHostToDevice, s));
  const int64_t offs[8] = {0, Ms, 0, F, 0, Nc, 0, Ns};
  HIP_OK(h, hipMemcpyAsync(d_off, offs, sizeof offs, hipMemcpyHostToDevice, s));
  HIP_OK(h, hipMemcpyAsync(d_t, tcur, 6 * sizeof(float), hipMemcpyHostToDevice, s));
  HIP_OK(h, hipMemcpyAsync(d_deg, degen, sizeof(int), hipMemcpyHostToDevice, s));
  llsr_s2s_batch b{};
  b.n_problems = 1;
  b.sharp = (const float*)d_sh; b.sharp_off = d_off;
  b.flat = (const float*)d_fl; b.flat_off = d_off + 2;
  b.corner_last = (const float*)d_cl; b.corner_last_off = d_off + 4;
  b.surf_last = (const float*)d_sl; b.surf_last_off = d_off + 6;
  b.transform_cur = d_t;
  b.is_degenerate = d_deg;
  b.report = d_rep;
  HIP_OK(h, hipEventRecord(m.e0, s));
  rc = llsr_scan2scan_batch(h, &b, s);
  if (rc != LLSR_OK) return rc;
  HIP_OK(h, hipEventRecord(m.e1, s));
  HIP_OK(h, hipMemcpyAsync(rep, d_rep, sizeof *rep, hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipMemcpyAsync(tcur, d_t, 6 * sizeof(float), hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipMemcpyAsync(degen, d_deg, sizeof(int), hipMemcpyDeviceToHost, s));
  rc = llsr_scan2scan_check(h);
  if (rc != LLSR_OK) return rc;
  float ms_ = 0.f;
  HIP_OK(h, hipEventElapsedTime(&ms_, m.e0, m.e1));
  rep->ms = ms_;
  return LLSR_OK;
}

// ---------------------------------------------------------------------------------------------
// End-to-end odometry (runFeatureAssociation, FA:2742-2853): see llsr_odo.hip.

static int32_t odo_alloc(llsr_handle* h) {
  auto& o = h->odo;
  if (o.pool) return LLSR_OK;
  const int B = h->max_batch;
  const size_t per = (size_t)h->dc.HW + kShadow;
  o.B = B;
  o.cap = (size_t)B * per;
  const size_t bytes = sizeof(float) * 12 * B + sizeof(int) * 3 * B + sizeof(float4) * kShadow +
                       sizeof(float4) * 8 * o.cap + sizeof(int64_t) * 6 * (B + 1) + sizeof(llsr_s2s_report) * B +
                       16 * 256;
  if (hipMalloc(&o.pool, bytes) != hipSuccess) {
    o.pool = nullptr;
    return fail(h, LLSR_ENOMEM, "odometry buffers");
  }
  char* q = (char*)o.pool;
  o.tcur = carve<float>(q, 6 * (size_t)B);
  o.tsum = carve<float>(q, 6 * (size_t)B);
  o.deg = carve<int>(q, B);
  o.inited = carve<int>(q, B);
  o.frames = carve<int>(q, B);
  o.shadow = carve<float4>(q, kShadow);
  o.sharp = carve<float4>(q, o.cap);
  o.flat = carve<float4>(q, o.cap);
  o.scan_c = carve<float4>(q, o.cap);
  o.scan_s = carve<float4>(q, o.cap);
  for (int k = 0; k < 2; ++k) {
    o.last_c[k] = carve<float4>(q, o.cap);
    o.last_s[k] = carve<float4>(q, o.cap);
  }
  o.off = carve<int64_t>(q, 6 * (size_t)(B + 1));
  o.report = carve<llsr_s2s_report>(q, B);
  if (hipHostMalloc((void**)&o.h_off, sizeof(int64_t) * 6 * (B + 1)) != hipSuccess ||
      hipHostMalloc((void**)&o.h_counts, sizeof(int) * kCnt * B) != hipSuccess)
    return fail(h, LLSR_ENOMEM, "pinned odometry staging");
  float sh[4 * kShadow];
  llsr_shadow_points(sh);
  HIP_OK(h, hipMemcpy(o.shadow, sh, sizeof sh, hipMemcpyHostToDevice));
  return llsr_odometry_reset(h);
}

extern "C" int32_t llsr_odometry_reset(llsr_handle* h) {
  if (!h) return LLSR_EINVAL;
  auto& o = h->odo;
  int32_t rc = llsr_reset_state(h);  // FA carry-over arrays (FA:167-198) of every slot
  if (rc != LLSR_OK || !o.pool) return rc;
  HIP_OK(h, hipSetDevice(h->device));
  const int B = o.B;
  HIP_OK(h, hipMemset(o.tcur, 0, sizeof(float) * 6 * B));
  HIP_OK(h, hipMemset(o.tsum, 0, sizeof(float) * 6 * B));
  HIP_OK(h, hipMemset(o.deg, 0, sizeof(int) * B));
  HIP_OK(h, hipMemset(o.inited, 0, sizeof(int) * B));
  HIP_OK(h, hipMemset(o.frames, 0, sizeof(int) * B));
  HIP_OK(h, hipMemset(o.off, 0, sizeof(int64_t) * 6 * (B + 1)));
  HIP_OK(h, hipMemset(o.report, 0, sizeof(llsr_s2s_report) * B));
  std::memset(o.h_off, 0, sizeof(int64_t) * 6 * (B + 1));
  o.cur = 0;
  return LLSR_OK;
}

extern "C" int32_t llsr_odometry_batch(llsr_handle* h, const float* d_xyzi, const int64_t* d_offsets, int32_t B,
                                       void* hip_stream) {
  if (!h) return LLSR_EINVAL;
  if (h->cfg.mode != LLSR_MODE_LM_APPLIED)
    return fail(h, LLSR_ENOSYS, "odometry needs LLSR_MODE_LM_APPLIED: faithful mode overwrites transformCur "
                                "from the /odom2 topic (updateInitialGuess, FA:2790), which has no input here");
  if (B < 1 || B > h->max_batch) return fail(h, LLSR_ERANGE, "batch size outside [1, max_batch]");
  HIP_OK(h, hipSetDevice(h->device));
  int32_t rc = odo_alloc(h);
  if (rc != LLSR_OK) return rc;
  auto& o = h->odo;
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  rc = llsr_process_batch(h, d_xyzi, d_offsets, B, s);
  if (rc != LLSR_OK) return rc;
  // the feature counts size the packed clouds: one host sync per batch
  HIP_OK(h, hipMemcpyAsync(o.h_counts, h->d.counts, sizeof(int) * kCnt * B, hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipStreamSynchronize(s));
  const int nb = o.B + 1;
  int64_t* hs = o.h_off;                       // sharp
  int64_t* hf = o.h_off + nb;                  // flat
  const int cur = o.cur, nxt = cur ^ 1;
  int64_t* hlc = o.h_off + (2 + cur) * nb;     // current last corner (from the previous batch)
  int64_t* hls = o.h_off + (4 + cur) * nb;
  int64_t* hnc = o.h_off + (2 + nxt) * nb;     // next last clouds
  int64_t* hns = o.h_off + (4 + nxt) * nb;
  int mMs = 0, mF = 0, mNc = 0, mNs = 0;
  hs[0] = hf[0] = hnc[0] = hns[0] = 0;
  for (int b = 0; b < B; ++b) {
    const int* c = o.h_counts + (size_t)b * kCnt;
    const int Ms = c[C_SHARP], F = c[C_F] + kShadow, M = c[C_M], L = c[C_L] + kShadow;
    hs[b + 1] = hs[b] + Ms;
    hf[b + 1] = hf[b] + F;
    hnc[b + 1] = hnc[b] + M;
    hns[b + 1] = hns[b] + L;
    mMs = Ms > mMs ? Ms : mMs;
    mF = F > mF ? F : mF;
    const int Nc = (int)(hlc[b + 1] - hlc[b]), Ns = (int)(hls[b + 1] - hls[b]);
    mNc = Nc > mNc ? Nc : mNc;
    mNs = Ns > mNs ? Ns : mNs;
  }
  // slots beyond B keep their (empty) ranges: offsets stay at the B-th value
  for (int b = B; b < o.B; ++b) {
    hs[b + 1] = hs[B]; hf[b + 1] = hf[B]; hnc[b + 1] = hnc[B]; hns[b + 1] = hns[B];
  }
  HIP_OK(h, hipMemcpyAsync(o.off, hs, sizeof(int64_t) * nb, hipMemcpyHostToDevice, s));
  HIP_OK(h, hipMemcpyAsync(o.off + nb, hf, sizeof(int64_t) * nb, hipMemcpyHostToDevice, s));
  HIP_OK(h, hipMemcpyAsync(o.off + (2 + nxt) * nb, hnc, sizeof(int64_t) * nb, hipMemcpyHostToDevice, s));
  HIP_OK(h, hipMemcpyAsync(o.off + (4 + nxt) * nb, hns, sizeof(int64_t) * nb, hipMemcpyHostToDevice, s));
  rc = llsr_scan2scan_reserve(h, o.B, mMs > 1 ? mMs : 1, mF, mNc > 1 ? mNc : 1, mNs > 1 ? mNs : 1);
  if (rc != LLSR_OK) return rc;
  OdoArgs a{};
  a.B = B;
  a.HW = h->dc.HW;
  a.counts = h->d.counts;
  a.loam = h->d.loam;
  a.sharp_ind = h->d.sharp;
  a.flat_ind = h->d.flat;
  a.less_sharp = h->d.less_sharp;
  a.lflat = h->d.lflat;
  a.shadow = o.shadow;
  a.sharp_off = o.off; a.sharp = o.sharp;
  a.flat_off = o.off + nb; a.flat = o.flat;
  a.nlast_c_off = o.off + (2 + nxt) * nb; a.nlast_c = o.last_c[nxt];
  a.nlast_s_off = o.off + (4 + nxt) * nb; a.nlast_s = o.last_s[nxt];
  a.scan_c = o.scan_c; a.scan_s = o.scan_s;
  a.tcur = o.tcur; a.tsum = o.tsum; a.inited = o.inited; a.frames = o.frames;
  k_odo_inputs<<<B, 256, 0, s>>>(a);
  HIP_OK(h, hipGetLastError());
  llsr_s2s_batch sb{};
  sb.n_problems = B;
  sb.sharp = (const float*)o.sharp; sb.sharp_off = o.off;
  sb.flat = (const float*)o.flat; sb.flat_off = o.off + nb;
  sb.corner_last = (const float*)o.last_c[cur]; sb.corner_last_off = o.off + (2 + cur) * nb;
  sb.surf_last = (const float*)o.last_s[cur]; sb.surf_last_off = o.off + (4 + cur) * nb;
  sb.transform_cur = o.tcur;
  sb.is_degenerate = o.deg;
  sb.report = o.report;
  // the LM instantiation follows this batch's clouds, not the (high-water) reserve
  rc = s2s_launch(h, &sb, s, std::max(std::max(mMs, mF), 1), std::max(mNc, 1));
  if (rc != LLSR_OK) return rc;
  k_odo_finish<<<B, 256, 0, s>>>(a);
  HIP_OK(h, hipGetLastError());
  HIP_OK(h, hipEventRecord(h->last_done, s));
  h->last_rec = true;
  o.cur = nxt;
  h->last_stream = s;
  return LLSR_OK;
}

extern "C" int32_t llsr_odometry_fetch(llsr_handle* h, int32_t b, llsr_odom_slot* out, float* corner_last,
                                       float* surf_last, float* corner_scan, float* surf_scan) {
  if (!h || !out) return LLSR_EINVAL;
  auto& o = h->odo;
  if (!o.pool) return fail(h, LLSR_EINVAL, "llsr_odometry_batch not called");
  if (b < 0 || b >= o.B) return fail(h, LLSR_ERANGE, "slot outside [0, max_batch)");
  int32_t rc = sync_last(h);
  if (rc) return rc;
  rc = llsr_scan2scan_check(h);
  if (rc) return rc;
  const int nb = o.B + 1;
  const int cur = o.cur;
  const int64_t* hlc = o.h_off + (2 + cur) * nb;
  const int64_t* hls = o.h_off + (4 + cur) * nb;
  std::memset(out, 0, sizeof *out);
  HIP_OK(h, d2h(&out->frames, o.frames + b, 1));
  HIP_OK(h, d2h(out->transform_cur, o.tcur + 6 * b, 6));
  HIP_OK(h, d2h(out->transform_sum, o.tsum + 6 * b, 6));
  HIP_OK(h, d2h(&out->lm, o.report + b, 1));
  out->n_corner_last = (int)(hlc[b + 1] - hlc[b]);
  out->n_surf_last = (int)(hls[b + 1] - hls[b]);
  const bool scans = out->frames > 1;  // the first scan of a slot publishes no scan clouds
  out->n_corner_scan = scans ? (int)(o.h_off[b + 1] - o.h_off[b]) : 0;
  out->n_surf_scan = scans ? (int)(o.h_off[nb + b + 1] - o.h_off[nb + b]) : 0;
  HIP_OK(h, d2h(corner_last, (const float*)(o.last_c[cur] + hlc[b]), 4 * (size_t)out->n_corner_last));
  HIP_OK(h, d2h(surf_last, (const float*)(o.last_s[cur] + hls[b]), 4 * (size_t)out->n_surf_last));
  HIP_OK(h, d2h(corner_scan, (const float*)(o.scan_c + o.h_off[b]), 4 * (size_t)out->n_corner_scan));
  HIP_OK(h, d2h(surf_scan, (const float*)(o.scan_s + o.h_off[nb + b]), 4 * (size_t)out->n_surf_scan));
  return LLSR_OK;
}

// ---------------------------------------------------------------------------------------------
// Mapping chain (MapOptimization::run, MO:1854-1896): the odometry batch, then per slot the pose
// glue on the host (llsr_mapping.h) around batched device work — adjustOutlierCloud, one
// segmented VoxelGrid for every slot's downsampleCurrentScan, the slots' local maps, and one
// scan-to-map batch over all slots.

namespace llsr {
// adjustOutlierCloud (FA:2600-2610): the IP outlier cloud of slot b (d.outl, [B][HW]) with
// x, y, z <- y, z, x, packed at off[b].
__global__ void k_mapping_outliers(const float4* outl, int HW, const int64_t* off, float4* out) {
  const int b = blockIdx.y;
  const int64_t o0 = off[b], n = off[b + 1] - o0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 p = outl[(size_t)b * HW + i];
    out[o0 + i] = make_float4(p.y, p.z, p.x, p.w);
  }
}
}  // namespace llsr

// Grow a device float4 buffer to hold `need` points, keeping its first `keep` points.
static int32_t mp_grow(llsr_handle* h, float4*& p, size_t& cap, size_t need, size_t keep, hipStream_t s) {
  if (need <= cap && p) return LLSR_OK;
  size_t n = cap ? cap : (size_t)1 << 16;
  while (n < need) n *= 2;
  float4* q = nullptr;
  if (hipMalloc(&q, n * sizeof(float4)) != hipSuccess) return fail(h, LLSR_ENOMEM, "mapping buffers");
  if (p && keep) HIP_OK(h, hipMemcpyAsync(q, p, keep * sizeof(float4), hipMemcpyDeviceToDevice, s));
  HIP_OK(h, sync_handle_streams(h));
  HIP_OK(h, hipStreamSynchronize(s));
  if (p) HIP_OK(h, hipFree(p));
  p = q;
  cap = n;
  return LLSR_OK;
}

extern "C" int32_t llsr_mapping_reset(llsr_handle* h) {
  if (!h) return LLSR_EINVAL;
  auto& mp = h->mp;
  if (!mp.live) return fail(h, LLSR_EINVAL, "llsr_mapping_init not called");
  int32_t rc = llsr_odometry_reset(h);
  if (rc != LLSR_OK) return rc;
  for (auto& sl : mp.slot) {
    llsr_map* m = sl.map;
    if (llsr_map_reset(m) != LLSR_OK) return fail(h, LLSR_EINVAL, "llsr_map_reset");
    sl = llsr_handle::MapSlot{};
    sl.map = m;
  }
  const int B = (int)mp.slot.size();
  HIP_OK(h, hipMemset(mp.d_deg, 0, sizeof(int) * B));      // isDegenerate = false (MO:285)
  HIP_OK(h, hipMemset(mp.d_matP, 0, sizeof(float) * 36 * B));  // matP zeroed (MO:286)
  return LLSR_OK;
}

// Release every mapping-chain allocation (slot stores, engine, state); mp.live becomes false.
static void mapping_free(llsr_handle* h) {
  auto& mp = h->mp;
  for (auto& sl : mp.slot)
    if (sl.map) llsr_map_destroy(sl.map);
  mp.slot.clear();
  if (mp.vg) llsr_map_destroy(mp.vg);
  mp.vg = nullptr;
  if (mp.small) (void)hipFree(mp.small);
  if (mp.hsmall) (void)hipHostFree(mp.hsmall);
  mp.small = mp.hsmall = nullptr;
  mp.live = false;
}

extern "C" int32_t llsr_mapping_init(llsr_handle* h, int32_t mo_mode, const llsr_map_config* map_cfg) {
  if (!h) return LLSR_EINVAL;
  if (mo_mode != LLSR_MODE_FAITHFUL && mo_mode != LLSR_MODE_LM_APPLIED) return fail(h, LLSR_EINVAL, "mo_mode");
  if (h->cfg.mode != LLSR_MODE_LM_APPLIED)
    return fail(h, LLSR_ENOSYS, "the mapping chain runs the odometry, which needs LLSR_MODE_LM_APPLIED");
  llsr_map_config mcfg;
  if (map_cfg) mcfg = *map_cfg;  // NULL: the YAML block of the handle's lidar
  else llsr_map_config_lidar(&mcfg, h->dc.H == 64 ? LLSR_LIDAR_HDL64E : LLSR_LIDAR_VLP16);
  if (mcfg.enable_loop_closure && mcfg.surrounding_keyframe_search_num < 1)
    return fail(h, LLSR_EINVAL, "surrounding_keyframe_search_num must be >= 1 with loop closure");
  HIP_OK(h, hipSetDevice(h->device));
  int32_t rc = odo_alloc(h);
  if (rc != LLSR_OK) return rc;
  auto& mp = h->mp;
  HIP_OK(h, sync_handle_streams(h));
  mapping_free(h);  // a repeated init rebuilds everything with the new map config
  mp.mode = mo_mode;
  mp.mcfg = mcfg;
  const int B = h->max_batch;
  mp.slot.resize(B);
  for (auto& sl : mp.slot)
    if (!(sl.map = llsr_map_create(&mp.mcfg, h->device))) { mapping_free(h); return fail(h, LLSR_ENOMEM, "llsr_map_create"); }
  if (!(mp.vg = llsr_map_create(&mp.mcfg, h->device))) { mapping_free(h); return fail(h, LLSR_ENOMEM, "llsr_map_create"); }
  const size_t nb = (size_t)B + 1;
  const size_t dbytes = sizeof(float) * 6 * B + sizeof(llsr_lm_report) * B + 2 * sizeof(int) * B +
                        2 * sizeof(float) * 36 * B + sizeof(int64_t) * 5 * nb + 10 * 256;
  const size_t hbytes = sizeof(float) * 6 * B + sizeof(llsr_lm_report) * B + sizeof(int64_t) * 5 * nb +
                        sizeof(int) * B + sizeof(float) * 6 * B + 8 * 256;
  if (hipMalloc(&mp.small, dbytes) != hipSuccess) { mp.small = nullptr; mapping_free(h); return fail(h, LLSR_ENOMEM, "mapping state"); }
  if (hipHostMalloc(&mp.hsmall, hbytes) != hipSuccess) { mp.hsmall = nullptr; mapping_free(h); return fail(h, LLSR_ENOMEM, "mapping staging"); }
  char* q = (char*)mp.small;
  mp.d_pose = carve<float>(q, 6 * (size_t)B);
  mp.d_rep = carve<llsr_lm_report>(q, B);
  mp.d_deg = carve<int>(q, B);
  mp.d_matP = carve<float>(q, 36 * (size_t)B);
  mp.d_off = carve<int64_t>(q, 5 * nb);
  mp.d_deg_bak = carve<int>(q, B);
  mp.d_matP_bak = carve<float>(q, 36 * (size_t)B);
  q = (char*)mp.hsmall;
  mp.h_pose = carve<float>(q, 6 * (size_t)B);
  mp.h_rep = carve<llsr_lm_report>(q, B);
  mp.h_off = carve<int64_t>(q, 5 * nb);
  mp.h_frames = carve<int>(q, B);
  mp.h_tsum = carve<float>(q, 6 * (size_t)B);
  mp.live = true;
  return llsr_mapping_reset(h);
}

// MapOptimization::run for the slots in `step` (their pose glue already applied by the caller).
static int32_t mapping_mo(llsr_handle* h, int32_t B, hipStream_t s, const std::vector<char>& step) {
  auto& mp = h->mp;
  auto& o = h->odo;
  int32_t rc = LLSR_OK;
  const int NB = o.B, nb = NB + 1;
  // this frame's AssociationOut clouds (the batch flipped o.cur to them)
  const int64_t* hs = o.h_off;                     // cloud_corner_scan (sharp, TransformToEnd)
  const int64_t* hf = o.h_off + nb;                // cloud_surf_scan (flat + shadow, TransformToEnd)
  const int64_t* hlc = o.h_off + (2 + o.cur) * nb; // cloud_corner_last
  const int64_t* hls = o.h_off + (4 + o.cur) * nb; // cloud_surf_last (+ shadow)
  // adjustOutlierCloud of this frame's IP outliers (FA:2720)
  int64_t* hol = mp.h_off + 4 * (size_t)nb;
  hol[0] = 0;
  int maxO = 0;
  for (int b = 0; b < NB; ++b) {
    const int n = (b < B && step[b]) ? o.h_counts[(size_t)b * kCnt + C_O] : 0;
    hol[b + 1] = hol[b] + n;
    maxO = n > maxO ? n : maxO;
  }
  rc = mp_grow(h, mp.outl, mp.cap_outl, (size_t)hol[NB] + 1, 0, s);
  if (rc != LLSR_OK) return rc;
  HIP_OK(h, hipMemcpyAsync(mp.d_off + 4 * (size_t)nb, hol, sizeof(int64_t) * nb, hipMemcpyHostToDevice, s));
  if (maxO > 0) {
    const int gx = (maxO + 255) / 256 < 64 ? (maxO + 255) / 256 : 64;
    k_mapping_outliers<<<dim3(gx, B), 256, 0, s>>>(h->d.outl, h->dc.HW, mp.d_off + 4 * (size_t)nb, mp.outl);
    HIP_OK(h, hipGetLastError());
  }
  // downsampleCurrentScan (MO:1234-1258) of every slot in one segmented VoxelGrid; segments by
  // kind so each kind's per-slot results are contiguous: [corner last][surf last, outlier]...
  // [corner scan][surf scan]
  const float lc = mp.mcfg.corner_leaf, lsf = mp.mcfg.surf_leaf, lo = mp.mcfg.outlier_leaf;
  const int S5 = 5 * NB;
  std::vector<const float4*> src(S5);
  std::vector<long long> cnt(S5, 0), dso(S5 + 1), toto(NB + 1);
  std::vector<float> leaf(S5);
  long long total = 0;
  for (int b = 0; b < NB; ++b) {
    const bool on = b < B && step[b];
    src[b] = o.last_c[o.cur] + hlc[b];          cnt[b] = on ? hlc[b + 1] - hlc[b] : 0;          leaf[b] = lc;
    src[NB + 2 * b] = o.last_s[o.cur] + hls[b]; cnt[NB + 2 * b] = on ? hls[b + 1] - hls[b] : 0; leaf[NB + 2 * b] = lsf;
    src[NB + 2 * b + 1] = mp.outl + hol[b];     cnt[NB + 2 * b + 1] = hol[b + 1] - hol[b];      leaf[NB + 2 * b + 1] = lo;
    src[3 * NB + b] = o.scan_c + hs[b];         cnt[3 * NB + b] = on ? hs[b + 1] - hs[b] : 0;   leaf[3 * NB + b] = lc;
    src[4 * NB + b] = o.scan_s + hf[b];         cnt[4 * NB + b] = on ? hf[b + 1] - hf[b] : 0;   leaf[4 * NB + b] = lsf;
  }
  for (long long c : cnt) total += c;
  rc = mp_grow(h, mp.ds, mp.cap_ds, (size_t)total + 1, 0, s);
  if (rc != LLSR_OK) return rc;
  rc = llsr_mapping::voxel_multi(mp.vg, src.data(), cnt.data(), leaf.data(), S5, mp.ds, dso.data(), s);
  if (rc != LLSR_OK) return fail(h, rc, std::string("downsample: ") + llsr_map_last_error(mp.vg));
  // laserCloudSurfTotalLastDS = surf leaf over SurfLastDS + OutlierLastDS (MO:1260-1266)
  std::vector<const float4*> tsrc(NB);
  std::vector<long long> tcnt(NB);
  std::vector<float> tleaf(NB, lsf);
  for (int b = 0; b < NB; ++b) {
    tsrc[b] = mp.ds + dso[NB + 2 * b];
    tcnt[b] = dso[NB + 2 * b + 2] - dso[NB + 2 * b];
  }
  rc = mp_grow(h, mp.tot, mp.cap_tot, (size_t)(dso[3 * NB] - dso[NB]) + 1, 0, s);
  if (rc != LLSR_OK) return rc;
  rc = llsr_mapping::voxel_multi(mp.vg, tsrc.data(), tcnt.data(), tleaf.data(), NB, mp.tot, toto.data(), s);
  if (rc != LLSR_OK) return fail(h, rc, std::string("downsample: ") + llsr_map_last_error(mp.vg));
  // extractSurroundingKeyFrames (MO:1096-1232) around currentRobotPosPoint, every slot with
  // keyframes in one pass (a slot without keyframes keeps an empty local map, MO:1097)
  std::vector<llsr_map*> emaps;
  std::vector<int> eslot;
  std::vector<float> epos;
  for (int b = 0; b < B; ++b) {
    auto& sl = mp.slot[b];
    if (!step[b]) continue;
    sl.mrep = llsr_map_report{};
    sl.n_cq = (int)(dso[3 * NB + b + 1] - dso[3 * NB + b]);
    sl.n_sq = (int)(toto[b + 1] - toto[b]);
    if (llsr_map_num_keyframes(sl.map) == 0) continue;
    emaps.push_back(sl.map);
    eslot.push_back(b);
    epos.insert(epos.end(), sl.robot, sl.robot + 3);
  }
  const int nE = (int)emaps.size();
  std::vector<llsr_map_report> ereps(nE > 0 ? nE : 1);
  std::vector<long long> eoc(nE + 1, 0), eos(nE + 1, 0);
  const float4* lmap = nullptr;
  if (nE > 0) {
    rc = llsr_mapping::extract_multi(mp.vg, emaps.data(), nE, epos.data(), ereps.data(), &lmap, eoc.data(),
                                     eos.data(), s);
    if (rc != LLSR_OK) return fail(h, rc, std::string("extract: ") + llsr_map_last_error(mp.vg));
  } else {
    rc = mp_grow(h, mp.cmap, mp.cap_cmap, 1, 0, s);  // a valid (empty) map base for the batch
    if (rc != LLSR_OK) return rc;
    lmap = mp.cmap;
  }
  int64_t* hcq = mp.h_off;
  int64_t* hsq = mp.h_off + nb;
  int64_t* hmc = mp.h_off + 2 * (size_t)nb;
  int64_t* hms = mp.h_off + 3 * (size_t)nb;
  long long mMc = 1, mMs = 1, mQc = 1, mQs = 1;
  {
    long long cc = eoc[0], cs = eos[0];
    int e = 0;
    for (int b = 0; b < NB; ++b) {
      hcq[b] = dso[3 * NB + b];
      hsq[b] = toto[b];
      hmc[b] = cc;
      hms[b] = cs;
      if (e < nE && eslot[e] == b) {
        mp.slot[b].mrep = ereps[e];
        cc = eoc[e + 1];
        cs = eos[e + 1];
        ++e;
      }
      mMc = std::max(mMc, (long long)(cc - hmc[b]));
      mMs = std::max(mMs, (long long)(cs - hms[b]));
      mQc = std::max(mQc, (long long)(dso[3 * NB + b + 1] - dso[3 * NB + b]));
      mQs = std::max(mQs, (long long)(toto[b + 1] - toto[b]));
    }
    hmc[NB] = cc;
    hms[NB] = cs;
    hcq[NB] = dso[4 * NB];
    hsq[NB] = toto[NB];
  }
  // scan2MapOptimization (MO:1572-1610): every slot is a problem; slots without a step, or whose
  // map fails MO:1573, stay inactive and keep their pose and LM members
  rc = llsr_scan2map_reserve(h, NB, (int32_t)mMc, (int32_t)mMs, (int32_t)mQc, (int32_t)mQs);
  if (rc != LLSR_OK) return rc;
  for (int b = 0; b < NB; ++b)
    for (int k = 0; k < 6; ++k) mp.h_pose[6 * b + k] = mp.slot[b].pose.transformTobeMapped[k];
  HIP_OK(h, hipMemcpyAsync(mp.d_pose, mp.h_pose, sizeof(float) * 6 * NB, hipMemcpyHostToDevice, s));
  HIP_OK(h, hipMemcpyAsync(mp.d_off, mp.h_off, sizeof(int64_t) * 4 * nb, hipMemcpyHostToDevice, s));
  llsr_s2m_batch sb{};
  sb.n_problems = NB;
  sb.corner_q = (const float*)mp.ds; sb.corner_q_off = mp.d_off;
  sb.surf_q = (const float*)mp.tot; sb.surf_q_off = mp.d_off + nb;
  sb.corner_map = (const float*)lmap; sb.corner_map_off = mp.d_off + 2 * (size_t)nb;
  sb.surf_map = (const float*)lmap; sb.surf_map_off = mp.d_off + 3 * (size_t)nb;
  sb.pose = mp.d_pose;
  sb.report = mp.d_rep;
  S2MOpts opt;
  opt.mode = mp.mode;
  opt.deg_in = opt.deg_out = mp.d_deg;
  opt.matP_in = opt.matP_out = mp.d_matP;
  rc = s2m_batch(h, &sb, s, opt);
  if (rc != LLSR_OK) return rc;
  HIP_OK(h, hipMemcpyAsync(mp.h_pose, mp.d_pose, sizeof(float) * 6 * NB, hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipMemcpyAsync(mp.h_rep, mp.d_rep, sizeof(llsr_lm_report) * NB, hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipStreamSynchronize(s));
  // transformUpdate (MO:1608) and saveKeyFramesAndFactor (MO:1612-1755)
  for (int b = 0; b < B; ++b) {
    if (!step[b]) continue;
    auto& sl = mp.slot[b];
    auto& P = sl.pose;
    sl.lm = mp.h_rep[b];
    sl.lm_ran = (hmc[b + 1] - hmc[b] > 10 && hms[b + 1] - hms[b] > 100) ? 1 : 0;
    if (sl.lm_ran) {
      for (int k = 0; k < 6; ++k) P.transformTobeMapped[k] = mp.h_pose[6 * b + k];
      llsr_mapping::transform_update(P);
    }
    for (int k = 0; k < 3; ++k) sl.robot[k] = P.transformAftMapped[3 + k];
    const bool first = llsr_map_num_keyframes(sl.map) == 0;
    const float* est = first ? P.transformTobeMapped : P.transformAftMapped;  // iSAM2's latestEstimate
    const float kp[6] = {est[3], est[4], est[5], est[0], est[1], est[2]};
    for (int k = 0; k < 6; ++k) {
      P.transformLast[k] = est[k];
      if (!first) P.transformTobeMapped[k] = P.transformAftMapped[k];
    }
    const int kf = llsr_map_add_keyframe(
        sl.map, kp, (const float*)(o.scan_c + hs[b]), (int32_t)(hs[b + 1] - hs[b]),
        (const float*)(mp.ds + dso[NB + 2 * b]), (int32_t)(dso[NB + 2 * b + 1] - dso[NB + 2 * b]),
        (const float*)(mp.ds + dso[NB + 2 * b + 1]), (int32_t)(dso[NB + 2 * b + 2] - dso[NB + 2 * b + 1]), s);
    if (kf < 0) return fail(h, kf, std::string("add_keyframe: ") + llsr_map_last_error(sl.map));
    sl.keyposes.insert(sl.keyposes.end(), kp, kp + 6);
    sl.mo_frames += 1;
  }
#ifdef LLSR_S2S_PROF
  {  // diagnostics build only: fail this call's MapOptimization part once, after its keyframes were
     // added, when slot 0 reaches MapOptimization frame LLSR_MO_FAIL_AT (tests/test_gpu_mapping_rollback.py)
    static bool fired = false;
    const char* at = std::getenv("LLSR_MO_FAIL_AT");
    if (at && !fired && step[0] && mp.slot[0].mo_frames == std::atoi(at)) {
      fired = true;
      return fail(h, LLSR_EIO, "injected MapOptimization failure (LLSR_MO_FAIL_AT)");
    }
  }
#endif
  return LLSR_OK;
}

extern "C" int32_t llsr_mapping_batch(llsr_handle* h, const float* d_xyzi, const int64_t* d_offsets, int32_t B,
                                      void* hip_stream) {
  if (!h) return LLSR_EINVAL;
  auto& mp = h->mp;
  if (!mp.live) return fail(h, LLSR_EINVAL, "llsr_mapping_init not called");
  if (B < 1 || B > h->max_batch) return fail(h, LLSR_ERANGE, "batch size outside [1, max_batch]");
  HIP_OK(h, hipSetDevice(h->device));
  hipStream_t s = hip_stream ? (hipStream_t)hip_stream : h->stream;
  int32_t rc = llsr_odometry_batch(h, d_xyzi, d_offsets, B, s);
  if (rc != LLSR_OK) return rc;
  auto& o = h->odo;
  HIP_OK(h, hipMemcpyAsync(mp.h_frames, o.frames, sizeof(int) * B, hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipMemcpyAsync(mp.h_tsum, o.tsum, sizeof(float) * 6 * B, hipMemcpyDeviceToHost, s));
  HIP_OK(h, hipStreamSynchronize(s));
  rc = llsr_scan2scan_check(h);
  if (rc != LLSR_OK) return rc;
  // MapOptimization's members of the B slots before this frame: an error below restores them
  struct Snap {
    llsr_handle::MapSlot slot;  // (keyposes: only its length is restored)
    size_t n_keyposes;
    int n_keyframes;
    llsr_mapping::MapSel sel;
  };
  std::vector<Snap> snap(B);
  for (int b = 0; b < B; ++b) {
    const auto& sl = mp.slot[b];
    snap[b].slot.pose = sl.pose;
    std::memcpy(snap[b].slot.robot, sl.robot, sizeof sl.robot);
    snap[b].slot.mo_frames = sl.mo_frames; snap[b].slot.lm_ran = sl.lm_ran;
    snap[b].slot.n_cq = sl.n_cq; snap[b].slot.n_sq = sl.n_sq; snap[b].slot.cycle = sl.cycle;
    snap[b].slot.lm = sl.lm; snap[b].slot.mrep = sl.mrep;
    snap[b].n_keyposes = sl.keyposes.size();
    snap[b].n_keyframes = llsr_map_num_keyframes(sl.map);
    snap[b].sel = llsr_mapping::map_selection(sl.map);
  }
  std::vector<char> step(o.B, 0);  // slots that receive an AssociationOut this call
  for (int b = 0; b < B; ++b) {
    auto& sl = mp.slot[b];
    sl.frames = mp.h_frames[b];
    // FA:2781-2784: the first scan sends nothing; FA:2818-2821: every mapping_frequency_divider-th
    // frame after it sends an AssociationOut
    if (sl.frames >= 2 && ++sl.cycle == h->cfg.mapping_frequency_divider) {
      sl.cycle = 0;
      step[b] = 1;
    }
    if (!step[b]) continue;
    llsr_mapping::odometry_roundtrip(mp.h_tsum + 6 * b, sl.pose.transformSum);  // OdometryToTransform
    llsr_mapping::transform_associate_to_map(sl.pose);
  }
  bool any = false;
  for (char c : step) any |= c != 0;
  if (any) {  // the LM members (isDegenerate, matP) before this frame, restored if it fails
    HIP_OK(h, hipMemcpyAsync(mp.d_deg_bak, mp.d_deg, sizeof(int) * o.B, hipMemcpyDeviceToDevice, s));
    HIP_OK(h, hipMemcpyAsync(mp.d_matP_bak, mp.d_matP, sizeof(float) * 36 * o.B, hipMemcpyDeviceToDevice, s));
  }
  rc = any ? mapping_mo(h, B, s, step) : LLSR_OK;
  if (rc != LLSR_OK) {
    const std::string msg = h->err;
    (void)hipStreamSynchronize(s);
    for (int b = 0; b < B; ++b) {
      auto& sl = mp.slot[b];
      const auto& sn = snap[b].slot;
      sl.pose = sn.pose;
      std::memcpy(sl.robot, sn.robot, sizeof sl.robot);
      sl.mo_frames = sn.mo_frames; sl.lm_ran = sn.lm_ran; sl.n_cq = sn.n_cq; sl.n_sq = sn.n_sq;
      sl.cycle = sn.cycle; sl.lm = sn.lm; sl.mrep = sn.mrep;
      sl.keyposes.resize(snap[b].n_keyposes);
      llsr_mapping::truncate_keyframes(sl.map, snap[b].n_keyframes);
      llsr_mapping::set_map_selection(sl.map, snap[b].sel);
    }
    (void)hipMemcpy(mp.d_deg, mp.d_deg_bak, sizeof(int) * o.B, hipMemcpyDeviceToDevice);
    (void)hipMemcpy(mp.d_matP, mp.d_matP_bak, sizeof(float) * 36 * o.B, hipMemcpyDeviceToDevice);
    return fail(h, rc, msg);
  }
  HIP_OK(h, hipEventRecord(h->last_done, s));
  h->last_rec = true;
  h->last_stream = s;
  return LLSR_OK;
}

extern "C" int32_t llsr_mapping_fetch(llsr_handle* h, int32_t b, llsr_mapping_slot* out) {
  if (!h || !out) return LLSR_EINVAL;
  auto& mp = h->mp;
  if (!mp.live) return fail(h, LLSR_EINVAL, "llsr_mapping_init not called");
  if (b < 0 || b >= (int)mp.slot.size()) return fail(h, LLSR_ERANGE, "slot outside [0, max_batch)");
  const auto& sl = mp.slot[b];
  std::memset(out, 0, sizeof *out);
  out->frames = sl.frames;
  out->mo_frames = sl.mo_frames;
  out->keyframes = (int32_t)(sl.keyposes.size() / 6);
  out->lm_ran = sl.lm_ran;
  for (int k = 0; k < 6; ++k) {
    out->transform_sum[k] = sl.pose.transformSum[k];
    out->transform_tobe_mapped[k] = sl.pose.transformTobeMapped[k];
    out->transform_bef_mapped[k] = sl.pose.transformBefMapped[k];
    out->transform_aft_mapped[k] = sl.pose.transformAftMapped[k];
  }
  out->n_corner_q = sl.n_cq;
  out->n_surf_q = sl.n_sq;
  out->lm = sl.lm;
  out->map = sl.mrep;
  return LLSR_OK;
}

extern "C" int32_t llsr_mapping_keyposes(llsr_handle* h, int32_t b, float* out, int32_t cap) {
  if (!h) return LLSR_EINVAL;
  auto& mp = h->mp;
  if (!mp.live) return fail(h, LLSR_EINVAL, "llsr_mapping_init not called");
  if (b < 0 || b >= (int)mp.slot.size()) return fail(h, LLSR_ERANGE, "slot outside [0, max_batch)");
  const auto& kp = mp.slot[b].keyposes;
  const int n = (int)(kp.size() / 6);
  if (out && cap > 0) std::memcpy(out, kp.data(), sizeof(float) * 6 * (size_t)(n < cap ? n : cap));
  return n;
}

extern "C" int32_t llsr_mapping_associate(const float* ts_fa, const float* bef, const float* aft, float* ts,
                                          float* tobe, float* incre) {
  if (!ts_fa || !bef || !aft || !ts || !tobe) return LLSR_EINVAL;
  llsr_mapping::MoPoses P;
  for (int k = 0; k < 6; ++k) {
    P.transformBefMapped[k] = bef[k];
    P.transformAftMapped[k] = aft[k];
  }
  llsr_mapping::odometry_roundtrip(ts_fa, P.transformSum);
  llsr_mapping::transform_associate_to_map(P);
  for (int k = 0; k < 6; ++k) {
    ts[k] = P.transformSum[k];
    tobe[k] = P.transformTobeMapped[k];
    if (incre) incre[k] = P.transformIncre[k];
  }
  return LLSR_OK;
}

// ---- TransformFusion (transformFusion.cpp, TF:65-304): host-side scalar glue ----------------
extern "C" int32_t llsr_fusion_init(llsr_fusion_state* st) {
  if (!st) return LLSR_EINVAL;
  std::memset(st, 0, sizeof *st);
  return LLSR_OK;
}

extern "C" int32_t llsr_pose_to_odometry(const float* pose, const float* twist6, llsr_odometry_msg* out) {
  if (!pose || !out) return LLSR_EINVAL;
  llsr_mapping::pose_to_odometry(pose, twist6, *out);
  return LLSR_OK;
}

extern "C" int32_t llsr_odometry_to_transform(const llsr_odometry_msg* in, float* transform) {
  if (!in || !transform) return LLSR_EINVAL;
  llsr_mapping::odometry_to_transform(*in, transform);
  return LLSR_OK;
}

extern "C" int32_t llsr_fusion_laser_odometry(llsr_fusion_state* st, const llsr_odometry_msg* laser_odometry,
                                              llsr_odometry_msg* integrated) {
  if (!st || !laser_odometry || !integrated) return LLSR_EINVAL;
  // TF:190-192: OdometryToTransform, then transformAssociateToMap (TF:65-186 = MO:458-581 with
  // transformMapped in place of transformTobeMapped)
  llsr_mapping::MoPoses P;
  llsr_mapping::odometry_to_transform(*laser_odometry, P.transformSum);
  for (int k = 0; k < 6; ++k) {
    P.transformBefMapped[k] = st->transform_bef_mapped[k];
    P.transformAftMapped[k] = st->transform_aft_mapped[k];
    P.transformIncre[k] = st->transform_incre[k];
  }
  llsr_mapping::transform_associate_to_map(P);
  for (int k = 0; k < 6; ++k) {
    st->transform_sum[k] = P.transformSum[k];
    st->transform_incre[k] = P.transformIncre[k];
    st->transform_mapped[k] = P.transformTobeMapped[k];
  }
  // TF:194-206: q.setRPY(mapped[2], -mapped[0], -mapped[1]); /integrated_to_init
  llsr_mapping::pose_to_odometry(st->transform_mapped, nullptr, *integrated);
  return LLSR_OK;
}

extern "C" int32_t llsr_fusion_aft_mapped(llsr_fusion_state* st, const llsr_odometry_msg* m) {
  if (!st || !m) return LLSR_EINVAL;
  llsr_mapping::odometry_to_transform(*m, st->transform_aft_mapped);  // TF:284-297: -pitch, -yaw, roll, position
  for (int k = 0; k < 3; ++k) {                                       // TF:299-304
    st->transform_bef_mapped[k] = (float)m->twist_angular[k];
    st->transform_bef_mapped[3 + k] = (float)m->twist_linear[k];
  }
  return LLSR_OK;
}

// ---- FA end of scan on the FA node's own thread (host side, no handle) ------------------------
// integrateTransformation (FA:2537-2568) and TransformToEnd (FA:1414-1490) as k_odo_finish runs
// them, for a node whose FA thread owns its clouds: the same functions
// (llsr_odo.h) compiled for the host, with the same glibc-exact sin / cos / asin / atan2 ports.
extern "C" int32_t llsr_integrate_transformation(float* transform_sum, const float* transform_cur) {
  if (!transform_sum || !transform_cur) return LLSR_EINVAL;
  float ts[6], tc[6];
  for (int k = 0; k < 6; ++k) {
    ts[k] = transform_sum[k];
    tc[k] = transform_cur[k];
  }
  llsr::odo_integrate(ts, tc);
  for (int k = 0; k < 6; ++k) transform_sum[k] = ts[k];
  return LLSR_OK;
}

extern "C" int32_t llsr_transform_to_end(const float* transform_cur, const float* in_xyzi, int32_t n,
                                         float* out_xyzi) {
  if (!transform_cur || n < 0 || (n > 0 && (!in_xyzi || !out_xyzi))) return LLSR_EINVAL;
  float tc[6];
  for (int k = 0; k < 6; ++k) tc[k] = transform_cur[k];
  for (int32_t i = 0; i < n; ++i) {  // in place allowed: each row is read before it is written
    const float* r = in_xyzi + 4 * (size_t)i;
    const float4 q = llsr::odo_to_end(tc, make_float4(r[0], r[1], r[2], r[3]));
    float* o = out_xyzi + 4 * (size_t)i;
    o[0] = q.x;
    o[1] = q.y;
    o[2] = q.z;
    o[3] = q.w;
  }
  return LLSR_OK;
}
