// llsr_map.hip — MapOptimization's local map on the device: the keyframe store
// (saveKeyFramesAndFactor, mapOptmization.cpp:1686-1752), extractSurroundingKeyFrames in both of
// its branches (the loop-closure queue of recent keyframes MO:1099-1151, the key-pose radius search
// MO:1152-1223) with the local-map VoxelGrids (MO:1224-1231), downsampleCurrentScan
// (MO:1234-1267), and the segmented VoxelGrid they all run on.
//
// VoxelGrid (pcl::VoxelGrid<PointXYZI>::applyFilter, PCL 1.10, downsample_all_data) of S clouds at
// once, every step a device pass over HBM:
//   k_vg_minmax    per-chunk min / max of x, y, z, folded into the cloud's bounds with order-
//                  preserving uint atomics (min / max are order independent, so exact);
//   k_vg_params    per cloud: the (max - min) * inv + 1 product check (over INT32_MAX: PCL returns
//                  the input unchanged — here every point becomes its own voxel, idx = its index,
//                  which reproduces that bit for bit), min_b = floor(min * inv), the div products;
//   k_vg_keys      PCL's index_vector entries (voxel idx << 32 | point index), in input order;
//   k_is_level /   libstdc++'s std::sort of every cloud's index_vector by voxel idx, exactly
//   k_is_leaf      (equal ids in introsort's order, which is the order PCL sums a voxel in);
//   k_vg_unpack    (cloud << 32 | voxel idx) keys + point indices for the passes below;
//   k_vg_heads     run heads, exclusive scan -> output slot of every voxel (ascending idx per
//                  cloud, the PCL output order; the per-cloud output offsets fall out of the scan);
//   k_vg_centroid  one lane per voxel sums its run in float (x, y, z, intensity) and divides by
//                  the run length, as PCL does for its sorted run.
// Host work per call is bookkeeping (block tables, the key-pose radius test over K poses, the
// surroundingExistingKeyPosesID list); every point of every cloud is touched only on the device.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <chrono>
#include <cstdint>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/llsr.h"
#include "llsr_isort.h"
#include "llsr_libm.h"
#include "llsr_mapping.h"

namespace {

using namespace llsr;
using llsr_libm::cosf_;
using llsr_libm::sinf_;

struct VgSeg {            // one cloud of a VoxelGrid call
  const float4* src;
  long long n;
  float inv;              // 1.0f / leaf (PCL: inverse_leaf_size_ = 1 / leaf_size_, float)
  int pad;
};
struct VgPar {            // per-cloud PCL parameters
  int minb[3];
  unsigned mul1, mul2;
  int pass;               // product check failed: input returned unchanged
};
struct Chunk {            // a block's share: points [b, e) of cloud seg
  int seg, pad;
  long long b, e;
};
constexpr int kChunk = 4096;  // points per block in the chunked passes (256 lanes x 16)

__device__ __forceinline__ unsigned ord(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord(unsigned o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__global__ void k_vg_init(unsigned* mm, int S) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  for (int a = 0; a < 3; ++a) {
    mm[6 * s + a] = 0xffffffffu;
    mm[6 * s + 3 + a] = 0u;
  }
}

__global__ __launch_bounds__(256) void k_vg_minmax(const Chunk* ch, const VgSeg* segs, unsigned* mm) {
  const Chunk c = ch[blockIdx.x];
  const float4* p = segs[c.seg].src;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (long long i = c.b + threadIdx.x; i < c.e; i += blockDim.x) {
    const float4 q = p[i];
    mn[0] = fminf(mn[0], q.x); mx[0] = fmaxf(mx[0], q.x);
    mn[1] = fminf(mn[1], q.y); mx[1] = fmaxf(mx[1], q.y);
    mn[2] = fminf(mn[2], q.z); mx[2] = fmaxf(mx[2], q.z);
  }
  for (int o = 32; o > 0; o >>= 1)
    for (int a = 0; a < 3; ++a) {
      mn[a] = fminf(mn[a], __shfl_xor(mn[a], o));
      mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o));
    }
  __shared__ float red[4][6];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int a = 0; a < 3; ++a) { red[w][a] = mn[a]; red[w][3 + a] = mx[a]; }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int a = threadIdx.x;
    float v = red[0][a];
    for (int k = 1; k < 4; ++k) v = a < 3 ? fminf(v, red[k][a]) : fmaxf(v, red[k][a]);
    if (a < 3) atomicMin(&mm[6 * c.seg + a], ord(v));
    else atomicMax(&mm[6 * c.seg + a], ord(v));
  }
}

__global__ void k_vg_params(const VgSeg* segs, const unsigned* mm, VgPar* par, int S) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  VgPar q{};
  if (segs[s].n > 0) {
    const float inv = segs[s].inv;
    float mn[3], mx[3];
    for (int a = 0; a < 3; ++a) { mn[a] = unord(mm[6 * s + a]); mx[a] = unord(mm[6 * s + 3 + a]); }
    // PCL: int64(float) + 1 per axis, product > INT32_MAX. Truncated in double (exact for these
    // magnitudes; an f32 -> i64 conversion here crashes the gfx950 instruction selector), and the
    // product in double is exact wherever it is near the INT32_MAX threshold.
    const float ex = (mx[0] - mn[0]) * inv, ey = (mx[1] - mn[1]) * inv, ez = (mx[2] - mn[2]) * inv;
    const double dx = trunc((double)ex) + 1, dy = trunc((double)ey) + 1, dz = trunc((double)ez) + 1;
    q.pass = dx * dy * dz > 2147483647.0;
    int div[3];
    for (int a = 0; a < 3; ++a) {
      q.minb[a] = (int)floorf(mn[a] * inv);
      div[a] = (int)floorf(mx[a] * inv) - q.minb[a] + 1;
    }
    q.mul1 = (unsigned)div[0];
    q.mul2 = (unsigned)div[0] * (unsigned)div[1];
  }
  par[s] = q;
}

// PCL's index_vector entry of each point: (voxel id << 32 | point index), in input order.
__global__ __launch_bounds__(256) void k_vg_keys(const Chunk* ch, const VgSeg* segs, const VgPar* par,
                                                 const long long* base, unsigned long long* kk) {
  const Chunk c = ch[blockIdx.x];
  const float4* p = segs[c.seg].src;
  const float inv = segs[c.seg].inv;
  const VgPar q = par[c.seg];
  const long long o = base[c.seg];
  for (long long i = c.b + threadIdx.x; i < c.e; i += blockDim.x) {
    unsigned idx;
    if (q.pass) {
      idx = (unsigned)i;
    } else {
      const float4 v = p[i];
      const int i0 = (int)(floorf(v.x * inv) - (float)q.minb[0]);
      const int i1 = (int)(floorf(v.y * inv) - (float)q.minb[1]);
      const int i2 = (int)(floorf(v.z * inv) - (float)q.minb[2]);
      idx = (unsigned)i0 + (unsigned)i1 * q.mul1 + (unsigned)i2 * q.mul2;
    }
    kk[o + i] = ((unsigned long long)idx << 32) | (unsigned)i;
  }
}

// ---- std::sort(index_vector) by voxel id, exactly as libstdc++ leaves equal ids ----------------
// Every segment is sorted on its own (llsr_isort.h): ranges above kIsLeaf are partitioned in
// global memory, one 1024-thread workgroup per range and level (k_is_level: the same parallel
// statement of __unguarded_partition as the wave version, with the stop lists in Lb / Rb); ranges
// of at most kIsLeaf elements finish in LDS, one wave each, with the depth limit they inherited
// (k_is_leaf). A range whose depth limit runs out above kIsLeaf is heap-sorted by one lane (the
// median-of-3 killer case; never met by point clouds).
struct IsRange {
  long long f, l;  // [f, l) in the packed key array
  int d, pad;      // remaining depth limit
};
constexpr int kIsLeaf = 1024;  // measured: 2048 -> 1024 local map 355 -> 369 extracts/s (512: same)
constexpr int kIsT = 1024;       // threads of k_is_level
constexpr int kIsE = 4;          // elements per lane per tile

__device__ void is_push(IsRange r, IsRange* nxt, int* n_nxt, IsRange* leaves, int* n_leaves) {
  const long long n = r.l - r.f;
  if (n <= 1) return;
  if (n > kIsLeaf) nxt[atomicAdd(n_nxt, 1)] = r;
  else leaves[atomicAdd(n_leaves, 1)] = r;
}

__global__ __launch_bounds__(kIsT) void k_is_level(unsigned long long* kk, const IsRange* in, const int* n_in,
                                                   IsRange* nxt, int* n_nxt, IsRange* leaves, int* n_leaves, int* Lb,
                                                   int* Rb) {
  if ((int)blockIdx.x >= *n_in) return;  // the grid is an upper bound on this level's ranges
  const IsRange r = in[blockIdx.x];
  unsigned long long* a = kk + r.f;
  int* Lp = Lb + r.f;
  int* Rp = Rb + r.f;
  const int n = (int)(r.l - r.f);
  const int t = threadIdx.x, w = t >> 6, ln = t & 63;
  const unsigned long long ltm = (1ull << ln) - 1ull;
  const VoxLess lt;
  if (r.d == 0) {  // __partial_sort(first, last, last)
    if (t == 0) heap_sort_range(reinterpret_cast<uint64_t*>(a), 0, n, lt);
    return;
  }
  if (t == 0) {  // __move_median_to_first(first, first + 1, mid, last - 1)
    const int x = 1, y = n / 2, z = n - 1;
    int m;
    if (lt(a[x], a[y])) m = lt(a[y], a[z]) ? y : (lt(a[x], a[z]) ? z : x);
    else m = lt(a[x], a[z]) ? x : (lt(a[y], a[z]) ? z : y);
    const unsigned long long v = a[0]; a[0] = a[m]; a[m] = v;
  }
  __syncthreads();
  const unsigned long long P = a[0];
  __shared__ int wcnt[kIsT / 64];
  __shared__ int s_first;
  // stop lists: L = ascending positions in [1, n) with !(a < P); R = descending positions in
  // [0, n) with !(P < a)
  int nL = 0, nR = 0;
  for (int side = 0; side < 2; ++side) {
    int tot_all = 0;
    for (int t0 = 0; t0 < n; t0 += kIsT * kIsE) {
      unsigned long long m[kIsE];
      int cnt = 0;
#pragma unroll
      for (int e = 0; e < kIsE; ++e) {
        const int k = t0 + (w * kIsE + e) * 64 + ln;  // k-th position in scan order
        bool f;
        if (side == 0) f = k + 1 < n && !lt(a[k + 1], P);
        else f = k < n && !lt(P, a[n - 1 - k]);
        m[e] = __ballot(f);
        cnt += (int)__popcll(m[e]);
      }
      if (ln == 0) wcnt[w] = cnt;
      __syncthreads();
      int off = 0, tot = 0;
      for (int q = 0; q < kIsT / 64; ++q) {
        off += q < w ? wcnt[q] : 0;
        tot += wcnt[q];
      }
      off += tot_all;
#pragma unroll
      for (int e = 0; e < kIsE; ++e) {
        const int k = t0 + (w * kIsE + e) * 64 + ln;
        if ((m[e] >> ln) & 1ull) {
          const int pos = off + (int)__popcll(m[e] & ltm);
          if (side == 0) Lp[pos] = k + 1;
          else Rp[pos] = n - 1 - k;
        }
        off += (int)__popcll(m[e]);
      }
      tot_all += tot;
      __syncthreads();
    }
    if (side == 0) nL = tot_all;
    else nR = tot_all;
  }
  // k* = first k < min(nL, nR) with !(L[k] < R[k]) (monotone): kIsT-ary search
  const int nm = nL < nR ? nL : nR;
  int lo = 0, hi = nm;  // good below lo, bad from hi
  while (hi > lo) {
    const int step = (hi - lo + kIsT - 1) / kIsT;
    if (t == 0) s_first = kIsT;
    __syncthreads();
    const int k = lo + t * step;
    if (k < hi && !(Lp[k] < Rp[k])) atomicMin(&s_first, t);
    __syncthreads();
    const int tb = s_first;
    __syncthreads();
    if (tb < kIsT) {
      const int nlo = tb > 0 ? lo + (tb - 1) * step + 1 : lo;
      hi = lo + tb * step;
      lo = nlo;
    } else {
      const int tlast = min(kIsT - 1, (hi - 1 - lo) / step);
      lo = lo + tlast * step + 1;
    }
  }
  const int ks = lo;
  const int cut = (ks > 0 && (ks >= nL || Lp[ks] >= Rp[ks - 1])) ? Rp[ks - 1] : Lp[ks];
  for (int k = t; k < ks; k += kIsT) {
    const int x = Lp[k], y = Rp[k];
    const unsigned long long v = a[x]; a[x] = a[y]; a[y] = v;
  }
  if (t == 0) {
    is_push(IsRange{r.f, r.f + cut, r.d - 1, 0}, nxt, n_nxt, leaves, n_leaves);
    is_push(IsRange{r.f + cut, r.l, r.d - 1, 0}, nxt, n_nxt, leaves, n_leaves);
  }
}

// One wave per range of at most kIsLeaf elements: the rest of its introsort, in LDS.
__global__ __launch_bounds__(64) void k_is_leaf(unsigned long long* kk, const IsRange* leaves) {
  __shared__ uint64_t key[kIsLeaf];
  __shared__ uint16_t Lp[kIsLeaf], Rp[kIsLeaf];
  __shared__ int stk[3 * kSortStack];
  const IsRange r = leaves[blockIdx.x];
  const int n = (int)(r.l - r.f);
  for (int k = threadIdx.x; k < n; k += 64) key[k] = kk[r.f + k];
  wave_sync_lds();
  exact_introsort(key, n, Lp, Rp, stk, VoxLess{}, r.d);
  for (int k = threadIdx.x; k < n; k += 64) kk[r.f + k] = key[k];
}

// Sorted index_vector -> the (segment << 32 | voxel id, point index) pairs the head / centroid
// passes read.
__global__ __launch_bounds__(256) void k_vg_unpack(const Chunk* ch, const long long* base,
                                                   const unsigned long long* kk, unsigned long long* key, int* val) {
  const Chunk c = ch[blockIdx.x];
  const long long o = base[c.seg];
  for (long long i = c.b + threadIdx.x; i < c.e; i += blockDim.x) {
    const unsigned long long v = kk[o + i];
    key[o + i] = ((unsigned long long)c.seg << 32) | (v >> 32);
    val[o + i] = (int)(unsigned)(v & 0xffffffffull);
  }
}

__global__ void k_vg_heads(const unsigned long long* key, int* flag, long long N) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  flag[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}

__global__ void k_vg_centroid(const unsigned long long* key, const int* val, const int* flag, const int* rank,
                              const VgSeg* segs, float4* out, long long N) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N || !flag[i]) return;
  const unsigned long long k = key[i];
  const float4* p = segs[(int)(k >> 32)].src;
  float sx = 0, sy = 0, sz = 0, si = 0;
  long long j = i;
  do {
    const float4 v = p[val[j]];
    sx += v.x; sy += v.y; sz += v.z; si += v.w;
    ++j;
  } while (j < N && key[j] == k);
  const float n = (float)(j - i);
  out[rank[i]] = make_float4(sx / n, sy / n, sz / n, si / n);
}

// out_off[s] = output slot of cloud s's first voxel (= rank at its first sorted position, which
// for an empty cloud is the next cloud's first slot); out_off[S] = voxel total.
__global__ void k_vg_offsets(const long long* base, const int* flag, const int* rank, long long N, int S,
                             long long* out_off) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > S) return;
  const long long total = N > 0 ? (long long)rank[N - 1] + flag[N - 1] : 0;
  const long long b = base[s];
  out_off[s] = b < N ? (long long)rank[b] : total;
}

// transformPointCloud(cloudIn, transformIn) (MO:671-701) of one keyframe chunk per block.
struct XfChunk {
  const float4* src;   // keyframe cloud chunk in its map's store
  long long dst;       // offset in the assembled map (points)
  int n, pad;
  float t[6];          // x, y, z, roll, pitch, yaw
};

__global__ __launch_bounds__(256) void k_map_transform(const XfChunk* ch, float4* map) {
  const XfChunk c = ch[blockIdx.x];
  const float tx = c.t[0], ty = c.t[1], tz = c.t[2], roll = c.t[3], pitch = c.t[4], yaw = c.t[5];
  const float cy = cosf_(yaw), sy = sinf_(yaw), cr = cosf_(roll), sr = sinf_(roll), cp = cosf_(pitch),
              sp = sinf_(pitch);
  for (int k = threadIdx.x; k < c.n; k += blockDim.x) {
    const float4 q = c.src[k];
    const float x1 = cy * q.x - sy * q.y;
    const float y1 = sy * q.x + cy * q.y;
    const float z1 = q.z;
    const float x2 = x1;
    const float y2 = cr * y1 - sr * z1;
    const float z2 = sr * y1 + cr * z1;
    map[c.dst + k] = make_float4(cp * x2 + sp * z2 + tx, y2 + ty, -sp * x2 + cp * z2 + tz, q.w);
  }
}

template <class T>
hipError_t grow(T*& p, size_t& cap, size_t need) {
  if (need <= cap) return hipSuccess;
  size_t n = cap ? cap : 1024;
  while (n < need) n += n / 2 + 1;
  if (p) {
    hipError_t e = hipFree(p);
    if (e != hipSuccess) return e;
    p = nullptr;
  }
  cap = 0;
  hipError_t e = hipMalloc(&p, n * sizeof(T));
  if (e == hipSuccess) cap = n;
  return e;
}


}  // namespace

struct llsr_map {
  llsr_map_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // keyframe store: packed points, host-side index
  float4* store = nullptr;
  size_t store_cap = 0, store_used = 0;
  struct Kf { float pose[6]; long long off[3]; int n[3]; };  // corner, surf, outlier
  std::vector<Kf> kf;
  // the local map's keyframe list: surroundingExistingKeyPosesID (radius branch) or the indices of
  // recent{Corner,Surf,Outlier}CloudKeyFrames, oldest first (loop-closure branch); with the
  // latestFrameID of MO:1126-1134 (0 from the constructor, MO:301)
  llsr_mapping::MapSel sel;
  // VoxelGrid scratch
  unsigned long long *key = nullptr, *key2 = nullptr;
  int *val = nullptr, *val2 = nullptr, *flag = nullptr, *rank = nullptr;
  size_t cap_key = 0, cap_key2 = 0, cap_val = 0, cap_val2 = 0, cap_flag = 0, cap_rank = 0;
  void* tmp = nullptr;
  size_t cap_tmp = 0;
  unsigned* mm = nullptr;
  size_t cap_mm = 0;
  VgPar* par = nullptr;
  size_t cap_par = 0;
  char* dtab = nullptr;        // device tables (segments, chunks, bases, out offsets)
  size_t cap_dtab = 0;
  char* htab = nullptr;        // pinned host staging of the same
  size_t cap_htab = 0;
  // local-map assembly
  float4* mapbuf = nullptr;    // [corner map | surf map]
  size_t cap_map = 0;
  float4* dsbuf = nullptr;     // VoxelGrid output staging
  size_t cap_ds = 0;
  float4* poses = nullptr;     // selected key poses (x, y, z, index)
  size_t cap_poses = 0;
  char* hstage = nullptr;      // pinned staging of the extract's own uploads (poses, chunk table)
  size_t cap_hstage = 0;
  char* dxf = nullptr;         // device chunk table of k_map_transform
  size_t cap_dxf = 0;
  char* isbuf = nullptr;       // exact introsort: range lists + counters
  size_t cap_isbuf = 0;
  int* hcnt = nullptr;         // pinned counters
};

static int32_t mfail(llsr_map* m, int32_t code, const std::string& msg) {
  if (m) m->err = msg;
  return code;
}

#define MAP_OK(m, expr)                                                          \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess)                                                        \
      return mfail(m, LLSR_EIO, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

namespace {

struct VgCloud {
  const float4* src;
  long long n;
  float leaf;
};

hipError_t host_grow(char*& p, size_t& cap, size_t need) {
  if (need <= cap) return hipSuccess;
  size_t n = cap ? cap : 4096;
  while (n < need) n *= 2;
  if (p) {
    hipError_t e = hipHostFree(p);
    if (e != hipSuccess) return e;
    p = nullptr;
  }
  cap = 0;
  hipError_t e = hipHostMalloc(&p, n);
  if (e == hipSuccess) cap = n;
  return e;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// The segmented VoxelGrid: clouds -> d_out packed (capacity sum n), out_off[S+1] on the host.
int32_t vg_run(llsr_map* m, const std::vector<VgCloud>& cl, float4* d_out, long long* out_off, hipStream_t s) {
  const int S = (int)cl.size();
  long long N = 0;
  std::vector<long long> base(S + 1);
  for (int k = 0; k < S; ++k) {
    if (cl[k].n < 0 || !(cl[k].leaf > 0)) return mfail(m, LLSR_EINVAL, "voxel grid: bad cloud size or leaf");
    base[k] = N;
    N += cl[k].n;
  }
  base[S] = N;
  if (N >= (long long)INT32_MAX) return mfail(m, LLSR_ERANGE, "voxel grid: more than 2^31 points");
  if (N == 0) {
    for (int k = 0; k <= S; ++k) out_off[k] = 0;
    return LLSR_OK;
  }
  // host tables: segments, chunks, bases
  std::vector<Chunk> ch;
  for (int k = 0; k < S; ++k)
    for (long long b = 0; b < cl[k].n; b += kChunk) ch.push_back({k, 0, b, std::min(cl[k].n, b + kChunk)});
  const size_t o_seg = 0, o_ch = align256(S * sizeof(VgSeg)), o_base = o_ch + align256(ch.size() * sizeof(Chunk)),
               o_out = o_base + align256((S + 1) * sizeof(long long)),
               bytes = o_out + align256((S + 1) * sizeof(long long));
  MAP_OK(m, host_grow(m->htab, m->cap_htab, bytes));
  MAP_OK(m, grow(m->dtab, m->cap_dtab, bytes));
  VgSeg* hs = reinterpret_cast<VgSeg*>(m->htab + o_seg);
  for (int k = 0; k < S; ++k) hs[k] = {cl[k].src, cl[k].n, 1.0f / cl[k].leaf, 0};
  std::memcpy(m->htab + o_ch, ch.data(), ch.size() * sizeof(Chunk));
  std::memcpy(m->htab + o_base, base.data(), (S + 1) * sizeof(long long));
  MAP_OK(m, hipMemcpyAsync(m->dtab, m->htab, o_out, hipMemcpyHostToDevice, s));
  const VgSeg* dseg = reinterpret_cast<const VgSeg*>(m->dtab + o_seg);
  const Chunk* dch = reinterpret_cast<const Chunk*>(m->dtab + o_ch);
  const long long* dbase = reinterpret_cast<const long long*>(m->dtab + o_base);
  long long* doff = reinterpret_cast<long long*>(m->dtab + o_out);
  // scratch
  MAP_OK(m, grow(m->key, m->cap_key, N));
  MAP_OK(m, grow(m->key2, m->cap_key2, N));
  MAP_OK(m, grow(m->val, m->cap_val, N));
  MAP_OK(m, grow(m->val2, m->cap_val2, N));
  MAP_OK(m, grow(m->flag, m->cap_flag, N));
  MAP_OK(m, grow(m->rank, m->cap_rank, N));
  MAP_OK(m, grow(m->mm, m->cap_mm, 6 * (size_t)S));
  MAP_OK(m, grow(m->par, m->cap_par, (size_t)S));
  size_t tb_scan = 0;
  MAP_OK(m, hipcub::DeviceScan::ExclusiveSum(nullptr, tb_scan, m->flag, m->rank, (int)N, s));
  MAP_OK(m, grow(reinterpret_cast<char*&>(m->tmp), m->cap_tmp, tb_scan));
  const int nch = (int)ch.size();
  k_vg_init<<<(S + 63) / 64, 64, 0, s>>>(m->mm, S);
  k_vg_minmax<<<nch, 256, 0, s>>>(dch, dseg, m->mm);
  k_vg_params<<<(S + 63) / 64, 64, 0, s>>>(dseg, m->mm, m->par, S);
  k_vg_keys<<<nch, 256, 0, s>>>(dch, dseg, m->par, dbase, m->key);
  MAP_OK(m, hipGetLastError());
  // std::sort of every segment's index_vector (m->key), the stop lists in flag / rank
  {
    std::vector<IsRange> big, small;
    for (int k = 0; k < S; ++k) {
      const long long n = cl[k].n;
      if (n < 2) continue;
      int lg = 0;
      while ((2ll << lg) <= n) ++lg;  // std::__lg
      const IsRange r{base[k], base[k] + n, 2 * lg, 0};
      (n > kIsLeaf ? big : small).push_back(r);
    }
    const size_t capA = (size_t)(N / kIsLeaf) + S + 2;
    const size_t capL = 84 * ((size_t)(N / kIsLeaf) + 1) + S + 2;
    const size_t o_b = align256(capA * sizeof(IsRange)), o_l = o_b + o_b,
                 o_c = o_l + align256(capL * sizeof(IsRange)), bytes_is = o_c + 256;  // dcnt: 4 ints
    MAP_OK(m, grow(m->isbuf, m->cap_isbuf, bytes_is));
    if (!m->hcnt) MAP_OK(m, hipHostMalloc((void**)&m->hcnt, 4 * sizeof(int)));
    IsRange* lA = reinterpret_cast<IsRange*>(m->isbuf);
    IsRange* lB = reinterpret_cast<IsRange*>(m->isbuf + o_b);
    IsRange* lL = reinterpret_cast<IsRange*>(m->isbuf + o_l);
    int* dcnt = reinterpret_cast<int*>(m->isbuf + o_c);
    // the host tables above were uploaded from htab asynchronously: stage the ranges after them
    const size_t o_h = align256(bytes), o_h2 = o_h + align256(big.size() * sizeof(IsRange) + 1),
                 hneed = o_h2 + align256(small.size() * sizeof(IsRange) + 1);  // big, then small ranges
    MAP_OK(m, hipStreamSynchronize(s));
    MAP_OK(m, host_grow(m->htab, m->cap_htab, hneed + align256((S + 1) * sizeof(long long))));
    // (host_grow may have moved htab: re-stage the offsets area after the sort, below)
    if (!big.empty()) {
      std::memcpy(m->htab + o_h, big.data(), big.size() * sizeof(IsRange));
      MAP_OK(m, hipMemcpyAsync(lA, m->htab + o_h, big.size() * sizeof(IsRange), hipMemcpyHostToDevice, s));
    }
    if (!small.empty()) {
      std::memcpy(m->htab + o_h2, small.data(), small.size() * sizeof(IsRange));
      MAP_OK(m, hipMemcpyAsync(lL, m->htab + o_h2, small.size() * sizeof(IsRange), hipMemcpyHostToDevice, s));
    }
    int nA = (int)big.size();
    m->hcnt[0] = nA;                 // dcnt[0]: ranges of the current level (device-side)
    m->hcnt[1] = (int)small.size();  // dcnt[1]: leaves
    m->hcnt[2] = 0;                  // dcnt[2]: ranges of the next level
    // (the pinned staging above is not touched again before the next synchronisation below)
    MAP_OK(m, hipMemcpyAsync(dcnt, m->hcnt, 3 * sizeof(int), hipMemcpyHostToDevice, s));
    // partition levels in batches of kLevels launches between host checks: each launch's grid is
    // an upper bound on its level's ranges (a range pushes at most two; capA bounds them all, the
    // ranges above kIsLeaf being disjoint), blocks past the device-side count exit at once
    constexpr int kLevels = 4;
    int* dA = dcnt;
    int* dB = dcnt + 2;
    while (nA > 0) {
      int bound = nA;
      for (int k = 0; k < kLevels; ++k) {
        MAP_OK(m, hipMemsetAsync(dB, 0, sizeof(int), s));
        k_is_level<<<bound, kIsT, 0, s>>>(m->key, lA, dA, lB, dB, lL, dcnt + 1, m->flag, m->rank);
        MAP_OK(m, hipGetLastError());
        std::swap(lA, lB);
        std::swap(dA, dB);
        bound = (int)std::min<size_t>(2 * (size_t)bound, capA);
      }
      MAP_OK(m, hipMemcpyAsync(m->hcnt, dA, sizeof(int), hipMemcpyDeviceToHost, s));
      MAP_OK(m, hipMemcpyAsync(m->hcnt + 1, dcnt + 1, sizeof(int), hipMemcpyDeviceToHost, s));
      MAP_OK(m, hipStreamSynchronize(s));
      nA = m->hcnt[0];
      if ((size_t)nA > capA || (size_t)m->hcnt[1] > capL) return mfail(m, LLSR_EIO, "voxel grid: introsort range lists overflow");
    }
    const int nLeaves = m->hcnt[1];
    if (nLeaves > 0) k_is_leaf<<<nLeaves, 64, 0, s>>>(m->key, lL);
    k_vg_unpack<<<nch, 256, 0, s>>>(dch, dbase, m->key, m->key2, m->val2);
    MAP_OK(m, hipGetLastError());
  }
  const int nb = (int)((N + 255) / 256);
  k_vg_heads<<<nb, 256, 0, s>>>(m->key2, m->flag, N);
  size_t tb = m->cap_tmp;
  MAP_OK(m, hipcub::DeviceScan::ExclusiveSum(m->tmp, tb, m->flag, m->rank, (int)N, s));
  k_vg_centroid<<<nb, 256, 0, s>>>(m->key2, m->val2, m->flag, m->rank, dseg, d_out, N);
  k_vg_offsets<<<(S + 64) / 64, 64, 0, s>>>(dbase, m->flag, m->rank, N, S, doff);
  MAP_OK(m, hipGetLastError());
  long long* hoff = reinterpret_cast<long long*>(m->htab + o_out);
  MAP_OK(m, hipMemcpyAsync(hoff, doff, (S + 1) * sizeof(long long), hipMemcpyDeviceToHost, s));
  MAP_OK(m, hipStreamSynchronize(s));
  std::memcpy(out_off, hoff, (S + 1) * sizeof(long long));
  return LLSR_OK;
}

hipStream_t pick(llsr_map* m, void* s) { return s ? static_cast<hipStream_t>(s) : m->stream; }

}  // namespace

extern "C" int32_t llsr_map_config_default(llsr_map_config* c) {
  if (!c) return LLSR_EINVAL;
  c->surrounding_radius = 50.0f;
  c->keypose_leaf = 1.0f;
  c->corner_leaf = 0.2f;
  c->surf_leaf = 0.4f;
  c->outlier_leaf = 0.4f;
  c->enable_loop_closure = 0;               // CFG:23
  c->surrounding_keyframe_search_num = 50;  // CFG:27
  return LLSR_OK;
}

extern "C" int32_t llsr_map_config_lidar(llsr_map_config* c, int32_t lidar) {
  if (!c) return LLSR_EINVAL;
  if (lidar != LLSR_LIDAR_VLP16 && lidar != LLSR_LIDAR_HDL64E) return LLSR_EINVAL;
  llsr_map_config_default(c);  // radius 50 and search num 50 in both blocks (CFG:26-27, 162-163)
  c->enable_loop_closure = lidar == LLSR_LIDAR_HDL64E ? 1 : 0;  // CFG:159
  return LLSR_OK;
}

namespace llsr_mapping {
MapSel map_selection(const llsr_map* m) { return m->sel; }
void set_map_selection(llsr_map* m, const MapSel& s) { m->sel = s; }
void truncate_keyframes(llsr_map* m, int keep) {
  if (keep < 0 || keep >= (int)m->kf.size()) return;
  m->store_used = (size_t)m->kf[keep].off[0];
  m->kf.resize(keep);
}
}  // namespace llsr_mapping

extern "C" llsr_map* llsr_map_create(const llsr_map_config* cfg, int32_t dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || dev >= n) return nullptr;
  // a loop-closure queue of fewer than one keyframe would pop from an empty deque (MO:1130)
  if (cfg && cfg->enable_loop_closure && cfg->surrounding_keyframe_search_num < 1) return nullptr;
  llsr_map* m = new (std::nothrow) llsr_map();
  if (!m) return nullptr;
  if (cfg) m->cfg = *cfg;
  else llsr_map_config_default(&m->cfg);
  m->device = dev;
  if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) {
    delete m;
    return nullptr;
  }
  return m;
}

extern "C" void llsr_map_destroy(llsr_map* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  (void)hipStreamSynchronize(m->stream);
  void* dev[] = {m->store, m->key, m->key2, m->val, m->val2, m->flag, m->rank, m->tmp, m->mm, m->par, m->dtab,
                 m->mapbuf, m->dsbuf, m->poses, m->dxf, m->isbuf};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  if (m->htab) (void)hipHostFree(m->htab);
  if (m->hstage) (void)hipHostFree(m->hstage);
  if (m->hcnt) (void)hipHostFree(m->hcnt);
  (void)hipStreamDestroy(m->stream);
  delete m;
}

extern "C" const char* llsr_map_last_error(const llsr_map* m) { return m ? m->err.c_str() : "null map"; }

extern "C" int32_t llsr_map_reset(llsr_map* m) {
  if (!m) return LLSR_EINVAL;
  m->kf.clear();
  m->sel = llsr_mapping::MapSel{};
  m->store_used = 0;
  return LLSR_OK;
}

extern "C" int32_t llsr_map_num_keyframes(const llsr_map* m) { return m ? (int32_t)m->kf.size() : LLSR_EINVAL; }

extern "C" int32_t llsr_map_voxel_grid(llsr_map* m, const float* d_in, const int64_t* off, int32_t S,
                                       const float* leaf, float* d_out, int64_t* out_off, void* hip_stream) {
  if (!m || !off || !leaf || !out_off || S < 1) return mfail(m, LLSR_EINVAL, "voxel_grid: bad arguments");
  if (off[S] > 0 && (!d_in || !d_out)) return mfail(m, LLSR_EINVAL, "voxel_grid: null cloud");
  MAP_OK(m, hipSetDevice(m->device));
  std::vector<VgCloud> cl(S);
  for (int k = 0; k < S; ++k) {
    if (off[k + 1] < off[k]) return mfail(m, LLSR_EINVAL, "voxel_grid: offsets must be non-decreasing");
    cl[k] = {reinterpret_cast<const float4*>(d_in) + off[k], off[k + 1] - off[k], leaf[k]};
  }
  std::vector<long long> o(S + 1);
  const int32_t rc = vg_run(m, cl, reinterpret_cast<float4*>(d_out), o.data(), pick(m, hip_stream));
  if (rc != LLSR_OK) return rc;
  for (int k = 0; k <= S; ++k) out_off[k] = o[k];
  return LLSR_OK;
}

extern "C" int32_t llsr_map_downsample_scan(llsr_map* m, const float* cl, int32_t ncl, const float* sl, int32_t nsl,
                                            const float* ol, int32_t nol, const float* cs, int32_t ncs,
                                            const float* ss, int32_t nss, float* d_out, int64_t* out_off,
                                            void* hip_stream) {
  if (!m || !d_out || !out_off || ncl < 0 || nsl < 0 || nol < 0 || ncs < 0 || nss < 0)
    return mfail(m, LLSR_EINVAL, "downsample_scan: bad arguments");
  MAP_OK(m, hipSetDevice(m->device));
  const hipStream_t s = pick(m, hip_stream);
  auto f4 = [](const float* p) { return reinterpret_cast<const float4*>(p); };
  const std::vector<VgCloud> five = {{f4(cl), ncl, m->cfg.corner_leaf},  {f4(sl), nsl, m->cfg.surf_leaf},
                                     {f4(ol), nol, m->cfg.outlier_leaf}, {f4(cs), ncs, m->cfg.corner_leaf},
                                     {f4(ss), nss, m->cfg.surf_leaf}};
  float4* out = reinterpret_cast<float4*>(d_out);
  long long o[6];
  int32_t rc = vg_run(m, five, out, o, s);
  if (rc != LLSR_OK) return rc;
  // laserCloudSurfTotalLast = SurfLastDS + OutlierLastDS, contiguous at [o[1], o[3]) (MO:1261-1266)
  const std::vector<VgCloud> total = {{out + o[1], o[3] - o[1], m->cfg.surf_leaf}};
  long long t[2];
  rc = vg_run(m, total, out + o[5], t, s);
  if (rc != LLSR_OK) return rc;
  for (int k = 0; k < 6; ++k) out_off[k] = o[k];
  out_off[6] = o[5] + t[1];
  return LLSR_OK;
}

// The mapping chain's batched downsampleCurrentScan (llsr_mapping.h): one segmented VoxelGrid over
// clouds at arbitrary device addresses, all slots at once.
int32_t llsr_mapping::voxel_multi(llsr_map* m, const float4* const* src, const long long* n, const float* leaf,
                                  int S, float4* out, long long* out_off, hipStream_t s) {
  if (!m || S < 1) return LLSR_EINVAL;
  std::vector<VgCloud> cl(S);
  for (int k = 0; k < S; ++k) cl[k] = {src[k], n[k], leaf[k]};
  return vg_run(m, cl, out, out_off, s);
}

extern "C" int32_t llsr_map_add_keyframe(llsr_map* m, const float pose[6], const float* c, int32_t nc,
                                         const float* su, int32_t ns, const float* o, int32_t no, void* hip_stream) {
  if (!m || !pose || nc < 0 || ns < 0 || no < 0 || (nc && !c) || (ns && !su) || (no && !o))
    return mfail(m, LLSR_EINVAL, "add_keyframe: bad arguments");
  MAP_OK(m, hipSetDevice(m->device));
  const hipStream_t s = pick(m, hip_stream);
  const size_t need = m->store_used + (size_t)nc + ns + no;
  if (need > m->store_cap) {
    size_t n = m->store_cap ? m->store_cap : (size_t)1 << 20;
    while (n < need) n *= 2;
    float4* p = nullptr;
    MAP_OK(m, hipMalloc(&p, n * sizeof(float4)));
    if (m->store_used) MAP_OK(m, hipMemcpyAsync(p, m->store, m->store_used * sizeof(float4), hipMemcpyDeviceToDevice, s));
    MAP_OK(m, hipStreamSynchronize(s));
    if (m->store) MAP_OK(m, hipFree(m->store));
    m->store = p;
    m->store_cap = n;
  }
  llsr_map::Kf k{};
  std::memcpy(k.pose, pose, sizeof k.pose);
  const float* src[3] = {c, su, o};
  const int cnt[3] = {nc, ns, no};
  for (int a = 0; a < 3; ++a) {
    k.off[a] = (long long)m->store_used;
    k.n[a] = cnt[a];
    if (cnt[a])
      MAP_OK(m, hipMemcpyAsync(m->store + m->store_used, src[a], cnt[a] * sizeof(float4), hipMemcpyDefault, s));
    m->store_used += cnt[a];
  }
  m->kf.push_back(k);
  return (int32_t)m->kf.size() - 1;
}

// extractSurroundingKeyFrames (MO:1096-1232) of n maps at once, with `eng`'s VoxelGrid engine and
// buffers: one key-pose VoxelGrid over every map's poses in radius, one transform launch over every
// listed keyframe, one VoxelGrid over the n corner and n surf maps. The local maps land in eng's
// dsbuf: map i's corner map at [off_c[i], off_c[i+1]), its surf map at [off_s[i], off_s[i+1]).
int32_t llsr_mapping::extract_multi(llsr_map* eng, llsr_map* const* maps, int n, const float* pos,
                                    llsr_map_report* reps, const float4** out, long long* off_c, long long* off_s,
                                    hipStream_t s) {
  llsr_map* m = eng;
  if (!m || n < 1) return LLSR_EINVAL;
  const auto t0 = std::chrono::steady_clock::now();
  // radiusSearch (MO:1157-1159): d^2 = ((0 + dx^2) + dy^2) + dz^2 < float(r^2), over K poses
  // (radius-branch maps only; a loop-closure map selects no poses here)
  std::vector<float4> sel;
  std::vector<long long> sel_off(n + 1, 0);
  for (int i = 0; i < n; ++i) {
    llsr_map* mi = maps[i];
    std::memset(&reps[i], 0, sizeof reps[i]);
    const float r2 = (float)((double)mi->cfg.surrounding_radius * (double)mi->cfg.surrounding_radius);
    const int K = mi->cfg.enable_loop_closure ? 0 : (int)mi->kf.size();
    const size_t s0 = sel.size();
    for (int k = 0; k < K; ++k) {
      const float* p = mi->kf[k].pose;
      float d = 0;
      for (int a = 0; a < 3; ++a) {
        const float df = pos[3 * i + a] - p[a];
        d += df * df;
      }
      if (d < r2) sel.push_back(make_float4(p[0], p[1], p[2], (float)k));
    }
    reps[i].n_in_radius = (int32_t)(sel.size() - s0);
    sel_off[i + 1] = (long long)sel.size();
  }
  // surroundingKeyPosesDS (MO:1166-1167) on the device; intensity = the mean keyframe index
  std::vector<std::vector<int>> ds_ids(n);
  if (!sel.empty()) {
    const size_t P = sel.size();
    MAP_OK(m, grow(m->poses, m->cap_poses, 2 * P));
    MAP_OK(m, host_grow(m->hstage, m->cap_hstage, 2 * P * sizeof(float4)));
    std::memcpy(m->hstage, sel.data(), P * sizeof(float4));
    MAP_OK(m, hipMemcpyAsync(m->poses, m->hstage, P * sizeof(float4), hipMemcpyHostToDevice, s));
    std::vector<VgCloud> pc(n);
    for (int i = 0; i < n; ++i) pc[i] = {m->poses + sel_off[i], sel_off[i + 1] - sel_off[i], maps[i]->cfg.keypose_leaf};
    std::vector<long long> po(n + 1);
    int32_t rc = vg_run(m, pc, m->poses + P, po.data(), s);
    if (rc != LLSR_OK) return rc;
    float4* hds = reinterpret_cast<float4*>(m->hstage) + P;
    MAP_OK(m, hipMemcpyAsync(hds, m->poses + P, po[n] * sizeof(float4), hipMemcpyDeviceToHost, s));
    MAP_OK(m, hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i)
      for (long long q = po[i]; q < po[i + 1]; ++q) ds_ids[i].push_back((int)hds[q].w);
  }
  // MO:1169-1189: drop listed keyframes no downsampled pose names; MO:1190-1222: append new ones;
  // MO:1224-1228: corner map = corner clouds; surf map = surf + outlier clouds, in list order
  std::vector<XfChunk> xc;
  std::vector<long long> rc_off(n + 1, 0), rs_off(n + 1, 0);
  for (int i = 0; i < n; ++i) {
    llsr_map* mi = maps[i];
    std::vector<int>& ids = mi->sel.ids;
    const int K = (int)mi->kf.size();
    if (mi->cfg.enable_loop_closure) {
      // MO:1099-1145. cloudKeyPoses3D[i].intensity == i (MO:1695-1697), so thisKeyInd == i.
      const int N = mi->cfg.surrounding_keyframe_search_num;
      if ((int)ids.size() < N) {
        // queue not full: rebuild it from the newest keyframe backwards, push_front until N
        std::vector<int> q;
        for (int k = K - 1; k >= 0; --k) {
          q.push_back(k);
          if ((int)q.size() >= N) break;
        }
        ids.assign(q.rbegin(), q.rend());
        reps[i].n_transformed = (int32_t)ids.size();
      } else if (mi->sel.latest_frame_id != K - 1) {
        // full: pop the oldest, push the newest (only when a keyframe was added since)
        ids.erase(ids.begin());
        mi->sel.latest_frame_id = K - 1;
        ids.push_back(K - 1);
        reps[i].n_transformed = 1;
      }
    } else {
      reps[i].n_poses_ds = (int32_t)ds_ids[i].size();
      std::vector<int> kept;
      for (int id : ids)
        for (int d : ds_ids[i])
          if (d == id) { kept.push_back(id); break; }
      ids.swap(kept);
      for (int d : ds_ids[i]) {
        bool found = false;
        for (int id : ids)
          if (id == d) { found = true; break; }
        if (!found) {
          if (d < 0 || d >= K) return mfail(m, LLSR_ERANGE, "extract: key pose index out of range");
          ids.push_back(d);
          ++reps[i].n_transformed;
        }
      }
    }
    reps[i].n_keyframes = (int32_t)ids.size();
    long long nc = 0, ns = 0;
    for (int id : ids) nc += mi->kf[id].n[0];
    for (int id : ids) ns += mi->kf[id].n[1] + mi->kf[id].n[2];
    reps[i].n_corner_map = nc;
    reps[i].n_surf_map = ns;
    rc_off[i + 1] = rc_off[i] + nc;
    rs_off[i + 1] = rs_off[i] + ns;
  }
  const long long NC = rc_off[n], NS = rs_off[n];
  for (int i = 0; i < n; ++i) {
    llsr_map* mi = maps[i];
    long long dc = rc_off[i], dsf = NC + rs_off[i];
    auto add = [&](const llsr_map::Kf& k, int a, long long& dst) {
      for (int b = 0; b < k.n[a]; b += 1024) {
        XfChunk x{};
        x.src = mi->store + k.off[a] + b;
        x.dst = dst + b;
        x.n = std::min(1024, k.n[a] - b);
        std::memcpy(x.t, k.pose, sizeof x.t);
        xc.push_back(x);
      }
      dst += k.n[a];
    };
    for (int id : mi->sel.ids) {
      add(mi->kf[id], 0, dc);
      add(mi->kf[id], 1, dsf);
      add(mi->kf[id], 2, dsf);
    }
  }
  MAP_OK(m, grow(m->mapbuf, m->cap_map, (size_t)(NC + NS)));
  MAP_OK(m, grow(m->dsbuf, m->cap_ds, (size_t)(NC + NS)));
  if (!xc.empty()) {
    // hstage is free here: the key-pose VoxelGrid above ended with a stream sync
    const size_t bytes = xc.size() * sizeof(XfChunk);
    MAP_OK(m, host_grow(m->hstage, m->cap_hstage, bytes));
    MAP_OK(m, grow(m->dxf, m->cap_dxf, bytes));
    std::memcpy(m->hstage, xc.data(), bytes);
    MAP_OK(m, hipMemcpyAsync(m->dxf, m->hstage, bytes, hipMemcpyHostToDevice, s));
    k_map_transform<<<(int)xc.size(), 256, 0, s>>>(reinterpret_cast<const XfChunk*>(m->dxf), m->mapbuf);
    MAP_OK(m, hipGetLastError());
  }
  // MO:1225-1231: VoxelGrid corner / surf of every map
  std::vector<VgCloud> mc(2 * n);
  for (int i = 0; i < n; ++i) {
    mc[i] = {m->mapbuf + rc_off[i], rc_off[i + 1] - rc_off[i], maps[i]->cfg.corner_leaf};
    mc[n + i] = {m->mapbuf + NC + rs_off[i], rs_off[i + 1] - rs_off[i], maps[i]->cfg.surf_leaf};
  }
  std::vector<long long> o(2 * n + 1);
  const int32_t rc = vg_run(m, mc, m->dsbuf, o.data(), s);
  if (rc != LLSR_OK) return rc;
  for (int i = 0; i <= n; ++i) {
    off_c[i] = o[i];
    off_s[i] = o[n + i];
  }
  const float ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  for (int i = 0; i < n; ++i) {
    reps[i].n_corner_ds = o[i + 1] - o[i];
    reps[i].n_surf_ds = o[n + i + 1] - o[n + i];
    reps[i].ms = ms;
  }
  *out = m->dsbuf;
  return LLSR_OK;
}

extern "C" int32_t llsr_map_extract(llsr_map* m, const float pos[3], float* d_corner, int64_t cap_c, float* d_surf,
                                    int64_t cap_s, llsr_map_report* rep, void* hip_stream) {
  if (!m || !pos || !rep) return mfail(m, LLSR_EINVAL, "extract: bad arguments");
  const auto t0 = std::chrono::steady_clock::now();
  std::memset(rep, 0, sizeof *rep);
  MAP_OK(m, hipSetDevice(m->device));
  const hipStream_t s = pick(m, hip_stream);
  if (m->kf.empty()) return LLSR_OK;  // MO:1097
  const float4* out = nullptr;
  long long oc[2], os[2];
  int32_t rc = llsr_mapping::extract_multi(m, &m, 1, pos, rep, &out, oc, os, s);
  if (rc != LLSR_OK) return rc;
  if (rep->n_corner_ds > cap_c || rep->n_surf_ds > cap_s)
    return mfail(m, LLSR_ERANGE, "extract: local map exceeds the output capacity");
  if (rep->n_corner_ds && !d_corner) return mfail(m, LLSR_EINVAL, "extract: null corner output");
  if (rep->n_surf_ds && !d_surf) return mfail(m, LLSR_EINVAL, "extract: null surf output");
  if (rep->n_corner_ds)
    MAP_OK(m, hipMemcpyAsync(d_corner, out + oc[0], rep->n_corner_ds * sizeof(float4), hipMemcpyDeviceToDevice, s));
  if (rep->n_surf_ds)
    MAP_OK(m, hipMemcpyAsync(d_surf, out + os[0], rep->n_surf_ds * sizeof(float4), hipMemcpyDeviceToDevice, s));
  MAP_OK(m, hipStreamSynchronize(s));
  rep->ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return LLSR_OK;
}

extern "C" int32_t llsr_map_keyframe_ids(const llsr_map* m, int32_t* out, int32_t cap) {
  if (!m) return LLSR_EINVAL;
  const int n = (int)m->sel.ids.size();
  for (int k = 0; k < n && k < cap; ++k) out[k] = m->sel.ids[k];
  return n;
}
