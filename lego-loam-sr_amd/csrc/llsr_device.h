// llsr_device.h — shared device-side declarations: the per-batch configuration block, the
// handle's device buffers, and small wave/block primitives for CDNA4 (64-lane waves).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "llsr_libm.h"

namespace llsr {

// Per-slot counter words (counts[b * kCnt + ...]).
enum : int {
  C_NPTS = 0,      // finite input points
  C_FIRST = 1,     // first finite raw index (atomicMin)
  C_LAST = 2,      // last finite raw index (atomicMax)
  C_S = 3,         // segmented points
  C_O = 4,         // outliers
  C_K = 5,         // near-ground cloud size
  C_INL = 6,       // RANSAC inliers
  C_RIT = 7,       // RANSAC iterations
  C_M = 8,         // cornerPointsLessSharp
  C_SHARP = 9,     // cornerPointsSharp
  C_F = 10,        // surfPointsFlat (without shadow points)
  C_L = 11,        // surfPointsLessFlat
  C_HALF = 12,     // adjustDistortion halfPassed split index
  C_EXACT = 13,    // rings whose curvature sort took the exact libstdc++ path (ties)
  C_PHOUT = 14,    // rings where the carried cloudSmoothness[4] index fell outside the ring window
  kCnt = 16
};

// Everything a kernel needs to know about the sensor, precomputed on the host with the same
// float/double conversions as the reference constructors (IP:117-121, FA:152-154).
struct DevCfg {
  int H, W, HW;
  float ip_resX, ip_resY, ip_angBottom;
  float segThr, sinX, cosX, sinY, cosY;
  int use_kitti, gsi, pointNum, lineNum;
  float scan_period, edge_thr, surf_thr;
  float fa_resY, sinResX, RatioXY, RatioZ, DBFr;
  float gnd_cos[3];  // ground angle test thresholds on the cosine for D = 12.5, 60, 25 deg (llsr_libm.h)
  int ccl_lds;  // union-find parent array fits LDS (H <= 16 && HW <= 32000)
  int lbl_band; // otherwise: rows per LDS union-find band of k_label<false> (band * W ints <= 72 KB: two workgroups per CU)
  int exact_vg;   // LLSR_VOXEL_ORDER_PCL: the less-flat VoxelGrid sums in std::sort's tie order
  int dbg_phase;  // diagnostics only: kernels return at phase boundary >= dbg_phase (default: never)
};

// Device buffers owned by the handle; every per-slot array has stride HW (or H for rings).
struct DevBufs {
  int* counts;          // [B][kCnt]
  float* orient;        // [B][4]
  int* cell_pt;         // [B][HW] raw point index or -1
  float* range;         // [B][HW]
  float4* full;         // [B][HW] the kept raw point (x, y, z, raw intensity); NaN, NaN, NaN, 0 where
                        // empty. fullCloud's intensity row + col / 1e4 is derived (cell_intensity).
  int8_t* ground;       // [B][HW]
  int* label;           // [B][HW]
  float4* near_pts;     // [B][HW] near-ground cloud (w = cell index)
  int* shuf;            // [B][HW] RANSAC shuffled_indices_
  int* ccl_a;           // [B][HW] scratch (global-mode union-find parent / stats)
  unsigned long long* ccl_b;  // [B][HW] scratch (global-mode row masks)
  int* start_ring;      // [B][H]
  int* end_ring;        // [B][H]
  float4* seg;          // [B][HW] segmented cloud (IP frame)
  uint8_t* seg_ground;  // [B][HW] (zero beyond S: CloudInfo arrays have length H*W)
  uint32_t* seg_col;    // [B][HW]
  float* seg_range;     // [B][HW]
  float* seg_int;       // [B][HW]
  float4* outl;         // [B][HW]
  float* outl_int;      // [B][HW]
  float4* loam;         // [B][HW] segmented cloud after adjustDistortion
  float* curv;          // [B][HW]
  uint8_t* picked;      // [B][HW] FA carry-over state cloudNeighborPicked
  int8_t* clabel;       // [B][HW] FA carry-over state cloudLabel
  int* ring_cnt;        // [B][3][H] edges, flats, less-flat per ring
  int* edge_tmp;        // [B][HW] per-ring edge lists at their ring's start position
  int* flat_tmp;        // [B][HW]
  float4* lflat_tmp;    // [B][HW]
  int* less_sharp;      // [B][HW]
  int* cluster;         // [B][HW]
  int* sharp;           // [B][HW]
  int* flat;            // [B][HW]
  float4* lflat;        // [B][HW]
  float4* db_pts;       // [B][HW] DBSCAN point records: (x0, y0, z0, kxy)
  float* db_kz;         // [B][HW]
  uint32_t* db_adj;     // [B][kAdjCap][kAdjWords] eps-neighbourhood bitmask rows
  uint32_t* mt0;        // [624] RANSAC's mt19937 state after seed(12345) and its first twist
  int* phantom;         // [B] FA carry-over state: cloudSmoothness[4].ind (value is always 0)
  int* seg_zero;        // [B] seg_ground / seg_col / seg_range are zero on [seg_zero, HW) (k_segment's
                        // last S; HW after llsr_reset_state), so a batch clears only [S, seg_zero)
};

// C_HALF before k_fa_points when k_segment's first tile of cells holds no passing point
constexpr int kHalfUnknown = -2;

// adjustDistortion's first orientation branch (FA:578-583) and its halfPassed test (FA:584-586)
__device__ __forceinline__ float ori_branch1(float o, float start) {
  constexpr double kPi_ = 3.14159265358979323846;
  if ((double)o < (double)start - kPi_ / 2) o = (float)(o + 2 * kPi_);
  else if ((double)o > (double)start + kPi_ * 3 / 2) o = (float)(o - 2 * kPi_);
  return o;
}
// o = -atan2f(y, x) of a segmented point
__device__ __forceinline__ bool half_passed(float o, float start) {
  return (double)(ori_branch1(o, start) - start) > 3.14159265358979323846;
}

// halfPassed's test (FA:578-586) on o = -atan2f(y, x) from project_cell_fast's atan2 (|err| < 1e-6
// rad): with d = o - start its outcome changes only at d = -pi, -pi/2, pi and 3 pi / 2 (the branch
// cuts and the test, o + 2 pi and o - 2 pi folded in), so the approximation decides it exactly when
// d is 1e-5 away from each; otherwise, and for zero / huge operands, the exact libm path.
// 1 / 0: passes / fails, 2: undecided (take the exact path)
__device__ __forceinline__ int half_passed_fast(float y, float x, float start) {
  const float ax = fabsf(y), bx = fabsf(x);
  const float mx = fmaxf(ax, bx), mn = fminf(ax, bx);
  if (!(mn > 0.0f && mx < 1e30f)) return 2;
  const float t = mn * __builtin_amdgcn_rcpf(mx);
  const float u = t * t;
  float pa = __builtin_fmaf(u, -0x1.09b84ap-8f, 0x1.6633d8p-6f);
  pa = __builtin_fmaf(u, pa, -0x1.ca08a0p-5f);
  pa = __builtin_fmaf(u, pa, 0x1.8af1c2p-4f);
  pa = __builtin_fmaf(u, pa, -0x1.1cd946p-3f);
  pa = __builtin_fmaf(u, pa, 0x1.988174p-3f);
  pa = __builtin_fmaf(u, pa, -0x1.554c3ap-2f);
  pa = __builtin_fmaf(u, pa, 0x1.ffffeap-1f);
  float ha = pa * t;
  ha = ax > bx ? 1.57079637f - ha : ha;
  ha = x < 0.0f ? 3.14159274f - ha : ha;
  ha = y < 0.0f ? -ha : ha;
  const double dd = (double)-ha - (double)start;
  constexpr double kPi_ = 3.14159265358979323846, e = 1e-5;
  if (!(fabs(dd + kPi_) > e && fabs(dd + kPi_ / 2) > e && fabs(dd - kPi_) > e && fabs(dd - 1.5 * kPi_) > e)) return 2;
  return (dd < -kPi_ / 2 ? dd > -kPi_ : (dd <= 1.5 * kPi_ && dd > kPi_)) ? 1 : 0;
}
__device__ __forceinline__ bool half_passed_any(float y, float x, float start) {
  const int r = half_passed_fast(y, x, start);
  return r == 2 ? half_passed(-llsr_libm::atan2f_(y, x), start) : r == 1;
}

// DBSCAN adjacency capacity per scan (edge candidates); larger M falls back to on-the-fly rows.
constexpr int kAdjCap = 2048;
constexpr int kAdjWords = kAdjCap / 32;

// fullCloud's intensity of cell (row i, col j): (float)(i + j / 10000.0) (IP:341); the double
// division is a multiply by 1e-4 where both give the same float (tests/test_oracle.py)
__device__ __forceinline__ float cell_intensity(int H, int W, int i, int j) {
  return (float)((double)(float)i + (H <= 256 && W <= 8192 ? (double)(float)j * 1e-4 : (double)(float)j / 10000.0));
}

// ---- wave / block primitives (wave64) ------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// __ballot of a bool: HIP's __ballot takes an int, which the backend materialises per lane and
// compares against zero again (two VALU instructions per ballot in the sort's partition loops)
__device__ __forceinline__ unsigned long long ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// lanes 0 .. n-1 as a wave mask (n clamped to [0, 64]; uniform n: scalar instructions only)
__device__ __forceinline__ unsigned long long lanes_below(int n) {
  return n >= 64 ? ~0ull : n <= 0 ? 0ull : (1ull << n) - 1ull;
}

// set bits of m below this lane, __popcll(m & ((1ull << lane) - 1)), as two mbcnt instructions
// (the and / popcount form costs four and keeps the lane mask in two registers)
__device__ __forceinline__ int lane_rank(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Lane exchanges as VALU ops (ds_bpermute, what __shfl_* compile to, queues in the LDS pipe):
// DPP row / quad permutations and gfx950's v_permlane16/32_swap.
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {  // v of lane (lane ^ J), J < 64
  const int l = threadIdx.x & 63;
  if constexpr (J == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  } else if constexpr (J == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
  } else if constexpr (J == 4) {  // row_ror:n: lane i reads lane (i - n) mod 16 of its row
    const uint32_t a = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false);
    const uint32_t b = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x12C, 0xf, 0xf, false);
    return (l & 4) ? a : b;
  } else if constexpr (J == 8) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);
  } else if constexpr (J == 16) {  // odd 16-lane rows of the first operand <-> even rows of the second
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (l & 16) ? r[0] : r[1];
  } else {  // upper 32 lanes of the first operand <-> lower 32 of the second
    static_assert(J == 32, "lane_xor: J < 64");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (l & 32) ? r[0] : r[1];
  }
}
template <int J>
__device__ __forceinline__ uint64_t lane_xor(uint64_t v) {
  return ((uint64_t)lane_xor<J>((uint32_t)(v >> 32)) << 32) | lane_xor<J>((uint32_t)v);
}
template <int J, class T>
__device__ __forceinline__ T lane_xor_t(T v) {  // any 4- or 8-byte type
  if constexpr (sizeof(T) == 4) return __builtin_bit_cast(T, lane_xor<J>(__builtin_bit_cast(uint32_t, v)));
  else return __builtin_bit_cast(T, lane_xor<J>(__builtin_bit_cast(uint64_t, v)));
}

// inclusive scan (32-bit integers): DPP row_shr within 16-lane rows, then row_bcast:15 / :31
template <class T>
__device__ __forceinline__ T wave_incl_scan_add(T x) {
  static_assert(sizeof(T) == 4, "wave_incl_scan_add: 32-bit integers");
  const int l = lane_id(), rl = l & 15;
  int v = (int)x, t;
  t = __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, false); if (rl >= 1) v += t;   // row_shr:1
  t = __builtin_amdgcn_mov_dpp(v, 0x112, 0xf, 0xf, false); if (rl >= 2) v += t;   // row_shr:2
  t = __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, false); if (rl >= 4) v += t;   // row_shr:4
  t = __builtin_amdgcn_mov_dpp(v, 0x118, 0xf, 0xf, false); if (rl >= 8) v += t;   // row_shr:8
  t = __builtin_amdgcn_mov_dpp(v, 0x142, 0xf, 0xf, false); if ((l & 31) >= 16) v += t;  // row_bcast:15
  t = __builtin_amdgcn_mov_dpp(v, 0x143, 0xf, 0xf, false); if (l >= 32) v += t;   // row_bcast:31
  return (T)v;
}

template <class T>
__device__ __forceinline__ T wave_reduce_add(T x) {
  x += lane_xor_t<32>(x); x += lane_xor_t<16>(x); x += lane_xor_t<8>(x);
  x += lane_xor_t<4>(x); x += lane_xor_t<2>(x); x += lane_xor_t<1>(x);
  return x;
}

template <class T>
__device__ __forceinline__ T wave_reduce_min(T x) {
  T y;
  y = lane_xor_t<32>(x); x = y < x ? y : x;
  y = lane_xor_t<16>(x); x = y < x ? y : x;
  y = lane_xor_t<8>(x); x = y < x ? y : x;
  y = lane_xor_t<4>(x); x = y < x ? y : x;
  y = lane_xor_t<2>(x); x = y < x ? y : x;
  y = lane_xor_t<1>(x); x = y < x ? y : x;
  return x;
}

template <class T>
__device__ __forceinline__ T wave_reduce_max(T x) {
  T y;
  y = lane_xor_t<32>(x); x = y > x ? y : x;
  y = lane_xor_t<16>(x); x = y > x ? y : x;
  y = lane_xor_t<8>(x); x = y > x ? y : x;
  y = lane_xor_t<4>(x); x = y > x ? y : x;
  y = lane_xor_t<2>(x); x = y > x ? y : x;
  y = lane_xor_t<1>(x); x = y > x ? y : x;
  return x;
}

// Exclusive prefix sum over the block; `tmp` holds >= blockDim/64 ints of LDS.
// Returns the exclusive prefix of v; *total receives the block sum. Contains barriers.
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* total) {
  const int l = lane_id(), w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  int x = wave_incl_scan_add(v);
  if (l == 63) tmp[w] = x;
  __syncthreads();
  if (w == 0) {
    int t = l < nw ? tmp[l] : 0;
    t = wave_incl_scan_add(t);
    if (l < nw) tmp[l] = t;
  }
  __syncthreads();
  int pre = w ? tmp[w - 1] : 0;
  *total = tmp[nw - 1];
  __syncthreads();
  return pre + x - v;
}

__device__ __forceinline__ int block_reduce_add(int v, int* tmp) {
  int t;
  block_excl_scan(v, tmp, &t);
  return t;
}

__device__ __forceinline__ int block_reduce_min(int v, int* tmp) {
  const int l = lane_id(), w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_reduce_min(v);
  if (l == 0) tmp[w] = v;
  __syncthreads();
  int r = tmp[0];
  for (int k = 1; k < nw; ++k) r = tmp[k] < r ? tmp[k] : r;
  __syncthreads();
  return r;
}

// x86-64 truncating conversions (cvttss2si / cvttsd2si): NaN / out of range -> INT_MIN.
__host__ __device__ __forceinline__ int trunc_i32(double v) {
  if (!(v > -2147483649.0 && v < 2147483648.0)) return (int)0x80000000;
  return (int)v;
}

}  // namespace llsr
