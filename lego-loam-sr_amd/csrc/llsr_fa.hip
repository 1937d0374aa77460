// llsr_fa.hip — FeatureAssociation feature stage on gfx950 (featureAssociation.cpp = FA,
// lines 565-899 and 1159-1387): LOAM-frame swap + relative time, curvature, occlusion masks,
// per-ring greedy edge/flat selection, per-ring VoxelGrid of less-flat points, DBSCAN edge
// refinement. Built with -ffp-contract=off; float order follows the reference exactly.
#include <cfloat>
#include <climits>

#include "llsr_device.h"
#include "llsr_isort.h"
#include "llsr_libm.h"

namespace llsr {

using namespace llsr_libm;
constexpr double kPi = 3.14159265358979323846;

// ---------------------------------------------------------------------------------------------
// K7 per-point stage: adjustDistortion (FA:565-598), calculateSmoothnessOurs (FA:817-848),
// markOccludedPoints (FA:851-899). One workgroup (256 threads) per (tile of kFaTile segmented
// points, scan): ~17 tiles of a VLP-16 scan in flight at once instead of one workgroup walking them.
// halfPassed is a one-way latch, so the serial loop equals: points up to the first index whose
// first-branch orientation passes start + pi use branch 1, later ones branch 2; k_segment leaves
// that index in C_HALF (kHalfUnknown when its first tile holds none, then each workgroup finds it).
// Curvature reads an LDS tile of LOAM points with a +-5 halo. Occlusion writes become a gather
// over the +-6 window of per-point flags. FA carry-over arrays (picked, cloudLabel) are per slot.
// ---------------------------------------------------------------------------------------------
constexpr int kFaT = 256;
constexpr int kFaTile = 4 * kFaT - 12;  // 1012 points: with the +-5 point halo and the +-6 flag halo, 4 slots per lane

// LOAM-frame point of segmented point i (FA:565-598): orientation branch by the halfPassed latch
// (`first`), relative time, intensity = ring + scan_period * relTime.
__device__ __forceinline__ float4 loam_point(const DevCfg& c, float4 p, int i, int first, float start, float endo,
                                             float diff) {
  float o = -atan2f_(p.y, p.x);  // point.x = y, point.z = x (FA:573-577)
  if (i <= first) {
    o = ori_branch1(o, start);
  } else {
    o = (float)(o + 2 * kPi);
    if ((double)o < (double)endo - kPi * 3 / 2) o = (float)(o + 2 * kPi);
    else if ((double)o > (double)endo + kPi / 2) o = (float)(o - 2 * kPi);
  }
  const float relTime = (o - start) / diff;
  const float inten = (float)(int)(p.w) + c.scan_period * relTime;
  return make_float4(p.y, p.z, p.x, inten);
}

__global__ __launch_bounds__(kFaT) void k_fa_points(DevCfg c, DevBufs d) {
  constexpr int kTile = kFaTile;
  __shared__ float4 tp[kTile + 10];
  __shared__ uint8_t fl[kTile + 12];  // bit0 A_i, bit1 B_i, bit2 C_i for i in [t0-6, t0+T+6)
  __shared__ int tmp[kFaT / 64];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * kTile;
  const size_t base = (size_t)b * c.HW;
  const int tid = threadIdx.x;
  constexpr int nt = kFaT;
  const int* cnt = d.counts + b * kCnt;
  const int S = cnt[C_S];
  if (t0 >= S) return;
  const float start = d.orient[b * 4 + 0], endo = d.orient[b * 4 + 1], diff = d.orient[b * 4 + 2];
  const float4* seg = d.seg + base;
  float4* loam = d.loam + base;

  int first = cnt[C_HALF];  // nothing writes it during this launch: uniform over the workgroup
  if (first == kHalfUnknown) {
    // the latch lies past k_segment's first tile (or nowhere): the smallest passing index, chunk
    // by chunk (later chunks only hold larger indices)
    first = INT_MAX;
    for (int c0 = 0; c0 < S; c0 += 4 * nt) {
      const int i0 = c0 + tid;
      float4 pp[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) pp[u] = i0 + u * nt < S ? seg[i0 + u * nt] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * nt;
        if (i >= S) continue;
        if (i < first && half_passed_any(pp[u].y, pp[u].x, start)) first = i;
      }
      first = block_reduce_min(first, tmp);
      if (first != INT_MAX) break;
    }
  }

  const float* rng = d.seg_range + base;
  const uint32_t* col = d.seg_col + base;
  uint8_t* picked = d.picked + base;
  int8_t* clabel = d.clabel + base;
  float* curv = d.curv + base;
  // ONE round of loads: the tile's points with their +-5 halo and the occlusion inputs (range,
  // column of i; the neighbours' from the adjacent lanes, the wave's edge lanes loading their one
  // outside value), all in flight together. Slot q = tid + u * nt of both covers [0, 4 nt).
  const int ln = lane_id();
  float4 pp[4];
  float r1[4], rx[4];
  uint32_t c1[4], cx[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = tid + u * nt, k = t0 - 5 + q;
    pp[u] = (q < kTile + 10 && k >= 0 && k < S) ? seg[k] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = tid + u * nt, i = t0 - 6 + q;
    const bool in = i >= 0 && i < S;
    r1[u] = in ? rng[i] : 0.0f;
    c1[u] = in ? col[i] : 0u;
    const int ie = ln == 0 ? i - 1 : i + 1;  // lane 0: i - 1; lane 63: i + 1 (the others unused)
    const bool ine = (ln == 0 || ln == 63) && ie >= 0 && ie < S;
    rx[u] = ine ? rng[ie] : 0.0f;
    cx[u] = ine ? col[ie] : 0u;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = tid + u * nt, k = t0 - 5 + q;
    if (q >= kTile + 10) continue;
    if (k >= 0 && k < S) {
      const float4 lp = loam_point(c, pp[u], k, first, start, endo, diff);
      tp[q] = lp;
      if (q >= 5 && q < kTile + 5) loam[k] = lp;
    } else {
      tp[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  // occlusion flags of the tile (+ halo)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int q = tid + u * nt, i = t0 - 6 + q;
    const float up = __shfl_up(r1[u], 1, 64), dn = __shfl_down(r1[u], 1, 64);
    const uint32_t cdn = (uint32_t)__shfl_down((int)c1[u], 1, 64);
    uint8_t f = 0;
    if (i >= 5 && i < S - 6) {
      const float r0 = ln == 0 ? rx[u] : up, r2 = ln == 63 ? rx[u] : dn;
      const uint32_t c2 = ln == 63 ? cx[u] : cdn;
      const float d1 = r1[u], d2 = r2;
      const int colDiff = abs((int)(c2 - c1[u]));
      if (colDiff < 10) {
        if ((double)(d1 - d2) > 0.3) f |= 1;
        else if ((double)(d2 - d1) > 0.3) f |= 2;
      }
      const float diff1 = fabs_((float)(r0 - r1[u]));
      const float diff2 = fabs_((float)(r2 - r1[u]));
      if ((double)diff1 > 0.02 * (double)r1[u] && (double)diff2 > 0.02 * (double)r1[u]) f |= 4;
    }
    fl[q] = f;
  }
  __syncthreads();
  for (int q0 = tid; q0 < kTile; q0 += nt) {
    const int k = t0 + q0;
    if (k >= S) break;
    const bool inner = k >= 5 && k < S - 5;
    float cv = 0.0f;
    if (inner) {
      const int q = q0 + 5;
      float dx = 0.f, dy = 0.f, dz = 0.f;
#pragma unroll
      for (int m = -5; m < 6; ++m) dx += tp[q + m].x;
      dx -= 11 * tp[q].x;
#pragma unroll
      for (int m = -5; m < 6; ++m) dy += tp[q + m].y;
      dy -= 11 * tp[q].y;
#pragma unroll
      for (int m = -5; m < 6; ++m) dz += tp[q + m].z;
      dz -= 11 * tp[q].z;
      const float4 p = tp[q];
      cv = sqrt_(dx * dx + dy * dy + dz * dz) / sqrt_(p.x * p.x + p.y * p.y + p.z * p.z) / 10;
    }
    curv[k] = cv;
    // picked[k]: reset on [5, S-5) by the smoothness loop, then any occlusion write
    bool occ = false;
    const int fq = q0 + 6;  // fl index of i = k
    if (fl[fq] & 4) occ = true;
#pragma unroll
    for (int m = 0; m <= 5; ++m) occ |= (fl[fq + m] & 1) != 0;   // A_i, i in [k, k+5]
#pragma unroll
    for (int m = 1; m <= 6; ++m) occ |= (fl[fq - m] & 2) != 0;   // B_i, i in [k-6, k-1]
    const uint8_t old = inner ? (uint8_t)0 : picked[k];  // only the 10 edge points keep theirs
    picked[k] = old | (occ ? (uint8_t)1 : (uint8_t)0);
    if (inner) clabel[k] = 0;
  }
}

void launch_fa_points(const DevCfg& c, const DevBufs& d, int B, hipStream_t s) {
  k_fa_points<<<dim3((c.HW + kFaTile - 1) / kFaTile, B), kFaT, 0, s>>>(c, d);
}

// ---------------------------------------------------------------------------------------------
// K8 per-ring selection (FA:1165-1271). One workgroup (256 threads) per (scan, ring).
// Reference order: cloudSmoothness[sp, ep) sorted by value (ties by index here; the reference's
// introsort leaves tie order unspecified), position 4 = the never-overwritten phantom {0, ind 0}
// (FA:169, 819), position ep unsorted. The edge loop visits ep, then ep-1..sp; the flat loop
// sp..ep. An entry can only be selected if it passes the static tests (threshold, ground flag,
// not already picked before the loop), and skipping entries that fail them does not change what
// the loop does to the others. So the block compacts the statically eligible entries, sorts only
// those, and lane 0 replays the serial loop over them against an LDS window [sp-5, ep+5] of
// picked/col/ground/label. Ring windows are disjoint (11 positions separate ep_r and sp_{r+1}).
// Less-flat points are then compacted and voxel-downsampled (PCL VoxelGrid, leaf 0.2).
// ---------------------------------------------------------------------------------------------
constexpr int kRingMax = 2048;  // >= max W
constexpr int kWin = kRingMax + 16;

// Block sort of n2 (power of two, 256 <= n2 <= 64 * 4 * 8) keys (u64 or u32) in LDS, ascending, by
// the 4 waves of the workgroup, the bitonic network with every stage whose partners lie in one wave
// run in registers: lane exchanges through DPP row / quad permutations and gfx950's
// v_permlane16/32_swap (VALU ops; ds_bpermute sits in the LDS queue), partners 64 or more apart
// between a lane's own registers. Only the stages that pair different waves' quarters read the LDS
// (each wave computes its own positions' results from the values it needs), so a sort costs five
// barriers. The full bitonic network's compare-exchanges (padding ~0 keys stay at the end).
// One compare-exchange of a key with its partner's value o: the min when this position takes the
// min (lower index of an ascending pair or upper of a descending one), else the max. Equal keys
// are interchangeable. One compare, the mask flip and a select per 32-bit word.
template <class T>
__device__ __forceinline__ T cx(T v, T o, bool want_min) {
  return ((o < v) == want_min) ? o : v;
}
// Stages J, J/2, ..., 1 of a bitonic merge of size SZ on the keys v[k] at positions base + 64 k + lane
// (SZ <= 64 K: direction from the position; SZ > 64 K: `up` for the whole wave).
template <int K, int SZ, int J, class T>
__device__ __forceinline__ void wave_merge(T (&v)[K], int base, bool up_all) {
  const int lane = threadIdx.x & 63;
  if constexpr (J >= 64) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      constexpr int d = J >> 6;
      if ((k & d) == 0) {
        const bool up = SZ > 64 * K ? up_all : (((base + k * 64) & SZ) == 0);
        const T a = v[k], b = v[k + d];
        const bool sw = (b < a) == up;
        v[k] = sw ? b : a;
        v[k + d] = sw ? a : b;
      }
    }
  } else {
    const bool lower = (lane & J) == 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const bool up = SZ > 64 * K ? up_all : (((base + k * 64 + lane) & SZ) == 0);
      v[k] = cx(v[k], lane_xor<J>(v[k]), lower == up);
    }
  }
  if constexpr (J > 1) wave_merge<K, SZ, J / 2>(v, base, up_all);
}
template <int K, int SZ, class T>
__device__ __forceinline__ void wave_sort_from(T (&v)[K], int base) {
  wave_merge<K, SZ, SZ / 2>(v, base, true);
  if constexpr (SZ < 64 * K) wave_sort_from<K, SZ * 2>(v, base);
}
template <int K, class T>
__device__ void block4_sort_k(T* key) {
  constexpr int Q = 64 * K;  // keys per wave, position w Q + 64 k + lane
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  T v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = key[w * Q + k * 64 + lane];
  // every quarter sorted with the full network's directions below size Q (up = position & size == 0)
  wave_sort_from<K, 2>(v, w * Q);
  // merge of size 2Q (ascending for waves 0-1, descending for 2-3): stage Q pairs wave w with w ^ 1
  const bool up2 = (w & 2) == 0;
#pragma unroll
  for (int k = 0; k < K; ++k) key[w * Q + k * 64 + lane] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = cx(v[k], key[(w ^ 1) * Q + k * 64 + lane], ((w & 1) == 0) == up2);
  wave_merge<K, 2 * Q, Q / 2>(v, w * Q, up2);
  __syncthreads();
  // merge of size 4Q, ascending: stages 2Q (w with w ^ 2) and Q (w with w ^ 1) from the four values
  // of the position group, then the in-wave stages
#pragma unroll
  for (int k = 0; k < K; ++k) key[w * Q + k * 64 + lane] = v[k];
  __syncthreads();
  const bool lo2 = (w & 2) == 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int p = k * 64 + lane;
    const T a = cx(v[k], key[(w ^ 2) * Q + p], lo2);                // this position after stage 2Q
    const T b = cx(key[(w ^ 1) * Q + p], key[(w ^ 3) * Q + p], lo2);  // its stage-Q partner after 2Q
    v[k] = cx(a, b, (w & 1) == 0);
  }
  wave_merge<K, 4 * Q, Q / 2>(v, w * Q, true);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) key[w * Q + k * 64 + lane] = v[k];
  __syncthreads();
}
// n2 <= 128 keys: wave 0 alone, in registers
template <int K, class T>
__device__ void wave0_sort_k(T* key) {
  if (threadIdx.x < 64) {
    T v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = key[k * 64 + threadIdx.x];
    wave_sort_from<K, 2>(v, 0);
#pragma unroll
    for (int k = 0; k < K; ++k) key[k * 64 + threadIdx.x] = v[k];
  }
  __syncthreads();
}
// n2 = 64 * K for K in {1, 2, 4, 8, 16, 32}
template <class T>
__device__ void block4_sort(T* key, int n2) {
  switch (n2) {
    case 64: wave0_sort_k<1>(key); break;
    case 128: wave0_sort_k<2>(key); break;
    case 256: block4_sort_k<1>(key); break;
    case 512: block4_sort_k<2>(key); break;
    case 1024: block4_sort_k<4>(key); break;
    default: block4_sort_k<8>(key); break;
  }
}

__device__ __forceinline__ int pow2_ceil(int n) {
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  return n2;
}

// Diagnostics (llsr_debug_exact_sort): the exact std::sort k_select_ring runs (block_introsort,
// 256 threads) on one array of n <= kRingMax values; out receives the original positions in sorted
// order.
__global__ __launch_bounds__(256) void k_debug_exact_sort(const float* vals, int n, int* out, long long* prof) {
  __shared__ uint64_t key[kRingMax];
  __shared__ uint16_t Lp[kRingMax], Rp[kRingMax];
  __shared__ BlockSortLds bsl;
  for (int t = threadIdx.x; t < n; t += 256) key[t] = ((uint64_t)__float_as_uint(vals[t]) << 32) | (uint32_t)t;
  __syncthreads();
  long long t0 = 0;
  if (prof && threadIdx.x == 0) t0 = clock64();
  block_introsort<256>(key, n, Lp, Rp, bsl, CurvLess{}, prof ? prof + 1 : nullptr);
  if (prof && threadIdx.x == 0) prof[0] = clock64() - t0;
  for (int t = threadIdx.x; t < n; t += 256) out[t] = (int)(uint32_t)key[t];
}

// Diagnostics (llsr_debug_exact_sort32): the PCL-order VoxelGrid's sort on 32-bit keys (rank << 11 |
// position, VoxLess32) of n <= kRingMax ranks < 2^21, as k_vox_pcl runs it (block_introsort, 256
// threads); out receives the original positions in sorted order.
__global__ __launch_bounds__(256) void k_debug_exact_sort32(const uint32_t* ranks, int n, int* out) {
  __shared__ uint32_t key[kRingMax];
  __shared__ uint16_t Lp[kRingMax], Rp[kRingMax];
  __shared__ BlockSortLds bsl;
  for (int t = threadIdx.x; t < n; t += 256) key[t] = (ranks[t] << 11) | (uint32_t)t;
  block_introsort<256>(key, n, Lp, Rp, bsl, VoxLess32{});
  __syncthreads();
  for (int t = threadIdx.x; t < n; t += 256) out[t] = (int)(key[t] & 0x7ffu);
}

// Serial greedy pick (FA:1175-1259) over a candidate list already in visiting order, by one wave:
// each chunk of 64 candidates reads `picked` once; the first still-alive candidate is selected,
// candidates inside its suppression interval die, repeat. Steps per chunk = picks in the chunk.
// Returns the number selected; writes labels, picked and the output list in selection order.
// wflag[w]: bits 0-2 forward reach, 3-5 backward reach, 6 ground, 7 picked (k_select_ring).
template <class Order>
__device__ __forceinline__ int greedy_wave(Order order, int nc, int ws, uint8_t* wflag, int8_t* wlab, int8_t lab,
                                           int* outp) {
  const int l = lane_id();
  const unsigned long long lt = (1ull << l) - 1ull;
  int nsel = 0;
  for (int t0 = 0; t0 < nc; t0 += 64) {
    const int t = t0 + l;
    const bool valid = t < nc;
    const int ind = valid ? order(t) : 0;
    const int w = valid ? ind - ws : 0;
    const int r = valid ? wflag[w] : 0x80;
    bool alive = valid && (r & 0x80) == 0;
    const int lo = w - ((r >> 3) & 7), hi = w + (r & 7);
    unsigned long long sel = 0ull;
    unsigned long long m = __ballot(alive);
    while (m) {
      const int s = __ffsll((long long)m) - 1;
      const int slo = __builtin_amdgcn_readlane(lo, s), shi = __builtin_amdgcn_readlane(hi, s);  // s is uniform
      sel |= 1ull << s;
      if (l > s && w >= slo && w <= shi) alive = false;
      if (l == s) alive = false;
      m = __ballot(alive);
    }
    if ((sel >> l) & 1ull) {
      wlab[w] = lab;
      outp[nsel + __popcll(sel & lt)] = ind;
      // other bits of the bytes are static during the passes: concurrent read-or-writes agree
      for (int q = lo; q <= hi; ++q) wflag[q] = (uint8_t)(wflag[q] | 0x80);
    }
    nsel += __popcll(sel);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  return nsel;
}

__global__ __launch_bounds__(256, 5) void k_select_ring(DevCfg c, DevBufs d) {
  // LDS < 32 KB -> 5 workgroups per CU. The window keeps two bytes per position: a flag byte
  // (suppression reach forward | backward << 3 (FA:1186-1205), ground << 6, picked << 7) and the
  // label; the VoxelGrid's voxel ids use key[] (dead after the greedy passes); the greedy passes read
  // the visiting order straight from the sorted keys.
  __shared__ uint64_t key[kRingMax];
  __shared__ uint32_t win_raw[2 * kWin / 4];
  uint8_t* wflag = reinterpret_cast<uint8_t*>(win_raw);
  int8_t* wlab = reinterpret_cast<int8_t*>(wflag + kWin);
  __shared__ uint16_t cfirst[kWin / 64 + 1];  // column of the first position of every 64
  __shared__ uint16_t cpos[kRingMax];
  __shared__ uint16_t rstart[kRingMax + 1];
  __shared__ int tmp[8];
  __shared__ float red[6][4];
  __shared__ int s_cnt;
  const int i = blockIdx.x, b = blockIdx.y;
  const int H = c.H, HW = c.HW;
  const size_t base = (size_t)b * HW;
  const int tid = threadIdx.x, nt = blockDim.x;
  int* rc = d.ring_cnt + (size_t)b * 3 * H;
  const int sp = d.start_ring[b * H + i];
  const int ep = d.end_ring[b * H + i] - 1;
  if (sp >= ep) {
    if (tid == 0) { rc[i] = 0; rc[H + i] = 0; rc[2 * H + i] = 0; }
    return;
  }
  const float* curv = d.curv + base;
  const int ws = sp - 5 > 0 ? sp - 5 : 0;
  const int we = ep + 5 < HW - 1 ? ep + 5 : HW - 1;
  const int wn = we - ws + 1;
  if (c.dbg_phase <= -2) return;
  // the whole window (and its curvatures, kept in registers for both candidate passes) is loaded
  // in one round trip: kPer positions per lane, all loads in flight together (blockDim.x == 256)
  constexpr int kPer = (kWin + 255) / 256;
  float cvr[kPer];
  uint32_t cl[kPer];
  uint32_t pkm = 0, gdm = 0;  // picked / ground bit per slot
  {
    uint8_t pk[kPer], gd[kPer];
    int8_t lb[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int t = tid + u * 256, pos = ws + t;
      cl[u] = 0;
      if (t < wn) {
        pk[u] = d.picked[base + pos];
        gd[u] = d.seg_ground[base + pos];
        lb[u] = d.clabel[base + pos];
        cl[u] = d.seg_col[base + pos];
        cvr[u] = curv[pos];
      }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int t = tid + u * 256;
      if (t < wn) {
        wlab[t] = lb[u];
        pkm |= (pk[u] != 0 ? 1u : 0u) << u;
        gdm |= (gd[u] != 0 ? 1u : 0u) << u;
        if ((t & 63) == 0) cfirst[t >> 6] = (uint16_t)cl[u];
      }
    }
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  if (c.dbg_phase <= -1) return;
  // Marking from `ind` runs forward while consecutive column gaps stay <= 10 (at most 5 steps,
  // stopping at H*W) and likewise backward (stopping at 0). Column indices are static, so the
  // reach of every selectable position is computed up front: one bit per window position marks a
  // stop between t and t + 1 (a gap > 10 or the window end, which also bounds H*W), and the
  // forward / backward reach is the distance to the nearest stop bit (ctz / clz of 64 bits).
  {
    uint64_t* gbits = reinterpret_cast<uint64_t*>(key);  // key[] is free until the edge candidates
    const int l = lane_id();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int t = tid + u * 256;
      const int dn = __shfl_down((int)cl[u], 1, 64);
      const int nx = l < 63 ? dn : (t + 1 < wn ? (int)cfirst[(t + 1) >> 6] : 0);
      const bool stop = t + 1 >= wn || abs(nx - (int)cl[u]) > 10;
      const uint64_t m = __ballot(t < wn && stop);
      if (l == 0 && (t >> 6) <= (wn >> 6)) gbits[t >> 6] = m;
    }
    __syncthreads();
    const int nw = (wn >> 6) + 1;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int t = tid + u * 256;
      if (t >= wn) break;
      const int k = t >> 6, sh = t & 63;
      uint64_t fw = gbits[k] >> sh;
      if (sh && k + 1 < nw) fw |= gbits[k + 1] << (64 - sh);
      const int f = fw ? min(5, __ffsll((long long)fw) - 1) : 5;
      int bk = 0;
      if (t > 0) {
        const int q = t - 1, kq = q >> 6, s2 = q & 63;
        uint64_t bw = gbits[kq] << (63 - s2);
        if (s2 < 63 && kq > 0) bw |= gbits[kq - 1] >> (s2 + 1);
        bk = min(min(5, t), bw ? (int)__clzll((long long)bw) : 64);
      }
      wflag[t] = (uint8_t)(f | (bk << 3) | (((gdm >> u) & 1u) << 6) | (((pkm >> u) & 1u) << 7));
    }
  }
  __syncthreads();
  // ---- the sorted range [sp, ep) of cloudSmoothness (FA:1172) ----
  // Position 4 (ring 0's sp) holds whatever the previous frame's ring-0 sort left there: value 0
  // (it is always a minimum) and a carried index `ph` (0 until an exact zero displaces it).
  const int nRng = ep - sp;
  const int ph = sp == 4 ? d.phantom[b] : 0;
  const bool ph_in = ph >= ws && ph - ws < wn;
  const float ph_curv = ph < 5 ? 0.0f : curv[ph];  // cloudCurvature[0..4] is never written (FA:819)
  if (sp == 4 && !ph_in && tid == 0) atomicAdd(&d.counts[b * kCnt + C_PHOUT], 1);
  __shared__ BlockSortLds bsl;  // block_introsort's top ranges and per-wave stacks
  __shared__ int s_flag, s_exact;
  // exact-order triggers: ties between eligible keys (found after each fast sort) and, in ring 0, an
  // exact zero that could take position 4 from the phantom for the next frame
  if (tid == 0) s_flag = 0;
  __syncthreads();
  if (sp == 4) {
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int p = ws + tid + u * 256;
      if (p >= 5 && p < ep && cvr[u] == 0.0f) s_flag = 1;
    }
  }
  // curvature of an entry's index as the eligibility tests read it (cloudCurvature[ind])
  auto curv_of = [&](int ind) { return ind < 5 ? 0.0f : curv[ind]; };
  // key[0, nRng) = the full range sorted exactly as std::sort leaves it; updates the phantom
  auto exact_sort = [&]() {
    for (int t = tid; t < nRng; t += nt) {
      const int p = sp + t;
      const float v = p == 4 ? 0.0f : curv[p];
      const int ind = p == 4 ? ph : p;
      key[t] = ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)ind;
    }
    block_introsort<256>(key, nRng, cpos, rstart, bsl, CurvLess{});
    if (tid == 0) {
      if (sp == 4) d.phantom[b] = (int)(uint32_t)key[0];
      atomicAdd(&d.counts[b * kCnt + C_EXACT], 1);
      s_exact = 1;
    }
    __syncthreads();
  };
  // compaction of the exactly sorted entries passing `elig`, in visiting order (descending for the
  // edge loop, ascending for the flat loop), into cpos; wave 0; returns the count
  auto compact_sorted = [&](bool descending, auto elig) {
    const int l = lane_id();
    int cnt = 0;
    for (int c0 = 0; c0 < nRng; c0 += 64) {
      const int k = c0 + l;
      const int t = descending ? nRng - 1 - k : k;
      const bool e = k < nRng && elig((int)(uint32_t)key[t]);
      const unsigned long long m = __ballot(e);
      if (e) cpos[cnt + __popcll(m & ((1ull << l) - 1ull))] = (uint16_t)t;
      cnt += __popcll(m);
    }
    return cnt;
  };
  auto edge_elig = [&](int ind) {
    const int w = ind - ws;
    return w >= 0 && w < wn && (wflag[w] & 0xC0) == 0 && curv_of(ind) > c.edge_thr;
  };
  auto flat_elig = [&](int ind) {
    const int w = ind - ws;
    return w >= 0 && w < wn && (wflag[w] & 0xC0) == 0x40 && curv_of(ind) < c.surf_thr;
  };
  // wave-aggregated append of the statically eligible keys of the fast path
  auto append = [&](bool edge) {
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int p = ws + tid + u * 256;
      const bool in = p >= sp && p < ep && (p != 4 || ph_in);
      const int ind = p == 4 ? ph : p;
      const float v = p == 4 ? 0.0f : cvr[u];          // the sort value
      const float ve = p == 4 ? ph_curv : cvr[u];     // cloudCurvature[ind]
      const int w = in ? ind - ws : 0;
      const int fg = in ? (wflag[w] & 0xC0) : 0x80;  // picked | ground
      const bool e = in && (edge ? (fg == 0 && ve > c.edge_thr) : (fg == 0x40 && ve < c.surf_thr));
      const unsigned long long m = __ballot(e);
      int wb = 0;
      if (lane_id() == 0 && m) wb = atomicAdd(&s_cnt, (int)__popcll(m));
      wb = __builtin_amdgcn_readlane(wb, 0);
      if (e) key[wb + __popcll(m & ((1ull << lane_id()) - 1ull))] = ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)ind;
    }
  };
  // adjacent equal values in the fast-sorted eligible keys [lo, hi); also reports an earlier trigger
  auto ties = [&](int lo, int hi) {
    for (int t = lo + tid; t + 1 < hi; t += nt)
      if ((uint32_t)(key[t] >> 32) == (uint32_t)(key[t + 1] >> 32)) s_flag = 1;
    __syncthreads();
    return s_flag != 0;
  };
  if (tid == 0) s_exact = 0;
  __syncthreads();
  // ---- edges: eligible entries visited in descending sorted order, the unsorted ep first ----
  const bool epE = curv[ep] > c.edge_thr && (wflag[ep - ws] & 0x40) == 0;
  const int e0 = epE ? 1 : 0;
  append(true);
  __syncthreads();
  if (c.dbg_phase <= 0) return;
  int nE = s_cnt;
  int n2 = max(pow2_ceil(nE), 64);
  for (int t = nE + tid; t < n2; t += nt) key[t] = 0ull;
  __syncthreads();
  block4_sort<uint64_t>(key, n2);
  if (c.dbg_phase <= 1) return;
  // (n2 - nE zero keys sort first: the eligible keys are key[n2 - nE, n2))
  if (ties(n2 - nE, n2)) {
    exact_sort();
    if (tid < 64) {
      const int cnt = compact_sorted(true, edge_elig);
      auto order = [&](int t) { return t < e0 ? ep : (int)(uint32_t)key[cpos[t - e0]]; };
      const int sel = greedy_wave(order, cnt + e0, ws, wflag, wlab, (int8_t)1, d.edge_tmp + base + sp);
      if (tid == 0) { rc[i] = sel; s_cnt = 0; }
    }
  } else if (tid < 64) {
    auto order = [&](int t) { return t < e0 ? ep : (int)(uint32_t)key[n2 - 1 - (t - e0)]; };
    const int cnt = greedy_wave(order, nE + e0, ws, wflag, wlab, (int8_t)1, d.edge_tmp + base + sp);
    if (tid == 0) { rc[i] = cnt; s_cnt = 0; }
  }
  __syncthreads();
  if (c.dbg_phase <= 2) return;
  // ---- flats: eligible entries in ascending sorted order, the unsorted ep last ----
  const bool epF = curv[ep] < c.surf_thr && (wflag[ep - ws] & 0x40) != 0;
  if (s_exact) {
    if (tid < 64) {
      const int cnt = compact_sorted(false, flat_elig);
      auto order = [&](int t) { return t < cnt ? (int)(uint32_t)key[cpos[t]] : ep; };
      const int sel = greedy_wave(order, cnt + (epF ? 1 : 0), ws, wflag, wlab, (int8_t)-1, d.flat_tmp + base + sp);
      if (tid == 0) rc[H + i] = sel;
    }
  } else {
    append(false);
    __syncthreads();
    const int nF = s_cnt;
    n2 = max(pow2_ceil(nF), 64);
    for (int t = nF + tid; t < n2; t += nt) key[t] = ~0ull;
    __syncthreads();
    block4_sort<uint64_t>(key, n2);
    if (ties(0, nF)) {
      exact_sort();
      if (tid < 64) {
        const int cnt = compact_sorted(false, flat_elig);
        auto order = [&](int t) { return t < cnt ? (int)(uint32_t)key[cpos[t]] : ep; };
        const int sel = greedy_wave(order, cnt + (epF ? 1 : 0), ws, wflag, wlab, (int8_t)-1, d.flat_tmp + base + sp);
        if (tid == 0) rc[H + i] = sel;
      }
    } else if (tid < 64) {
      auto order = [&](int t) { return t < nF ? (int)(uint32_t)key[t] : ep; };
      const int cnt = greedy_wave(order, nF + (epF ? 1 : 0), ws, wflag, wlab, (int8_t)-1, d.flat_tmp + base + sp);
      if (tid == 0) rc[H + i] = cnt;
    }
  }
  __syncthreads();
  if (c.dbg_phase <= 3) return;
  for (int t = tid; t < wn; t += nt) {
    d.picked[base + ws + t] = (uint8_t)(wflag[t] >> 7);
    d.clabel[base + ws + t] = wlab[t];
  }
  // ---- less-flat candidates k in [sp, ep] with cloudLabel[k] <= 0 (FA:1262-1266) ----
  const int n = ep - sp + 1;
  const int per = (n + nt - 1) / nt;
  const int k0 = min(tid * per, n), k1 = min(k0 + per, n);
  int mine = 0;
  for (int k = k0; k < k1; ++k) mine += wlab[sp + k - ws] <= 0;
  int L;
  int pos = block_excl_scan(mine, tmp, &L);
  for (int k = k0; k < k1; ++k)
    if (wlab[sp + k - ws] <= 0) cpos[pos++] = (uint16_t)k;
  __syncthreads();
  if (c.dbg_phase <= 4) return;
  const float4* lp = d.loam + base + sp;
  // ---- VoxelGrid(0.2) applyFilter (PCL 1.10), centroids summed in (voxel, input) order ----
  // each lane's candidates (t = tid + 256 u, L <= 2048) are gathered once, for the bounds and the keys
  constexpr int kLp = kRingMax / 256;
  float4 lpr[kLp];
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
#pragma unroll
  for (int u = 0; u < kLp; ++u)
    if (tid + u * 256 < L) lpr[u] = lp[cpos[tid + u * 256]];
#pragma unroll
  for (int u = 0; u < kLp; ++u) {
    if (tid + u * 256 >= L) continue;
    const float4 p = lpr[u];
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  for (int a = 0; a < 3; ++a) { mn[a] = wave_reduce_min(mn[a]); mx[a] = wave_reduce_max(mx[a]); }
  if (lane_id() == 0)
    for (int a = 0; a < 3; ++a) { red[a][tid >> 6] = mn[a]; red[3 + a][tid >> 6] = mx[a]; }
  __syncthreads();
  for (int a = 0; a < 3; ++a) {
    mn[a] = fminf(fminf(red[a][0], red[a][1]), fminf(red[a][2], red[a][3]));
    mx[a] = fmaxf(fmaxf(red[3 + a][0], red[3 + a][1]), fmaxf(red[3 + a][2], red[3 + a][3]));
  }
  const float inv = 1.0f / 0.2f;
  float4* out = d.lflat_tmp + base + sp;
  if (L == 0) {
    if (tid == 0) rc[2 * H + i] = 0;
    return;
  }
  const long long dx = (long long)((mx[0] - mn[0]) * inv) + 1, dy = (long long)((mx[1] - mn[1]) * inv) + 1,
                  dz = (long long)((mx[2] - mn[2]) * inv) + 1;
  if (dx * dy * dz > (long long)INT_MAX) {  // PCL: leaf too small -> output = input
    for (int t = tid; t < L; t += nt) out[t] = lp[cpos[t]];
    if (tid == 0) rc[2 * H + i] = L;
    return;
  }
  int minb[3], div[3];
  for (int a = 0; a < 3; ++a) {
    minb[a] = (int)floorf(mn[a] * inv);
    div[a] = (int)floorf(mx[a] * inv) - minb[a] + 1;
  }
  const int mul1 = div[0], mul2 = div[0] * div[1];
  // voxel id of every candidate, in ring order (points of one voxel are mostly consecutive)
  // (in key[]: dead after the greedy passes; every key[] write below comes after the barriers that
  // end the vk[] reads, and a lane's own ids stay in vkr)
  uint32_t* vk = reinterpret_cast<uint32_t*>(key);
  uint32_t vkr[kLp];
#pragma unroll
  for (int u = 0; u < kLp; ++u) {
    const int t = tid + u * 256;
    vkr[u] = 0u;
    if (t >= L) continue;
    const float4 p = lpr[u];
    const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
    const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
    const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
    vkr[u] = (uint32_t)(i0 + i1 * mul1 + i2 * mul2);
    vk[t] = vkr[u];
  }
  __syncthreads();
  __shared__ int scnt[kLp * 4 + 1];
  const int wv = tid >> 6, ln = lane_id();
  const unsigned long long ltm = (1ull << ln) - 1ull;
  int V;
  auto slot_scan = [&]() {  // exclusive scan of scnt[0 .. kLp*4) in place, total in scnt[kLp*4]
    __syncthreads();
    if (wv == 0) {
      const int v = ln < kLp * 4 ? scnt[ln] : 0;
      const int incl = wave_incl_scan_add(v);
      if (ln < kLp * 4) scnt[ln] = incl - v;
      if (ln == 63) scnt[kLp * 4] = incl;
    }
    __syncthreads();
  };
  // runs of equal voxel id in ring order -> one sort key per run, (voxel id, run index), sorted
  // (block4_sort); run starts in rstart. Position t = u * 256 + tid in slot u of a lane; run
  // indices from per-(slot, wave) ballot counts scanned in (slot, wave) = ring order.
  auto sort_runs = [&]() {
    unsigned long long mR[kLp];
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      const int t = u * 256 + tid;
      mR[u] = __ballot(t < L && (t == 0 || vkr[u] != vk[t - 1]));
      if (ln == 0) scnt[u * 4 + wv] = (int)__popcll(mR[u]);
    }
    slot_scan();
    const int R = scnt[kLp * 4];
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      if (!((mR[u] >> ln) & 1ull)) continue;
      const int t = u * 256 + tid;
      const int ro = scnt[u * 4 + wv] + (int)__popcll(mR[u] & ltm);
      rstart[ro] = (uint16_t)t;
      key[ro] = ((uint64_t)vkr[u] << 32) | (uint32_t)ro;
    }
    if (tid == 0) rstart[R] = (uint16_t)L;
    const int R2 = max(pow2_ceil(R), 64);
    for (int t = R + tid; t < R2; t += nt) key[t] = ~0ull;
    __syncthreads();
    block4_sort<uint64_t>(key, R2);
    return R;
  };
  if (c.exact_vg) {
    // LLSR_VOXEL_ORDER_PCL (llsr_set_voxel_order): std::sort(index_vector) by voxel id alone (PCL
    // 1.10 voxel_grid.hpp) and the centroids summed in that order run in k_vox_pcl, a kernel of
    // its own with a small LDS footprint (more rings per CU for the sort's dependent chains). It
    // sorts 32-bit keys (rank << 11 | candidate): each voxel id replaced by its dense rank among the
    // ring's ids, which keeps the outcome of every comparison; the ranks come from the sorted voxel
    // runs. The keys and the candidate positions go to the scratch slots of the ring's positions
    // (ccl_a / ccl_b, dead since k_label), and rc[2H + i] = -1 - L marks the ring pending.
    if (c.dbg_phase <= 5) return;
    const int R = sort_runs();
    uint16_t* rrank = reinterpret_cast<uint16_t*>(win_raw);  // run -> rank of its voxel id
    const unsigned long long lem = ltm | (1ull << ln);
    unsigned long long mH[kLp];
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      const int t = u * 256 + tid;
      mH[u] = __ballot(t < R && (t == 0 || (key[t] >> 32) != (key[t - 1] >> 32)));
      if (ln == 0) scnt[u * 4 + wv] = (int)__popcll(mH[u]);
    }
    slot_scan();
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      const int t = u * 256 + tid;
      if (t < R) rrank[(uint32_t)key[t]] = (uint16_t)(scnt[u * 4 + wv] + (int)__popcll(mH[u] & lem) - 1);
    }
    __syncthreads();
    uint32_t* gk = reinterpret_cast<uint32_t*>(d.ccl_a + base) + sp;
    uint16_t* gc = reinterpret_cast<uint16_t*>(d.ccl_b + base) + sp;
    for (int r = tid; r < R; r += nt) {
      const uint32_t rk = (uint32_t)rrank[r] << 11;
      const int qe = rstart[r + 1];
      for (int q = rstart[r]; q < qe; ++q) gk[q] = rk | (uint32_t)q;
    }
    for (int t = tid; t < L; t += nt) gc[t] = cpos[t];
    if (tid == 0) rc[2 * H + i] = -1 - L;
    return;
  } else {
    // LLSR_VOXEL_ORDER_INPUT: each voxel summed run by run in ring order (sorted runs)
    if (c.dbg_phase <= 5) return;
    const int R = sort_runs();
    if (c.dbg_phase <= 6) return;
    // voxels = groups of sorted runs with equal id; sum members in (run start, position) order.
    // Sorted run t = u * 256 + tid sits in slot u of a lane, so a wave's voxel heads of one slot are
    // consecutive voxels and their centroids are stored contiguously; output positions come from
    // per-(slot, wave) ballot counts scanned in (slot, wave) = sorted order.
    unsigned long long mH[kLp];
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      const int t = u * 256 + tid;
      const bool head = t < R && (t == 0 || (key[t] >> 32) != (key[t - 1] >> 32));
      mH[u] = __ballot(head);
      if (ln == 0) scnt[u * 4 + wv] = (int)__popcll(mH[u]);
    }
    slot_scan();
    V = scnt[kLp * 4];
#pragma unroll
    for (int u = 0; u < kLp; ++u) {
      const int t = u * 256 + tid;
      if (!((mH[u] >> ln) & 1ull)) continue;
      const uint32_t vid = (uint32_t)(key[t] >> 32);
      float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
      int cntp = 0;
      for (int e = t; e < R && (uint32_t)(key[e] >> 32) == vid; ++e) {
        const int run = (int)(uint32_t)key[e];
        // two of the run's points in flight per step, summed in order
        const int qe = rstart[run + 1];
        for (int q = rstart[run]; q < qe; q += 2) {
          const bool two = q + 1 < qe;
          const float4 p0 = lp[cpos[q]];
          const float4 p1 = two ? lp[cpos[q + 1]] : make_float4(0.f, 0.f, 0.f, 0.f);
          sx += p0.x; sy += p0.y; sz += p0.z; si += p0.w;
          ++cntp;
          if (two) {
            sx += p1.x; sy += p1.y; sz += p1.z; si += p1.w;
            ++cntp;
          }
        }
      }
      const float nn = (float)cntp;
      const int vo = scnt[u * 4 + wv] + (int)__popcll(mH[u] & ltm);
      out[vo] = make_float4(sx / nn, sy / nn, sz / nn, si / nn);
    }
  }
  if (tid == 0) rc[2 * H + i] = V;
}

// ---------------------------------------------------------------------------------------------
// K8b the less-flat VoxelGrid in PCL order (LLSR_VOXEL_ORDER_PCL; FA:1268-1271, PCL 1.10
// VoxelGrid::applyFilter): each pending ring's (voxel id << 32 | candidate) keys sorted by voxel id
// exactly as libstdc++'s std::sort leaves them (block_introsort, llsr_isort.h), then one lane per
// voxel sums its points in that order. Split from k_select_ring so the sort runs at 8 workgroups
// per CU (32-bit keys: 17 KB LDS, <= 64 VGPRs) instead of 5: its chains of dependent LDS steps
// want rings in flight. grid (H, B), block 256.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 8) void k_vox_pcl(DevCfg c, DevBufs d) {
  __shared__ uint32_t key[kRingMax];
  __shared__ uint16_t Lp[kRingMax], Rp[kRingMax];
  __shared__ BlockSortLds bsl;
  constexpr int kLp = kRingMax / 256;
  __shared__ int scnt[kLp * 4 + 1];
  const int i = blockIdx.x, b = blockIdx.y, H = c.H;
  int* rc = d.ring_cnt + (size_t)b * 3 * H;
  const int r = rc[2 * H + i];
  if (r >= 0) return;  // no candidates, or written by k_select_ring (input order / oversized grid)
  const int L = -1 - r;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int sp = d.start_ring[b * H + i];
  const size_t base = (size_t)b * c.HW;
  const uint32_t* gk = reinterpret_cast<const uint32_t*>(d.ccl_a + base) + sp;
  const uint16_t* gc = reinterpret_cast<const uint16_t*>(d.ccl_b + base) + sp;
  for (int t = tid; t < L; t += nt) key[t] = gk[t];
  // barriers on entry and exit (diagnostic phases 100 / 101 / 102: the block-wide part, the
  // partitions, the whole sort)
  block_introsort<256>(key, L, Lp, Rp, bsl, VoxLess32{}, nullptr, c.dbg_phase >= 100 ? c.dbg_phase - 100 : 1 << 30);
  if (c.dbg_phase <= 102) return;
  uint16_t* cpos = Lp;  // the sort's scratch is free again
  for (int t = tid; t < L; t += nt) cpos[t] = gc[t];
  const float4* lp = d.loam + base + sp;
  float4* out = d.lflat_tmp + base + sp;
  const int wv = tid >> 6, ln = lane_id();
  const unsigned long long ltm = (1ull << ln) - 1ull;
  // voxel heads in sorted order; sorted position t = u * 256 + tid sits in slot u of a lane, so a
  // wave's heads of one slot are consecutive voxels and their centroids are stored contiguously;
  // output positions come from per-(slot, wave) ballot counts scanned in (slot, wave) = sorted order.
  unsigned long long mH[kLp];
#pragma unroll
  for (int u = 0; u < kLp; ++u) {
    const int t = u * 256 + tid;
    const bool head = t < L && (t == 0 || (key[t] >> 11) != (key[t - 1] >> 11));
    mH[u] = __ballot(head);
    if (ln == 0) scnt[u * 4 + wv] = (int)__popcll(mH[u]);
  }
  __syncthreads();
  if (wv == 0) {  // exclusive scan of scnt[0 .. kLp*4) in place, total in scnt[kLp*4]
    const int v = ln < kLp * 4 ? scnt[ln] : 0;
    const int incl = wave_incl_scan_add(v);
    if (ln < kLp * 4) scnt[ln] = incl - v;
    if (ln == 63) scnt[kLp * 4] = incl;
  }
  __syncthreads();
  const int V = scnt[kLp * 4];
#pragma unroll
  for (int u = 0; u < kLp; ++u) {
    const int t = u * 256 + tid;
    if (!((mH[u] >> ln) & 1ull)) continue;
    const uint32_t vr = key[t] >> 11;
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    int e = t;
    for (; e < L && (key[e] >> 11) == vr; ++e) {
      const float4 p = lp[cpos[key[e] & 0x7ffu]];
      sx += p.x; sy += p.y; sz += p.z; si += p.w;
    }
    const float nn = (float)(e - t);
    const int vo = scnt[u * 4 + wv] + (int)__popcll(mH[u] & ltm);
    out[vo] = make_float4(sx / nn, sy / nn, sz / nn, si / nn);
  }
  if (tid == 0) rc[2 * H + i] = V;
}

// ---------------------------------------------------------------------------------------------
// K9a concatenate the per-ring lists in ring order (FA:1165 loop) and prepare the DBSCAN point
// records of the edge candidates: lidar-frame (x0, y0, z0) = LOAM (z, x, y), kxy, kz
// (FA:1326-1336). One workgroup (256 threads) per scan.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fa_concat(DevCfg c, DevBufs d) {
  __shared__ int roff[3][65];
  __shared__ int rsp[64];
  const int b = blockIdx.x;
  const int H = c.H;
  const size_t base = (size_t)b * c.HW;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int* rc = d.ring_cnt + (size_t)b * 3 * H;
  if (tid < 64) {
    for (int q = 0; q < 3; ++q) {
      const int v = tid < H ? rc[q * H + tid] : 0;
      const int incl = wave_incl_scan_add(v);
      if (tid < H) roff[q][tid] = incl - v;
      if (tid == 63) roff[q][H] = incl;
    }
  }
  if (tid < H) rsp[tid] = d.start_ring[b * H + tid];
  __syncthreads();
  const int M = roff[0][H];
  // all rings of a list at once: output a comes from ring r with roff[r] <= a < roff[r + 1]
  for (int q = 0; q < 3; ++q) {
    const int tot = roff[q][H];
    for (int a = tid; a < tot; a += nt) {
      int lo = 0, hi = H - 1;  // largest r with roff[q][r] <= a (never an empty ring)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (roff[q][mid] <= a) lo = mid;
        else hi = mid - 1;
      }
      const size_t src = base + rsp[lo] + (a - roff[q][lo]);
      if (q == 0) d.less_sharp[base + a] = d.edge_tmp[src];
      else if (q == 1) d.flat[base + a] = d.flat_tmp[src];
      else d.lflat[base + a] = d.lflat_tmp[src];
    }
  }
  __syncthreads();
  const float4* loam = d.loam + base;
  for (int a = tid; a < M; a += nt) {
    const float4 p = loam[d.less_sharp[base + a]];
    const float x0 = p.z, y0 = p.x, z0 = p.y;
    const float AB = atan2f_(z0, sqrt_(x0 * x0 + y0 * y0));
    const float kxy = sqrt_(x0 * x0 + y0 * y0) * c.sinResX * c.RatioXY;
    const float kz = (sqrt_(x0 * x0 + y0 * y0) * tanf_(AB + c.fa_resY) -
                      sqrt_(x0 * x0 + y0 * y0) * tanf_(AB - c.fa_resY)) / 2 * c.RatioZ;
    d.db_pts[base + a] = make_float4(x0, y0, z0, kxy);
    d.db_kz[base + a] = kz;
  }
  if (tid == 0) {
    int* cnt = d.counts + b * kCnt;
    cnt[C_M] = M;
    cnt[C_F] = roff[1][H];
    cnt[C_L] = roff[2][H];
  }
}

// eps test of FA:1353-1354 with point i as the centre and j's scales
__device__ __forceinline__ bool db_near(const DevCfg& c, float4 pi, float4 pj, float kzj) {
  const float eps = sqrt_((pi.x - pj.x) * (pi.x - pj.x) / (pj.w * pj.w) +
                          (pi.y - pj.y) * (pi.y - pj.y) / (pj.w * pj.w) +
                          (pi.z - pj.z) * (pi.z - pj.z) / (kzj * kzj));
  return eps <= c.DBFr;
}

// Certified fast form of db_near: the squared scaled distance from hardware reciprocals (all three
// terms are >= 0, so its relative error against the reference's float evaluation is < 1e-6) decides
// eps <= DBFr whenever it is more than 2e-5 (relative) away from DBFr^2: below, sqrt(s) < DBFr and
// its rounding cannot exceed DBFr; above, sqrt(s) exceeds DBFr by > 4 ulp. Pairs in the band, zero or
// non-finite scales and NaN coordinates take the exact expression.
__device__ __forceinline__ bool db_near_fast(const DevCfg& c, float4 pi, float4 pj, float kzj) {
  const float dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
  const float k2 = pj.w * pj.w, z2 = kzj * kzj;
  if (c.DBFr > 0.0f && k2 > 1e-30f && k2 < 1e30f && z2 > 1e-30f && z2 < 1e30f) {
    const float s = (dx * dx + dy * dy) * __builtin_amdgcn_rcpf(k2) + dz * dz * __builtin_amdgcn_rcpf(z2);
    const float r2 = c.DBFr * c.DBFr;
    if (s < r2 * (1.0f - 2e-5f)) return true;
    if (s > r2 * (1.0f + 2e-5f)) return false;
  }
  return db_near(c, pi, pj, kzj);
}

// ---------------------------------------------------------------------------------------------
// K9b eps-neighbourhood bitmask for every (i, j) of a scan (M <= kAdjCap). A wave task is 64
// consecutive j (one per lane) against kAdjRows consecutive rows i: the lane's point j, the two
// hardware reciprocals of its scales and the fast path's eligibility are computed once per task,
// then each row costs a wave-uniform load of point i, the scaled distance and a ballot stored as
// two words. Decisions are db_near_fast's (the same reciprocals, the same float expression, the
// exact db_near inside the band). Takes the O(M^2) float work off DBSCAN's serial merge.
// grid (32, B), block 256.
// ---------------------------------------------------------------------------------------------
// A wave's LDS instructions execute in issue order, so lanes of one wave only need the compiler
// not to move memory operations across these points (no s_waitcnt, no cache maintenance).
__device__ __forceinline__ void wave_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

constexpr int kAdjRows = 16;

__global__ __launch_bounds__(256) void k_dbscan_adj(DevCfg c, DevBufs d, const float4* __restrict__ db_pts) {
  const int b = blockIdx.y;
  const size_t base = (size_t)b * c.HW;
  const int M = d.counts[b * kCnt + C_M];
  if (M > kAdjCap) return;
  const int nch = (M + 63) / 64, ngr = (M + kAdjRows - 1) / kAdjRows;
  const int wv = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int nwv = (gridDim.x * blockDim.x) >> 6;
  const int l = lane_id();
  uint32_t* adj = d.db_adj + (size_t)b * kAdjCap * kAdjWords;
  const float4* __restrict__ pts = db_pts + base;  // d.db_pts as a restrict argument: scalar loads
  const float r2 = c.DBFr * c.DBFr, lo = r2 * (1.0f - 2e-5f), hi = r2 * (1.0f + 2e-5f);
  __shared__ unsigned long long sb[4][kAdjRows];  // each wave's row ballots, read back as words
  const int wl = threadIdx.x >> 6;
  for (int task = wv; task < nch * ngr; task += nwv) {
    const int ch = task % nch, i0 = (task / nch) * kAdjRows;
    const int j = ch * 64 + l;
    const bool inj = j < M;
    const float4 pj = inj ? pts[j] : make_float4(0.f, 0.f, 0.f, 1.f);
    const float kz = inj ? d.db_kz[base + j] : 1.0f;
    const float k2 = pj.w * pj.w, z2 = kz * kz;
    const bool fast = c.DBFr > 0.0f && k2 > 1e-30f && k2 < 1e30f && z2 > 1e-30f && z2 < 1e30f;
    const float rk = __builtin_amdgcn_rcpf(k2), rz = __builtin_amdgcn_rcpf(z2);
    // the task's row points: wave-uniform addresses of a read-only array, so scalar loads, all in
    // flight before the first row (rows past M repeat row M - 1; their bits are never stored);
    // the rows' ballots gather in lanes 2r (low word) / 2r+1 (high word) and leave in ONE store
    uint32_t out = 0u;
    constexpr int kHalf = kAdjRows / 2;  // 8 rows' points at a time in SGPRs (16 would spill)
#pragma unroll
    for (int r = 0; r < kAdjRows; ++r) {
      float3 prw[kHalf];
      if (r % kHalf == 0) {
#pragma unroll
        for (int e = 0; e < kHalf; ++e) {
          const float4 q = pts[min(i0 + r + e, M - 1)];
          prw[e] = make_float3(q.x, q.y, q.z);
        }
      }
      const float3 pr = prw[r % kHalf];
      const float4 pi = make_float4(pr.x, pr.y, pr.z, 0.0f);  // (db_near reads no pi.w)
      const float dx = pi.x - pj.x, dy = pi.y - pj.y, dz = pi.z - pj.z;
      const float s = (dx * dx + dy * dy) * rk + dz * dz * rz;
      bool nb = fast && s < lo;
      if (inj && !(fast && (s < lo || s > hi))) nb = db_near(c, pi, pj, kz);
      nb = nb && inj;
      const unsigned long long m = __ballot(nb);
      if (l == 0) sb[wl][r] = m;
    }
    wave_order();
    if (l < 2 * kAdjRows) out = reinterpret_cast<const uint32_t*>(sb[wl])[l];
    wave_order();  // the next task's writes after these reads
    const int w = 2 * ch + (l & 1);
    if (l < 2 * kAdjRows && i0 + (l >> 1) < M && w < kAdjWords) adj[(size_t)(i0 + (l >> 1)) * kAdjWords + w] = out;
  }
}

// ---------------------------------------------------------------------------------------------
// K9c DBSCAN merge (FA:1342-1386) + cluster run-length filter (FA:1281-1305), ONE WAVE per scan.
// The reference relabels every point whose label is in the neighbours' label list, including
// label 0 (so all still-unlabelled points collapse into min_label). That is a merge of label
// classes, done here with a union-find over label nodes 1..M plus "zero" nodes: Z0 holds every
// not-yet-visited point, and visiting i moves i into a fresh zero node (cluster[i] = 0). A merge
// unions the neighbours' classes — and, when a neighbour is unlabelled, every live zero class —
// into min_label; a new label only re-points the neighbours. Checked against a literal
// transcription of the loop in tests/test_dbscan_uf.py. Per point: O(degree) work.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <bool lds>
__device__ __forceinline__ int uf_root(int* par, int x) {  // path halving
  while (true) {
    const int p = par[x];
    if (p == x) return x;
    const int gp = par[p];
    par[x] = gp;
    if (gp == p) return p;
    x = gp;
  }
}

// Minimum of v over lanes with `valid`, for 0 <= v < 2^nbits, by ballots (scalar work only);
// returns 999999999 when no lane is valid.
__device__ __forceinline__ int wave_min_ballot(int v, bool valid, int nbits) {
  unsigned long long cand = __ballot(valid);
  if (!cand) return 999999999;
  const int l = lane_id();
  int res = 0;
  for (int bt = nbits - 1; bt >= 0; --bt) {
    const unsigned long long z = __ballot(((cand >> l) & 1ull) && !((v >> bt) & 1));
    if (z) cand = z;
    else res |= 1 << bt;
  }
  return res;
}


// kRowBlk adjacency rows are staged into LDS per block (one load latency per block instead of one
// per point: the rows of a 300-point scan come from L2 / the Infinity Cache, ~1 us away), the next
// block's words waiting in registers (kPF per lane) while the current one is merged.
constexpr int kRowBlk = 32;

template <bool lds, int kPF = 1>
__device__ __forceinline__ void dbscan_merge(const DevCfg& c, const DevBufs& d, size_t base, int b, int M,
                                             int* par, int* raw, int* nb, int* rt, int* live, int* shn,
                                             uint32_t* rowbuf = nullptr) {
  auto sync_ = [&]() {
    if (lds) wave_order();
    else __threadfence_block();
  };
  const int l = lane_id();
  const unsigned long long lt = (1ull << l) - 1ull;
  const int Z0 = M + 1;
  for (int x = l; x < 2 * M + 3; x += 64) par[x] = x;
  for (int j = l; j < M; j += 64) raw[j] = Z0;
  if (l == 0) { live[0] = Z0; shn[0] = 1; }
  sync_();
  const bool pre = M <= kAdjCap;
  const uint32_t* adj = d.db_adj + (size_t)b * kAdjCap * kAdjWords;
  const int W32 = (M + 31) / 32;
  int label = 0;
  // rows are <= 64 words when precomputed (M <= kAdjCap)
  const bool staged = lds && pre && kRowBlk * W32 <= 64 * kPF;
  const int bw = kRowBlk * W32;  // words per staged block
  uint32_t pf[kPF];
  auto fetch_block = [&](int blk) {
#pragma unroll
    for (int e = 0; e < kPF; ++e) {
      const int idx = l + 64 * e;
      const int r = idx / (W32 > 0 ? W32 : 1), w = idx - r * W32;
      const int row = blk * kRowBlk + r;
      pf[e] = (idx < bw && row < M) ? adj[(size_t)row * kAdjWords + w] : 0u;
    }
  };
  if (staged && M > 0) fetch_block(0);
  uint32_t nextw = (!staged && pre && M > 0 && l < W32) ? adj[l] : 0u;
  for (int i = 0; i < M; ++i) {
    const int zi = M + 2 + i;
    if (l == 0) raw[i] = zi;
    // neighbour list of i in increasing j
    int deg = 0;
    bool i_in = false;
    const float4 pi = pre ? make_float4(0.f, 0.f, 0.f, 0.f) : d.db_pts[base + i];
    uint32_t roww;
    if (staged) {
      if (i % kRowBlk == 0) {
#pragma unroll
        for (int e = 0; e < kPF; ++e)
          if (l + 64 * e < bw) rowbuf[l + 64 * e] = pf[e];
        wave_order();
        fetch_block(i / kRowBlk + 1);
      }
      roww = l < W32 ? rowbuf[(i % kRowBlk) * W32 + l] : 0u;
    } else {
      roww = nextw;  // prefetch row i+1 while merging row i
      if (pre) nextw = (i + 1 < M && l < W32) ? adj[(size_t)(i + 1) * kAdjWords + l] : 0u;
    }
    for (int w0 = 0; w0 < W32; w0 += 64) {
      const int w = w0 + l;
      uint32_t word = 0u;
      if (w < W32) {
        if (pre) {
          word = roww;
        } else {
          for (int q = 0; q < 32; ++q) {
            const int j = 32 * w + q;
            if (j < M && db_near(c, pi, d.db_pts[base + j], d.db_kz[base + j])) word |= 1u << q;
          }
        }
      }
      if (w == (i >> 5)) i_in = (word >> (i & 31)) & 1u;
      const int cnt = __popc(word);
      const int ex = wave_incl_scan_add(cnt) - cnt;
      int pos = deg + ex;
      while (word) {
        const int q = __ffs(word) - 1;
        word &= word - 1u;
        nb[pos++] = 32 * w + q;
      }
      deg += __builtin_amdgcn_readlane(ex + cnt, 63);
    }
    i_in = __ballot(i_in) != 0ull;
    sync_();
    int lmin = 999999999;
    bool zero = false;
    for (int k = l; k < deg; k += 64) {
      const int r = uf_root<lds>(par, raw[nb[k]]);
      rt[k] = r;
      if (r > M) zero = true;
      else if (r < lmin) lmin = r;
    }
    lmin = wave_reduce_min(lmin);
    zero = __ballot(zero) != 0ull;
    sync_();
    if (lmin <= label) {
      for (int k = l; k < deg; k += 64) {
        const int r = rt[k];
        if (r <= M && r != lmin) par[r] = lmin;
        raw[nb[k]] = lmin;
      }
      if (zero) {
        const int nl = shn[0];
        for (int k = l; k <= nl; k += 64) {
          const int z = k < nl ? live[k] : zi;
          const int r = uf_root<lds>(par, z);
          if (r > M) par[r] = lmin;
        }
        sync_();
        if (l == 0) shn[0] = 0;
      } else if (!i_in && l == 0) {
        live[shn[0]] = zi;
        shn[0] += 1;
      }
    } else {
      label += 1;
      for (int k = l; k < deg; k += 64) raw[nb[k]] = label;
      if (!i_in && l == 0) {
        live[shn[0]] = zi;
        shn[0] += 1;
      }
    }
    sync_();
  }
  // final labels -> raw (as CL) and the output array
  for (int j = l; j < M; j += 64) {
    const int r = uf_root<lds>(par, raw[j]);
    const int v = r > M ? 0 : r;
    d.cluster[base + j] = v;
    nb[j] = v;
  }
  sync_();
  // ---- run lengths of the sorted labels, last run dropped; keep label r+1 if run r >= 4 ----
  int* CL = nb;
  int* hist = rt;
  const int NL = label + 1;
  for (int q = l; q < NL; q += 64) hist[q] = 0;
  sync_();
  for (int a = l; a < M; a += 64) atomicAdd(&hist[CL[a]], 1);
  sync_();
  int lmax = -1;
  for (int q = l; q < NL; q += 64)
    if (hist[q] > 0) lmax = q;
  lmax = wave_reduce_max(lmax);
  uint32_t* keep = (uint32_t*)par;  // label-indexed bitmap, par no longer needed
  const int nwLb = (NL + 1 + 31) / 32;
  for (int w = l; w < nwLb; w += 64) keep[w] = 0u;
  sync_();
  int run = 0;
  for (int q0 = 0; q0 < NL; q0 += 64) {
    const int q = q0 + l;
    const bool pres = q < NL && hist[q] > 0;
    const unsigned long long m = __ballot(pres);
    const int r = run + __popcll(m & lt);
    if (pres && q != lmax && hist[q] >= 4 && r + 1 < NL) atomicOr(&keep[(r + 1) >> 5], 1u << ((r + 1) & 31));
    run += __popcll(m);
  }
  sync_();
  int ns = 0;
  for (int a0 = 0; a0 < M; a0 += 64) {
    const int a = a0 + l;
    const bool kp = a < M && ((keep[CL[a] >> 5] >> (CL[a] & 31)) & 1u);
    const unsigned long long m = __ballot(kp);
    if (kp) d.sharp[base + ns + __popcll(m & lt)] = d.less_sharp[base + a];
    ns += __popcll(m);
  }
  if (l == 0) d.counts[b * kCnt + C_SHARP] = ns;
}

// One wave per scan, so the LDS footprint sets how many scans a CU runs at once: kDbL = 1024
// (24.6 KB, VLP-16-sized scans, M ~ 300) fits every SIMD of a CU; 2048 (49 KB) serves HDL-64E.
template <int kDbL>
__global__ __launch_bounds__(64) void k_dbscan_merge(DevCfg c, DevBufs d) {
  constexpr int kPF = kRowBlk * (kDbL / 32) / 64;  // staged words per lane (M <= kDbL)
  __shared__ uint32_t sRows[kRowBlk * (kDbL / 32)];
  __shared__ int sPar[2 * kDbL + 4];
  __shared__ int sRaw[kDbL];
  __shared__ int sNb[kDbL];
  __shared__ int sRt[kDbL + 1];
  __shared__ int sLive[kDbL + 1];
  __shared__ int sN[1];
  const int b = blockIdx.x;
  const size_t base = (size_t)b * c.HW;
  const int M = d.counts[b * kCnt + C_M];
  if (M <= kDbL) {
    dbscan_merge<true, kPF>(c, d, base, b, M, sPar, sRaw, sNb, sRt, sLive, sN, sRows);
  } else {  // global scratch: ccl_b (2*HW ints) parent, ccl_a raw, cluster nb, edge_tmp rt, shuf live
    dbscan_merge<false>(c, d, base, b, M, (int*)(d.ccl_b + base), d.ccl_a + base, d.flat_tmp + base,
                        d.edge_tmp + base, d.shuf + base, d.shuf + base + c.HW - 1);
  }
}

}  // namespace llsr

namespace llsr {
template __global__ void k_dbscan_merge<1024>(DevCfg, DevBufs);
template __global__ void k_dbscan_merge<2048>(DevCfg, DevBufs);
}  // namespace llsr
