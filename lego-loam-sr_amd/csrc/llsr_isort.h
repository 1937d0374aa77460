// llsr_isort.h — libstdc++'s std::sort reproduced exactly on the device, for the two places where
// the reference sorts with a comparator that ignores part of the element, so the order of EQUAL
// keys is whatever libstdc++'s introsort leaves and it changes results:
//   * the per-ring cloudSmoothness sort by value (FA:1172): the greedy edge / flat pick visits tied
//     candidates in that order (llsr_fa.hip);
//   * pcl::VoxelGrid's std::sort of (voxel id, point index) by voxel id (PCL 1.10 voxel_grid.hpp,
//     every downSizeFilter of FA / MO): each centroid sums its voxel's points in that order
//     (llsr_fa.hip's per-ring less-flat filter, llsr_map.hip's segmented filter).
// Keys are uint64 (sort key << 32 | payload); the comparator sees the whole word.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "llsr_device.h"

namespace llsr {

// The sort compares values only, so the order of EQUAL values is whatever libstdc++'s introsort
// leaves, and it decides which of two tied candidates the greedy loop visits first. One wave
// reproduces it on key[0, n) (value bits << 32 | ind): __introsort_loop (median of
// (first+1, mid, last-1) to first, __unguarded_partition, depth limit 2*lg(n) -> heap sort),
// then __final_insertion_sort (threshold 16). Each partition is evaluated in parallel: the k-th
// stop of the left scan over the original range is L[k] (!(a < pivot)), of the right scan R[k]
// (!(pivot < a), from last-1 down to the pivot slot); pairs k < k* = #{k : L[k] < R[k]} are
// swapped and the cut is R[k*-1] when k* > 0 and L[k*] is missing or >= R[k*-1], else L[k*].
// Sub-ranges are independent (the depth limit travels with each) and the final insertion sort
// never crosses a leaf boundary, so it runs as one insertion sort per leaf. The serial statement
// of this formulation is checked against std::sort by tests/native/introsort_check.cpp; the
// device against the oracle's std::sort by tests/test_gpu_features_ties.py.
__device__ __forceinline__ bool key_lt(uint64_t a, uint64_t b) {
  return __uint_as_float((uint32_t)(a >> 32)) < __uint_as_float((uint32_t)(b >> 32));
}
// the comparators: cloudSmoothness by value (FA:1172), PCL's cloud_point_index_idx by voxel id
struct CurvLess {
  __device__ bool operator()(uint64_t a, uint64_t b) const { return key_lt(a, b); }
};
struct VoxLess {
  __device__ bool operator()(uint64_t a, uint64_t b) const { return (uint32_t)(a >> 32) < (uint32_t)(b >> 32); }
};
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// libstdc++ __adjust_heap (with __push_heap) on key[f, f+len), one lane
template <class Lt>
__device__ void heap_adjust(uint64_t* key, int f, int hole, int len, uint64_t val, Lt lt) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (lt(key[f + second], key[f + second - 1])) second--;
    key[f + hole] = key[f + second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    key[f + hole] = key[f + second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && lt(key[f + parent], val)) {
    key[f + hole] = key[f + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  key[f + hole] = val;
}
// __partial_sort(first, last, last) = __make_heap + __sort_heap, one lane
template <class Lt>
__device__ void heap_sort_range(uint64_t* key, int f, int l, Lt lt) {
  const int len = l - f;
  if (len >= 2)
    for (int parent = (len - 2) / 2;; --parent) {
      heap_adjust(key, f, parent, len, key[f + parent], lt);
      if (parent == 0) break;
    }
  for (int last = l; last - f > 1;) {
    --last;
    const uint64_t val = key[last];
    key[last] = key[f];
    heap_adjust(key, f, 0, last - f, val, lt);
  }
}
constexpr int kSortStack = 64;

// ---- ranges of at most 64 elements: the rest of their introsort in registers -----------------
// Lane i holds element f + i. Partitions, the heap-sort fallback and the final insertion sort of
// the range's leaves (an insertion sort with a strict comparator is a stable sort, so each leaf's
// result is its stable sort, computed from ranks) all run on register values with ballots and
// lane shuffles; only the load and the final store touch LDS.
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
// position of the k-th (0-based) set bit of m, from bit 0; k < popcount(m)
__device__ __forceinline__ int select_bit(uint64_t m, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t low = m & ((1ull << w) - 1ull);
    const int c = __popcll(low);
    if (k >= c) { k -= c; m >>= w; pos += w; }
    else m = low;
  }
  return pos;
}
// libstdc++ heap sort of lanes [f, e) (all lanes execute; every index is wave-uniform)
template <class Lt>
__device__ void reg_heap_adjust(uint64_t& v, int f, int hole, int len, uint64_t val, Lt lt) {
  const int l = lane_id();
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (lt(rdlane64(v, f + second), rdlane64(v, f + second - 1))) second--;
    const uint64_t x = rdlane64(v, f + second);
    if (l == f + hole) v = x;
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    const uint64_t x = rdlane64(v, f + second - 1);
    if (l == f + hole) v = x;
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && lt(rdlane64(v, f + parent), val)) {
    const uint64_t x = rdlane64(v, f + parent);
    if (l == f + hole) v = x;
    hole = parent;
    parent = (hole - 1) / 2;
  }
  if (l == f + hole) v = val;
}
template <class Lt>
__device__ void reg_heap_sort(uint64_t& v, int f, int e, Lt lt) {
  const int l = lane_id();
  const int len = e - f;
  if (len >= 2)
    for (int parent = (len - 2) / 2;; --parent) {
      reg_heap_adjust(v, f, parent, len, rdlane64(v, f + parent), lt);
      if (parent == 0) break;
    }
  for (int last = e; last - f > 1;) {
    --last;
    const uint64_t val = rdlane64(v, last);
    const uint64_t top = rdlane64(v, f);
    if (l == last) v = top;
    reg_heap_adjust(v, f, 0, last - f, val, lt);
  }
}
// key[f, f + n), n <= 64, remaining depth limit d: finished exactly as std::sort would.
template <class Lt>
__device__ void small_sort(uint64_t* key, int f, int n, int d, Lt lt) {
  const int l = lane_id();
  const unsigned long long ltm = (1ull << l) - 1ull;
  const unsigned long long lem = l == 63 ? ~0ull : (2ull << l) - 1ull;  // bits <= l
  uint64_t v = l < n ? key[f + l] : 0ull;
  int dep = d;                  // depth limit of the range starting at this lane
  unsigned long long bnd = 1ull, leafm = 0ull;
  int cur = 0;
  while (cur < n) {
    const unsigned long long above = cur == 63 ? 0ull : bnd & ~((2ull << cur) - 1ull);
    const int e = above ? __ffsll((long long)above) - 1 : n;
    const int dd = __builtin_amdgcn_readlane(dep, cur);
    if (e - cur <= 16) { leafm |= 1ull << cur; cur = e; continue; }
    if (dd == 0) { reg_heap_sort(v, cur, e, lt); leafm |= 1ull << cur; cur = e; continue; }
    // __move_median_to_first(first, first + 1, mid, last - 1)
    const int a = cur + 1, b = cur + (e - cur) / 2, c = e - 1;
    const uint64_t va = rdlane64(v, a), vb = rdlane64(v, b), vc = rdlane64(v, c);
    int mi;
    uint64_t vm;
    if (lt(va, vb)) {
      if (lt(vb, vc)) { mi = b; vm = vb; }
      else if (lt(va, vc)) { mi = c; vm = vc; }
      else { mi = a; vm = va; }
    } else if (lt(va, vc)) { mi = a; vm = va; }
    else if (lt(vb, vc)) { mi = c; vm = vc; }
    else { mi = b; vm = vb; }
    const uint64_t v0 = rdlane64(v, cur);
    if (l == cur) v = vm;
    else if (l == mi) v = v0;
    const uint64_t P = vm;
    // __unguarded_partition: stop lists L (ascending, (cur, e)) and R (descending, [cur, e))
    const unsigned long long mL = __ballot(l > cur && l < e && !lt(v, P));
    const unsigned long long mR = __ballot(l >= cur && l < e && !lt(P, v));
    const int nL = __popcll(mL), nR = __popcll(mR), nm = nL < nR ? nL : nR;
    const int Lk = l < nL ? select_bit(mL, l) : 64;
    const int Rk = l < nR ? select_bit(mR, nR - 1 - l) : -1;
    const int ks = __popcll(__ballot(l < nm && Lk < Rk));  // monotone: lanes 0 .. ks-1
    const int Lks = __builtin_amdgcn_readlane(Lk, ks < 63 ? ks : 63);
    const int Rks = __builtin_amdgcn_readlane(Rk, ks > 0 ? ks - 1 : 0);
    const int cut = (ks > 0 && (ks >= nL || Lks >= Rks)) ? Rks : Lks;
    // pairs k < ks swap L[k] <-> R[k]
    const int kL = __popcll(mL & ltm);
    const int kR = l == 63 ? 0 : __popcll(mR >> (l + 1));
    const int toR = __shfl(Rk, kL & 63), toL = __shfl(Lk, kR & 63);
    int src = l;
    if (((mL >> l) & 1ull) && kL < ks) src = toR;
    else if (((mR >> l) & 1ull) && kR < ks) src = toL;
    v = shfl64(v, src);
    if (l == cur || l == cut) dep = dd - 1;
    bnd |= 1ull << cut;
  }
  // each leaf's insertion sort = its stable sort
  const int s0 = 63 - __clzll((long long)(leafm & lem));
  const unsigned long long up = leafm & ~lem;
  const int t0 = up ? __ffsll((long long)up) - 1 : n;
  int len = l < n ? t0 - s0 : 0;
  int mx = len;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { const int y = __shfl_xor(mx, o); mx = y > mx ? y : mx; }
  int rank = 0;
  for (int q = 0; q < mx; ++q) {
    const int sq = s0 + q;
    const uint64_t w = shfl64(v, sq < 64 ? sq : 63);
    if (q < len && (lt(w, v) || (!lt(v, w) && sq < l))) ++rank;
  }
  if (l < n) key[f + s0 + rank] = v;
  wave_sync_lds();
}

// Executed by one full wave (64 lanes). Lp / Rp: n uint16 each; stk: 3 * kSortStack ints.
// key[0, n) ends up as std::sort leaves it. depth0 < 0: the whole array (depth limit 2 * lg(n));
// else a sub-range of a larger sort that inherits the remaining depth limit of its parent range
// (llsr_map.hip's segmented VoxelGrid). Ranges above 64 elements are partitioned in LDS; each range
// of at most 64 is finished in registers (small_sort).
template <class Lt>
__device__ void exact_introsort(uint64_t* key, int n, uint16_t* Lp, uint16_t* Rp, int* stk, Lt lt,
                                int depth0 = -1) {
  const int l = lane_id();
  const unsigned long long ltm = (1ull << l) - 1ull;
  wave_sync_lds();
  if (n <= 1) return;
  const int lg = 31 - __clz(n);
  int sp = 0;  // stack depth (wave-uniform)
  int rf = 0, rl = n, rd = depth0 < 0 ? 2 * lg : depth0;
  while (true) {
    bool heaped = false;
    while (rl - rf > 64) {
      if (rd == 0) {
        if (l == 0) heap_sort_range(key, rf, rl, lt);
        wave_sync_lds();
        heaped = true;
        break;
      }
      rd--;
      const int mid = rf + (rl - rf) / 2;
      if (l == 0) {  // __move_median_to_first(first, first+1, mid, last-1)
        const int a = rf + 1, b = mid, c = rl - 1;
        int m;
        if (lt(key[a], key[b])) m = lt(key[b], key[c]) ? b : (lt(key[a], key[c]) ? c : a);
        else m = lt(key[a], key[c]) ? a : (lt(key[b], key[c]) ? c : b);
        const uint64_t t = key[rf]; key[rf] = key[m]; key[m] = t;
      }
      wave_sync_lds();
      const uint64_t P = key[rf];
      int nL = 0, nR = 0;
      for (int c0 = rf + 1; c0 < rl; c0 += 64) {
        const int i = c0 + l;
        const bool f = i < rl && !lt(key[i], P);
        const unsigned long long m = __ballot(f);
        if (f) Lp[nL + __popcll(m & ltm)] = (uint16_t)i;
        nL += __popcll(m);
      }
      for (int c0 = rl - 1; c0 >= rf; c0 -= 64) {
        const int j = c0 - l;
        const bool f = j >= rf && !lt(P, key[j]);
        const unsigned long long m = __ballot(f);
        if (f) Rp[nR + __popcll(m & ltm)] = (uint16_t)j;
        nR += __popcll(m);
      }
      wave_sync_lds();
      const int nm = nL < nR ? nL : nR;
      int ks = nm;  // first k with !(L[k] < R[k]) (monotone)
      for (int c0 = 0; c0 < nm; c0 += 64) {
        const int k = c0 + l;
        const unsigned long long m = __ballot(k < nm && !(Lp[k] < Rp[k]));
        if (m) { ks = c0 + __ffsll((long long)m) - 1; break; }
      }
      const int cut = (ks > 0 && (ks >= nL || Lp[ks] >= Rp[ks - 1])) ? Rp[ks - 1] : Lp[ks];
      for (int k = l; k < ks; k += 64) {
        const int a = Lp[k], b = Rp[k];
        const uint64_t t = key[a]; key[a] = key[b]; key[b] = t;
      }
      wave_sync_lds();
      // the right part waits (at most one entry per level of the current path: <= 2*lg(n) + 1
      // <= 23 < kSortStack); the left part continues here
      if (l == 0) { stk[3 * sp] = cut; stk[3 * sp + 1] = rl; stk[3 * sp + 2] = rd; }
      ++sp;
      rl = cut;
    }
    if (!heaped && rl - rf > 1) small_sort(key, rf, rl - rf, rd, lt);
    wave_sync_lds();
    if (sp == 0) break;
    --sp;
    rf = stk[3 * sp]; rl = stk[3 * sp + 1]; rd = stk[3 * sp + 2];
  }
  wave_sync_lds();
}

// ---- the whole workgroup on one array ----------------------------------------------------------
// block_introsort: the same std::sort, with the ranges above 64 elements partitioned level by level
// by every thread of the workgroup at once. libstdc++'s recursion only ever touches disjoint
// sub-ranges, each carrying its own depth limit, so the order in which they are partitioned does
// not change the result: a level partitions every open range (> 64 elements, depth left) together.
// Per level each thread classifies a contiguous chunk of positions (L stop: !(a < pivot) in
// (first, last); R stop: !(pivot < a) in [first, last), as in exact_introsort) and ONE block scan of
// the packed (L, R) counts gives every stop its rank inside its range (ranks minus the range's base;
// R ranks counted from the right end). The stop lists go to Lp / Rp at the range's own offset, the
// pairs k < ks swap (the L side of pair k tests L[k] < R[k] and the last such k writes ks), and
// lane j of wave 0 computes range j's cut and children. Finished ranges (<= 64 elements, or depth 0:
// libstdc++'s heap sort) get a mark in their first key's payload bits 24-31 (which no caller uses:
// payloads are indices < 2^24; the comparators read only the high word); after the last level the
// marks are listed, stripped, and the waves finish the ranges round-robin (small_sort in registers,
// the rare heap sort by one lane). n <= 2048 = 8 positions per thread.
constexpr int kBsRanges = 32;  // open ranges have > 64 elements and are disjoint: < 2048 / 64
struct BlockSortLds {
  int first[kBsRanges], last[kBsRanges], dep[kBsRanges], ks[kBsRanges];
  int glf[kBsRanges], grf[kBsRanges], gll[kBsRanges], grl[kBsRanges];  // (L, R) stops before first / last
  uint64_t piv[kBsRanges];
  int scan[16];
  int na, nr;
};
constexpr uint32_t kBsMark = 0x80000000u;        // payload bit 31: a finished range starts here
constexpr uint64_t kBsStrip = ~0xFF000000ull;    // payload bits 24-31: the mark and the range's depth

template <int kNT, class Lt>
__device__ void block_introsort(uint64_t* key, int n, uint16_t* Lp, uint16_t* Rp, BlockSortLds& s, Lt lt) {
  static_assert(kNT % 64 == 0 && kNT * 8 >= 2048, "block_introsort: 8 positions per thread cover 2048");
  constexpr int kPer = 2048 / kNT;
  constexpr int kNW = kNT / 64;
  const int tid = threadIdx.x, l = lane_id(), w = tid >> 6;
  __syncthreads();  // key[0, n) written by the caller
  if (n <= 1) return;
  const int lg = 31 - __clz(n);
  if (n <= 64) {  // std::sort's whole loop inside one small range
    if (w == 0) small_sort(key, 0, n, 2 * lg, lt);
    __syncthreads();
    return;
  }
  if (tid == 0) {
    s.first[0] = 0;
    s.last[0] = n;
    s.dep[0] = 2 * lg;
    s.na = 1;
  }
  __syncthreads();
  const int per = (n + kNT - 1) / kNT;
  const int c0 = min(tid * per, n), c1 = min(c0 + per, n);
  // the open range holding position i, walking up from the chunk's first (ranges sorted by first)
  auto range_of = [&](int na, int& jj, int i) {
    while (jj + 1 < na && s.first[jj + 1] <= i) ++jj;
    return jj >= 0 && i < s.last[jj];
  };
  auto chunk_range = [&](int na) {  // the last range with first <= c0, or -1
    int lo = 0, hi = na - 1;
    if (s.first[0] > c0) return -1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s.first[mid] <= c0) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  while (true) {
    const int na = s.na;
    if (na == 0) break;
    // __move_median_to_first(first, first + 1, mid, last - 1); the pivot
    if (w == 0 && l < na) {
      const int f = s.first[l], e = s.last[l];
      const int a = f + 1, b = f + (e - f) / 2, c = e - 1;
      const uint64_t va = key[a], vb = key[b], vc = key[c];
      int m;
      if (lt(va, vb)) m = lt(vb, vc) ? b : (lt(va, vc) ? c : a);
      else m = lt(va, vc) ? a : (lt(vb, vc) ? c : b);
      const uint64_t vm = m == a ? va : (m == b ? vb : vc);
      key[m] = key[f];
      key[f] = vm;
      s.piv[l] = vm;
      s.ks[l] = 0;
    }
    __syncthreads();
    // stops of this thread's positions
    const int j0 = chunk_range(na);
    uint32_t mL = 0, mR = 0;
    {
      int jj = j0;
#pragma unroll 1
      for (int u = 0; u < kPer; ++u) {
        const int i = c0 + u;
        if (i >= c1 || !range_of(na, jj, i)) continue;
        const uint64_t v = key[i], P = s.piv[jj];
        if (i > s.first[jj] && !lt(v, P)) mL |= 1u << u;
        if (!lt(P, v)) mR |= 1u << u;
      }
    }
    int tot;
    const int ex = block_excl_scan((int)(__popc(mL) | (__popc(mR) << 16)), s.scan, &tot);
    const int gl0 = ex & 0xffff, gr0 = ex >> 16;  // stops before c0 (whole array)
    // each range's counts at its first and past its last position
    {
      int jj = j0;
#pragma unroll 1
      for (int u = 0; u < kPer; ++u) {
        const int i = c0 + u;
        if (i >= c1 || !range_of(na, jj, i)) continue;
        const uint32_t below = (1u << u) - 1u;
        const int gl = gl0 + __popc(mL & below), gr = gr0 + __popc(mR & below);
        if (i == s.first[jj]) { s.glf[jj] = gl; s.grf[jj] = gr; }
        if (i == s.last[jj] - 1) { s.gll[jj] = gl + (int)((mL >> u) & 1u); s.grl[jj] = gr + (int)((mR >> u) & 1u); }
      }
    }
    __syncthreads();
    // L[k] / R[k] at the range's offset (L ascending, R from the right end)
    {
      int jj = j0;
#pragma unroll 1
      for (int u = 0; u < kPer; ++u) {
        const int i = c0 + u;
        if (i >= c1 || !range_of(na, jj, i)) continue;
        const uint32_t below = (1u << u) - 1u;
        const int f = s.first[jj];
        if ((mL >> u) & 1u) Lp[f + gl0 + __popc(mL & below) - s.glf[jj]] = (uint16_t)i;
        if ((mR >> u) & 1u) Rp[f + s.grl[jj] - (gr0 + __popc(mR & below)) - 1] = (uint16_t)i;
      }
    }
    __syncthreads();
    // pairs k < ks swap; the L side of pair k checks L[k] < R[k] (monotone in k)
    {
      int jj = j0;
#pragma unroll 1
      for (int u = 0; u < kPer; ++u) {
        const int i = c0 + u;
        if (i >= c1 || !((mL >> u) & 1u) || !range_of(na, jj, i)) continue;
        const int f = s.first[jj];
        const int k = gl0 + __popc(mL & ((1u << u) - 1u)) - s.glf[jj];
        const int nL = s.gll[jj] - s.glf[jj], nR = s.grl[jj] - s.grf[jj], nm = nL < nR ? nL : nR;
        if (k < nm) {
          const int r = Rp[f + k];
          if (i < r) {
            const uint64_t a = key[i];
            key[i] = key[r];
            key[r] = a;
            if (!(k + 1 < nm && Lp[f + k + 1] < Rp[f + k + 1])) s.ks[jj] = k + 1;
          }
        }
      }
    }
    __syncthreads();
    // lane j of wave 0: range j's cut, its children; open ones (> 64, depth left) form the next
    // level's list in position order, the others get their start mark (and depth)
    if (w == 0) {
      int f = 0, e = 0, cut = 0, d = 0;
      bool o0 = false, o1 = false;
      if (l < na) {
        f = s.first[l];
        e = s.last[l];
        d = s.dep[l] - 1;
        const int ks = s.ks[l], nL = s.gll[l] - s.glf[l];
        cut = (ks > 0 && (ks >= nL || Lp[f + ks] >= Rp[f + ks - 1])) ? Rp[f + ks - 1] : Lp[f + ks];
        o0 = cut - f > 64 && d > 0;
        o1 = e - cut > 64 && d > 0;
        const uint64_t mk = (uint64_t)(kBsMark | ((uint32_t)d << 24));
        if (!o0 && cut > f) key[f] |= mk;
        if (!o1 && e > cut) key[cut] |= mk;
      }
      const int c = (o0 ? 1 : 0) + (o1 ? 1 : 0);
      const int incl = wave_incl_scan_add(c);
      const int ex0 = incl - c;
      const int nna = __builtin_amdgcn_readlane(incl, 63);
      wave_sync_lds();  // every lane has read its old entry
      if (o0) { s.first[ex0] = f; s.last[ex0] = cut; s.dep[ex0] = d; }
      if (o1) { const int o = ex0 + (o0 ? 1 : 0); s.first[o] = cut; s.last[o] = e; s.dep[o] = d; }
      if (l == 0) s.na = nna;
    }
    __syncthreads();
  }
  // list the finished ranges (starts -> Lp, depths -> Rp) and strip the marks
  uint32_t mk = 0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = c0 + u;
    if (i < c1 && ((uint32_t)key[i] & kBsMark)) mk |= 1u << u;
  }
  int nr;
  const int rb = block_excl_scan(__popc(mk), s.scan, &nr);
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    if (!((mk >> u) & 1u)) continue;
    const int i = c0 + u;
    const uint64_t v = key[i];
    const int k = rb + __popc(mk & ((1u << u) - 1u));
    Lp[k] = (uint16_t)i;
    Rp[k] = (uint16_t)(((uint32_t)v >> 24) & 0x7f);
    key[i] = v & kBsStrip;
  }
  __syncthreads();
  for (int k = w; k < nr; k += kNW) {
    const int f = Lp[k], e = k + 1 < nr ? Lp[k + 1] : n, d = Rp[k];
    if (e - f <= 64) {
      small_sort(key, f, e - f, d, lt);
    } else {  // depth exhausted above 64 elements: libstdc++'s __partial_sort of the range
      if (l == 0) heap_sort_range(key, f, e, lt);
      wave_sync_lds();
    }
  }
  __syncthreads();
}

}  // namespace llsr
