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
// Executed by one full wave (64 lanes). Lp / Rp: n uint16 each; stk: 3 * kSortStack ints;
// leaf: (n + 64) / 64 uint64 words. Returns nothing; key[0, n) ends up as std::sort leaves it.
// depth0 < 0: the whole array (depth limit 2 * lg(n)); else a sub-range of a larger sort that
// inherits the remaining depth limit of its parent range (llsr_map.hip's segmented VoxelGrid).
template <class Lt>
__device__ void exact_introsort(uint64_t* key, int n, uint16_t* Lp, uint16_t* Rp, int* stk, uint64_t* leaf, Lt lt,
                                int depth0 = -1) {
  const int l = lane_id();
  const unsigned long long ltm = (1ull << l) - 1ull;
  for (int w = l; w <= (n >> 6); w += 64) leaf[w] = 0ull;
  wave_sync_lds();
  if (n <= 1) return;
  const int lg = 31 - __clz(n);
  int sp = 0;  // stack depth (wave-uniform)
  int rf = 0, rl = n, rd = depth0 < 0 ? 2 * lg : depth0;
  while (true) {
    while (rl - rf > 16) {
      if (rd == 0) {
        if (l == 0) heap_sort_range(key, rf, rl, lt);
        wave_sync_lds();
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
    if (l == 0) leaf[rf >> 6] |= 1ull << (rf & 63);
    wave_sync_lds();
    if (sp == 0) break;
    --sp;
    rf = stk[3 * sp]; rl = stk[3 * sp + 1]; rd = stk[3 * sp + 2];
  }
  // one insertion sort per leaf block: lane w takes the leaves starting in word w, w + 64, ...
  const int nw = (n + 63) >> 6;
  for (int w = l; w < nw; w += 64) {
    uint64_t bits = leaf[w];
    while (bits) {
      const int s0 = (w << 6) + __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      int e = n;  // next leaf start after s0
      if (bits) {
        e = (w << 6) + __ffsll((long long)bits) - 1;
      } else {
        for (int w2 = w + 1; w2 < nw; ++w2)
          if (leaf[w2]) { e = (w2 << 6) + __ffsll((long long)leaf[w2]) - 1; break; }
      }
      for (int i = s0 + 1; i < e; ++i) {
        const uint64_t val = key[i];
        int j = i;
        while (j > s0 && lt(val, key[j - 1])) { key[j] = key[j - 1]; --j; }
        key[j] = val;
      }
    }
  }
  wave_sync_lds();
}


}  // namespace llsr
