// llsr_isort.h — libstdc++'s std::sort reproduced exactly on the device, for the two places where
// the reference sorts with a comparator that ignores part of the element, so the order of EQUAL
// keys is whatever libstdc++'s introsort leaves and it changes results:
//   * the per-ring cloudSmoothness sort by value (FA:1172): the greedy edge / flat pick visits tied
//     candidates in that order (llsr_fa.hip);
//   * pcl::VoxelGrid's std::sort of (voxel id, point index) by voxel id (PCL 1.10 voxel_grid.hpp,
//     every downSizeFilter of FA / MO): each centroid sums its voxel's points in that order
//     (llsr_fa.hip's per-ring less-flat filter, llsr_map.hip's segmented filter).
// Keys are uint64 (sort key << 32 | payload) or uint32 (VoxLess32: dense voxel rank << 11 | candidate);
// the comparator reads the sort-key bits only.
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
// 32-bit VoxelGrid keys (dense voxel rank << 11 | candidate): the rank bits only
struct VoxLess32 {
  __device__ bool operator()(uint32_t a, uint32_t b) const { return (a >> 11) < (b >> 11); }
};
// `a < P` and `P < a` against one pivot P, as the partitions test every element of a range
template <class K, class Lt>
struct PivotTest {
  K P;
  Lt lt;
  __device__ PivotTest(K p, Lt l) : P(p), lt(l) {}
  __device__ bool below(K a) const { return lt(a, P); }
  __device__ bool above(K a) const { return lt(P, a); }
};
// VoxLess32 reads the rank bits (>> 11) only: a < P iff a < (P & ~0x7ff), P < a iff a > (P | 0x7ff),
// one compare of the whole key each
template <>
struct PivotTest<uint32_t, VoxLess32> {
  uint32_t lo, hi;
  __device__ PivotTest(uint32_t p, VoxLess32) : lo(p & ~0x7ffu), hi(p | 0x7ffu) {}
  __device__ bool below(uint32_t a) const { return a < lo; }
  __device__ bool above(uint32_t a) const { return a > hi; }
};
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// libstdc++ __adjust_heap (with __push_heap) on key[f, f+len), one lane
template <class K, class Lt>
__device__ void heap_adjust(K* key, int f, int hole, int len, K val, Lt lt) {
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
template <class K, class Lt>
__device__ void heap_sort_range(K* key, int f, int l, Lt lt) {
  const int len = l - f;
  if (len >= 2)
    for (int parent = (len - 2) / 2;; --parent) {
      heap_adjust(key, f, parent, len, key[f + parent], lt);
      if (parent == 0) break;
    }
  for (int last = l; last - f > 1;) {
    --last;
    const K val = key[last];
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
__device__ __forceinline__ uint64_t rdlane_k(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rdlane_k(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t shfl_k(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t shfl_k(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src); }
// the word the comparators read (VoxLess / CurvLess: the high word of a 64-bit key; a 32-bit key
// whole) and a key holding only that word
__device__ __forceinline__ uint32_t cmp_word(uint64_t k) { return (uint32_t)(k >> 32); }
__device__ __forceinline__ uint32_t cmp_word(uint32_t k) { return k; }
__device__ __forceinline__ void from_cmp_word(uint32_t w, uint64_t& k) { k = (uint64_t)w << 32; }
__device__ __forceinline__ void from_cmp_word(uint32_t w, uint32_t& k) { k = w; }
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
template <class K, class Lt>
__device__ void reg_heap_adjust(K& v, int f, int hole, int len, K val, Lt lt) {
  const int l = lane_id();
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (lt(rdlane_k(v, f + second), rdlane_k(v, f + second - 1))) second--;
    const K x = rdlane_k(v, f + second);
    if (l == f + hole) v = x;
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    const K x = rdlane_k(v, f + second - 1);
    if (l == f + hole) v = x;
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;
  while (hole > top && lt(rdlane_k(v, f + parent), val)) {
    const K x = rdlane_k(v, f + parent);
    if (l == f + hole) v = x;
    hole = parent;
    parent = (hole - 1) / 2;
  }
  if (l == f + hole) v = val;
}
template <class K, class Lt>
__device__ void reg_heap_sort(K& v, int f, int e, Lt lt) {
  const int l = lane_id();
  const int len = e - f;
  if (len >= 2)
    for (int parent = (len - 2) / 2;; --parent) {
      reg_heap_adjust(v, f, parent, len, rdlane_k(v, f + parent), lt);
      if (parent == 0) break;
    }
  for (int last = e; last - f > 1;) {
    --last;
    const K val = rdlane_k(v, last);
    const K top = rdlane_k(v, f);
    if (l == last) v = top;
    reg_heap_adjust(v, f, 0, last - f, val, lt);
  }
}
// key[f, f + n), n <= 64, holds one or more independent ranges (the set bits of `bnd`: their
// starts, bit 0 always set), each with its remaining depth limit in `dep` of its start lane; every
// range is finished exactly as std::sort would (libstdc++'s loop below 64 elements, then the final
// insertion sort of its leaves). The ranges' partitions run side by side: each lane works on the
// range that holds it (a segment of lanes), one partition step of every open segment per pass.
// Lp[f, f + n) and Rp[f, f + n) are scratch: each step lists a segment's L stops and R stops
// (ascending) at the segment's own offset as lane numbers, so the k-th pair, ks and the cut are LDS
// reads. A segment of at most 16 elements is a leaf; one above 16 whose depth limit is spent is
// heap-sorted in registers (rare), one segment at a time.
template <class K, class Lt>
__device__ void seg_small_sort(K* key, uint16_t* Lp, uint16_t* Rp, int f, int n, unsigned long long bnd,
                               int dep, Lt lt) {
  const int l = lane_id();
  const unsigned long long lem = l == 63 ? ~0ull : (2ull << l) - 1ull;  // bits <= l
  K v = l < n ? key[f + l] : K(0);
  auto seg_of = [&](int& s, int& e) {  // the segment [s, e) holding this lane
    s = 63 - __clzll((long long)(bnd & lem));
    const unsigned long long up = bnd & ~lem;
    e = up ? __ffsll((long long)up) - 1 : n;
  };
  {  // every lane holds its segment's depth limit (given on each range's first lane)
    int s, e;
    seg_of(s, e);
    dep = __shfl(dep, s);
  }
  while (true) {
    int s, e;
    seg_of(s, e);
    const int dd = dep;
    const bool work = l < n && e - s > 16 && dd > 0;
    if (!ballot(work)) break;
    const unsigned long long segm = (e >= 64 ? ~0ull : ((1ull << e) - 1ull)) & ~((1ull << s) - 1ull);
    // __move_median_to_first(first, first + 1, mid, last - 1) of this lane's segment
    const int a = s + 1, b = s + (e - s) / 2, c = e - 1;
    const K va = shfl_k(v, a & 63), vb = shfl_k(v, b & 63), vc = shfl_k(v, c & 63), v0 = shfl_k(v, s);
    int mi;
    K vm;
    if (lt(va, vb)) {
      if (lt(vb, vc)) { mi = b; vm = vb; }
      else if (lt(va, vc)) { mi = c; vm = vc; }
      else { mi = a; vm = va; }
    } else if (lt(va, vc)) { mi = a; vm = va; }
    else if (lt(vb, vc)) { mi = c; vm = vc; }
    else { mi = b; vm = vb; }
    if (work) {
      if (l == s) v = vm;
      else if (l == mi) v = v0;
    }
    const PivotTest<K, Lt> P(vm, lt);
    // __unguarded_partition: stop lists L ((s, e)) and R ([s, e)), ascending, in LDS; one round of
    // reads gives every lane its pair (k = l - s) and, for a stop, the partner it would swap with
    const bool isL = work && l > s && !P.below(v), isR = work && !P.above(v);
    const unsigned long long mL = ballot(isL), mR = ballot(isR);
    const int nL = __popcll(mL & segm), nR = __popcll(mR & segm), nm = nL < nR ? nL : nR;
    const int kL = lane_rank(mL & segm), kRa = lane_rank(mR & segm), kR = nR - 1 - kRa;
    uint16_t* L = Lp + f + s;
    uint16_t* R = Rp + f + s;
    if (isL) L[kL] = (uint16_t)l;
    if (isR) R[kRa] = (uint16_t)l;
    wave_sync_lds();
    const int k = l - s;
    const bool kin = work && k < nm;
    const int Lk = kin ? L[k] : 64, Rk = kin ? R[nR - 1 - k] : -1;
    const int pl = isL && kL < nm ? R[nR - 1 - kL] : l;  // L[kL]'s pair R_kL
    const int pr = isR && kR < nm ? L[kR] : l;           // R_kR's pair L[kR]
    wave_sync_lds();
    const int ks = __popcll(ballot(kin && Lk < Rk) & segm);  // monotone: the segment's first ks
    // L[ks] and R_{ks-1} (the k-th R stop from the right) are the lanes holding those ranks
    const unsigned long long bL = ballot(isL && kL == ks) & segm, bR = ballot(isR && kR == ks - 1) & segm;
    const int Lks = bL ? __ffsll((long long)bL) - 1 : 0;
    const int Rks = bR ? __ffsll((long long)bR) - 1 : 0;
    const int cut = (ks > 0 && (ks >= nL || Lks >= Rks)) ? Rks : Lks;
    // pairs k < ks swap L[k] <-> R_k
    const int src = isL && kL < ks ? pl : (isR && kR < ks ? pr : l);
    v = shfl_k(v, src);
    // both parts one level deeper; the cut starts the right part (none when cut == e)
    bnd |= ballot(work && l == cut);
    if (work) dep = dd - 1;
  }
  // segments above 16 with no depth left: libstdc++'s heap sort, in registers
  unsigned long long heapm = 0ull;
  {
    int s, e;
    seg_of(s, e);
    unsigned long long hs = ballot(l < n && l == s && e - s > 16 && dep == 0);
    heapm = hs;
    while (hs) {
      const int hs0 = __ffsll((long long)hs) - 1;
      hs &= hs - 1ull;
      const unsigned long long up = bnd & ~(hs0 == 63 ? ~0ull : (2ull << hs0) - 1ull);
      const int he = up ? __ffsll((long long)up) - 1 : n;
      reg_heap_sort(v, hs0, he, lt);
    }
  }
  // each leaf's insertion sort = its stable sort (<= 16 elements; a heap-sorted segment is sorted
  // already): the rank of every element among its leaf's, the leaf read back from LDS at once
  int s0, t0;
  seg_of(s0, t0);
  const int len = l < n ? t0 - s0 : 0;
  if (l < n) key[f + l] = v;
  wave_sync_lds();
  int rank = l - s0;
  if (l < n && !((heapm >> s0) & 1ull)) {
    rank = 0;
#pragma unroll
    for (int h = 0; h < 16; h += 8) {
      uint32_t w[8];  // the comparators read one word of the key (cmp_word)
#pragma unroll
      for (int q = 0; q < 8; ++q) w[q] = cmp_word(key[f + min(s0 + h + q, n - 1)]);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        K wq;
        from_cmp_word(w[q], wq);
        if (h + q < len && (lt(wq, v) || (!lt(v, wq) && s0 + h + q < l))) ++rank;
      }
    }
  }
  wave_sync_lds();
  if (l < n) key[f + s0 + rank] = v;
  wave_sync_lds();
}
// one range key[f, f + n), n <= 64, with depth limit d
template <class K, class Lt>
__device__ __forceinline__ void small_sort(K* key, uint16_t* Lp, uint16_t* Rp, int f, int n, int d, Lt lt) {
  seg_small_sort(key, Lp, Rp, f, n, 1ull, d, lt);
}

// ---- libstdc++'s heap sort of a range above 64 elements, by one wave ---------------------------
// __make_heap: the sift-downs of one depth touch disjoint subtrees, so a depth's parents run on
// parallel lanes (deepest depth first, as libstdc++'s decreasing parent order implies). Each pop
// (__pop_heap + __adjust_heap + __push_heap) is evaluated from the heap as it stands before it: the
// hole's path to a leaf follows the larger child (right unless right < left), chosen for a whole
// 6-level subtree below the hole at once (lane i loads the two children of subtree node i; the
// choices are one ballot, the walk a few scalar steps per level); the values move up the path by
// one place, and the popped value settles where __push_heap stops: above the deepest path
// position whose (moved-up) parent is not less than it, which is one ballot over the path.
template <class K, class Lt>
__device__ void wave_heap_sort(K* key, int f, int e, Lt lt) {
  const int l = lane_id();
  const int len0 = e - f;
  if (len0 < 2) return;
  {
    const int lastp = (len0 - 2) / 2;
    for (int d = 31 - __clz(lastp + 1); d >= 0; --d) {
      const int lo = (1 << d) - 1, hi = min((2 << d) - 2, lastp);
      for (int p = lo + l; p <= hi; p += 64) heap_adjust(key, f, p, len0, key[f + p], lt);
      wave_sync_lds();
    }
  }
  for (int len = len0 - 1; len >= 1; --len) {
    // __pop_heap(first, first + len + 1, first + len): value = last, last = root
    const K value = key[f + len];
    const K root = key[f];
    const int lim = (len - 1) / 2;
    int hole = 0, L = 0;
    int pnode = 0, pnext = 0;  // lane t < L: path node p_t and the child p_{t+1} the hole moved to
    K pchild = 0;       // lane t < L: the value of p_{t+1} before the pop
    bool more = hole < lim;
    while (more) {
      // the subtree of 63 nodes below the hole: lane i = its BFS node i, at absolute index a
      const int lv = 31 - __clz(l + 1);
      const int a = ((hole + 1) << lv) - 1 + (l + 1 - (1 << lv));
      bool right = false;
      K chosen = 0;
      if (l < 63 && a < lim) {
        const K cl = key[f + 2 * a + 1], cr = key[f + 2 * a + 2];
        right = !lt(cr, cl);  // __adjust_heap: second = right child, then -- if right < left
        chosen = right ? cr : cl;
      }
      const unsigned long long rm = ballot(right);
      int i = 0, ai = hole;
      for (int k = 0; k < 6; ++k) {
        if (!(ai < lim)) break;
        const int ci = 2 * i + ((rm >> i) & 1ull ? 2 : 1);
        const int ca = 2 * ai + ((rm >> i) & 1ull ? 2 : 1);
        const K cv = rdlane_k(chosen, i);
        if (l == L) { pnode = ai; pnext = ca; pchild = cv; }
        ++L;
        i = ci;
        ai = ca;
      }
      hole = ai;
      more = hole < lim;  // 6 levels done with the hole still above the last parent: next subtree
    }
    if ((len & 1) == 0 && hole == (len - 2) / 2) {  // the last parent's only (left) child
      const K cv = key[f + 2 * hole + 1];
      if (l == L) { pnode = hole; pnext = 2 * hole + 1; pchild = cv; }
      ++L;
      hole = 2 * hole + 1;
    }
    // __push_heap from the hole: path position t + 1 moves up while its new parent value (the old
    // value of p_{t+1}) is less than `value`; it stops at j = 1 + the deepest t < L where it is not
    const unsigned long long stay = ballot(l < L && !lt(pchild, value));
    const int j = stay ? 64 - __clzll((long long)stay) : 0;
    const int pj = __builtin_amdgcn_readlane(pnode, j < L ? j : 0);
    wave_sync_lds();
    if (l == 0) key[f + len] = root;
    if (l < j) key[f + pnode] = pchild;
    if (l == 0) key[f + (j < L ? pj : hole)] = value;
    wave_sync_lds();
    (void)pnext;
  }
}

// Executed by one full wave (64 lanes). Lp / Rp: n uint16 each; stk: 3 * kStack ints.
// key[0, n) ends up as std::sort leaves it. depth0 < 0: the whole array (depth limit 2 * lg(n));
// else a sub-range of a larger sort that inherits the remaining depth limit of its parent range
// (llsr_map.hip's segmented VoxelGrid, block_introsort's ranges). Ranges above 64 elements are
// partitioned in LDS: one pass lists the L stops (ascending) and the R stops (ascending; R[k], the
// k-th from the right, is Rp[nR - 1 - k]); each range of at most 64 is finished in registers
// (small_sort), a range above 64 whose depth limit is spent by wave_heap_sort. The stack holds at
// most one entry per level of the current path: <= depth limit + 1 entries.
template <class K, class Lt, int kStack = kSortStack>
__device__ void exact_introsort(K* key, int n, uint16_t* Lp, uint16_t* Rp, int* stk, Lt lt,
                                int depth0 = -1) {
  const int l = lane_id();
  wave_sync_lds();
  if (n <= 1) return;
  const int lg = 31 - __clz(n);
  int sp = 0;  // stack depth (wave-uniform)
  int rf = 0, rl = n, rd = depth0 < 0 ? 2 * lg : depth0;
  while (true) {
    bool heaped = false;
    while (rl - rf > 64) {
      if (rd == 0) {
        wave_heap_sort(key, rf, rl, lt);
        heaped = true;
        break;
      }
      rd--;
      // __move_median_to_first(first, first+1, mid, last-1)
      const int a = rf + 1, b = rf + (rl - rf) / 2, c = rl - 1;
      const K va = key[a], vb = key[b], vc = key[c], vf = key[rf];
      int m;
      if (lt(va, vb)) m = lt(vb, vc) ? b : (lt(va, vc) ? c : a);
      else m = lt(va, vc) ? a : (lt(vb, vc) ? c : b);
      const K P = m == a ? va : (m == b ? vb : vc);
      wave_sync_lds();
      if (l == 0) { key[m] = vf; key[rf] = P; }
      wave_sync_lds();
      int nL = 0, nR = 0;
      const PivotTest<K, Lt> pt(P, lt);
      for (int c0 = rf; c0 < rl; c0 += 64) {
        const int i = c0 + l;
        const K v = i < rl ? key[i] : K(0);
        const bool fl = i < rl && i > rf && !pt.below(v);
        const bool fr = i < rl && !pt.above(v);
        const unsigned long long in = lanes_below(rl - c0);
        const unsigned long long mL = in & (c0 == rf ? ~1ull : ~0ull) & ~ballot(pt.below(v)), mR = in & ~ballot(pt.above(v));
        if (fl) Lp[nL + lane_rank(mL)] = (uint16_t)i;
        if (fr) Rp[nR + lane_rank(mR)] = (uint16_t)i;
        nL += __popcll(mL);
        nR += __popcll(mR);
      }
      wave_sync_lds();
      const int nm = nL < nR ? nL : nR;
      int ks = nm;  // first k with !(L[k] < R[k]) (monotone)
      for (int c0 = 0; c0 < nm; c0 += 64) {
        const int k = c0 + l;
        const unsigned long long m = ballot(k < nm && !(Lp[k] < Rp[nR - 1 - k]));
        if (m) { ks = c0 + __ffsll((long long)m) - 1; break; }
      }
      const int cut = (ks > 0 && (ks >= nL || Lp[ks] >= Rp[nR - ks])) ? Rp[nR - ks] : Lp[ks];
      for (int k = l; k < ks; k += 64) {
        const int a2 = Lp[k], b2 = Rp[nR - 1 - k];
        const K t = key[a2]; key[a2] = key[b2]; key[b2] = t;
      }
      wave_sync_lds();
      // the right part waits; the left part continues here (one entry per level of the path: at
      // most the depth limit; a full stack traps instead of overrunning into its neighbours)
      if (sp >= kStack) __builtin_trap();
      if (l == 0) { stk[3 * sp] = cut; stk[3 * sp + 1] = rl; stk[3 * sp + 2] = rd; }
      ++sp;
      rl = cut;
    }
    if (!heaped && rl - rf > 1) small_sort(key, Lp, Rp, rf, rl - rf, rd, lt);
    wave_sync_lds();
    if (sp == 0) break;
    --sp;
    rf = stk[3 * sp]; rl = stk[3 * sp + 1]; rd = stk[3 * sp + 2];
  }
  wave_sync_lds();
}

// ---- the whole workgroup on one array ----------------------------------------------------------
// block_introsort: the same std::sort by the workgroup. libstdc++'s recursion only ever touches
// disjoint sub-ranges, each carrying its own depth limit, so the order in which they are processed
// does not change the result. Ranges above kBsBig elements (the top of the recursion, and the long
// chains of lopsided splits the voxel ids of a ring produce) are partitioned by the whole
// workgroup, one at a time (block_partition: each thread classifies a contiguous chunk, one block
// scan ranks the stops); every smaller range, or a large one whose depth limit is spent, goes to a
// list that is dealt to the waves (largest first, each to the least loaded wave). Each wave then
// finishes its ranges on its own as exact_introsort does: partition in LDS (stop lists at the
// range's own offset of Lp / Rp), continue with the left part, the right part on the wave's private
// stack; a range of at most 64 elements in registers (small_sort), one above 64 with no depth left
// by wave_heap_sort. n <= 2048.
constexpr int kBsBig = 512;
constexpr int kBsList = 64;   // the dealt ranges: two per block partition at most, and few of those
constexpr int kBsStack = 24;  // one entry per level of a path: <= depth limit (2 lg 2048 = 22) + 1
struct BlockSortLds {
  int rng[kBsList];             // first | last << 12 | depth << 24
  int owner[kBsList];           // the wave that finishes range k
  int big[kBsStack];            // the block's pending large ranges
  int stk[4][kBsStack];         // the waves' pending right parts
  int scan[16];
  int nr, ks;
  uint64_t piv;
};

// One libstdc++ partition step of key[rf, rl) by one wave (rf + 1 < rl): the median of three to
// rf, __unguarded_partition over (rf, rl) with the stop lists at Lp / Rp + rf; returns the cut.
template <class K, class Lt>
__device__ __forceinline__ int wave_partition(K* key, uint16_t* Lp, uint16_t* Rp, int rf, int rl, Lt lt) {
  const int l = lane_id();
  // __move_median_to_first(first, first+1, mid, last-1)
  const int a = rf + 1, b = rf + (rl - rf) / 2, c = rl - 1;
  const K va = key[a], vb = key[b], vc = key[c], vf = key[rf];
  int m;
  if (lt(va, vb)) m = lt(vb, vc) ? b : (lt(va, vc) ? c : a);
  else m = lt(va, vc) ? a : (lt(vb, vc) ? c : b);
  const K P = m == a ? va : (m == b ? vb : vc);
  wave_sync_lds();
  if (l == 0) { key[m] = vf; key[rf] = P; }
  wave_sync_lds();
  // __unguarded_partition: L stops (!(a < P), (rf, rl)) and R stops (!(P < a), [rf, rl)), both
  // listed ascending (R[k], the k-th from the right, is Rp[nR - 1 - k]); two chunks of 64 per step
  int nL = 0, nR = 0;
  const PivotTest<K, Lt> pt(P, lt);
  for (int c0 = rf; c0 < rl; c0 += 128) {
    const int i0 = c0 + l, i1 = c0 + 64 + l;
    const K v0 = i0 < rl ? key[i0] : K(0), v1 = i1 < rl ? key[i1] : K(0);
    const bool fl0 = i0 < rl && i0 > rf && !pt.below(v0), fr0 = i0 < rl && !pt.above(v0);
    const bool fl1 = i1 < rl && !pt.below(v1), fr1 = i1 < rl && !pt.above(v1);
    // the masks from one ballot per key compare, the index bounds as scalar masks (a ballot of a
    // combined predicate is materialised per lane and compared again)
    const unsigned long long in0 = lanes_below(rl - c0), in1 = lanes_below(rl - c0 - 64);
    const unsigned long long mL0 = in0 & (c0 == rf ? ~1ull : ~0ull) & ~ballot(pt.below(v0)), mR0 = in0 & ~ballot(pt.above(v0));
    const unsigned long long mL1 = in1 & ~ballot(pt.below(v1)), mR1 = in1 & ~ballot(pt.above(v1));
    const int nL1 = nL + __popcll(mL0), nR1 = nR + __popcll(mR0);
    if (fl0) Lp[rf + nL + lane_rank(mL0)] = (uint16_t)i0;
    if (fr0) Rp[rf + nR + lane_rank(mR0)] = (uint16_t)i0;
    if (fl1) Lp[rf + nL1 + lane_rank(mL1)] = (uint16_t)i1;
    if (fr1) Rp[rf + nR1 + lane_rank(mR1)] = (uint16_t)i1;
    nL = nL1 + __popcll(mL1);
    nR = nR1 + __popcll(mR1);
  }
  wave_sync_lds();
  const uint16_t* L = Lp + rf;
  const uint16_t* R = Rp + rf;
  const int nm = nL < nR ? nL : nR;
  int ks = nm;  // first k with !(L[k] < R[k]) (monotone)
  for (int c0 = 0; c0 < nm; c0 += 128) {
    const int k0 = c0 + l, k1 = c0 + 64 + l;
    const int a0 = k0 < nm ? L[k0] : 0, b0 = k0 < nm ? R[nR - 1 - k0] : 0;
    const int a1 = k1 < nm ? L[k1] : 0, b1 = k1 < nm ? R[nR - 1 - k1] : 0;
    const unsigned long long m0 = ballot(k0 < nm && !(a0 < b0)), m1 = ballot(k1 < nm && !(a1 < b1));
    if (m0) { ks = c0 + __ffsll((long long)m0) - 1; break; }
    if (m1) { ks = c0 + 64 + __ffsll((long long)m1) - 1; break; }
  }
  const int cut = (ks > 0 && (ks >= nL || L[ks] >= R[nR - ks])) ? R[nR - ks] : L[ks];
  for (int k0 = l; k0 < ks; k0 += 128) {
    const int k1 = k0 + 64;
    const bool two = k1 < ks;
    const int x0 = L[k0], y0 = R[nR - 1 - k0];
    const int x1 = two ? L[k1] : 0, y1 = two ? R[nR - 1 - k1] : 0;
    const K p0 = key[x0], q0 = key[y0];
    const K p1 = two ? key[x1] : K(0), q1 = two ? key[y1] : K(0);
    key[x0] = q0;
    key[y0] = p0;
    if (two) { key[x1] = q1; key[y1] = p1; }
  }
  wave_sync_lds();
  return cut;
}

// One libstdc++ partition step of key[rf, rl) by the whole workgroup (kNT threads); returns the
// cut (uniform). Thread t classifies positions [rf + t * per, +per); one block scan of the packed
// (L, R) stop counts gives every stop its rank; the first k with !(L[k] < R[k]) is an LDS min.
template <int kNT, class K, class Lt>
__device__ __forceinline__ int block_partition(K* key, uint16_t* Lp, uint16_t* Rp, int rf, int rl, BlockSortLds& s,
                                               Lt lt) {
  const int tid = threadIdx.x;
  if (tid == 0) {  // __move_median_to_first(first, first+1, mid, last-1)
    const int a = rf + 1, b = rf + (rl - rf) / 2, c = rl - 1;
    const K va = key[a], vb = key[b], vc = key[c], vf = key[rf];
    int m;
    if (lt(va, vb)) m = lt(vb, vc) ? b : (lt(va, vc) ? c : a);
    else m = lt(va, vc) ? a : (lt(vb, vc) ? c : b);
    const K P = m == a ? va : (m == b ? vb : vc);
    key[m] = vf;
    key[rf] = P;
    s.piv = P;
    s.ks = 0x7fffffff;
  }
  __syncthreads();
  const PivotTest<K, Lt> pt((K)s.piv, lt);
  const int per = (rl - rf + kNT - 1) / kNT;
  const int c0 = min(rf + tid * per, rl), c1 = min(c0 + per, rl);
  uint32_t mL = 0, mR = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int i = c0 + u;
    if (i >= c1) continue;
    const K v = key[i];
    if (i > rf && !pt.below(v)) mL |= 1u << u;
    if (!pt.above(v)) mR |= 1u << u;
  }
  int tot;
  const int ex = block_excl_scan((int)(__popc(mL) | (__popc(mR) << 16)), s.scan, &tot);
  const int nL = tot & 0xffff, nR = tot >> 16;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t below = (1u << u) - 1u;
    if ((mL >> u) & 1u) Lp[rf + (ex & 0xffff) + __popc(mL & below)] = (uint16_t)(c0 + u);
    if ((mR >> u) & 1u) Rp[rf + (ex >> 16) + __popc(mR & below)] = (uint16_t)(c0 + u);
  }
  __syncthreads();
  const uint16_t* L = Lp + rf;
  const uint16_t* R = Rp + rf;
  const int nm = nL < nR ? nL : nR;
  {  // ks = the first k with !(L[k] < R[k]) (monotone), nm if none
    const int pk = (nm + kNT - 1) / kNT;
    const int k0 = min(tid * pk, nm), k1 = min(k0 + pk, nm);
    int kf = 0x7fffffff;
    for (int k = k0; k < k1; ++k)
      if (!(L[k] < R[nR - 1 - k])) { kf = k; break; }
    if (kf != 0x7fffffff) atomicMin(&s.ks, kf);
  }
  __syncthreads();
  const int ks = min(s.ks, nm);
  {
    const int pk = (ks + kNT - 1) / kNT;
    const int k0 = min(tid * pk, ks), k1 = min(k0 + pk, ks);
    for (int k = k0; k < k1; ++k) {
      const int x = L[k], y = R[nR - 1 - k];
      const K t = key[x];
      key[x] = key[y];
      key[y] = t;
    }
  }
  const int cut = (ks > 0 && (ks >= nL || L[ks] >= R[nR - ks])) ? R[nR - ks] : L[ks];
  __syncthreads();
  return cut;
}

// prof (diagnostics only, k_debug_exact_sort): prof[0] = clocks of the block-wide part; per wave w,
// prof[1 + 4 w + 0..3] = clocks in wave partitions, small_sort, wave_heap_sort, and idle at the end
template <int kNT, class K, class Lt>
__device__ __forceinline__ void block_introsort(K* key, int n, uint16_t* Lp, uint16_t* Rp, BlockSortLds& s, Lt lt,
                                                long long* prof = nullptr, int stop = 1 << 30) {
  static_assert(kNT == 256, "block_introsort: four waves");
  const int tid = threadIdx.x, l = lane_id(), w = tid >> 6;
  long long tc = prof ? clock64() : 0, tpw = 0, tsm = 0, thp = 0;
  auto stamp = [&](long long& acc) {
    if (prof) {
      const long long t1 = clock64();
      acc += t1 - tc;
      tc = t1;
    }
  };
  __syncthreads();  // key[0, n) written by the caller
  if (n <= 1) return;
  const int lg = 31 - __clz(n);
  if (n <= 64) {  // std::sort's whole loop inside one small range
    if (w == 0) small_sort(key, Lp, Rp, 0, n, 2 * lg, lt);
    __syncthreads();
    return;
  }
  auto enc = [](int f, int e, int d) { return f | (e << 12) | (d << 24); };
  // large ranges, block-wide, left part first (the right part waits on the block's stack); the
  // counters are uniform copies every thread keeps (thread 0 writes the arrays). Near a full list
  // the remaining ranges go to the list as they are (the waves finish any size).
  {
    int rf = 0, rl = n, rd = 2 * lg;
    int nbig = 0, nr = 0;
    while (true) {
      while (rl - rf > kBsBig && rd > 0 && nr < kBsList - 2) {
        rd--;
        const int cut = block_partition<kNT>(key, Lp, Rp, rf, rl, s, lt);
        if (rl - cut > kBsBig && rd > 0) {
          if (nbig >= kBsStack) __builtin_trap();  // cannot: <= one entry per level of the path
          if (tid == 0) s.big[nbig] = enc(cut, rl, rd);
          ++nbig;
        } else if (rl > cut) {
          if (tid == 0) s.rng[nr] = enc(cut, rl, rd);
          ++nr;
        }
        rl = cut;
      }
      if (rl > rf) {
        if (tid == 0) s.rng[nr] = enc(rf, rl, rd);
        ++nr;
      }
      if (nbig == 0) break;
      __syncthreads();
      --nbig;
      const int it = s.big[nbig];
      rf = it & 0xfff;
      rl = (it >> 12) & 0xfff;
      rd = (it >> 24) & 0x3f;
    }
    if (tid == 0) s.nr = nr;
  }
  __syncthreads();
  if (prof && tid == 0) prof[0] = clock64() - tc;
  if (stop <= 0) return;  // diagnostics (phase timing): the block-wide part only
  // deal the list: largest first, each to the least loaded wave (elements as the load)
  if (w == 0) {
    const int cnt = s.nr;
    const int sz = l < cnt ? ((s.rng[l] >> 12) & 0xfff) - (s.rng[l] & 0xfff) : -1;
    if (l == 0) {
      int ld0 = 0, ld1 = 0, ld2 = 0, ld3 = 0;
      unsigned long long taken = 0;
      for (int r = 0; r < cnt; ++r) {
        int best = 0, bs = -1;
        for (int k = 0; k < cnt; ++k) {
          const int z = __builtin_amdgcn_readlane(sz, k);
          if (!((taken >> k) & 1ull) && z > bs) { bs = z; best = k; }
        }
        taken |= 1ull << best;
        const int m01 = min(ld0, ld1), m23 = min(ld2, ld3);
        const int wm = m01 <= m23 ? (ld0 <= ld1 ? 0 : 1) : (ld2 <= ld3 ? 2 : 3);
        if (wm == 0) ld0 += bs; else if (wm == 1) ld1 += bs; else if (wm == 2) ld2 += bs; else ld3 += bs;
        s.owner[best] = wm;
      }
    }
  }
  __syncthreads();
  // every wave finishes its ranges alone; consecutive ranges of at most 64 elements (left-first
  // order emits them in position order) are collected in a window of <= 64 lanes and finished
  // together by seg_small_sort
  const int nr = s.nr;
  int* stk = s.stk[w];
  if (prof) tc = clock64();
  int wf = 0, wn = 0, wdep = 0;
  unsigned long long wb = 0ull;
  auto flush = [&]() {
    if (wn > 1 && stop > 1) seg_small_sort(key, Lp, Rp, wf, wn, wb, wdep, lt);  // stop 1: partitions only
    wn = 0;
  };
  auto emit = [&](int rf, int rl, int rd) {
    const int len = rl - rf;
    if (len <= 0) return;
    if (wn > 0 && rf == wf + wn && wn + len <= 64) {
      wb |= 1ull << wn;
      if (l == wn) wdep = rd;
      wn += len;
    } else {
      flush();
      wf = rf;
      wn = len;
      wb = 1ull;
      if (l == 0) wdep = rd;
    }
  };
  for (int k = 0; k < nr; ++k) {
    if (s.owner[k] != w) continue;
    const int it = s.rng[k];
    int rf = it & 0xfff, rl = (it >> 12) & 0xfff, rd = (it >> 24) & 0x3f;
    int sp = 0;
    while (true) {
      while (rl - rf > 64 && rd > 0) {
        rd--;
        const int cut = wave_partition(key, Lp, Rp, rf, rl, lt);
        if (sp >= kBsStack) __builtin_trap();  // cannot: <= one entry per level of the path
        if (l == 0) stk[sp] = enc(cut, rl, rd);
        ++sp;
        rl = cut;
      }
      stamp(tpw);
      if (rl - rf > 64) {
        wave_heap_sort(key, rf, rl, lt);  // depth limit spent: __partial_sort
        stamp(thp);
      } else {
        emit(rf, rl, rd);
        stamp(tsm);
      }
      wave_sync_lds();
      if (sp == 0) break;
      --sp;
      const int nx = stk[sp];
      rf = nx & 0xfff;
      rl = (nx >> 12) & 0xfff;
      rd = (nx >> 24) & 0x3f;
    }
  }
  flush();
  stamp(tsm);
  long long tend = prof ? clock64() : 0;
  __syncthreads();
  if (prof && l == 0) {
    prof[1 + 4 * w] = tpw; prof[2 + 4 * w] = tsm; prof[3 + 4 * w] = thp; prof[4 + 4 * w] = clock64() - tend;
  }
}

}  // namespace llsr
