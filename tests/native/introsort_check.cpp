// introsort_check.cpp — TEST HARNESS (tests/test_introsort.py).
//
// The device reproduces libstdc++'s std::sort (bits/stl_algo.h: __introsort_loop with
// __move_median_to_first + __unguarded_partition, heap-sort fallback at depth 2*lg(n),
// __final_insertion_sort with threshold 16) for the per-ring curvature sort of
// extractFeaturesOurs (featureAssociation.cpp:1172), whose order of EQUAL values decides the
// greedy edge / flat selection. On the GPU each partition is computed by one wave in parallel:
//   * the k-th stop of the left scan in the ORIGINAL range is L_k (positions with !(a < pivot)),
//     the k-th stop of the right scan R_k (positions with !(pivot < a), from the right, down to
//     the pivot slot itself);
//   * k* = #{k : L_k < R_k} (monotone); pairs k < k* are swapped (disjoint positions);
//   * the cut is R_{k*-1} if k* > 0 and (L_{k*} does not exist or L_{k*} >= R_{k*-1}), else L_{k*};
//   * sub-ranges are independent, so they may be processed in any order (the depth limit travels
//     with each range); the final insertion sort never moves an element across a leaf boundary,
//     so it is one insertion sort per leaf block.
// This program checks that formulation (written serially here, the same arithmetic as
// llsr_fa.hip's exact_introsort) against std::sort on tie-heavy inputs, including inputs that
// exhaust the depth limit. Prints "<cases> <mismatches> <heap_fallbacks>"; exit 1 on mismatch.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <utility>
#include <vector>

using Elem = std::pair<float, int>;
static bool less_v(const Elem& a, const Elem& b) { return a.first < b.first; }

static void move_median_to_first(std::vector<Elem>& v, int result, int a, int b, int c) {
  if (less_v(v[a], v[b])) {
    if (less_v(v[b], v[c])) std::swap(v[result], v[b]);
    else if (less_v(v[a], v[c])) std::swap(v[result], v[c]);
    else std::swap(v[result], v[a]);
  } else if (less_v(v[a], v[c])) {
    std::swap(v[result], v[a]);
  } else if (less_v(v[b], v[c])) {
    std::swap(v[result], v[c]);
  } else {
    std::swap(v[result], v[b]);
  }
}

// libstdc++ __adjust_heap / __push_heap / __make_heap / __sort_heap on v[f, l)
static void push_heap(std::vector<Elem>& v, int f, int hole, int top, Elem val) {
  int parent = (hole - 1) / 2;
  while (hole > top && less_v(v[f + parent], val)) {
    v[f + hole] = v[f + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  v[f + hole] = val;
}
static void adjust_heap(std::vector<Elem>& v, int f, int hole, int len, Elem val) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (less_v(v[f + second], v[f + second - 1])) second--;
    v[f + hole] = v[f + second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    v[f + hole] = v[f + second - 1];
    hole = second - 1;
  }
  push_heap(v, f, hole, top, val);
}
static void heap_sort(std::vector<Elem>& v, int f, int l) {
  const int len = l - f;
  if (len >= 2) {
    for (int parent = (len - 2) / 2;; --parent) {
      adjust_heap(v, f, parent, len, v[f + parent]);
      if (parent == 0) break;
    }
  }
  for (int last = l; last - f > 1;) {
    --last;
    const Elem val = v[last];
    v[last] = v[f];
    adjust_heap(v, f, 0, last - f, val);
  }
}

static int heap_fallbacks = 0;

static void formulation_sort(std::vector<Elem>& v) {
  const int n = (int)v.size();
  if (n <= 1) return;
  int lg = 0;
  while ((2 << lg) <= n) ++lg;  // std::__lg(n)
  std::vector<char> bstart(n + 1, 0);
  struct R { int f, l, d; };
  std::vector<R> stack{{0, n, 2 * lg}};
  while (!stack.empty()) {
    R r = stack.back();
    stack.pop_back();
    while (r.l - r.f > 16) {
      if (r.d == 0) {
        heap_sort(v, r.f, r.l);
        ++heap_fallbacks;
        break;
      }
      r.d--;
      move_median_to_first(v, r.f, r.f + 1, r.f + (r.l - r.f) / 2, r.l - 1);
      const float P = v[r.f].first;
      std::vector<int> L, Rr;
      for (int i = r.f + 1; i < r.l; ++i)
        if (!(v[i].first < P)) L.push_back(i);
      for (int j = r.l - 1; j >= r.f; --j)
        if (!(P < v[j].first)) Rr.push_back(j);
      int ks = 0;
      while (ks < (int)L.size() && ks < (int)Rr.size() && L[ks] < Rr[ks]) ++ks;
      const int cut = (ks > 0 && (ks >= (int)L.size() || L[ks] >= Rr[ks - 1])) ? Rr[ks - 1] : L[ks];
      for (int k = 0; k < ks; ++k) std::swap(v[L[k]], v[Rr[k]]);
      stack.push_back({cut, r.l, r.d});
      r.l = cut;
    }
    bstart[r.f] = 1;
  }
  // one insertion sort per leaf block
  for (int s = 0; s < n;) {
    int e = s + 1;
    while (e < n && !bstart[e]) ++e;
    for (int i = s + 1; i < e; ++i) {
      const Elem val = v[i];
      int j = i;
      while (j > s && less_v(val, v[j - 1])) { v[j] = v[j - 1]; --j; }
      v[j] = val;
    }
    s = e;
  }
}

int main() {
  std::mt19937 g(20240607);
  int cases = 0, bad = 0;
  auto check = [&](std::vector<Elem> a) {
    std::vector<Elem> ref = a;
    std::sort(ref.begin(), ref.end(), less_v);
    formulation_sort(a);
    ++cases;
    for (size_t k = 0; k < a.size(); ++k)
      if (a[k].second != ref[k].second) { ++bad; return; }
  };
  for (int t = 0; t < 30000; ++t) {
    const int n = std::uniform_int_distribution<int>(0, t < 20000 ? 300 : 2048)(g);
    const int levels = std::uniform_int_distribution<int>(1, 40)(g);
    std::vector<Elem> a(n);
    for (int i = 0; i < n; ++i) a[i] = {(float)std::uniform_int_distribution<int>(0, levels)(g) * 0.25f, i};
    if (t % 5 == 0) std::sort(a.begin(), a.end(), less_v);                      // presorted
    if (t % 5 == 1) std::reverse(a.begin(), a.end());
    check(a);
  }
  // median-of-3 killers (Musser): exhaust the depth limit -> the heap-sort fallback
  for (int n : {64, 100, 250, 512, 1000, 2000, 2048}) {
    for (int ties = 0; ties < 2; ++ties) {
      std::vector<Elem> a(n);
      const int k = n / 2;
      for (int i = 0; i < k; ++i) {
        a[i] = {(float)((i % 2 == 0) ? i + 1 : k + i + (i % 2)), i};
        a[k + i] = {(float)(2 * (i + 1)), k + i};
      }
      if (ties)
        for (int i = 0; i < n; ++i) a[i].first = (float)((int)a[i].first / 3);
      check(a);
    }
  }
  printf("%d %d %d\n", cases, bad, heap_fallbacks);
  return bad ? 1 : 0;
}
