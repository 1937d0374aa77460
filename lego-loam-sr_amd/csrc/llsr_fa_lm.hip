// llsr_fa_lm.hip — FeatureAssociation scan-to-scan LM on gfx950 (updateTransformation,
// featureAssociation.cpp:2505-2535) for a batch of independent scans.
//
// k_s2s_lm: one kThreads-thread workgroup per scan (512, or 256 for the <1024, 1024> instantiation,
// llsr_s2s.h) runs the whole two-phase optimisation in-kernel
// (no host round trips): surf phase (FA:2508-2516) then corner phase (FA:2519-2527), each up to
// 100 iterations. Per iteration:
//   A  on iterations % 5 == 0 the kNN-1 of every query (q = tid, tid + kThreads, ...) after
//      TransformToStart (FA:1389-1412) in the last cloud: the sparse corner cloud is scanned from
//      LDS, the surf cloud searched over shells of its 1 m cell grid (llsr_grid.h), and queries
//      the shells leave open are resolved by a block-wide scan; then the ring-constrained scans
//      for the second / third tripod point in the last cloud's own order (FA:1588-1647,
//      1737-1803). Every iteration: the line / plane coefficient (FA:1650-1695, 1806-1842) and
//      the Jacobian row of calculateTransformation{Surf,Corner} (FA:1893-1913, 2046-2062) into an
//      LDS row buffer (zeros without a correspondence; the valid rows are counted);
//   B  12 lanes of wave 0 sum the rows in correspondence order — one lane per entry of the
//      3x3 AtA / 3-vector AtB — the oracle's summation order exactly;
//   C  thread 0: ColPivHouseholderQR solve, SelfAdjointEigenSolver degeneracy test at
//      iteration 0, projection, pose update, NaN reset, stop test (FA:1915-2009, 2064-2142).
// Float / double typing follows each reference line, sin/cos are the glibc ports, so results
// are bit-identical to the CPU restatement (oracle/oracle_fa_lm.cpp).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "llsr_device.h"
#include "llsr_eigen.h"
#include "llsr_grid.h"
#include "llsr_isort.h"
#include "llsr_s2s.h"

namespace llsr {

using llsr_libm::cosf_;
using llsr_libm::fabs_;
using llsr_libm::fbits;
using llsr_libm::sinf_;
using llsr_libm::sqrt_;

namespace {

constexpr int kMaxShell = 2;  // grid shells searched before the exact block-wide scan (queries in sparse regions)
constexpr int kFbMax = 256;       // queries per kNN iteration whose shells did not settle (block scan)
constexpr int kIx = 5;            // ints per query in S2SArgs::idx
constexpr int kWalkBudget = 200;  // per-lane surf walk steps before the whole-wave walk takes over

// TransformToStart (FA:1389-1412)
__device__ __forceinline__ float4 to_start(const float* t, float4 pi) {
  const float s = 10 * (pi.w - (float)trunc_i32(pi.w));
  const float rx = s * t[0], ry = s * t[1], rz = s * t[2];
  const float tx = s * t[3], ty = s * t[4], tz = s * t[5];
  const float crz = cosf_(rz), srz = sinf_(rz);
  const float crx = cosf_(rx), srx = sinf_(rx);
  const float cry = cosf_(ry), sry = sinf_(ry);
  const float x1 = crz * (pi.x - tx) + srz * (pi.y - ty);
  const float y1 = -srz * (pi.x - tx) + crz * (pi.y - ty);
  const float z1 = (pi.z - tz);
  const float x2 = x1;
  const float y2 = crx * y1 + srx * z1;
  const float z2 = -srx * y1 + crx * z1;
  return make_float4(cry * x2 - sry * z2, y2, sry * x2 + cry * z2, pi.w);
}

// (last - sel)^2 as written at FA:1609-1614
__device__ __forceinline__ float sqdis(float4 a, float4 b) {
  return (a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z);
}

// nanoflann L2_Simple (query - point), accumulated from 0
__device__ __forceinline__ float l2(float4 q, float4 p) {
  float d = 0.0f, t;
  t = q.x - p.x; d += t * t;
  t = q.y - p.y; d += t * t;
  t = q.z - p.z; d += t * t;
  return d;
}

// Nearest neighbour of q in grid g of problem p (KdTreeFLANN::nearestKSearch, k = 1; ties ->
// lower index) over growing shells of 1 m cells. Returns true once the searched shells provably
// contain the nearest point or nothing nearer than dist_sqr can remain outside them; false when
// kMaxShell shells do not settle it (the caller then scans the whole cloud, nn1_block).
// (bi, bd) may start from a known point of the cloud (the previous kNN pass's answer: a real
// candidate, so the lexicographic minimum is unchanged) — cells farther than it are not probed.
__device__ bool nn1_shells(const CellGrid& g, int p, float4 q, float dist_sqr, int& bi, float& bd) {
  const CellSlot* tab = g.table(p);
  const float4* pts = g.cells(p);
  const int cx = cell_coord(q.x), cy = cell_coord(q.y), cz = cell_coord(q.z);
  // squared gap of q to the cell slab at offset dd along one axis, rounded as l2 rounds: a point
  // of that slab has |fl(q - p)| >= this gap (rounding is monotone and symmetric)
  auto gap2 = [](float v, int c, int dd) {
    const float g = dd < 0 ? v - (float)(c + dd + 1) : dd > 0 ? (float)(c + dd) - v : 0.0f;
    return g * g;
  };
  for (int h = 0; h <= kMaxShell; ++h) {
    for (int dx = -h; dx <= h; ++dx)
      for (int dy = -h; dy <= h; ++dy) {
        const int step = (h == 0 || dx == -h || dx == h || dy == -h || dy == h) ? 1 : 2 * h;
        const float lxy = gap2(q.x, cx, dx) + gap2(q.y, cy, dy);
        for (int dz = -h; dz <= h; dz += step) {
          // a cell whose every point is farther than bd cannot change the (d, index) minimum, and
          // one with none nearer than dist_sqr cannot give a correspondence (finish rejects nd >= it)
          const float lb = lxy + gap2(q.z, cz, dz);
          if (lb > bd || lb >= dist_sqr) continue;
          const int s = grid_find(tab, g.log2T, cell_key(cx + dx, cy + dy, cz + dz));
          if (s < 0) continue;
          const int st = tab[s].start, n = tab[s].count;
          for (int j = st; j < st + n; ++j) {
            const float4 c = pts[j];
            const float d = l2(q, c);
            const int id = (int)fbits(c.w);
            if (nn_before(d, id, bd, bi)) { bd = d; bi = id; }
          }
        }
      }
    // every point outside the searched block is at least r away (float slack 1e-5)
    float r = q.x - (float)(cx - h);
    r = fminf(r, (float)(cx + h + 1) - q.x);
    r = fminf(r, q.y - (float)(cy - h));
    r = fminf(r, (float)(cy + h + 1) - q.y);
    r = fminf(r, q.z - (float)(cz - h));
    r = fminf(r, (float)(cz + h + 1) - q.z);
    const float r2 = r * r * (1.0f - 1e-5f);
    if (bd < r2 || r2 >= dist_sqr) return true;
  }
  return false;
}

// Exact nearest neighbour by a scan in index order with strict '<' (ties -> lower index, as the
// shells).
__device__ __forceinline__ void nn1_scan(const float4* pts, int n, float4 q, int& bi, float& bd) {
  bd = INFINITY;
  bi = INT_MAX;
  for (int k = 0; k < n; ++k) {
    const float d = l2(q, pts[k]);
    if (d < bd) { bd = d; bi = k; }
  }
}

// nn1_scan for up to kMulti queries at once by the whole block: each thread scans an interleaved
// slice of the cloud in index order against every query, then each query's (d, index) minima are
// reduced with the index tie-break — equal to nn1_scan per query, with one pass over the cloud
// for kMulti queries. Contains barriers: every thread of the block must call it.
constexpr int kMulti = 2;  // 2 (from 4): 113 instead of 166 spilled VGPRs at the 4-waves bound
template <int kNT>
__device__ void nn1_block_multi(const float4* pts, int n, const float4* qs, int nq, int* bi, float* bd,
                                float (*red_d)[kNT / 64], int (*red_i)[kNT / 64]) {
  float d[kMulti];
  int id[kMulti];
#pragma unroll
  for (int j = 0; j < kMulti; ++j) { d[j] = INFINITY; id[j] = INT_MAX; }
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const float4 p = pts[k];
#pragma unroll
    for (int j = 0; j < kMulti; ++j)
      if (j < nq) {
        const float dd = l2(qs[j], p);
        if (dd < d[j]) { d[j] = dd; id[j] = k; }
      }
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int j = 0; j < kMulti; ++j) {
    for (int off = 32; off; off >>= 1) {
      const float od = __shfl_xor(d[j], off, 64);
      const int oi = __shfl_xor(id[j], off, 64);
      if (nn_before(od, oi, d[j], id[j])) { d[j] = od; id[j] = oi; }
    }
    if (lane_id() == 0) { red_d[j][w] = d[j]; red_i[j][w] = id[j]; }
  }
  __syncthreads();
  for (int j = 0; j < nq; ++j) {
    float bdj = red_d[j][0];
    int bij = red_i[j][0];
    for (int k = 1; k < nw; ++k)
      if (nn_before(red_d[j][k], red_i[j][k], bdj, bij)) { bdj = red_d[j][k]; bij = red_i[j][k]; }
    bd[j] = bdj;
    bi[j] = bij;
  }
  __syncthreads();
}

// findCorrespondingCornerFeatures search (FA:1587-1648) around the nearest neighbour nn (squared
// distance nd); `fwd` = the reference's forward bound (cornerPointsSharpNum), clamped to the last
// cloud.
// The two linear scans of the tripod searches walk the last cloud away from the nearest neighbour
// until the ring leaves [cs - 2.5, cs + 2.5]; they read 8 points per step (all loads in flight at
// once) and replay the serial test on them in order, so the result is the serial loop's.
constexpr int kScan = 8;

template <class Visit>
__device__ __forceinline__ void scan_up(const float4* pts, int from, int end, int cs, Visit visit) {
  for (int j0 = from; j0 < end; j0 += kScan) {
    float4 c[kScan];
#pragma unroll
    for (int u = 0; u < kScan; ++u) c[u] = j0 + u < end ? pts[j0 + u] : make_float4(0.f, 0.f, 0.f, 0.f);
    bool stop = false;
#pragma unroll
    for (int u = 0; u < kScan; ++u) {
      if (stop || j0 + u >= end) continue;
      const int rj = trunc_i32(c[u].w);
      if ((double)rj > (double)cs + 2.5) stop = true;
      else visit(j0 + u, c[u], rj);
    }
    if (stop) return;
  }
}

template <class Visit>
__device__ __forceinline__ void scan_down(const float4* pts, int from, int cs, Visit visit) {
  for (int j0 = from; j0 >= 0; j0 -= kScan) {
    float4 c[kScan];
#pragma unroll
    for (int u = 0; u < kScan; ++u) c[u] = j0 - u >= 0 ? pts[j0 - u] : make_float4(0.f, 0.f, 0.f, 0.f);
    bool stop = false;
#pragma unroll
    for (int u = 0; u < kScan; ++u) {
      if (stop || j0 - u < 0) continue;
      const int rj = trunc_i32(c[u].w);
      if ((double)rj < (double)cs - 2.5) stop = true;
      else visit(j0 - u, c[u], rj);
    }
    if (stop) return;
  }
}

// findCorrespondingCornerFeatures search (FA:1587-1648) around the nearest neighbour nn (squared
// distance nd); `fwd` = the reference's forward bound (cornerPointsSharpNum), clamped to the last
// cloud.
__device__ void corner_finish(const float4* cl, int Nc, int fwd, float4 sel, float dist_sqr, int nn, float nd,
                              int& i1, int& i2) {
  i1 = -1;
  i2 = -1;
  if (!(nd < dist_sqr)) return;
  i1 = nn;
  const int cs = trunc_i32(cl[nn].w);
  float m2 = dist_sqr;
  int b2 = -1;
  const int end = fwd < Nc ? fwd : Nc;
  scan_up(cl, nn + 1, end, cs, [&](int j, float4 c, int rj) {
    const float d = sqdis(c, sel);
    if (rj > cs && d < m2) { m2 = d; b2 = j; }
  });
  scan_down(cl, nn - 1, cs, [&](int j, float4 c, int rj) {
    const float d = sqdis(c, sel);
    if (rj < cs && d < m2) { m2 = d; b2 = j; }
  });
  i2 = b2;
}

// Squared-distance lower bound of q to a block's box, summed in sqdis' order: every point of the
// block has fl(sqdis) >= this value (each rounded gap and square is monotone in its exact value),
// so a block whose bound is >= the current minimum cannot change a strict '<' minimum. NaN
// coordinates give NaN bounds, which never skip.
__device__ __forceinline__ float box_lb(const float4& lo, const float4& hi, float4 q) {
  const float gx = q.x < lo.x ? lo.x - q.x : (q.x > hi.x ? q.x - hi.x : 0.0f);
  const float gy = q.y < lo.y ? lo.y - q.y : (q.y > hi.y ? q.y - hi.y : 0.0f);
  const float gz = q.z < lo.z ? lo.z - q.z : (q.z > hi.z ? q.z - hi.z : 0.0f);
  return gx * gx + gy * gy + gz * gz;
}

// findCorrespondingSurfFeatures search (FA:1724-1809): the up-walk visits nn+1 .. end-1 until a
// ring above cs + 2.5, the down-walk nn-1 .. 0 until a ring below cs - 2.5, each point updating the
// nearest same-ring (m2) or other-ring (m3) candidate with strict '<'. Whole 8-point blocks
// (aligned to the box array) and whole 64-point superblocks that contain no walk stop and whose
// box cannot beat the minimum they would be tested against are skipped: the visits that remain
// are the walk's, in its order, so the result is the serial loop's.
// w2 / w3: skip bounds from the previous kNN pass (the next float above the distance of its
// same-ring / other-ring choice, when the nearest neighbour and hence the walk's range and classes
// are unchanged; INFINITY otherwise): a block whose box is farther holds only points farther than a
// point of the same class and range, so it cannot hold the argmin.
// budget: the most 8-point steps (a block visited or skipped, a superblock skipped) the two walks
// may take; false when it ran out (i2 / i3 then meaningless: the caller walks that query again
// another way), true with the result otherwise.
__device__ bool surf_finish(const float4* sl, const float4* box, const float4* box2, int Ns, int fwd, float4 sel,
                            float dist_sqr, int nn, float nd, float w2, float w3, int& i1, int& i2, int& i3,
                            int budget = INT_MAX) {
  i1 = -1;
  i2 = -1;
  i3 = -1;
  if (!(nd < dist_sqr)) return true;
  int spent = 0;
  i1 = nn;
  const int cs = trunc_i32(sl[nn].w);
  float m2 = dist_sqr, m3 = dist_sqr;
  int b2 = -1, b3 = -1;
  const int end = fwd < Ns ? fwd : Ns;
  // the minimum a block of rings [rlo, rhi] is tested against: the up-walk tests rings <= cs
  // against m2, the down-walk rings >= cs; the rest against m3
  auto bound_up = [&](float rlo, float rhi) {
    const float b2 = fminf(m2, w2), b3 = fminf(m3, w3);
    return rhi <= (float)cs ? b2 : rlo > (float)cs ? b3 : fmaxf(b2, b3);
  };
  auto bound_dn = [&](float rlo, float rhi) {
    const float b2 = fminf(m2, w2), b3 = fminf(m3, w3);
    return rlo >= (float)cs ? b2 : rhi < (float)cs ? b3 : fmaxf(b2, b3);
  };
  // up-walk: single points up to the next block boundary, then blocks
  int j = nn + 1;
  bool stop = false;
  auto up_visit = [&](int jj, float4 c) {
    const int rj = trunc_i32(c.w);
    if ((double)rj > (double)cs + 2.5) { stop = true; return; }
    const float d = sqdis(c, sel);
    if (rj <= cs) {
      if (d < m2) { m2 = d; b2 = jj; }
    } else {
      if (d < m3) { m3 = d; b3 = jj; }
    }
  };
  for (; j < end && (j & 7) && !stop; ++j) up_visit(j, sl[j]);
  for (; j < end && !stop; j += kScan) {
    if (++spent > budget) return false;
    if ((j & 63) == 0 && j + 64 <= end) {  // a whole superblock
      const float4 lo = box2[2 * (j >> 6)], hi = box2[2 * (j >> 6) + 1];
      if ((double)(int)hi.w <= (double)cs + 2.5 && box_lb(lo, hi, sel) >= bound_up(lo.w, hi.w)) {
        j += 64 - kScan;
        continue;
      }
    }
    if (j + kScan <= end) {
      const float4 lo = box[2 * (j >> 3)], hi = box[2 * (j >> 3) + 1];
      if ((double)(int)hi.w <= (double)cs + 2.5 && box_lb(lo, hi, sel) >= bound_up(lo.w, hi.w)) continue;
    }
    float4 c[kScan];
#pragma unroll
    for (int u = 0; u < kScan; ++u) c[u] = j + u < end ? sl[j + u] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < kScan; ++u)
      if (!stop && j + u < end) up_visit(j + u, c[u]);
  }
  // down-walk: single points down to a block's last index, then blocks [j - 7, j]
  j = nn - 1;
  stop = false;
  auto down_visit = [&](int jj, float4 c) {
    const int rj = trunc_i32(c.w);
    if ((double)rj < (double)cs - 2.5) { stop = true; return; }
    const float d = sqdis(c, sel);
    if (rj >= cs) {
      if (d < m2) { m2 = d; b2 = jj; }
    } else {
      if (d < m3) { m3 = d; b3 = jj; }
    }
  };
  for (; j >= 0 && (j & 7) != 7 && !stop; --j) down_visit(j, sl[j]);
  for (; j >= 0 && !stop; j -= kScan) {
    if (++spent > budget) return false;
    if ((j & 63) == 63) {  // superblock [j - 63, j]
      const float4 lo = box2[2 * (j >> 6)], hi = box2[2 * (j >> 6) + 1];
      if ((double)(int)lo.w >= (double)cs - 2.5 && box_lb(lo, hi, sel) >= bound_dn(lo.w, hi.w)) {
        j -= 64 - kScan;
        continue;
      }
    }
    const float4 lo = box[2 * (j >> 3)], hi = box[2 * (j >> 3) + 1];  // block [j - 7, j]
    if ((double)(int)lo.w >= (double)cs - 2.5 && box_lb(lo, hi, sel) >= bound_dn(lo.w, hi.w)) continue;
    float4 c[kScan];
#pragma unroll
    for (int u = 0; u < kScan; ++u) c[u] = sl[j - u];
#pragma unroll
    for (int u = 0; u < kScan; ++u)
      if (!stop) down_visit(j - u, c[u]);
  }
  i2 = b2;
  i3 = b3;
  return true;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// surf_finish for the queries of one wave, walked by the whole wave one query at a time (every lane
// of the wave calls it; `act` marks a lane holding a query). A walk visits 64 points at once, lane
// order = walk order: the first lane meeting a ring outside the band ends the walk (lanes after it
// are not visited), and the lowest lane of the chunk's minimum is the serial loop's first strict
// '<' minimum (an earlier chunk's equal minimum is kept). Whole 64-point superblocks are tested 64
// at a time, one per lane, against the current minima; skipping is only ever a shortcut (a block
// whose box cannot beat the minimum it would be tested against and that holds no stop changes
// nothing), so the result is the serial loop's.
__device__ void surf_finish_wave(const float4* sl, const float4* box2, int end, float4 sel, float dist_sqr, bool act,
                                 int nn, float nd, float w2l, float w3l, int& i1, int& i2, int& i3) {
  const bool walk = act && nd < dist_sqr;
  i1 = walk ? nn : -1;
  i2 = -1;
  i3 = -1;
  const int lane = lane_id();
  uint64_t pend = __ballot(walk);
  while (pend) {
    const int l = __builtin_ctzll(pend);
    pend &= pend - 1;
    const float4 q = make_float4(readlane_f(sel.x, l), readlane_f(sel.y, l), readlane_f(sel.z, l), 0.0f);
    const int n0 = __builtin_amdgcn_readlane(nn, l);
    const int cs = trunc_i32(sl[n0].w);
    float m2 = dist_sqr, m3 = dist_sqr;
    int b2 = -1, b3 = -1;
    // one chunk: lane -> index idx (valid when `in`); true when the walk stops in it
    auto visit = [&](int idx, bool in, bool up) {
      const float4 c = in ? sl[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
      const int r = trunc_i32(c.w);
      const bool st = in && (up ? (double)r > (double)cs + 2.5 : (double)r < (double)cs - 2.5);
      const uint64_t sm = __ballot(st);
      const bool v = in && (sm == 0 || lane < __builtin_ctzll(sm));
      const float d = sqdis(c, q);
      const bool same = up ? r <= cs : r >= cs;
      const float d2 = v && same && d < m2 ? d : INFINITY;
      const float d3 = v && !same && d < m3 ? d : INFINITY;
      const float x2 = wave_reduce_min(d2), x3 = wave_reduce_min(d3);
      if (x2 < m2) {
        m2 = x2;
        b2 = __builtin_amdgcn_readlane(idx, __builtin_ctzll(__ballot(d2 == x2)));
      }
      if (x3 < m3) {
        m3 = x3;
        b3 = __builtin_amdgcn_readlane(idx, __builtin_ctzll(__ballot(d3 == x3)));
      }
      return sm != 0;
    };
    const float w2 = readlane_f(w2l, l), w3 = readlane_f(w3l, l);  // surf_finish's skip bounds
    auto bound_up = [&](float rlo, float rhi) {
      const float b2 = fminf(m2, w2), b3 = fminf(m3, w3);
      return rhi <= (float)cs ? b2 : rlo > (float)cs ? b3 : fmaxf(b2, b3);
    };
    auto bound_dn = [&](float rlo, float rhi) {
      const float b2 = fminf(m2, w2), b3 = fminf(m3, w3);
      return rlo >= (float)cs ? b2 : rhi < (float)cs ? b3 : fmaxf(b2, b3);
    };
    // up-walk n0 + 1 .. end - 1: the head up to a superblock boundary, then superblocks
    int j = n0 + 1;
    bool stop = false;
    const int hend = min((j + 63) & ~63, end);
    if (j < hend) {
      stop = visit(j + lane, j + lane < hend, true);
      j = hend;
    }
    while (!stop && j < end) {
      const int j0 = j, sb = (j0 >> 6) + lane;
      const bool full = (sb + 1) * 64 <= end;
      float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
      if (full) { lo = box2[2 * sb]; hi = box2[2 * sb + 1]; }
      const bool nostop = full && (double)(int)hi.w <= (double)cs + 2.5;
      int f0 = 0;
      for (;;) {
        const bool skip = nostop && box_lb(lo, hi, q) >= bound_up(lo.w, hi.w);
        const uint64_t need = __ballot(!skip) & (~0ull << f0);
        if (!need) { j = j0 + 64 * 64; break; }
        const int f = __builtin_ctzll(need), base = j0 + 64 * f;
        if (base >= end) { j = end; break; }
        stop = visit(base + lane, base + lane < end, true);
        if (stop || f == 63) { j = base + 64; break; }
        f0 = f + 1;
      }
    }
    // down-walk n0 - 1 .. 0: the head down to a superblock's first index, then superblocks
    j = n0 - 1;
    stop = false;
    if (j >= 0 && (j & 63) != 63) {
      const int hlo = j & ~63;
      stop = visit(j - lane, j - lane >= hlo, false);
      j = hlo - 1;
    }
    while (!stop && j >= 0) {
      const int j0 = j, sb = (j0 >> 6) - lane;  // superblock [64 sb, 64 sb + 63]
      float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
      if (sb >= 0) { lo = box2[2 * sb]; hi = box2[2 * sb + 1]; }
      const bool nostop = sb >= 0 && (double)(int)lo.w >= (double)cs - 2.5;
      int f0 = 0;
      for (;;) {
        const bool skip = nostop && box_lb(lo, hi, q) >= bound_dn(lo.w, hi.w);
        const uint64_t need = __ballot(!skip) & (~0ull << f0);
        if (!need) { j = j0 - 64 * 64; break; }
        const int f = __builtin_ctzll(need), top = j0 - 64 * f;
        if (top < 0) { j = -1; break; }
        stop = visit(top - lane, true, false);
        if (stop || f == 63) { j = top - 64; break; }
        f0 = f + 1;
      }
    }
    if (lane == l) {
      i2 = b2;
      i3 = b3;
    }
  }
}

// brute-force kNN-1 of J queries per thread over the LDS corner cloud (index order, strict '<')
template <int J>
__device__ __forceinline__ void corner_brute(const float4* cl, int Nc, const float4* qs, float* bd, int* bi) {
  int k = 0;
  for (; k + 8 <= Nc; k += 8) {  // 8 LDS reads in flight, then the in-order tests
    float4 c[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) c[u] = cl[k + u];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const float d = l2(qs[j], c[u]);
        if (d < bd[j]) { bd[j] = d; bi[j] = k + u; }
      }
  }
  for (; k < Nc; ++k) {
    const float4 c = cl[k];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const float d = l2(qs[j], c);
      if (d < bd[j]) { bd[j] = d; bi[j] = k; }
    }
  }
}

// Jacobian constants of calculateTransformationSurf (FA:1858-1891) / ...Corner (FA:2025-2043)
struct JacSurf {
  float a1, a2, a3, a4, a5, a6, a7, a8, a9, a10, a11, crx, b2, b6, c1, c2, c3, c4, c5, c6, c7, c8, c9;
  JacSurf() = default;
  __device__ explicit JacSurf(const float* t) {
    const float srx = sinf_(t[0]), crx_ = cosf_(t[0]);
    const float sry = sinf_(t[1]), cry = cosf_(t[1]);
    const float srz = sinf_(t[2]), crz = cosf_(t[2]);
    const float tx = t[3], ty = t[4], tz = t[5];
    crx = crx_;
    a1 = crx * sry * srz; a2 = crx * crz * sry; a3 = srx * sry;
    a4 = tx * a1 - ty * a2 - tz * a3;
    a5 = srx * srz; a6 = crz * srx;
    a7 = ty * a6 - tz * crx - tx * a5;
    a8 = crx * cry * srz; a9 = crx * cry * crz; a10 = cry * srx;
    a11 = tz * a10 + ty * a9 - tx * a8;
    const float b1 = -crz * sry - cry * srx * srz;
    b2 = cry * crz * srx - sry * srz;
    const float b5 = cry * crz - srx * sry * srz;
    b6 = cry * srz + crz * srx * sry;
    c1 = -b6; c2 = b5; c3 = tx * b6 - ty * b5; c4 = -crx * crz; c5 = crx * srz;
    c6 = ty * c5 + tx * -c4; c7 = b2; c8 = -b1; c9 = tx * -b2 - ty * -b1;
  }
  __device__ void row(float4 p, float cx, float cy, float cz, float* J) const {
    J[0] = (-a1 * p.x + a2 * p.y + a3 * p.z + a4) * cx + (a5 * p.x - a6 * p.y + crx * p.z + a7) * cy +
           (a8 * p.x - a9 * p.y - a10 * p.z + a11) * cz;
    J[1] = (c1 * p.x + c2 * p.y + c3) * cx + (c4 * p.x - c5 * p.y + c6) * cy + (c7 * p.x + c8 * p.y + c9) * cz;
    J[2] = -b6 * cx + c4 * cy + b2 * cz;
  }
};

struct JacCorner {
  float b1, b2, b3, b4, b5, b6, b7, b8, c5, srx;
  JacCorner() = default;
  __device__ explicit JacCorner(const float* t) {
    srx = sinf_(t[0]);
    const float crx = cosf_(t[0]);
    const float sry = sinf_(t[1]), cry = cosf_(t[1]);
    const float srz = sinf_(t[2]), crz = cosf_(t[2]);
    const float tx = t[3], ty = t[4], tz = t[5];
    b1 = -crz * sry - cry * srx * srz;
    b2 = cry * crz * srx - sry * srz;
    b3 = crx * cry;
    b4 = tx * -b1 + ty * -b2 + tz * b3;
    b5 = cry * crz - srx * sry * srz;
    b6 = cry * srz + crz * srx * sry;
    b7 = crx * sry;
    b8 = tz * b7 - ty * b6 - tx * b5;
    c5 = crx * srz;
  }
  __device__ void row(float4 p, float cx, float cy, float cz, float* J) const {
    J[0] = (b1 * p.x + b2 * p.y - b3 * p.z + b4) * cx + (b5 * p.x + b6 * p.y - b7 * p.z + b8) * cz;
    J[1] = -b5 * cx + c5 * cy + b1 * cz;
    J[2] = b7 * cx - srx * cy - b3 * cz;
  }
};

}  // namespace

// Phase C of one iteration (thread 0): ColPivHouseholderQR solve, the iteration-0 degeneracy test
// and matP, the projection, pose update, NaN reset and stop test (FA:1915-2009 / 2064-2142).
// Not inlined: the kernel's register allocation then does not carry the solver's temporaries
// (its peak sat here), and the call runs once per iteration on one lane.
__device__ __noinline__ int s2s_solve_step(float* t, float* matP, const float* sums, int* isDeg, int it, bool surf) {
  float AtA[9], AtB[3], X[3];
  for (int k = 0; k < 9; ++k) AtA[k] = sums[k];  // lane r + 3c -> column-major (r, c)
  for (int k = 0; k < 3; ++k) AtB[k] = sums[9 + k];
  llsr_eigen::colpiv_qr_solve<3, 3>(AtA, AtB, X);
  if (it == 0) {
    float E[3], V[9], V2[9];
    llsr_eigen::eig3(AtA, E, V);
    for (int k = 0; k < 9; ++k) V2[k] = V[k];
    int deg = 0;
    for (int i = 2; i >= 0; --i) {
      if (E[i] < 10) {
        for (int j = 0; j < 3; ++j) V2[i + 3 * j] = 0;
        deg = 1;
      } else {
        break;
      }
    }
    *isDeg = deg;
    float Vi[9];
    llsr_eigen::inverse3(V, Vi);         // matV.inverse(): cofactors (FA:1983 / 2118)
    llsr_eigen::prod33(Vi, V2, matP);    // matP = matV.inverse() * matV2
  }
  if (*isDeg) {  // matX = matP * matX2 (FA:1986-1990 / 2121-2125)
    const float X2[3] = {X[0], X[1], X[2]};
    llsr_eigen::prod31(matP, X2, X);
  }
  const float r2d = (float)(180.0 / 3.14159265358979323846);  // FA:56
  double dR, dT;
  if (surf) {
    t[0] += X[0]; t[2] += X[1]; t[4] += X[2];
    const double e0 = (double)(r2d * X[0]), e1 = (double)(r2d * X[1]), e2 = (double)(X[2] * 100);
    dR = (double)(float)sqrt(e0 * e0 + e1 * e1);
    dT = (double)(float)sqrt(e2 * e2);
  } else {
    t[1] += X[0]; t[3] += X[1]; t[5] += X[2];
    const double e0 = (double)(r2d * X[0]), e1 = (double)(X[1] * 100), e2 = (double)(X[2] * 100);
    dR = (double)(float)sqrt(e0 * e0);
    dT = (double)(float)sqrt(e1 * e1 + e2 * e2);
  }
  for (int k = 0; k < 6; ++k)
    if (t[k] != t[k]) t[k] = 0;
  return (dR < 0.1 && dT < 0.1) ? 1 : 0;
}

// k_s2s_boxes: per 8-point block of laserCloudSurfLast (index order), the box of its points and
// the range of their rings (trunc of the intensity, as the walks read it); lanes 8m .. 8m + 7 then
// combine their blocks into the box of 64-point superblock m. NaN coordinates stay out of the
// boxes (fminf / fmaxf): their distances are NaN, which never update a minimum.
__global__ void k_s2s_boxes(S2SArgs a) {
  const CellGrid& g = a.grids.g[1];
  const int p = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = g.count(p);
  const float4* pts = g.src + g.off[p];
  float4 lo = make_float4(INFINITY, INFINITY, INFINITY, INFINITY);
  float4 hi = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  for (int j = 8 * k; j < 8 * k + 8 && j < n; ++j) {
    const float4 c = pts[j];
    const float r = (float)trunc_i32(c.w);
    lo = make_float4(fminf(lo.x, c.x), fminf(lo.y, c.y), fminf(lo.z, c.z), fminf(lo.w, r));
    hi = make_float4(fmaxf(hi.x, c.x), fmaxf(hi.y, c.y), fmaxf(hi.z, c.z), fmaxf(hi.w, r));
  }
  if (8 * k < n) {
    float4* b = a.sbox + ((size_t)p * ((g.cap + 7) / 8) + k) * 2;
    b[0] = lo;
    b[1] = hi;
  }
#pragma unroll
  for (int o = 1; o < 8; o <<= 1) {
    lo = make_float4(fminf(lo.x, __shfl_xor(lo.x, o, 64)), fminf(lo.y, __shfl_xor(lo.y, o, 64)),
                     fminf(lo.z, __shfl_xor(lo.z, o, 64)), fminf(lo.w, __shfl_xor(lo.w, o, 64)));
    hi = make_float4(fmaxf(hi.x, __shfl_xor(hi.x, o, 64)), fmaxf(hi.y, __shfl_xor(hi.y, o, 64)),
                     fmaxf(hi.z, __shfl_xor(hi.z, o, 64)), fmaxf(hi.w, __shfl_xor(hi.w, o, 64)));
  }
  if ((k & 7) == 0 && 8 * k < n) {
    float4* b = a.sbox2 + ((size_t)p * ((g.cap + 63) / 64) + (k >> 3)) * 2;
    b[0] = lo;
    b[1] = hi;
  }
}

// Diagnostic build only (make prof -> libllsr_prof.so): thread 0 accumulates the wall clock of
// each phase and the report's transform_cur carries {A with kNN, A, B, C} in 10 ns ticks.
#ifdef LLSR_S2S_PROF
#define LLSR_STAMP(acc)                                    \
  do {                                                     \
    if (tid == 0) {                                        \
      const unsigned long long t1_ = wall_clock64();       \
      acc += t1_ - tprev;                                  \
      tprev = t1_;                                         \
    }                                                      \
  } while (0)
#else
#define LLSR_STAMP(acc) do {} while (0)
#endif

// kLdsRows: Jacobian rows kept in LDS (16 B each; larger phases use the HBM buffer); kLdsCorner:
// laserCloudCornerLast kept in LDS for a brute-force kNN-1 (larger clouds use the cell grid).
// Three instantiations (llsr_s2s.h), chosen per launch from the batch's largest clouds: 1024 / 1024
// (39 KB, 4 workgroups per CU: VLP-16-sized scans), 2560 / 1536 (78 KB, 2 per CU: HDL-64E, whose
// ~2.1-2.2k flat queries would otherwise sum their rows from HBM every surf iteration) and
// 2048 / 2048 (77 KB) otherwise.
template <int kLdsRows, int kLdsCorner, int kNT>
__global__ __launch_bounds__(kNT, 4) void k_s2s_lm(S2SArgs a) {
  constexpr int kThreads = kNT;  // (shadows the default: the instantiation's workgroup size)
  const int p = blockIdx.x;
  const int tid = threadIdx.x;
#ifdef LLSR_S2S_PROF
  unsigned long long tprev = wall_clock64(), tAks = 0, tAkc = 0, tA = 0, tB = 0, tC = 0, tF = 0, tW = 0;
  int nfb_total = 0;  // queries the surf / corner shells left to the block-wide scan (report.degenerate >> 1)
#endif
  __shared__ float t[6];
  __shared__ float matP[9];
  __shared__ float sums[12];
  __shared__ int isDeg, stop, n_corr[2], iters[2];
  __shared__ float4 lrows_raw[kLdsRows];  // the LDS rows as four arrays (J0, J1, J2, b): phase B
  float* const lrow4 = reinterpret_cast<float*>(lrows_raw);  // reads 4 consecutive rows of a column at once
  __shared__ uint8_t lvalid[kLdsRows];
  __shared__ uint16_t lvix[kLdsRows];  // phase B: the rows holding a correspondence, in order
  __shared__ float4 lcl[kLdsCorner];
  // the large instantiations (HDL-64E-sized clouds) take the whole-wave surf walks; the 1024 /
  // 1024 one keeps the per-lane walks, faster on VLP-16 clouds
  constexpr bool kBig = kLdsRows > 1024;
  __shared__ int fbq[kFbMax], nfb, nvalid, nrow;
  __shared__ float bpart[5][12];  // phase B: per-depth-block AtA partial sums
  __shared__ float red_d[kMulti][kThreads / 64];
  __shared__ int red_i[kMulti][kThreads / 64];
  const CellGrid& gc = a.grids.g[0];
  const CellGrid& gs = a.grids.g[1];
  const int64_t ms0 = a.sharp_off[p], ms1 = a.sharp_off[p + 1], f0 = a.flat_off[p], f1 = a.flat_off[p + 1];
  const int64_t nc = gc.off[p + 1] - gc.off[p], ns = gs.off[p + 1] - gs.off[p];
  const bool bad = ms1 < ms0 || f1 < f0 || nc < 0 || ns < 0 || ms1 - ms0 > a.cap_sharp || f1 - f0 > a.cap_flat ||
                   nc > gc.cap || ns > gs.cap;
  const int Ms = bad ? 0 : (int)(ms1 - ms0), F = bad ? 0 : (int)(f1 - f0);
  const int Nc = bad ? 0 : (int)nc, Ns = bad ? 0 : (int)ns;
  if (tid == 0) {
    for (int k = 0; k < 6; ++k) t[k] = a.tcur[6 * p + k];
    isDeg = a.degen[p];
    n_corr[0] = n_corr[1] = 0;
    iters[0] = iters[1] = 0;
    nfb = 0;
    nvalid = 0;
    if (bad) atomicOr(a.error, 1);
  }
  __syncthreads();
  const bool skipped = bad || Nc < 10 || Ns < 100;  // FA:2506
  if (!skipped) {
    const bool corner_lds = Nc <= kLdsCorner;
    const float4* clg = gc.src + gc.off[p];
    if (corner_lds) {  // visible to every thread after the barrier at the top of the first phase
      for (int k = tid; k < Nc; k += kThreads) lcl[k] = clg[k];
    }
    const float4* sl = gs.src + gs.off[p];
    const float4* sbox = a.sbox + (size_t)p * ((gs.cap + 7) / 8) * 2;
    const float4* sbox2 = a.sbox2 + (size_t)p * ((gs.cap + 63) / 64) * 2;
    const int capq = a.cap_sharp > a.cap_flat ? a.cap_sharp : a.cap_flat;
    // per query: [0..2] the correspondence (i1 = nearest, i2, i3) the rows read; [3..4] the kNN
    // pass's (nearest, d^2) until the tripod search turns them into [0..2]
    int* idx = a.idx + (size_t)p * capq * kIx;
    float4* grows = a.rows + (size_t)p * capq;
    uint8_t* gvalid = a.valid + (size_t)p * capq;
    // the two phases as two instantiations of one body (0: surf, FA:2508-2516; 1: corner,
    // FA:2519-2527), so each keeps only its own Jacobian constants live (the kernel's VGPR peak)
    auto run_phase = [&](auto tag) {
      constexpr bool surf = decltype(tag)::value;
      const int phase = surf ? 0 : 1;
      const float4* qry = surf ? a.flat + f0 : a.sharp + ms0;
      const int Q = surf ? F : Ms;
      // the rows of this phase: LDS when they fit (phase B re-reads them serially every iteration)
      float4* rows = grows;  // (the HBM rows when the phase's rows do not fit LDS)
      uint8_t* vf = Q <= kLdsRows ? lvalid : gvalid;  // row q holds a correspondence (laserCloudOri order)
      if (tid == 0)
        for (int k = 0; k < 9; ++k) matP[k] = (k % 4 == 0) ? 1.0f : 0.0f;
      __syncthreads();
      int it = 0;
      for (it = 0; it < 100; ++it) {
        // ---- A: correspondences + Jacobian rows at the current transformCur ----
        float tl[6];
        for (int k = 0; k < 6; ++k) tl[k] = t[k];
        // the Jacobian constants depend only on transformCur: once per iteration, not per query
        [[maybe_unused]] JacSurf js;
        [[maybe_unused]] JacCorner jc;
        if constexpr (surf) js = JacSurf(tl);
        else jc = JacCorner(tl);
        const bool knn = it % 5 == 0;
        // the ring-constrained tripod search around a found nearest neighbour (FA:1588-1647 /
        // FA:1737-1803) and the correspondence indices it leaves in idx
        // the nearest neighbour (index, squared distance) of query q, parked in idx; the tripod
        // searches then run from ONE call site below (one inlined copy of the walks keeps the
        // kernel at 128 VGPRs with fewer spills than three copies)
        auto park = [&](int q, int nn, float nd) {
          int* ix = idx + kIx * q;
          ix[3] = nn;
          ix[4] = __float_as_int(nd);
        };
        // the previous kNN pass of this phase (it >= 5): its nearest neighbour seeds the shells, and
        // when the new nearest neighbour is the same point its tripod points bound the walks
        const bool warm = it > 0;
        auto walk_bounds = [&](const int* ix, float4 sel, int nn, float& w2, float& w3) {
          w2 = w3 = INFINITY;
          if (warm && ix[0] == nn && nn >= 0) {
            if (ix[1] >= 0) w2 = __int_as_float(__float_as_int(sqdis(sl[ix[1]], sel)) + 1);
            if (ix[2] >= 0) w3 = __int_as_float(__float_as_int(sqdis(sl[ix[2]], sel)) + 1);
          }
        };
        auto finish = [&](int q, float4 sel, int nn, float nd) {
          int i1, i2, i3 = -1;
          if (surf) {
            float w2, w3;
            walk_bounds(idx + kIx * q, sel, nn, w2, w3);
            surf_finish(sl, sbox, sbox2, Ns, F, sel, a.dist_sqr, nn, nd, w2, w3, i1, i2, i3);
          } else if (corner_lds) {  // LDS-typed accesses (a generic pointer would issue flat loads)
            corner_finish(lcl, Nc, Ms, sel, a.dist_sqr, nn, nd, i1, i2);
          } else {
            corner_finish(clg, Nc, Ms, sel, a.dist_sqr, nn, nd, i1, i2);
          }
          int* ix = idx + kIx * q;
          ix[0] = i1; ix[1] = i2; ix[2] = i3;
        };
        if (knn) {  // kNN-1 every 5th iteration (FA:1588 / 1724)
          if (!surf && corner_lds) {
            // the sparse corner cloud from LDS: each thread scans it once for up to kMulti of its
            // queries (index order, strict '<': nn1_scan per query)
            for (int q0 = tid; q0 < Q; q0 += kThreads * kMulti) {
              float4 qs[kMulti];
              float bd[kMulti];
              int bi[kMulti];
#pragma unroll
              for (int j = 0; j < kMulti; ++j) {
                const int q = q0 + j * kThreads;
                qs[j] = q < Q ? to_start(tl, qry[q]) : make_float4(0.f, 0.f, 0.f, 0.f);
                bd[j] = INFINITY;
                bi[j] = INT_MAX;
              }
              // queries this wave holds (wave-uniform): no distance work for empty slots
              const int wq = Q - (q0 - lane_id());
              const int nj = wq > 3 * kThreads ? 4 : wq > 2 * kThreads ? 3 : wq > kThreads ? 2 : 1;
              if (nj == 1) corner_brute<1>(lcl, Nc, qs, bd, bi);
              else corner_brute<2>(lcl, Nc, qs, bd, bi);
#pragma unroll
              for (int j = 0; j < kMulti; ++j)
                if (q0 + j * kThreads < Q) park(q0 + j * kThreads, bi[j], bd[j]);
            }
          }
          for (int q = tid; q < Q && !(!surf && corner_lds); q += kThreads) {
            const float4 sel = to_start(tl, qry[q]);
            int nn = INT_MAX;
            float nd = INFINITY;
            if (surf && warm) {  // seed: the previous pass's nearest neighbour
              const int pn = idx[kIx * q];
              if (pn >= 0) { nn = pn; nd = l2(sel, sl[pn]); }
            }
            const bool ok = nn1_shells(surf ? gs : gc, p, sel, a.dist_sqr, nn, nd);
            if (ok) {
              park(q, nn, nd);
            } else {
              const int k = atomicAdd(&nfb, 1);
              if (k < kFbMax) {
                fbq[k] = q;
              } else {  // overflow of the queue: the serial scan (same result)
                nn1_scan(surf ? sl : clg, surf ? Ns : Nc, sel, nn, nd);
                park(q, nn, nd);
              }
            }
          }
          __syncthreads();
          if (surf) LLSR_STAMP(tAks);
          else LLSR_STAMP(tAkc);
          // queries the shells left open: the whole block scans the cloud, kMulti queries per pass
          const int nq = nfb < kFbMax ? nfb : kFbMax;
#ifdef LLSR_S2S_PROF
          if (tid == 0) nfb_total += nfb;
#endif
          for (int k0 = 0; k0 < nq; k0 += kMulti) {
            const int m = nq - k0 < kMulti ? nq - k0 : kMulti;
            float4 qs[kMulti];
#pragma unroll
            for (int j = 0; j < kMulti; ++j) qs[j] = j < m ? to_start(tl, qry[fbq[k0 + j]]) : make_float4(0.f, 0.f, 0.f, 0.f);
            int nn[kMulti];
            float nd[kMulti];
            nn1_block_multi<kThreads>(surf ? sl : clg, surf ? Ns : Nc, qs, m, nn, nd, red_d, red_i);
#pragma unroll
            for (int j = 0; j < kMulti; ++j)
              if (j < m && tid == j) park(fbq[k0 + j], nn[j], nd[j]);
          }
          if (tid == 0) nfb = 0;
          __syncthreads();
          if (surf) LLSR_STAMP(tAks);
          else LLSR_STAMP(tAkc);
          if constexpr (surf && kBig) {
            // each lane walks its own query up to kWalkBudget 8-point steps; the whole wave then walks
            // the queries that ran out, one at a time (HDL-64E: the shadow points' queries, whose
            // ring band holds most of the cloud, would keep a per-lane walk's wave busy alone)
            for (int q0 = 0; q0 < Q; q0 += kThreads) {
              const int q = q0 + tid;
              const bool act = q < Q;
              int* ix = idx + kIx * (act ? q : 0);
              int nn = -1;
              float nd = INFINITY, w2 = INFINITY, w3 = INFINITY;
              float4 sel = make_float4(0.f, 0.f, 0.f, 0.f);
              if (act) {
                nn = ix[3];
                nd = __int_as_float(ix[4]);
                sel = to_start(tl, qry[q]);
                walk_bounds(ix, sel, nn, w2, w3);
              }
              int i1 = -1, i2 = -1, i3 = -1;
              bool done = true;
              if (act) done = surf_finish(sl, sbox, sbox2, Ns, F, sel, a.dist_sqr, nn, nd, w2, w3, i1, i2, i3, kWalkBudget);
              if (__ballot(!done)) {
                int j1, j2, j3;
                surf_finish_wave(sl, sbox2, F < Ns ? F : Ns, sel, a.dist_sqr, !done, nn, nd, w2, w3, j1, j2, j3);
                if (!done) { i1 = j1; i2 = j2; i3 = j3; }
              }
              if (act) { ix[0] = i1; ix[1] = i2; ix[2] = i3; }
            }
          } else {
            for (int q = tid; q < Q; q += kThreads) {
              const int* ix = idx + kIx * q;
              finish(q, to_start(tl, qry[q]), ix[3], __int_as_float(ix[4]));
            }
          }
          __syncthreads();
          if (surf) LLSR_STAMP(tW);
          else LLSR_STAMP(tF);
        }
        int nval = 0;
        for (int q = tid; q < Q; q += kThreads) {
          const float4 pi = qry[q];
          const float4 sel = to_start(tl, pi);
          const int* ix = idx + kIx * q;
          float4 row = make_float4(0.f, 0.f, 0.f, 0.f);  // no correspondence: adds exact zeros
          bool valid = false;
          if constexpr (surf) {
            if (ix[1] >= 0 && ix[2] >= 0) {
              const float4 t1 = sl[ix[0]], t2 = sl[ix[1]], t3 = sl[ix[2]];
              float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
              float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
              float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
              float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
              const float ps = sqrt_(pa * pa + pb * pb + pc * pc);
              pa /= ps; pb /= ps; pc /= ps; pd /= ps;
              const float pd2 = pa * sel.x + pb * sel.y + pc * sel.z + pd;
              float s = 1;
              if (it >= 5)
                s = (float)(1 - 1.8 * (double)fabs_(pd2) /
                                    (double)sqrt_(sqrt_(sel.x * sel.x + sel.y * sel.y + sel.z * sel.z)));
              if ((double)s > 0.1 && pd2 != 0) {
                float J[3];
                js.row(pi, s * pa, s * pb, s * pc, J);
                row = make_float4(J[0], J[1], J[2], (float)(-0.05 * (double)(s * pd2)));
                valid = true;
              }
            }
          } else if (ix[1] >= 0) {  // corner
            float4 t1, t2;
            if (corner_lds) { t1 = lcl[ix[0]]; t2 = lcl[ix[1]]; }
            else { t1 = clg[ix[0]]; t2 = clg[ix[1]]; }
            const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
            const float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
            const float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
            const float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
            const float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
            const float a012 = sqrt_(m11 * m11 + m22 * m22 + m33 * m33);
            const float l12 = sqrt_((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
            const float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
            const float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
            const float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
            const float ld2 = a012 / l12;
            float s = 1;
            if (it >= 5) s = (float)(1 - 1.8 * (double)fabs_(ld2));
            if ((double)s > 0.1 && ld2 != 0) {
              float J[3];
              jc.row(pi, s * la, s * lb, s * lc, J);
              row = make_float4(J[0], J[1], J[2], (float)(-0.05 * (double)(s * ld2)));
              valid = true;
            }
          }
          if (Q <= kLdsRows) {
            lrow4[q] = row.x;
            lrow4[kLdsRows + q] = row.y;
            lrow4[2 * kLdsRows + q] = row.z;
            lrow4[3 * kLdsRows + q] = row.w;
            lvalid[q] = valid ? 1 : 0;
          }
          else { grows[q] = row; gvalid[q] = valid ? 1 : 0; }
          nval += valid ? 1 : 0;
        }
        if (nval) atomicAdd(&nvalid, nval);
        __syncthreads();
        LLSR_STAMP(tA);
        // ---- B: AtA / AtB as Eigen evaluates matAt * matA and matAt * matB (FA:1953-1955) ----
        // Lane r + 3c sums AtA(r, c), lanes 9..11 AtB: the products of two components of each
        // correspondence's row in correspondence order. matAt * matA is Eigen's GEMM: each depth
        // block of kc rows (llsr_eigen::gemm_kc) is summed from zero and added to the result; below
        // N + 6 < 20 it is the lazy coefficient product, and matAt * matB always is (a sum that
        // starts from the first product). Rows without a correspondence are skipped.
        if (Q <= kLdsRows) {
          // rows in LDS: wave 0 lists the rows holding a correspondence (ballot compaction, order
          // kept), the block moves them to the front of lrows in that order (stable, in place: a
          // row only moves down, every read before the first write), then the sums read contiguous
          // rows. Each GEMM depth block of AtA is its own lane (12 entries x blocks <= 64 lanes of
          // wave 0), summed from zero; lanes 0..8 then add the blocks in order. AtB (lanes 9..11)
          // and the lazy product are single chains over all rows.
          if (tid < 64) {
            int N = 0;
            for (int q0 = 0; q0 < Q; q0 += 64) {
              const int q = q0 + tid;
              const bool v = q < Q && lvalid[q] != 0;
              const unsigned long long m = __ballot(v);
              if (v) lvix[N + __popcll(m & ((1ull << tid) - 1ull))] = (uint16_t)q;
              N += __popcll(m);
            }
            if (tid == 0) nrow = N;
          }
          __syncthreads();
          const int N = nrow;
          // in steps of 2 rows per lane (fewer registers live across the barrier): a step's sources
          // lvix[i] >= i lie at or beyond its destinations and beyond every earlier step's
          constexpr int kMvS = 2;
          for (int c0 = 0; c0 < N; c0 += kMvS * kThreads) {
            float4 mv[kMvS];
#pragma unroll
            for (int u = 0; u < kMvS; ++u) {
              const int i = c0 + tid + u * kThreads;
              if (i < N) {
                const int r = lvix[i];
                mv[u] = make_float4(lrow4[r], lrow4[kLdsRows + r], lrow4[2 * kLdsRows + r], lrow4[3 * kLdsRows + r]);
              }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kMvS; ++u) {
              const int i = c0 + tid + u * kThreads;
              if (i < N) {
                lrow4[i] = mv[u].x;
                lrow4[kLdsRows + i] = mv[u].y;
                lrow4[2 * kLdsRows + i] = mv[u].z;
                lrow4[3 * kLdsRows + i] = mv[u].w;
              }
            }
            __syncthreads();
          }
          const bool lazyAll = N + 6 < 20;
          const int kc = lazyAll ? N : llsr_eigen::gemm_kc(N, 3, 3);
          const int nblk = lazyAll || N == 0 ? 1 : (N + kc - 1) / kc;
          if (tid < 64) {
            // lane = entry (0..11) + 12 * block; AtB entries and the lazy product use block 0 only
            const int e = tid % 12, blk = tid / 12;
            const bool lazy = e >= 9 || lazyAll;
            // the lazy lanes (AtB, or everything when lazyAll) always sum on block 0: their result
            // is read below whatever nblk is; the GEMM-blocked lanes only when the blocks fit
            const bool act = lazy ? blk == 0 : (blk < nblk && 12 * nblk <= 64);
            const int ra = e < 9 ? e % 3 : e - 9, rb = e < 9 ? e / 3 : 3;
            const float* ca = lrow4 + ra * kLdsRows;  // the two columns this lane multiplies
            const float* cb = lrow4 + rb * kLdsRows;
            float c = 0.0f;
            if (act) {
              const int b0 = lazy ? 0 : blk * kc, b1 = lazy ? N : min(N, b0 + kc);
              int i = b0;
              if (lazy && N > 0) { c = ca[0] * cb[0]; i = 1; }  // the coefficient product
              for (; i < b1 && (i & 7); ++i) c = c + ca[i] * cb[i];
              // 8 rows per step, each column read as two 16-byte loads; the next step's loads are
              // in flight while this step's products are added in order (the only serial part)
              if (i + 8 <= b1) {
                float4 xa0 = *reinterpret_cast<const float4*>(ca + i), xa1 = *reinterpret_cast<const float4*>(ca + i + 4);
                float4 xb0 = *reinterpret_cast<const float4*>(cb + i), xb1 = *reinterpret_cast<const float4*>(cb + i + 4);
                for (; i + 16 <= b1; i += 8) {
                  const float4 ya0 = *reinterpret_cast<const float4*>(ca + i + 8);
                  const float4 ya1 = *reinterpret_cast<const float4*>(ca + i + 12);
                  const float4 yb0 = *reinterpret_cast<const float4*>(cb + i + 8);
                  const float4 yb1 = *reinterpret_cast<const float4*>(cb + i + 12);
                  c = c + xa0.x * xb0.x; c = c + xa0.y * xb0.y; c = c + xa0.z * xb0.z; c = c + xa0.w * xb0.w;
                  c = c + xa1.x * xb1.x; c = c + xa1.y * xb1.y; c = c + xa1.z * xb1.z; c = c + xa1.w * xb1.w;
                  xa0 = ya0; xa1 = ya1; xb0 = yb0; xb1 = yb1;
                }
                c = c + xa0.x * xb0.x; c = c + xa0.y * xb0.y; c = c + xa0.z * xb0.z; c = c + xa0.w * xb0.w;
                c = c + xa1.x * xb1.x; c = c + xa1.y * xb1.y; c = c + xa1.z * xb1.z; c = c + xa1.w * xb1.w;
                i += 8;
              }
              for (; i < b1; ++i) c = c + ca[i] * cb[i];
              if (!lazy) bpart[blk][e] = c;
            }
            wave_sync_lds();
            if (tid < 12) {
              if (lazy) {
                sums[tid] = c;
              } else if (12 * nblk <= 64) {
                float tot = 0.0f;
                for (int x = 0; x < nblk; ++x) tot = tot + 1.0f * bpart[x][tid];
                sums[tid] = tot;
              } else {  // more depth blocks than wave 0 has lanes for: one lane per entry
                float tot = 0.0f;
                for (int b0 = 0; b0 < N; b0 += kc) {
                  const int b1 = min(N, b0 + kc);
                  float cs = 0.0f;
                  for (int i = b0; i < b1; ++i) cs = cs + ca[i] * cb[i];
                  tot = tot + 1.0f * cs;
                }
                sums[tid] = tot;
              }
            }
          }
        } else if (Q > kLdsRows && tid < 12) {
          const int ra = tid < 9 ? tid % 3 : tid - 9, rb = tid < 9 ? tid / 3 : 3;
          const float* rf = reinterpret_cast<const float*>(rows);
          const int N = nvalid;
          const bool lazy = tid >= 9 || N + 6 < 20;
          const int kc = lazy ? 0x7fffffff : llsr_eigen::gemm_kc(N, 3, 3);
          float tot = 0.0f, c = 0.0f;
          int cnt = 0;
          bool first = true;
          // branch-free: rows without a correspondence are selected out (never added), the
          // products of 8 rows are formed before their in-order additions
          auto add = [&](bool ok, float pr) {
            if (lazy) {
              c = ok ? (first ? pr : c + pr) : c;
              first = first && !ok;
            } else {
              const float cn = ok ? c + pr : c;
              const int kn = cnt + (ok ? 1 : 0);
              const bool fl = kn == kc;
              tot = fl ? tot + 1.0f * cn : tot;
              c = fl ? 0.0f : cn;
              cnt = fl ? 0 : kn;
            }
          };
          int q = 0;
          for (; q + 8 <= Q; q += 8) {
            float pv[8];
            bool ok[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              ok[u] = vf[q + u] != 0;
              pv[u] = rf[4 * (q + u) + ra] * rf[4 * (q + u) + rb];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) add(ok[u], pv[u]);
          }
          for (; q < Q; ++q) add(vf[q] != 0, rf[4 * q + ra] * rf[4 * q + rb]);
          sums[tid] = lazy ? c : (cnt ? tot + 1.0f * c : tot);
        }
        __syncthreads();
        LLSR_STAMP(tB);
        // ---- C: solve and update (thread 0) ----
        if (tid == 0) {
          stop = 0;
          const int cnt = nvalid;
          nvalid = 0;  // counted again by the next phase A (after the end-of-iteration barrier)
          n_corr[phase] = cnt;
          if (cnt >= 10) stop = s2s_solve_step(t, matP, sums, &isDeg, it, surf);  // FA:2514 / 2525
        }
        __syncthreads();
        LLSR_STAMP(tC);
        if (stop) break;
      }
      if (tid == 0) iters[phase] = it;
      __syncthreads();
    };
    run_phase(std::true_type{});
    run_phase(std::false_type{});
  }
  if (tid == 0) {
    llsr_s2s_report& r = a.report[p];
    r.surf_iterations = skipped ? 0 : iters[0];
    r.corner_iterations = skipped ? 0 : iters[1];
    r.n_surf_corr = n_corr[0];
    r.n_corner_corr = n_corr[1];
    r.degenerate = isDeg;
    r.skipped = skipped ? 1 : 0;
    for (int k = 0; k < 6; ++k) {
      r.transform_cur[k] = t[k];
      a.tcur[6 * p + k] = t[k];
    }
    r.ms = 0.0f;
#ifdef LLSR_S2S_PROF
    // phase ticks and the shell fallback count to the diagnostics buffer (llsr_debug_s2s_prof); the
    // report keeps its ABI meaning in every build
    float* pf = a.prof + 8 * (size_t)p;
    pf[0] = (float)tAks; pf[1] = (float)tAkc; pf[2] = (float)tA; pf[3] = (float)tB;
    pf[4] = (float)tC; pf[5] = (float)tF; pf[6] = (float)tW; pf[7] = (float)nfb_total;
#endif
    a.degen[p] = isDeg;
  }
}

template __global__ void k_s2s_lm<2048, 2048, 512>(S2SArgs);
template __global__ void k_s2s_lm<2560, 1536, 512>(S2SArgs);
template __global__ void k_s2s_lm<1024, 1024, 256>(S2SArgs);

}  // namespace llsr
