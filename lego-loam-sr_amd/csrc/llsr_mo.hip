// llsr_mo.hip — MapOptimization scan-to-map on gfx950: a batch of independent problems
// (scan2MapOptimization, mapOptmization.cpp:1572-1610), each = corner/surf query clouds of one
// scan + its corner/surf local maps + the pose transformTobeMapped.
//
// Per batch:
//   k_s2m_setup        problem bookkeeping, capacity checks, the MO:1573 guard
//   k_grid_*           1 m cell grids of both maps (kdtreeCornerFromMap / kdtreeSurfFromMap
//                      setInputCloud, MO:1575-1576), llsr_grid.h
//   k_s2m_iter  x it   one launch per LM iteration (MO:1578-1608) over (query block, problem):
//                      pointAssociateToMap, kNN-5, the corner line / surf plane coefficient, the
//                      Jacobian row, compacted per block in laserCloudOri order
//   k_s2m_solve x it   one workgroup per problem: the normal equations in Eigen's order, then
//                      LMOptimization's solve / degeneracy / update / stop test
//   k_s2m_finish       pose + llsr_lm_report out
//
// kNN-5 (nanoflann, exact, sorted) only matters when all five neighbours lie within d^2 < 1.0
// (MO:1279 / MO:1386), so a 1 m grid over the 27 neighbouring cells finds them exactly. Each
// thread keeps the five smallest (d^2, map index) pairs: identical to inserting candidates in
// index order with strict '<' (the restatement in oracle/oracle_mo.cpp), independent of the
// order the cells are visited; cells that cannot hold a better pair are not probed (knn5). The per-correspondence arithmetic repeats the reference's float
// and double operations one for one (-ffp-contract=off, glibc sinf/cosf ports, Eigen 3.3.7
// restatements in llsr_eigen.h), so correspondences and coefficients are bit-identical to the
// oracle, and the normal equations are summed in the reference's Eigen order: the float path is
// bit-identical to the oracle (tests/test_gpu_mo.py).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cstdint>

#include "../../include/llsr.h"
#include "llsr_device.h"
#include "llsr_eigen.h"
#include "llsr_grid.h"
#include "llsr_lm.h"
#include "llsr_mo.h"

// LLSR_S2M_DBG stage stops of k_s2m_solve exist only in the diagnostic build (make prof)
#ifdef LLSR_S2S_PROF
#define S2M_DBG(a) ((a).dbg)
#else
#define S2M_DBG(a) 0
#endif

namespace llsr {

using llsr_libm::bitsf;
using llsr_libm::cosf_;
using llsr_libm::fabs_;
using llsr_libm::fbits;
using llsr_libm::sinf_;
using llsr_libm::sqrt_;

namespace {

struct Best5 {
  float d[5];
  int i[5];
};

// The 27 neighbour cells in the order kNN-5 visits them: the query's own cell, the 6 face
// neighbours, the 12 edge and the 8 corner neighbours (packed as (dx+1) | (dy+1) << 2 | (dz+1) << 4),
// so the 5th-best distance tightens early and prunes the farther cells.
__constant__ unsigned char kCellOrder[27] = {
    21,                                          // (0, 0, 0)
    20, 22, 17, 25, 5, 37,                       // faces
    16, 18, 24, 26, 4, 6, 36, 38, 1, 9, 33, 41,  // edges
    0, 2, 8, 10, 32, 34, 40, 42};                // corners

// kNN-5 with d^2 < 1.0 around q in one map; returns true when five were found.
// The result is the five smallest (d^2, index) pairs of the cells' points with d^2 < 1.0, in any
// visiting order. A cell is skipped when no point in it can enter that set: its box lies at squared
// distance LB from q, every point's float d^2 (three rounded differences, squares and sums) is at
// least LB (1 - 5 eps) minus the rounding of the box gaps (< 1e-7 absolute), so a cell with
// LB > lim (1 + 1e-5) + 4e-6 holds only points with d^2 > lim, where lim = 1.0, or the current 5th
// distance once five are held (a tie at lim would need d^2 == lim). Exact, therefore, and typically
// 7 of the 27 cells are probed (the center, the faces and a few edges; tests/test_gpu_mo.py).
__device__ bool knn5(const CellSlot* __restrict__ tab, int log2T, const float4* __restrict__ pts,
                     float qx, float qy, float qz, Best5& b) {
#pragma unroll
  for (int k = 0; k < 5; ++k) { b.d[k] = INFINITY; b.i[k] = INT_MAX; }
  const int cx = cell_coord(qx), cy = cell_coord(qy), cz = cell_coord(qz);
  // distances from q to its cell's lower / upper faces per axis (cell_coord's sentinel cell for
  // NaN / huge coordinates: gaps become NaN / huge, no cell is skipped wrongly since LB > lim fails
  // for NaN and a huge q finds nothing anyway)
  const float lx = qx - floorf(qx), ly = qy - floorf(qy), lz = qz - floorf(qz);
  const float ux = 1.0f - lx, uy = 1.0f - ly, uz = 1.0f - lz;
  // cells visited one at a time (not unrolled): keeps the kernel's VGPRs low, which beat issuing
  // all probes up front on MI355X (latency-bound gathers, 8 waves per SIMD)
#pragma unroll 1
  for (int c = 0; c < 27; ++c) {
    const int o = kCellOrder[c];
    const int ox = (o & 3) - 1, oy = ((o >> 2) & 3) - 1, oz = (o >> 4) - 1;
    const float gx = ox < 0 ? lx : (ox > 0 ? ux : 0.0f);
    const float gy = oy < 0 ? ly : (oy > 0 ? uy : 0.0f);
    const float gz = oz < 0 ? lz : (oz > 0 ? uz : 0.0f);
    const float lb = gx * gx + gy * gy + gz * gz;
    const float lim = b.d[4] < 1.0f ? b.d[4] : 1.0f;
    if (lb > lim * 1.00001f + 4e-6f) continue;
    const int s = grid_find(tab, log2T, cell_key(cx + ox, cy + oy, cz + oz));
    if (s < 0) continue;
    const int st = tab[s].start, n = tab[s].count;
    float4 pn = n > 0 ? pts[st] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = st; j < st + n; ++j) {
      const float4 p = pn;  // the next point's load is in flight while this one is tested
      if (j + 1 < st + n) pn = pts[j + 1];
      float d = 0.0f;
      float t = qx - p.x; d += t * t;  // nanoflann L2 accumulation order
      t = qy - p.y; d += t * t;
      t = qz - p.z; d += t * t;
      const int id = (int)fbits(p.w);
      if (!(d < 1.0f) || !nn_before(d, id, b.d[4], b.i[4])) continue;
      b.d[4] = d; b.i[4] = id;
#pragma unroll
      for (int k = 4; k > 0; --k)
        if (nn_before(b.d[k], b.i[k], b.d[k - 1], b.i[k - 1])) {
          const float td = b.d[k]; b.d[k] = b.d[k - 1]; b.d[k - 1] = td;
          const int ti = b.i[k]; b.i[k] = b.i[k - 1]; b.i[k - 1] = ti;
        }
    }
  }
  return b.d[4] < 1.0f;
}

// pointAssociateToMap (MO:606-620) with the cached sin/cos of transformTobeMapped.
struct Assoc {
  float cR, sR, cP, sP, cY, sY, tx, ty, tz;
  __device__ void apply(float px, float py, float pz, float& ox, float& oy, float& oz) const {
    const float x1 = cY * px - sY * py;
    const float y1 = sY * px + cY * py;
    const float z1 = pz;
    const float x2 = x1;
    const float y2 = cR * y1 - sR * z1;
    const float z2 = sR * y1 + cR * z1;
    ox = cP * x2 + sP * z2 + tx;
    oy = y2 + ty;
    oz = -sP * x2 + cP * z2 + tz;
  }
};

// cornerOptimization body (MO:1274-1375) for one query; returns false when rejected.
__device__ bool corner_coeff(const CellSlot* tab, int log2T, const float4* pts, const float4* mapP,
                             float x0, float y0, float z0, float& la, float& lb, float& lc, float& ld) {
  Best5 nb;
  if (!knn5(tab, log2T, pts, x0, y0, z0, nb)) return false;
  float mx[5], my[5], mz[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const float4 m = mapP[nb.i[j]];
    mx[j] = m.x; my[j] = m.y; mz[j] = m.z;
  }
  float cx = 0, cy = 0, cz = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) { cx += mx[j]; cy += my[j]; cz += mz[j]; }
  cx /= 5; cy /= 5; cz /= 5;
  float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const float ax = mx[j] - cx, ay = my[j] - cy, az = mz[j] - cz;
    a11 += ax * ax; a12 += ax * ay; a13 += ax * az; a22 += ay * ay; a23 += ay * az; a33 += az * az;
  }
  a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
  const float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33};
  float D1[3], V1[9];
  llsr_eigen::eig3(A1, D1, V1);
  if (!(D1[2] > 3 * D1[1])) return false;
  const float x1 = (float)(cx + 0.1 * V1[0]), y1 = (float)(cy + 0.1 * V1[3]), z1 = (float)(cz + 0.1 * V1[6]);
  const float x2 = (float)(cx - 0.1 * V1[0]), y2 = (float)(cy - 0.1 * V1[3]), z2 = (float)(cz - 0.1 * V1[6]);
  const float u = (x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1);
  const float v = (x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1);
  const float w = (y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1);
  const float a012 = sqrt_(u * u + v * v + w * w);
  const float l12 = sqrt_((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
  const float a = ((y1 - y2) * u + (z1 - z2) * v) / a012 / l12;
  const float b = -((x1 - x2) * u - (z1 - z2) * w) / a012 / l12;
  const float c = -((x1 - x2) * v + (y1 - y2) * w) / a012 / l12;
  const float ld2 = a012 / l12;
  const float s = (float)(1 - 0.9 * (double)fabs_(ld2));
  if (!((double)s > 0.1)) return false;
  la = s * a; lb = s * b; lc = s * c; ld = s * ld2;
  return true;
}

// surfOptimization body (MO:1383-1440) for one query.
__device__ bool surf_coeff(const CellSlot* tab, int log2T, const float4* pts, const float4* mapP,
                           float x0, float y0, float z0, float& la, float& lb, float& lc, float& ld) {
  Best5 nb;
  if (!knn5(tab, log2T, pts, x0, y0, z0, nb)) return false;
  float A0[15];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const float4 m = mapP[nb.i[j]];
    A0[j] = m.x; A0[5 + j] = m.y; A0[10 + j] = m.z;
  }
  const float B0[5] = {-1, -1, -1, -1, -1};
  float X0[3];
  llsr_eigen::colpiv_qr_solve<5, 3>(A0, B0, X0);
  float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
  const float ps = sqrt_(pa * pa + pb * pb + pc * pc);
  pa /= ps; pb /= ps; pc /= ps; pd /= ps;
#pragma unroll
  for (int j = 0; j < 5; ++j)
    if (fabs_(pa * A0[j] + pb * A0[5 + j] + pc * A0[10 + j] + pd) > 0.2f) return false;
  const float pd2 = pa * x0 + pb * y0 + pc * z0 + pd;
  const float r = sqrt_(sqrt_(x0 * x0 + y0 * y0 + z0 * z0));
  const float s = (float)(1 - 0.9 * (double)fabs_(pd2) / (double)r);
  if (!((double)s > 0.1)) return false;
  la = s * pa; lb = s * pb; lc = s * pc; ld = s * pd2;
  return true;
}

}  // namespace

__global__ void k_s2m_setup(S2MArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.P) return;
  S2MProb& st = a.prob[p];
  const int64_t qc0 = a.cq_off[p], qc1 = a.cq_off[p + 1], qs0 = a.sq_off[p], qs1 = a.sq_off[p + 1];
  const int64_t mc0 = a.cm_off[p], mc1 = a.cm_off[p + 1], ms0 = a.sm_off[p], ms1 = a.sm_off[p + 1];
  st.qc0 = qc0; st.qs0 = qs0; st.mc0 = mc0; st.ms0 = ms0;
  st.Qc = (int)(qc1 - qc0); st.Qs = (int)(qs1 - qs0); st.Mc = (int)(mc1 - mc0); st.Ms = (int)(ms1 - ms0);
  int bad = 0;
  if (qc1 < qc0 || qs1 < qs0 || mc1 < mc0 || ms1 < ms0) bad = 1;
  if (st.Qc > a.cap_qc || st.Qs > a.cap_qs || st.Mc > a.cap_mc || st.Ms > a.cap_ms) bad = 1;
  if (bad) {
    atomicOr(a.error, 1);
    st.Qc = st.Qs = st.Mc = st.Ms = 0;
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) { st.pose[k] = a.pose[6 * p + k]; st.matX0[k] = 0.0f; }
  st.iter = 0; st.converged = 0; st.nc = 0; st.ns = 0;
  st.degenerate = a.deg_in ? a.deg_in[p] : 0;
  if (a.matP_in)
    for (int k = 0; k < 36; ++k) st.matP[k] = a.matP_in[36 * p + k];
  st.min_lambda = 0.0f; st.cf_mean = 0.0f;
  st.active = (!bad && st.Mc > 10 && st.Ms > 100) ? 1 : 0;  // MO:1573
  st.cR = cosf_(st.pose[0]); st.sR = sinf_(st.pose[0]);
  st.cP = cosf_(st.pose[1]); st.sP = sinf_(st.pose[1]);
  st.cY = cosf_(st.pose[2]); st.sY = sinf_(st.pose[2]);
  if (st.active) atomicAdd(a.n_active, 1);
}

using llsr_lm::kRed;

__device__ void lm_step(const S2MArgs& a, S2MProb& st, const float* red) {
  // LMOptimization (MO:1444-1570) after the Jacobian build; the solve / update / stop test is
  // llsr_lm::lm_update (shared with the oracle's split-sum restatement).
  st.iter += 1;
  const int iterCount = st.iter - 1;
  st.nc = (int)red[28];
  st.ns = (int)red[29];
  bool conv = false;
  if (st.nc + st.ns >= 50)  // MO:1453
    conv = llsr_lm::lm_update(st, red, iterCount, a.applied != 0, a.stop_thres);
  if (conv) st.converged = 1;
  if (conv || st.iter >= a.iter_max) {
    st.active = 0;
    atomicSub(a.n_active, 1);
  }
}

// One query of cornerOptimization (MO:1274-1375) / surfOptimization (MO:1383-1440) at the current
// pose: false without a correspondence, else its Jacobian row (LMOptimization MO:1465-1490), the
// right-hand side matB = -step_size * coeff.intensity and |coeff.intensity| (MO:1558).
template <bool kCorner>
__device__ __forceinline__ bool query_row(const S2MArgs& a, const S2MProb& st, int p, int qi, float* J, float& bb,
                                          float& ald) {
  const int Q = kCorner ? st.Qc : st.Qs;
  if (qi >= Q) return false;
  const float4 q = reinterpret_cast<const float4*>(kCorner ? a.cq : a.sq)[(kCorner ? st.qc0 : st.qs0) + qi];
  Assoc as{st.cR, st.sR, st.cP, st.sP, st.cY, st.sY, st.pose[3], st.pose[4], st.pose[5]};
  float x0, y0, z0;
  as.apply(q.x, q.y, q.z, x0, y0, z0);
  float la, lb, lc, ld;
  bool ok;
  if constexpr (kCorner) {
    const float4* mp = reinterpret_cast<const float4*>(a.cm) + st.mc0;
    ok = corner_coeff(a.grids.g[0].table(p), a.grids.g[0].log2T, a.grids.g[0].cells(p), mp,
                      x0, y0, z0, la, lb, lc, ld);
  } else {
    const float4* mp = reinterpret_cast<const float4*>(a.sm) + st.ms0;
    ok = surf_coeff(a.grids.g[1].table(p), a.grids.g[1].log2T, a.grids.g[1].cells(p), mp,
                    x0, y0, z0, la, lb, lc, ld);
  }
  if (!ok) return false;
  // Jacobian row (MO:1465-1490) at the current pose; srx.. are the same sin/cos values
  const float srx = st.sR, crx = st.cR, sry = st.sP, cry = st.cP, srz = st.sY, crz = st.cY;
  const float px = q.x, py = q.y, pz = q.z;
  J[0] = (crx * sry * srz * px + crx * crz * sry * py - srx * sry * pz) * la +
         (-srx * srz * px - crz * srx * py - crx * pz) * lb +
         (crx * cry * srz * px + crx * cry * crz * py - cry * srx * pz) * lc;
  J[1] = ((cry * srx * srz - crz * sry) * px + (sry * srz + cry * crz * srx) * py + crx * cry * pz) * la +
         ((-cry * crz - srx * sry * srz) * px + (cry * srz - crz * srx * sry) * py - crx * sry * pz) * lc;
  J[2] = ((crz * srx * sry - cry * srz) * px + (-cry * crz - srx * sry * srz) * py) * la +
         (crx * crz * px - crx * srz * py) * lb +
         ((sry * srz + cry * crz * srx) * px + (crz * sry - cry * srx * srz) * py) * lc;
  J[3] = la; J[4] = lb; J[5] = lc;
  bb = -a.step_size * ld;
  ald = fabs_(ld);
  return true;
}

// The split mode's per-query words: v[0..20] the AtA upper triangle, v[21..26] AtB, v[27]
// |coeff.intensity|, v[28] / v[29] = 1 for a corner / surf correspondence; all zero without one.
template <bool kCorner>
__device__ __forceinline__ void query_terms(const S2MArgs& a, const S2MProb& st, int p, int qi, float* v) {
#pragma unroll
  for (int k = 0; k < kRed; ++k) v[k] = 0.0f;
  float J[6], bb, ald;
  if (!query_row<kCorner>(a, st, p, qi, J, bb, ald)) return;
  int k = 0;
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = r; c < 6; ++c, ++k) v[k] = J[r] * J[c];
#pragma unroll
  for (int c = 0; c < 6; ++c) v[21 + c] = J[c] * bb;
  v[27] = ald;
  v[kCorner ? 28 : 29] = 1.0f;
}

// ---- the float path (llsr_scan2map_batch): Eigen's summation order ------------------------
// LMOptimization's matA rows are the correspondences in laserCloudOri order: the corner queries
// that found one, in query order, then the surf queries (MO:1582-1583). Each 256-query block of
// k_s2m_iter writes its rows compacted in that order (a.rows, 8 floats: J[6], matB, |intensity|)
// and its row count; k_s2m_solve (one workgroup per problem) then sums them
// exactly as the reference's Eigen 3.3.7 build does (llsr_eigen.h, oracle_eigen.h gemm_ata /
// gemv_atb) — matAt * matA per GEMM depth block of kc rows from zero, rows 4-5 x columns 0-3
// through gebp's four-accumulator path, the depth blocks added in order; matAt * matB and CF_all
// left to right — one lane per sum (the depth blocks spread over three waves), and runs the LM
// step. The
// result is bit-identical to the oracle's statement; one launch per LM iteration.
namespace {
constexpr int kRedWords = 29;   // AtA: 21 upper-triangle entries + the 8 of rows 4-5 x columns 0-3

// Exclusive prefix of the problem's block row counts into pre[0..blocks] (LDS).
__device__ void block_prefix(const S2MArgs& a, int p, int* pre, int* tmp) {
  const int nb = a.blocks, t = threadIdx.x;
  const int per = (nb + 255) / 256, b0 = t * per, b1 = min(nb, b0 + per);
  const int* cnt = a.bcnt + (size_t)p * nb;
  int s = 0;
  for (int b = b0; b < b1; ++b) s += cnt[b];
  tmp[t] = s;
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int k = 0; k < 256; ++k) { const int v = tmp[k]; tmp[k] = acc; acc += v; }
  }
  __syncthreads();
  s = tmp[t];
  for (int b = b0; b < b1; ++b) { pre[b] = s; s += cnt[b]; }
  if (b1 == nb && b0 < b1) pre[nb] = s;
  if (nb == 0 && t == 0) pre[0] = 0;
  __syncthreads();
}

// Rows [r0, r0 + d) of the problem's matA into lrow (LDS, 8 floats per row), all threads: each
// lane locates four rows at a time, then issues their eight loads at once.
__device__ void stage_rows(const S2MArgs& a, int p, const int* pre, int r0, int d, float4* lrow) {
  const int nb = a.blocks;
  constexpr int kU = 4;
  for (int i0 = 0; i0 < d; i0 += kU * 256) {
  const float4* src[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int i = i0 + threadIdx.x + u * 256;
    src[u] = nullptr;
    if (i < d) {
      const int g = r0 + i;
      int lo = 0, hi = nb - 1;  // the block b with pre[b] <= g < pre[b + 1]
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= g) lo = mid;
        else hi = mid - 1;
      }
      src[u] = a.rows + (((size_t)p * nb + lo) * 256 + (g - pre[lo])) * 2;
    }
  }
  float4 v0[kU], v1[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u)
    if (src[u]) { v0[u] = src[u][0]; v1[u] = src[u][1]; }
#pragma unroll
  for (int u = 0; u < kU; ++u)
    if (src[u]) {
      const int i = i0 + threadIdx.x + u * 256;
      lrow[2 * i] = v0[u];
      lrow[2 * i + 1] = v1[u];
    }
  }
}

// The problem's normal equations in Eigen's order and the LM step (MO:1444-1570), by one
// workgroup. The rows stream through LDS a.solve_rows at a time (all of them at once for the usual
// few thousand correspondences, so the waves never wait on each other); wave 0 lanes 0..6 sum matAt * matB (6,
// from the first product) and CF_all (from zero) over every row; waves 1..3 own the depth blocks of
// matAt * matA round robin (block x: wave 1 + x % 3), 29 lanes each (the 21 upper-triangle
// entries, then rows 4-5 x columns 0-3 through gebp's four-accumulator path), each block summed
// from zero; thread 0 adds the blocks in order and runs the LM step.
__device__ void s2m_assemble_solve(const S2MArgs& a, int p, int* pre, int* tmp, float4* lrow) {
  S2MProb& st = a.prob[p];
  block_prefix(a, p, pre, tmp);
  if (S2M_DBG(a) == 1) return;
  const int N = pre[a.blocks];
  const int nc = pre[a.blocks_c];
  const int t = threadIdx.x, wv = t >> 6, ln = t & 63;
  // per-depth-block sums: the first kLdsDepthBlocks in LDS, the rest (N above ~44k rows) in the
  // problem's global spill rows (a.blk_spill, sized at reserve for the reserved query counts)
  constexpr int kLdsDepthBlocks = 64;
  __shared__ float s_blk[kLdsDepthBlocks][kRedWords];
  __shared__ float s_b[7];
  float* spill = a.blk_spill + (size_t)p * a.spill_cap * kRedWords;
  auto blk = [&](int x, int e) -> float& {
    return x < kLdsDepthBlocks ? s_blk[x][e] : spill[(size_t)(x - kLdsDepthBlocks) * kRedWords + e];
  };
  const int kc = N >= 50 ? llsr_eigen::gemm_kc(N, 6, 6) : 1;
  const int nkb = N >= 50 ? (N + kc - 1) / kc : 0;
  const bool fits = nkb <= kLdsDepthBlocks + a.spill_cap;  // always, for clouds within the reserve
  // lane roles: wave 0 lanes < 7 -> matB / CF; waves 1..3 lanes < 29 -> AtA
  int ia = 0, ib = 0;
  bool sw = false;
  if (wv == 0) {
    ia = ln < 6 ? ln : 7;
    ib = 6;
  } else if (ln < 21) {
    int i = 0, k = ln;
    while (k >= 6 - i) { k -= 6 - i; ++i; }
    ia = i; ib = i + k;
  } else if (ln < kRedWords) {
    sw = true; ia = 4 + (ln - 21) / 4; ib = (ln - 21) % 4;
  }
  const bool busy = (wv == 0 && ln < 7) || (wv > 0 && ln < kRedWords);
  float c = 0.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f, C3 = 0.0f;
  if (N >= 50) {
    for (int r0 = 0; r0 < N; r0 += a.solve_rows) {
      const int d = min(a.solve_rows, N - r0);
      stage_rows(a, p, pre, r0, d, lrow);
      __syncthreads();
      if (S2M_DBG(a) == 2 || !fits) continue;
      const float* lr = reinterpret_cast<const float*>(lrow);
      if (busy && wv == 0 && S2M_DBG(a) != 5) {
        // the products do not depend on the running sum: load 8 rows ahead, then add in order;
        // loads unconditional and the CF lane's factor a select, so the loop has no branch
        const int ib2 = ln < 6 ? 6 : 7, ia2 = ln < 6 ? ia : 7;
        const bool mul = ln < 6;
        int q = 0;
        if (r0 == 0) {
          const float x = lr[ia2], y = lr[ib2];
          c = mul ? x * y : c + x;
          q = 1;
        }
        for (; q + 32 <= d; q += 32) {
          float v[32];
#pragma unroll
          for (int u = 0; u < 32; ++u) {
            const float x = lr[8 * (q + u) + ia2], y = lr[8 * (q + u) + ib2];
            v[u] = x * (mul ? y : 1.0f);
          }
#pragma unroll
          for (int u = 0; u < 32; ++u) c = c + v[u];
        }
        for (; q < d; ++q) {
          const float x = lr[8 * q + ia2], y = lr[8 * q + ib2];
          c = c + x * (mul ? y : 1.0f);
        }
      } else if (wv > 0 && S2M_DBG(a) != 4 && d == N) {
        // every row is in LDS: each depth block runs on 53 lanes of one wave without selects —
        // lanes 0..20 the upper-triangle entries (c = c + a_i a_j over the block), lanes 21..52 the
        // 8 swapped entries x 4 accumulators (lane u sums rows q = u mod 4 below endk4), merged as
        // (C0 + C1) + (C2 + C3) and followed by the remainder rows on the entry's first lane
        const bool nrm = ln < 21;
        const int e8 = (ln - 21) >> 2, u4 = (ln - 21) & 3;
        int fa = ia, fb = ib;
        if (!nrm && ln < 53) { fa = 4 + e8 / 4; fb = e8 % 4; }
        for (int x = wv - 1; x < nkb; x += 3) {
          const int k2 = x * kc, db = min(kc, N - k2), endk4 = (db / 4) * 4;
          const int q0 = nrm ? 0 : u4, qs = nrm ? 1 : 4, qe = nrm ? db : endk4;
          float acc = 0.0f;
          int q = q0;
          for (; q + 7 * qs < qe; q += 8 * qs) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const float* row = lr + 8 * (k2 + q + u * qs);
              v[u] = nrm ? row[fa] * row[fb] : row[fb] * row[fa];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc = nrm ? acc + v[u] : v[u] + acc;
          }
          for (; q < qe; q += qs) {
            const float* row = lr + 8 * (k2 + q);
            acc = nrm ? acc + row[fa] * row[fb] : row[fb] * row[fa] + acc;
          }
          // swapped entries: merge the four accumulators on the entry's first lane
          const int base = 21 + 4 * e8;
          const float a0 = __shfl(acc, base & 63), a1 = __shfl(acc, (base + 1) & 63);
          const float a2 = __shfl(acc, (base + 2) & 63), a3 = __shfl(acc, (base + 3) & 63);
          if (ln < 21) {
            blk(x, ln) = acc;
          } else if (ln < 53 && u4 == 0) {
            float cc = (a0 + a1) + (a2 + a3);
            for (int qq = endk4; qq < db; ++qq) {
              const float* row = lr + 8 * (k2 + qq);
              cc = row[fb] * row[fa] + cc;
            }
            blk(x, 21 + e8) = cc;
          }
        }
      } else if (busy && wv > 0 && S2M_DBG(a) != 4) {
        // the rows stream in chunks: the depth-block segments of this chunk that belong to this wave
        for (int g = r0; g < r0 + d;) {
          const int x = g / kc, k2 = x * kc, db = min(kc, N - k2);
          const int ge = min(k2 + db, r0 + d);
          if (x % 3 == wv - 1) {
            const int endk4 = (db / 4) * 4;
            // branch-free per row: gebp's four accumulators by qq mod 4 below endk4 (swapped
            // lanes), the merge at endk4, then c = c + product
            auto step = [&](int qq, float pr) {
              const bool mn = sw && qq < endk4;
              const int uu = qq & 3;
              C0 = (mn && uu == 0) ? pr + C0 : C0;
              C1 = (mn && uu == 1) ? pr + C1 : C1;
              C2 = (mn && uu == 2) ? pr + C2 : C2;
              C3 = (mn && uu == 3) ? pr + C3 : C3;
              const float cb = (sw && qq == endk4) ? (C0 + C1) + (C2 + C3) : c;
              c = mn ? c : cb + pr;
            };
            int gg = g;
            for (; gg + 8 <= ge; gg += 8) {
              float v[8];  // the products, 8 rows ahead of the in-order additions
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const float* row = lr + 8 * (gg + u - r0);
                v[u] = row[ia] * row[ib];
              }
#pragma unroll
              for (int u = 0; u < 8; ++u) step(gg + u - k2, v[u]);
            }
            for (; gg < ge; ++gg) {
              const float* row = lr + 8 * (gg - r0);
              step(gg - k2, row[ia] * row[ib]);
            }
            if (ge == k2 + db) {  // the depth block is complete
              const float v = (sw && endk4 == db) ? (C0 + C1) + (C2 + C3) : c;
              blk(x, ln) = v;
              c = 0.0f; C0 = 0.0f; C1 = 0.0f; C2 = 0.0f; C3 = 0.0f;
            }
          }
          g = ge;
        }
      }
      __syncthreads();
    }
    if (wv == 0 && ln < 7) s_b[ln] = c;
  }
  __syncthreads();
  if (t != 0 || (S2M_DBG(a) >= 2 && S2M_DBG(a) <= 5)) return;
  st.iter += 1;
  const int iterCount = st.iter - 1;
  st.nc = nc;
  st.ns = N - nc;
  bool conv = false;
  if (N >= 50 && fits) {  // MO:1453
    float wsum[kRedWords];
    for (int e = 0; e < kRedWords; ++e) wsum[e] = 0.0f;
    for (int x = 0; x < nkb; ++x)
      for (int e = 0; e < kRedWords; ++e) wsum[e] = wsum[e] + 1.0f * blk(x, e);
    float AtA[36];
    int e = 0;
    for (int r = 0; r < 6; ++r)
      for (int q = r; q < 6; ++q, ++e) { AtA[r + 6 * q] = wsum[e]; AtA[q + 6 * r] = wsum[e]; }
    for (int r = 4; r < 6; ++r)
      for (int q = 0; q < 4; ++q, ++e) AtA[r + 6 * q] = wsum[e];
    conv = llsr_lm::lm_update_full(st, AtA, s_b, s_b[6], N, iterCount, a.applied != 0, a.stop_thres);
  } else if (N >= 50) {
    atomicOr(a.error, 4);  // more depth blocks than reserved (not reachable within the reserve)
  }
  if (conv) st.converged = 1;
  if (conv || st.iter >= a.iter_max) {
    st.active = 0;
    atomicSub(a.n_active, 1);
  }
}
}  // namespace

template <bool kCorner>
__device__ __forceinline__ void s2m_block(const S2MArgs& a, int p, int qb) {
  S2MProb& st = a.prob[p];
  if (!st.active) return;
  __shared__ int wcnt[4];
  float J[6], bb = 0.0f, ald = 0.0f;
  const bool ok = query_row<kCorner>(a, st, p, qb * 256 + threadIdx.x, J, bb, ald);
  const unsigned long long m = __ballot(ok);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) wcnt[w] = __popcll(m);
  __syncthreads();
  const int gb = (kCorner ? 0 : a.blocks_c) + qb;
  int base = 0;
  for (int k = 0; k < w; ++k) base += wcnt[k];
  if (ok) {
    float4* r = a.rows + (((size_t)p * a.blocks + gb) * 256 + base + __popcll(m & ((1ull << lane) - 1))) * 2;
    r[0] = make_float4(J[0], J[1], J[2], J[3]);
    r[1] = make_float4(J[4], J[5], bb, ald);
  }
  if (threadIdx.x == 0) a.bcnt[(size_t)p * a.blocks + gb] = (wcnt[0] + wcnt[1]) + (wcnt[2] + wcnt[3]);
}

// XCD-aware placement of the (problem, query block) workgroups: the dispatcher deals workgroups
// round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch), so with a plain
// (blocks, P) grid every problem's blocks land on all 8 XCDs and each XCD's L2 fetches the same
// local map. Linear workgroup L -> XCD class x = L % 8 and slot j = L / 8; class x runs the blocks
// of problems x, x + 8, x + 16, ... in order, so a problem's map is read through one L2 (and
// k_s2m_solve's workgroup p, class p % 8, finds its rows there). Placement only: results do not
// depend on it. Grid: 8 * ceil(P / 8) * nb workgroups; false = padding.
__device__ __forceinline__ bool xcd_problem_block(int nb, int P, int& p, int& b) {
  const int L = (int)blockIdx.x;
  const int j = L >> 3;
  const int pp = j / nb;
  b = j - pp * nb;
  p = pp * 8 + (L & 7);
  return p < P;
}

// grid 8 * ceil(P / 8) * blocks (xcd_problem_block): corner blocks first, then surf blocks; the
// branch is block-uniform. 8 waves per SIMD (64 VGPRs, 10 spilled): the kNN gathers are latency-
// bound, more waves hide more of them (lm_applied 31.3k -> 32.9k, faithful 1.52k -> 1.66k problems/s).
__global__ __launch_bounds__(256, 8) void k_s2m_iter(S2MArgs a) {
  int p, b;
  if (!xcd_problem_block(a.blocks, a.P, p, b)) return;
  if (b < a.blocks_c)
    s2m_block<true>(a, p, b);
  else
    s2m_block<false>(a, p, b - a.blocks_c);
}

// grid P, 256 threads, dynamic LDS a.solve_lds bytes: one workgroup per problem assembles the
// normal equations from the rows k_s2m_iter wrote (the kernel boundary makes them visible: no
// device-scope fences, which would write back every L2 on MI355X's eight XCDs) and solves.
__global__ __launch_bounds__(256) void k_s2m_solve(S2MArgs a) {
  const int p = blockIdx.x;
  if (!a.prob[p].active) return;
  extern __shared__ int s_dyn[];  // [blocks + 1] block prefix, then a.solve_rows matA rows
  __shared__ int tmp[256];
  float4* lrow = reinterpret_cast<float4*>(s_dyn + ((a.blocks + 4) & ~3));
  s2m_assemble_solve(a, p, s_dyn, tmp, lrow);
}

// ---- split-correspondence mode (llsr_scan2map_shard_*) ----------------------
// Every term is rounded once to int64 fixed point (llsr_lm::ne_term) and summed with integer
// adds: the wave / block sums and the global atomics are exact, so the words do not depend on
// how the queries are split over blocks or ranks, nor on the order the atomics land.
template <bool kCorner>
__device__ __forceinline__ void s2m_block_fx(const S2MArgs& a, int p, int qb) {
  const S2MProb& st = a.prob[p];
  if (!st.active) return;
  __shared__ long long wsum[4][kRed + 1];
  float v[kRed];
  query_terms<kCorner>(a, st, p, qb * 256 + threadIdx.x, v);
  const int w = threadIdx.x >> 6;
  int bad = 0;  // terms outside the fixed-point range: contribute 0, counted in word 31
#pragma unroll
  for (int k = 0; k < kRed; ++k) {
    bad += llsr_lm::ne_bad(k, v[k]);
    const long long s = wave_reduce_add(llsr_lm::ne_term(k, v[k]));
    if (lane_id() == 0) wsum[w][k] = s;
  }
  {
    const long long s = wave_reduce_add((long long)bad);
    if (lane_id() == 0) wsum[w][kRed] = s;
  }
  __syncthreads();
  if (threadIdx.x <= kRed) {
    const int k = threadIdx.x;
    const long long t = wsum[0][k] + wsum[1][k] + wsum[2][k] + wsum[3][k];
    const int word = k < kRed ? k : llsr_lm::kNeOverflow;
    if (t != 0)
      atomicAdd(reinterpret_cast<unsigned long long*>(a.ne + (size_t)p * llsr_lm::kNeWords + word),
                (unsigned long long)t);
  }
}

// grid 8 * ceil(P / 8) * nb with nb = ceil(blocks_c / world) + ceil(blocks_s / world)
// (xcd_problem_block): rank r takes the corner blocks r, r + world, ... and likewise the surf blocks.
__global__ __launch_bounds__(256, 8) void k_s2m_iter_fx(S2MArgs a, int nb) {
  int p, bx;
  if (!xcd_problem_block(nb, a.P, p, bx)) return;
  const int bcw = (a.blocks_c + a.world - 1) / a.world;
  if (bx < bcw)
    s2m_block_fx<true>(a, p, bx * a.world + a.rank);
  else
    s2m_block_fx<false>(a, p, (bx - bcw) * a.world + a.rank);
}

// One thread per problem: the summed words (all ranks) -> the LM step.
__global__ __launch_bounds__(64) void k_s2m_solve_fx(S2MArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.P) return;
  S2MProb& st = a.prob[p];
  if (!st.active) return;
  const long long* w = a.ne + (size_t)p * llsr_lm::kNeWords;
  if (w[llsr_lm::kNeOverflow] != 0) atomicOr(a.error, 2);  // reported by llsr_scan2map_shard_step
  float red[kRed];
  llsr_lm::ne_to_red(w, red);
  lm_step(a, st, red);
}

__global__ void k_s2m_finish(S2MArgs a) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.P) return;
  const S2MProb& st = a.prob[p];
  llsr_lm_report& r = a.report[p];
  r.iterations = st.iter;
  r.converged = st.converged;
  r.degenerate = st.degenerate;
  r.min_lambda = st.min_lambda;
  r.cf_mean = st.cf_mean;
  r.n_corner_corr = st.nc;
  r.n_surf_corr = st.ns;
  for (int k = 0; k < 6; ++k) {
    r.matX0[k] = st.matX0[k];
    r.pose[k] = st.pose[k];
    a.pose[6 * p + k] = st.pose[k];
  }
  r.ms = 0.0f;
  if (a.deg_out) a.deg_out[p] = st.degenerate;
  if (a.matP_out)
    for (int k = 0; k < 36; ++k) a.matP_out[36 * p + k] = st.matP[k];
}

}  // namespace llsr
