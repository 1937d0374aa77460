// llsr_ip.hip — ImageProjection on gfx950: projection, ground segmentation, connected-component
// labelling and segmented-cloud extraction for a batch of scans (one slot per scan).
//
// Reference: LeGO-LOAM/src/imageProjection.cpp (IP). Each kernel names the lines it restates.
// Built with -ffp-contract=off: every float/double expression below evaluates in the same order
// and precision as the reference's x86-64 -O3 build, so outputs are bit-identical.
#include <cfloat>
#include <climits>

#include "llsr_device.h"
#include "llsr_libm.h"

namespace llsr {

using namespace llsr_libm;

constexpr double kPi = 3.14159265358979323846;

__device__ __forceinline__ bool finite3(float4 p) {
  return __builtin_isfinite(p.x) && __builtin_isfinite(p.y) && __builtin_isfinite(p.z);
}

__device__ __forceinline__ int project_cell(const DevCfg& c, float4 p, float* range_out) {
  const float range = sqrt_(p.x * p.x + p.y * p.y + p.z * p.z);
  *range_out = range;
  const float va = asinf_(p.z / range);
  const int row = trunc_i32((double)((va + c.ip_angBottom) / c.ip_resY));
  if (row < 0 || row >= c.H) return -1;
  const float ha = atan2f_(p.x, p.y);
  int col = trunc_i32(-round(((double)ha - kPi / 2) / (double)c.ip_resX) + c.W * 0.5);
  if (col >= c.W) col -= c.W;
  if (col < 0 || col >= c.W || (double)range < 0.1) return -1;
  return col + row * c.W;
}

// Certified fast path for project_cell. The cell depends on asinf/atan2f only through a truncated
// (row) and a rounded (column) quotient, both monotone in the angle, so an approximation with a
// known error bound decides the cell exactly unless the quotient lies within that bound of a
// decision boundary; only then (and for |z/r| >= 0.5, zero / non-finite operands, a range within
// 1 % of the 0.1 m cut) the lane takes the exact libm path.
// Row: s = z / r from the hardware reciprocal square root (<= 1 ulp) and a multiply: within
// 2.5 * 2^-23 |s| of the reference's correctly rounded sqrt and divide, so the angle within
// 3.5e-7 |s| <= 1.75e-7 (|s| < 0.5, asin' <= 1.155); asinf_ below 0.5 IS the fdlibm odd polynomial
// (same ops as asinf_); the quotient by res_Y is a multiply by the reciprocal (|err| <= 2^-22 |q|).
// Margin around every non-zero integer: 1e-5 |q| + 1e-6 + 4e-7 / res_Y (trunc maps (-1, 1) to 0).
// Column: atan2 from a hardware reciprocal (<= 1 ulp) and a degree-15 odd minimax polynomial (3.7e-8
// on [0, 1]) plus the octant fix-ups: |ha - atan2f_| < 1e-6 rad (measured < 6e-7, tests/test_libm.py);
// the double quotient (ha - pi/2) / res_X becomes a float multiply (|err| <= 2^-22 |q| + 3e-7 /
// res_X), and the margin 4e-6 / res_X + 2.4e-7 |q| around every half-integer covers both with 2-4x
// to spare. round(q) and the W / 2 offset are integer arithmetic for even W.
// Bit-exact by construction; tests/test_gpu_projection_edges.py puts points on the boundaries.
// Returns the row (>= 0) and *colp, or -1 (no cell); *ok = false: undecided, use project_cell.
__device__ __forceinline__ int project_cell_fast(const DevCfg& c, float4 p, float invResY, float invResX,
                                                 bool* ok, int* colp) {
  const float r2 = p.x * p.x + p.y * p.y + p.z * p.z;  // the reference's sqrt argument, same ops
  const float s = p.z * __builtin_amdgcn_rsqf(r2);
  const uint32_t is = fbits(s) & 0x7fffffffu;
  // |s| < 0.5 (false for NaN); range = fl(sqrt(r2)) vs 0.1 decided away from r2 in [0.0099, 0.0101]
  bool good = is < 0x3f000000u && (r2 < 0.0099f || r2 > 0.0101f);
  const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f,
              p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  const float t2 = s * s;
  const float w = t2 * (p0 + t2 * (p1 + t2 * (p2 + t2 * (p3 + t2 * p4))));
  const float va = is < 0x32000000u ? s : s + s * w;
  const float qr = (va + c.ip_angBottom) * invResY;
  const float rr = __builtin_rintf(qr);
  good = good && (rr == 0.0f || fabsf(qr - rr) > 1e-5f * fabsf(qr) + 1e-6f + 4e-7f * invResY);
  const int row = (int)__builtin_truncf(qr);
  const float a = p.x, b = p.y;
  const float ax = fabsf(a), bx = fabsf(b);
  const float mx = fmaxf(ax, bx), mn = fminf(ax, bx);
  good = good && mn > 0.0f && mx < 1e30f;
  if (!good || row < 0 || row >= c.H) {
    *ok = good;
    return -1;
  }
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
  ha = b < 0.0f ? 3.14159274f - ha : ha;
  ha = a < 0.0f ? -ha : ha;
  const float qc = (ha - 1.57079637f) * invResX;
  const float fl = __builtin_floorf(qc);
  good = fabsf(qc - fl - 0.5f) > 4e-6f * invResX + 2.4e-7f * fabsf(qc);
  *ok = good;
  const float rq = qc - fl < 0.5f ? fl : fl + 1.0f;  // round(qc) away from the half-integers
  int col;
  if ((c.W & 1) == 0) col = (c.W >> 1) - (int)rq;   // -round + W * 0.5, exact in integers
  else col = trunc_i32(-(double)rq + c.W * 0.5);
  if (col >= c.W) col -= c.W;
  if (col < 0 || col >= c.W || r2 < 0.0099f) return -1;  // (double)fl(sqrt(r2)) < 0.1
  *colp = col;
  return row;
}

// project_cell's (row, col) through the certified fast path, the exact libm path where it cannot
// decide; returns the row or -1
__device__ __forceinline__ int project_cell_any(const DevCfg& c, float4 p, float invResY, float invResX, int* colp) {
  bool ok;
  int row = project_cell_fast(c, p, invResY, invResX, &ok, colp);
  if (!ok) {
    float r;
    const int cell = project_cell(c, p, &r);
    row = cell < 0 ? -1 : cell / c.W;
    if (cell >= 0) *colp = cell - row * c.W;
  }
  return row;
}

// ---------------------------------------------------------------------------------------------
// K1 project: removeNaNFromPointCloud (IP:198) + projectPointCloud row/col (IP:305-336).
// One thread per raw point; the serial "last writer wins" of IP:337-347 becomes atomicMax of
// the raw index per cell (the compacted order preserves raw order). Also counts finite points
// and the first/last finite index for findStartEndAngle (IP:430-436).
// The winners go to a COLUMN-major scratch table (ccl_a, dead until k_label): Velodyne order
// fires all rings of one azimuth back to back, so a wave's stores land in one or two 128-byte
// lines instead of 64 (row-major: one line per ring). k_gather_column turns it row-major.
// (Measured per 512 HDL-64E scans: per-wave counter atomics 4.17 ms -> per-workgroup 0.36 ms; a
// plain-store pass plus an atomicMax fix-up pass for colliding cells was slower, 0.61 ms.)
// grid (ceil(maxN/256), B), block 256.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_project(DevCfg c, const float4* __restrict__ pts,
                                                 const int64_t* __restrict__ off, DevBufs d) {
  const int b = blockIdx.y;
  const int64_t o0 = off[b], n = off[b + 1] - o0;
  // grid-stride over the scan: every raw point is projected whatever the grid's width; the
  // finite-point count and first / last finite index are reduced per workgroup (3 atomics each)
  int npts = 0, first = INT_MAX, last = -1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 p = pts[o0 + i];
    if (!finite3(p)) continue;
    ++npts;
    first = min(first, (int)i);
    last = max(last, (int)i);
    int col;
    const int row = project_cell_any(c, p, 1.0f / c.ip_resY, 1.0f / c.ip_resX, &col);
    if (row >= 0) atomicMax(&d.ccl_a[(size_t)b * c.HW + (size_t)col * c.H + row], (int)i);
  }
  __shared__ int red[3][4];
  npts = wave_reduce_add(npts);
  first = wave_reduce_min(first);
  last = wave_reduce_max(last);
  if (lane_id() == 0) { red[0][threadIdx.x >> 6] = npts; red[1][threadIdx.x >> 6] = first; red[2][threadIdx.x >> 6] = last; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int w = 1; w < nw; ++w) {
      npts += red[0][w];
      first = min(first, red[1][w]);
      last = max(last, red[2][w]);
    }
    if (npts) {
      int* cnt = d.counts + b * kCnt;
      atomicAdd(&cnt[C_NPTS], npts);
      atomicMin(&cnt[C_FIRST], first);
      atomicMax(&cnt[C_LAST], last);
    }
  }
}

// groundRemovalOurs' per-column test (IP:524-629) as a step over one column's state, so a lane can
// carry two columns at once: their serial 16-row chains interleave (ILP) instead of running in two
// rounds of lanes.
struct GndState {
  bool haveRV = false, obs = false;
  float RVx = 0.f, RVy = 0.f, RVz = 0.f, lx = 0.f, ly = 0.f, lz = 0.f;
};
__device__ __forceinline__ int8_t ground_step(const DevCfg& c, GndState& st, float4 f, int i) {
  int8_t g;
  if (f.w == 0.0f) {
    g = -1;
  } else if (!st.haveRV) {
    const float d0 = sqrt_(f.x * f.x + f.y * f.y);
    st.RVx = f.x / d0; st.RVy = f.y / d0; st.RVz = 0.0f;
    st.haveRV = true;
    st.lx = f.x; st.ly = f.y; st.lz = f.z;
    g = 1;
  } else {
    const float TVx = f.x - st.lx, TVy = f.y - st.ly, TVz = f.z - st.lz;
    // (float)(acosf(x) / deg) <= D  <=>  gnd_cos(D) <= x <= 1  (llsr_libm.h ground_cos_threshold)
    const float x = (TVx * st.RVx + TVy * st.RVy + TVz * st.RVz) /
                    (sqrt_(TVx * TVx + TVy * TVy + TVz * TVz) *
                     sqrt_(st.RVx * st.RVx + st.RVy * st.RVy + st.RVz * st.RVz));
    const float xs = c.use_kitti ? (i < 16 ? c.gnd_cos[1] : c.gnd_cos[2]) : c.gnd_cos[0];
    if (x >= xs && x <= 1.0f) { st.RVx += TVx; st.RVy += TVy; st.RVz += TVz; g = 1; }
    else g = 0;
    st.lx = f.x; st.ly = f.y; st.lz = f.z;
  }
  // Filter (IP:620-628): after the first 0 of the column every 1 becomes 2.
  if (g == 0) st.obs = true;
  else if (g == 1 && st.obs) g = 2;
  return g;
}

// ---------------------------------------------------------------------------------------------
// K2 gather + ground column pass: builds range_mat/full_cloud for each cell (IP:337-347,
// resetParameters IP:170-179) and runs groundRemovalOurs' per-column vector test and Filter
// (IP:524-629) in the same sweep. One thread per (scan, column), rows bottom-up. The wave's 64
// columns of k_project's column-major winner table are one contiguous run of 64 * H ints: loaded
// coalesced into LDS (column stride H + 1 against bank conflicts), then read per column; the
// row-major cell->point map is written here.
// grid (ceil(W/64), B), block 64, dynamic LDS 64 * (H + 1) ints.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_gather_column(DevCfg c, const float4* __restrict__ pts,
                                                      const int64_t* __restrict__ off, DevBufs d) {
  extern __shared__ int lwin[];
  const int b = blockIdx.y;
  const int j0 = blockIdx.x * blockDim.x;
  const int j = j0 + threadIdx.x;
  const int64_t o0 = off[b];
  const size_t base = (size_t)b * c.HW;
  {
    const int ncol = min(64, c.W - j0);
    const int* src = d.ccl_a + base + (size_t)j0 * c.H;  // columns j0 .. j0 + ncol - 1, row 0 first
    for (int t = threadIdx.x; t < ncol * c.H; t += 64) {
      const int cj = t / c.H, ci = t - cj * c.H;
      lwin[cj * (c.H + 1) + ci] = src[t];
    }
  }
  __syncthreads();
  if (j >= c.W) return;
  const int* colw = lwin + threadIdx.x * (c.H + 1);  // this column's winners, row 0 first
  const float qnan = __builtin_nanf("");
  GndState st;
  // rows in groups of kR: the group's winner points are gathered with all loads in flight, then
  // the column's serial ground chain runs over them (one load latency per group, not per row)
  constexpr int kR = 8;
  for (int i0 = 0; i0 < c.H; i0 += kR) {
    float4 pg[kR];
    int wg[kR];
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      wg[u] = i0 + u < c.H ? colw[i0 + u] : -1;
      pg[u] = wg[u] >= 0 ? pts[o0 + wg[u]] : make_float4(qnan, qnan, qnan, 0.0f);
    }
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const int i = i0 + u;
      if (i >= c.H) break;
      const int cell = j + i * c.W;
      const float4 p = pg[u];
      d.cell_pt[base + cell] = wg[u];
      d.range[base + cell] = wg[u] >= 0 ? sqrt_(p.x * p.x + p.y * p.y + p.z * p.z) : FLT_MAX;
      d.full[base + cell] = p;
      // IP:535: NaN cells (and a real point at row 0, col 0) have intensity 0
      const float w = wg[u] >= 0 ? cell_intensity(c.H, c.W, i, j) : 0.0f;
      d.ground[base + cell] = ground_step(c, st, make_float4(p.x, p.y, p.z, w), i);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// K1+K2 fused for range images that fit LDS (H <= 16, H*W <= 32000, e.g. VLP-16): one workgroup per scan.
// The claim pass projects every raw point once (coalesced reads) and resolves IP:337-347's serial
// "last writer wins" with an LDS atomicMax of the raw index per cell, each cell's winner writing its
// range and its raw point (x, y, z, raw intensity: fullCloud with the intensity row + col / 1e4
// derived where needed, cell_intensity); a sweep of the final winner table writes the cell ->
// point map and the resetParameters values of empty cells (IP:170-179); the per-column ground test
// + Filter (IP:524-629) reads the kept points back. No global atomics.
// ---------------------------------------------------------------------------------------------
// columns j0 and j1 (j1 >= W: none), their cells loaded 8 rows at a time ahead of the tests;
// cellf(cell) = (x, y, z, w) with w == 0 exactly for the cells groundRemoval skips (IP:535)
template <class CellF>
__device__ __forceinline__ void ground_columns2(const DevCfg& c, CellF cellf, int8_t* ground, int j0, int j1) {
  GndState s0, s1;
  const bool has1 = j1 < c.W;
  constexpr int kR = 8;
  for (int i0 = 0; i0 < c.H; i0 += kR) {
    float4 f0[kR], f1[kR];
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const bool in = i0 + u < c.H;
      f0[u] = in ? cellf(j0 + (i0 + u) * c.W) : make_float4(0.f, 0.f, 0.f, 0.f);
      f1[u] = in && has1 ? cellf(j1 + (i0 + u) * c.W) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const int i = i0 + u;
      if (i >= c.H) break;
      const int8_t g0 = ground_step(c, s0, f0[u], i);
      const int8_t g1 = ground_step(c, s1, f1[u], i);
      ground[j0 + i * c.W] = g0;
      if (has1) ground[j1 + i * c.W] = g1;
    }
  }
}

// The cell table holds each cell's winning raw index (LDS atomicMax; -1 = empty), 115 KB for
// VLP-16, next to the 25 KB pass-2 transpose tile.
__global__ __launch_bounds__(1024) void k_project_fused(DevCfg c, const float4* __restrict__ pts,
                                                        const int64_t* __restrict__ off, DevBufs d) {
  extern __shared__ int cidx[];
  __shared__ int tmp[32];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int HW = c.HW;
  const size_t base = (size_t)b * HW;
  const int64_t o0 = off[b];
  const int n = (int)(off[b + 1] - o0);
  for (int q = tid; q < HW; q += nt) cidx[q] = -1;
  __syncthreads();
  int nfin = 0, first = INT_MAX, last = -1;
  const float invResY = 1.0f / c.ip_resY, invResX = 1.0f / c.ip_resX;
  const float qnan = __builtin_nanf("");
  const int W = c.W;
  // Chunks of nt raw points in DESCENDING index order. "Last writer wins" (IP:337-347) makes a
  // cell's point the largest raw index mapped to it, so once a chunk has raised the LDS winner table
  // (atomicMax) a cell holding an index of THIS chunk is final: no later-processed (lower-index)
  // point can take it. Its winner emits the cell's range and point from registers, so the claim
  // pass reads the raw points from HBM exactly once. A firing-ordered stream (Velodyne:
  // the rings of one azimuth are consecutive) puts a chunk's cells in a band of ~nt / H columns:
  // winners inside the 64-column band starting at the chunk's smallest column go through an LDS
  // tile written out row by row (full lines); any other winner (wrap-around, unordered input)
  // writes its cell directly.
  // Chunks of kU * nt points (kU per lane, the loads of the next two chunks in flight during this
  // chunk's barriers); the tile holds the band's points, and "won in this chunk" is read back from
  // the winner table (index within the chunk's range).
  constexpr int kU = 2, kTC = 128, kTP = kTC + 1;  // padded rows
  __shared__ float4 tfull[16 * kTP];
  __shared__ int s_cmin[2];
  if (tid < 2) s_cmin[tid] = INT_MAX;
  const int C = kU * nt;
  const int nch = (n + C - 1) / C;
  // two chunks of loads in flight (buffers A / B alternate, so no register copy waits on a load
  // that is still outstanding)
  float4 pa[kU], pb[kU];
  auto load = [&](float4 (&buf)[kU], int ch) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = ch * C + u * nt + tid;
      buf[u] = (ch >= 0 && i < n) ? pts[o0 + i] : make_float4(qnan, 0.f, 0.f, 0.f);
    }
  };
  auto chunk = [&](int ch, const float4 (&pp)[kU]) {
    const int par = ch & 1;
    const int lo = ch * C, hi = lo + C;  // this chunk's raw index range
    if (tid == 0) s_cmin[par ^ 1] = INT_MAX;  // the next chunk's
    int cell[kU], row[kU], col[kU];
    int cm = INT_MAX;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = lo + u * nt + tid;
      cell[u] = -1;
      row[u] = 0;
      col[u] = INT_MAX;
      if (!finite3(pp[u])) continue;
      ++nfin;
      first = i < first ? i : first;
      last = i > last ? i : last;
      int cc;
      const int rw = project_cell_any(c, pp[u], invResY, invResX, &cc);
      if (rw >= 0) {
        cell[u] = cc + rw * W;
        atomicMax(&cidx[cell[u]], i);
        row[u] = rw;
        col[u] = cc;
        cm = cc < cm ? cc : cm;
      }
    }
    cm = wave_reduce_min(cm);
    if (lane_id() == 0 && cm != INT_MAX) atomicMin(&s_cmin[par], cm);
    __syncthreads();
    const int c0 = s_cmin[par];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = lo + u * nt + tid;
      if (cell[u] < 0 || cidx[cell[u]] != i) continue;
      const float4 p = pp[u];
      if (col[u] - c0 < kTC) {
        tfull[row[u] * kTP + (col[u] - c0)] = p;
      } else {
        d.range[base + cell[u]] = sqrt_(p.x * p.x + p.y * p.y + p.z * p.z);
        d.full[base + cell[u]] = p;
      }
    }
    __syncthreads();
    if (c0 != INT_MAX) {  // row-major over the tile: the cells this chunk won
      for (int t = tid; t < c.H * kTC; t += nt) {
        const int trow = t / kTC, ck = t % kTC, tcol = c0 + ck;
        if (tcol >= W) continue;
        const int wpi = cidx[trow * W + tcol];
        if (wpi < lo || wpi >= hi) continue;
        const float4 f = tfull[trow * kTP + ck];
        const size_t q = base + (size_t)trow * W + tcol;
        d.range[q] = sqrt_(f.x * f.x + f.y * f.y + f.z * f.z);
        d.full[q] = f;
      }
    }
    __syncthreads();
  };
  load(pa, nch - 1);
  load(pb, nch - 2);
  __syncthreads();
  for (int ch = nch - 1; ch >= 0; ch -= 2) {
    float4 pp[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) pp[u] = pa[u];
    load(pa, ch - 2);
    chunk(ch, pp);
    if (ch == 0) break;
#pragma unroll
    for (int u = 0; u < kU; ++u) pp[u] = pb[u];
    load(pb, ch - 3);
    chunk(ch - 1, pp);
  }
  nfin = block_reduce_add(nfin, tmp);
  first = block_reduce_min(first, tmp);
  last = -block_reduce_min(-last, tmp);
  if (tid == 0) {
    int* cnt = d.counts + b * kCnt;
    cnt[C_NPTS] = nfin;
    cnt[C_FIRST] = first;
    cnt[C_LAST] = last;
  }
  if (c.dbg_phase <= 0) return;
  // the cell -> point map from the final winner table; cells no point reached keep the
  // resetParameters range (IP:170-179)
  for (int q = tid; q < HW; q += nt) {
    const int w = cidx[q];
    d.cell_pt[base + q] = w;
    if (w < 0) {
      d.range[base + q] = FLT_MAX;
      d.full[base + q] = make_float4(qnan, qnan, qnan, 0.0f);
    }
  }
  __syncthreads();
  if (c.dbg_phase <= 1) return;
  // the column ground test on the winners' points (w == 0: empty, or the point of cell (0, 0))
  const float4* full = d.full + base;
  auto cellf = [&](int q) {
    const float4 p = full[q];
    return make_float4(p.x, p.y, p.z, (cidx[q] < 0 || q == 0) ? 0.0f : 1.0f);
  };
  for (int j = tid; j < c.W; j += 2 * nt) ground_columns2(c, cellf, d.ground + base, j, j + nt);
}

// ---------------------------------------------------------------------------------------------
// K3 ADD (IP:631-671): per row, a forward then a backward recurrence "2 -> 1 if a ground cell
// sits one or two columns behind and the step is short". The state before column j is the pair
// (g'[j-2]==1, g'[j-1]==1), so each column is a map on 4 states; a wave composes the maps of
// its 64 lane-chunks with a shuffle scan and replays each chunk from its exact incoming state.
// Bit-identical to the serial loop. One wave per row. grid (ceil(H/4), B), block 256.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t st_apply(uint32_t f, uint32_t s) { return (f >> (2 * s)) & 3u; }
__device__ __forceinline__ uint32_t st_compose(uint32_t g, uint32_t f) {  // g after f
  uint32_t h = 0;
#pragma unroll
  for (uint32_t s = 0; s < 4; ++s) h |= st_apply(g, st_apply(f, s)) << (2 * s);
  return h;
}
// map of one column: s=(a|b<<1) -> (b | c<<1), c = one || (cand && (a||b))
__device__ __forceinline__ uint32_t st_column(bool one, bool cand) {
  uint32_t f = 0;
#pragma unroll
  for (uint32_t s = 0; s < 4; ++s) {
    const uint32_t a = s & 1u, bb = s >> 1;
    const uint32_t cc = one ? 1u : (cand && (a | bb)) ? 1u : 0u;
    f |= (bb | (cc << 1)) << (2 * s);
  }
  return f;
}

// st_compose(st_column(one, cand), F) on the packed table directly: every 2-bit entry v = (a | b<<1)
// becomes b | c<<1, c = one || (cand && (a || b)) — four bit operations instead of the generic loop.
__device__ __forceinline__ uint32_t st_push(uint32_t F, bool one, bool cand) {
  const uint32_t lo = (F >> 1) & 0x55u;
  const uint32_t hi = one ? 0xAAu : cand ? (((F | (F >> 1)) & 0x55u) << 1) : 0u;
  return lo | hi;
}

__device__ __forceinline__ bool add_test(const float4* __restrict__ full, int cell, int nb) {
  const float4 p = full[cell], q = full[nb];
  const float r = sqrt_(p.x * p.x + p.y * p.y + p.z * p.z);
  const float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
  const float dr = sqrt_(dx * dx + dy * dy + dz * dz);
  return (double)dr <= 0.061 * (double)r && (double)dz <= 0.1;
}

// 8 waves per SIMD (45 VGPRs, no spills): 0.190 -> 0.154 ms per 1024 VLP-16 scans; the same bound
// on k_segment / k_ground_elev_ransac spills and was slower
__global__ __launch_bounds__(256, 8) void k_ground_add(DevCfg c, DevBufs d) {
  __shared__ int8_t grow[4][2048];
  const int b = blockIdx.y;
  const int wv = threadIdx.x >> 6, l = lane_id();
  const int i = blockIdx.x * 4 + wv;
  if (i >= c.H) return;
  const int W = c.W;
  const size_t rbase = (size_t)b * c.HW + (size_t)i * W;
  int8_t* g = grow[wv];
  for (int j = l; j < W; j += 64) g[j] = d.ground[rbase + j];
  __builtin_amdgcn_wave_barrier();
  const float4* full = d.full + rbase;
  const int CH = (W + 63) / 64;
  const uint32_t kId = 0xE4u;  // identity map on 4 states

  // ---- forward pass, j = 2 .. W-1 ----
  {
    const int j0 = l * CH, j1 = min(j0 + CH, W);
    uint32_t F = kId;
    uint64_t candBits = 0;  // CH <= 64
    for (int j = j0; j < j1; ++j) {
      if (j < 2) continue;
      const bool two = g[j] == 2;
      const bool cand = two && add_test(full, j, j - 2);
      if (cand) candBits |= 1ull << (j - j0);
      F = st_push(F, g[j] == 1, cand);
    }
    // exclusive scan of maps over lanes (lane order = column order)
    uint32_t incl = F;
#pragma unroll
    for (int dlt = 1; dlt < 64; dlt <<= 1) {
      const uint32_t y = __shfl_up(incl, dlt, 64);
      if (l >= dlt) incl = st_compose(incl, y);
    }
    uint32_t excl = __shfl_up(incl, 1, 64);
    if (l == 0) excl = kId;
    const uint32_t s0 = (g[0] == 1 ? 1u : 0u) | (g[1] == 1 ? 2u : 0u);
    uint32_t s = st_apply(excl, s0);
    __builtin_amdgcn_wave_barrier();
    for (int j = j0; j < j1; ++j) {
      if (j < 2) continue;
      const bool cand = (candBits >> (j - j0)) & 1ull;
      const uint32_t a = s & 1u, bb = s >> 1;
      bool one = g[j] == 1;
      if (cand && (a | bb)) { g[j] = 1; one = true; }
      s = bb | ((one ? 1u : 0u) << 1);
    }
  }
  __builtin_amdgcn_wave_barrier();
  // ---- backward pass, j = W-3 .. 0, neighbours j+1, j+2 ----
  {
    // lane l owns the l-th chunk counted from the right end.
    const int hi = W - 3;  // first column visited
    const int j1 = hi - l * CH, j0 = max(j1 - CH + 1, 0);  // chunk [j0, j1], visited descending
    uint32_t F = kId;
    uint64_t candBits = 0;
    for (int j = j1; j >= j0; --j) {
      const bool two = g[j] == 2;
      const bool cand = two && add_test(full, j, j + 2);
      if (cand) candBits |= 1ull << (j1 - j);
      F = st_push(F, g[j] == 1, cand);
    }
    uint32_t incl = F;
#pragma unroll
    for (int dlt = 1; dlt < 64; dlt <<= 1) {
      const uint32_t y = __shfl_up(incl, dlt, 64);
      if (l >= dlt) incl = st_compose(incl, y);
    }
    uint32_t excl = __shfl_up(incl, 1, 64);
    if (l == 0) excl = kId;
    const uint32_t s0 = (g[W - 1] == 1 ? 1u : 0u) | (g[W - 2] == 1 ? 2u : 0u);
    uint32_t s = st_apply(excl, s0);
    __builtin_amdgcn_wave_barrier();
    for (int j = j1; j >= j0; --j) {
      const bool cand = (candBits >> (j1 - j)) & 1ull;
      const uint32_t a = s & 1u, bb = s >> 1;
      bool one = g[j] == 1;
      if (cand && (a | bb)) { g[j] = 1; one = true; }
      s = bb | ((one ? 1u : 0u) << 1);
    }
  }
  __builtin_amdgcn_wave_barrier();
  for (int j = l; j < W; j += 64) d.ground[rbase + j] = g[j];
}

// ---------------------------------------------------------------------------------------------
// Device mt19937 (== boost::mt19937 / std::mt19937) for PCL's SampleConsensusModel RNG.
// ---------------------------------------------------------------------------------------------
struct MT {
  uint32_t mt[624];
  int idx;
};
__device__ uint32_t mt_next(MT& m) {
  if (m.idx >= 624) {
    for (int k = 0; k < 624; ++k) {
      const uint32_t y = (m.mt[k] & 0x80000000u) | (m.mt[(k + 1) % 624] & 0x7fffffffu);
      m.mt[k] = m.mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    m.idx = 0;
  }
  uint32_t y = m.mt[m.idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

__device__ __forceinline__ float ransac_dist(const float cf[4], float4 q) {
  // Eigen SSE dot of 4 floats: (c0 p0 + c2 p2) + (c1 p1 + c3 * 1)
  return fabs_((cf[0] * q.x + cf[2] * q.z) + (cf[1] * q.y + cf[3] * 1.0f));
}

// ---------------------------------------------------------------------------------------------
// K4 ELEVATION + NEAR + RANSAC + final ground (IP:673-735). One workgroup (512 or 1024 threads) per
// scan: a last-valid carry scan over columns, a row-major compaction of near-ground cells, and
// PCL 1.10's RandomSampleConsensus driven by lane 0 with inlier counting spread over the block.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_ground_elev_ransac(DevCfg c, DevBufs d) {
  __shared__ float colz[2048];
  __shared__ int colok[2048];
  __shared__ uint64_t colm2[2048];  // per column: rows with ground == 2 (H <= 64)
  __shared__ int tmp[32];
  __shared__ MT rng;
  __shared__ int sh_int[8];
  __shared__ float sh_cf[4], best_cf[4];
  const int b = blockIdx.x;
  const int W = c.W, H = c.H, HW = c.HW;
  const size_t base = (size_t)b * HW;
  int8_t* g = d.ground + base;
  const float4* full = d.full + base;
  const int tid = threadIdx.x, nt = blockDim.x;

  // ---- ELEVATION: per-column ground count and top ground z (IP:676-687) ----
  // The column's ground bytes are loaded 16 rows at a time (all in flight), reduced to bit masks;
  // only the top ground cell's z is fetched, and the cells == 2 are remembered for the Filter pass.
  for (int j = tid; j < W; j += nt) {
    uint64_t m1 = 0ull, m2 = 0ull;
    for (int i0 = 0; i0 < H; i0 += 16) {
      int8_t gv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) gv[u] = i0 + u < H ? g[j + (i0 + u) * W] : (int8_t)0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        m1 |= (uint64_t)(gv[u] == 1) << (i0 + u);
        m2 |= (uint64_t)(gv[u] == 2) << (i0 + u);
      }
    }
    const int cnt = __popcll(m1);
    colz[j] = m1 ? full[j + (63 - __clzll((long long)m1)) * W].z : 0.0f;
    colok[j] = cnt >= 5 ? j : -1;
    colm2[j] = m2;
  }
  __syncthreads();
  // last-valid carry across columns: max-scan of colok (block-sequential chunks of 2)
  {
    const int per = (W + nt - 1) / nt;
    const int j0 = tid * per, j1 = min(j0 + per, W);
    int last = -1;
    for (int j = j0; j < j1; ++j) last = colok[j] > last ? colok[j] : last;
    // inclusive max-scan over threads
    const int l = lane_id(), w = tid >> 6;
    int x = last;
    for (int dl = 1; dl < 64; dl <<= 1) {
      int y = __shfl_up(x, dl, 64);
      if (l >= dl) x = y > x ? y : x;
    }
    if (l == 63) tmp[w] = x;
    __syncthreads();
    int pre = -1;
    for (int k = 0; k < w; ++k) pre = tmp[k] > pre ? tmp[k] : pre;
    int ex = __shfl_up(x, 1, 64);
    if (l == 0) ex = -1;
    int run = ex > pre ? ex : pre;
    __syncthreads();
    for (int j = j0; j < j1; ++j) {
      run = colok[j] > run ? colok[j] : run;
      colok[j] = run;  // index of the carried column, -1 = initial -1.3
    }
  }
  __syncthreads();
  for (int j = tid; j < W; j += nt) {
    const float EH = colok[j] >= 0 ? colz[colok[j]] : -1.3f;
    const uint64_t m2 = colm2[j];
    for (int i0 = 0; i0 < H && (m2 >> i0); i0 += 16) {
      float z[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) z[u] = (m2 >> (i0 + u)) & 1ull ? full[j + (i0 + u) * W].z : 0.0f;
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if ((m2 >> (i0 + u)) & 1ull) g[j + (i0 + u) * W] = ((double)z[u] < (double)EH + 0.3) ? 1 : 0;
    }
  }
  __syncthreads();

  if (c.dbg_phase <= 0) return;
  // ---- NEAR (IP:701-715): row-major compaction, intensity = linear index ----
  // Cells interleaved across lanes per slot (t0 + u * blockDim + tid): loads and the compacted
  // stores of a wave are contiguous; row-major positions from per-(slot, wave) ballot counts.
  float4* nearp = d.near_pts + base;
  int K = 0;
  constexpr int kC = 4;
  __shared__ int ncnt[2][kC * 16 + 1];
  const int nw = nt >> 6, wv = tid >> 6, ln = lane_id();
  int par = 0;
  // the next tile's ground flags are loaded before this tile's barriers (one load latency per tile
  // instead of two: the points' loads depend on the flags)
  int8_t gn[kC];
#pragma unroll
  for (int u = 0; u < kC; ++u) gn[u] = u * nt + tid < HW ? g[u * nt + tid] : (int8_t)0;
  for (int t0 = 0; t0 < HW; t0 += kC * nt, par ^= 1) {
    int8_t gv[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) gv[u] = gn[u];
    float4 p[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) p[u] = gv[u] == 1 ? full[t0 + u * nt + tid] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int cell = t0 + kC * nt + u * nt + tid;
      gn[u] = cell < HW ? g[cell] : (int8_t)0;
    }
    bool nearc[kC];
    float depth[kC];
    unsigned long long mN[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      depth[u] = sqrt_(p[u].x * p[u].x + p[u].y * p[u].y);
      nearc[u] = gv[u] == 1 && (double)depth[u] <= 10;
      mN[u] = __ballot(nearc[u]);
      if (ln == 0) ncnt[par][u * nw + wv] = (int)__popcll(mN[u]);
    }
    __syncthreads();
    if (wv == 0) {
      const int v = ln < kC * nw ? ncnt[par][ln] : 0;
      const int incl = wave_incl_scan_add(v);
      if (ln < kC * nw) ncnt[par][ln] = incl - v;
      if (ln == 63) ncnt[par][kC * 16] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      if (!nearc[u]) continue;
      const int cell = t0 + u * nt + tid;
      const int pos = K + ncnt[par][u * nw + wv] + (int)__popcll(mN[u] & ((1ull << ln) - 1ull));
      nearp[pos] = make_float4(p[u].x, p[u].y, p[u].z, (float)cell);
      if ((double)depth[u] <= 5) g[cell] = 0;
    }
    K += ncnt[par][kC * 16];
  }
  int* shuf = d.shuf + base;
  for (int k = tid; k < K; k += nt) shuf[k] = k;
  __syncthreads();
  if (c.dbg_phase <= 1) return;

  // ---- RANSAC (PCL 1.10 RandomSampleConsensus::computeModel, threshold 0.5) ----
  // sh_int: 0 stop, 1 valid-model, 2 iterations, 3 best count, 4 skipped, 5 have-best
  __shared__ double kk;
  for (int k = tid; k < 624; k += nt) rng.mt[k] = d.mt0[k];  // seeded and twisted on the host
  if (tid == 0) {
    rng.idx = 0;
    sh_int[0] = K < 3 ? 1 : 0;
    sh_int[2] = K < 3 ? INT_MAX - 1 : 0;
    sh_int[3] = -INT_MAX;
    sh_int[4] = 0;
    sh_int[5] = 0;
    kk = 1.0;
  }
  __syncthreads();
  const double log_probability = log(1.0 - 0.99);
  const double one_over = K > 0 ? 1.0 / (double)K : 0.0;
  while (true) {
    if (tid == 0) {
      sh_int[1] = 0;
      if (!(sh_int[0] == 0 && sh_int[2] < kk && sh_int[4] < 100000)) {
        sh_int[0] = 1;
      } else {
        bool ok = false;
        for (int tries = 0; tries < 1000 && !ok; ++tries) {
          for (int q = 0; q < 3; ++q) {
            const int r = (int)(mt_next(rng) >> 1);
            const int sw = q + (int)((unsigned)r % (unsigned)(K - q));
            const int t = shuf[q]; shuf[q] = shuf[sw]; shuf[sw] = t;
          }
          const float4 p0 = nearp[shuf[0]], p1 = nearp[shuf[1]], p2 = nearp[shuf[2]];
          const float r0 = (p1.x - p0.x) / (p2.x - p0.x), r1 = (p1.y - p0.y) / (p2.y - p0.y),
                      r2 = (p1.z - p0.z) / (p2.z - p0.z);
          ok = (r0 != r1) || (r2 != r1);
        }
        if (!ok) {
          sh_int[0] = 1;
        } else {
          const float4 p0 = nearp[shuf[0]], p1 = nearp[shuf[1]], p2 = nearp[shuf[2]];
          const float a0 = p1.x - p0.x, a1 = p1.y - p0.y, a2 = p1.z - p0.z;
          const float b0 = p2.x - p0.x, b1 = p2.y - p0.y, b2 = p2.z - p0.z;
          const float r0 = a0 / b0, r1 = a1 / b1, r2 = a2 / b2;
          if (r0 == r1 && r2 == r1) {
            sh_int[4] += 1;
          } else {
            float cf[4];
            cf[0] = a1 * b2 - a2 * b1;
            cf[1] = a2 * b0 - a0 * b2;
            cf[2] = a0 * b1 - a1 * b0;
            cf[3] = 0.0f;
            const float sq = (cf[0] * cf[0] + cf[2] * cf[2]) + (cf[1] * cf[1] + cf[3] * cf[3]);
            if (sq > 0.0f) {
              const float nrm = sqrt_(sq);
              for (int q = 0; q < 4; ++q) cf[q] = cf[q] / nrm;
            }
            cf[3] = -1.0f * ((cf[0] * p0.x + cf[2] * p0.z) + (cf[1] * p0.y + cf[3] * 1.0f));
            for (int q = 0; q < 4; ++q) sh_cf[q] = cf[q];
            sh_int[1] = 1;
          }
        }
      }
    }
    __syncthreads();
    if (sh_int[0]) break;
    if (!sh_int[1]) continue;
    float cf[4] = {sh_cf[0], sh_cf[1], sh_cf[2], sh_cf[3]};
    int cnt = 0;
    for (int k = tid; k < K; k += nt)
      if ((double)ransac_dist(cf, nearp[k]) < 0.5) ++cnt;
    cnt = block_reduce_add(cnt, tmp);
    if (tid == 0) {
      if (cnt > sh_int[3]) {
        sh_int[3] = cnt;
        for (int q = 0; q < 4; ++q) best_cf[q] = cf[q];
        sh_int[5] = 1;
        const double w = (double)cnt * one_over;
        double p_no = 1.0 - pow(w, 3.0);
        p_no = fmax(2.220446049250313e-16, p_no);
        p_no = fmin(1.0 - 2.220446049250313e-16, p_no);
        kk = log_probability / log(p_no);
      }
      sh_int[2] += 1;
      if (sh_int[2] > 10000) sh_int[0] = 1;
    }
    __syncthreads();
  }
  if (c.dbg_phase <= 2) return;
  // ---- inliers with depth <= 5 become ground again (IP:727-735) ----
  int ninl = 0;
  if (sh_int[5]) {
    const float cf[4] = {best_cf[0], best_cf[1], best_cf[2], best_cf[3]};
    constexpr int kF = 4;  // points per lane with their loads in flight together
    for (int k0 = 0; k0 < K; k0 += kF * nt) {
      float4 q[kF];
#pragma unroll
      for (int u = 0; u < kF; ++u) {
        const int k = k0 + u * nt + tid;
        q[u] = k < K ? nearp[k] : make_float4(0.f, 0.f, 0.f, -1.f);
      }
#pragma unroll
      for (int u = 0; u < kF; ++u) {
        if (q[u].w < 0.0f || !((double)ransac_dist(cf, q[u]) < 0.5)) continue;
        ++ninl;
        const int cell = (int)q[u].w;
        const float depth = sqrt_(q[u].x * q[u].x + q[u].y * q[u].y);  // the near cloud holds the cell's x, y, z
        if ((double)depth <= 5) g[cell] = 1;
      }
    }
  }
  ninl = block_reduce_add(ninl, tmp);
  if (tid == 0) {
    int* cnt = d.counts + b * kCnt;
    cnt[C_K] = K;
    cnt[C_INL] = ninl;
    cnt[C_RIT] = sh_int[2];
  }
}

// ---------------------------------------------------------------------------------------------
// K5 cloudSegmentation labelling (IP:783-789 driving labelComponents IP:847-931).
// The BFS edge test is symmetric, so each BFS visits exactly one connected component of the
// label-0 cells (4-neighbourhood, columns wrap, rows do not), seeded at its smallest linear
// index. We compute components with a lock-free union-find (link to the smaller root, so the
// root is that seed), then size and the row set of the non-seed members (lineCountFlag is set
// only for pushed cells, IP:904), feasibility (IP:912-922), and label = 1 + rank of the seed
// among feasible components in row-major order; infeasible -> 999999. One workgroup per scan.
// LDS mode (VLP-16 size): parent array in LDS; else global scratch with workgroup-scope atomics.
// ---------------------------------------------------------------------------------------------
template <class Acc>
__device__ __forceinline__ int uf_find(Acc& P, int x) {
  while (true) {
    const int p = P.ld(x);
    if (p == x) return x;
    const int gp = P.ld(p);
    if (gp == p) return p;
    P.st(x, gp);  // path halving; benign race (values only move toward the root)
    x = gp;
  }
}
template <class Acc>
__device__ __forceinline__ void uf_unite(Acc& P, int a, int b) {
  while (true) {
    a = uf_find(P, a);
    b = uf_find(P, b);
    if (a == b) return;
    if (a > b) { const int t = a; a = b; b = t; }
    const int old = P.cas(b, b, a);  // hook larger root under smaller
    if (old == b) return;
    b = old;
  }
}
struct LdsAcc {
  int* p;
  __device__ int ld(int i) { return __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
  __device__ void st(int i, int v) { __hip_atomic_store(p + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
  __device__ int cas(int i, int e, int v) {
    __hip_atomic_compare_exchange_strong(p + i, &e, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return e;
  }
};

__device__ __forceinline__ bool seg_edge(const DevCfg& c, float ra, float rb, bool horiz) {
  const float d1 = ra < rb ? rb : ra;  // std::max(a, b) = (a < b) ? b : a
  const float d2 = rb < ra ? rb : ra;  // std::min(a, b) = (b < a) ? b : a
  const float sA = horiz ? c.sinX : c.sinY, cA = horiz ? c.cosX : c.cosY;
  const float tang = d2 * sA / (d1 - d2 * cA);
  return tang > c.segThr;
}

template <bool kLds>
__global__ __launch_bounds__(1024) void k_label(DevCfg c, DevBufs d) {
  extern __shared__ int lds_parent[];
  __shared__ int tmp[32];
  const int b = blockIdx.x;
  const int W = c.W, H = c.H, HW = c.HW;
  const size_t base = (size_t)b * HW;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int8_t* g = d.ground + base;
  const float* rng = d.range + base;
  int* lab = d.label + base;
  LdsAcc P{kLds ? lds_parent : d.ccl_a + base};

  if constexpr (kLds) {
    // label_mat init (IP:752-759): -1 for ground or empty, else 0 -> union-find singleton; and the
    // BFS edge test of every cell with its right (wrapping, IP:884-886) and lower neighbour as two
    // bits in LDS (ebits, after the parent words), from ranges loaded kE cells per lane at once —
    // the union pass then reads LDS only (its global loads sat behind data-dependent branches)
    uint8_t* ebits = reinterpret_cast<uint8_t*>(lds_parent + HW);
    constexpr int kE = 4;
    for (int t0 = 0; t0 < HW; t0 += kE * nt) {
      float r[kE], rr[kE], rd[kE];
      int8_t gv[kE];
#pragma unroll
      for (int u = 0; u < kE; ++u) {
        const int cell = t0 + u * nt + tid;
        if (cell >= HW) continue;
        const int i = cell / W, j = cell - i * W;
        gv[u] = g[cell];
        r[u] = rng[cell];
        rr[u] = rng[(j + 1 < W) ? cell + 1 : cell + 1 - W];
        rd[u] = i + 1 < H ? rng[cell + W] : FLT_MAX;
      }
      // A wave holds 64 consecutive cells of slot u: the right edges between neighbours of one row
      // inside the wave are resolved here, each cell pointing straight at the first cell of its
      // linked run (the run's smallest index, so the union-find invariant "root = smallest cell"
      // holds); only the wave's last right edge, the row wrap and the down edges are left for the
      // union pass.
      const int ln = lane_id();
#pragma unroll
      for (int u = 0; u < kE; ++u) {
        const int cell = t0 + u * nt + tid;
        const bool in = cell < HW;
        const int i = in ? cell / W : 0, j = in ? cell - i * W : 0;
        const bool l0 = in && !(gv[u] == 1 || r[u] == FLT_MAX);
        const bool er = in && seg_edge(c, r[u], rr[u], true);
        const bool ed = in && i + 1 < H && seg_edge(c, r[u], rd[u], false);
        const bool l0n = __shfl_down(l0 ? 1 : 0, 1, 64) != 0;  // the next lane's cell (j + 1 if j + 1 < W)
        const bool link = er && l0 && l0n && ln < 63 && j + 1 < W;  // resolved in the wave
        const unsigned long long lk = __ballot(link);
        const unsigned long long heads = ~(lk << 1);                 // lane 0 always starts a run
        const int head = 63 - __clzll((long long)(heads & ((2ull << ln) - 1ull)));
        if (!in) continue;
        P.st(cell, l0 ? cell - (ln - head) : -1);
        ebits[cell] = (uint8_t)((er && !link ? 1 : 0) | (ed ? 2 : 0));
      }
    }
    __syncthreads();
    if (c.dbg_phase <= 0) return;
    for (int cell = tid; cell < HW; cell += nt) {
      const int e = ebits[cell];
      if (e == 0 || P.ld(cell) < 0) continue;
      const int i = cell / W, j = cell - i * W;
      const int right = (j + 1 < W) ? cell + 1 : cell + 1 - W;  // wrap (IP:884-886)
      if ((e & 1) && P.ld(right) >= 0) uf_unite(P, cell, right);
      if ((e & 2) && P.ld(cell + W) >= 0) uf_unite(P, cell, cell + W);
    }
    __syncthreads();
  } else {
    // H*W does not fit LDS: bands of lbl_band rows are united in LDS (local indices, link to the
    // smaller root, so a band root is its band component's smallest cell), their roots written to
    // the global parent array (every cell -> its band root), then only the down edges across band
    // boundaries are united there. Same components, same roots (the smallest cell) as one
    // union-find over the whole image; the global atomics touch ~H / lbl_band rows instead of all.
    const int R = c.lbl_band;
    LdsAcc L{lds_parent};
    for (int r0 = 0; r0 < H; r0 += R) {
      const int r1 = r0 + R < H ? r0 + R : H;
      const int c0 = r0 * W, nb = (r1 - r0) * W;
      for (int q = tid; q < nb; q += nt) {
        const int cell = c0 + q;
        const bool l0 = !(g[cell] == 1 || rng[cell] == FLT_MAX);
        L.st(q, l0 ? q : -1);
      }
      __syncthreads();
      for (int q = tid; q < nb; q += nt) {
        if (L.ld(q) < 0) continue;
        const int cell = c0 + q;
        const int i = cell / W, j = cell - i * W;
        const float r = rng[cell];
        const int rq = (j + 1 < W) ? q + 1 : q + 1 - W;  // wrap (IP:884-886)
        if (L.ld(rq) >= 0 && seg_edge(c, r, rng[c0 + rq], true)) uf_unite(L, q, rq);
        if (i + 1 < r1) {
          const int dq = q + W;
          if (L.ld(dq) >= 0 && seg_edge(c, r, rng[c0 + dq], false)) uf_unite(L, q, dq);
        }
      }
      __syncthreads();
      // walks (the band is final); a member's word becomes its root (a concurrent walk reading it
      // still sees an ancestor; roots are never written here)
      for (int q = tid; q < nb; q += nt) {
        int x = L.ld(q);
        if (x >= 0) {
          for (int px = L.ld(x); px != x; px = L.ld(x)) x = px;
          if (x != q) L.st(q, x);
        }
        P.st(c0 + q, x < 0 ? -1 : c0 + x);
      }
      __syncthreads();
      // Band component stats in the band root's LDS word, as in the LDS path: 0x80000000 |
      // size << 16 | rows (bit i - r0, lbl_band <= 16) of its non-root members
      for (int q = tid; q < nb; q += nt)
        if (L.ld(q) == q) L.st(q, (int)(0x80000000u | (1u << 16)));
      __syncthreads();
      for (int q = tid; q < nb; q += nt) {
        const int x = L.ld(q);
        if (x < 0) continue;  // not label 0, or a root (stats word)
        atomicAdd(&lds_parent[x], 1 << 16);
        atomicOr(&lds_parent[x], 1 << ((c0 + q) / W - r0));
      }
      __syncthreads();
      // lab: -1 (not label 0), the band root's cell (member) or the band stats (band root)
      for (int q = tid; q < nb; q += nt) {
        const int x = L.ld(q);
        lab[c0 + q] = x >= 0 ? c0 + x : x;
      }
      __syncthreads();
    }
    if (c.dbg_phase <= 0) return;
    for (int r1 = R; r1 < H; r1 += R)
      for (int j = tid; j < W; j += nt) {
        const int a = (r1 - 1) * W + j, bc = r1 * W + j;
        if (P.ld(a) >= 0 && P.ld(bc) >= 0 && seg_edge(c, rng[a], rng[bc], false)) uf_unite(P, a, bc);
      }
    __syncthreads();
  }
  if (c.dbg_phase <= 1) return;
  if constexpr (kLds) {
    // Everything stays in the LDS word of each cell: -1 = not label 0; a member holds its root's
    // index (>= 0); a root holds 0x80000000 | size << 16 | row mask of its pushed members (size <=
    // HW <= 32000 keeps the word != -1), later 0x80000000 | label. Global memory sees the labels once.
    // read-only walks: the only stores are P[cell] = its root, so every word a concurrent walk
    // reads is still an ancestor (path halving here could store a stale grandparent over a root)
    for (int cell = tid; cell < HW; cell += nt) {
      int x = P.ld(cell);
      if (x < 0) continue;
      for (int px = P.ld(x); px != x; px = P.ld(x)) x = px;
      P.st(cell, x);
    }
    __syncthreads();
    if (c.dbg_phase <= 2) return;
    for (int cell = tid; cell < HW; cell += nt)
      if (P.ld(cell) == cell) P.st(cell, (int)(0x80000000u | (1u << 16)));
    __syncthreads();
    for (int cell = tid; cell < HW; cell += nt) {
      const int root = P.ld(cell);
      if (root < 0) continue;
      atomicAdd(&lds_parent[root], 1 << 16);
      atomicOr(&lds_parent[root], 1 << (cell / W));
    }
    __syncthreads();
    if (c.dbg_phase <= 3) return;
    constexpr int kC = 4;
    int rank = 0;
    for (int t0 = 0; t0 < HW; t0 += kC * nt) {
      const int c0 = t0 + kC * tid;
      bool root[kC], feas[kC];
      int nf = 0;
#pragma unroll
      for (int u = 0; u < kC; ++u) {
        const int v = c0 + u < HW ? P.ld(c0 + u) : -1;
        root[u] = v < 0 && v != -1;
        const int size = (int)(((unsigned)v >> 16) & 0x7fffu), lines = __popc((unsigned)v & 0xffffu);
        feas[u] = root[u] && (size >= 30 || (size >= c.pointNum && lines >= c.lineNum));
        nf += feas[u];
      }
      int tot;
      int ex = rank + block_excl_scan(nf, tmp, &tot);  // barriers: all root words read
#pragma unroll
      for (int u = 0; u < kC; ++u)
        if (root[u]) P.st(c0 + u, (int)(0x80000000u | (unsigned)(feas[u] ? ++ex : 999999)));
      rank += tot;
    }
    __syncthreads();
    if (c.dbg_phase <= 4) return;
    for (int cell = tid; cell < HW; cell += nt) {
      const int v = P.ld(cell);
      lab[cell] = v == -1 ? -1 : v < 0 ? (v & 0x7fffffff) : (P.ld(v) & 0x7fffffff);
    }
    return;
  }
  // Global mode: component stats from the band components. A band root whose global root is
  // itself is a component seed: it takes its band's stats with plain stores (lab = 0x80000000 |
  // size, rows in ccl_b); the other band roots (components crossing a band boundary) then add
  // theirs, their own row included, with atomics.
  const int R = c.lbl_band;
  unsigned long long* rowA = d.ccl_b + base;
  // the cell sweeps below take kU cells per lane with their loads in flight together (one global
  // load latency per kU cells: nearly every cell only needs its word to be skipped)
  constexpr int kU = 8;
  for (int c0 = 0; c0 < HW; c0 += kU * nt) {
    int v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int cell = c0 + u * nt + tid;
      v[u] = cell < HW ? lab[cell] : -1;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int cell = c0 + u * nt + tid;
      if (v[u] >= -1 || uf_find(P, cell) != cell) continue;  // -1, a member, or a joined band root
      rowA[cell] = (unsigned long long)(v[u] & 0xffff) << ((cell / W) / R * R);
      lab[cell] = (int)(0x80000000u | (((unsigned)v[u] >> 16) & 0x7fffu));
    }
  }
  __syncthreads();
  for (int c0 = 0; c0 < HW; c0 += kU * nt) {
    int v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int cell = c0 + u * nt + tid;
      v[u] = cell < HW ? lab[cell] : -1;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int cell = c0 + u * nt + tid;
      if (v[u] >= -1 || P.ld(cell) == cell) continue;  // only band roots joined to another seed
      const int gr = uf_find(P, cell);
      const int row = cell / W;
      __hip_atomic_fetch_add(&lab[gr], (int)(((unsigned)v[u] >> 16) & 0x7fffu), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_or(&rowA[gr], ((unsigned long long)(v[u] & 0xffff) << (row / R * R)) | (1ull << row),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  __syncthreads();
  // feasibility and rank of feasible seeds in row-major order: tiles of 4 consecutive cells per
  // lane, one block scan of the lane counts per tile; a seed's lab becomes 0x80000000 | label
  constexpr int kC = 4;
  int rank = 0;
  for (int t0 = 0; t0 < HW; t0 += kC * nt) {
    const int c0 = t0 + kC * tid;
    bool root[kC], feas[kC];
    int nf = 0;
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int cell = c0 + u;
      root[u] = cell < HW && P.ld(cell) == cell;
      feas[u] = false;
      if (root[u]) {
        const int size = lab[cell] & 0x7fffffff, lines = __popcll(rowA[cell]);
        feas[u] = size >= 30 || (size >= c.pointNum && lines >= c.lineNum);
      }
      nf += feas[u];
    }
    int tot;
    int ex = rank + block_excl_scan(nf, tmp, &tot);  // barriers: all stat reads done
#pragma unroll
    for (int u = 0; u < kC; ++u)
      if (root[u]) lab[c0 + u] = (int)(0x80000000u | (unsigned)(feas[u] ? ++ex : 999999));
    rank += tot;
  }
  __syncthreads();
  // every label-0 cell takes its seed's label (a seed's own word may already hold the final value:
  // both forms read the same through the mask)
  for (int c0 = 0; c0 < HW; c0 += kU * nt) {
    int v[kU], gr[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int cell = c0 + u * nt + tid;
      v[u] = cell < HW ? lab[cell] : -1;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int cell = c0 + u * nt + tid;
      gr[u] = v[u] == -1 ? -1 : uf_find(P, v[u] >= 0 ? v[u] : cell);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int cell = c0 + u * nt + tid;
      if (gr[u] >= 0)
        lab[cell] = __hip_atomic_load(&lab[gr[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & 0x7fffffff;
    }
  }
}

template __global__ void k_label<true>(DevCfg, DevBufs);
template __global__ void k_label<false>(DevCfg, DevBufs);

// halfPassed's exact test, out of line: the rare undecided points of k_segment's first tile (inlined,
// the libm code's registers would spill k_segment's SGPRs)
__device__ __attribute__((noinline)) bool half_passed_exact(float y, float x, float start) {
  return half_passed(-atan2f_(y, x), start);
}

// Diagnostics (llsr_debug_half_passed): per (y, x, start) triple the fast test's code (0 / 1 / 2 =
// fails / passes / undecided), half_passed_any and the exact test
__global__ void k_debug_half_passed(const float* yxs, int n, uint8_t* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float y = yxs[3 * t], x = yxs[3 * t + 1], st = yxs[3 * t + 2];
  out[3 * t] = (uint8_t)half_passed_fast(y, x, st);
  out[3 * t + 1] = half_passed_any(y, x, st) ? 1 : 0;
  out[3 * t + 2] = half_passed_exact(y, x, st) ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------
// K6 segmented / outlier extraction (IP:791-832) + findStartEndAngle (IP:430-445).
// Row-major block compaction; ring start/end indices fall out of the running count at each
// row boundary. One workgroup per scan.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_segment(DevCfg c, const float4* __restrict__ pts,
                                                  const int64_t* __restrict__ off, DevBufs d) {
  const int b = blockIdx.x;
  const int W = c.W, H = c.H, HW = c.HW;
  const size_t base = (size_t)b * HW;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int8_t* g = d.ground + base;
  const int* lab = d.label + base;
  int* cnt = d.counts + b * kCnt;
  __shared__ float s_start;
  __shared__ int s_half;  // adjustDistortion's halfPassed latch among the first tile's segmented points
  constexpr int kUnd = 64;
  __shared__ float4 s_und[kUnd];  // points the fast halfPassed test left undecided: x, y, -, index
  __shared__ int s_nund;
  if (tid == 0) {
    s_half = INT_MAX;
    s_nund = 0;
    float o0 = 0.f, o1 = 0.f, o2 = 0.f;
    if (cnt[C_NPTS] > 0) {
      const float4 a = pts[off[b] + cnt[C_FIRST]], e = pts[off[b] + cnt[C_LAST]];
      o0 = -atan2f_(a.y, a.x);
      o1 = (float)(-atan2f_(e.y, e.x) + 2 * kPi);
      if (o1 - o0 > 3 * kPi) o1 = (float)(o1 - 2 * kPi);
      else if (o1 - o0 < kPi) o1 = (float)(o1 + 2 * kPi);
      o2 = o1 - o0;
    }
    d.orient[b * 4 + 0] = o0;
    d.orient[b * 4 + 1] = o1;
    d.orient[b * 4 + 2] = o2;
    s_start = o0;
  }
  // 0 = skip, 1 = segmented, 2 = outlier
  auto kind = [&](int cell, int L, int8_t gv) -> int {
    const int i = cell / W, j = cell - i * W;
    if (!(L > 0 || gv == 1)) return 0;
    if (L == 999999) return (i > c.gsi && j % 5 == 0) ? 2 : 0;
    if (gv == 1 && (j % 5 != 0 && j > 5 && j < W - 5)) return 0;
    return 1;
  };
  // Row-major compaction in tiles of 4 * blockDim cells, cell t0 + u * blockDim + tid in slot u of
  // a lane, so every load and every output store of one slot is contiguous across the wave (the
  // kept cells of a wave land in consecutive output positions). Offsets: per (slot, wave) ballot
  // counts, one scan of those <= 64 words in (slot, wave) = row-major order. The label / ground
  // loads of the next tile are issued before this tile's scan.
  constexpr int kC = 4;
  __shared__ int wcnt[2][kC * 16 + 1];  // packed segmented | outlier << 16 counts, double-buffered
  const int nw = nt >> 6, wv = tid >> 6, l = lane_id();
  const unsigned long long lt = (1ull << l) - 1ull;
  int baseS = 0, baseO = 0;
  int labn[kC];
  int8_t gn[kC];
  auto load_kind = [&](int t0) {
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int cell = t0 + u * nt + tid;
      labn[u] = cell < HW ? lab[cell] : 0;
      gn[u] = cell < HW ? g[cell] : (int8_t)0;
    }
  };
  load_kind(0);
  int par = 0;
  for (int t0 = 0; t0 < HW; t0 += kC * nt, par ^= 1) {
    int kk[kC];
    int8_t gc[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int cell = t0 + u * nt + tid;
      gc[u] = gn[u];
      kk[u] = cell < HW ? kind(cell, labn[u], gn[u]) : 0;
    }
    float4 f[kC];
    float rg[kC], vs[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      if (kk[u] == 0) continue;
      const int cell = t0 + u * nt + tid;
      const size_t q = base + cell;
      const float4 p = d.full[q];
      const int ci = cell / W;
      f[u] = make_float4(p.x, p.y, p.z, cell_intensity(H, W, ci, cell - ci * W));
      vs[u] = p.w;
      rg[u] = kk[u] == 1 ? d.range[q] : 0.0f;
    }
    if (t0 + kC * nt < HW) load_kind(t0 + kC * nt);
    unsigned long long mS[kC], mO[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      mS[u] = __ballot(kk[u] == 1);
      mO[u] = __ballot(kk[u] == 2);
      if (l == 0) wcnt[par][u * nw + wv] = (int)__popcll(mS[u]) | ((int)__popcll(mO[u]) << 16);
    }
    __syncthreads();
    if (wv == 0) {
      const int v = l < kC * nw ? wcnt[par][l] : 0;
      const int incl = wave_incl_scan_add(v);
      if (l < kC * nw) wcnt[par][l] = incl - v;
      if (l == 63) wcnt[par][kC * 16] = incl;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int cell = t0 + u * nt + tid;
      if (cell >= HW) break;
      const int ex = wcnt[par][u * nw + wv];
      const int ps = baseS + (ex & 0xffff) + (int)__popcll(mS[u] & lt);
      const int po = baseO + (ex >> 16) + (int)__popcll(mO[u] & lt);
      const int i = cell / W, j = cell - i * W;
      if (j == 0) {
        d.start_ring[b * H + i] = ps - 1 + 5;
        if (i > 0) d.end_ring[b * H + i - 1] = ps - 1 - 5;
      }
      if (kk[u] == 1) {
        // halfPassed (FA:584): the latch is the smallest passing index, and the first tile holds
        // the smallest indices (row 0: half a turn in, normally); k_fa_points searches otherwise
        // (ps grows with the lane within a slot: the wave's first passing lane holds its minimum)
        // (undecided lanes, rare, queue for the exact test after the loop)
        if (t0 == 0) {
          const int hp = half_passed_fast(f[u].y, f[u].x, s_start);
          const unsigned long long mp = ballot(hp == 1);
          if (mp && l == __builtin_ctzll(mp)) atomicMin(&s_half, ps);
          if (hp == 2) {
            const int k = atomicAdd(&s_nund, 1);
            if (k < kUnd) s_und[k] = make_float4(f[u].x, f[u].y, 0.0f, __int_as_float(ps));
          }
        }
        d.seg[base + ps] = f[u];
        d.seg_ground[base + ps] = gc[u] == 1;
        d.seg_col[base + ps] = (uint32_t)j;
        d.seg_range[base + ps] = rg[u];
        d.seg_int[base + ps] = vs[u];
      } else if (kk[u] == 2) {
        d.outl[base + po] = f[u];
        d.outl_int[base + po] = vs[u];
      }
    }
    const int tot = wcnt[par][kC * 16];
    baseS += tot & 0xffff;
    baseO += tot >> 16;
  }
  const int S = baseS, O = baseO;
  __syncthreads();
  const int nund = s_nund;
  if (nund > 0 && nund <= kUnd && tid < nund) {
    const float4 q = s_und[tid];
    if (half_passed_exact(q.y, q.x, s_start)) atomicMin(&s_half, __float_as_int(q.w));
  }
  __syncthreads();  // s_half final
  if (tid == 0) {  // (more undecided points than the queue holds: k_fa_points searches)
    cnt[C_HALF] = (s_half == INT_MAX || nund > kUnd) ? kHalfUnknown : s_half;
    d.end_ring[b * H + H - 1] = S - 1 - 5;
    cnt[C_S] = S;
    cnt[C_O] = O;
  }
  // CloudInfo arrays are H*W long and zero past S (IP:184-186); FA reads a few past S. They are
  // zero past the slot's previous S already (d.seg_zero), so only [S, previous S) is cleared.
  const int zend = min(d.seg_zero[b], HW);
  __syncthreads();  // every thread read the old bound
  if (tid == 0) d.seg_zero[b] = S;
  for (int k = S + tid; k < zend; k += nt) {
    d.seg_ground[base + k] = 0;
    d.seg_col[base + k] = 0u;
    d.seg_range[base + k] = 0.0f;
  }
}

}  // namespace llsr
