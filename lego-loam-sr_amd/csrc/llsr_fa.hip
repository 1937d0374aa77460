// llsr_fa.hip — FeatureAssociation feature stage on gfx950 (featureAssociation.cpp = FA,
// lines 565-899 and 1159-1387): LOAM-frame swap + relative time, curvature, occlusion masks,
// per-ring greedy edge/flat selection, per-ring VoxelGrid of less-flat points, DBSCAN edge
// refinement. Built with -ffp-contract=off; float order follows the reference exactly.
#include <cfloat>
#include <climits>

#include "llsr_device.h"
#include "llsr_libm.h"

namespace llsr {

using namespace llsr_libm;
constexpr double kPi = 3.14159265358979323846;

// ---------------------------------------------------------------------------------------------
// K7 per-point stage: adjustDistortion (FA:565-598), calculateSmoothnessOurs (FA:817-848),
// markOccludedPoints (FA:851-899). One workgroup (1024 threads) per scan.
// halfPassed is a one-way latch, so the serial loop equals: points up to the first index whose
// first-branch orientation passes start + pi use branch 1, later ones branch 2 (block min).
// Curvature reads an LDS tile of LOAM points with a +-5 halo. Occlusion writes become a gather
// over the +-6 window of per-point flags. FA carry-over arrays (picked, cloudLabel) are per slot.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float ori_branch1(float o, float start) {
  if ((double)o < (double)start - kPi / 2) o = (float)(o + 2 * kPi);
  else if ((double)o > (double)start + kPi * 3 / 2) o = (float)(o - 2 * kPi);
  return o;
}

constexpr int kTile = 1024;

__global__ __launch_bounds__(1024) void k_fa_points(DevCfg c, DevBufs d) {
  __shared__ float4 tp[kTile + 10];
  __shared__ uint8_t fl[kTile + 12];  // bit0 A_i, bit1 B_i, bit2 C_i for i in [t0-6, t0+T+6)
  __shared__ int tmp[32];
  const int b = blockIdx.x;
  const size_t base = (size_t)b * c.HW;
  const int tid = threadIdx.x, nt = blockDim.x;
  int* cnt = d.counts + b * kCnt;
  const int S = cnt[C_S];
  const float start = d.orient[b * 4 + 0], endo = d.orient[b * 4 + 1], diff = d.orient[b * 4 + 2];
  const float4* seg = d.seg + base;
  float4* loam = d.loam + base;

  int first = INT_MAX;
  for (int i = tid; i < S; i += nt) {
    const float4 p = seg[i];
    const float o = ori_branch1(-atan2f_(p.y, p.x), start);
    if ((double)(o - start) > kPi && i < first) first = i;
  }
  first = block_reduce_min(first, tmp);
  for (int i = tid; i < S; i += nt) {
    const float4 p = seg[i];
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
    loam[i] = make_float4(p.y, p.z, p.x, inten);
  }
  if (tid == 0) cnt[C_HALF] = first;
  __syncthreads();

  const float* rng = d.seg_range + base;
  const uint32_t* col = d.seg_col + base;
  uint8_t* picked = d.picked + base;
  int8_t* clabel = d.clabel + base;
  float* curv = d.curv + base;
  for (int t0 = 0; t0 < S; t0 += kTile) {
    for (int q = tid; q < kTile + 10; q += nt) {
      const int k = t0 - 5 + q;
      tp[q] = (k >= 0 && k < S) ? loam[k] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    for (int q = tid; q < kTile + 12; q += nt) {
      const int i = t0 - 6 + q;
      uint8_t f = 0;
      if (i >= 5 && i < S - 6) {
        const float d1 = rng[i], d2 = rng[i + 1];
        const int colDiff = abs((int)(col[i + 1] - col[i]));
        if (colDiff < 10) {
          if ((double)(d1 - d2) > 0.3) f |= 1;
          else if ((double)(d2 - d1) > 0.3) f |= 2;
        }
        const float diff1 = fabs_((float)(rng[i - 1] - rng[i]));
        const float diff2 = fabs_((float)(rng[i + 1] - rng[i]));
        if ((double)diff1 > 0.02 * (double)rng[i] && (double)diff2 > 0.02 * (double)rng[i]) f |= 4;
      }
      fl[q] = f;
    }
    __syncthreads();
    const int k = t0 + tid;
    if (tid < kTile && k < S) {
      const bool inner = k >= 5 && k < S - 5;
      float cv = 0.0f;
      if (inner) {
        const int q = tid + 5;
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
      const int fq = k - t0 + 6;  // fl index of i = k
      if (fl[fq] & 4) occ = true;
#pragma unroll
      for (int m = 0; m <= 5; ++m) occ |= (fl[fq + m] & 1) != 0;   // A_i, i in [k, k+5]
#pragma unroll
      for (int m = 1; m <= 6; ++m) occ |= (fl[fq - m] & 2) != 0;   // B_i, i in [k-6, k-1]
      const uint8_t old = picked[k];
      picked[k] = (inner ? (uint8_t)0 : old) | (occ ? (uint8_t)1 : (uint8_t)0);
      if (inner) clabel[k] = 0;
    }
    __syncthreads();
  }
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

__device__ __forceinline__ void bitonic_sort_u64(uint64_t* key, int n2) {
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < n2; t += blockDim.x) {
        const int ixj = t ^ j;
        if (ixj > t) {
          const uint64_t a = key[t], e = key[ixj];
          const bool up = (t & k) == 0;
          if ((a > e) == up) { key[t] = e; key[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ int pow2_ceil(int n) {
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  return n2;
}

__global__ __launch_bounds__(256) void k_select_ring(DevCfg c, DevBufs d) {
  __shared__ uint64_t key[kRingMax];
  __shared__ uint8_t wpick[kWin];
  __shared__ uint8_t wgnd[kWin];
  __shared__ int8_t wlab[kWin];
  __shared__ uint16_t wcol[kWin];
  __shared__ uint16_t cpos[kRingMax];
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
  for (int t = tid; t < wn; t += nt) {
    const int pos = ws + t;
    wpick[t] = d.picked[base + pos];
    wgnd[t] = d.seg_ground[base + pos];
    wlab[t] = d.clabel[base + pos];
    wcol[t] = (uint16_t)d.seg_col[base + pos];
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  auto suppress = [&](int ind) {
    wpick[ind - ws] = 1;
    for (int l = 1; l <= 5; ++l) {
      if (ind + l >= HW) continue;
      const int cd = abs((int)wcol[ind + l - ws] - (int)wcol[ind + l - 1 - ws]);
      if (cd > 10) break;
      wpick[ind + l - ws] = 1;
    }
    for (int l = -1; l >= -5; --l) {
      if (ind + l < 0) continue;
      const int cd = abs((int)wcol[ind + l - ws] - (int)wcol[ind + l + 1 - ws]);
      if (cd > 10) break;
      wpick[ind + l - ws] = 1;
    }
  };
  // ---- edges: statically eligible sorted-part entries, visited in descending key order ----
  for (int p = sp + tid; p < ep; p += nt) {
    const int ind = p == 4 ? 0 : p;
    const float v = p == 4 ? 0.0f : curv[p];
    const int w = ind - ws;
    if (wpick[w] == 0 && v > c.edge_thr && wgnd[w] == 0)
      key[atomicAdd(&s_cnt, 1)] = ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)ind;
  }
  __syncthreads();
  int nE = s_cnt;
  int n2 = pow2_ceil(nE);
  for (int t = nE + tid; t < n2; t += nt) key[t] = 0ull;
  __syncthreads();
  bitonic_sort_u64(key, n2);
  if (tid == 0) {
    int cnt = 0;
    for (int t = -1; t < nE; ++t) {
      int ind;
      float v;
      if (t < 0) { ind = ep; v = curv[ep]; }  // the unsorted entry at ep is visited first
      else { const uint64_t k = key[n2 - 1 - t]; ind = (int)(uint32_t)k; v = __uint_as_float((uint32_t)(k >> 32)); }
      const int w = ind - ws;
      if (wpick[w] == 0 && v > c.edge_thr && wgnd[w] == 0) {
        wlab[w] = 1;
        d.edge_tmp[base + sp + cnt++] = ind;
        suppress(ind);
      }
    }
    rc[i] = cnt;
    s_cnt = 0;
  }
  __syncthreads();
  // ---- flats: ascending key order, entry ep last ----
  for (int p = sp + tid; p < ep; p += nt) {
    const int ind = p == 4 ? 0 : p;
    const float v = p == 4 ? 0.0f : curv[p];
    const int w = ind - ws;
    if (wpick[w] == 0 && v < c.surf_thr && wgnd[w] == 1)
      key[atomicAdd(&s_cnt, 1)] = ((uint64_t)__float_as_uint(v) << 32) | (uint32_t)ind;
  }
  __syncthreads();
  const int nF = s_cnt;
  n2 = pow2_ceil(nF);
  for (int t = nF + tid; t < n2; t += nt) key[t] = ~0ull;
  __syncthreads();
  bitonic_sort_u64(key, n2);
  if (tid == 0) {
    int cnt = 0;
    for (int t = 0; t <= nF; ++t) {
      int ind;
      float v;
      if (t == nF) { ind = ep; v = curv[ep]; }
      else { const uint64_t k = key[t]; ind = (int)(uint32_t)k; v = __uint_as_float((uint32_t)(k >> 32)); }
      const int w = ind - ws;
      if (wpick[w] == 0 && v < c.surf_thr && wgnd[w] == 1) {
        wlab[w] = -1;
        d.flat_tmp[base + sp + cnt++] = ind;
        suppress(ind);
      }
    }
    rc[H + i] = cnt;
  }
  __syncthreads();
  for (int t = tid; t < wn; t += nt) {
    d.picked[base + ws + t] = wpick[t];
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
  const float4* lp = d.loam + base + sp;
  // ---- VoxelGrid(0.2) applyFilter (PCL 1.10), centroids summed in (voxel, input) order ----
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int t = tid; t < L; t += nt) {
    const float4 p = lp[cpos[t]];
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
  const int L2 = pow2_ceil(L);
  for (int t = tid; t < L2; t += nt) {
    uint64_t k = ~0ull;
    if (t < L) {
      const float4 p = lp[cpos[t]];
      const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
      const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
      const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
      k = ((uint64_t)(uint32_t)(i0 + i1 * mul1 + i2 * mul2) << 32) | (uint32_t)t;
    }
    key[t] = k;
  }
  __syncthreads();
  bitonic_sort_u64(key, L2);
  const int perv = (L + nt - 1) / nt;
  const int v0 = min(tid * perv, L), v1 = min(v0 + perv, L);
  int heads = 0;
  for (int t = v0; t < v1; ++t) heads += (t == 0 || (key[t] >> 32) != (key[t - 1] >> 32));
  int V;
  int vo = block_excl_scan(heads, tmp, &V);
  for (int t = v0; t < v1; ++t) {
    if (!(t == 0 || (key[t] >> 32) != (key[t - 1] >> 32))) continue;
    const uint32_t vid = (uint32_t)(key[t] >> 32);
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    int e = t;
    while (e < L && (uint32_t)(key[e] >> 32) == vid) {
      const float4 p = lp[cpos[(uint32_t)key[e]]];
      sx += p.x; sy += p.y; sz += p.z; si += p.w;
      ++e;
    }
    const float nn = (float)(e - t);
    out[vo++] = make_float4(sx / nn, sy / nn, sz / nn, si / nn);
  }
  if (tid == 0) rc[2 * H + i] = V;
}

// ---------------------------------------------------------------------------------------------
// K9 concatenate per-ring lists (ring order, FA:1165) and DBSCAN_EdgeFeature (FA:1318-1387)
// + cluster run-length filter (FA:1281-1305). ONE WAVE per scan: the serial merge loop over i
// needs a neighbourhood pass, a min-label reduction and a relabel pass per point; inside one wave
// these are ordered by the wave's own LDS ordering (no workgroup barriers). The O(M^2) tests run
// 64-wide. Points / labels live in LDS when M <= kDb, else in per-slot global scratch.
// Semantics reproduced exactly: in_label_list always holds the labels of the eps-neighbours as
// read before any update (with cluster[i] = 0), so the relabel also collapses every point whose
// label is 0 — including not-yet-visited ones — into min_label (FA:1369-1375).
// ---------------------------------------------------------------------------------------------
constexpr int kDb = 2048;

__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64) void k_fa_finish(DevCfg c, DevBufs d) {
  __shared__ int roff[3][65];
  __shared__ float4 sP[kDb];
  __shared__ int sAux[kDb + 1];   // kz (as float bits) during the merge, label histogram after
  __shared__ int sCl[kDb];
  __shared__ uint32_t sIn[kDb / 32];
  __shared__ uint32_t sLb[kDb / 32 + 1];
  const int b = blockIdx.x;
  const int H = c.H;
  const size_t base = (size_t)b * c.HW;
  const int l = threadIdx.x;
  const int* rc = d.ring_cnt + (size_t)b * 3 * H;
  // ring offsets (exclusive scan over <= 64 rings, three lists)
  for (int q = 0; q < 3; ++q) {
    const int v = l < H ? rc[q * H + l] : 0;
    const int incl = wave_incl_scan_add(v);
    if (l < H) roff[q][l] = incl - v;
    if (l == 63) roff[q][H] = incl;
  }
  wave_fence();
  const int M = roff[0][H], F = roff[1][H], Lf = roff[2][H];
  for (int r = 0; r < H; ++r) {
    const int sp = d.start_ring[b * H + r];
    for (int t = l; t < rc[r]; t += 64) d.less_sharp[base + roff[0][r] + t] = d.edge_tmp[base + sp + t];
    for (int t = l; t < rc[H + r]; t += 64) d.flat[base + roff[1][r] + t] = d.flat_tmp[base + sp + t];
    for (int t = l; t < rc[2 * H + r]; t += 64) d.lflat[base + roff[2][r] + t] = d.lflat_tmp[base + sp + t];
  }
  __threadfence_block();

  const bool lds = M <= kDb;
  float4* P = lds ? sP : d.db_pts + base;
  int* AUX = lds ? sAux : (int*)(d.db_kz + base);
  int* CL = lds ? sCl : d.cluster + base;
  uint32_t* IN = lds ? sIn : (uint32_t*)(d.ccl_b + base);
  const int nwIn = (M + 31) / 32, nwLb = (M + 1 + 31) / 32;
  uint32_t* LB = lds ? sLb : IN + nwIn;
  const float4* loam = d.loam + base;
  for (int a = l; a < M; a += 64) {
    const float4 p = loam[d.less_sharp[base + a]];
    const float x0 = p.z, y0 = p.x, z0 = p.y;  // LOAM -> lidar axes (FA:1327-1329)
    const float AB = atan2f_(z0, sqrt_(x0 * x0 + y0 * y0));
    const float kxy = sqrt_(x0 * x0 + y0 * y0) * c.sinResX * c.RatioXY;
    const float kz = (sqrt_(x0 * x0 + y0 * y0) * tanf_(AB + c.fa_resY) -
                      sqrt_(x0 * x0 + y0 * y0) * tanf_(AB - c.fa_resY)) / 2 * c.RatioZ;
    P[a] = make_float4(x0, y0, z0, kxy);
    AUX[a] = __float_as_int(kz);
    CL[a] = 0;
  }
  for (int w = l; w < nwIn; w += 64) IN[w] = 0u;
  for (int w = l; w < nwLb; w += 64) LB[w] = 0u;
  __threadfence_block();
  int label = 0;
  for (int i = 0; i < M; ++i) {
    const float4 pi = P[i];
    int lmin = 999999999;
    for (int j = l; j < M; j += 64) {
      const float4 pj = P[j];
      const float kzj = __int_as_float(AUX[j]);
      const float eps = sqrt_((pi.x - pj.x) * (pi.x - pj.x) / (pj.w * pj.w) +
                              (pi.y - pj.y) * (pi.y - pj.y) / (pj.w * pj.w) +
                              (pi.z - pj.z) * (pi.z - pj.z) / (kzj * kzj));
      if (eps <= c.DBFr) {
        const int lj = j == i ? 0 : CL[j];
        atomicOr(&IN[j >> 5], 1u << (j & 31));
        atomicOr(&LB[lj >> 5], 1u << (lj & 31));
        if (lj != 0 && lj < lmin) lmin = lj;
      }
    }
    lmin = wave_reduce_min(lmin);
    if (lds) wave_fence(); else __threadfence_block();
    if (lmin <= label) {
      for (int j = l; j < M; j += 64) {
        const int cur = j == i ? 0 : CL[j];
        if (((IN[j >> 5] >> (j & 31)) & 1u) || ((LB[cur >> 5] >> (cur & 31)) & 1u)) CL[j] = lmin;
        else if (j == i) CL[j] = 0;
      }
    } else {
      label += 1;
      for (int j = l; j < M; j += 64) {
        if ((IN[j >> 5] >> (j & 31)) & 1u) CL[j] = label;
        else if (j == i) CL[j] = 0;
      }
    }
    if (lds) wave_fence(); else __threadfence_block();
    for (int w = l; w < nwIn; w += 64) IN[w] = 0u;
    for (int w = l; w <= (label >> 5) && w < nwLb; w += 64) LB[w] = 0u;
    if (lds) wave_fence(); else __threadfence_block();
  }
  // ---- run lengths of the sorted labels, last run dropped; keep label r+1 if run r >= 4 ----
  int* hist = AUX;
  const int NL = label + 1;
  for (int q = l; q < NL; q += 64) hist[q] = 0;
  __threadfence_block();
  for (int a = l; a < M; a += 64) atomicAdd(&hist[CL[a]], 1);
  __threadfence_block();
  int lmax = -1;
  for (int q = l; q < NL; q += 64)
    if (hist[q] > 0) lmax = q;
  lmax = wave_reduce_max(lmax);
  for (int w = l; w < nwLb; w += 64) LB[w] = 0u;
  __threadfence_block();
  const unsigned long long lt = (1ull << l) - 1ull;
  int run = 0;
  for (int q0 = 0; q0 < NL; q0 += 64) {
    const int q = q0 + l;
    const bool pres = q < NL && hist[q] > 0;
    const unsigned long long m = __ballot(pres);
    const int r = run + __popcll(m & lt);
    if (pres && q != lmax && hist[q] >= 4 && r + 1 < NL) atomicOr(&LB[(r + 1) >> 5], 1u << ((r + 1) & 31));
    run += __popcll(m);
  }
  __threadfence_block();
  int ns = 0;
  for (int a0 = 0; a0 < M; a0 += 64) {
    const int a = a0 + l;
    const bool keep = a < M && ((LB[CL[a] >> 5] >> (CL[a] & 31)) & 1u);
    const unsigned long long m = __ballot(keep);
    if (keep) d.sharp[base + ns + __popcll(m & lt)] = d.less_sharp[base + a];
    ns += __popcll(m);
  }
  if (lds)
    for (int a = l; a < M; a += 64) d.cluster[base + a] = CL[a];
  if (l == 0) {
    int* cnt = d.counts + b * kCnt;
    cnt[C_M] = M;
    cnt[C_SHARP] = ns;
    cnt[C_F] = F;
    cnt[C_L] = Lf;
  }
}

}  // namespace llsr
