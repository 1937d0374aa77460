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
// cloudSmoothness[sp, ep) is sorted by value (ties by index; the reference's introsort leaves
// tie order unspecified), position 4 carries the never-overwritten phantom {0, ind 0}
// (FA:169, 819), position ep stays unsorted. Lane 0 then runs the serial edge (ep..sp) and flat
// (sp..ep) loops against an LDS window [sp-5, ep+5] of picked/col/ground/curvature; ring windows
// are disjoint (11 positions separate ep_r from sp_{r+1}), so rings run concurrently.
// Less-flat points are compacted and voxel-downsampled (PCL VoxelGrid leaf 0.2) in-block.
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

__global__ __launch_bounds__(256) void k_select_ring(DevCfg c, DevBufs d) {
  __shared__ uint64_t key[kRingMax];
  __shared__ uint8_t wpick[kWin];
  __shared__ uint8_t wgnd[kWin];
  __shared__ int8_t wlab[kWin];
  __shared__ uint32_t wcol[kWin];
  __shared__ float wcurv[kWin];
  __shared__ float4 cand[kRingMax];
  __shared__ int tmp[8];
  __shared__ float red[6][4];
  __shared__ int nvox;
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
  const int nsort = ep - sp;
  int n2 = 1;
  while (n2 < nsort) n2 <<= 1;
  for (int t = tid; t < n2; t += nt) {
    uint64_t k = ~0ull;
    if (t < nsort) {
      const int pos = sp + t;
      k = pos == 4 ? 0ull : ((uint64_t)__float_as_uint(curv[pos]) << 32) | (uint32_t)pos;
    }
    key[t] = k;
  }
  const int ws = sp - 5 > 0 ? sp - 5 : 0;
  const int we = ep + 5 < HW - 1 ? ep + 5 : HW - 1;
  const int wn = we - ws + 1;
  for (int t = tid; t < wn; t += nt) {
    const int pos = ws + t;
    wpick[t] = d.picked[base + pos];
    wgnd[t] = d.seg_ground[base + pos];
    wlab[t] = d.clabel[base + pos];
    wcol[t] = d.seg_col[base + pos];
    wcurv[t] = curv[pos];
  }
  __syncthreads();
  bitonic_sort_u64(key, n2);

  if (tid == 0) {
    auto suppress = [&](int ind) {
      wpick[ind - ws] = 1;
      for (int l = 1; l <= 5; ++l) {
        if (ind + l >= HW) continue;
        const int cd = abs((int)(wcol[ind + l - ws] - wcol[ind + l - 1 - ws]));
        if (cd > 10) break;
        wpick[ind + l - ws] = 1;
      }
      for (int l = -1; l >= -5; --l) {
        if (ind + l < 0) continue;
        const int cd = abs((int)(wcol[ind + l - ws] - wcol[ind + l + 1 - ws]));
        if (cd > 10) break;
        wpick[ind + l - ws] = 1;
      }
    };
    int nE = 0, nF = 0;
    for (int k = ep; k >= sp; --k) {
      const int ind = k == ep ? ep : (int)(uint32_t)key[k - sp];
      const int w = ind - ws;
      if (wpick[w] == 0 && wcurv[w] > c.edge_thr && wgnd[w] == 0) {
        wlab[w] = 1;
        d.edge_tmp[base + sp + nE++] = ind;
        suppress(ind);
      }
    }
    for (int k = sp; k <= ep; ++k) {
      const int ind = k == ep ? ep : (int)(uint32_t)key[k - sp];
      const int w = ind - ws;
      if (wpick[w] == 0 && wcurv[w] < c.surf_thr && wgnd[w] == 1) {
        wlab[w] = -1;
        d.flat_tmp[base + sp + nF++] = ind;
        suppress(ind);
      }
    }
    rc[i] = nE;
    rc[H + i] = nF;
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
  const float4* loam = d.loam + base;
  for (int k = k0; k < k1; ++k)
    if (wlab[sp + k - ws] <= 0) cand[pos++] = loam[sp + k];
  __syncthreads();
  // ---- VoxelGrid(0.2) applyFilter (PCL 1.10), centroids summed in (voxel, input) order ----
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int t = tid; t < L; t += nt) {
    const float4 p = cand[t];
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
  const long long dx = (long long)((mx[0] - mn[0]) * inv) + 1, dy = (long long)((mx[1] - mn[1]) * inv) + 1,
                  dz = (long long)((mx[2] - mn[2]) * inv) + 1;
  if (L == 0) {
    if (tid == 0) rc[2 * H + i] = 0;
    return;
  }
  if (dx * dy * dz > (long long)INT_MAX) {  // PCL: leaf too small -> output = input
    for (int t = tid; t < L; t += nt) out[t] = cand[t];
    if (tid == 0) rc[2 * H + i] = L;
    return;
  }
  int minb[3], div[3];
  for (int a = 0; a < 3; ++a) {
    minb[a] = (int)floorf(mn[a] * inv);
    div[a] = (int)floorf(mx[a] * inv) - minb[a] + 1;
  }
  const int mul1 = div[0], mul2 = div[0] * div[1];
  int L2 = 1;
  while (L2 < L) L2 <<= 1;
  for (int t = tid; t < L2; t += nt) {
    uint64_t k = ~0ull;
    if (t < L) {
      const float4 p = cand[t];
      const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
      const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
      const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
      k = ((uint64_t)(uint32_t)(i0 + i1 * mul1 + i2 * mul2) << 32) | (uint32_t)t;
    }
    key[t] = k;
  }
  __syncthreads();
  bitonic_sort_u64(key, L2);
  // voxel heads -> ordinal via block scan over contiguous chunks
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
      const float4 p = cand[(uint32_t)key[e]];
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
// + cluster run-length filter (FA:1281-1305). One workgroup (1024 threads) per scan.
// The O(M^2) neighbourhood tests run in parallel across the block for each i; the serial
// label-merge semantics (collapse through label 0, relabel of every member label) are applied
// exactly with LDS bitmaps. Points/labels live in LDS when M <= kDbLds, else in global scratch.
// ---------------------------------------------------------------------------------------------
constexpr int kDbLds = 4096;

__global__ __launch_bounds__(1024) void k_fa_finish(DevCfg c, DevBufs d) {
  __shared__ int roff[3][65];
  __shared__ float4 sP[kDbLds];
  __shared__ float sKz[kDbLds];
  __shared__ int sCl[kDbLds + 1];
  __shared__ uint32_t sIn[2][kDbLds / 32];
  __shared__ uint32_t sLb[2][kDbLds / 32 + 1];
  __shared__ int sMin[2];
  __shared__ int tmp[32];
  const int b = blockIdx.x;
  const int H = c.H;
  const size_t base = (size_t)b * c.HW;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int* rc = d.ring_cnt + (size_t)b * 3 * H;
  if (tid < 3) {
    int acc = 0;
    for (int r = 0; r < H; ++r) { roff[tid][r] = acc; acc += rc[tid * H + r]; }
    roff[tid][H] = acc;
  }
  __syncthreads();
  const int M = roff[0][H], F = roff[1][H], Lf = roff[2][H];
  for (int r = 0; r < H; ++r) {
    const int sp = d.start_ring[b * H + r];
    for (int t = tid; t < rc[r]; t += nt) d.less_sharp[base + roff[0][r] + t] = d.edge_tmp[base + sp + t];
    for (int t = tid; t < rc[H + r]; t += nt) d.flat[base + roff[1][r] + t] = d.flat_tmp[base + sp + t];
    for (int t = tid; t < rc[2 * H + r]; t += nt) d.lflat[base + roff[2][r] + t] = d.lflat_tmp[base + sp + t];
  }
  __syncthreads();

  // ---- DBSCAN_EdgeFeature ----
  const bool lds = M <= kDbLds;
  float4* P = lds ? sP : d.db_pts + base;
  float* KZ = lds ? sKz : d.db_kz + base;
  int* CL = lds ? sCl : d.cluster + base;
  uint32_t* IN0 = lds ? sIn[0] : (uint32_t*)(d.ccl_b + base);
  const int nwIn = (M + 31) / 32;
  uint32_t* IN1 = IN0 + (lds ? kDbLds / 32 : nwIn);
  uint32_t* LB0 = lds ? sLb[0] : IN1 + nwIn;
  const int nwLb = (M + 1 + 31) / 32;
  uint32_t* LB1 = LB0 + (lds ? kDbLds / 32 + 1 : nwLb);
  const float4* loam = d.loam + base;
  for (int a = tid; a < M; a += nt) {
    const float4 p = loam[d.less_sharp[base + a]];
    const float x0 = p.z, y0 = p.x, z0 = p.y;
    const float rxy = sqrt_(x0 * x0 + y0 * y0);
    const float AB = atan2f_(z0, rxy);
    const float kxy = sqrt_(x0 * x0 + y0 * y0) * c.sinResX * c.RatioXY;
    const float kz = (sqrt_(x0 * x0 + y0 * y0) * tanf_(AB + c.fa_resY) -
                      sqrt_(x0 * x0 + y0 * y0) * tanf_(AB - c.fa_resY)) / 2 * c.RatioZ;
    P[a] = make_float4(x0, y0, z0, kxy);
    KZ[a] = kz;
    CL[a] = 0;
  }
  for (int w = tid; w < nwIn; w += nt) { IN0[w] = 0u; IN1[w] = 0u; }
  for (int w = tid; w < nwLb; w += nt) { LB0[w] = 0u; LB1[w] = 0u; }
  if (tid == 0) { sMin[0] = 999999999; sMin[1] = 999999999; }
  __syncthreads();
  int label = 0;
  for (int i = 0; i < M; ++i) {
    uint32_t* IN = (i & 1) ? IN1 : IN0;
    uint32_t* LB = (i & 1) ? LB1 : LB0;
    uint32_t* INo = (i & 1) ? IN0 : IN1;
    uint32_t* LBo = (i & 1) ? LB0 : LB1;
    const float4 pi = P[i];
    int lmin = 999999999;
    for (int j = tid; j < M; j += nt) {
      const float4 pj = P[j];
      const float kzj = KZ[j];
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
    if (lane_id() == 0 && lmin < 999999999) atomicMin(&sMin[i & 1], lmin);
    // clear the other buffers (used by iteration i-1, consumed before the last barrier)
    for (int w = tid; w < nwIn; w += nt) INo[w] = 0u;
    for (int w = tid; w < nwLb; w += nt) LBo[w] = 0u;
    if (tid == 0) sMin[(i + 1) & 1] = 999999999;
    __syncthreads();
    const int minLabel = sMin[i & 1];
    if (minLabel <= label) {
      for (int j = tid; j < M; j += nt) {
        const int cur = j == i ? 0 : CL[j];
        const bool inj = (IN[j >> 5] >> (j & 31)) & 1u;
        if (inj || ((LB[cur >> 5] >> (cur & 31)) & 1u)) CL[j] = minLabel;
        else if (j == i) CL[j] = 0;
      }
    } else {
      label += 1;
      for (int j = tid; j < M; j += nt) {
        const bool inj = (IN[j >> 5] >> (j & 31)) & 1u;
        if (inj) CL[j] = label;
        else if (j == i) CL[j] = 0;
      }
    }
    __syncthreads();
  }
  // ---- run lengths of sorted labels, last run dropped; label r+1 kept if run r >= 4 ----
  // labels are in [0, label]; histogram into KZ's storage (no longer needed)
  int* hist = lds ? (int*)sKz : (int*)(d.db_kz + base);
  const int NL = label + 1;
  for (int l = tid; l < NL; l += nt) hist[l] = 0;
  __syncthreads();
  for (int a = tid; a < M; a += nt) atomicAdd(&hist[CL[a]], 1);
  __syncthreads();
  int lmax = -1;
  for (int l = tid; l < NL; l += nt)
    if (hist[l] > 0) lmax = l;
  lmax = wave_reduce_max(lmax);
  if (lane_id() == 0) tmp[tid >> 6] = lmax;
  __syncthreads();
  lmax = -1;
  for (int w = 0; w < (nt >> 6); ++w) lmax = tmp[w] > lmax ? tmp[w] : lmax;
  __syncthreads();
  // rank of each present label among present labels (ascending)
  const int perl = (NL + nt - 1) / nt;
  const int l0 = min(tid * perl, NL), l1 = min(l0 + perl, NL);
  int pres = 0;
  for (int l = l0; l < l1; ++l) pres += hist[l] > 0;
  int tot;
  int r = block_excl_scan(pres, tmp, &tot);
  // inlier marks go into LB0 (label-indexed bitmap); clear it first
  for (int w = tid; w < nwLb; w += nt) LB0[w] = 0u;
  __syncthreads();
  for (int l = l0; l < l1; ++l) {
    if (hist[l] <= 0) continue;
    if (l != lmax && hist[l] >= 4) {
      const int lab = r + 1;
      if (lab < NL) atomicOr(&LB0[lab >> 5], 1u << (lab & 31));
    }
    ++r;
  }
  __syncthreads();
  const int perm = (M + nt - 1) / nt;
  const int a0 = min(tid * perm, M), a1 = min(a0 + perm, M);
  int ns = 0;
  for (int a = a0; a < a1; ++a) ns += (LB0[CL[a] >> 5] >> (CL[a] & 31)) & 1u;
  int NS;
  int ps = block_excl_scan(ns, tmp, &NS);
  for (int a = a0; a < a1; ++a)
    if ((LB0[CL[a] >> 5] >> (CL[a] & 31)) & 1u) d.sharp[base + ps++] = d.less_sharp[base + a];
  if (lds)
    for (int a = tid; a < M; a += nt) d.cluster[base + a] = CL[a];
  if (tid == 0) {
    int* cnt = d.counts + b * kCnt;
    cnt[C_M] = M;
    cnt[C_SHARP] = NS;
    cnt[C_F] = F;
    cnt[C_L] = Lf;
  }
}

}  // namespace llsr
