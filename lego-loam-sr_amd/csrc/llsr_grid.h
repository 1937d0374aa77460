// llsr_grid.h — 1 m cell grids over per-problem point clouds, the device replacement for the
// reference's per-scan nanoflann kd-trees (KdTreeFLANN::setInputCloud; MO:1575-1576 for the
// local maps, FA:2714-2717 for the last corner / surf clouds).
//
// A grid is an open-addressing table of occupied cells (packed floor(x), floor(y), floor(z))
// plus a cell-contiguous copy of the cloud storing (x, y, z, original index bits). Searches
// break distance ties by the original index, so the order of points inside the copy (filled
// with atomics) never changes a result. Built by k_grid_{clear, insert, alloc, scatter} for
// two clouds per problem at once (blockIdx.z).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llsr {

struct CellSlot {
  uint64_t key;  // packed cell or kCellEmpty
  int start;     // first point of the cell in `sorted`
  int count;
};

constexpr uint64_t kCellEmpty = ~0ull;

struct CellGrid {
  const float4* src;    // the clouds, concatenated over the batch
  const int64_t* off;   // [P+1]
  int cap;              // points per problem reserved
  int log2T;            // table slots per problem = 1 << log2T (> cap, grid_log2_table)
  CellSlot* tab;        // [P][1 << log2T]
  float4* sorted;       // [P][cap]
  int2* where;          // [P][cap] (slot, rank) of each point
  int* cursor;          // [P]
  __device__ __forceinline__ int count(int p) const {
    const int64_t n = off[p + 1] - off[p];
    return n < 0 ? 0 : (n > cap ? cap : (int)n);
  }
  __device__ __forceinline__ const CellSlot* table(int p) const { return tab + ((size_t)p << log2T); }
  __device__ __forceinline__ const float4* cells(int p) const { return sorted + (size_t)p * cap; }
};

struct CellGrids2 {
  CellGrid g[2];
  int P;
};

__device__ __forceinline__ int cell_coord(float v) {
  // floor() to a cell index; NaN / huge coordinates land in a far sentinel cell (their distance
  // tests fail anyway, so where they are bucketed cannot change a result)
  const float f = floorf(v);
  return (f > -1048000.0f && f < 1048000.0f) ? (int)f : 1048500;
}

__device__ __forceinline__ uint64_t cell_key(int a, int b, int c) {
  return ((uint64_t)(uint32_t)(a + 1048576) << 42) | ((uint64_t)(uint32_t)(b + 1048576) << 21) |
         (uint64_t)(uint32_t)(c + 1048576);
}

__device__ __forceinline__ uint32_t cell_hash(uint64_t k, int log2T) {
  return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - log2T));
}

// Probe for `key`; returns the slot or -1 (the table is never full: more slots than points).
__device__ __forceinline__ int grid_find(const CellSlot* __restrict__ tab, int log2T, uint64_t key) {
  const uint32_t mask = (1u << log2T) - 1u;
  uint32_t s = cell_hash(key, log2T);
  for (;;) {
    const uint64_t k = tab[s].key;
    if (k == key) return (int)s;
    if (k == kCellEmpty) return -1;
    s = (s + 1) & mask;
  }
}

// (d, index) lexicographic order: the result of inserting candidates in index order with
// nanoflann's strict '<' (KNNResultSet::addPoint).
__device__ __forceinline__ bool nn_before(float da, int ia, float db, int ib) {
  return da < db || (da == db && ia < ib);
}

// Table size for `cap` points per problem.
// Table slots: the smallest power of two ABOVE the point capacity, so at least one slot stays
// empty even if every point had its own cell (grid_find and the insert probes end at an empty
// slot). Clouds hold several points per 1 m cell, so the load is low in practice; k_grid_clear and
// k_grid_alloc sweep the whole table, so a 2x margin doubled their cost (measured: scan-to-map grid
// build 3.7 ms per 256-problem step with 2x).
inline int grid_log2_table(int cap) {
  int l = 4;
  while ((1ll << l) <= (long long)(cap > 1 ? cap : 1)) ++l;
  return l;
}

__global__ void k_grid_clear(CellGrids2 g);
__global__ void k_grid_insert(CellGrids2 g);
__global__ void k_grid_alloc(CellGrids2 g);
__global__ void k_grid_scatter(CellGrids2 g);

// Enqueue the four build kernels for both grids of P problems.
inline void grid_build(const CellGrids2& g, hipStream_t s) {
  const int T = 1 << (g.g[0].log2T > g.g[1].log2T ? g.g[0].log2T : g.g[1].log2T);
  const int M = g.g[0].cap > g.g[1].cap ? g.g[0].cap : g.g[1].cap;
  k_grid_clear<<<dim3((T + 255) / 256, g.P, 2), 256, 0, s>>>(g);
  if (M > 0) k_grid_insert<<<dim3((M + 1023) / 1024, g.P, 2), 256, 0, s>>>(g);  // kInsChunk
  k_grid_alloc<<<dim3((T + 4095) / 4096, g.P, 2), 256, 0, s>>>(g);                // 256 * kAllocPer
  if (M > 0) k_grid_scatter<<<dim3((M + 255) / 256, g.P, 2), 256, 0, s>>>(g);
}

}  // namespace llsr
