// llsr_grid.hip — build kernels of the per-problem cell grids (llsr_grid.h). blockIdx.y =
// problem, blockIdx.z = which of the two grids.
#include "llsr_device.h"
#include "llsr_grid.h"

namespace llsr {

__global__ void k_grid_clear(CellGrids2 gg) {
  const CellGrid& g = gg.g[blockIdx.z];
  const int p = blockIdx.y;
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s == 0) g.cursor[p] = 0;
  if (s >= (1u << g.log2T)) return;
  CellSlot& t = g.tab[((size_t)p << g.log2T) + s];
  t.key = kCellEmpty;
  t.start = 0;
  t.count = 0;
}

// Points are inserted a chunk of kInsChunk at a time per workgroup: the chunk's distinct cells are
// first gathered in an LDS hash (their points' ranks by LDS atomics; a wave's run of equal keys,
// common in scan / VoxelGrid order, takes one), then each distinct cell probes / claims its global
// slot and takes its points' ranks with ONE count atomic. Global atomics execute at the memory side,
// so this is what the build pays for: one per distinct cell per chunk instead of one per run.
constexpr int kInsChunk = 1024;            // points per workgroup (256 threads x 4)
constexpr int kInsLds = 2 * kInsChunk;     // LDS hash slots (load <= 1/2)

__device__ __forceinline__ uint32_t lds_hash(uint64_t k) {
  return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - 11)) & (kInsLds - 1);
}

__global__ __launch_bounds__(256) void k_grid_insert(CellGrids2 gg) {
  static_assert(kInsLds == 1 << 11, "lds_hash width");
  __shared__ uint64_t lkey[kInsLds];
  __shared__ int lcnt[kInsLds];
  __shared__ int lpos[kInsLds];        // global slot, then (after the claims) global base rank
  __shared__ uint16_t ldist[kInsChunk];  // distinct LDS slots of the chunk
  __shared__ int ndist;
  const CellGrid& g = gg.g[blockIdx.z];
  const int p = blockIdx.y;
  const int n = g.count(p);
  const int c0 = blockIdx.x * kInsChunk;
  if (c0 >= n) return;  // block-uniform
  const int tid = threadIdx.x, l = lane_id();
  for (int s = tid; s < kInsLds; s += 256) { lkey[s] = kCellEmpty; lcnt[s] = 0; }
  if (tid == 0) ndist = 0;
  __syncthreads();
  // phase 1: LDS slot and chunk-local rank of every point (u-major: a wave holds 64 consecutive points)
  int slot[4], rank[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = c0 + u * 256 + tid;
    const bool in = k < n;
    uint64_t key = kCellEmpty;
    if (in) {
      const float4 q = g.src[g.off[p] + k];
      key = cell_key(cell_coord(q.x), cell_coord(q.y), cell_coord(q.z));
    }
    const uint64_t prev = __shfl_up(key, 1, 64);
    const bool head = in && (l == 0 || prev != key);
    const unsigned long long heads = __ballot(head);
    const unsigned long long live = __ballot(in);
    const int start = 63 - __clzll((long long)(heads & ((2ull << l) - 1ull)));
    int hs = 0, hb = 0;
    if (head) {
      const unsigned long long after = heads & ~((2ull << l) - 1ull);
      const int end = after ? __ffsll((long long)after) - 1 : 64 - __clzll((long long)live);
      uint32_t h = lds_hash(key);
      for (;;) {
        const uint64_t kk = atomicCAS((unsigned long long*)&lkey[h], (unsigned long long)kCellEmpty,
                                      (unsigned long long)key);
        if (kk == kCellEmpty) ldist[atomicAdd(&ndist, 1)] = (uint16_t)h;
        if (kk == kCellEmpty || kk == key) break;
        h = (h + 1) & (kInsLds - 1);
      }
      hs = (int)h;
      hb = atomicAdd(&lcnt[h], end - l);
    }
    slot[u] = __shfl(hs, start, 64);
    rank[u] = __shfl(hb, start, 64) + (l - start);
  }
  __syncthreads();
  // phase 2: one global probe / claim and one count atomic per distinct cell of the chunk
  CellSlot* tab = g.tab + ((size_t)p << g.log2T);
  const uint32_t mask = (1u << g.log2T) - 1u;
  const int nd = ndist;
  for (int j = tid; j < nd; j += 256) {
    const int ls = ldist[j];
    const uint64_t key = lkey[ls];
    uint32_t h = cell_hash(key, g.log2T);
    for (;;) {  // a plain load first: most cells already exist (a few points per cell)
      uint64_t kk = __hip_atomic_load((unsigned long long*)&tab[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (kk == kCellEmpty)
        kk = atomicCAS((unsigned long long*)&tab[h].key, (unsigned long long)kCellEmpty, (unsigned long long)key);
      if (kk == kCellEmpty || kk == key) break;
      h = (h + 1) & mask;
    }
    const int base = atomicAdd(&tab[h].count, lcnt[ls]);
    lpos[ls] = (int)h;
    lcnt[ls] = base;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = c0 + u * 256 + tid;
    if (k < n) g.where[(size_t)p * g.cap + k] = make_int2(lpos[slot[u]], lcnt[slot[u]] + rank[u]);
  }
}

// Cell ranges: each thread sums the counts of kAllocPer slots, a block scan of those sums, then
// ONE cursor atomic per block of 256 * kAllocPer slots (the cells' order in the copy is irrelevant:
// searches break ties by original index).
constexpr int kAllocPer = 16;

__global__ __launch_bounds__(256) void k_grid_alloc(CellGrids2 gg) {
  const CellGrid& g = gg.g[blockIdx.z];
  const int p = blockIdx.y;
  const uint32_t T = 1u << g.log2T;
  const uint32_t b0 = blockIdx.x * 256u * kAllocPer;
  if (b0 >= T) return;  // block-uniform
  CellSlot* tab = g.tab + ((size_t)p << g.log2T);
  int c[kAllocPer];
  int sum = 0;
#pragma unroll
  for (int u = 0; u < kAllocPer; ++u) {
    const uint32_t s = b0 + u * 256u + threadIdx.x;
    c[u] = s < T ? tab[s].count : 0;
    sum += c[u];
  }
  __shared__ int wtot[4];
  __shared__ int base;
  const int incl = wave_incl_scan_add(sum);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 63) wtot[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(&g.cursor[p], wtot[0] + wtot[1] + wtot[2] + wtot[3]);
  __syncthreads();
  int o = base + incl - sum;
  for (int k = 0; k < w; ++k) o += wtot[k];
#pragma unroll
  for (int u = 0; u < kAllocPer; ++u) {
    if (c[u] > 0) tab[b0 + u * 256u + threadIdx.x].start = o;
    o += c[u];
  }
}

__global__ void k_grid_scatter(CellGrids2 gg) {
  const CellGrid& g = gg.g[blockIdx.z];
  const int p = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= g.count(p)) return;
  const float4 q = g.src[g.off[p] + k];
  const int2 w = g.where[(size_t)p * g.cap + k];
  const CellSlot* tab = g.tab + ((size_t)p << g.log2T);
  g.sorted[(size_t)p * g.cap + tab[w.x].start + w.y] = make_float4(q.x, q.y, q.z, __uint_as_float((uint32_t)k));
}

}  // namespace llsr
