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

// Consecutive points of a cloud often share a cell (scan order, VoxelGrid order), so lanes of a
// wave holding a run of equal keys insert once: the run's first lane probes / claims the slot and
// takes the run's ranks with ONE count atomic; the others derive slot and rank from it.
__global__ void k_grid_insert(CellGrids2 gg) {
  const CellGrid& g = gg.g[blockIdx.z];
  const int p = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = g.count(p);
  if ((int)(blockIdx.x * blockDim.x) >= n) return;  // block-uniform: every lane of a live wave stays
  const bool in = k < n;
  uint64_t key = kCellEmpty;
  if (in) {
    const float4 q = g.src[g.off[p] + k];
    key = cell_key(cell_coord(q.x), cell_coord(q.y), cell_coord(q.z));
  }
  const int l = lane_id();
  const uint64_t prev = __shfl_up(key, 1, 64);
  const bool head = in && (l == 0 || prev != key);
  const unsigned long long heads = __ballot(head);
  const unsigned long long live = __ballot(in);
  const int start = 63 - __clzll((long long)(heads & ((2ull << l) - 1ull)));  // this lane's run head
  int s = 0, base = 0;
  if (head) {
    const unsigned long long after = heads & ~((2ull << l) - 1ull);
    const int end = after ? __ffsll((long long)after) - 1 : 64 - __clzll((long long)live);
    CellSlot* tab = g.tab + ((size_t)p << g.log2T);
    const uint32_t mask = (1u << g.log2T) - 1u;
    uint32_t h = cell_hash(key, g.log2T);
    for (;;) {  // a plain load first: most cells already exist (a few points per cell)
      uint64_t kk = __hip_atomic_load((unsigned long long*)&tab[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (kk == kCellEmpty)
        kk = atomicCAS((unsigned long long*)&tab[h].key, (unsigned long long)kCellEmpty, (unsigned long long)key);
      if (kk == kCellEmpty || kk == key) break;
      h = (h + 1) & mask;
    }
    s = (int)h;
    base = atomicAdd(&tab[h].count, end - l);
  }
  s = __shfl(s, start, 64);
  base = __shfl(base, start, 64);
  if (in) g.where[(size_t)p * g.cap + k] = make_int2(s, base + (l - start));
}

__global__ __launch_bounds__(256) void k_grid_alloc(CellGrids2 gg) {
  // Cell ranges: a block scan of the slot counts, then ONE cursor atomic per block (the cells'
  // order in the copy is irrelevant: searches break ties by original index).
  const CellGrid& g = gg.g[blockIdx.z];
  const int p = blockIdx.y;
  const uint32_t T = 1u << g.log2T;
  if (blockIdx.x * blockDim.x >= T) return;  // block-uniform
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  CellSlot* tab = g.tab + ((size_t)p << g.log2T);
  const int c = s < T ? tab[s].count : 0;
  __shared__ int wtot[4];
  __shared__ int base;
  const int incl = wave_incl_scan_add(c);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 63) wtot[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(&g.cursor[p], wtot[0] + wtot[1] + wtot[2] + wtot[3]);
  __syncthreads();
  int o = base;
  for (int k = 0; k < w; ++k) o += wtot[k];
  if (c > 0) tab[s].start = o + incl - c;
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
