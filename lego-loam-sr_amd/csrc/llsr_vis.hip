// llsr_vis.hip — ImageProjection's visualization topics on gfx950 (publishClouds,
// imageProjection.cpp:933-967) for one slot of the last batch, from the slot's images.
#include "llsr_device.h"

namespace llsr {

// ---------------------------------------------------------------------------------------------
// Visualization clouds of one slot (publishClouds' topics, IP:933-967): _full_cloud and
// _full_info_cloud dense per cell (IP:337-347: x, y, z with intensity row + col / 1e4, resp. the
// range; resetParameters' nanPoint — NaN x, y, z, intensity 0 — for cells no point reached,
// IP:170-179), the ground / nonground / unknownground clouds (the full-cloud points of the cells
// whose final ground_mat is 1 / 0 / 2, row-major, IP:760-769) and _segmented_cloud_pure (cells with
// 0 < label != 999999, intensity = label, row-major, IP:833-842). One workgroup; the four
// compacted clouds keep row-major order through per-chunk block scans. out: 6 arrays of HW float4
// (full, info, ground, nonground, unknown, pure), cnt: 4 counts.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_vis_clouds(DevCfg c, DevBufs d, int b, float4* out, int* cnt) {
  __shared__ int tmp[32];
  const int HW = c.HW, W = c.W;
  const size_t base = (size_t)b * HW;
  float4* full = out;
  float4* info = out + HW;
  float4* cat[4] = {out + 2 * (size_t)HW, out + 3 * (size_t)HW, out + 4 * (size_t)HW, out + 5 * (size_t)HW};
  int run[4] = {0, 0, 0, 0};
  const float qnan = __builtin_nanf("");
  for (int t0 = 0; t0 < HW; t0 += blockDim.x) {
    const int cell = t0 + threadIdx.x;
    const bool in = cell < HW;
    float4 fp = make_float4(qnan, qnan, qnan, 0.0f), ip = fp;
    int g = -9, lab = 0;
    if (in) {
      const int i = cell / W, j = cell - i * W;
      const float4 p = d.full[base + cell];
      if (d.cell_pt[base + cell] >= 0) {
        fp = make_float4(p.x, p.y, p.z, cell_intensity(c.H, W, i, j));
        ip = make_float4(p.x, p.y, p.z, d.range[base + cell]);
      }
      full[cell] = fp;
      info[cell] = ip;
      g = d.ground[base + cell];
      lab = d.label[base + cell];
    }
    const bool sel[4] = {g == 1, g == 0, g == 2, in && lab > 0 && lab != 999999};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int tot;
      const int pos = run[k] + block_excl_scan(sel[k] ? 1 : 0, tmp, &tot);
      if (sel[k]) cat[k][pos] = k < 3 ? fp : make_float4(fp.x, fp.y, fp.z, (float)lab);
      run[k] += tot;
    }
  }
  if (threadIdx.x < 4) cnt[threadIdx.x] = run[threadIdx.x];
}

}  // namespace llsr
