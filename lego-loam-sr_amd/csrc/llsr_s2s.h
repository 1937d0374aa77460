// llsr_s2s.h — device data of the scan-to-scan LM batch (llsr_fa_lm.hip).
#pragma once
#include <stdint.h>

#include "../../include/llsr.h"
#include "llsr_grid.h"

namespace llsr {

struct S2SArgs {
  int P;
  float dist_sqr;              // nearest_feature_search_distance^2 (FA:152)
  int cap_sharp, cap_flat;     // queries per problem reserved
  const float4* sharp; const int64_t* sharp_off;   // cornerPointsSharp
  const float4* flat;  const int64_t* flat_off;    // surfPointsFlat (+ shadow points)
  CellGrids2 grids;            // g[0] laserCloudCornerLast, g[1] laserCloudSurfLast
  float* tcur;                 // [P][6] transformCur in/out
  int* degen;                  // [P] isDegenerate in/out
  llsr_s2s_report* report;     // [P]
  int* idx;                    // [P][max(cap_sharp, cap_flat)][5] correspondence indices + kNN pass
  float4* rows;                // [P][max(cap_sharp, cap_flat)] Jacobian row (3) + b (0 without a correspondence)
  uint8_t* valid;              // [P][max(cap_sharp, cap_flat)] 1: the row holds a correspondence
  int* error;                  // capacity violations
  float4* sbox;                // [P][ceil(cap / 8)][2] bounding boxes of 8-point blocks of laserCloudSurfLast
                               // in index order: (min x, y, z, min ring), (max x, y, z, max ring)
  float4* sbox2;               // [P][ceil(cap / 64)][2] the same for 64-point superblocks
  float* prof;                 // [P][8] diagnostics build only (LLSR_S2S_PROF): phase ticks + fallbacks
};

// bounding boxes of the surf-last cloud's 8-point blocks (the tripod walks skip a block whose box
// cannot hold a nearer point); grid (ceil(ceil(cap / 8) / 256), P), block 256
__global__ void k_s2s_boxes(S2SArgs a);

// k_s2s_lm: one kNT-thread workgroup per problem (512 for the large instantiations: HDL-64E clouds,
// 256 -> 512 took the LM 39.3 -> 32.6 ms in round 2; 256 for <1024, 1024>: four workgroups per CU
// instead of two, so a 1024-scan VLP-16 batch runs in one round instead of two, LM 6.98 -> 4.82 ms
// in round 5). Its reductions, strides and row compaction assume blockDim.x == kNT, so it is only
// launched through s2s_lm_launch, which takes the block size from the template.
template <int kLdsRows, int kLdsCorner, int kNT>
__global__ void k_s2s_lm(S2SArgs a);  // instantiated for <1024, 1024, 256>, <2560, 1536, 512>, <2048, 2048, 512>

template <int kLdsRows, int kLdsCorner, int kNT>
inline void s2s_lm_launch(int P, hipStream_t s, const S2SArgs& a) {
  k_s2s_lm<kLdsRows, kLdsCorner, kNT><<<P, kNT, 0, s>>>(a);
}

}  // namespace llsr
