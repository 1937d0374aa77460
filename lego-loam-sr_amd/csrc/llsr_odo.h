// llsr_odo.h — device data of the end-to-end odometry batch (llsr_odo.hip, llsr_odometry_*).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace llsr {

constexpr int kShadow = 160;  // GenerateShadowPoint: 16 x 10 virtual points (FA:412-450)

struct OdoArgs {
  int B, HW;
  const int* counts;                       // [B][kCnt] of the feature batch
  const float4* loam;                      // [B][HW] segmented cloud in the LOAM frame
  const int* sharp_ind;                    // [B][HW] cornerPointsSharp as segmented indices
  const int* flat_ind;                     // [B][HW] surfPointsFlat (without shadow points)
  const int* less_sharp;                   // [B][HW] cornerPointsLessSharp
  const float4* lflat;                     // [B][HW] surfPointsLessFlat points
  const float4* shadow;                    // [160]
  const int64_t* sharp_off; float4* sharp; // LM queries of this batch, packed [B+1]
  const int64_t* flat_off; float4* flat;
  const int64_t* nlast_c_off; float4* nlast_c;  // the next last clouds, packed [B+1]
  const int64_t* nlast_s_off; float4* nlast_s;
  float4* scan_c; float4* scan_s;          // TransformToEnd'd sharp / flat (offsets of sharp / flat)
  float* tcur;                             // [B][6] transformCur (after the LM)
  float* tsum;                             // [B][6] transformSum
  int* inited;                             // [B] systemInitedLM
  int* frames;                             // [B]
};

__global__ void k_odo_inputs(OdoArgs a);
__global__ void k_odo_finish(OdoArgs a);

}  // namespace llsr
