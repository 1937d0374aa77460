// llsr_odo.h — device data of the end-to-end odometry batch (llsr_odo.hip, llsr_odometry_*).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "llsr_device.h"
#include "llsr_libm.h"

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

// The per-scan pose arithmetic of FA's end of scan, shared by k_odo_finish and the host entry points
// llsr_transform_to_end / llsr_integrate_transformation (the FA node's thread calls those on its own
// clouds). Float typing and operation order follow the reference lines; sin / cos / asin / atan2 are
// the glibc ports of llsr_libm.h on both sides (use_imu_undistortion is false in every config block,
// CFG:59/127/195).
using llsr_libm::asinf_;
using llsr_libm::atan2f_;
using llsr_libm::cosf_;
using llsr_libm::sinf_;

// TransformToEnd (FA:1414-1490), use_imu_undistortion == false branch.
__host__ __device__ __forceinline__ float4 odo_to_end(const float* tc, float4 pi) {
  const float s = 10 * (pi.w - (float)trunc_i32(pi.w));
  float rx = s * tc[0], ry = s * tc[1], rz = s * tc[2];
  float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
  const float x1 = cosf_(rz) * (pi.x - tx) + sinf_(rz) * (pi.y - ty);
  const float y1 = -sinf_(rz) * (pi.x - tx) + cosf_(rz) * (pi.y - ty);
  const float z1 = (pi.z - tz);
  const float x2 = x1;
  const float y2 = cosf_(rx) * y1 + sinf_(rx) * z1;
  const float z2 = -sinf_(rx) * y1 + cosf_(rx) * z1;
  const float x3 = cosf_(ry) * x2 - sinf_(ry) * z2;
  const float y3 = y2;
  const float z3 = sinf_(ry) * x2 + cosf_(ry) * z2;
  rx = tc[0]; ry = tc[1]; rz = tc[2];
  tx = tc[3]; ty = tc[4]; tz = tc[5];
  const float x4 = cosf_(ry) * x3 + sinf_(ry) * z3;
  const float y4 = y3;
  const float z4 = -sinf_(ry) * x3 + cosf_(ry) * z3;
  const float x5 = x4;
  const float y5 = cosf_(rx) * y4 - sinf_(rx) * z4;
  const float z5 = sinf_(rx) * y4 + cosf_(rx) * z4;
  return make_float4(cosf_(rz) * x5 - sinf_(rz) * y5 + tx, sinf_(rz) * x5 + cosf_(rz) * y5 + ty, z5 + tz,
                     (float)trunc_i32(pi.w));
}

// AccumulateRotation (FA:1552-1578)
__host__ __device__ __forceinline__ void odo_accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz,
                                                            float& ox, float& oy, float& oz) {
  const float srx = cosf_(lx) * cosf_(cx) * sinf_(ly) * sinf_(cz) - cosf_(cx) * cosf_(cz) * sinf_(lx) -
                    cosf_(lx) * cosf_(ly) * sinf_(cx);
  ox = -asinf_(srx);
  const float srycrx = sinf_(lx) * (cosf_(cy) * sinf_(cz) - cosf_(cz) * sinf_(cx) * sinf_(cy)) +
                       cosf_(lx) * sinf_(ly) * (cosf_(cy) * cosf_(cz) + sinf_(cx) * sinf_(cy) * sinf_(cz)) +
                       cosf_(lx) * cosf_(ly) * cosf_(cx) * sinf_(cy);
  const float crycrx = cosf_(lx) * cosf_(ly) * cosf_(cx) * cosf_(cy) -
                       cosf_(lx) * sinf_(ly) * (cosf_(cz) * sinf_(cy) - cosf_(cy) * sinf_(cx) * sinf_(cz)) -
                       sinf_(lx) * (sinf_(cy) * sinf_(cz) + cosf_(cy) * cosf_(cz) * sinf_(cx));
  oy = atan2f_(srycrx / cosf_(ox), crycrx / cosf_(ox));
  const float srzcrx = sinf_(cx) * (cosf_(lz) * sinf_(ly) - cosf_(ly) * sinf_(lx) * sinf_(lz)) +
                       cosf_(cx) * sinf_(cz) * (cosf_(ly) * cosf_(lz) + sinf_(lx) * sinf_(ly) * sinf_(lz)) +
                       cosf_(lx) * cosf_(cx) * cosf_(cz) * sinf_(lz);
  const float crzcrx = cosf_(lx) * cosf_(lz) * cosf_(cx) * cosf_(cz) -
                       cosf_(cx) * sinf_(cz) * (cosf_(ly) * sinf_(lz) - cosf_(lz) * sinf_(lx) * sinf_(ly)) -
                       sinf_(cx) * (sinf_(ly) * sinf_(lz) + cosf_(ly) * cosf_(lz) * sinf_(lx));
  oz = atan2f_(srzcrx / cosf_(ox), crzcrx / cosf_(ox));
}

// integrateTransformation (FA:2537-2568), no IMU.
__host__ __device__ __forceinline__ void odo_integrate(float* ts, const float* tc) {
  float rx, ry, rz;
  odo_accumulate_rotation(ts[0], ts[1], ts[2], -tc[0], -tc[1], -tc[2], rx, ry, rz);
  const float x1 = cosf_(rz) * (tc[3]) - sinf_(rz) * (tc[4]);
  const float y1 = sinf_(rz) * (tc[3]) + cosf_(rz) * (tc[4]);
  const float z1 = tc[5];
  const float x2 = x1;
  const float y2 = cosf_(rx) * y1 - sinf_(rx) * z1;
  const float z2 = sinf_(rx) * y1 + cosf_(rx) * z1;
  const float tx = ts[3] - (cosf_(ry) * x2 + sinf_(ry) * z2);
  const float ty = ts[4] - y2;
  const float tz = ts[5] - (-sinf_(ry) * x2 + cosf_(ry) * z2);
  ts[0] = rx; ts[1] = ry; ts[2] = rz;
  ts[3] = tx; ts[4] = ty; ts[5] = tz;
}


}  // namespace llsr
