// llsr_odo.hip — the device glue of FeatureAssociation's per-scan loop around the scan-to-scan LM
// (runFeatureAssociation, featureAssociation.cpp:2742-2853), for a batch of independent
// sequences (one slot each), so IP -> features -> LM -> last clouds never leaves HBM:
//
//   k_odo_inputs   cornerPointsSharp / surfPointsFlat (+ the 160 GenerateShadowPoint points,
//                  FA:1310-1314) gathered from the feature stage into the LM's packed inputs
//   (k_grid_* + k_s2s_lm: updateTransformation against the slot's last clouds, llsr_fa_lm.hip)
//   k_odo_finish   first scan of a slot: checkSystemInitialization (FA:2291-2315);
//                  afterwards integrateTransformation (FA:2537-2568 with AccumulateRotation
//                  FA:1552-1578) and publishCloudsLast (FA:2660-2712): TransformToEnd
//                  (FA:1414-1490) of the less-sharp / less-flat clouds, which become the next
//                  last clouds (+ shadow points on the surf side), and of the sharp / flat
//                  clouds, which are the MapOptimization scan inputs (AssociationOut).
// Float typing and operation order follow the reference lines; sin/cos/asin/atan2 are the glibc
// ports of llsr_libm.h (use_imu_undistortion is false in every config block, CFG:59/127/195).
#include <hip/hip_runtime.h>

#include "llsr_device.h"
#include "llsr_libm.h"
#include "llsr_odo.h"

namespace llsr {

using llsr_libm::asinf_;
using llsr_libm::atan2f_;
using llsr_libm::cosf_;
using llsr_libm::sinf_;

// TransformToEnd (FA:1414-1490), use_imu_undistortion == false branch.
__device__ __forceinline__ float4 to_end(const float* tc, float4 pi) {
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
__device__ __forceinline__ void accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz,
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
__device__ __forceinline__ void integrate(float* ts, const float* tc) {
  float rx, ry, rz;
  accumulate_rotation(ts[0], ts[1], ts[2], -tc[0], -tc[1], -tc[2], rx, ry, rz);
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

// grid B, block 256: the LM's query clouds of slot b, packed at the host-computed offsets.
__global__ __launch_bounds__(256) void k_odo_inputs(OdoArgs a) {
  const int b = blockIdx.x;
  const int* cnt = a.counts + b * kCnt;
  const size_t base = (size_t)b * a.HW;
  const int Ms = cnt[C_SHARP], F = cnt[C_F];
  float4* sharp = a.sharp + a.sharp_off[b];
  float4* flat = a.flat + a.flat_off[b];
  for (int k = threadIdx.x; k < Ms; k += blockDim.x) sharp[k] = a.loam[base + a.sharp_ind[base + k]];
  for (int k = threadIdx.x; k < F + kShadow; k += blockDim.x)
    flat[k] = k < F ? a.loam[base + a.flat_ind[base + k]] : a.shadow[k - F];
}

// grid B, block 256: after the LM of slot b (transformCur in a.tcur).
__global__ __launch_bounds__(256) void k_odo_finish(OdoArgs a) {
  const int b = blockIdx.x;
  const int* cnt = a.counts + b * kCnt;
  const size_t base = (size_t)b * a.HW;
  const int M = cnt[C_M], L = cnt[C_L], Ms = cnt[C_SHARP], F = cnt[C_F];
  const bool inited = a.inited[b] != 0;
  float tc[6];
  for (int k = 0; k < 6; ++k) tc[k] = a.tcur[6 * b + k];
  float4* cl = a.nlast_c + a.nlast_c_off[b];
  float4* sl = a.nlast_s + a.nlast_s_off[b];
  if (!inited) {  // checkSystemInitialization (FA:2291-2315): the clouds as they are
    for (int k = threadIdx.x; k < M; k += blockDim.x) cl[k] = a.loam[base + a.less_sharp[base + k]];
    for (int k = threadIdx.x; k < L + kShadow; k += blockDim.x) sl[k] = k < L ? a.lflat[base + k] : a.shadow[k - L];
  } else {  // publishCloudsLast (FA:2666-2707)
    for (int k = threadIdx.x; k < M; k += blockDim.x) cl[k] = to_end(tc, a.loam[base + a.less_sharp[base + k]]);
    for (int k = threadIdx.x; k < L + kShadow; k += blockDim.x)
      sl[k] = k < L ? to_end(tc, a.lflat[base + k]) : a.shadow[k - L];
    float4* sc = a.scan_c + a.sharp_off[b];
    float4* ss = a.scan_s + a.flat_off[b];
    for (int k = threadIdx.x; k < Ms; k += blockDim.x) sc[k] = to_end(tc, a.sharp[a.sharp_off[b] + k]);
    for (int k = threadIdx.x; k < F + kShadow; k += blockDim.x) ss[k] = to_end(tc, a.flat[a.flat_off[b] + k]);
  }
  if (threadIdx.x == 0) {
    if (inited) {
      float ts[6];
      for (int k = 0; k < 6; ++k) ts[k] = a.tsum[6 * b + k];
      integrate(ts, tc);
      for (int k = 0; k < 6; ++k) a.tsum[6 * b + k] = ts[k];
    }
    a.inited[b] = 1;
    a.frames[b] += 1;
  }
}

}  // namespace llsr
