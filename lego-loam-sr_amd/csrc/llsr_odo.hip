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
    for (int k = threadIdx.x; k < M; k += blockDim.x) cl[k] = odo_to_end(tc, a.loam[base + a.less_sharp[base + k]]);
    for (int k = threadIdx.x; k < L + kShadow; k += blockDim.x)
      sl[k] = k < L ? odo_to_end(tc, a.lflat[base + k]) : a.shadow[k - L];
    float4* sc = a.scan_c + a.sharp_off[b];
    float4* ss = a.scan_s + a.flat_off[b];
    for (int k = threadIdx.x; k < Ms; k += blockDim.x) sc[k] = odo_to_end(tc, a.sharp[a.sharp_off[b] + k]);
    for (int k = threadIdx.x; k < F + kShadow; k += blockDim.x) ss[k] = odo_to_end(tc, a.flat[a.flat_off[b] + k]);
  }
  if (threadIdx.x == 0) {
    if (inited) {
      float ts[6];
      for (int k = 0; k < 6; ++k) ts[k] = a.tsum[6 * b + k];
      odo_integrate(ts, tc);
      for (int k = 0; k < 6; ++k) a.tsum[6 * b + k] = ts[k];
    }
    a.inited[b] = 1;
    a.frames[b] += 1;
  }
}

}  // namespace llsr
