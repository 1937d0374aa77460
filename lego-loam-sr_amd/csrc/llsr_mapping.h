// llsr_mapping.h — the scalar glue of MapOptimization::run (mapOptmization.cpp:1854-1896) that sits
// between the batched kernels of the mapping chain (llsr_mapping_*): per sequence and frame a few
// dozen float / double operations, evaluated on the host side of the library exactly as the
// reference's x86-64 build evaluates them (glibc float sinf / cosf / asinf / atan2f for the float
// overloads, glibc double sin / cos / asin / atan2 inside tf2; no FMA contraction).
//   * the odometry handoff: FeatureAssociation::publishOdometry builds laser_odometry from
//     transformSum through tf2::Quaternion::setRPY (featureAssociation.cpp:2612-2625) and
//     MapOptimization reads it back with OdometryToTransform (utility.h:99-113,
//     tf2::Matrix3x3::getRPY);
//   * transformAssociateToMap (mapOptmization.cpp:458-581) and transformUpdate (MO:583-589).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "../../include/llsr.h"

namespace llsr_mapping {

// Which keyframes make up a llsr_map's local map between extractSurroundingKeyFrames calls
// (MO:1096-1232): the radius branch's surroundingExistingKeyPosesID, or the loop-closure branch's
// queue of recent keyframes (their indices, oldest first) and latestFrameID. The queue holds
// indices rather than the transformed clouds of MO:1115-1143: a key pose never changes after
// saveKeyFramesAndFactor stores it (correctPoses acts only after a closed loop, MO:1758, and the
// loop-closure thread is commented out, MO:174), so transforming at extract time gives the same
// points.
struct MapSel {
  std::vector<int> ids;
  int latest_frame_id = 0;
};
MapSel map_selection(const llsr_map* m);
void set_map_selection(llsr_map* m, const MapSel& s);

// Segmented VoxelGrid (llsr_map.hip's engine) over S clouds src[k] (device, n[k] points, leaf[k]):
// results packed into `out` (capacity sum n) in segment order, offsets out_off[S+1] on the host.
// Synchronises s.
int32_t voxel_multi(llsr_map* m, const float4* const* src, const long long* n, const float* leaf, int S,
                    float4* out, long long* out_off, hipStream_t s);
// extractSurroundingKeyFrames of n maps around pos[n][3] in one pass of `eng`'s engine: the local
// maps in *out (eng-owned, valid until its next use), map i's corner map at [off_c[i], off_c[i+1]),
// surf map at [off_s[i], off_s[i+1]); reps[i] as llsr_map_extract. A map without keyframes yields
// empty maps (the caller skips the call for it, MO:1097). Synchronises s.
int32_t extract_multi(llsr_map* eng, llsr_map* const* maps, int n, const float* pos, llsr_map_report* reps,
                      const float4** out, long long* off_c, long long* off_s, hipStream_t s);
// Drop keyframes from index `keep` on (a failed frame's keyframe, llsr_mapping_batch rollback).
void truncate_keyframes(llsr_map* m, int keep);

// tf2::Quaternion::setRPY (tf2/LinearMath/Quaternion.h), double. The reference's GCC -O3 build
// merges each tf2Cos(a) / tf2Sin(a) pair into one glibc sincos(a) call (GCC's sincos pass), and
// glibc's sincos can differ from separate sin / cos in the last bit (e.g. q.w of setRPY(0.963,
// -2.970, 1.414) by 2 ulps); clang does not merge, so the call is written out.
inline void tf2_set_rpy(double roll, double pitch, double yaw, double q[4]) {
  const double halfYaw = yaw * 0.5, halfPitch = pitch * 0.5, halfRoll = roll * 0.5;
  double cosYaw, sinYaw, cosPitch, sinPitch, cosRoll, sinRoll;
  ::sincos(halfYaw, &sinYaw, &cosYaw);
  ::sincos(halfPitch, &sinPitch, &cosPitch);
  ::sincos(halfRoll, &sinRoll, &cosRoll);
  q[0] = sinRoll * cosPitch * cosYaw - cosRoll * sinPitch * sinYaw;
  q[1] = cosRoll * sinPitch * cosYaw + sinRoll * cosPitch * sinYaw;
  q[2] = cosRoll * cosPitch * sinYaw - sinRoll * sinPitch * cosYaw;
  q[3] = cosRoll * cosPitch * cosYaw + sinRoll * sinPitch * sinYaw;
}

// tf2::Matrix3x3(q).getRPY(roll, pitch, yaw) (tf2/LinearMath/Matrix3x3.h: setRotation +
// getEulerYPR, solution 1), double
inline void tf2_get_rpy(const double q[4], double& roll, double& pitch, double& yaw) {
  const double d = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  const double s = 2.0 / d;
  const double xs = q[0] * s, ys = q[1] * s, zs = q[2] * s;
  const double wx = q[3] * xs, wy = q[3] * ys, wz = q[3] * zs;
  const double xx = q[0] * xs, xy = q[0] * ys, xz = q[0] * zs;
  const double yy = q[1] * ys, yz = q[1] * zs, zz = q[2] * zs;
  const double m00 = 1.0 - (yy + zz), m10 = xy + wz, m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
  if (std::fabs(m20) >= 1) {
    yaw = 0;
    const double delta = std::atan2(m21, m22);
    pitch = m20 < 0 ? 3.141592653589793238 / 2.0 : -3.141592653589793238 / 2.0;
    roll = delta;
  } else {
    pitch = -std::asin(m20);
    roll = std::atan2(m21 / std::cos(pitch), m22 / std::cos(pitch));
    yaw = std::atan2(m10 / std::cos(pitch), m00 / std::cos(pitch));
  }
}

// laser_odometry of publishOdometry (FA:2612-2625) read back by OdometryToTransform (UT:99-113):
// orientation = (-q.y, -q.z, q.x, q.w) of setRPY(ts[2], -ts[0], -ts[1]); OdometryToTransform
// rebuilds tf2::Quaternion(o.z, -o.x, -o.y, o.w) = q and takes getRPY.
inline void odometry_roundtrip(const float ts[6], float out[6]) {
  double q[4];
  tf2_set_rpy((double)ts[2], -(double)ts[0], -(double)ts[1], q);
  const double ox = -q[1], oy = -q[2], oz = q[0], ow = q[3];  // geometry_msgs orientation
  const double q2[4] = {oz, -ox, -oy, ow};
  double roll, pitch, yaw;
  tf2_get_rpy(q2, roll, pitch, yaw);
  out[0] = (float)(-pitch);
  out[1] = (float)(-yaw);
  out[2] = (float)roll;
  out[3] = (float)(double)ts[3];  // position.x/y/z: float -> double -> float
  out[4] = (float)(double)ts[4];
  out[5] = (float)(double)ts[5];
}

// the publishers' pose -> nav_msgs/Odometry encoding (FA:2612-2625, MO:704-723, TF:193-206)
inline void pose_to_odometry(const float pose[6], const float* twist6, llsr_odometry_msg& m) {
  double q[4];
  tf2_set_rpy((double)pose[2], -(double)pose[0], -(double)pose[1], q);  // float args -> double
  m.orientation[0] = -q[1];
  m.orientation[1] = -q[2];
  m.orientation[2] = q[0];
  m.orientation[3] = q[3];
  for (int k = 0; k < 3; ++k) {
    m.position[k] = (double)pose[3 + k];
    m.twist_angular[k] = twist6 ? (double)twist6[k] : 0.0;
    m.twist_linear[k] = twist6 ? (double)twist6[3 + k] : 0.0;
  }
}

// OdometryToTransform (UT:99-113)
inline void odometry_to_transform(const llsr_odometry_msg& m, float t[6]) {
  const double q2[4] = {m.orientation[2], -m.orientation[0], -m.orientation[1], m.orientation[3]};
  double roll, pitch, yaw;
  tf2_get_rpy(q2, roll, pitch, yaw);
  t[0] = (float)(-pitch);
  t[1] = (float)(-yaw);
  t[2] = (float)roll;
  for (int k = 0; k < 3; ++k) t[3 + k] = (float)m.position[k];
}

// MapOptimization's pose members (mapOptimization.h), one sequence
struct MoPoses {
  float transformSum[6] = {0};
  float transformIncre[6] = {0};
  float transformTobeMapped[6] = {0};
  float transformBefMapped[6] = {0};
  float transformAftMapped[6] = {0};
  float transformLast[6] = {0};
};

// transformAssociateToMap (MO:458-581): the float overloads of sin / cos / asin / atan2
inline void transform_associate_to_map(MoPoses& m) {
  const float* S = m.transformSum;
  const float* B = m.transformBefMapped;
  const float* A = m.transformAftMapped;
  float* T = m.transformTobeMapped;
  float* I = m.transformIncre;
  float x1 = std::cos(S[1]) * (B[3] - S[3]) - std::sin(S[1]) * (B[5] - S[5]);
  float y1 = B[4] - S[4];
  float z1 = std::sin(S[1]) * (B[3] - S[3]) + std::cos(S[1]) * (B[5] - S[5]);
  float x2 = x1;
  float y2 = std::cos(S[0]) * y1 + std::sin(S[0]) * z1;
  float z2 = -std::sin(S[0]) * y1 + std::cos(S[0]) * z1;
  I[3] = std::cos(S[2]) * x2 + std::sin(S[2]) * y2;
  I[4] = -std::sin(S[2]) * x2 + std::cos(S[2]) * y2;
  I[5] = z2;
  const float sbcx = std::sin(S[0]), cbcx = std::cos(S[0]);
  const float sbcy = std::sin(S[1]), cbcy = std::cos(S[1]);
  const float sbcz = std::sin(S[2]), cbcz = std::cos(S[2]);
  const float sblx = std::sin(B[0]), cblx = std::cos(B[0]);
  const float sbly = std::sin(B[1]), cbly = std::cos(B[1]);
  const float sblz = std::sin(B[2]), cblz = std::cos(B[2]);
  const float salx = std::sin(A[0]), calx = std::cos(A[0]);
  const float saly = std::sin(A[1]), caly = std::cos(A[1]);
  const float salz = std::sin(A[2]), calz = std::cos(A[2]);
  const float srx = -sbcx * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz) -
                    cbcx * sbcy *
                        (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                         calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                    cbcx * cbcy *
                        (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                         calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx);
  T[0] = -std::asin(srx);
  const float srycrx =
      sbcx * (cblx * cblz * (caly * salz - calz * salx * saly) - cblx * sblz * (caly * calz + salx * saly * salz) +
              calx * saly * sblx) -
      cbcx * cbcy *
          ((caly * calz + salx * saly * salz) * (cblz * sbly - cbly * sblx * sblz) +
           (caly * salz - calz * salx * saly) * (sbly * sblz + cbly * cblz * sblx) - calx * cblx * cbly * saly) +
      cbcx * sbcy *
          ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
           (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) + calx * cblx * saly * sbly);
  const float crycrx =
      sbcx * (cblx * sblz * (calz * saly - caly * salx * salz) - cblx * cblz * (saly * salz + caly * calz * salx) +
              calx * caly * sblx) +
      cbcx * cbcy *
          ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
           (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) + calx * caly * cblx * cbly) -
      cbcx * sbcy *
          ((saly * salz + caly * calz * salx) * (cbly * sblz - cblz * sblx * sbly) +
           (calz * saly - caly * salx * salz) * (cbly * cblz + sblx * sbly * sblz) - calx * caly * cblx * sbly);
  T[1] = std::atan2(srycrx / std::cos(T[0]), crycrx / std::cos(T[0]));
  const float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) *
                           (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                            calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) -
                       (cbcy * cbcz + sbcx * sbcy * sbcz) *
                           (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                            calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) +
                       cbcx * sbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
  const float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) *
                           (calx * calz * (cbly * sblz - cblz * sblx * sbly) -
                            calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly) -
                       (sbcy * sbcz + cbcy * cbcz * sbcx) *
                           (calx * salz * (cblz * sbly - cbly * sblx * sblz) -
                            calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx) +
                       cbcx * cbcz * (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz);
  T[2] = std::atan2(srzcrx / std::cos(T[0]), crzcrx / std::cos(T[0]));
  x1 = std::cos(T[2]) * I[3] - std::sin(T[2]) * I[4];
  y1 = std::sin(T[2]) * I[3] + std::cos(T[2]) * I[4];
  z1 = I[5];
  x2 = x1;
  y2 = std::cos(T[0]) * y1 - std::sin(T[0]) * z1;
  z2 = std::sin(T[0]) * y1 + std::cos(T[0]) * z1;
  T[3] = A[3] - (std::cos(T[1]) * x2 + std::sin(T[1]) * z2);
  T[4] = A[4] - y2;
  T[5] = A[5] - (-std::sin(T[1]) * x2 + std::cos(T[1]) * z2);
}

// transformUpdate (MO:583-589)
inline void transform_update(MoPoses& m) {
  for (int i = 0; i < 6; ++i) {
    m.transformBefMapped[i] = m.transformSum[i];
    m.transformAftMapped[i] = m.transformTobeMapped[i];
  }
}

}  // namespace llsr_mapping
