// oracle_mapping.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h). The scalar pose bookkeeping of
// MapOptimization::run (mapOptmization.cpp:1854-1896) restated on the CPU for the mapping-chain
// parity tests; the clouds go through the oracle's VoxelGrid / keyframe store / scan2map and the
// per-frame composition lives in oracle_py.py (OracleMapping).
//
// Arithmetic follows the reference's x86-64 build: the odometry handoff is tf2 (double,
// tf2/LinearMath/Quaternion.h setRPY, Matrix3x3.h setRotation + getEulerYPR solution 1), and
// transformAssociateToMap calls sin / cos / asin / atan2 on float arguments, which resolve to the
// float overloads (tf2's LinearMath/Scalar.h includes <math.h>, whose libstdc++ wrapper puts
// std::sin(float) etc. in the global namespace) — glibc sinf / cosf / asinf / atan2f here.
#include <math.h>

#include <cmath>
#include <cstdint>

#include "oracle.h"

namespace {

struct Quat { double x, y, z, w; };

// tf2::Quaternion::setRPY(roll, pitch, yaw)
Quat set_rpy(double roll, double pitch, double yaw) {
  const double halfYaw = yaw * 0.5;
  const double halfPitch = pitch * 0.5;
  const double halfRoll = roll * 0.5;
  // tf2Cos / tf2Sin of one angle: GCC -O3 (the reference's build) emits one glibc sincos call for
  // each pair; written out so the statement does not depend on this build's optimiser
  double cosYaw, sinYaw, cosPitch, sinPitch, cosRoll, sinRoll;
  ::sincos(halfYaw, &sinYaw, &cosYaw);
  ::sincos(halfPitch, &sinPitch, &cosPitch);
  ::sincos(halfRoll, &sinRoll, &cosRoll);
  Quat q;
  q.x = sinRoll * cosPitch * cosYaw - cosRoll * sinPitch * sinYaw;
  q.y = cosRoll * sinPitch * cosYaw + sinRoll * cosPitch * sinYaw;
  q.z = cosRoll * cosPitch * sinYaw - sinRoll * sinPitch * cosYaw;
  q.w = cosRoll * cosPitch * cosYaw + sinRoll * sinPitch * sinYaw;
  return q;
}

// tf2::Matrix3x3(q).getRPY(roll, pitch, yaw): setRotation, then getEulerYPR (solution 1)
void get_rpy(const Quat& q, double& roll, double& pitch, double& yaw) {
  const double d = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;  // length2 = dot(q, q)
  const double s = 2.0 / d;
  const double xs = q.x * s, ys = q.y * s, zs = q.z * s;
  const double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
  const double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
  const double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
  double m[3][3];
  m[0][0] = 1.0 - (yy + zz); m[0][1] = xy - wz;         m[0][2] = xz + wy;
  m[1][0] = xy + wz;         m[1][1] = 1.0 - (xx + zz); m[1][2] = yz - wx;
  m[2][0] = xz - wy;         m[2][1] = yz + wx;         m[2][2] = 1.0 - (xx + yy);
  const double kPi = 3.1415926535897932384626433832795029;
  if (::fabs(m[2][0]) >= 1) {
    yaw = 0;
    const double delta = ::atan2(m[2][1], m[2][2]);
    pitch = (m[2][0] < 0) ? kPi / 2.0 : -kPi / 2.0;
    roll = delta;
  } else {
    pitch = -::asin(m[2][0]);
    roll = ::atan2(m[2][1] / ::cos(pitch), m[2][2] / ::cos(pitch));
    yaw = ::atan2(m[1][0] / ::cos(pitch), m[0][0] / ::cos(pitch));
  }
}

}  // namespace

// publishOdometry (FA:2612-2625) -> nav_msgs::Odometry -> OdometryToTransform (utility.h:99-113)
extern "C" void oracle_odometry_to_transform(const float* transformSum_fa, float* transformSum_mo) {
  const float* ts = transformSum_fa;
  const Quat q = set_rpy(ts[2], -ts[0], -ts[1]);  // float -> tf2Scalar (double)
  // geometry_msgs orientation (x, y, z, w) = (-q.y, -q.z, q.x, q.w)
  const double ox = -q.y, oy = -q.z, oz = q.x, ow = q.w;
  double roll, pitch, yaw;
  get_rpy(Quat{oz, -ox, -oy, ow}, roll, pitch, yaw);
  transformSum_mo[0] = (float)-pitch;
  transformSum_mo[1] = (float)-yaw;
  transformSum_mo[2] = (float)roll;
  for (int k = 3; k < 6; ++k) transformSum_mo[k] = (float)(double)ts[k];  // position: float -> double -> float
}

// transformAssociateToMap (MO:458-581), one statement per reference statement.
extern "C" void oracle_associate_to_map(const float* transformSum, const float* transformBefMapped,
                                        const float* transformAftMapped, float* transformTobeMapped,
                                        float* transformIncre) {
  const float* sum = transformSum;
  const float* bef = transformBefMapped;
  const float* aft = transformAftMapped;
  float* tobe = transformTobeMapped;
  float* inc = transformIncre;
  float x1 = cos(sum[1]) * (bef[3] - sum[3]) - sin(sum[1]) * (bef[5] - sum[5]);
  float y1 = bef[4] - sum[4];
  float z1 = sin(sum[1]) * (bef[3] - sum[3]) + cos(sum[1]) * (bef[5] - sum[5]);

  float x2 = x1;
  float y2 = cos(sum[0]) * y1 + sin(sum[0]) * z1;
  float z2 = -sin(sum[0]) * y1 + cos(sum[0]) * z1;

  inc[3] = cos(sum[2]) * x2 + sin(sum[2]) * y2;
  inc[4] = -sin(sum[2]) * x2 + cos(sum[2]) * y2;
  inc[5] = z2;

  float sbcx = sin(sum[0]);
  float cbcx = cos(sum[0]);
  float sbcy = sin(sum[1]);
  float cbcy = cos(sum[1]);
  float sbcz = sin(sum[2]);
  float cbcz = cos(sum[2]);

  float sblx = sin(bef[0]);
  float cblx = cos(bef[0]);
  float sbly = sin(bef[1]);
  float cbly = cos(bef[1]);
  float sblz = sin(bef[2]);
  float cblz = cos(bef[2]);

  float salx = sin(aft[0]);
  float calx = cos(aft[0]);
  float saly = sin(aft[1]);
  float caly = cos(aft[1]);
  float salz = sin(aft[2]);
  float calz = cos(aft[2]);

  // the three bracketed factors shared by srx / srzcrx / crzcrx
  #define ORA_F1 (salx * sblx + calx * cblx * salz * sblz + calx * calz * cblx * cblz)
  #define ORA_F2 (calx * calz * (cbly * sblz - cblz * sblx * sbly) - calx * salz * (cbly * cblz + sblx * sbly * sblz) + cblx * salx * sbly)
  #define ORA_F3 (calx * salz * (cblz * sbly - cbly * sblx * sblz) - calx * calz * (sbly * sblz + cbly * cblz * sblx) + cblx * cbly * salx)
  float srx = -sbcx * ORA_F1 - cbcx * sbcy * ORA_F2 - cbcx * cbcy * ORA_F3;
  tobe[0] = -asin(srx);

  float srycrx = sbcx * (cblx * cblz * (caly * salz - calz * salx * saly) -
                         cblx * sblz * (caly * calz + salx * saly * salz) + calx * saly * sblx) -
                 cbcx * cbcy *
                     ((caly * calz + salx * saly * salz) * (cblz * sbly - cbly * sblx * sblz) +
                      (caly * salz - calz * salx * saly) * (sbly * sblz + cbly * cblz * sblx) -
                      calx * cblx * cbly * saly) +
                 cbcx * sbcy *
                     ((caly * calz + salx * saly * salz) * (cbly * cblz + sblx * sbly * sblz) +
                      (caly * salz - calz * salx * saly) * (cbly * sblz - cblz * sblx * sbly) +
                      calx * cblx * saly * sbly);
  float crycrx = sbcx * (cblx * sblz * (calz * saly - caly * salx * salz) -
                         cblx * cblz * (saly * salz + caly * calz * salx) + calx * caly * sblx) +
                 cbcx * cbcy *
                     ((saly * salz + caly * calz * salx) * (sbly * sblz + cbly * cblz * sblx) +
                      (calz * saly - caly * salx * salz) * (cblz * sbly - cbly * sblx * sblz) +
                      calx * caly * cblx * cbly) -
                 cbcx * sbcy *
                     ((saly * salz + caly * calz * salx) * (cbly * sblz - cblz * sblx * sbly) +
                      (calz * saly - caly * salx * salz) * (cbly * cblz + sblx * sbly * sblz) -
                      calx * caly * cblx * sbly);
  tobe[1] = atan2(srycrx / cos(tobe[0]), crycrx / cos(tobe[0]));

  float srzcrx = (cbcz * sbcy - cbcy * sbcx * sbcz) * ORA_F3 - (cbcy * cbcz + sbcx * sbcy * sbcz) * ORA_F2 +
                 cbcx * sbcz * ORA_F1;
  float crzcrx = (cbcy * sbcz - cbcz * sbcx * sbcy) * ORA_F2 - (sbcy * sbcz + cbcy * cbcz * sbcx) * ORA_F3 +
                 cbcx * cbcz * ORA_F1;
  #undef ORA_F1
  #undef ORA_F2
  #undef ORA_F3
  tobe[2] = atan2(srzcrx / cos(tobe[0]), crzcrx / cos(tobe[0]));

  x1 = cos(tobe[2]) * inc[3] - sin(tobe[2]) * inc[4];
  y1 = sin(tobe[2]) * inc[3] + cos(tobe[2]) * inc[4];
  z1 = inc[5];

  x2 = x1;
  y2 = cos(tobe[0]) * y1 - sin(tobe[0]) * z1;
  z2 = sin(tobe[0]) * y1 + cos(tobe[0]) * z1;

  tobe[3] = aft[3] - (cos(tobe[1]) * x2 + sin(tobe[1]) * z2);
  tobe[4] = aft[4] - y2;
  tobe[5] = aft[5] - (-sin(tobe[1]) * x2 + cos(tobe[1]) * z2);
}

// ---- TransformFusion (transformFusion.cpp) — the node's two handlers, one statement per line ----
// Messages are 13 doubles: orientation x, y, z, w; position x, y, z; twist angular x, y, z; twist
// linear x, y, z. The state is TransformFusion's members, 5 x 6 floats: transformSum,
// transformIncre, transformMapped, transformBefMapped, transformAftMapped.

// the publishers' encoding: FA:2612-2625 (transformSum), MO:704-723 (transformAftMapped, twist =
// transformBefMapped), TF:193-206 (transformMapped)
extern "C" void oracle_pose_to_odometry(const float* pose, const float* twist, double* msg) {
  const Quat q = set_rpy(pose[2], -pose[0], -pose[1]);
  msg[0] = -q.y;  // orientation.x = -geoQuat.y
  msg[1] = -q.z;
  msg[2] = q.x;
  msg[3] = q.w;
  msg[4] = pose[3];
  msg[5] = pose[4];
  msg[6] = pose[5];
  for (int k = 0; k < 6; ++k) msg[7 + k] = twist ? twist[k] : 0.0;
}

// OdometryToTransform (utility.h:99-113)
static void odometry_to_transform_msg(const double* msg, float* transform) {
  double roll, pitch, yaw;
  get_rpy(Quat{msg[2], -msg[0], -msg[1], msg[3]}, roll, pitch, yaw);
  transform[0] = -pitch;
  transform[1] = -yaw;
  transform[2] = roll;
  transform[3] = msg[4];
  transform[4] = msg[5];
  transform[5] = msg[6];
}

// TransformFusion::laserOdometryHandler (TF:188-208)
extern "C" void oracle_fusion_laser_odometry(float* st, const double* laserOdometry, double* laserOdometry2) {
  float* transformSum = st;
  float* transformIncre = st + 6;
  float* transformMapped = st + 12;
  float* transformBefMapped = st + 18;
  float* transformAftMapped = st + 24;
  odometry_to_transform_msg(laserOdometry, transformSum);
  oracle_associate_to_map(transformSum, transformBefMapped, transformAftMapped, transformMapped, transformIncre);
  oracle_pose_to_odometry(transformMapped, nullptr, laserOdometry2);
}

// TransformFusion::odomAftMappedHandler (TF:282-304)
extern "C" void oracle_fusion_aft_mapped(float* st, const double* odomAftMapped) {
  float* transformBefMapped = st + 18;
  float* transformAftMapped = st + 24;
  double roll, pitch, yaw;
  get_rpy(Quat{odomAftMapped[2], -odomAftMapped[0], -odomAftMapped[1], odomAftMapped[3]}, roll, pitch, yaw);
  transformAftMapped[0] = -pitch;
  transformAftMapped[1] = -yaw;
  transformAftMapped[2] = roll;
  transformAftMapped[3] = odomAftMapped[4];
  transformAftMapped[4] = odomAftMapped[5];
  transformAftMapped[5] = odomAftMapped[6];
  transformBefMapped[0] = odomAftMapped[7];
  transformBefMapped[1] = odomAftMapped[8];
  transformBefMapped[2] = odomAftMapped[9];
  transformBefMapped[3] = odomAftMapped[10];
  transformBefMapped[4] = odomAftMapped[11];
  transformBefMapped[5] = odomAftMapped[12];
}
