// llsr_lm.h — LMOptimization's solve / degeneracy / pose update / stop test (MO:1505-1568) on
// already-summed normal equations, and the int64 fixed-point words that the split-correspondence
// scan-to-map sums across GPUs. Device code (llsr_mo.hip); the oracle restates the
// same step independently (oracle/oracle_mo.cpp mo_lm_solve / ofx).
#pragma once
#include <stdint.h>

#include "llsr_eigen.h"
#include "llsr_libm.h"

namespace llsr_lm {

// Words per problem of the reduced normal equations: AtA upper triangle (21, row-major r <= c),
// AtB (6), sum |coeff.intensity| (1), #corner, #surf correspondences (2), 1 spare, and word 31 =
// the number of terms that were out of the fixed-point range (non-finite or |v| >= 2^32).
constexpr int kNeWords = 32;
constexpr int kRed = 30;
constexpr int kNeOverflow = 31;

// Fixed point for the exchanged sums: every per-correspondence term is rounded once to a
// multiple of 2^-30 and the sums are plain int64 additions — associative, so any split of the
// correspondences over blocks / GPUs and any all-reduce order give identical words. Range: a
// term with |v| < 2^32 is at most 2^62 in the word; the sums are exact while the total stays below
// 2^63, i.e. sum |term| < 2^33 (e.g. 20k correspondences with |J|^2 up to 4e5, points ~600 m
// away). A term outside |v| < 2^32 (or NaN / inf) contributes 0 and is counted in word 31, which
// the solve step turns into an error instead of a silently wrong pose.
constexpr double kNeScale = 1073741824.0;  // 2^30
LLSR_HD bool ne_in_range(float v) { return llsr_libm::fabs_(v) < 4294967296.0f; }  // false for NaN
LLSR_HD long long ne_fix(float v) { return ne_in_range(v) ? (long long)__builtin_rint((double)v * kNeScale) : 0; }
LLSR_HD float ne_unfix(long long w) { return (float)((double)w / kNeScale); }
// Word k of one correspondence: the counts (28, 29) stay plain integers.
LLSR_HD long long ne_term(int k, float v) { return k >= 28 ? (long long)v : ne_fix(v); }
LLSR_HD int ne_bad(int k, float v) { return (k < 28 && !ne_in_range(v)) ? 1 : 0; }

// Summed words -> the float reduction vector lm_update consumes.
LLSR_HD void ne_to_red(const long long* w, float* red) {
  for (int k = 0; k < 28; ++k) red[k] = ne_unfix(w[k]);
  red[28] = (float)w[28];
  red[29] = (float)w[29];
}

// One LMOptimization after the Jacobian build (MO:1505-1568) for a problem whose N = nc + ns
// >= 50 (the caller checks MO:1453). St provides pose[6], cR/sR/cP/sP/cY/sY (cached cos / sin
// of pose[0..2]), matP[36], matX0[6], min_lambda, cf_mean, degenerate — matP and degenerate are
// MapOptimization members (mapOptimization.h:279-281): set at iteration 0 and reused after.
// `red`: AtA upper triangle (21), AtB (6), sum |d|, #corner, #surf. Returns the stop test.
// lm_update_full: the same on the full column-major matAtA[36], matAtB[6], CF_all and N.
template <class St>
LLSR_HD bool lm_update_full(St& st, const float* AtA, const float* AtB, float cf_all, int N, int iterCount,
                            bool applied, float stop_thres) {
  using llsr_libm::cosf_;
  using llsr_libm::sinf_;
  float X[6];
  llsr_eigen::colpiv_qr_solve<6, 6>(AtA, AtB, X);  // matAtA.colPivHouseholderQr().solve(matAtB)
  if (iterCount == 0) {  // MO:1507-1531
    float E[6], V[36], V2[36], Vi[36];
    llsr_eigen::eig_sym<6>(AtA, E, V);
    st.min_lambda = E[0];
    for (int k = 0; k < 36; ++k) V2[k] = V[k];
    bool deg = false;
    for (int i = 5; i >= 0; --i) {
      if (E[i] < 100) {
        for (int j = 0; j < 6; ++j) V2[i + 6 * j] = 0;
        deg = true;
      } else {
        break;
      }
    }
    st.degenerate = deg ? 1 : 0;
    llsr_eigen::inverse_lu<6>(V, Vi);      // matV.inverse() (PartialPivLU)
    llsr_eigen::prod66(Vi, V2, st.matP);   // matP = matV.inverse() * matV2
    for (int k = 0; k < 6; ++k) st.matX0[k] = X[k];
  }
  if (st.degenerate) {  // MO:1533-1536
    float X2[6];
    for (int k = 0; k < 6; ++k) X2[k] = X[k];
    llsr_eigen::prod61(st.matP, X2, X);
  }
  if (applied) {  // MO:1539-1545 (commented out in the reference: faithful mode skips it)
    for (int k = 0; k < 6; ++k) st.pose[k] += X[k];
    st.cR = cosf_(st.pose[0]); st.sR = sinf_(st.pose[0]);
    st.cP = cosf_(st.pose[1]); st.sP = sinf_(st.pose[1]);
    st.cY = cosf_(st.pose[2]); st.sY = sinf_(st.pose[2]);
  }
  const float r2d = 57.29577951308232f;  // pcl::rad2deg(float)
  const double e0 = (double)(X[0] * r2d), e1 = (double)(X[1] * r2d), e2 = (double)(X[2] * r2d);
  const double t0 = (double)(X[3] * 100), t1 = (double)(X[4] * 100), t2 = (double)(X[5] * 100);
  const float deltaR = (float)__builtin_sqrt(e0 * e0 + e1 * e1 + e2 * e2);
  const float deltaT = (float)__builtin_sqrt(t0 * t0 + t1 * t1 + t2 * t2);
  st.cf_mean = cf_all / (float)N;
  return deltaR < stop_thres && deltaT < stop_thres;
}

template <class St>
LLSR_HD bool lm_update(St& st, const float* red, int iterCount, bool applied, float stop_thres) {
  const int N = (int)red[28] + (int)red[29];
  float AtA[36];
  int q = 0;
  for (int r = 0; r < 6; ++r)
    for (int c = r; c < 6; ++c, ++q) { AtA[r + 6 * c] = red[q]; AtA[c + 6 * r] = red[q]; }
  return lm_update_full(st, AtA, red + 21, red[27], N, iterCount, applied, stop_thres);
}

}  // namespace llsr_lm
