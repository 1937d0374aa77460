// llsr_eigen.h — restatements of the Eigen 3.3.7 dense routines the MapOptimization LM calls,
// in float, usable on host and device:
//   * SelfAdjointEigenSolver<Matrix3f> (mapOptmization.cpp:1320) — scaling to [-1,1], the 3x3
//     closed-form tridiagonalisation, implicit symmetric QR steps with Givens rotations
//     accumulated into Q, ascending sort. The corner residual uses ROW 0 of the eigenvector
//     matrix (MO:1329-1334), so each eigenvector's SIGN matters; this follows Eigen's algorithm
//     step by step to reproduce them.
//   * SelfAdjointEigenSolver<Matrix<float,6,6>> (MO:1512) — Householder tridiagonalisation +
//     the same QR iteration (eigenvalues drive min_lambda / degeneracy).
//   * ColPivHouseholderQR::solve (MO:1398 5x3 plane fit, MO:1505 6x6 normal equations).
// Eigen itself is absent from this image; these are checked against numpy
// (tests/test_linalg.py) for values and against the algorithm for signs.
#pragma once
#include <stdint.h>

#include "llsr_libm.h"

namespace llsr_eigen {

using llsr_libm::fabs_;
using llsr_libm::sqrt_;

LLSR_HD float hypot_(float x, float y) {  // Eigen 3.3 internal::hypot_impl
  const float ax = fabs_(x), ay = fabs_(y);
  float p, qp;
  if (ax > ay) { p = ax; qp = ay / p; }
  else { p = ay; qp = ax / p; }
  if (p == 0.0f) return 0.0f;
  return p * sqrt_(1.0f + qp * qp);
}

// JacobiRotation::makeGivens (real case)
LLSR_HD void make_givens(float p, float q, float& c, float& s) {
  if (q == 0.0f) {
    c = p < 0.0f ? -1.0f : 1.0f;
    s = 0.0f;
  } else if (p == 0.0f) {
    c = 0.0f;
    s = q < 0.0f ? 1.0f : -1.0f;
  } else if (fabs_(p) > fabs_(q)) {
    const float t = q / p;
    float u = sqrt_(1.0f + t * t);
    if (p < 0.0f) u = -u;
    c = 1.0f / u;
    s = -t * c;
  } else {
    const float t = p / q;
    float u = sqrt_(1.0f + t * t);
    if (q < 0.0f) u = -u;
    s = -1.0f / u;
    c = -t * s;
  }
}

// internal::tridiagonal_qr_step (ColMajor), Q is n x n column-major
LLSR_HD void tridiagonal_qr_step(float* diag, float* subdiag, int start, int end, float* Q, int n) {
  const float td = (diag[end - 1] - diag[end]) * 0.5f;
  const float e = subdiag[end - 1];
  float mu = diag[end];
  if (td == 0.0f) {
    mu -= fabs_(e);
  } else {
    const float e2 = e * e;
    const float h = hypot_(td, e);
    if (e2 == 0.0f) mu -= (e / (td + (td > 0.0f ? 1.0f : -1.0f))) * (e / h);
    else mu -= e2 / (td + (td > 0.0f ? h : -h));
  }
  float x = diag[start] - mu;
  float z = subdiag[start];
  for (int k = start; k < end; ++k) {
    float c, s;
    make_givens(x, z, c, s);
    const float sdk = s * diag[k] + c * subdiag[k];
    const float dkp1 = s * subdiag[k] + c * diag[k + 1];
    diag[k] = c * (c * diag[k] - s * subdiag[k]) - s * (c * subdiag[k] - s * diag[k + 1]);
    diag[k + 1] = s * sdk + c * dkp1;
    subdiag[k] = c * sdk - s * dkp1;
    if (k > start) subdiag[k - 1] = c * subdiag[k - 1] - s * z;
    x = subdiag[k];
    if (k < end - 1) {
      z = -s * subdiag[k + 1];
      subdiag[k + 1] = c * subdiag[k + 1];
    }
    // Q = Q * G  (applyOnTheRight(k, k+1, rot) == rotation in the plane with rot^T)
    for (int i = 0; i < n; ++i) {
      const float xi = Q[i + k * n], yi = Q[i + (k + 1) * n];
      Q[i + k * n] = c * xi + (-s) * yi;
      Q[i + (k + 1) * n] = -(-s) * xi + c * yi;
    }
  }
}

// internal::computeFromTridiagonal_impl (Eigen 3.3.7 deflation test) + ascending sort.
// Returns 0 on success (Eigen's Success), 1 when the iteration limit was hit.
LLSR_HD int compute_from_tridiagonal(float* diag, float* subdiag, int n, float* Q) {
  const float considerAsZero = 1.17549435e-38f;  // numeric_limits<float>::min()
  const float precision = 2.0f * 1.1920929e-07f;  // 2 * epsilon
  const int maxIterations = 30;
  int end = n - 1, start = 0, iter = 0;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (fabs_(subdiag[i]) <= (fabs_(diag[i]) + fabs_(diag[i + 1])) * precision ||
          fabs_(subdiag[i]) <= considerAsZero)
        subdiag[i] = 0.0f;
    while (end > 0 && subdiag[end - 1] == 0.0f) end--;
    if (end <= 0) break;
    iter++;
    if (iter > maxIterations * n) break;
    start = end - 1;
    while (start > 0 && subdiag[start - 1] != 0.0f) start--;
    tridiagonal_qr_step(diag, subdiag, start, end, Q, n);
  }
  const int info = iter <= maxIterations * n ? 0 : 1;
  if (info == 0) {
    for (int i = 0; i < n - 1; ++i) {
      int k = 0;  // minCoeff(&k) over segment(i, n-i): first minimum
      float m = diag[i];
      for (int q = 1; q < n - i; ++q)
        if (diag[i + q] < m) { m = diag[i + q]; k = q; }
      if (k > 0) {
        const float t = diag[i]; diag[i] = diag[k + i]; diag[k + i] = t;
        for (int r = 0; r < n; ++r) {
          const float u = Q[r + i * n]; Q[r + i * n] = Q[r + (k + i) * n]; Q[r + (k + i) * n] = u;
        }
      }
    }
  }
  return info;
}

// SelfAdjointEigenSolver<Matrix3f>::compute on the lower triangle of A (column-major).
// evals ascending; evecs column-major (eigenvector k = column k).
LLSR_HD int eig3(const float* A, float* evals, float* V) {
  float m[9];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 3; ++r) m[r + 3 * c] = r >= c ? A[r + 3 * c] : 0.0f;  // triangularView<Lower>
  float scale = 0.0f;
  for (int q = 0; q < 9; ++q) scale = fabs_(m[q]) > scale ? fabs_(m[q]) : scale;
  if (scale == 0.0f) scale = 1.0f;
  for (int c = 0; c < 3; ++c)
    for (int r = c; r < 3; ++r) m[r + 3 * c] /= scale;
  float diag[3], sub[2];
  // tridiagonalization_inplace_selector<MatrixType, 3, false>
  const float tol = 1.17549435e-38f;
  diag[0] = m[0];
  const float v1norm2 = m[2] * m[2];  // mat(2,0)
  if (v1norm2 <= tol) {
    diag[1] = m[4];
    diag[2] = m[8];
    sub[0] = m[1];
    sub[1] = m[5];
    for (int q = 0; q < 9; ++q) V[q] = (q % 4 == 0) ? 1.0f : 0.0f;
  } else {
    const float beta = sqrt_(m[1] * m[1] + v1norm2);
    const float invBeta = 1.0f / beta;
    const float m01 = m[1] * invBeta;
    const float m02 = m[2] * invBeta;
    const float q = 2.0f * m01 * m[5] + m02 * (m[8] - m[4]);
    diag[1] = m[4] + m02 * q;
    diag[2] = m[8] - m02 * q;
    sub[0] = beta;
    sub[1] = m[5] - m01 * q;
    // mat << 1,0,0, 0,m01,m02, 0,m02,-m01  (row-wise comma initialiser), stored column-major
    V[0] = 1.0f; V[3] = 0.0f; V[6] = 0.0f;
    V[1] = 0.0f; V[4] = m01;  V[7] = m02;
    V[2] = 0.0f; V[5] = m02;  V[8] = -m01;
  }
  const int info = compute_from_tridiagonal(diag, sub, 3, V);
  for (int k = 0; k < 3; ++k) evals[k] = diag[k] * scale;
  return info;
}

// MatrixBase::makeHouseholder on v[0..m): returns tau, beta; v[1..m) becomes the essential part.
LLSR_HD void make_householder(float* v, int m, float& tau, float& beta) {
  float tailSq = 0.0f;
  for (int q = 1; q < m; ++q) tailSq += v[q] * v[q];
  const float c0 = v[0];
  const float tol = 1.17549435e-38f;
  if (tailSq <= tol) {
    tau = 0.0f;
    beta = c0;
    for (int q = 1; q < m; ++q) v[q] = 0.0f;
  } else {
    beta = sqrt_(c0 * c0 + tailSq);
    if (c0 >= 0.0f) beta = -beta;
    for (int q = 1; q < m; ++q) v[q] = v[q] / (c0 - beta);
    tau = (beta - c0) / beta;
  }
}

// SelfAdjointEigenSolver<Matrix<float,6,6>>: Householder tridiagonalisation (Eigen's
// tridiagonalization_inplace + HouseholderSequence evaluation) + the QR iteration above.
template <int N>
LLSR_HD int eig_sym(const float* A, float* evals, float* V) {
  float m[N * N];
  for (int c = 0; c < N; ++c)
    for (int r = 0; r < N; ++r) m[r + N * c] = r >= c ? A[r + N * c] : 0.0f;
  float scale = 0.0f;
  for (int q = 0; q < N * N; ++q) scale = fabs_(m[q]) > scale ? fabs_(m[q]) : scale;
  if (scale == 0.0f) scale = 1.0f;
  for (int c = 0; c < N; ++c)
    for (int r = c; r < N; ++r) m[r + N * c] /= scale;
  // full symmetric working copy (Eigen reads the lower triangle through selfadjointView)
  float h[N];
  for (int i = 0; i < N - 1; ++i) {
    const int rs = N - i - 1;
    float* v = &m[(i + 1) + N * i];
    float tau, beta;
    make_householder(v, rs, tau, beta);
    v[0] = 1.0f;
    // p = tau * A_sub * v  (A_sub = lower-stored symmetric block)
    float p[N];
    for (int r = 0; r < rs; ++r) {
      float acc = 0.0f;
      for (int c = 0; c < rs; ++c) {
        const int R = i + 1 + r, Cc = i + 1 + c;
        const float a = R >= Cc ? m[R + N * Cc] : m[Cc + N * R];
        acc += a * (tau * v[c]);
      }
      p[r] = acc;
    }
    float dot = 0.0f;
    for (int r = 0; r < rs; ++r) dot += p[r] * v[r];
    const float alpha = tau * -0.5f * dot;
    for (int r = 0; r < rs; ++r) p[r] += alpha * v[r];
    // rank-2 update of the lower triangle: A -= v p' + p v'
    for (int c = 0; c < rs; ++c)
      for (int r = c; r < rs; ++r) {
        const int R = i + 1 + r, Cc = i + 1 + c;
        m[R + N * Cc] = m[R + N * Cc] - (v[r] * p[c] + p[r] * v[c]);
      }
    v[0] = beta;
    h[i] = tau;
  }
  float diag[N], sub[N];
  for (int k = 0; k < N; ++k) diag[k] = m[k + N * k];
  for (int k = 0; k < N - 1; ++k) sub[k] = m[(k + 1) + N * k];
  // Q = H_0 H_1 ... H_{N-2}, vectors stored below the subdiagonal (shift 1)
  for (int q = 0; q < N * N; ++q) V[q] = (q % (N + 1) == 0) ? 1.0f : 0.0f;
  for (int k = N - 2; k >= 0; --k) {
    const int cs = N - k - 1;  // bottom-right corner size
    const int o = k + 1;
    float ess[N];
    ess[0] = 1.0f;
    for (int q = 1; q < cs; ++q) ess[q] = m[(o + q) + N * k];
    const float tau = h[k];
    if (tau == 0.0f) continue;
    // applyHouseholderOnTheLeft on V[o.., o..]
    for (int c = 0; c < cs; ++c) {
      float t = 0.0f;
      for (int q = 1; q < cs; ++q) t += ess[q] * V[(o + q) + N * (o + c)];
      t += V[o + N * (o + c)];
      V[o + N * (o + c)] -= tau * t;
      for (int q = 1; q < cs; ++q) V[(o + q) + N * (o + c)] -= tau * ess[q] * t;
    }
  }
  const int info = compute_from_tridiagonal(diag, sub, N, V);
  for (int k = 0; k < N; ++k) evals[k] = diag[k] * scale;
  return info;
}

// ColPivHouseholderQR<Matrix<float, R, C>>(A).solve(b): least-squares x (A column-major, R x C).
// Every loop has a compile-time trip count and the pivot swap / un-permutation select by
// comparison instead of indexing with a runtime column, so on the device the arrays stay in
// registers; the arithmetic and its order are those of Eigen's algorithm.
template <int R, int C>
LLSR_HD void colpiv_qr_solve(const float* Ain, const float* b, float* x) {
  float A[R * C];
#pragma unroll
  for (int q = 0; q < R * C; ++q) A[q] = Ain[q];
  constexpr int size = R < C ? R : C;
  float hc[C], nu[C], nd[C];
  int perm[C];
#pragma unroll
  for (int k = 0; k < C; ++k) perm[k] = k;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    float sq = 0.0f;
#pragma unroll
    for (int r = 0; r < R; ++r) sq += A[r + R * k] * A[r + R * k];
    nd[k] = sqrt_(sq);
    nu[k] = nd[k];
  }
  float maxn = 0.0f;
#pragma unroll
  for (int k = 0; k < C; ++k) maxn = nu[k] > maxn ? nu[k] : maxn;
  const float eps = 1.1920929e-07f;
  const float thr_helper = (maxn * eps) * (maxn * eps) / (float)R;
  const float downdate_thr = sqrt_(eps);
  int nonzero = size;
  float maxpivot = 0.0f;
#pragma unroll
  for (int k = 0; k < size; ++k) {
    int big = k;
    float bn = nu[k];
#pragma unroll
    for (int j = k + 1; j < C; ++j)
      if (nu[j] > bn) { bn = nu[j]; big = j; }
    if (nonzero == size && bn * bn < thr_helper * (float)(R - k)) nonzero = k;
#pragma unroll
    for (int j = k + 1; j < C; ++j) {
      if (j == big) {
#pragma unroll
        for (int r = 0; r < R; ++r) { const float t = A[r + R * k]; A[r + R * k] = A[r + R * j]; A[r + R * j] = t; }
        float t = nu[k]; nu[k] = nu[j]; nu[j] = t;
        t = nd[k]; nd[k] = nd[j]; nd[j] = t;
        const int ti = perm[k]; perm[k] = perm[j]; perm[j] = ti;
      }
    }
    float tau, beta;
    make_householder(&A[k + R * k], R - k, tau, beta);
    A[k + R * k] = beta;
    if (fabs_(beta) > maxpivot) maxpivot = fabs_(beta);
    hc[k] = tau;
    // apply H_k to the remaining columns
    if (tau != 0.0f) {
#pragma unroll
      for (int j = k + 1; j < C; ++j) {
        float t = 0.0f;
#pragma unroll
        for (int r = k + 1; r < R; ++r) t += A[r + R * k] * A[r + R * j];
        t += A[k + R * j];
        A[k + R * j] -= tau * t;
#pragma unroll
        for (int r = k + 1; r < R; ++r) A[r + R * j] -= tau * A[r + R * k] * t;
      }
    }
#pragma unroll
    for (int j = k + 1; j < C; ++j) {
      if (nu[j] != 0.0f) {
        float temp = fabs_(A[k + R * j]) / nu[j];
        temp = (1.0f + temp) * (1.0f - temp);
        temp = temp < 0.0f ? 0.0f : temp;
        const float ratio = nu[j] / nd[j];
        const float temp2 = temp * (ratio * ratio);
        if (temp2 <= downdate_thr) {
          float sq = 0.0f;
#pragma unroll
          for (int r = k + 1; r < R; ++r) sq += A[r + R * j] * A[r + R * j];
          nd[j] = sqrt_(sq);
          nu[j] = nd[j];
        } else {
          nu[j] *= sqrt_(temp);
        }
      }
    }
  }
  // c = Q^T b, then solve R_top c = c, then un-permute
  float cv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) cv[r] = b[r];
#pragma unroll
  for (int k = 0; k < size; ++k) {
    const float tau = hc[k];
    if (k >= nonzero || tau == 0.0f) continue;
    float t = cv[k];
#pragma unroll
    for (int r = k + 1; r < R; ++r) t += A[r + R * k] * cv[r];
    cv[k] -= tau * t;
#pragma unroll
    for (int r = k + 1; r < R; ++r) cv[r] -= tau * A[r + R * k] * t;
  }
#pragma unroll
  for (int i = size - 1; i >= 0; --i) {
    if (i >= nonzero) continue;
    float acc = cv[i];
#pragma unroll
    for (int j = i + 1; j < size; ++j)
      if (j < nonzero) acc -= A[i + R * j] * cv[j];
    cv[i] = acc / A[i + R * i];
  }
#pragma unroll
  for (int j = 0; j < C; ++j) {
    float v = 0.0f;
#pragma unroll
    for (int i = 0; i < size; ++i)
      if (i < nonzero && perm[i] == j) v = cv[i];
    x[j] = v;
  }
}

}  // namespace llsr_eigen
