// llsr_eigen.h — the Eigen 3.3.7 dense routines of the hot path, in float, on host and device:
//   * ColPivHouseholderQR<Matrix<float,R,C>>::solve   FA:1956 / 2094 (3x3), MO:1398 (5x3), MO:1505 (6x6)
//   * SelfAdjointEigenSolver<Matrix3f>                FA:1966 / 2101, MO:1320
//   * SelfAdjointEigenSolver<Matrix<float,6,6>>       MO:1512
//   * MatrixBase::inverse()                           FA:1983 / 2118 (3x3 cofactors), MO:1530 (6x6,
//                                                     PartialPivLU)
//   * the lazy products matV.inverse() * matV2 and matP * matX2 (FA:1983-1989, MO:1530-1536)
//   * the depth blocking of Eigen's GEMM for matAt * matA (FA:1954 / 2092)
//
// Restates the algorithms of Eigen 3.3.7 (MPL-2.0, http://eigen.tuxfamily.org; Eigen is absent
// from this image) as the reference's build runs them — GCC -O3, baseline x86-64: SSE2 Packet4f,
// no FMA — including the order in which each reduction adds (the kernel Eigen dispatches to
// decides it: Redux.h, GeneralMatrixVector.h, SelfadjointMatrixVector.h, ProductEvaluators.h).
// The oracle restates the same routines independently (oracle/oracle_eigen.h); the two are
// cross-checked bit for bit on random and rank-deficient matrices by tests/test_eigen_restatement.py.
//
// Every loop has a compile-time trip count (or is fully unrolled), so on the device the matrices
// stay in registers; runtime column indices are replaced by compare-and-select.
#pragma once
#include <stdint.h>

#include "llsr_libm.h"

namespace llsr_eigen {

using llsr_libm::fabs_;
using llsr_libm::sqrt_;

constexpr float kEps = 1.1920928955078125e-07f;   // NumTraits<float>::epsilon()
constexpr float kMin = 1.17549435082228751e-38f;  // numeric_limits<float>::min()

// ---- Redux.h --------------------------------------------------------------------------------
// fixed size, not vectorised: redux_novec_unroller adds the two halves
template <int N>
LLSR_HD float sum_halves(const float* e) {
  if constexpr (N == 0) return 0.0f;
  else if constexpr (N == 1) return e[0];
  else return sum_halves<N / 2>(e) + sum_halves<N - N / 2>(e + N / 2);
}
// predux<Packet4f>
LLSR_HD float predux(float a0, float a1, float a2, float a3) { return (a0 + a2) + (a1 + a3); }
// fixed size, vectorised (N < 8): one packet, predux, tail by halves
template <int N>
LLSR_HD float sum_fixed(const float* e) {
  static_assert(N < 8, "one packet at most");
  if constexpr (N < 4) return sum_halves<N>(e);
  else if constexpr (N == 4) return predux(e[0], e[1], e[2], e[3]);
  else return predux(e[0], e[1], e[2], e[3]) + sum_halves<N - 4>(e + 4);
}
// dynamic size, vectorised expression (n < 8, alignedStart 0): a packet when n >= 4, then the
// tail one by one; below one packet, left to right
LLSR_HD float sum_dyn(const float* e, int n) {
  if (n <= 0) return 0.0f;
  if (n >= 4) {
    float r = predux(e[0], e[1], e[2], e[3]);
#pragma unroll
    for (int i = 4; i < 8; ++i)
      if (i < n) r = r + e[i];
    return r;
  }
  float r = e[0];
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < n) r = r + e[i];
  return r;
}

// ---- GeneralMatrixVector.h: the alignment peeling of the row-major GEMV ----------------------
LLSR_HD constexpr int first_aligned(int off, int size) {
  return ((4 - (off & 3)) & 3) < size ? ((4 - (off & 3)) & 3) : size;
}
struct GemvPlan { int a0, a1; };  // scalar head [0, a0), packet body [a0, a1), scalar tail
LLSR_HD constexpr GemvPlan gemv_plan(int loff0, int boff, int d, int rows) {
  return (first_aligned(loff0, d) == d || first_aligned(boff, rows) == rows)
             ? GemvPlan{0, 0}
             : GemvPlan{first_aligned(boff, d), first_aligned(boff, d) + ((d - first_aligned(boff, d)) & ~3)};
}

// ---- Householder.h ----------------------------------------------------------------------------
// makeHouseholderInPlace on v[0..n) (n <= 6, compile-time after unrolling)
LLSR_HD void make_householder(float* v, int n, float& tau, float& beta) {
  float sq[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) sq[q] = q + 1 < n ? v[q + 1] * v[q + 1] : 0.0f;
  const float tailSq = n > 1 ? sum_dyn(sq, n - 1) : 0.0f;
  const float c0 = v[0];
  if (tailSq <= kMin) {
    tau = 0.0f;
    beta = c0;
#pragma unroll
    for (int q = 1; q < 6; ++q)
      if (q < n) v[q] = 0.0f;
  } else {
    beta = sqrt_(c0 * c0 + tailSq);
    if (c0 >= 0.0f) beta = -beta;
    const float den = c0 - beta;
#pragma unroll
    for (int q = 1; q < 6; ++q)
      if (q < n) v[q] = v[q] / den;
    tau = (beta - c0) / beta;
  }
}

// applyHouseholderOnTheLeft(essential, tau) on the rows x cols block at M (leading dimension LD,
// element (0,0) at float offset moff of aligned storage, essential at eoff), the GEMV flavour
// (cols is dynamic at compile time in every caller).
template <int LD>
LLSR_HD void apply_householder_gemv(float* M, int moff, int rows, int cols, const float* ess, int eoff, float tau) {
  if (rows == 1) {
    const float f = 1.0f - tau;
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (j < cols) M[j * LD] = M[j * LD] * f;
    return;
  }
  if (tau == 0.0f) return;
  const int d = rows - 1;
  const GemvPlan g = gemv_plan(moff + 1, eoff, d, cols);
  float tmp[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    if (j >= cols) continue;
    const float* l = M + 1 + j * LD;
    float t = 0.0f;
#pragma unroll
    for (int q = 0; q < 5; ++q)
      if (q < g.a0 && q < d) t = t + l[q] * ess[q];
    if (g.a1 > g.a0) {
      float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int q = 0; q < 5; ++q)
        if (q >= g.a0 && q < g.a1) p[(q - g.a0) & 3] = l[q] * ess[q] + p[(q - g.a0) & 3];
      t = t + predux(p[0], p[1], p[2], p[3]);
    }
#pragma unroll
    for (int q = 0; q < 5; ++q)
      if (q >= g.a1 && q < d) t = t + l[q] * ess[q];
    tmp[j] = 0.0f + t;
  }
#pragma unroll
  for (int j = 0; j < 6; ++j)
    if (j < cols) {
      tmp[j] = tmp[j] + M[j * LD];
      M[j * LD] = M[j * LD] - tau * tmp[j];
    }
  float tess[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) tess[q] = q < d ? tau * ess[q] : 0.0f;
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int q = 0; q < 5; ++q)
      if (j < cols && q < d) M[1 + q + j * LD] = M[1 + q + j * LD] - tmp[j] * tess[q];
}

// ---- ColPivHouseholderQR.h: computeInPlace + solve(b) -----------------------------------------
// A column-major R x C (R >= C, C <= 6). The storage is Matrix<float,R,C> (16-byte aligned when
// R*C*4 is a multiple of 16, which is the only case where the GEMV peeling can reach a packet).
template <int R, int C>
LLSR_HD void colpiv_qr_solve(const float* Ain, const float* b, float* x) {
  float A[R * C];
#pragma unroll
  for (int q = 0; q < R * C; ++q) A[q] = Ain[q];
  constexpr int size = R < C ? R : C;
  float hc[C], nu[C], nd[C];
  int perm[C], tr[C];
#pragma unroll
  for (int k = 0; k < C; ++k) {  // m_qr.col(k).norm(): fixed-size column
    float sq[R];
#pragma unroll
    for (int r = 0; r < R; ++r) sq[r] = A[r + R * k] * A[r + R * k];
    nd[k] = sqrt_(sum_fixed<R>(sq));
    nu[k] = nd[k];
  }
  float maxn = nu[0];
#pragma unroll
  for (int k = 1; k < C; ++k) maxn = nu[k] > maxn ? nu[k] : maxn;
  const float me = maxn * kEps;
  const float thr_helper = me * me / (float)R;
  const float downdate_thr = sqrt_(kEps);
  int nonzero = size;
#pragma unroll
  for (int k = 0; k < size; ++k) {
    int big = k;
    float bn = nu[k];
#pragma unroll
    for (int j = k + 1; j < C; ++j)
      if (nu[j] > bn) { bn = nu[j]; big = j; }
    if (nonzero == size && bn * bn < thr_helper * (float)(R - k)) nonzero = k;
    tr[k] = big;
#pragma unroll
    for (int j = k + 1; j < C; ++j) {
      if (j == big) {
#pragma unroll
        for (int r = 0; r < R; ++r) { const float t = A[r + R * k]; A[r + R * k] = A[r + R * j]; A[r + R * j] = t; }
        float t = nu[k]; nu[k] = nu[j]; nu[j] = t;
        t = nd[k]; nd[k] = nd[j]; nd[j] = t;
      }
    }
    float beta;
    make_householder(&A[k + R * k], R - k, hc[k], beta);
    A[k + R * k] = beta;
    if (k + 1 < C) apply_householder_gemv<R>(&A[k + R * (k + 1)], k + R * (k + 1), R - k, C - k - 1, &A[k + 1 + R * k],
                                             k + 1 + R * k, hc[k]);
#pragma unroll
    for (int j = k + 1; j < C; ++j) {
      if (nu[j] != 0.0f) {
        float temp = fabs_(A[k + R * j]) / nu[j];
        temp = (1.0f + temp) * (1.0f - temp);
        temp = temp < 0.0f ? 0.0f : temp;
        const float ratio = nu[j] / nd[j];
        const float temp2 = temp * (ratio * ratio);
        if (temp2 <= downdate_thr) {
          float sq[R];
#pragma unroll
          for (int r = 0; r < R; ++r) sq[r] = r < R - k - 1 ? A[k + 1 + r + R * j] * A[k + 1 + r + R * j] : 0.0f;
          nd[j] = sqrt_(sum_dyn(sq, R - k - 1));
          nu[j] = nd[j];
        } else {
          nu[j] = nu[j] * sqrt_(temp);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < C; ++k) perm[k] = k;
#pragma unroll
  for (int k = 0; k < size; ++k)
#pragma unroll
    for (int j = k + 1; j < C; ++j)
      if (j == tr[k]) { const int t = perm[k]; perm[k] = perm[j]; perm[j] = t; }
  if (nonzero == 0) {
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = 0.0f;
    return;
  }
  // c = Q^T b: H_k applied with the InnerProduct form (the rhs is a vector)
  float c[R];
#pragma unroll
  for (int r = 0; r < R; ++r) c[r] = b[r];
#pragma unroll
  for (int k = 0; k < size; ++k) {
    if (k >= nonzero) continue;
    const float tau = hc[k];
    if (R - k == 1) {
      c[k] = c[k] * (1.0f - tau);
      continue;
    }
    if (tau == 0.0f) continue;
    float e[R];
#pragma unroll
    for (int q = 0; q < R; ++q) e[q] = q < R - k - 1 ? A[k + 1 + q + R * k] * c[k + 1 + q] : 0.0f;
    const float t = sum_dyn(e, R - k - 1) + c[k];
    c[k] = c[k] - tau * t;
#pragma unroll
    for (int q = 0; q < R; ++q)
      if (q < R - k - 1) c[k + 1 + q] = c[k + 1 + q] - t * (tau * A[k + 1 + q + R * k]);
  }
  // triangular_solve_vector<Upper, ColMajor>: column-oriented, from the last row up
#pragma unroll
  for (int i = size - 1; i >= 0; --i) {
    if (i >= nonzero) continue;
    if (c[i] != 0.0f) {
      c[i] = c[i] / A[i + R * i];
#pragma unroll
      for (int q = 0; q < size; ++q)
        if (q < i) c[q] = c[q] - c[i] * A[q + R * i];
    }
  }
#pragma unroll
  for (int j = 0; j < C; ++j) {
    float v = 0.0f;
#pragma unroll
    for (int i = 0; i < size; ++i)
      if (i < nonzero && perm[i] == j) v = c[i];
    x[j] = v;
  }
}

// ---- SelfAdjointEigenSolver.h -------------------------------------------------------------
LLSR_HD float hypot_(float x, float y) {  // internal::hypot_impl
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

// internal::tridiagonal_qr_step (ColMajor); Q n x n column-major, Q = Q * G
template <int N>
LLSR_HD void tridiagonal_qr_step(float* diag, float* subdiag, int start, int end, float* Q) {
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
    // applyOnTheRight(k, k+1, rot): apply_rotation_in_the_plane with (c, -s), which returns
    // early for the identity rotation
    if (c == 1.0f && s == 0.0f) continue;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const float xi = Q[i + k * N], yi = Q[i + (k + 1) * N];
      Q[i + k * N] = c * xi + (-s) * yi;
      Q[i + (k + 1) * N] = -(-s) * xi + c * yi;
    }
  }
}

// computeFromTridiagonal_impl (Eigen 3.3.7 deflation test) + ascending sort; 0 = Success.
template <int N>
LLSR_HD int compute_from_tridiagonal(float* diag, float* subdiag, float* Q) {
  const float precision = 2.0f * kEps;
  const int maxIterations = 30;
  int end = N - 1, start = 0, iter = 0;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (fabs_(subdiag[i]) <= (fabs_(diag[i]) + fabs_(diag[i + 1])) * precision || fabs_(subdiag[i]) <= kMin)
        subdiag[i] = 0.0f;
    while (end > 0 && subdiag[end - 1] == 0.0f) end--;
    if (end <= 0) break;
    iter++;
    if (iter > maxIterations * N) break;
    start = end - 1;
    while (start > 0 && subdiag[start - 1] != 0.0f) start--;
    tridiagonal_qr_step<N>(diag, subdiag, start, end, Q);
  }
  const int info = iter <= maxIterations * N ? 0 : 1;
  if (info == 0) {
    for (int i = 0; i < N - 1; ++i) {
      int k = 0;  // minCoeff(&k) over segment(i, N-i): first minimum
      float m = diag[i];
      for (int q = 1; q < N - i; ++q)
        if (diag[i + q] < m) { m = diag[i + q]; k = q; }
      if (k > 0) {
        const float t = diag[i]; diag[i] = diag[k + i]; diag[k + i] = t;
#pragma unroll
        for (int r = 0; r < N; ++r) {
          const float u = Q[r + i * N]; Q[r + i * N] = Q[r + (k + i) * N]; Q[r + (k + i) * N] = u;
        }
      }
    }
  }
  return info;
}

template <int N>
LLSR_HD float scale_lower(const float* A, float* m) {
#pragma unroll
  for (int c = 0; c < N; ++c)
#pragma unroll
    for (int r = 0; r < N; ++r) m[r + N * c] = r >= c ? A[r + N * c] : 0.0f;  // triangularView<Lower>
  float scale = 0.0f;
#pragma unroll
  for (int q = 0; q < N * N; ++q) scale = fabs_(m[q]) > scale ? fabs_(m[q]) : scale;
  if (scale == 0.0f) scale = 1.0f;
#pragma unroll
  for (int c = 0; c < N; ++c)
#pragma unroll
    for (int r = c; r < N; ++r) m[r + N * c] /= scale;
  return scale;
}

// SelfAdjointEigenSolver<Matrix3f>::compute on the lower triangle of A (column-major).
// evals ascending; evecs column-major (eigenvector k = column k).
LLSR_HD int eig3(const float* A, float* evals, float* V) {
  float m[9];
  const float scale = scale_lower<3>(A, m);
  float diag[3], sub[2];
  // tridiagonalization_inplace_selector<MatrixType, 3, false>
  diag[0] = m[0];
  const float v1norm2 = m[2] * m[2];  // mat(2,0)
  if (v1norm2 <= kMin) {
    diag[1] = m[4];
    diag[2] = m[8];
    sub[0] = m[1];
    sub[1] = m[5];
#pragma unroll
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
  const int info = compute_from_tridiagonal<3>(diag, sub, V);
#pragma unroll
  for (int k = 0; k < 3; ++k) evals[k] = diag[k] * scale;
  return info;
}

// SelfAdjointEigenSolver<Matrix<float,N,N>> (4 <= N <= 6): tridiagonalization_inplace — for
// each column a Householder reflector, p = h * A v by selfadjoint_matrix_vector_product's
// column loop (size <= 8), p += (h * -0.5 * p.v) v, the rank-2 update — then the in-place
// HouseholderSequence evaluation of Q (m_eivec, aligned) and the QR iteration.
template <int N>
LLSR_HD int eig_sym(const float* A, float* evals, float* V) {
  float* m = V;
  const float scale = scale_lower<N>(A, m);
  float h[N];
#pragma unroll
  for (int i = 0; i < N - 1; ++i) {
    const int rs = N - i - 1;
    float* v = &m[(i + 1) + N * i];
    float tau, beta;
    make_householder(v, rs, tau, beta);
    v[0] = 1.0f;
    float p[N];
#pragma unroll
    for (int r = 0; r < N; ++r) p[r] = 0.0f;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j >= rs) continue;
      const float t1 = tau * v[j];
      float t2 = 0.0f;
      p[j] = p[j] + m[(i + 1 + j) + N * (i + 1 + j)] * t1;
#pragma unroll
      for (int r = 0; r < N; ++r) {
        if (r <= j || r >= rs) continue;
        const float a = m[(i + 1 + r) + N * (i + 1 + j)];
        p[r] = p[r] + a * t1;
        t2 = t2 + a * v[r];
      }
      p[j] = p[j] + tau * t2;
    }
    float e[N];
#pragma unroll
    for (int r = 0; r < N; ++r) e[r] = r < rs ? p[r] * v[r] : 0.0f;
    const float s = (tau * -0.5f) * sum_dyn(e, rs);
#pragma unroll
    for (int r = 0; r < N; ++r)
      if (r < rs) p[r] = p[r] + s * v[r];
#pragma unroll
    for (int c = 0; c < N; ++c)
#pragma unroll
      for (int r = 0; r < N; ++r) {
        if (c >= rs || r < c || r >= rs) continue;
        float& a = m[(i + 1 + r) + N * (i + 1 + c)];
        a = a + ((-v[c]) * p[r] + (-p[c]) * v[r]);
      }
    v[0] = beta;
    h[i] = tau;
  }
  float diag[N], sub[N];
#pragma unroll
  for (int k = 0; k < N; ++k) diag[k] = m[k + N * k];
#pragma unroll
  for (int k = 0; k < N - 1; ++k) sub[k] = m[(k + 1) + N * k];
  sub[N - 1] = 0.0f;
#pragma unroll
  for (int k = 0; k < N; ++k) m[k + N * k] = 1.0f;
#pragma unroll
  for (int c = 1; c < N; ++c)
#pragma unroll
    for (int r = 0; r < c; ++r) m[r + N * c] = 0.0f;
#pragma unroll
  for (int k = N - 2; k >= 0; --k) {
    const int cs = N - k - 1, o = k + 1;
    apply_householder_gemv<N>(&m[o + N * o], o + N * o, cs, cs, &m[(k + 2) + N * k], (k + 2) + N * k, h[k]);
#pragma unroll
    for (int r = 0; r < N; ++r)
      if (r > k) m[r + N * k] = 0.0f;
  }
  const int info = compute_from_tridiagonal<N>(diag, sub, m);
#pragma unroll
  for (int k = 0; k < N; ++k) evals[k] = diag[k] * scale;
  return info;
}

// ---- InverseImpl.h: matV.inverse() --------------------------------------------------------------
// compute_inverse<3>: cofactor_3x3, det = c0*m00 + (c1*m10 + c2*m20), inv(i,j) = cof(j,i) / det
LLSR_HD void inverse3(const float* m, float* inv) {
#define LLSR_M(r, c) m[(r) + 3 * (c)]
#define LLSR_COF(i, j)                                                                       \
  (LLSR_M(((i) + 1) % 3, ((j) + 1) % 3) * LLSR_M(((i) + 2) % 3, ((j) + 2) % 3) -            \
   LLSR_M(((i) + 1) % 3, ((j) + 2) % 3) * LLSR_M(((i) + 2) % 3, ((j) + 1) % 3))
  const float c0 = LLSR_COF(0, 0), c1 = LLSR_COF(1, 0), c2 = LLSR_COF(2, 0);
  const float det = c0 * LLSR_M(0, 0) + (c1 * LLSR_M(1, 0) + c2 * LLSR_M(2, 0));
  const float invdet = 1.0f / det;
  inv[0] = c0 * invdet; inv[3] = c1 * invdet; inv[6] = c2 * invdet;
  inv[1] = LLSR_COF(0, 1) * invdet; inv[4] = LLSR_COF(1, 1) * invdet; inv[7] = LLSR_COF(2, 1) * invdet;
  inv[2] = LLSR_COF(0, 2) * invdet; inv[5] = LLSR_COF(1, 2) * invdet; inv[8] = LLSR_COF(2, 2) * invdet;
#undef LLSR_COF
#undef LLSR_M
}

// compute_inverse<Dynamic>: partialPivLu().inverse() = PartialPivLU::solve(Identity) —
// unblocked_lu (first maximal |pivot|, full row swap, column divided by the pivot, rank-1
// update), P * I, then triangular_solve_matrix UnitLower and Upper (one small panel,
// column-oriented, reciprocal of the diagonal).
template <int N>
LLSR_HD void inverse_lu(const float* m, float* inv) {
  float lu[N * N];
#pragma unroll
  for (int q = 0; q < N * N; ++q) lu[q] = m[q];
  int tr[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    int row = k;
    float big = fabs_(lu[k + N * k]);
#pragma unroll
    for (int r = k + 1; r < N; ++r)
      if (fabs_(lu[r + N * k]) > big) { big = fabs_(lu[r + N * k]); row = r; }
    tr[k] = row;
    if (big != 0.0f) {
#pragma unroll
      for (int r = k + 1; r < N; ++r)
        if (r == row)
#pragma unroll
          for (int c = 0; c < N; ++c) { const float t = lu[k + N * c]; lu[k + N * c] = lu[r + N * c]; lu[r + N * c] = t; }
      const float piv = lu[k + N * k];
#pragma unroll
      for (int r = k + 1; r < N; ++r) lu[r + N * k] = lu[r + N * k] / piv;
    }
#pragma unroll
    for (int c = k + 1; c < N; ++c)
#pragma unroll
      for (int r = k + 1; r < N; ++r) lu[r + N * c] = lu[r + N * c] - lu[r + N * k] * lu[k + N * c];
  }
#pragma unroll
  for (int q = 0; q < N * N; ++q) inv[q] = (q % (N + 1) == 0) ? 1.0f : 0.0f;
#pragma unroll
  for (int k = 0; k < N; ++k)
#pragma unroll
    for (int r = k + 1; r < N; ++r)
      if (r == tr[k])
#pragma unroll
        for (int c = 0; c < N; ++c) { const float t = inv[k + N * c]; inv[k + N * c] = inv[r + N * c]; inv[r + N * c] = t; }
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float b = inv[i + N * j] * 1.0f;
#pragma unroll
      for (int r = i + 1; r < N; ++r) inv[r + N * j] = inv[r + N * j] - b * lu[r + N * i];
    }
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    const float a = 1.0f / lu[i + N * i];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      inv[i + N * j] = inv[i + N * j] * a;
      const float b = inv[i + N * j];
#pragma unroll
      for (int r = 0; r < i; ++r) inv[r + N * j] = inv[r + N * j] - b * lu[r + N * i];
    }
  }
}

// ---- ProductEvaluators.h: the lazy products after the inverse ------------------------------------
// scalar coefficient (lhs.row(r)' .* rhs.col(c)).sum() by halves; packet lane: pmul, then pmadd in k order
template <int N>
LLSR_HD float lazy_coeff(const float* L, int r, const float* Rc) {
  float e[N];
#pragma unroll
  for (int k = 0; k < N; ++k) e[k] = L[r + N * k] * Rc[k];
  return sum_halves<N>(e);
}
template <int N>
LLSR_HD float lazy_lane(const float* L, int r, const float* Rc) {
  float acc = L[r] * Rc[0];
#pragma unroll
  for (int k = 1; k < N; ++k) acc = L[r + N * k] * Rc[k] + acc;
  return acc;
}
// matP = matV.inverse() * matV2 and matX = matP * matX2 for 3x3 (FA): every coefficient scalar
LLSR_HD void prod33(const float* A, const float* B, float* out) {
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) out[r + 3 * c] = lazy_coeff<3>(A, r, &B[3 * c]);
}
LLSR_HD void prod31(const float* A, const float* x, float* out) {
#pragma unroll
  for (int r = 0; r < 3; ++r) out[r] = lazy_coeff<3>(A, r, x);
}
// 6x6 (MO): the aliasing temporary is assigned by slices — even columns rows 0-3 by packet,
// odd columns rows 2-5 — and the 6x1 product rows 0-3 by packet, rows 4-5 scalar
LLSR_HD void prod66(const float* A, const float* B, float* out) {
#pragma unroll
  for (int c = 0; c < 6; ++c)
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const int p0 = (c & 1) ? 2 : 0;
      out[r + 6 * c] = (r >= p0 && r < p0 + 4) ? lazy_lane<6>(A, r, &B[6 * c]) : lazy_coeff<6>(A, r, &B[6 * c]);
    }
}
LLSR_HD void prod61(const float* A, const float* x, float* out) {
#pragma unroll
  for (int r = 0; r < 6; ++r) out[r] = r < 4 ? lazy_lane<6>(A, r, x) : lazy_coeff<6>(A, r, x);
}

// ---- GeneralMatrixMatrix.h: the depth block kc of matAt * matA -------------------------------------
// evaluateProductBlockingSizesHeuristic (single thread, SSE: mr = 8, nr = 4, KcFactor 1) for an
// m x n result of depth k with a `l1`-byte L1 data cache (32 KiB assumed; CPU-dependent in the
// reference, which queries CPUID). Each block's products are summed from zero and added to the
// result. Below `rows + 2*cols < 20` Eigen uses the lazy coefficient product (no blocks).
LLSR_HD int gemm_kc(int k, int m, int n, int l1 = 32 * 1024) {
  const int mx = k > m ? (k > n ? k : n) : (m > n ? m : n);
  if (mx < 48) return k;
  int max_kc = ((l1 - 8 * 4 * 4) / (8 * 4 + 4 * 4)) & ~7;
  if (max_kc < 1) max_kc = 1;
  if (k <= max_kc) return k;
  return (k % max_kc) == 0 ? max_kc : max_kc - 8 * ((max_kc - 1 - (k % max_kc)) / (8 * (k / max_kc + 1)));
}

}  // namespace llsr_eigen
