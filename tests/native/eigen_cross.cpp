// eigen_cross.cpp — TEST HARNESS (built and run by tests/test_eigen_restatement.py).
//
// Cross-checks the device's Eigen 3.3.7 restatement (lego-loam-sr_amd/csrc/llsr_eigen.h, compiled
// for the host) against the oracle's independent one (oracle/oracle_eigen.h) bit for bit, on the
// matrix shapes of the hot path: 3x3 / 6x6 normal equations (random Jacobians, rank-deficient and
// scaled ones), 5x3 plane fits, 3x3 covariances, and the degeneracy projection
// matP = matV.inverse() * matV2, matX = matP * matX2 (FA:1983-1989, MO:1530-1536).
// Prints one line per check: "<name> <cases> <mismatches>"; exit status 1 on any mismatch.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../lego-loam-sr_amd/csrc/llsr_eigen.h"
#include "../../oracle/oracle_eigen.h"

static bool same(const float* a, const float* b, int n) { return std::memcmp(a, b, sizeof(float) * n) == 0; }

struct Rng {
  std::mt19937 g;
  explicit Rng(uint32_t s) : g(s) {}
  float u(float lo, float hi) { return std::uniform_real_distribution<float>(lo, hi)(g); }
  int i(int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(g); }
};

// Normal equations of n random Jacobian rows of width W, with optional rank deficiency
// (a column scaled towards zero or two columns made dependent) and an overall scale.
template <int W>
static void normal_eq(Rng& r, float* AtA, float* AtB, int n, int mode) {
  float rows[4096 * W], b[4096];
  const float scale = std::pow(10.0f, r.u(-3.0f, 3.0f));
  for (int q = 0; q < n; ++q) {
    for (int c = 0; c < W; ++c) rows[q * W + c] = r.u(-1.0f, 1.0f) * scale;
    if (mode == 1) rows[q * W + (W - 1)] *= 1e-3f;                    // one weak direction
    if (mode == 2) rows[q * W + 1] = rows[q * W + 0] * 0.5f;          // exactly dependent columns
    if (mode == 3) for (int c = W / 2; c < W; ++c) rows[q * W + c] *= 1e-4f;  // half the directions weak
    b[q] = r.u(-0.1f, 0.1f);
  }
  oeig::gemm_ata(rows, n, W, AtA);
  oeig::gemv_atb(rows, b, n, W, AtB);
}

int main() {
  int bad_total = 0;
  auto report = [&](const char* name, int cases, int bad) {
    std::printf("%s %d %d\n", name, cases, bad);
    bad_total += bad;
  };
  Rng r(12345);
  {  // 3x3 QR solve + eig + degeneracy projection (FA)
    int bad = 0, cases = 0;
    for (int t = 0; t < 20000; ++t) {
      float AtA[9], AtB[3];
      normal_eq<3>(r, AtA, AtB, r.i(10, 800), t % 4);
      float xd[3], xo[3];
      llsr_eigen::colpiv_qr_solve<3, 3>(AtA, AtB, xd);
      oeig::colpiv_qr_solve(AtA, 3, 3, AtB, xo);
      float Ed[3], Vd[9], Eo[3], Vo[9];
      llsr_eigen::eig3(AtA, Ed, Vd);
      oeig::eig_sym3(AtA, Eo, Vo);
      float V2[9], Id[9], Io[9], Pd[9], Po[9], Xd[3], Xo[3];
      std::memcpy(V2, Vo, sizeof V2);
      for (int i = 2; i >= 0; --i) {
        if (Eo[i] < 10.0f * (t % 2 ? 1e6f : 1.0f)) { for (int j = 0; j < 3; ++j) V2[i + 3 * j] = 0.0f; }
        else break;
      }
      llsr_eigen::inverse3(Vd, Id);
      oeig::inverse3(Vo, Io);
      llsr_eigen::prod33(Id, V2, Pd);
      oeig::prod33(Io, V2, Po);
      llsr_eigen::prod31(Pd, xd, Xd);
      oeig::prod31(Po, xo, Xo);
      ++cases;
      if (!same(xd, xo, 3) || !same(Ed, Eo, 3) || !same(Vd, Vo, 9) || !same(Id, Io, 9) || !same(Pd, Po, 9) ||
          !same(Xd, Xo, 3)) {
        if (bad < 5) std::printf("  mismatch3 case %d\n", t);
        ++bad;
      }
    }
    report("fa_3x3", cases, bad);
  }
  {  // 6x6 QR solve + eig + PartialPivLU inverse + projection (MO)
    int bad = 0, cases = 0;
    for (int t = 0; t < 20000; ++t) {
      float AtA[36], AtB[6];
      normal_eq<6>(r, AtA, AtB, r.i(50, 3000), t % 4);
      float xd[6], xo[6];
      llsr_eigen::colpiv_qr_solve<6, 6>(AtA, AtB, xd);
      oeig::colpiv_qr_solve(AtA, 6, 6, AtB, xo);
      float Ed[6], Vd[36], Eo[6], Vo[36];
      llsr_eigen::eig_sym<6>(AtA, Ed, Vd);
      oeig::eig_sym_n(AtA, 6, Eo, Vo);
      float V2[36], Id[36], Io[36], Pd[36], Po[36], Xd[6], Xo[6];
      std::memcpy(V2, Vo, sizeof V2);
      for (int i = 5; i >= 0; --i) {
        if (Eo[i] < 100.0f * (t % 2 ? 1e6f : 1.0f)) { for (int j = 0; j < 6; ++j) V2[i + 6 * j] = 0.0f; }
        else break;
      }
      llsr_eigen::inverse_lu<6>(Vd, Id);
      oeig::inverse_lu(Vo, 6, Io);
      llsr_eigen::prod66(Id, V2, Pd);
      oeig::prod66(Io, V2, Po);
      llsr_eigen::prod61(Pd, xd, Xd);
      oeig::prod61(Po, xo, Xo);
      ++cases;
      if (!same(xd, xo, 6) || !same(Ed, Eo, 6) || !same(Vd, Vo, 36) || !same(Id, Io, 36) || !same(Pd, Po, 36) ||
          !same(Xd, Xo, 6)) {
        if (bad < 5) std::printf("  mismatch6 case %d (x %d e %d v %d inv %d p %d X %d)\n", t, !same(xd, xo, 6),
                                 !same(Ed, Eo, 6), !same(Vd, Vo, 36), !same(Id, Io, 36), !same(Pd, Po, 36),
                                 !same(Xd, Xo, 6));
        ++bad;
      }
    }
    report("mo_6x6", cases, bad);
  }
  {  // 5x3 plane fit (MO:1398) on near-planar, exactly planar and degenerate neighbourhoods
    int bad = 0, cases = 0;
    for (int t = 0; t < 50000; ++t) {
      float A[15];
      const float nx = r.u(-1, 1), ny = r.u(-1, 1), nz = r.u(-1, 1), d = r.u(-30, 30);
      for (int j = 0; j < 5; ++j) {
        float x = r.u(-40, 40), y = r.u(-40, 40), z;
        if (t % 3 == 0) z = r.u(-3, 3);                                   // random points
        else z = (nz != 0.0f) ? -(d + nx * x + ny * y) / nz : 0.0f;       // on a plane
        if (t % 3 == 2) { x = std::round(x * 50) / 50; y = std::round(y * 50) / 50; z = std::round(z * 50) / 50; }
        if (t % 7 == 0 && j > 0) { x = A[0]; y = A[5]; }                  // repeated xy
        A[j] = x; A[5 + j] = y; A[10 + j] = z;
      }
      const float B[5] = {-1, -1, -1, -1, -1};
      float xd[3], xo[3];
      llsr_eigen::colpiv_qr_solve<5, 3>(A, B, xd);
      oeig::colpiv_qr_solve(A, 5, 3, B, xo);
      ++cases;
      if (!same(xd, xo, 3)) { if (bad < 5) std::printf("  mismatch53 case %d\n", t); ++bad; }
    }
    report("mo_5x3", cases, bad);
  }
  {  // 3x3 covariance eigen (MO:1320): 5 points on / near a line
    int bad = 0, cases = 0;
    for (int t = 0; t < 50000; ++t) {
      float px[5], py[5], pz[5];
      const float dx = r.u(-1, 1), dy = r.u(-1, 1), dz = r.u(-1, 1), cx = r.u(-50, 50), cy = r.u(-50, 50);
      for (int j = 0; j < 5; ++j) {
        const float s = r.u(-0.5f, 0.5f), n = (t % 2) ? r.u(-0.01f, 0.01f) : 0.0f;
        px[j] = cx + s * dx + n; py[j] = cy + s * dy - n; pz[j] = s * dz + n;
      }
      float mx = 0, my = 0, mz = 0;
      for (int j = 0; j < 5; ++j) { mx += px[j]; my += py[j]; mz += pz[j]; }
      mx /= 5; my /= 5; mz /= 5;
      float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
      for (int j = 0; j < 5; ++j) {
        const float ax = px[j] - mx, ay = py[j] - my, az = pz[j] - mz;
        a11 += ax * ax; a12 += ax * ay; a13 += ax * az; a22 += ay * ay; a23 += ay * az; a33 += az * az;
      }
      const float A[9] = {a11 / 5, a12 / 5, a13 / 5, a12 / 5, a22 / 5, a23 / 5, a13 / 5, a23 / 5, a33 / 5};
      float Ed[3], Vd[9], Eo[3], Vo[9];
      llsr_eigen::eig3(A, Ed, Vd);
      oeig::eig_sym3(A, Eo, Vo);
      ++cases;
      if (!same(Ed, Eo, 3) || !same(Vd, Vo, 9)) { if (bad < 5) std::printf("  mismatch_cov case %d\n", t); ++bad; }
    }
    report("mo_cov3", cases, bad);
  }
  {  // gemm_kc against the oracle's statement over every depth of interest
    int bad = 0;
    for (int k = 1; k < 20000; ++k)
      if (llsr_eigen::gemm_kc(k, 3, 3) != oeig::gemm_kc(k, 3, 3) || llsr_eigen::gemm_kc(k, 6, 6) != oeig::gemm_kc(k, 6, 6))
        ++bad;
    report("gemm_kc", 19999, bad);
  }
  return bad_total ? 1 : 0;
}
