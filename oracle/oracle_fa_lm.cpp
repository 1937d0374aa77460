// oracle_fa_lm.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Scalar CPU restatement of FeatureAssociation::updateTransformation (FA = featureAssociation.cpp:
// 2505-2535): TransformToStart (FA:1389-1412), findCorrespondingSurfFeatures (FA:1699-1844),
// calculateTransformationSurf (FA:1846-2010), findCorrespondingCornerFeatures (FA:1580-1697),
// calculateTransformationCorner (FA:2013-2143); plus TransformToEnd (FA:1414-1490, no-IMU
// branch) and GenerateShadowPoint (FA:412-439) that produce its inputs.
//
// Float/double typing follows each reference line (float sin/cos/sqrt overloads, double
// literals 1.8 / 0.05 / 2.5 promote). kNN-1 (nanoflann KdTreeFLANN::nearestKSearch(k = 1)) is
// an exact brute-force minimum with strict '<' in index order: equal distances keep the lower
// index (nanoflann keeps the first found in tree order; equal float distances are measure-zero
// on the synthetic scenes). Built a second time against the reference's own nanoflann.hpp
// (-DLLSR_ORACLE_NANOFLANN, oracle/_ref) as a cross-check.
//
// Reference undefined behaviour, restated deterministically and documented in DESIGN.md:
//   * the forward neighbour scans are bounded by the CURRENT query count (`j < cornerPointsSharpNum`
//     FA:1599, `j < surfPointsFlatNum` FA:1742), not the last cloud's size; when that bound
//     exceeds the last cloud the reference reads past its end — clamped here;
//   * matP is an uninitialised local at iterCount >= 1 (FA:1856, 2022); it holds, in practice,
//     what the previous call left in the same stack slot, i.e. the iteration-0 value of the
//     phase — restated that way (identity if iteration 0 of the phase built no system).
#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>

#include "../include/llsr.h"
#include "oracle.h"
#include "oracle_eigen.h"
#ifdef LLSR_ORACLE_NANOFLANN
#include "nanoflann.hpp"
#endif

namespace {

struct P4 { float x, y, z, i; };

#ifdef LLSR_ORACLE_NANOFLANN
struct CloudAdaptor {
  const P4* pts = nullptr;
  size_t n = 0;
  size_t kdtree_get_point_count() const { return n; }
  float kdtree_get_pt(const size_t idx, int dim) const { return (&pts[idx].x)[dim]; }
  template <class BBOX> bool kdtree_get_bbox(BBOX&) const { return false; }
};
using KdTree = nanoflann::KDTreeSingleIndexAdaptor<nanoflann::SO3_Adaptor<float, CloudAdaptor>, CloudAdaptor, 3, int>;
struct Nn1 {
  CloudAdaptor ad;
  KdTree* tree = nullptr;
  ~Nn1() { delete tree; }
  void build(const P4* p, int n) {
    ad.pts = p;
    ad.n = (size_t)n;
    delete tree;
    tree = new KdTree(3, ad);
    tree->buildIndex();
  }
  void query(const P4& q, int& idx, float& d2) const {
    nanoflann::KNNResultSet<float, int> rs(1);
    rs.init(&idx, &d2);
    tree->findNeighbors(rs, &q.x, nanoflann::SearchParams());
  }
};
#define ORACLE_FN(name) ref_##name
#else
struct Nn1 {  // exact nearest neighbour, lowest index on ties
  const P4* pts = nullptr;
  int n = 0;
  void build(const P4* p, int np) { pts = p; n = np; }
  void query(const P4& q, int& idx, float& d2) const {
    idx = -1;
    d2 = INFINITY;
    for (int k = 0; k < n; ++k) {
      float d = 0.0f, t;  // nanoflann L2_Simple accumulation order
      t = q.x - pts[k].x; d += t * t;
      t = q.y - pts[k].y; d += t * t;
      t = q.z - pts[k].z; d += t * t;
      if (d < d2) { d2 = d; idx = k; }
    }
  }
};
#define ORACLE_FN(name) oracle_##name
#endif

struct Coeff { P4 ori; float cx, cy, cz, ci; };

struct S2S {
  const llsr_config* cfg;
  float t[6];              // transformCur
  bool isDegenerate;
  float matP[9];           // column-major
  const P4 *sharp, *flat, *cl, *sl;
  int Ms, F, Nc, Ns;
  Nn1 kc, ks;
  std::vector<int> ci1, ci2, si1, si2, si3;  // pointSearchCornerInd1/2, pointSearchSurfInd1/2/3
  std::vector<Coeff> sel;
  float distSqr;

  // TransformToStart (FA:1389-1412)
  P4 to_start(const P4& pi) const {
    const float s = 10 * (pi.i - (float)(int)pi.i);
    const float rx = s * t[0], ry = s * t[1], rz = s * t[2];
    const float tx = s * t[3], ty = s * t[4], tz = s * t[5];
    const float x1 = std::cos(rz) * (pi.x - tx) + std::sin(rz) * (pi.y - ty);
    const float y1 = -std::sin(rz) * (pi.x - tx) + std::cos(rz) * (pi.y - ty);
    const float z1 = (pi.z - tz);
    const float x2 = x1;
    const float y2 = std::cos(rx) * y1 + std::sin(rx) * z1;
    const float z2 = -std::sin(rx) * y1 + std::cos(rx) * z1;
    P4 po;
    po.x = std::cos(ry) * x2 - std::sin(ry) * z2;
    po.y = y2;
    po.z = std::sin(ry) * x2 + std::cos(ry) * z2;
    po.i = pi.i;
    return po;
  }

  static float sqdis(const P4& a, const P4& b) {
    return (a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z);
  }

  // findCorrespondingCornerFeatures (FA:1580-1697)
  void corner_corr(int iterCount) {
    for (int i = 0; i < Ms; ++i) {
      const P4 pointSel = to_start(sharp[i]);
      if (iterCount % 5 == 0) {
        int nn;
        float nd;
        kc.query(pointSel, nn, nd);
        int closestPointInd = -1, minPointInd2 = -1;
        if (nd < distSqr) {
          closestPointInd = nn;
          const int closestPointScan = (int)cl[closestPointInd].i;
          float minPointSqDis2 = distSqr;
          const int fwd_end = Ms < Nc ? Ms : Nc;  // reference bound j < cornerPointsSharpNum (clamped)
          for (int j = closestPointInd + 1; j < fwd_end; j++) {
            if ((double)(int)cl[j].i > closestPointScan + 2.5) break;
            const float d = sqdis(cl[j], pointSel);
            if ((int)cl[j].i > closestPointScan && d < minPointSqDis2) { minPointSqDis2 = d; minPointInd2 = j; }
          }
          for (int j = closestPointInd - 1; j >= 0; j--) {
            if ((double)(int)cl[j].i < closestPointScan - 2.5) break;
            const float d = sqdis(cl[j], pointSel);
            if ((int)cl[j].i < closestPointScan && d < minPointSqDis2) { minPointSqDis2 = d; minPointInd2 = j; }
          }
        }
        ci1[i] = closestPointInd;
        ci2[i] = minPointInd2;
      }
      if (ci2[i] >= 0) {
        const P4 t1 = cl[ci1[i]], t2 = cl[ci2[i]];
        const float x0 = pointSel.x, y0 = pointSel.y, z0 = pointSel.z;
        const float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
        const float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
        const float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
        const float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
        const float a012 = std::sqrt(m11 * m11 + m22 * m22 + m33 * m33);
        const float l12 = std::sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
        const float la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
        const float lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
        const float lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
        const float ld2 = a012 / l12;
        float s = 1;
        if (iterCount >= 5) s = (float)(1 - 1.8 * (double)std::fabs(ld2));
        if ((double)s > 0.1 && ld2 != 0) sel.push_back({sharp[i], s * la, s * lb, s * lc, s * ld2});
      }
    }
  }

  // findCorrespondingSurfFeatures (FA:1699-1844)
  void surf_corr(int iterCount) {
    for (int i = 0; i < F; ++i) {
      const P4 pointSel = to_start(flat[i]);
      if (iterCount % 5 == 0) {
        int nn;
        float nd;
        ks.query(pointSel, nn, nd);
        int closestPointInd = -1, minPointInd2 = -1, minPointInd3 = -1;
        if (nd < distSqr) {
          closestPointInd = nn;
          const int closestPointScan = (int)sl[closestPointInd].i;
          float minPointSqDis2 = distSqr, minPointSqDis3 = distSqr;
          const int fwd_end = F < Ns ? F : Ns;  // reference bound j < surfPointsFlatNum (clamped)
          for (int j = closestPointInd + 1; j < fwd_end; j++) {
            if ((double)(int)sl[j].i > closestPointScan + 2.5) break;
            const float d = sqdis(sl[j], pointSel);
            if ((int)sl[j].i <= closestPointScan) {
              if (d < minPointSqDis2) { minPointSqDis2 = d; minPointInd2 = j; }
            } else {
              if (d < minPointSqDis3) { minPointSqDis3 = d; minPointInd3 = j; }
            }
          }
          for (int j = closestPointInd - 1; j >= 0; j--) {
            if ((double)(int)sl[j].i < closestPointScan - 2.5) break;
            const float d = sqdis(sl[j], pointSel);
            if ((int)sl[j].i >= closestPointScan) {
              if (d < minPointSqDis2) { minPointSqDis2 = d; minPointInd2 = j; }
            } else {
              if (d < minPointSqDis3) { minPointSqDis3 = d; minPointInd3 = j; }
            }
          }
        }
        si1[i] = closestPointInd;
        si2[i] = minPointInd2;
        si3[i] = minPointInd3;
      }
      if (si2[i] >= 0 && si3[i] >= 0) {
        const P4 t1 = sl[si1[i]], t2 = sl[si2[i]], t3 = sl[si3[i]];
        float pa = (t2.y - t1.y) * (t3.z - t1.z) - (t3.y - t1.y) * (t2.z - t1.z);
        float pb = (t2.z - t1.z) * (t3.x - t1.x) - (t3.z - t1.z) * (t2.x - t1.x);
        float pc = (t2.x - t1.x) * (t3.y - t1.y) - (t3.x - t1.x) * (t2.y - t1.y);
        float pd = -(pa * t1.x + pb * t1.y + pc * t1.z);
        const float ps = std::sqrt(pa * pa + pb * pb + pc * pc);
        pa /= ps; pb /= ps; pc /= ps; pd /= ps;
        const float pd2 = pa * pointSel.x + pb * pointSel.y + pc * pointSel.z + pd;
        float s = 1;
        if (iterCount >= 5)
          s = (float)(1 - 1.8 * (double)std::fabs(pd2) /
                              (double)std::sqrt(std::sqrt(pointSel.x * pointSel.x + pointSel.y * pointSel.y +
                                                          pointSel.z * pointSel.z)));
        if ((double)s > 0.1 && pd2 != 0) sel.push_back({flat[i], s * pa, s * pb, s * pc, s * pd2});
      }
    }
  }

  // Shared tail of calculateTransformation{Surf,Corner} (FA:1952-1990 / 2089-2125): matAtA =
  // matAt * matA and matAtB = matAt * matB as Eigen evaluates them, the 3x3 column-pivoting QR
  // solve, the iteration-0 eigen decomposition with degeneracy test (eigenvalues scanned from the
  // largest, rows of matV2 zeroed), matP = matV.inverse() * matV2 (cofactor inverse), and the
  // projection matX = matP * matX2 — all through oracle_eigen.h.
  void solve3(int iterCount, const std::vector<float>& rows, const std::vector<float>& b, float* X) {
    const int n = (int)b.size();
    float AtA[9], AtB[3];
    oeig::gemm_ata(rows.data(), n, 3, AtA);
    oeig::gemv_atb(rows.data(), b.data(), n, 3, AtB);
    oeig::colpiv_qr_solve(AtA, 3, 3, AtB, X);
    if (iterCount == 0) {
      float E[3], V[9], V2[9], Vi[9];
      oeig::eig_sym3(AtA, E, V);
      std::memcpy(V2, V, sizeof V2);
      isDegenerate = false;
      const float eignThre[3] = {10, 10, 10};
      for (int i = 2; i >= 0; --i) {
        if (E[i] < eignThre[i]) {
          for (int j = 0; j < 3; ++j) V2[i + 3 * j] = 0;
          isDegenerate = true;
        } else {
          break;
        }
      }
      oeig::inverse3(V, Vi);
      oeig::prod33(Vi, V2, matP);
    }
    if (isDegenerate) {
      const float X2[3] = {X[0], X[1], X[2]};
      oeig::prod31(matP, X2, X);
    }
  }

  // calculateTransformationSurf (FA:1846-2010); returns false when converged
  bool calc_surf(int iterCount) {
    const float srx = std::sin(t[0]), crx = std::cos(t[0]);
    const float sry = std::sin(t[1]), cry = std::cos(t[1]);
    const float srz = std::sin(t[2]), crz = std::cos(t[2]);
    const float tx = t[3], ty = t[4], tz = t[5];
    const float a1 = crx * sry * srz, a2 = crx * crz * sry, a3 = srx * sry;
    const float a4 = tx * a1 - ty * a2 - tz * a3;
    const float a5 = srx * srz, a6 = crz * srx;
    const float a7 = ty * a6 - tz * crx - tx * a5;
    const float a8 = crx * cry * srz, a9 = crx * cry * crz, a10 = cry * srx;
    const float a11 = tz * a10 + ty * a9 - tx * a8;
    const float b1 = -crz * sry - cry * srx * srz, b2 = cry * crz * srx - sry * srz;
    const float b5 = cry * crz - srx * sry * srz, b6 = cry * srz + crz * srx * sry;
    const float c1 = -b6, c2 = b5, c3 = tx * b6 - ty * b5, c4 = -crx * crz, c5 = crx * srz;
    const float c6 = ty * c5 + tx * -c4, c7 = b2, c8 = -b1, c9 = tx * -b2 - ty * -b1;
    std::vector<float> rows, bv;
    rows.reserve(3 * sel.size());
    bv.reserve(sel.size());
    for (const Coeff& co : sel) {
      const P4& p = co.ori;
      const float arx = (-a1 * p.x + a2 * p.y + a3 * p.z + a4) * co.cx + (a5 * p.x - a6 * p.y + crx * p.z + a7) * co.cy +
                        (a8 * p.x - a9 * p.y - a10 * p.z + a11) * co.cz;
      const float arz = (c1 * p.x + c2 * p.y + c3) * co.cx + (c4 * p.x - c5 * p.y + c6) * co.cy + (c7 * p.x + c8 * p.y + c9) * co.cz;
      const float aty = -b6 * co.cx + c4 * co.cy + b2 * co.cz;
      rows.insert(rows.end(), {arx, arz, aty});  // matA(i, 0..2) (FA:1946-1948)
      bv.push_back((float)(-0.05 * (double)co.ci));  // matB(i, 0) (FA:1949)
    }
    float X[3];
    solve3(iterCount, rows, bv, X);
    t[0] += X[0];
    t[2] += X[1];
    t[4] += X[2];
    for (int i = 0; i < 6; ++i)
      if (std::isnan(t[i])) t[i] = 0;
    const float r2d = (float)(180.0 / M_PI);  // FA:56 const float RAD2DEG
    const double e0 = (double)(r2d * X[0]), e1 = (double)(r2d * X[1]), e2 = (double)(X[2] * 100);
    const float deltaR = (float)std::sqrt(e0 * e0 + e1 * e1);
    const float deltaT = (float)std::sqrt(e2 * e2);
    return !((double)deltaR < 0.1 && (double)deltaT < 0.1);
  }

  // calculateTransformationCorner (FA:2013-2143)
  bool calc_corner(int iterCount) {
    const float srx = std::sin(t[0]), crx = std::cos(t[0]);
    const float sry = std::sin(t[1]), cry = std::cos(t[1]);
    const float srz = std::sin(t[2]), crz = std::cos(t[2]);
    const float tx = t[3], ty = t[4], tz = t[5];
    const float b1 = -crz * sry - cry * srx * srz, b2 = cry * crz * srx - sry * srz, b3 = crx * cry;
    const float b4 = tx * -b1 + ty * -b2 + tz * b3;
    const float b5 = cry * crz - srx * sry * srz, b6 = cry * srz + crz * srx * sry, b7 = crx * sry;
    const float b8 = tz * b7 - ty * b6 - tx * b5;
    const float c5 = crx * srz;
    std::vector<float> rows, bv;
    rows.reserve(3 * sel.size());
    bv.reserve(sel.size());
    for (const Coeff& co : sel) {
      const P4& p = co.ori;
      const float ary = (b1 * p.x + b2 * p.y - b3 * p.z + b4) * co.cx + (b5 * p.x + b6 * p.y - b7 * p.z + b8) * co.cz;
      const float atx = -b5 * co.cx + c5 * co.cy + b1 * co.cz;
      const float atz = b7 * co.cx - srx * co.cy - b3 * co.cz;
      rows.insert(rows.end(), {ary, atx, atz});  // matA(i, 0..2) (FA:2085-2087)
      bv.push_back((float)(-0.05 * (double)co.ci));
    }
    float X[3];
    solve3(iterCount, rows, bv, X);
    t[1] += X[0];
    t[3] += X[1];
    t[5] += X[2];
    for (int i = 0; i < 6; ++i)
      if (std::isnan(t[i])) t[i] = 0;
    const float r2d = (float)(180.0 / M_PI);
    const double e0 = (double)(r2d * X[0]), e1 = (double)(X[1] * 100), e2 = (double)(X[2] * 100);
    const float deltaR = (float)std::sqrt(e0 * e0);
    const float deltaT = (float)std::sqrt(e1 * e1 + e2 * e2);
    return !((double)deltaR < 0.1 && (double)deltaT < 0.1);
  }
};

}  // namespace

extern "C" int32_t ORACLE_FN(scan2scan)(const llsr_config* cfg, const float* sharp, int32_t Ms, const float* flat,
                                        int32_t F, const float* cl, int32_t Nc, const float* sl, int32_t Ns,
                                        float* transform_cur, int32_t* is_degenerate, llsr_s2s_report* rep) {
  if (!cfg || !transform_cur || !is_degenerate || !rep || Ms < 0 || F < 0 || Nc < 0 || Ns < 0) return LLSR_EINVAL;
  std::memset(rep, 0, sizeof *rep);
  S2S S;
  S.cfg = cfg;
  std::memcpy(S.t, transform_cur, sizeof S.t);
  S.isDegenerate = *is_degenerate != 0;
  for (int k = 0; k < 9; ++k) S.matP[k] = (k % 4 == 0) ? 1.0f : 0.0f;
  S.sharp = reinterpret_cast<const P4*>(sharp);
  S.flat = reinterpret_cast<const P4*>(flat);
  S.cl = reinterpret_cast<const P4*>(cl);
  S.sl = reinterpret_cast<const P4*>(sl);
  S.Ms = Ms; S.F = F; S.Nc = Nc; S.Ns = Ns;
  S.distSqr = cfg->nearest_feature_search_distance * cfg->nearest_feature_search_distance;  // FA:152
  auto t0 = std::chrono::steady_clock::now();
  if (Nc < 10 || Ns < 100) {  // FA:2506
    rep->skipped = 1;
  } else {
    S.kc.build(S.cl, Nc);
    S.ks.build(S.sl, Ns);
    S.ci1.assign(Ms, -1); S.ci2.assign(Ms, -1);
    S.si1.assign(F, -1); S.si2.assign(F, -1); S.si3.assign(F, -1);
    int it1 = 0;
    for (it1 = 0; it1 < 100; ++it1) {
      S.sel.clear();
      S.surf_corr(it1);
      rep->n_surf_corr = (int32_t)S.sel.size();
      if (S.sel.size() < 10) continue;
      if (!S.calc_surf(it1)) break;
    }
    for (int k = 0; k < 9; ++k) S.matP[k] = (k % 4 == 0) ? 1.0f : 0.0f;
    int it2 = 0;
    for (it2 = 0; it2 < 100; ++it2) {
      S.sel.clear();
      S.corner_corr(it2);
      rep->n_corner_corr = (int32_t)S.sel.size();
      if (S.sel.size() < 10) continue;
      if (!S.calc_corner(it2)) break;
    }
    rep->surf_iterations = it1;
    rep->corner_iterations = it2;
  }
  auto t1 = std::chrono::steady_clock::now();
  std::memcpy(transform_cur, S.t, sizeof S.t);
  std::memcpy(rep->transform_cur, S.t, sizeof S.t);
  *is_degenerate = S.isDegenerate ? 1 : 0;
  rep->degenerate = *is_degenerate;
  rep->ms = (float)std::chrono::duration<double, std::milli>(t1 - t0).count();
  return LLSR_OK;
}

#ifndef LLSR_ORACLE_NANOFLANN
// TransformToEnd (FA:1414-1490), use_imu_undistortion == false branch.
extern "C" void oracle_transform_to_end(const float* tc, float* xyzi, int32_t n) {
  P4* p = reinterpret_cast<P4*>(xyzi);
  for (int k = 0; k < n; ++k) {
    const P4 pi = p[k];
    const float s = 10 * (pi.i - (float)(int)pi.i);
    float rx = s * tc[0], ry = s * tc[1], rz = s * tc[2];
    float tx = s * tc[3], ty = s * tc[4], tz = s * tc[5];
    const float x1 = std::cos(rz) * (pi.x - tx) + std::sin(rz) * (pi.y - ty);
    const float y1 = -std::sin(rz) * (pi.x - tx) + std::cos(rz) * (pi.y - ty);
    const float z1 = (pi.z - tz);
    const float x2 = x1;
    const float y2 = std::cos(rx) * y1 + std::sin(rx) * z1;
    const float z2 = -std::sin(rx) * y1 + std::cos(rx) * z1;
    const float x3 = std::cos(ry) * x2 - std::sin(ry) * z2;
    const float y3 = y2;
    const float z3 = std::sin(ry) * x2 + std::cos(ry) * z2;
    rx = tc[0]; ry = tc[1]; rz = tc[2];
    tx = tc[3]; ty = tc[4]; tz = tc[5];
    const float x4 = std::cos(ry) * x3 + std::sin(ry) * z3;
    const float y4 = y3;
    const float z4 = -std::sin(ry) * x3 + std::cos(ry) * z3;
    const float x5 = x4;
    const float y5 = std::cos(rx) * y4 - std::sin(rx) * z4;
    const float z5 = std::sin(rx) * y4 + std::cos(rx) * z4;
    P4 po;
    po.x = std::cos(rz) * x5 - std::sin(rz) * y5 + tx;
    po.y = std::sin(rz) * x5 + std::cos(rz) * y5 + ty;
    po.z = z5 + tz;
    po.i = (float)(int)pi.i;
    p[k] = po;
  }
}

// AccumulateRotation (FA:1552-1578): float sin / cos / asin / atan2 overloads.
static void accumulate_rotation(float cx, float cy, float cz, float lx, float ly, float lz, float& ox, float& oy,
                                float& oz) {
  float srx = std::cos(lx) * std::cos(cx) * std::sin(ly) * std::sin(cz) -
              std::cos(cx) * std::cos(cz) * std::sin(lx) - std::cos(lx) * std::cos(ly) * std::sin(cx);
  ox = -std::asin(srx);
  float srycrx = std::sin(lx) * (std::cos(cy) * std::sin(cz) - std::cos(cz) * std::sin(cx) * std::sin(cy)) +
                 std::cos(lx) * std::sin(ly) * (std::cos(cy) * std::cos(cz) + std::sin(cx) * std::sin(cy) * std::sin(cz)) +
                 std::cos(lx) * std::cos(ly) * std::cos(cx) * std::sin(cy);
  float crycrx = std::cos(lx) * std::cos(ly) * std::cos(cx) * std::cos(cy) -
                 std::cos(lx) * std::sin(ly) * (std::cos(cz) * std::sin(cy) - std::cos(cy) * std::sin(cx) * std::sin(cz)) -
                 std::sin(lx) * (std::sin(cy) * std::sin(cz) + std::cos(cy) * std::cos(cz) * std::sin(cx));
  oy = std::atan2(srycrx / std::cos(ox), crycrx / std::cos(ox));
  float srzcrx = std::sin(cx) * (std::cos(lz) * std::sin(ly) - std::cos(ly) * std::sin(lx) * std::sin(lz)) +
                 std::cos(cx) * std::sin(cz) * (std::cos(ly) * std::cos(lz) + std::sin(lx) * std::sin(ly) * std::sin(lz)) +
                 std::cos(lx) * std::cos(cx) * std::cos(cz) * std::sin(lz);
  float crzcrx = std::cos(lx) * std::cos(lz) * std::cos(cx) * std::cos(cz) -
                 std::cos(cx) * std::sin(cz) * (std::cos(ly) * std::sin(lz) - std::cos(lz) * std::sin(lx) * std::sin(ly)) -
                 std::sin(cx) * (std::sin(ly) * std::sin(lz) + std::cos(ly) * std::cos(lz) * std::sin(lx));
  oz = std::atan2(srzcrx / std::cos(ox), crzcrx / std::cos(ox));
}

// integrateTransformation (FA:2537-2568), use_imu_undistortion == false: transformSum in place.
extern "C" void oracle_integrate_transformation(float* ts, const float* tc) {
  float rx, ry, rz;
  accumulate_rotation(ts[0], ts[1], ts[2], -tc[0], -tc[1], -tc[2], rx, ry, rz);
  const float x1 = std::cos(rz) * (tc[3]) - std::sin(rz) * (tc[4]);
  const float y1 = std::sin(rz) * (tc[3]) + std::cos(rz) * (tc[4]);
  const float z1 = tc[5];
  const float x2 = x1;
  const float y2 = std::cos(rx) * y1 - std::sin(rx) * z1;
  const float z2 = std::sin(rx) * y1 + std::cos(rx) * z1;
  const float tx = ts[3] - (std::cos(ry) * x2 + std::sin(ry) * z2);
  const float ty = ts[4] - y2;
  const float tz = ts[5] - (-std::sin(ry) * x2 + std::cos(ry) * z2);
  ts[0] = rx; ts[1] = ry; ts[2] = rz;
  ts[3] = tx; ts[4] = ty; ts[5] = tz;
}

// GenerateShadowPoint (FA:412-439): 16 x 10 virtual points, lidar_to_body_centor (FA:300).
extern "C" void oracle_shadow_points(float* out) {
  const double c0 = 0.008, c1 = 0.0, c2 = -0.035;
  const int row_size = 16, col_size = 10;
  const double row_angle = (std::atan2(0.120, 0.05) * 2) / (row_size - 1);
  const double col_angle = (std::atan2(0.077, 0.05) * 2) / (col_size - 1);
  int k = 0;
  for (int row = 0; row < row_size; row++) {
    const float row_x = (float)(0.05 * std::tan((((row_size - 1.0) / 2.0) * row_angle) - (row * row_angle)));
    for (int col = 0; col < col_size; col++) {
      const float col_y = (float)(0.05 * std::tan((((col_size - 1.0) / 2.0) * col_angle) - (col * col_angle)));
      out[4 * k + 0] = (float)(col_y + c1);
      out[4 * k + 1] = (float)(-(0.035f + 0.05f) + c2);
      out[4 * k + 2] = (float)(row_x + c0);
      out[4 * k + 3] = (float)((double)((float)row + (float)17) + (double)(float)col / 10000.0);
      ++k;
    }
  }
}
#endif
