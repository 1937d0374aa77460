// oracle_mo.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Scalar CPU restatement of MapOptimization::scan2MapOptimization (MO = mapOptmization.cpp:
// 1572-1610) with cornerOptimization (MO:1269-1377), surfOptimization (MO:1379-1442),
// LMOptimization (MO:1444-1570) and pointAssociateToMap (MO:591-620).
//
// kNN-5 (nanoflann KdTreeFLANN::nearestKSearch, eps 0, sorted) is restated exactly where it can
// matter: a correspondence is kept only when the 5th nearest squared distance is < 1.0, so the
// search is a 1 m uniform grid over the 27 neighbouring cells; squared distances accumulate as
// ((0 + dx^2) + dy^2) + dz^2 (nanoflann.hpp:431-439, L2_Simple_Adaptor behind the SO3_Adaptor of
// nanoflann_pcl.h) and equal distances keep the lower index. Eigen calls go through the oracle's
// own restatement (oracle_eigen.h), independent of the device's.
//
// Built a second time by oracle/Makefile with -DLLSR_ORACLE_NANOFLANN against the reference's
// own vendored kd-tree (LeGO-LOAM/include/lego_loam/nanoflann.hpp, included by path, std-only;
// output oracle/_ref/libref_mo.so, never committed): the same restatement with the reference's
// kNN, used to cross-check the grid (tests/test_mo_oracle.py) and as the MO CPU baseline.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../include/llsr.h"
#include "oracle.h"
#include "oracle_eigen.h"
#ifdef LLSR_ORACLE_NANOFLANN
#include "nanoflann.hpp"
#endif

namespace {

struct P4 { float x, y, z, i; };

struct Grid {
  const P4* pts = nullptr;
  int n = 0;
  std::unordered_map<long long, std::vector<int>> cells;
  static long long key(int a, int b, int c) {
    return ((long long)(a + 1048576) << 42) | ((long long)(b + 1048576) << 21) | (long long)(c + 1048576);
  }
  void build(const P4* p, int np) {
    pts = p;
    n = np;
    cells.clear();
    for (int k = 0; k < np; ++k)
      cells[key((int)std::floor(p[k].x), (int)std::floor(p[k].y), (int)std::floor(p[k].z))].push_back(k);
  }
  // 5 nearest with d2 < 1.0, ascending; returns how many (only 5 means "accepted").
  int knn5(const P4& q, int* idx, float* d2) const {
    int cnt = 0;
    const int cx = (int)std::floor(q.x), cy = (int)std::floor(q.y), cz = (int)std::floor(q.z);
    // candidates in index order so equal distances resolve like a first-found insertion
    std::vector<int> cand;
    for (int a = -1; a <= 1; ++a)
      for (int b = -1; b <= 1; ++b)
        for (int c = -1; c <= 1; ++c) {
          auto it = cells.find(key(cx + a, cy + b, cz + c));
          if (it != cells.end()) cand.insert(cand.end(), it->second.begin(), it->second.end());
        }
    std::sort(cand.begin(), cand.end());
    for (int k : cand) {
      float d = 0.0f;
      float t = q.x - pts[k].x; d += t * t;
      t = q.y - pts[k].y; d += t * t;
      t = q.z - pts[k].z; d += t * t;
      if (!(d < 1.0f)) continue;
      if (cnt == 5 && !(d < d2[4])) continue;
      int pos = cnt < 5 ? cnt : 4;
      if (cnt < 5) ++cnt;
      while (pos > 0 && d < d2[pos - 1]) { d2[pos] = d2[pos - 1]; idx[pos] = idx[pos - 1]; --pos; }
      d2[pos] = d; idx[pos] = k;
    }
    return cnt;
  }
};

#ifdef LLSR_ORACLE_NANOFLANN
// KdTreeFLANN<PointType> of nanoflann_pcl.h: KDTreeSingleIndexAdaptor<SO3_Adaptor<float, .>, ., 3,
// int>, leaf size 10, nearestKSearch = KNNResultSet<float, int>(k) + findNeighbors(SearchParams())
struct CloudAdaptor {
  const P4* pts = nullptr;
  size_t n = 0;
  size_t kdtree_get_point_count() const { return n; }
  float kdtree_get_pt(const size_t idx, int dim) const { return (&pts[idx].x)[dim]; }
  template <class BBOX> bool kdtree_get_bbox(BBOX&) const { return false; }
};
using KdTree = nanoflann::KDTreeSingleIndexAdaptor<nanoflann::SO3_Adaptor<float, CloudAdaptor>, CloudAdaptor, 3, int>;
struct Knn {
  CloudAdaptor ad;
  KdTree* tree = nullptr;
  ~Knn() { delete tree; }
  void build(const P4* p, int np) {
    ad.pts = p;
    ad.n = (size_t)np;
    delete tree;
    tree = new KdTree(3, ad);
    tree->buildIndex();
  }
  // same contract as Grid::knn5: 5 when the five nearest all have d^2 < 1.0
  int knn5(const P4& q, int* idx, float* d2) const {
    nanoflann::KNNResultSet<float, int> rs(5);
    rs.init(idx, d2);
    tree->findNeighbors(rs, &q.x, nanoflann::SearchParams());
    return (rs.size() == 5 && d2[4] < 1.0f) ? 5 : 0;
  }
};
#define ORACLE_FN(name) ref_##name
#else
using Knn = Grid;
#define ORACLE_FN(name) oracle_##name
#endif

struct Coeff { P4 ori; float cx, cy, cz, ci; };

// cornerOptimization body (MO:1274-1375) for one map-frame query point; false when rejected.
bool corner_coeff(const Knn& gc, const P4* cornerM, const P4& sel_p, float& la_, float& lb_, float& lc_,
                  float& ld_) {
  int idx[5];
  float d2[5];
  if (gc.knn5(sel_p, idx, d2) < 5) return false;
  float cx = 0, cy = 0, cz = 0;
  for (int j = 0; j < 5; ++j) { cx += cornerM[idx[j]].x; cy += cornerM[idx[j]].y; cz += cornerM[idx[j]].z; }
  cx /= 5; cy /= 5; cz /= 5;
  float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
  for (int j = 0; j < 5; ++j) {
    const float ax = cornerM[idx[j]].x - cx, ay = cornerM[idx[j]].y - cy, az = cornerM[idx[j]].z - cz;
    a11 += ax * ax; a12 += ax * ay; a13 += ax * az; a22 += ay * ay; a23 += ay * az; a33 += az * az;
  }
  a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
  const float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33};  // column-major
  float D1[3], V1[9];
  oeig::eig_sym3(A1, D1, V1);
  if (!(D1[2] > 3 * D1[1])) return false;
  const float x0 = sel_p.x, y0 = sel_p.y, z0 = sel_p.z;
  // ROW 0 of matV1: V(0,0), V(0,1), V(0,2) (column-major: [0], [3], [6])
  const float x1 = (float)(cx + 0.1 * V1[0]), y1 = (float)(cy + 0.1 * V1[3]), z1 = (float)(cz + 0.1 * V1[6]);
  const float x2 = (float)(cx - 0.1 * V1[0]), y2 = (float)(cy - 0.1 * V1[3]), z2 = (float)(cz - 0.1 * V1[6]);
  const float a012 = std::sqrt(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                               ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                               ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)));
  const float l12 = std::sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
  const float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                    (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) / a012 / l12;
  const float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                     (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
  const float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                     (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
  const float ld2 = a012 / l12;
  const float s = (float)(1 - 0.9 * std::fabs(ld2));
  if (!(s > 0.1)) return false;
  la_ = s * la; lb_ = s * lb; lc_ = s * lc; ld_ = s * ld2;
  return true;
}

// surfOptimization body (MO:1383-1440) for one map-frame query point; false when rejected.
bool surf_coeff(const Knn& gs, const P4* surfM, const P4& sel_p, float& la_, float& lb_, float& lc_, float& ld_) {
  int idx[5];
  float d2[5];
  if (gs.knn5(sel_p, idx, d2) < 5) return false;
  float A0[15];  // 5x3 column-major
  for (int j = 0; j < 5; ++j) { A0[j] = surfM[idx[j]].x; A0[5 + j] = surfM[idx[j]].y; A0[10 + j] = surfM[idx[j]].z; }
  const float B0[5] = {-1, -1, -1, -1, -1};
  float X0[3];
  oeig::colpiv_qr_solve(A0, 5, 3, B0, X0);  // matA0.colPivHouseholderQr().solve(matB0)
  float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
  const float ps = std::sqrt(pa * pa + pb * pb + pc * pc);
  pa /= ps; pb /= ps; pc /= ps; pd /= ps;
  for (int j = 0; j < 5; ++j)
    if (std::fabs(pa * surfM[idx[j]].x + pb * surfM[idx[j]].y + pc * surfM[idx[j]].z + pd) > 0.2) return false;
  const float pd2 = pa * sel_p.x + pb * sel_p.y + pc * sel_p.z + pd;
  const float s = (float)(1 - 0.9 * std::fabs(pd2) /
                                 std::sqrt(std::sqrt(sel_p.x * sel_p.x + sel_p.y * sel_p.y + sel_p.z * sel_p.z)));
  if (!(s > 0.1)) return false;
  la_ = s * pa; lb_ = s * pb; lc_ = s * pc; ld_ = s * pd2;
  return true;
}

// pointAssociateToMap (MO:606-620) with the sin/cos of updatePointAssociateToMapSinCos (MO:591-604).
P4 associate(const float* t, const P4& pi) {
  const float cRoll = std::cos(t[0]), sRoll = std::sin(t[0]);
  const float cPitch = std::cos(t[1]), sPitch = std::sin(t[1]);
  const float cYaw = std::cos(t[2]), sYaw = std::sin(t[2]);
  const float x1 = cYaw * pi.x - sYaw * pi.y;
  const float y1 = sYaw * pi.x + cYaw * pi.y;
  const float z1 = pi.z;
  const float x2 = x1;
  const float y2 = cRoll * y1 - sRoll * z1;
  const float z2 = sRoll * y1 + cRoll * z1;
  P4 po;
  po.x = cPitch * x2 + sPitch * z2 + t[3];
  po.y = y2 + t[4];
  po.z = -sPitch * x2 + cPitch * z2 + t[5];
  po.i = pi.i;
  return po;
}

// Jacobian row of LMOptimization (MO:1465-1490) at pose t; a[6] = (arx, ary, arz, cx, cy, cz).
void jacobian_row(const float* t, const Coeff& co, float* a) {
  const float srx = std::sin(t[0]), crx = std::cos(t[0]);
  const float sry = std::sin(t[1]), cry = std::cos(t[1]);
  const float srz = std::sin(t[2]), crz = std::cos(t[2]);
  const P4& p = co.ori;
  a[0] = (crx * sry * srz * p.x + crx * crz * sry * p.y - srx * sry * p.z) * co.cx +
         (-srx * srz * p.x - crz * srx * p.y - crx * p.z) * co.cy +
         (crx * cry * srz * p.x + crx * cry * crz * p.y - cry * srx * p.z) * co.cz;
  a[1] = ((cry * srx * srz - crz * sry) * p.x + (sry * srz + cry * crz * srx) * p.y + crx * cry * p.z) * co.cx +
         ((-cry * crz - srx * sry * srz) * p.x + (cry * srz - crz * srx * sry) * p.y - crx * sry * p.z) * co.cz;
  a[2] = ((crz * srx * sry - cry * srz) * p.x + (-cry * crz - srx * sry * srz) * p.y) * co.cx +
         (crx * crz * p.x - crx * srz * p.y) * co.cy +
         ((sry * srz + cry * crz * srx) * p.x + (crz * sry - cry * srx * srz) * p.y) * co.cz;
  a[3] = co.cx;
  a[4] = co.cy;
  a[5] = co.cz;
}

// LMOptimization from the solve to the degeneracy projection (MO:1505-1537), on the assembled
// normal equations. matP / isDegenerate are MapOptimization members (mapOptimization.h:279-281,
// zeroed at construction MO:285-286): set at iteration 0, reused by the later iterations.
struct MoLm {
  bool isDegenerate = false;
  float matP[36] = {0};
  float min_lambda = 0.0f;
  float matX0[6] = {0};
};
void mo_lm_solve(MoLm& s, const float* AtA, const float* AtB, int iterCount, float* X) {
  oeig::colpiv_qr_solve(AtA, 6, 6, AtB, X);
  if (iterCount == 0) {
    float E[6], V[36], V2[36], Vi[36];
    oeig::eig_sym_n(AtA, 6, E, V);
    s.min_lambda = E[0];
    std::memcpy(V2, V, sizeof V2);
    s.isDegenerate = false;
    const float eignThre[6] = {100, 100, 100, 100, 100, 100};
    for (int i = 5; i >= 0; --i) {
      if (E[i] < eignThre[i]) {
        for (int j = 0; j < 6; ++j) V2[i + 6 * j] = 0;  // matV2(i, j): row i (MO:1522-1524)
        s.isDegenerate = true;
      } else {
        break;
      }
    }
    oeig::inverse_lu(V, 6, Vi);       // matV.inverse(): PartialPivLU
    oeig::prod66(Vi, V2, s.matP);     // matP = matV.inverse() * matV2 (MO:1530)
    std::memcpy(s.matX0, X, sizeof s.matX0);
  }
  if (s.isDegenerate) {
    float X2[6];
    std::memcpy(X2, X, sizeof X2);
    oeig::prod61(s.matP, X2, X);      // matX = matP * matX2 (MO:1533-1536)
  }
}

// The stop test (MO:1546-1553): pcl::rad2deg(float), std::pow(float, int) in double.
bool mo_converged(const float* X, float stop_thres) {
  const float r2d = 57.29577951308232f;
  const float deltaR = (float)std::sqrt(std::pow(X[0] * r2d, 2) + std::pow(X[1] * r2d, 2) + std::pow(X[2] * r2d, 2));
  const float deltaT = (float)std::sqrt(std::pow(X[3] * 100, 2) + std::pow(X[4] * 100, 2) + std::pow(X[5] * 100, 2));
  return deltaR < stop_thres && deltaT < stop_thres;
}

}  // namespace

// scan2MapOptimization with the optimiser's members carried in and out: isDegenerate / matP
// (mapOptimization.h:279-281) keep their values across frames, and an iteration 0 with fewer than
// 50 correspondences (MO:1453) leaves them untouched for the later iterations of the next frames.
extern "C" int32_t ORACLE_FN(scan2map_carry)(const llsr_config* cfg, const float* cq, int32_t Qc, const float* sq,
                                         int32_t Qs, const float* cm, int32_t Mc, const float* sm, int32_t Ms,
                                         float* pose, int32_t* degenerate, float* matP, llsr_lm_report* rep) {
  if (!cfg || !pose || !rep || !degenerate || !matP || Qc < 0 || Qs < 0 || Mc < 0 || Ms < 0) return LLSR_EINVAL;
  const P4* cornerQ = reinterpret_cast<const P4*>(cq);
  const P4* surfQ = reinterpret_cast<const P4*>(sq);
  const P4* cornerM = reinterpret_cast<const P4*>(cm);
  const P4* surfM = reinterpret_cast<const P4*>(sm);
  std::memset(rep, 0, sizeof *rep);
  float t[6];
  std::memcpy(t, pose, sizeof t);
  if (!(Mc > 10 && Ms > 100)) {  // MO:1573
    std::memcpy(rep->pose, t, sizeof t);
    return LLSR_OK;
  }
  auto t0 = std::chrono::steady_clock::now();
  Knn gc, gs;
  gc.build(cornerM, Mc);
  gs.build(surfM, Ms);
  const bool applied = cfg->mode == LLSR_MODE_LM_APPLIED;
  MoLm lm;
  lm.isDegenerate = *degenerate != 0;
  std::memcpy(lm.matP, matP, sizeof lm.matP);
  float CF_mean = 0.0f;
  int iters = 0, converged = 0, nc = 0, ns = 0;
  std::vector<Coeff> sel;
  std::vector<float> rows, bv;
  for (int iterCount = 0; iterCount < cfg->iterCountThres; ++iterCount) {
    sel.clear();
    ++iters;
    // ---- cornerOptimization (MO:1269-1377) ----
    int ncor = 0;
    for (int i = 0; i < Qc; ++i) {
      Coeff co{cornerQ[i], 0, 0, 0, 0};
      if (corner_coeff(gc, cornerM, associate(t, cornerQ[i]), co.cx, co.cy, co.cz, co.ci)) { sel.push_back(co); ++ncor; }
    }
    // ---- surfOptimization (MO:1379-1442) ----
    int nsur = 0;
    for (int i = 0; i < Qs; ++i) {
      Coeff co{surfQ[i], 0, 0, 0, 0};
      if (surf_coeff(gs, surfM, associate(t, surfQ[i]), co.cx, co.cy, co.cz, co.ci)) { sel.push_back(co); ++nsur; }
    }
    nc = ncor; ns = nsur;
    // ---- LMOptimization (MO:1444-1570) ----
    const int N = (int)sel.size();
    if (N < 50) continue;  // returns false: not converged, no update
    rows.resize((size_t)6 * N);
    bv.resize(N);
    for (int i = 0; i < N; ++i) {
      jacobian_row(t, sel[i], &rows[(size_t)6 * i]);
      bv[i] = -cfg->step_size * sel[i].ci;  // matB(i, 0) = -step_size * coeff.intensity
    }
    float AtA[36], AtB[6], X[6];
    oeig::gemm_ata(rows.data(), N, 6, AtA);  // matAtA = matAt * matA (GEMM)
    oeig::gemv_atb(rows.data(), bv.data(), N, 6, AtB);
    mo_lm_solve(lm, AtA, AtB, iterCount, X);
    if (iterCount == 0) std::memcpy(rep->matX0, lm.matX0, sizeof lm.matX0);
    if (applied)
      for (int k = 0; k < 6; ++k) t[k] += X[k];
    float CF_all = 0;
    for (int i = 0; i < N; ++i) CF_all += std::fabs(sel[i].ci);
    CF_mean = CF_all / N;
    if (mo_converged(X, cfg->stop_thres)) { converged = 1; break; }
  }
  const bool isDegenerate = lm.isDegenerate;
  const float min_lambda = lm.min_lambda;
  auto t1 = std::chrono::steady_clock::now();
  rep->iterations = iters;
  rep->converged = converged;
  rep->degenerate = isDegenerate ? 1 : 0;
  rep->min_lambda = min_lambda;
  rep->cf_mean = CF_mean;
  rep->n_corner_corr = nc;
  rep->n_surf_corr = ns;
  rep->ms = (float)std::chrono::duration<double, std::milli>(t1 - t0).count();
  std::memcpy(rep->pose, t, sizeof t);
  std::memcpy(pose, t, sizeof t);
  *degenerate = isDegenerate ? 1 : 0;
  std::memcpy(matP, lm.matP, sizeof lm.matP);
  return LLSR_OK;
}

// One scan2MapOptimization call of a freshly constructed MapOptimization (members zeroed, MO:285-286).
extern "C" int32_t ORACLE_FN(scan2map)(const llsr_config* cfg, const float* cq, int32_t Qc, const float* sq,
                                   int32_t Qs, const float* cm, int32_t Mc, const float* sm, int32_t Ms,
                                   float* pose, llsr_lm_report* rep) {
  int32_t deg = 0;
  float matP[36] = {0};
  return ORACLE_FN(scan2map_carry)(cfg, cq, Qc, sq, Qs, cm, Mc, sm, Ms, pose, &deg, matP, rep);
}

// ---- split-correspondence scan-to-map, int64 fixed-point sums (llsr_scan2map_shard_*) -------
// The CPU statement of the split mode, written independently of the
// device: per LM iteration every rank sums the fixed-point terms of its 256-query blocks (block b
// of each kind goes to rank b % world), the ranks' words are added, and the LMOptimization tail
// (mo_lm_solve above: QR, eigen, PartialPivLU inverse, projection) runs on the total. Used by the
// gloo tests as a rank's engine and by the GPU tests as the bit-exact reference for the device's
// split mode. Word layout (LLSR_NE_WORDS = 32): AtA upper triangle row-major (21), AtB (6),
// sum |coeff.intensity|, #corner, #surf, 2 spare. A term is round-to-nearest-even(v * 2^30) as an
// int64; a non-finite term or one with |v| >= 2^32 is counted in word 31 and contributes 0.
namespace ofx {
constexpr int kWords = LLSR_NE_WORDS;
constexpr double kScale = 1073741824.0;  // 2^30
inline void add_term(int64_t* ne, int k, float v) {
  if (k >= 28) { ne[k] += (int64_t)v; return; }
  if (!(std::fabs(v) < 4294967296.0f)) { ne[31] += 1; return; }
  ne[k] += (int64_t)std::nearbyint((double)v * kScale);
}
inline float word(int64_t w) { return (float)((double)w / kScale); }
}  // namespace ofx

struct oracle_s2m_shard {
  llsr_config cfg;
  std::vector<P4> cq, sq, cm, sm;
  Knn gc, gs;
  MoLm lm;
  float pose[6];
  float cf_mean = 0.0f;
  int iter = 0, active = 0, converged = 0, nc = 0, ns = 0;
};

extern "C" oracle_s2m_shard* ORACLE_FN(s2m_shard_create)(const llsr_config* cfg, const float* cq, int32_t Qc,
                                                         const float* sq, int32_t Qs, const float* cm, int32_t Mc,
                                                         const float* sm, int32_t Ms, const float* pose) {
  if (!cfg || !pose || Qc < 0 || Qs < 0 || Mc < 0 || Ms < 0) return nullptr;
  auto* s = new oracle_s2m_shard();
  s->cfg = *cfg;
  const P4* p4[4] = {reinterpret_cast<const P4*>(cq), reinterpret_cast<const P4*>(sq),
                     reinterpret_cast<const P4*>(cm), reinterpret_cast<const P4*>(sm)};
  s->cq.assign(p4[0], p4[0] + Qc);
  s->sq.assign(p4[1], p4[1] + Qs);
  s->cm.assign(p4[2], p4[2] + Mc);
  s->sm.assign(p4[3], p4[3] + Ms);
  std::memcpy(s->pose, pose, sizeof s->pose);
  s->active = (Mc > 10 && Ms > 100) ? 1 : 0;  // MO:1573
  if (s->active) {
    s->gc.build(s->cm.data(), Mc);
    s->gs.build(s->sm.data(), Ms);
  }
  return s;
}

extern "C" void ORACLE_FN(s2m_shard_destroy)(oracle_s2m_shard* s) { delete s; }

// Rank `rank` of `world`: the LLSR_NE_WORDS int64 words of this rank's query blocks.
extern "C" void ORACLE_FN(s2m_shard_partial)(oracle_s2m_shard* s, int32_t rank, int32_t world, int64_t* ne) {
  for (int k = 0; k < ofx::kWords; ++k) ne[k] = 0;
  if (!s->active || world < 1) return;
  const float* t = s->pose;
  auto add = [&](const Coeff& co, bool corner) {
    float a[6];
    jacobian_row(t, co, a);
    const float bb = -s->cfg.step_size * co.ci;
    int k = 0;
    for (int r = 0; r < 6; ++r)
      for (int c = r; c < 6; ++c, ++k) ofx::add_term(ne, k, a[r] * a[c]);
    for (int c = 0; c < 6; ++c) ofx::add_term(ne, 21 + c, a[c] * bb);
    ofx::add_term(ne, 27, std::fabs(co.ci));
    ofx::add_term(ne, corner ? 28 : 29, 1.0f);
  };
  for (int i = 0; i < (int)s->cq.size(); ++i) {
    if ((i / 256) % world != rank) continue;
    Coeff co{s->cq[i], 0, 0, 0, 0};
    if (corner_coeff(s->gc, s->cm.data(), associate(t, s->cq[i]), co.cx, co.cy, co.cz, co.ci)) add(co, true);
  }
  for (int i = 0; i < (int)s->sq.size(); ++i) {
    if ((i / 256) % world != rank) continue;
    Coeff co{s->sq[i], 0, 0, 0, 0};
    if (surf_coeff(s->gs, s->sm.data(), associate(t, s->sq[i]), co.cx, co.cy, co.cz, co.ci)) add(co, false);
  }
}

// LMOptimization on the summed words of all ranks; returns 1 while the problem is still active.
extern "C" int32_t ORACLE_FN(s2m_shard_step)(oracle_s2m_shard* s, const int64_t* ne) {
  if (!s->active) return 0;
  s->iter += 1;
  const int iterCount = s->iter - 1;
  s->nc = (int)ne[28];
  s->ns = (int)ne[29];
  const int N = s->nc + s->ns;
  bool conv = false;
  if (N >= 50) {  // MO:1453
    float AtA[36], AtB[6], X[6];
    int k = 0;
    for (int r = 0; r < 6; ++r)
      for (int c = r; c < 6; ++c, ++k) AtA[r + 6 * c] = AtA[c + 6 * r] = ofx::word(ne[k]);
    for (int c = 0; c < 6; ++c) AtB[c] = ofx::word(ne[21 + c]);
    mo_lm_solve(s->lm, AtA, AtB, iterCount, X);
    if (s->cfg.mode == LLSR_MODE_LM_APPLIED)
      for (int q = 0; q < 6; ++q) s->pose[q] += X[q];
    s->cf_mean = ofx::word(ne[27]) / (float)N;
    conv = mo_converged(X, s->cfg.stop_thres);
  }
  if (conv) s->converged = 1;
  if (conv || s->iter >= s->cfg.iterCountThres) s->active = 0;
  return s->active;
}

extern "C" void ORACLE_FN(s2m_shard_result)(const oracle_s2m_shard* s, float* pose, llsr_lm_report* rep) {
  std::memset(rep, 0, sizeof *rep);
  rep->iterations = s->iter;
  rep->converged = s->converged;
  rep->degenerate = s->lm.isDegenerate ? 1 : 0;
  rep->min_lambda = s->lm.min_lambda;
  rep->cf_mean = s->cf_mean;
  rep->n_corner_corr = s->nc;
  rep->n_surf_corr = s->ns;
  std::memcpy(rep->matX0, s->lm.matX0, sizeof s->lm.matX0);
  std::memcpy(rep->pose, s->pose, sizeof s->pose);
  std::memcpy(pose, s->pose, sizeof s->pose);
}

// kNN-5 of Q queries against one map (cross-check hook): idx/d2 [Q][5]; returns #accepted and
// writes -1 indices for rejected queries.
extern "C" int32_t ORACLE_FN(knn5_batch)(const float* map, int32_t M, const float* q, int32_t Q, int32_t* idx,
                                         float* d2) {
  Knn k;
  k.build(reinterpret_cast<const P4*>(map), M);
  int acc = 0;
  for (int i = 0; i < Q; ++i) {
    if (k.knn5(reinterpret_cast<const P4*>(q)[i], idx + 5 * i, d2 + 5 * i) == 5) {
      ++acc;
    } else {
      for (int j = 0; j < 5; ++j) { idx[5 * i + j] = -1; d2[5 * i + j] = 0.0f; }
    }
  }
  return acc;
}

#ifndef LLSR_ORACLE_NANOFLANN
extern "C" int32_t oracle_eig3(const float* A, float* e, float* v) { return oeig::eig_sym3(A, e, v); }
extern "C" int32_t oracle_eig6(const float* A, float* e, float* v) { return oeig::eig_sym_n(A, 6, e, v); }
extern "C" void oracle_qr_solve_5x3(const float* A, const float* b, float* x) { oeig::colpiv_qr_solve(A, 5, 3, b, x); }
extern "C" void oracle_qr_solve_6x6(const float* A, const float* b, float* x) { oeig::colpiv_qr_solve(A, 6, 6, b, x); }
extern "C" void oracle_inverse3(const float* A, float* inv) { oeig::inverse3(A, inv); }
extern "C" void oracle_inverse6(const float* A, float* inv) { oeig::inverse_lu(A, 6, inv); }
#endif
