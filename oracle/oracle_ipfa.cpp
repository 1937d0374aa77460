// oracle_ipfa.cpp — TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Scalar CPU restatement of LeGO-LOAM-SR's ImageProjection (IP = imageProjection.cpp) and the
// FeatureAssociation feature stage (FA = featureAssociation.cpp), plus the PCL 1.10 pieces the
// reference calls (RandomSampleConsensus + SampleConsensusModelPlane, VoxelGrid). Types and
// operation order follow the reference as written (float vs double promotion noted inline);
// build with -O3 -ffp-contract=off like the reference's baseline x86-64 build (no FMA).
// Unqualified float math resolves to the float overloads.
#include "oracle.h"
#include "oracle_voxel.h"

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstring>
#include <random>
#include <vector>

namespace {

const double kDegToRad = M_PI / 180.0;  // utility.h:49 (double)

struct P4 { float x, y, z, i; };

// x86-64 cvttss2si/cvttsd2si: NaN and out-of-range give INT_MIN (the reference's build target).
inline int trunc_i32(double v) {
  if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
  return (int)v;
}

// ------------------------------------------------------------------------------------------
// PCL 1.10 RandomSampleConsensus<PointXYZI> with SampleConsensusModelPlane (IP:716-721).
// Model RNG: boost::mt19937 seeded 12345 per model instance, drawn through
// boost::uniform_int<>(0, INT_MAX) => raw >> 1 (bucket size 2). Eigen's SSE reductions pair
// lanes (0+2)+(1+3) for 4-float dot/squaredNorm.
// ------------------------------------------------------------------------------------------
struct PlaneRansac {
  const std::vector<P4>* pts;
  std::vector<int> shuffled;
  std::mt19937 gen;
  int iterations = 0;
  explicit PlaneRansac(const std::vector<P4>& p, uint32_t seed) : pts(&p), gen(seed) {
    shuffled.resize(p.size());
    for (size_t k = 0; k < p.size(); ++k) shuffled[k] = (int)k;
  }
  int rnd() { return (int)(gen() >> 1); }
  static float dot4(const float a[4], const float b[4]) {
    return (a[0] * b[0] + a[2] * b[2]) + (a[1] * b[1] + a[3] * b[3]);
  }
  bool good(const int s[3]) const {
    const P4 &p0 = (*pts)[s[0]], &p1 = (*pts)[s[1]], &p2 = (*pts)[s[2]];
    float r0 = (p1.x - p0.x) / (p2.x - p0.x), r1 = (p1.y - p0.y) / (p2.y - p0.y),
          r2 = (p1.z - p0.z) / (p2.z - p0.z);
    return (r0 != r1) || (r2 != r1);
  }
  bool sample(int s[3]) {  // SampleConsensusModel::getSamples, max_sample_checks_ = 1000
    const size_t n = shuffled.size();
    for (int tries = 0; tries < 1000; ++tries) {
      for (size_t k = 0; k < 3; ++k)
        std::swap(shuffled[k], shuffled[k + (size_t)rnd() % (n - k)]);
      s[0] = shuffled[0]; s[1] = shuffled[1]; s[2] = shuffled[2];
      if (good(s)) return true;
    }
    return false;
  }
  bool fit(const int s[3], float c[4]) const {  // computeModelCoefficients
    const P4 &p0 = (*pts)[s[0]], &p1 = (*pts)[s[1]], &p2 = (*pts)[s[2]];
    float a0 = p1.x - p0.x, a1 = p1.y - p0.y, a2 = p1.z - p0.z;
    float b0 = p2.x - p0.x, b1 = p2.y - p0.y, b2 = p2.z - p0.z;
    float r0 = a0 / b0, r1 = a1 / b1, r2 = a2 / b2;
    if (r0 == r1 && r2 == r1) return false;
    c[0] = a1 * b2 - a2 * b1;
    c[1] = a2 * b0 - a0 * b2;
    c[2] = a0 * b1 - a1 * b0;
    c[3] = 0.0f;
    float sq = (c[0] * c[0] + c[2] * c[2]) + (c[1] * c[1] + c[3] * c[3]);
    if (sq > 0.0f) {
      float nrm = std::sqrt(sq);
      for (int k = 0; k < 4; ++k) c[k] = c[k] / nrm;
    }
    float p[4] = {p0.x, p0.y, p0.z, 1.0f};
    c[3] = -1.0f * dot4(c, p);
    return true;
  }
  float dist(const float c[4], const P4& q) const {
    float p[4] = {q.x, q.y, q.z, 1.0f};
    return std::fabs(dot4(c, p));
  }
  // RandomSampleConsensus::computeModel + getInliers; threshold 0.5 (IP:719).
  void run(double thr, std::vector<int>& inliers) {
    inliers.clear();
    const int K = (int)pts->size();
    const int max_iterations = 10000;  // RandomSampleConsensus ctor
    const double probability = 0.99;
    iterations = 0;
    if (K < 3) { iterations = INT_MAX - 1; return; }
    int best = -INT_MAX;
    double k = 1.0;
    const double log_probability = std::log(1.0 - probability);
    const double one_over_indices = 1.0 / (double)K;
    unsigned skipped = 0;
    const unsigned max_skip = (unsigned)max_iterations * 10u;
    float bestc[4] = {0, 0, 0, 0};
    bool have = false;
    while (iterations < k && skipped < max_skip) {
      int s[3];
      if (!sample(s)) break;
      float c[4];
      if (!fit(s, c)) { ++skipped; continue; }
      int cnt = 0;
      for (int q = 0; q < K; ++q)
        if ((double)dist(c, (*pts)[q]) < thr) ++cnt;
      if (cnt > best) {
        best = cnt;
        std::memcpy(bestc, c, sizeof bestc);
        have = true;
        double w = (double)best * one_over_indices;
        double p_no = 1.0 - std::pow(w, 3.0);
        p_no = std::max(std::numeric_limits<double>::epsilon(), p_no);
        p_no = std::min(1.0 - std::numeric_limits<double>::epsilon(), p_no);
        k = log_probability / std::log(p_no);
      }
      ++iterations;
      if (iterations > max_iterations) break;
    }
    if (!have) return;
    for (int q = 0; q < K; ++q)
      if ((double)dist(bestc, (*pts)[q]) < thr) inliers.push_back(q);
  }
};

// PCL 1.10 VoxelGrid<PointXYZI>::applyFilter (FA:1268-1270), restated in oracle_voxel.h.
void voxel_grid(const std::vector<P4>& in, float leaf, std::vector<P4>& out, bool stable) {
  std::vector<float> o;
  oracle_voxel::voxel_grid(reinterpret_cast<const float*>(in.data()), in.size(), leaf, o, stable);
  out.resize(o.size() / 4);
  std::memcpy(out.data(), o.data(), o.size() * sizeof(float));
}

}  // namespace

// ------------------------------------------------------------------------------------------
struct oracle_state {
  // false (default): the less-flat VoxelGrid sums each voxel in std::sort's order, as PCL
  // (LLSR_VOXEL_ORDER_PCL, the device's default); true: in input order (LLSR_VOXEL_ORDER_INPUT)
  bool vg_stable = false;
  llsr_config cfg;
  int H, W, HW;
  // IP derived constants (IP:117-121, 849)
  float ip_resX, ip_resY, ip_angBottom, segTheta, segThr, sinX, cosX, sinY, cosY;
  // FA derived constants (FA:152-154, 415-431)
  float fa_resX, fa_resY, sinResX;
  std::vector<P4> shadow;  // GenerateShadowPoint
  // FA carry-over (FA:168-198): sized H*W once, never cleared.
  std::vector<std::pair<float, size_t>> smooth;
  std::vector<float> curv;
  std::vector<int> picked, pickedPlane, clabel;
  // last-scan scratch kept for oracle_ransac_inliers
  std::vector<P4> near;
  double ip_ms = 0, fa_ms = 0;
};

static void init_consts(oracle_state* s) {
  const llsr_config& c = s->cfg;
  s->H = c.num_vertical_scans;
  s->W = c.num_horizontal_scans;
  s->HW = s->H * s->W;
  s->ip_resX = (float)((M_PI * 2) / s->W);
  s->ip_resY = (float)(kDegToRad * (c.vertical_angle_top - c.vertical_angle_bottom) / float(s->H - 1));
  s->ip_angBottom = (float)(-(c.vertical_angle_bottom - 0.1) * kDegToRad);
  s->segTheta = (float)(c.segment_theta * kDegToRad);
  s->segThr = std::tan(s->segTheta);
  s->sinX = std::sin(s->ip_resX); s->cosX = std::cos(s->ip_resX);
  s->sinY = std::sin(s->ip_resY); s->cosY = std::cos(s->ip_resY);
  s->fa_resX = (float)((M_PI * 2) / s->W);
  s->fa_resY = (float)(kDegToRad * (c.vertical_angle_top - c.vertical_angle_bottom) / float(s->H - 1));
  s->sinResX = std::sin(s->fa_resX);
  // GenerateShadowPoint (FA:412-432): doubles, stored through float members.
  s->shadow.clear();
  const int row_size = 16, col_size = 10;
  const double row_angle = (std::atan2(0.120, 0.05) * 2) / (row_size - 1);
  const double col_angle = (std::atan2(0.077, 0.05) * 2) / (col_size - 1);
  const double l2b[3] = {0.008, 0.0, -0.035};
  for (int r = 0; r < row_size; ++r) {
    float row_x = (float)(0.05 * std::tan((((row_size - 1.0) / 2.0) * row_angle) - (r * row_angle)));
    for (int q = 0; q < col_size; ++q) {
      float col_y = (float)(0.05 * std::tan((((col_size - 1.0) / 2.0) * col_angle) - (q * col_angle)));
      P4 p;
      p.x = (float)(col_y + l2b[1]);
      p.y = (float)(-(0.035f + 0.05f) + l2b[2]);
      p.z = (float)(row_x + l2b[0]);
      p.i = (float)((float)r + (float)17 + (float)q / 10000.0);
      s->shadow.push_back(p);
    }
  }
}

extern "C" oracle_state* oracle_create(const llsr_config* cfg) {
  if (!cfg || cfg->use_vlp32c || cfg->num_vertical_scans < 2 || cfg->num_horizontal_scans < 16)
    return nullptr;
  oracle_state* s = new oracle_state();
  s->cfg = *cfg;
  init_consts(s);
  oracle_reset(s);
  return s;
}

extern "C" void oracle_destroy(oracle_state* s) { delete s; }

extern "C" void oracle_reset(oracle_state* s) {
  s->smooth.assign(s->HW, {0.0f, 0});
  s->curv.assign(s->HW, 0.0f);
  s->picked.assign(s->HW, 0);
  s->pickedPlane.assign(s->HW, 0);
  s->clabel.assign(s->HW, 0);
}

extern "C" void oracle_stage_ms(const oracle_state* s, double* ip, double* fa) {
  if (ip) *ip = s->ip_ms;
  if (fa) *fa = s->fa_ms;
}

// libstdc++ std::sort by value (the comparator of FA:1172, utility.h:57-61) of n values; out[k] =
// the input position at sorted position k (test hook for the device's exact tie order).
extern "C" void oracle_std_sort_by_value(const float* vals, int32_t n, int32_t* out) {
  std::vector<std::pair<float, size_t>> v((size_t)n);
  for (int k = 0; k < n; ++k) v[k] = {vals[k], (size_t)k};
  std::sort(v.begin(), v.end(),
            [](const std::pair<float, size_t>& a, const std::pair<float, size_t>& b) { return a.first < b.first; });
  for (int k = 0; k < n; ++k) out[k] = (int32_t)v[k].second;
}

// cloudSmoothness[4].ind, the entry the next frame's ring-0 sort starts from (test hook)
extern "C" int32_t oracle_phantom_index(const oracle_state* s) { return (int32_t)s->smooth[4].second; }
extern "C" void oracle_set_voxel_order(oracle_state* s, int32_t pcl) { s->vg_stable = pcl == 0; }

extern "C" int32_t oracle_ransac_inliers(oracle_state* s, uint32_t seed, int32_t* out, int32_t cap) {
  PlaneRansac rs(s->near, seed);
  std::vector<int> inl;
  rs.run(0.5, inl);
  int n = (int)inl.size();
  for (int k = 0; k < n && k < cap; ++k) out[k] = inl[k];
  return n;
}

// ------------------------------------------------------------------------------------------
extern "C" int32_t oracle_process_scan(oracle_state* s, const float* xyzi, int32_t nraw,
                                       llsr_scan_out* out) {
  if (!s || !out || nraw < 0 || (nraw > 0 && !xyzi)) return LLSR_EINVAL;
  const llsr_config& cfg = s->cfg;
  const int H = s->H, W = s->W, HW = s->HW;
  auto t0 = std::chrono::steady_clock::now();

  // ---- cloudHandler: resetParameters (IP:147-187) + removeNaNFromPointCloud (IP:196-198) ----
  std::vector<P4> cloud;
  std::vector<int> rawIndex;
  cloud.reserve(nraw);
  for (int k = 0; k < nraw; ++k) {
    P4 p{xyzi[4 * k], xyzi[4 * k + 1], xyzi[4 * k + 2], xyzi[4 * k + 3]};
    if (!std::isfinite(p.x) || !std::isfinite(p.y) || !std::isfinite(p.z)) continue;
    cloud.push_back(p);
    rawIndex.push_back(k);
  }
  const int N = (int)cloud.size();
  const float qnan = std::numeric_limits<float>::quiet_NaN();
  std::vector<float> rangeMat(HW, FLT_MAX);
  std::vector<int8_t> g(HW, 0);
  std::vector<int> lab(HW, 0);
  std::vector<int> cellPt(HW, -1);
  std::vector<P4> full(HW, P4{qnan, qnan, qnan, 0.0f});
  std::vector<P4> visual(HW, P4{qnan, qnan, qnan, 0.0f});

  // ---- findStartEndAngle (IP:430-445) ----
  float ori[3] = {0, 0, 0};
  if (N > 0) {
    const P4& a = cloud.front();
    const P4& b = cloud.back();
    ori[0] = -std::atan2(a.y, a.x);
    ori[1] = (float)(-std::atan2(b.y, b.x) + 2 * M_PI);
    if (ori[1] - ori[0] > 3 * M_PI) ori[1] = (float)(ori[1] - 2 * M_PI);
    else if (ori[1] - ori[0] < M_PI) ori[1] = (float)(ori[1] + 2 * M_PI);
    ori[2] = ori[1] - ori[0];
  }

  // ---- projectPointCloud, non-VLP-32c branch (IP:301-348) ----
  for (int k = 0; k < N; ++k) {
    P4 p = cloud[k];
    float range = std::sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    float va = std::asin(p.z / range);
    int row = trunc_i32((double)((va + s->ip_angBottom) / s->ip_resY));
    if (row < 0 || row >= H) continue;
    float ha = std::atan2(p.x, p.y);
    int col = trunc_i32(-std::round(((double)ha - M_PI_2) / (double)s->ip_resX) + W * 0.5);
    if (col >= W) col -= W;
    if (col < 0 || col >= W) continue;
    if (range < 0.1) continue;
    const int cell = col + row * W;
    rangeMat[cell] = range;
    visual[cell] = p;
    p.i = (float)((double)(float)row + (double)(float)col / 10000.0);
    full[cell] = p;
    cellPt[cell] = rawIndex[k];
  }

  // ---- groundRemovalOurs: column pass + Filter (IP:524-629) ----
  for (int j = 0; j < W; ++j) {
    bool haveRV = false, obs = false;
    float RVx = 0, RVy = 0, RVz = 0;
    int lower = 0;
    for (int i = 0; i < H; ++i) {
      const int c = j + i * W;
      if (full[c].i == 0) { g[c] = -1; continue; }
      if (!haveRV) {
        float d0 = std::sqrt(full[c].x * full[c].x + full[c].y * full[c].y);
        RVx = full[c].x / d0; RVy = full[c].y / d0; RVz = 0;
        haveRV = true; lower = c; g[c] = 1;
      } else {
        float TVx = full[c].x - full[lower].x, TVy = full[c].y - full[lower].y,
              TVz = full[c].z - full[lower].z;
        float ang = (float)(std::acos((TVx * RVx + TVy * RVy + TVz * RVz) /
                                      (std::sqrt(TVx * TVx + TVy * TVy + TVz * TVz) *
                                       std::sqrt(RVx * RVx + RVy * RVy + RVz * RVz))) / kDegToRad);
        g[c] = 1;
        float D;
        if (cfg.use_kitti) D = i < 16 ? 60.0f : 25.0f;
        else D = 12.5f;
        if (ang <= D) { RVx += TVx; RVy += TVy; RVz += TVz; g[c] = 1; }
        else g[c] = 0;
        lower = c;
      }
    }
    for (int i = 0; i < H; ++i) {
      const int c = j + i * W;
      if (g[c] != 0 && !obs) continue;
      obs = true;
      if (g[c] == 1) g[c] = 2;
    }
  }
  // ---- ADD (IP:631-671): forward then backward recurrence per row ----
  auto addTest = [&](int c, int nb) {
    const P4 &p = full[c], &q = full[nb];
    float r = std::sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    float dx = p.x - q.x, dy = p.y - q.y, dz = p.z - q.z;
    float dr = std::sqrt(dx * dx + dy * dy + dz * dz);
    return (double)dr <= 0.061 * (double)r && (double)dz <= 0.1;
  };
  for (int i = 0; i < H; ++i) {
    for (int j = 2; j < W; ++j) {
      const int c = j + i * W;
      if (g[c] != 2) continue;
      bool nb = g[c - 2] == 1 || g[c - 1] == 1;
      if (nb && addTest(c, c - 2)) g[c] = 1;
    }
    for (int j = W - 3; j > -1; --j) {
      const int c = j + i * W;
      if (g[c] != 2) continue;
      bool nb = g[c + 2] == 1 || g[c + 1] == 1;
      if (nb && addTest(c, c + 2)) g[c] = 1;
    }
  }
  // ---- ELEVATION (IP:673-698): last-valid carry across columns ----
  {
    float EHt = -1.3f, EH = -1.3f;
    for (int j = 0; j < W; ++j) {
      int cnt = 0;
      for (int i = 0; i < H; ++i)
        if (g[j + i * W] == 1) { ++cnt; EHt = full[j + i * W].z; }
      if (cnt >= 5) EH = EHt;
      for (int i = 0; i < H; ++i) {
        const int c = j + i * W;
        if (g[c] == 2) g[c] = ((double)full[c].z < (double)EH + 0.3) ? 1 : 0;
      }
    }
  }
  // ---- NEAR + RANSAC (IP:700-735) ----
  s->near.clear();
  for (int c = 0; c < HW; ++c) {
    float depth = std::sqrt(full[c].x * full[c].x + full[c].y * full[c].y);
    if ((double)depth <= 10 && g[c] == 1) {
      P4 p = full[c];
      p.i = (float)c;
      s->near.push_back(p);
      if ((double)depth <= 5) g[c] = 0;
    }
  }
  std::vector<int> inl;
  PlaneRansac rs(s->near, 12345u);
  rs.run(0.5, inl);
  for (int q : inl) {
    int c = (int)s->near[q].i;
    float depth = std::sqrt(full[c].x * full[c].x + full[c].y * full[c].y);
    if ((double)depth <= 5) g[c] = 1;
  }
  // ---- Push Back (IP:751-759) ----
  for (int c = 0; c < HW; ++c)
    if (g[c] == 1 || rangeMat[c] == FLT_MAX) lab[c] = -1;

  // ---- cloudSegmentation: BFS labelComponents (IP:783-789, 847-931) ----
  {
    int labelCount = 1;
    std::vector<int> queue(HW), all(HW);
    std::vector<char> lineFlag(H);
    const int di[4] = {0, -1, 1, 0}, dj[4] = {-1, 0, 0, 1};
    for (int seed = 0; seed < HW; ++seed) {
      if (lab[seed] != 0) continue;
      int qh = 0, qt = 0, na = 0;
      std::fill(lineFlag.begin(), lineFlag.end(), 0);
      queue[qt++] = seed;
      all[na++] = seed;
      while (qh < qt) {
        const int from = queue[qh++];
        const int fi = from / W, fj = from % W;
        lab[from] = labelCount;
        for (int d = 0; d < 4; ++d) {
          int ni = fi + di[d], nj = fj + dj[d];
          if (ni < 0 || ni >= H) continue;
          if (nj < 0) nj = W - 1;
          if (nj >= W) nj = 0;
          const int to = nj + ni * W;
          if (lab[to] != 0) continue;
          float d1 = std::max(rangeMat[from], rangeMat[to]);
          float d2 = std::min(rangeMat[from], rangeMat[to]);
          float sA = di[d] == 0 ? s->sinX : s->sinY;
          float cA = di[d] == 0 ? s->cosX : s->cosY;
          float tang = d2 * sA / (d1 - d2 * cA);
          if (tang > s->segThr) {
            queue[qt++] = to;
            lab[to] = labelCount;
            lineFlag[ni] = 1;
            all[na++] = to;
          }
        }
      }
      bool feasible = false;
      if (na >= 30) feasible = true;
      else if (na >= cfg.segment_valid_point_num) {
        int lines = 0;
        for (int i = 0; i < H; ++i) lines += lineFlag[i] ? 1 : 0;
        if (lines >= cfg.segment_valid_line_num) feasible = true;
      }
      if (feasible) ++labelCount;
      else for (int k = 0; k < na; ++k) lab[all[k]] = 999999;
    }
  }
  // ---- segmented / outlier extraction (IP:791-832) ----
  std::vector<P4> seg, outl;
  std::vector<float> segInt, outInt, segRange;
  std::vector<uint8_t> segGround;
  std::vector<uint32_t> segCol;
  std::vector<int32_t> startRing(H), endRing(H);
  int S = 0;
  for (int i = 0; i < H; ++i) {
    startRing[i] = S - 1 + 5;
    for (int j = 0; j < W; ++j) {
      const int c = j + i * W;
      if (lab[c] > 0 || g[c] == 1) {
        if (lab[c] == 999999) {
          if (i > cfg.ground_scan_index && j % 5 == 0) {
            outl.push_back(full[c]);
            outInt.push_back(visual[c].i);
          }
          continue;
        }
        if (g[c] == 1 && (j % 5 != 0 && j > 5 && j < W - 5)) continue;
        segGround.push_back(g[c] == 1);
        segCol.push_back((uint32_t)j);
        segRange.push_back(rangeMat[c]);
        seg.push_back(full[c]);
        segInt.push_back(visual[c].i);
        ++S;
      }
    }
    endRing[i] = S - 1 - 5;
  }
  auto t1 = std::chrono::steady_clock::now();

  // ================= FeatureAssociation feature stage (FA:2766-2775) =================
  // CloudInfo arrays have length H*W (IP:184-186): zero beyond S.
  std::vector<uint32_t> colInd(HW, 0u);
  std::vector<float> rng(HW, 0.0f);
  std::vector<uint8_t> gflag(HW, 0);
  for (int k = 0; k < S; ++k) { colInd[k] = segCol[k]; rng[k] = segRange[k]; gflag[k] = segGround[k]; }

  // ---- adjustDistortion (FA:565-598, IMU block skipped: imuPointerLast < 0) ----
  std::vector<P4> pc(S);
  {
    bool halfPassed = false;
    for (int k = 0; k < S; ++k) {
      P4 p;
      p.x = seg[k].y; p.y = seg[k].z; p.z = seg[k].x;
      float o = -std::atan2(p.x, p.z);
      if (!halfPassed) {
        if (o < ori[0] - M_PI / 2) o = (float)(o + 2 * M_PI);
        else if (o > ori[0] + M_PI * 3 / 2) o = (float)(o - 2 * M_PI);
        if (o - ori[0] > M_PI) halfPassed = true;
      } else {
        o = (float)(o + 2 * M_PI);
        if (o < ori[1] - M_PI * 3 / 2) o = (float)(o + 2 * M_PI);
        else if (o > ori[1] + M_PI / 2) o = (float)(o - 2 * M_PI);
      }
      float relTime = (o - ori[0]) / ori[2];
      p.i = (float)(int)(seg[k].i) + cfg.scan_period * relTime;
      pc[k] = p;
    }
  }
  // ---- calculateSmoothnessOurs (FA:817-848) ----
  for (int k = 5; k < S - 5; ++k) {
    float dx = 0, dy = 0, dz = 0;
    for (int q = -5; q < 6; ++q) dx += pc[k + q].x;
    dx -= 11 * pc[k].x;
    for (int q = -5; q < 6; ++q) dy += pc[k + q].y;
    dy -= 11 * pc[k].y;
    for (int q = -5; q < 6; ++q) dz += pc[k + q].z;
    dz -= 11 * pc[k].z;
    float c = std::sqrt(dx * dx + dy * dy + dz * dz) /
              std::sqrt(pc[k].x * pc[k].x + pc[k].y * pc[k].y + pc[k].z * pc[k].z) / 10;
    s->curv[k] = c;
    s->picked[k] = 0;
    s->pickedPlane[k] = 0;
    s->clabel[k] = 0;
    s->smooth[k] = {c, (size_t)k};
  }
  // ---- markOccludedPoints (FA:851-899) ----
  for (int k = 5; k < S - 6; ++k) {
    float d1 = rng[k], d2 = rng[k + 1];
    int colDiff = std::abs(int(colInd[k + 1] - colInd[k]));
    if (colDiff < 10) {
      if (d1 - d2 > 0.3) {
        for (int q = k - 5; q <= k; ++q) s->picked[q] = s->pickedPlane[q] = 1;
      } else if (d2 - d1 > 0.3) {
        for (int q = k + 1; q <= k + 6; ++q) s->picked[q] = s->pickedPlane[q] = 1;
      }
    }
    float diff1 = std::fabs(float(rng[k - 1] - rng[k]));
    float diff2 = std::fabs(float(rng[k + 1] - rng[k]));
    if (diff1 > 0.02 * rng[k] && diff2 > 0.02 * rng[k]) s->picked[k] = s->pickedPlane[k] = 1;
  }
  // ---- extractFeaturesOurs (FA:1159-1272) ----
  std::vector<int> lessSharp, flat;
  std::vector<P4> lessFlat;
  const int colSize = HW;  // segmented_cloud_col_ind.size()
  auto suppress = [&](int ind) {
    s->picked[ind] = 1;
    for (int l = 1; l <= 5; ++l) {
      if (ind + l >= colSize) continue;
      int cd = std::abs(int(colInd[ind + l] - colInd[ind + l - 1]));
      if (cd > 10) break;
      s->picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; --l) {
      if (ind + l < 0) continue;
      int cd = std::abs(int(colInd[ind + l] - colInd[ind + l + 1]));
      if (cd > 10) break;
      s->picked[ind + l] = 1;
    }
  };
  for (int i = 0; i < H; ++i) {
    const int sp = startRing[i], ep = endRing[i] - 1;
    if (sp >= ep) continue;
    std::sort(s->smooth.begin() + sp, s->smooth.begin() + ep,
              [](const std::pair<float, size_t>& a, const std::pair<float, size_t>& b) {
                return a.first < b.first;
              });
    for (int k = ep; k >= sp; --k) {
      const int ind = (int)s->smooth[k].second;
      if (s->picked[ind] == 0 && s->curv[ind] > cfg.edge_threshold && gflag[ind] == 0) {
        s->clabel[ind] = 1;
        lessSharp.push_back(ind);
        suppress(ind);
      }
    }
    for (int k = sp; k <= ep; ++k) {
      const int ind = (int)s->smooth[k].second;
      if (s->picked[ind] == 0 && s->curv[ind] < cfg.surf_threshold && gflag[ind] == 1) {
        s->clabel[ind] = -1;
        flat.push_back(ind);
        suppress(ind);
      }
    }
    std::vector<P4> ringLess, ringDS;
    for (int k = sp; k <= ep; ++k)
      if (s->clabel[k] <= 0) ringLess.push_back(pc[k]);
    voxel_grid(ringLess, 0.2f, ringDS, s->vg_stable);
    lessFlat.insert(lessFlat.end(), ringDS.begin(), ringDS.end());
  }
  // ---- DBSCAN_EdgeFeature (FA:1318-1387) ----
  const int M = (int)lessSharp.size();
  std::vector<int> cluster(M, 0);
  {
    std::vector<float> kxy(M), kz(M);
    for (int a = 0; a < M; ++a) {
      const P4& p = pc[lessSharp[a]];
      float x0 = p.z, y0 = p.x, z0 = p.y;
      float AB = std::atan2(z0, std::sqrt(x0 * x0 + y0 * y0));
      kxy[a] = std::sqrt(x0 * x0 + y0 * y0) * s->sinResX * cfg.RatioXY;
      kz[a] = (std::sqrt(x0 * x0 + y0 * y0) * std::tan(AB + s->fa_resY) -
               std::sqrt(x0 * x0 + y0 * y0) * std::tan(AB - s->fa_resY)) / 2 * cfg.RatioZ;
    }
    int label = 0;
    std::vector<int> inIdx, inLab;
    for (int a = 0; a < M; ++a) {
      cluster[a] = 0;
      const P4& pa = pc[lessSharp[a]];
      float x0 = pa.z, y0 = pa.x, z0 = pa.y;
      inIdx.clear(); inLab.clear();
      for (int b = 0; b < M; ++b) {
        const P4& pb = pc[lessSharp[b]];
        float xj = pb.z, yj = pb.x, zj = pb.y;
        float eps = std::sqrt((x0 - xj) * (x0 - xj) / (kxy[b] * kxy[b]) +
                              (y0 - yj) * (y0 - yj) / (kxy[b] * kxy[b]) +
                              (z0 - zj) * (z0 - zj) / (kz[b] * kz[b]));
        if (eps <= cfg.DBFr) { inIdx.push_back(b); inLab.push_back(cluster[b]); }
      }
      int minLab = 999999999;
      for (int b : inIdx)
        if (cluster[b] != 0 && cluster[b] < minLab) minLab = cluster[b];
      if (minLab <= label) {
        std::sort(inLab.begin(), inLab.end());
        inLab.erase(std::unique(inLab.begin(), inLab.end()), inLab.end());
        for (int b = 0; b < M; ++b)
          for (int L : inLab)
            if (cluster[b] == L) cluster[b] = minLab;
        for (int b : inIdx) cluster[b] = minLab;
      } else {
        label += 1;
        for (int b : inIdx) cluster[b] = label;
      }
    }
  }
  // cluster run lengths, last run dropped (FA:1281-1305)
  std::vector<int> sharp;
  {
    std::vector<int> sorted = cluster;
    std::sort(sorted.begin(), sorted.end());
    std::vector<int> runs;
    int cnt = 1;
    for (int a = 0; a < (int)sorted.size() - 1; ++a) {
      if (sorted[a + 1] - sorted[a] == 0) ++cnt;
      else { runs.push_back(cnt); cnt = 1; }
    }
    std::vector<int> inlierLab;
    for (int a = 0; a < (int)runs.size(); ++a)
      if (runs[a] >= 4) inlierLab.push_back(a + 1);
    for (int a = 0; a < M; ++a)
      for (int L : inlierLab)
        if (cluster[a] == L) sharp.push_back(lessSharp[a]);
  }
  auto t2 = std::chrono::steady_clock::now();
  s->ip_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
  s->fa_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();

  // ================= outputs =================
  out->n_points = N;
  std::memcpy(out->orientation, ori, sizeof ori);
  if (out->range_image) std::memcpy(out->range_image, rangeMat.data(), sizeof(float) * HW);
  if (out->cell_point) std::memcpy(out->cell_point, cellPt.data(), sizeof(int32_t) * HW);
  if (out->ground_image) std::memcpy(out->ground_image, g.data(), HW);
  if (out->label_image) std::memcpy(out->label_image, lab.data(), sizeof(int32_t) * HW);
  if (out->start_ring_index) std::memcpy(out->start_ring_index, startRing.data(), 4 * H);
  if (out->end_ring_index) std::memcpy(out->end_ring_index, endRing.data(), 4 * H);
  out->n_segmented = S;
  for (int k = 0; k < S; ++k) {
    if (out->seg_xyzi) std::memcpy(out->seg_xyzi + 4 * k, &seg[k], 16);
    if (out->seg_ground_flag) out->seg_ground_flag[k] = segGround[k];
    if (out->seg_col_ind) out->seg_col_ind[k] = segCol[k];
    if (out->seg_range) out->seg_range[k] = segRange[k];
    if (out->seg_intensity) out->seg_intensity[k] = segInt[k];
    if (out->loam_xyzi) std::memcpy(out->loam_xyzi + 4 * k, &pc[k], 16);
    if (out->curvature) out->curvature[k] = (k >= 5 && k < S - 5) ? s->curv[k] : 0.0f;
    if (out->picked) out->picked[k] = (uint8_t)s->picked[k];
    if (out->label) out->label[k] = (int8_t)s->clabel[k];
  }
  out->n_outlier = (int32_t)outl.size();
  for (size_t k = 0; k < outl.size(); ++k) {
    if (out->outlier_xyzi) std::memcpy(out->outlier_xyzi + 4 * k, &outl[k], 16);
    if (out->outlier_intensity) out->outlier_intensity[k] = outInt[k];
  }
  out->n_near = (int32_t)s->near.size();
  out->n_ransac_inliers = (int32_t)inl.size();
  out->ransac_iterations = rs.iterations;
  out->n_less_sharp = M;
  for (int a = 0; a < M; ++a) {
    if (out->less_sharp_ind) out->less_sharp_ind[a] = lessSharp[a];
    if (out->dbscan_cluster) out->dbscan_cluster[a] = cluster[a];
  }
  out->n_sharp = (int32_t)sharp.size();
  if (out->sharp_ind) std::copy(sharp.begin(), sharp.end(), out->sharp_ind);
  out->n_flat = (int32_t)flat.size();
  if (out->flat_ind) std::copy(flat.begin(), flat.end(), out->flat_ind);
  out->n_less_flat = (int32_t)lessFlat.size();
  if (out->less_flat_xyzi)
    for (size_t k = 0; k < lessFlat.size(); ++k) std::memcpy(out->less_flat_xyzi + 4 * k, &lessFlat[k], 16);
  return LLSR_OK;
}
