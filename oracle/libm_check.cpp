// libm_check.cpp — TEST INFRASTRUCTURE (oracle/). Pins the device libm restatement
// (lego-loam-sr_amd/csrc/llsr_libm.h) against the host glibc float functions the reference
// links (imageProjection.cpp:313,321,559; featureAssociation.cpp:577,1330-1332).
//
//   libm_check [stride] [threads] [only]   (only: run just the functions whose name starts so)
// stride=1 sweeps all 2^32 inputs per unary function; atan2f is checked on a dense grid of
// (y, x) pairs plus every exponent/sign combination. Exit status = number of mismatching
// functions (0 = bit-identical everywhere tested).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <atomic>
#include "../lego-loam-sr_amd/csrc/llsr_libm.h"

using namespace llsr_libm;

static bool same(float a, float b) {
  if (std::isnan(a) && std::isnan(b)) return true;
  return fbits(a) == fbits(b);
}

static const char* g_only = "";
template <class F, class G>
static long sweep(const char* name, F port, G ref, uint64_t lo, uint64_t hi, uint64_t stride,
                  int nthreads) {
  if (std::strncmp(name, g_only, std::strlen(g_only)) != 0) return 0;
  std::atomic<long> bad{0};
  std::atomic<int> shown{0};
  std::vector<std::thread> th;
  for (int t = 0; t < nthreads; ++t) {
    th.emplace_back([&, t]() {
      for (uint64_t u = lo + (uint64_t)t * stride; u < hi; u += stride * (uint64_t)nthreads) {
        float x = bitsf((uint32_t)u);
        float a = port(x), b = ref(x);
        if (!same(a, b)) {
          if (shown.fetch_add(1) < 5)
            std::printf("  %s mismatch x=%a (0x%08x): port=%a glibc=%a\n", name, x, (uint32_t)u, a, b);
          bad.fetch_add(1);
        }
      }
    });
  }
  for (auto& x : th) x.join();
  std::printf("%-8s [%08llx,%08llx) stride %llu: %ld mismatches\n", name, (unsigned long long)lo,
              (unsigned long long)hi, (unsigned long long)stride, bad.load());
  return bad.load();
}

int main(int argc, char** argv) {
  uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  int nthreads = argc > 2 ? atoi(argv[2]) : (int)std::thread::hardware_concurrency();
  if (nthreads < 1) nthreads = 1;
  g_only = argc > 3 ? argv[3] : "";
  int failed = 0;
  const uint64_t ALL = 1ull << 32;
  failed += sweep("asinf", asinf_, [](float x) { return std::asin(x); }, 0, ALL, stride, nthreads) != 0;
  failed += sweep("acosf", acosf_, [](float x) { return std::acos(x); }, 0, ALL, stride, nthreads) != 0;
  failed += sweep("atanf", atanf_, [](float x) { return std::atan(x); }, 0, ALL, stride, nthreads) != 0;
  // tanf: |x| < 120 (0x42f00000) for both signs — the restated domain.
  failed += sweep("tanf+", tanf_, [](float x) { return std::tan(x); }, 0, 0x42f00000ull, stride, nthreads) != 0;
  failed += sweep("tanf-", tanf_, [](float x) { return std::tan(x); }, 0x80000000ull,
                  0x80000000ull + 0x42f00000ull, stride, nthreads) != 0;
  // sinf / cosf on |x| < 120 (glibc's reduce_fast domain; the restated domain)
  failed += sweep("sinf+", sinf_, [](float x) { return std::sin(x); }, 0, 0x42f00000ull, stride, nthreads) != 0;
  failed += sweep("sinf-", sinf_, [](float x) { return std::sin(x); }, 0x80000000ull, 0x80000000ull + 0x42f00000ull, stride, nthreads) != 0;
  failed += sweep("cosf+", cosf_, [](float x) { return std::cos(x); }, 0, 0x42f00000ull, stride, nthreads) != 0;
  failed += sweep("cosf-", cosf_, [](float x) { return std::cos(x); }, 0x80000000ull, 0x80000000ull + 0x42f00000ull, stride, nthreads) != 0;
  // atan2f: y sweeps a strided subset of all floats, x from a structured set.
  {
    std::vector<float> xs;
    const float base[] = {1.0f, -1.0f, 0.0f, -0.0f, INFINITY, -INFINITY, 1e-30f, -1e-30f,
                          3.0f, -7.5f, 1e30f, -1e30f, 0.3f, -0.3f, 1e-40f, 12.25f, -100.0f};
    for (float b : base) xs.push_back(b);
    uint32_t s = 12345u;
    for (int i = 0; i < 48; ++i) {  // random finite x over many magnitudes
      s = s * 1664525u + 1013904223u;
      xs.push_back(bitsf((s & 0x807fffffu) | ((uint32_t)(80 + (s >> 24) % 96) << 23)));
    }
    long bad = 0;
    for (float xv : xs) {
      bad += sweep("atan2f", [xv](float y) { return atan2f_(y, xv); },
                   [xv](float y) { return std::atan2(y, xv); }, 0, ALL, stride * 61, nthreads);
    }
    failed += bad != 0;
  }
  // ground angle test as a threshold on the cosine (llsr_libm.h ground_cos_threshold)
  for (float D : {12.5f, 25.0f, 60.0f}) {
    const float xs = ground_cos_threshold(D);
    char name[16];
    std::snprintf(name, sizeof name, "gnd%g", D);
    failed += sweep(name, [xs](float x) { return (float)(x >= xs && x <= 1.0f); },
                    [D](float x) { return (float)((float)((double)std::acos(x) / (M_PI / 180.0)) <= D); },
                    0, ALL, stride, nthreads) != 0;
  }
  std::printf("libm_check: %d function(s) with mismatches\n", failed);
  return failed;
}
