// llsr_libm.h — bit-exact restatements of the glibc (2.31–2.35, sysdeps/ieee754/flt-32)
// single-precision elementary functions that the LeGO-LOAM-SR hot path calls on floats.
//
// Why: the reference computes row/column indices, ground angles and DBSCAN scales with glibc
// float libm (imageProjection.cpp:313 asinf, :321 atan2f, :559 acosf; featureAssociation.cpp:577
// atan2f, :1330 atan2f, :1332 tanf). The device's own ocml functions round differently in a few
// ULPs, which flips row/column truncation and threshold tests. These ports follow the fdlibm
// algorithms glibc ships for these functions, written with explicit IEEE-754 single ops so they
// produce identical bits on the host (g++ -ffp-contract=off) and on gfx950 (hipcc
// -ffp-contract=off, correctly-rounded f32 divide/sqrt — hipcc's default).
//
// The float ports below follow fdlibm as shipped in glibc's sysdeps/ieee754/flt-32 (e_asinf.c,
// e_acosf.c, e_atan2f.c, s_atanf.c, k_tanf.c, s_tanf.c: "Conversion to float by Ian Lance Taylor,
// Cygnus Support, ian@cygnus.com"), whose notice is preserved as its licence requires:
//
//   ====================================================
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//
//   Developed at SunPro, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this
//   software is freely granted, provided that this notice
//   is preserved.
//   ====================================================
//
// Validation: oracle/libm_check.cpp compares every function against the host glibc over all
// 2^32 float inputs (asinf, acosf, atanf; tanf, sinf, cosf on |x| < 120) and over dense
// random/structured pairs for atan2f. See DESIGN.md §2.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define LLSR_HD __host__ __device__ __forceinline__
#else
#define LLSR_HD static inline
#endif

namespace llsr_libm {

LLSR_HD uint32_t fbits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __float_as_uint(f);
#else
  uint32_t u; memcpy(&u, &f, 4); return u;
#endif
}
LLSR_HD float bitsf(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __uint_as_float(u);
#else
  float f; memcpy(&f, &u, 4); return f;
#endif
}
LLSR_HD float fabs_(float x) { return bitsf(fbits(x) & 0x7fffffffu); }
// IEEE correctly-rounded single sqrt on both sides.
LLSR_HD float sqrt_(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_sqrtf(x);
#else
  return __builtin_sqrtf(x);
#endif
}

// ---- asinf: glibc e_asinf.c (x + x^3 p(x^2) form, pio2_hi rounded up) ----------------------
LLSR_HD float asinf_(float x) {
  const float one = 1.0f, huge = 1.0e30f;
  const float pio2_hi = 1.57079637050628662109375f;
  const float pio2_lo = -4.37113900018624283e-8f;
  const float pio4_hi = 0.785398185253143310546875f;
  const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f,
              p3 = 2.417951451e-2f, p4 = 4.216630880e-2f;
  int32_t hx = (int32_t)fbits(x);
  int32_t ix = hx & 0x7fffffff;
  float t, w, p, q, c, r, s;
  if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
  if (ix > 0x3f800000) return (x - x) / (x - x);
  if (ix < 0x3f000000) {
    if (ix < 0x32000000) {
      if (huge + x > one) return x;
    } else {
      t = x * x;
      w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
      return x + x * w;
    }
  }
  w = one - fabs_(x);
  t = w * 0.5f;
  p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
  s = sqrt_(t);
  if (ix >= 0x3F79999A) {
    t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
  } else {
    w = bitsf(fbits(s) & 0xfffff000u);
    c = (t - w * w) / (s + w);
    r = p;
    p = 2.0f * s * r - (pio2_lo - 2.0f * c);
    q = pio4_hi - 2.0f * w;
    t = pio4_hi - (p - q);
  }
  return hx > 0 ? t : -t;
}

// ---- acosf: glibc e_acosf.c (fdlibm rational R(z)=p/q) --------------------------------------
LLSR_HD float acosf_(float x) {
  const float one = 1.0f, pi = 3.1415925026e+00f, pio2_hi = 1.5707962513e+00f,
              pio2_lo = 7.5497894159e-08f;
  const float pS0 = 1.6666667163e-01f, pS1 = -3.2556581497e-01f, pS2 = 2.0121252537e-01f,
              pS3 = -4.0055535734e-02f, pS4 = 7.9153501429e-04f, pS5 = 3.4793309169e-05f,
              qS1 = -2.4033949375e+00f, qS2 = 2.0209457874e+00f, qS3 = -6.8828397989e-01f,
              qS4 = 7.7038154006e-02f;
  int32_t hx = (int32_t)fbits(x);
  int32_t ix = hx & 0x7fffffff;
  float z, p, q, r, w, s, c, df;
  if (ix == 0x3f800000) {
    if (hx > 0) return 0.0f;
    return pi + 2.0f * pio2_lo;
  } else if (ix > 0x3f800000) {
    return (x - x) / (x - x);
  }
  if (ix < 0x3f000000) {
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;
    z = x * x;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx < 0) {
    z = (one + x) * 0.5f;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    s = sqrt_(z);
    r = p / q;
    w = r * s - pio2_lo;
    return pi - 2.0f * (s + w);
  } else {
    z = (one - x) * 0.5f;
    s = sqrt_(z);
    df = bitsf(fbits(s) & 0xfffff000u);
    c = (z - df * df) / (s + df);
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    w = r * s + c;
    return 2.0f * (df + w);
  }
}

// ---- atanf: glibc s_atanf.c (fdlibm, 11-term odd/even split) --------------------------------
LLSR_HD float atanf_(float x) {
  const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f,
              atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
  const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f,
              atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
              aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
              aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
              aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  const float one = 1.0f, huge = 1.0e30f;
  int32_t hx = (int32_t)fbits(x);
  int32_t ix = hx & 0x7fffffff;
  if (ix >= 0x4c000000) {
    if (ix > 0x7f800000) return x + x;
    return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
  }
  if (ix < 0x31000000) {
    if (huge + x > one) return x;
  }
  // The four reductions of fdlibm as ONE quotient (a |x| + b) / (c |x| + d) with per-range
  // constants, so lanes of a wave in different ranges share one division instead of running up
  // to four divergent ones. Each is the same float operation sequence as its branch:
  //   id 0: (2|x| - 1) / (|x| + 2)     id 1: (|x| - 1) / (|x| + 1)
  //   id 2: (|x| - 1.5) / (1.5|x| + 1) id 3: (0|x| - 1) / (|x| + 0) = -1 / |x|
  // and id -1 keeps x: (1 x + 0) / (0 x + 1) = x exactly (x != 0 here).
  const int id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
  const float xin = id < 0 ? x : fabs_(x);
  const float ca = id == 0 ? 2.0f : id == 3 ? 0.0f : one;
  const float cb = id < 0 ? 0.0f : id == 2 ? -1.5f : -one;
  const float cc = id < 0 ? 0.0f : id == 2 ? 1.5f : one;
  const float cd = id < 0 ? one : id == 0 ? 2.0f : id == 3 ? 0.0f : one;
  x = (ca * xin + cb) / (cc * xin + cd);
  float z = x * x;
  float w = z * z;
  float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return hx < 0 ? -z : z;
}

// ---- atan2f: glibc e_atan2f.c -----------------------------------------------------------------
LLSR_HD float atan2f_(float y, float x) {
  const float tiny = 1.0e-30f, zero = 0.0f, pi_o_4 = 7.8539818525e-01f,
              pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
  int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
  int32_t hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return atanf_(y);
  int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    switch (m) {
      case 0: case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    } else {
      switch (m) {
        case 0: return zero;
        case 1: return -zero;
        case 2: return pi + tiny;
        default: return -pi - tiny;
      }
    }
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  int32_t k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0f;
  else z = atanf_(fabs_(y / x));
  switch (m) {
    case 0: return z;
    case 1: return bitsf(fbits(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

// ---- tanf: glibc s_tanf.c + k_tanf.c; argument reduction only for |x| < 3pi/4 ---------------
// (the hot path only evaluates tanf(atan2f(z, r_xy) +- res_Y) with |arg| <= pi/2 + res_Y).
LLSR_HD float kernel_tanf_(float x, float y, int iy) {
  const float one = 1.0f, pio4 = 7.8539812565e-01f, pio4lo = 3.7748947079e-08f;
  const float T0 = 3.3333334327e-01f, T1 = 1.3333334029e-01f, T2 = 5.3968254477e-02f,
              T3 = 2.1869488060e-02f, T4 = 8.8632395491e-03f, T5 = 3.5920790397e-03f,
              T6 = 1.4562094584e-03f, T7 = 5.8804126456e-04f, T8 = 2.4646313977e-04f,
              T9 = 7.8179444245e-05f, T10 = 7.1407252108e-05f, T11 = -1.8558637748e-05f,
              T12 = 2.5907305826e-05f;
  int32_t hx = (int32_t)fbits(x);
  int32_t ix = hx & 0x7fffffff;
  float z, r, v, w, s;
  if (ix < 0x39000000) {
    if ((int)x == 0) {
      if ((ix | (iy + 1)) == 0) return one / fabs_(x);
      else if (iy == 1) return x;
      else return -one / x;
    }
  }
  if (ix >= 0x3f2ca140) {
    if (hx < 0) { x = -x; y = -y; }
    z = pio4 - x;
    w = pio4lo - y;
    x = z + w; y = 0.0f;
    if (fabs_(x) < 0x1p-13f)
      return (float)((1 - ((hx >> 30) & 2)) * iy) * (1.0f - 2.0f * (float)iy * x);
  }
  z = x * x;
  w = z * z;
  r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
  v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
  s = z * x;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  w = x + r;
  if (ix >= 0x3f2ca140) {
    v = (float)iy;
    return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
  }
  if (iy == 1) return w;
  float a, t;
  z = bitsf(fbits(w) & 0xfffff000u);
  v = r - (z - x);
  t = a = -1.0f / w;
  t = bitsf(fbits(t) & 0xfffff000u);
  s = 1.0f + t * z;
  return t + a * (s + t * v);
}

LLSR_HD float tanf_(float x) {
  int32_t hx = (int32_t)fbits(x);
  int32_t ix = hx & 0x7fffffff;
  if (ix <= 0x3f490fda) return kernel_tanf_(x, 0.0f, 1);
  if (ix >= 0x7f800000) return x - x;
  // glibc's __ieee754_rem_pio2f reuses the sincosf "reduce_fast" step (double precision,
  // 2/pi prescaled by 2^24 so the quadrant lands in bits 24..31). It is exact for |x| <= 120;
  // beyond that (never reached: the hot path's arguments are bounded by pi/2 + res_Y) return
  // NaN so a misuse is loud, never silently inexact.
  if (ix < 0x42f00000) {
    double dx = (double)x;
    double r = dx * 0x1.45F306DC9C883p+23;
    int32_t n = ((int32_t)r + 0x800000) >> 24;
    dx = dx - (double)n * 0x1.921FB54442D18p0;
    float y0 = (float)dx;
    float y1 = (float)(dx - (double)y0);
    return kernel_tanf_(y0, y1, 1 - ((n & 1) << 1));
  }
  return bitsf(0x7fc00000u);
}


// ---- sinf / cosf: glibc >= 2.28 sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c (sincosf.h):
// double-precision polynomials after reduce_fast (|x| < 120). Larger |x| is outside the hot
// path's domain (angles of a 6-DoF pose) and returns NaN so a misuse is loud.
struct SinCosTab {
  double sign[4];
  double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
LLSR_HD const SinCosTab& sincos_tab(int k) {
  static const SinCosTab T[2] = {
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
       0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
       0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
      {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
       -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
       0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
  return T[k];
}
LLSR_HD uint32_t abstop12(float x) { return (fbits(x) >> 20) & 0x7ff; }
// x86-64 glibc dispatches sinf/cosf (and only those of the functions used here) through an
// ifunc to a copy of this code built with -mfma -mavx2 (sysdeps/x86_64/fpu/multiarch/s_sinf.c),
// so every multiply feeding an add is one fused op there; restated with explicit fma so host
// and device agree with what the reference gets on any FMA-capable x86 (libm_check pins it).
LLSR_HD float sinf_poly(double x, double x2, const SinCosTab& p, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = __builtin_fma(x2, p.s3, p.s2);
    const double x7 = x3 * x2;
    const double s = __builtin_fma(x3, p.s1, x);
    return (float)__builtin_fma(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = __builtin_fma(x2, p.c4, p.c3);
  const double c1 = __builtin_fma(x2, p.c1, p.c0);
  const double x6 = x4 * x2;
  const double c = __builtin_fma(x4, p.c2, c1);
  return (float)__builtin_fma(x6, c2, c);
}
LLSR_HD double reduce_fast_(double x, const SinCosTab& p, int* np) {
  const double r = x * p.hpi_inv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return __builtin_fma(-(double)n, p.hpi, x);
}
LLSR_HD float sinf_(float y) {
  double x = y;
  int n;
  const SinCosTab* p = &sincos_tab(0);
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
    const double s = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return y;
    return sinf_poly(x, s, *p, 0);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast_(x, *p, &n);
    const double s = p->sign[n & 3];
    if (n & 2) p = &sincos_tab(1);
    return sinf_poly(x * s, x * x, *p, n);
  } else if (abstop12(y) < abstop12(__builtin_inff())) {
    return bitsf(0x7fc00000u);
  }
  return (y - y) / (y - y);
}
LLSR_HD float cosf_(float y) {
  double x = y;
  int n;
  const SinCosTab* p = &sincos_tab(0);
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
    const double x2 = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return sinf_poly(x, x2, *p, 1);
  } else if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast_(x, *p, &n);
    const double s = p->sign[n & 3];
    if (n & 2) p = &sincos_tab(1);
    return sinf_poly(x * s, x * x, *p, n ^ 1);
  } else if (abstop12(y) < abstop12(__builtin_inff())) {
    return bitsf(0x7fc00000u);
  }
  return (y - y) / (y - y);
}

// ---- groundRemovalOurs' angle test (imageProjection.cpp:555-566) as one comparison ----------
// The reference keeps a cell as ground iff (float)(acosf(x) / (pi/180)) <= D, x = TV.RV/(|TV||RV|).
// That predicate is monotone in x (acosf_ non-increasing on [-1, 1], NaN for |x| > 1 or NaN x),
// so it equals  xs <= x <= 1  with xs = the smallest float it accepts; ground_cos_threshold finds
// xs by bisection over the ordered float bits. oracle/libm_check ("gnd" rows) verifies the
// equivalence over all 2^32 x for every D the reference uses (12.5, 25, 60 degrees).
LLSR_HD float ground_angle_deg(float x) {
  return (float)((double)acosf_(x) / (3.14159265358979323846 / 180.0));
}
LLSR_HD bool ground_angle_ok(float x, float D) { return ground_angle_deg(x) <= D; }
LLSR_HD float ground_cos_threshold(float D) {
  auto key2f = [](int32_t k) { return bitsf(k < 0 ? (0x80000000u | (uint32_t)(-k)) : (uint32_t)k); };
  int32_t lo = -(int32_t)0x3f800000, hi = 0x3f800000;  // keys of -1 (rejected) and 1 (accepted)
  while (hi - lo > 1) {
    const int32_t mid = lo + (hi - lo) / 2;
    if (ground_angle_ok(key2f(mid), D)) hi = mid;
    else lo = mid;
  }
  return key2f(hi);
}

}  // namespace llsr_libm
