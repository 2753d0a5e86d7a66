// ORACLE (test infrastructure only) -- restatement of glibc 2.35 single-precision
// sinf/cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h; the ARM
// optimized-routines algorithm), as dispatched by glibc's x86_64 IFUNC to the
// FMA variant (__sinf_fma / __cosf_fma, built with -mfma -mavx2 and GCC's default
// fp-contract=fast, so every `a + b*c` is one fused multiply-add).
//
// Why it exists: the reference computes the steered-BRIEF rotation with
// `a = (float)cos(angle), b = (float)sin(angle)` on float angles
// (orb_extractor.cc:105-106) -> glibc cosf/sinf.  Descriptor bits depend on
// the exact float values, so the GPU kernel and this oracle share the same
// algorithm.  tests/test_sincosf.py checks this restatement against the
// host libm for EVERY float in [0, 2*pi] (the range IC_Angle can produce).
//
// Only the |x| < 120 path is restated: angles fed by the extractor are in
// [0, 2*pi] (fastAtan2 degrees in [0, 360] times pi/180).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

namespace oracle {

struct SinCosTab {
  double sign[4];
  double hpi_inv;  // 2/pi * 2^24 (x86_64 has no TOINT_INTRINSICS)
  double hpi;      // pi/2
  double c0, c1, c2, c3, c4;
  double s1, s2, s3;
};

static const SinCosTab kSinCosTab[2] = {
    {{1.0, -1.0, -1.0, 1.0},
     0x1.45F306DC9C883p+23,
     0x1.921FB54442D18p0,
     0x1p0,
     -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5,
     -0x1.6c087e89a359dp-10,
     0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7,
     -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0},
     0x1.45F306DC9C883p+23,
     0x1.921FB54442D18p0,
     -0x1p0,
     0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5,
     0x1.6c087e89a359dp-10,
     -0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7,
     -0x1.994eb3774cf24p-13},
};

static inline uint32_t sc_abstop12(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  return (u >> 20) & 0x7ff;
}

// Odd n -> cosine polynomial, even n -> sine polynomial.
static inline float sc_poly(double x, double x2, const SinCosTab* p, int n) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = std::fma(x2, p->s3, p->s2);
    double x7 = x3 * x2;
    double s = std::fma(x3, p->s1, x);
    return (float)std::fma(x7, s1, s);
  }
  double x4 = x2 * x2;
  double c2 = std::fma(x2, p->c4, p->c3);
  double c1 = std::fma(x2, p->c1, p->c0);
  double x6 = x4 * x2;
  double c = std::fma(x4, p->c2, c1);
  return (float)std::fma(x6, c2, c);
}

// Range reduction x -> r in [-pi/4, pi/4], quadrant n (scaled-int rounding).
static inline double sc_reduce(double x, const SinCosTab* p, int* np) {
  double r = x * p->hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return std::fma(-(double)n, p->hpi, x);
}

static const float kPio4f = 0x1.921FB6p-1f;

static inline float glibc_sinf(float y) {
  double x = y;
  const SinCosTab* p = &kSinCosTab[0];
  if (sc_abstop12(y) < sc_abstop12(kPio4f)) {
    double s = x * x;
    if (sc_abstop12(y) < sc_abstop12(0x1p-12f)) return y;
    return sc_poly(x, s, p, 0);
  }
  int n;
  x = sc_reduce(x, p, &n);
  double s = p->sign[n & 3];
  if (n & 2) p = &kSinCosTab[1];
  return sc_poly(x * s, x * x, p, n);
}

static inline float glibc_cosf(float y) {
  double x = y;
  const SinCosTab* p = &kSinCosTab[0];
  if (sc_abstop12(y) < sc_abstop12(kPio4f)) {
    double x2 = x * x;
    if (sc_abstop12(y) < sc_abstop12(0x1p-12f)) return 1.0f;
    return sc_poly(x, x2, p, 1);
  }
  int n;
  x = sc_reduce(x, p, &n);
  double s = p->sign[n & 3];
  if (n & 2) p = &kSinCosTab[1];
  return sc_poly(x * s, x * x, p, n ^ 1);
}

}  // namespace oracle
