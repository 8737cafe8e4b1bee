/*
 * trig.h — the transcendental functions of the pose arithmetic: sin, tan
 * and acos in FP64, written with +, -, *, /, sqrt and floor only.
 *
 * GTSAM 4.2.0's Rot3/Pose3 Expmap and Logmap (SO3.cpp ExpmapFunctor and
 * Logmap, Pose3.cpp Expmap and Logmap) call std::sin,
 * std::acos and std::tan. The device and glibc implementations of those
 * differ in the last bit for some arguments, and the Between/Prior rows
 * amplify such a bit: 1 - theta / (2 tan(theta/2)) cancels for small
 * rotations and acos is ill-conditioned near 1. This header is the single
 * implementation that both sides use instead — the kernels (se3.hpp) and
 * the CPU oracle (oracle/oracle.c) — so that the two evaluate the same
 * IEEE operations in the same order and round identically. The basic
 * operations are correctly rounded on both sides (gfx950 FP64 division and
 * square root as HIP lowers them without fast-math; SSE2 on the host), and
 * the header must be compiled without FMA contraction: se3.hpp includes it
 * under `#pragma clang fp contract(off)`, the oracle is plain gcc -std=c99
 * on x86-64 (no contraction).
 *
 * Accuracy against mpmath (tests/test_trig.py): sin within 1 ulp, tan
 * within 2 ulp, acos within 1 ulp on their whole domain of use (|x| below
 * 2^19 pi/2 for sin and tan).
 *
 * Method. sin/tan: x = n pi/2 + r with |r| <= pi/4 by a three-part
 * Cody-Waite reduction (pi/2 split in 33 + 33 + 53 bits, so n * part is
 * exact for |n| < 2^20), then Taylor polynomials of sin and cos in r^2 up
 * to r^17 and r^18 (truncation below 1e-19 relative at pi/4); cos keeps
 * the rounding of 1 - r^2/2 (the fdlibm kernel form). acos: |x| <= 1/2 by
 * pi/2 - asin(x), otherwise by 2 asin(sqrt((1 - |x|)/2)), the square root
 * split in a 32-bit head and a correction; asin(s) = s + s z P(z), z = s^2
 * <= 1/4, P the Taylor series of asin to z^26 (truncation below 1e-18).
 * Coefficients are the nearest doubles of the exact series terms (checked
 * by tests/test_trig.py).
 */
#ifndef DYNOHIP_TRIG_H
#define DYNOHIP_TRIG_H

#include <math.h>
#include <string.h>

#if defined(__HIPCC__)
#define DHT_FN static __host__ __device__ inline
#else
#define DHT_FN static inline
#endif

/* pi/2 in three parts: 33 bits, 33 bits, 53 bits */
#define DHT_PIO2_1 0x1.921fb54400000p+0
#define DHT_PIO2_2 0x1.0b4611a600000p-34
#define DHT_PIO2_3 0x1.3198a2e037073p-69
#define DHT_INV_PIO2 0x1.45f306dc9c883p-1
/* pi/2 = HI + LO, pi = 2 HI + 2 LO */
#define DHT_PIO2_HI 0x1.921fb54442d18p+0
#define DHT_PIO2_LO 0x1.1a62633145c07p-54
#define DHT_PI_HI 0x1.921fb54442d18p+1

/* sin r = r + r z (S1 + z S2 + ... + z^7 S8), S_k = (-1)^k / (2k+1)! */
#define DHT_S1 -0x1.5555555555555p-3
#define DHT_S2 0x1.1111111111111p-7
#define DHT_S3 -0x1.a01a01a01a01ap-13
#define DHT_S4 0x1.71de3a556c734p-19
#define DHT_S5 -0x1.ae64567f544e4p-26
#define DHT_S6 0x1.6124613a86d09p-33
#define DHT_S7 -0x1.ae7f3e733b81fp-41
#define DHT_S8 0x1.952c77030ad4ap-49
/* cos r = 1 - z/2 + z^2 (C1 + z C2 + ... + z^7 C8), C_k = (-1)^(k+1) / (2k+2)! */
#define DHT_C1 0x1.5555555555555p-5
#define DHT_C2 -0x1.6c16c16c16c17p-10
#define DHT_C3 0x1.a01a01a01a01ap-16
#define DHT_C4 -0x1.27e4fb7789f5cp-22
#define DHT_C5 0x1.1eed8eff8d898p-29
#define DHT_C6 -0x1.93974a8c07c9dp-37
#define DHT_C7 0x1.ae7f3e733b81fp-45
#define DHT_C8 -0x1.6827863b97d97p-53

/* the reduction: x - n pi/2 = r + rr (|rr| <= ulp(r)/2), returns n mod 4
   (x finite). x - n P1 and n P2 are exact; the rounding of their
   difference is recovered exactly (|x - n P1| >= |n P2|) and carried in rr
   with the third part. */
DHT_FN int dht_reduce(double x, double* r, double* rr) {
  const double fn = floor(x * DHT_INV_PIO2 + 0.5);
  const double a = x - fn * DHT_PIO2_1;
  const double b = fn * DHT_PIO2_2;
  const double r1 = a - b;
  const double t = ((a - r1) - b) - fn * DHT_PIO2_3;
  const double y0 = r1 + t;
  *r = y0;
  *rr = (r1 - y0) + t;
  const double q = fn - 4.0 * floor(fn * 0.25);
  return (int)q;
}

/* sin(r + rr) and cos(r + rr) on |r| <= pi/4, rr the tail of the reduced
   argument: sin(r + rr) = sin r + rr cos r ~ r + r z P + rr (1 - z/2),
   cos(r + rr) = cos r - rr sin r ~ cos r - r rr */
DHT_FN double dht_ksin(double r, double rr) {
  const double z = r * r;
  const double v = z * r;
  const double p = DHT_S2 + z * (DHT_S3 + z * (DHT_S4 + z * (DHT_S5 + z * (DHT_S6 + z * (DHT_S7 + z * DHT_S8)))));
  return r - ((z * (0.5 * rr - v * p) - rr) - v * DHT_S1);
}

DHT_FN double dht_kcos(double r, double rr) {
  const double z = r * r;
  const double p =
      DHT_C1 + z * (DHT_C2 + z * (DHT_C3 + z * (DHT_C4 + z * (DHT_C5 + z * (DHT_C6 + z * (DHT_C7 + z * DHT_C8))))));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + ((z * z) * p - r * rr));
}

DHT_FN double dht_sin(double x) {
  if (x - x != 0.0) return x - x; /* NaN for NaN and +-inf */
  double r, rr;
  const int n = dht_reduce(x, &r, &rr);
  switch (n) {
    case 0: return dht_ksin(r, rr);
    case 1: return dht_kcos(r, rr);
    case 2: return -dht_ksin(r, rr);
    default: return -dht_kcos(r, rr);
  }
}

DHT_FN double dht_tan(double x) {
  if (x - x != 0.0) return x - x;
  double r, rr;
  const int n = dht_reduce(x, &r, &rr);
  const double s = dht_ksin(r, rr), c = dht_kcos(r, rr);
  return (n & 1) ? -c / s : s / c;
}

/* asin(s) = s + s z P(z), P(z) = sum_{n>=1} A_n z^(n-1),
   A_n = (2n)! / (4^n (n!)^2 (2n+1)) */
DHT_FN double dht_asin_p(double z) {
  double p = 0x1.1052bc5fa960ap-9;
  p = 0x1.208d3570ae5a6p-9 + z * p;
  p = 0x1.3275586c5f2f0p-9 + z * p;
  p = 0x1.464c0950f7d47p-9 + z * p;
  p = 0x1.5c5f56efaaaabp-9 + z * p;
  p = 0x1.750de64d7d05fp-9 + z * p;
  p = 0x1.90cb77f60c7cep-9 + z * p;
  p = 0x1.b026f57b13b14p-9 + z * p;
  p = 0x1.d3d2a8e0dd67dp-9 + z * p;
  p = 0x1.fcaf8fb6db6dbp-9 + z * p;
  p = 0x1.15ee9d45d1746p-8 + z * p;
  p = 0x1.31683bdef7bdfp-8 + z * p;
  p = 0x1.51ba308d3dcb1p-8 + z * p;
  p = 0x1.782dda12f684cp-8 + z * p;
  p = 0x1.a6863d70a3d71p-8 + z * p;
  p = 0x1.df3bd37a6f4dfp-8 + z * p;
  p = 0x1.12ef3cf3cf3cfp-7 + z * p;
  p = 0x1.3fde50d79435ep-7 + z * p;
  p = 0x1.7a87878787878p-7 + z * p;
  p = 0x1.c99999999999ap-7 + z * p;
  p = 0x1.1c4ec4ec4ec4fp-6 + z * p;
  p = 0x1.6e8ba2e8ba2e9p-6 + z * p;
  p = 0x1.f1c71c71c71c7p-6 + z * p;
  p = 0x1.6db6db6db6db7p-5 + z * p;
  p = 0x1.3333333333333p-4 + z * p;
  p = 0x1.5555555555555p-3 + z * p;
  return z * p;
}

DHT_FN double dht_acos(double x) {
  const double ax = fabs(x);
  if (!(ax <= 1.0)) return (x - x) / (x - x); /* NaN outside [-1, 1] */
  if (ax <= 0.5) {
    const double q = dht_asin_p(x * x); /* asin(x) = x + x q */
    return DHT_PIO2_HI - (x - (DHT_PIO2_LO - x * q));
  }
  const double z = (1.0 - ax) * 0.5; /* exact */
  const double s = sqrt(z);
  const double q = dht_asin_p(z);
  if (x < 0.0) return DHT_PI_HI - 2.0 * (s + (s * q - DHT_PIO2_LO));
  if (z == 0.0) return 0.0; /* x = 1 */
  /* s = df + c exactly to ~2^-100: df the high 32 bits of s */
  double df = s;
  unsigned long long bits;
  memcpy(&bits, &df, sizeof(bits));
  bits &= 0xffffffff00000000ULL;
  memcpy(&df, &bits, sizeof(bits));
  const double c = (z - df * df) / (s + df);
  return 2.0 * (df + (c + s * q));
}

#endif /* DYNOHIP_TRIG_H */
