// glibc_powf.hpp -- glibc 2.35 powf, restated for the device (and the host
// test that pins it).
//
// Where it is used: vtkm::Pow(float, float) is std::pow -> powf in the
// reference's CPU build.  The -direct colour mode's Phong term calls
// pow(max(cosPhi, 0), 20) (VTK-m RayTracer SurfaceColor::Shade; the
// reference's own copies RayTracerNormals.cxx:121-122, RayTracerAlbedo.cxx:
// 121-122).  glibc's powf is NOT correctly rounded: a correctly rounded x^20
// (double repeated squaring) differs from it on 44 279 of the floats in [0, 1].
// So this file restates glibc's algorithm (sysdeps/ieee754/flt-32/e_powf.c,
// Szabolcs Nagy's design) with glibc's own tables.
//
// Build variant: x86-64 libm picks an FMA build of e_powf.c by ifunc on
// FMA-capable CPUs (sysdeps/x86_64/fpu/multiarch/e_powf.c).  That build
// contracts every a*b+c of log2_inline/exp2_inline into an fma.  It is what
// the host libm returns on this image: the restatement below, with those fmas,
// equals libm's powf on every float in [0, 1.01] for y = 20 (tests/
// test_direct.py, exhaustive, CPU); the non-FMA build would differ on one.
//
// Tables: __powf_log2_data and __exp2f_data, extracted from this image's
// libm.so.6 by tools/extract_glibc_powf.py (the test re-extracts and compares).
#pragma once
#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#define RTP_PF_FN __host__ __device__ inline
#else
#define RTP_PF_FN inline
#endif

namespace rtp_glibc {

constexpr uint64_t kPowfLog2Tab[32] = {
    0x3ff661ec79f8f3beull, 0xbfdefec65b963019ull, 0x3ff571ed4aaf883dull, 0xbfdb0b6832d4fca4ull,
    0x3ff49539f0f010b0ull, 0xbfd7418b0a1fb77bull, 0x3ff3c995b0b80385ull, 0xbfd39de91a6dcf7bull,
    0x3ff30d190c8864a5ull, 0xbfd01d9bf3f2b631ull, 0x3ff25e227b0b8ea0ull, 0xbfc97c1d1b3b7af0ull,
    0x3ff1bb4a4a1a343full, 0xbfc2f9e393af3c9full, 0x3ff12358f08ae5baull, 0xbfb960cbbf788d5cull,
    0x3ff0953f419900a7ull, 0xbfaa6f9db6475fceull, 0x3ff0000000000000ull, 0x0000000000000000ull,
    0x3fee608cfd9a47acull, 0x3fb338ca9f24f53dull, 0x3feca4b31f026aa0ull, 0x3fc476a9543891baull,
    0x3feb2036576afce6ull, 0x3fce840b4ac4e4d2ull, 0x3fe9c2d163a1aa2dull, 0x3fd40645f0c6651cull,
    0x3fe886e6037841edull, 0x3fd88e9c2c1b9ff8ull, 0x3fe767dcf5534862ull, 0x3fdce0a44eb17bccull};
constexpr uint64_t kPowfLog2Poly[5] = {
    0x3fd27616c9496e0bull, 0xbfd71969a075c67aull, 0x3fdec70a6ca7baddull, 0xbfe7154748bef6c8ull, 0x3ff71547652ab82bull};
constexpr uint64_t kExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
constexpr uint64_t kExp2fShiftScaled = 0x42e8000000000000ull;
constexpr uint64_t kExp2fPoly[3] = {
    0x3fac6af84b912394ull, 0x3fcebfce50fac4f3ull, 0x3fe62e42ff0c52d6ull};

RTP_PF_FN double u2d(uint64_t u) {
  double d;
  memcpy(&d, &u, 8);
  return d;
}
RTP_PF_FN uint64_t d2u(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}
RTP_PF_FN float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
RTP_PF_FN uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

// e_powf.c checkint: 0 not an integer, 1 odd integer, 2 even integer
RTP_PF_FN int checkint(uint32_t iy) {
  int e = iy >> 23 & 0xff;
  if (e < 0x7f) return 0;
  if (e > 0x7f + 23) return 2;
  if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
  if (iy & (1u << (0x7f + 23 - e))) return 1;
  return 2;
}
RTP_PF_FN int zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000 - 1; }

// log2_inline (POWF_LOG2_TABLE_BITS = 4, POWF_SCALE_BITS = 0), FMA build
RTP_PF_FN double log2_inline(uint32_t ix) {
  const uint32_t OFF = 0x3f330000;
  const uint32_t tmp = ix - OFF;
  const int i = (tmp >> (23 - 4)) % 16;
  const uint32_t top = tmp & 0xff800000;
  const uint32_t iz = ix - top;
  const int k = (int32_t)top >> 23;
  const double invc = u2d(kPowfLog2Tab[2 * i]), logc = u2d(kPowfLog2Tab[2 * i + 1]);
  const double z = (double)u2f(iz);
  const double r = __builtin_fma(z, invc, -1.0);
  const double y0 = logc + (double)k;
  const double r2 = r * r;
  double y = __builtin_fma(u2d(kPowfLog2Poly[0]), r, u2d(kPowfLog2Poly[1]));
  const double p = __builtin_fma(u2d(kPowfLog2Poly[2]), r, u2d(kPowfLog2Poly[3]));
  const double r4 = r2 * r2;
  double q = __builtin_fma(u2d(kPowfLog2Poly[4]), r, y0);
  q = __builtin_fma(p, r2, q);
  y = __builtin_fma(y, r4, q);
  return y;
}

// exp2_inline (EXP2F_TABLE_BITS = 5), FMA build
RTP_PF_FN float exp2_inline(double xd, uint32_t sign_bias) {
  const double shift = u2d(kExp2fShiftScaled);
  double kd = xd + shift;
  const uint64_t ki = d2u(kd);
  kd -= shift;
  const double r = xd - kd;
  uint64_t t = kExp2fTab[ki % 32];
  const uint64_t ski = ki + sign_bias;
  t += ski << (52 - 5);
  const double s = u2d(t);
  const double z = __builtin_fma(u2d(kExp2fPoly[0]), r, u2d(kExp2fPoly[1]));
  const double r2 = r * r;
  double y = __builtin_fma(u2d(kExp2fPoly[2]), r, 1.0);
  y = __builtin_fma(z, r2, y);
  y = y * s;
  return (float)y;
}

// __powf (e_powf.c) in round-to-nearest without errno: y must not be
// zero/inf/NaN (the caller's exponent is the constant 20).
RTP_PF_FN float powf(float x, float y) {
  uint32_t sign_bias = 0;
  uint32_t ix = f2u(x);
  const uint32_t iy = f2u(y);
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    // x is subnormal, zero, negative, inf or nan
    if (zeroinfnan(ix)) {
      float x2 = x * x;
      if ((ix & 0x80000000u) && checkint(iy) == 1) x2 = -x2;
      return (iy & 0x80000000u) ? 1.0f / x2 : x2;
    }
    if (ix & 0x80000000u) {  // finite negative x
      const int yint = checkint(iy);
      if (yint == 0) return (x - x) / (x - x);  // __math_invalidf: NaN
      if (yint == 1) sign_bias = 1u << (5 + 11);
      ix &= 0x7fffffff;
    }
    if (ix < 0x00800000u) {  // subnormal: normalize
      ix = f2u(u2f(ix) * 0x1p23f);
      ix &= 0x7fffffff;
      ix -= 23u << 23;
    }
  }
  const double logx = log2_inline(ix);
  const double ylogx = (double)y * logx;
  if (((d2u(ylogx) >> 47) & 0xffff) >= (d2u(126.0) >> 47)) {
    // |y*log(x)| >= 126
    if (ylogx > 0x1.fffffffd1d571p+6) return sign_bias ? -__builtin_huge_valf() : __builtin_huge_valf();
    if (ylogx <= -150.0) return sign_bias ? -0.0f : 0.0f;
  }
  return exp2_inline(ylogx, sign_bias);
}

}  // namespace rtp_glibc
