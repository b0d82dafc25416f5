// rtp_device.hpp -- CDNA4 device math for the path-tracing hot path.
//
// Bit-exactness contract: every function reproduces the IEEE float/double
// operation sequence of the reference's CPU (g++, x86-64 SSE2) build.  The
// translation unit is compiled with -ffp-contract=off and HIP's default
// correctly-rounded f32 division/sqrt (checked in the .s: v_div_fixup_f32,
// v_sqrt_f32 + fma correction), and with denormals preserved.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rtp_layout.hpp"

#define RTP_DEV __device__ __forceinline__

namespace rtp {

constexpr double kPi = 3.14159265358979323846264338327950288;  // vtkm::Pi()
constexpr float kEps = 1e-5f;                                  // vtkm::Epsilon<float>()

struct f3 {
  float x, y, z;
};
RTP_DEV f3 mk(float x, float y, float z) { return f3{x, y, z}; }
RTP_DEV f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
RTP_DEV f3 ld3(const __attribute__((address_space(4))) float* p) { return f3{p[0], p[1], p[2]}; }  // kernarg / constant
RTP_DEV f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RTP_DEV f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RTP_DEV f3 scl(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
RTP_DEV f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
// vtkm::Dot: (a0*b0 + a1*b1) + a2*b2
RTP_DEV float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vtkm::Cross without VTKM_FMA (default x86-64 build)
RTP_DEV f3 cross(f3 a, f3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
RTP_DEV f3 de_nan(f3 c) {                                 // PdfWorklet.h:38-44
  if (!(c.x == c.x)) c.x = 0;
  if (!(c.y == c.y)) c.y = 0;
  if (!(c.z == c.z)) c.z = 0;
  return c;
}

// ------------------------------------------------- fast exact arithmetic ---
// Candidate short sequences for RN(1/x) and RN(sqrt(x)) without the scaling
// and special-case steps of the general IEEE lowering.  They are used only
// where rtp_verify_fast_math (exhaustive, every float of the stated range, on
// the device) shows them bit-identical to the IEEE operation.
RTP_DEV float rcp_nr1(float x) {  // v_rcp_f32 + one Newton step (fused)
  float r = __builtin_amdgcn_rcpf(x);
  float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}
RTP_DEV float rcp_nr2(float x) {  // + Markstein remainder correction
  float r = __builtin_amdgcn_rcpf(x);
  float e = __builtin_fmaf(-x, r, 1.0f);
  r = __builtin_fmaf(e, r, r);
  float q = r;
  float rem = __builtin_fmaf(-x, q, 1.0f);
  return __builtin_fmaf(rem, r, q);
}
RTP_DEV float sqrt_fast(float x) {  // v_sqrt_f32 + residual-based rounding fix (normal x)
  float s = __builtin_amdgcn_sqrtf(x);
  float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
  float rd = __builtin_fmaf(-sd, s, x), ru = __builtin_fmaf(-su, s, x);
  s = (rd <= 0.0f) ? sd : s;
  s = (ru > 0.0f) ? su : s;
  return s;
}

// RN(a / b) from r = RN(1 / b): q = RN(a r) is within one ulp of a / b, the
// remainder a - b q is exact with an FMA, and one FMA correction rounds to
// the correctly rounded quotient (Markstein's theorem; Muller et al.,
// Handbook of Floating-Point Arithmetic, 2nd ed., Thm 5.8), provided nothing
// over- or underflows.  Callers document why their operands stay in range;
// rtp_verify_fast_math kind 8 checks it exhaustively over divisors.
RTP_DEV float div_markstein(float a, float b, float r) {
  const float q = a * r;
  const float rem = __builtin_fmaf(-b, q, a);
  return __builtin_fmaf(rem, r, q);
}

// ------------------------------------------------------ exact wrappers ---
// rcp_nr1(x) == 1.0f/x and sqrt_fast(x) == sqrtf(x) bit for bit for every
// float with |x| in [2^-40, 2^40] (exhaustive device check, tools/
// verify_fast_math.py and tests/test_gpu_fast_math.py); outside that range
// (zero, denormal-scale, huge, Inf, NaN) the IEEE operation is used.
RTP_DEV bool fast_range(float x) { return fabsf(x) >= 0x1p-40f && fabsf(x) <= 0x1p40f; }
// The IEEE fallback sits behind a wave-uniform branch (ballot) holding an
// empty volatile asm, so the compiler cannot speculate it into the common
// path (it otherwise computes both and selects).
RTP_DEV float rcp_exact(float x) {  // 1.0f / x
  float r = rcp_nr1(x);
  const bool slow = !fast_range(x);
  if (__ballot(slow)) {
    asm volatile("");
    if (slow) r = 1.0f / x;
  }
  return r;
}
RTP_DEV float sqrt_exact(float x) {  // sqrtf(x)
  float s = sqrt_fast(x);
  const bool slow = !fast_range(x) || x < 0.0f;
  if (__ballot(slow)) {
    asm volatile("");
    if (slow) s = __builtin_sqrtf(x);
  }
  return s;
}
RTP_DEV float rsqrt_exact(float x) {  // 1 / sqrtf(x)  (vtkm::RMagnitude, CPU build)
  float r = rcp_nr1(sqrt_fast(x));
  const bool slow = !fast_range(x) || x < 0.0f;
  if (__ballot(slow)) {
    asm volatile("");
    if (slow) r = 1.0f / __builtin_sqrtf(x);
  }
  return r;
}
// 1/det of the quad tests.  The reciprocal is only used when !(|det| < kEps)
// (kEps = 1e-5 > 2^-40), so the small end of fast_range never matters: only
// |det| > 2^40 (or NaN) takes the IEEE path.
#ifndef RTP_DET_FALLBACK
#define RTP_DET_FALLBACK 1  // (0: timing experiments only -- not exact for |det| > 2^40)
#endif
RTP_DEV float rcp_det(float x) {
  float r = rcp_nr1(x);
  if (RTP_DET_FALLBACK) {
    const bool slow = !(fabsf(x) <= 0x1p40f);
    if (__ballot(slow)) {
      asm volatile("");
      if (slow) r = 1.0f / x;
    }
  }
  return r;
}
// vtkm::RMagnitude on the CPU build: 1 / sqrt(x.x)
RTP_DEV float rmag(f3 a) { return rsqrt_exact(dot(a, a)); }
RTP_DEV float magn(f3 a) { return sqrt_exact(dot(a, a)); }
RTP_DEV f3 unit_vector(f3 a) { return scl(a, rmag(a)); }  // vec3.h:38-42

// ------------------------------------------------------------------ RNG ---
// wangXor.h:30-38; the draw replaces the state (wangXor.h:55-59)
RTP_DEV uint32_t wang(uint32_t s) {
  s = (s ^ 61u) ^ (s >> 16);
  s *= 9u;
  s = s ^ (s >> 4);
  s *= 0x27d4eb2du;
  s = s ^ (s >> 15);
  return s;
}
// float(t) / 4294967295.f: the divisor rounds to 2^32, so the quotient is the
// exact scaling float(t) * 2^-32.
RTP_DEV float randf(uint32_t& s) {
  s = wang(s);
  return (float)s * 0x1p-32f;
}

// glibc 2.35 flt-32 sinf/cosf restated (see oracle/rtp_oracle.c; pinned
// bit-exact against libm for all floats in [0, 2pi]).  |x| < 120 path only.
struct SinCosT {
  double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};
__constant__ static const SinCosT kSC[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};

RTP_DEV uint32_t top12(float x) { return (__float_as_uint(x) >> 20) & 0x7ffu; }

// Evaluates the odd (sin) or even (cos) polynomial; the coefficients of table
// entry t are selected arithmetically (no divergent pointer).
RTP_DEV float sincos_poly(double x, double x2, int t, int n) {
  const SinCosT& p = kSC[t];
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = p.s2 + x2 * p.s3;
    double x7 = x3 * x2;
    double s = x + x3 * p.s1;
    return (float)(s + x7 * s1);
  } else {
    double x4 = x2 * x2;
    double c2 = p.c3 + x2 * p.c4;
    double c1 = p.c0 + x2 * p.c1;
    double x6 = x4 * x2;
    double c = c1 + x4 * p.c2;
    return (float)(c + x6 * c2);
  }
}
// is_cos = 0: sinf, 1: cosf
RTP_DEV float glibc_sincosf(float y, int is_cos) {
  double x = y;
  if (top12(y) < top12(0x1.921FB6p-1f)) {
    if (top12(y) < top12(0x1p-12f)) return is_cos ? 1.0f : y;
    return sincos_poly(x, x * x, 0, is_cos);
  }
  double r = x * kSC[0].hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  x = x - n * kSC[0].hpi;
  double s = kSC[0].sign[n & 3];
  return sincos_poly(x * s, x * x, (n & 2) ? 1 : 0, n ^ is_cos);
}
RTP_DEV float rtp_sinf(float y) { return glibc_sincosf(y, 0); }
RTP_DEV float rtp_cosf(float y) { return glibc_sincosf(y, 1); }

// sinf and cosf of the same argument, branch-free, each bit-identical to the
// functions above (|y| < 120).  For |y| < pi/4 glibc's small-argument path is
// the general path with n = 0 (x - 0*hpi == x, sign[0] == 1, table 0), so one
// reduction serves every lane; both polynomials are evaluated and n's parity
// says which is the sine.  Table 1 differs from table 0 only by negated cosine
// coefficients, and negation commutes with round-to-nearest, so the even
// polynomial of table 1 is exactly the negated one of table 0.
RTP_DEV void rtp_sincosf(float y, float* sin_out, float* cos_out) {
  const SinCosT& p = kSC[0];
  const double x0 = y;
  const double r = x0 * p.hpi_inv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  const double x = x0 - n * p.hpi;
  const double xs = ((n + 1) & 2) ? -x : x;  // sign[n & 3] = {1,-1,-1,1}
  const double x2 = x * x;
  // odd polynomial on xs (sinf_poly, n even branch)
  const double x3 = xs * x2;
  const double s1 = p.s2 + x2 * p.s3;
  const double x7 = x3 * x2;
  const float odd = (float)((xs + x3 * p.s1) + x7 * s1);
  // even polynomial, table 0 (sinf_poly, n odd branch)
  const double x4 = x2 * x2;
  const double c2 = p.c3 + x2 * p.c4;
  const double c1 = p.c0 + x2 * p.c1;
  const double x6 = x4 * x2;
  float even = (float)((c1 + x4 * p.c2) + x6 * c2);
  even = (n & 2) ? -even : even;
  float sv = (n & 1) ? even : odd;
  float cv = (n & 1) ? odd : even;
  const bool tiny = top12(y) < top12(0x1p-12f);
  *sin_out = tiny ? y : sv;
  *cos_out = tiny ? 1.0f : cv;
}

// ------------------------------------------------------------------ onb ---
struct Onb {
  f3 u, v, w;
};
RTP_DEV Onb build_from_w(f3 n) {  // onb.h:34-45
  Onb o;
  o.w = unit_vector(n);
  f3 a = (fabsf(o.w.x) > 0.9) ? mk(0, 1, 0) : mk(1, 0, 0);
  o.v = unit_vector(cross(o.w, a));
  o.u = cross(o.w, o.v);
  return o;
}
RTP_DEV f3 local(const Onb& o, f3 a) {  // onb.h:27-28
  return add(add(scl(o.u, a.x), scl(o.v, a.y)), scl(o.w, a.z));
}

// -------------------------------------------------------- intersection ---
// Lagae-Dutre ray/quad (Surface.h:31-161) on precomputed edges; returns the
// ray parameter through t_out.  The bilinear (u,v) are never read downstream.
// Branch-free form: every rejection test of the reference is evaluated on the
// same values and the hit is their conjunction (the early returns only skip
// work, they never change a value that a later test reads).
//
// Zero structure.  The edge vectors of most quads have exactly-zero
// components (axis-aligned walls, faces of boxes rotated about y).  The
// reference still multiplies by them; those products are +-0, and in a
// left-to-right sum x + (+-0) == x, (+-0) - x == -x for x != 0.  Dropping
// them can only change the SIGN of a zero result, and every such value only
// reaches a comparison with 0 (== for both zeros), a sum with a nonzero term,
// or a product that again only reaches such comparisons (det == +-0 is
// rejected by |det| < eps before its reciprocal matters).  Inputs are finite
// (ray directions are de-NaN'd / bounded, origins are hit points), so 0*x is
// +-0.  Hence every nonzero intermediate is bit-identical to the full form.
// M* are the compile-time masks of the nonzero edge components
// (rtp_layout.hpp kQuadKind); two-term sums are order-free (commutative).
constexpr int cross_mask(int me) {  // nonzero components of cross(full, e)
  return (((me >> 1) | (me >> 2)) & 1) | ((((me >> 2) | me) & 1) << 1) | (((me | (me >> 1)) & 1) << 2);
}
template <int ME, int I>
RTP_DEV float cross_c(const float (&a)[3], const float* e) {  // component I of cross(a, e)
  constexpr int i1 = (I + 1) % 3, i2 = (I + 2) % 3;
  constexpr bool p = (ME >> i2) & 1, q = (ME >> i1) & 1;
  if constexpr (p && q) return a[i1] * e[i2] - a[i2] * e[i1];
  else if constexpr (p) return a[i1] * e[i2];
  else if constexpr (q) return -(a[i2] * e[i1]);
  else return 0.0f;
}
template <int M>
RTP_DEV float dot_m(const float* x, const float* y) {  // vtkm::Dot without the structural-zero terms
  constexpr bool b0 = M & 1, b1 = (M >> 1) & 1, b2 = (M >> 2) & 1;
  if constexpr (b0 && b1 && b2) return (x[0] * y[0] + x[1] * y[1]) + x[2] * y[2];
  else if constexpr (b0 && b1) return x[0] * y[0] + x[1] * y[1];
  else if constexpr (b0 && b2) return x[0] * y[0] + x[2] * y[2];
  else if constexpr (b1 && b2) return x[1] * y[1] + x[2] * y[2];
  else if constexpr (b0) return x[0] * y[0];
  else if constexpr (b1) return x[1] * y[1];
  else if constexpr (b2) return x[2] * y[2];
  else return 0.0f;
}

// Packed pairs (v_pk_mul_f32 / v_pk_add_f32 round each half like the scalar
// instruction), used to run a parallelogram's two triangles side by side.
typedef float f2v __attribute__((ext_vector_type(2)));
template <int ME, int I>
RTP_DEV f2v cross_c2(const f2v (&a)[3], const float* e) {  // component I of cross(a, e), e shared
  constexpr int i1 = (I + 1) % 3, i2 = (I + 2) % 3;
  constexpr bool p = (ME >> i2) & 1, q = (ME >> i1) & 1;
  if constexpr (p && q) return a[i1] * e[i2] - a[i2] * e[i1];
  else if constexpr (p) return a[i1] * e[i2];
  else if constexpr (q) return -(a[i2] * e[i1]);
  else return f2v{0.0f, 0.0f};
}
template <int M>
RTP_DEV f2v dot_m2(const f2v (&x)[3], const float* y) {  // dot_m with a shared right-hand side
  constexpr bool b0 = M & 1, b1 = (M >> 1) & 1, b2 = (M >> 2) & 1;
  if constexpr (b0 && b1 && b2) return (x[0] * y[0] + x[1] * y[1]) + x[2] * y[2];
  else if constexpr (b0 && b1) return x[0] * y[0] + x[1] * y[1];
  else if constexpr (b0 && b2) return x[0] * y[0] + x[2] * y[2];
  else if constexpr (b1 && b2) return x[1] * y[1] + x[2] * y[2];
  else if constexpr (b0) return x[0] * y[0];
  else if constexpr (b1) return x[1] * y[1];
  else if constexpr (b2) return x[2] * y[2];
  else return f2v{0.0f, 0.0f};
}
template <int M>
RTP_DEV f2v dot_m2l(const float* x, const f2v (&y)[3]) {  // dot_m with a shared left-hand side
  constexpr bool b0 = M & 1, b1 = (M >> 1) & 1, b2 = (M >> 2) & 1;
  if constexpr (b0 && b1 && b2) return (x[0] * y[0] + x[1] * y[1]) + x[2] * y[2];
  else if constexpr (b0 && b1) return x[0] * y[0] + x[1] * y[1];
  else if constexpr (b0 && b2) return x[0] * y[0] + x[2] * y[2];
  else if constexpr (b1 && b2) return x[1] * y[1] + x[2] * y[2];
  else if constexpr (b0) return x[0] * y[0];
  else if constexpr (b1) return x[1] * y[1];
  else if constexpr (b2) return x[2] * y[2];
  else return f2v{0.0f, 0.0f};
}

// G: the quad's scan head (a DevQuad, or a QuadGeom copy already in
// registers); M: the quad in memory, read only for the second triangle's
// edges of a quad that is not an exact parallelogram.
template <int K, class G = DevQuad>
RTP_DEV bool quad_hit_masked(const G& Q, const DevQuad& M, f3 o, f3 d, float& t_out) {
  constexpr int M01 = kQuadKind[K].m01, M03 = kQuadKind[K].m03, M21 = kQuadKind[K].m21, M23 = kQuadKind[K].m23;
  constexpr int MP = cross_mask(M03), MQ = cross_mask(M01), MPp = cross_mask(M21), MQp = cross_mask(M23);
  const float dv[3] = {d.x, d.y, d.z};
  const float P[3] = {cross_c<M03, 0>(dv, Q.e03), cross_c<M03, 1>(dv, Q.e03), cross_c<M03, 2>(dv, Q.e03)};
  const float det = dot_m<M01 & MP>(Q.e01, P);
  const float inv_det = rcp_det(det);
  // (a parallelogram has e21 == -e03 and e23 == -e01, so only kinds whose
  // masks pair up can hold one)
  if constexpr (M21 == M03 && M23 == M01) if (Q.para) {
    // exact parallelogram (e21 == -e03, e23 == -e01 bit for bit): Pp == -P,
    // detp == det, Qp == -cross(Tp, e01), so the second triangle is the first
    // one's arithmetic on Tp = o - v11 with both results negated (negation
    // commutes with rounding).  Half .x is the (v00) triangle, .y the (v11)
    // one; both always evaluated, branch-free.
    const float ov[3] = {o.x, o.y, o.z};
    const f2v T2[3] = {f2v{ov[0], ov[0]} - f2v{Q.vv[0][0], Q.vv[0][1]},
                       f2v{ov[1], ov[1]} - f2v{Q.vv[1][0], Q.vv[1][1]},
                       f2v{ov[2], ov[2]} - f2v{Q.vv[2][0], Q.vv[2][1]}};
    const f2v al2 = dot_m2<MP>(T2, P) * inv_det;  // (alpha, -ap)
    const f2v Q2[3] = {cross_c2<M01, 0>(T2, Q.e01), cross_c2<M01, 1>(T2, Q.e01), cross_c2<M01, 2>(T2, Q.e01)};
    const f2v be2 = dot_m2l<MQ>(dv, Q2) * inv_det;  // (beta, -bp)
    const float Qv[3] = {Q2[0].x, Q2[1].x, Q2[2].x};
    const float t = dot_m<M03 & MQ>(Q.e03, Qv) * inv_det;
    const float alpha = al2.x, beta = be2.x;
    // ap < 0 <=> -al2.y < 0 <=> al2.y > 0 (NaN: false both ways; -(+-0) is
    // not < 0 and +-0 is not > 0), likewise bp; evaluated without short
    // circuits so no lane mask or max canonicalisation is generated;
    // !(a < 0) & !(b < 0) & !(c < 0) == !(minNum(a, b, c) < 0): minNum skips
    // NaN operands, whose terms are true (!(NaN < 0)); all three NaN gives
    // NaN, true as well; -0 is not < 0 either way (no signaling NaNs arise)
    const bool ok1 = !(fabsf(det) < kEps) & !(fminf(fminf(alpha, beta), t) < 0.0f);
    const bool second = (alpha + beta) > 1.0f;
    const bool bad2 = (al2.y > 0.0f) | (be2.y > 0.0f);
    t_out = t;
    return ok1 & !(second & bad2);
  }
  const float T[3] = {o.x - Q.vv[0][0], o.y - Q.vv[1][0], o.z - Q.vv[2][0]};
  const float alpha = dot_m<MP>(T, P) * inv_det;
  const float Qv[3] = {cross_c<M01, 0>(T, Q.e01), cross_c<M01, 1>(T, Q.e01), cross_c<M01, 2>(T, Q.e01)};
  const float beta = dot_m<MQ>(dv, Qv) * inv_det;
  const float t = dot_m<M03 & MQ>(Q.e03, Qv) * inv_det;
  bool ok = !(fabsf(det) < kEps) && !(alpha < 0.0f) && !(beta < 0.0f) && !(t < 0.0f);
  if (ok && (alpha + beta) > 1.0f) {
    const float Pp[3] = {cross_c<M21, 0>(dv, M.e21), cross_c<M21, 1>(dv, M.e21), cross_c<M21, 2>(dv, M.e21)};
    const float detp = dot_m<M23 & MPp>(M.e23, Pp);
    const float inv_detp = rcp_det(detp);
    const float Tp[3] = {o.x - Q.vv[0][1], o.y - Q.vv[1][1], o.z - Q.vv[2][1]};
    const float ap = dot_m<MPp>(Tp, Pp) * inv_detp;
    const float Qp[3] = {cross_c<M23, 0>(Tp, M.e23), cross_c<M23, 1>(Tp, M.e23), cross_c<M23, 2>(Tp, M.e23)};
    const float bp = dot_m<MQp>(dv, Qp) * inv_detp;
    ok = !(fabsf(detp) < kEps) && !(ap < 0.0f) && !(bp < 0.0f);
  }
  t_out = t;
  return ok;
}

// Q.kind is wave-uniform (every lane tests the same quad): scalar branch.
RTP_DEV bool quad_hit(const DevQuad& Q, f3 o, f3 d, float& t_out) {
  switch (Q.kind) {
    case 1: return quad_hit_masked<1>(Q, Q, o, d, t_out);
    case 2: return quad_hit_masked<2>(Q, Q, o, d, t_out);
    case 3: return quad_hit_masked<3>(Q, Q, o, d, t_out);
    case 4: return quad_hit_masked<4>(Q, Q, o, d, t_out);
    case 5: return quad_hit_masked<5>(Q, Q, o, d, t_out);
    case 6: return quad_hit_masked<6>(Q, Q, o, d, t_out);
    case 7: return quad_hit_masked<7>(Q, Q, o, d, t_out);
    case 8: return quad_hit_masked<8>(Q, Q, o, d, t_out);
    case 9: return quad_hit_masked<9>(Q, Q, o, d, t_out);
    case 10: return quad_hit_masked<10>(Q, Q, o, d, t_out);
    default: return quad_hit_masked<0>(Q, Q, o, d, t_out);
  }
}

// SphereLeafIntersector::hit (Surface.h:319-367): first acceptable root
RTP_DEV bool sphere_hit(f3 o, f3 d, float tmin, float tmax, f3 c, float rr, float& t_out) {
  f3 oc = sub(o, c);
  float a = dot(d, d);
  float b = dot(oc, d);
  float cc = dot(oc, oc) - rr;
  float disc = b * b - a * cc;
  if (disc > 0) {
    float sq = sqrt_exact(b * b - a * cc);
    float temp = (-b - sq) / a;
    if (temp < tmax && temp > tmin) {
      t_out = temp;
      return true;
    }
    temp = (-b + sq) / a;
    if (temp < tmax && temp > tmin) {
      t_out = temp;
      return true;
    }
  }
  return false;
}

// (float)(cosine / kPi) of cosine_pdf::value (ScatterWorklet.h:96-112) as a
// double product with the double reciprocal.  The two double results differ
// by at most one double ulp; tests/test_gpu_fast_math.py checks exhaustively
// (verify kind 5) that the float roundings agree for every float in [0, 2]
// (the argument is a dot of two unit vectors, used only when > 0).
RTP_DEV float cos_over_pi(float c) {
  constexpr double kInvPi = 1.0 / kPi;
  return (float)((double)c * kInvPi);
}

// ----------------------------------------------------------- sampling ---
RTP_DEV f3 random_cosine_direction(float r1, float r2) {  // PdfWorklet.h:47-53
  float z = sqrt_exact(1 - r2);
  float phi = (float)(2 * kPi * r1);
  float x = rtp_cosf(phi) * 2 * sqrt_exact(r2);
  float y = rtp_sinf(phi) * 2 * sqrt_exact(r2);
  return mk(x, y, z);
}
RTP_DEV f3 random_to_sphere(float rr, float dist2, float r1, float r2) {  // PdfWorklet.h:157-165
  float z = 1 + r2 * (sqrt_exact(1 - rr / dist2) - 1);
  float phi = (float)(2 * kPi * r1);
  float x = rtp_cosf(phi) * sqrt_exact(1 - z * z);
  float y = rtp_sinf(phi) * sqrt_exact(1 - z * z);
  return mk(x, y, z);
}

// QuadPDFWorklet::pdf_value (PdfWorklet.h:230-248).  The normal flip of
// intersect() is dropped: fabs(dot(v,-n)*k) == fabs(dot(v,n)*k) exactly.
RTP_DEV float quad_pdf_value(const DevLights& L, f3 o, f3 v, float rmag_v) {  // rmag_v == rmag(v)
  float t;
  if (quad_hit(L.quad, o, v, t) && t < 3.40282347e+38f && t > 0.001f) {
    float distance_squared = t * t * dot(v, v);
    float cosine = fabsf(dot(v, ld3(L.quad.n)) * rmag_v);
    return distance_squared / (cosine * L.area);
  }
  return 0;
}
// SpherePDFWorklet::pdf_value (PdfWorklet.h:333-346).  ctm >= 0: the
// caller already holds cos_theta_max = sqrt(1 - R^2/|c-o|^2) bit for bit (the
// light-sphere generator computes the same expression from the same hit
// point), so only lanes without it recompute.
RTP_DEV float sphere_pdf_value(const DevLights& L, f3 o, f3 v, float ctm = -1.0f) {
  float t;
  f3 c = ld3(L.sc);
  if (sphere_hit(o, v, 0.001f, 3.40282347e+38f, c, L.srr, t)) {
    float cos_theta_max = ctm;
    if (!(ctm >= 0.0f)) {
      f3 co = sub(c, o);
      cos_theta_max = sqrt_exact(1 - L.srr / dot(co, co));
    }
    float solid_angle = (float)(2 * kPi * (1 - cos_theta_max));
    return rcp_exact(solid_angle);  // 1 / solid_angle
  }
  return 0;
}

// DielectricWorklet (EmitWorklet.h:153-226)
// pow((double)(1 - cosine), 5.0) of schlick: x is a float value (24
// significant bits), so x^2 is exact in double and x^4 = h + l exactly (the
// error of a product is a double, recovered by an FMA); x^5 = (h + l) x =
// p + e + l x with p + e = h x exact.  The sum rounds once more: the result
// is the correctly rounded x^5 unless x^5 lies within ~2^-100 (relative) of a
// midpoint between doubles.  glibc's pow (the reference's; the oracle's) is
// correctly rounded but for such near-midpoint cases too, and the value
// reaches the image only through (float)(r0 + (1 - r0) x^5) and a comparison
// with a float draw.  Checked against this host's glibc pow for every float
// x with |x| in [2^-24, 2] (tests/cpp/pow5_check.cpp).  The ocml pow it
// replaces ran ~80 double operations in a call on 7 of 64 lanes in 94% of
// C2's bounce steps (r04c stats: 9% of the step).  Range: |1 - cosine| is 0
// or >= 2^-24 and <= 2.5, so nothing under- or overflows; NaN propagates.
RTP_DEV double pow5_exact(double x) {
  const double x2 = x * x;                      // exact
  const double h = x2 * x2;                     // x^4 rounded
  const double l = __builtin_fma(x2, x2, -h);   // ... and its exact error
  const double p = h * x;
  const double e = __builtin_fma(h, x, -p);     // h x = p + e exactly
  return p + (e + l * x);
}
// r0sq = ((1 - ref_idx) / (1 + ref_idx))^2 (precomputed on the host with the
// same float operations: DevScene::ior_r0sq)
RTP_DEV float schlick(float cosine, float r0sq) {
  return (float)(r0sq + (1 - r0sq) * pow5_exact((double)(1 - cosine)));
}
// ior_inv = (float)(1.0 / ref_idx) (DevScene::ior_inv)
RTP_DEV void dielectric_scatter(f3 dir, f3 n, float ref_idx, float r0sq, float ior_inv, float rnd, f3& sd) {
  f3 reflected = sub(dir, scl(n, 2 * dot(dir, n)));
  f3 refracted = mk(0, 0, 0);  // reference reads an uninitialised vec3 here when refraction fails and rnd==1
  f3 outward;
  float ni_over_nt, cosine;
  const float rm = rmag(dir);  // one 1/|dir| for the cosine and unit_vector(dir)
  if (dot(dir, n) > 0) {
    outward = neg(n);
    ni_over_nt = ref_idx;
    cosine = ref_idx * dot(dir, n) * rm;
  } else {
    outward = n;
    ni_over_nt = ior_inv;
    cosine = -dot(dir, n) * rm;
  }
  float reflect_prob;
  {  // refract (EmitWorklet.h:160-170)
    f3 uv = scl(dir, rm);
    float dt = dot(uv, outward);
    float discriminant = (float)(1.0 - ni_over_nt * ni_over_nt * (1 - dt * dt));
    if (discriminant > 0) {
      refracted = sub(scl(sub(uv, scl(outward, dt)), ni_over_nt), scl(outward, sqrt_exact(discriminant)));
      reflect_prob = schlick(cosine, r0sq);
    } else {
      reflect_prob = 1.0f;
    }
  }
  sd = ((double)rnd < (double)reflect_prob) ? reflected : refracted;
}

// One RNG step of a ray that is dead for this depth: the which draw
// (PdfWorklet.h:20) plus the generator's draws -- cosine 2, quad 3, sphere 2
// (PdfWorklet.h:71-72, 91-93, 210).  which(t) is monotone in the hash value,
// so it is decided by two integer thresholds computed on the host.
RTP_DEV uint32_t dead_step(uint32_t s, uint32_t t1, uint32_t t2) {
  uint32_t t = wang(s);
  uint32_t s2 = wang(wang(t));
  uint32_t s3 = wang(s2);
  return (t >= t1 && t < t2) ? s3 : s2;
}

}  // namespace rtp
