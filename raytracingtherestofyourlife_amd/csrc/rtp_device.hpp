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
RTP_DEV f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
RTP_DEV f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
RTP_DEV f3 scl(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
RTP_DEV f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
// vtkm::Dot: (a0*b0 + a1*b1) + a2*b2
RTP_DEV float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vtkm::Cross without VTKM_FMA (default x86-64 build)
RTP_DEV f3 cross(f3 a, f3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
// vtkm::RMagnitude on the CPU build: 1 / sqrt(x.x)
RTP_DEV float rmag(f3 a) { return 1.0f / __builtin_sqrtf(dot(a, a)); }
RTP_DEV float magn(f3 a) { return __builtin_sqrtf(dot(a, a)); }
RTP_DEV f3 unit_vector(f3 a) { return scl(a, rmag(a)); }  // vec3.h:38-42
RTP_DEV f3 de_nan(f3 c) {                                 // PdfWorklet.h:38-44
  if (!(c.x == c.x)) c.x = 0;
  if (!(c.y == c.y)) c.y = 0;
  if (!(c.z == c.z)) c.z = 0;
  return c;
}

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
RTP_DEV bool quad_hit(const DevQuad& Q, f3 o, f3 d, float& t_out) {
  const f3 e03 = ld3(Q.e03), e01 = ld3(Q.e01);
  f3 P = cross(d, e03);
  float det = dot(e01, P);
  if (fabsf(det) < kEps) return false;
  float inv_det = 1.0f / det;
  f3 T = sub(o, ld3(Q.v00));
  float alpha = dot(T, P) * inv_det;
  if (alpha < 0.0f) return false;
  f3 Qv = cross(T, e01);
  float beta = dot(d, Qv) * inv_det;
  if (beta < 0.0f) return false;
  if ((alpha + beta) > 1.0f) {
    const f3 e23 = ld3(Q.e23), e21 = ld3(Q.e21);
    f3 Pp = cross(d, e21);
    float detp = dot(e23, Pp);
    if (fabsf(detp) < kEps) return false;
    float inv_detp = 1.0f / detp;
    f3 Tp = sub(o, ld3(Q.v11));
    float ap = dot(Tp, Pp) * inv_detp;
    if (ap < 0.0f) return false;
    f3 Qp = cross(Tp, e23);
    float bp = dot(d, Qp) * inv_detp;
    if (bp < 0.0f) return false;
  }
  float t = dot(e03, Qv) * inv_det;
  if (t < 0.0f) return false;
  t_out = t;
  return true;
}

// SphereLeafIntersector::hit (Surface.h:319-367): first acceptable root
RTP_DEV bool sphere_hit(f3 o, f3 d, float tmin, float tmax, f3 c, float rr, float& t_out) {
  f3 oc = sub(o, c);
  float a = dot(d, d);
  float b = dot(oc, d);
  float cc = dot(oc, oc) - rr;
  float disc = b * b - a * cc;
  if (disc > 0) {
    float sq = __builtin_sqrtf(b * b - a * cc);
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

// ----------------------------------------------------------- sampling ---
RTP_DEV f3 random_cosine_direction(float r1, float r2) {  // PdfWorklet.h:47-53
  float z = __builtin_sqrtf(1 - r2);
  float phi = (float)(2 * kPi * r1);
  float x = rtp_cosf(phi) * 2 * __builtin_sqrtf(r2);
  float y = rtp_sinf(phi) * 2 * __builtin_sqrtf(r2);
  return mk(x, y, z);
}
RTP_DEV f3 random_to_sphere(float rr, float dist2, float r1, float r2) {  // PdfWorklet.h:157-165
  float z = 1 + r2 * (__builtin_sqrtf(1 - rr / dist2) - 1);
  float phi = (float)(2 * kPi * r1);
  float x = rtp_cosf(phi) * __builtin_sqrtf(1 - z * z);
  float y = rtp_sinf(phi) * __builtin_sqrtf(1 - z * z);
  return mk(x, y, z);
}

// QuadPDFWorklet::pdf_value (PdfWorklet.h:230-248).  The normal flip of
// intersect() is dropped: fabs(dot(v,-n)*k) == fabs(dot(v,n)*k) exactly.
RTP_DEV float quad_pdf_value(const DevLights& L, f3 o, f3 v) {
  float t;
  if (quad_hit(L.quad, o, v, t) && t < 3.40282347e+38f && t > 0.001f) {
    float distance_squared = t * t * dot(v, v);
    float cosine = fabsf(dot(v, ld3(L.quad.n)) * rmag(v));
    return distance_squared / (cosine * L.area);
  }
  return 0;
}
// SpherePDFWorklet::pdf_value (PdfWorklet.h:333-346)
RTP_DEV float sphere_pdf_value(const DevLights& L, f3 o, f3 v) {
  float t;
  f3 c = ld3(L.sc);
  if (sphere_hit(o, v, 0.001f, 3.40282347e+38f, c, L.srr, t)) {
    f3 co = sub(c, o);
    float cos_theta_max = __builtin_sqrtf(1 - L.srr / dot(co, co));
    float solid_angle = (float)(2 * kPi * (1 - cos_theta_max));
    return 1 / solid_angle;
  }
  return 0;
}

// DielectricWorklet (EmitWorklet.h:153-226)
RTP_DEV float schlick(float cosine, float ref_idx) {
  float r0 = (1 - ref_idx) / (1 + ref_idx);
  r0 = r0 * r0;
  return (float)(r0 + (1 - r0) * pow((double)(1 - cosine), 5.0));
}
RTP_DEV void dielectric_scatter(f3 dir, f3 n, float ref_idx, float rnd, f3& sd) {
  f3 reflected = sub(dir, scl(n, 2 * dot(dir, n)));
  f3 refracted = mk(0, 0, 0);  // reference reads an uninitialised vec3 here when refraction fails and rnd==1
  f3 outward;
  float ni_over_nt, cosine;
  if (dot(dir, n) > 0) {
    outward = neg(n);
    ni_over_nt = ref_idx;
    cosine = ref_idx * dot(dir, n) * rmag(dir);
  } else {
    outward = n;
    ni_over_nt = (float)(1.0 / ref_idx);
    cosine = -dot(dir, n) * rmag(dir);
  }
  float reflect_prob;
  {  // refract (EmitWorklet.h:160-170)
    f3 uv = unit_vector(dir);
    float dt = dot(uv, outward);
    float discriminant = (float)(1.0 - ni_over_nt * ni_over_nt * (1 - dt * dt));
    if (discriminant > 0) {
      refracted = sub(scl(sub(uv, scl(outward, dt)), ni_over_nt), scl(outward, __builtin_sqrtf(discriminant)));
      reflect_prob = schlick(cosine, ref_idx);
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
