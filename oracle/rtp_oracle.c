/*
 * rtp_oracle.c -- CPU restatement of the reference's path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see rtp_oracle.h).  Compile with gcc -O2
 * -ffp-contract=off and no fast-math: x86-64 SSE2 float/double arithmetic,
 * which is what a default g++ build of the reference performs.
 *
 * Every function cites the reference file:line it follows.  VTK-m (not
 * vendored, not in this container) semantics used by those lines:
 *   Dot(a,b)        = (a0*b0 + a1*b1) + a2*b2              (left to right)
 *   Cross(a,b)      = (a1*b2-a2*b1, a2*b0-a0*b2, a0*b1-a1*b0) (no VTKM_FMA on
 *                     a default x86-64 build, so no difference-of-products)
 *   RMagnitude(x)   = 1 / sqrt(Dot(x,x))   (CPU build; CUDA would use rsqrtf)
 *   Normalize(x)    : x = x * RMagnitude(x);   Magnitude = sqrt(Dot(x,x))
 *   Epsilon<float>  = 1e-5f;  Pi() is double;  Pi_180f() = 0.01745329251994329577f
 *   TriangleNormal(a,b,c) = Cross(b-a, c-a)
 *   float overloads of sqrt/cos/sin/fabs (libstdc++ <math.h>); pow(float,int)
 *   promotes to double; g++ evaluates call arguments right to left.
 */
#include "rtp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#if defined(__FP_FAST_FMA) || defined(__FAST_MATH__)
#error "oracle must be built without FMA contraction / fast-math"
#endif

static const double PI_D = 3.14159265358979323846264338327950288; /* vtkm::Pi() */
static const float PI_180F = 0.01745329251994329577f;             /* vtkm::Pi_180f() */
static const float EPS_F = 1e-5f;                                 /* vtkm::Epsilon<float>() */

typedef struct {
  float x, y, z;
} v3;

static inline v3 mk(float x, float y, float z) {
  v3 r = {x, y, z};
  return r;
}
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 scl(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float rmag(v3 a) { return 1 / sqrtf(dot(a, a)); }
static inline float mag(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 unit_vector(v3 a) { return scl(a, rmag(a)); } /* vec3.h:38-42 */
static inline v3 de_nan(v3 c) {                                /* PdfWorklet.h:38-44 */
  if (!(c.x == c.x)) c.x = 0;
  if (!(c.y == c.y)) c.y = 0;
  if (!(c.z == c.z)) c.z = 0;
  return c;
}
static inline v3 ld(const float p[3]) { return mk(p[0], p[1], p[2]); }

/* ---------------------------------------------------------------- RNG --- */
/* wangXor.h:30-38 */
uint32_t rtpo_wang32(uint32_t seed) {
  seed = (seed ^ 61) ^ (seed >> 16);
  seed *= 9;
  seed = seed ^ (seed >> 4);
  seed *= 0x27d4eb2d;
  seed = seed ^ (seed >> 15);
  return seed;
}
/* wangXor.h:55-59 -- the state is replaced by the hash; 1.0f is reachable */
float rtpo_randf(uint32_t* seed) {
  uint32_t t = rtpo_wang32(*seed);
  *seed = t;
  return (float)t / 4294967295.f;
}
/* PdfWorklet.h:19-21 with type_size 3 (WhichGenerateDir.cxx:10) */
static inline int which_of(float r) {
  int w = (int)(r * 3 + 1);
  return 3 < w ? 3 : w;
}
int32_t rtpo_which(uint32_t hash_value) { return which_of((float)hash_value / 4294967295.f); }

/* ---------------------------------------------- glibc sinf / cosf ------ */
/* Restatement of glibc 2.35 sysdeps/ieee754/flt-32/{s_sinf.c,s_cosf.c,
 * sincosf.h,sincosf_data.c} (the float sin/cos the reference's g++ build
 * calls from PdfWorklet.h:50-51,162-163).  Verified bit-exact against this
 * host's libm for every float in [0, 2*pi] (tests/test_oracle_primitives.py),
 * both with and without FMA contraction.  Only the |x| < 120 path is needed:
 * arguments are float(2*pi*r), r in [0,1]. */
typedef struct {
  double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
} sincos_t;
static const sincos_t SC[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
static inline uint32_t top12(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  return (u >> 20) & 0x7ff;
}
static inline float sinf_poly(double x, double x2, const sincos_t* p, int n) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = p->s2 + x2 * p->s3;
    double x7 = x3 * x2;
    double s = x + x3 * p->s1;
    return (float)(s + x7 * s1);
  } else {
    double x4 = x2 * x2;
    double c2 = p->c3 + x2 * p->c4;
    double c1 = p->c0 + x2 * p->c1;
    double x6 = x4 * x2;
    double c = c1 + x4 * p->c2;
    return (float)(c + x6 * c2);
  }
}
static inline double reduce_fast(double x, const sincos_t* p, int* np) {
  double r = x * p->hpi_inv;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return x - n * p->hpi;
}
float rtpo_sinf(float y) {
  double x = y;
  const sincos_t* p = &SC[0];
  int n;
  if (top12(y) < top12(0x1.921FB6p-1f)) {
    if (top12(y) < top12(0x1p-12f)) return y;
    return sinf_poly(x, x * x, p, 0);
  }
  if (!(top12(y) < top12(120.0f))) return sinf(y); /* unreachable for this path */
  x = reduce_fast(x, p, &n);
  double s = p->sign[n & 3];
  if (n & 2) p = &SC[1];
  return sinf_poly(x * s, x * x, p, n);
}
float rtpo_cosf(float y) {
  double x = y;
  const sincos_t* p = &SC[0];
  int n;
  if (top12(y) < top12(0x1.921FB6p-1f)) {
    if (top12(y) < top12(0x1p-12f)) return 1.0f;
    return sinf_poly(x, x * x, p, 1);
  }
  if (!(top12(y) < top12(120.0f))) return cosf(y); /* unreachable for this path */
  x = reduce_fast(x, p, &n);
  double s = p->sign[n & 3];
  if (n & 2) p = &SC[1];
  return sinf_poly(x * s, x * x, p, n ^ 1);
}

/* ---------------------------------------------------------------- onb --- */
/* onb.h:30-45 */
typedef struct {
  v3 u, v, w;
} onb;
static inline onb build_from_w(v3 n) {
  onb o;
  o.w = unit_vector(n);
  v3 a = (fabsf(o.w.x) > 0.9) ? mk(0, 1, 0) : mk(1, 0, 0);
  o.v = unit_vector(cross(o.w, a));
  o.u = cross(o.w, o.v);
  return o;
}
static inline v3 local(const onb* o, v3 a) { /* onb.h:27-28: a0*u + a1*v + a2*w */
  return add(add(scl(o->u, a.x), scl(o->v, a.y)), scl(o->w, a.z));
}

/* ------------------------------------------------------- intersection --- */
/* QuadLeafIntersector::hit, Surface.h:31-161 (Lagae-Dutre).  The bilinear
 * (u,v) it also computes are never read downstream and are omitted. */
static int quad_hit(v3 o, v3 d, v3 v00, v3 v10, v3 v11, v3 v01, float* t_out) {
  v3 E03 = sub(v01, v00);
  v3 P = cross(d, E03);
  v3 E01 = sub(v10, v00);
  float det = dot(E01, P);
  if (fabsf(det) < EPS_F) return 0;
  float inv_det = 1.0f / det;
  v3 T = sub(o, v00);
  float alpha = dot(T, P) * inv_det;
  if (alpha < 0.0) return 0;
  v3 Q = cross(T, E01);
  float beta = dot(d, Q) * inv_det;
  if (beta < 0.0) return 0;
  if ((alpha + beta) > 1.0f) {
    v3 E23 = sub(v01, v11);
    v3 E21 = sub(v10, v11);
    v3 Pp = cross(d, E21);
    float detp = dot(E23, Pp);
    if (fabsf(detp) < EPS_F) return 0;
    float inv_detp = 1.0f / detp;
    v3 Tp = sub(o, v11);
    float ap = dot(Tp, Pp) * inv_detp;
    if (ap < 0.0f) return 0;
    v3 Qp = cross(Tp, E23);
    float bp = dot(d, Qp) * inv_detp;
    if (bp < 0.0f) return 0;
  }
  float t = dot(E03, Q) * inv_det;
  if (t < 0.0) return 0;
  *t_out = t;
  return 1;
}

typedef struct {
  float t;
  v3 n, p;
} hitrec;

/* QuadLeafIntersector::intersect, Surface.h:163-199 */
static int quad_intersect(v3 o, v3 d, float tmin, float tmax, v3 q, v3 r, v3 s, v3 t, hitrec* rec) {
  float T;
  int h = quad_hit(o, d, q, r, s, t, &T);
  h = h && (T < tmax) && (T > tmin);
  if (h) {
    v3 n = cross(sub(r, q), sub(s, q)); /* TriangleNormal(q,r,s) */
    n = scl(n, rmag(n));                /* Normalize */
    if (dot(n, d) > 0.f) n = neg(n);
    rec->t = T;
    rec->p = add(o, scl(d, T));
    rec->n = n;
  }
  return h;
}

/* SphereLeafIntersector::hit, Surface.h:319-367 (uv, Surface.h:312-317, unused) */
static int sphere_hit(v3 o, v3 d, float tmin, float tmax, v3 center, float radius, hitrec* rec) {
  v3 oc = sub(o, center);
  float a = dot(d, d);
  float b = dot(oc, d);
  float c = dot(oc, oc) - radius * radius;
  float discriminant = b * b - a * c;
  if (discriminant > 0) {
    float temp = (-b - sqrtf(b * b - a * c)) / a;
    if (temp < tmax && temp > tmin) {
      rec->t = temp;
      rec->p = add(o, scl(d, temp));
      rec->n = mk((rec->p.x - center.x) / radius, (rec->p.y - center.y) / radius, (rec->p.z - center.z) / radius);
      return 1;
    }
    temp = (-b + sqrtf(b * b - a * c)) / a;
    if (temp < tmax && temp > tmin) {
      rec->t = temp;
      rec->p = add(o, scl(d, temp));
      rec->n = mk((rec->p.x - center.x) / radius, (rec->p.y - center.y) / radius, (rec->p.z - center.z) / radius);
      return 1;
    }
  }
  return 0;
}

/* ------------------------------------------------------------- scene --- */
static inline float d555(double v) { return (float)(v / 555.0); } /* Vec<float,3> / 555.0 */

typedef struct {
  float m[4][4];
} mat4;

/* CornellBox::invert, CornellBox.cpp:10-35: mat = Translate(265,0,295) *
 * Transpose(Rotate(-15 deg, y)); pts[i] = mat * (p,1).  Transform3DRotate is
 * VTK-m's Rodrigues form in float; MatrixMultiply sums k = 0..3 in order. */
static void cb_invert(float pts[4][3]) {
  const float angle = -15;
  float ax = 0.f, ay = 1.f, az = 0.f;
  {
    v3 axis = mk(ax, ay, az);
    axis = scl(axis, rmag(axis)); /* vtkm::Normal */
    ax = axis.x;
    ay = axis.y;
    az = axis.z;
  }
  float rad = PI_180F * angle;
  float sA = sinf(rad), cA = cosf(rad);
  mat4 R;
  R.m[0][0] = ax * ax * (1 - cA) + cA;
  R.m[0][1] = ax * ay * (1 - cA) - az * sA;
  R.m[0][2] = ax * az * (1 - cA) + ay * sA;
  R.m[0][3] = 0;
  R.m[1][0] = ay * ax * (1 - cA) + az * sA;
  R.m[1][1] = ay * ay * (1 - cA) + cA;
  R.m[1][2] = ay * az * (1 - cA) - ax * sA;
  R.m[1][3] = 0;
  R.m[2][0] = az * ax * (1 - cA) - ay * sA;
  R.m[2][1] = az * ay * (1 - cA) + ax * sA;
  R.m[2][2] = az * az * (1 - cA) + cA;
  R.m[2][3] = 0;
  R.m[3][0] = 0;
  R.m[3][1] = 0;
  R.m[3][2] = 0;
  R.m[3][3] = 1;
  mat4 RT, T, M;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) RT.m[i][j] = R.m[j][i];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) T.m[i][j] = (i == j) ? 1.f : 0.f;
  T.m[0][3] = 265;
  T.m[1][3] = 0;
  T.m[2][3] = 295;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      float sum = T.m[i][0] * RT.m[0][j];
      for (int k = 1; k < 4; k++) sum = sum + T.m[i][k] * RT.m[k][j];
      M.m[i][j] = sum;
    }
  for (int p = 0; p < 4; p++) {
    float v[4] = {pts[p][0], pts[p][1], pts[p][2], 1.f};
    float o[3];
    for (int i = 0; i < 3; i++) o[i] = M.m[i][0] * v[0] + M.m[i][1] * v[1] + M.m[i][2] * v[2] + M.m[i][3] * v[3];
    pts[p][0] = o[0];
    pts[p][1] = o[1];
    pts[p][2] = o[2];
  }
}

static void cb_push_point(rtpo_scene* s, float x, float y, float z) {
  s->points[s->n_points][0] = x;
  s->points[s->n_points][1] = y;
  s->points[s->n_points][2] = z;
  s->n_points++;
}
/* one quad cell: points appended in order, QuadIds row [cellId, p0..p3] */
static void cb_quad(rtpo_scene* s, int* cell, const float pts[4][3], int divide, int midx, int tidx) {
  int base = s->n_points;
  for (int i = 0; i < 4; i++) {
    if (divide)
      cb_push_point(s, d555(pts[i][0]), d555(pts[i][1]), d555(pts[i][2]));
    else
      cb_push_point(s, pts[i][0], pts[i][1], pts[i][2]);
  }
  for (int i = 0; i < 4; i++) s->field[s->n_field++] = (float)*cell; /* buildQuad :56-59 */
  int q = s->n_quads++;
  s->quad_ids[q][0] = *cell;
  for (int i = 0; i < 4; i++) s->quad_ids[q][1 + i] = base + i;
  s->quad_mat[q] = midx;
  s->quad_tex[q] = tidx;
  (*cell)++;
}
static void set4(float p[4][3], float a0, float a1, float a2, float b0, float b1, float b2, float c0, float c1,
                 float c2, float d0, float d1, float d2) {
  p[0][0] = a0, p[0][1] = a1, p[0][2] = a2;
  p[1][0] = b0, p[1][1] = b1, p[1][2] = b2;
  p[2][0] = c0, p[2][1] = c1, p[2][2] = c2;
  p[3][0] = d0, p[3][1] = d1, p[3][2] = d2;
}
/* CornellBox::buildBox, CornellBox.cpp:63-139 (duplicated near/far faces,
 * no sides or bottom -- kept as is) */
static void cb_box(rtpo_scene* s, int* cell, v3 n, v3 f) {
  float p[4][3];
  set4(p, n.x, n.y, n.z, f.x, n.y, n.z, f.x, f.y, n.z, n.x, f.y, n.z);
  cb_quad(s, cell, p, 1, 1, 1);
  set4(p, n.x, n.y, f.z, f.x, n.y, f.z, f.x, f.y, f.z, n.x, f.y, f.z);
  cb_quad(s, cell, p, 1, 1, 1);
  set4(p, n.x, f.y, n.z, f.x, f.y, n.z, f.x, f.y, f.z, n.x, f.y, f.z);
  cb_quad(s, cell, p, 1, 1, 1);
  set4(p, n.x, n.y, n.z, f.x, n.y, n.z, f.x, f.y, n.z, n.x, f.y, n.z);
  cb_quad(s, cell, p, 1, 1, 1);
  set4(p, n.x, n.y, f.z, f.x, n.y, f.z, f.x, f.y, f.z, n.x, f.y, f.z);
  cb_quad(s, cell, p, 1, 1, 1);
}

/* CornellBox::buildDataSet, CornellBox.cpp:141-418 + the extractors
 * (MapperPathTracer.cxx:178-197: SphereExtractor radius 90/555.0,
 * QuadExtractor in cell order skipping the vertex cell) */
void rtpo_cornell_box(int32_t variant, rtpo_scene* s) {
  memset(s, 0, sizeof(*s));
  const float tex[4][3] = {{0.65, 0.05, 0.05}, {0.73, 0.73, 0.73}, {0.12, 0.45, 0.15}, {15, 15, 15}};
  const int mt[5] = {0, 0, 0, 1, 2}, tt[5] = {0, 1, 2, 3, 0};
  s->n_tex = 4;
  memcpy(s->tex, tex, sizeof(tex));
  s->n_mat = 5;
  s->n_tex_type = 5;
  for (int i = 0; i < 5; i++) s->mat_type[i] = mt[i], s->tex_type[i] = tt[i];
  int cell = 0;
  float p[4][3];
  /* yz_rect x=555 green (:175-186) */
  set4(p, 555, 0, 0, 555, 555, 0, 555, 555, 555, 555, 0, 555);
  cb_quad(s, &cell, p, 1, 2, 2);
  /* yz_rect x=0 red (:189-200); first point is vec3(0,0,0) undivided */
  set4(p, 0, 0, 0, 0, 555, 0, 0, 555, 555, 0, 0, 555);
  cb_quad(s, &cell, p, 1, 0, 0); /* four field values (:197-200), like every quad: 89 for 89 points */
  /* light (:204-215) */
  set4(p, 213, 554, 227, 343, 554, 227, 343, 554, 332, 213, 554, 332);
  cb_quad(s, &cell, p, 1, 3, 3);
  /* ceiling (:218-229) */
  set4(p, 0, 555, 0, 555, 555, 0, 555, 555, 555, 0, 555, 555);
  cb_quad(s, &cell, p, 1, 1, 1);
  /* floor (:232-243) */
  set4(p, 0, 0, 0, 555, 0, 0, 555, 0, 555, 0, 0, 555);
  cb_quad(s, &cell, p, 1, 1, 1);
  /* back wall (:247-258) */
  set4(p, 0, 0, 555, 555, 0, 555, 555, 555, 555, 0, 555, 555);
  cb_quad(s, &cell, p, 1, 1, 1);
  if (variant == 3) { /* C3 scene (rtp_oracle.h) */
    s->light_box_pointids[0] = 0;
    s->light_box_pointids[1] = 8;
    s->light_box_pointids[2] = 9;
    s->light_box_pointids[3] = 10;
    s->light_box_pointids[4] = 11;
    s->light_sphere_point = s->n_points; /* sphere 0 centre */
    s->ior = 1.5f;
    uint32_t st = RTPO_C3_SEED;
    for (int k = 0; k < RTPO_C3_SPHERES; k++) {
      float cx = 190, cy = 90, cz = 190, rad = 90;
      int mat = 4, tex = 0;
      if (k > 0) {
        float u4, u5;
        for (;;) { /* redraw spheres that would intersect sphere 0 */
          const float u0 = rtpo_randf(&st), u1 = rtpo_randf(&st), u2 = rtpo_randf(&st);
          const float u3 = rtpo_randf(&st);
          u4 = rtpo_randf(&st);
          u5 = rtpo_randf(&st);
          rad = 8.0f + 22.0f * u3;
          cx = rad + (555.0f - 2.0f * rad) * u0;
          cy = rad + (555.0f - 2.0f * rad) * u1;
          cz = rad + (555.0f - 2.0f * rad) * u2;
          const float dx = cx - 190.0f, dy = cy - 90.0f, dz = cz - 190.0f, g = 92.0f + rad;
          if (!(dx * dx + dy * dy + dz * dz < g * g)) break;
        }
        if (u4 < 0.8f) {
          mat = (int)(3.0f * u5);
          if (mat > 2) mat = 2;
          tex = mat;
        }
      }
      s->sphere_point[k] = s->n_points;
      cb_push_point(s, d555(cx), d555(cy), d555(cz));
      s->field[s->n_field++] = (float)cell++; /* vertex cell (:364 pattern) */
      s->sphere_radius[k] = d555(rad);
      s->sphere_mat[k] = mat;
      s->sphere_tex[k] = tex;
    }
    s->n_spheres = RTPO_C3_SPHERES;
    for (int i = 0; i < s->n_field; i++) s->field[i] /= (float)s->n_field; /* :389-390 */
    return;
  }
  /* small rotated box (:262-353) incl. the y=333 vertex typo (:327) */
  set4(p, 0, 0, 165, 165, 0, 165, 165, 330, 165, 0, 330, 165);
  cb_invert(p);
  cb_quad(s, &cell, p, 1, 1, 1);
  set4(p, 0, 0, 0, 165, 0, 0, 165, 330, 0, 0, 330, 0);
  cb_invert(p);
  cb_quad(s, &cell, p, 1, 1, 1);
  set4(p, 165, 0, 0, 165, 330, 0, 165, 330, 165, 165, 0, 165);
  cb_invert(p);
  cb_quad(s, &cell, p, 1, 1, 1);
  set4(p, 0, 0, 0, 0, 330, 0, 0, 330, 165, 0, 0, 165);
  cb_invert(p);
  cb_quad(s, &cell, p, 1, 1, 1);
  set4(p, 0, 333, 0, 165, 330, 0, 165, 330, 165, 0, 330, 165);
  cb_invert(p);
  cb_quad(s, &cell, p, 1, 1, 1);
  set4(p, 0, 0, 0, 165, 0, 0, 165, 0, 165, 0, 0, 165);
  cb_invert(p);
  cb_quad(s, &cell, p, 1, 1, 1);
  /* sphere vertex cell (:357-365) */
  float scx = -335, scy = 90, scz = 290;
  if (variant == 1) scx = 190, scy = 90, scz = 190;
  if (variant == 2) scx = 440, scy = 200, scz = 150;
  const float sphere_radii = 90;
  s->sphere_point[0] = s->n_points;
  cb_push_point(s, d555(scx), d555(scy), d555(scz));
  s->sphere_radius[0] = (float)(90 / 555.0); /* ExtractCells(cellset, 90/555.0) */
  s->sphere_mat[0] = 4;
  s->sphere_tex[0] = 0;
  s->n_spheres = 1;
  s->field[s->n_field++] = (float)cell; /* vertex cell (:364) */
  cell++;
  /* boxes (:368-386) */
  v3 bc = mk(135, 90, 290);
  cb_box(s, &cell, mk(bc.x - sphere_radii, 0, bc.z - sphere_radii), mk(bc.x + sphere_radii, 180, bc.z + sphere_radii));
  cb_box(s, &cell, mk(50, 0, 50), mk(450, 100, 100));
  /* light coupling (MapperPathTracer.cxx:141-148) */
  s->light_box_pointids[0] = 0;
  s->light_box_pointids[1] = 8;
  s->light_box_pointids[2] = 9;
  s->light_box_pointids[3] = 10;
  s->light_box_pointids[4] = 11;
  s->light_sphere_point = 4 * 12;
  s->ior = 1.5f;
  for (int i = 0; i < s->n_field; i++) s->field[i] /= (float)s->n_field; /* :389-390 */
}

/* ------------------------------------------------------------ camera --- */
/* Camera::SetParameters/SetUp (Camera.cxx:624-637, 767-776), the look vector
 * (Camera.cxx:908-909) and RayGen's constructor (Camera.cxx:437-474) with
 * fovX := fovY (Camera.cxx:925-931) and _zoom = 0. */
void rtpo_camera_setup(const float pos[3], const float look_at[3], const float up_in[3], float fov_y_deg,
                       int32_t nx, int32_t ny, float cam[12]) {
  v3 up = ld(up_in);
  if (!(up.x == 0.f && up.y == 1.f && up.z == 0.f)) up = scl(up, rmag(up)); /* SetUp: Normalize if changed */
  v3 position = ld(pos);
  v3 look = sub(ld(look_at), position);
  look = scl(look, rmag(look));
  float thx = tanf((fov_y_deg * PI_180F) * .5f);
  float thy = tanf((fov_y_deg * PI_180F) * .5f);
  v3 u = cross(look, up);
  u = scl(u, rmag(u));
  v3 v = cross(u, look);
  v = scl(v, rmag(v));
  v3 dx = scl(u, (2 * thx / (float)nx));
  v3 dy = scl(v, (2 * thy / (float)ny));
  v3 nlook = scl(look, rmag(look));
  float out[12] = {position.x, position.y, position.z, nlook.x, nlook.y, nlook.z,
                   dx.x,       dx.y,       dx.z,       dy.x,    dy.y,    dy.z};
  memcpy(cam, out, sizeof(out));
}

/* Camera::RayGen::operator(), Camera.cxx:482-524 (2 draws per pixel) */
static inline v3 raygen(const float cam[12], int32_t nx, int32_t ny, int64_t idx, uint32_t* seed) {
  int i = (int32_t)idx % nx;
  int j = (int32_t)idx / nx;
  float ru = rtpo_randf(seed);
  float rv = rtpo_randf(seed);
  v3 nlook = ld(cam + 3), dx = ld(cam + 6), dy = ld(cam + 9);
  v3 rd = add(add(nlook, scl(dx, ((2.f * ((float)i + (1.f - ru)) - (float)nx) / 2.0f))),
              scl(dy, ((2.f * ((float)j + (rv)) - (float)ny) / 2.0f)));
  if (rd.x == 0.f) rd.x += 0.0000001f;
  if (rd.y == 0.f) rd.y += 0.0000001f;
  if (rd.z == 0.f) rd.z += 0.0000001f;
  float sq_mag = sqrtf(dot(rd, rd));
  return mk(rd.x / sq_mag, rd.y / sq_mag, rd.z / sq_mag);
}

/* -------------------------------------------------- sampling helpers --- */
/* CosineWorketletGenerateDir::random_cosine_direction, PdfWorklet.h:47-53
 * (the reference's 2*sqrt(r2) -- directions are neither unit nor cosine
 * distributed; kept) */
static inline v3 random_cosine_direction(float r1, float r2) {
  float z = sqrtf(1 - r2);
  float phi = (float)(2 * PI_D * r1);
  float x = rtpo_cosf(phi) * 2 * sqrtf(r2);
  float y = rtpo_sinf(phi) * 2 * sqrtf(r2);
  return mk(x, y, z);
}
/* SphereWorkletGenerateDir::random_to_sphere, PdfWorklet.h:157-165 */
static inline v3 random_to_sphere(float radius, float distance_squared, float r1, float r2) {
  float z = 1 + r2 * (sqrtf(1 - radius * radius / distance_squared) - 1);
  float phi = (float)(2 * PI_D * r1);
  float x = rtpo_cosf(phi) * sqrtf(1 - z * z);
  float y = rtpo_sinf(phi) * sqrtf(1 - z * z);
  return mk(x, y, z);
}

typedef struct {
  v3 q, r, s, t;   /* light quad points light_box_pointids[1..4] */
  v3 g1, g2;       /* generation corners pts[pointIndex[1]], pts[pointIndex[3]] */
  v3 sph_c;        /* light sphere centre */
  float sph_r;     /* SphereRadii[0] */
} lights;

static void setup_lights(const rtpo_scene* sc, lights* L) {
  const int32_t* id = sc->light_box_pointids;
  L->q = ld(sc->points[id[1]]);
  L->r = ld(sc->points[id[2]]);
  L->s = ld(sc->points[id[3]]);
  L->t = ld(sc->points[id[4]]);
  L->g1 = ld(sc->points[id[1]]);
  L->g2 = ld(sc->points[id[3]]);
  L->sph_c = ld(sc->points[sc->light_sphere_point]);
  L->sph_r = sc->sphere_radius[0];
}

/* QuadWorkletGenerateDir, PdfWorklet.h:89-136 (3 draws) */
static inline v3 gen_quad(const lights* L, v3 p, uint32_t* seed) {
  float x0 = L->g1.x, x1 = L->g2.x, z0 = L->g1.z, z1 = L->g2.z, y0 = L->g1.y, y1 = L->g1.y;
  float r1 = rtpo_randf(seed);
  float r2 = rtpo_randf(seed);
  float r3 = rtpo_randf(seed);
  v3 rp = mk(x0 + r1 * (x1 - x0), y0 + r2 * (y1 - y0), z0 + r3 * (z1 - z0));
  return sub(rp, p);
}
/* SphereWorkletGenerateDir, PdfWorklet.h:167-212 (2 draws; g++ evaluates
 * random(p, getRandF(seed), getRandF(seed), ...) right to left, so r1 is the
 * SECOND draw) */
static inline v3 gen_sphere(const lights* L, v3 p, uint32_t* seed) {
  float first = rtpo_randf(seed);
  float second = rtpo_randf(seed);
  float r1 = second, r2 = first;
  v3 direction = sub(L->sph_c, p);
  float distance_squared = dot(direction, direction);
  onb uvw = build_from_w(direction);
  return de_nan(local(&uvw, random_to_sphere(L->sph_r, distance_squared, r1, r2)));
}
/* CosineWorketletGenerateDir, PdfWorklet.h:63-79 (2 draws) */
static inline v3 gen_cosine(v3 n, uint32_t* seed) {
  float r1 = rtpo_randf(seed);
  float r2 = rtpo_randf(seed);
  onb uvw = build_from_w(n);
  return de_nan(local(&uvw, random_cosine_direction(r1, r2)));
}
/* QuadPDFWorklet::pdf_value, PdfWorklet.h:230-248 */
static inline float quad_pdf_value(const lights* L, v3 o, v3 v) {
  hitrec rec;
  if (quad_intersect(o, v, 0.001f, FLT_MAX, L->q, L->r, L->s, L->t, &rec)) {
    float qr = mag(sub(L->r, L->q));
    float qt = mag(sub(L->t, L->q));
    float area = qr * qt;
    float rect = rec.t;
    float distance_squared = rect * rect * dot(v, v);
    float cosine = fabsf(dot(v, rec.n) * rmag(v));
    return distance_squared / (cosine * area);
  }
  return 0;
}
/* SpherePDFWorklet::pdf_value, PdfWorklet.h:333-346 */
static inline float sphere_pdf_value(const lights* L, v3 o, v3 v) {
  hitrec rec;
  if (sphere_hit(o, v, 0.001f, FLT_MAX, L->sph_c, L->sph_r, &rec)) {
    float cos_theta_max = sqrtf(1 - L->sph_r * L->sph_r / dot(sub(L->sph_c, o), sub(L->sph_c, o)));
    float solid_angle = (float)(2 * PI_D * (1 - cos_theta_max));
    return 1 / solid_angle;
  }
  return 0;
}
/* DielectricWorklet::schlick / refract / reflect, EmitWorklet.h:153-175 */
static inline float schlick(float cosine, float ref_idx) {
  float r0 = (1 - ref_idx) / (1 + ref_idx);
  r0 = r0 * r0;
  return (float)(r0 + (1 - r0) * pow((double)(1 - cosine), 5.0));
}
static inline int refract(v3 v, v3 n, float ni_over_nt, v3* refracted) {
  v3 uv = unit_vector(v);
  float dt = dot(uv, n);
  float discriminant = (float)(1.0 - ni_over_nt * ni_over_nt * (1 - dt * dt));
  if (discriminant > 0) {
    *refracted = sub(scl(sub(uv, scl(n, dt)), ni_over_nt), scl(n, sqrtf(discriminant)));
    return 1;
  }
  return 0;
}
/* DielectricWorklet::scatter, EmitWorklet.h:180-226.  When refraction fails
 * and the draw is exactly 1.0f the reference reads an uninitialised vec3;
 * this restatement (and the HIP path) use (0,0,0) there. */
static inline void dielectric_scatter(v3 dir, v3 n, v3 p, float ref_idx, double rnd, v3* so, v3* sd) {
  v3 reflected = sub(dir, scl(n, 2 * dot(dir, n)));
  v3 refracted = mk(0, 0, 0);
  v3 outward;
  float ni_over_nt, cosine, reflect_prob;
  if (dot(dir, n) > 0) {
    outward = neg(n);
    ni_over_nt = ref_idx;
    cosine = ref_idx * dot(dir, n) * rmag(dir);
  } else {
    outward = n;
    ni_over_nt = (float)(1.0 / ref_idx);
    cosine = -dot(dir, n) * rmag(dir);
  }
  if (refract(dir, outward, ni_over_nt, &refracted))
    reflect_prob = schlick(cosine, ref_idx);
  else
    reflect_prob = 1.0;
  *so = p;
  *sd = (rnd < reflect_prob) ? reflected : refracted;
}

/* ------------------------------------------- scalar per-pixel variant --- */
/* Intersect one ray against every quad (index order, strict closest) then
 * every sphere with tmax from the quads -- the closest-hit semantics of
 * BVHTraverser.h:128-227 + Surface.h:208-254, 376-409 (a BVH only changes
 * the visiting order, which matters for exactly equal t only). */
static int scene_hit(const rtpo_scene* sc, v3 o, v3 d, hitrec* rec, int* hm, int* ht) {
  int hit = 0;
  float closest = FLT_MAX;
  const float tmin = (float)0.001;
  for (int q = 0; q < sc->n_quads; q++) {
    const int32_t* id = sc->quad_ids[q];
    hitrec tmp;
    if (quad_intersect(o, d, tmin, closest, ld(sc->points[id[1]]), ld(sc->points[id[2]]), ld(sc->points[id[3]]),
                       ld(sc->points[id[4]]), &tmp)) {
      *rec = tmp;
      closest = tmp.t;
      *hm = sc->quad_mat[q];
      *ht = sc->quad_tex[q];
      hit = 1;
    }
  }
  float tmax = hit ? closest : FLT_MAX; /* BVHTraverser.h:225-226 */
  for (int k = 0; k < sc->n_spheres; k++) {
    hitrec tmp;
    if (sphere_hit(o, d, tmin, tmax, ld(sc->points[sc->sphere_point[k]]), sc->sphere_radius[k], &tmp)) {
      tmax = tmp.t;
      *rec = tmp;
      *hm = sc->sphere_mat[k];
      *ht = sc->sphere_tex[k];
      hit = 1;
    }
  }
  return hit;
}

/* One pixel, S samples x D depths, in the stage order of
 * MapperPathTracer.cxx:278-354. A/E hold attenuation/emitted per depth. */
static void trace_pixel(const rtpo_scene* sc, const lights* L, const float cam[12], int32_t nx, int32_t ny,
                        int32_t spp, int32_t depth, uint32_t seed0, int64_t pix, v3* A, v3* E, float out[4],
                        uint32_t* seed_out, uint32_t* live_out) {
  uint32_t seed = seed0;
  float col[3] = {0, 0, 0};
  uint32_t live = 0;
  hitrec hrec;
  memset(&hrec, 0, sizeof(hrec));
  v3 sA = mk(0, 0, 0), sO = mk(0, 0, 0), sD = mk(0, 0, 0);
  const float weight = (float)(1.0 / (float)2); /* lightables = 2, MapperPathTracer.cxx:218 */
  for (int s = 0; s < spp; s++) {
    v3 dir = raygen(cam, nx, ny, pix, &seed);
    v3 org = ld(cam);
    int alive = 1, spec = 0;
    for (int d = 0; d < depth; d++) {
      float sum = 0;
      /* intersect, MapperPathTracer.cxx:408-435 */
      int hit = 0, hm = 0, ht = 0;
      if (alive) {
        live++;
        hit = scene_hit(sc, org, dir, &hrec, &hm, &ht);
      }
      /* CollectIntersecttWorklet, SurfaceWorklets.h:104-109 */
      if (!(alive && hit)) {
        alive = 0;
        A[d] = mk(1.0f, 1.0f, 1.0f);
        E[d] = mk(0.0f, 0.0f, 0.0f);
      }
      /* applyMaterials, MapperPathTracer.cxx:451-479 / EmitWorklet.h */
      if (alive) {
        int mt = sc->mat_type[hm];
        v3 albedo = ld(sc->tex[sc->tex_type[ht]]);
        if (mt == 0) { /* LambertianWorklet :58-70 */
          E[d] = mk(0, 0, 0);
          sA = albedo;
          spec = 0;
        } else if (mt == 1) { /* DiffuseLightWorklet :124-133 */
          E[d] = (dot(hrec.n, dir) < 0.0) ? albedo : mk(0, 0, 0);
          alive = 0;
          spec = 0;
        } else if (mt == 2) { /* DielectricWorklet :257-270 */
          float r = rtpo_randf(&seed);
          sA = mk(1, 1, 1);
          dielectric_scatter(dir, hrec.n, hrec.p, sc->ior, r, &sO, &sD);
          spec = 1;
          E[d] = mk(0, 0, 0);
        }
      }
      /* generateRays, MapperPathTracer.cxx:481-503 (every ray draws) */
      v3 gen = mk(0, 0, 0);
      int w = which_of(rtpo_randf(&seed));
      if (w <= 1) gen = gen_cosine(hrec.n, &seed);
      if (w == 2) gen = gen_quad(L, hrec.p, &seed);
      if (w == 3) gen = gen_sphere(L, hrec.p, &seed);
      /* applyPDFs, MapperPathTracer.cxx:505-538 */
      if (alive) sum += weight * quad_pdf_value(L, hrec.p, gen);
      if (alive) {
        (void)rtpo_randf(&seed); /* SpherePDFWorklet :391, discarded */
        sum += weight * sphere_pdf_value(L, hrec.p, gen);
      }
      /* PDFCosineWorklet, ScatterWorklet.h:79-116 (bit 1 is never set) */
      v3 atten = mk(1.0f, 1.0f, 1.0f);
      v3 out_o = org, out_d = dir;
      if (alive) {
        if (spec) {
          atten = sA;
          out_o = sO;
          out_d = sD;
        } else {
          onb uvw = build_from_w(hrec.n);
          out_o = hrec.p;
          out_d = gen;
          float cv;
          {
            float cosine = dot(unit_vector(gen), uvw.w);
            cv = (cosine > 0) ? (float)(cosine / PI_D) : 0;
          }
          double pdf_val = 0.5 * sum + 0.5 * cv;
          float sp;
          {
            float cosine = dot(hrec.n, unit_vector(out_d));
            sp = (cosine < 0) ? 0 : (float)(cosine / PI_D);
          }
          double sctr = sp / pdf_val;
          atten = mk((float)(sA.x * sctr), (float)(sA.y * sctr), (float)(sA.z * sctr));
        }
      }
      A[d] = atten;
      org = out_o;
      dir = out_d;
    }
    /* backward radiance, MapperPathTracer.cxx:328-348, then cols += s (:350) */
    v3 sum = add(E[depth - 1], mk(0, 0, 0));
    for (int d = depth - 2; d >= 0; d--) {
      sum = mk(A[d].x * sum.x, A[d].y * sum.y, A[d].z * sum.z);
      sum = add(E[d], sum);
    }
    col[0] = col[0] + sum.x;
    col[1] = col[1] + sum.y;
    col[2] = col[2] + sum.z;
  }
  out[0] = col[0];
  out[1] = col[1];
  out[2] = col[2];
  out[3] = 0.0f;
  if (seed_out) *seed_out = seed;
  if (live_out) *live_out = live;
}

void rtpo_render_pixels(const rtpo_scene* sc, const float cam[12], int32_t nx, int32_t ny, int32_t spp,
                        int32_t depth, uint32_t seed_base, const int64_t* pixels, int64_t npix, float* out_rgba,
                        uint32_t* out_seed, uint32_t* out_live, int32_t nthreads) {
  if (depth < 1 || spp < 0) return;
  lights L;
  setup_lights(sc, &L);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
  {
    v3* A = (v3*)malloc(sizeof(v3) * depth);
    v3* E = (v3*)malloc(sizeof(v3) * depth);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
    for (int64_t k = 0; k < npix; k++) {
      int64_t pix = pixels[k];
      trace_pixel(sc, &L, cam, nx, ny, spp, depth, seed_base + (uint32_t)pix, pix, A, E, out_rgba + 4 * k,
                  out_seed ? out_seed + k : NULL, out_live ? out_live + k : NULL);
    }
    free(A);
    free(E);
  }
  (void)nthreads;
}

/* -------------------------------------------- stage-structured (SoA) --- */
/* Every stage is a pass over all N rays, exactly as the worklet dispatches
 * of RenderCellsImpl: same arrays, same order, dead rays dispatched too.
 * Per-depth buffers A/E are depth-major [d*N + i] (Ray.h:268-275). */
typedef struct {
  float *ox, *oy, *oz, *dx, *dy, *dz;
  uint8_t* status;
  float *ht, *hnx, *hny, *hnz, *hpx, *hpy, *hpz; /* HitRecord (U,V unused) */
  int32_t *hm, *htx;                              /* HitId */
  float *sox, *soy, *soz, *sdx, *sdy, *sdz, *sax, *say, *saz; /* ScatterRecord */
  float *gx, *gy, *gz, *sum, *tmin;
  int32_t* which;
  float *Ax, *Ay, *Az, *Ex, *Ey, *Ez;
  float *tx, *ty, *tz;                            /* sumtotl */
  uint32_t* seeds;
  uint32_t* live;
} soa_t;

#define FOR_RAYS for (int64_t i = 0; i < n; i++)
#define OMP_FOR _Pragma("omp parallel for schedule(static) num_threads(nthreads)")

int32_t rtpo_render_soa(const rtpo_scene* sc, const float cam[12], int32_t nx, int32_t ny, int32_t spp,
                        int32_t depth, uint32_t seed_base, int32_t row_begin, int32_t row_end, float* out_rgba,
                        uint32_t* out_seed, uint32_t* out_live, int32_t nthreads) {
  if (depth < 1 || spp < 0 || row_begin < 0 || row_end > ny || row_begin >= row_end) return -1;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#else
  nthreads = 1;
#endif
  lights L;
  setup_lights(sc, &L);
  const int64_t first = (int64_t)row_begin * nx;
  const int64_t n = (int64_t)(row_end - row_begin) * nx;
  soa_t R;
  float** fl[] = {&R.ox, &R.oy, &R.oz, &R.dx, &R.dy, &R.dz, &R.ht, &R.hnx, &R.hny, &R.hnz, &R.hpx, &R.hpy,
                  &R.hpz, &R.sox, &R.soy, &R.soz, &R.sdx, &R.sdy, &R.sdz, &R.sax, &R.say, &R.saz, &R.gx, &R.gy,
                  &R.gz, &R.sum, &R.tmin, &R.tx, &R.ty, &R.tz};
  for (size_t k = 0; k < sizeof(fl) / sizeof(fl[0]); k++) *fl[k] = (float*)calloc(n, sizeof(float));
  float** dl[] = {&R.Ax, &R.Ay, &R.Az, &R.Ex, &R.Ey, &R.Ez};
  for (size_t k = 0; k < 6; k++) *dl[k] = (float*)calloc(n * depth, sizeof(float));
  R.status = (uint8_t*)calloc(n, 1);
  R.hm = (int32_t*)calloc(n, 4);
  R.htx = (int32_t*)calloc(n, 4);
  R.which = (int32_t*)calloc(n, 4);
  R.seeds = (uint32_t*)calloc(n, 4);
  R.live = (uint32_t*)calloc(n, 4);
  float* cols = (float*)calloc(n * 3, sizeof(float));
  const float weight = (float)(1.0 / (float)2);
  const float tmin_c = (float)0.001;
  /* seeds[i] = i (MapperPathTracer.cxx:265-267) */
  OMP_FOR FOR_RAYS R.seeds[i] = seed_base + (uint32_t)(first + i);
  for (int s = 0; s < spp; s++) {
    /* CreateRays (Camera.cxx:879-960) + Status = 8 */
    OMP_FOR FOR_RAYS {
      v3 d = raygen(cam, nx, ny, first + i, &R.seeds[i]);
      R.dx[i] = d.x, R.dy[i] = d.y, R.dz[i] = d.z;
      R.ox[i] = cam[0], R.oy[i] = cam[1], R.oz[i] = cam[2];
      R.status[i] = 1u << 3;
    }
    for (int dep = 0; dep < depth; dep++) {
      float* Ax = R.Ax + (int64_t)dep * n;
      float* Ay = R.Ay + (int64_t)dep * n;
      float* Az = R.Az + (int64_t)dep * n;
      float* Ex = R.Ex + (int64_t)dep * n;
      float* Ey = R.Ey + (int64_t)dep * n;
      float* Ez = R.Ez + (int64_t)dep * n;
      OMP_FOR FOR_RAYS { R.sum[i] = 0; R.ht[i] = FLT_MAX; R.tmin[i] = tmin_c; }
      /* quad traversal (BVHTraverser over QuadLeafIntersector) */
      OMP_FOR FOR_RAYS {
        if (R.status[i] & 8) R.live[i]++;
        if (!(R.status[i] & 8)) continue;
        v3 o = mk(R.ox[i], R.oy[i], R.oz[i]), d = mk(R.dx[i], R.dy[i], R.dz[i]);
        float closest = R.ht[i];
        int hit = 0;
        for (int q = 0; q < sc->n_quads; q++) {
          const int32_t* id = sc->quad_ids[q];
          hitrec tmp;
          if (quad_intersect(o, d, R.tmin[i], closest, ld(sc->points[id[1]]), ld(sc->points[id[2]]),
                             ld(sc->points[id[3]]), ld(sc->points[id[4]]), &tmp)) {
            R.ht[i] = tmp.t;
            R.hnx[i] = tmp.n.x, R.hny[i] = tmp.n.y, R.hnz[i] = tmp.n.z;
            R.hpx[i] = tmp.p.x, R.hpy[i] = tmp.p.y, R.hpz[i] = tmp.p.z;
            R.hm[i] = sc->quad_mat[q];
            R.htx[i] = sc->quad_tex[q];
            closest = tmp.t;
            hit = 1;
          }
        }
        R.status[i] |= (uint8_t)(hit << 2);
        R.ht[i] = hit ? closest : FLT_MAX;
      }
      /* sphere traversal */
      OMP_FOR FOR_RAYS {
        if (!(R.status[i] & 8)) continue;
        v3 o = mk(R.ox[i], R.oy[i], R.oz[i]), d = mk(R.dx[i], R.dy[i], R.dz[i]);
        float closest = R.ht[i];
        int hit = 0;
        for (int k = 0; k < sc->n_spheres; k++) {
          hitrec tmp;
          if (sphere_hit(o, d, R.tmin[i], closest, ld(sc->points[sc->sphere_point[k]]), sc->sphere_radius[k],
                         &tmp)) {
            closest = tmp.t;
            R.hnx[i] = tmp.n.x, R.hny[i] = tmp.n.y, R.hnz[i] = tmp.n.z;
            R.hpx[i] = tmp.p.x, R.hpy[i] = tmp.p.y, R.hpz[i] = tmp.p.z;
            R.hm[i] = sc->sphere_mat[k];
            R.htx[i] = sc->sphere_tex[k];
            hit = 1;
          }
        }
        R.status[i] |= (uint8_t)(hit << 2);
        if ((R.status[i] & 8) && (R.status[i] & 4)) R.ht[i] = closest;
      }
      /* CollectIntersecttWorklet */
      OMP_FOR FOR_RAYS {
        uint8_t st = R.status[i];
        if (!((st & 8) && (st & 4))) {
          st &= (uint8_t)~8u;
          Ax[i] = 1.0f, Ay[i] = 1.0f, Az[i] = 1.0f;
          Ex[i] = 0.0f, Ey[i] = 0.0f, Ez[i] = 0.0f;
        }
        st &= (uint8_t)~4u;
        R.status[i] = st;
      }
      /* LambertianWorklet */
      OMP_FOR FOR_RAYS {
        uint8_t st = R.status[i];
        if (!(st & 2) && (st & 8) && sc->mat_type[R.hm[i]] == 0) {
          const float* c = sc->tex[sc->tex_type[R.htx[i]]];
          R.sax[i] = c[0], R.say[i] = c[1], R.saz[i] = c[2];
          R.status[i] = (uint8_t)((st | 8u) & ~16u);
          Ex[i] = 0, Ey[i] = 0, Ez[i] = 0;
        }
      }
      /* DiffuseLightWorklet */
      OMP_FOR FOR_RAYS {
        uint8_t st = R.status[i];
        if (!(st & 2) && (st & 8) && sc->mat_type[R.hm[i]] == 1) {
          const float* c = sc->tex[sc->tex_type[R.htx[i]]];
          v3 nn = mk(R.hnx[i], R.hny[i], R.hnz[i]), d = mk(R.dx[i], R.dy[i], R.dz[i]);
          int em = dot(nn, d) < 0.0;
          Ex[i] = em ? c[0] : 0, Ey[i] = em ? c[1] : 0, Ez[i] = em ? c[2] : 0;
          R.status[i] = 0; /* fin &= (false << 3) */
        }
      }
      /* DielectricWorklet */
      OMP_FOR FOR_RAYS {
        uint8_t st = R.status[i];
        if (!(st & 2) && (st & 8) && sc->mat_type[R.hm[i]] == 2) {
          float r = rtpo_randf(&R.seeds[i]);
          v3 so, sd;
          dielectric_scatter(mk(R.dx[i], R.dy[i], R.dz[i]), mk(R.hnx[i], R.hny[i], R.hnz[i]),
                             mk(R.hpx[i], R.hpy[i], R.hpz[i]), sc->ior, r, &so, &sd);
          R.sax[i] = 1, R.say[i] = 1, R.saz[i] = 1;
          R.sox[i] = so.x, R.soy[i] = so.y, R.soz[i] = so.z;
          R.sdx[i] = sd.x, R.sdy[i] = sd.y, R.sdz[i] = sd.z;
          R.status[i] = (uint8_t)(st | 8u | 16u);
          Ex[i] = 0, Ey[i] = 0, Ez[i] = 0;
        }
      }
      /* WhichGenerateDir (all rays) */
      OMP_FOR FOR_RAYS R.which[i] = which_of(rtpo_randf(&R.seeds[i]));
      /* CosineGenerateDir */
      OMP_FOR FOR_RAYS {
        if (R.which[i] <= 1) {
          v3 g = gen_cosine(mk(R.hnx[i], R.hny[i], R.hnz[i]), &R.seeds[i]);
          R.gx[i] = g.x, R.gy[i] = g.y, R.gz[i] = g.z;
        }
      }
      /* QuadGenerateDir */
      OMP_FOR FOR_RAYS {
        if (R.which[i] == 2) {
          v3 g = gen_quad(&L, mk(R.hpx[i], R.hpy[i], R.hpz[i]), &R.seeds[i]);
          R.gx[i] = g.x, R.gy[i] = g.y, R.gz[i] = g.z;
        }
      }
      /* SphereGenerateDir */
      OMP_FOR FOR_RAYS {
        if (R.which[i] == 3) {
          v3 g = gen_sphere(&L, mk(R.hpx[i], R.hpy[i], R.hpz[i]), &R.seeds[i]);
          R.gx[i] = g.x, R.gy[i] = g.y, R.gz[i] = g.z;
        }
      }
      /* QuadPdf */
      OMP_FOR FOR_RAYS {
        if (R.status[i] & 8)
          R.sum[i] += weight * quad_pdf_value(&L, mk(R.hpx[i], R.hpy[i], R.hpz[i]), mk(R.gx[i], R.gy[i], R.gz[i]));
      }
      /* SpherePdf */
      OMP_FOR FOR_RAYS {
        if (R.status[i] & 8) {
          (void)rtpo_randf(&R.seeds[i]);
          R.sum[i] += weight * sphere_pdf_value(&L, mk(R.hpx[i], R.hpy[i], R.hpz[i]), mk(R.gx[i], R.gy[i], R.gz[i]));
        }
      }
      /* PDFCosineWorklet */
      OMP_FOR FOR_RAYS {
        uint8_t st = R.status[i];
        if (!(st & 2)) {
          v3 atten = mk(1.0f, 1.0f, 1.0f);
          v3 oo = mk(R.ox[i], R.oy[i], R.oz[i]), od = mk(R.dx[i], R.dy[i], R.dz[i]);
          if (st & 8) {
            if (st & 16) {
              atten = mk(R.sax[i], R.say[i], R.saz[i]);
              oo = mk(R.sox[i], R.soy[i], R.soz[i]);
              od = mk(R.sdx[i], R.sdy[i], R.sdz[i]);
            } else {
              v3 nn = mk(R.hnx[i], R.hny[i], R.hnz[i]);
              v3 g = mk(R.gx[i], R.gy[i], R.gz[i]);
              onb uvw = build_from_w(nn);
              oo = mk(R.hpx[i], R.hpy[i], R.hpz[i]);
              od = g;
              float cv;
              {
                float cosine = dot(unit_vector(g), uvw.w);
                cv = (cosine > 0) ? (float)(cosine / PI_D) : 0;
              }
              double pdf_val = 0.5 * R.sum[i] + 0.5 * cv;
              float sp;
              {
                float cosine = dot(nn, unit_vector(od));
                sp = (cosine < 0) ? 0 : (float)(cosine / PI_D);
              }
              double sctr = sp / pdf_val;
              atten = mk((float)(R.sax[i] * sctr), (float)(R.say[i] * sctr), (float)(R.saz[i] * sctr));
            }
          }
          Ax[i] = atten.x, Ay[i] = atten.y, Az[i] = atten.z;
          R.ox[i] = oo.x, R.oy[i] = oo.y, R.oz[i] = oo.z;
          R.dx[i] = od.x, R.dy[i] = od.y, R.dz[i] = od.z;
        }
        R.status[i] = (uint8_t)(st & ~(st >> 3));
      }
    }
    /* backward SliceTransform passes (MapperPathTracer.cxx:328-348) */
    {
      const int64_t off = (int64_t)(depth - 1) * n;
      OMP_FOR FOR_RAYS {
        R.tx[i] = R.Ex[off + i] + 0.0f;
        R.ty[i] = R.Ey[off + i] + 0.0f;
        R.tz[i] = R.Ez[off + i] + 0.0f;
      }
    }
    for (int dep = depth - 2; dep >= 0; dep--) {
      const int64_t off = (int64_t)dep * n;
      OMP_FOR FOR_RAYS {
        R.tx[i] = R.Ax[off + i] * R.tx[i];
        R.ty[i] = R.Ay[off + i] * R.ty[i];
        R.tz[i] = R.Az[off + i] * R.tz[i];
      }
      OMP_FOR FOR_RAYS {
        R.tx[i] = R.Ex[off + i] + R.tx[i];
        R.ty[i] = R.Ey[off + i] + R.ty[i];
        R.tz[i] = R.Ez[off + i] + R.tz[i];
      }
    }
    /* cols += sumtotl (:350) */
    OMP_FOR FOR_RAYS {
      cols[3 * i + 0] = cols[3 * i + 0] + R.tx[i];
      cols[3 * i + 1] = cols[3 * i + 1] + R.ty[i];
      cols[3 * i + 2] = cols[3 * i + 2] + R.tz[i];
    }
  }
  FOR_RAYS {
    out_rgba[4 * i + 0] = cols[3 * i + 0];
    out_rgba[4 * i + 1] = cols[3 * i + 1];
    out_rgba[4 * i + 2] = cols[3 * i + 2];
    out_rgba[4 * i + 3] = 0.0f;
    if (out_seed) out_seed[i] = R.seeds[i];
    if (out_live) out_live[i] = R.live[i];
  }
  for (size_t k = 0; k < sizeof(fl) / sizeof(fl[0]); k++) free(*fl[k]);
  for (size_t k = 0; k < 6; k++) free(*dl[k]);
  free(R.status), free(R.hm), free(R.htx), free(R.which), free(R.seeds), free(R.live), free(cols);
  return 0;
}

/* NormalizeFunctor, main.cc:253-287 (alpha is normalised too; rgb de-NaN'd) */
void rtpo_normalize(float* rgba, int64_t n, int32_t spp) {
  const float samplecount = (float)spp;
  for (int64_t i = 0; i < n; i++) {
    float* c = rgba + 4 * i;
    for (int k = 0; k < 3; k++)
      if (!(c[k] == c[k])) c[k] = 0;
    for (int k = 0; k < 4; k++) c[k] = sqrtf(c[k] / samplecount);
  }
}

/* Test helper: compare the sinf/cosf restatement with this host's libm on
 * every stride-th float in [lo, hi] (bit patterns).  Returns the mismatch
 * count; *checked receives the number of floats compared. */
int64_t rtpo_check_sincos_vs_libm(float lo, float hi, uint32_t stride, int64_t* checked) {
  uint32_t a, b;
  memcpy(&a, &lo, 4);
  memcpy(&b, &hi, 4);
  int64_t bad = 0, n = 0;
  if (stride == 0) stride = 1;
  for (uint64_t u = a; u <= b; u += stride) {
    uint32_t uu = (uint32_t)u;
    float f;
    memcpy(&f, &uu, 4);
    float s0 = rtpo_sinf(f), s1 = sinf(f), c0 = rtpo_cosf(f), c1 = cosf(f);
    if (memcmp(&s0, &s1, 4) != 0 || memcmp(&c0, &c1, 4) != 0) bad++;
    n++;
  }
  if (checked) *checked = n;
  return bad;
}

/* ================================================================ -direct ===
 * main.cc -direct (runRay / runNorms / runAlbedo, :120-251; generate(),
 * :386-431).  One View3D::Paint (View3D.cxx:53-64) of a quad mapper
 * (MapperQuad.cxx:86-150): Canvas::Clear, rays from VTK-m's raytracing
 * Camera, RayTracer::Render (IntersectRays, IntersectionData, SurfaceX::
 * Shade), CanvasRayTracer::WriteToCanvas, BlendBackground.
 *
 * VTK-m pieces restated from VTK-m 1.6's published sources (not vendored in
 * the reference; version not pinned):
 *  - Canvas::Clear: colour (0,0,0,0), depth 1.001f;
 *  - Camera::CreateRaysImpl with image-subset mode ON (boundingBox non-empty;
 *    the reference's own copy switched it off for the path only,
 *    Camera.cxx:1069) -> FindSubset, then PerspectiveRayGen; the reference's
 *    copies of both are Camera.cxx:339-423 and :963-1060;
 *  - BVH closest hit: distance = MaxDistance (inf) and hitIdx = -1 on a
 *    miss; quads in index order, tmin = 0 < t < tmax strict;
 *  - QuadIntersector::IntersectionData: intersection = o + t*d; normal =
 *    Normalize(TriangleNormal(p0,p1,p2)) flipped against the ray; scalar =
 *    (field[QuadIds[0]] - min) * invDelta (QuadIds[0] is the cell id);
 *  - SurfaceColor::Shade writes the shaded colour-map colour; the Normals /
 *    Albedo variants are the reference's RayTracerNormals.cxx:84-141 and
 *    RayTracerAlbedo.cxx:84-145;
 *  - WriteToCanvas (SurfaceConverter): depth = 0.5*(VP*p).z/(VP*p).w + 0.5,
 *    colour blended over the cleared canvas and clamped to [0,1] with
 *    std::min/std::max (CPU build: NaN -> 1);
 *  - Camera view/projection matrices (MatrixHelpers::ViewMatrix,
 *    Camera3DStruct::CreateProjectionMatrix);
 *  - ColorTable construction from (x,r,g,b) / (x,a,mid,sharp) quadruples
 *    (AddPoint: sorted insert, equal x overwrites, out-of-[0,1] colours
 *    dropped), Sample(n): n float-spaced values over the table range, linear
 *    RGB interpolation, clamped outside the nodes, std::round(c*255). */
typedef struct {
  float m[4][4];
} dmat4;
static dmat4 m4_identity(void) {
  dmat4 r;
  memset(&r, 0, sizeof(r));
  for (int i = 0; i < 4; i++) r.m[i][i] = 1.f;
  return r;
}
/* vtkm::MatrixMultiply: product(r,c) = Dot(row r, column c), left to right */
static dmat4 m4_mul(const dmat4* a, const dmat4* b) {
  dmat4 r;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      float acc = a->m[i][0] * b->m[0][j];
      acc = acc + a->m[i][1] * b->m[1][j];
      acc = acc + a->m[i][2] * b->m[2][j];
      acc = acc + a->m[i][3] * b->m[3][j];
      r.m[i][j] = acc;
    }
  return r;
}
static void m4_vec(const float m[16], const float v[4], float out[4]) {
  for (int i = 0; i < 4; i++) {
    float acc = m[4 * i + 0] * v[0];
    acc = acc + m[4 * i + 1] * v[1];
    acc = acc + m[4 * i + 2] * v[2];
    acc = acc + m[4 * i + 3] * v[3];
    out[i] = acc;
  }
}
/* MatrixHelpers::ViewMatrix(position, lookAt, up) */
static dmat4 view_matrix(v3 position, v3 look_at, v3 up) {
  v3 view_dir = sub(position, look_at);
  v3 right = cross(up, view_dir);
  v3 ru = cross(view_dir, right);
  view_dir = scl(view_dir, rmag(view_dir));
  right = scl(right, rmag(right));
  ru = scl(ru, rmag(ru));
  dmat4 m = m4_identity();
  m.m[0][0] = right.x, m.m[0][1] = right.y, m.m[0][2] = right.z;
  m.m[1][0] = ru.x, m.m[1][1] = ru.y, m.m[1][2] = ru.z;
  m.m[2][0] = view_dir.x, m.m[2][1] = view_dir.y, m.m[2][2] = view_dir.z;
  m.m[0][3] = -dot(right, position);
  m.m[1][3] = -dot(ru, position);
  m.m[2][3] = -dot(view_dir, position);
  return m;
}
/* Camera3DStruct::CreateProjectionMatrix (zoom 1, no pan) */
static dmat4 projection_matrix(int32_t w, int32_t h, float fov_deg, float near_plane, float far_plane) {
  dmat4 m = m4_identity();
  const float aspect = (float)w / (float)h;
  float fov_rad = fov_deg * PI_180F;
  fov_rad = tanf(fov_rad * 0.5f);
  const float size = near_plane * fov_rad;
  const float left = -size * aspect, right = size * aspect, bottom = -size, top = size;
  m.m[0][0] = 2.f * near_plane / (right - left);
  m.m[1][1] = 2.f * near_plane / (top - bottom);
  m.m[0][2] = (right + left) / (right - left);
  m.m[1][2] = (top + bottom) / (top - bottom);
  m.m[2][2] = -(far_plane + near_plane) / (far_plane - near_plane);
  m.m[3][2] = -1.f;
  m.m[2][3] = -(2.f * far_plane * near_plane) / (far_plane - near_plane);
  m.m[3][3] = 0.f;
  dmat4 T = m4_identity(), Z = m4_identity(); /* Transform3DTranslate(0,0,0), Transform3DScale(1,1,1) */
  dmat4 tm = m4_mul(&T, &m);
  return m4_mul(&Z, &tm);
}
static inline float stdmax(float a, float b) { return (a < b) ? b : a; } /* (std::max)(a, b) */
static inline float stdmin(float a, float b) { return (b < a) ? b : a; } /* (std::min)(a, b) */

void rtpo_direct_setup(const rtpo_scene* sc, const float pos[3], const float look_at[3], const float up_in[3],
                       float fov_y_deg, float clip_near, float clip_far, int32_t nx, int32_t ny,
                       rtpo_direct_cam* out) {
  memset(out, 0, sizeof(*out));
  /* raytracing::Camera::SetParameters on a fresh camera (500x500, fov 30):
   * SetUp (normalised if changed), SetFieldOfView, SetHeight, SetWidth
   * (Camera.cxx:624-637, 641-684, 716-764).  The net FovX is fovY for a
   * square canvas, else 2*atan(w/h * tan(fovY/2)). */
  v3 up = ld(up_in);
  if (!(up.x == 0.f && up.y == 1.f && up.z == 0.f)) up = scl(up, rmag(up));
  float fov_x = fov_y_deg;
  if (nx != ny) {
    const float fovy_rad = fov_y_deg * PI_180F;
    const float vertical = tanf(0.5f * fovy_rad);
    const float aspect = (float)nx / (float)ny;
    const float horizontal = aspect * vertical;
    const float fovx_rad = 2.0f * atanf(horizontal);
    fov_x = fovx_rad / PI_180F;
  }
  v3 position = ld(pos);
  v3 look = sub(ld(look_at), position); /* CreateRaysImpl: Look = LookAt - Position, Normalize */
  look = scl(look, rmag(look));
  /* PerspectiveRayGen constructor (Camera.cxx:351-392), zoom 1 */
  const float thx = tanf((fov_x * PI_180F) * .5f);
  const float thy = tanf((fov_y_deg * PI_180F) * .5f);
  v3 ru = cross(look, up);
  ru = scl(ru, rmag(ru));
  v3 rv = cross(ru, look);
  rv = scl(rv, rmag(rv));
  v3 dx = scl(ru, (2 * thx / (float)nx));
  v3 dy = scl(rv, (2 * thy / (float)ny));
  const float zoom = 1.f;
  dx = mk(dx.x / zoom, dx.y / zoom, dx.z / zoom);
  dy = mk(dy.x / zoom, dy.y / zoom, dy.z / zoom);
  v3 nlook = scl(look, rmag(look));
  memcpy(out->eye, &position, 12);
  memcpy(out->nlook, &nlook, 12);
  memcpy(out->dx, &dx, 12);
  memcpy(out->dy, &dy, 12);
  out->nx = nx, out->ny = ny;
  /* view-projection of the vtkm::rendering::Camera (raw ViewUp) */
  dmat4 V = view_matrix(position, ld(look_at), ld(up_in));
  dmat4 P = projection_matrix(nx, ny, fov_y_deg, clip_near, clip_far);
  dmat4 VP = m4_mul(&P, &V);
  memcpy(out->vp, VP.m, sizeof(VP.m));
  /* shape bounds: union of the quads' AABBs (AABBSurface.h:36-78) */
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int q = 0; q < sc->n_quads; q++) {
    const int32_t* id = sc->quad_ids[q];
    float mn[3], mx[3];
    for (int k = 0; k < 3; k++) mn[k] = mx[k] = sc->points[id[1]][k];
    for (int c = 2; c <= 4; c++)
      for (int k = 0; k < 3; k++) {
        mn[k] = stdmin(mn[k], sc->points[id[c]][k]);
        mx[k] = stdmax(mx[k], sc->points[id[c]][k]);
      }
    for (int k = 0; k < 3; k++) {
      const float eps = stdmax(1e-6f, 1.0e-4f * (mx[k] - mn[k]));
      mn[k] -= eps;
      mx[k] += eps;
      lo[k] = lo[k] < mn[k] ? lo[k] : mn[k];
      hi[k] = hi[k] > mx[k] ? hi[k] : mx[k];
    }
  }
  /* FindSubset (Camera.cxx:963-1060) */
  if (sc->n_quads == 0 || (position.x >= lo[0] && position.x <= hi[0] && position.y >= lo[1] &&
                           position.y <= hi[1] && position.z >= lo[2] && position.z <= hi[2])) {
    out->sub_x0 = 0, out->sub_y0 = 0, out->sub_w = nx, out->sub_h = ny;
  } else {
    float xmin = INFINITY, ymin = INFINITY, zmin = INFINITY, xmax = -INFINITY, ymax = -INFINITY, zmax = -INFINITY;
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          const float e[4] = {i ? hi[0] : lo[0], j ? hi[1] : lo[1], k ? hi[2] : lo[2], 1.f};
          float t[4];
          m4_vec(out->vp, e, t);
          for (int a = 0; a < 3; a++) t[a] = t[a] / t[3];
          t[0] = (t[0] * 0.5f + 0.5f) * (float)nx;
          t[1] = (t[1] * 0.5f + 0.5f) * (float)ny;
          t[2] = (t[2] * 0.5f + 0.5f);
          zmin = stdmin(zmin, t[2]);
          zmax = stdmax(zmax, t[2]);
          if (t[2] < 0 || t[2] > 1) continue;
          xmin = stdmin(xmin, t[0]);
          ymin = stdmin(ymin, t[1]);
          xmax = stdmax(xmax, t[0]);
          ymax = stdmax(ymax, t[1]);
        }
    xmin -= .001f;
    xmax += .001f;
    ymin -= .001f;
    ymax += .001f;
    xmin = floorf(stdmin(stdmax(0.f, xmin), (float)nx));
    xmax = ceilf(stdmin(stdmax(0.f, xmax), (float)nx));
    ymin = floorf(stdmin(stdmax(0.f, ymin), (float)ny));
    ymax = ceilf(stdmin(stdmax(0.f, ymax), (float)ny));
    const int32_t dxp = (int32_t)xmax - (int32_t)xmin, dyp = (int32_t)ymax - (int32_t)ymin;
    if (zmax < 0 || xmin >= xmax || ymin >= ymax) {
      out->sub_x0 = 0, out->sub_y0 = 0, out->sub_w = 1, out->sub_h = 1;
    } else {
      out->sub_x0 = (int32_t)xmin, out->sub_y0 = (int32_t)ymin, out->sub_w = dxp, out->sub_h = dyp;
    }
  }
  /* SurfaceX::run: light = Position + (2,2,2)*Up; Shade: viewDir normalised */
  v3 light = add(position, mk(2.f * up.x, 2.f * up.y, 2.f * up.z));
  v3 vd = sub(position, ld(look_at));
  vd = scl(vd, rmag(vd));
  memcpy(out->light, &light, 12);
  memcpy(out->view_dir, &vd, 12);
}

void rtpo_quad_scalars(const rtpo_scene* sc, float* out) {
  /* Actor::Init: scalar range = field min/max (double of the float values);
   * GetScalar's constructor takes them as float */
  float mn = INFINITY, mx = -INFINITY;
  for (int i = 0; i < sc->n_field; i++) {
    mn = sc->field[i] < mn ? sc->field[i] : mn;
    mx = sc->field[i] > mx ? sc->field[i] : mx;
  }
  const float inv = (mx - mn != 0.f) ? 1.f / (mx - mn) : 1.f / mn;
  for (int q = 0; q < sc->n_quads; q++) {
    const int32_t cell = sc->quad_ids[q][0];
    const float s = (cell >= 0 && cell < sc->n_field) ? sc->field[cell] : 0.f;
    out[q] = (s - mn) * inv;
  }
}

typedef struct {
  double x;
  float v[4];
} ct_node;
/* ColorTable::AddPoint / AddPointAlpha: sorted insert, an equal x overwrites */
static int ct_add(ct_node* nodes, int n, double x, const float* v, int nv) {
  int pos = 0;
  while (pos < n && nodes[pos].x < x) pos++;
  if (pos < n && nodes[pos].x == x) {
    memcpy(nodes[pos].v, v, sizeof(float) * nv);
    return n;
  }
  memmove(nodes + pos + 1, nodes + pos, sizeof(ct_node) * (n - pos));
  nodes[pos].x = x;
  memcpy(nodes[pos].v, v, sizeof(float) * nv);
  return n + 1;
}
static float ct_uchar(float t) { return (float)(unsigned char)roundf(t * 255.0f) * (1.0f / 255.0f); }

int32_t rtpo_sample_color_table(const double* rgb, int32_t n_rgb, const double* alpha, int32_t n_alpha,
                                const double nan_color[3], int32_t n_samples, float* out) {
  if (n_samples < 2 || n_rgb < 0 || n_alpha < 0) return -1;
  ct_node cn[256], an[256];
  int nc = 0, na = 0;
  double rmin = INFINITY, rmax = -INFINITY;
  if (n_rgb > 0 && n_rgb % 4 == 0)
    for (int i = 0; i + 3 < n_rgb && nc < 255; i += 4) {
      const float v[3] = {(float)rgb[i + 1], (float)rgb[i + 2], (float)rgb[i + 3]};
      if (v[0] < 0 || v[0] > 1 || v[1] < 0 || v[1] > 1 || v[2] < 0 || v[2] > 1) continue;
      nc = ct_add(cn, nc, rgb[i], v, 3);
      rmin = rgb[i] < rmin ? rgb[i] : rmin;
      rmax = rgb[i] > rmax ? rgb[i] : rmax;
    }
  if (n_alpha > 0 && n_alpha % 4 == 0)
    for (int i = 0; i + 3 < n_alpha && na < 255; i += 4) {
      const float v[3] = {(float)alpha[i + 1], (float)alpha[i + 2], (float)alpha[i + 3]};
      if (v[0] < 0 || v[0] > 1 || v[1] < 0 || v[1] > 1 || v[2] < 0 || v[2] > 1) continue;
      na = ct_add(an, na, alpha[i], v, 3);
      rmin = alpha[i] < rmin ? alpha[i] : rmin;
      rmax = alpha[i] > rmax ? alpha[i] : rmax;
    }
  if (nc == 0 && na == 0) rmin = rmax = 0;
  const double d_samples = (double)(n_samples - 1);
  const double d_delta = (rmax - rmin) / d_samples;
  const float f_samples = (float)(n_samples - 1);
  const float f_start = (float)rmin;
  const float f_delta = (float)(rmax - rmin) / f_samples;
  const float f_end = f_start + (f_delta * f_samples);
  const int use_f = fabs((double)f_end - rmax) <= 0.002 && fabs((double)f_delta - d_delta) <= 0.002;
  for (int i = 0; i < n_samples; i++) {
    double x;
    if (use_f)
      x = (double)(i == 0 ? f_start : (i == n_samples - 1 ? f_end : f_start + ((float)i * f_delta)));
    else
      x = i == 0 ? rmin : (i == n_samples - 1 ? rmax : rmin + ((double)i * d_delta));
    float c[3];
    if (x != x) {
      for (int k = 0; k < 3; k++) c[k] = (float)nan_color[k];
    } else if (nc == 0) {
      c[0] = c[1] = c[2] = 0.f;
    } else if (x <= cn[0].x) {
      memcpy(c, cn[0].v, 12);
    } else if (x >= cn[nc - 1].x) {
      memcpy(c, cn[nc - 1].v, 12);
    } else {
      int s = 1;
      while (cn[s].x < x) s++;
      const int f = s - 1;
      const float w = (float)((x - cn[f].x) / (cn[s].x - cn[f].x));
      for (int k = 0; k < 3; k++) c[k] = (1.0f - w) * cn[f].v[k] + w * cn[s].v[k]; /* vtkm::Lerp */
    }
    float a;
    if (na == 0) {
      a = 1.f;
    } else if (x <= an[0].x) {
      a = an[0].v[0];
    } else if (x >= an[na - 1].x) {
      a = an[na - 1].v[0];
    } else { /* linear between opacity nodes (midpoint 0.5, sharpness 0 only) */
      int s = 1;
      while (an[s].x < x) s++;
      const int f = s - 1;
      const float w = (float)((x - an[f].x) / (an[s].x - an[f].x));
      a = (1.0f - w) * an[f].v[0] + w * an[s].v[0];
    }
    out[4 * i + 0] = ct_uchar(c[0]);
    out[4 * i + 1] = ct_uchar(c[1]);
    out[4 * i + 2] = ct_uchar(c[2]);
    out[4 * i + 3] = ct_uchar(a);
  }
  return 0;
}

void rtpo_render_direct(const rtpo_scene* sc, const rtpo_direct_cam* cam, const float* quad_scalar,
                        const float* cmap, int32_t cmap_n, const float bg[4], int32_t composite, int32_t aov,
                        float* out_rgba, float* out_depth) {
  const int32_t nx = cam->nx, ny = cam->ny;
  const v3 eye = ld(cam->eye), nlook = ld(cam->nlook), ddx = ld(cam->dx), ddy = ld(cam->dy);
  const v3 L = ld(cam->light), V = ld(cam->view_dir);
#pragma omp parallel for schedule(static)
  for (int64_t idx = 0; idx < (int64_t)nx * ny; idx++) {
    const int32_t i = (int32_t)(idx % nx), j = (int32_t)(idx / nx);
    float c[4] = {0.f, 0.f, 0.f, 0.f}; /* Canvas::Clear */
    float depth = 1.001f;
    if (i >= cam->sub_x0 && i < cam->sub_x0 + cam->sub_w && j >= cam->sub_y0 && j < cam->sub_y0 + cam->sub_h) {
      /* PerspectiveRayGen::operator() (Camera.cxx:394-421) */
      v3 rd = add(add(nlook, scl(ddx, ((2.f * (float)i - (float)nx) / 2.0f))),
                  scl(ddy, ((2.f * (float)j - (float)ny) / 2.0f)));
      if (rd.x == 0.f) rd.x += 0.0000001f;
      if (rd.y == 0.f) rd.y += 0.0000001f;
      if (rd.z == 0.f) rd.z += 0.0000001f;
      const float sq_mag = sqrtf(dot(rd, rd));
      const v3 d = mk(rd.x / sq_mag, rd.y / sq_mag, rd.z / sq_mag);
      /* closest quad hit, index order, 0 < t < tmax */
      int hq = -1;
      float closest = INFINITY;
      for (int q = 0; q < sc->n_quads; q++) {
        const int32_t* id = sc->quad_ids[q];
        float T;
        if (quad_hit(eye, d, ld(sc->points[id[1]]), ld(sc->points[id[2]]), ld(sc->points[id[3]]),
                     ld(sc->points[id[4]]), &T) &&
            T < closest && T > 0.f) {
          closest = T;
          hq = q;
        }
      }
      float rc[4] = {0.f, 0.f, 0.f, 0.f}; /* Rays.Buffers[0].InitConst(0) */
      const float dist = closest;          /* MaxDistance (inf) on a miss */
      if (hq >= 0) {
        const int32_t* id = sc->quad_ids[hq];
        const v3 p = add(eye, scl(d, dist));
        v3 n = cross(sub(ld(sc->points[id[2]]), ld(sc->points[id[1]])), sub(ld(sc->points[id[3]]), ld(sc->points[id[1]])));
        n = scl(n, rmag(n));
        if (dot(n, d) > 0.f) n = neg(n);
        v3 ldir = sub(L, p);
        ldir = scl(ldir, rmag(ldir));
        float cos_t = dot(n, ldir);
        cos_t = stdmin(stdmax(cos_t, 0.f), 1.f);
        v3 refl = sub(scl(n, 2.f * dot(ldir, n)), ldir);
        refl = scl(refl, rmag(refl));
        const float cos_p = dot(refl, V);
        if (aov == RTPO_AOV_COLOR) {
          const float spec = powf(stdmax(cos_p, 0.f), 20.f);
          const float sf = quad_scalar[hq] * (float)(cmap_n - 1);
          int32_t ci = (sf > -2147483649.0f && sf < 2147483648.0f) ? (int32_t)sf : INT32_MIN; /* cvttss2si */
          ci = ci > 0 ? ci : 0;
          ci = ci < cmap_n - 1 ? ci : cmap_n - 1;
          for (int k = 0; k < 4; k++) rc[k] = cmap[4 * ci + k];
          for (int k = 0; k < 3; k++) rc[k] *= stdmin(0.5f + 0.7f * cos_t + 0.7f * spec, 1.f);
        } else if (aov == RTPO_AOV_NORMALS) {
          rc[0] = n.x, rc[1] = n.y, rc[2] = n.z, rc[3] = 1.0f;
        } else {
          rc[0] = (cos_p * refl.x) / (cos_t * ldir.x);
          rc[1] = (cos_p * refl.y) / (cos_t * ldir.y);
          rc[2] = (cos_p * refl.z) / (cos_t * ldir.z);
          rc[3] = 1.0f;
        }
      }
      /* WriteToCanvas / SurfaceConverter */
      const v3 ip = add(eye, scl(d, dist));
      const float pt[4] = {ip.x, ip.y, ip.z, 1.f};
      float np[4];
      m4_vec(cam->vp, pt, np);
      const float z = np[2] / np[3];
      depth = 0.5f * z + 0.5f;
      const float a = 1.f - rc[3];
      float o[4];
      o[0] = rc[0] + c[0] * a;
      o[1] = rc[1] + c[1] * a;
      o[2] = rc[2] + c[2] * a;
      o[3] = c[3] * a + rc[3];
      for (int k = 0; k < 4; k++) c[k] = stdmin(1.f, stdmax(o[k], 0.f));
    }
    if (composite && !(c[3] >= 1.f)) { /* BlendBackground */
      const float a = bg[3] * (1.f - c[3]);
      c[0] = c[0] + bg[0] * a;
      c[1] = c[1] + bg[1] * a;
      c[2] = c[2] + bg[2] * a;
      c[3] = a + c[3];
    }
    memcpy(out_rgba + 4 * idx, c, 16);
    if (out_depth) out_depth[idx] = depth;
  }
}
