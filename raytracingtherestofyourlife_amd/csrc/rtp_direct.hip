// rtp_direct.hip -- the -direct mode of main.cc (runRay / runNorms /
// runAlbedo, main.cc:120-251, 623-651) on gfx950: one lane per canvas pixel.
//
// The reference renders each AOV with its own View3D::Paint (View3D.cxx:
// 53-64): clear the canvas, cast the VTK-m raytracing Camera's rays, closest
// quad hit, QuadIntersector::IntersectionData, the mapper's SurfaceX::Shade,
// CanvasRayTracer::WriteToCanvas and BlendBackground -- three intersection
// passes over the same rays for colour, normals and albedo.  Here one launch
// intersects each ray once and writes every requested AOV plus the depth
// buffer; each output is bit-identical to its own reference render because
// the three renders share rays, hits and depth and each starts from a cleared
// canvas.  Scene data (DevScene) is wave-uniform and read with scalar loads,
// as in the path kernels; the only per-lane memory traffic is the output
// (16 B per AOV + 4 B depth per pixel, coalesced), so the kernel is bound by
// the closest-hit VALU work, not by HBM.
#include <hip/hip_runtime.h>

#include "glibc_powf.hpp"
#include "rtp_device.hpp"

namespace rtp {

namespace {

constexpr uint64_t kNoKey = ~0ull;

// Closest quad over the kind groups with the (t, reference index) key of the
// path kernels; here tmin = 0 (camera rays: MinDistance 0, strict '>').
// Positive floats order like their bit patterns, so the smallest key is the
// index-order strict-'<' winner of the reference's scan.
template <int K>
RTP_DEV void scan_direct(const DevScene* __restrict__ sc, int g, f3 o, f3 d, uint64_t& best) {
  const int b = sc->kind_begin[g], e = sc->kind_begin[g + 1];
  for (int q = b; q < e; q++) {
    const DevQuad& Q = sc->quads[q];
    float t;
    const bool ok = quad_hit_masked<K>(Q, Q, o, d, t);
    const uint64_t key = (uint64_t)__float_as_uint(t) << 32 | Q.key_lo;
    best = (ok && t > 0.0f && key < best) ? key : best;
  }
}

RTP_DEV uint64_t closest_quad(const DevScene* __restrict__ sc, f3 o, f3 d) {
  uint64_t key = kNoKey;
  scan_direct<1>(sc, 0, o, d, key);
  scan_direct<2>(sc, 1, o, d, key);
  scan_direct<3>(sc, 2, o, d, key);
  scan_direct<4>(sc, 3, o, d, key);
  scan_direct<5>(sc, 4, o, d, key);
  scan_direct<6>(sc, 5, o, d, key);
  scan_direct<7>(sc, 6, o, d, key);
  scan_direct<8>(sc, 7, o, d, key);
  scan_direct<9>(sc, 8, o, d, key);
  scan_direct<10>(sc, 9, o, d, key);
  scan_direct<0>(sc, 10, o, d, key);
  return key;
}

// (std::max)(a, b) / (std::min)(a, b) of the CPU build (vtkm::Max / Min):
// NaN propagates from the first argument of max, min(1, NaN) is 1
RTP_DEV float std_max(float a, float b) { return (a < b) ? b : a; }
RTP_DEV float std_min(float a, float b) { return (b < a) ? b : a; }

// vtkm::Int32(x) on x86-64 (cvttss2si): out-of-range and NaN give INT32_MIN
RTP_DEV int32_t cvt_i32_x86(float x) {
  return (x > -2147483649.0f && x < 2147483648.0f) ? (int32_t)x : (int32_t)0x80000000u;
}

RTP_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// CanvasRayTracer::WriteToCanvas (SurfaceConverter) over a cleared canvas,
// then Canvas::BlendBackground
RTP_DEV float4 to_canvas(float4 rc, const DirectParams& p) {
  const float a = 1.f - rc.w;
  float o0 = rc.x + 0.f * a, o1 = rc.y + 0.f * a, o2 = rc.z + 0.f * a, o3 = 0.f * a + rc.w;
  float4 c = make_float4(std_min(1.f, std_max(o0, 0.f)), std_min(1.f, std_max(o1, 0.f)),
                         std_min(1.f, std_max(o2, 0.f)), std_min(1.f, std_max(o3, 0.f)));
  if (p.composite && !(c.w >= 1.f)) {
    const float b = p.bg[3] * (1.f - c.w);
    c.x = c.x + p.bg[0] * b;
    c.y = c.y + p.bg[1] * b;
    c.z = c.z + p.bg[2] * b;
    c.w = b + c.w;
  }
  return c;
}

}  // namespace

__global__ void __launch_bounds__(256) rtp_render_direct_kernel(const DevScene* __restrict__ sc, DirectParams p) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= p.npix) return;
  const int32_t i = (int32_t)(idx % p.nx), j = (int32_t)(idx / p.nx);
  float depth = 1.001f;  // Canvas::Clear
  float4 rc_color = make_float4(0.f, 0.f, 0.f, 0.f), rc_norm = rc_color, rc_alb = rc_color;
  const bool in_sub = i >= p.sub_x0 && i < p.sub_x0 + p.sub_w && j >= p.sub_y0 && j < p.sub_y0 + p.sub_h;
  if (in_sub) {
    // PerspectiveRayGen::operator() (Camera.cxx:394-421)
    const f3 nlook = ld3(p.nlook), ddx = ld3(p.dx), ddy = ld3(p.dy), eye = ld3(p.eye);
    f3 rd = add(add(nlook, scl(ddx, ((2.f * (float)i - (float)p.nx) / 2.0f))),
                scl(ddy, ((2.f * (float)j - (float)p.ny) / 2.0f)));
    if (rd.x == 0.f) rd.x += 0.0000001f;
    if (rd.y == 0.f) rd.y += 0.0000001f;
    if (rd.z == 0.f) rd.z += 0.0000001f;
    const float sq_mag = sqrt_exact(dot(rd, rd));
    const f3 d = mk(rd.x / sq_mag, rd.y / sq_mag, rd.z / sq_mag);
    const uint64_t key = closest_quad(sc, eye, d);
    const bool hit = key != kNoKey;
    // BVH traversal: distance = MaxDistance (inf) unless a quad was hit
    const float dist = hit ? __uint_as_float((uint32_t)(key >> 32)) : __builtin_huge_valf();
    if (hit) {
      const DevQuad& Q = sc->quads[key & 0xff];
      // QuadIntersector::IntersectionData: intersection, normal, scalar
      const f3 pnt = add(eye, scl(d, dist));
      f3 n = ld3(Q.n);  // Normalize(TriangleNormal(p0, p1, p2))
      if (dot(n, d) > 0.f) n = neg(n);
      // SurfaceX::Shade (RayTracerNormals.cxx:106-134, RayTracerAlbedo.cxx:106-134)
      f3 ldir = sub(ld3(p.light), pnt);
      ldir = scl(ldir, rmag(ldir));
      float cos_t = dot(n, ldir);
      cos_t = std_min(std_max(cos_t, 0.f), 1.f);
      f3 refl = sub(scl(n, 2.f * dot(ldir, n)), ldir);
      refl = scl(refl, rmag(refl));
      const float cos_p = dot(refl, ld3(p.view_dir));
      if (p.color) {
        const float spec = rtp_glibc::powf(std_max(cos_p, 0.f), 20.f);
        int32_t ci = cvt_i32_x86(p.qscalar[Q.orig] * (float)(p.cmap_n - 1));
        ci = ci > 0 ? ci : 0;
        ci = ci < p.cmap_n - 1 ? ci : p.cmap_n - 1;
        rc_color = ld4(p.cmap + 4 * ci);
        const float k = std_min(0.5f + 0.7f * cos_t + 0.7f * spec, 1.f);
        rc_color.x *= k;
        rc_color.y *= k;
        rc_color.z *= k;
      }
      rc_norm = make_float4(n.x, n.y, n.z, 1.0f);
      rc_alb = make_float4((cos_p * refl.x) / (cos_t * ldir.x), (cos_p * refl.y) / (cos_t * ldir.y),
                           (cos_p * refl.z) / (cos_t * ldir.z), 1.0f);
    }
    // WriteToCanvas depth: 0.5 * (VP * (o + t d)).z / .w + 0.5
    const f3 ip = add(eye, scl(d, dist));
    const float* m = p.vp;
    const float zc = ((m[8] * ip.x + m[9] * ip.y) + m[10] * ip.z) + m[11] * 1.f;
    const float wc = ((m[12] * ip.x + m[13] * ip.y) + m[14] * ip.z) + m[15] * 1.f;
    depth = 0.5f * (zc / wc) + 0.5f;
  }
  if (p.color) reinterpret_cast<float4*>(p.color)[idx] = to_canvas(rc_color, p);
  if (p.normals) reinterpret_cast<float4*>(p.normals)[idx] = to_canvas(rc_norm, p);
  if (p.albedo) reinterpret_cast<float4*>(p.albedo)[idx] = to_canvas(rc_alb, p);
  if (p.depth) p.depth[idx] = depth;
}

// powf restatement evaluated elementwise (tests: device powf vs the host libm)
__global__ void rtp_eval_powf_kernel(const float* __restrict__ x, float y, float* __restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = rtp_glibc::powf(x[i], y);
}

}  // namespace rtp

extern "C" hipError_t rtp_launch_direct(const rtp::DevScene* scene, const rtp::DirectParams* p, hipStream_t stream) {
  if (p->npix <= 0) return hipSuccess;
  const int64_t blocks = (p->npix + 255) / 256;
  hipLaunchKernelGGL(rtp::rtp_render_direct_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, scene, *p);
  return hipGetLastError();
}

extern "C" hipError_t rtp_launch_eval_powf(const float* x, float y, float* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(rtp::rtp_eval_powf_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, y, out, n);
  return hipGetLastError();
}
