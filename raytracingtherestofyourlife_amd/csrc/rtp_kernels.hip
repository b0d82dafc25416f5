// rtp_kernels.hip -- CDNA4 (gfx950) kernels of the path-tracing hot path.
//
// rtp_render_pixels_kernel: one lane per pixel, the lane runs the pixel's
// whole sample x depth loop (MapperPathTracer.cxx:278-354) with the fused
// per-depth stage sequence of SURVEY.md 3.2.  Scene and light data are read
// with wave-uniform (scalar) loads; the only per-lane memory traffic is the
// attenuation history (needed for the reference's back-to-front radiance
// product, MapperPathTracer.cxx:328-348), kept depth-major [d][pixel] exactly
// like the reference's ChannelBuffers so a wave's stores are coalesced.
#include <hip/hip_runtime.h>

#include "rtp_device.hpp"

namespace rtp {

// Closest hit over every quad (index order, strict '<') then every sphere
// with tmax from the quads: the closest-hit semantics of
// BVHTraverser.h:128-227 over Surface.h:208-254 / 376-409.
struct Hit {
  float t;
  int kind;  // -1 none, 0 quad, 1 sphere
  int idx;
};

RTP_DEV Hit closest_hit(const DevScene* __restrict__ sc, f3 o, f3 d) {
  Hit h{3.40282347e+38f, -1, 0};
  const float tmin = 0.001f;
  const int nq = sc->n_quads;
  for (int q = 0; q < nq; q++) {
    float t;
    if (quad_hit(sc->quads[q], o, d, t) && t < h.t && t > tmin) {
      h.t = t;
      h.kind = 0;
      h.idx = q;
    }
  }
  const int ns = sc->n_spheres;
  for (int k = 0; k < ns; k++) {
    const DevSphere& S = sc->spheres[k];
    float t;
    if (sphere_hit(o, d, tmin, h.t, ld3(S.c), S.rr, t)) {
      h.t = t;
      h.kind = 1;
      h.idx = k;
    }
  }
  return h;
}

__global__ void __launch_bounds__(256) rtp_render_pixels_kernel(KParams p) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.npix) return;
  const DevScene* __restrict__ sc = p.scene;
  const int64_t pix = p.pixel_ids ? p.pixel_ids[k] : p.pixel_begin + k;
  const uint32_t t1 = sc->which_t1, t2 = sc->which_t2;
  const float ior = sc->ior;
  const DevLights& L = sc->light;

  uint32_t seed = p.seed_base + (uint32_t)pix;  // seeds[i] = i (MapperPathTracer.cxx:265-267)
  float cr = 0.f, cg = 0.f, cb = 0.f;
  uint32_t live = 0;
  const int pi = (int32_t)pix % p.nx, pj = (int32_t)pix / p.nx;
  const f3 eye = ld3(p.cam.eye), nlook = ld3(p.cam.nlook), cdx = ld3(p.cam.dx), cdy = ld3(p.cam.dy);
  float4* __restrict__ hist = reinterpret_cast<float4*>(p.hist) + k;
  const int64_t hstride = p.npix;
  const int D = p.depth;

  for (int s = 0; s < p.spp; s++) {
    // Camera::RayGen (Camera.cxx:482-524)
    f3 dir;
    {
      float ru = randf(seed);
      float rv = randf(seed);
      f3 rd = add(add(nlook, scl(cdx, ((2.f * ((float)pi + (1.f - ru)) - (float)p.nx) / 2.0f))),
                  scl(cdy, ((2.f * ((float)pj + rv) - (float)p.ny) / 2.0f)));
      if (rd.x == 0.f) rd.x += 0.0000001f;
      if (rd.y == 0.f) rd.y += 0.0000001f;
      if (rd.z == 0.f) rd.z += 0.0000001f;
      float sq_mag = __builtin_sqrtf(dot(rd, rd));
      dir = mk(rd.x / sq_mag, rd.y / sq_mag, rd.z / sq_mag);
    }
    f3 org = eye;
    bool alive = true;
    int klight = -1;
    f3 emit = mk(0.f, 0.f, 0.f);
    bool nonfinite = false;

    for (int d = 0; d < D; d++) {
      if (!alive) {
        seed = dead_step(seed, t1, t2);
        continue;
      }
      live++;
      // intersect + CollectIntersecttWorklet (SurfaceWorklets.h:104-109)
      Hit h = closest_hit(sc, org, dir);
      if (h.kind < 0) {
        alive = false;
        seed = dead_step(seed, t1, t2);
        continue;
      }
      f3 hp = add(org, scl(dir, h.t));
      f3 hn;
      int mt;
      f3 alb;
      if (h.kind == 0) {
        const DevQuad& Q = sc->quads[h.idx];
        hn = ld3(Q.n);
        if (dot(hn, dir) > 0.f) hn = neg(hn);  // Surface.h:184-185
        mt = Q.mt;
        alb = ld3(Q.alb);
      } else {
        const DevSphere& S = sc->spheres[h.idx];
        hn = mk((hp.x - S.c[0]) / S.r, (hp.y - S.c[1]) / S.r, (hp.z - S.c[2]) / S.r);
        mt = S.mt;
        alb = ld3(S.alb);
      }
      // applyMaterials (EmitWorklet.h)
      if (mt == 1) {  // DiffuseLightWorklet: emit, path ends (status &= 0)
        emit = (dot(hn, dir) < 0.0f) ? alb : mk(0.f, 0.f, 0.f);
        klight = d;
        alive = false;
        seed = dead_step(seed, t1, t2);  // the dead ray still draws which + generator
        continue;
      }
      f3 atten;
      if (mt == 2) {  // DielectricWorklet: 1 draw before generation, specular
        float r = randf(seed);
        f3 sd;
        dielectric_scatter(dir, hn, ior, r, sd);
        // generation + discarded sphere-pdf draw only advance the stream
        seed = dead_step(seed, t1, t2);
        (void)randf(seed);
        atten = mk(1.f, 1.f, 1.f);
        org = hp;
        dir = sd;
      } else {  // LambertianWorklet
        // generateRays: which + generator (PdfWorklet.h:19-213)
        f3 gen;
        uint32_t tw = wang(seed);
        seed = tw;
        if (tw < t1) {  // cosine
          float r1 = randf(seed);
          float r2 = randf(seed);
          Onb uvw = build_from_w(hn);
          gen = de_nan(local(uvw, random_cosine_direction(r1, r2)));
        } else if (tw < t2) {  // light quad
          float r1 = randf(seed);
          float r2 = randf(seed);
          float r3 = randf(seed);
          f3 rp = mk(L.gx0 + r1 * L.gdx, L.gy0 + r2 * L.gdy, L.gz0 + r3 * L.gdz);
          gen = sub(rp, hp);
        } else {  // light sphere; g++ evaluates the two draws right to left
          float first = randf(seed);
          float second = randf(seed);
          f3 c = ld3(L.sc);
          f3 direction = sub(c, hp);
          float dist2 = dot(direction, direction);
          Onb uvw = build_from_w(direction);
          gen = de_nan(local(uvw, random_to_sphere(L.srr, dist2, second, first)));
        }
        // applyPDFs: QuadPDFWorklet, SpherePDFWorklet (1 discarded draw)
        const float weight = 0.5f;
        float sum = 0;
        sum += weight * quad_pdf_value(L, hp, gen);
        (void)randf(seed);
        sum += weight * sphere_pdf_value(L, hp, gen);
        // PDFCosineWorklet (ScatterWorklet.h:96-112), mixture in double
        Onb uvw = build_from_w(hn);
        float cv;
        {
          float cosine = dot(unit_vector(gen), uvw.w);
          cv = (cosine > 0) ? (float)(cosine / kPi) : 0.f;
        }
        double pdf_val = 0.5 * (double)sum + 0.5 * (double)cv;
        float sp;
        {
          float cosine = dot(hn, unit_vector(gen));
          sp = (cosine < 0) ? 0.f : (float)(cosine / kPi);
        }
        double sctr = (double)sp / pdf_val;
        atten = mk((float)(alb.x * sctr), (float)(alb.y * sctr), (float)(alb.z * sctr));
        org = hp;
        dir = gen;
      }
      if (d <= D - 2) {
        hist[(int64_t)d * hstride] = make_float4(atten.x, atten.y, atten.z, 0.f);
        nonfinite |= !(__builtin_isfinite(atten.x) && __builtin_isfinite(atten.y) && __builtin_isfinite(atten.z));
      }
    }
    // backward radiance (MapperPathTracer.cxx:328-348): s = E[D-1]+0, then
    // s = A[d]*s; s = E[d]+s.  Dead depths contribute A=1, E=0 exactly.
    float sx, sy, sz;
    if (klight >= 0) {
      sx = emit.x + 0.0f;
      sy = emit.y + 0.0f;
      sz = emit.z + 0.0f;
      for (int d = klight - 1; d >= 0; d--) {
        float4 a = hist[(int64_t)d * hstride];
        sx = a.x * sx;
        sy = a.y * sy;
        sz = a.z * sz;
        sx = 0.0f + sx;
        sy = 0.0f + sy;
        sz = 0.0f + sz;
      }
    } else {
      const float v = nonfinite ? __builtin_nanf("") : 0.0f;
      sx = sy = sz = v;
    }
    cr = cr + sx;
    cg = cg + sy;
    cb = cb + sz;
  }
  reinterpret_cast<float4*>(p.out)[k] = make_float4(cr, cg, cb, 0.f);
  if (p.seed_out) p.seed_out[k] = seed;
  if (p.live_out) p.live_out[k] = live;
}

// ------------------------------------------------------- diagnostics ---
__global__ void rtp_eval_primitive_kernel(int kind, const void* in, void* out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* fi = static_cast<const float*>(in);
  const uint32_t* ui = static_cast<const uint32_t*>(in);
  float* fo = static_cast<float*>(out);
  uint32_t* uo = static_cast<uint32_t*>(out);
  switch (kind) {
    case 0: fo[i] = rtp_sinf(fi[i]); break;
    case 1: fo[i] = rtp_cosf(fi[i]); break;
    case 2: fo[i] = 1.0f / __builtin_sqrtf(fi[i]); break;
    case 3: uo[i] = wang(ui[i]); break;
    default: break;
  }
}

}  // namespace rtp

// ----------------------------------------------------------- launchers ---
extern "C" hipError_t rtp_launch_render(const rtp::KParams* p, hipStream_t stream) {
  const int block = 256;
  const int64_t grid = (p->npix + block - 1) / block;
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(rtp::rtp_render_pixels_kernel, dim3((unsigned)grid), dim3(block), 0, stream, *p);
  return hipGetLastError();
}

extern "C" hipError_t rtp_launch_eval_primitive(int kind, const void* in, void* out, int64_t n, hipStream_t stream) {
  const int block = 256;
  const int64_t grid = (n + block - 1) / block;
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(rtp::rtp_eval_primitive_kernel, dim3((unsigned)grid), dim3(block), 0, stream, kind, in, out, n);
  return hipGetLastError();
}
