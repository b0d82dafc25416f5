// rtp_layout.hpp -- device-resident scene and launch-parameter layout shared by
// the host (rtp_host.cpp) and the HIP kernels (rtp_kernels.hip).
//
// Everything here is RAY-INDEPENDENT data precomputed once on the host with
// the same float operations the reference performs per ray (edge vectors,
// normalised quad normals, light-quad area, r*r ...), so the per-ray
// arithmetic in the kernel is bit-identical to the reference's.
#pragma once
#include <stdint.h>

namespace rtp {

constexpr int kMaxQuads = 256;
constexpr int kMaxSpheres = 256;

// One quad of the Lagae-Dutre test (Surface.h:31-161) with v00=q, v10=r,
// v11=s, v01=t.  128 B, read with uniform (scalar) loads.
struct alignas(16) DevQuad {
  float v00[3], e01[3], e03[3];  // e01 = v10-v00, e03 = v01-v00
  float v11[3], e21[3], e23[3];  // e21 = v10-v11, e23 = v01-v11
  float n[3];                    // Normalize(TriangleNormal(q,r,s)), unflipped
  float alb[3];                  // tex[texType[texIdx]]
  int32_t mt;                    // matType[matIdx]
  int32_t pad[7];
};

struct alignas(16) DevSphere {
  float c[3];
  float r;
  float rr;  // radius*radius (Surface.h:328)
  float alb[3];
  int32_t mt;
  int32_t pad[7];
};

struct alignas(16) DevLights {
  DevQuad quad;   // light quad for QuadPDFWorklet (PdfWorklet.h:230-248)
  float area;     // Magnitude(r-q) * Magnitude(t-q)
  float gx0, gdx; // QuadWorkletGenerateDir: x0, x1-x0  (PdfWorklet.h:125-134)
  float gy0, gdy; //                          y0, y1-y0 (= 0)
  float gz0, gdz; //                          z0, z1-z0
  float sc[3];    // light sphere centre / radius (PdfWorklet.h:205-210, 392-396)
  float sr, srr;
  int32_t pad[2];
};

struct alignas(16) DevScene {
  int32_t n_quads;
  int32_t n_spheres;
  uint32_t which_t1;  // smallest hash with which >= 2   (PdfWorklet.h:20)
  uint32_t which_t2;  // smallest hash with which == 3
  float ior;
  int32_t pad[3];
  DevLights light;
  DevQuad quads[kMaxQuads];
  DevSphere spheres[kMaxSpheres];
};

// camera constants (Camera.cxx:437-474): eye, nlook, delta_x, delta_y
struct DevCamera {
  float eye[3], nlook[3], dx[3], dy[3];
};

struct KParams {
  const DevScene* scene;
  DevCamera cam;
  int32_t nx, ny, spp, depth;
  uint32_t seed_base;
  int64_t pixel_begin;
  const int64_t* pixel_ids;  // nullable
  int64_t npix;
  float* out;                // float4[npix]
  uint32_t* seed_out;        // nullable
  uint32_t* live_out;        // nullable
  float* hist;               // float4[(depth-1) * npix] attenuation history
};

}  // namespace rtp
