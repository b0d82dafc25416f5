/*
 * rtp_oracle.h -- CPU restatement of m-kim/raytracingtherestofyourlife's
 * Monte Carlo path-tracing loop (MapperPathTracer::RenderCellsImpl).
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (librtp.so, the HIP
 * kernels, the Python package) links, loads or calls this code.  It is used
 * by tests/ (as the parity checker), by __graft_entry__.smoke() (checker) and
 * by bench.py's cpu_baseline leg (timed CPU baseline, kind "port").
 *
 * Parity status: PARITY UNPINNED against the reference itself.  The reference
 * cannot be compiled here (needs VTK-m, absent) and holds no
 * tests, golden images or fixtures for this path, so this restatement is only
 * partially pinned, by (i) known-answer tests
 * probed on this host (RNG, glibc sinf/cosf bit-exactness, g++ argument
 * evaluation order) and (ii) the two internal variants (scalar per-pixel and
 * stage-structured SoA) agreeing bit-for-bit.  VTK-m behaviour that the
 * reference relies on is restated from its published semantics and each
 * assumption is listed in DESIGN.md section "Oracle assumptions".
 */
#ifndef RTP_ORACLE_H
#define RTP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTPO_MAX_POINTS 8192
#define RTPO_MAX_QUADS 2048
#define RTPO_MAX_SPHERES 2048
#define RTPO_MAX_MATS 16

/* Scene in the reference's own representation (CornellBox.cpp:141-418,
 * MapperPathTracer.cxx:141-148, 178-197).  quad_ids rows are the
 * QuadExtractor layout [cellId, p0, p1, p2, p3]. */
typedef struct {
  int32_t n_points;
  float points[RTPO_MAX_POINTS][3];
  int32_t n_quads;
  int32_t quad_ids[RTPO_MAX_QUADS][5];
  int32_t quad_mat[RTPO_MAX_QUADS]; /* matIdx[0] */
  int32_t quad_tex[RTPO_MAX_QUADS]; /* texIdx[0] */
  int32_t n_spheres;
  int32_t sphere_point[RTPO_MAX_SPHERES]; /* SphereIds */
  float sphere_radius[RTPO_MAX_SPHERES];  /* SphereRadii */
  int32_t sphere_mat[RTPO_MAX_SPHERES];   /* matIdx[1] */
  int32_t sphere_tex[RTPO_MAX_SPHERES];   /* texIdx[1] */
  int32_t n_mat;
  int32_t mat_type[RTPO_MAX_MATS];
  int32_t n_tex_type;
  int32_t tex_type[RTPO_MAX_MATS];
  int32_t n_tex;
  float tex[RTPO_MAX_MATS][3];
  int32_t light_box_pointids[5]; /* (0,8,9,10,11) MapperPathTracer.cxx:141 */
  int32_t light_sphere_point;    /* 48, MapperPathTracer.cxx:145 */
  float ior;                     /* 1.5, MapperPathTracer.cxx:467 */
  /* the "point_var" point field (CornellBox.cpp:36-60, 163-418): each cell
   * pushes its cell index once per point it adds (the red wall five times,
   * :189-200), then every value is divided by the value count (:389-390).
   * Read by the -direct mappers only. */
  int32_t n_field;
  float field[RTPO_MAX_POINTS + 16];
} rtpo_scene;

/* Camera constants shared by every RayGen invocation:
 * cam[0..2] eye, [3..5] nlook, [6..8] delta_x, [9..11] delta_y. */
void rtpo_camera_setup(const float pos[3], const float look_at[3], const float up[3], float fov_y_deg,
                       int32_t nx, int32_t ny, float cam[12]);

/* variant 0: reference scene (CornellBox.cpp:141-418, glass sphere at x=-335,
 *            outside the box).
 * variant 1: same, sphere moved to (190,90,190) (notebook cell 2) so the
 *            dielectric path is exercised (it overlaps the tall box: most
 *            pixels NaN-poison, a stress case for the NaN semantics).
 * variant 2: sphere floating at (440,200,150), clear of every box (a clean
 *            visible glass sphere).
 * variant 3: the C3 stress scene (BASELINE.json configs[2], SURVEY.md 8(d);
 *            build-defined because the reference's SphereExtractor breaks for
 *            more than one sphere): the six walls with the light, no boxes,
 *            RTPO_C3_SPHERES spheres.  Sphere 0 is the glass sphere at the
 *            notebook position (190,90,190), radius 90 (the light-sphere target
 *            of the mixture pdf).  Spheres 1.. draw u0..u5 from the reference's
 *            own RNG (getRandF, seed RTPO_C3_SEED) and set, in 555-units and
 *            float arithmetic: r = 8 + 22*u3, centre_k = r + (555 - 2r)*u_k;
 *            a sphere with |centre - (190,90,190)|^2 < (92 + r)^2 is redrawn
 *            (a hit point inside the light sphere makes the reference's
 *            sphere sampler NaN and poisons the pixel); u4 < 0.8: lambertian
 *            matIdx = texIdx = min(2, int(3*u5)), else dielectric (4, 0).
 *            Coordinates are then /555.0 in double. */
#define RTPO_C3_SPHERES 1000
#define RTPO_C3_SEED 3u
void rtpo_cornell_box(int32_t variant, rtpo_scene* out);

/* Scalar per-pixel render of an arbitrary pixel subset (pixels are fully
 * independent because seed[i] = seed_base + i, MapperPathTracer.cxx:265-267).
 * out_rgba[4*k..] receives the un-normalised canvas sum for pixels[k]
 * (alpha := 0); out_seed / out_live (nullable) the final RNG state and the
 * number of live ray-bounces of that pixel.  nthreads <= 0: all cores. */
void rtpo_render_pixels(const rtpo_scene* sc, const float cam[12], int32_t nx, int32_t ny, int32_t spp,
                        int32_t depth, uint32_t seed_base, const int64_t* pixels, int64_t npix,
                        float* out_rgba, uint32_t* out_seed, uint32_t* out_live, int32_t nthreads);

/* Stage-structured SoA render of the full nx*ny canvas: the same per-stage
 * passes over all rays as RenderCellsImpl (no compaction, cost ~ N*S*D).
 * This is the timed CPU baseline.  Must agree bit-for-bit with
 * rtpo_render_pixels.  rows restricts work to image rows [row_begin,row_end)
 * (a bounded sample for timing); pass 0, ny for the whole image. */
int32_t rtpo_render_soa(const rtpo_scene* sc, const float cam[12], int32_t nx, int32_t ny, int32_t spp,
                        int32_t depth, uint32_t seed_base, int32_t row_begin, int32_t row_end,
                        float* out_rgba, uint32_t* out_seed, uint32_t* out_live, int32_t nthreads);

/* ---------------------------------------------------------------------
 * -direct mode (main.cc:120-251, 623-651; generate() :386-431): the
 * MapperQuad / MapperQuadNormals / MapperQuadAlbedo one-bounce renders of
 * the quads (QuadExtractor: the sphere's vertex cell is not drawn).  One call
 * is one View3D::Paint: Canvas::Clear, camera rays of VTK-m's raytracing
 * Camera (PerspectiveRayGen over the FindSubset pixel rectangle), closest hit,
 * QuadIntersector::IntersectionData, the SurfaceX::Shade of the mapper,
 * CanvasRayTracer::WriteToCanvas (depth + blend + clamp), BlendBackground.
 * VTK-m pieces not present in the reference are restated from VTK-m 1.6's
 * published behaviour ("direct mode"): parity unpinned there. */
typedef struct {
  float eye[3], nlook[3], dx[3], dy[3]; /* PerspectiveRayGen (Camera.cxx:339-392) */
  int32_t nx, ny;
  int32_t sub_x0, sub_y0, sub_w, sub_h; /* FindSubset pixel rectangle (Camera.cxx:963-1060) */
  float vp[16];                         /* projection * view, row-major (WriteToCanvas) */
  float light[3];                       /* Position + (2,2,2)*Up (RayTracerNormals.cxx:155-156) */
  float view_dir[3];                    /* Normalize(Position - LookAt) */
} rtpo_direct_cam;

#define RTPO_AOV_COLOR 1
#define RTPO_AOV_NORMALS 2
#define RTPO_AOV_ALBEDO 4

void rtpo_direct_setup(const rtpo_scene* sc, const float pos[3], const float look_at[3], const float up[3],
                       float fov_y_deg, float clip_near, float clip_far, int32_t nx, int32_t ny,
                       rtpo_direct_cam* out);
/* QuadIntersector GetScalar per quad: (field[cellId] - min) * invDelta over
 * the actor's scalar range (min/max of the whole field) */
void rtpo_quad_scalars(const rtpo_scene* sc, float* out);
/* ColorTable(name, RGB, nanColor, rgbPoints, alphaPoints) + Mapper::
 * SetActiveColorTable's Sample(n) into Vec4ui_8 and *(1/255.f) */
int32_t rtpo_sample_color_table(const double* rgb_points, int32_t n_rgb, const double* alpha_points,
                                int32_t n_alpha, const double nan_color[3], int32_t n_samples, float* out_rgba);
/* One mapper render into out_rgba (float4 per pixel) and out_depth
 * (nullable); aov is one RTPO_AOV_* flag. */
void rtpo_render_direct(const rtpo_scene* sc, const rtpo_direct_cam* cam, const float* quad_scalar,
                        const float* cmap, int32_t cmap_n, const float bg[4], int32_t composite, int32_t aov,
                        float* out_rgba, float* out_depth);

/* NormalizeFunctor (main.cc:253-287): de-NaN rgb, then sqrt(x / spp). */
void rtpo_normalize(float* rgba, int64_t n, int32_t spp);

/* primitives, exported for known-answer tests */
uint32_t rtpo_wang32(uint32_t seed);
float rtpo_randf(uint32_t* seed);
float rtpo_sinf(float x);
float rtpo_cosf(float x);
int32_t rtpo_which(uint32_t hash_value);
int64_t rtpo_check_sincos_vs_libm(float lo, float hi, uint32_t stride, int64_t* checked);

#ifdef __cplusplus
}
#endif
#endif
