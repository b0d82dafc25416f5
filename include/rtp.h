/*
 * rtp.h -- C ABI of the MI355X-native Monte Carlo path tracer (librtp.so).
 *
 * Drop-in boundary for vtkm::rendering::MapperPathTracer
 * (reference MapperPathTracer.h:44-159, MapperPathTracer.cxx:94-406).  Plain
 * pointers and sizes only; no VTK-m, HIP or torch types in the signatures.
 * The reference exposes a C++ class, so the "binding" a maintainer adds is
 * the header-only C++ shim include/rtp/rendering.hpp (same class and method
 * names) -- see INTEGRATION.md.
 *
 * Mapping to the reference:
 *   rtp_create / rtp_destroy      MapperPathTracer ctor/dtor (:94-153); one
 *                                 context per GPU (HIP device ordinal).
 *   rtp_set_scene                 the scene half of the ctor (matIdx, texIdx,
 *                                 matType, texType, tex) + the cell set and
 *                                 coordinates handed to RenderCells
 *                                 (extract/buildBVH, :178-197, :437-449) +
 *                                 the hard-coded light coupling (:141-148,
 *                                 :218, :467).
 *   rtp_render                    SetCanvas + RenderCells (:155-172,
 *                                 :356-383): fills the canvas colour buffer
 *                                 (Vec4f per pixel) with the UN-normalised
 *                                 per-pixel sum over spp samples.
 *   rtp_render_device             same, output already in device memory (the
 *                                 HBM-resident path used by bench.py and the
 *                                 multi-GPU tile shard).
 *   rtp_normalize                 NormalizeFunctor, main.cc:253-287.
 *   rtp_write_pnm                 save(), main.cc:325-384 (P3, buffer order).
 *   rtp_cornell_box               CornellBox::buildDataSet (CornellBox.cpp).
 *
 * Errors: every entry point returns an rtp_status; rtp_last_error() gives a
 * thread-local message (the reference throws vtkm::cont::ErrorBadValue).
 *
 * Concurrency: a context is driven by one host thread at a time (like the
 * reference's mapper).  Its renders are ordered even when they are enqueued
 * on different streams: each launch waits for the context's previous one,
 * because they share the context's scratch (path history, progress counter).
 * rtp_set_scene and rtp_destroy wait for queued renders before replacing or
 * freeing device buffers.  Use one context per stream for concurrent renders.
 */
#ifndef RTP_H
#define RTP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTP_ABI_VERSION 3

typedef enum {
  RTP_OK = 0,
  RTP_ERR_INVALID_ARGUMENT = -1, /* ErrorBadValue in the reference */
  RTP_ERR_NO_SCENE = -2,
  RTP_ERR_DEVICE = -3,           /* HIP runtime failure / no GPU */
  RTP_ERR_OUT_OF_MEMORY = -4,
} rtp_status;

typedef struct rtp_context rtp_context;

/* vtkm::rendering::Camera fields read by pathtracing::Camera::SetParameters
 * (Camera.cxx:624-637).  Zoom and clipping range do not affect the path. */
typedef struct {
  float position[3];
  float look_at[3];
  float view_up[3];
  float fov_y_deg; /* applied to both axes (Camera.cxx:925-931) */
} rtp_camera;

/* Scene in the reference's representation.  quad_points holds, per quad,
 * the QuadExtractor point ids [p0 p1 p2 p3] (= QuadIds[1..4]); the Lagae-
 * Dutre test takes v00=p0, v10=p1, v11=p2, v01=p3 (Surface.h:174). */
typedef struct {
  const float* points; /* float3[n_points] */
  int32_t n_points;
  const int32_t* quad_points; /* int32[4*n_quads] */
  const int32_t* quad_mat;    /* matIdx[0] */
  const int32_t* quad_tex;    /* texIdx[0] */
  int32_t n_quads;
  const int32_t* sphere_point;  /* SphereIds */
  const float* sphere_radius;   /* SphereRadii */
  const int32_t* sphere_mat;    /* matIdx[1] */
  const int32_t* sphere_tex;    /* texIdx[1] */
  int32_t n_spheres;
  const int32_t* mat_type; /* 0 lambertian, 1 diffuse light, 2 dielectric */
  int32_t n_mat;
  const int32_t* tex_type;
  int32_t n_tex_type;
  const float* tex_rgb; /* float3[n_tex] */
  int32_t n_tex;
  int32_t light_quad_points[4]; /* light_box_pointids[1..4] (8,9,10,11) */
  int32_t light_sphere_point;   /* light_sphere_pointids[0] (48); radius = sphere_radius[0] */
  float ior;                    /* DielectricWorklet ref_idx (1.5) */
} rtp_scene_desc;

typedef struct {
  uint64_t samples;      /* pixels * spp */
  uint64_t live_bounces; /* ray-bounces processed while the path was alive */
  uint64_t nan_pixels;   /* pixels whose rgb sum is NaN before normalisation */
  double kernel_ms;      /* device time of the render kernel(s) */
} rtp_stats;

/* optional per-pixel diagnostics (device or host pointers matching the call) */
typedef struct {
  uint32_t* final_seed;   /* RNG state after the last sample (nullable) */
  uint32_t* live_bounces; /* live ray-bounces per pixel (nullable) */
} rtp_pixel_aux;

const char* rtp_last_error(void);
int32_t rtp_abi_version(void);

rtp_status rtp_create(int32_t device, rtp_context** out);
void rtp_destroy(rtp_context* ctx);

rtp_status rtp_set_scene(rtp_context* ctx, const rtp_scene_desc* scene);

/* Full canvas render into host memory (rgba_out: float4[nx*ny]). */
rtp_status rtp_render(rtp_context* ctx, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                      int32_t depth, uint32_t seed_base, float* rgba_out, rtp_stats* stats);

/* rtp_render_device over the 16x16 tiles of a round-robin tile deal: rank
 * `rank` of `world` owns tiles t = rank, rank + world, ... of the canvas in
 * row-major tile order, each tile's pixels row-major (the order of
 * shard.tile_pixels; the multi-GPU sharding of SURVEY.md 8(e)).
 * d_rgba_out: device float4[256 * tiles owned]: entry 256 q + e is pixel
 * (16 tx + e % 16, 16 ty + e / 16) of the rank's q-th tile (tx, ty).  A canvas
 * that is not whole tiles (C4's 1080 rows) has clipped tiles on its right and
 * top edges: their entries outside the canvas are rendered like the others
 * (camera rays past the frame, seeds of no real pixel) and are to be ignored
 * (shard.tile_entries).  Every entry inside the canvas equals
 * rtp_render_device on that pixel, without a pixel list. */
rtp_status rtp_render_tiles_device(rtp_context* ctx, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                                   int32_t depth, uint32_t seed_base, int32_t rank, int32_t world, float* d_rgba_out,
                                   void* hip_stream, rtp_stats* stats);

/* Device-resident render of a pixel set on hip_stream (0 = null stream).
 * Pixels: d_pixel_ids (device int64[pixel_count]) when non-NULL, else the
 * contiguous range [pixel_begin, pixel_begin+pixel_count).  d_rgba_out is a
 * device float4[pixel_count] (entry k <-> k-th pixel of the set).  aux
 * pointers, when non-NULL, are device arrays of pixel_count.  Asynchronous:
 * returns after enqueueing; stats->kernel_ms is only filled when
 * stats != NULL, which synchronises the stream. */
rtp_status rtp_render_device(rtp_context* ctx, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                             int32_t depth, uint32_t seed_base, int64_t pixel_begin, int64_t pixel_count,
                             const int64_t* d_pixel_ids, float* d_rgba_out, const rtp_pixel_aux* aux,
                             void* hip_stream, rtp_stats* stats);

/* rtp_render_device with a wave plan: the launch runs n_waves persistent
 * waves and wave w owns the entries [d_wave_begin[w], d_wave_begin[w+1]) of
 * the pixel set (each range <= 128 entries; d_wave_begin: device
 * int32[n_waves+1], non-decreasing, ending at pixel_count).  Grouping pixels
 * of similar cost into the same wave keeps its lanes busy to the end (a
 * pixel's samples are one sequential chain).  Results are identical to
 * rtp_render_device for any plan.  Scenes without the sphere BVH only.
 * NOT asynchronous like rtp_render_device: the plan is copied to the host and
 * validated before the launch, which waits for the work already queued on
 * hip_stream (an experiment's entry point: a bad plan is an error, not a
 * silently clamped launch). */
rtp_status rtp_render_planned_device(rtp_context* ctx, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                                     int32_t depth, uint32_t seed_base, int64_t pixel_begin, int64_t pixel_count,
                                     const int64_t* d_pixel_ids, const int32_t* d_wave_begin, int32_t n_waves,
                                     float* d_rgba_out, const rtp_pixel_aux* aux, void* hip_stream,
                                     rtp_stats* stats);

/* Host-memory variant of rtp_render_device for an arbitrary pixel list
 * (golden pixel subsets); aux pointers are host arrays. */
rtp_status rtp_render_pixels(rtp_context* ctx, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                             int32_t depth, uint32_t seed_base, const int64_t* pixel_ids, int64_t pixel_count,
                             float* rgba_out, const rtp_pixel_aux* aux, rtp_stats* stats);

/* Host-side helpers of the application layer (main.cc). */
rtp_status rtp_normalize(float* rgba, int64_t n_pixels, int32_t spp);
rtp_status rtp_write_pnm(const char* path, const float* rgba, int32_t nx, int32_t ny);

/* CornellBox::buildDataSet.  variant 0: the reference scene (glass sphere
 * outside the box); 1: sphere at (190,90,190) (notebook cell 2; overlaps the
 * tall box); 2: sphere floating at (440,200,150), clear of the boxes;
 * 3: the C3 stress scene -- the six walls with the light and 1000 spheres
 * (sphere 0: glass at (190,90,190), the light-sphere target; spheres 1..999
 * from the reference's RNG, see oracle/rtp_oracle.h for the exact recipe).
 * The returned descriptor points into library-owned static storage. */
rtp_status rtp_cornell_box(int32_t variant, rtp_scene_desc* out);

/* ------------------------------------------------------------------------
 * -direct mode (main.cc:120-251, 623-651; generate() :386-431): the quad
 * mappers MapperQuad (colour), MapperQuadNormals and MapperQuadAlbedo
 * (MapperQuad*.cxx:86-150) painted by View3D (View3D.cxx:53-64).  One call
 * renders any subset of the three AOVs and the canvas depth buffer with one
 * intersection pass; each output equals the canvas colour buffer of its own
 * reference render (runRay / runNorms / runAlbedo each start from a cleared
 * canvas), and depth equals the canvas depth buffer of any of them.  Only
 * quads are drawn (the mappers use the QuadExtractor alone). */
typedef enum {
  RTP_AOV_COLOR = 1,   /* MapperQuad: RayTracer SurfaceColor (Phong over the colour map) */
  RTP_AOV_NORMALS = 2, /* MapperQuadNormals: RayTracerNormals.cxx:84-141 */
  RTP_AOV_ALBEDO = 4,  /* MapperQuadAlbedo: RayTracerAlbedo.cxx:84-145 */
} rtp_aov;

typedef struct {
  float clip_near, clip_far; /* vtkm::rendering::Camera::SetClippingRange (main.cc:615: 0.1, 5) */
  float background[4];       /* View3D background colour (main.cc:181: 0,0,0,1) */
  int32_t composite_background; /* Mapper::SetCompositeBackground (MapperQuad.cxx:46-49: on) */
  /* per quad, in rtp_scene_desc order: the actor's field at QuadIds[0] (the
   * cell id) normalised over the scalar range -- QuadIntersector::
   * IntersectionData's GetScalar; rtp_quad_scalars computes it */
  const float* quad_scalar;
  /* Mapper::ColorMap: float4[color_map_size] (Mapper::SetActiveColorTable,
   * 1024 samples of the actor's colour table; rtp_sample_color_table) */
  const float* color_map;
  int32_t color_map_size;
} rtp_direct_desc;

/* Host buffers (nullable each, at least one non-NULL): rgba float4[nx*ny] per
 * AOV, depth float[nx*ny].  aovs is informational: an AOV is rendered iff its
 * buffer is non-NULL.  Synchronous. */
rtp_status rtp_render_direct(rtp_context* ctx, const rtp_camera* cam, int32_t nx, int32_t ny,
                             const rtp_direct_desc* desc, float* color_rgba, float* normals_rgba,
                             float* albedo_rgba, float* depth, rtp_stats* stats);
/* Same with device buffers on hip_stream (0 = null stream); asynchronous
 * unless stats != NULL. */
rtp_status rtp_render_direct_device(rtp_context* ctx, const rtp_camera* cam, int32_t nx, int32_t ny,
                                    const rtp_direct_desc* desc, float* d_color_rgba, float* d_normals_rgba,
                                    float* d_albedo_rgba, float* d_depth, void* hip_stream, rtp_stats* stats);

/* Host helpers of the -direct application layer (no device needed). */
/* vtkm::cont::ColorTable(name, RGB, nanColor, rgbPoints, alphaPoints) sampled
 * by Mapper::SetActiveColorTable: n_samples float4 colours (uint8 / 255). */
rtp_status rtp_sample_color_table(const double* rgb_points, int32_t n_rgb, const double* alpha_points,
                                  int32_t n_alpha, const double nan_color[3], int32_t n_samples, float* out_rgba);
/* QuadIntersector GetScalar per quad: (field[quad_cell[q]] - min) * invDelta
 * with min/max over the whole field (Actor::Init's scalar range). */
rtp_status rtp_quad_scalars(const float* field, int32_t n_field, const int32_t* quad_cell, int32_t n_quads,
                            float* out);
/* CornellBox's "point_var" field and the cell id of each quad
 * (CornellBox.cpp:36-60, 163-418; QuadIds[0]); library-owned storage. */
rtp_status rtp_cornell_point_field(int32_t variant, const float** field, int32_t* n_field,
                                   const int32_t** quad_cell, int32_t* n_quads);
/* save() of a Float32 buffer (main.cc:346-359): NaN -> 0, sqrt, int(255.99*c). */
rtp_status rtp_write_pnm_depth(const char* path, const float* depth, int32_t nx, int32_t ny);
/* Diagnostics: the device powf restatement (glibc_powf.hpp) elementwise. */
rtp_status rtp_eval_powf(rtp_context* ctx, const float* x, float y, float* out, int64_t n);

/* ------------------------------------------------------------------------
 * RNG jump tables.  A path that ends before depthcount still draws the
 * reference's random numbers for every remaining depth;
 * the renderer skips them with tables of the dead-depth map over all 2^32
 * RNG states (chain tables for 32/16/8/4 depths, direct tables for the
 * counts depth-50 samples mostly have: 224 GiB of HBM by default, built once
 * per device and process, shared by its contexts).  Results are identical
 * with and without them; they only change speed and setup cost.
 *   RTP_FF_TABLES_AUTO  (default) build them in two stages, each before the
 *                       launch that takes the samples launched on the device
 *                       past its break-even count (setup time / time saved
 *                       per sample): the chain tables (64 GiB) at
 *                       auto_samples, the direct tables at
 *                       auto_samples_direct (once the chain tables exist:
 *                       their sample count + the direct stage's estimated
 *                       setup -- 0.07 s + 2.5x the chain tables' measured
 *                       allocation -- over the time it saves per sample).
 *                       A one-shot render such as main.cc's never pays the
 *                       setup
 *   RTP_FF_TABLES_OFF   hash every dead depth on this context
 *   RTP_FF_TABLES_ON    build now (a long-lived renderer / service)
 * Environment: RTP_FF_POLICY=auto|on|off sets the default of new contexts. */
typedef enum {
  RTP_FF_TABLES_AUTO = 0,
  RTP_FF_TABLES_OFF = 1,
  RTP_FF_TABLES_ON = 2,
} rtp_ff_policy;

typedef struct {
  int32_t policy;         /* this context's rtp_ff_policy */
  int32_t built;          /* 0 none, 1 the chain tables, 2 chain + direct tables */
  int32_t chain_tables;   /* tables for 32, 16, 8, 4, ... dead depths */
  int32_t direct_first;   /* direct tables for counts [direct_first, +direct_count) */
  int32_t direct_count;
  uint64_t bytes;         /* device memory the tables hold */
  double alloc_ms;        /* host time of their allocation (includes the driver's clearing) */
  double build_ms;        /* device time of the build kernel */
  uint64_t samples_seen;  /* samples launched on the device by this process */
  uint64_t auto_samples;  /* the AUTO policy's break-even counts: chain tables, */
  uint64_t auto_samples_direct; /* direct tables (RTP_FF_AUTO_SAMPLES=chain[,direct]) */
} rtp_ff_info;

rtp_status rtp_set_ff_tables(rtp_context* ctx, int32_t policy);
rtp_status rtp_get_ff_tables(rtp_context* ctx, rtp_ff_info* out);

/* Diagnostics: evaluate a device primitive elementwise (tests only).
 * kind 0: glibc-exact sinf port, 1: cosf port, 2: 1/sqrtf(x) (RMagnitude),
 * 3: wang32 (bit pattern in/out), 4 / 5: the RNG jump tables (state after
 * 16 / 32 dead depths; RTP_ERR_DEVICE if they are not built), 6: the state
 * after one dead depth, 7: the first direct table (direct_first depths).
 * in/out: n 4-byte elements, host memory. */
rtp_status rtp_eval_primitive(rtp_context* ctx, int32_t kind, const void* in, void* out, int64_t n);

/* Diagnostics: with RTP_DEBUG_STATS=1 in the environment the render kernel
 * records per-wave counters (bounce steps, live lanes, fast-forward batches,
 * shader-clock cycles per phase); this sums them over waves into out[0..n_out)
 * (out[kDbgCounters], if requested, = the longest wave lifetime) and returns
 * the wave count of the last such launch (0 if none).  n_out < 0: copy the raw
 * per-wave records (waves * kDbgCounters values) instead. */
int32_t rtp_debug_counters(rtp_context* ctx, uint64_t* out, int32_t n_out);

/* Diagnostics: the closest hit of n rays (o, d: 6 floats each, host memory)
 * through the quad prefilter and through the exact scan of every quad.
 * out (host, 7 u32 per ray): prefiltered (t bits, kind, index), exact (t
 * bits, kind, index), 1 if the ray fell back to the exact scan. */
rtp_status rtp_debug_closest_hit(rtp_context* ctx, const float* rays, int64_t n, uint32_t* out);

/* Diagnostics: how the current scene's spheres are searched by a render
 * (rtp_render*, without RTP_DEBUG_STATS or a wave plan): 0 every sphere in
 * order (fewer than 9 spheres), 1 the threaded sphere BVH in global memory,
 * 2 the same walk over each block's LDS copy of a wider-leaved tree (opt-in:
 * RTP_BVH_LDS=1 at rtp_set_scene, and only when its nodes and spheres fit the
 * LDS). */
int32_t rtp_sphere_walk(rtp_context* ctx);

/* Diagnostics: the octant mask of the current scene's global sphere walk (a
 * ray in direction octant o walks the near-to-far copy o & mask; 7: all 8
 * copies, the default for the host SAH and the device LBVH builds alike;
 * RTP_BVH_OCT_MASK narrows it for experiments); -1 without a sphere BVH.  The
 * value is copied back from the device scene the kernels read (-2 if that
 * copy fails, -3 if it disagrees with the context's host mirror). */
int32_t rtp_sphere_walk_oct_mask(rtp_context* ctx);

/* Diagnostics: exhaustively compare a fast device arithmetic sequence with the
 * IEEE operation for every float bit pattern in [lo_bits, hi_bits].  kind 0:
 * rcp (v_rcp + 1 Newton step) vs 1.0f/x; 1: rcp + remainder correction; 2:
 * fast sqrt vs sqrtf; 3/4: 1/sqrt with rcp kind 0/1; 5: (float)(x*(1/pi)) vs
 * (float)(x/pi) in double; 6/7: the branch-free sincos vs the sinf/cosf
 * ports.  *mismatches = count,
 * *first_bad = smallest mismatching bit pattern (0xffffffff if none). */
rtp_status rtp_verify_fast_math(rtp_context* ctx, int32_t kind, uint32_t lo_bits, uint32_t hi_bits,
                                uint64_t* mismatches, uint32_t* first_bad);

#ifdef __cplusplus
}
#endif
#endif /* RTP_H */
