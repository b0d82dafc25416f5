// rtp_layout.hpp -- device-resident scene and launch-parameter layout shared by
// the host (rtp_host.cpp) and the HIP kernels (rtp_kernels.hip).
//
// Everything here is RAY-INDEPENDENT data precomputed once on the host with
// the same float operations the reference performs per ray (edge vectors,
// normalised quad normals, light-quad area, r*r ...), so the per-ray
// arithmetic in the kernel is bit-identical to the reference's.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace rtp {

constexpr int kMaxQuads = 256;
constexpr int kMaxDepth = 16383;    // remaining dead depths fit the 14-bit field of the pool's slots (kRemMask)
constexpr int kMaxSpp = 8388607;    // 256 slots * spp fits the pool's 32-bit sample cursors (kSteal: see pool_body)
constexpr int kPoolSlots = 128;  // pixel slots per persistent wave of the pool kernel (a planned wave's range bound)
constexpr int kMaxSpheres = 256;          // held inline in DevScene (scalar loads)
constexpr int kMaxSpheresBvh = 1 << 22;   // spheres behind the BVH (global memory)
constexpr int kBvhMinSpheres = 9;         // scenes with more spheres use the BVH
constexpr int kBvhGpuMinSpheres = 262144;  // from this size the BVH is built on the device (rtp_bvh_gpu.hip)
#ifndef RTP_BVH_LEAF
#define RTP_BVH_LEAF 1  // measured best on C3: 1 < 2 < 4 < 7 (367 / 407 / 469 / 564 ms at 16 spp)
#endif
constexpr int kBvhLeafSize = RTP_BVH_LEAF;  // leaf size bound (<= 7: 3-bit count field)

// Zero-structure kinds of quads: the masks of the nonzero components of the
// edge vectors (e01, e03, e21, e23).  A kind's test (quad_hit_masked) drops
// every product with a structurally zero component at compile time; the host
// assigns the kind from exact zeros.  Kind 0 is the general quad; 1..6 are
// axis-aligned rectangles (e01 along I, e03 along J); 7..9 are the faces of
// boxes rotated about y (edges in the xz-plane or along y); 10 is a quad with
// general first-triangle edges and a flat second triangle.
constexpr int kQuadKinds = 11;
struct QuadKindMasks {
  int m01, m03, m21, m23;
};
constexpr QuadKindMasks kQuadKind[kQuadKinds] = {
    {7, 7, 7, 7},                                                               // 0 general
    {1, 2, 2, 1}, {1, 4, 4, 1}, {2, 1, 1, 2}, {2, 4, 4, 2}, {4, 1, 1, 4}, {4, 2, 2, 4},  // 1..6 axis-aligned
    {5, 2, 2, 5}, {2, 5, 5, 2}, {5, 5, 5, 5},                                  // 7..9 rotated about y
    {7, 7, 5, 5}};  // 10: the small box's top (CornellBox.cpp's y=333 vertex): only e21/e23 are flat

// One quad of the Lagae-Dutre test (Surface.h:31-161) with v00=q, v10=r,
// v11=s, v01=t.  Read with uniform (scalar) loads.  The first 64 bytes are
// everything the closest-hit scan of an exact parallelogram reads (QuadGeom):
// the scan fetches them as one s_load_dwordx16, the next quad's while it
// tests the current one.
struct alignas(16) DevQuad {
  float vv[3][2];                // (v00[k], v11[k]) interleaved: one SGPR pair per axis for packed math
  float e01[3], e03[3];          // e01 = v10-v00, e03 = v01-v00
  uint32_t key_lo;               // orig << 8 | scan position: low word of the (t, orig) hit key
  int32_t para;                  // e23 == -e01 and e21 == -e03 bit for bit (exact parallelogram)
  int32_t orig;                  // index in the reference's quad order (tie-break of equal t)
  int32_t kind;                  // index into kQuadKind
  float e21[3], e23[3];          // e21 = v10-v11, e23 = v01-v11
  float n[3];                    // Normalize(TriangleNormal(q,r,s)), unflipped
  float alb[3];                  // tex[texType[texIdx]]
  int32_t mt;                    // matType[matIdx]
  int32_t pad[3];
};
// The scan-time head of a DevQuad (same field offsets).
struct alignas(16) QuadGeom {
  float vv[3][2];
  float e01[3], e03[3];
  uint32_t key_lo;
  int32_t para;
  int32_t orig;
  int32_t kind;
};
static_assert(sizeof(DevQuad) == 128 && sizeof(QuadGeom) == 64 && offsetof(DevQuad, e21) == 64,
              "DevQuad: 64-byte scan head + 64-byte tail");
static_assert(offsetof(DevQuad, key_lo) == offsetof(QuadGeom, key_lo) &&
                  offsetof(DevQuad, para) == offsetof(QuadGeom, para) &&
                  offsetof(DevQuad, e03) == offsetof(QuadGeom, e03),
              "QuadGeom mirrors the head of DevQuad");

struct alignas(16) DevSphere {
  float c[3];
  float r;
  float rr;  // radius*radius (Surface.h:328)
  float alb[3];
  int32_t mt;
  int32_t pad[7];
};

// Sphere record in BVH leaf order (global memory, per-lane loads).
struct alignas(16) DevSphereG {
  float c[3];
  float rr;      // radius*radius
  int32_t orig;  // index in the scene's sphere order (tie-break, material lookup)
  int32_t pad[3];
};

static_assert(sizeof(DevSphereG) == 32 && offsetof(DevSphereG, orig) == 16, "spheres_bvh reads DevSphereG as 2 x 16 B");

// Threaded (stackless) BVH node in depth-first order: on a hit of an inner
// node traversal continues at i+1 (its left child); on a miss, or after a
// leaf, at `skip` (the first node after this subtree; n_nodes ends the walk).
// The boxes are padded so that culling is conservative (rtp_host.cpp).
struct alignas(16) BvhNode {
  float lo[3];
  int32_t skip;
  float hi[3];
  int32_t leaf;  // 0: inner; kBvhLeafSphere: one embedded sphere; else (first << 3) | count
};
// leaf value of a one-sphere leaf that holds the sphere itself: lo = centre,
// hi[0] = radius^2, hi[1] = sphere index (int bits)
constexpr int32_t kBvhLeafSphere = -1;
// The walks read a compact copy of the octant arrays (DevScene::cnodes, 16 B
// per node, index for index the BvhNode arrays): one 16-byte gather per node
// visit instead of two.  On C3 the walk's gathers held the texture data
// path 91% busy (TD_TD_BUSY, r03t) while VALU issue sat at 0.49.  Four
// words per node:
//   sphere leaf (BvhNode::leaf == kBvhLeafSphere): x, y, z = the centre's
//     float bits, w = r^2 bits | kCBvhSphereBit.  The walk goes on at i + 1
//     (a leaf's skip); the sphere's scene index is cidx[i], read only for the
//     final hit and for exact t ties.
//   inner node or multi-sphere leaf: x = half2(lo.x, lo.y), y = half2(lo.z,
//     hi.x), z = half2(hi.y, hi.z), each rounded outward (lo down, hi up:
//     the box only grows, so culling stays conservative); w = skip (inner
//     node) or kCBvhLeafBit | (first << 3 | count) (leaf: next is i + 1).
constexpr uint32_t kCBvhSphereBit = 0x80000000u, kCBvhLeafBit = 0x40000000u;
#ifndef RTP_BVH_EMBED
#define RTP_BVH_EMBED 1
#endif

// The same threaded walk out of LDS (rtp_render_pool_lds): a second tree
// over the same spheres with leaves of up to kLdsWalkLeaf spheres (SAH,
// bvh_build), flattened and compacted like the global one (8 octant copies of
// 16-byte nodes), and its spheres in leaf order as (centre, r^2) float4s.
// Each 16-wave block copies both into its LDS; the walk's node and leaf
// gathers are then LDS reads instead of texture-path gathers (on C3 those held
// TD 93% busy per CU, r03y).  Used when the copy fits beside the block's pools
// (rtp_lds_walk_capacity(); C3: 8 x ~460 nodes + 1000 spheres = 74 KB).
// Bigger leaves keep the eight copies small: a leaf costs one box test and
// then its spheres' exact tests (tools/bvh_walk_sim.cpp: per C3 ray 27.5
// visits and 10 sphere tests at leaves <= 6, 36 and 4 at leaves of 1).
#ifndef RTP_LDS_WALK_LEAF
#define RTP_LDS_WALK_LEAF 6
#endif
constexpr int kLdsWalkLeaf = RTP_LDS_WALK_LEAF;
static_assert(kLdsWalkLeaf >= 1 && kLdsWalkLeaf <= 7, "a leaf's count has 3 bits");
constexpr int kLdsBvhWavesPerBlock = 16;

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

// Axis-plane quad of the closest-hit prefilter (kinds 1..6: every vertex
// shares coordinate `axis` bit for bit).  (cb, cc) +- (rb, rc) bounds the
// quad in the two other coordinates (b = axis+1, c = axis+2 mod 3), widened
// outward on the host.  Read with uniform (scalar) loads.
constexpr int kMaxPre = 32;  // prefiltered quads; the key packs the index in 5 bits
struct alignas(16) PreQuad {
  float cb, cc;    // centre along axis+1, axis+2 (adjacent: one SGPR pair for packed math)
  float rb, rc;    // half extents
  float x;         // the plane: coordinate `axis` of every vertex
  int32_t qpos;    // position in DevScene::quads
  int32_t pad[2];
};
static_assert(sizeof(PreQuad) == 32, "the prefilter scan reads a PreQuad as one s_load_dwordx8");

// The same quads for the prefilter's exact test in the plane's own axes:
// e01 = b along axis i, e03 = c along axis j, a the third; s = +1 if
// j == i+1 (mod 3) else -1 (the cross products' sign); the vertex v00 and
// v11 coordinates permuted to (i, a, j).  Exact parallelograms only.
struct alignas(16) PreExact {
  float b, bs, c, cs;  // bs = s*b, cs = s*c
  float vi, va, vj;    // v00
  float wi, wa, wj;    // v11
  int32_t i, s;
  uint32_t key_lo;     // DevQuad::key_lo
  int32_t pad[3];
};

struct alignas(16) DevScene {
  int32_t n_quads;
  int32_t n_spheres;
  // quads are stored grouped by kind in the scan order 1..kQuadKinds-1, 0:
  // group g (g-th in that order) occupies [kind_begin[g], kind_begin[g+1])
  int32_t kind_begin[kQuadKinds + 1];
  uint32_t which_t1;  // smallest hash with which >= 2   (PdfWorklet.h:20)
  uint32_t which_t2;  // smallest hash with which == 3
  float ior;
  int32_t n_nodes;                 // BVH scenes (n_spheres >= kBvhMinSpheres): nodes per octant copy
  int32_t n_lw_nodes;              // LDS walk: nodes per octant copy of lw_nodes (0: no LDS walk)
  // DielectricWorklet constants of ior, with the reference's float/double
  // operations (EmitWorklet.h:153-170): r0 = ((1 - ior) / (1 + ior))^2 of
  // schlick, and ni_over_nt = (float)(1.0 / ior) of a ray entering the glass
  float ior_r0sq, ior_inv;
  const BvhNode* nodes;            // 8 * n_nodes: one threaded copy per ray-direction octant
  const DevSphereG* sph_geom;      // BVH leaf order
  const DevSphere* sph_all;        // scene order (materials of the hit sphere)
  DevLights light;
  DevQuad quads[kMaxQuads];
  DevSphere spheres[kMaxSpheres];
  // closest-hit prefilter over the axis-plane quads (groups 0..5 = kinds 1..6):
  // n_pre == kind_begin[6] when enabled, else 0; pre[] grouped by plane axis,
  // [pre_begin[a], pre_begin[a+1]); pre_scale = max |vertex coordinate| of them
  int32_t n_pre;
  int32_t pre_begin[4];
  float pre_scale;
  int32_t pad2[2];
  PreQuad pre[kMaxPre];
  PreExact prex[kMaxPre];  // by quad position (< n_pre)
  const uint32_t* cnodes;    // 8 * n_nodes compact nodes (4 words each; kCBvhSphereBit above)
  const int32_t* cidx;       // 8 * n_nodes: a sphere leaf's scene index (else -1)
  // the LDS walk's tree (kLdsWalkLeaf): global copies, loaded into each block's LDS
  const uint32_t* lw_nodes;  // 8 * n_lw_nodes compact nodes
  const int32_t* lw_cidx;    // 8 * n_lw_nodes: an embedded sphere's scene index (else -1)
  const float* lw_sph;       // n_lw_sph float4s (centre, r^2) in the leaf order of lw_nodes
  const int32_t* lw_orig;    // n_lw_sph: the scene index of each
  int32_t n_lw_sph;
  // the global walk's copies: a ray in octant o walks copy (o & oct_mask);
  // bits left out of the mask order those axes' splits left child first
  // (fewer distinct copies: a smaller footprint in the texture cache)
  int32_t oct_mask;
  int32_t pad3[2];
};
// The pool kernel's scans prefetch up to two records past the last quad or
// prefilter record; these must stay inside DevScene (values never used).
static_assert(offsetof(DevScene, spheres) == offsetof(DevScene, quads) + sizeof(DevQuad) * kMaxQuads &&
                  sizeof(DevSphere) * kMaxSpheres >= 2 * sizeof(DevQuad),
              "quads[] is followed by at least two quads' worth of DevScene");
static_assert(offsetof(DevScene, prex) == offsetof(DevScene, pre) + sizeof(PreQuad) * kMaxPre &&
                  sizeof(PreExact) * kMaxPre >= 2 * sizeof(PreQuad),
              "pre[] is followed by at least two records' worth of DevScene");

// camera constants (Camera.cxx:437-474): eye, nlook, delta_x, delta_y
struct DevCamera {
  float eye[3], nlook[3], dx[3], dy[3];
};

constexpr int kFfTables = 6;  // jump tables for 32, 16, 8, 4, 2, 1 dead depths (default 4 built)
constexpr int kFfMaxSteps = 64;  // build kernel: tables for 1..63 dead depths
// the fused table build's outputs: t[r] receives the state after r dead
// depths (null: no table for r)
struct FfBuildOut {
  uint32_t* t[kFfMaxSteps];
};

struct KParams {
  DevCamera cam;
  int32_t nx, ny, spp, depth;
  uint32_t seed_base;
  int64_t pixel_begin;
  const int64_t* pixel_ids;  // nullable
  // tile deal (tile_world > 0, pixel_ids null): entry k is pixel (k & 255) of
  // the rank's (k >> 8)-th 16x16 tile, tiles dealt round-robin in row-major
  // order over a canvas of tile_tx tiles per row (shard.tile_pixels' order)
  int32_t tile_tx, tile_world, tile_rank, tile_pad;
  int64_t npix;
  float* out;                // float4[npix]
  uint32_t* seed_out;        // nullable
  uint32_t* live_out;        // nullable
  float* hist;               // float4[(depth-1) * lanes] attenuation history, depth-major
  unsigned long long* dbg;   // nullable: per-wave counters (kDbgCounters each), diagnostics only
  unsigned long long* progress;  // 2 words zeroed before launch: [0] samples finished by all waves (issue-priority
                                 // balancing), [1] entries claimed by work stealing (pool kernel kSteal)
  // RNG jump tables (nullable): ff[j][s] = the state after (32 >> j) dead
  // depths from state s (2^32 entries each, 16 GiB; rtp_host.cpp)
  const uint32_t* ff[kFfTables];
  // direct tables (nullable): ffd[(r - ffd_first) << 32 | s] = the state after
  // r dead depths from s, for r in [ffd_first, ffd_first + ffd_count)
  const uint32_t* ffd;
  int32_t ffd_first, ffd_count;
  // planned launch (nullable): wave w owns entries [wave_begin[w], wave_begin[w+1])
  const int32_t* wave_begin;
};

// -direct mode (main.cc:120-251): one launch renders the requested AOVs of
// the quad mappers (MapperQuad colour, MapperQuadNormals, MapperQuadAlbedo)
// and the canvas depth, one lane per pixel of the canvas.
struct DirectParams {
  float eye[3], nlook[3], dx[3], dy[3];  // PerspectiveRayGen (Camera.cxx:351-392)
  int32_t nx, ny;
  int32_t sub_x0, sub_y0, sub_w, sub_h;  // FindSubset pixel rectangle (Camera.cxx:963-1060)
  float vp[16];                          // projection * view, row-major (WriteToCanvas)
  float light[3];                        // Position + (2,2,2)*Up
  float view_dir[3];                     // Normalize(Position - LookAt)
  float bg[4];                           // background colour (BlendBackground)
  int32_t composite;                     // CompositeBackground
  int32_t cmap_n;                        // colour-map entries
  const float* qscalar;                  // normalised scalar per kept quad (DevQuad::orig order)
  const float* cmap;                     // float4[cmap_n]
  float* color;                          // float4 per pixel (nullable)
  float* normals;                        // float4 per pixel (nullable)
  float* albedo;                         // float4 per pixel (nullable)
  float* depth;                          // float per pixel (nullable)
  int64_t npix;                          // nx * ny
};

// per-wave diagnostic counters of the pool kernel (RTP_DEBUG_STATS=1)
enum DbgCounter {
  kDbgBounceSteps = 0,   // loop iterations that ran a bounce
  kDbgBounceLanes,       // sum over those iterations of lanes with a live path
  kDbgFfPhases,          // fast-forward batches
  kDbgFfLanes,           // sum of batch sizes
  kDbgFfIters,           // sum of per-batch loop trip counts (max remaining depths)
  kDbgCyclesBounce,      // s_memtime cycles spent in bounce steps (incl. refill)
  kDbgCyclesFf,          // s_memtime cycles spent in fast-forward batches
  kDbgCyclesTotal,       // whole wave lifetime
  kDbgCyclesIntersect,   // inside bounce(): closest_hit
  kDbgCyclesShade,       // inside bounce(): material + generate + pdfs + scatter
  kDbgCyclesEnd,         // path end: radiance product + slot update + queue push
  kDbgCyclesRefill,      // refill: READY pop + camera ray
  kDbgRealStart,         // s_memrealtime (100 MHz, chip-wide) at wave start (raw, not summed)
  kDbgRealEnd,           // ... at wave end
  kDbgHwId,              // HW_REG_HW_ID of the wave (SIMD/CU/SE placement)
  kDbgTailSteps,         // bounce steps taken while < 64 of the wave's pixels were unfinished
  kDbgTailLanes,         // live lanes summed over those steps
  kDbgTailCycles,        // s_memtime cycles from the first such step to the wave's end
  kDbgFallbackSteps,     // bounce steps in which some lane ran the exact scan of the prefiltered quads
  kDbgFallbackLanes,     // lanes that did, summed over all bounce steps
  // exec occupancy per region (round 4): how often a region ran in a wave
  // (visits) and the lanes active when it started (sum of popcount(exec))
  kDbgRefillVisits,      // refill with >= 1 lane taking a sample: camera ray
  kDbgRefillLanes,
  kDbgHitVisits,         // shade_hit past the miss test (a surface was hit)
  kDbgHitLanes,
  kDbgGenVisits,         // the Lambertian branch: generator + pdfs + mixture
  kDbgGenLanes,
  kDbgCyclesGen,         //   s_memtime cycles in the generator (which draw .. gen)
  kDbgCyclesPdf,         //   ... in the pdfs, the mixture and the scatter (gen .. atten)
  kDbgEndVisits,         // path-end bookkeeping (a lane's path ended this step)
  kDbgEndLanes,
  kDbgFfRadVisits,       // fast-forward batch: the radiance product (light-hit samples)
  kDbgFfRadLanes,
  kDbgFfRadRows,         //   history rows read, summed over lanes
  kDbgDeadLanes,         // hashed dead depths after the tables: active lanes summed over trips
  kDbgDielVisits,        // the dielectric branch (glass hits)
  kDbgDielLanes,
  kDbgCyclesDiel,        //   s_memtime cycles in it
  kDbgLightVisits,       // light hits (the path ends with an emission)
  kDbgLightLanes,
  kDbgBoxFreeSteps,      // bounce steps in which no live lane's closest hit is an exact-scan quad (the
                         //   rotated box's faces): the most a wave-uniform box reject could skip (r06)
  kDbgBoxLanes,          // live lanes whose closest hit is one, summed over bounce steps
  kDbgCounters
};

}  // namespace rtp
