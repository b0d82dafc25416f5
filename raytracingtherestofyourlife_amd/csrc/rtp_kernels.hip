// rtp_kernels.hip -- CDNA4 (gfx950) kernels of the path-tracing hot path.
//
// Both kernels run the fused per-depth stage sequence of SURVEY.md 3.2 (one
// call of bounce() == one depth of MapperPathTracer.cxx:286-305 for one ray)
// and differ only in how work is mapped to lanes:
//
//  v1  rtp_render_lockstep: one lane per pixel; the lane walks its pixel's
//      samples and depths in order (MapperPathTracer.cxx:278-354).  Lanes of
//      a wave stay on the same depth, so a wave executes a live bounce as long
//      as ANY of its 64 paths is alive -- kept as the simple reference mapping.
//
//  v2  rtp_render_pool (default): persistent waves.  Each wave owns a pool of
//      pixels in LDS (RNG state, colour sum, sample count).  A lane always
//      carries a LIVE path: when its path ends, the lane banks the sample's
//      contribution into the pixel's slot, queues the pixel for the RNG
//      fast-forward of its remaining dead depths, and immediately starts the
//      next sample of a READY pixel.  The fast-forwards (pure integer Wang
//      hashing) run in full-wave batches when the READY queue
//      runs dry.  Per-pixel sample order, draw order and summation order are
//      exactly the reference's; only the interleaving across pixels changes.
//
// Scene and light data are wave-uniform and arrive through a const __restrict__
// kernel argument, so the compiler reads them with scalar loads into SGPRs.
// The only per-lane global memory traffic is the attenuation history needed
// by the reference's back-to-front radiance product (MapperPathTracer.cxx:
// 328-348), stored depth-major [d][lane] like the reference's ChannelBuffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "rtp_device.hpp"

// One compiled path.  The alternatives measured and rejected in rounds 1-2
// (and the RTP_DUP cost-attribution probes behind DESIGN.md 4.1's tables) are
// in git history: `git show c9f7859:raytracingtherestofyourlife_amd/csrc/
// rtp_kernels.hip`.  The numeric scheduling constants below stay tunable.
#ifndef RTP_FF_MARGIN
#define RTP_FF_MARGIN 12  // pool kernel: fast-forward when READY holds fewer than idle lanes + this
#endif
// history rows of a finished sample loaded together in the fast-forward batch
#ifndef RTP_HIST_PREFETCH
#define RTP_HIST_PREFETCH 6
#endif
constexpr int kHistPrefetch = RTP_HIST_PREFETCH;
// and the rest kHistChunk at a time (r03r: 4 rows per wait, -0.4% at N = 1,
// -1.1% at the 1/8 share, against two per wait)
#ifndef RTP_HIST_CHUNK
#define RTP_HIST_CHUNK 4
#endif
constexpr int kHistChunk = RTP_HIST_CHUNK;
#ifndef RTP_WALK_DONE
// pool kernel, sphere-BVH scenes: a loop iteration walks the BVH until this
// many of the wave's paths have finished their walks (or all have)
#define RTP_WALK_DONE 48
#endif
#ifndef RTP_CRIT_FF
#define RTP_CRIT_FF 100  // pool kernel: lag (per mille of the wave's average samples) that makes a pixel critical
#endif

namespace rtp {

typedef uint32_t u16v __attribute__((ext_vector_type(16)));  // 64 bytes: one s_load_dwordx16

struct Hit {
  float t;
  int kind;  // -1 none, 0 quad, 1 sphere
  int idx;
};

// Closest hit over every quad then every sphere with tmax from the quads: the
// closest-hit semantics of BVHTraverser.h:128-227 over Surface.h:208-254 /
// 376-409 with quads visited in index order and a strict '<'.  That scan
// returns the lexicographic minimum of (t, index) over the hits, so the quads
// can be visited grouped by zero-structure kind (one tight loop per kind) as
// long as equal t is broken by the original index.
// The (t, orig) minimum as one unsigned 64-bit key {bits(t), orig << 8 | q}:
// an accepted t is > 0.001, and positive floats order like their bit
// patterns, so key order is exactly "t, then reference index".  The scan
// position q rides in the low bits (orig is unique, so it never decides).
static_assert(kMaxQuads <= 256, "key_lo packs orig and the scan position in 8 bits each");
constexpr uint64_t kNoHitKey = (uint64_t)0x7f7fffffu << 32 | 0xffffffffu;  // {FLT_MAX, none}
// The scan reads the quads' 64-byte scan heads (QuadGeom) as one
// s_load_dwordx16 each, the NEXT quad's issued before the current one is
// tested, so its scalar-load latency hides behind the test's VALU work (the
// field-by-field loads compiled to ~5 dependent s_load / s_waitcnt round
// trips per quad).  The two head registers ping-pong (no copy of the
// prefetched head per quad) and the walk is a pointer (2 SALU per prefetch
// address, not ~7 for a clamped index).  `cur` holds quad b's head on entry
// and quad e's (the next group's first: the groups are contiguous in scan
// order) on exit.
RTP_DEV u16v quad_head(const DevScene* __restrict__ sc, int q) {
  return reinterpret_cast<const u16v*>(sc->quads)[2 * min(q, kMaxQuads - 1)];
}
template <int K>
RTP_DEV void scan_one(const DevQuad& M, const u16v& head, f3 o, f3 d, uint64_t& best) {
  QuadGeom G;
  __builtin_memcpy(&G, &head, sizeof(G));
  float t;
  const bool ok = quad_hit_masked<K>(G, M, o, d, t);
  const uint64_t key = (uint64_t)__float_as_uint(t) << 32 | G.key_lo;
  best = (ok && t > 0.001f && key < best) ? key : best;
}
RTP_DEV u16v head_at(const DevQuad* q) { return *reinterpret_cast<const u16v*>(q); }
template <int K>
RTP_DEV void scan_kind_pf(const DevScene* __restrict__ sc, int b, int e, f3 o, f3 d, uint64_t& best, u16v& cur) {
  // (the prefetches read at most two records past quads[] -- still inside
  // DevScene, whose spheres[] follow -- and those values are never used)
  const DevQuad* qp = sc->quads + b;
  for (int n = e - b; n > 0; n -= 2, qp += 2) {
    const u16v nxt = head_at(qp + 1);
    scan_one<K>(qp[0], cur, o, d, best);
    if (n == 1) {
      cur = nxt;
      break;
    }
    cur = head_at(qp + 2);
    scan_one<K>(qp[1], nxt, o, d, best);
  }
}

// SphereLeafIntersector::hit's accepted root without the tmax test: the
// reference takes r1 = (-b-sq)/a if tmin < r1 < tmax, else r2 = (-b+sq)/a if
// tmin < r2 < tmax.  r1 <= r2 (a > 0), so r1 >= tmax rules out r2 too: the
// accepted root is "r1 if r1 > tmin else r2", accepted iff it is > tmin and
// < tmax.  It does not depend on tmax, so spheres may be visited in any order.
RTP_DEV bool sphere_root(f3 o, f3 d, float tmin, f3 c, float rr, float& t_out) {
  f3 oc = sub(o, c);
  float a = dot(d, d);
  float b = dot(oc, d);
  float cc = dot(oc, oc) - rr;
  float disc = b * b - a * cc;
  if (!(disc > 0)) return false;
  float sq = sqrt_exact(b * b - a * cc);
  float r1 = (-b - sq) / a;
  float t = r1 > tmin ? r1 : (-b + sq) / a;
  t_out = t;
  return t > tmin;
}

// Threaded-BVH walk over the spheres (scenes with >= kBvhMinSpheres).  The
// brute-force scan in index order with a strict '<' returns the
// lexicographic minimum of (t, quads before spheres, sphere index); the walk
// visits spheres in BVH order and keeps that minimum explicitly.  Node boxes
// only cull (padded on the host; compared with slack here), so no sphere
// whose root could win is skipped.  (Loading node i+1 while testing i was
// faster with flat loads and 16% slower with global ones: DESIGN.md 4.1.)
typedef float f4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) f4v GF4;
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u4v GU4;
typedef const __attribute__((address_space(1))) int32_t GI32;
// 1/d per component for the slab tests (tiny components clamped)
RTP_DEV float slab_rcp(float v) { return __builtin_amdgcn_rcpf(fabsf(v) < 1e-20f ? copysignf(1e-20f, v) : v); }
// A ray's view of the sphere BVH: the compact copy of the tree ordered
// near-to-far for its direction octant (rtp_layout.hpp kCBvhSphereBit) and
// that copy's sphere-index table.  (Global, address space 1, pointers: through
// the generic ones loaded from the scene the walk compiled to flat loads.)
// The slab test runs as fma(box, 1/d, -o/d): one rounding of o/d per
// component instead of a rounded (box - o) per face.  The boxes only cull,
// and each sphere lies at least the host's pad inside its boxes on every
// axis (rtp_host.cpp: 0.002 r + 1e-5 + 2^-16 (|c| + r)), so a ray through
// a sphere crosses every box around it over a parameter interval 2 pad / |d|
// wider than the sphere's: far above these roundings (2^-24 |o| / |d|).
struct BvhRay {
  GU4* nodes;
  GI32* cidx;
  GI32* orig;           // LDS walk: the scene index of a leaf-order sphere position (kind 3 hits)
  float ix, iy, iz;     // 1/d (clamped)
  float ox, oy, oz;     // -o/d
};
RTP_DEV int ray_octant(f3 d) { return (d.x < 0.f ? 1 : 0) | (d.y < 0.f ? 2 : 0) | (d.z < 0.f ? 4 : 0); }
// kLds: the LDS walk's tree (its global side tables; the nodes are read from LDS)
template <bool kLds = false>
RTP_DEV BvhRay bvh_ray(const DevScene* __restrict__ sc, f3 o, f3 d) {
  const int oct = ray_octant(d) & (kLds ? 7 : sc->oct_mask);
  const int64_t base = (int64_t)oct * (kLds ? sc->n_lw_nodes : sc->n_nodes);
  BvhRay R;
  R.nodes = (GU4*)((kLds ? sc->lw_nodes : sc->cnodes) + 4 * base);
  R.cidx = (GI32*)((kLds ? sc->lw_cidx : sc->cidx) + base);
  R.orig = (GI32*)sc->lw_orig;
  R.ix = slab_rcp(d.x);
  R.iy = slab_rcp(d.y);
  R.iz = slab_rcp(d.z);
  R.ox = -(o.x * R.ix);
  R.oy = -(o.y * R.iy);
  R.oz = -(o.z * R.iz);
  return R;
}
// During a walk a sphere hit is h.kind == 2 with h.idx the leaf's node (the
// sphere's scene index is cidx[node]), or, in the LDS walk's multi-sphere
// leaves, h.kind == 3 with h.idx the sphere's leaf-order position (scene index
// orig[pos]); bvh_resolve turns either into kind 1 with the scene index.
// Kind 1 hits (the global walk's multi-sphere leaves) carry the index.
RTP_DEV int bvh_hit_index(const Hit& h, const BvhRay& R) {
  return h.kind == 2 ? R.cidx[h.idx] : h.kind == 3 ? R.orig[h.idx] : h.idx;
}
RTP_DEV void bvh_resolve(Hit& h, const BvhRay& R) {
  if (h.kind >= 2) {
    h.idx = bvh_hit_index(h, R);
    h.kind = 1;
  }
}
// the closest-sphere update: the (t, scene index) minimum, quads winning t
// ties; `ref` is the hit's kind-`kind` reference, `orig` reads its scene index
// (only for an exact tie between spheres: rare)
template <class Orig>
RTP_DEV void bvh_accept(Hit& h, float t, int kind, int ref, const BvhRay& R, Orig orig) {
  if (t < h.t) {
    h.t = t;
    h.kind = kind;
    h.idx = ref;
  } else if (t == h.t && h.kind >= 1) {
    if (orig() < bvh_hit_index(h, R)) {
      h.kind = kind;
      h.idx = ref;
    }
  }
}
RTP_DEV float half_lo(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xffffu)); }
RTP_DEV float half_hi(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16)); }
// One node of the walk: node ni (its 16 bytes v) is tested against the ray
// and the best hit so far; returns the next node (>= n_nodes: the walk is
// done).  A sphere leaf runs the exact root test (no box); an inner node's
// box (padded on the host, rounded outward to half precision, compared with
// slack here) only culls.
// kLds: the LDS walk (rtp_render_pool_lds): a multi-sphere leaf's spheres
// are (centre, r^2) float4s in the block's LDS (lsph), else 32-byte
// DevSphereG records in global memory (geom_g).
typedef const __attribute__((address_space(3))) f4v LF4;
typedef const __attribute__((address_space(3))) u4v LU4;
template <bool kLds = false>
RTP_DEV int bvh_visit(GF4* __restrict__ geom_g, LF4* __restrict__ lsph, const BvhRay& R, f3 o, f3 d, u4v v, int ni,
                      Hit& h) {
  if ((int32_t)v.w < 0) {  // a sphere leaf: centre, r^2
    float t;
    if (sphere_root(o, d, 0.001f, mk(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z)),
                    __uint_as_float(v.w & ~kCBvhSphereBit), t))
      bvh_accept(h, t, 2, ni, R, [&] { return R.cidx[ni]; });
    return ni + 1;
  }
  const float x0 = __builtin_fmaf(half_lo(v.x), R.ix, R.ox), x1 = __builtin_fmaf(half_hi(v.y), R.ix, R.ox);
  const float y0 = __builtin_fmaf(half_hi(v.x), R.iy, R.oy), y1 = __builtin_fmaf(half_lo(v.z), R.iy, R.oy);
  const float z0 = __builtin_fmaf(half_lo(v.y), R.iz, R.oz), z1 = __builtin_fmaf(half_hi(v.z), R.iz, R.oz);
  const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
  const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
  const float slack = 1e-5f * fabsf(tf) + 1e-7f;
  const bool hit = tn <= tf + slack && tf >= 0.0f && tn <= h.t * 1.00001f + 1e-7f;
  const bool leaf = (v.w & kCBvhLeafBit) != 0;
  if (hit && leaf) {  // a multi-sphere leaf: its spheres in leaf order
    const int first = (int)((v.w & ~kCBvhLeafBit) >> 3), cnt = (int)(v.w & 7u);
    for (int j = first; j < first + cnt; j++) {
      float t;
      if constexpr (kLds) {
        const f4v g0 = lsph[j];  // c, rr
        if (sphere_root(o, d, 0.001f, mk(g0.x, g0.y, g0.z), g0.w, t)) bvh_accept(h, t, 3, j, R, [&] { return R.orig[j]; });
      } else {
        const f4v g0 = geom_g[2 * j], g1 = geom_g[2 * j + 1];  // c, rr | orig
        if (sphere_root(o, d, 0.001f, mk(g0.x, g0.y, g0.z), g0.w, t))
          bvh_accept(h, t, 1, __float_as_int(g1.x), R, [&] { return __float_as_int(g1.x); });
      }
    }
  }
  return (hit || leaf) ? ni + 1 : (int)v.w;
}
// Threaded-BVH walk over the spheres (scenes with >= kBvhMinSpheres).  The
// brute-force scan in index order with a strict '<' returns the
// lexicographic minimum of (t, quads before spheres, sphere index); the walk
// visits spheres in BVH order and keeps that minimum explicitly, so no
// sphere whose root could win is skipped and the order does not matter.
RTP_DEV void spheres_bvh(const DevScene* __restrict__ sc, f3 o, f3 d, Hit& h) {
  const BvhRay R = bvh_ray(sc, o, d);
  const int nn = sc->n_nodes;
  GF4* __restrict__ geom_g = (GF4*)sc->sph_geom;  // DevSphereG: 2 x 16 B
  int ni = 0;
  u4v v = R.nodes[0];
  while (ni < nn) {
    const int next = bvh_visit(geom_g, nullptr, R, o, d, v, ni, h);
    if (next < nn) v = R.nodes[next];
    ni = next;
  }
  bvh_resolve(h, R);
}

// qshade: the block's LDS copy of the quads' shading data (n, alb, mt) so
// the hit's material is an LDS gather instead of a global one.
// Every quad of a scene (kMaxQuads, 8 KiB): with a table that could be
// absent, the compiler merged the LDS and global reads of the hit's record
// into 7 flat loads (waited on both counters); now they are 2 ds_read_b128.
constexpr int kLdsQuads = kMaxQuads, kQShadeFloats = 8;  // per quad: n, alb, mt, pad
// The block's LDS table also holds the prefilter's PreExact records (after
// the shading data): the candidate's record is then 4 ds_read_b128 instead of
// 4 global loads (L2 hits) on every bounce's critical path (C2 kernel -1.7%,
// r03c; an LDS copy of the quads in round 1 had been slower).
constexpr int kPrexLdsOffset = kLdsQuads * kQShadeFloats;
constexpr int kQTableFloats = kPrexLdsOffset + kMaxPre * 16;

RTP_DEV void fill_qshade(const DevScene* __restrict__ sc, float* s_qshade) {
  for (int i = threadIdx.x; i < sc->n_quads * kQShadeFloats; i += blockDim.x) {
    const DevQuad& Q = sc->quads[i / kQShadeFloats];
    const int f = i % kQShadeFloats;
    s_qshade[i] = f < 3 ? Q.n[f] : f < 6 ? Q.alb[f - 3] : f == 6 ? __int_as_float(Q.mt) : 0.f;
  }
  const float* px = reinterpret_cast<const float*>(sc->prex);
  for (int i = threadIdx.x; i < sc->n_pre * 16; i += blockDim.x) s_qshade[kPrexLdsOffset + i] = px[i];
}

// Closest-hit prefilter over the axis-plane quads (kinds 1..6).
// The exact Lagae-Dutre test costs ~40 VALU per quad and every quad meets
// some lane of a wave, so the scan paid it for all of them.  The prefilter
// instead takes, per quad, the ray's parameter at the quad's plane and the
// hit point's distance outside the quad's box, both in a few ops, with an
// error margin m >= the difference between these approximations and the
// exact test's own roundings:
//   m = 2^-18 * (|t| * max(max|d|, 1) + max|o| + scene scale + 1),
// about six times the worst case of either computation (a handful of
// roundings each of |t*d|, |o| and the vertex coordinates).
// A quad the exact test accepts (0.001 < t, inside) is therefore a
// candidate, and t - m is a lower bound of its exact t.  Each lane keeps its
// two smallest lower bounds, runs the exact test on the first (quad_hit_axis
// on the quad's PreExact record, a per-lane load from the small global prex
// table: the kind's own parallelogram arithmetic in the quad's axes, bit-equal
// to it), and is done when the second lower bound exceeds the best exact hit:
// every other candidate's exact t is larger, so it loses whatever its index.
// Otherwise -- near an edge, a near tie, no finite ray, coordinates beyond
// kPreLim -- the lane runs the exact scan of every axis-plane quad, as
// without the prefilter.  (The host disables the prefilter for scenes it
// does not cover, and with RTP_PREFILTER=0: DevScene::n_pre == 0.)
constexpr float kPreTmin = 0.0005f;  // candidates: approximate t above this (accepted hits: t > 0.001)
constexpr float kPreLimD = 16.0f;    // larger |o| or |d| components: exact scan (margin bound below tmin)
constexpr float kPreK = 0x1p-18f;    // margin factor, 64 units of 2^-24
template <int A>
RTP_DEV float comp(f3 v) {
  if constexpr (A == 0) return v.x;
  else if constexpr (A == 1) return v.y;
  else return v.z;
}
// k1 <= k2: the two smallest candidate keys {bits(t - m) & ~31, quad position}
// (positive floats order like their bit patterns; rounding the low bits
// down keeps the lower bound).  No candidate: ~0u.
// Each PreQuad is one s_load_dwordx8, the next one's issued before the
// current one is tested (as scan_kind_pf); `cur` carries quad b's record in
// and quad e's (the next axis group's first) out.  v_and_or_b32 / v_med3_u32
// are inline asm: the compiler emits 2 + 2 ops for them, which left the
// prefilter at break-even.
typedef uint32_t u8v __attribute__((ext_vector_type(8)));
RTP_DEV u8v pre_rec(const DevScene* __restrict__ sc, int i) {
  return reinterpret_cast<const u8v*>(sc->pre)[min(i, kMaxPre - 1)];
}
template <int A>
RTP_DEV void pre_axis(const DevScene* __restrict__ sc, int b, int e, f3 o, f3 d, float ma, float mb, uint32_t& k1,
                      uint32_t& k2, u8v& cur) {
  constexpr int B = (A + 1) % 3, C = (A + 2) % 3;
  if (b == e) return;
  const float inv = __builtin_amdgcn_rcpf(comp<A>(d));
  const float oa = comp<A>(o);
  const f2v obc = f2v{comp<B>(o), comp<C>(o)}, dbc = f2v{comp<B>(d), comp<C>(d)};
  // the candidate key of one quad (~0u: not a candidate)
  auto key_of = [&](const PreQuad& P) -> uint32_t {
    const float t = (P.x - oa) * inv;
    // the two in-plane coordinates as one packed FMA and one packed subtract
    const f2v u = __builtin_elementwise_fma(f2v{t, t}, dbc, obc) - f2v{P.cb, P.cc};
    const float ub = fabsf(u.x) - P.rb, uc = fabsf(u.y) - P.rc;
    const float m = __builtin_fmaf(fabsf(t), ma, mb);
    // t = +-inf (d[A] ~ 0) gives NaN or inf here and at worst a key above
    // every finite one; the exact test rejects such a quad (|det| < eps)
    const bool ok = (fmaxf(ub, uc) <= m) & (t > kPreTmin);
    uint32_t key;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(key) : "v"(__float_as_uint(t - m)), "v"(~31u), "s"((uint32_t)P.qpos));
    return ok ? key : ~0u;
  };
  auto fold = [&](uint32_t key) {  // keep the two smallest keys
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(k2) : "v"(k1), "v"(k2), "v"(key));
    k1 = min(k1, key);
  };
  // ping-pong heads, pointer walk (as scan_kind_pf; prefetches past pre[]
  // stay inside DevScene: prex[] follows)
  auto as_pre = [](const u8v& v) {
    PreQuad P;
    __builtin_memcpy(&P, &v, sizeof(P));
    return P;
  };
  const PreQuad* pq = sc->pre + b;
  for (int n = e - b; n > 0; n -= 2, pq += 2) {
    const u8v nxt = *reinterpret_cast<const u8v*>(pq + 1);
    fold(key_of(as_pre(cur)));
    if (n == 1) {
      cur = nxt;
      break;
    }
    cur = *reinterpret_cast<const u8v*>(pq + 2);
    fold(key_of(as_pre(nxt)));
  }
}

// quad_hit_masked<K>'s parallelogram path for an axis-plane quad of any of
// the kinds 1..6, the kind chosen per lane: the same products, sums and
// signs (derived in DESIGN.md 4.1), on o and d permuted into the quad's axes.
RTP_DEV bool quad_hit_axis(const PreExact& E, f3 o, f3 d, float& t_out) {
  const bool x0 = E.i == 0, x1 = E.i == 1, pos = E.s > 0;
  auto perm = [&](f3 v, float& vi, float& va, float& vj) {
    const float r0 = x0 ? v.x : (x1 ? v.y : v.z);
    const float r1 = x0 ? v.y : (x1 ? v.z : v.x);
    const float r2 = x0 ? v.z : (x1 ? v.x : v.y);
    vi = r0;
    vj = pos ? r1 : r2;
    va = pos ? r2 : r1;
  };
  float oi, oa, oj, di, da, dj;
  perm(o, oi, oa, oj);
  perm(d, di, da, dj);
  const float Pa = di * E.cs;     // s * d_i c
  const float Pi = -(da * E.cs);  // -s * d_a c
  const float det = E.b * Pi;
  const float inv_det = rcp_det(det);
  const f2v Ta = f2v{oa, oa} - f2v{E.va, E.wa};
  const f2v Ti = f2v{oi, oi} - f2v{E.vi, E.wi};
  const f2v Tj = f2v{oj, oj} - f2v{E.vj, E.wj};
  const f2v al2 = (Ti * Pi + Ta * Pa) * inv_det;  // (alpha, -ap)
  const f2v Qj = Ta * E.bs;                       // s * T_a b
  const f2v Qa = -(Tj * E.bs);                    // -s * T_j b
  const f2v be2 = (f2v{dj, dj} * Qj + f2v{da, da} * Qa) * inv_det;  // (beta, -bp)
  const float t = (E.c * Qj.x) * inv_det;
  const bool ok1 = !(fabsf(det) < kEps) & !(fminf(fminf(al2.x, be2.x), t) < 0.0f);  // (see quad_hit_masked)
  const bool second = (al2.x + be2.x) > 1.0f;
  const bool bad2 = (al2.y > 0.0f) | (be2.y > 0.0f);
  t_out = t;
  return ok1 & !(second & bad2);
}

// kSpheres = false: the quads only (the pool kernel's resumable sphere-BVH
// walk, spheres_bvh_step, continues from the quads' hit).
template <bool kBvh, bool kSpheres = true>
RTP_DEV Hit closest_hit(const DevScene* __restrict__ sc, f3 o, f3 d, bool prefilter,
                        uint32_t* full_out, const float* lds_prex) {
  Hit h{3.40282347e+38f, -1, 0};
  const float tmin = 0.001f;
  // the (t, orig) key minimum: the order the kinds are scanned in is free
  uint64_t key = kNoHitKey;
  bool full = true;  // this lane needs the exact scan of the axis-plane quads (kinds 1..6)
  const bool pre = prefilter && sc->n_pre > 0;  // wave-uniform
  {  // kinds 7..10 and 0: the exact scan, always (their keys are final)
    const int g6 = sc->kind_begin[6], g7 = sc->kind_begin[7], g8 = sc->kind_begin[8], g9 = sc->kind_begin[9],
              g10 = sc->kind_begin[10], g11 = sc->kind_begin[11];
    u16v cur = quad_head(sc, g6);
    scan_kind_pf<7>(sc, g6, g7, o, d, key, cur);
    scan_kind_pf<8>(sc, g7, g8, o, d, key, cur);
    scan_kind_pf<9>(sc, g8, g9, o, d, key, cur);
    scan_kind_pf<10>(sc, g9, g10, o, d, key, cur);
    scan_kind_pf<0>(sc, g10, g11, o, d, key, cur);
  }
  if (pre) {
    const bool lane_ok = (int)(fabsf(o.x) <= kPreLimD) & (int)(fabsf(o.y) <= kPreLimD) &
                         (int)(fabsf(o.z) <= kPreLimD) & (int)(fabsf(d.x) <= kPreLimD) &
                         (int)(fabsf(d.y) <= kPreLimD) & (int)(fabsf(d.z) <= kPreLimD);
    const float dmax = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), 1.0f));
    const float omax = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float ma = kPreK * dmax, mb = kPreK * (omax + (sc->pre_scale + 1.0f));
    uint32_t k1 = ~0u, k2 = ~0u;
    const int p0 = sc->pre_begin[0], p1 = sc->pre_begin[1], p2 = sc->pre_begin[2], p3 = sc->pre_begin[3];
    u8v pcur = pre_rec(sc, p0);
    pre_axis<0>(sc, p0, p1, o, d, ma, mb, k1, k2, pcur);
    pre_axis<1>(sc, p1, p2, o, d, ma, mb, k1, k2, pcur);
    pre_axis<2>(sc, p2, p3, o, d, ma, mb, k1, k2, pcur);
    // the candidate's PreExact record from the block's LDS table: four
    // 16-byte reads issued together (every lane: k1 = ~0u reads record 31,
    // in bounds, unused)
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v* lx = reinterpret_cast<const f4v*>(lds_prex) + 4 * (k1 & 31u);
    f4v xr[4] = {lx[0], lx[1], lx[2], lx[3]};
    static_assert(sizeof(PreExact) == sizeof(xr), "PreExact is four 16-byte loads");
    if (lane_ok && k1 != ~0u) {  // (finite o, d: the generic arithmetic equals the kind's)
      PreExact Q;
      __builtin_memcpy(&Q, xr, sizeof(Q));
      float t;
      const bool ok = quad_hit_axis(Q, o, d, t);
      const uint64_t kq = (uint64_t)__float_as_uint(t) << 32 | Q.key_lo;
      key = (ok && t > 0.001f && kq < key) ? kq : key;
    }
    full = !lane_ok || (k2 & ~31u) <= (uint32_t)(key >> 32);  // k2 = ~0u (none) never is
  }
  if (full_out) *full_out = !pre ? 2u : full ? 1u : 0u;  // 2: prefilter off for this scene
  if (__ballot(full)) {
    if (full) {
      const int g0 = sc->kind_begin[0], g1 = sc->kind_begin[1], g2 = sc->kind_begin[2], g3 = sc->kind_begin[3],
                g4 = sc->kind_begin[4], g5 = sc->kind_begin[5], g6 = sc->kind_begin[6];
      u16v cur = quad_head(sc, g0);
      scan_kind_pf<1>(sc, g0, g1, o, d, key, cur);
      scan_kind_pf<2>(sc, g1, g2, o, d, key, cur);
      scan_kind_pf<3>(sc, g2, g3, o, d, key, cur);
      scan_kind_pf<4>(sc, g3, g4, o, d, key, cur);
      scan_kind_pf<5>(sc, g4, g5, o, d, key, cur);
      scan_kind_pf<6>(sc, g5, g6, o, d, key, cur);
    }
  }
  if (key != kNoHitKey) {
    h.t = __uint_as_float((uint32_t)(key >> 32));
    h.kind = 0;
    h.idx = (int)(key & 0xffu);
  }
  static_assert(kQuadKinds == 11, "closest_hit scans every kind");
  if constexpr (!kSpheres) {
  } else if constexpr (kBvh) {
    spheres_bvh(sc, o, d, h);
  } else {
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
  }
  return h;
}

// Camera::RayGen (Camera.cxx:482-524): 2 draws, jittered direction
template <class Cam>  // DevCamera, or one read through an address-space-4 (kernarg) reference
RTP_DEV f3 camera_ray(const Cam& cam, int pi, int pj, int nx, int ny, uint32_t& seed) {
  float ru = randf(seed);
  float rv = randf(seed);
  f3 rd = add(add(ld3(cam.nlook), scl(ld3(cam.dx), ((2.f * ((float)pi + (1.f - ru)) - (float)nx) / 2.0f))),
              scl(ld3(cam.dy), ((2.f * ((float)pj + rv) - (float)ny) / 2.0f)));
  if (rd.x == 0.f) rd.x += 0.0000001f;
  if (rd.y == 0.f) rd.y += 0.0000001f;
  if (rd.z == 0.f) rd.z += 0.0000001f;
  float sq_mag = __builtin_sqrtf(dot(rd, rd));
  // rd.x / sq_mag, ... as Markstein divisions by one reciprocal: rd =
  // nlook + a*dx + b*dy with dx, dy orthogonal to the unit nlook (Camera.cxx:
  // 437-474), so sq_mag is >= ~1 and at most ~|tan(fov/2)| + 1 < 2^26 for fov
  // <= 180: inside rcp_nr1's exact range [2^-40, 2^40]; each |component| is
  // <= sq_mag and >= 1e-7 (the zero fix above), so no quotient or remainder
  // under- or overflows.
  const float r = rcp_nr1(sq_mag);
  return mk(div_markstein(rd.x, sq_mag, r), div_markstein(rd.y, sq_mag, r), div_markstein(rd.z, sq_mag, r));
}

struct Path {
  f3 org, dir;
  int d;           // current depth (the path is alive at the start of depth d)
  bool nonfinite;  // some stored A[d'] (d' <= D-2) is +-Inf or NaN
};

enum BounceResult { kAlive = 0, kMissed = 1, kLight = 2 };

// One depth for a ray that is alive at its start:
// intersect, collect, material, generate, pdfs, scatter.  Advances the RNG by
// exactly the reference's draws for this depth and stores A[d] at hist_d
// (when d <= D-2).  On kLight, `emit` receives E[d].
RTP_DEV unsigned long long stamp(bool on) { return on ? __builtin_amdgcn_s_memtime() : 0ull; }
// Stats build only (RTP_DEBUG_STATS=1): counters updated from divergent code
// go straight to the wave's record in global memory (gdbg = p.dbg + wave *
// kDbgCounters, zeroed before the launch), from its first active lane.
// dbg_region: one visit and the lanes active at the region's start;
// dbg_add: the sum of v over the active lanes.
RTP_DEV void dbg_region(unsigned long long* gdbg, int c) {
  const uint64_t m = __ballot(true);
  if ((int)(threadIdx.x & 63) == (int)__builtin_ctzll(m)) {
    atomicAdd(gdbg + c, 1ull);
    atomicAdd(gdbg + c + 1, (unsigned long long)__popcll(m));
  }
}
RTP_DEV void dbg_add(unsigned long long* gdbg, int c, unsigned long long v) { atomicAdd(gdbg + c, v); }

// kDeferDead: a path that misses or hits the light at depth k leaves its
// depth-k draws (which + generator, exactly one dead step) to the caller's
// fast-forward instead of drawing them here.
// qshade: the block's LDS quad table (fill_qshade).
template <bool kBvh, bool kDeferDead>
RTP_DEV int shade_hit(const DevScene* __restrict__ sc, Path& ps, uint32_t& seed, f3& emit, float4* __restrict__ hist_d,
                      int D, const float* qshade, const Hit h, unsigned long long* dbg = nullptr);
template <bool kBvh, bool kDeferDead = false>
RTP_DEV int bounce(const DevScene* __restrict__ sc, Path& ps, uint32_t& seed, f3& emit, float4* __restrict__ hist_d,
                   int D, unsigned long long* dbg, const float* qshade, unsigned long long* gdbg = nullptr) {
  const bool st = dbg != nullptr;
  const unsigned long long t0 = stamp(st);
  const f3 org = ps.org, dir = ps.dir;
  // intersect + CollectIntersecttWorklet (SurfaceWorklets.h:104-109)
  uint32_t fb = 0;  // (stats) 1: this lane ran the exact scan of the prefiltered quads
  Hit h = closest_hit<kBvh>(sc, org, dir, true, st ? &fb : nullptr, qshade + kPrexLdsOffset);
  if (st) {
    const unsigned long long m = __ballot(fb == 1u);
    dbg[kDbgFallbackSteps] += m ? 1 : 0;
    dbg[kDbgFallbackLanes] += (unsigned long long)__popcll(m);
  }
  if (gdbg) {  // (stats) lanes whose closest hit is one of the exact-scan quads (kinds 7..10, 0)
    const uint64_t mb = __ballot(h.kind == 0 && h.idx >= sc->kind_begin[6]);
    if ((int)(threadIdx.x & 63) == (int)__builtin_ctzll(__ballot(true))) {
      if (mb == 0) dbg_add(gdbg, kDbgBoxFreeSteps, 1ull);
      dbg_add(gdbg, kDbgBoxLanes, (unsigned long long)__popcll(mb));
    }
  }
  if (st) {
    const unsigned long long t1s = __builtin_amdgcn_s_memtime();
    dbg[kDbgCyclesIntersect] += t1s - t0;
  }
  return shade_hit<kBvh, kDeferDead>(sc, ps, seed, emit, hist_d, D, qshade, h, gdbg);
}

// The rest of one depth once the closest hit h is known: collect, material,
// generate, pdfs, scatter (bounce() above; the pool kernel's resumable
// sphere-BVH walk calls it directly for the lanes whose walk has finished).
// dbg (stats build only): the wave's global counter record (dbg_region).
template <bool kBvh, bool kDeferDead>
RTP_DEV int shade_hit(const DevScene* __restrict__ sc, Path& ps, uint32_t& seed, f3& emit, float4* __restrict__ hist_d,
                      int D, const float* qshade, const Hit h, unsigned long long* dbg) {
  const uint32_t t1 = sc->which_t1, t2 = sc->which_t2;
  const DevLights& L = sc->light;
  const f3 org = ps.org, dir = ps.dir;
  const int d = ps.d;
  if (h.kind < 0) {
    if (!kDeferDead) seed = dead_step(seed, t1, t2);  // which + generator draws of the now-dead ray
    return kMissed;
  }
  if (dbg) dbg_region(dbg, kDbgHitVisits);
  f3 hp = add(org, scl(dir, h.t));
  f3 hn;
  int mt;
  f3 alb;
  if (h.kind == 0) {
    // (an LDS table always: a global fallback here made the compiler read
    // both through one flat pointer)
    const float4* r = reinterpret_cast<const float4*>(qshade + h.idx * kQShadeFloats);  // 16-byte aligned
    const float4 r0 = r[0], r1 = r[1];
    hn = mk(r0.x, r0.y, r0.z);
    alb = mk(r0.w, r1.x, r1.y);
    mt = __float_as_int(r1.z);
    if (dot(hn, dir) > 0.f) hn = neg(hn);  // Surface.h:184-185
  } else {
    const DevSphere& S = kBvh ? sc->sph_all[h.idx] : sc->spheres[h.idx];
    hn = mk((hp.x - S.c[0]) / S.r, (hp.y - S.c[1]) / S.r, (hp.z - S.c[2]) / S.r);
    mt = S.mt;
    alb = ld3(S.alb);
  }
  // applyMaterials (EmitWorklet.h)
  if (mt == 1) {  // DiffuseLightWorklet: emit, path ends (status &= 0)
    if (dbg) dbg_region(dbg, kDbgLightVisits);
    emit = (dot(hn, dir) < 0.0f) ? alb : mk(0.f, 0.f, 0.f);
    if (!kDeferDead) seed = dead_step(seed, t1, t2);
    return kLight;
  }
  f3 atten;
  // The RNG draws of both scattering materials, taken together (one pass for
  // the dielectric and Lambertian lanes instead of one per branch): the
  // dielectric's own draw (DielectricWorklet, EmitWorklet.h), then for both
  // the which draw and the generator's 2 / 3 / 2 draws (PdfWorklet.h:20,
  // 63-213; a dielectric discards the direction: dead_step's advance) and
  // SpherePDFWorklet's discarded draw (no draw lies between the generator and
  // it: quad_pdf_value draws none).
  const bool glass = mt == 2;
  float rglass = 0.0f;
  if (glass) rglass = randf(seed);
  const uint32_t tw = wang(seed);  // which (PdfWorklet.h:20)
  seed = tw;
  const bool is_cos = tw < t1, is_quad = !is_cos && tw < t2;
  const float ra = randf(seed);
  const float rb = randf(seed);
  uint32_t s3 = seed;
  const float rc = randf(s3);
  seed = is_quad ? s3 : seed;
  (void)randf(seed);  // SpherePDFWorklet's discarded draw
  if (glass) {  // DielectricWorklet: specular
    const unsigned long long td0 = stamp(dbg != nullptr);
    if (dbg) dbg_region(dbg, kDbgDielVisits);
    f3 sd;
    dielectric_scatter(dir, hn, sc->ior, sc->ior_r0sq, sc->ior_inv, rglass, sd);
    atten = mk(1.f, 1.f, 1.f);
    ps.org = hp;
    ps.dir = sd;
    if (dbg) {
      const unsigned long long td1 = __builtin_amdgcn_s_memtime();
      if ((int)(threadIdx.x & 63) == (int)__builtin_ctzll(__ballot(true))) dbg_add(dbg, kDbgCyclesDiel, td1 - td0);
    }
  } else {  // LambertianWorklet
    const unsigned long long tg0 = stamp(dbg != nullptr);
    if (dbg) dbg_region(dbg, kDbgGenVisits);
    f3 gen;
    float sph_ctm = -1.0f;  // sqrt(1 - R^2/|c-hp|^2) when the generator made it (sphere_pdf_value reuses it)
    // The three generators as one branch-free pass.  Cosine (PdfWorklet.h:
    // 63-79) and light-sphere (:193-213) directions share the ONB, the
    // sincos of phi = 2*pi*r1 and local(); they differ in w, in which draw
    // is r1 (g++ evaluates the sphere generator's draws right to left), and
    // in z and the radial factor.  The light-quad point (:112-137) needs a
    // third draw, taken only by its lanes (drawn above).
    const f3 rp = mk(L.gx0 + ra * L.gdx, L.gy0 + rb * L.gdy, L.gz0 + rc * L.gdz);
    const f3 genq = sub(rp, hp);
    const f3 direction = sub(ld3(L.sc), hp);
    const float r1 = is_cos ? ra : rb, r2 = is_cos ? rb : ra;
    const f3 wdir = is_cos ? hn : direction;
    const Onb guvw = build_from_w(wdir);
    const float phi = (float)(2 * kPi * r1);
    float sphi, cphi;
    rtp_sincosf(phi, &sphi, &cphi);
    // cosine: z = sqrt(1-r2), x = (cos(phi)*2)*sqrt(r2); sphere: z = 1 + r2*(sqrt(1-R^2/d^2)-1),
    // x = cos(phi)*sqrt(1-z*z) (and (c*1)*s == c*s exactly)
    const float dist2 = dot(direction, direction);
    const float q = sqrt_exact(is_cos ? 1 - r2 : 1 - L.srr / dist2);
    sph_ctm = is_cos ? -1.0f : q;
    const float z = is_cos ? q : 1 + r2 * (q - 1);
    const float rad = sqrt_exact(is_cos ? r2 : 1 - z * z);
    const float m = is_cos ? 2.0f : 1.0f;
    const f3 gcs = de_nan(local(guvw, mk(cphi * m * rad, sphi * m * rad, z)));
    gen = is_quad ? genq : gcs;
    const unsigned long long tg1 = stamp(dbg != nullptr);
    // applyPDFs: QuadPDFWorklet, SpherePDFWorklet (1 discarded draw)
    const float weight = 0.5f;
    float sum = 0;
    // 1/|gen| once: QuadPDFWorklet's rmag and both unit_vector(gen) below
    const float rg = rmag(gen);
    sum += weight * quad_pdf_value(L, hp, gen, rg);
    sum += weight * sphere_pdf_value(L, hp, gen, sph_ctm);  // (its discarded draw: above)
    // PDFCosineWorklet (ScatterWorklet.h:96-112): mixture in double
    const f3 ug = scl(gen, rg);       // unit_vector(gen)
    const f3 w_hn = unit_vector(hn);  // build_from_w(hn).w (u and v are unused here)
    float cv;
    {
      float cosine = dot(ug, w_hn);
      cv = (cosine > 0) ? cos_over_pi(cosine) : 0.f;
    }
    double pdf_val = 0.5 * (double)sum + 0.5 * (double)cv;
    float sp;
    {
      float cosine = dot(hn, ug);
      sp = (cosine < 0) ? 0.f : cos_over_pi(cosine);
    }
    double sctr = (double)sp / pdf_val;
    atten = mk((float)(alb.x * sctr), (float)(alb.y * sctr), (float)(alb.z * sctr));
    ps.org = hp;
    ps.dir = gen;
    if (dbg) {  // (wave cycles: added once, by the first active lane)
      const unsigned long long tg2 = __builtin_amdgcn_s_memtime();
      if ((int)(threadIdx.x & 63) == (int)__builtin_ctzll(__ballot(true))) {
        dbg_add(dbg, kDbgCyclesGen, tg1 - tg0);
        dbg_add(dbg, kDbgCyclesPdf, tg2 - tg1);
      }
    }
  }
  if (d <= D - 2) {
    *hist_d = make_float4(atten.x, atten.y, atten.z, 0.f);
    ps.nonfinite |= !(__builtin_isfinite(atten.x) && __builtin_isfinite(atten.y) && __builtin_isfinite(atten.z));
  }
  return kAlive;
}

// Back-to-front radiance (MapperPathTracer.cxx:328-348) of a finished path:
// s = E[D-1]+0; s = A[d]*s; s = E[d]+s for d = D-2..0.  Depths after the end
// contribute A=1, E=0 exactly, so for a light hit at depth k this is
// s = E_k (+0), then s = 0 + A[d]*s for d = k-1..0; for any other ending it
// is +0, or NaN if some stored A was not finite (Inf*0 / NaN propagation).
RTP_DEV f3 path_radiance(int result, int k, f3 emit, bool nonfinite, const float4* __restrict__ hist,
                         int64_t stride) {
  if (result != kLight) {
    const float v = nonfinite ? __builtin_nanf("") : 0.0f;
    return mk(v, v, v);
  }
  float sx = emit.x + 0.0f, sy = emit.y + 0.0f, sz = emit.z + 0.0f;
  for (int dd = k - 1; dd >= 0; dd--) {
    float4 a = hist[(int64_t)dd * stride];
    sx = a.x * sx;
    sy = a.y * sy;
    sz = a.z * sz;
    sx = 0.0f + sx;
    sy = 0.0f + sy;
    sz = 0.0f + sz;
  }
  return mk(sx, sy, sz);
}

// Tile-deal index arithmetic: q = ti / tx from a float reciprocal, then one
// correction each way (ti < 2^24, so the estimate is off by at most one).
template <class KP>
RTP_DEV int64_t tile_pixel(const KP& p, int k) {
  const int ti = (k >> 8) * p.tile_world + p.tile_rank, within = k & 255;
  int ty = (int)((float)ti * __builtin_amdgcn_rcpf((float)p.tile_tx));
  ty += (ty + 1) * p.tile_tx <= ti;
  ty -= ty * p.tile_tx > ti;
  const int tx = ti - ty * p.tile_tx;
  return (int64_t)(ty * 16 + (within >> 4)) * p.nx + tx * 16 + (within & 15);
}
// The pixel's column and row directly (refill): the tile deal gives them
// without forming the linear index; a pixel index is split by a float
// reciprocal quotient with one correction each way, exact while every index
// is below 2^24 (the estimate is then off by at most one), else by integer
// division (a wave-uniform branch).  The compiler's signed % and / cost ~40
// VALU per refill.
template <bool kTiles = false, class KP>
RTP_DEV void pixel_xy(const KP& p, int k, int& pi, int& pj) {
  if constexpr (kTiles) {
    const int ti = (k >> 8) * p.tile_world + p.tile_rank, within = k & 255;
    int ty = (int)((float)ti * __builtin_amdgcn_rcpf((float)p.tile_tx));
    ty += (ty + 1) * p.tile_tx <= ti;
    ty -= ty * p.tile_tx > ti;
    const int tx = ti - ty * p.tile_tx;
    pj = ty * 16 + (within >> 4);
    pi = tx * 16 + (within & 15);
  } else {
    const int u = (int)(p.pixel_ids ? p.pixel_ids[k] : p.pixel_begin + k);  // in [0, nx * ny)
    const int nx = p.nx;
    if ((int64_t)nx * p.ny <= (int64_t)1 << 24) {
      int q = (int)((float)u * __builtin_amdgcn_rcpf((float)nx));
      q += (q + 1) * nx <= u;
      q -= q * nx > u;
      pj = q;
      pi = u - q * nx;
    } else {
      pj = (int)((uint32_t)u / (uint32_t)nx);
      pi = u - pj * nx;
    }
  }
}
// kTiles: a separate kernel instance (rtp_render_tiles_device).  A runtime
// branch here changed the compiler's code for the whole scheduling loop of
// the other modes (+9% time), as other additions to the refill path did.
template <bool kTiles = false, class KP>
RTP_DEV int64_t pixel_of(const KP& p, int k) {  // k < npix <= INT32_MAX (launch() checks)
  if constexpr (kTiles) return tile_pixel(p, k);
  else return p.pixel_ids ? p.pixel_ids[k] : p.pixel_begin + k;
}

// ------------------------------------------------------------------ v1 ---
template <bool kBvh>
__global__ void __launch_bounds__(256) rtp_render_lockstep(const DevScene* __restrict__ sc, KParams p) {
  __shared__ __align__(16) float s_qshade[kQTableFloats];
  fill_qshade(sc, s_qshade);
  __syncthreads();
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= p.npix) return;
  const int64_t pix = pixel_of(p, k);
  const uint32_t t1 = sc->which_t1, t2 = sc->which_t2;
  uint32_t seed = p.seed_base + (uint32_t)pix;  // seeds[i] = i (MapperPathTracer.cxx:265-267)
  float cr = 0.f, cg = 0.f, cb = 0.f;
  uint32_t live = 0;
  const int pi = (int32_t)pix % p.nx, pj = (int32_t)pix / p.nx;
  float4* __restrict__ hist = reinterpret_cast<float4*>(p.hist) + k;
  const int64_t stride = p.npix;
  const int D = p.depth;
  for (int s = 0; s < p.spp; s++) {
    Path ps;
    ps.dir = camera_ray(p.cam, pi, pj, p.nx, p.ny, seed);
    ps.org = ld3(p.cam.eye);
    ps.nonfinite = false;
    int result = kAlive, k_end = D;
    f3 emit = mk(0.f, 0.f, 0.f);
    for (int d = 0; d < D; d++) {
      if (result != kAlive) {
        seed = dead_step(seed, t1, t2);
        continue;
      }
      live++;
      ps.d = d;
      result = bounce<kBvh>(sc, ps, seed, emit, hist + (int64_t)d * stride, D, nullptr, s_qshade);
      if (result != kAlive) k_end = d;
    }
    f3 c = path_radiance(result, k_end, emit, ps.nonfinite, hist, stride);
    cr = cr + c.x;
    cg = cg + c.y;
    cb = cb + c.z;
  }
  reinterpret_cast<float4*>(p.out)[k] = make_float4(cr, cg, cb, 0.f);
  if (p.seed_out) p.seed_out[k] = seed;
  if (p.live_out) p.live_out[k] = live;
}

// ------------------------------------------------------------------ v2 ---
constexpr int kWavesPerBlock = 4;
#ifndef RTP_POOL
#define RTP_POOL 128
#endif
constexpr int kPool = RTP_POOL;  // pixel slots per wave (power of two: queue index = cursor & (kPool-1))
static_assert(kPool == kPoolSlots || RTP_POOL != 128, "rtp_layout.hpp kPoolSlots is the production pool size");
static_assert((kPool & (kPool - 1)) == 0 && kPool >= 64, "pool size must be a power of two >= 64");
// LDS per wave: seed, r, g, b, samples, live (u32) + rem, q_ready, q_ff (u16):
// 30 B x 128 slots x 4 waves + the 2 KB quad shading table = 17 KiB per
// block.  Occupancy is set by VGPRs (5 waves per SIMD at <= 96, below).
// Measured on C2 / C3 / C4: 128 slots at 5 waves beat 256 slots at 4 waves
// by 6 / 10 / 5%; 256 slots at 5 waves (LDS booked to the last byte) and
// 128 slots at 6 waves (80 VGPRs, spills) were slower.
constexpr int kSlotBytes = 6 * 4 + 3 * 2;
// s_rem packs the remaining dead depths with how the sample's path ended
constexpr int kRemMask = 0x3fff, kEndLight = 0x4000, kEndNonfinite = 0x8000;
static_assert(kMaxDepth <= kRemMask, "the remaining dead depths fit s_rem's count field");
constexpr int kPoolLdsBytes = kWavesPerBlock * kPool * kSlotBytes;

RTP_DEV uint32_t lane_rank(uint64_t mask) {  // number of set mask bits below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
RTP_DEV void wave_sync() {  // order LDS traffic between lanes of this wave (no cross-wave barrier)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Issue-priority balancing: the SIMD arbiter favours older waves, so with a
// static split of pixels the youngest wave of each SIMD finished ~1/3 later
// than the oldest, and the SIMD ran its last milliseconds with one or two
// waves (little latency hiding).  Every kPrioPeriod finished samples a wave publishes
// its finished samples to a global counter and sets s_setprio from how far
// its own completed fraction lags the global one.
#ifndef RTP_PRIO_BALANCE
#define RTP_PRIO_BALANCE 1
#endif
#ifndef RTP_PRIO_THR
#define RTP_PRIO_THR 0.0002f
#endif
#ifndef RTP_PRIO_PERIOD
#define RTP_PRIO_PERIOD 128
#endif
constexpr int kPrioPeriod = RTP_PRIO_PERIOD;

RTP_DEV void set_priority(float lag) {  // s_setprio needs an immediate
  if (lag > RTP_PRIO_THR) __builtin_amdgcn_s_setprio(3);
  else if (lag > 0.0f) __builtin_amdgcn_s_setprio(2);
  else if (lag > -RTP_PRIO_THR) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

#ifndef RTP_POOL_MIN_WAVES_PER_EU
#define RTP_POOL_MIN_WAVES_PER_EU 5
#endif
// gfx950 allocates VGPRs in granules of 8: 5 waves per SIMD need <= 96.  The
// waves-per-EU hint alone settles at 102 (4 waves); the hard cap costs one
// spilled 64-bit value (16 B of scratch).
#ifndef RTP_POOL_MAX_VGPR
#define RTP_POOL_MAX_VGPR 96
#endif
// byte offset of the KParams argument in rtp_render_pool's kernarg segment:
// the first argument (the scene pointer) rounded up to KParams' alignment
// (also checked against the code object's argument metadata by
// tests/test_abi.py)
constexpr int kKParamsOffset =
    (int)((sizeof(const DevScene*) + alignof(KParams) - 1) / alignof(KParams) * alignof(KParams));
static_assert(alignof(KParams) <= 16 && kKParamsOffset == 8, "KParams follows the 8-byte scene pointer");
typedef const __attribute__((address_space(4))) KParams CKP;
// The kernel arguments re-read where they are used (scalar loads from the
// kernarg segment): values loaded once and kept live through the scheduling
// loop were SGPRs spilled to VGPR lanes (v_readlane in the hot path).
RTP_DEV CKP& kparams() {
  CKP* pp = (CKP*)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() +
                   kKParamsOffset);
  asm volatile("" : "+s"(pp));
  return *pp;
}
typedef const __attribute__((address_space(1))) uint32_t GU32;
// kPlan: a planned launch (KParams::wave_begin): wave w owns the entries
// [wave_begin[w], wave_begin[w+1]) -- up to kPool of them, grouped by their
// expected cost -- instead of the interleaved entries j * n_waves + w.
// The pool kernel's body; kWPB waves per block, kLdsBvh: the sphere BVH is
// walked out of the block's LDS copy (s_bvh: the LDS walk's compact nodes,
// then its leaf spheres; rtp_render_pool_lds).
// kSteal: a launch with more entries than its waves' pools hold (C3, C4,
// C5 on one GPU).  The waves are the resident ones; a slot whose pixel has
// all its samples writes the pixel out and claims the next unclaimed entry
// (one atomic per batch), so no wave idles while entries remain, instead of
// waves of 128 pixels each running in generations with a tail per wave.
template <bool kStats, bool kBvh, bool kTiles, bool kPlan, int kWPB, bool kLdsBvh, bool kSteal = false>
__device__ __forceinline__ void pool_body(const DevScene* __restrict__ sc, const KParams& p, int n_waves,
                                          unsigned char* smem, float* s_qshade, uint32_t* s_bvh,
                                          uint32_t* s_entry_all = nullptr) {
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  const int w = blockIdx.x * kWPB + wib;  // global wave id
  // the quads' shading data into LDS (the block's only barrier, before any wave leaves)
  fill_qshade(sc, s_qshade);  // (n_quads <= kMaxQuads = kLdsQuads)
  if constexpr (kLdsBvh) {  // and the LDS walk's tree (its size checked on the host: rtp_lds_walk_capacity)
    const int nn = 8 * sc->n_lw_nodes, ns = sc->n_lw_sph;
    u4v* dst = reinterpret_cast<u4v*>(s_bvh);
    GU4* const gn = (GU4*)sc->lw_nodes;
    GU4* const gs = (GU4*)sc->lw_sph;
    for (int i = threadIdx.x; i < nn; i += blockDim.x) dst[i] = gn[i];
    for (int i = threadIdx.x; i < ns; i += blockDim.x) dst[nn + i] = gs[i];
  }
  __syncthreads();
  if (w >= n_waves) return;  // whole wave leaves; no block-level barriers follow
  unsigned char* base = smem + (size_t)wib * kPool * kSlotBytes;
  uint32_t* s_seed = reinterpret_cast<uint32_t*>(base);
  float* s_r = reinterpret_cast<float*>(s_seed + kPool);
  float* s_g = s_r + kPool;
  float* s_b = s_g + kPool;
  uint32_t* s_samples = reinterpret_cast<uint32_t*>(s_b + kPool);
  uint32_t* s_live = s_samples + kPool;
  uint16_t* s_rem = reinterpret_cast<uint16_t*>(s_live + kPool);
  uint16_t* q_ready = s_rem + kPool;
  uint16_t* q_ff = q_ready + kPool;
  uint32_t* s_entry = kSteal ? s_entry_all + wib * kPool : nullptr;  // kSteal: the slot's entry

  const uint32_t t1 = sc->which_t1, t2 = sc->which_t2;
  const int D = p.depth, S = p.spp;
  // slot j of wave w <-> list entry k = j * n_waves + w (pixels interleaved over waves)
  // or, planned, k = wave_begin[w] + j
  int n_slots, wbase = 0;
  if constexpr (kPlan) {  // (the host checked the plan; the clamps keep a bad one inside the buffers)
    wbase = p.wave_begin[w];
    n_slots = max(0, min(min(kPool, p.wave_begin[w + 1] - wbase), (int)(p.npix - wbase)));
  } else {
    const int64_t left = p.npix - w;
    n_slots = left <= 0 ? 0 : (int)min<int64_t>(kPool, (left + n_waves - 1) / n_waves);
  }
  for (int j = lane; j < n_slots; j += 64) {
    const int64_t k = kPlan ? (int64_t)(wbase + j) : (int64_t)j * n_waves + w;
    if constexpr (kSteal) s_entry[j] = (uint32_t)k;
    s_seed[j] = p.seed_base + (uint32_t)pixel_of<kTiles>(p, k);  // seeds[i] = i (MapperPathTracer.cxx:265-267)
    s_r[j] = 0.f;
    s_g[j] = 0.f;
    s_b[j] = 0.f;
    s_samples[j] = 0u;
    s_live[j] = 0u;
    s_rem[j] = 0;
    q_ready[j] = (uint16_t)j;
  }
  wave_sync();
  // wave-uniform, monotone queue cursors
  // (uint32: under kSteal a wave's finished-sample count ff_tail runs over
  // every pixel it claims -- C5 on one GPU: ~2.6e10 -- so it wraps; only the
  // differences of cursors (each < 2^31: <= kPool * spp) and their low bits
  // (the ring index) are used, and unsigned arithmetic wraps exactly)
  uint32_t ready_head = 0, ready_tail = (S > 0) ? n_slots : 0, ff_head = 0, ff_tail = 0;
  int unfinished = n_slots;                // stats only: pixels with samples still to run
  unsigned long long t_tail = 0;

  // attenuation history per pixel SLOT, D rows: a pixel has one sample in
  // flight, so its history survives until the fast-forward batch that
  // computes the sample's radiance (row k of a light hit holds E_k)
  // depth-major [d][wave*kPool + slot]: the hot depths 0..4 of all slots
  // stay dense.  (A slot-major layout, one pixel's rows in one 128-byte line,
  // measured no faster: r03c, profiles/r03c_ab_history_prex.txt.)
  float4* __restrict__ const hist_base = reinterpret_cast<float4*>(p.hist) + (int64_t)w * kPool;
  const int64_t stride = (int64_t)n_waves * kPool;
  float4* __restrict__ hist = hist_base;  // per lane: hist_base + slot of its path
  const f3 eye = ld3(p.cam.eye);

  // diagnostics (uniform branch on a kernel argument; off in production)
  // (compiled in only for the kStats instantiation: the counters cost ~30 VGPRs)
  unsigned long long dbg[kStats ? kDbgCounters : 1] = {};
  constexpr bool want_dbg = kStats;
  unsigned long long* const gdbg = want_dbg ? p.dbg + (int64_t)w * kDbgCounters : nullptr;
  const unsigned long long t_start = want_dbg ? __builtin_amdgcn_s_memtime() : 0ull;
  if (p.dbg && lane == 0) {  // placement + start time (RTP_DEBUG_STATS=1|2)
    p.dbg[(int64_t)w * kDbgCounters + kDbgRealStart] = __builtin_amdgcn_s_memrealtime();
    p.dbg[(int64_t)w * kDbgCounters + kDbgHwId] =
        (unsigned)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID
  }

  uint32_t published = 0;  // wave-uniform: ff_tail when the finished samples were last added to p.progress
  // kSteal (wave-uniform): slots still holding a pixel, and the samples of the
  // pixels already written out (the fair-share average is over the others)
  int live_slots = n_slots;
  uint32_t retired = 0;  // (the samples of the written-out pixels, mod 2^32 like ff_tail)
  bool critical_ff = false;  // wave-uniform: a critical (far-lagging) pixel waits in the FF queue

  bool has_path = false;
  int slot = 0;
  uint32_t seed = 0;
  // Sphere-BVH scenes (global walk): the closest-hit search is resumable.
  // A path's walk spans as many loop iterations as it needs; an iteration
  // walks until RTP_WALK_DONE of the wave's paths have finished theirs, and
  // only those are shaded.  The walks' lengths differ several-fold between
  // lanes (C3: 17 of 64 lanes per VALU instruction when every lane's walk ran
  // to its end inside one iteration); now a long walk no longer holds the
  // other 63 lanes.  The walk is the same walk (same nodes, same order, same
  // running minimum), so the hit is bit-identical.
  constexpr bool kWalk = kBvh;
  int wni = -1;                             // the path's next BVH node; -1: its quads are not scanned yet
  Hit wh{3.40282347e+38f, -1, 0};           // its closest hit so far
  Path ps;
  ps.org = eye;
  ps.dir = mk(0.f, 0.f, 1.f);
  ps.d = 0;
  ps.nonfinite = false;

  for (;;) {
    const uint64_t idle = __ballot(!has_path);
    const int n_idle = __popcll(idle);
    const int n_ready = (int)(ready_tail - ready_head);
    const int n_ff = (int)(ff_tail - ff_head);
    if ((n_ready < n_idle + RTP_FF_MARGIN || critical_ff) && n_ff > 0) {
      critical_ff = false;
      // ---- batch RNG fast-forward over the remaining dead depths of finished
      //      samples (1 + {2,3,2} draws per depth) ----
      const unsigned long long t0 = want_dbg ? __builtin_amdgcn_s_memtime() : 0ull;
      const int n = min(64, n_ff);
      const bool mine = lane < n;
      int fslot = 0, frem = 0;
      uint32_t fseed = 0;
      if (mine) {
        fslot = q_ff[(ff_head + lane) & (kPool - 1)];
        fseed = s_seed[fslot];
        frem = s_rem[fslot];
      }
      // the first jump-table read is issued before the radiance loads below,
      // so its latency overlaps theirs: the direct table of the sample's
      // remaining count when there is one (then it is the only read), else
      // the 32-depth table
      uint32_t early = 0;
      const int frc = frem & kRemMask;
      CKP& FP = kparams();
      const bool has_direct = mine && FP.ffd != nullptr && (unsigned)(frc - FP.ffd_first) < (unsigned)FP.ffd_count;
      const bool has_early = mine && !has_direct && FP.ff[0] != nullptr && frc >= 32;
      if (has_direct || has_early) {
        GU32* src = (GU32*)(has_direct ? FP.ffd + ((uint64_t)(frc - FP.ffd_first) << 32) : FP.ff[0]);
        early = src[fseed];
      }
      if (mine) {
        // back-to-front radiance of the pixel's finished sample (path_radiance),
        // banked in sample order before the pixel's next sample can start
        const int flags = frem;
        frem &= kRemMask;
        f3 c;
        if (flags & kEndLight) {
          const int k_end = D - frem;  // a light hit ends the path: rem = D - 1 - k_end + 1
          if (want_dbg) {
            dbg_region(gdbg, kDbgFfRadVisits);
            dbg_add(gdbg, kDbgFfRadRows, (unsigned long long)(k_end + 1));
          }
          const float4* __restrict__ hp = hist_base + fslot;
          // rows k_end (E) and k_end-1 .. k_end-5 issued together (clamped to
          // row 0; rows below 0 are not applied), the rest two per trip;
          // products in the reference's order (depth k_end-1 down to 0).
          // One wait instead of up to three dependent round trips: C2 -1%
          // (r03f, profiles/r03f_ab_history_prefetch.txt).
          f3 rw[kHistPrefetch];
#pragma unroll
          for (int i = 0; i < kHistPrefetch; i++) {
            const float4 v = hp[(int64_t)max(k_end - i, 0) * stride];
            rw[i] = mk(v.x, v.y, v.z);
          }
          float sx = rw[0].x + 0.0f, sy = rw[0].y + 0.0f, sz = rw[0].z + 0.0f;
#pragma unroll
          for (int i = 1; i < kHistPrefetch; i++) {
            const bool on = k_end - i >= 0;
            sx = on ? 0.0f + rw[i].x * sx : sx;
            sy = on ? 0.0f + rw[i].y * sy : sy;
            sz = on ? 0.0f + rw[i].z * sz : sz;
          }
          int dd = k_end - kHistPrefetch;
          // the remaining rows kHistChunk at a time, each chunk's loads
          // issued together (one wait per chunk)
          for (; dd >= 0; dd -= kHistChunk) {
            f3 rc[kHistChunk];
#pragma unroll
            for (int i = 0; i < kHistChunk; i++) {
              const float4 v = hp[(int64_t)max(dd - i, 0) * stride];
              rc[i] = mk(v.x, v.y, v.z);
            }
#pragma unroll
            for (int i = 0; i < kHistChunk; i++) {
              const bool on = dd - i >= 0;
              sx = on ? 0.0f + rc[i].x * sx : sx;
              sy = on ? 0.0f + rc[i].y * sy : sy;
              sz = on ? 0.0f + rc[i].z * sz : sz;
            }
          }
          c = mk(sx, sy, sz);
        } else {
          const float v = (flags & kEndNonfinite) ? __builtin_nanf("") : 0.0f;
          c = mk(v, v, v);
        }
        s_r[fslot] = s_r[fslot] + c.x;  // cols += sumtotl (MapperPathTracer.cxx:350), in sample order
        s_g[fslot] = s_g[fslot] + c.y;
        s_b[fslot] = s_b[fslot] + c.z;
      }
      // jump over 32 / 16 / 8 / 4 dead depths with one table read each
      // (HBM-resident tables of the dead-step map, built once per device),
      // then hash the few remaining depths
      if (has_direct) {
        fseed = early;
        frem = 0;
      } else if (has_early) {
        fseed = early;
        frem -= 32;
      }
#pragma unroll
      for (int j = 1; j < kFfTables; j++) {
        GU32* __restrict__ tab = (GU32*)kparams().ff[j];
        if (tab != nullptr && mine && frem >= (32 >> j)) {
          fseed = tab[fseed];
          frem -= 32 >> j;
        }
      }
      int iters = 0;
      for (int i = 0;; i++) {
        const bool act = mine && i < frem;
        if (!__any(act)) break;
        if (act) fseed = dead_step(fseed, t1, t2);
        if (want_dbg) {
          const uint64_t am = __ballot(act);
          if (lane == 0) dbg_add(gdbg, kDbgDeadLanes, (unsigned long long)__popcll(am));
        }
        iters++;
      }
      bool again = false;
      if (mine) s_seed[fslot] = fseed;
      if (mine) again = s_samples[fslot] < (uint32_t)S;
      if (want_dbg) unfinished -= __popcll(__ballot(mine && !again));
      if constexpr (kSteal) {
        // pixels with all their samples: written out, their slots take the
        // next unclaimed entries (claimed in launch order after the initial
        // n_waves * kPool)
        const uint64_t done = __ballot(mine && !again);
        if (done) {
          const int nd = __popcll(done);
          unsigned long long base = 0;
          if (lane == 0) base = atomicAdd(kparams().progress + 1, (unsigned long long)nd);
          base = __shfl(base, 0) + (unsigned long long)n_waves * kPool;
          retired += (uint32_t)(nd * S);
          if (mine && !again) {
            const int64_t k = (int64_t)s_entry[fslot];
            reinterpret_cast<float4*>(p.out)[k] = make_float4(s_r[fslot], s_g[fslot], s_b[fslot], 0.f);
            if (p.seed_out) p.seed_out[k] = s_seed[fslot];
            if (p.live_out) p.live_out[k] = s_live[fslot];
            const unsigned long long kn = base + lane_rank(done);
            if (kn < (unsigned long long)p.npix) {  // a fresh pixel in this slot, at the front of READY below
              s_entry[fslot] = (uint32_t)kn;
              s_seed[fslot] = p.seed_base + (uint32_t)pixel_of<kTiles>(p, (int)kn);
              s_r[fslot] = 0.f;
              s_g[fslot] = 0.f;
              s_b[fslot] = 0.f;
              s_samples[fslot] = 0u;
              s_live[fslot] = 0u;
              s_rem[fslot] = 0;
              again = true;
            }
          }
          live_slots -= __popcll(__ballot(mine && !again));
        }
      }
      // Fair share: a pixel whose completed samples are at or below the
      // wave's average (ff_tail / n_slots) goes to the FRONT of the READY
      // ring, the others to the back.  FIFO alone let cheap pixels (short
      // paths, back sooner) take more than their share of lanes, so the
      // expensive pixels' sequential sample chains ran on alone at the end
      // (17% of bounce steps with ~12 of 64 lanes live).
      // (samples * slots <= 2^23 * 2^7; ff_tail (no stealing) and ff_tail - retired (the
      // held pixels' finished samples) are <= 2^7 * spp: 32 bits suffice)
      const bool urgent = again && (kSteal ? s_samples[fslot] * (uint32_t)live_slots <= (uint32_t)(ff_tail - retired)
                                           : s_samples[fslot] * (uint32_t)n_slots <= (uint32_t)ff_tail);
      const uint64_t pu = __ballot(urgent), pn = __ballot(again && !urgent);
      ready_head -= (uint32_t)__popcll(pu);
      if (urgent) q_ready[(ready_head + lane_rank(pu)) & (kPool - 1)] = (uint16_t)fslot;
      if (again && !urgent) q_ready[(ready_tail + lane_rank(pn)) & (kPool - 1)] = (uint16_t)fslot;
      ready_tail += __popcll(pn);
      ff_head += n;
      wave_sync();
      if (want_dbg) {
        dbg[kDbgFfPhases] += 1;
        dbg[kDbgFfLanes] += (unsigned long long)n;
        dbg[kDbgFfIters] += (unsigned long long)iters;
        dbg[kDbgCyclesFf] += __builtin_amdgcn_s_memtime() - t0;
      }
      // on into the refill, which takes the pixels this batch made READY,
      // and the bounce: a sample's chain spends no iteration of its own on
      // the fast-forward
    }
    // ---- refill idle lanes with the next sample of READY pixels ----
    const unsigned long long tb = stamp(want_dbg);
    const int take = min(n_idle, (int)(ready_tail - ready_head));
    if (!has_path) {
      const int r = (int)lane_rank(idle);
      if (r < take) {
        if (want_dbg) dbg_region(gdbg, kDbgRefillVisits);
        slot = q_ready[(ready_head + r) & (kPool - 1)];
        seed = s_seed[slot];
        hist = hist_base + slot;
        // the camera and tile constants re-read from the kernel arguments
        // here (kparams): kept live through the loop they were SGPRs spilled
        // to VGPR lanes, ~30 v_readlane per refill (through the kernarg
        // segment pointer: &p would copy p to scratch)
        CKP& P = kparams();
        int pi, pj;
        pixel_xy<kTiles>(P, kSteal ? (int)s_entry[slot] : kPlan ? wbase + slot : slot * n_waves + w, pi,
                         pj);  // (32-bit index: a 64-bit one spilled)
        ps.dir = camera_ray(P.cam, pi, pj, P.nx, P.ny, seed);
        ps.org = ld3(P.cam.eye);
        ps.d = 0;
        ps.nonfinite = false;
        has_path = true;
      }
    }
    ready_head += take;
    if (!__any(has_path) && ff_tail == ff_head) break;  // nothing live, nothing READY, nothing to fast-forward
    if (want_dbg) dbg[kDbgCyclesRefill] += __builtin_amdgcn_s_memtime() - tb;
    // ---- one depth of every live path ----
    bool ended = false;
    const unsigned long long ta = stamp(want_dbg);
    unsigned long long tbnc = ta;
    bool shade = has_path;
    if constexpr (kWalk) {
      const int nn = kLdsBvh ? sc->n_lw_nodes : sc->n_nodes;
      if (has_path && wni < 0) {  // a new ray: the quads first (their hit bounds the walk)
        wh = closest_hit<false, false>(sc, ps.org, ps.dir, true, nullptr, s_qshade + kPrexLdsOffset);
        wni = 0;
      }
      const uint64_t pm = __ballot(has_path);
      const int need = min(RTP_WALK_DONE, __popcll(pm));
      bool walking = has_path && wni < nn;
      if (__ballot(walking)) {
        const f3 o = ps.org, d = ps.dir;
        const BvhRay R = bvh_ray<kLdsBvh>(sc, o, d);
        GF4* __restrict__ geom_g = (GF4*)sc->sph_geom;
        // the LDS walk: this octant's copy of the nodes, then the leaf spheres
        LU4* const lnodes = (LU4*)s_bvh + (kLdsBvh ? ray_octant(d) * nn : 0);
        LF4* const lsph = (LF4*)s_bvh + (kLdsBvh ? 8 * nn : 0);
#ifndef RTP_BVH_NT
#define RTP_BVH_NT 0  // (experiment: the walk's node gathers as non-temporal loads)
#endif
        auto node = [&](int i) {
          if constexpr (kLdsBvh) return lnodes[i];
          else if constexpr (RTP_BVH_NT) return __builtin_nontemporal_load(R.nodes + i);
          else return R.nodes[i];
        };
        u4v v = u4v{0u, 0u, 0u, 0u};
        if (walking) v = node(wni);
        for (;;) {
          const uint64_t wm = __ballot(walking);
          if (wm == 0 || __popcll(pm & ~wm) >= need) break;
          if (walking) {
            const int next = bvh_visit<kLdsBvh>(geom_g, lsph, R, o, d, v, wni, wh);
            walking = next < nn;
            if (walking) v = node(next);
            wni = next;
          }
        }
        if (has_path && !walking) bvh_resolve(wh, R);
      }
      shade = has_path && !walking;
      if (want_dbg) dbg[kDbgCyclesIntersect] += stamp(want_dbg) - ta;
    }
    if (shade) {
      f3 emit = mk(0.f, 0.f, 0.f);
      int res;
      if constexpr (kWalk) {
        res = shade_hit<kBvh, true>(sc, ps, seed, emit, hist + (int64_t)ps.d * stride, D, s_qshade, wh,
                                    gdbg);  // (stats build: the region counters; nullptr otherwise)
        wni = -1;
      } else {
        res = bounce<kBvh, true>(sc, ps, seed, emit, hist + (int64_t)ps.d * stride, D, want_dbg ? dbg : nullptr,
                                 s_qshade, gdbg);
      }
      tbnc = stamp(want_dbg);
      if (res == kAlive && ps.d < D - 1) {
        ps.d++;
      } else {
        const int k_end = ps.d;
        if (want_dbg) dbg_region(gdbg, kDbgEndVisits);
        // the radiance product runs in the fast-forward batch (above)
        if (res == kLight) hist[(int64_t)k_end * stride] = make_float4(emit.x, emit.y, emit.z, 0.f);
        // dead depths left: D-1-k_end, plus depth k_end's own draws when the
        // path died there (bounce<.., true> left them to the fast-forward)
        const int rem = D - 1 - k_end + (res != kAlive ? 1 : 0);
        s_rem[slot] = (uint16_t)(rem | (res == kLight ? kEndLight : 0) | (ps.nonfinite ? kEndNonfinite : 0));
        s_samples[slot] = s_samples[slot] + 1u;
        s_live[slot] = s_live[slot] + (uint32_t)(k_end + 1);
        s_seed[slot] = seed;
        ended = true;
        has_path = false;
      }
    }
    if (want_dbg) {
      const unsigned long long te = __builtin_amdgcn_s_memtime();
      dbg[kDbgCyclesShade] += tbnc - ta;  // minus the intersect share, subtracted on the host
      dbg[kDbgCyclesEnd] += te - tbnc;
    }
    const uint64_t fin = __ballot(ended);
    if (ended) q_ff[(ff_tail + lane_rank(fin)) & (kPool - 1)] = (uint16_t)slot;
#if RTP_CRIT_FF > 0
    // A pixel whose finished samples lag the wave's average by more than
    // RTP_CRIT_FF/1000 runs its sample chain on the critical path (its path
    // length keeps it behind): its fast-forward is not left waiting for the
    // READY queue to run dry -- the batch runs in the next iteration.
    // (a scheduling heuristic: single precision is plenty; kSteal: fresh
    // pixels always lag, so no critical batches)
    if (!kSteal && __ballot(ended && (float)(s_samples[slot] * (uint32_t)n_slots) * 1000.0f <
                              (float)ff_tail * (float)(1000 - RTP_CRIT_FF)))
      critical_ff = true;
#endif
    ff_tail += __popcll(fin);
    wave_sync();
    if (RTP_PRIO_BALANCE && ff_tail - published >= (uint32_t)kPrioPeriod) {
      unsigned long long g = 0;
      if (lane == 0) g = atomicAdd(kparams().progress, (unsigned long long)(ff_tail - published));
      g = __shfl(g, 0) + (unsigned long long)(ff_tail - published);
      published = ff_tail;
      float lag;
      if constexpr (kSteal) {
        // remaining samples: this wave's (its held pixels') against the
        // average wave's, npix * S - g over the waves.  While unclaimed
        // entries remain, the average includes them and every wave sits
        // below it (priority 0: the stealing balances); once they are gone
        // the waves with the most work left get the issue slots.  In units
        // of a full pool's samples, like the fractions below.
        const float mine_left = (float)live_slots * (float)S - (float)(ff_tail - retired);
        const float avg_left = ((float)kparams().npix * (float)S - (float)g) / (float)n_waves;
        lag = (mine_left - avg_left) / ((float)kPool * (float)S);
      } else {
        // completed fractions: global g / (npix*S) vs own ff_tail / (n_slots*S)
        lag = ((float)g / (float)kparams().npix - (float)ff_tail / (float)n_slots) / (float)S;
      }
      set_priority(lag);
    }
    if (want_dbg && unfinished < 64) {
      if (t_tail == 0) t_tail = __builtin_amdgcn_s_memtime();
      dbg[kDbgTailSteps] += 1;
      dbg[kDbgTailLanes] += (unsigned long long)__popcll(__ballot(has_path || ended));
    }
    if (want_dbg) {
      dbg[kDbgBounceSteps] += 1;
      dbg[kDbgBounceLanes] += (unsigned long long)__popcll(__ballot(has_path || ended));
      dbg[kDbgCyclesBounce] += __builtin_amdgcn_s_memtime() - tb;
    }
  }
  if (!kStats && p.dbg && lane == 0)  // RTP_DEBUG_STATS=2: lifetime only
    p.dbg[(int64_t)w * kDbgCounters + kDbgRealEnd] = __builtin_amdgcn_s_memrealtime();
  if (want_dbg && lane == 0) {
    dbg[kDbgCyclesTotal] = __builtin_amdgcn_s_memtime() - t_start;
    dbg[kDbgRealEnd] = __builtin_amdgcn_s_memrealtime();
    dbg[kDbgTailCycles] = t_tail ? __builtin_amdgcn_s_memtime() - t_tail : 0;
    for (int c = 0; c < (kStats ? kDbgRefillVisits : 0); c++)  // (the later counters are accumulated in place)
      if (c != kDbgRealStart && c != kDbgHwId) p.dbg[(int64_t)w * kDbgCounters + c] = dbg[c];
  }
  wave_sync();
  for (int j = lane; j < (kSteal ? 0 : n_slots); j += 64) {  // (kSteal: written as they finished)
    const int64_t k = kPlan ? (int64_t)(wbase + j) : (int64_t)j * n_waves + w;
    reinterpret_cast<float4*>(p.out)[k] = make_float4(s_r[j], s_g[j], s_b[j], 0.f);
    if (p.seed_out) p.seed_out[k] = s_seed[j];
    if (p.live_out) p.live_out[k] = s_live[j];
  }
}

#if RTP_POOL_MAX_VGPR > 0
#define RTP_POOL_VGPR_ATTR __attribute__((amdgpu_num_vgpr(RTP_POOL_MAX_VGPR)))
#else
#define RTP_POOL_VGPR_ATTR
#endif
template <bool kStats, bool kBvh, bool kTiles = false, bool kPlan = false, bool kSteal = false>
__global__ void __launch_bounds__(256, RTP_POOL_MIN_WAVES_PER_EU) RTP_POOL_VGPR_ATTR
    rtp_render_pool(const DevScene* __restrict__ sc, KParams p, int n_waves) {
  __shared__ __align__(16) unsigned char smem[kPoolLdsBytes];
  __shared__ __align__(16) float s_qshade[kQTableFloats];
  if constexpr (kSteal) {
    __shared__ uint32_t s_entry[kWavesPerBlock * kPool];
    pool_body<kStats, kBvh, kTiles, kPlan, kWavesPerBlock, false, true>(sc, p, n_waves, smem, s_qshade, nullptr,
                                                                        s_entry);
  } else {
    pool_body<kStats, kBvh, kTiles, kPlan, kWavesPerBlock, false>(sc, p, n_waves, smem, s_qshade, nullptr);
  }
}

// Scenes whose LDS walk tree fits (DevScene::lw_nodes, rtp_lds_walk_capacity):
// one 16-wave block per CU (4 waves per SIMD, <= 128 VGPRs) shares one LDS
// copy of the tree -- dynamic LDS after the waves' pools, the quad tables and
// (kSteal) the slots' entries.
template <bool kTiles, bool kSteal>
__global__ void __launch_bounds__(64 * kLdsBvhWavesPerBlock, 1) __attribute__((amdgpu_num_vgpr(128)))
    rtp_render_pool_lds(const DevScene* __restrict__ sc, KParams p, int n_waves) {
  __shared__ __align__(16) unsigned char smem[kLdsBvhWavesPerBlock * kPool * kSlotBytes];
  __shared__ __align__(16) float s_qshade[kQTableFloats];
  extern __shared__ __align__(16) uint32_t s_dyn[];
  if constexpr (kSteal) {
    __shared__ uint32_t s_entry[kLdsBvhWavesPerBlock * kPool];
    pool_body<false, true, kTiles, false, kLdsBvhWavesPerBlock, true, true>(sc, p, n_waves, smem, s_qshade, s_dyn,
                                                                            s_entry);
  } else {
    pool_body<false, true, kTiles, false, kLdsBvhWavesPerBlock, true>(sc, p, n_waves, smem, s_qshade, s_dyn);
  }
}
constexpr int kLdsWalkStaticBytes =
    kLdsBvhWavesPerBlock * kPool * kSlotBytes + kQTableFloats * 4 + kLdsBvhWavesPerBlock * kPool * 4;
constexpr int kLdsWalkDynBytes = 160 * 1024 - kLdsWalkStaticBytes;  // the tree's share of the CU's 160 KiB
static_assert(kPool != 128 || kLdsWalkDynBytes >= 64 * 1024, "the LDS walk keeps room for a C3-size tree");

// ------------------------------------------------------- diagnostics ---
__global__ void rtp_eval_primitive_kernel(int kind, const void* in, void* out, int64_t n, const uint32_t* tab,
                                          uint32_t t1, uint32_t t2) {
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
    case 4: uo[i] = tab[ui[i]]; break;          // jump-table gather (ff16 / ff32)
    case 5: uo[i] = dead_step(ui[i], t1, t2); break;
    default: break;
  }
}

// closest_hit with and without the prefilter on a list of rays (o, d: 6
// floats each): out[7 i ..] = prefiltered (t bits, kind, idx), exact scan
// (t bits, kind, idx), 1 if the lane fell back to the exact scan.
template <bool kBvh>
__global__ void __launch_bounds__(256) rtp_eval_closest_kernel(const DevScene* __restrict__ sc,
                                                               const float* __restrict__ rays, uint32_t* out,
                                                               int64_t n) {
  __shared__ __align__(16) float s_qshade[kQTableFloats];
  fill_qshade(sc, s_qshade);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = rays + 6 * i;
  const f3 o = mk(r[0], r[1], r[2]), d = mk(r[3], r[4], r[5]);
  uint32_t full = 0;
  const Hit a = closest_hit<kBvh>(sc, o, d, true, &full, s_qshade + kPrexLdsOffset);
  const Hit b = closest_hit<kBvh>(sc, o, d, false, nullptr, nullptr);
  uint32_t* w = out + 7 * i;
  w[0] = __float_as_uint(a.t), w[1] = (uint32_t)a.kind, w[2] = (uint32_t)a.idx;
  w[3] = __float_as_uint(b.t), w[4] = (uint32_t)b.kind, w[5] = (uint32_t)b.idx;
  w[6] = full;
}

// RNG jump tables, all in one pass: thread s iterates the dead-step map from
// state s (= base + i) up to max_r steps and, after step r, stores the state
// into every table that tabulates r dead depths (out.t[r] != null: the chain
// tables for 32 / 16 / 8 / 4 ... depths and the direct tables of the counts
// a finished sample most often has).  The stores of a wave go to consecutive
// states, so each is one coalesced 256-byte write; the build costs max_r dead
// steps per state instead of the sum of every table's depth count.
__global__ void __launch_bounds__(256) rtp_build_ff_tables_kernel(FfBuildOut out, int max_r, uint32_t t1, uint32_t t2,
                                                                   uint64_t base, uint64_t count) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  uint32_t s = (uint32_t)(base + i);
  for (int r = 1; r <= max_r; r++) {
    s = dead_step(s, t1, t2);
    uint32_t* __restrict__ T = out.t[r];  // wave-uniform
    if (T != nullptr) T[base + i] = s;
  }
}

// Exhaustive equivalence check of a fast sequence against the IEEE operation
// for every float bit pattern in [lo, hi] (one lane per pattern).
__global__ void rtp_verify_fast_math_kernel(int kind, uint32_t lo, uint64_t count, unsigned long long* bad,
                                            uint32_t* first_bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t bits = lo + (uint32_t)i;
  const float x = __uint_as_float(bits);
  float want = 0.f, got = 0.f;
  switch (kind) {
    case 0: want = 1.0f / x; got = rcp_nr1(x); break;
    case 1: want = 1.0f / x; got = rcp_nr2(x); break;
    case 2: want = __builtin_sqrtf(x); got = sqrt_fast(x); break;
    case 3: want = 1.0f / __builtin_sqrtf(x); got = rcp_nr1(sqrt_fast(x)); break;
    case 4: want = 1.0f / __builtin_sqrtf(x); got = rcp_nr2(sqrt_fast(x)); break;
    case 5: want = (float)((double)x / kPi); got = cos_over_pi(x); break;
    case 6: { float s, c; rtp_sincosf(x, &s, &c); want = rtp_sinf(x); got = s; break; }
    case 7: { float s, c; rtp_sincosf(x, &s, &c); want = rtp_cosf(x); got = c; break; }
    case 8: {  // x as the divisor of div_markstein, 32 numerators spread over [-x, x] and beyond
      const float r = rcp_nr1(x);
      uint32_t h = bits;
      for (int k = 0; k < 32; k++) {
        h = wang(h + (uint32_t)k);
        const float a = x * ((float)(int32_t)h * 0x1p-31f) * (k < 24 ? 1.0f : 1024.0f);
        const float w = a / x, g = div_markstein(a, x, r);
        if (__float_as_uint(w) != __float_as_uint(g) && fabsf(w) >= 0x1p-120f) {  // (normal quotients)
          want = w;
          got = g;
          break;
        }
      }
      break;
    }
    default: break;
  }
  if (__float_as_uint(want) != __float_as_uint(got)) {
    atomicAdd(bad, 1ull);
    atomicMin(first_bad, bits);
  }
}

}  // namespace rtp

// ----------------------------------------------------------- launchers ---
extern "C" hipError_t rtp_launch_verify_fast_math(int kind, uint32_t lo, uint64_t count, unsigned long long* bad,
                                                  uint32_t* first_bad, hipStream_t stream) {
  const int block = 256;
  const uint64_t grid = (count + block - 1) / block;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(rtp::rtp_verify_fast_math_kernel, dim3((unsigned)grid), dim3(block), 0, stream, kind, lo, count,
                     bad, first_bad);
  return hipGetLastError();
}
namespace {
template <bool kStats, bool kBvh>
int resident_blocks_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rtp::rtp_render_pool<kStats, kBvh>, 256, 0) != hipSuccess ||
      nb <= 0)
    nb = 1;
  return nb;
}
// (the occupancy of the LDS walk's instances at the largest tree: one block
// per CU; also sets their dynamic-LDS limit)
int lds_bvh_resident_blocks_per_cu() {
  static int cached = -1;
  if (cached > 0) return cached;
  const int dyn = rtp::kLdsWalkDynBytes;
  const void* k[4] = {reinterpret_cast<const void*>(rtp::rtp_render_pool_lds<false, false>),
                      reinterpret_cast<const void*>(rtp::rtp_render_pool_lds<true, false>),
                      reinterpret_cast<const void*>(rtp::rtp_render_pool_lds<false, true>),
                      reinterpret_cast<const void*>(rtp::rtp_render_pool_lds<true, true>)};
  for (const void* f : k) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, dyn);
  auto occ = [dyn](auto kernel) {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, 64 * rtp::kLdsBvhWavesPerBlock, dyn) != hipSuccess ||
        b <= 0)
      b = 1;
    return b;
  };
  const int nb = std::min(std::min(occ(rtp::rtp_render_pool_lds<false, false>), occ(rtp::rtp_render_pool_lds<true, false>)),
                          std::min(occ(rtp::rtp_render_pool_lds<false, true>), occ(rtp::rtp_render_pool_lds<true, true>)));
  cached = nb;
  return cached;
}
// bvh: 0 no sphere BVH, 1 the global threaded walk, 2 the LDS walk
int pool_resident_waves(bool stats, int bvh) {
  static int cached[2][3] = {{-1, -1, -1}, {-1, -1, -1}};
  int& c = cached[stats][bvh];
  if (c > 0) return c;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (bvh == 2) {
    c = cus * lds_bvh_resident_blocks_per_cu() * rtp::kLdsBvhWavesPerBlock;
    return c;
  }
  const int nb = stats ? (bvh ? resident_blocks_per_cu<true, true>() : resident_blocks_per_cu<true, false>())
                       : (bvh ? resident_blocks_per_cu<false, true>() : resident_blocks_per_cu<false, false>());
  c = cus * nb * rtp::kWavesPerBlock;
  if (const char* v = getenv("RTP_VERBOSE")) {
    if (v[0] == '1') {
      int lds_cu = 0;
      (void)hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
      hipFuncAttributes fa{};
      (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(rtp::rtp_render_pool<false, false>));
      fprintf(stderr, "rtp: pool kernel %d CUs x %d blocks of %d waves; LDS %zu B per block, %d B per CU; %d VGPRs\n",
              cus, nb, rtp::kWavesPerBlock, (size_t)fa.sharedSizeBytes, lds_cu, fa.numRegs);
    }
  }
  return c;
}
int kernel_variant() {
  const char* e = getenv("RTP_KERNEL");
  if (e && e[0] == '1') return 1;
  return 2;
}
}  // namespace

// Work plan: how many lanes' worth of attenuation history the launch needs.
extern "C" int64_t rtp_plan_history_lanes(int64_t npix, int spp, int bvh, int* variant_out, int* waves_out) {
  const int v = kernel_variant();
  if (variant_out) *variant_out = v;
  if (v == 1) {
    if (waves_out) *waves_out = (int)((npix + 63) / 64);
    return npix;
  }
  // pixels per wave when the launch cannot fill every resident wave: 80, so
  // that a lane often serves two pixels (the cheap pixels fill the lanes the
  // expensive ones' sample chains leave idle) while the waves per SIMD stay
  // few (each step of a chain is faster).  Rank 0's share of the C2 frame
  // under the N-rank tile deal, kernel ms (r03k/l, profiles/r03k_*):
  //   px/wave:  64    80    96    112   128
  //   N = 2:    95.5  83.6  86.5  79.0  88.7
  //   N = 4:    74.0  64.4  65.1  69.0  73.8
  //   N = 8:    58.7  58.6  59.2   --   65.0
  // (non-monotone: which pixels share a wave decides its longest chain).
  // Below a third of the resident waves at 64 pixels (C1, the 1/8 share)
  // the steps already run at one wave's latency: fewer waves gain nothing,
  // and a second pixel on a lane only lengthens its chain (C1: 0.70 -> 0.80
  // ms at 80), so such launches keep 64.  RTP_WAVE_PIXELS overrides
  // (experiments).
  // Long chains (spp >= 2048) on a share that fills 1.5-2.5 waves per SIMD
  // at 128 pixels per wave take 128: every pixel's chain is then ~2x the
  // average sample chain of a lane's two pixels, so the lanes stay full, and
  // fewer waves per SIMD make each step of the longest chains faster (the
  // per-step cost rises ~2.5 k cycles per extra wave on a SIMD, 13 k alone:
  // tools/lat_bench.hip).  C4's 1/8 share (259 200 pixels, 4096 spp), kernel
  // ms (r04c): 80 px/wave 388, 96 323, 112 354, 128 310.  C2's shares keep
  // 64/80 (1000 spp: 128 px/wave was 9-10% slower at N = 2, 4, 8).
  const char* st = getenv("RTP_DEBUG_STATS");
  const int64_t resident = pool_resident_waves(st && st[0] == '1', bvh);
  const int64_t simds = std::max<int64_t>(1, resident / RTP_POOL_MIN_WAVES_PER_EU);
  int wave_px = (npix + 63) / 64 * 3 < resident ? 64 : 80;
  if (spp >= 2048 && npix * 2 >= simds * 128 * 3 && npix * 2 <= simds * 128 * 5) wave_px = 128;
  if (const char* e = getenv("RTP_WAVE_PIXELS")) wave_px = std::max(1, std::min(rtp::kPool, atoi(e)));
  const int64_t by_lanes = (npix + wave_px - 1) / wave_px;
  const int64_t by_pool = (npix + rtp::kPool - 1) / rtp::kPool;
  int64_t W = std::min<int64_t>(by_lanes, resident);
  W = std::max<int64_t>(W, by_pool);
  W = std::max<int64_t>(W, 1);
  if (waves_out) *waves_out = (int)W;
  return W * rtp::kPool;
}

// Waves of the stealing instances that fit the chip at once: their own
// occupancy (the s_entry table adds 2 KiB of LDS per block), the smaller of
// the contiguous / pixel-list and tile-deal instances.  A stealing launch
// larger than this would leave blocks waiting for a free CU, and their
// statically assigned first entries would run as a tail after the stolen work.
namespace {
template <bool kBvh>
int steal_blocks_per_cu() {
  int a = 0, b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, rtp::rtp_render_pool<false, kBvh, false, false, true>, 256, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rtp::rtp_render_pool<false, kBvh, true, false, true>, 256, 0) !=
          hipSuccess)
    return 1;
  return std::max(1, std::min(a, b));
}
int steal_resident_waves(int bvh) {
  static int cached[2] = {-1, -1};
  int& c = cached[bvh ? 1 : 0];
  if (c > 0) return c;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  c = cus * (bvh ? steal_blocks_per_cu<true>() : steal_blocks_per_cu<false>()) * rtp::kWavesPerBlock;
  return c;
}
}  // namespace

// Work stealing (pool_body kSteal) when a launch's entries exceed what the
// resident waves' pools hold: the resident waves, each refilling its slots
// from the unclaimed entries.  Returns the waves (0: no stealing).
extern "C" int rtp_plan_steal(int64_t npix, int bvh) {
  const int64_t resident = pool_resident_waves(false, bvh);
  if (npix <= resident * rtp::kPool) return 0;
  if (bvh == 2) return (int)resident;  // (its instances' occupancy: lds_bvh_resident_blocks_per_cu)
  return std::min<int>((int)resident, steal_resident_waves(bvh));
}

// Bytes of LDS the LDS walk's tree may take (nodes of 8 octant copies plus
// the leaf spheres, 16 B each): what the 16-wave block leaves of the CU's 160 KiB.
extern "C" int rtp_lds_walk_capacity(void) { return std::max(0, rtp::kLdsWalkDynBytes); }

extern "C" hipError_t rtp_launch_eval_closest(const rtp::DevScene* scene, const float* rays, uint32_t* out,
                                              int64_t n, int bvh, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  if (bvh) hipLaunchKernelGGL(rtp::rtp_eval_closest_kernel<true>, g, b, 0, stream, scene, rays, out, n);
  else hipLaunchKernelGGL(rtp::rtp_eval_closest_kernel<false>, g, b, 0, stream, scene, rays, out, n);
  return hipGetLastError();
}
extern "C" hipError_t rtp_launch_render(const rtp::DevScene* scene, const rtp::KParams* p, int variant, int waves,
                                        int bvh, hipStream_t stream, int lds_bytes) {
  if (p->npix <= 0) return hipSuccess;
  if (variant == 1 && p->tile_world > 0) return hipErrorNotSupported;  // (v1 takes pixel lists or ranges)
  if (variant == 1) {
    const int64_t grid = (p->npix + 255) / 256;
    if (bvh)
      hipLaunchKernelGGL(rtp::rtp_render_lockstep<true>, dim3((unsigned)grid), dim3(256), 0, stream, scene, *p);
    else
      hipLaunchKernelGGL(rtp::rtp_render_lockstep<false>, dim3((unsigned)grid), dim3(256), 0, stream, scene, *p);
  } else if (bvh == 2) {  // the sphere BVH walked out of LDS
    if (p->wave_begin || lds_bytes <= 0 || lds_bytes > rtp::kLdsWalkDynBytes) return hipErrorNotSupported;
    (void)lds_bvh_resident_blocks_per_cu();  // (sets the kernels' dynamic-LDS limit once)
    const int blocks = (waves + rtp::kLdsBvhWavesPerBlock - 1) / rtp::kLdsBvhWavesPerBlock;
    const dim3 g((unsigned)blocks), b(64 * rtp::kLdsBvhWavesPerBlock);
    const size_t dyn = (size_t)lds_bytes;
    const bool steal = (int64_t)waves * rtp::kPool < p->npix;  // rtp_plan_steal
    if (steal && p->tile_world > 0) hipLaunchKernelGGL((rtp::rtp_render_pool_lds<true, true>), g, b, dyn, stream, scene, *p, waves);
    else if (steal) hipLaunchKernelGGL((rtp::rtp_render_pool_lds<false, true>), g, b, dyn, stream, scene, *p, waves);
    else if (p->tile_world > 0) hipLaunchKernelGGL((rtp::rtp_render_pool_lds<true, false>), g, b, dyn, stream, scene, *p, waves);
    else hipLaunchKernelGGL((rtp::rtp_render_pool_lds<false, false>), g, b, dyn, stream, scene, *p, waves);
  } else {
    const int blocks = (waves + rtp::kWavesPerBlock - 1) / rtp::kWavesPerBlock;
    const char* st = getenv("RTP_DEBUG_STATS");
    const bool stats = p->dbg && st && st[0] == '1';
    const dim3 g((unsigned)blocks), b(256);
    if (p->wave_begin) {  // a planned launch (pixel list or range, no BVH)
      if (bvh || p->tile_world > 0) return hipErrorNotSupported;
      if (stats) hipLaunchKernelGGL((rtp::rtp_render_pool<true, false, false, true>), g, b, 0, stream, scene, *p, waves);
      else hipLaunchKernelGGL((rtp::rtp_render_pool<false, false, false, true>), g, b, 0, stream, scene, *p, waves);
    } else if ((int64_t)waves * rtp::kPool < p->npix) {  // more entries than slots: work stealing (rtp_plan_steal)
      if (stats) return hipErrorNotSupported;
      if (p->tile_world > 0) {
        if (bvh) hipLaunchKernelGGL((rtp::rtp_render_pool<false, true, true, false, true>), g, b, 0, stream, scene, *p, waves);
        else hipLaunchKernelGGL((rtp::rtp_render_pool<false, false, true, false, true>), g, b, 0, stream, scene, *p, waves);
      } else {
        if (bvh) hipLaunchKernelGGL((rtp::rtp_render_pool<false, true, false, false, true>), g, b, 0, stream, scene, *p, waves);
        else hipLaunchKernelGGL((rtp::rtp_render_pool<false, false, false, false, true>), g, b, 0, stream, scene, *p, waves);
      }
    } else if (p->tile_world > 0) {  // the tile deal: its own instances, no stats variant
      if (bvh) hipLaunchKernelGGL((rtp::rtp_render_pool<false, true, true>), g, b, 0, stream, scene, *p, waves);
      else hipLaunchKernelGGL((rtp::rtp_render_pool<false, false, true>), g, b, 0, stream, scene, *p, waves);
    } else if (stats && bvh) hipLaunchKernelGGL((rtp::rtp_render_pool<true, true>), g, b, 0, stream, scene, *p, waves);
    else if (stats) hipLaunchKernelGGL((rtp::rtp_render_pool<true, false>), g, b, 0, stream, scene, *p, waves);
    else if (bvh) hipLaunchKernelGGL((rtp::rtp_render_pool<false, true>), g, b, 0, stream, scene, *p, waves);
    else hipLaunchKernelGGL((rtp::rtp_render_pool<false, false>), g, b, 0, stream, scene, *p, waves);
  }
  return hipGetLastError();
}

extern "C" hipError_t rtp_launch_build_ff_tables(const rtp::FfBuildOut* out, int max_r, uint32_t t1, uint32_t t2,
                                                 hipStream_t stream) {
  if (max_r < 1 || max_r >= rtp::kFfMaxSteps) return hipErrorInvalidValue;
  const uint64_t total = 1ull << 32, chunk = 1ull << 30;
  for (uint64_t base = 0; base < total; base += chunk) {
    hipLaunchKernelGGL(rtp::rtp_build_ff_tables_kernel, dim3((unsigned)(chunk / 256)), dim3(256), 0, stream, *out,
                       max_r, t1, t2, base, chunk);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

extern "C" hipError_t rtp_launch_eval_primitive(int kind, const void* in, void* out, int64_t n, const uint32_t* tab,
                                                uint32_t t1, uint32_t t2, hipStream_t stream) {
  const int block = 256;
  const int64_t grid = (n + block - 1) / block;
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(rtp::rtp_eval_primitive_kernel, dim3((unsigned)grid), dim3(block), 0, stream, kind, in, out, n,
                     tab, t1, t2);
  return hipGetLastError();
}
