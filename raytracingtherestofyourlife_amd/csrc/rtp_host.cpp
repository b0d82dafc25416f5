// rtp_host.cpp -- host side of librtp.so: the C ABI declared in include/rtp.h.
//
// Mirrors vtkm::rendering::MapperPathTracer (MapperPathTracer.cxx:94-538):
// the scene/material tables, the camera set-up of pathtracing::Camera
// (Camera.cxx:437-474, 624-776, 879-960) and the render entry point.  All
// ray-independent quantities are precomputed here with the reference's own
// float operations (compiled with -ffp-contract=off; x86-64 SSE2 arithmetic
// is IEEE single/double, the same as the reference's g++ build).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rtp.h"
#include "rtp_context.hpp"
#include "rtp_layout.hpp"

extern "C" int64_t rtp_plan_history_lanes(int64_t npix, int spp, int bvh, int* variant_out, int* waves_out);
extern "C" int rtp_plan_steal(int64_t npix, int bvh);
extern "C" hipError_t rtp_launch_render(const rtp::DevScene* scene, const rtp::KParams* p, int variant, int waves, int bvh,
                                        hipStream_t stream, int lds_bytes);
extern "C" int rtp_lds_walk_capacity(void);
extern "C" hipError_t rtp_launch_eval_primitive(int kind, const void* in, void* out, int64_t n, const uint32_t* tab,
                                                uint32_t t1, uint32_t t2, hipStream_t stream);
extern "C" hipError_t rtp_launch_build_ff_tables(const rtp::FfBuildOut* out, int max_r, uint32_t t1, uint32_t t2,
                                                 hipStream_t stream);
extern "C" hipError_t rtp_compact_bvh(const rtp::BvhNode* d_nodes, int64_t total, uint32_t* d_cn, int32_t* d_cidx,
                                      hipStream_t stream);
extern "C" hipError_t rtp_build_bvh_gpu(const float4* d_cr, int n, float3 lo, float3 ext, rtp::BvhNode* d_nodes,
                                        rtp::DevSphereG* d_geom, hipStream_t stream);
extern "C" hipError_t rtp_launch_eval_closest(const rtp::DevScene* scene, const float* rays, uint32_t* out,
                                              int64_t n, int bvh, hipStream_t stream);
extern "C" hipError_t rtp_launch_verify_fast_math(int kind, uint32_t lo, uint64_t count, unsigned long long* bad,
                                                  uint32_t* first_bad, hipStream_t stream);

namespace {

thread_local std::string g_err;

rtp_status fail(rtp_status st, const std::string& msg) {
  g_err = msg;
  return st;
}
rtp_status hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? RTP_ERR_OUT_OF_MEMORY : RTP_ERR_DEVICE,
              std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr)                                 \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

// ---------------------------------------------------- host vector math ---
struct v3 {
  float x, y, z;
};
inline v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline v3 scl(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline v3 cross(v3 a, v3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float rmag(v3 a) { return 1 / std::sqrt(dot(a, a)); }
inline v3 normalize(v3 a) { return scl(a, rmag(a)); }  // vtkm::Normalize (CPU build)
inline v3 ld(const float* p) { return {p[0], p[1], p[2]}; }
inline void st(float* d, v3 a) { d[0] = a.x, d[1] = a.y, d[2] = a.z; }

// which = min(3, int(r*3+1)), r = float(t)/4294967295.f  (PdfWorklet.h:20)
int which_of_hash(uint32_t t) {
  float r = (float)t / 4294967295.f;
  int w = (int)(r * 3 + 1);
  return w < 3 ? w : 3;
}
// smallest hash value with which >= w (which is monotone in t)
uint32_t which_threshold(int w) {
  uint64_t lo = 0, hi = 0x100000000ull;  // answer in [lo, hi]
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (which_of_hash((uint32_t)mid) >= w)
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo > 0xffffffffull ? 0xffffffffu : (uint32_t)lo;
}

void fill_quad(rtp::DevQuad& Q, v3 q, v3 r, v3 s, v3 t) {
  std::memset(&Q, 0, sizeof(Q));
  for (int k = 0; k < 3; k++) Q.vv[k][0] = (&q.x)[k], Q.vv[k][1] = (&s.x)[k];
  st(Q.e01, sub(r, q));
  st(Q.e03, sub(t, q));
  st(Q.e21, sub(r, s));
  st(Q.e23, sub(t, s));
  st(Q.n, normalize(cross(sub(r, q), sub(s, q))));  // TriangleNormal(q,r,s), Surface.h:182-183
  // zero-structure kind (exact zeros only; see quad_hit_masked)
  auto mask_of = [](const float* e) {
    int m = 0;
    for (int k = 0; k < 3; k++)
      if (e[k] != 0.0f) m |= 1 << k;
    return m;
  };
  const int m01 = mask_of(Q.e01), m03 = mask_of(Q.e03), m21 = mask_of(Q.e21), m23 = mask_of(Q.e23);
  // exact parallelogram (see quad_hit_masked): value equality; the sign of a
  // zero component only ever changes the sign of a zero intermediate
  Q.para = 1;
  for (int k = 0; k < 3; k++)
    if (!(-Q.e01[k] == Q.e23[k] && -Q.e03[k] == Q.e21[k])) Q.para = 0;
  Q.kind = 0;
  for (int k = 1; k < rtp::kQuadKinds; k++) {
    const rtp::QuadKindMasks& K = rtp::kQuadKind[k];
    if (K.m01 == m01 && K.m03 == m03 && K.m21 == m21 && K.m23 == m23) Q.kind = k;
  }
  // Kinds 1..6 are axis-plane rectangles: their masks force s = (r_I, t_J),
  // so e23 == -e01 and e21 == -e03 exactly and they are always exact
  // parallelograms (the prefilter's exact test, quad_hit_axis, relies on it;
  // setup_prefilter re-checks Q.para).  An in-plane quad that is not a
  // parallelogram has a non-rectangular mask set and is kind 0.
}

bool bit_equal(const float* a, const float* b, int n) { return std::memcmp(a, b, sizeof(float) * n) == 0; }

// Closest-hit prefilter tables (rtp_kernels.hip closest_hit):
// the quads of groups 0..5 (kinds 1..6, edges along two axes) lie in a plane
// x[axis] = const, bit for bit.  Each gets that plane and a box around its
// vertices in the other two coordinates, widened outward by a few ulps so
// that the float box contains the real one.  Enabled only when every such
// quad qualifies, they fit kMaxPre, and the scene is within the coordinate
// range the kernel's error margins assume (|x| <= kPreLim).
constexpr float kPreLim = 16.0f;
void setup_prefilter(rtp::DevScene* h, const rtp_scene_desc* s, const std::vector<int>& kept) {
  h->n_pre = 0;
  for (int a = 0; a <= 3; a++) h->pre_begin[a] = 0;
  h->pre_scale = 0.0f;
  const int n = h->kind_begin[6];
  if (n <= 0 || n > rtp::kMaxPre) return;
  const char* e = getenv("RTP_PREFILTER");
  if (e && e[0] == '0') return;
  std::vector<int> axis_of(n);
  std::vector<rtp::PreQuad> pq(n);
  float scale = 0.0f;
  for (int q = 0; q < n; q++) {
    const rtp::DevQuad& Q = h->quads[q];
    const rtp::QuadKindMasks& K = rtp::kQuadKind[Q.kind];
    const int flat = 7 & ~(K.m01 | K.m03);
    if (Q.kind < 1 || Q.kind > 6 || (flat != 1 && flat != 2 && flat != 4)) return;
    const int a = flat == 1 ? 0 : flat == 2 ? 1 : 2, b = (a + 1) % 3, c = (a + 2) % 3;
    if (!Q.para) return;  // (unreachable: kinds 1..6 are exact parallelograms, see fill_quad)
    {
      const int ei = K.m01 == 1 ? 0 : K.m01 == 2 ? 1 : 2, ej = K.m03 == 1 ? 0 : K.m03 == 2 ? 1 : 2;
      const int ea = 3 - ei - ej;
      rtp::PreExact& E = h->prex[q];
      std::memset(&E, 0, sizeof(E));
      E.i = ei;
      E.s = (ej == (ei + 1) % 3) ? 1 : -1;
      E.b = Q.e01[ei], E.c = Q.e03[ej];
      E.bs = E.s > 0 ? E.b : -E.b, E.cs = E.s > 0 ? E.c : -E.c;
      E.vi = Q.vv[ei][0], E.va = Q.vv[ea][0], E.vj = Q.vv[ej][0];
      E.wi = Q.vv[ei][1], E.wa = Q.vv[ea][1], E.wj = Q.vv[ej][1];
      E.key_lo = Q.key_lo;
    }
    const int32_t* id = s->quad_points + 4 * kept[Q.orig];
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    const float x = s->points[3 * id[0] + a];
    for (int k = 0; k < 4; k++) {
      const float* v = s->points + 3 * id[k];
      if (!(v[a] == x)) return;  // not in one axis plane
      for (int j = 0; j < 3; j++) {
        if (!std::isfinite(v[j])) return;
        lo[j] = std::min(lo[j], (double)v[j]);
        hi[j] = std::max(hi[j], (double)v[j]);
        scale = std::max(scale, std::fabs(v[j]));
      }
    }
    auto centre_half = [&](int j, float& cen, float& half) {
      cen = (float)(0.5 * (lo[j] + hi[j]));
      const double need = std::max(hi[j] - (double)cen, (double)cen - lo[j]);
      half = (float)need;
      for (int u = 0; u < 2; u++) half = std::nextafter(half, INFINITY);  // >= need after rounding
    };
    rtp::PreQuad& P = pq[q];
    std::memset(&P, 0, sizeof(P));
    P.x = x;
    centre_half(b, P.cb, P.rb);
    centre_half(c, P.cc, P.rc);
    P.qpos = q;
    axis_of[q] = a;
  }
  if (!(scale <= kPreLim)) return;
  int pos = 0;
  for (int a = 0; a < 3; a++) {
    h->pre_begin[a] = pos;
    for (int q = 0; q < n; q++)
      if (axis_of[q] == a) h->pre[pos++] = pq[q];
  }
  h->pre_begin[3] = pos;
  h->pre_scale = scale;
  h->n_pre = n;
}

// RNG jump tables.  A dead depth consumes 1 + {2,3,2} draws chosen by the
// `which` draw against two constant thresholds (lightables = 2,
// MapperPathTracer.cxx:218; PdfWorklet.h:20), so "advance the state over k
// dead depths" is a fixed map of the 32-bit state.  Chain table j tabulates
// it for k = 32 >> j over all 2^32 states (16 GiB each), and the direct
// tables for each k in [d_first, d_first + d_count): a finished sample whose
// remaining count falls in the direct block is fast-forwarded by ONE gather,
// others by a chain of gathers plus a few hashed depths (rtp_render_pool).
// Defaults: 4 chain tables (32, 16, 8, 4) and direct tables 41..50 (the
// counts a depth-50 render's samples mostly have), 224 GiB in all;
// RTP_FF_TABLES=n (0..6) / RTP_FF_DIRECT=n / RTP_FF_DIRECT_FIRST=r change
// the set, and it shrinks to the free device memory (8 GiB kept free).
// The tables are per device and process, shared by every context, and built
// by the policy of rtp_set_ff_tables (include/rtp.h): what they cost
// (allocation + build, measured here) against what they save per sample.
struct FfTables {
  uint32_t* t[rtp::kFfTables] = {};
  uint32_t* direct = nullptr;  // d_count tables of 2^32 entries, contiguous
  int d_first = 0, d_count = 0, n_chain = 0;
  int stage = 0;  // built so far: 1 chain tables, 2 + direct tables
  double alloc_ms = 0, build_ms = 0;
  double chain_alloc_ms = -1;  // the chain stage's own allocation time (-1: not built)
  uint64_t chain_at = 0;       // samples_seen when the chain stage was built
  uint64_t bytes = 0;
  uint64_t samples_seen = 0;  // samples launched on this device (the AUTO policy's count)
};
std::mutex g_ff_mu;
FfTables g_ff[64];

int ff_policy_default() {
  const char* e = getenv("RTP_FF_POLICY");
  if (e && !std::strcmp(e, "on")) return RTP_FF_TABLES_ON;
  if (e && !std::strcmp(e, "off")) return RTP_FF_TABLES_OFF;
  return RTP_FF_TABLES_AUTO;
}

// AUTO builds in two stages, each once the samples launched on the device
// (this launch included) reach its break-even count: setup time over the
// kernel time it saves per sample (C2 on MI355X; round 5,
// profiles/r05z_ff_policy.txt: no tables 126.0 ms, chain tables 106.8 ms,
// all 98.9 ms per 6.4e8 samples):
//  - chain tables (64 GiB): 0.12 s build + an allocation that takes 1 ms to
//    ~1.5 s depending on the box (the driver clearing the memory), saving
//    3.0e-11 s/sample: 7.5e9 samples, ~12 C2 renders (allows ~0.1 s of
//    allocation);
//  - direct tables (+160 GiB): 0.07 s more build + 2.5x the chain stage's
//    measured allocation time, saving 1.23e-11 s/sample: counted from the
//    chain stage, ~9 C2 renders where allocation is fast, ~450 where the
//    chain's 64 GiB took 1.4 s; 3e11 samples before the chain stage is built.
// RTP_FF_AUTO_SAMPLES=chain[,direct] overrides (absolute counts).
constexpr double kFfChainSavePerSample = 3.0e-11, kFfDirectSavePerSample = 1.23e-11;
constexpr double kFfDirectBuildS = 0.07, kFfDirectAllocRatio = 160.0 / 64.0;
void ff_auto_samples(uint64_t& chain, uint64_t& direct, const FfTables* T = nullptr) {
  chain = 7500000000ull;
  direct = 300000000000ull;
  if (const char* e = getenv("RTP_FF_AUTO_SAMPLES")) {
    char* end = nullptr;
    chain = std::strtoull(e, &end, 10);
    direct = (end && *end == ',') ? std::strtoull(end + 1, nullptr, 10) : chain;
    return;
  }
  if (T && T->chain_alloc_ms >= 0) {
    const double setup_s = kFfDirectBuildS + kFfDirectAllocRatio * T->chain_alloc_ms / 1e3;
    direct = std::min<uint64_t>(direct, T->chain_at + (uint64_t)(setup_s / kFfDirectSavePerSample));
  }
  (void)kFfChainSavePerSample;
}

// Allocate and build the tables of a device up to `stage` (caller holds
// g_ff_mu): 1 the chain tables, 2 also the direct block.  The new tables are
// allocated and built through local pointers and published into T only once
// the build kernel has finished: a launch that took its snapshot (FfSnap)
// earlier, and may still be running on another stream, never sees a table
// that is half built, and a failed build frees only what it allocated.
void ff_build(FfTables& T, int stage) {
  if (T.stage >= stage) return;
  int want = 4, nd = 10, first = 41;
  if (const char* env = getenv("RTP_FF_TABLES")) want = std::max(0, std::min(rtp::kFfTables, atoi(env)));
  if (const char* env = getenv("RTP_FF_DIRECT")) nd = std::max(0, std::min(32, atoi(env)));
  if (const char* env = getenv("RTP_FF_DIRECT_FIRST")) first = std::max(1, atoi(env));
  if (first + nd > rtp::kFfMaxSteps) nd = std::max(0, rtp::kFfMaxSteps - first);
  if (want == 0) nd = 0;  // (RTP_FF_TABLES=0: no tables at all)
  const size_t bytes = (size_t)4 << 32, reserve = 8ull << 30;
  auto fits = [&](size_t n) {
    size_t free_b = 0, total_b = 0;
    return hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b >= n + reserve;
  };
  rtp::FfBuildOut out{};
  uint32_t* chain[rtp::kFfTables] = {};
  uint32_t* direct = nullptr;
  int n_chain = 0, d_count = 0;
  int max_r = 0;
  const auto t0 = std::chrono::steady_clock::now();
  if (T.stage < 1) {
    for (int j = 0; j < want; j++) {
      if (!fits(bytes) || hipMalloc(&chain[j], bytes) != hipSuccess) {
        chain[j] = nullptr;
        break;
      }
      n_chain = j + 1;
      out.t[32 >> j] = chain[j];
      max_r = std::max(max_r, 32 >> j);
    }
  }
  if (stage >= 2 && nd > 0) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
      nd = std::min<int>(nd, free_b > reserve ? (int)((free_b - reserve) / bytes) : 0);
    else
      nd = 0;
    if (nd > 0 && hipMalloc(&direct, bytes * (size_t)nd) == hipSuccess) {
      d_count = nd;
      for (int k = 0; k < nd; k++) {
        out.t[first + k] = direct + (size_t)k * (bytes / 4);
        max_r = std::max(max_r, first + k);
      }
    } else {
      direct = nullptr;
    }
  }
  (void)hipGetLastError();
  const double alloc_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  T.alloc_ms += alloc_ms;
  if (T.stage < 1 && stage == 1 && n_chain > 0) {  // the AUTO policy's estimate of the direct stage's cost
    T.chain_alloc_ms = alloc_ms;
    T.chain_at = T.samples_seen;
  }
  T.stage = stage;  // (a failed stage is not retried)
  if (max_r > 0) {
    const uint32_t t1 = which_threshold(2), t2 = which_threshold(3);
    hipEvent_t a = nullptr, b = nullptr;
    bool ok = hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess;
    ok = ok && hipEventRecord(a, nullptr) == hipSuccess;
    ok = ok && rtp_launch_build_ff_tables(&out, max_r, t1, t2, nullptr) == hipSuccess;
    ok = ok && hipEventRecord(b, nullptr) == hipSuccess && hipEventSynchronize(b) == hipSuccess;
    float ms = 0;
    if (ok) (void)hipEventElapsedTime(&ms, a, b);
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    (void)hipGetLastError();
    if (!ok) {  // nothing was published: free this stage's own allocations
      for (uint32_t* p : chain)
        if (p) (void)hipFree(p);
      if (direct) (void)hipFree(direct);
      return;
    }
    T.build_ms += ms;
  }
  // publish (the build has completed)
  for (int j = 0; j < n_chain; j++) T.t[j] = chain[j];
  if (n_chain > 0) T.n_chain = n_chain;
  if (d_count > 0) {
    T.direct = direct;
    T.d_first = first;
    T.d_count = d_count;
  }
  T.bytes = bytes * (size_t)(T.n_chain + T.d_count);
}

// What one launch reads of a device's tables: a copy taken under g_ff_mu,
// so a later stage being built by another thread cannot change it.
struct FfSnap {
  const uint32_t* t[rtp::kFfTables] = {};
  const uint32_t* direct = nullptr;
  int d_first = 0, d_count = 0;
};

// The tables a launch of `samples` samples on `device` uses under `policy`
// (built first when the policy says so).  The tables, once published, stay
// until the process ends.
FfSnap ff_tables(int device, int policy, uint64_t samples) {
  std::lock_guard<std::mutex> lk(g_ff_mu);
  FfTables& T = g_ff[device & 63];
  T.samples_seen += samples;
  if (policy == RTP_FF_TABLES_ON) {
    ff_build(T, 2);
  } else if (policy == RTP_FF_TABLES_AUTO) {
    uint64_t chain = 0, direct = 0;
    ff_auto_samples(chain, direct, &T);
    if (T.samples_seen >= direct) ff_build(T, 2);
    else if (T.samples_seen >= chain) ff_build(T, 1);
  }
  FfSnap s;
  if (policy == RTP_FF_TABLES_OFF) return s;
  for (int j = 0; j < rtp::kFfTables; j++) s.t[j] = T.t[j];
  s.direct = T.direct;
  s.d_first = T.d_first;
  s.d_count = T.d_count;
  return s;
}

// Sphere BVH (replaces the VTK-m LinearBVH of buildBVH, MapperPathTracer.cxx:
// 437-449, for scenes with many spheres).  Binned SAH (16 bins per axis) with
// deterministic partitions, leaves of <= kBvhLeafSize spheres.  The tree is
// flattened eight times, once per ray-direction octant: each copy is a
// depth-first "threaded" array (hit: next node; miss or leaf done: skip) that
// visits the child on the near side of the split axis first, so a lane walks
// near-to-far without a stack and the closest-hit bound culls early.  Boxes
// only cull: each sphere box is padded by 0.2% of its radius + 1e-5 so that
// every point the device's float sphere test can return lies inside it, and
// the kernel compares against a slack-widened [0, t_best] interval.  The
// closest hit is the lexicographic min of (t, kind, index) whatever the order.
struct BvhPrim {
  float lo[3], hi[3], cen[3];
  int32_t idx;
};
struct TNode {
  float lo[3], hi[3];
  int axis = 0, left = -1, right = -1, first = 0, count = 0;
};

float half_area(const float lo[3], const float hi[3]) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}

int bvh_build(std::vector<BvhPrim>& P, int b, int e, std::vector<TNode>& T, std::vector<int32_t>& order,
              int leaf_size = rtp::kBvhLeafSize) {
  const int me = (int)T.size();
  T.emplace_back();
  TNode nd;
  float clo[3], chi[3];
  for (int k = 0; k < 3; k++) {
    nd.lo[k] = clo[k] = INFINITY;
    nd.hi[k] = chi[k] = -INFINITY;
  }
  for (int i = b; i < e; i++)
    for (int k = 0; k < 3; k++) {
      nd.lo[k] = std::min(nd.lo[k], P[i].lo[k]);
      nd.hi[k] = std::max(nd.hi[k], P[i].hi[k]);
      clo[k] = std::min(clo[k], P[i].cen[k]);
      chi[k] = std::max(chi[k], P[i].cen[k]);
    }
  const int n = e - b;
  if (n <= leaf_size) {
    nd.first = (int)order.size();
    nd.count = n;
    for (int i = b; i < e; i++) order.push_back(P[i].idx);
    T[me] = nd;
    return me;
  }
  // binned SAH
  constexpr int kBins = 16;
  int best_ax = -1, best_split = 0;
  float best_cost = INFINITY;
  for (int ax = 0; ax < 3; ax++) {
    const float ext = chi[ax] - clo[ax];
    if (!(ext > 0)) continue;
    int cnt[kBins] = {};
    float blo[kBins][3], bhi[kBins][3];
    for (int j = 0; j < kBins; j++)
      for (int k = 0; k < 3; k++) blo[j][k] = INFINITY, bhi[j][k] = -INFINITY;
    for (int i = b; i < e; i++) {
      int j = (int)((P[i].cen[ax] - clo[ax]) / ext * kBins);
      j = std::min(kBins - 1, std::max(0, j));
      cnt[j]++;
      for (int k = 0; k < 3; k++) blo[j][k] = std::min(blo[j][k], P[i].lo[k]), bhi[j][k] = std::max(bhi[j][k], P[i].hi[k]);
    }
    for (int s = 1; s < kBins; s++) {  // split between bins s-1 and s
      float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      int nl = 0, nr = 0;
      for (int j = 0; j < kBins; j++) {
        if (!cnt[j]) continue;
        float* lo = j < s ? llo : rlo;
        float* hi = j < s ? lhi : rhi;
        (j < s ? nl : nr) += cnt[j];
        for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], blo[j][k]), hi[k] = std::max(hi[k], bhi[j][k]);
      }
      if (!nl || !nr) continue;
      const float cost = nl * half_area(llo, lhi) + nr * half_area(rlo, rhi);
      if (cost < best_cost) best_cost = cost, best_ax = ax, best_split = s;
    }
  }
  int mid;
  if (best_ax >= 0) {
    const int ax = best_ax;
    const float ext = chi[ax] - clo[ax];
    auto bin = [&](const BvhPrim& x) {
      return std::min(kBins - 1, std::max(0, (int)((x.cen[ax] - clo[ax]) / ext * kBins)));
    };
    mid = (int)(std::stable_partition(P.begin() + b, P.begin() + e, [&](const BvhPrim& x) { return bin(x) < best_split; }) -
                P.begin());
    nd.axis = ax;
  } else {  // coincident centroids: median split by index
    std::sort(P.begin() + b, P.begin() + e, [](const BvhPrim& x, const BvhPrim& y) { return x.idx < y.idx; });
    mid = b + n / 2;
    nd.axis = 0;
  }
  nd.left = bvh_build(P, b, mid, T, order, leaf_size);
  nd.right = bvh_build(P, mid, e, T, order, leaf_size);
  T[me] = nd;
  return me;
}

// inner nodes of the sphere BVH above this depth are dropped from the walks'
// arrays (bvh_flatten below)
constexpr int kBvhDropDepth = 2;
constexpr float kBvhDropArea = 0.6f;  // (0: off)

// threaded flattening for one octant (bit k set: direction component k < 0)
// A one-sphere leaf carries the sphere itself (rtp::kBvhLeafSphere): lo =
// centre, hi[0] = r*r, hi[1] = the sphere's index (as int bits), so the walk
// runs the exact root test without a box test or a second dependent load.
// Inner nodes above depth `drop` are not emitted: their children take their
// place in the order (the skip of the node before them then lands on their
// first emitted descendant), so the walk treats their boxes as hit.  A box
// only culls, so this changes which nodes a ray visits, never its hit.  The
// top boxes (the whole sphere cloud, its halves) are hit by nearly every ray
// from inside the room: each one dropped is one dependent gather and box test
// fewer per walk.
// Below that, with drop_sa > 0, an inner node with two inner children is
// dropped too when its surface area exceeds drop_sa of its parent's (a ray
// that reaches it would hit its box with about that probability: dropping it
// saves one visit when it would be hit and costs one when it would not).
void bvh_flatten(const std::vector<TNode>& T, int t, int oct, const std::vector<int32_t>& order,
                 const std::vector<rtp::DevSphere>& sph, std::vector<rtp::BvhNode>& out, int depth = 0,
                 int drop = 0, float drop_sa = 0.f, float parent_area = 0.f) {
  const TNode& n = T[t];
  const float area = half_area(n.lo, n.hi);
  const bool inner2 = n.left >= 0 && T[n.left].left >= 0 && T[n.right].left >= 0;
  if (n.left >= 0 && (depth < drop || (drop_sa > 0.f && inner2 && parent_area > 0.f && area > drop_sa * parent_area))) {
    const bool neg = (oct >> n.axis) & 1;
    const float pa = parent_area > 0.f ? parent_area : area;  // the nearest emitted ancestor's (or the root's)
    bvh_flatten(T, neg ? n.right : n.left, oct, order, sph, out, depth + 1, drop, drop_sa, pa);
    bvh_flatten(T, neg ? n.left : n.right, oct, order, sph, out, depth + 1, drop, drop_sa, pa);
    return;
  }
  const int me = (int)out.size();
  out.emplace_back();
  rtp::BvhNode nd{};
  const TNode& s = T[t];
  std::memcpy(nd.lo, s.lo, sizeof(nd.lo));
  std::memcpy(nd.hi, s.hi, sizeof(nd.hi));
  if (s.left < 0) {
    if (RTP_BVH_EMBED && s.count == 1) {
      const rtp::DevSphere& S = sph[order[s.first]];
      std::memcpy(nd.lo, S.c, sizeof(nd.lo));
      nd.hi[0] = S.rr;
      int32_t orig = order[s.first];
      std::memcpy(&nd.hi[1], &orig, sizeof(orig));
      nd.hi[2] = 0.f;
      nd.leaf = rtp::kBvhLeafSphere;
    } else {
      nd.leaf = (s.first << 3) | s.count;
    }
  } else {
    const bool neg = (oct >> s.axis) & 1;  // moving toward lower coordinates: right (upper) child first
    bvh_flatten(T, neg ? s.right : s.left, oct, order, sph, out, depth + 1, drop, drop_sa, area);
    bvh_flatten(T, neg ? s.left : s.right, oct, order, sph, out, depth + 1, drop, drop_sa, area);
    nd.leaf = 0;
  }
  nd.skip = (int32_t)out.size();
  out[me] = nd;
}

}  // namespace

// error reporting for the other translation units of librtp.so
rtp_status rtp_internal_fail(rtp_status st, const std::string& msg) { return fail(st, msg); }

namespace {
rtp_status drain(rtp_context* c) {
  if (c->pending) {
    HIP_TRY(hipEventSynchronize(c->done));
    c->pending = false;
  }
  return RTP_OK;
}
}  // namespace

extern "C" {

const char* rtp_last_error(void) { return g_err.c_str(); }
int32_t rtp_abi_version(void) { return RTP_ABI_VERSION; }

rtp_status rtp_create(int32_t device, rtp_context** out) {
  if (!out) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_create: out is NULL");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return fail(RTP_ERR_DEVICE, "rtp_create: no HIP device available");
  if (device < 0 || device >= n) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_create: device ordinal out of range");
  HIP_TRY(hipSetDevice(device));
  rtp_context* c = new rtp_context();
  c->device = device;
  c->ff_policy = ff_policy_default();
  e = hipMalloc(&c->d_scene, sizeof(rtp::DevScene));
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "hipMalloc(scene)");
  }
  e = hipMalloc(&c->d_progress, 16);
  if (e != hipSuccess) {
    (void)hipFree(c->d_scene);
    delete c;
    return hip_fail(e, "hipMalloc(progress)");
  }
  HIP_TRY(hipEventCreate(&c->ev0));
  HIP_TRY(hipEventCreate(&c->ev1));
  HIP_TRY(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
  *out = c;
  return RTP_OK;
}

void rtp_destroy(rtp_context* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)drain(c);
  if (c->d_scene) (void)hipFree(c->d_scene);
  if (c->d_hist) (void)hipFree(c->d_hist);
  if (c->d_dbg) (void)hipFree(c->d_dbg);
  if (c->d_progress) (void)hipFree(c->d_progress);
  if (c->d_nodes) (void)hipFree(c->d_nodes);
  if (c->d_sph_geom) (void)hipFree(c->d_sph_geom);
  if (c->d_sph_all) (void)hipFree(c->d_sph_all);
  for (void* p : {(void*)c->d_lw_nodes, (void*)c->d_lw_cidx, (void*)c->d_lw_sph, (void*)c->d_lw_orig})
    if (p) (void)hipFree(p);
  if (c->d_cnodes) (void)hipFree(c->d_cnodes);
  if (c->d_cidx) (void)hipFree(c->d_cidx);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->d_direct) (void)hipFree(c->d_direct);
  delete c;
}

// extract + buildBVH (MapperPathTracer.cxx:178-197, 437-449) and the light
// coupling of the constructor (:141-148).  Quads that repeat an earlier quad
// bit-for-bit (same vertices in the same order, same material and texture --
// buildBox emits two such pairs per box, CornellBox.cpp:114-137) are dropped:
// under the strict '<' closest test the later copy can never win, so the hit
// record is unchanged.
rtp_status rtp_set_scene(rtp_context* c, const rtp_scene_desc* s) {
  if (!c || !s) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: NULL argument");
  if (s->n_points <= 0 || !s->points) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: no points");
  if (s->n_quads < 0 || s->n_spheres < 0 || s->n_spheres > rtp::kMaxSpheresBvh)
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: bad primitive counts");
  if (s->n_spheres < 1)
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: the light sphere radius is SphereRadii[0]; need >= 1 sphere");
  auto pt_ok = [&](int32_t id) { return id >= 0 && id < s->n_points; };
  auto mat_ok = [&](int32_t m) { return m >= 0 && m < s->n_mat && s->mat_type[m] >= 0 && s->mat_type[m] <= 2; };
  auto tex_ok = [&](int32_t t) {
    return t >= 0 && t < s->n_tex_type && s->tex_type[t] >= 0 && s->tex_type[t] < s->n_tex;
  };
  rtp::DevScene* h = new rtp::DevScene();
  std::memset(h, 0, sizeof(*h));
  // (after the memset: every octant its own walk order -- the device LBVH
  // build keeps all 8; the host SAH build may narrow it, RTP_BVH_OCT_MASK)
  h->oct_mask = 7;
  std::vector<int> kept;
  std::vector<rtp::DevQuad> built;
  for (int q = 0; q < s->n_quads; q++) {
    const int32_t* id = s->quad_points + 4 * q;
    for (int k = 0; k < 4; k++)
      if (!pt_ok(id[k])) {
        delete h;
        return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: quad point id out of range");
      }
    if (!mat_ok(s->quad_mat[q]) || !tex_ok(s->quad_tex[q])) {
      delete h;
      return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: quad material/texture index out of range");
    }
    bool dup = false;
    for (int j : kept) {
      const int32_t* jd = s->quad_points + 4 * j;
      bool same = s->quad_mat[j] == s->quad_mat[q] && s->quad_tex[j] == s->quad_tex[q];
      for (int k = 0; k < 4 && same; k++) same = bit_equal(s->points + 3 * jd[k], s->points + 3 * id[k], 3);
      if (same) {
        dup = true;
        break;
      }
    }
    if (dup) continue;
    if ((int)kept.size() >= rtp::kMaxQuads) {
      delete h;
      return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: too many distinct quads");
    }
    rtp::DevQuad Q;
    fill_quad(Q, ld(s->points + 3 * id[0]), ld(s->points + 3 * id[1]), ld(s->points + 3 * id[2]),
              ld(s->points + 3 * id[3]));
    Q.mt = s->mat_type[s->quad_mat[q]];
    st(Q.alb, ld(s->tex_rgb + 3 * s->tex_type[s->quad_tex[q]]));
    Q.orig = (int32_t)kept.size();  // rank in the reference's (index) order
    kept.push_back(q);
    built.push_back(Q);
  }
  // group by kind (scan order 1..kQuadKinds-1, then 0); the device scan
  // compares (t, orig) lexicographically, which is exactly the reference's
  // index-order strict '<' scan, so the grouping changes no result.
  {
    int pos = 0;
    for (int g = 0; g < rtp::kQuadKinds; g++) {
      const int kind = (g + 1) % rtp::kQuadKinds;
      h->kind_begin[g] = pos;
      for (const rtp::DevQuad& Q : built)
        if (Q.kind == kind) {
          h->quads[pos] = Q;
          h->quads[pos].key_lo = ((uint32_t)Q.orig << 8) | (uint32_t)pos;  // both < kMaxQuads = 256
          pos++;
        }
    }
    h->kind_begin[rtp::kQuadKinds] = pos;
    if (const char* v = getenv("RTP_VERBOSE")) {
      if (v[0] == '1') {
        fprintf(stderr, "rtp: %d quads by scan group (kind: count / exact parallelograms):", pos);
        for (int g = 0; g < rtp::kQuadKinds; g++) {
          int np = 0;
          for (int i = h->kind_begin[g]; i < h->kind_begin[g + 1]; i++) np += h->quads[i].para ? 1 : 0;
          fprintf(stderr, " %d: %d/%d", (g + 1) % rtp::kQuadKinds, h->kind_begin[g + 1] - h->kind_begin[g], np);
        }
        fprintf(stderr, "\n");
      }
    }
  }
  setup_prefilter(h, s, kept);
  h->n_quads = (int32_t)kept.size();
  // the -direct mode's inputs: kept quad -> reference index, and the shape
  // bounds (union of the quads' padded AABBs, AABBSurface.h:36-78)
  std::vector<int32_t> kept_ref(kept.begin(), kept.end());
  float blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int q = 0; q < s->n_quads; q++) {
    const int32_t* id = s->quad_points + 4 * q;
    float mn[3], mx[3];
    for (int k = 0; k < 3; k++) mn[k] = mx[k] = s->points[3 * id[0] + k];
    for (int c2 = 1; c2 < 4; c2++)
      for (int k = 0; k < 3; k++) {
        const float v = s->points[3 * id[c2] + k];
        mn[k] = (v < mn[k]) ? v : mn[k];  // vtkm::Min / Max: (std::min)/(std::max)
        mx[k] = (mx[k] < v) ? v : mx[k];
      }
    for (int k = 0; k < 3; k++) {
      const float ext = 1.0e-4f * (mx[k] - mn[k]);
      const float eps = (1e-6f < ext) ? ext : 1e-6f;
      mn[k] -= eps;
      mx[k] += eps;
      blo[k] = std::min(blo[k], mn[k]);
      bhi[k] = std::max(bhi[k], mx[k]);
    }
  }
  std::vector<rtp::DevSphere> sph(s->n_spheres);
  for (int k = 0; k < s->n_spheres; k++) {
    if (!pt_ok(s->sphere_point[k]) || !mat_ok(s->sphere_mat[k]) || !tex_ok(s->sphere_tex[k]) ||
        !(s->sphere_radius[k] > 0.0f)) {
      delete h;
      return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: sphere index or radius out of range");
    }
    rtp::DevSphere& S = sph[k];
    std::memset(&S, 0, sizeof(S));
    st(S.c, ld(s->points + 3 * s->sphere_point[k]));
    S.r = s->sphere_radius[k];
    S.rr = S.r * S.r;
    S.mt = s->mat_type[s->sphere_mat[k]];
    st(S.alb, ld(s->tex_rgb + 3 * s->tex_type[s->sphere_tex[k]]));
  }
  const bool use_bvh = s->n_spheres >= rtp::kBvhMinSpheres;
  // which builder makes the sphere BVH: the host's binned SAH (better trees,
  // O(n log n) on one core) or the device LBVH (rtp_bvh_gpu.hip) for large
  // scenes; RTP_BVH_BUILD=host|gpu overrides
  bool gpu_build = use_bvh && s->n_spheres >= rtp::kBvhGpuMinSpheres;
  if (const char* bb = getenv("RTP_BVH_BUILD")) {
    if (!std::strcmp(bb, "gpu")) gpu_build = use_bvh;
    if (!std::strcmp(bb, "host")) gpu_build = false;
  }
  std::vector<rtp::BvhNode> nodes;
  std::vector<rtp::DevSphereG> geom;
  // the LDS walk's tree (kLdsWalkLeaf) in BvhNode form, its leaf order and size
  std::vector<rtp::BvhNode> lw_nodes;
  std::vector<int32_t> lw_order;
  int lw_per_oct = 0;
  if (!use_bvh) {
    for (int k = 0; k < s->n_spheres; k++) h->spheres[k] = sph[k];
  } else if (gpu_build) {
    h->n_nodes = 2 * s->n_spheres - 1;  // nodes and sphere records are built on the device below
  } else {
    std::vector<BvhPrim> P(s->n_spheres);
    for (int k = 0; k < s->n_spheres; k++) {
      const rtp::DevSphere& S = sph[k];
      // (+ 2^-16 of the coordinates' magnitude: the walk's fma slab test,
      // rtp_kernels.hip BvhRay, stays far inside the margin at any scale)
      const float pad = 0.002f * S.r + 1e-5f +
                        0x1p-16f * (std::max(std::fabs(S.c[0]), std::max(std::fabs(S.c[1]), std::fabs(S.c[2]))) + S.r);
      for (int a = 0; a < 3; a++) {
        P[k].lo[a] = S.c[a] - S.r - pad;
        P[k].hi[a] = S.c[a] + S.r + pad;
        P[k].cen[a] = S.c[a];
      }
      P[k].idx = k;
    }
    const std::vector<BvhPrim> P0 = P;  // (bvh_build reorders P)
    std::vector<int32_t> order;
    std::vector<TNode> tree;
    bvh_build(P, 0, s->n_spheres, tree, order);
    // inner nodes above this depth are not emitted (bvh_flatten; RTP_BVH_DROP overrides)
    int drop = kBvhDropDepth;
    float drop_sa = kBvhDropArea;
    if (const char* dd = getenv("RTP_BVH_DROP")) drop = std::max(0, std::min(16, atoi(dd)));
    if (const char* da = getenv("RTP_BVH_DROP_SA")) drop_sa = (float)atof(da);
    // the copies the walk reads: octant o walks copy (o & oct_mask)
    // (RTP_BVH_OCT_MASK; the other copies are built the same and never read)
    int oct_mask = 7;
    if (const char* om = getenv("RTP_BVH_OCT_MASK")) oct_mask = atoi(om) & 7;
    h->oct_mask = oct_mask;
    int per_oct = 0;
    for (int oct = 0; oct < 8; oct++) {  // 8 copies of n_nodes entries, indices local to each copy
      std::vector<rtp::BvhNode> one;
      bvh_flatten(tree, 0, oct & oct_mask, order, sph, one, 0, drop, drop_sa);
      per_oct = (int)one.size();  // (the same nodes are dropped in every octant's order)
      nodes.insert(nodes.end(), one.begin(), one.end());
    }
    // The LDS walk's tree (opt-in, RTP_BVH_LDS=1): leaves of up to
    // kLdsWalkLeaf spheres, flattened the same way, used when its 8 copies
    // plus the leaf spheres fit the block's LDS (the stats build and planned
    // launches walk the global tree).  On C3 at 16 spp (r04h/r04i, kernel ms):
    // LDS walk 324, the global walk over the same leaves-of-6 tree 349, the
    // global walk over the leaves-of-1 tree 186 -- the LDS copy saves 7% of the
    // texture-path gathers' cost, the bigger leaves it needs to fit cost 88%
    // (10 exact sphere tests per ray instead of 4: DESIGN.md 4.2).
    const char* le = getenv("RTP_BVH_LDS");
    if (le && le[0] == '1') {
      std::vector<BvhPrim> P2 = P0;
      std::vector<TNode> tree2;
      bvh_build(P2, 0, s->n_spheres, tree2, lw_order, rtp::kLdsWalkLeaf);
      for (int oct = 0; oct < 8; oct++) {
        std::vector<rtp::BvhNode> one;
        bvh_flatten(tree2, 0, oct, lw_order, sph, one, 0, drop, drop_sa);
        lw_per_oct = (int)one.size();
        lw_nodes.insert(lw_nodes.end(), one.begin(), one.end());
      }
      const int64_t bytes = (int64_t)16 * (8 * (int64_t)lw_per_oct + (int64_t)lw_order.size());
      if (bytes > rtp_lds_walk_capacity()) {
        lw_nodes.clear();
        lw_order.clear();
        lw_per_oct = 0;
      }
    }
    geom.resize(order.size());
    for (size_t j = 0; j < order.size(); j++) {
      const rtp::DevSphere& S = sph[order[j]];
      std::memset(&geom[j], 0, sizeof(geom[j]));
      std::memcpy(geom[j].c, S.c, sizeof(S.c));
      geom[j].rr = S.rr;
      geom[j].orig = order[j];
    }
    h->n_nodes = (int32_t)per_oct;
  }
  h->n_spheres = s->n_spheres;
  // lights (MapperPathTracer.cxx:141-148): light quad = light_box_pointids[1..4]
  const int32_t* lq = s->light_quad_points;
  for (int k = 0; k < 4; k++)
    if (!pt_ok(lq[k])) {
      delete h;
      return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: light quad point id out of range");
    }
  if (!pt_ok(s->light_sphere_point)) {
    delete h;
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_scene: light sphere point id out of range");
  }
  v3 q = ld(s->points + 3 * lq[0]), r = ld(s->points + 3 * lq[1]), ss = ld(s->points + 3 * lq[2]),
     t = ld(s->points + 3 * lq[3]);
  fill_quad(h->light.quad, q, r, ss, t);
  {
    float qr = std::sqrt(dot(sub(r, q), sub(r, q)));  // vtkm::Magnitude
    float qt = std::sqrt(dot(sub(t, q), sub(t, q)));
    h->light.area = qr * qt;  // PdfWorklet.h:236-239
  }
  // QuadWorkletGenerateDir uses pts[pointIndex[1]] and pts[pointIndex[3]]
  {
    float x0 = q.x, x1 = ss.x, z0 = q.z, z1 = ss.z, y0 = q.y, y1 = q.y;
    h->light.gx0 = x0, h->light.gdx = x1 - x0;
    h->light.gy0 = y0, h->light.gdy = y1 - y0;
    h->light.gz0 = z0, h->light.gdz = z1 - z0;
  }
  st(h->light.sc, ld(s->points + 3 * s->light_sphere_point));
  h->light.sr = s->sphere_radius[0];  // SphereRadii[0] (PdfWorklet.h:205-210)
  h->light.srr = h->light.sr * h->light.sr;
  h->ior = s->ior;
  {  // schlick's r0^2 and 1/ior with the reference's operations (float, float; double then float)
    float r0 = (1 - h->ior) / (1 + h->ior);
    h->ior_r0sq = r0 * r0;
    h->ior_inv = (float)(1.0 / h->ior);
  }
  h->which_t1 = which_threshold(2);
  h->which_t2 = which_threshold(3);
  hipError_t e = hipSetDevice(c->device);
  if (c->pending) {  // a queued render may still read the old scene
    if (e == hipSuccess) e = hipEventSynchronize(c->done);
    c->pending = false;
  }
  for (void** p : {(void**)&c->d_nodes, (void**)&c->d_sph_geom, (void**)&c->d_sph_all, (void**)&c->d_cnodes,
                   (void**)&c->d_cidx, (void**)&c->d_lw_nodes, (void**)&c->d_lw_cidx, (void**)&c->d_lw_sph,
                   (void**)&c->d_lw_orig})
    if (*p && e == hipSuccess) {
      e = hipFree(*p);
      *p = nullptr;
    }
  if (use_bvh && gpu_build && e == hipSuccess) {
    const int n = s->n_spheres;
    std::vector<float4> cr(n);
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int k = 0; k < n; k++) {
      cr[k] = make_float4(sph[k].c[0], sph[k].c[1], sph[k].c[2], sph[k].r);
      for (int a = 0; a < 3; a++) lo[a] = std::min(lo[a], sph[k].c[a]), hi[a] = std::max(hi[a], sph[k].c[a]);
    }
    float4* d_cr = nullptr;
    e = hipMalloc(&c->d_nodes, (size_t)8 * h->n_nodes * sizeof(rtp::BvhNode));
    if (e == hipSuccess) e = hipMalloc(&c->d_sph_geom, (size_t)n * sizeof(rtp::DevSphereG));
    if (e == hipSuccess) e = hipMalloc(&c->d_sph_all, sph.size() * sizeof(rtp::DevSphere));
    if (e == hipSuccess) e = hipMalloc(&d_cr, (size_t)n * sizeof(float4));
    if (e == hipSuccess) e = hipMemcpy(d_cr, cr.data(), (size_t)n * sizeof(float4), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = rtp_build_bvh_gpu(d_cr, n, make_float3(lo[0], lo[1], lo[2]),
                            make_float3(hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]), c->d_nodes, c->d_sph_geom,
                            nullptr);
    if (d_cr) (void)hipFree(d_cr);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_sph_all, sph.data(), sph.size() * sizeof(rtp::DevSphere), hipMemcpyHostToDevice);
    h->nodes = c->d_nodes;
    h->sph_geom = c->d_sph_geom;
    h->sph_all = c->d_sph_all;
  } else if (use_bvh && e == hipSuccess) {
    e = hipMalloc(&c->d_nodes, nodes.size() * sizeof(rtp::BvhNode));
    if (e == hipSuccess) e = hipMalloc(&c->d_sph_geom, geom.size() * sizeof(rtp::DevSphereG));
    if (e == hipSuccess) e = hipMalloc(&c->d_sph_all, sph.size() * sizeof(rtp::DevSphere));
    if (e == hipSuccess)
      e = hipMemcpy(c->d_nodes, nodes.data(), nodes.size() * sizeof(rtp::BvhNode), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_sph_geom, geom.data(), geom.size() * sizeof(rtp::DevSphereG), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_sph_all, sph.data(), sph.size() * sizeof(rtp::DevSphere), hipMemcpyHostToDevice);
    h->nodes = c->d_nodes;
    h->sph_geom = c->d_sph_geom;
    h->sph_all = c->d_sph_all;
    if (e == hipSuccess && lw_per_oct > 0) {  // the LDS walk's tree: compacted like the global one
      const int64_t total = (int64_t)8 * lw_per_oct, ns = (int64_t)lw_order.size();
      std::vector<float> lsph(4 * ns);
      for (int64_t j = 0; j < ns; j++) {
        const rtp::DevSphere& S = sph[lw_order[j]];
        lsph[4 * j] = S.c[0], lsph[4 * j + 1] = S.c[1], lsph[4 * j + 2] = S.c[2], lsph[4 * j + 3] = S.rr;
      }
      rtp::BvhNode* d_tmp = nullptr;
      e = hipMalloc(&d_tmp, (size_t)total * sizeof(rtp::BvhNode));
      if (e == hipSuccess) e = hipMalloc(&c->d_lw_nodes, (size_t)total * 16);
      if (e == hipSuccess) e = hipMalloc(&c->d_lw_cidx, (size_t)total * sizeof(int32_t));
      if (e == hipSuccess) e = hipMalloc(&c->d_lw_sph, (size_t)ns * 16);
      if (e == hipSuccess) e = hipMalloc(&c->d_lw_orig, (size_t)ns * sizeof(int32_t));
      if (e == hipSuccess)
        e = hipMemcpy(d_tmp, lw_nodes.data(), (size_t)total * sizeof(rtp::BvhNode), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(c->d_lw_sph, lsph.data(), (size_t)ns * 16, hipMemcpyHostToDevice);
      if (e == hipSuccess)
        e = hipMemcpy(c->d_lw_orig, lw_order.data(), (size_t)ns * sizeof(int32_t), hipMemcpyHostToDevice);
      if (e == hipSuccess) e = rtp_compact_bvh(d_tmp, total, c->d_lw_nodes, c->d_lw_cidx, nullptr);
      if (d_tmp) (void)hipFree(d_tmp);
      h->lw_nodes = c->d_lw_nodes;
      h->lw_cidx = c->d_lw_cidx;
      h->lw_sph = c->d_lw_sph;
      h->lw_orig = c->d_lw_orig;
      h->n_lw_nodes = lw_per_oct;
      h->n_lw_sph = (int32_t)ns;
    }
  }
  if (use_bvh && e == hipSuccess) {  // the walks' compact copy of the octant arrays
    const int64_t total = (int64_t)8 * h->n_nodes;
    e = hipMalloc(&c->d_cnodes, (size_t)total * 16);
    if (e == hipSuccess) e = hipMalloc(&c->d_cidx, (size_t)total * sizeof(int32_t));
    if (e == hipSuccess) e = rtp_compact_bvh(c->d_nodes, total, c->d_cnodes, c->d_cidx, nullptr);
    h->cnodes = c->d_cnodes;
    h->cidx = c->d_cidx;
  }
  if (e == hipSuccess) e = hipMemcpy(c->d_scene, h, sizeof(*h), hipMemcpyHostToDevice);
  c->lw_bytes = h->n_lw_nodes > 0 ? 16 * (8 * h->n_lw_nodes + h->n_lw_sph) : 0;
  c->use_bvh = use_bvh;
  c->oct_mask = use_bvh ? h->oct_mask : 0;  // (read before the host copy is freed)
  delete h;
  if (e != hipSuccess) return hip_fail(e, "rtp_set_scene upload");
  c->kept_quads = std::move(kept_ref);
  c->n_ref_quads = s->n_quads;
  for (int k = 0; k < 3; k++) c->quad_lo[k] = blo[k], c->quad_hi[k] = bhi[k];
  c->has_scene = true;
  return RTP_OK;
}

}  // extern "C"

namespace {

// pathtracing::Camera::SetParameters -> CreateRaysImpl -> RayGen ctor
void camera_setup(const rtp_camera* cam, int32_t nx, int32_t ny, rtp::DevCamera* out) {
  v3 up = ld(cam->view_up);
  if (!(up.x == 0.f && up.y == 1.f && up.z == 0.f)) up = normalize(up);  // SetUp (Camera.cxx:767-776)
  v3 pos = ld(cam->position);
  v3 look = normalize(sub(ld(cam->look_at), pos));  // Camera.cxx:908-909
  const float pi_180f = 0.01745329251994329577f;    // vtkm::Pi_180f()
  float thx = tanf((cam->fov_y_deg * pi_180f) * .5f);
  float thy = tanf((cam->fov_y_deg * pi_180f) * .5f);
  v3 u = normalize(cross(look, up));
  v3 v = normalize(cross(u, look));
  st(out->eye, pos);
  st(out->dx, scl(u, (2 * thx / (float)nx)));
  st(out->dy, scl(v, (2 * thy / (float)ny)));
  st(out->nlook, normalize(look));
}

rtp_status check_render_args(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                             int32_t depth) {
  if (!c || !cam) return fail(RTP_ERR_INVALID_ARGUMENT, "render: NULL argument");
  if (!c->has_scene) return fail(RTP_ERR_NO_SCENE, "render: rtp_set_scene was not called");
  if (nx <= 0 || ny <= 0) return fail(RTP_ERR_INVALID_ARGUMENT, "Camera width/height must be greater than zero.");
  if ((int64_t)nx * ny > INT32_MAX) return fail(RTP_ERR_INVALID_ARGUMENT, "render: canvas too large");
  if (!(cam->fov_y_deg > 0)) return fail(RTP_ERR_INVALID_ARGUMENT, "Camera feild of view must be greater than zero.");
  if (cam->fov_y_deg > 180) return fail(RTP_ERR_INVALID_ARGUMENT, "Camera feild of view must be less than 180.");
  if (spp < 0) return fail(RTP_ERR_INVALID_ARGUMENT, "render: samplecount must be >= 0");
  // depthcount < 1 makes the reference read emitted[(depth-1)*N] out of range
  // (MapperPathTracer.cxx:328-331); rejected here.
  if (depth < 1) return fail(RTP_ERR_INVALID_ARGUMENT, "render: depthcount must be >= 1");
  // device-side bookkeeping limits: the pool kernel packs the remaining dead
  // depths into 14 bits and counts a wave's finished samples (<= 256 * spp)
  // in 32-bit signed cursors
  if (depth > rtp::kMaxDepth) return fail(RTP_ERR_INVALID_ARGUMENT, "render: depthcount must be <= 16383");
  if (spp > rtp::kMaxSpp) return fail(RTP_ERR_INVALID_ARGUMENT, "render: samplecount must be <= 8388607");
  return RTP_OK;
}

rtp_status ensure_hist(rtp_context* c, size_t bytes) {
  if (bytes <= c->hist_bytes) return RTP_OK;
  rtp_status rs = drain(c);
  if (rs != RTP_OK) return rs;
  if (c->d_hist) HIP_TRY(hipFree(c->d_hist));
  c->d_hist = nullptr;
  c->hist_bytes = 0;
  HIP_TRY(hipMalloc(&c->d_hist, bytes));
  c->hist_bytes = bytes;
  return RTP_OK;
}

rtp_status launch(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp, int32_t depth,
                  uint32_t seed_base, int64_t pixel_begin, int64_t npix, const int64_t* d_ids, float* d_out,
                  uint32_t* d_seed, uint32_t* d_live, hipStream_t stream, double* kernel_ms,
                  const int32_t* tile = nullptr, const int32_t* d_wave_begin = nullptr, int plan_waves = 0) {
  // the kernels index a launch's entries with 32-bit integers
  if (npix > INT32_MAX) return fail(RTP_ERR_INVALID_ARGUMENT, "render: more than 2^31-1 pixels in one launch");
  HIP_TRY(hipSetDevice(c->device));
  rtp::KParams p{};
  if (tile) p.tile_tx = tile[0], p.tile_world = tile[1], p.tile_rank = tile[2];
  camera_setup(cam, nx, ny, &p.cam);
  p.nx = nx, p.ny = ny, p.spp = spp, p.depth = depth;
  p.seed_base = seed_base;
  p.pixel_begin = pixel_begin;
  p.pixel_ids = d_ids;
  p.npix = npix;
  p.out = d_out;
  p.seed_out = d_seed;
  p.live_out = d_live;
  int variant = 2, waves = 0;
  // the sphere BVH's walk: 2 out of LDS when the tree fits (rtp_render_pool_lds),
  // 1 the global threaded walk (also for the diagnostics build and wave plans)
  const char* stats_env = getenv("RTP_DEBUG_STATS");
  const bool stats_on = stats_env && stats_env[0] == '1';
  const int bvh = !c->use_bvh ? 0 : (c->lw_bytes > 0 && !stats_on && !d_wave_begin) ? 2 : 1;
  int64_t lanes = rtp_plan_history_lanes(npix, spp, bvh, &variant, &waves);
  if (d_wave_begin) {  // a planned launch: the caller's waves
    if (variant != 2 || c->use_bvh || tile)
      return fail(RTP_ERR_INVALID_ARGUMENT, "render: a wave plan needs the pool kernel, no BVH, no tile deal");
    waves = plan_waves;
    lanes = (int64_t)plan_waves * 128;
  }
  p.wave_begin = d_wave_begin;
  // more entries than the resident waves' pools hold: the resident waves
  // steal entries (RTP_STEAL=0: waves of 128 entries in generations)
  if (variant == 2 && !d_wave_begin && !stats_on && spp > 0) {
    const char* se = getenv("RTP_STEAL");
    const int sw = (se && se[0] == '0') ? 0 : rtp_plan_steal(npix, bvh);
    if (sw > 0) {
      waves = sw;
      lanes = (int64_t)sw * 128;
    }
  }
  // D rows per lane (row k of a light hit holds E_k), rounded up to 8 (a
  // slot-major history pads each slot to whole 128-byte lines)
  size_t hist_need = (size_t)((depth + 7) & ~7) * (size_t)lanes * 16;
  rtp_status rs = ensure_hist(c, hist_need);
  if (rs != RTP_OK) return rs;
  p.hist = c->d_hist;
  p.dbg = nullptr;
  p.progress = c->d_progress;
  if (variant == 2) {
    const FfSnap ft = ff_tables(c->device, c->ff_policy, (uint64_t)npix * (uint64_t)spp);
    for (int j = 0; j < rtp::kFfTables; j++) p.ff[j] = ft.t[j];
    p.ffd = ft.direct, p.ffd_first = ft.d_first, p.ffd_count = ft.d_count;
  }
  if (c->pending) HIP_TRY(hipStreamWaitEvent(stream, c->done, 0));
  HIP_TRY(hipMemsetAsync(c->d_progress, 0, 16, stream));  // [0] progress, [1] entries stolen (kSteal)
  {
    const char* e = getenv("RTP_DEBUG_STATS");
    if (e && (e[0] == '1' || e[0] == '2') && variant == 2) {  // 2: timestamps in the production kernel
      if (c->d_dbg) (void)hipFree(c->d_dbg);
      c->d_dbg = nullptr;
      HIP_TRY(hipMalloc(&c->d_dbg, (size_t)waves * rtp::kDbgCounters * 8));
      HIP_TRY(hipMemsetAsync(c->d_dbg, 0, (size_t)waves * rtp::kDbgCounters * 8, stream));
      c->dbg_waves = waves;
      p.dbg = c->d_dbg;
    }
  }
  if (kernel_ms) HIP_TRY(hipEventRecord(c->ev0, stream));
  HIP_TRY(rtp_launch_render(c->d_scene, &p, variant, waves, bvh, stream, c->lw_bytes));
  HIP_TRY(hipEventRecord(c->done, stream));
  c->pending = true;
  if (kernel_ms) {
    HIP_TRY(hipEventRecord(c->ev1, stream));
    HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *kernel_ms = ms;
  }
  return RTP_OK;
}

// host-buffer render of an optional pixel list (nullptr: contiguous range)
rtp_status render_host(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp, int32_t depth,
                       uint32_t seed_base, const int64_t* ids, int64_t npix, float* rgba_out,
                       const rtp_pixel_aux* aux, rtp_stats* stats) {
  HIP_TRY(hipSetDevice(c->device));
  if (npix == 0) {
    if (stats) *stats = rtp_stats{};
    return RTP_OK;
  }
  int64_t* d_ids = nullptr;
  float* d_out = nullptr;
  uint32_t *d_seed = nullptr, *d_live = nullptr;
  rtp_status rs = RTP_OK;
  double ms = 0;
  std::vector<uint32_t> live(npix);
  auto cleanup = [&]() {
    if (d_ids) (void)hipFree(d_ids);
    if (d_out) (void)hipFree(d_out);
    if (d_seed) (void)hipFree(d_seed);
    if (d_live) (void)hipFree(d_live);
  };
  hipError_t e = hipMalloc(&d_out, (size_t)npix * 16);
  if (e == hipSuccess) e = hipMalloc(&d_live, (size_t)npix * 4);
  if (e == hipSuccess && aux && aux->final_seed) e = hipMalloc(&d_seed, (size_t)npix * 4);
  if (e == hipSuccess && ids) {
    e = hipMalloc(&d_ids, (size_t)npix * 8);
    if (e == hipSuccess) e = hipMemcpy(d_ids, ids, (size_t)npix * 8, hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    cleanup();
    return hip_fail(e, "render: device buffers");
  }
  rs = launch(c, cam, nx, ny, spp, depth, seed_base, 0, npix, d_ids, d_out, d_seed, d_live, nullptr, &ms);
  if (rs == RTP_OK) {
    e = hipMemcpy(rgba_out, d_out, (size_t)npix * 16, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(live.data(), d_live, (size_t)npix * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && d_seed) e = hipMemcpy(aux->final_seed, d_seed, (size_t)npix * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) rs = hip_fail(e, "render: copy back");
  }
  cleanup();
  if (rs != RTP_OK) return rs;
  if (aux && aux->live_bounces) std::memcpy(aux->live_bounces, live.data(), (size_t)npix * 4);
  if (stats) {
    stats->samples = (uint64_t)npix * (uint64_t)spp;
    uint64_t lb = 0, nan = 0;
    for (int64_t i = 0; i < npix; i++) {
      lb += live[i];
      const float* px = rgba_out + 4 * i;
      nan += (std::isnan(px[0]) || std::isnan(px[1]) || std::isnan(px[2])) ? 1 : 0;
    }
    stats->live_bounces = lb;
    stats->nan_pixels = nan;
    stats->kernel_ms = ms;
  }
  return RTP_OK;
}

}  // namespace

extern "C" {

rtp_status rtp_render(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp, int32_t depth,
                      uint32_t seed_base, float* rgba_out, rtp_stats* stats) {
  rtp_status rs = check_render_args(c, cam, nx, ny, spp, depth);
  if (rs != RTP_OK) return rs;
  if (!rgba_out) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render: rgba_out is NULL");
  return render_host(c, cam, nx, ny, spp, depth, seed_base, nullptr, (int64_t)nx * ny, rgba_out, nullptr, stats);
}

rtp_status rtp_render_pixels(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                             int32_t depth, uint32_t seed_base, const int64_t* pixel_ids, int64_t pixel_count,
                             float* rgba_out, const rtp_pixel_aux* aux, rtp_stats* stats) {
  rtp_status rs = check_render_args(c, cam, nx, ny, spp, depth);
  if (rs != RTP_OK) return rs;
  if (pixel_count < 0 || (pixel_count > 0 && (!pixel_ids || !rgba_out)))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_pixels: bad pixel list / output");
  const int64_t npx = (int64_t)nx * ny;
  for (int64_t i = 0; i < pixel_count; i++)
    if (pixel_ids[i] < 0 || pixel_ids[i] >= npx)
      return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_pixels: pixel id out of range");
  return render_host(c, cam, nx, ny, spp, depth, seed_base, pixel_ids, pixel_count, rgba_out, aux, stats);
}

rtp_status rtp_render_device(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                             int32_t depth, uint32_t seed_base, int64_t pixel_begin, int64_t pixel_count,
                             const int64_t* d_pixel_ids, float* d_rgba_out, const rtp_pixel_aux* aux,
                             void* hip_stream, rtp_stats* stats) {
  rtp_status rs = check_render_args(c, cam, nx, ny, spp, depth);
  if (rs != RTP_OK) return rs;
  if (pixel_count < 0 || (pixel_count > 0 && !d_rgba_out))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_device: bad output");
  if (!d_pixel_ids && (pixel_begin < 0 || pixel_begin + pixel_count > (int64_t)nx * ny))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_device: pixel range outside the canvas");
  if (pixel_count == 0) return RTP_OK;
  double ms = 0;
  rs = launch(c, cam, nx, ny, spp, depth, seed_base, pixel_begin, pixel_count, d_pixel_ids, d_rgba_out,
              aux ? aux->final_seed : nullptr, aux ? aux->live_bounces : nullptr, (hipStream_t)hip_stream,
              stats ? &ms : nullptr);
  if (rs == RTP_OK && stats) {
    stats->samples = (uint64_t)pixel_count * (uint64_t)spp;
    stats->live_bounces = 0;
    stats->nan_pixels = 0;
    stats->kernel_ms = ms;
  }
  return rs;
}

// rtp_render_device with a wave plan (include/rtp.h).
rtp_status rtp_render_planned_device(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                                     int32_t depth, uint32_t seed_base, int64_t pixel_begin, int64_t pixel_count,
                                     const int64_t* d_pixel_ids, const int32_t* d_wave_begin, int32_t n_waves,
                                     float* d_rgba_out, const rtp_pixel_aux* aux, void* hip_stream, rtp_stats* stats) {
  rtp_status rs = check_render_args(c, cam, nx, ny, spp, depth);
  if (rs != RTP_OK) return rs;
  if (pixel_count <= 0 || !d_rgba_out || !d_wave_begin || n_waves <= 0 || n_waves > (1 << 24))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_planned_device: bad plan / output");
  if (!d_pixel_ids && (pixel_begin < 0 || pixel_begin + pixel_count > (int64_t)nx * ny))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_planned_device: pixel range outside the canvas");
  {  // the plan must cover [0, pixel_count) exactly, in order, <= 128 entries per wave (one pool)
    HIP_TRY(hipSetDevice(c->device));
    std::vector<int32_t> plan((size_t)n_waves + 1);
    HIP_TRY(hipMemcpyAsync(plan.data(), d_wave_begin, plan.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                           (hipStream_t)hip_stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)hip_stream));
    bool ok = plan[0] == 0 && plan[n_waves] == pixel_count;
    for (int32_t w = 0; ok && w < n_waves; w++) ok = plan[w] <= plan[w + 1] && plan[w + 1] - plan[w] <= rtp::kPoolSlots;
    if (!ok)
      return fail(RTP_ERR_INVALID_ARGUMENT,
                  "rtp_render_planned_device: wave_begin must rise from 0 to pixel_count in steps of at most 128");
  }
  double ms = 0;
  rs = launch(c, cam, nx, ny, spp, depth, seed_base, pixel_begin, pixel_count, d_pixel_ids, d_rgba_out,
              aux ? aux->final_seed : nullptr, aux ? aux->live_bounces : nullptr, (hipStream_t)hip_stream,
              stats ? &ms : nullptr, nullptr, d_wave_begin, n_waves);
  if (rs == RTP_OK && stats) {
    *stats = rtp_stats{};
    stats->samples = (uint64_t)pixel_count * (uint64_t)spp;
    stats->kernel_ms = ms;
  }
  return rs;
}

// rtp_render_device over the rank's tiles of a round-robin 16x16 tile deal
// (shard.tile_pixels) without a pixel list: the kernel computes each entry's
// pixel, which saves the refill's gather of its id (C4's 1/8 share: 263 vs
// 276 ms on the same pixels, profiles/r04y_tiles_vs_list.txt).  Clipped edge
// tiles are rendered whole; their entries outside the canvas are ignored by
// the caller (shard.tile_entries): 0.7% more work on C4's 1080 rows.
rtp_status rtp_render_tiles_device(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, int32_t spp,
                                   int32_t depth, uint32_t seed_base, int32_t rank, int32_t world, float* d_rgba_out,
                                   void* hip_stream, rtp_stats* stats) {
  rtp_status rs = check_render_args(c, cam, nx, ny, spp, depth);
  if (rs != RTP_OK) return rs;
  if (world < 1 || rank < 0 || rank >= world)
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_tiles_device: rank outside [0, world)");
  const int64_t tx = (nx + 15) / 16, ty = (ny + 15) / 16;
  const int64_t tiles = tx * ty;
  // (the entries' pixel indices, up to 16 ty * nx, stay 32-bit in the kernel)
  if (tiles >= (1 << 24) || 16 * ty * (int64_t)nx >= ((int64_t)1 << 31))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_tiles_device: canvas too large");
  const int64_t mine = tiles / world + (rank < tiles % world ? 1 : 0);
  if (mine == 0) return RTP_OK;
  if (!d_rgba_out) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_render_tiles_device: bad output");
  const int32_t tile[3] = {(int32_t)tx, world, rank};
  double ms = 0;
  rs = launch(c, cam, nx, ny, spp, depth, seed_base, 0, mine * 256, nullptr, d_rgba_out, nullptr, nullptr,
              (hipStream_t)hip_stream, stats ? &ms : nullptr, tile);
  if (rs == RTP_OK && stats) {
    stats->samples = (uint64_t)mine * 256 * (uint64_t)spp;
    stats->live_bounces = 0;
    stats->nan_pixels = 0;
    stats->kernel_ms = ms;
  }
  return rs;
}

// Diagnostics: sums of the pool kernel's per-wave counters from the last launch
// made with RTP_DEBUG_STATS=1 (order of rtp::DbgCounter); returns the number
// of waves, 0 if none were recorded.
int32_t rtp_debug_counters(rtp_context* c, uint64_t* out, int32_t n_out) {
  if (!c || !c->d_dbg || !out) return 0;
  std::vector<unsigned long long> h((size_t)c->dbg_waves * rtp::kDbgCounters);
  if (hipMemcpy(h.data(), c->d_dbg, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  if (n_out < 0) {  // raw per-wave records: out must hold waves * kDbgCounters values
    std::memcpy(out, h.data(), h.size() * 8);
    return c->dbg_waves;
  }
  for (int k = 0; k < n_out && k < rtp::kDbgCounters; k++) {
    uint64_t acc = 0;
    for (int w = 0; w < c->dbg_waves; w++) acc += h[(size_t)w * rtp::kDbgCounters + k];
    out[k] = acc;
  }
  if (n_out > rtp::kDbgCounters) {  // extra slot: max wave lifetime
    uint64_t mx = 0;
    for (int w = 0; w < c->dbg_waves; w++) mx = std::max<uint64_t>(mx, h[(size_t)w * rtp::kDbgCounters + rtp::kDbgCyclesTotal]);
    out[rtp::kDbgCounters] = mx;
  }
  return c->dbg_waves;
}

rtp_status rtp_eval_primitive(rtp_context* c, int32_t kind, const void* in, void* out, int64_t n) {
  if (!c || !in || !out || n < 0 || kind < 0 || kind > 7)
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_eval_primitive: bad arguments");
  if (n == 0) return RTP_OK;
  HIP_TRY(hipSetDevice(c->device));
  const uint32_t* tab = nullptr;
  if (kind == 4 || kind == 5 || kind == 7) {
    const FfSnap ft = ff_tables(c->device, c->ff_policy, 0);
    tab = kind == 4 ? ft.t[1] : kind == 5 ? ft.t[0] : ft.direct;  // 16 / 32 dead depths, direct_first
    if (!tab) return fail(RTP_ERR_DEVICE, "rtp_eval_primitive: RNG jump tables are not built (policy or memory)");
  }
  const int dk = kind <= 3 ? kind : (kind == 6 ? 5 : 4);  // device kinds: 4 gather, 5 one dead step
  void *din = nullptr, *dout = nullptr;
  HIP_TRY(hipMalloc(&din, (size_t)n * 4));
  hipError_t e = hipMalloc(&dout, (size_t)n * 4);
  if (e == hipSuccess) e = hipMemcpy(din, in, (size_t)n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = rtp_launch_eval_primitive(dk, din, dout, n, tab, which_threshold(2), which_threshold(3), nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost);
  (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  if (e != hipSuccess) return hip_fail(e, "rtp_eval_primitive");
  return RTP_OK;
}

// Diagnostics: the closest hit of host rays with and without the quad
// prefilter (rtp_eval_closest_kernel; 7 u32 per ray).
rtp_status rtp_debug_closest_hit(rtp_context* c, const float* rays, int64_t n, uint32_t* out) {
  if (!c || !rays || !out || n < 0) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_debug_closest_hit: bad arguments");
  if (!c->d_scene) return fail(RTP_ERR_NO_SCENE, "rtp_debug_closest_hit: no scene set");
  if (n == 0) return RTP_OK;
  HIP_TRY(hipSetDevice(c->device));
  void *din = nullptr, *dout = nullptr;
  HIP_TRY(hipMalloc(&din, (size_t)n * 24));
  hipError_t e = hipMalloc(&dout, (size_t)n * 28);
  if (e == hipSuccess) e = hipMemcpy(din, rays, (size_t)n * 24, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = rtp_launch_eval_closest(c->d_scene, static_cast<const float*>(din), static_cast<uint32_t*>(dout), n,
                                c->use_bvh ? 1 : 0, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 28, hipMemcpyDeviceToHost);
  (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  if (e != hipSuccess) return hip_fail(e, "rtp_debug_closest_hit");
  return RTP_OK;
}

int32_t rtp_sphere_walk(rtp_context* c) {
  if (!c || !c->has_scene || !c->use_bvh) return 0;
  return c->lw_bytes > 0 ? 2 : 1;
}

int32_t rtp_sphere_walk_oct_mask(rtp_context* c) {
  if (!c || !c->has_scene || !c->use_bvh) return -1;
  // the value the kernels read: DevScene::oct_mask of the device copy (the
  // host field is a mirror, checked against it)
  int32_t dm = -1;
  if (hipSetDevice(c->device) != hipSuccess ||
      hipMemcpy(&dm, reinterpret_cast<const char*>(c->d_scene) + offsetof(rtp::DevScene, oct_mask), sizeof(dm),
                hipMemcpyDeviceToHost) != hipSuccess)
    return -2;
  return dm == c->oct_mask ? dm : -3;
}

// Diagnostics: exhaustive device check of a fast arithmetic sequence (kind,
// see rtp_verify_fast_math_kernel) over float bit patterns [lo_bits, hi_bits].
rtp_status rtp_verify_fast_math(rtp_context* c, int32_t kind, uint32_t lo_bits, uint32_t hi_bits,
                                uint64_t* mismatches, uint32_t* first_bad) {
  if (!c || !mismatches || hi_bits < lo_bits || kind < 0 || kind > 8)
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_verify_fast_math: bad args");
  HIP_TRY(hipSetDevice(c->device));
  unsigned long long* d_bad = nullptr;
  uint32_t* d_first = nullptr;
  HIP_TRY(hipMalloc(&d_bad, 8));
  HIP_TRY(hipMalloc(&d_first, 4));
  HIP_TRY(hipMemset(d_bad, 0, 8));
  HIP_TRY(hipMemset(d_first, 0xff, 4));
  const uint64_t total = (uint64_t)hi_bits - lo_bits + 1;
  const uint64_t chunk = 1ull << 30;
  for (uint64_t off = 0; off < total; off += chunk) {
    const uint64_t n = std::min<uint64_t>(chunk, total - off);
    HIP_TRY(rtp_launch_verify_fast_math(kind, lo_bits + (uint32_t)off, n, d_bad, d_first, nullptr));
  }
  unsigned long long bad = 0;
  uint32_t first = 0;
  HIP_TRY(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&first, d_first, 4, hipMemcpyDeviceToHost));
  (void)hipFree(d_bad);
  (void)hipFree(d_first);
  *mismatches = bad;
  if (first_bad) *first_bad = first;
  return RTP_OK;
}

rtp_status rtp_set_ff_tables(rtp_context* c, int32_t policy) {
  if (!c || policy < RTP_FF_TABLES_AUTO || policy > RTP_FF_TABLES_ON)
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_set_ff_tables: bad arguments");
  c->ff_policy = policy;
  if (policy == RTP_FF_TABLES_ON) {
    HIP_TRY(hipSetDevice(c->device));
    (void)ff_tables(c->device, policy, 0);  // build now, outside any timed render
  }
  return RTP_OK;
}

rtp_status rtp_get_ff_tables(rtp_context* c, rtp_ff_info* out) {
  if (!c || !out) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_get_ff_tables: bad arguments");
  std::lock_guard<std::mutex> lk(g_ff_mu);
  const FfTables& T = g_ff[c->device & 63];
  *out = rtp_ff_info{};
  out->policy = c->ff_policy;
  out->built = T.d_count > 0 ? 2 : T.n_chain > 0 ? 1 : 0;
  out->chain_tables = T.n_chain;
  out->direct_first = T.d_first;
  out->direct_count = T.d_count;
  out->bytes = T.bytes;
  out->alloc_ms = T.alloc_ms;
  out->build_ms = T.build_ms;
  out->samples_seen = T.samples_seen;
  uint64_t chain = 0, direct = 0;
  ff_auto_samples(chain, direct, &T);
  out->auto_samples = chain;
  out->auto_samples_direct = direct;
  return RTP_OK;
}

// NormalizeFunctor (main.cc:253-287): de-NaN rgb, then sqrt(c / spp) on all
// four channels.
rtp_status rtp_normalize(float* rgba, int64_t n, int32_t spp) {
  if (!rgba || n < 0) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_normalize: bad arguments");
  const float samplecount = (float)spp;
  for (int64_t i = 0; i < n; i++) {
    float* px = rgba + 4 * i;
    for (int k = 0; k < 3; k++)
      if (!(px[k] == px[k])) px[k] = 0;
    for (int k = 0; k < 4; k++) px[k] = std::sqrt(px[k] / samplecount);
  }
  return RTP_OK;
}

// save() (main.cc:325-384): P3 header "nx ny 255", one "r g b" line per
// pixel in buffer order (row 0 = camera bottom), int(255.99*c) unclamped,
// NaN pixels written as 0.
rtp_status rtp_write_pnm(const char* path, const float* rgba, int32_t nx, int32_t ny) {
  if (!path || !rgba || nx <= 0 || ny <= 0) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_write_pnm: bad arguments");
  FILE* f = std::fopen(path, "w");
  if (!f) return fail(RTP_ERR_INVALID_ARGUMENT, std::string("Couldn't save pnm: ") + path);
  std::fprintf(f, "P3\n%d %d 255\n", nx, ny);
  const int64_t n = (int64_t)nx * ny;
  for (int64_t i = 0; i < n; i++) {
    float c[3] = {rgba[4 * i], rgba[4 * i + 1], rgba[4 * i + 2]};
    if ((c[0] != c[0]) || (c[1] != c[1]) || (c[2] != c[2])) c[0] = c[1] = c[2] = 0.0f;
    std::fprintf(f, "%d %d %d\n", (int)(255.99 * c[0]), (int)(255.99 * c[1]), (int)(255.99 * c[2]));
  }
  std::fclose(f);
  return RTP_OK;
}

}  // extern "C"
