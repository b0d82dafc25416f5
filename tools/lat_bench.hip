// lat_bench.hip -- latency and throughput of the bounce step's parts on one
// MI355X, outside the pool kernel's scheduling (development tool).
//
// Each lane runs a chain of bounces in the C2 scene (Cornell box, variant 0):
// a random ray from a random point inside the room, then from each hit point
// on: closest_hit (+ shade_hit: material, generator, pdfs, scatter) exactly as
// the render kernel runs them (the device functions of rtp_kernels.hip,
// included below).  A path that dies restarts from a random point.  W waves
// per SIMD (grid = CUs x W blocks of 4 waves): W = 1 gives a lone wave's
// latency per step, W = 5 the pool kernel's occupancy.
//
// modes: 0 closest_hit only (prefilter on)
//        1 closest_hit + shade_hit (a bounce step without the pool's bookkeeping)
//        2 closest_hit with the prefilter off (exact scan of every quad)
//        3 shade_hit only (the hit of the first ray, re-shaded each step)
//        4 one jump-table gather per step (HBM latency: a dependent 4-byte
//          gather from a 16 GiB table, the fast-forward's chain read)
//        5 the ray advance alone (random point / direction: the other modes' overhead)
//        6 closest_hit's always-exact scan alone (kinds 7..10, 0)
//        7 closest_hit's prefilter alone (axis-plane quads + the candidate's exact test)
//        8 closest_hit SPLIT over lane pairs: lanes 2i and 2i+1 carry the same
//          ray, each scans half of every quad group (and of the prefilter's
//          records), the pair combines its keys with DPP swaps -- a wave
//          carries 32 rays (the strong-scaling experiment: a short share's
//          idle issue slots spent on halving each step's intersection)
//        9 mode 8 + shade_hit (shaded on both lanes of the pair, like mode 1)
//       10 check: mode 8's hit against closest_hit's on the same rays (prints
//          the mismatch count; not a timing)
//       11 TWO rays per lane in one instruction stream: closest_hit of both
//          rays in the same quad loops (each scalar-loaded head tested against
//          both: ILP instead of a second wave; cycles per step = both rays)
//       12 mode 11 + shade_hit of each ray (a step of two paths per lane)
//       13 check: mode 11's two hits against closest_hit's (mismatch count)
// (built with -DRTP_DET_FALLBACK=0: the quad tests without their |det| > 2^40 branch)
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fno-fast-math
//        -I raytracingtherestofyourlife_amd/csrc tools/lat_bench.hip
//        -L raytracingtherestofyourlife_amd -lrtp -Wl,-rpath,<that dir> -o tools/lat_bench
// usage: tools/lat_bench [iters] [modes...]
#include "../raytracingtherestofyourlife_amd/csrc/rtp_kernels.hip"
#include "../raytracingtherestofyourlife_amd/csrc/rtp_context.hpp"

#include <vector>

namespace lb {
using namespace rtp;

RTP_DEV f3 rand_dir(uint32_t& s) {
  for (;;) {
    const float x = 2.f * randf(s) - 1.f, y = 2.f * randf(s) - 1.f, z = 2.f * randf(s) - 1.f;
    const float q = x * x + y * y + z * z;
    if (q > 1e-4f && q <= 1.f) return mk(x, y, z);
  }
}
RTP_DEV f3 rand_point(uint32_t& s) {
  return mk(0.05f + 0.9f * randf(s), 0.05f + 0.9f * randf(s), 0.05f + 0.9f * randf(s));
}

// ---- lane-pair split of closest_hit (modes 8, 9) ----
// swap with the pair partner (DPP quad_perm [1,0,3,2])
RTP_DEV uint32_t pair_swap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
RTP_DEV uint64_t pair_min(uint64_t k) {
  const uint64_t o = (uint64_t)pair_swap((uint32_t)(k >> 32)) << 32 | pair_swap((uint32_t)k);
  return o < k ? o : k;
}
// quads [b, e) of kind K: this lane takes positions b + 2j + odd (an odd count
// leaves the last quad to both lanes); the heads are selected per lane
template <int K>
RTP_DEV void scan_kind_split(const DevScene* __restrict__ sc, int b, int e, f3 o, f3 d, uint64_t& best, bool odd) {
  for (int q = b; q < e; q += 2) {
    const int qb = min(q + 1, e - 1);
    const u16v ha = head_at(sc->quads + q), hb = head_at(sc->quads + qb);
    u16v h;
#pragma unroll
    for (int i = 0; i < 16; i++) h[i] = odd ? hb[i] : ha[i];
    const DevQuad& M = sc->quads[odd ? qb : q];  // (read only by a non-parallelogram's second triangle)
    scan_one<K>(M, h, o, d, best);
  }
}
template <int A>
RTP_DEV void pre_axis_split(const DevScene* __restrict__ sc, int b, int e, f3 o, f3 d, float ma, float mb, uint32_t& k1,
                            uint32_t& k2, bool odd) {
  constexpr int B = (A + 1) % 3, C = (A + 2) % 3;
  if (b == e) return;
  const float inv = __builtin_amdgcn_rcpf(comp<A>(d));
  const float oa = comp<A>(o);
  const f2v obc = f2v{comp<B>(o), comp<C>(o)}, dbc = f2v{comp<B>(d), comp<C>(d)};
  for (int q = b; q < e; q += 2) {
    const int qb = min(q + 1, e - 1);
    const PreQuad Pa = sc->pre[q], Pb = sc->pre[qb];
    const float px = odd ? Pb.x : Pa.x, cb = odd ? Pb.cb : Pa.cb, cc = odd ? Pb.cc : Pa.cc;
    const float rb = odd ? Pb.rb : Pa.rb, rc = odd ? Pb.rc : Pa.rc;
    const uint32_t qpos = odd ? (uint32_t)Pb.qpos : (uint32_t)Pa.qpos;
    const float t = (px - oa) * inv;
    const f2v u = __builtin_elementwise_fma(f2v{t, t}, dbc, obc) - f2v{cb, cc};
    const float ub = fabsf(u.x) - rb, uc = fabsf(u.y) - rc;
    const float m = __builtin_fmaf(fabsf(t), ma, mb);
    const bool ok = (fmaxf(ub, uc) <= m) & (t > kPreTmin);
    const uint32_t key = ok ? ((__float_as_uint(t - m) & ~31u) | qpos) : ~0u;
    k2 = max(k1, min(k2, key));
    k1 = min(k1, key);
  }
}
RTP_DEV Hit closest_hit_split(const DevScene* __restrict__ sc, f3 o, f3 d, const float* lds_prex) {
  const bool odd = (threadIdx.x & 1) != 0;
  uint64_t key = kNoHitKey;
  {
    const int g6 = sc->kind_begin[6], g7 = sc->kind_begin[7], g8 = sc->kind_begin[8], g9 = sc->kind_begin[9],
              g10 = sc->kind_begin[10], g11 = sc->kind_begin[11];
    scan_kind_split<7>(sc, g6, g7, o, d, key, odd);
    scan_kind_split<8>(sc, g7, g8, o, d, key, odd);
    scan_kind_split<9>(sc, g8, g9, o, d, key, odd);
    scan_kind_split<10>(sc, g9, g10, o, d, key, odd);
    scan_kind_split<0>(sc, g10, g11, o, d, key, odd);
  }
  const bool lane_ok = (int)(fabsf(o.x) <= kPreLimD) & (int)(fabsf(o.y) <= kPreLimD) & (int)(fabsf(o.z) <= kPreLimD) &
                       (int)(fabsf(d.x) <= kPreLimD) & (int)(fabsf(d.y) <= kPreLimD) & (int)(fabsf(d.z) <= kPreLimD);
  const float dmax = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), 1.0f));
  const float omax = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
  const float ma = kPreK * dmax, mb = kPreK * (omax + (sc->pre_scale + 1.0f));
  uint32_t k1 = ~0u, k2 = ~0u;
  const int p0 = sc->pre_begin[0], p1 = sc->pre_begin[1], p2 = sc->pre_begin[2], p3 = sc->pre_begin[3];
  pre_axis_split<0>(sc, p0, p1, o, d, ma, mb, k1, k2, odd);
  pre_axis_split<1>(sc, p1, p2, o, d, ma, mb, k1, k2, odd);
  pre_axis_split<2>(sc, p2, p3, o, d, ma, mb, k1, k2, odd);
  {  // the pair's two smallest keys
    const uint32_t o1 = pair_swap(k1), o2 = pair_swap(k2);
    k2 = min(max(k1, o1), min(k2, o2));
    k1 = min(k1, o1);
  }
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* lx = reinterpret_cast<const f4v*>(lds_prex) + 4 * (k1 & 31u);
  f4v xr[4] = {lx[0], lx[1], lx[2], lx[3]};
  if (lane_ok && k1 != ~0u) {
    PreExact Q;
    __builtin_memcpy(&Q, xr, sizeof(Q));
    float t;
    const bool ok = quad_hit_axis(Q, o, d, t);
    const uint64_t kq = (uint64_t)__float_as_uint(t) << 32 | Q.key_lo;
    key = (ok && t > 0.001f && kq < key) ? kq : key;
  }
  key = pair_min(key);
  const bool full = !lane_ok || (k2 & ~31u) <= (uint32_t)(key >> 32);
  if (__ballot(full)) {
    if (full) {
      const int g0 = sc->kind_begin[0], g1 = sc->kind_begin[1], g2 = sc->kind_begin[2], g3 = sc->kind_begin[3],
                g4 = sc->kind_begin[4], g5 = sc->kind_begin[5], g6 = sc->kind_begin[6];
      scan_kind_split<1>(sc, g0, g1, o, d, key, odd);
      scan_kind_split<2>(sc, g1, g2, o, d, key, odd);
      scan_kind_split<3>(sc, g2, g3, o, d, key, odd);
      scan_kind_split<4>(sc, g3, g4, o, d, key, odd);
      scan_kind_split<5>(sc, g4, g5, o, d, key, odd);
      scan_kind_split<6>(sc, g5, g6, o, d, key, odd);
    }
    key = pair_min(key);  // (both lanes of a pair take the same branch)
  }
  Hit h{3.40282347e+38f, -1, 0};
  if (key != kNoHitKey) {
    h.t = __uint_as_float((uint32_t)(key >> 32));
    h.kind = 0;
    h.idx = (int)(key & 0xffu);
  }
  const int ns = sc->n_spheres;
  for (int k = 0; k < ns; k++) {
    const DevSphere& S = sc->spheres[k];
    float t;
    if (sphere_hit(o, d, 0.001f, h.t, ld3(S.c), S.rr, t)) {
      h.t = t;
      h.kind = 1;
      h.idx = k;
    }
  }
  return h;
}

// ---- two rays per lane in one instruction stream (modes 11-13) ----
// closest_hit<false> for rays A and B together: every scalar-loaded quad head
// and prefilter record is tested against both rays, so the two rays'
// dependent chains can interleave (ILP in place of a second wave on a SIMD
// that a short launch leaves half empty).  Same keys, same minimum as two
// closest_hit calls (mode 13).  act_a / act_b: the lane carries that ray.
// (r04v: a pool kernel with two paths per lane built on this,
// rtp_render_pool_pair in git 9f948ac, was 44-47% slower on C4's 1/8 and
// 1/4 shares)
template <int K>
RTP_DEV void scan_kind_pf2(const DevScene* __restrict__ sc, int b, int e, f3 oa, f3 da, uint64_t& ba, f3 ob, f3 db,
                           uint64_t& bb, u16v& cur) {
  const DevQuad* qp = sc->quads + b;
  for (int n = e - b; n > 0; n -= 2, qp += 2) {
    const u16v nxt = head_at(qp + 1);
    scan_one<K>(qp[0], cur, oa, da, ba);
    scan_one<K>(qp[0], cur, ob, db, bb);
    if (n == 1) {
      cur = nxt;
      break;
    }
    cur = head_at(qp + 2);
    scan_one<K>(qp[1], nxt, oa, da, ba);
    scan_one<K>(qp[1], nxt, ob, db, bb);
  }
}
struct PreRay {
  float inv, oa, ma, mb;
  f2v obc, dbc;
  uint32_t k1, k2;
};
template <int A>
RTP_DEV void pre_setup(PreRay& r, f3 o, f3 d) {
  constexpr int B = (A + 1) % 3, C = (A + 2) % 3;
  r.inv = __builtin_amdgcn_rcpf(comp<A>(d));
  r.oa = comp<A>(o);
  r.obc = f2v{comp<B>(o), comp<C>(o)};
  r.dbc = f2v{comp<B>(d), comp<C>(d)};
}
RTP_DEV void pre_fold(PreRay& r, const PreQuad& P) {
  const float t = (P.x - r.oa) * r.inv;
  const f2v u = __builtin_elementwise_fma(f2v{t, t}, r.dbc, r.obc) - f2v{P.cb, P.cc};
  const float ub = fabsf(u.x) - P.rb, uc = fabsf(u.y) - P.rc;
  const float m = __builtin_fmaf(fabsf(t), r.ma, r.mb);
  const bool ok = (fmaxf(ub, uc) <= m) & (t > kPreTmin);
  uint32_t key;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(key) : "v"(__float_as_uint(t - m)), "v"(~31u), "s"((uint32_t)P.qpos));
  key = ok ? key : ~0u;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r.k2) : "v"(r.k1), "v"(r.k2), "v"(key));
  r.k1 = min(r.k1, key);
}
template <int A>
RTP_DEV void pre_axis2(const DevScene* __restrict__ sc, int b, int e, f3 oa, f3 da, PreRay& ra, f3 ob, f3 db, PreRay& rb,
                       u8v& cur) {
  if (b == e) return;
  pre_setup<A>(ra, oa, da);
  pre_setup<A>(rb, ob, db);
  auto as_pre = [](const u8v& v) {
    PreQuad P;
    __builtin_memcpy(&P, &v, sizeof(P));
    return P;
  };
  const PreQuad* pq = sc->pre + b;
  for (int n = e - b; n > 0; n -= 2, pq += 2) {
    const u8v nxt = *reinterpret_cast<const u8v*>(pq + 1);
    const PreQuad P0 = as_pre(cur);
    pre_fold(ra, P0);
    pre_fold(rb, P0);
    if (n == 1) {
      cur = nxt;
      break;
    }
    cur = *reinterpret_cast<const u8v*>(pq + 2);
    const PreQuad P1 = as_pre(nxt);
    pre_fold(ra, P1);
    pre_fold(rb, P1);
  }
}
RTP_DEV void pre_candidate(f3 o, f3 d, const PreRay& r, bool lane_ok, const float* lds_prex, uint64_t& key) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* lx = reinterpret_cast<const f4v*>(lds_prex) + 4 * (r.k1 & 31u);
  f4v xr[4] = {lx[0], lx[1], lx[2], lx[3]};
  if (lane_ok && r.k1 != ~0u) {
    PreExact Q;
    __builtin_memcpy(&Q, xr, sizeof(Q));
    float t;
    const bool ok = quad_hit_axis(Q, o, d, t);
    const uint64_t kq = (uint64_t)__float_as_uint(t) << 32 | Q.key_lo;
    key = (ok && t > 0.001f && kq < key) ? kq : key;
  }
}
RTP_DEV bool pre_lane_ok(f3 o, f3 d) {
  return (int)(fabsf(o.x) <= kPreLimD) & (int)(fabsf(o.y) <= kPreLimD) & (int)(fabsf(o.z) <= kPreLimD) &
         (int)(fabsf(d.x) <= kPreLimD) & (int)(fabsf(d.y) <= kPreLimD) & (int)(fabsf(d.z) <= kPreLimD);
}
RTP_DEV void pre_margins(const DevScene* __restrict__ sc, f3 o, f3 d, PreRay& r) {
  const float dmax = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), 1.0f));
  const float omax = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
  r.ma = kPreK * dmax;
  r.mb = kPreK * (omax + (sc->pre_scale + 1.0f));
  r.k1 = ~0u;
  r.k2 = ~0u;
}
RTP_DEV Hit key_hit(const DevScene* __restrict__ sc, uint64_t key, f3 o, f3 d) {
  Hit h{3.40282347e+38f, -1, 0};
  if (key != kNoHitKey) {
    h.t = __uint_as_float((uint32_t)(key >> 32));
    h.kind = 0;
    h.idx = (int)(key & 0xffu);
  }
  const int ns = sc->n_spheres;
  for (int k = 0; k < ns; k++) {
    const DevSphere& S = sc->spheres[k];
    float t;
    if (sphere_hit(o, d, 0.001f, h.t, ld3(S.c), S.rr, t)) {
      h.t = t;
      h.kind = 1;
      h.idx = k;
    }
  }
  return h;
}
RTP_DEV void closest_hit2(const DevScene* __restrict__ sc, f3 oa, f3 da, Hit& ha, bool act_a, f3 ob, f3 db, Hit& hb,
                          bool act_b, const float* lds_prex) {
  uint64_t ka = kNoHitKey, kb = kNoHitKey;
  {
    const int g6 = sc->kind_begin[6], g7 = sc->kind_begin[7], g8 = sc->kind_begin[8], g9 = sc->kind_begin[9],
              g10 = sc->kind_begin[10], g11 = sc->kind_begin[11];
    u16v cur = quad_head(sc, g6);
    scan_kind_pf2<7>(sc, g6, g7, oa, da, ka, ob, db, kb, cur);
    scan_kind_pf2<8>(sc, g7, g8, oa, da, ka, ob, db, kb, cur);
    scan_kind_pf2<9>(sc, g8, g9, oa, da, ka, ob, db, kb, cur);
    scan_kind_pf2<10>(sc, g9, g10, oa, da, ka, ob, db, kb, cur);
    scan_kind_pf2<0>(sc, g10, g11, oa, da, ka, ob, db, kb, cur);
  }
  bool fa = true, fb = true;  // the lane needs the exact scan of the axis-plane quads for ray A / B
  if (sc->n_pre > 0) {          // (wave-uniform)
    const bool oka = pre_lane_ok(oa, da), okb = pre_lane_ok(ob, db);
    PreRay ra, rb;
    pre_margins(sc, oa, da, ra);
    pre_margins(sc, ob, db, rb);
    const int p0 = sc->pre_begin[0], p1 = sc->pre_begin[1], p2 = sc->pre_begin[2], p3 = sc->pre_begin[3];
    u8v pcur = pre_rec(sc, p0);
    pre_axis2<0>(sc, p0, p1, oa, da, ra, ob, db, rb, pcur);
    pre_axis2<1>(sc, p1, p2, oa, da, ra, ob, db, rb, pcur);
    pre_axis2<2>(sc, p2, p3, oa, da, ra, ob, db, rb, pcur);
    pre_candidate(oa, da, ra, oka, lds_prex, ka);
    pre_candidate(ob, db, rb, okb, lds_prex, kb);
    fa = !oka || (ra.k2 & ~31u) <= (uint32_t)(ka >> 32);
    fb = !okb || (rb.k2 & ~31u) <= (uint32_t)(kb >> 32);
  }
  fa = fa && act_a;
  fb = fb && act_b;
  if (__ballot(fa | fb)) {
    if (fa | fb) {  // the exact scan for both rays (a full scan's minimum is the exact one either way)
      const int g0 = sc->kind_begin[0], g1 = sc->kind_begin[1], g2 = sc->kind_begin[2], g3 = sc->kind_begin[3],
                g4 = sc->kind_begin[4], g5 = sc->kind_begin[5], g6 = sc->kind_begin[6];
      u16v cur = quad_head(sc, g0);
      scan_kind_pf2<1>(sc, g0, g1, oa, da, ka, ob, db, kb, cur);
      scan_kind_pf2<2>(sc, g1, g2, oa, da, ka, ob, db, kb, cur);
      scan_kind_pf2<3>(sc, g2, g3, oa, da, ka, ob, db, kb, cur);
      scan_kind_pf2<4>(sc, g3, g4, oa, da, ka, ob, db, kb, cur);
      scan_kind_pf2<5>(sc, g4, g5, oa, da, ka, ob, db, kb, cur);
      scan_kind_pf2<6>(sc, g5, g6, oa, da, ka, ob, db, kb, cur);
    }
  }
  ha = key_hit(sc, ka, oa, da);
  hb = key_hit(sc, kb, ob, db);
}

// the two parts of closest_hit (rtp_kernels.hip), each alone
template <int kPart>
RTP_DEV uint64_t ch_part(const DevScene* __restrict__ sc, f3 o, f3 d, const float* lds_prex) {
  uint64_t key = kNoHitKey;
  if constexpr (kPart == 0) {
    const int g6 = sc->kind_begin[6], g7 = sc->kind_begin[7], g8 = sc->kind_begin[8], g9 = sc->kind_begin[9],
              g10 = sc->kind_begin[10], g11 = sc->kind_begin[11];
    u16v cur = quad_head(sc, g6);
    scan_kind_pf<7>(sc, g6, g7, o, d, key, cur);
    scan_kind_pf<8>(sc, g7, g8, o, d, key, cur);
    scan_kind_pf<9>(sc, g8, g9, o, d, key, cur);
    scan_kind_pf<10>(sc, g9, g10, o, d, key, cur);
    scan_kind_pf<0>(sc, g10, g11, o, d, key, cur);
  } else {
    const float dmax = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fmaxf(fabsf(d.z), 1.0f));
    const float omax = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float ma = kPreK * dmax, mb = kPreK * (omax + (sc->pre_scale + 1.0f));
    uint32_t k1 = ~0u, k2 = ~0u;
    const int p0 = sc->pre_begin[0], p1 = sc->pre_begin[1], p2 = sc->pre_begin[2], p3 = sc->pre_begin[3];
    u8v pcur = pre_rec(sc, p0);
    pre_axis<0>(sc, p0, p1, o, d, ma, mb, k1, k2, pcur);
    pre_axis<1>(sc, p1, p2, o, d, ma, mb, k1, k2, pcur);
    pre_axis<2>(sc, p2, p3, o, d, ma, mb, k1, k2, pcur);
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v* lx = reinterpret_cast<const f4v*>(lds_prex) + 4 * (k1 & 31u);
    f4v xr[4] = {lx[0], lx[1], lx[2], lx[3]};
    if (k1 != ~0u) {
      PreExact Q;
      __builtin_memcpy(&Q, xr, sizeof(Q));
      float t;
      const bool ok = quad_hit_axis(Q, o, d, t);
      const uint64_t kq = (uint64_t)__float_as_uint(t) << 32 | Q.key_lo;
      key = (ok && t > 0.001f && kq < key) ? kq : key;
    }
    key ^= (uint64_t)k2;
  }
  return key;
}

template <int kMode>
__global__ void __launch_bounds__(256) lat_kernel(const DevScene* __restrict__ sc, int iters, float4* hist,
                                                  const uint32_t* __restrict__ tab, unsigned long long* cycles,
                                                  float* sink) {
  __shared__ __align__(16) float s_qshade[kQTableFloats];
  fill_qshade(sc, s_qshade);
  __syncthreads();
  const int gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  constexpr bool kSplit = kMode == 8 || kMode == 9 || kMode == 10;  // lane pairs share a ray (identical per-lane state)
  const int ray = kSplit ? (int)(blockIdx.x * blockDim.x + threadIdx.x) >> 1 : (int)(blockIdx.x * blockDim.x + threadIdx.x);
  uint32_t seed = 0x9e3779b9u * (ray + 1);
  Path ps;
  ps.org = rand_point(seed);
  ps.dir = rand_dir(seed);
  ps.d = 0;
  ps.nonfinite = false;
  float acc = 0.f;
  float4* hd = hist + ray;
  // the second ray of modes 11..13 (its own seed and history row)
  uint32_t seedb = 0x85ebca6bu * (ray + 1) + 17u;
  Path pb;
  pb.org = rand_point(seedb);
  pb.dir = rand_dir(seedb);
  pb.d = 0;
  pb.nonfinite = false;
  float4* hdb = hist + (size_t)gridDim.x * blockDim.x + ray;
  Hit h0{};
  Path p0 = ps;
  if (kMode == 3) h0 = closest_hit<false>(sc, ps.org, ps.dir, true, nullptr, s_qshade + kPrexLdsOffset);
  uint32_t ts = seed;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if constexpr (kMode == 4) {
      ts = tab[ts];
      acc += (float)(ts & 1u);
    } else if constexpr (kMode == 5) {
      acc += ps.dir.x;
      ps.org = add(ps.org, scl(ps.dir, 1e-3f * randf(seed)));
      ps.dir = rand_dir(seed);
    } else if constexpr (kMode == 6 || kMode == 7) {
      const uint64_t k = ch_part<kMode - 6>(sc, ps.org, ps.dir, s_qshade + kPrexLdsOffset);
      acc += __uint_as_float((uint32_t)(k >> 32) & 0x3fffffffu);
      ps.org = add(ps.org, scl(ps.dir, 1e-3f * randf(seed)));
      ps.dir = rand_dir(seed);
    } else if constexpr (kSplit) {
      const Hit h = closest_hit_split(sc, ps.org, ps.dir, s_qshade + kPrexLdsOffset);
      if constexpr (kMode == 10) {
        const Hit w = closest_hit<false>(sc, ps.org, ps.dir, true, nullptr, s_qshade + kPrexLdsOffset);
        acc += (__float_as_uint(w.t) != __float_as_uint(h.t) || w.kind != h.kind || w.idx != h.idx) ? 1.f : 0.f;
        ps.org = h.kind >= 0 ? add(ps.org, scl(ps.dir, h.t)) : rand_point(seed);
        ps.dir = rand_dir(seed);
      } else if constexpr (kMode == 8) {
        acc += h.t;
        ps.org = h.kind >= 0 ? add(ps.org, scl(ps.dir, h.t)) : rand_point(seed);
        ps.dir = rand_dir(seed);
      } else {
        f3 emit;
        const int r = shade_hit<false, true>(sc, ps, seed, emit, hd, 50, s_qshade, h);
        if (r != kAlive) {
          acc += emit.x;
          ps.org = rand_point(seed);
          ps.dir = rand_dir(seed);
        }
      }
    } else if constexpr (kMode >= 11) {
      Hit ha, hb;
      closest_hit2(sc, ps.org, ps.dir, ha, true, pb.org, pb.dir, hb, true, s_qshade + kPrexLdsOffset);
      if constexpr (kMode == 13) {  // check against closest_hit on the same rays
        const Hit wa = closest_hit<false>(sc, ps.org, ps.dir, true, nullptr, s_qshade + kPrexLdsOffset);
        const Hit wb = closest_hit<false>(sc, pb.org, pb.dir, true, nullptr, s_qshade + kPrexLdsOffset);
        acc += (__float_as_uint(wa.t) != __float_as_uint(ha.t) || wa.kind != ha.kind || wa.idx != ha.idx) ? 1.f : 0.f;
        acc += (__float_as_uint(wb.t) != __float_as_uint(hb.t) || wb.kind != hb.kind || wb.idx != hb.idx) ? 1.f : 0.f;
      }
      if constexpr (kMode == 11 || kMode == 13) {
        if constexpr (kMode == 11) acc += ha.t + hb.t;
        ps.org = ha.kind >= 0 ? add(ps.org, scl(ps.dir, ha.t)) : rand_point(seed);
        ps.dir = rand_dir(seed);
        pb.org = hb.kind >= 0 ? add(pb.org, scl(pb.dir, hb.t)) : rand_point(seedb);
        pb.dir = rand_dir(seedb);
      } else {
        f3 emit;
        const int r = shade_hit<false, true>(sc, ps, seed, emit, hd, 50, s_qshade, ha);
        if (r != kAlive) {
          acc += emit.x;
          ps.org = rand_point(seed);
          ps.dir = rand_dir(seed);
        }
        const int rb = shade_hit<false, true>(sc, pb, seedb, emit, hdb, 50, s_qshade, hb);
        if (rb != kAlive) {
          acc += emit.x;
          pb.org = rand_point(seedb);
          pb.dir = rand_dir(seedb);
        }
      }
    } else if constexpr (kMode == 3) {
      ps = p0;
      f3 emit;
      const int r = shade_hit<false, true>(sc, ps, seed, emit, hd, 50, s_qshade, h0);
      acc += ps.dir.x + (float)r;
    } else {
      const Hit h = closest_hit<false>(sc, ps.org, ps.dir, kMode != 2, nullptr, s_qshade + kPrexLdsOffset);
      if constexpr (kMode == 0 || kMode == 2) {
        acc += h.t;
        ps.org = h.kind >= 0 ? add(ps.org, scl(ps.dir, h.t)) : rand_point(seed);
        ps.dir = rand_dir(seed);
      } else {
        f3 emit;
        const int r = shade_hit<false, true>(sc, ps, seed, emit, hd, 50, s_qshade, h);
        if (r != kAlive) {
          acc += emit.x;
          ps.org = rand_point(seed);
          ps.dir = rand_dir(seed);
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cycles[gw] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void fill_tab(uint32_t* t, uint64_t n, uint64_t base) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t x = (uint32_t)(base + i) * 2654435761u;
    x ^= x >> 15;
    t[i] = x * 2246822519u;
  }
}

template <int kMode>
void run(const DevScene* sc, int cus, int w, int iters, float4* hist, const uint32_t* tab, unsigned long long* cyc,
         float* sink) {
  const int blocks = cus * w;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(lat_kernel<kMode>, dim3(blocks), dim3(256), 0, nullptr, sc, 4, hist, tab, cyc, sink);  // warm
  (void)hipEventRecord(a, nullptr);
  hipLaunchKernelGGL(lat_kernel<kMode>, dim3(blocks), dim3(256), 0, nullptr, sc, iters, hist, tab, cyc, sink);
  (void)hipEventRecord(b, nullptr);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned long long> c((size_t)blocks * 4);
  (void)hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
  double sum = 0, mx = 0;
  for (auto v : c) sum += (double)v, mx = std::max(mx, (double)v);
  double bad = 0;
  if (kMode == 10 || kMode == 13) {
    std::vector<float> sk((size_t)blocks * 256);
    (void)hipMemcpy(sk.data(), sink, sk.size() * 4, hipMemcpyDeviceToHost);
    for (float v : sk) bad += v;
  }
  printf("{\"mismatches\": %.0f, \"mode\": %d, \"waves_per_simd\": %d, \"iters\": %d, \"kernel_ms\": %.3f, \"cycles_per_step\": %.1f, "
         "\"max_cycles_per_step\": %.1f, \"ns_per_step_wall\": %.2f, \"wave_steps_per_us\": %.1f}\n",
         bad, kMode, w, iters, ms, sum / c.size() / iters, mx / iters, ms * 1e6 / iters, (double)c.size() * iters / (ms * 1e3));
  fflush(stdout);
}
}  // namespace lb

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  std::vector<int> modes;
  for (int i = 2; i < argc; i++) modes.push_back(atoi(argv[i]));
  if (modes.empty()) modes = {0, 1, 2, 3, 4, 5, 6, 7};
  rtp_context* ctx = nullptr;
  if (rtp_create(0, &ctx) != RTP_OK) {
    fprintf(stderr, "rtp_create: %s\n", rtp_last_error());
    return 1;
  }
  rtp_scene_desc d{};
  if (rtp_cornell_box(0, &d) != RTP_OK || rtp_set_scene(ctx, &d) != RTP_OK) {
    fprintf(stderr, "scene: %s\n", rtp_last_error());
    return 1;
  }
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int maxw = 5;
  float4* hist = nullptr;
  uint32_t* tab = nullptr;
  unsigned long long* cyc = nullptr;
  float* sink = nullptr;
  (void)hipMalloc(&hist, (size_t)cus * maxw * 256 * 16 * 64);
  (void)hipMalloc(&cyc, (size_t)cus * maxw * 4 * 8);
  (void)hipMalloc(&sink, (size_t)cus * maxw * 256 * 4);
  const size_t tab_n = (size_t)1 << 32;
  bool have_tab = false;
  for (int m : modes) have_tab |= m == 4;
  if (have_tab) {  // a scrambled map: the gather chain is data-dependent and spans the whole table
    if (hipMalloc(&tab, tab_n * 4) != hipSuccess) return 1;
    for (uint64_t base = 0; base < tab_n; base += 1ull << 30)  // (a dispatch holds < 2^32 work-items)
      hipLaunchKernelGGL(lb::fill_tab, dim3((unsigned)((1ull << 30) / 256)), dim3(256), 0, nullptr, tab + base,
                         (uint64_t)(1ull << 30), base);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
  }
  for (int m : modes)
    for (int w = 1; w <= maxw; w++) {
      switch (m) {
        case 0: lb::run<0>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 1: lb::run<1>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 2: lb::run<2>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 3: lb::run<3>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 4: lb::run<4>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 5: lb::run<5>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 6: lb::run<6>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 7: lb::run<7>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 8: lb::run<8>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 9: lb::run<9>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 10: lb::run<10>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 11: lb::run<11>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 12: lb::run<12>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        case 13: lb::run<13>(ctx->d_scene, cus, w, iters, hist, tab, cyc, sink); break;
        default: break;
      }
    }
  rtp_destroy(ctx);
  return 0;
}
