// bvh_walk_sim.cpp -- CPU walk statistics of sphere-BVH layouts on the C3
// scene (development tool: which layout fits the LDS and what a walk costs).
//
// Builds the host's binned-SAH tree (rtp_host.cpp bvh_build: 16 bins, the
// same sphere-box pad) for a leaf-size bound, then walks random rays from
// points inside the room (outside every sphere), bounded by the walls, with
//   threaded: the 8 octant-ordered threaded copies (bvh_flatten, top-box drop
//             depth 2 + area ratio 0.6): one box or sphere per visit;
//   stack:    one copy, children as a pair (both boxes tested per visit, near
//             child first, far child pushed): visits, max stack depth;
//   wide4:    the binary tree collapsed to 4-wide nodes (a node's children are
//             its binary grandchildren, or children where those are leaves):
//             every child box tested per visit, hit children visited near to
//             far through a stack, sphere leaves tested after their box.
// Prints per-ray means: node visits, box tests, sphere tests, max stack depth,
// and the layout sizes.  `bvh_walk_sim <rays> builders`: one-sphere leaves
// built with 16 / 32 / 64 bins or a full sweep SAH, threaded visits per ray.  build: g++ -O2 -std=c++17 tools/bvh_walk_sim.cpp
//   -Iinclude -Lraytracingtherestofyourlife_amd -lrtp -Wl,-rpath,$PWD/raytracingtherestofyourlife_amd
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rtp.h"

struct Prim {
  float lo[3], hi[3], cen[3];
  int idx;
};
struct Node {
  float lo[3], hi[3];
  int axis = 0, left = -1, right = -1, first = 0, count = 0, depth = 0;
};
static float half_area(const float* lo, const float* hi) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}
static int build(std::vector<Prim>& P, int b, int e, std::vector<Node>& T, std::vector<int>& order, int leaf, int depth) {
  const int me = (int)T.size();
  T.emplace_back();
  Node nd;
  nd.depth = depth;
  float clo[3], chi[3];
  for (int k = 0; k < 3; k++) nd.lo[k] = clo[k] = INFINITY, nd.hi[k] = chi[k] = -INFINITY;
  for (int i = b; i < e; i++)
    for (int k = 0; k < 3; k++) {
      nd.lo[k] = std::min(nd.lo[k], P[i].lo[k]);
      nd.hi[k] = std::max(nd.hi[k], P[i].hi[k]);
      clo[k] = std::min(clo[k], P[i].cen[k]);
      chi[k] = std::max(chi[k], P[i].cen[k]);
    }
  const int n = e - b;
  if (n <= leaf) {
    nd.first = (int)order.size();
    nd.count = n;
    for (int i = b; i < e; i++) order.push_back(P[i].idx);
    T[me] = nd;
    return me;
  }
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
      int j = std::min(kBins - 1, std::max(0, (int)((P[i].cen[ax] - clo[ax]) / ext * kBins)));
      cnt[j]++;
      for (int k = 0; k < 3; k++) blo[j][k] = std::min(blo[j][k], P[i].lo[k]), bhi[j][k] = std::max(bhi[j][k], P[i].hi[k]);
    }
    for (int s = 1; s < kBins; s++) {
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
    auto bin = [&](const Prim& x) { return std::min(kBins - 1, std::max(0, (int)((x.cen[ax] - clo[ax]) / ext * kBins))); };
    mid = (int)(std::stable_partition(P.begin() + b, P.begin() + e, [&](const Prim& x) { return bin(x) < best_split; }) -
                P.begin());
    nd.axis = ax;
  } else {
    mid = b + n / 2;
  }
  nd.left = build(P, b, mid, T, order, leaf, depth + 1);
  nd.right = build(P, mid, e, T, order, leaf, depth + 1);
  T[me] = nd;
  return me;
}

// the same recursion with B bins per axis, or B = 0: a full sweep (every
// split between centroid-sorted neighbours on each axis, ties by index)
static int build_b(std::vector<Prim>& P, int b, int e, std::vector<Node>& T, std::vector<int>& order, int B, int depth) {
  if (B > 0 && B != 16) {
    // binned with B bins (copy of build()'s logic with a runtime bin count)
    const int me = (int)T.size();
    T.emplace_back();
    Node nd;
    nd.depth = depth;
    float clo[3], chi[3];
    for (int k = 0; k < 3; k++) nd.lo[k] = clo[k] = INFINITY, nd.hi[k] = chi[k] = -INFINITY;
    for (int i = b; i < e; i++)
      for (int k = 0; k < 3; k++) {
        nd.lo[k] = std::min(nd.lo[k], P[i].lo[k]), nd.hi[k] = std::max(nd.hi[k], P[i].hi[k]);
        clo[k] = std::min(clo[k], P[i].cen[k]), chi[k] = std::max(chi[k], P[i].cen[k]);
      }
    const int n = e - b;
    if (n <= 1) {
      nd.first = (int)order.size();
      nd.count = n;
      for (int i = b; i < e; i++) order.push_back(P[i].idx);
      T[me] = nd;
      return me;
    }
    int best_ax = -1, best_split = 0;
    float best_cost = INFINITY;
    std::vector<int> cnt(B);
    std::vector<float> blo(3 * B), bhi(3 * B);
    for (int ax = 0; ax < 3; ax++) {
      const float ext = chi[ax] - clo[ax];
      if (!(ext > 0)) continue;
      std::fill(cnt.begin(), cnt.end(), 0);
      std::fill(blo.begin(), blo.end(), INFINITY);
      std::fill(bhi.begin(), bhi.end(), -INFINITY);
      for (int i = b; i < e; i++) {
        const int j = std::min(B - 1, std::max(0, (int)((P[i].cen[ax] - clo[ax]) / ext * B)));
        cnt[j]++;
        for (int k = 0; k < 3; k++) blo[3 * j + k] = std::min(blo[3 * j + k], P[i].lo[k]), bhi[3 * j + k] = std::max(bhi[3 * j + k], P[i].hi[k]);
      }
      for (int sp = 1; sp < B; sp++) {
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int nl = 0, nr = 0;
        for (int j = 0; j < B; j++) {
          if (!cnt[j]) continue;
          float* lo = j < sp ? llo : rlo;
          float* hi = j < sp ? lhi : rhi;
          (j < sp ? nl : nr) += cnt[j];
          for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], blo[3 * j + k]), hi[k] = std::max(hi[k], bhi[3 * j + k]);
        }
        if (!nl || !nr) continue;
        const float cost = nl * half_area(llo, lhi) + nr * half_area(rlo, rhi);
        if (cost < best_cost) best_cost = cost, best_ax = ax, best_split = sp;
      }
    }
    int mid = b + n / 2;
    if (best_ax >= 0) {
      const int ax = best_ax;
      const float ext = chi[ax] - clo[ax];
      mid = (int)(std::stable_partition(P.begin() + b, P.begin() + e, [&](const Prim& x) {
                    return std::min(B - 1, std::max(0, (int)((x.cen[ax] - clo[ax]) / ext * B))) < best_split;
                  }) - P.begin());
      nd.axis = ax;
    }
    nd.left = build_b(P, b, mid, T, order, B, depth + 1);
    nd.right = build_b(P, mid, e, T, order, B, depth + 1);
    T[me] = nd;
    return me;
  }
  if (B == 16) return build(P, b, e, T, order, 1, depth);
  // full sweep
  const int me = (int)T.size();
  T.emplace_back();
  Node nd;
  nd.depth = depth;
  for (int k = 0; k < 3; k++) nd.lo[k] = INFINITY, nd.hi[k] = -INFINITY;
  for (int i = b; i < e; i++)
    for (int k = 0; k < 3; k++) nd.lo[k] = std::min(nd.lo[k], P[i].lo[k]), nd.hi[k] = std::max(nd.hi[k], P[i].hi[k]);
  const int n = e - b;
  if (n <= 1) {
    nd.first = (int)order.size();
    nd.count = n;
    for (int i = b; i < e; i++) order.push_back(P[i].idx);
    T[me] = nd;
    return me;
  }
  int best_ax = 0, best_i = n / 2;
  float best_cost = INFINITY;
  std::vector<float> racc(n);
  for (int ax = 0; ax < 3; ax++) {
    std::sort(P.begin() + b, P.begin() + e, [ax](const Prim& x, const Prim& y) {
      return x.cen[ax] < y.cen[ax] || (x.cen[ax] == y.cen[ax] && x.idx < y.idx);
    });
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = n - 1; i >= 1; i--) {  // right boxes: prims [i, n)
      for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], P[b + i].lo[k]), hi[k] = std::max(hi[k], P[b + i].hi[k]);
      racc[i] = (n - i) * half_area(lo, hi);
    }
    for (int k = 0; k < 3; k++) lo[k] = INFINITY, hi[k] = -INFINITY;
    for (int i = 1; i < n; i++) {  // left: prims [0, i)
      for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], P[b + i - 1].lo[k]), hi[k] = std::max(hi[k], P[b + i - 1].hi[k]);
      const float cost = i * half_area(lo, hi) + racc[i];
      if (cost < best_cost) best_cost = cost, best_ax = ax, best_i = i;
    }
  }
  const int ax = best_ax;
  std::sort(P.begin() + b, P.begin() + e, [ax](const Prim& x, const Prim& y) {
    return x.cen[ax] < y.cen[ax] || (x.cen[ax] == y.cen[ax] && x.idx < y.idx);
  });
  nd.axis = ax;
  nd.left = build_b(P, b, b + best_i, T, order, B, depth + 1);
  nd.right = build_b(P, b + best_i, e, T, order, B, depth + 1);
  T[me] = nd;
  return me;
}

struct Sph {
  float c[3], r, rr;
};
static bool sphere_t(const float* o, const float* d, const Sph& s, float& t) {
  const float oc[3] = {o[0] - s.c[0], o[1] - s.c[1], o[2] - s.c[2]};
  const float a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
  const float b = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
  const float c = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - s.rr;
  const float disc = b * b - a * c;
  if (!(disc > 0)) return false;
  const float sq = std::sqrt(disc);
  float r1 = (-b - sq) / a;
  t = r1 > 0.001f ? r1 : (-b + sq) / a;
  return t > 0.001f;
}
static bool box_hit(const float* o, const float* inv, const float* lo, const float* hi, float tmax, float& tn) {
  float t0 = 0.f, t1 = tmax;
  for (int k = 0; k < 3; k++) {
    float a = (lo[k] - o[k]) * inv[k], b = (hi[k] - o[k]) * inv[k];
    if (a > b) std::swap(a, b);
    t0 = std::max(t0, a);
    t1 = std::min(t1, b);
  }
  tn = t0;
  return t0 <= t1;
}

// 4-wide collapse: the children of binary node i as up to 4 binary node ids
static int wide_children(const std::vector<Node>& T, int i, int out[4]) {
  int n = 0;
  for (int c : {T[i].left, T[i].right}) {
    if (T[c].left < 0) out[n++] = c;
    else out[n++] = T[c].left, out[n++] = T[c].right;
  }
  return n;
}
struct Stats {
  double visits = 0, boxes = 0, spheres = 0, maxstack = 0, pushes = 0;
  int maxstack_all = 0;
};

int main(int argc, char** argv) {
  const int nrays = argc > 1 ? atoi(argv[1]) : 20000;
  rtp_scene_desc d{};
  if (rtp_cornell_box(3, &d) != RTP_OK) {
    fprintf(stderr, "%s\n", rtp_last_error());
    return 1;
  }
  std::vector<Sph> S(d.n_spheres);
  for (int k = 0; k < d.n_spheres; k++) {
    const float* p = d.points + 3 * d.sphere_point[k];
    S[k] = {{p[0], p[1], p[2]}, d.sphere_radius[k], d.sphere_radius[k] * d.sphere_radius[k]};
  }
  // rays: origins inside the room outside every sphere, uniform directions
  uint32_t st = 12345;
  auto rnd = [&]() {
    st ^= st << 13, st ^= st >> 17, st ^= st << 5;
    return (st >> 8) * 0x1p-24f;
  };
  std::vector<float> rays;
  while ((int)rays.size() < 6 * nrays) {
    float o[3] = {0.01f + 0.98f * rnd(), 0.01f + 0.98f * rnd(), 0.01f + 0.98f * rnd()};
    bool inside = false;
    for (const Sph& s : S) {
      const float dx = o[0] - s.c[0], dy = o[1] - s.c[1], dz = o[2] - s.c[2];
      if (dx * dx + dy * dy + dz * dz <= s.rr) inside = true;
    }
    if (inside) continue;
    float v[3];
    for (;;) {
      v[0] = 2 * rnd() - 1, v[1] = 2 * rnd() - 1, v[2] = 2 * rnd() - 1;
      const float q = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
      if (q > 1e-3f && q <= 1) break;
    }
    rays.insert(rays.end(), {o[0], o[1], o[2], v[0], v[1], v[2]});
  }
  auto wall_t = [](const float* o, const float* dd) {
    float t = INFINITY;
    for (int k = 0; k < 3; k++) {
      if (dd[k] > 0) t = std::min(t, (1.f - o[k]) / dd[k]);
      if (dd[k] < 0) t = std::min(t, (0.f - o[k]) / dd[k]);
    }
    return t;
  };
  printf("# C3 scene: %d spheres; %d rays from points in the room\n", d.n_spheres, nrays);
  if (argc > 2 && !strcmp(argv[2], "quant")) {
    // binary "pair" nodes: a visit loads one 16-byte node holding BOTH
    // children's boxes quantised to `bits` per coordinate on a grid over the
    // root box (rounded outward), tests both, goes to the near hit child and
    // pushes the far one; a sphere child is tested exactly at once (one more
    // 16-byte load for its centre and r^2).  Loads per ray = node visits +
    // sphere tests, against the threaded walk's one load per visit.
    std::vector<Prim> P(S.size());
    for (size_t k = 0; k < S.size(); k++) {
      const float pad = 0.002f * S[k].r + 1e-5f;
      for (int a = 0; a < 3; a++)
        P[k].lo[a] = S[k].c[a] - S[k].r - pad, P[k].hi[a] = S[k].c[a] + S[k].r + pad, P[k].cen[a] = S[k].c[a];
      P[k].idx = (int)k;
    }
    std::vector<Node> T;
    std::vector<int> order;
    build(P, 0, (int)P.size(), T, order, 1, 0);
    for (int bits : {6, 8, 10, 16, 0}) {
      std::vector<Node> Q = T;  // quantised boxes (bits 0: exact)
      if (bits) {
        const float cells = (float)((1 << bits) - 1);
        for (Node& nd : Q)
          for (int a = 0; a < 3; a++) {
            const float lo0 = T[0].lo[a], ext = T[0].hi[a] - T[0].lo[a];
            nd.lo[a] = lo0 + ext * std::floor((nd.lo[a] - lo0) / ext * cells) / cells;
            nd.hi[a] = lo0 + ext * std::ceil((nd.hi[a] - lo0) / ext * cells) / cells;
          }
      }
      double visits = 0, sph = 0;
      int worst = 0;
      for (int r2 = 0; r2 < nrays; r2++) {
        const float* o2 = &rays[6 * r2];
        const float* d2 = o2 + 3;
        const float inv2[3] = {1.f / d2[0], 1.f / d2[1], 1.f / d2[2]};
        float best = wall_t(o2, d2);
        std::vector<std::pair<int, float>> stk;
        int cur = 0, v = 0, sp = 0;
        for (;;) {
          if (cur >= 0) {
            const Node& nd = Q[cur];
            v++;
            int nxt[2];
            float tnx[2];
            int nh = 0;
            for (int c : {nd.left, nd.right}) {
              float tn;
              if (!box_hit(o2, inv2, Q[c].lo, Q[c].hi, best, tn)) continue;
              if (Q[c].left < 0) {
                float t;
                sp++;
                if (sphere_t(o2, d2, S[order[Q[c].first]], t) && t < best) best = t;
                continue;
              }
              nxt[nh] = c, tnx[nh] = tn, nh++;
            }
            if (nh == 2) {
              if (tnx[1] < tnx[0]) std::swap(nxt[0], nxt[1]), std::swap(tnx[0], tnx[1]);
              stk.push_back({nxt[1], tnx[1]});
              worst = std::max(worst, (int)stk.size());
              cur = nxt[0];
            } else {
              cur = nh ? nxt[0] : -1;
            }
          } else {
            if (stk.empty()) break;
            auto e = stk.back();
            stk.pop_back();
            if (e.second <= best) cur = e.first;
          }
        }
        visits += v;
        sph += sp;
      }
      printf("pair nodes, boxes %s%d bits: %.2f node visits + %.2f sphere tests = %.2f 16-byte loads per ray (threaded: one per visit), max stack %d\n",
             bits ? "" : "exact (", bits, visits / nrays, sph / nrays, (visits + sph) / nrays, worst);
    }
    return 0;
  }
  if (argc > 2 && !strcmp(argv[2], "builders")) {  // one-sphere leaves: the tree builder's effect on the threaded walk
    for (int B : {16, 32, 64, 0}) {
      std::vector<Prim> P(S.size());
      for (size_t k = 0; k < S.size(); k++) {
        const float pad = 0.002f * S[k].r + 1e-5f;
        for (int a = 0; a < 3; a++)
          P[k].lo[a] = S[k].c[a] - S[k].r - pad, P[k].hi[a] = S[k].c[a] + S[k].r + pad, P[k].cen[a] = S[k].c[a];
        P[k].idx = (int)k;
      }
      std::vector<Node> T;
      std::vector<int> order;
      build_b(P, 0, (int)P.size(), T, order, B, 0);
      double sah = 0, v = 0, sp = 0;
      for (const Node& nd : T) sah += nd.left < 0 ? 0.0 : half_area(nd.lo, nd.hi);
      sah /= half_area(T[0].lo, T[0].hi);
      for (int r2 = 0; r2 < nrays; r2++) {
        const float* o2 = &rays[6 * r2];
        const float* d2 = o2 + 3;
        const float inv2[3] = {1.f / d2[0], 1.f / d2[1], 1.f / d2[2]};
        float best = wall_t(o2, d2);
        std::vector<int> stk{0};
        while (!stk.empty()) {
          const int i = stk.back();
          stk.pop_back();
          const Node& nd = T[i];
          v++;
          if (nd.left < 0) {
            float t;
            sp++;
            if (sphere_t(o2, d2, S[order[nd.first]], t) && t < best) best = t;
            continue;
          }
          float tn;
          if (!box_hit(o2, inv2, nd.lo, nd.hi, best, tn)) continue;
          const bool neg = d2[nd.axis] < 0;
          stk.push_back(neg ? nd.left : nd.right);
          stk.push_back(neg ? nd.right : nd.left);
        }
      }
      printf("builder %s%d: inner-node area sum / root %.2f | threaded walk %.2f visits %.2f sphere tests per ray\n",
             B ? "binned " : "sweep", B, sah, v / nrays, sp / nrays);
    }
    return 0;
  }
  for (int leaf : {1, 2, 3, 4, 6}) {
    std::vector<Prim> P(S.size());
    for (size_t k = 0; k < S.size(); k++) {
      const float pad = 0.002f * S[k].r + 1e-5f;
      for (int a = 0; a < 3; a++)
        P[k].lo[a] = S[k].c[a] - S[k].r - pad, P[k].hi[a] = S[k].c[a] + S[k].r + pad, P[k].cen[a] = S[k].c[a];
      P[k].idx = (int)k;
    }
    std::vector<Node> T;
    std::vector<int> order;
    build(P, 0, (int)P.size(), T, order, leaf, 0);
    int depth = 0, leaves = 0, inner = 0;
    for (const Node& n : T) depth = std::max(depth, n.depth), (n.left < 0 ? leaves : inner)++;
    // threaded walk = depth-first near-first traversal with box culling at every node (top drop ignored)
    Stats th, th_oracle, sk, wd;
    std::vector<double> depth_visits(32, 0.0);
    for (int r = 0; r < nrays; r++) {
      const float* o = &rays[6 * r];
      const float* dd = o + 3;
      const float inv[3] = {1.f / dd[0], 1.f / dd[1], 1.f / dd[2]};
      // threaded: visit node; if box hit (or leaf) continue into it (pass 0:
      // bounded by the walls; pass 1: by the true closest hit, the bound a
      // perfect first guess would give -- how many visits culling could save)
      float t_true = wall_t(o, dd);
      for (const Sph& s2 : S) {
        float t;
        if (sphere_t(o, dd, s2, t) && t < t_true) t_true = t;
      }
      for (int pass = 0; pass < 2; pass++) {
        Stats& acc = pass ? th_oracle : th;
        float best = pass ? t_true * 1.00001f : wall_t(o, dd);
        int visits = 0, spheres = 0;
        std::vector<int> stk{0};
        while (!stk.empty()) {
          const int i = stk.back();
          stk.pop_back();
          const Node& n = T[i];
          visits++;
          if (pass == 0) depth_visits[std::min(n.depth, 31)]++;
          if (n.left < 0 && n.count == 1) {  // embedded sphere: exact test, no box
            float t;
            spheres++;
            if (sphere_t(o, dd, S[order[n.first]], t) && t < best) best = t;
            continue;
          }
          float tn;
          if (!box_hit(o, inv, n.lo, n.hi, best, tn)) continue;
          if (n.left < 0) {
            for (int j = 0; j < n.count; j++) {
              float t;
              spheres++;
              if (sphere_t(o, dd, S[order[n.first + j]], t) && t < best) best = t;
            }
            continue;
          }
          const bool neg = dd[n.axis] < 0;
          stk.push_back(neg ? n.left : n.right);
          stk.push_back(neg ? n.right : n.left);
        }
        acc.visits += visits;
        acc.spheres += spheres;
      }
      // stack walk over child pairs
      {
        float best = wall_t(o, dd);
        int visits = 0, spheres = 0, boxes = 0, maxs = 0, pushes = 0;
        std::vector<std::pair<int, float>> stk;
        int cur = 0;
        for (;;) {
          if (cur >= 0) {
            const Node& n = T[cur];
            visits++;
            if (n.left < 0) {  // (root leaf only)
              for (int j = 0; j < n.count; j++) {
                float t;
                spheres++;
                if (sphere_t(o, dd, S[order[n.first + j]], t) && t < best) best = t;
              }
              cur = -1;
              continue;
            }
            int nxt[2];
            float tnx[2];
            int nh = 0;
            for (int c : {n.left, n.right}) {
              const Node& ch = T[c];
              float tn;
              boxes++;
              if (!box_hit(o, inv, ch.lo, ch.hi, best, tn)) continue;
              if (ch.left < 0) {
                for (int j = 0; j < ch.count; j++) {
                  float t;
                  spheres++;
                  if (sphere_t(o, dd, S[order[ch.first + j]], t) && t < best) best = t;
                }
                continue;
              }
              nxt[nh] = c, tnx[nh] = tn, nh++;
            }
            if (nh == 2) {
              if (tnx[1] < tnx[0]) std::swap(nxt[0], nxt[1]), std::swap(tnx[0], tnx[1]);
              stk.push_back({nxt[1], tnx[1]});
              pushes++;
              maxs = std::max(maxs, (int)stk.size());
              cur = nxt[0];
            } else if (nh == 1) {
              cur = nxt[0];
            } else {
              cur = -1;
            }
          } else {
            if (stk.empty()) break;
            auto e = stk.back();
            stk.pop_back();
            if (e.second <= best) cur = e.first;
          }
        }
        sk.visits += visits;
        sk.spheres += spheres;
        sk.boxes += boxes;
        sk.maxstack += maxs;
        sk.pushes += pushes;
        sk.maxstack_all = std::max(sk.maxstack_all, maxs);
      }
      // 4-wide walk
      {
        float best = wall_t(o, dd);
        int visits = 0, spheres = 0, boxes = 0, maxs = 0;
        std::vector<std::pair<int, float>> stk{{0, 0.f}};
        while (!stk.empty()) {
          auto e = stk.back();
          stk.pop_back();
          if (e.second > best) continue;
          const Node& n = T[e.first];
          if (n.left < 0) {  // a leaf (root only, or pushed leaf)
            for (int j = 0; j < n.count; j++) {
              float t;
              spheres++;
              if (sphere_t(o, dd, S[order[n.first + j]], t) && t < best) best = t;
            }
            continue;
          }
          visits++;
          int ch[4];
          const int nc = wide_children(T, e.first, ch);
          std::vector<std::pair<float, int>> hits;
          for (int k = 0; k < nc; k++) {
            float tn;
            boxes++;
            if (box_hit(o, inv, T[ch[k]].lo, T[ch[k]].hi, best, tn)) hits.push_back({tn, ch[k]});
          }
          std::sort(hits.begin(), hits.end());
          for (int k = (int)hits.size() - 1; k >= 0; k--) stk.push_back({hits[k].second, hits[k].first});
          maxs = std::max(maxs, (int)stk.size());
        }
        wd.visits += visits;
        wd.spheres += spheres;
        wd.boxes += boxes;
        wd.maxstack += maxs;
        wd.maxstack_all = std::max(wd.maxstack_all, maxs);
      }
    }
    const double n = nrays;
    printf("leaf<=%d: %d nodes (%d inner, %d leaves), depth %d | threaded: %.1f visits %.1f sphere tests per ray, "
           "8 octant copies x 16 B = %.0f KB | stack: %.1f visits %.1f box tests %.1f sphere tests %.2f pushes, "
           "max stack mean %.1f / worst %d, one copy x 32 B per inner node = %.0f KB\n",
           leaf, (int)T.size(), inner, leaves, depth, th.visits / n, th.spheres / n, 8.0 * T.size() * 16 / 1024,
           sk.visits / n, sk.boxes / n, sk.spheres / n, sk.pushes / n, sk.maxstack / n, sk.maxstack_all,
           inner * 32.0 / 1024);
    {
      double tot = 0, cum = 0;
      for (double v : depth_visits) tot += v;
      printf("   threaded visits by node depth (cumulative share; nodes at depth <= k per octant copy):");
      int nodes_le = 0;
      for (int k = 0; k < 14; k++) {
        cum += depth_visits[k];
        for (const Node& nd : T) nodes_le += nd.depth == k;
        printf(" %d:%.2f/%d", k, cum / tot, nodes_le);
      }
      printf("\n");
    }
    // fewer octant copies: near-first only at nodes split along a covered
    // axis (mask bit k: axis k's sign picks the copy), left child first elsewhere
    for (int cover : {7, 5, 1, 2, 4, 0}) {
      double v = 0;
      for (int r2 = 0; r2 < nrays; r2++) {
        const float* o2 = &rays[6 * r2];
        const float* d2 = o2 + 3;
        const float inv2[3] = {1.f / d2[0], 1.f / d2[1], 1.f / d2[2]};
        float best = wall_t(o2, d2);
        std::vector<int> stk{0};
        while (!stk.empty()) {
          const int i = stk.back();
          stk.pop_back();
          const Node& nd = T[i];
          v++;
          if (nd.left < 0 && nd.count == 1) {
            float t;
            if (sphere_t(o2, d2, S[order[nd.first]], t) && t < best) best = t;
            continue;
          }
          float tn;
          if (!box_hit(o2, inv2, nd.lo, nd.hi, best, tn)) continue;
          if (nd.left < 0) {
            for (int j = 0; j < nd.count; j++) {
              float t;
              if (sphere_t(o2, d2, S[order[nd.first + j]], t) && t < best) best = t;
            }
            continue;
          }
          const bool neg = ((cover >> nd.axis) & 1) && d2[nd.axis] < 0;
          stk.push_back(neg ? nd.left : nd.right);
          stk.push_back(neg ? nd.right : nd.left);
        }
      }
      printf("   threaded, copies for axes mask %d (%d copies): %.1f visits per ray\n", cover,
             1 << __builtin_popcount(cover), v / nrays);
    }
    printf("   threaded with the true hit as the initial bound: %.1f visits %.1f sphere tests per ray\n",
           th_oracle.visits / n, th_oracle.spheres / n);
    printf("   wide4: %.1f node visits %.1f box tests %.1f sphere tests per ray, max stack mean %.1f / worst %d; "
           "gathers per ray: threaded %.1f x 16 B = %.0f B, wide4 (48-B quantized nodes + 16-B spheres) %.1f x 16 B = %.0f B\n",
           wd.visits / n, wd.boxes / n, wd.spheres / n, wd.maxstack / n, wd.maxstack_all, th.visits / n,
           16 * th.visits / n, (3 * wd.visits + wd.spheres) / n, 16 * (3 * wd.visits + wd.spheres) / n);
  }
  return 0;
}
