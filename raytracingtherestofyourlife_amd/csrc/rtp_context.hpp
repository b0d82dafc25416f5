// rtp_context.hpp -- the rtp_context behind the C ABI (include/rtp.h),
// shared by rtp_host.cpp (path mode) and rtp_direct_host.cpp (-direct mode).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/rtp.h"

#include "rtp_layout.hpp"

struct rtp_context {
  int device = 0;
  rtp::DevScene* d_scene = nullptr;
  bool has_scene = false;
  float* d_hist = nullptr;
  size_t hist_bytes = 0;
  unsigned long long* d_dbg = nullptr;  // RTP_DEBUG_STATS=1: per-wave counters of the last launch
  int dbg_waves = 0;
  unsigned long long* d_progress = nullptr;  // global finished-sample counter of the pool kernel
  // many-sphere scenes: threaded BVH + sphere records (rtp_layout.hpp)
  rtp::BvhNode* d_nodes = nullptr;
  uint32_t* d_cnodes = nullptr;  // compact copy of d_nodes (the walks read it)
  int32_t* d_cidx = nullptr;     // scene index of each compact sphere leaf
  rtp::DevSphereG* d_sph_geom = nullptr;
  rtp::DevSphere* d_sph_all = nullptr;
  // the LDS walk's tree (rtp_layout.hpp kLdsWalkLeaf): compact nodes, their
  // embedded spheres' scene indices, leaf spheres (float4) and their indices
  uint32_t* d_lw_nodes = nullptr;
  int32_t* d_lw_cidx = nullptr;
  float* d_lw_sph = nullptr;
  int32_t* d_lw_orig = nullptr;
  int lw_bytes = 0;  // its LDS footprint (0: the scene has no LDS walk)
  bool use_bvh = false;
  int oct_mask = 0;  // the global walk's octant mask (DevScene::oct_mask) of the current scene
  int ff_policy = 0;  // rtp_ff_policy (RNG jump tables)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // Completion of the last launch.  The history buffer and the progress
  // counter are per-context scratch, so a launch on any stream first waits
  // for the previous one, and the host waits before it frees or rewrites a
  // buffer a queued kernel may still read.
  hipEvent_t done = nullptr;
  bool pending = false;
  // -direct mode (rtp_direct_host.cpp): reference index of each kept
  // (de-duplicated) quad in DevQuad::orig order, the reference's quad count,
  // the quads' shape bounds, and device scratch for the per-call scalar
  // table and colour map
  std::vector<int32_t> kept_quads;
  int32_t n_ref_quads = 0;
  float quad_lo[3] = {0, 0, 0}, quad_hi[3] = {0, 0, 0};
  float* d_direct = nullptr;
  size_t direct_bytes = 0;
};
// thread-local last-error message of the C ABI (rtp_host.cpp)
rtp_status rtp_internal_fail(rtp_status st, const std::string& msg);
