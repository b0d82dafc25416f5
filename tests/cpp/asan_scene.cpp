// asan_scene.cpp -- the C ABI's scene and render entry points under the host
// AddressSanitizer + UBSan (built by build.build_asan(): every host
// translation unit of librtp -- rtp_host.cpp, rtp_direct_host.cpp,
// scene_cornell.cpp and the launch stubs of the .hip files -- compiled with
// -Xarch_host -fsanitize=address,undefined; device code unchanged).
//
// Without a HIP device: rtp_create must fail with RTP_ERR_DEVICE and the
// host-only helpers (scene tables, normalise, PNM) run sanitized.
// With one: the scene replacements the reference's ctor/SetData sequence can
// produce (MapperPathTracer.cxx:100-140 builds the scene per mapper), i.e.
// Cornell -> the C3 sphere BVH (host SAH and device LBVH) -> Cornell, each
// followed by a small render, and the octant mask read back from the device
// scene (the mask was once read from freed memory).
// Prints "OK nodev" or "OK gpu" and exits 0 when every check passes.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rtp.h"

static int failures = 0;
#define EXPECT(cond)                                               \
  do {                                                             \
    if (!(cond)) {                                                 \
      std::fprintf(stderr, "FAIL %d: %s (%s)\n", __LINE__, #cond,  \
                   rtp_last_error() ? rtp_last_error() : "");      \
      failures++;                                                  \
    }                                                              \
  } while (0)

static void host_helpers(const char* pnm) {
  rtp_scene_desc d{};
  for (int v = 0; v < 4; v++) EXPECT(rtp_cornell_box(v, &d) == RTP_OK && d.n_quads > 0);
  EXPECT(rtp_cornell_box(3, &d) == RTP_OK && d.n_spheres == 1000);
  std::vector<float> px = {4.f, NAN, 16.f, 7.f, 0.f, 1.f, 2.f, 3.f};
  EXPECT(rtp_normalize(px.data(), 2, 4) == RTP_OK && px[0] == 1.f && px[1] == 0.f);
  EXPECT(rtp_write_pnm(pnm, px.data(), 2, 1) == RTP_OK);
}

static rtp_camera cornell_camera() {
  // main.cc:616-622 (rtp::DefaultCamera)
  rtp_camera c{};
  const float a = (float)(278 / 555.0), b = (float)(-800 / 555.0);
  for (int k = 0; k < 3; k++) c.position[k] = k == 2 ? b : a, c.look_at[k] = a, c.view_up[k] = k == 1 ? 1.f : 0.f;
  c.fov_y_deg = 40.f;
  return c;
}

static void render_small(rtp_context* ctx) {
  const int nx = 16, ny = 12, spp = 2, depth = 8;
  std::vector<float> rgba((size_t)4 * nx * ny, -1.f);
  rtp_stats st{};
  const rtp_camera cam = cornell_camera();
  EXPECT(rtp_render(ctx, &cam, nx, ny, spp, depth, 0, rgba.data(), &st) == RTP_OK);
  EXPECT(st.samples == (uint64_t)nx * ny * spp);
  int finite = 0;
  for (int i = 0; i < nx * ny; i++) finite += std::isfinite(rgba[4 * i]) && rgba[4 * i] >= 0.f;
  EXPECT(finite > nx * ny / 2);
}

int main(int argc, char** argv) {
  host_helpers(argc > 1 ? argv[1] : "/tmp/rtp_asan_scene.pnm");
  rtp_context* ctx = nullptr;
  const rtp_status st = rtp_create(0, &ctx);
  if (st == RTP_ERR_DEVICE) {
    EXPECT(ctx == nullptr);
    if (failures) return 1;
    std::printf("OK nodev\n");
    return 0;
  }
  EXPECT(st == RTP_OK && ctx);
  if (!ctx) return 1;
  rtp_scene_desc d{};
  const char* builds[2] = {"host", "gpu"};
  for (const char* b : builds) {
    setenv("RTP_BVH_BUILD", b, 1);
    EXPECT(rtp_cornell_box(0, &d) == RTP_OK && rtp_set_scene(ctx, &d) == RTP_OK);
    EXPECT(rtp_sphere_walk_oct_mask(ctx) == -1);
    render_small(ctx);
    EXPECT(rtp_cornell_box(3, &d) == RTP_OK && rtp_set_scene(ctx, &d) == RTP_OK);
    EXPECT(rtp_sphere_walk(ctx) == 1);
    EXPECT(rtp_sphere_walk_oct_mask(ctx) == 7);
    render_small(ctx);
  }
  setenv("RTP_BVH_OCT_MASK", "3", 1);  // the host build honours the experiment's narrower mask
  setenv("RTP_BVH_BUILD", "host", 1);
  EXPECT(rtp_cornell_box(3, &d) == RTP_OK && rtp_set_scene(ctx, &d) == RTP_OK);
  EXPECT(rtp_sphere_walk_oct_mask(ctx) == 3);
  unsetenv("RTP_BVH_OCT_MASK");
  EXPECT(rtp_cornell_box(0, &d) == RTP_OK && rtp_set_scene(ctx, &d) == RTP_OK);
  EXPECT(rtp_sphere_walk_oct_mask(ctx) == -1);
  render_small(ctx);
  rtp_destroy(ctx);
  if (failures) return 1;
  std::printf("OK gpu\n");
  return 0;
}
