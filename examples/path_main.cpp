// path_main.cpp -- the path-traced modes of the reference's main.cc (parse,
// runPath, save, generateHemisphere; main.cc:54-119, 289-384, 385-427,
// 504-664) written against rtp/rendering.hpp, i.e. the reference driver on
// the MI355X path.
//
//   rtp_path [-x 128] [-y 128] [-samplecount 10] [-raydepth 5]
//            [-hemisphere [-phicount 15] [-thetacount 15]]
//            [-o output] [-raw prefix] [-variant 0] [-device 0]
//            [-rank 0 -world 1] [-dry-run]
//
// Writes <o>.pnm like main.cc, or <o>-<phi>-<theta>.pnm per hemisphere view
// (generate(), "%.4f" formatting).  -raw additionally dumps the normalised
// float RGBA buffer (nx*ny*4 float32, buffer order) to <raw> (single view) or
// <raw>-<phi>-<theta>.f32 (hemisphere) for bit-exact comparisons.  -rank/-world shard the hemisphere views (view v
// goes to rank v mod world; no communication).  -dry-run prints the views
// (phi, theta, camera position as float bit patterns) and renders nothing.
// -direct: the quad mappers' one-bounce AOVs (main.cc:623-651, generate()
// :399-420): direct.pnm, depth.pnm, normals.pnm, albedo.pnm (or
// direct-<phi>-<theta>.pnm ... per hemisphere view), all four from one launch.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include <cmath>
#include <cstdint>
#include <vector>

#include "rtp/rendering.hpp"

namespace {

struct View {
  float phi, theta;
  rtp::Vec3f pos;
};

// generateHemisphere (main.cc:504-561) with the parameters main() passes
// (:583-595): phi in [0, 1) by 1/phiCount, theta in [0, 2pi) by
// (float)(2pi)/thetaCount, radius -1078/555 around (278,278,278)/555.  Float
// variables as declared there; the phi bound is compared in double
// (phiEnd - 0.5*rPhi); cos/sin of float arguments are the float overloads.
std::vector<View> hemisphere_views(int phiCount, int thetaCount) {
  std::vector<View> v;
  const float phiBegin = 0.0, phiEnd = 1.0;
  const float thetaEnd = 2 * 3.14159265358979323846;  // 2*vtkm::Pi()
  const float rTheta = thetaEnd / (static_cast<float>(thetaCount));
  const float thetaBegin = 0;
  const float rPhi = (phiEnd - phiBegin) / float(phiCount);
  const float r = -1078 / 555.0;
  for (float phi = phiBegin; phi < (phiEnd - 0.5 * rPhi); phi += rPhi)
    for (float theta = thetaBegin; theta < thetaEnd; theta += rTheta) {
      const float px = r * std::cos(theta) * std::sin(phi);
      const float py = r * std::sin(theta) * std::sin(phi);
      const float pz = r * std::cos(phi);
      v.push_back({phi, theta, {(float)(px + 278 / 555.0), (float)(py + 278 / 555.0), (float)(pz + 278 / 555.0)}});
    }
  return v;
}

uint32_t bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

}  // namespace

int main(int argc, char** argv) {
  int x = 128, y = 128, s = 10, depth = 5, variant = 0, device = 0;  // main.cc:56-62 defaults
  int phiCount = 15, thetaCount = 15, rank = 0, world = 1;
  bool hemi = false, dry = false, direct = false;
  std::string out = "output", raw;
  for (int i = 1; i < argc; i++) {
    auto next = [&](const char* flag) -> const char* {
      if (!std::strcmp(argv[i], flag) && i + 1 < argc) return argv[++i];
      return nullptr;
    };
    const char* v;
    if ((v = next("-x"))) x = std::atoi(v);
    else if ((v = next("-y"))) y = std::atoi(v);
    else if ((v = next("-samplecount"))) s = std::atoi(v);
    else if ((v = next("-raydepth"))) depth = std::atoi(v);
    else if ((v = next("-o"))) out = v;
    else if ((v = next("-raw"))) raw = v;
    else if ((v = next("-variant"))) variant = std::atoi(v);
    else if ((v = next("-device"))) device = std::atoi(v);
    else if ((v = next("-phicount"))) phiCount = std::atoi(v);
    else if ((v = next("-thetacount"))) thetaCount = std::atoi(v);
    else if ((v = next("-rank"))) rank = std::atoi(v);
    else if ((v = next("-world"))) world = std::atoi(v);
    else if (!std::strcmp(argv[i], "-hemisphere")) hemi = true;
    else if (!std::strcmp(argv[i], "-dry-run")) dry = true;
    else if (!std::strcmp(argv[i], "-direct")) direct = true;
  }
  if (world < 1 || rank < 0 || rank >= world || phiCount < 1 || thetaCount < 1) {
    std::cerr << "rtp_path: bad -rank/-world/-phicount/-thetacount" << std::endl;
    return 2;
  }
  std::vector<View> views;
  if (hemi) {
    const std::vector<View> all = hemisphere_views(phiCount, thetaCount);
    for (size_t k = rank; k < all.size(); k += world) views.push_back(all[k]);
  }
  if (dry) {
    for (const View& w : views)
      std::printf("%.4f-%.4f %08x %08x %08x\n", w.phi, w.theta, bits(w.pos[0]), bits(w.pos[1]), bits(w.pos[2]));
    return 0;
  }
  try {
    const auto t0 = std::chrono::steady_clock::now();
    rtp::CornellBox cb;
    cb.variant = variant;
    cb.buildDataSet();
    rtp::rendering::CanvasRayTracer canvas(x, y);
    rtp::rendering::Camera cam = rtp::DefaultCamera();
    auto dev = std::make_shared<rtp::Device>(device);
    auto render = [&](const std::string& suffix) {  // generate() / the default branch of main()
      if (direct) {  // runRay + depth, runNorms, runAlbedo (main.cc:399-420, 625-650)
        const rtp::rendering::DirectBuffers b = rtp::RunDirect(x, y, cam, cb, dev);
        rtp::SavePNM("direct" + suffix + ".pnm", b.color, x, y);
        rtp::SaveDepthPNM("depth" + suffix + ".pnm", b.depth, x, y);
        rtp::SavePNM("normals" + suffix + ".pnm", b.normals, x, y);
        rtp::SavePNM("albedo" + suffix + ".pnm", b.albedo, x, y);
        return;
      }
      rtp::runPath(x, y, s, depth, canvas, cam, cb, dev);
      rtp::SavePNM(out + suffix + ".pnm", canvas);
      if (!raw.empty()) {
        const std::string fn = suffix.empty() ? raw : raw + suffix + ".f32";
        FILE* f = std::fopen(fn.c_str(), "wb");
        if (!f) throw rtp::ErrorBadValue("cannot open " + fn);
        const auto& c = canvas.GetColorBuffer();
        std::fwrite(c.data(), sizeof(rtp::Vec4f), c.size(), f);
        std::fclose(f);
      }
    };
    if (hemi) {
      // generateHemisphere's own camera: near plane 1, not main()'s 0.1
      // (main.cc:519 `SetClippingRange(01.f, 5.f)`; it moves the depth AOV)
      cam.SetClippingRange(1.0f, 5.f);
      for (const View& w : views) {
        char suffix[64];
        std::snprintf(suffix, sizeof(suffix), "-%.4f-%.4f", w.phi, w.theta);
        cam.SetPosition(w.pos);
        render(suffix);
      }
    } else {
      render("");
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << " Elapsed time         = " << el << std::endl;
  } catch (const std::exception& e) {
    std::cerr << "rtp_path: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
