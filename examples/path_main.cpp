// path_main.cpp -- the path-traced mode of the reference's main.cc (parse,
// runPath, save; main.cc:54-119, 289-384, 562-664) written against
// rtp/rendering.hpp, i.e. the reference driver on the MI355X path.
//
//   rtp_path [-x 128] [-y 128] [-samplecount 10] [-raydepth 5]
//            [-o output] [-raw file.f32] [-variant 0] [-device 0]
//
// Writes <o>.pnm like main.cc.  -raw additionally dumps the normalised float
// RGBA buffer (nx*ny*4 float32, buffer order) for bit-exact comparisons.
// -hemisphere and -direct are not on the path tracer's route (out of scope).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "rtp/rendering.hpp"

int main(int argc, char** argv) {
  int x = 128, y = 128, s = 10, depth = 5, variant = 0, device = 0;  // main.cc:56-62 defaults
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
    else if (!std::strcmp(argv[i], "-hemisphere") || !std::strcmp(argv[i], "-direct")) {
      std::cerr << argv[i] << ": not part of the path-tracing route (see DESIGN.md, out of scope)\n";
      return 2;
    }
  }
  try {
    const auto t0 = std::chrono::steady_clock::now();
    rtp::CornellBox cb;
    cb.variant = variant;
    cb.buildDataSet();
    rtp::rendering::CanvasRayTracer canvas(x, y);
    rtp::rendering::Camera cam = rtp::DefaultCamera();
    auto dev = std::make_shared<rtp::Device>(device);
    rtp::runPath(x, y, s, depth, canvas, cam, cb, dev);
    rtp::SavePNM(out + ".pnm", canvas);
    if (!raw.empty()) {
      FILE* f = std::fopen(raw.c_str(), "wb");
      if (!f) throw rtp::ErrorBadValue("cannot open " + raw);
      const auto& c = canvas.GetColorBuffer();
      std::fwrite(c.data(), sizeof(rtp::Vec4f), c.size(), f);
      std::fclose(f);
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::cout << " Elapsed time         = " << el << std::endl;
  } catch (const std::exception& e) {
    std::cerr << "rtp_path: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
