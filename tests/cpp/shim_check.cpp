// shim_check.cpp -- CPU checks of rtp/rendering.hpp (no GPU needed): the
// reference's error behaviour (MapperPathTracer.cxx:155-172 ErrorBadValue on a
// non-CanvasRayTracer canvas), the CornellBox table, NormalizeFunctor and the
// PNM writer.  Prints "OK" and exits 0 when every check passes.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>

#include "rtp/rendering.hpp"

static int failures = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::cerr << "FAIL " << __LINE__ << ": " #cond << std::endl;     \
      failures++;                                                      \
    }                                                                  \
  } while (0)

template <class E, class F>
bool throws(F f) {
  try {
    f();
  } catch (const E&) {
    return true;
  } catch (...) {
    return false;
  }
  return false;
}

int main(int argc, char** argv) {
  using namespace rtp;
  CornellBox cb;
  cb.buildDataSet();
  EXPECT(cb.ds.GetCellSet().quads.size() == 22);  // 6 walls + 2 x 8 box quads (CornellBox.cpp)
  EXPECT(cb.ds.GetCellSet().spheres.size() == 1);
  EXPECT(cb.matType.size() == 5 && cb.matType[3] == 1 && cb.matType[4] == 2);
  EXPECT(cb.lightQuad[0] == 8 && cb.lightSphere == 48);

  rendering::Canvas plain(4, 4);
  rendering::CanvasRayTracer canvas(4, 4);
  rendering::MapperPathTracer mapper(2, 3, cb.matIdx, cb.texIdx, cb.matType, cb.texType, cb.tex);
  EXPECT(throws<ErrorBadValue>([&] { mapper.SetCanvas(&plain); }));
  rendering::Field f;
  rendering::ColorTable ct;
  rendering::Range r;
  rendering::Camera cam = DefaultCamera();
  EXPECT(throws<ErrorBadValue>([&] { mapper.RenderCells(cb.ds.GetCellSet(), cb.coord, f, ct, cam, r); }));
  mapper.SetCanvas(&canvas);
  EXPECT(mapper.GetCanvas() == &canvas);
  auto copy = mapper.NewCopy();
  EXPECT(copy->GetCanvas() == &canvas);  // shares the internals
  std::vector<int32_t> bad_mat[2] = {{0, 1}, {4}}, bad_tex[2] = {{0, 1}, {0}};
  rendering::MapperPathTracer wrong(2, 3, bad_mat, bad_tex, cb.matType, cb.texType, cb.tex);
  wrong.SetCanvas(&canvas);
  EXPECT(throws<ErrorBadValue>([&] { wrong.RenderCells(cb.ds.GetCellSet(), cb.coord, f, ct, cam, r); }));
  EXPECT(throws<ErrorBadValue>([&] { rendering::CanvasRayTracer c(0, 3); }));

  // NormalizeFunctor: sqrt(deNaN(c)/S) per rgb channel
  std::vector<Vec4f> cols = {{4.f, NAN, 16.f, 7.f}, {0.f, 1.f, 2.f, 3.f}};
  Normalize(cols, 4);
  EXPECT(cols[0][0] == 1.f && cols[0][1] == 0.f && cols[0][2] == 2.f);
  EXPECT(cols[1][1] == std::sqrt(1.f / 4.f));

  // save(): P3, buffer order, int(255.99*c), whole pixel zeroed on NaN
  const std::string path = argc > 1 ? argv[1] : "/tmp/rtp_shim_check.pnm";
  canvas.GetColorBuffer()[0] = {0.5f, 1.0f, 0.0f, 0.f};
  canvas.GetColorBuffer()[1] = {0.5f, NAN, 1.0f, 0.f};
  SavePNM(path, canvas);
  std::ifstream in(path);
  std::stringstream ss;
  ss << in.rdbuf();
  EXPECT(ss.str().rfind("P3\n4 4 255\n127 255 0\n0 0 0\n", 0) == 0);

  // -direct host helpers (no device): the colour table of main.cc and the
  // GetScalar per quad over the point field
  const std::vector<Vec4f> cmap = MainPalletColorTable().Sample(1024);
  EXPECT(cmap.size() == 1024 && cmap[0][3] == 1.f);
  EXPECT(std::fabs(cmap[0][0] - 13 / 255.f) < 1e-7f && std::fabs(cmap[1023][1] - 186 / 255.f) < 1e-7f);
  EXPECT(cb.ds.quadCells.size() == 22 && cb.ds.quadCells[12] == 13);  // the sphere's vertex cell is 12
  const std::vector<float> qs = rendering::QuadScalars(cb.ds.GetField("point_var"), cb.ds.quadCells);
  EXPECT(qs[0] == 0.f && qs[21] > qs[12] && qs[21] <= 1.f);
  EXPECT(throws<ErrorBadValue>([&] { cb.ds.GetField("nope"); }));
  rendering::MapperQuadNormals qm;
  EXPECT(throws<ErrorBadValue>([&] { qm.SetCanvas(&plain); }));

  if (failures) return 1;
  std::cout << "OK" << std::endl;
  return 0;
}
