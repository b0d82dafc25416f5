// rtp/vtkm_compat.hpp -- the VTK-m names the reference's main.cc uses, over
// rtp/rendering.hpp and the librtp C ABI, so that main.cc compiles and runs
// UNCHANGED against librtp.so (the drop-in boundary of SURVEY.md 8(b)):
//
//   cd include/vtkm_compat && g++ -std=c++17 -I.. -x c++ - -L<pkg> -lrtp < main.cc
//
// (main.cc read from stdin: its quoted includes -- "MapperPathTracer.h",
// "CornellBox.h", "View3D.h", ... -- then resolve in include/vtkm_compat/
// instead of next to main.cc; raytracingtherestofyourlife_amd/build.py
// build_main_unchanged).  Every header main.cc includes has a same-named file
// under include/vtkm_compat/ that includes this one.
//
// Only the surface main.cc touches (main.cc:11-42 includes; 120-251 the
// -direct mappers, View3D, Scene, Actor, ColorTable; 253-323 NormalizeFunctor,
// runPath, vtkm::cont::Algorithm::Transform; 325-384 save() through
// ArrayHandle portals; 460-664 Camera, CanvasRayTracer, Timer, Initialize,
// vtkm::Pi/Sqrt/Sin/Cos).  The path tracer itself is MapperPathTracer over the
// HIP kernels (rtp_render); there is no CPU path.
#pragma once

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "rendering.hpp"

#ifndef VTKM_EXEC_CONT
#define VTKM_EXEC_CONT
#endif
#ifndef VTKM_EXEC
#define VTKM_EXEC
#endif
#ifndef VTKM_CONT
#define VTKM_CONT
#endif

namespace vtkm {
using Float32 = float;
using Float64 = double;
using Id = int64_t;
using IdComponent = int32_t;
using UInt8 = uint8_t;
template <class T, int N>
using Vec = rtp::Vec<T, N>;
using Vec3f_32 = Vec<Float32, 3>;
using Vec4f_32 = Vec<Float32, 4>;
using Range = rtp::rendering::Range;

inline constexpr Float64 Pi() { return 3.14159265358979323846; }
inline constexpr Float32 Pif() { return 3.14159265358979323846f; }
// the scalar math functions: the C library's overload for the argument type
inline Float32 Sqrt(Float32 x) { return std::sqrt(x); }
inline Float64 Sqrt(Float64 x) { return std::sqrt(x); }
inline Float32 Sin(Float32 x) { return std::sin(x); }
inline Float64 Sin(Float64 x) { return std::sin(x); }
inline Float32 Cos(Float32 x) { return std::cos(x); }
inline Float64 Cos(Float64 x) { return std::cos(x); }
// ... and componentwise on a Vec (NormalizeFunctor: vtkm::Sqrt(tmp / samplecount))
template <class T, int N>
inline Vec<T, N> Sqrt(const Vec<T, N>& v) {
  Vec<T, N> r;
  for (int i = 0; i < N; i++) r[i] = Sqrt(v[i]);
  return r;
}

namespace cont {
template <class T>
using ArrayHandle = rtp::ArrayHandle<T>;
using Field = rtp::Field;
using CoordinateSystem = rtp::CoordinateSystem;
using DataSet = rtp::DataSet;
using ErrorBadValue = rtp::ErrorBadValue;

// vtkm::cont::Initialize: nothing to set up (the HIP device opens with the
// first mapper that renders)
inline void Initialize() {}
inline void Initialize(int&, char**) {}

enum class ColorSpace { RGB, HSV, HSV_WRAP, LAB, DIVERGING };

// vtkm::cont::ColorTable: the constructor runRay / runAlbedo use (name,
// colour space, NaN colour, rgb points and alpha values, main.cc:173-176),
// and a preset (runNorms: the normals mapper never samples it)
class ColorTable : public rtp::rendering::ColorTable {
 public:
  enum struct Preset { DEFAULT, COOL_TO_WARM, COOL_TO_WARM_EXTENDED, VIRIDIS, INFERNO, BLACK_BODY_RADIATION };
  ColorTable() = default;
  explicit ColorTable(Preset) {
    name = "preset";
    rgbPoints = {0.0, 0.23, 0.299, 0.754, 1.0, 0.706, 0.016, 0.150};
  }
  ColorTable(const std::string& nm, ColorSpace, const Vec<double, 3>& nan, const std::vector<double>& rgb,
             const std::vector<double>& alpha) {
    name = nm;
    nanColor = rtp::Vec3f((float)nan[0], (float)nan[1], (float)nan[2]);
    rgbPoints = rgb;
    alphaPoints = alpha;
  }
};

// vtkm::cont::Algorithm::Transform(a, b, out, f): out[i] = f(a[i], b[i])
// (in place when the arrays alias, as in runPath)
struct Algorithm {
  template <class A, class B, class C, class F>
  static void Transform(const A& a, const B& b, C& out, F f) {
    const size_t n = a.size();
    out.resize(n);
    for (size_t i = 0; i < n; i++) {
      const auto x = a[i], y = b[i];
      out[i] = f(x, y);
    }
  }
};

// vtkm::cont::Timer: wall time between Start and Stop, in seconds
class Timer {
 public:
  void Start() {
    t0_ = clock::now();
    running_ = true;
  }
  void Stop() {
    t1_ = clock::now();
    running_ = false;
  }
  Float64 GetElapsedTime() const {
    return std::chrono::duration<Float64>((running_ ? clock::now() : t1_) - t0_).count();
  }

 private:
  using clock = std::chrono::steady_clock;
  clock::time_point t0_{}, t1_{};
  bool running_ = false;
};
}  // namespace cont

namespace rendering {
using Canvas = rtp::rendering::Canvas;
using CanvasRayTracer = rtp::rendering::CanvasRayTracer;
using Camera = rtp::rendering::Camera;
using MapperPathTracer = rtp::rendering::MapperPathTracer;
using Mapper = rtp::rendering::MapperQuadBase;  // the mappers View3D paints with (-direct)

class Color {
 public:
  Color(float r = 0.f, float g = 0.f, float b = 0.f, float a = 1.f) : Components(r, g, b, a) {}
  rtp::Vec4f Components;
};

// vtkm::rendering::Actor: the cell set, coordinates, scalar field and colour
// table of one scene actor
class Actor {
 public:
  Actor(const rtp::CellSet& cells, const rtp::CoordinateSystem& coords, const rtp::Field& field,
        const cont::ColorTable& ct)
      : cells_(&cells), coords_(&coords), field_(field), ct_(ct) {}
  const rtp::CellSet& GetCells() const { return *cells_; }
  const rtp::CoordinateSystem& GetCoordinates() const { return *coords_; }
  const rtp::Field& GetScalarField() const { return field_; }
  const cont::ColorTable& GetColorTable() const { return ct_; }

 private:
  const rtp::CellSet* cells_;
  const rtp::CoordinateSystem* coords_;
  rtp::Field field_;
  cont::ColorTable ct_;
};

class Scene {
 public:
  void AddActor(const Actor& a) { actors_.push_back(a); }
  int GetNumberOfActors() const { return (int)actors_.size(); }
  const Actor& GetActor(int i) const { return actors_.at((size_t)i); }

 private:
  std::vector<Actor> actors_;
};

namespace pathtracing {
// View3D (View3D.cxx): Paint clears the canvas and renders every actor with
// the view's mapper (the colour mapper samples the actor's colour table,
// vtkm Mapper::SetActiveColorTable), background composited
class View3D {
 public:
  View3D(const Scene& scene, Mapper& mapper, Canvas& canvas, const Camera& camera, const Color& background,
         const Color& foreground)
      : scene_(scene), mapper_(mapper), canvas_(canvas), camera_(camera), background_(background) {
    (void)foreground;
  }
  void Initialize() {}
  void Paint() {
    auto* c = dynamic_cast<CanvasRayTracer*>(&canvas_);
    if (!c) throw cont::ErrorBadValue("Ray Tracer: bad canvas type. Must be CanvasRayTracer");
    c->Clear();
    mapper_.SetCanvas(c);
    mapper_.SetBackground(background_.Components);
    for (int i = 0; i < scene_.GetNumberOfActors(); i++) {
      const Actor& a = scene_.GetActor(i);
      if (dynamic_cast<rtp::rendering::MapperQuad*>(&mapper_)) mapper_.SetActiveColorTable(a.GetColorTable());
      mapper_.RenderCells(a.GetCells(), a.GetCoordinates(), a.GetScalarField(), a.GetCells().quadCells, camera_);
    }
  }

 private:
  const Scene& scene_;
  Mapper& mapper_;
  Canvas& canvas_;
  Camera camera_;
  Color background_;
};
}  // namespace pathtracing
}  // namespace rendering
}  // namespace vtkm

// pathtracing/vec3.h
using vec3 = vtkm::Vec<vtkm::Float32, 3>;

// CornellBox.h: the scene builder (CornellBox.cpp through rtp_cornell_box)
using CornellBox = rtp::CornellBox;

// MapperQuad.h, MapperQuadNormals.h, MapperQuadAlbedo.h
namespace path {
namespace rendering {
using MapperQuad = rtp::rendering::MapperQuad;
using MapperQuadNormals = rtp::rendering::MapperQuadNormals;
using MapperQuadAlbedo = rtp::rendering::MapperQuadAlbedo;
}  // namespace rendering
}  // namespace path
