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
#include <cstdio>
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

enum class CopyFlag { Off = 0, On = 1 };
enum CellShapeIdEnum { CELL_SHAPE_EMPTY = 0, CELL_SHAPE_VERTEX = 1, CELL_SHAPE_TRIANGLE = 5, CELL_SHAPE_QUAD = 9 };
struct TopologyElementTagPoint {};
struct TopologyElementTagCell {};

inline constexpr Float64 Pi() { return 3.14159265358979323846; }
template <class T>
inline constexpr T Pi_180() {
  return T(0.01745329251994329576923690768489);
}
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
inline Float32 RSqrt(Float32 x) { return 1.0f / std::sqrt(x); }  // the CPU build's RSqrt
inline Float64 RSqrt(Float64 x) { return 1.0 / std::sqrt(x); }

// VectorAnalysis: sums left to right, like vtkm::Dot's loop
template <class T, int N>
inline T Dot(const Vec<T, N>& a, const Vec<T, N>& b) {
  T r = T(a[0] * b[0]);
  for (int i = 1; i < N; i++) r = T(r + a[i] * b[i]);
  return r;
}
template <class T, int N>
inline T MagnitudeSquared(const Vec<T, N>& v) {
  return Dot(v, v);
}
template <class T, int N>
inline T Magnitude(const Vec<T, N>& v) {
  return Sqrt(MagnitudeSquared(v));
}
template <class T, int N>
inline T RMagnitude(const Vec<T, N>& v) {
  return RSqrt(MagnitudeSquared(v));
}
template <class T, int N>
inline Vec<T, N> Normal(const Vec<T, N>& v) {
  return v * RMagnitude(v);
}
template <class T>
inline Vec<T, 3> Cross(const Vec<T, 3>& a, const Vec<T, 3>& b) {
  return Vec<T, 3>(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}

// Matrix and Transform3D (CornellBox::invert): vtkm's formulas and
// summation order (MatrixMultiply: Dot of a row and a column)
template <class T, int R, int C>
struct Matrix {
  T m[R][C] = {};
  T& operator()(int i, int j) { return m[i][j]; }
  const T& operator()(int i, int j) const { return m[i][j]; }
};
template <class T, int N>
inline Matrix<T, N, N> MatrixIdentity() {
  Matrix<T, N, N> r;
  for (int i = 0; i < N; i++) r(i, i) = T(1);
  return r;
}
template <class T>
inline Matrix<T, 4, 4> Transform3DTranslate(const T& x, const T& y, const T& z) {
  Matrix<T, 4, 4> r = MatrixIdentity<T, 4>();
  r(0, 3) = x;
  r(1, 3) = y;
  r(2, 3) = z;
  return r;
}
template <class T>
inline Matrix<T, 4, 4> Transform3DRotate(T angleDegrees, const Vec<T, 3>& axisOfRotation) {
  const T angleRadians = Pi_180<T>() * angleDegrees;
  const Vec<T, 3> a = Normal(axisOfRotation);
  const T s = Sin(angleRadians), c = Cos(angleRadians);
  Matrix<T, 4, 4> r;
  r(0, 0) = a[0] * a[0] * (1 - c) + c;
  r(0, 1) = a[0] * a[1] * (1 - c) - a[2] * s;
  r(0, 2) = a[0] * a[2] * (1 - c) + a[1] * s;
  r(1, 0) = a[1] * a[0] * (1 - c) + a[2] * s;
  r(1, 1) = a[1] * a[1] * (1 - c) + c;
  r(1, 2) = a[1] * a[2] * (1 - c) - a[0] * s;
  r(2, 0) = a[2] * a[0] * (1 - c) - a[1] * s;
  r(2, 1) = a[2] * a[1] * (1 - c) + a[0] * s;
  r(2, 2) = a[2] * a[2] * (1 - c) + c;
  r(3, 3) = T(1);
  return r;
}
template <class T>
inline Matrix<T, 4, 4> Transform3DRotate(T angleDegrees, T x, T y, T z) {
  return Transform3DRotate(angleDegrees, Vec<T, 3>(x, y, z));
}
template <class T, int R, int C>
inline Matrix<T, C, R> MatrixTranspose(const Matrix<T, R, C>& a) {
  Matrix<T, C, R> r;
  for (int i = 0; i < R; i++)
    for (int j = 0; j < C; j++) r(j, i) = a(i, j);
  return r;
}
template <class T, int R, int K, int C>
inline Matrix<T, R, C> MatrixMultiply(const Matrix<T, R, K>& a, const Matrix<T, K, C>& b) {
  Matrix<T, R, C> r;
  for (int i = 0; i < R; i++)
    for (int j = 0; j < C; j++) {
      T acc = T(a(i, 0) * b(0, j));
      for (int k = 1; k < K; k++) acc = T(acc + a(i, k) * b(k, j));
      r(i, j) = acc;
    }
  return r;
}
template <class T, int R, int C>
inline Vec<T, R> MatrixMultiply(const Matrix<T, R, C>& a, const Vec<T, C>& v) {
  Vec<T, R> r;
  for (int i = 0; i < R; i++) {
    T acc = T(a(i, 0) * v[0]);
    for (int k = 1; k < C; k++) acc = T(acc + a(i, k) * v[k]);
    r[i] = acc;
  }
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

template <class T>
inline ArrayHandle<T> make_ArrayHandle(const std::vector<T>& v, CopyFlag) {
  return ArrayHandle<T>(v.begin(), v.end());
}
template <class T>
struct ArrayHandleCounting {
  T start, step;
  int64_t n;
  ArrayHandleCounting(T s, T d, int64_t count) : start(s), step(d), n(count) {}
  int64_t GetNumberOfValues() const { return n; }
  T Get(int64_t i) const { return T(start + T(i) * step); }
};
template <class T, class U>
inline void ArrayCopy(const ArrayHandleCounting<T>& src, ArrayHandle<U>& dst) {
  dst.resize((size_t)src.GetNumberOfValues());
  for (int64_t i = 0; i < src.GetNumberOfValues(); i++) dst[(size_t)i] = U(src.Get(i));
}
template <class T, class U>
inline void ArrayCopy(const ArrayHandle<T>& src, ArrayHandle<U>& dst) {
  dst.assign(src.begin(), src.end());
}

using DynamicCellSet = rtp::CellSet;
template <class... A>
struct CellSetExplicit {};

// DataSetBuilderExplicit::Create: the explicit cell set (shapes, point counts,
// connectivity) as the mappers take it -- the quads (QuadExtractor: quad
// cells, their cell ids) and the vertex cells (SphereExtractor: sphere
// centres; the extractor's radius is the mapper's, MapperPathTracer.cxx:182)
class DataSetBuilderExplicit {
 public:
  DataSet Create(const ArrayHandle<Vec<Float32, 3>>& coords, const ArrayHandle<UInt8>& shapes,
                 const ArrayHandle<IdComponent>& numIndices, const ArrayHandle<Id>& conn,
                 const std::string& coordsName = "coords") {
    (void)coordsName;
    if (shapes.size() != numIndices.size()) throw ErrorBadValue("DataSetBuilderExplicit: shapes/numIndices sizes");
    DataSet ds;
    ds.coords = rtp::CoordinateSystem(coords.begin(), coords.end());
    int64_t off = 0;
    ds.cells.offsets.push_back(0);
    for (size_t c = 0; c < shapes.size(); c++) {
      const int n = numIndices[c];
      if (off + n > (int64_t)conn.size()) throw ErrorBadValue("DataSetBuilderExplicit: connectivity too short");
      if (shapes[c] == CELL_SHAPE_QUAD && n == 4) {
        ds.cells.quads.push_back({(int32_t)conn[off], (int32_t)conn[off + 1], (int32_t)conn[off + 2], (int32_t)conn[off + 3]});
        ds.cells.quadCells.push_back((int32_t)c);
      } else if (shapes[c] == CELL_SHAPE_VERTEX && n == 1) {
        ds.cells.spheres.push_back((int32_t)conn[off]);
      }
      off += n;
      ds.cells.offsets.push_back(off);
    }
    ds.quadCells = ds.cells.quadCells;
    return ds;
  }
};

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

namespace io {
namespace writer {
// VTKDataSetWriter: a legacy-format ASCII unstructured grid (points, the
// quad and vertex cells, the point fields)
class VTKDataSetWriter {
 public:
  explicit VTKDataSetWriter(const std::string& fname) : fname_(fname) {}
  void WriteDataSet(const cont::DataSet& ds) const {
    std::FILE* f = std::fopen(fname_.c_str(), "w");
    if (!f) throw cont::ErrorBadValue("VTKDataSetWriter: cannot open " + fname_);
    const auto& P = ds.GetCoordinateSystem();
    const auto& C = ds.GetCellSet();
    std::fprintf(f, "# vtk DataFile Version 3.0\nvtk output\nASCII\nDATASET UNSTRUCTURED_GRID\nPOINTS %zu float\n",
                 P.size());
    for (const auto& p : P) std::fprintf(f, "%.9g %.9g %.9g\n", p[0], p[1], p[2]);
    const size_t nc = C.quads.size() + C.spheres.size();
    std::fprintf(f, "CELLS %zu %zu\n", nc, 5 * C.quads.size() + 2 * C.spheres.size());
    for (const auto& q : C.quads) std::fprintf(f, "4 %d %d %d %d\n", q[0], q[1], q[2], q[3]);
    for (int32_t s : C.spheres) std::fprintf(f, "1 %d\n", s);
    std::fprintf(f, "CELL_TYPES %zu\n", nc);
    for (size_t i = 0; i < C.quads.size(); i++) std::fprintf(f, "9\n");
    for (size_t i = 0; i < C.spheres.size(); i++) std::fprintf(f, "1\n");
    bool header = false;
    for (const auto& fld : ds.fields)
      if (fld.values.size() == P.size()) {
        if (!header) std::fprintf(f, "POINT_DATA %zu\n", P.size());
        header = true;
        std::fprintf(f, "SCALARS %s float 1\nLOOKUP_TABLE default\n", fld.name.c_str());
        for (float v : fld.values) std::fprintf(f, "%.9g\n", v);
      }
    std::fclose(f);
  }

 private:
  std::string fname_;
};
}  // namespace writer
}  // namespace io

namespace rendering {
namespace raytracing {
// QuadExtractor: (cell id, p0, p1, p2, p3) of every quad cell
class QuadExtractor {
 public:
  void ExtractCells(const rtp::CellSet& cells) {
    ids_.clear();
    for (size_t q = 0; q < cells.quads.size(); q++)
      ids_.push_back(Vec<Id, 5>((Id)(q < cells.quadCells.size() ? cells.quadCells[q] : (int32_t)q), (Id)cells.quads[q][0],
                                (Id)cells.quads[q][1], (Id)cells.quads[q][2], (Id)cells.quads[q][3]));
  }
  cont::ArrayHandle<Vec<Id, 5>> GetQuadIds() const { return ids_; }
  Id GetNumberOfQuads() const { return (Id)ids_.size(); }

 private:
  cont::ArrayHandle<Vec<Id, 5>> ids_;
};
}  // namespace raytracing
namespace pathtracing {
// SphereExtractor (pathtracing/SphereExtractor.h): the vertex cells' points
// with one constant radius
class SphereExtractor {
 public:
  void ExtractCells(const rtp::CellSet& cells, Float32 radius) {
    ids_.assign(cells.spheres.begin(), cells.spheres.end());
    radii_.assign(cells.spheres.size(), radius);
  }
  cont::ArrayHandle<Id> GetPointIds() const { return ids_; }
  cont::ArrayHandle<Float32> GetRadii() const { return radii_; }
  Id GetNumberOfSpheres() const { return (Id)ids_.size(); }

 private:
  cont::ArrayHandle<Id> ids_;
  cont::ArrayHandle<Float32> radii_;
};
}  // namespace pathtracing

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

// MapperQuad.h, MapperQuadNormals.h, MapperQuadAlbedo.h
namespace path {
namespace rendering {
using MapperQuad = rtp::rendering::MapperQuad;
using MapperQuadNormals = rtp::rendering::MapperQuadNormals;
using MapperQuadAlbedo = rtp::rendering::MapperQuadAlbedo;
}  // namespace rendering
}  // namespace path
