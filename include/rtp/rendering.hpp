// rtp/rendering.hpp -- header-only C++ host interface over the librtp C ABI
// (include/rtp.h) that mirrors the reference's MapperPathTracer surface, so a
// host program written against vtkm::rendering::MapperPathTracer (main.cc's
// runPath) reads the same:
//
//   rtp::CornellBox cb; cb.buildDataSet();
//   rtp::rendering::CanvasRayTracer canvas(nx, ny);
//   rtp::rendering::Camera cam; cam.SetPosition(...); ...
//   rtp::rendering::MapperPathTracer mapper(spp, depth, cb.matIdx, cb.texIdx,
//                                           cb.matType, cb.texType, cb.tex);
//   mapper.SetCanvas(&canvas);
//   mapper.RenderCells(cb.ds.GetCellSet(), cb.coord, field, ct, cam, sr);
//   rtp::Normalize(canvas.GetColorBuffer(), spp);       // NormalizeFunctor
//   rtp::SavePNM("output.pnm", canvas);                  // save(), main.cc:325-384
//
// The -direct mode (main.cc:120-251) has the quad mappers MapperQuad,
// MapperQuadNormals and MapperQuadAlbedo (MapperQuad*.cxx:86-150) with
// runRay / runNorms / runAlbedo, and RunDirect: all three AOVs + depth from
// one launch.
//
// Reference: MapperPathTracer.h:44-159, MapperPathTracer.cxx:94-406 (ctor,
// SetCanvas, RenderCells, StartScene/EndScene, NewCopy), main.cc:253-384
// (NormalizeFunctor, runPath, save), CornellBox.h:9-55.
//
// Errors follow the reference: a bad canvas type or bad argument throws
// rtp::ErrorBadValue (vtkm::cont::ErrorBadValue); device failures throw
// rtp::ErrorExecution.  There is no CPU path: without a HIP device every
// render throws.
#pragma once

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../rtp.h"

namespace rtp {

// vtkm::Vec<T, N> as the host code uses it: N components (std::array
// storage, so a std::vector of them is a plain T array for the C ABI),
// componentwise arithmetic with scalars and vectors, a scalar fills every
// component (vtkm::Vec(const T&)), N scalars of any arithmetic type convert
// one by one (vec3(278/555.0, ...): a double divide, then float).
template <class T, int N>
struct Vec : std::array<T, N> {
  using ComponentType = T;
  static constexpr int NUM_COMPONENTS = N;
  Vec() : std::array<T, N>{} {}
  Vec(const T& v) { this->fill(v); }  // NOLINT: implicit like vtkm::Vec
  template <class... A, std::enable_if_t<sizeof...(A) == N && (N > 1), int> = 0>
  Vec(A... a) : std::array<T, N>{{static_cast<T>(a)...}} {}  // NOLINT
  Vec(const std::array<T, N>& a) : std::array<T, N>(a) {}     // NOLINT
  Vec& operator=(const T& v) {
    this->fill(v);
    return *this;
  }
#define RTP_VEC_OP(op)                                                  \
  friend Vec operator op(const Vec& a, const Vec& b) {                  \
    Vec r;                                                              \
    for (int i = 0; i < N; i++) r[i] = a[i] op b[i];                    \
    return r;                                                           \
  }                                                                     \
  friend Vec operator op(const Vec& a, const T& s) {                    \
    Vec r;                                                              \
    for (int i = 0; i < N; i++) r[i] = a[i] op s;                       \
    return r;                                                           \
  }                                                                     \
  friend Vec operator op(const T& s, const Vec& a) {                    \
    Vec r;                                                              \
    for (int i = 0; i < N; i++) r[i] = s op a[i];                       \
    return r;                                                           \
  }
  RTP_VEC_OP(+)
  RTP_VEC_OP(-)
  RTP_VEC_OP(*)
  RTP_VEC_OP(/)
#undef RTP_VEC_OP
};
// a float Vec with a double scalar computes in double, then rounds each
// component to float (vtkm's mixed-precision Vec operators: the reference's
// scene points are vec3(x) / 555.0, CornellBox.cpp)
template <int N>
Vec<float, N> operator/(const Vec<float, N>& a, double s) {
  Vec<float, N> r;
  for (int i = 0; i < N; i++) r[i] = (float)((double)a[i] / s);
  return r;
}
template <int N>
Vec<float, N> operator*(const Vec<float, N>& a, double s) {
  Vec<float, N> r;
  for (int i = 0; i < N; i++) r[i] = (float)((double)a[i] * s);
  return r;
}
using Vec3f = Vec<float, 3>;
using Vec4f = Vec<float, 4>;
static_assert(sizeof(Vec3f) == 12 && sizeof(Vec4f) == 16, "Vec: N packed components");

// vtkm::cont::ArrayHandle as the host code uses it: a std::vector with the
// portal accessors main.cc's save() reads (GetNumberOfValues, ReadPortal().Get).
template <class T>
struct ArrayHandle : std::vector<T> {
  using ValueType = T;
  using std::vector<T>::vector;
  ArrayHandle() = default;
  ArrayHandle(const std::vector<T>& v) : std::vector<T>(v) {}  // NOLINT
  ArrayHandle& operator=(const std::vector<T>& v) {
    std::vector<T>::operator=(v);
    return *this;
  }
  struct Portal {
    const ArrayHandle* a;
    T Get(int64_t i) const { return (*a)[(size_t)i]; }
    int64_t GetNumberOfValues() const { return (int64_t)a->size(); }
  };
  struct WPortal {
    ArrayHandle* a;
    T Get(int64_t i) const { return (*a)[(size_t)i]; }
    void Set(int64_t i, const T& v) const { (*a)[(size_t)i] = v; }
    int64_t GetNumberOfValues() const { return (int64_t)a->size(); }
  };
  int64_t GetNumberOfValues() const { return (int64_t)this->size(); }
  void Allocate(int64_t n) { this->resize((size_t)n); }
  Portal ReadPortal() const { return Portal{this}; }
  WPortal WritePortal() { return WPortal{this}; }
};

struct ErrorBadValue : std::invalid_argument {
  using std::invalid_argument::invalid_argument;
};
struct ErrorExecution : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void Check(rtp_status s) {
  if (s == RTP_OK) return;
  const char* m = rtp_last_error();
  const std::string msg = m ? m : "rtp error";
  if (s == RTP_ERR_INVALID_ARGUMENT || s == RTP_ERR_NO_SCENE) throw ErrorBadValue(msg);
  throw ErrorExecution(msg);
}

// One rtp_context (one HIP device).  Shared by MapperPathTracer copies.
class Device {
 public:
  explicit Device(int ordinal = 0) {
    rtp_context* c = nullptr;
    Check(rtp_create(ordinal, &c));
    ctx_.reset(c, rtp_destroy);
  }
  rtp_context* get() const { return ctx_.get(); }

 private:
  std::shared_ptr<rtp_context> ctx_;
};

// ------------------------------------------------------------------ scene --
// The parts of vtkm::cont::DynamicCellSet / CoordinateSystem the path tracer
// consumes: QuadExtractor rows (p0..p3) and the vertex cells (sphere centres)
// with their radii (MapperPathTracer::extract, MapperPathTracer.cxx:178-197).
struct CellSet {
  std::vector<std::array<int32_t, 4>> quads;
  std::vector<int32_t> spheres;
  std::vector<float> radii;
  std::vector<int32_t> quadCells;  // QuadIds[0]: the cell id of each quad (the quad mappers' field lookup)
  std::vector<int64_t> offsets;    // an explicit cell set's point offsets per cell (CellSetExplicit), if built so
  // (vtkm::cont::DynamicCellSet::Cast<CellSetExplicit<>>() and its offsets, CornellBox::extract)
  template <class T>
  const CellSet& Cast() const {
    return *this;
  }
  template <class A, class B>
  ArrayHandle<int64_t> GetOffsetsArray(A, B) const {
    return ArrayHandle<int64_t>(offsets);
  }
  int64_t GetNumberOfCells() const { return offsets.empty() ? (int64_t)(quads.size() + spheres.size()) : (int64_t)offsets.size() - 1; }
};
// vtkm::cont::CoordinateSystem: the points, with SetData / GetData().Cast<>()
struct CoordinateSystem : std::vector<Vec3f> {
  using std::vector<Vec3f>::vector;
  CoordinateSystem() = default;
  CoordinateSystem(const std::vector<Vec3f>& v) : std::vector<Vec3f>(v) {}  // NOLINT
  void SetData(const std::vector<Vec3f>& v) { std::vector<Vec3f>::operator=(v); }
  struct Data {
    const CoordinateSystem* c;
    template <class T>
    T Cast() const {
      return T(c->begin(), c->end());
    }
  };
  Data GetData() const { return Data{this}; }
  int64_t GetNumberOfPoints() const { return (int64_t)size(); }
};

// vtkm::cont::Field with point association: one value per entry.
struct Field {
  enum struct Association { ANY, WHOLE_MESH, POINTS, CELL_SET };
  std::string name;
  std::vector<float> values;
  Field() = default;
  Field(std::string n, std::vector<float> v) : name(std::move(n)), values(std::move(v)) {}
  Field(std::string n, Association, const std::vector<float>& v) : name(std::move(n)), values(v) {}
  const std::string& GetName() const { return name; }
};

struct DataSet {
  CellSet cells;
  CoordinateSystem coords;
  std::vector<int32_t> quadCells;  // QuadIds[0]: the cell id of each quad
  std::vector<Field> fields;
  const CellSet& GetCellSet() const { return cells; }
  const CoordinateSystem& GetCoordinateSystem() const { return coords; }
  void AddField(const Field& f) {
    for (Field& g : fields)
      if (g.name == f.name) {
        g = f;
        return;
      }
    fields.push_back(f);
  }
  const Field& GetField(const std::string& name) const {
    for (const Field& f : fields)
      if (f.name == name) return f;
    throw ErrorBadValue("No field with requested name: " + name);
  }
};

// CornellBox (CornellBox.h:9-55): matIdx/texIdx are arrays of two index lists,
// [0] for quads and [1] for spheres, as in the reference.
struct CornellBox {
  int variant = 0;  // 0 reference scene; 1, 2: visible-sphere variants (rtp.h)
  std::vector<int32_t> matIdx[2], texIdx[2];
  std::vector<int32_t> matType, texType;
  std::vector<Vec3f> tex;
  CoordinateSystem coord;
  DataSet ds;
  std::array<int32_t, 4> lightQuad{};
  int32_t lightSphere = 0;
  float ior = 1.5f;

  void buildDataSet() {
    rtp_scene_desc d{};
    Check(rtp_cornell_box(variant, &d));
    coord.resize(d.n_points);
    for (int i = 0; i < d.n_points; i++) coord[i] = {d.points[3 * i], d.points[3 * i + 1], d.points[3 * i + 2]};
    ds.cells.quads.resize(d.n_quads);
    for (int q = 0; q < d.n_quads; q++)
      for (int k = 0; k < 4; k++) ds.cells.quads[q][k] = d.quad_points[4 * q + k];
    ds.cells.spheres.assign(d.sphere_point, d.sphere_point + d.n_spheres);
    ds.cells.radii.assign(d.sphere_radius, d.sphere_radius + d.n_spheres);
    matIdx[0].assign(d.quad_mat, d.quad_mat + d.n_quads);
    texIdx[0].assign(d.quad_tex, d.quad_tex + d.n_quads);
    matIdx[1].assign(d.sphere_mat, d.sphere_mat + d.n_spheres);
    texIdx[1].assign(d.sphere_tex, d.sphere_tex + d.n_spheres);
    matType.assign(d.mat_type, d.mat_type + d.n_mat);
    texType.assign(d.tex_type, d.tex_type + d.n_tex_type);
    tex.resize(d.n_tex);
    for (int i = 0; i < d.n_tex; i++) tex[i] = {d.tex_rgb[3 * i], d.tex_rgb[3 * i + 1], d.tex_rgb[3 * i + 2]};
    for (int k = 0; k < 4; k++) lightQuad[k] = d.light_quad_points[k];
    lightSphere = d.light_sphere_point;
    ior = d.ior;
    const float* fv = nullptr;
    const int32_t* qc = nullptr;
    int32_t nf = 0, nq = 0;
    Check(rtp_cornell_point_field(variant, &fv, &nf, &qc, &nq));
    ds.quadCells.assign(qc, qc + nq);
    ds.cells.quadCells = ds.quadCells;
    ds.coords = coord;
    ds.fields.assign(1, Field{"point_var", std::vector<float>(fv, fv + nf)});  // CornellBox.cpp:411-416
  }
};

namespace rendering {

// The vtkm::rendering::Camera fields the path tracer reads (pathtracing/
// Camera.cxx:624-637, 715-764).  Zoom and clipping range never reach RayGen.
class Camera {
 public:
  void SetPosition(const Vec3f& p) { position_ = p; }
  void SetLookAt(const Vec3f& p) { look_at_ = p; }
  void SetViewUp(const Vec3f& p) { view_up_ = p; }
  void SetFieldOfView(float deg) { fov_ = deg; }
  void SetClippingRange(float n, float f) { clip_ = {n, f}; }
  void SetZoom(float z) { zoom_ = z; }
  const Vec3f& GetPosition() const { return position_; }
  const Vec3f& GetLookAt() const { return look_at_; }
  const Vec3f& GetViewUp() const { return view_up_; }
  float GetFieldOfView() const { return fov_; }
  const std::array<float, 2>& GetClippingRange() const { return clip_; }

  rtp_camera ToC() const {
    rtp_camera c{};
    for (int k = 0; k < 3; k++) {
      c.position[k] = position_[k];
      c.look_at[k] = look_at_[k];
      c.view_up[k] = view_up_[k];
    }
    c.fov_y_deg = fov_;
    return c;
  }

 private:
  Vec3f position_{0.f, 0.f, 1.f}, look_at_{0.f, 0.f, 0.f}, view_up_{0.f, 1.f, 0.f};
  float fov_ = 60.f, zoom_ = 1.f;
  std::array<float, 2> clip_{0.01f, 1000.f};
};

// vtkm::rendering::Canvas: colour buffer Vec4f per pixel, index j*nx + i
// (row 0 = camera bottom); depth buffer float per pixel (written by the
// -direct mappers).  The mappers render into a CanvasRayTracer only
// (MapperPathTracer.cxx:155-172).
class Canvas {
 public:
  Canvas(int w, int h) : width_(w), height_(h) {
    if (w <= 0 || h <= 0) throw ErrorBadValue("Canvas: width and height must be positive");
    color_.assign((size_t)w * h, Vec4f{0.f, 0.f, 0.f, 0.f});
    depth_.assign((size_t)w * h, 1.001f);
  }
  virtual ~Canvas() = default;
  int GetWidth() const { return width_; }
  int GetHeight() const { return height_; }
  ArrayHandle<Vec4f>& GetColorBuffer() { return color_; }
  const ArrayHandle<Vec4f>& GetColorBuffer() const { return color_; }
  ArrayHandle<float>& GetDepthBuffer() { return depth_; }
  const ArrayHandle<float>& GetDepthBuffer() const { return depth_; }
  // Canvas::Clear (VTK-m): colour 0, depth 1.001
  void Clear() {
    std::fill(color_.begin(), color_.end(), Vec4f{0.f, 0.f, 0.f, 0.f});
    std::fill(depth_.begin(), depth_.end(), 1.001f);
  }

 private:
  int width_, height_;
  ArrayHandle<Vec4f> color_;
  ArrayHandle<float> depth_;
};

class CanvasRayTracer : public Canvas {
 public:
  CanvasRayTracer(int w, int h) : Canvas(w, h) {}
};

using Field = rtp::Field;  // ignored by the path tracer (MapperPathTracer.cxx:356-383)

// vtkm::cont::ColorTable(name, RGB, nanColor, rgbPoints, alphaPoints):
// (x, r, g, b) and (x, alpha, midpoint, sharpness) quadruples.  Ignored by
// the path tracer; sampled by the quad mappers (Mapper::SetActiveColorTable).
struct ColorTable {
  std::string name;
  Vec3f nanColor{0.5f, 0.f, 0.f};
  std::vector<double> rgbPoints, alphaPoints{0.0, 1.0, 0.5, 0.0, 1.0, 1.0, 0.5, 0.0};
  std::vector<Vec4f> Sample(int n = 1024) const {
    std::vector<Vec4f> out((size_t)n);
    const double nanc[3] = {nanColor[0], nanColor[1], nanColor[2]};
    Check(rtp_sample_color_table(rgbPoints.data(), (int32_t)rgbPoints.size(), alphaPoints.data(),
                                 (int32_t)alphaPoints.size(), nanc, n, out.data()->data()));
    return out;
  }
};
struct Range {};  // ignored

// vtkm::rendering::MapperPathTracer.  RenderCells leaves the UN-normalised
// per-pixel sum over `sc` samples in the canvas colour buffer; normalisation
// is the caller's job (main.cc:317-321).
class MapperPathTracer {
 public:
  // The HIP device is opened on first use (RenderCells) unless one is given.
  MapperPathTracer(int sc, int dc, std::vector<int32_t>* matIdx, std::vector<int32_t>* texIdx,
                   std::vector<int32_t>& matType, std::vector<int32_t>& texType, std::vector<Vec3f>& tex,
                   std::shared_ptr<Device> device = nullptr, int device_ordinal = 0)
      : samplecount(sc), depthcount(dc), MatIdx(matIdx), TexIdx(texIdx), MatType(matType), TexType(texType),
        Tex(tex), internals_(std::make_shared<Internals>(Internals{std::move(device), device_ordinal, nullptr, true, {}})) {
    if (!matIdx || !texIdx) throw ErrorBadValue("MapperPathTracer: matIdx/texIdx must point to two index lists");
  }
  // The reference's own index arrays (vtkm::Id: 64-bit, CornellBox.h:13-14),
  // narrowed once into lists the mapper owns.
  MapperPathTracer(int sc, int dc, ArrayHandle<int64_t>* matIdx, ArrayHandle<int64_t>* texIdx,
                   std::vector<int32_t>& matType, std::vector<int32_t>& texType, std::vector<Vec3f>& tex,
                   std::shared_ptr<Device> device = nullptr, int device_ordinal = 0)
      : MapperPathTracer(sc, dc, Narrow(matIdx, texIdx), matType, texType, tex, std::move(device), device_ordinal) {}

  // MapperPathTracer.cxx:155-172
  void SetCanvas(Canvas* canvas) {
    if (canvas != nullptr && dynamic_cast<CanvasRayTracer*>(canvas) == nullptr)
      throw ErrorBadValue("Ray Tracer: bad canvas type. Must be CanvasRayTracer");
    internals_->canvas = static_cast<CanvasRayTracer*>(canvas);
  }
  Canvas* GetCanvas() const { return internals_->canvas; }
  void SetCompositeBackground(bool on) { internals_->composite_background = on; }
  void StartScene() {}
  void EndScene() {}
  // shallow copy sharing the internals (:403-406)
  std::unique_ptr<MapperPathTracer> NewCopy() const { return std::unique_ptr<MapperPathTracer>(new MapperPathTracer(*this)); }

  // The scene coupling of the reference constructor (:141-148): light quad =
  // QuadIds row (0,8,9,10,11), light sphere = point 48, ior 1.5.
  void SetLights(const std::array<int32_t, 4>& quad, int32_t sphere_point, float ior = 1.5f) {
    light_quad_ = quad;
    light_sphere_ = sphere_point;
    ior_ = ior;
  }

  // MapperPathTracer.cxx:356-383 -> RenderCellsImpl :199-355
  void RenderCells(const CellSet& cellset, const CoordinateSystem& coords, const Field&, const ColorTable&,
                   const Camera& camera, const Range&) {
    CanvasRayTracer* canvas = internals_->canvas;
    if (!canvas) throw ErrorBadValue("MapperPathTracer: SetCanvas was not called");
    SetScene(cellset, coords);
    const rtp_camera cam = camera.ToC();
    rtp_stats st{};
    Check(rtp_render(device(), &cam, canvas->GetWidth(), canvas->GetHeight(), samplecount,
                     depthcount, 0u, canvas->GetColorBuffer().data()->data(), &st));
    last_stats = st;
  }

  const int samplecount, depthcount;  // as in the reference: (sc, dc)
  std::vector<int32_t>*MatIdx, *TexIdx;
  std::vector<int32_t>&MatType, &TexType;
  std::vector<Vec3f>& Tex;
  rtp_stats last_stats{};

 private:
  struct Internals {
    std::shared_ptr<Device> device;
    int ordinal;
    CanvasRayTracer* canvas;
    bool composite_background;
    std::shared_ptr<std::vector<int32_t>> owned_idx;  // narrowed matIdx[0..1], texIdx[0..1] (64-bit inputs)
  };
  using OwnedIdx = std::shared_ptr<std::vector<int32_t>>;
  static OwnedIdx Narrow(const ArrayHandle<int64_t>* m, const ArrayHandle<int64_t>* t) {
    if (!m || !t) throw ErrorBadValue("MapperPathTracer: matIdx/texIdx must point to two index lists");
    OwnedIdx o(new std::vector<int32_t>[4], std::default_delete<std::vector<int32_t>[]>());
    for (int k = 0; k < 2; k++) {
      o.get()[k].assign(m[k].begin(), m[k].end());
      o.get()[2 + k].assign(t[k].begin(), t[k].end());
    }
    return o;
  }
  MapperPathTracer(int sc, int dc, OwnedIdx own, std::vector<int32_t>& matType, std::vector<int32_t>& texType,
                   std::vector<Vec3f>& tex, std::shared_ptr<Device> device, int device_ordinal)
      : MapperPathTracer(sc, dc, own.get(), own.get() + 2, matType, texType, tex, std::move(device), device_ordinal) {
    internals_->owned_idx = std::move(own);
  }

  rtp_context* device() {
    if (!internals_->device) internals_->device = std::make_shared<Device>(internals_->ordinal);
    return internals_->device->get();
  }

  void SetScene(const CellSet& cs, const CoordinateSystem& coords) {
    const size_t nq = cs.quads.size(), ns = cs.spheres.size();
    if (MatIdx[0].size() != nq || TexIdx[0].size() != nq || MatIdx[1].size() != ns || TexIdx[1].size() != ns)
      throw ErrorBadValue("MapperPathTracer: matIdx/texIdx sizes do not match the cell set");
    std::vector<float> radii = cs.radii;
    if (radii.size() != ns) radii.assign(ns, 90.0f / 555.0f);  // extract() default radius (:182)
    rtp_scene_desc d{};
    d.points = coords.empty() ? nullptr : coords.data()->data();
    d.n_points = (int32_t)coords.size();
    d.quad_points = cs.quads.empty() ? nullptr : cs.quads.data()->data();
    d.quad_mat = MatIdx[0].data();
    d.quad_tex = TexIdx[0].data();
    d.n_quads = (int32_t)nq;
    d.sphere_point = cs.spheres.data();
    d.sphere_radius = radii.data();
    d.sphere_mat = MatIdx[1].data();
    d.sphere_tex = TexIdx[1].data();
    d.n_spheres = (int32_t)ns;
    d.mat_type = MatType.data();
    d.n_mat = (int32_t)MatType.size();
    d.tex_type = TexType.data();
    d.n_tex_type = (int32_t)TexType.size();
    d.tex_rgb = Tex.empty() ? nullptr : Tex.data()->data();
    d.n_tex = (int32_t)Tex.size();
    for (int k = 0; k < 4; k++) d.light_quad_points[k] = light_quad_[k];
    d.light_sphere_point = light_sphere_;
    d.ior = ior_;
    Check(rtp_set_scene(device(), &d));
  }

  std::shared_ptr<Internals> internals_;
  std::array<int32_t, 4> light_quad_{8, 9, 10, 11};
  int32_t light_sphere_ = 48;
  float ior_ = 1.5f;
};

// -direct mode: the quad mappers (MapperQuad*.cxx:86-150).  RenderCells
// paints the mapper's AOV and the depth into the canvas like View3D::Paint
// (cleared canvas, background (0,0,0,1) composited).
inline std::vector<float> QuadScalars(const Field& f, const std::vector<int32_t>& quadCells) {
  std::vector<float> out(quadCells.size());
  Check(rtp_quad_scalars(f.values.data(), (int32_t)f.values.size(), quadCells.data(), (int32_t)quadCells.size(),
                         out.data()));
  return out;
}

struct DirectBuffers {
  std::vector<Vec4f> color, normals, albedo;
  std::vector<float> depth;
};

// One rtp_render_direct launch: the AOVs whose bit is set in `aovs`, + depth.
inline DirectBuffers RenderDirect(rtp_context* ctx, const Camera& camera, int nx, int ny,
                                  const std::vector<float>& qscalar, const std::vector<Vec4f>& cmap, int aovs,
                                  const Vec4f& background = {0.f, 0.f, 0.f, 1.f}, bool composite = true) {
  DirectBuffers b;
  const size_t n = (size_t)nx * ny;
  if (aovs & RTP_AOV_COLOR) b.color.resize(n);
  if (aovs & RTP_AOV_NORMALS) b.normals.resize(n);
  if (aovs & RTP_AOV_ALBEDO) b.albedo.resize(n);
  b.depth.resize(n);
  rtp_direct_desc d{};
  d.clip_near = camera.GetClippingRange()[0];
  d.clip_far = camera.GetClippingRange()[1];
  for (int k = 0; k < 4; k++) d.background[k] = background[k];
  d.composite_background = composite ? 1 : 0;
  d.quad_scalar = qscalar.data();
  d.color_map = cmap.empty() ? nullptr : cmap.data()->data();
  d.color_map_size = (int32_t)cmap.size();
  const rtp_camera cam = camera.ToC();
  auto ptr = [](std::vector<Vec4f>& v) { return v.empty() ? nullptr : v.data()->data(); };
  Check(rtp_render_direct(ctx, &cam, nx, ny, &d, ptr(b.color), ptr(b.normals), ptr(b.albedo), b.depth.data(),
                          nullptr));
  return b;
}

class MapperQuadBase {
 public:
  explicit MapperQuadBase(int aov, std::shared_ptr<Device> device = nullptr) : aov_(aov), device_(std::move(device)) {}
  virtual ~MapperQuadBase() = default;
  void SetCanvas(Canvas* canvas) {  // MapperQuad.cxx:65-79
    if (canvas != nullptr && dynamic_cast<CanvasRayTracer*>(canvas) == nullptr)
      throw ErrorBadValue("Ray Tracer: bad canvas type. Must be CanvasRayTracer");
    canvas_ = static_cast<CanvasRayTracer*>(canvas);
  }
  Canvas* GetCanvas() const { return canvas_; }
  void SetCompositeBackground(bool on) { composite_ = on; }
  void SetBackground(const Vec4f& bg) { background_ = bg; }
  void SetActiveColorTable(const ColorTable& ct) { colorMap_ = ct.Sample(1024); }  // vtkm Mapper: 1024 samples
  void StartScene() {}
  void EndScene() {}
  // MapperQuad.cxx:86-150 over a scene with quads only (QuadExtractor)
  void RenderCells(const CellSet& cellset, const CoordinateSystem& coords, const Field& scalarField,
                   const std::vector<int32_t>& quadCells, const Camera& camera) {
    if (!canvas_) throw ErrorBadValue("MapperQuad: SetCanvas was not called");
    const size_t nq = cellset.quads.size();
    std::vector<int32_t> zq(nq, 0), one(1, 0);
    std::vector<float> rad(1, 1.f), tex(3, 0.f);
    rtp_scene_desc d{};
    d.points = coords.empty() ? nullptr : coords.data()->data();
    d.n_points = (int32_t)coords.size();
    d.quad_points = nq ? cellset.quads.data()->data() : nullptr;
    d.quad_mat = zq.data();
    d.quad_tex = zq.data();
    d.n_quads = (int32_t)nq;
    d.sphere_point = one.data();  // the ABI's light-sphere slot; spheres are not drawn here
    d.sphere_radius = rad.data();
    d.sphere_mat = one.data();
    d.sphere_tex = one.data();
    d.n_spheres = 1;
    d.mat_type = one.data();
    d.n_mat = 1;
    d.tex_type = one.data();
    d.n_tex_type = 1;
    d.tex_rgb = tex.data();
    d.n_tex = 1;
    for (int k = 0; k < 4; k++) d.light_quad_points[k] = nq ? cellset.quads[0][k] : 0;
    d.light_sphere_point = 0;
    d.ior = 1.5f;
    Check(rtp_set_scene(device(), &d));
    const std::vector<float> qs = nq ? QuadScalars(scalarField, quadCells) : std::vector<float>();
    DirectBuffers b = RenderDirect(device(), camera, canvas_->GetWidth(), canvas_->GetHeight(), qs,
                                   aov_ == RTP_AOV_COLOR ? colorMap_ : std::vector<Vec4f>(), aov_, background_,
                                   composite_);
    canvas_->GetColorBuffer() = aov_ == RTP_AOV_COLOR ? b.color : (aov_ == RTP_AOV_NORMALS ? b.normals : b.albedo);
    canvas_->GetDepthBuffer() = b.depth;
  }

 private:
  rtp_context* device() {
    if (!device_) device_ = std::make_shared<Device>(0);
    return device_->get();
  }
  int aov_;
  std::shared_ptr<Device> device_;
  CanvasRayTracer* canvas_ = nullptr;
  bool composite_ = true;
  Vec4f background_{0.f, 0.f, 0.f, 1.f};
  std::vector<Vec4f> colorMap_;
};
struct MapperQuad : MapperQuadBase {  // VTK-m RayTracer colour: Phong over the colour map
  explicit MapperQuad(std::shared_ptr<Device> d = nullptr) : MapperQuadBase(RTP_AOV_COLOR, std::move(d)) {}
};
struct MapperQuadNormals : MapperQuadBase {  // RayTracerNormals.cxx
  explicit MapperQuadNormals(std::shared_ptr<Device> d = nullptr) : MapperQuadBase(RTP_AOV_NORMALS, std::move(d)) {}
};
struct MapperQuadAlbedo : MapperQuadBase {  // RayTracerAlbedo.cxx
  explicit MapperQuadAlbedo(std::shared_ptr<Device> d = nullptr) : MapperQuadBase(RTP_AOV_ALBEDO, std::move(d)) {}
};

}  // namespace rendering

// The ct_12_quad colour table of runRay / runAlbedo (main.cc:150-176).
inline rendering::ColorTable MainPalletColorTable() {
  const std::vector<double> c1 = {0.65, 0.05, 0.05}, c2 = {0.73, 0.73, 0.73}, c3 = {0.12, 0.45, 0.15};
  const int num_quads = 12 + 6 + 6;
  rendering::ColorTable ct;
  ct.name = "pallet_color_table";
  ct.nanColor = {0.f, 0.f, 0.f};
  ct.rgbPoints.insert(ct.rgbPoints.end(), c3.begin(), c3.end());
  ct.rgbPoints.insert(ct.rgbPoints.end(), c1.begin(), c1.end());
  ct.rgbPoints.insert(ct.rgbPoints.end(), c2.begin(), c2.end());
  for (int i = 0; i < num_quads - 3; i++) ct.rgbPoints.insert(ct.rgbPoints.end(), c2.begin(), c2.end());
  ct.alphaPoints.assign(num_quads, 1.0);
  return ct;
}

// runRay / runNorms / runAlbedo (main.cc:120-251): one mapper paints the canvas.
template <typename M>
inline void runQuadMapper(rendering::CanvasRayTracer& canvas, const rendering::Camera& cam, const CornellBox& cb,
                          std::shared_ptr<Device> device = nullptr) {
  M mapper(std::move(device));
  mapper.SetCanvas(&canvas);
  mapper.SetActiveColorTable(MainPalletColorTable());
  canvas.Clear();  // View3D::Paint
  mapper.RenderCells(cb.ds.GetCellSet(), cb.coord, cb.ds.GetField("point_var"), cb.ds.quadCells, cam);
}
inline void runRay(rendering::CanvasRayTracer& c, const rendering::Camera& cam, const CornellBox& cb,
                   std::shared_ptr<Device> d = nullptr) {
  runQuadMapper<rendering::MapperQuad>(c, cam, cb, std::move(d));
}
inline void runNorms(rendering::CanvasRayTracer& c, const rendering::Camera& cam, const CornellBox& cb,
                     std::shared_ptr<Device> d = nullptr) {
  runQuadMapper<rendering::MapperQuadNormals>(c, cam, cb, std::move(d));
}
inline void runAlbedo(rendering::CanvasRayTracer& c, const rendering::Camera& cam, const CornellBox& cb,
                      std::shared_ptr<Device> d = nullptr) {
  runQuadMapper<rendering::MapperQuadAlbedo>(c, cam, cb, std::move(d));
}

// The -direct block of main.cc (:623-651) in one launch: colour, normals,
// albedo and depth on the Cornell box, each equal to its own mapper render.
inline rendering::DirectBuffers RunDirect(int nx, int ny, const rendering::Camera& cam, const CornellBox& cb,
                                          std::shared_ptr<Device> device) {
  rtp_scene_desc d{};
  Check(rtp_cornell_box(cb.variant, &d));
  Check(rtp_set_scene(device->get(), &d));
  const std::vector<float> qs = rendering::QuadScalars(cb.ds.GetField("point_var"), cb.ds.quadCells);
  return rendering::RenderDirect(device->get(), cam, nx, ny, qs, MainPalletColorTable().Sample(1024),
                                 RTP_AOV_COLOR | RTP_AOV_NORMALS | RTP_AOV_ALBEDO);
}

// save() of a colour buffer (main.cc:325-384)
inline void SavePNM(const std::string& path, const std::vector<Vec4f>& colors, int nx, int ny) {
  Check(rtp_write_pnm(path.c_str(), colors.data()->data(), nx, ny));
}
// save() of the depth buffer (main.cc:346-359)
inline void SaveDepthPNM(const std::string& path, const std::vector<float>& depth, int nx, int ny) {
  Check(rtp_write_pnm_depth(path.c_str(), depth.data(), nx, ny));
}

// NormalizeFunctor (main.cc:253-287): c = sqrt(deNaN(c) / samplecount), in place.
inline void Normalize(std::vector<Vec4f>& colors, int samplecount) {
  Check(rtp_normalize(colors.data()->data(), (int64_t)colors.size(), samplecount));
}

// save() (main.cc:325-384): P3 header, buffer order, int(255.99*c) per channel.
inline void SavePNM(const std::string& path, const rendering::CanvasRayTracer& canvas) {
  Check(rtp_write_pnm(path.c_str(), canvas.GetColorBuffer().data()->data(), canvas.GetWidth(), canvas.GetHeight()));
}

// The camera of main.cc:616-622.
inline rendering::Camera DefaultCamera() {
  rendering::Camera cam;
  cam.SetClippingRange(0.1f, 5.f);
  const float a = (float)(278 / 555.0), b = (float)(-800 / 555.0);  // double divide, then float (vec3)
  cam.SetPosition({a, a, b});
  cam.SetFieldOfView(40.f);
  cam.SetViewUp({0.f, 1.f, 0.f});
  cam.SetLookAt({a, a, a});
  return cam;
}

// runPath (main.cc:289-323)
inline void runPath(int nx, int ny, int samplecount, int depthcount, rendering::Canvas& canvas,
                    rendering::Camera& cam, CornellBox& cb, std::shared_ptr<Device> device = nullptr) {
  (void)nx;
  (void)ny;
  rendering::MapperPathTracer mapper(samplecount, depthcount, cb.matIdx, cb.texIdx, cb.matType, cb.texType, cb.tex,
                                     std::move(device));
  mapper.SetLights(cb.lightQuad, cb.lightSphere, cb.ior);
  mapper.SetCanvas(&canvas);
  rendering::Field field;
  rendering::ColorTable ct;
  rendering::Range sr;
  mapper.RenderCells(cb.ds.GetCellSet(), cb.coord, field, ct, cam, sr);
  Normalize(static_cast<rendering::CanvasRayTracer&>(canvas).GetColorBuffer(), samplecount);
}

}  // namespace rtp
