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
// Reference: MapperPathTracer.h:44-159, MapperPathTracer.cxx:94-406 (ctor,
// SetCanvas, RenderCells, StartScene/EndScene, NewCopy), main.cc:253-384
// (NormalizeFunctor, runPath, save), CornellBox.h:9-55.
//
// Errors follow the reference: a bad canvas type or bad argument throws
// rtp::ErrorBadValue (vtkm::cont::ErrorBadValue); device failures throw
// rtp::ErrorExecution.  There is no CPU path: without a HIP device every
// render throws.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../rtp.h"

namespace rtp {

using Vec3f = std::array<float, 3>;
using Vec4f = std::array<float, 4>;

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
};
using CoordinateSystem = std::vector<Vec3f>;

struct DataSet {
  CellSet cells;
  const CellSet& GetCellSet() const { return cells; }
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

class Canvas {
 public:
  Canvas(int w, int h) : width_(w), height_(h) {
    if (w <= 0 || h <= 0) throw ErrorBadValue("Canvas: width and height must be positive");
  }
  virtual ~Canvas() = default;
  int GetWidth() const { return width_; }
  int GetHeight() const { return height_; }

 private:
  int width_, height_;
};

// Colour buffer: Vec4f per pixel, index j*nx + i (row 0 = camera bottom).
class CanvasRayTracer : public Canvas {
 public:
  CanvasRayTracer(int w, int h) : Canvas(w, h), color_((size_t)w * h, Vec4f{0.f, 0.f, 0.f, 0.f}) {}
  std::vector<Vec4f>& GetColorBuffer() { return color_; }
  const std::vector<Vec4f>& GetColorBuffer() const { return color_; }

 private:
  std::vector<Vec4f> color_;
};

struct Field {};       // ignored by the path tracer (MapperPathTracer.cxx:356-383)
struct ColorTable {};  // ignored
struct Range {};       // ignored

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
        Tex(tex), internals_(std::make_shared<Internals>(Internals{std::move(device), device_ordinal, nullptr, true})) {
    if (!matIdx || !texIdx) throw ErrorBadValue("MapperPathTracer: matIdx/texIdx must point to two index lists");
  }

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
  };

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

}  // namespace rendering

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
