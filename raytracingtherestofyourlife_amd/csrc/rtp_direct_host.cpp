// rtp_direct_host.cpp -- host side of the -direct mode (include/rtp.h):
// the camera, subset and matrix set-up of the quad mappers' render
// (MapperQuad.cxx:86-150 over VTK-m's raytracing Camera, RayTracer and
// CanvasRayTracer), the colour-table sampling of Mapper::SetActiveColorTable,
// the QuadIntersector scalar, and the depth PNM writer of main.cc.  Compiled
// with -ffp-contract=off like rtp_host.cpp: every ray-independent constant is
// computed with the float operations of the reference's CPU build.
//
// VTK-m behaviour not present in the reference's sources is restated from
// VTK-m 1.6's published code (version not pinned; DESIGN.md "direct mode"):
// Canvas::Clear (colour 0, depth 1.001), image-subset ray generation,
// MatrixHelpers::ViewMatrix, CreateProjectionMatrix, WriteToCanvas,
// BlendBackground, ColorTable::AddPoint / Sample, ColorToUChar.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtp.h"
#include "rtp_context.hpp"
#include "rtp_layout.hpp"

extern "C" hipError_t rtp_launch_direct(const rtp::DevScene* scene, const rtp::DirectParams* p, hipStream_t stream);
extern "C" hipError_t rtp_launch_eval_powf(const float* x, float y, float* out, int64_t n, hipStream_t stream);

namespace {

rtp_status fail(rtp_status st, const std::string& msg) { return rtp_internal_fail(st, msg); }
rtp_status hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? RTP_ERR_OUT_OF_MEMORY : RTP_ERR_DEVICE,
              std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr)                                 \
  do {                                                \
    hipError_t e_ = (expr);                           \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

struct v3 {
  float x, y, z;
};
inline v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline v3 scl(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline v3 cross(v3 a, v3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline v3 normalize(v3 a) { return scl(a, 1 / std::sqrt(dot(a, a))); }  // vtkm::Normalize (CPU build)
inline v3 ld(const float* p) { return {p[0], p[1], p[2]}; }
inline void st(float* d, v3 a) { d[0] = a.x, d[1] = a.y, d[2] = a.z; }
inline float std_max(float a, float b) { return (a < b) ? b : a; }  // vtkm::Max on the CPU build
inline float std_min(float a, float b) { return (b < a) ? b : a; }  // vtkm::Min
constexpr float kPi180f = 0.01745329251994329577f;                  // vtkm::Pi_180f()

struct M4 {
  float m[4][4];
};
M4 identity() {
  M4 r{};
  for (int i = 0; i < 4; i++) r.m[i][i] = 1.f;
  return r;
}
// vtkm::MatrixMultiply: each entry a left-to-right Dot of a row and a column
M4 mul(const M4& a, const M4& b) {
  M4 r;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      float acc = a.m[i][0] * b.m[0][j];
      for (int k = 1; k < 4; k++) acc = acc + a.m[i][k] * b.m[k][j];
      r.m[i][j] = acc;
    }
  return r;
}
void mul_vec(const M4& a, const float v[4], float out[4]) {
  for (int i = 0; i < 4; i++) {
    float acc = a.m[i][0] * v[0];
    for (int k = 1; k < 4; k++) acc = acc + a.m[i][k] * v[k];
    out[i] = acc;
  }
}

// vtkm::rendering::MatrixHelpers::ViewMatrix(position, lookAt, up)
M4 view_matrix(v3 position, v3 look_at, v3 up) {
  v3 view_dir = sub(position, look_at);
  v3 right = cross(up, view_dir);
  v3 ru = cross(view_dir, right);
  view_dir = normalize(view_dir);
  right = normalize(right);
  ru = normalize(ru);
  M4 m = identity();
  m.m[0][0] = right.x, m.m[0][1] = right.y, m.m[0][2] = right.z;
  m.m[1][0] = ru.x, m.m[1][1] = ru.y, m.m[1][2] = ru.z;
  m.m[2][0] = view_dir.x, m.m[2][1] = view_dir.y, m.m[2][2] = view_dir.z;
  m.m[0][3] = -dot(right, position);
  m.m[1][3] = -dot(ru, position);
  m.m[2][3] = -dot(view_dir, position);
  return m;
}

// Camera::Camera3DStruct::CreateProjectionMatrix with zoom 1 and no pan
// (Z * (T * P), both identity here but multiplied as VTK-m does)
M4 projection_matrix(int32_t w, int32_t h, float fov_deg, float n, float f) {
  M4 m = identity();
  const float aspect = (float)w / (float)h;
  float fov_rad = fov_deg * kPi180f;
  fov_rad = std::tan(fov_rad * 0.5f);
  const float size = n * fov_rad;
  const float left = -size * aspect, right = size * aspect, bottom = -size, top = size;
  m.m[0][0] = 2.f * n / (right - left);
  m.m[1][1] = 2.f * n / (top - bottom);
  m.m[0][2] = (right + left) / (right - left);
  m.m[1][2] = (top + bottom) / (top - bottom);
  m.m[2][2] = -(f + n) / (f - n);
  m.m[3][2] = -1.f;
  m.m[2][3] = -(2.f * f * n) / (f - n);
  m.m[3][3] = 0.f;
  const M4 T = identity(), Z = identity();
  return mul(Z, mul(T, m));
}

// Everything ray-independent of one direct render.
void direct_setup(const rtp_context* c, const rtp_camera* cam, const rtp_direct_desc* dd, int32_t nx, int32_t ny,
                  rtp::DirectParams* p) {
  // raytracing::Camera::SetParameters on a fresh camera (Camera.cxx:624-637):
  // SetUp normalises a changed up vector (:767-776); SetFieldOfView /
  // SetHeight / SetWidth (:641-684, 716-764) leave FovX = FovY for a square
  // canvas and 2*atan(w/h * tan(fovY/2)) otherwise.
  v3 up = ld(cam->view_up);
  if (!(up.x == 0.f && up.y == 1.f && up.z == 0.f)) up = normalize(up);
  float fov_x = cam->fov_y_deg;
  if (nx != ny) {
    const float fovy_rad = cam->fov_y_deg * kPi180f;
    const float vertical = std::tan(0.5f * fovy_rad);
    const float aspect = (float)nx / (float)ny;
    const float horizontal = aspect * vertical;
    const float fovx_rad = 2.0f * std::atan(horizontal);
    fov_x = fovx_rad / kPi180f;
  }
  const v3 pos = ld(cam->position);
  const v3 look = normalize(sub(ld(cam->look_at), pos));  // CreateRaysImpl: Look = LookAt - Position
  // PerspectiveRayGen's constructor (Camera.cxx:351-392), zoom 1
  const float thx = std::tan((fov_x * kPi180f) * .5f);
  const float thy = std::tan((cam->fov_y_deg * kPi180f) * .5f);
  const v3 ru = normalize(cross(look, up));
  const v3 rv = normalize(cross(ru, look));
  v3 dx = scl(ru, (2 * thx / (float)nx));
  v3 dy = scl(rv, (2 * thy / (float)ny));
  const float zoom = 1.f;
  dx = {dx.x / zoom, dx.y / zoom, dx.z / zoom};
  dy = {dy.x / zoom, dy.y / zoom, dy.z / zoom};
  st(p->eye, pos);
  st(p->nlook, normalize(look));
  st(p->dx, dx);
  st(p->dy, dy);
  p->nx = nx, p->ny = ny;
  // CanvasRayTracer::WriteToCanvas / FindSubset: projection * view of the
  // vtkm::rendering::Camera (raw ViewUp)
  const M4 vp = mul(projection_matrix(nx, ny, cam->fov_y_deg, dd->clip_near, dd->clip_far),
                    view_matrix(pos, ld(cam->look_at), ld(cam->view_up)));
  std::memcpy(p->vp, vp.m, sizeof(vp.m));
  // Camera::FindSubset over the quads' shape bounds (Camera.cxx:963-1060)
  const float* lo = c->quad_lo;
  const float* hi = c->quad_hi;
  if (c->n_ref_quads == 0 || (pos.x >= lo[0] && pos.x <= hi[0] && pos.y >= lo[1] && pos.y <= hi[1] &&
                              pos.z >= lo[2] && pos.z <= hi[2])) {
    p->sub_x0 = 0, p->sub_y0 = 0, p->sub_w = nx, p->sub_h = ny;
  } else {
    float xmin = INFINITY, ymin = INFINITY, zmin = INFINITY, xmax = -INFINITY, ymax = -INFINITY, zmax = -INFINITY;
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        for (int k = 0; k < 2; k++) {
          const float e[4] = {i ? hi[0] : lo[0], j ? hi[1] : lo[1], k ? hi[2] : lo[2], 1.f};
          float t[4];
          mul_vec(vp, e, t);
          for (int a = 0; a < 3; a++) t[a] = t[a] / t[3];
          t[0] = (t[0] * 0.5f + 0.5f) * (float)nx;
          t[1] = (t[1] * 0.5f + 0.5f) * (float)ny;
          t[2] = (t[2] * 0.5f + 0.5f);
          zmin = std_min(zmin, t[2]);
          zmax = std_max(zmax, t[2]);
          if (t[2] < 0 || t[2] > 1) continue;
          xmin = std_min(xmin, t[0]);
          ymin = std_min(ymin, t[1]);
          xmax = std_max(xmax, t[0]);
          ymax = std_max(ymax, t[1]);
        }
    xmin -= .001f;
    xmax += .001f;
    ymin -= .001f;
    ymax += .001f;
    xmin = std::floor(std_min(std_max(0.f, xmin), (float)nx));
    xmax = std::ceil(std_min(std_max(0.f, xmax), (float)nx));
    ymin = std::floor(std_min(std_max(0.f, ymin), (float)ny));
    ymax = std::ceil(std_min(std_max(0.f, ymax), (float)ny));
    if (zmax < 0 || xmin >= xmax || ymin >= ymax) {
      p->sub_x0 = 0, p->sub_y0 = 0, p->sub_w = 1, p->sub_h = 1;
    } else {
      p->sub_x0 = (int32_t)xmin, p->sub_y0 = (int32_t)ymin;
      p->sub_w = (int32_t)xmax - (int32_t)xmin, p->sub_h = (int32_t)ymax - (int32_t)ymin;
    }
  }
  // SurfaceX::run (RayTracerNormals.cxx:150-163): light = Position + (2,2,2)*Up
  st(p->light, add(pos, v3{2.f * up.x, 2.f * up.y, 2.f * up.z}));
  st(p->view_dir, normalize(sub(pos, ld(cam->look_at))));
  for (int k = 0; k < 4; k++) p->bg[k] = dd->background[k];
  p->composite = dd->composite_background ? 1 : 0;
  p->npix = (int64_t)nx * ny;
}

rtp_status check_direct(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, const rtp_direct_desc* dd,
                        bool any_out) {
  if (!c || !cam || !dd) return fail(RTP_ERR_INVALID_ARGUMENT, "render_direct: NULL argument");
  if (!c->has_scene) return fail(RTP_ERR_NO_SCENE, "render_direct: rtp_set_scene was not called");
  if (nx <= 0 || ny <= 0) return fail(RTP_ERR_INVALID_ARGUMENT, "Camera width/height must be greater than zero.");
  if ((int64_t)nx * ny > INT32_MAX) return fail(RTP_ERR_INVALID_ARGUMENT, "render_direct: canvas too large");
  if (!(cam->fov_y_deg > 0)) return fail(RTP_ERR_INVALID_ARGUMENT, "Camera feild of view must be greater than zero.");
  if (cam->fov_y_deg > 180) return fail(RTP_ERR_INVALID_ARGUMENT, "Camera feild of view must be less than 180.");
  if (!any_out) return fail(RTP_ERR_INVALID_ARGUMENT, "render_direct: no output buffer");
  if (c->n_ref_quads > 0 && !dd->quad_scalar)
    return fail(RTP_ERR_INVALID_ARGUMENT, "render_direct: quad_scalar is NULL");
  return RTP_OK;
}

// upload the scalar table (kept-quad order) and the colour map into the
// context's scratch; the previous launch may still read it
rtp_status stage_inputs(rtp_context* c, const rtp_direct_desc* dd, bool need_cmap, hipStream_t stream,
                        rtp::DirectParams* p) {
  const size_t nk = c->kept_quads.size();
  const int32_t cm = need_cmap ? std::max(dd->color_map_size, 0) : 0;
  if (need_cmap && (cm < 1 || !dd->color_map))
    return fail(RTP_ERR_INVALID_ARGUMENT, "render_direct: the colour AOV needs a colour map (Mapper::ColorMap)");
  std::vector<float> host(nk + 4 * (size_t)cm + 4);
  for (size_t k = 0; k < nk; k++) host[k] = dd->quad_scalar[c->kept_quads[k]];
  const size_t cm_off = (nk + 3) & ~size_t(3);  // float4-aligned colour map
  host.resize(cm_off + 4 * (size_t)cm + 1);
  if (cm) std::memcpy(host.data() + cm_off, dd->color_map, sizeof(float) * 4 * cm);
  const size_t bytes = host.size() * sizeof(float);
  if (c->pending) {
    HIP_TRY(hipEventSynchronize(c->done));
    c->pending = false;
  }
  if (bytes > c->direct_bytes) {
    if (c->d_direct) HIP_TRY(hipFree(c->d_direct));
    c->d_direct = nullptr;
    c->direct_bytes = 0;
    HIP_TRY(hipMalloc(&c->d_direct, bytes));
    c->direct_bytes = bytes;
  }
  HIP_TRY(hipMemcpyAsync(c->d_direct, host.data(), bytes, hipMemcpyHostToDevice, stream));
  p->qscalar = c->d_direct;
  p->cmap = c->d_direct + cm_off;
  p->cmap_n = cm;
  return RTP_OK;
}

rtp_status launch_direct(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny, const rtp_direct_desc* dd,
                         float* color, float* normals, float* albedo, float* depth, hipStream_t stream,
                         double* kernel_ms) {
  HIP_TRY(hipSetDevice(c->device));
  rtp::DirectParams p{};
  direct_setup(c, cam, dd, nx, ny, &p);
  rtp_status rs = stage_inputs(c, dd, color != nullptr, stream, &p);
  if (rs != RTP_OK) return rs;
  p.color = color, p.normals = normals, p.albedo = albedo, p.depth = depth;
  if (kernel_ms) HIP_TRY(hipEventRecord(c->ev0, stream));
  HIP_TRY(rtp_launch_direct(c->d_scene, &p, stream));
  HIP_TRY(hipEventRecord(c->done, stream));
  c->pending = true;
  if (kernel_ms) {
    HIP_TRY(hipEventRecord(c->ev1, stream));
    HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    *kernel_ms = ms;
  }
  return RTP_OK;
}

// ColorTable node (x, value) kept sorted by x (ColorTable::AddPoint)
struct CtNode {
  double x;
  float v[3];
};
void ct_add(std::vector<CtNode>& nodes, double x, const float v[3]) {
  auto it = std::lower_bound(nodes.begin(), nodes.end(), x, [](const CtNode& n, double k) { return n.x < k; });
  if (it != nodes.end() && it->x == x) {
    std::memcpy(it->v, v, sizeof(it->v));
    return;
  }
  CtNode n{x, {v[0], v[1], v[2]}};
  nodes.insert(it, n);
}
bool outside01(const float v[3]) {
  for (int k = 0; k < 3; k++)
    if (v[k] < 0 || v[k] > 1) return true;
  return false;
}
// ColorTableBase::MapThroughColorSpace / MapThroughOpacitySpace (RGB space,
// clamping on): the node values, linearly interpolated (vtkm::Lerp)
void ct_map(const std::vector<CtNode>& nodes, double x, int nv, float* out) {
  if (nodes.empty()) {
    for (int k = 0; k < nv; k++) out[k] = 0.f;
    return;
  }
  if (x <= nodes.front().x) {
    std::memcpy(out, nodes.front().v, sizeof(float) * nv);
    return;
  }
  if (x >= nodes.back().x) {
    std::memcpy(out, nodes.back().v, sizeof(float) * nv);
    return;
  }
  auto it = std::lower_bound(nodes.begin(), nodes.end(), x, [](const CtNode& n, double k) { return n.x < k; });
  const CtNode& b = *it;
  const CtNode& a = *(it - 1);
  const float w = (float)((x - a.x) / (b.x - a.x));
  for (int k = 0; k < nv; k++) out[k] = (1.0f - w) * a.v[k] + w * b.v[k];
}
// colorconversion::ColorToUChar then Mapper::SetActiveColorTable's * (1/255.f)
float to_ui8_float(float t) { return (float)(uint8_t)std::round(t * 255.0f) * (1.0f / 255.0f); }

}  // namespace

extern "C" {

rtp_status rtp_render_direct(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny,
                             const rtp_direct_desc* dd, float* color, float* normals, float* albedo, float* depth,
                             rtp_stats* stats) {
  rtp_status rs = check_direct(c, cam, nx, ny, dd, color || normals || albedo || depth);
  if (rs != RTP_OK) return rs;
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)nx * ny;
  float* d[4] = {nullptr, nullptr, nullptr, nullptr};
  float* h[4] = {color, normals, albedo, depth};
  const size_t sz[4] = {16 * n, 16 * n, 16 * n, 4 * n};
  hipError_t e = hipSuccess;
  for (int k = 0; k < 4 && e == hipSuccess; k++)
    if (h[k]) e = hipMalloc(&d[k], sz[k]);
  double ms = 0;
  if (e == hipSuccess) {
    rs = launch_direct(c, cam, nx, ny, dd, d[0], d[1], d[2], d[3], nullptr, &ms);
    for (int k = 0; k < 4 && rs == RTP_OK; k++)
      if (h[k] && (e = hipMemcpy(h[k], d[k], sz[k], hipMemcpyDeviceToHost)) != hipSuccess)
        rs = hip_fail(e, "render_direct: copy back");
  } else {
    rs = hip_fail(e, "render_direct: device buffers");
  }
  for (float* p : d)
    if (p) (void)hipFree(p);
  if (rs == RTP_OK && stats) {
    *stats = rtp_stats{};
    stats->samples = n;
    stats->kernel_ms = ms;
  }
  return rs;
}

rtp_status rtp_render_direct_device(rtp_context* c, const rtp_camera* cam, int32_t nx, int32_t ny,
                                    const rtp_direct_desc* dd, float* color, float* normals, float* albedo,
                                    float* depth, void* hip_stream, rtp_stats* stats) {
  rtp_status rs = check_direct(c, cam, nx, ny, dd, color || normals || albedo || depth);
  if (rs != RTP_OK) return rs;
  double ms = 0;
  rs = launch_direct(c, cam, nx, ny, dd, color, normals, albedo, depth, (hipStream_t)hip_stream,
                     stats ? &ms : nullptr);
  if (rs == RTP_OK && stats) {
    *stats = rtp_stats{};
    stats->samples = (uint64_t)nx * ny;
    stats->kernel_ms = ms;
  }
  return rs;
}

// ColorTable(name, colorSpace, nanColor, rgbPoints, alphaPoints) ->
// FillColorTableFromDataPointer / FillOpacityTableFromDataPointer
// (quadruples; AddPoint: sorted insert, equal x overwrites, colours outside
// [0,1] dropped) -> Sample(n): n values from Min to Max of the table range in
// float when float resolves them (tolerance 0.002), colours interpolated per
// node pair, std::round(c * 255) -> uint8 -> * (1/255.f).
rtp_status rtp_sample_color_table(const double* rgb, int32_t n_rgb, const double* alpha, int32_t n_alpha,
                                  const double nan_color[3], int32_t n_samples, float* out) {
  if (n_samples < 2 || n_rgb < 0 || n_alpha < 0 || !out || (n_rgb && !rgb) || (n_alpha && !alpha))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_sample_color_table: bad arguments");
  std::vector<CtNode> cn, an;
  double rmin = INFINITY, rmax = -INFINITY;
  if (n_rgb > 0 && n_rgb % 4 == 0)
    for (int32_t i = 0; i < n_rgb; i += 4) {
      const float v[3] = {(float)rgb[i + 1], (float)rgb[i + 2], (float)rgb[i + 3]};
      if (outside01(v)) continue;
      ct_add(cn, rgb[i], v);
      rmin = std::min(rmin, rgb[i]);
      rmax = std::max(rmax, rgb[i]);
    }
  if (n_alpha > 0 && n_alpha % 4 == 0)
    for (int32_t i = 0; i < n_alpha; i += 4) {
      const float v[3] = {(float)alpha[i + 1], (float)alpha[i + 2], (float)alpha[i + 3]};
      if (outside01(v)) continue;
      ct_add(an, alpha[i], v);
      rmin = std::min(rmin, alpha[i]);
      rmax = std::max(rmax, alpha[i]);
    }
  if (cn.empty() && an.empty()) rmin = rmax = 0;
  const double d_delta = (rmax - rmin) / (double)(n_samples - 1);
  const float f_samples = (float)(n_samples - 1);
  const float f_start = (float)rmin;
  const float f_delta = (float)(rmax - rmin) / f_samples;
  const float f_end = f_start + (f_delta * f_samples);
  const bool use_f = std::fabs((double)f_end - rmax) <= 0.002 && std::fabs((double)f_delta - d_delta) <= 0.002;
  for (int32_t i = 0; i < n_samples; i++) {
    double x;
    if (use_f)
      x = (double)(i == 0 ? f_start : (i == n_samples - 1 ? f_end : f_start + ((float)i * f_delta)));
    else
      x = i == 0 ? rmin : (i == n_samples - 1 ? rmax : rmin + ((double)i * d_delta));
    float col[3], a[3];
    if (std::isnan(x)) {
      for (int k = 0; k < 3; k++) col[k] = nan_color ? (float)nan_color[k] : 0.f;
    } else {
      ct_map(cn, x, 3, col);
    }
    if (an.empty())
      a[0] = 1.f;
    else
      ct_map(an, x, 1, a);
    out[4 * i + 0] = to_ui8_float(col[0]);
    out[4 * i + 1] = to_ui8_float(col[1]);
    out[4 * i + 2] = to_ui8_float(col[2]);
    out[4 * i + 3] = to_ui8_float(a[0]);
  }
  return RTP_OK;
}

rtp_status rtp_quad_scalars(const float* field, int32_t n_field, const int32_t* quad_cell, int32_t n_quads,
                            float* out) {
  if (n_field < 1 || n_quads < 0 || !field || (n_quads && (!quad_cell || !out)))
    return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_quad_scalars: bad arguments");
  float mn = INFINITY, mx = -INFINITY;  // Actor::Init: the field's range
  for (int32_t i = 0; i < n_field; i++) {
    mn = std::min(mn, field[i]);
    mx = std::max(mx, field[i]);
  }
  // GetScalar's constructor (QuadIntersector): 1/(max-min), or 1/min for a flat field
  const float inv = (mx - mn != 0.f) ? 1.f / (mx - mn) : 1.f / mn;
  for (int32_t q = 0; q < n_quads; q++) {
    const int32_t cell = quad_cell[q];
    if (cell < 0 || cell >= n_field) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_quad_scalars: cell id out of range");
    out[q] = (field[cell] - mn) * inv;
  }
  return RTP_OK;
}

// save<vtkm::Float32> (main.cc:346-359): NaN -> 0, sqrt, int(255.99*c) x3
rtp_status rtp_write_pnm_depth(const char* path, const float* depth, int32_t nx, int32_t ny) {
  if (!path || !depth || nx <= 0 || ny <= 0) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_write_pnm_depth: bad arguments");
  FILE* f = std::fopen(path, "w");
  if (!f) return fail(RTP_ERR_INVALID_ARGUMENT, std::string("Couldn't save pnm: ") + path);
  std::fprintf(f, "P3\n%d %d 255\n", nx, ny);
  const int64_t n = (int64_t)nx * ny;
  for (int64_t i = 0; i < n; i++) {
    float col = depth[i];
    if (col != col) col = 0.f;
    col = std::sqrt(col);
    const int v = (int)(255.99 * col);
    std::fprintf(f, "%d %d %d\n", v, v, v);
  }
  std::fclose(f);
  return RTP_OK;
}

rtp_status rtp_eval_powf(rtp_context* c, const float* x, float y, float* out, int64_t n) {
  if (!c || !x || !out || n < 0) return fail(RTP_ERR_INVALID_ARGUMENT, "rtp_eval_powf: bad arguments");
  if (n == 0) return RTP_OK;
  HIP_TRY(hipSetDevice(c->device));
  float *dx = nullptr, *dout = nullptr;
  HIP_TRY(hipMalloc(&dx, (size_t)n * 4));
  hipError_t e = hipMalloc(&dout, (size_t)n * 4);
  if (e == hipSuccess) e = hipMemcpy(dx, x, (size_t)n * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = rtp_launch_eval_powf(dx, y, dout, n, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  if (dout) (void)hipFree(dout);
  if (e != hipSuccess) return hip_fail(e, "rtp_eval_powf");
  return RTP_OK;
}

}  // extern "C"
