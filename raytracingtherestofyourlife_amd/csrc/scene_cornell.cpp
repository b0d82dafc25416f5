// scene_cornell.cpp -- CornellBox::buildDataSet (CornellBox.cpp:141-418) for
// the C ABI (rtp_cornell_box).  Produces the reference's 89 points, 22 quads
// (QuadExtractor order, vertex cell skipped), 1 sphere and the material
// tables, with the reference's float/double arithmetic:
//   * every coordinate is Vec<float,3>(x) / 555.0 (double divide -> float)
//   * the small box is rotated by VTK-m's Transform3DRotate(-15 deg, y) in
//     float, transposed, pre-multiplied by Translate(265,0,295)
//     (CornellBox::invert, :10-35)
//   * buildBox's duplicated faces and the y=333 vertex typo are kept.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/rtp.h"

namespace {

struct SceneStore {
  std::vector<float> points;
  std::vector<int32_t> quad_points, quad_mat, quad_tex;
  std::vector<int32_t> sphere_point, sphere_mat, sphere_tex;
  std::vector<float> sphere_radius;
  int32_t mat_type[5] = {0, 0, 0, 1, 2};  // lambertian x3, light, dielectric (:149-154)
  int32_t tex_type[5] = {0, 1, 2, 3, 0};  // red, white, green, light, dielectric (:156-161)
  // vec3(0.65, 0.05, 0.05) etc.: double literals converted to float (:144-147)
  float tex_rgb[12] = {(float)0.65, (float)0.05, (float)0.05, (float)0.73, (float)0.73, (float)0.73,
                       (float)0.12, (float)0.45, (float)0.15, 15.f,         15.f,         15.f};

  // the "point_var" field (CornellBox.cpp:36-60): each cell pushes its cell
  // index once per point it adds; QuadIds[0] (the cell id) per quad
  std::vector<float> field;
  std::vector<int32_t> quad_cell;
  int cell = 0;

  void add_quad(const float p[4][3], int mat, int tex) {
    const int base = (int)(points.size() / 3);
    for (int i = 0; i < 4; i++)
      for (int k = 0; k < 3; k++) points.push_back((float)((double)p[i][k] / 555.0));
    for (int i = 0; i < 4; i++) quad_points.push_back(base + i);
    quad_mat.push_back(mat);
    quad_tex.push_back(tex);
    for (int i = 0; i < 4; i++) field.push_back((float)cell);
    quad_cell.push_back(cell++);
  }
  void add_vertex_cell() { field.push_back((float)cell++); }  // sphere vertex cell (:357-365)
  void finish_field() {                                       // val /= float(vecField.size()) (:389-390)
    const float n = (float)field.size();
    for (float& v : field) v /= n;
  }
};

using P4 = float[4][3];

constexpr int kC3Spheres = 1000;
constexpr uint32_t kC3Seed = 3u;

// wangXor getRandF (wangXor.h:30-38, 55-59): float(t) / 4294967295.f == float(t) * 2^-32
float draw(uint32_t& s) {
  s = (s ^ 61u) ^ (s >> 16);
  s *= 9u;
  s = s ^ (s >> 4);
  s *= 0x27d4eb2du;
  s = s ^ (s >> 15);
  return (float)s * 0x1p-32f;
}

void rect(P4& p, std::initializer_list<float> v) {
  auto it = v.begin();
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 3; k++) p[i][k] = *it++;
}

// CornellBox::invert (CornellBox.cpp:10-35)
void invert(P4& pts) {
  const float angle = -15.f;
  float axis[3] = {0.f, 1.f, 0.f};
  {  // vtkm::Normal
    float r = 1 / std::sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
    for (float& a : axis) a = a * r;
  }
  const float rad = 0.01745329251994329577f * angle;  // Pi_180<float>() * angle
  const float sn = std::sin(rad), cs = std::cos(rad);
  const float x = axis[0], y = axis[1], z = axis[2];
  float R[4][4] = {{x * x * (1 - cs) + cs, x * y * (1 - cs) - z * sn, x * z * (1 - cs) + y * sn, 0},
                   {y * x * (1 - cs) + z * sn, y * y * (1 - cs) + cs, y * z * (1 - cs) - x * sn, 0},
                   {z * x * (1 - cs) - y * sn, z * y * (1 - cs) + x * sn, z * z * (1 - cs) + cs, 0},
                   {0, 0, 0, 1}};
  float T[4][4] = {{1, 0, 0, 265}, {0, 1, 0, 0}, {0, 0, 1, 295}, {0, 0, 0, 1}};
  float M[4][4];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      float acc = T[i][0] * R[j][0];  // right factor is R^T: (R^T)[k][j] = R[j][k]
      for (int k = 1; k < 4; k++) acc = acc + T[i][k] * R[j][k];
      M[i][j] = acc;
    }
  for (auto& pt : pts) {
    const float v[4] = {pt[0], pt[1], pt[2], 1.f};
    float o[3];
    for (int i = 0; i < 3; i++) o[i] = M[i][0] * v[0] + M[i][1] * v[1] + M[i][2] * v[2] + M[i][3] * v[3];
    std::memcpy(pt, o, sizeof(o));
  }
}

// CornellBox::buildBox (:63-139): near, far, top, near (dup), far (dup)
void box(SceneStore& s, const float n[3], const float f[3]) {
  P4 p;
  rect(p, {n[0], n[1], n[2], f[0], n[1], n[2], f[0], f[1], n[2], n[0], f[1], n[2]});
  s.add_quad(p, 1, 1);
  rect(p, {n[0], n[1], f[2], f[0], n[1], f[2], f[0], f[1], f[2], n[0], f[1], f[2]});
  s.add_quad(p, 1, 1);
  rect(p, {n[0], f[1], n[2], f[0], f[1], n[2], f[0], f[1], f[2], n[0], f[1], f[2]});
  s.add_quad(p, 1, 1);
  rect(p, {n[0], n[1], n[2], f[0], n[1], n[2], f[0], f[1], n[2], n[0], f[1], n[2]});
  s.add_quad(p, 1, 1);
  rect(p, {n[0], n[1], f[2], f[0], n[1], f[2], f[0], f[1], f[2], n[0], f[1], f[2]});
  s.add_quad(p, 1, 1);
}

void build(SceneStore& s, int variant) {
  P4 p;
  rect(p, {555, 0, 0, 555, 555, 0, 555, 555, 555, 555, 0, 555});  // green wall (:175-186)
  s.add_quad(p, 2, 2);
  rect(p, {0, 0, 0, 0, 555, 0, 0, 555, 555, 0, 0, 555});  // red wall (:189-200)
  s.add_quad(p, 0, 0);  // (four field values like every quad, :197-200: 89 values for the 89 points)
  rect(p, {213, 554, 227, 343, 554, 227, 343, 554, 332, 213, 554, 332});  // light (:204-215)
  s.add_quad(p, 3, 3);
  rect(p, {0, 555, 0, 555, 555, 0, 555, 555, 555, 0, 555, 555});  // ceiling
  s.add_quad(p, 1, 1);
  rect(p, {0, 0, 0, 555, 0, 0, 555, 0, 555, 0, 0, 555});  // floor
  s.add_quad(p, 1, 1);
  rect(p, {0, 0, 555, 555, 0, 555, 555, 555, 555, 0, 555, 555});  // back wall
  s.add_quad(p, 1, 1);
  if (variant == 3) {  // C3 stress scene: walls + light + kC3Spheres spheres (rtp.h)
    uint32_t st = kC3Seed;
    for (int k = 0; k < kC3Spheres; k++) {
      float cx = 190, cy = 90, cz = 190, rad = 90;
      int mat = 4, tex = 0;
      if (k > 0) {
        float u4, u5;
        for (;;) {  // redraw spheres that would intersect sphere 0
          const float u0 = draw(st), u1 = draw(st), u2 = draw(st), u3 = draw(st);
          u4 = draw(st);
          u5 = draw(st);
          rad = 8.0f + 22.0f * u3;
          cx = rad + (555.0f - 2.0f * rad) * u0;
          cy = rad + (555.0f - 2.0f * rad) * u1;
          cz = rad + (555.0f - 2.0f * rad) * u2;
          const float dx = cx - 190.0f, dy = cy - 90.0f, dz = cz - 190.0f, g = 92.0f + rad;
          if (!(dx * dx + dy * dy + dz * dz < g * g)) break;
        }
        if (u4 < 0.8f) {
          mat = std::min(2, (int)(3.0f * u5));
          tex = mat;
        }
      }
      s.sphere_point.push_back((int32_t)(s.points.size() / 3));
      for (float v : {cx, cy, cz}) s.points.push_back((float)((double)v / 555.0));
      s.sphere_radius.push_back((float)((double)rad / 555.0));
      s.sphere_mat.push_back(mat);
      s.sphere_tex.push_back(tex);
      s.add_vertex_cell();
    }
    s.finish_field();
    return;
  }
  const std::initializer_list<float> small_box[6] = {
      {0, 0, 165, 165, 0, 165, 165, 330, 165, 0, 330, 165},  {0, 0, 0, 165, 0, 0, 165, 330, 0, 0, 330, 0},
      {165, 0, 0, 165, 330, 0, 165, 330, 165, 165, 0, 165},  {0, 0, 0, 0, 330, 0, 0, 330, 165, 0, 0, 165},
      {0, 333, 0, 165, 330, 0, 165, 330, 165, 0, 330, 165}, {0, 0, 0, 165, 0, 0, 165, 0, 165, 0, 0, 165}};
  for (const auto& r : small_box) {
    rect(p, r);
    invert(p);
    s.add_quad(p, 1, 1);
  }
  // glass sphere vertex cell (:357-365); the extractor radius is 90/555.0
  float c[3] = {-335.f, 90.f, 290.f};
  if (variant == 1) c[0] = 190.f, c[1] = 90.f, c[2] = 190.f;  // notebook cell 2 position
  if (variant == 2) c[0] = 440.f, c[1] = 200.f, c[2] = 150.f;  // floating, clear of the boxes
  s.sphere_point.push_back((int32_t)(s.points.size() / 3));
  for (float v : c) s.points.push_back((float)((double)v / 555.0));
  s.sphere_radius.push_back((float)(90 / 555.0));
  s.sphere_mat.push_back(4);
  s.sphere_tex.push_back(0);
  s.add_vertex_cell();
  const float rad = 90;
  const float bc[3] = {135, 90, 290};
  const float n1[3] = {bc[0] - rad, 0, bc[2] - rad}, f1[3] = {bc[0] + rad, 180, bc[2] + rad};
  box(s, n1, f1);
  const float n2[3] = {50, 0, 50}, f2[3] = {450, 100, 100};
  box(s, n2, f2);
  s.finish_field();
}

SceneStore g_store[4];
std::once_flag g_once[4];

}  // namespace

extern "C" rtp_status rtp_cornell_box(int32_t variant, rtp_scene_desc* out) {
  if (!out || variant < 0 || variant > 3) return RTP_ERR_INVALID_ARGUMENT;
  std::call_once(g_once[variant], [variant] { build(g_store[variant], variant); });
  const SceneStore& s = g_store[variant];
  std::memset(out, 0, sizeof(*out));
  out->points = s.points.data();
  out->n_points = (int32_t)(s.points.size() / 3);
  out->quad_points = s.quad_points.data();
  out->quad_mat = s.quad_mat.data();
  out->quad_tex = s.quad_tex.data();
  out->n_quads = (int32_t)s.quad_mat.size();
  out->sphere_point = s.sphere_point.data();
  out->sphere_radius = s.sphere_radius.data();
  out->sphere_mat = s.sphere_mat.data();
  out->sphere_tex = s.sphere_tex.data();
  out->n_spheres = (int32_t)s.sphere_point.size();
  out->mat_type = s.mat_type;
  out->n_mat = 5;
  out->tex_type = s.tex_type;
  out->n_tex_type = 5;
  out->tex_rgb = s.tex_rgb;
  out->n_tex = 4;
  // MapperPathTracer.cxx:141-148
  out->light_quad_points[0] = 8;
  out->light_quad_points[1] = 9;
  out->light_quad_points[2] = 10;
  out->light_quad_points[3] = 11;
  out->light_sphere_point = s.sphere_point[0];  // 4 * 12 for variants 0..2
  out->ior = 1.5f;
  return RTP_OK;
}

extern "C" rtp_status rtp_cornell_point_field(int32_t variant, const float** field, int32_t* n_field,
                                              const int32_t** quad_cell, int32_t* n_quads) {
  if (!field || !n_field || !quad_cell || !n_quads || variant < 0 || variant > 3) return RTP_ERR_INVALID_ARGUMENT;
  std::call_once(g_once[variant], [variant] { build(g_store[variant], variant); });
  const SceneStore& s = g_store[variant];
  *field = s.field.data();
  *n_field = (int32_t)s.field.size();
  *quad_cell = s.quad_cell.data();
  *n_quads = (int32_t)s.quad_cell.size();
  return RTP_OK;
}
