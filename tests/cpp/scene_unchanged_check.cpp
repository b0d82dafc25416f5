// scene_unchanged_check.cpp -- the reference's own CornellBox (CornellBox.h /
// CornellBox.cpp, compiled unchanged over include/vtkm_compat) against the
// library's scene builder (rtp_cornell_box, csrc/scene_cornell.cpp): the same
// points bit for bit, the same quads, vertex cells, material and texture
// tables.  Built by build.build_main_unchanged where the reference exists; no
// GPU needed.  Prints "OK" and exits 0 when every check passes.
#include <cstdio>
#include <cstring>

#include "CornellBox.h"  // the reference's header (the compile puts the reference tree on the quote path)

static int failures = 0;
#define EXPECT(cond)                                           \
  do {                                                         \
    if (!(cond)) {                                             \
      std::fprintf(stderr, "FAIL %d: %s\n", __LINE__, #cond);  \
      failures++;                                              \
    }                                                          \
  } while (0)

int main() {
  CornellBox cb;
  cb.buildDataSet();
  rtp_scene_desc d{};
  EXPECT(rtp_cornell_box(0, &d) == RTP_OK);
  // points: the data set's coordinates and the CornellBox's coord, bit for bit
  const auto& P = cb.ds.GetCoordinateSystem();
  EXPECT((int)P.size() == d.n_points && (int)cb.coord.size() == d.n_points);
  for (int i = 0; i < d.n_points && i < (int)P.size(); i++)
    for (int k = 0; k < 3; k++) {
      EXPECT(std::memcmp(&P[i][k], &d.points[3 * i + k], 4) == 0);
      EXPECT(std::memcmp(&cb.coord[i][k], &d.points[3 * i + k], 4) == 0);
    }
  const auto& C = cb.ds.GetCellSet();
  EXPECT((int)C.quads.size() == d.n_quads);
  for (int q = 0; q < d.n_quads && q < (int)C.quads.size(); q++)
    for (int k = 0; k < 4; k++) EXPECT(C.quads[q][k] == d.quad_points[4 * q + k]);
  EXPECT((int)C.spheres.size() == d.n_spheres && d.n_spheres == 1 && C.spheres[0] == d.sphere_point[0]);
  EXPECT((int)cb.matIdx[0].size() == d.n_quads && (int)cb.matIdx[1].size() == d.n_spheres);
  for (int q = 0; q < d.n_quads; q++) EXPECT(cb.matIdx[0][q] == d.quad_mat[q] && cb.texIdx[0][q] == d.quad_tex[q]);
  EXPECT(cb.matIdx[1][0] == d.sphere_mat[0] && cb.texIdx[1][0] == d.sphere_tex[0]);
  EXPECT((int)cb.matType.size() == d.n_mat && (int)cb.texType.size() == d.n_tex_type && (int)cb.tex.size() == d.n_tex);
  for (int i = 0; i < d.n_mat; i++) EXPECT(cb.matType[i] == d.mat_type[i]);
  for (int i = 0; i < d.n_tex_type; i++) EXPECT(cb.texType[i] == d.tex_type[i]);
  for (int i = 0; i < d.n_tex; i++)
    for (int k = 0; k < 3; k++) EXPECT(std::memcmp(&cb.tex[i][k], &d.tex_rgb[3 * i + k], 4) == 0);
  // the quad cells' ids and the point field the -direct mappers read
  const float* fv = nullptr;
  const int32_t* qc = nullptr;
  int32_t nf = 0, nq = 0;
  EXPECT(rtp_cornell_point_field(0, &fv, &nf, &qc, &nq) == RTP_OK);
  EXPECT(nq == (int)C.quadCells.size());
  for (int i = 0; i < nq && i < (int)C.quadCells.size(); i++) EXPECT(C.quadCells[i] == qc[i]);
  const auto& F = cb.ds.GetField("point_var");
  EXPECT((int)F.values.size() == nf);
  for (int i = 0; i < nf && i < (int)F.values.size(); i++) EXPECT(std::memcmp(&F.values[i], &fv[i], 4) == 0);
  // CornellBox::extract over the shim's extractors
  cb.extract();
  EXPECT((int)cb.QuadIds.size() == d.n_quads && (int)cb.SphereIds.size() == 1);
  EXPECT(cb.SphereRadii.size() == 1 && cb.SphereRadii[0] == (float)(90.0 / 555.0));
  if (failures) return 1;
  std::printf("OK\n");
  return 0;
}
