// host_sanitize.cc — the library's host-only code under AddressSanitizer +
// UndefinedBehaviorSanitizer (sanitizers on host code; the GPU
// pool runs no GPU sanitizers).  Built by tests/test_host_sanitizers.py with
// the ROCm clang for the host (no offload), together with
//   dealii-ns-gls_amd/host/mesh.cc            the mesh generator (libglsmesh)
//   dealii-ns-gls_amd/csrc/brick_discovery.cc brick discovery (libglsamd)
// and exercises every mesh entry point and the discovery on shuffled cell
// lists; any sanitizer report fails the run (-fno-sanitize-recover).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#include "../../dealii-ns-gls_amd/csrc/op_internal.h"
#include "../../include/gls_mesh.h"

static int fails = 0;
#define CHECK(c)                                                      \
  do                                                                  \
    {                                                                 \
      if (!(c))                                                       \
        {                                                             \
          std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);     \
          ++fails;                                                    \
        }                                                             \
    }                                                                 \
  while (0)

// every per-mesh query, the constraint mask, measures, brick hint and the
// discovery of the cell list in generator order and shuffled
static void
exercise(glsMesh *m)
{
  const int     dim = gls_mesh_dim(m), k = gls_mesh_degree(m);
  const int64_t nc = gls_mesh_n_cells(m), nn = gls_mesh_n_nodes(m);
  const int     npc = dim == 3 ? (k + 1) * (k + 1) * (k + 1) : (k + 1) * (k + 1);
  const uint32_t *cn = gls_mesh_cell_nodes(m);
  for (int64_t i = 0; i < nc * npc; ++i)
    CHECK(cn[i] < (uint64_t)nn);
  std::vector<uint8_t> mask((size_t)nn);
  CHECK(gls_mesh_constraint_mask(m, 0x2u, 0x4u, 0x18u, mask.data()) == 0);
  std::vector<double> meas((size_t)nc), hmin((size_t)nc);
  CHECK(gls_mesh_cell_measure(m, meas.data(), hmin.data()) == 0);
  for (int64_t c = 0; c < nc; ++c)
    CHECK(meas[(size_t)c] > 0 && hmin[(size_t)c] > 0);
  int dims[3] = {0, 0, 0};
  CHECK(gls_mesh_brick(m, dims) == 0);

  std::vector<uint32_t> cells(cn, cn + nc * npc);
  for (int shuffled = 0; shuffled < 2; ++shuffled)
    {
      if (shuffled)
        {
          std::vector<int64_t> perm((size_t)nc);
          std::iota(perm.begin(), perm.end(), 0);
          std::shuffle(perm.begin(), perm.end(), std::mt19937_64(7));
          for (int64_t c = 0; c < nc; ++c)
            for (int j = 0; j < npc; ++j)
              cells[(size_t)(c * npc + j)] = cn[perm[(size_t)c] * npc + j];
        }
      gls::BrickPlan plan;
      const bool     ok = gls::discover_bricks(dim, k, nc, cells.data(), plan);
      if (ok)
        {
          CHECK((int64_t)plan.perm.size() == nc);
          std::vector<char> seen((size_t)nc, 0);
          for (int64_t c : plan.perm)
            {
              CHECK(c >= 0 && c < nc);
              if (c >= 0 && c < nc)
                seen[(size_t)c] = 1;
            }
          for (char s : seen)
            CHECK(s);
        }
    }
}

int
main()
{
  // cylinder channels (grid_cylinder.h) and hyper cubes, every degree, two
  // refinements, with the child lattices between consecutive levels
  for (int dim = 2; dim <= 3; ++dim)
    for (int k = 1; k <= 2; ++k)
      {
        glsMesh *lv[2] = {nullptr, nullptr};
        for (int r = 0; r < 2; ++r)
          {
            CHECK(gls_mesh_cylinder(dim, k, r, 2.2, 0.41, 0.2, 0.1, 0.0, &lv[r]) == 0);
            if (lv[r])
              exercise(lv[r]);
          }
        if (lv[0] && lv[1])
          {
            const int npl = dim == 3 ? (2 * k + 1) * (2 * k + 1) * (2 * k + 1) :
                                       (2 * k + 1) * (2 * k + 1);
            std::vector<uint32_t> lat((size_t)(gls_mesh_n_cells(lv[0]) * npl));
            CHECK(gls_mesh_child_lattice(lv[0], lv[1], lat.data()) == 0);
            for (uint32_t v : lat)
              CHECK(v < (uint64_t)gls_mesh_n_nodes(lv[1]));
          }
        for (glsMesh *m : lv)
          gls_mesh_destroy(m);
      }
  for (int dim = 2; dim <= 3; ++dim)
    for (int k = 1; k <= 3; ++k)
      {
        glsMesh *m = nullptr;
        CHECK(gls_mesh_hypercube(dim, k, 2, &m) == 0);
        if (m)
          exercise(m);
        gls_mesh_destroy(m);
      }
  // an unstructured coarse mesh (the sphere deck's path): two hexes sharing a
  // face, tagged boundary faces, refined twice
  {
    const double  v[12 * 3] = {0, 0, 0, 1, 0, 0, 2, 0, 0, 0, 1, 0, 1, 1, 0, 2, 1, 0,
                               0, 0, 1, 1, 0, 1, 2, 0, 1, 0, 1, 1, 1, 1, 1, 2, 1, 1};
    const int32_t cells[2 * 8] = {0, 1, 3, 4, 6, 7, 9, 10, 1, 2, 4, 5, 7, 8, 10, 11};
    const int32_t bf[2 * 4]    = {0, 3, 6, 9, 2, 5, 8, 11};
    const int32_t ids[2]       = {1, 2};
    glsMesh      *m            = nullptr;
    CHECK(gls_mesh_from_coarse(3, 2, 2, 12, v, 2, cells, 2, bf, ids, &m) == 0);
    if (m)
      exercise(m);
    gls_mesh_destroy(m);
  }
  // error paths: bad arguments return a status and a message
  {
    glsMesh *m = nullptr;
    CHECK(gls_mesh_cylinder(4, 2, 0, 2.2, 0.41, 0.2, 0.1, 0.0, &m) != 0);
    CHECK(gls_mesh_last_error() != nullptr);
  }
  std::printf("host sanitizer run: %d failures\n", fails);
  return fails ? 1 : 0;
}
