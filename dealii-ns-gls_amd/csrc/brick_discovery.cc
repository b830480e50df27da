// Brick discovery for an arbitrary cell order.
//
// The brick kernel (brick.h) needs the cells of a brick as a structured
// bx x by x bz block whose local lexicographic node orders agree (one node
// lattice per brick).  gls_mesh_* meshes come in that order already
// (glsOpDesc::brick); a deal.II DoFHandler / MatrixFree cell order does not
// (operator_ns.cc:806-830 runs its cell_loop over MatrixFree's cell batches,
// whatever their order).  This finds the blocks from the connectivity alone:
//
//  1. aligned neighbours: cell c' is the +a neighbour of c when c's face
//     x_a = k is c''s face x_a = 0 corner by corner (same orientation of the
//     other axes) -- children of one refined coarse cell always are;
//  2. integer block coordinates by a breadth-first walk over aligned
//     neighbours, per connected component;
//  3. the block phase per component and axis from the cells without a -a
//     neighbour (coarse-cell or domain boundaries sit at phase 0);
//  4. bricks from the origins (coordinate = phase mod shape), each checked:
//     every cell present and unused, and the lattice consistent (a node at
//     one lattice position only, a lattice position with one node).
//
// The first shape that covers every cell wins; the operator then runs its
// cells in the discovered order (plan.perm: internal -> caller cell).
#include <algorithm>
#include <array>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "op_internal.h"

namespace gls
{
namespace
{
struct FaceKey
{
  uint32_t v[4];
  bool
  operator==(const FaceKey &o) const
  {
    return v[0] == o.v[0] && v[1] == o.v[1] && v[2] == o.v[2] && v[3] == o.v[3];
  }
};

struct FaceKeyHash
{
  size_t
  operator()(const FaceKey &k) const
  {
    uint64_t h = 1469598103934665603ULL;
    for (uint32_t x : k.v)
      h = (h ^ x) * 1099511628211ULL;
    return (size_t)h;
  }
};

// try one shape; fills perm on success
bool
tile(int dim, int k, int64_t nc, const uint32_t *cn, const std::vector<int64_t> &nb,
     const std::vector<int64_t> &coord, const std::vector<int32_t> &comp, int32_t n_comp,
     const int B[3], std::vector<int64_t> &perm)
{
  const int n = k + 1, nq = dim == 3 ? n * n * n : n * n;
  // phase per (component, axis): the most frequent coordinate residue of the
  // cells without an aligned -a neighbour
  std::vector<int32_t> phase((size_t)n_comp * 3, 0);
  {
    std::vector<int32_t> hist((size_t)n_comp * 3 * 8, 0);
    for (int64_t c = 0; c < nc; ++c)
      for (int a = 0; a < dim; ++a)
        if (nb[((size_t)c * 3 + a) * 2] < 0)
          {
            const int64_t r = ((coord[(size_t)c * 3 + a] % B[a]) + B[a]) % B[a];
            hist[((size_t)comp[c] * 3 + a) * 8 + r]++;
          }
    for (int32_t q = 0; q < n_comp; ++q)
      for (int a = 0; a < dim; ++a)
        {
          const int32_t *h = &hist[((size_t)q * 3 + a) * 8];
          phase[(size_t)q * 3 + a] = (int32_t)(std::max_element(h, h + B[a]) - h);
        }
  }
  // origins, ordered by (component, block z, y, x, z inside the block): the
  // layers of one block and neighbouring blocks stay consecutive (the
  // launch order's L2 reuse, build_bricks)
  std::vector<int64_t> org;
  for (int64_t c = 0; c < nc; ++c)
    {
      bool o = true;
      for (int a = 0; a < dim && o; ++a)
        {
          const int64_t x = coord[(size_t)c * 3 + a] - phase[(size_t)comp[c] * 3 + a];
          o = ((x % B[a]) + B[a]) % B[a] == 0;
        }
      if (o)
        org.push_back(c);
    }
  const int64_t G = dim == 3 && B[2] == 1 ? 4 : 1; // group z layers of 4
  auto fl = [](int64_t x, int64_t m) { return x >= 0 ? x / m : -((-x + m - 1) / m); };
  std::sort(org.begin(), org.end(), [&](int64_t p, int64_t q) {
    auto key = [&](int64_t c) {
      const int64_t *x = &coord[(size_t)c * 3];
      const int64_t zb = fl(x[2], B[2] * G);
      return std::array<int64_t, 6>{comp[c], zb, fl(x[1], B[1]), fl(x[0], B[0]), x[2], c};
    };
    return key(p) < key(q);
  });
  const int Lx = k * B[0] + 1, Ly = k * B[1] + 1, Lz = dim == 3 ? k * B[2] + 1 : 1;
  const int L  = Lx * Ly * Lz;
  std::vector<char>     used((size_t)nc, 0);
  std::vector<uint32_t> lat((size_t)L);
  std::vector<int64_t>  cells((size_t)B[0] * B[1] * B[2]);
  std::unordered_map<uint32_t, int> pos;
  perm.clear();
  perm.reserve((size_t)nc);
  auto walk = [&](int64_t c, int a, int steps) {
    for (int s = 0; s < steps && c >= 0; ++s)
      c = nb[((size_t)c * 3 + a) * 2 + 1];
    return c;
  };
  for (int64_t o : org)
    {
      if (used[o])
        continue;
      bool ok = true;
      for (int l = 0; l < B[2] && ok; ++l)
        {
          const int64_t cz = walk(o, 2, l);
          for (int j = 0; j < B[1] && ok; ++j)
            {
              const int64_t cy = walk(cz, 1, j);
              for (int i = 0; i < B[0] && ok; ++i)
                {
                  const int64_t c = walk(cy, 0, i);
                  ok = c >= 0 && !used[c];
                  if (ok)
                    cells[(size_t)i + B[0] * (j + (size_t)B[1] * l)] = c;
                }
            }
        }
      if (!ok)
        continue;
      std::fill(lat.begin(), lat.end(), UINT32_MAX);
      pos.clear();
      for (int lc = 0; lc < B[0] * B[1] * B[2] && ok; ++lc)
        {
          const int     cx = lc % B[0], cy = (lc / B[0]) % B[1], cz = lc / (B[0] * B[1]);
          const int64_t c  = cells[(size_t)lc];
          for (int p = 0; p < nq && ok; ++p)
            {
              const int i = p % n, j = (p / n) % n, l = dim == 3 ? p / (n * n) : 0;
              const int li = (cx * k + i) + Lx * ((cy * k + j) + Ly * (cz * k + l));
              const uint32_t node = cn[(size_t)c * nq + p];
              if (lat[li] == UINT32_MAX)
                {
                  auto it = pos.find(node);
                  if (it != pos.end() && it->second != li)
                    ok = false; // one node at two lattice positions (a wrap)
                  lat[li]   = node;
                  pos[node] = li;
                }
              else if (lat[li] != node)
                ok = false;
            }
        }
      if (!ok)
        continue;
      for (int lc = 0; lc < B[0] * B[1] * B[2]; ++lc)
        {
          used[cells[(size_t)lc]] = 1;
          perm.push_back(cells[(size_t)lc]);
        }
    }
  return (int64_t)perm.size() == nc;
}
} // namespace

bool
discover_bricks(int dim, int k, int64_t nc, const uint32_t *cn, BrickPlan &plan)
{
  const int n = k + 1, nq = dim == 3 ? n * n * n : n * n;
  if (nc <= 0)
    return false;
  // 1. aligned neighbours nb[(c * 3 + a) * 2 + s], s = 0: -a, 1: +a
  std::vector<int64_t> nb((size_t)nc * 6, -1);
  auto face = [&](int64_t c, int a, int side) {
    FaceKey key{{UINT32_MAX, UINT32_MAX, UINT32_MAX, UINT32_MAX}};
    const int u = (a + 1) % dim, v = (a + 2) % dim;
    int       t = 0;
    for (int vv = 0; vv < (dim == 3 ? 2 : 1); ++vv)
      for (int uu = 0; uu < 2; ++uu)
        {
          int idx[3] = {0, 0, 0};
          idx[a]     = side * k;
          idx[u]     = uu * k;
          if (dim == 3)
            idx[v] = vv * k;
          key.v[t++] = cn[(size_t)c * nq + idx[0] + n * (idx[1] + n * idx[2])];
        }
    return key;
  };
  for (int a = 0; a < dim; ++a)
    {
      std::unordered_map<FaceKey, int64_t, FaceKeyHash> minus;
      minus.reserve((size_t)nc * 2);
      for (int64_t c = 0; c < nc; ++c)
        {
          auto r = minus.emplace(face(c, a, 0), c);
          if (!r.second)
            r.first->second = -2; // two cells with one face: not conforming
        }
      for (int64_t c = 0; c < nc; ++c)
        {
          auto it = minus.find(face(c, a, 1));
          if (it == minus.end() || it->second < 0 || it->second == c)
            continue;
          const int64_t d = it->second;
          if (nb[((size_t)d * 3 + a) * 2] != -1)
            {
              nb[((size_t)d * 3 + a) * 2] = -2;
              continue;
            }
          nb[((size_t)c * 3 + a) * 2 + 1] = d;
          nb[((size_t)d * 3 + a) * 2]     = c;
        }
    }
  for (auto &x : nb)
    x = x < 0 ? -1 : x;
  // 2. coordinates per component
  std::vector<int64_t> coord((size_t)nc * 3, 0);
  std::vector<int32_t> comp((size_t)nc, -1);
  int32_t              n_comp = 0;
  std::vector<int64_t> queue;
  queue.reserve((size_t)nc);
  for (int64_t s = 0; s < nc; ++s)
    {
      if (comp[s] >= 0)
        continue;
      comp[s] = n_comp;
      queue.clear();
      queue.push_back(s);
      for (size_t h = 0; h < queue.size(); ++h)
        {
          const int64_t c = queue[h];
          for (int a = 0; a < dim; ++a)
            for (int sd = 0; sd < 2; ++sd)
              {
                const int64_t d = nb[((size_t)c * 3 + a) * 2 + sd];
                if (d < 0 || comp[d] >= 0)
                  continue;
                comp[d] = n_comp;
                for (int e = 0; e < 3; ++e)
                  coord[(size_t)d * 3 + e] = coord[(size_t)c * 3 + e];
                coord[(size_t)d * 3 + a] += sd ? 1 : -1;
                queue.push_back(d);
              }
        }
      ++n_comp;
    }
  // 3./4. shapes, largest first (brick.h limits: 4 x 4 footprint, 16 cells
  // in 3D; 8 x 8 in 2D)
  static const int S3[][3] = {{4, 4, 1}, {2, 2, 2}, {2, 2, 1}, {1, 1, 1}};
  static const int S2[][3] = {{8, 8, 1}, {4, 4, 1}, {2, 2, 1}, {1, 1, 1}};
  for (int s = 0; s < 4; ++s)
    {
      const int *B = dim == 3 ? S3[s] : S2[s];
      if (tile(dim, k, nc, cn, nb, coord, comp, n_comp, B, plan.perm))
        {
          plan.shape[0] = B[0], plan.shape[1] = B[1], plan.shape[2] = B[2];
          return true;
        }
    }
  plan.perm.clear();
  return false;
}
} // namespace gls
