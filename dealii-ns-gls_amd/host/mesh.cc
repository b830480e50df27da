// mesh.cc — host-side mesh / DoF / constraint setup (libglsmesh.so).
//
// Restates the part of the reference's deal.II setup pipeline that feeds the
// hot path (see include/gls_mesh.h for the interface):
//
//  * coarse mesh of the flow-past-cylinder channel, grid_cylinder.h:7-151
//    (2D: hyper_cube_with_cylindrical_hole + 8 subdivided rectangles merged)
//    and grid_cylinder.h:153-242 (3D: extrusion into 4 layers, shifted to
//    z in [-H/2, H/2]); boundary ids from face centres, :112-133 / :200-223;
//  * uniform global refinement (simulation.cc:316-326: every cell centre lies
//    left of x = length - position, so every cell is refined);
//  * new points placed like deal.II's manifolds do: points on the cylinder
//    surface by averaging in cylindrical coordinates (PolarManifold /
//    CylindricalManifold attached to manifold id 0, grid_cylinder.h:100,189),
//    every other new point by transfinite interpolation of the surrounding
//    vertices / line mid points / face mid points (FlatManifold with
//    interpolate_from_surrounding);
//  * MappingQ_k support points == the Q_k nodes of the cell; because the
//    geometry is refined with the same rules, the Q2 nodes of level r are the
//    vertices of level r + 1 (SURVEY §8d counting argument);
//  * nodes are identified topologically across coarse cells (shared coarse
//    vertex / edge / face + lattice coordinates), numbered in order of first
//    appearance in cell order (cache-friendly), cells ordered by coarse cell
//    (sorted by centre x, y, z -> contiguous cell ranges are x-slabs for the
//    multi-GPU partition) then lexicographically inside the coarse cell.
//
// Not a port of deal.II: this is an independent restatement; exact
// bit-parity of coordinates with deal.II's MappingQ is not claimed
// ("parity unpinned" for geometry).

#include "../../include/gls_mesh.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace
{
thread_local std::string g_err;

using P3 = std::array<double, 3>;

struct CoarseMesh
{
  int                             dim = 3;
  std::vector<P3>                 vertices;
  std::vector<std::array<int, 8>> cells; // 2^dim used, lexicographic
  // boundary id per (cell, face); -1 = interior face.  face f: axis f/2,
  // side f%2
  std::vector<std::array<int, 6>> face_bid;
};

} // namespace

struct glsMesh_
{
  int                   dim    = 3;
  int                   degree = 2;
  int                   n_ref  = 0;
  int64_t               n_coarse = 0;
  std::vector<uint32_t> cell_nodes;
  std::vector<double>   coords;
  std::vector<uint32_t> node_bid;
  std::vector<int32_t>  cell_coarse;
  int64_t               n_cells = 0;
  int64_t               n_nodes = 0;
  // slip normal axis per boundary id (-1 = not planar/axis aligned)
  int slip_axis[32];
  // per axis d: boundary ids of the axis-aligned planar faces with normal d
  // that touch the node (no-normal-flux constraints of flat walls); bit b of
  // nonplanar_bids: a face with id b is curved or oblique
  std::vector<uint32_t> node_axis_bid[3];
  uint32_t              nonplanar_bids = 0;
  // generator parameters (for child lattice consistency checks)
  std::vector<double> params;
};

namespace
{
// ---------------------------------------------------------------- geometry
struct CurvedSurface
{
  bool   active = false;
  double radius = 0.0; // cylinder (3D, axis z through origin) / circle (2D)

  bool
  on(const P3 &p) const
  {
    if (!active)
      return false;
    const double r = std::hypot(p[0], p[1]);
    return std::abs(r - radius) < 1e-10 * std::max(1.0, radius);
  }
};

inline P3
add(const P3 &a, const P3 &b)
{
  return {a[0] + b[0], a[1] + b[1], a[2] + b[2]};
}
inline P3
scale(const P3 &a, double s)
{
  return {a[0] * s, a[1] * s, a[2] * s};
}

// wrap an angle difference into (-pi, pi]
inline double
wrap(double d)
{
  while (d > M_PI)
    d -= 2 * M_PI;
  while (d <= -M_PI)
    d += 2 * M_PI;
  return d;
}

// Weighted average of points in cylindrical coordinates (r, phi, z), the
// angle unwrapped around the first point (ChartManifold with periodic phi).
P3
cyl_average(const P3 *pts, const double *w, int n)
{
  const double phi0 = std::atan2(pts[0][1], pts[0][0]);
  double       r = 0, phi = 0, z = 0;
  for (int i = 0; i < n; ++i)
    {
      const double ri = std::hypot(pts[i][0], pts[i][1]);
      const double pi = phi0 + wrap(std::atan2(pts[i][1], pts[i][0]) - phi0);
      r += w[i] * ri;
      phi += w[i] * pi;
      z += w[i] * pts[i][2];
    }
  return {r * std::cos(phi), r * std::sin(phi), z};
}

P3
edge_mid(const P3 &a, const P3 &b, const CurvedSurface &cs)
{
  if (cs.on(a) && cs.on(b))
    {
      const P3     p[2] = {a, b};
      const double w[2] = {0.5, 0.5};
      return cyl_average(p, w, 2);
    }
  return scale(add(a, b), 0.5);
}

// quad centre from 4 vertices + 4 line mid points (transfinite interpolation:
// lines +1/2, vertices -1/4); on the curved surface in cylindrical coords.
P3
quad_center(const P3 v[4], const P3 e[4], const CurvedSurface &cs)
{
  const bool curved = cs.on(v[0]) && cs.on(v[1]) && cs.on(v[2]) && cs.on(v[3]);
  if (curved)
    {
      P3     p[8];
      double w[8];
      for (int i = 0; i < 4; ++i)
        {
          p[i]     = v[i];
          w[i]     = -0.25;
          p[4 + i] = e[i];
          w[4 + i] = 0.5;
        }
      return cyl_average(p, w, 8);
    }
  P3 c = {0, 0, 0};
  for (int i = 0; i < 4; ++i)
    c = add(c, add(scale(e[i], 0.5), scale(v[i], -0.25)));
  return c;
}

// ------------------------------------------------------------ lattices
// Lattice of (n+1)^dim points of one coarse cell, refined recursively from
// its corners.  Index: i + (n+1)*(j + (n+1)*l).
struct Lattice
{
  int             dim;
  int             n;
  std::vector<P3> p;

  P3 &
  at(int i, int j, int l)
  {
    return p[i + (n + 1) * (j + (n + 1) * l)];
  }
};

Lattice
refine_lattice(const Lattice &in, const CurvedSurface &cs)
{
  Lattice out;
  out.dim        = in.dim;
  out.n          = 2 * in.n;
  const int N    = out.n + 1;
  const int Nz   = (in.dim == 3) ? N : 1;
  out.p.assign((size_t)N * N * Nz, P3{0, 0, 0});
  const int Mi   = in.n + 1;
  auto      inat = [&](int i, int j, int l) -> const P3 & {
    return in.p[i + Mi * (j + Mi * l)];
  };
  auto Q = [&](int i, int j, int l) -> P3 & {
    return out.p[i + N * (j + N * l)];
  };
  const int lz_in = (in.dim == 3) ? in.n : 0;
  // copy
  for (int l = 0; l <= lz_in; ++l)
    for (int j = 0; j <= in.n; ++j)
      for (int i = 0; i <= in.n; ++i)
        Q(2 * i, 2 * j, 2 * l) = inat(i, j, l);

  const int lmax = (in.dim == 3) ? out.n : 0;
  // edges: exactly one odd index
  for (int l = 0; l <= lmax; ++l)
    for (int j = 0; j <= out.n; ++j)
      for (int i = 0; i <= out.n; ++i)
        {
          const int odd = (i & 1) + (j & 1) + (l & 1);
          if (odd != 1)
            continue;
          if (i & 1)
            Q(i, j, l) = edge_mid(Q(i - 1, j, l), Q(i + 1, j, l), cs);
          else if (j & 1)
            Q(i, j, l) = edge_mid(Q(i, j - 1, l), Q(i, j + 1, l), cs);
          else
            Q(i, j, l) = edge_mid(Q(i, j, l - 1), Q(i, j, l + 1), cs);
        }
  // faces (3D) / cells (2D): exactly two odd indices
  for (int l = 0; l <= lmax; ++l)
    for (int j = 0; j <= out.n; ++j)
      for (int i = 0; i <= out.n; ++i)
        {
          const int odd = (i & 1) + (j & 1) + (l & 1);
          if (odd != 2)
            continue;
          // the two odd axes span the quad
          int a0, a1;
          if (!(i & 1))
            a0 = 1, a1 = 2;
          else if (!(j & 1))
            a0 = 0, a1 = 2;
          else
            a0 = 0, a1 = 1;
          int  idx[3] = {i, j, l};
          auto off    = [&](int d0, int d1) -> P3 & {
            int t[3] = {idx[0], idx[1], idx[2]};
            t[a0] += d0;
            t[a1] += d1;
            return Q(t[0], t[1], t[2]);
          };
          P3 v[4] = {off(-1, -1), off(1, -1), off(-1, 1), off(1, 1)};
          P3 e[4] = {off(0, -1), off(0, 1), off(-1, 0), off(1, 0)};
          Q(i, j, l) = quad_center(v, e, cs);
        }
  // hex centres (3D): three odd indices; transfinite: faces +1/2, lines
  // -1/4, vertices +1/8
  if (in.dim == 3)
    for (int l = 1; l <= out.n; l += 2)
      for (int j = 1; j <= out.n; j += 2)
        for (int i = 1; i <= out.n; i += 2)
          {
            P3 c = {0, 0, 0};
            for (int dl = -1; dl <= 1; ++dl)
              for (int dj = -1; dj <= 1; ++dj)
                for (int di = -1; di <= 1; ++di)
                  {
                    const int nz = (di != 0) + (dj != 0) + (dl != 0);
                    double    w  = 0;
                    if (nz == 1)
                      w = 0.5;
                    else if (nz == 2)
                      w = -0.25;
                    else if (nz == 3)
                      w = 0.125;
                    if (w != 0)
                      c = add(c, scale(Q(i + di, j + dj, l + dl), w));
                  }
            Q(i, j, l) = c;
          }
  return out;
}

// ------------------------------------------------------------ coarse meshes
// vertex merge by position (coarse meshes are tiny)
int
find_or_add_vertex(std::vector<P3> &verts, const P3 &p)
{
  for (size_t i = 0; i < verts.size(); ++i)
    if (std::abs(verts[i][0] - p[0]) < 1e-12 &&
        std::abs(verts[i][1] - p[1]) < 1e-12 &&
        std::abs(verts[i][2] - p[2]) < 1e-12)
      return (int)i;
  verts.push_back(p);
  return (int)verts.size() - 1;
}

// GridGenerator::subdivided_hyper_rectangle in 2D (corner points sorted)
void
add_rectangle(std::vector<std::array<P3, 4>> &quads, int nx, int ny,
              double x0, double y0, double x1, double y1)
{
  const double xa = std::min(x0, x1), xb = std::max(x0, x1);
  const double ya = std::min(y0, y1), yb = std::max(y0, y1);
  for (int j = 0; j < ny; ++j)
    for (int i = 0; i < nx; ++i)
      {
        const double u0 = xa + (xb - xa) * i / nx, u1 = xa + (xb - xa) * (i + 1) / nx;
        const double v0 = ya + (yb - ya) * j / ny, v1 = ya + (yb - ya) * (j + 1) / ny;
        quads.push_back({P3{u0, v0, 0}, P3{u1, v0, 0}, P3{u0, v1, 0}, P3{u1, v1, 0}});
      }
}

std::vector<std::array<P3, 4>>
cylinder_2d_quads(double length, double height, double pos, double D,
                  double shift, bool for_3D)
{
  std::vector<std::array<P3, 4>> q;
  // hyper_cube_with_cylindrical_hole(inner D/2, outer D): 8 cells between
  // the circle (radius D/2) and the square [-D, D]^2, one per 45 degrees.
  const double ri = D / 2., ro = D;
  for (int k = 0; k < 8; ++k)
    {
      auto inner = [&](int kk) {
        const double a = kk * M_PI / 4.;
        return P3{ri * std::cos(a), ri * std::sin(a), 0};
      };
      auto outer = [&](int kk) {
        kk %= 8;
        const double a = kk * M_PI / 4.;
        // even: edge mid points of the square, odd: its corners
        if (kk % 2 == 0)
          return P3{ro * std::round(std::cos(a)), ro * std::round(std::sin(a)), 0};
        return P3{ro * (std::cos(a) > 0 ? 1. : -1.), ro * (std::sin(a) > 0 ? 1. : -1.), 0};
      };
      // xi radial (inner -> outer), eta along increasing angle
      q.push_back({inner(k), outer(k), inner(k + 1), outer(k + 1)});
    }
  const double H = height;
  add_rectangle(q, 2, 1, -D, -D, D, -H / 2. + shift);
  add_rectangle(q, 2, 1, -D, D, D, H / 2. + shift);
  add_rectangle(q, 18, 2, D, -D, length - pos, D);
  add_rectangle(q, 18, 1, D, D, length - pos, H / 2. + shift);
  add_rectangle(q, 18, 1, D, -H / 2. + shift, length - pos, -D);
  const int nl = for_3D ? 4 : 1;
  add_rectangle(q, nl, 2, -pos, -D, -D, D);
  add_rectangle(q, nl, 1, -pos, D, -D, H / 2. + shift);
  add_rectangle(q, nl, 1, -pos, -H / 2. + shift, -D, -D);
  return q;
}

void
compute_face_bids(CoarseMesh &cm, double length, double height, double pos,
                  double shift, bool cylinder_rules)
{
  const int nv = 1 << cm.dim, nf = 2 * cm.dim, nvf = nv / 2;
  std::map<std::vector<int>, int> count;
  auto face_verts = [&](int c, int f) {
    const int        axis = f / 2, side = f % 2;
    std::vector<int> v;
    for (int k = 0; k < nv; ++k)
      if (((k >> axis) & 1) == side)
        v.push_back(cm.cells[c][k]);
    std::sort(v.begin(), v.end());
    return v;
  };
  for (size_t c = 0; c < cm.cells.size(); ++c)
    for (int f = 0; f < nf; ++f)
      count[face_verts(c, f)]++;
  cm.face_bid.assign(cm.cells.size(), std::array<int, 6>{-1, -1, -1, -1, -1, -1});
  for (size_t c = 0; c < cm.cells.size(); ++c)
    for (int f = 0; f < nf; ++f)
      {
        const auto fv = face_verts(c, f);
        if (count[fv] != 1)
          continue;
        P3 ctr = {0, 0, 0};
        for (int v : fv)
          ctr = add(ctr, cm.vertices[v]);
        ctr = scale(ctr, 1.0 / nvf);
        int bid = 0;
        if (cylinder_rules)
          {
            if (ctr[0] > length - pos - 1e-6)
              bid = 1;
            else if (ctr[0] < -pos + 1e-6)
              bid = 0;
            else if (std::abs(ctr[1] - (height / 2. + shift)) < 1e-6)
              bid = 4;
            else if (std::abs(ctr[1] - (-height / 2. + shift)) < 1e-6)
              bid = 3;
            else if (cm.dim == 3 && std::abs(ctr[2] - height / 2.) < 1e-6)
              bid = 6;
            else if (cm.dim == 3 && std::abs(ctr[2] + height / 2.) < 1e-6)
              bid = 5;
            else
              bid = 2;
          }
        cm.face_bid[c][f] = bid;
      }
}

// ------------------------------------------------------------ cell order
// Inside a coarse cell refined to nsub^dim cells, cells are ordered
// brick-major: bricks of b[d] = min(nsub, BRICK[d]) cells per direction in
// lexicographic order, cells lexicographic inside a brick.  The operator
// processes one brick per workgroup (see csrc/brick.h); 3D bricks are
// 4 x 4 x 2 cells so that the headline mesh (400 coarse cells, r = 2) yields
// 800 workgroups for the 256 CUs.
inline void
brick_dims(int nsub, int dim, int b[3])
{
  const int B[3] = {dim == 3 ? 4 : 8, dim == 3 ? 4 : 8, dim == 3 ? 2 : 1};
  for (int d = 0; d < 3; ++d)
    b[d] = (d < dim) ? (nsub < B[d] ? nsub : B[d]) : 1;
}

inline int64_t
local_cell_index(int cx, int cy, int cz, int nsub, int dim)
{
  int b[3];
  brick_dims(nsub, dim, b);
  const int     nbx = nsub / b[0], nby = nsub / b[1];
  const int64_t brick =
    (cx / b[0]) + (int64_t)nbx * ((cy / b[1]) + (int64_t)nby * (dim == 3 ? (cz / b[2]) : 0));
  const int64_t inner =
    (cx % b[0]) + (int64_t)b[0] * ((cy % b[1]) + (int64_t)b[1] * (dim == 3 ? (cz % b[2]) : 0));
  return brick * ((int64_t)b[0] * b[1] * b[2]) + inner;
}

inline void
local_cell_coords(int64_t r, int nsub, int dim, int &cx, int &cy, int &cz)
{
  int b[3];
  brick_dims(nsub, dim, b);
  const int     nbx = nsub / b[0], nby = nsub / b[1];
  const int64_t cpb   = (int64_t)b[0] * b[1] * b[2];
  const int64_t brick = r / cpb, inner = r % cpb;
  const int     bx = (int)(brick % nbx), by = (int)((brick / nbx) % nby),
            bz = dim == 3 ? (int)(brick / ((int64_t)nbx * nby)) : 0;
  const int ix = (int)(inner % b[0]), iy = (int)((inner / b[0]) % b[1]),
            iz = dim == 3 ? (int)(inner / ((int64_t)b[0] * b[1])) : 0;
  cx = bx * b[0] + ix;
  cy = by * b[1] + iy;
  cz = bz * b[2] + iz;
}

// ------------------------------------------------------------ fine mesh
struct KeyHash
{
  size_t
  operator()(const std::array<int64_t, 6> &k) const
  {
    uint64_t h = 1469598103934665603ULL;
    for (auto v : k)
      {
        h ^= (uint64_t)v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
        h *= 1099511628211ULL;
      }
    return h;
  }
};

glsMesh_ *
build_fine(const CoarseMesh &cm, int degree, int n_ref, const CurvedSurface &cs)
{
  auto *m     = new glsMesh_();
  m->dim      = cm.dim;
  m->degree   = degree;
  m->n_ref    = n_ref;
  m->n_coarse = (int64_t)cm.cells.size();
  for (int &a : m->slip_axis)
    a = -1;

  const int dim  = cm.dim;
  const int nsub = 1 << n_ref;        // fine cells per direction per coarse cell
  const int n    = degree * nsub;     // lattice intervals per direction
  const int N    = n + 1;
  const int Nz   = dim == 3 ? N : 1;
  const int kp   = degree + 1;
  const int nloc = dim == 3 ? kp * kp * kp : kp * kp;
  const int64_t cells_per_coarse = dim == 3 ? (int64_t)nsub * nsub * nsub : (int64_t)nsub * nsub;
  m->n_cells                     = cells_per_coarse * (int64_t)cm.cells.size();
  m->cell_nodes.resize((size_t)m->n_cells * nloc);
  m->cell_coarse.resize((size_t)m->n_cells);

  // lattice refinement needs n to be a power of two (k in {1,2}) unless the
  // cell is affine (hypercube), where points follow from linear interpolation
  const bool pow2 = (n & (n - 1)) == 0;

  std::unordered_map<std::array<int64_t, 6>, uint32_t, KeyHash> shared;
  shared.reserve(1 << 20);
  std::vector<double>   coords;
  std::vector<uint32_t> bids;
  coords.reserve((size_t)m->n_cells * dim * 2);
  const int nv = 1 << dim;

  std::vector<uint32_t> lattice_node((size_t)N * N * Nz);
  std::vector<uint32_t> axis_bid[3];

  for (size_t c = 0; c < cm.cells.size(); ++c)
    {
      // ---- lattice geometry
      Lattice lat;
      lat.dim = dim;
      if (pow2)
        {
          lat.n = 1;
          lat.p.resize(nv);
          for (int k = 0; k < nv; ++k)
            lat.p[k] = cm.vertices[cm.cells[c][k]];
          while (lat.n < n)
            lat = refine_lattice(lat, cs);
        }
      else
        {
          // affine/multilinear only (hypercube with degree 3): GLL points
          if (cs.active)
            throw std::runtime_error("degree 3 only supported on flat meshes");
          std::vector<double> g1 = {0.0, 0.5 - std::sqrt(5.0) / 10.0,
                                    0.5 + std::sqrt(5.0) / 10.0, 1.0};
          lat.n = n;
          lat.p.assign((size_t)N * N * Nz, P3{0, 0, 0});
          auto t = [&](int i) {
            const int cell = std::min(i / degree, nsub - 1);
            const int loc  = i - cell * degree;
            return (cell + g1[loc]) / nsub;
          };
          for (int l = 0; l < Nz; ++l)
            for (int j = 0; j < N; ++j)
              for (int i = 0; i < N; ++i)
                {
                  const double s[3] = {t(i), t(j), dim == 3 ? t(l) : 0.0};
                  P3           p    = {0, 0, 0};
                  for (int k = 0; k < nv; ++k)
                    {
                      double w = 1;
                      for (int d = 0; d < dim; ++d)
                        w *= ((k >> d) & 1) ? s[d] : 1 - s[d];
                      p = add(p, scale(cm.vertices[cm.cells[c][k]], w));
                    }
                  lat.p[i + N * (j + N * l)] = p;
                }
        }

      // ---- node identification
      const auto &V = cm.cells[c];
      for (int l = 0; l < Nz; ++l)
        for (int j = 0; j < N; ++j)
          for (int i = 0; i < N; ++i)
            lattice_node[i + N * (j + N * l)] = UINT32_MAX;

      auto get_node = [&](int i, int j, int l) -> uint32_t {
        uint32_t &slot = lattice_node[i + N * (j + N * l)];
        if (slot != UINT32_MAX)
          return slot;
        const int idx[3] = {i, j, l};
        int       nb     = 0; // number of coordinates on the coarse cell boundary
        for (int d = 0; d < dim; ++d)
          nb += (idx[d] == 0 || idx[d] == n);
        std::array<int64_t, 6> key{};
        bool                   is_shared = nb > 0;
        if (nb == dim)
          {
            int corner = 0;
            for (int d = 0; d < dim; ++d)
              corner |= (idx[d] == n) << d;
            key = {0, V[corner], 0, 0, 0, 0};
          }
        else if (nb == dim - 1)
          {
            // on a coarse edge: free axis a
            int a = 0;
            for (int d = 0; d < dim; ++d)
              if (!(idx[d] == 0 || idx[d] == n))
                a = d;
            int base = 0;
            for (int d = 0; d < dim; ++d)
              if (d != a)
                base |= (idx[d] == n) << d;
            const int va = V[base], vb = V[base | (1 << a)];
            const int t  = idx[a];
            key = {1, std::min(va, vb), std::max(va, vb), va < vb ? t : n - t, 0, 0};
          }
        else if (dim == 3 && nb == 1)
          {
            int a = 0;
            for (int d = 0; d < 3; ++d)
              if (idx[d] == 0 || idx[d] == n)
                a = d;
            const int side = idx[a] == n;
            int       a1 = -1, a2 = -1;
            for (int d = 0; d < 3; ++d)
              if (d != a)
                {
                  if (a1 < 0)
                    a1 = d;
                  else
                    a2 = d;
                }
            auto corner = [&](int s1, int s2) {
              return V[(side << a) | (s1 << a1) | (s2 << a2)];
            };
            // origin = corner with the smallest vertex id
            int best = -1, ps = 0, qs = 0;
            for (int s2 = 0; s2 < 2; ++s2)
              for (int s1 = 0; s1 < 2; ++s1)
                if (best < 0 || corner(s1, s2) < best)
                  best = corner(s1, s2), ps = s1, qs = s2;
            const int id1 = corner(1 - ps, qs), id2 = corner(ps, 1 - qs);
            const int u   = ps ? n - idx[a1] : idx[a1];
            const int v   = qs ? n - idx[a2] : idx[a2];
            if (id1 < id2)
              key = {2, best, id1, id2, u, v};
            else
              key = {2, best, id2, id1, v, u};
          }
        uint32_t id;
        if (is_shared)
          {
            auto it = shared.find(key);
            if (it != shared.end())
              {
                slot = it->second;
                return slot;
              }
            id = (uint32_t)(coords.size() / dim);
            shared.emplace(key, id);
          }
        else
          id = (uint32_t)(coords.size() / dim);
        const P3 &p = lat.p[i + N * (j + N * l)];
        for (int d = 0; d < dim; ++d)
          coords.push_back(p[d]);
        bids.push_back(0);
        slot = id;
        return id;
      };

      const int64_t cbase = (int64_t)c * cells_per_coarse;
      // brick-major cell order (see local_cell_index); node numbers follow
      // first appearance in that order, so a brick's nodes are clustered
      for (int64_t r = 0; r < cells_per_coarse; ++r)
            {
              int cx, cy, cz;
              local_cell_coords(r, nsub, dim, cx, cy, cz);
              const int64_t cell = cbase + r;
              m->cell_coarse[cell] = (int32_t)c;
              uint32_t *cn         = &m->cell_nodes[(size_t)cell * nloc];
              int       q          = 0;
              const int kz         = dim == 3 ? kp : 1;
              for (int l = 0; l < kz; ++l)
                for (int j = 0; j < kp; ++j)
                  for (int i = 0; i < kp; ++i)
                    cn[q++] = get_node(cx * degree + i, cy * degree + j,
                                       dim == 3 ? cz * degree + l : 0);
            }

      // ---- boundary ids of the lattice points on boundary faces
      for (int f = 0; f < 2 * dim; ++f)
        {
          const int bid = cm.face_bid[c][f];
          if (bid < 0)
            continue;
          const int a = f / 2, side = f % 2;
          // physical normal axis of the (flat, axis-aligned) coarse face
          int nax = -1;
          {
            std::vector<P3> fv;
            for (int k = 0; k < nv; ++k)
              if (((k >> a) & 1) == side)
                fv.push_back(cm.vertices[cm.cells[c][k]]);
            for (int d = 0; d < dim && nax < 0; ++d)
              {
                bool same = true;
                for (const P3 &q : fv)
                  same = same && std::abs(q[d] - fv[0][d]) <= 1e-12 * (1.0 + std::abs(fv[0][d]));
                if (same)
                  nax = d;
              }
            if (nax < 0)
              {
                nax = -1;
                m->nonplanar_bids |= 1u << bid;
              }
          }
          for (int l = 0; l < Nz; ++l)
            for (int j = 0; j < N; ++j)
              for (int i = 0; i < N; ++i)
                {
                  const int idx[3] = {i, j, l};
                  if (idx[a] != (side ? n : 0))
                    continue;
                  const uint32_t id = lattice_node[i + N * (j + N * l)];
                  bids[id] |= 1u << bid;
                  if (nax >= 0)
                    {
                      if (axis_bid[nax].size() <= id)
                        axis_bid[nax].resize((size_t)id + 1, 0u);
                      axis_bid[nax][id] |= 1u << bid;
                    }
                }
        }
    }
  m->coords   = std::move(coords);
  m->node_bid = std::move(bids);
  m->n_nodes  = (int64_t)m->node_bid.size();
  for (int d = 0; d < 3; ++d)
    {
      axis_bid[d].resize((size_t)m->n_nodes, 0u);
      m->node_axis_bid[d] = std::move(axis_bid[d]);
    }
  return m;
}

void
sort_coarse_cells(CoarseMesh &cm)
{
  const int                        nv = 1 << cm.dim;
  std::vector<std::pair<P3, int>> key;
  for (size_t c = 0; c < cm.cells.size(); ++c)
    {
      P3 ctr = {0, 0, 0};
      for (int k = 0; k < nv; ++k)
        ctr = add(ctr, cm.vertices[cm.cells[c][k]]);
      ctr = scale(ctr, 1.0 / nv);
      // quantize so that cells in one column sort deterministically
      for (auto &x : ctr)
        x = std::round(x * 1e9) / 1e9;
      key.push_back({ctr, (int)c});
    }
  std::sort(key.begin(), key.end());
  std::vector<std::array<int, 8>> cells;
  for (auto &k : key)
    cells.push_back(cm.cells[k.second]);
  cm.cells = cells;
}

} // namespace

extern "C" {

const char *
gls_mesh_last_error(void)
{
  return g_err.c_str();
}

int
gls_mesh_cylinder(int dim, int degree, int n_ref, double length, double height,
                  double pos, double D, double shift, glsMesh **out)
{
  try
    {
      if (!out || (dim != 2 && dim != 3) || degree < 1 || degree > 2 ||
          n_ref < 0 || n_ref > 6)
        throw std::runtime_error("gls_mesh_cylinder: invalid arguments");
      const auto quads = cylinder_2d_quads(length, height, pos, D, shift, dim == 3);
      CoarseMesh cm;
      cm.dim = dim;
      std::vector<std::array<int, 4>> q2;
      for (const auto &q : quads)
        {
          std::array<int, 4> ids;
          for (int k = 0; k < 4; ++k)
            ids[k] = find_or_add_vertex(cm.vertices, q[k]);
          q2.push_back(ids);
        }
      if (dim == 2)
        {
          for (const auto &q : q2)
            cm.cells.push_back({q[0], q[1], q[2], q[3], 0, 0, 0, 0});
        }
      else
        {
          // extrude_triangulation(tria1, 5 slices, height) then shift -H/2
          const int           nslice = 5;
          const size_t        nv2    = cm.vertices.size();
          std::vector<P3>     v3;
          for (int s = 0; s < nslice; ++s)
            for (size_t v = 0; v < nv2; ++v)
              v3.push_back({cm.vertices[v][0], cm.vertices[v][1],
                            height * s / (nslice - 1) - height / 2.});
          cm.vertices = v3;
          for (int s = 0; s + 1 < nslice; ++s)
            for (const auto &q : q2)
              {
                std::array<int, 8> c;
                for (int k = 0; k < 4; ++k)
                  {
                    c[k]     = q[k] + (int)(s * nv2);
                    c[4 + k] = q[k] + (int)((s + 1) * nv2);
                  }
                cm.cells.push_back(c);
              }
        }
      sort_coarse_cells(cm);
      compute_face_bids(cm, length, height, pos, shift, true);
      CurvedSurface cs;
      cs.active = true;
      cs.radius = D / 2.;
      glsMesh_ *m = build_fine(cm, degree, n_ref, cs);
      m->slip_axis[3] = 1;
      m->slip_axis[4] = 1;
      if (dim == 3)
        {
          m->slip_axis[5] = 2;
          m->slip_axis[6] = 2;
        }
      m->params = {0, (double)dim, (double)degree, length, height, pos, D, shift};
      *out      = m;
      return 0;
    }
  catch (const std::exception &e)
    {
      g_err = e.what();
      return 1;
    }
}

int
gls_mesh_hypercube(int dim, int degree, int n_ref, glsMesh **out)
{
  try
    {
      if (!out || (dim != 2 && dim != 3) || degree < 1 || degree > 3 ||
          n_ref < 0 || n_ref > 8)
        throw std::runtime_error("gls_mesh_hypercube: invalid arguments");
      CoarseMesh cm;
      cm.dim = dim;
      for (int k = 0; k < (1 << dim); ++k)
        cm.vertices.push_back({(double)(k & 1), (double)((k >> 1) & 1),
                               dim == 3 ? (double)((k >> 2) & 1) : 0.0});
      cm.cells.push_back({0, 1, 2, 3, dim == 3 ? 4 : 0, dim == 3 ? 5 : 0,
                          dim == 3 ? 6 : 0, dim == 3 ? 7 : 0});
      compute_face_bids(cm, 0, 0, 0, 0, false);
      CurvedSurface cs; // inactive
      glsMesh_     *m = build_fine(cm, degree, n_ref, cs);
      m->params       = {1, (double)dim, (double)degree};
      *out            = m;
      return 0;
    }
  catch (const std::exception &e)
    {
      g_err = e.what();
      return 1;
    }
}

int
gls_mesh_from_coarse(int dim, int degree, int n_ref, int64_t n_vertices, const double *vertices,
                     int64_t n_cells, const int32_t *cells, int64_t n_bfaces,
                     const int32_t *bface_vertices, const int32_t *bface_ids, glsMesh **out)
{
  try
    {
      if (!out || (dim != 2 && dim != 3) || degree < 1 || degree > 2 || n_ref < 0 ||
          n_ref > 8 || n_vertices <= 0 || n_cells <= 0 || !vertices || !cells ||
          (n_bfaces > 0 && (!bface_vertices || !bface_ids)))
        throw std::runtime_error("gls_mesh_from_coarse: invalid arguments");
      const int nv = 1 << dim, nvf = nv / 2;
      CoarseMesh cm;
      cm.dim = dim;
      for (int64_t v = 0; v < n_vertices; ++v)
        cm.vertices.push_back({vertices[v * dim], vertices[v * dim + 1],
                               dim == 3 ? vertices[v * dim + 2] : 0.0});
      for (int64_t c = 0; c < n_cells; ++c)
        {
          std::array<int, 8> cv{};
          for (int k = 0; k < nv; ++k)
            {
              const int32_t v = cells[c * nv + k];
              if (v < 0 || v >= n_vertices)
                throw std::runtime_error("gls_mesh_from_coarse: vertex index out of range");
              cv[k] = v;
            }
          cm.cells.push_back(cv);
        }
      // x-ordered coarse cells (contiguous slabs for the partitioner)
      sort_coarse_cells(cm);
      // GridIn::read_msh: a boundary face takes the physical tag of the
      // boundary element on it, 0 when there is none
      std::map<std::vector<int>, int> tagged;
      for (int64_t f = 0; f < n_bfaces; ++f)
        {
          std::vector<int> key(bface_vertices + f * nvf, bface_vertices + (f + 1) * nvf);
          std::sort(key.begin(), key.end());
          if (bface_ids[f] < 0 || bface_ids[f] > 31)
            throw std::runtime_error("gls_mesh_from_coarse: boundary id outside 0..31");
          tagged[key] = bface_ids[f];
        }
      compute_face_bids(cm, 0, 0, 0, 0, false);
      for (size_t c = 0; c < cm.cells.size(); ++c)
        for (int f = 0; f < 2 * dim; ++f)
          if (cm.face_bid[c][f] >= 0)
            {
              std::vector<int> key;
              for (int k = 0; k < nv; ++k)
                if (((k >> (f / 2)) & 1) == f % 2)
                  key.push_back(cm.cells[c][k]);
              std::sort(key.begin(), key.end());
              auto it             = tagged.find(key);
              cm.face_bid[c][f] = it == tagged.end() ? 0 : it->second;
            }
      CurvedSurface cs; // flat refinement (see gls_mesh.h)
      glsMesh_     *m = build_fine(cm, degree, n_ref, cs);
      m->params       = {2, (double)dim, (double)degree};
      *out            = m;
      return 0;
    }
  catch (const std::exception &e)
    {
      g_err = e.what();
      return 1;
    }
}

void
gls_mesh_destroy(glsMesh *m)
{
  delete m;
}

int
gls_mesh_dim(const glsMesh *m)
{
  return m->dim;
}
int
gls_mesh_degree(const glsMesh *m)
{
  return m->degree;
}
int64_t
gls_mesh_n_cells(const glsMesh *m)
{
  return m->n_cells;
}
int64_t
gls_mesh_n_nodes(const glsMesh *m)
{
  return m->n_nodes;
}
int64_t
gls_mesh_n_coarse_cells(const glsMesh *m)
{
  return m->n_coarse;
}
const uint32_t *
gls_mesh_cell_nodes(const glsMesh *m)
{
  return m->cell_nodes.data();
}
const double *
gls_mesh_node_coords(const glsMesh *m)
{
  return m->coords.data();
}
const uint32_t *
gls_mesh_node_boundary(const glsMesh *m)
{
  return m->node_bid.data();
}
const int32_t *
gls_mesh_cell_coarse(const glsMesh *m)
{
  return m->cell_coarse.data();
}

int
gls_mesh_constraint_mask(const glsMesh *m, uint32_t vel_ids, uint32_t p_ids,
                         uint32_t slip_ids, uint8_t *out)
{
  if (!m || !out)
    {
      g_err = "gls_mesh_constraint_mask: null argument";
      return 1;
    }
  const int dim = m->dim;
  // ids listed in the descriptor but absent from the mesh constrain nothing
  // (simulation.cc:407-414 lists walls 3 .. 3+2*dim-1 in every dimension)
  uint32_t present = 0;
  for (int64_t i = 0; i < m->n_nodes; ++i)
    present |= m->node_bid[i];
  slip_ids &= present;
  for (int b = 0; b < 32; ++b)
    if (((slip_ids >> b) & 1) && ((m->nonplanar_bids >> b) & 1))
      {
        g_err = "gls_mesh_constraint_mask: slip boundary id " +
                std::to_string(b) +
                " is not an axis-aligned planar wall (general no-normal-flux "
                "constraints are not pure Dirichlet)";
        return 2;
      }
  const uint8_t vel_bits = (uint8_t)((1u << dim) - 1);
  for (int64_t i = 0; i < m->n_nodes; ++i)
    {
      const uint32_t b    = m->node_bid[i];
      uint8_t        mask = 0;
      if (b & vel_ids)
        mask |= vel_bits;
      if (b & p_ids)
        mask |= (uint8_t)(1u << dim);
      // compute_no_normal_flux_constraints on flat axis-aligned walls: the
      // normal component of every wall face touching the node (both at an
      // edge where two walls meet)
      if (b & slip_ids)
        for (int d = 0; d < dim; ++d)
          if (m->node_axis_bid[d][i] & slip_ids)
            mask |= (uint8_t)(1u << d);
      out[i] = mask;
    }
  return 0;
}

int
gls_mesh_brick(const glsMesh *m, int *dims)
{
  if (!m || !dims)
    {
      g_err = "gls_mesh_brick: null argument";
      return 1;
    }
  brick_dims(1 << m->n_ref, m->dim, dims);
  return 0;
}

int
gls_mesh_child_lattice(const glsMesh *coarse, const glsMesh *fine,
                       uint32_t *out)
{
  if (!coarse || !fine || !out || coarse->dim != fine->dim ||
      coarse->degree != fine->degree || fine->n_ref != coarse->n_ref + 1 ||
      coarse->n_coarse != fine->n_coarse || coarse->params != fine->params)
    {
      g_err = "gls_mesh_child_lattice: meshes are not consecutive levels of "
              "the same generator";
      return 1;
    }
  const int     dim   = coarse->dim;
  const int     k     = coarse->degree;
  const int     kp    = k + 1;
  const int     L     = 2 * k + 1;
  const int     nloc  = dim == 3 ? kp * kp * kp : kp * kp;
  const int     nsc   = 1 << coarse->n_ref;
  const int     nsf   = 2 * nsc;
  const int64_t cpcC  = dim == 3 ? (int64_t)nsc * nsc * nsc : (int64_t)nsc * nsc;
  const int64_t cpcF  = dim == 3 ? (int64_t)nsf * nsf * nsf : (int64_t)nsf * nsf;
  const int     Lz    = dim == 3 ? L : 1;
  const int     nlat  = L * L * Lz;
  for (int64_t cell = 0; cell < coarse->n_cells; ++cell)
    {
      const int64_t c = cell / cpcC;
      int           cx, cy, cz;
      local_cell_coords(cell % cpcC, nsc, dim, cx, cy, cz);
      for (int l = 0; l < Lz; ++l)
        for (int j = 0; j < L; ++j)
          for (int i = 0; i < L; ++i)
            {
              const int ai = std::min(i / k, 1), aj = std::min(j / k, 1),
                        al = dim == 3 ? std::min(l / k, 1) : 0;
              const int64_t fcell =
                c * cpcF + local_cell_index(2 * cx + ai, 2 * cy + aj,
                                            dim == 3 ? 2 * cz + al : 0, nsf, dim);
              const int li = i - ai * k, lj = j - aj * k, ll = dim == 3 ? l - al * k : 0;
              const int q  = li + kp * (lj + kp * ll);
              out[cell * nlat + i + L * (j + L * l)] =
                fine->cell_nodes[(size_t)fcell * nloc + q];
            }
    }
  return 0;
}

int
gls_mesh_cell_measure(const glsMesh *m, double *measure_out,
                      double *min_vertex_distance_out)
{
  if (!m)
    {
      g_err = "gls_mesh_cell_measure: null mesh";
      return 1;
    }
  const int dim  = m->dim;
  const int k    = m->degree;
  const int kp   = k + 1;
  const int nloc = dim == 3 ? kp * kp * kp : kp * kp;
  const int nv   = 1 << dim;
  const double g[2] = {0.5 - 0.5 / std::sqrt(3.0), 0.5 + 0.5 / std::sqrt(3.0)};
  for (int64_t c = 0; c < m->n_cells; ++c)
    {
      double X[8][3] = {};
      for (int v = 0; v < nv; ++v)
        {
          const int i = (v & 1) * k, j = ((v >> 1) & 1) * k,
                    l = dim == 3 ? ((v >> 2) & 1) * k : 0;
          const uint32_t node = m->cell_nodes[(size_t)c * nloc + i + kp * (j + kp * l)];
          for (int d = 0; d < dim; ++d)
            X[v][d] = m->coords[(size_t)node * dim + d];
        }
      if (measure_out)
        {
          // exact integral of det J of the multilinear map (2-point Gauss)
          double vol = 0;
          const int nqz = dim == 3 ? 2 : 1;
          for (int qz = 0; qz < nqz; ++qz)
            for (int qy = 0; qy < 2; ++qy)
              for (int qx = 0; qx < 2; ++qx)
                {
                  const double s[3] = {g[qx], g[qy], dim == 3 ? g[qz] : 0};
                  double       J[3][3] = {};
                  for (int v = 0; v < nv; ++v)
                    for (int a = 0; a < dim; ++a)
                      {
                        double dphi = 1;
                        for (int b = 0; b < dim; ++b)
                          {
                            const int bit = (v >> b) & 1;
                            if (b == a)
                              dphi *= bit ? 1.0 : -1.0;
                            else
                              dphi *= bit ? s[b] : 1 - s[b];
                          }
                        for (int d = 0; d < dim; ++d)
                          J[d][a] += X[v][d] * dphi;
                      }
                  double det;
                  if (dim == 2)
                    det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
                  else
                    det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                          J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                          J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
                  vol += det * (dim == 3 ? 0.125 : 0.25);
                }
          measure_out[c] = vol;
        }
      if (min_vertex_distance_out)
        {
          double dmin = 1e300;
          for (int a = 0; a < nv; ++a)
            for (int b = a + 1; b < nv; ++b)
              {
                double s = 0;
                for (int d = 0; d < dim; ++d)
                  s += (X[a][d] - X[b][d]) * (X[a][d] - X[b][d]);
                dmin = std::min(dmin, std::sqrt(s));
              }
          min_vertex_distance_out[c] = dmin;
        }
    }
  return 0;
}

} // extern "C"
