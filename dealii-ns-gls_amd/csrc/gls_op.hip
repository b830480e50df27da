// gls_op.hip — host side of the C-ABI (include/gls_op.h): operator setup
// (MatrixFree-style compressed geometry, packed cell→node indices with the
// constrained-component bits, per-q tables), and the launch functions for the
// vmult / residual / diagonal / table-producer kernels of kernels.h.
#include "../../include/gls_op.h"
#include "brick.h"
#include "common.h"
#include "trace.h"
#include "kernels.h"
#include "op_internal.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

using namespace gls;

namespace gls
{
thread_local std::string g_err;

void
set_error(const std::string &s)
{
  g_err = s;
}

// ------------------------------------------------------------ 1D basis (host)
Basis1D::Basis1D(int k)
{
  n = k + 1;
  if (k == 1)
    nodes = {0.0, 1.0};
  else if (k == 2)
    nodes = {0.0, 0.5, 1.0};
  else if (k == 3)
    nodes = {0.0, 0.5 - std::sqrt(5.0) / 10.0, 0.5 + std::sqrt(5.0) / 10.0, 1.0};
  else
    throw std::runtime_error("degree > 3 not supported");
  // Gauss-Legendre on [0,1]
  qp.resize(n);
  qw.resize(n);
  for (int i = 0; i < n; ++i)
    {
      double z = std::cos(M_PI * (i + 0.75) / (n + 0.5)), pp = 0;
      for (int it = 0; it < 100; ++it)
        {
          double p1 = 1, p2 = 0;
          for (int j = 1; j <= n; ++j)
            {
              const double p3 = p2;
              p2              = p1;
              p1              = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
            }
          pp              = n * (z * p1 - p2) / (z * z - 1.0);
          const double z1 = z;
          z               = z1 - p1 / pp;
          if (std::abs(z - z1) < 1e-16)
            break;
        }
      qp[n - 1 - i] = 0.5 * (1.0 + z);
      qw[n - 1 - i] = 1.0 / ((1.0 - z * z) * pp * pp);
    }
  auto lagrange = [](const std::vector<double> &x, int i, double t, double &val, double &der) {
    const int m = (int)x.size();
    val = 1, der = 0;
    for (int j = 0; j < m; ++j)
      if (j != i)
        {
          double prod = 1.0 / (x[i] - x[j]);
          for (int l = 0; l < m; ++l)
            if (l != i && l != j)
              prod *= (t - x[l]) / (x[i] - x[l]);
          der += prod;
          val *= (t - x[j]) / (x[i] - x[j]);
        }
  };
  S.assign(n * n, 0);
  D.assign(n * n, 0);
  Dq.assign(n * n, 0);
  for (int q = 0; q < n; ++q)
    for (int i = 0; i < n; ++i)
      {
        double v, d;
        lagrange(nodes, i, qp[q], v, d);
        S[q * n + i] = v;
        D[q * n + i] = d;
        lagrange(qp, i, qp[q], v, d);
        Dq[q * n + i] = d;
      }
}

} // namespace gls

// operator state: struct glsOp_ in op_internal.h

namespace
{
template <typename T>
void
upload(void **dptr, const std::vector<T> &h)
{
  HIP_THROW(hipMalloc(dptr, std::max<size_t>(1, h.size() * sizeof(T))));
  if (!h.empty())
    HIP_THROW(hipMemcpy(*dptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
}

template <typename T>
std::vector<T>
convert(const std::vector<double> &v)
{
  return std::vector<T>(v.begin(), v.end());
}

// host twin of gls::qindex (kernels.h): [plane][cell][line] position of q
// point p of `cell`
int64_t
host_qindex(int dim, int n, int64_t cell, int p, int64_t ncell)
{
  const int lpc = dim == 3 ? n * n : n;
  return ((int64_t)(p / lpc) * ncell + cell) * lpc + (p % lpc);
}

// compute units of the operator's device (not the caller's current one):
// the brick layout, and with it the summation order, follows the device the
// operator lives on
int
op_cu_count(const glsOp_ *op)
{
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, op->device) !=
      hipSuccess)
    return 0;
  return n_cu;
}

// Brick decomposition: node lattice per brick, exclusive vs shared nodes,
// partial slots and the CSR that k_shared_reduce walks.
void
build_bricks(glsOp_ *op, const glsOpDesc *d, const char *cell_curved)
{
  const int dim = op->dim, k = op->degree, n = k + 1;
  const int bx = d->brick[0], by = d->brick[1];
  int       bz = dim == 3 ? d->brick[2] : 1;
  if (bx <= 0 || by <= 0 || bz <= 0)
    return;
  // 3D: run the bricks as their one-cell-thick z layers (each layer of a
  // lexicographic brick is a contiguous cell range): twice the workgroups
  // for the same cells evens out the per-CU load (800 4x4x2 bricks on 256
  // CUs leave a 32-brick second round) and the padded LDS lattice of a
  // 4x4x1 layer keeps 3 workgroups per CU (measured 59.6 -> 53.7 us before
  // the LDS re-layout)
  // Small bricks (bx by <= 4: the r1 level of a 2x2x2-refined coarse mesh)
  // keep up to 8 cells (bz layers) per brick: one round of the workgroup's
  // 4 waves x 2 cells instead of a 4-cell layer with two idle waves
  // 3D Q2 operators with many bricks: 4x4x2 bricks, 32 cells and 4 rounds
  // per workgroup (fewer shared nodes per cell, half the partial slots; the
  // relaxation operands read at the write-out), run by the 4-wave FP32 /
  // 3-wave FP64 two-layer kernels.  Against the one-layer kernels (5 waves
  // FP32, 4 FP64 since round 5) they pay only on long launches: from 8
  // generations of the one-layer kernel's slots on (two-layer bricks >= 8 x
  // its workgroups per CU x CUs) -- the sphere r3 (16,384 two-layer bricks)
  // 560 -> 530 us FP32, 918 -> 867 us FP64; below it the one-layer bricks
  // win (Re3900 r3, 6,400: FP32 172 -> 167 us, FP64 288-294 -> 287.5 us; r2
  // 26.8 -> 29.2 us FP32 with two layers) (profiles/r05/explore/
  // ab_two_layer_r3.txt, ab_two_layer_r2.txt).  GLS_TWO_LAYER=0 / 1 forces
  // them off / on.
  bool two_layer = dim == 3 && k == 2 && bx * by == 16 && bz % 2 == 0;
  if (two_layer)
    {
      const int64_t nb2 = d->n_cells / (2 * bx * by);
      const int     wgs = op->prec == GLS_F32 ? 5 : 4; // one-layer workgroups per CU
      const int     n_cu = op_cu_count(op);
      two_layer = n_cu > 0 && nb2 >= 8 * wgs * (int64_t)n_cu;
      if (const char *tl = getenv("GLS_TWO_LAYER"))
        two_layer = tl[0] == '1';
    }
  if (dim == 3)
    {
      int z = 1;
      while (bx * by * z * 2 <= 8 && bz % (z * 2) == 0)
        z *= 2;
      bz = two_layer ? 2 : z;
    }
  const int64_t cpb = (int64_t)bx * by * bz;
  if (d->n_cells % cpb != 0)
    throw std::runtime_error("gls_op_create: n_cells is not a multiple of the brick size");
  const int Lx = k * bx + 1, Ly = k * by + 1, Lz = dim == 3 ? k * bz + 1 : 1;
  const int L  = Lx * Ly * Lz;
  const int side_max = k * (dim == 3 ? 4 : 8) + 1;
  const int zl       = two_layer ? 2 : 1;
  const int lmax     = dim == 3 ? side_max * side_max * (zl * k + 1) : side_max * side_max;
  if (L > lmax || lmax > 729 || (dim == 3 && (bx > 4 || by > 4 || bx * by * bz > 16 * zl)) ||
      (dim == 2 && (bx > 8 || by > 8)))
    return; // lattice does not fit the brick kernel's LDS: per-cell path
  const int64_t nb_full = d->n_cells / cpb;
  const int     nq      = op->nq;
  // Work units: full bricks in mesh order, then the last n_split bricks
  // split into halves along y (bx x by/2 cells, the lattice's upper rows
  // unused).  Workgroups are dispatched in unit order, so the smaller units
  // fill the last dispatch wave and shorten the tail (LPT order).
  // Default: when the bricks leave a small last dispatch wave (fewer than a
  // quarter of the resident slots, 3 workgroups per CU), split twice that
  // many trailing bricks (Re3900 r2: 1,600 bricks on 768 slots -> 128 split,
  // measured 46.3 -> 45.1 us; splitting 0/256/512 was slower).
  int64_t n_split = 0;
  {
    const int n_cu = op_cu_count(op);
    if (n_cu > 0)
      {
        const int64_t slots = 3 * (int64_t)n_cu;
        const int64_t rem   = nb_full % slots;
        if (nb_full > slots && rem > 0 && rem < slots / 4)
          n_split = 2 * rem;
      }
  }
  if (two_layer)
    n_split = 0; // (one dispatch generation: no tail to split)
  if (by % 2 != 0)
    n_split = 0;
  n_split = std::max<int64_t>(0, std::min(n_split, nb_full));
  const int64_t nb = nb_full + n_split;
  // brick order: bricks that read no ghost node first, then the ones that
  // do, so a partitioned vmult runs the former while the ghost import is in
  // flight (deal.II's overlap of update_ghost_values with interior cells)
  std::vector<int64_t> order;
  order.reserve((size_t)nb_full);
  std::vector<char> ghosted((size_t)nb_full, 0);
  for (int64_t b = 0; b < nb_full; ++b)
    for (int64_t j = 0; j < cpb * nq && !ghosted[b]; ++j)
      ghosted[b] = d->cell_nodes[b * cpb * nq + j] >= (uint64_t)d->n_owned_nodes;
  for (int pass = 0; pass < 2; ++pass)
    for (int64_t b = 0; b < nb_full; ++b)
      if (ghosted[b] == pass)
        order.push_back(b);
  int64_t n_interior = 0;
  while (n_interior < nb_full - n_split && !ghosted[order[n_interior]])
    ++n_interior;

  // XCD-aware launch order: workgroup i of a launch is dispatched to XCD
  // i % 8, each XCD with its own L2.  Consecutive bricks of the mesh order
  // (the z layers of one refined coarse cell) share a lattice plane of src
  // nodes, so each XCD gets a contiguous run of bricks: launch slot i holds
  // brick start(i % 8) + i / 8 of the segment (a bijection for any length).
  // Applied to the interior and the boundary segment separately (they are
  // separate launches in the partitioned vmult); the split tail keeps its
  // LPT order.
  {
    const bool remap = true;
    auto        xcd   = [&](int64_t b0, int64_t b1) {
      const int64_t G = b1 - b0, q = G / 8, r = G % 8;
      if (G < 16)
        return;
      std::vector<int64_t> seg(order.begin() + b0, order.begin() + b1);
      for (int64_t i = 0; i < G; ++i)
        {
          const int64_t x = i % 8, j = i / 8;
          order[b0 + i] = seg[x * q + std::min<int64_t>(x, r) + j];
        }
    };
    // curved bricks (per-q geometry: longer lives) spread evenly over the
    // XCD runs of a segment, and first within each run: the generator's
    // order puts all of them (the cells around the cylinder) into one or two
    // XCDs' runs (Re3900 r2: 80 and 48 of 128), whose last bricks then end
    // the launch.  Each run takes a contiguous share of the curved bricks and
    // of the Cartesian ones in mesh order (lattice-plane sharing kept).
    const bool balance = cell_curved != nullptr;
    auto        spread  = [&](int64_t b0, int64_t b1) {
      const int64_t G = b1 - b0, q = G / 8, r = G % 8;
      if (G < 16)
        return;
      std::vector<int64_t> K, C;
      for (int64_t i = b0; i < b1; ++i)
        {
          bool cv = false;
          for (int64_t lc = 0; lc < cpb && !cv; ++lc)
            cv = cell_curved[(size_t)(order[(size_t)i] * cpb + lc)] != 0;
          (cv ? K : C).push_back(order[(size_t)i]);
        }
      if (K.empty() || C.empty())
        return;
      // run x: positions [x q + min(x, r), +q + (x < r)) of the segment (the
      // xcd lambda's split); curved shares as even as the counts allow
      const int64_t nk = (int64_t)K.size();
      size_t        ik = 0, ic = 0;
      int64_t       pos = b0;
      // (curved bricks first in the run measured 1-2 % faster than spread
      // through it or last: profiles/r04/explore/ab_curved_balance.txt)
      for (int x = 0; x < 8; ++x)
        {
          const int64_t len = q + (x < r ? 1 : 0);
          const int64_t kx  = nk * (x + 1) / 8 - nk * x / 8;
          for (int64_t t = 0; t < len; ++t)
            order[(size_t)pos++] = (t < kx && ik < K.size()) || ic >= C.size() ? K[ik++] : C[ic++];
        }
    };
    if (balance)
      {
        spread(0, n_interior);
        spread(n_interior, nb_full - n_split);
      }
    if (remap)
      {
        xcd(0, n_interior);
        xcd(n_interior, nb_full - n_split);
      }
  }
  std::vector<uint32_t> bcell0((size_t)nb), bncell((size_t)nb);
  for (int64_t b = 0; b < nb_full - n_split; ++b)
    bcell0[b] = (uint32_t)(order[b] * cpb), bncell[b] = (uint32_t)cpb;
  for (int64_t h = 0; h < 2 * n_split; ++h)
    {
      const int64_t b = nb_full - n_split + h;
      bcell0[b] = (uint32_t)(order[nb_full - n_split + h / 2] * cpb + (h % 2) * (cpb / 2));
      bncell[b] = (uint32_t)(cpb / 2);
    }
  std::vector<uint32_t> bnodes((size_t)nb * L, UINT32_MAX);
  for (int64_t b = 0; b < nb; ++b)
    for (int64_t lc = 0; lc < (int64_t)bncell[b]; ++lc)
      {
        const int     cx = (int)(lc % bx), cy = (int)((lc / bx) % by), cz = (int)(lc / (bx * by));
        const int64_t cell = bcell0[b] + lc;
        for (int p = 0; p < nq; ++p)
          {
            const int i = p % n, j = (p / n) % n, l = dim == 3 ? p / (n * n) : 0;
            const int li = (cx * k + i) + Lx * ((cy * k + j) + Ly * (cz * k + l));
            const uint32_t node = d->cell_nodes[cell * nq + p];
            uint32_t      &s    = bnodes[(size_t)b * L + li];
            if (s == UINT32_MAX)
              s = node;
            else if (s != node)
              throw std::runtime_error("gls_op_create: cells do not form the declared bricks "
                                       "(shared lattice nodes differ)");
          }
      }
  // brick multiplicity of each node
  std::vector<uint32_t> mult((size_t)d->n_nodes, 0), last((size_t)d->n_nodes, UINT32_MAX);
  for (int64_t b = 0; b < nb; ++b)
    for (int i = 0; i < L; ++i)
      {
        const uint32_t node = bnodes[(size_t)b * L + i];
        if (node == UINT32_MAX)
          continue;
        if (last[node] != (uint32_t)b)
          {
            last[node] = (uint32_t)b;
            mult[node]++;
          }
      }
  // targets: exclusive owned nodes -> node id; every other node is "shared":
  // its per-brick partials occupy a contiguous slot range [off[s], off[s+1])
  // in node order, so k_shared_reduce reads one contiguous run per node.
  // Owned nodes no brick touches get an empty range (identity / zero row).
  std::vector<uint32_t> target((size_t)nb * L);
  std::vector<int64_t>  shared_index((size_t)d->n_nodes, -1);
  std::vector<uint32_t> shared_nodes;
  for (int64_t node = 0; node < d->n_nodes; ++node)
    {
      const bool owned  = node < d->n_owned_nodes;
      const bool shared = mult[node] > 1                 // brick boundary
                          || (!owned && mult[node] > 0)  // ghost partial sums
                          || (owned && mult[node] == 0)  // untouched owned row
                          || (d->node_cmask[node] & 0xF); // identity / zero rows
      if (shared)
        {
          shared_index[node] = (int64_t)shared_nodes.size();
          shared_nodes.push_back((uint32_t)node);
        }
    }
  // order the shared nodes owned rows first, then by brick multiplicity
  // (then node): inside a class of multiplicity m node j's slots start at
  // slot0 + j * m, so k_shared_reduce computes its slot addresses instead of
  // loading them; the ghost rows (a partitioned operator's export block)
  // form a separately launchable tail
  const int64_t n_own_nodes = d->n_owned_nodes;
  std::stable_sort(shared_nodes.begin(), shared_nodes.end(), [&](uint32_t x, uint32_t y) {
    const bool gx = (int64_t)x >= n_own_nodes, gy = (int64_t)y >= n_own_nodes;
    return gx != gy ? gy : mult[x] < mult[y];
  });
  for (size_t s = 0; s < shared_nodes.size(); ++s)
    shared_index[shared_nodes[s]] = (int64_t)s;
  std::vector<uint32_t> off(shared_nodes.size() + 1, 0);
  for (size_t s = 0; s < shared_nodes.size(); ++s)
    off[s + 1] = off[s] + mult[shared_nodes[s]];
  // multiplicity classes of the shared nodes [s0, s1) (first[] relative to
  // s0); n = -1: too many classes (offset-table kernel)
  auto classes = [&](size_t s0, size_t s1) {
    ReduceClasses rc{};
    for (size_t s = s0; s < s1; ++s)
      {
        const uint32_t m = mult[shared_nodes[s]];
        if (rc.n == 0 || rc.mult[rc.n - 1] != m)
          {
            if (rc.n == ReduceClasses::MAX)
              {
                rc.n = -1;
                break;
              }
            rc.first[rc.n] = (uint32_t)(s - s0);
            rc.mult[rc.n]  = m;
            rc.slot0[rc.n] = off[s];
            rc.n++;
          }
      }
    if (rc.n >= 0)
      rc.first[rc.n] = (uint32_t)(s1 - s0);
    return rc;
  };
  size_t n_sh_own = 0;
  while (n_sh_own < shared_nodes.size() && (int64_t)shared_nodes[n_sh_own] < n_own_nodes)
    ++n_sh_own;
  op->n_shared_owned = (int64_t)n_sh_own;
  op->reduce_classes = classes(0, shared_nodes.size());
  op->reduce_owned   = classes(0, n_sh_own);
  op->reduce_ghost   = classes(n_sh_own, shared_nodes.size());
  const uint64_t n_slot_total = off.back();
  if (n_slot_total >= SHARED_BIT)
    throw std::runtime_error("gls_op_create: too many partial slots");
  std::vector<uint32_t> fill(shared_nodes.size(), 0);
  for (int64_t b = 0; b < nb; ++b)
    {
      // a node appears once per brick lattice
      for (int i = 0; i < L; ++i)
        {
          const uint32_t node = bnodes[(size_t)b * L + i];
          if (node == UINT32_MAX) // unused lattice node of a split brick
            {
              target[(size_t)b * L + i] = UNUSED_NODE;
              continue;
            }
          const int64_t s = shared_index[node];
          if (s < 0)
            target[(size_t)b * L + i] = node;
          else
            target[(size_t)b * L + i] = SHARED_BIT | (off[s] + fill[s]++);
        }
    }
  // resident smoothing sweeps (k_brick_sweeps): tagged-granule slot buffers
  // for operators small enough to be resident (FP32 3D Q2 levels of a few
  // thousand bricks of at most SWEEP_MAX_L lattice nodes) whose nodes are
  // shared by at most SWEEP_MAX_MULT bricks
  {
    uint32_t max_mult = 0;
    for (uint32_t node : shared_nodes)
      max_mult = std::max(max_mult, mult[node]);
    if (op->prec == GLS_F32 && dim == 3 && k == 2 && nb <= 4096 && n_slot_total > 0 &&
        L <= SWEEP_MAX_L &&
        max_mult <= (uint32_t)SWEEP_MAX_MULT && n_slot_total * 32 < (1ull << 31))
      {
        for (auto &g : op->d_sweep_gran)
          {
            HIP_THROW(hipMalloc(&g, (size_t)n_slot_total * 32));
            HIP_THROW(hipMemset(g, 0, (size_t)n_slot_total * 32));
          }
        HIP_THROW(hipMalloc(&op->d_sweep_err, sizeof(uint32_t)));
        HIP_THROW(hipMemset(op->d_sweep_err, 0, sizeof(uint32_t)));
        HIP_THROW(hipHostMalloc((void **)&op->h_sweep_flag, sizeof(uint32_t),
                                hipHostMallocMapped | hipHostMallocCoherent));
        *(volatile uint32_t *)op->h_sweep_flag = 0;
        HIP_THROW(hipHostGetDevicePointer((void **)&op->d_sweep_flag, op->h_sweep_flag, 0));
      }
  }
  const uint32_t slot = (uint32_t)n_slot_total;
  // packed node | cmask for the gather and the reduction
  for (auto &v : bnodes)
    v = v == UINT32_MAX ? UNUSED_NODE : v | (uint32_t)(d->node_cmask[v] & 0xF) << 28;
  for (auto &v : shared_nodes)
    v |= (uint32_t)(d->node_cmask[v] & 0xF) << 28;

  op->use_brick = true;
  op->bx = bx, op->by = by, op->bz = bz;
  op->L = L, op->Lx = Lx, op->Ly = Ly;
  op->n_bricks = nb;
  op->n_interior_bricks = n_interior;
  op->n_slots  = slot;
  op->n_shared = (int64_t)shared_nodes.size();
  op->brick_cell0 = bcell0;
  op->brick_ncell  = bncell;
  upload((void **)&op->d_brick_cell0, bcell0);
  upload((void **)&op->d_brick_nodes, bnodes);
  upload((void **)&op->d_brick_target, target);
  upload((void **)&op->d_shared_nodes, shared_nodes);
  upload((void **)&op->d_shared_off, off);
  {
    // node -> its index in the shared-node order (-1: exclusive to one brick),
    // for consumers that rebuild a deferred reduction (mg.hip k_restrict)
    std::vector<int32_t> si((size_t)d->n_nodes);
    for (size_t i = 0; i < si.size(); ++i)
      si[i] = (int32_t)shared_index[i];
    upload((void **)&op->d_shared_index, si);
  }
  HIP_THROW(hipMalloc(&op->d_partial,
                      std::max<size_t>(1, (size_t)slot * (dim + 1) * op->tsize())));
}

// storage field (kernels.h Fields) of canonical host field f: the host
// layout of gls_op_upload_tables / download_tables is delta1, delta2,
// U(dim), gradU(dim^2), gradP(dim), Ut_old(dim)
template <int dim>
int
storage_field_t(int f)
{
  using F = Fields<dim>;
  if (f == 0)
    return F::D1;
  if (f == 1)
    return F::D2;
  f -= 2;
  if (f < dim)
    return F::U + f;
  f -= dim;
  if (f < dim * dim)
    return F::GU + f;
  f -= dim * dim;
  if (f < dim)
    return F::GP + f;
  return F::UT + (f - dim);
}

int
storage_field(const glsOp_ *op, int f)
{
  return op->dim == 3 ? storage_field_t<3>(f) : storage_field_t<2>(f);
}

// host twin of gls::tab_index (kernels.h), f a storage field
size_t
host_tab_index(const glsOp_ *op, int64_t c, int q, int f)
{
  const int W = (int)(16 / op->tsize());
  return (size_t)(op->h_tab_cbase[c] + (int64_t)(f / W) * op->tab_gs + (int64_t)q * W + f % W);
}

// Per-q table layout (kernels.h tab_index): cells are grouped into chunks of
// CPW = 64 / nq cells — with bricks, the cells one wavefront of k_brick runs
// in one round — and a chunk stores its fields in 16-byte groups, lanes
// (cell slot, q) contiguous inside a group.
void
build_table_layout(glsOp_ *op)
{
  const int     W   = (int)(16 / op->tsize());
  const int     NG  = (op->nf_store + W - 1) / W;
  const int     nq  = op->nq;
  const int     CPW = std::max(1, 64 / nq);
  const int64_t gs  = (int64_t)CPW * nq * W;
  op->h_tab_cbase.assign((size_t)op->n_cells, 0);
  int64_t n_chunks = 0;
  if (op->use_brick)
    {
      std::vector<uint32_t> chunk0((size_t)op->n_bricks);
      for (int64_t b = 0; b < op->n_bricks; ++b)
        {
          chunk0[b] = (uint32_t)n_chunks;
          for (uint32_t lc = 0; lc < op->brick_ncell[b]; ++lc)
            op->h_tab_cbase[op->brick_cell0[b] + lc] =
              (n_chunks + lc / CPW) * NG * gs + (int64_t)(lc % CPW) * nq * W;
          n_chunks += (op->brick_ncell[b] + CPW - 1) / CPW;
        }
      upload((void **)&op->d_brick_chunk0, chunk0);
    }
  else
    {
      for (int64_t c = 0; c < op->n_cells; ++c)
        op->h_tab_cbase[c] = (c / CPW) * NG * gs + (c % CPW) * nq * W;
      n_chunks = (op->n_cells + CPW - 1) / CPW;
    }
  op->tab_gs    = gs;
  op->tab_elems = n_chunks * NG * gs;
  upload((void **)&op->d_tab_cbase, op->h_tab_cbase);
}

// geometry of one cell at all q: J[d][a] = dx_d / dxi_a by sum factorisation
void
cell_jacobians(int dim, const Basis1D &b, const double *X /* [nloc][dim] */,
               std::vector<double> &J /* [nq][dim][dim] */)
{
  // b.S / b.D are [q][i] with qp.size() quadrature points and n support
  // points (a mapping basis may differ in degree from the element's)
  const int n = b.n, m = (int)b.qp.size();
  const int nq = dim == 3 ? m * m * m : m * m, nl = dim == 3 ? n * n * n : n * n;
  J.assign((size_t)nq * dim * dim, 0.0);
  for (int q = 0; q < nq; ++q)
    {
      const int qa[3] = {q % m, (q / m) % m, dim == 3 ? q / (m * m) : 0};
      for (int i = 0; i < nl; ++i)
        {
          const int ia[3] = {i % n, (i / n) % n, dim == 3 ? i / (n * n) : 0};
          double    sv[3], dv[3];
          for (int a = 0; a < dim; ++a)
            {
              sv[a] = b.S[qa[a] * n + ia[a]];
              dv[a] = b.D[qa[a] * n + ia[a]];
            }
          for (int a = 0; a < dim; ++a)
            {
              double w = 1;
              for (int bb = 0; bb < dim; ++bb)
                w *= (bb == a) ? dv[bb] : sv[bb];
              if (w == 0.0)
                continue;
              for (int d = 0; d < dim; ++d)
                J[(q * dim + d) * dim + a] += X[i * dim + d] * w;
            }
        }
    }
}

// the Lagrange basis of MappingQ(m) (Gauss-Lobatto support points, as
// Basis1D(m)) and its derivative at the given quadrature points:
// S[q*n+i], D[q*n+i] with n = m + 1 and qp.size() points
Basis1D
mapping_basis(int m, const std::vector<double> &qp)
{
  Basis1D b(m);
  const int n = b.n, nq = (int)qp.size();
  b.qp = qp;
  b.S.assign((size_t)nq * n, 0.0);
  b.D.assign((size_t)nq * n, 0.0);
  for (int q = 0; q < nq; ++q)
    for (int i = 0; i < n; ++i)
      {
        double v = 1, dv = 0;
        for (int j = 0; j < n; ++j)
          if (j != i)
            {
              double prod = 1.0 / (b.nodes[i] - b.nodes[j]);
              for (int l = 0; l < n; ++l)
                if (l != i && l != j)
                  prod *= (qp[q] - b.nodes[l]) / (b.nodes[i] - b.nodes[l]);
              dv += prod;
              v *= (qp[q] - b.nodes[j]) / (b.nodes[i] - b.nodes[j]);
            }
        b.S[(size_t)q * n + i] = v;
        b.D[(size_t)q * n + i] = dv;
      }
  return b;
}

void
invert(int dim, const double *J, double *inv, double &det)
{
  if (dim == 2)
    {
      det    = J[0] * J[3] - J[1] * J[2];
      inv[0] = J[3] / det, inv[1] = -J[1] / det, inv[2] = -J[2] / det, inv[3] = J[0] / det;
    }
  else
    {
      det = J[0] * (J[4] * J[8] - J[5] * J[7]) - J[1] * (J[3] * J[8] - J[5] * J[6]) +
            J[2] * (J[3] * J[7] - J[4] * J[6]);
      inv[0] = (J[4] * J[8] - J[5] * J[7]) / det;
      inv[1] = (J[2] * J[7] - J[1] * J[8]) / det;
      inv[2] = (J[1] * J[5] - J[2] * J[4]) / det;
      inv[3] = (J[5] * J[6] - J[3] * J[8]) / det;
      inv[4] = (J[0] * J[8] - J[2] * J[6]) / det;
      inv[5] = (J[2] * J[3] - J[0] * J[5]) / det;
      inv[6] = (J[3] * J[7] - J[4] * J[6]) / det;
      inv[7] = (J[1] * J[6] - J[0] * J[7]) / det;
      inv[8] = (J[0] * J[4] - J[1] * J[3]) / det;
    }
}

template <typename T, int n>
Shape<T, n>
make_shape(const Basis1D &b)
{
  Shape<T, n> s;
  for (int q = 0; q < n; ++q)
    {
      for (int i = 0; i < n; ++i)
        {
          s.S[q][i]  = (T)b.S[q * n + i];
          s.Dq[q][i] = (T)b.Dq[q * n + i];
        }
      s.w[q] = (T)b.qw[q];
    }
  return s;
}

// ------------------------------------------------------------ dispatch
template <int dim, int k, typename T>
struct Impl
{
  static constexpr int n  = k + 1;
  static constexpr int nq = ipow(n, dim);

  static ApplyArgs<T, dim, n>
  args(const glsOp_ *op)
  {
    ApplyArgs<T, dim, n> a;
    a.nodes         = op->d_nodes;
    a.cell_geo      = op->d_cell_geo;
    a.geo_cart      = (const T *)op->d_geo_cart;
    a.n_cart        = op->n_cart;
    a.geo_gen       = (const T *)op->d_geo_gen;
    a.gen_stride    = op->n_gen * nq;
    a.tab           = (const T *)op->d_tab;
    a.tab_cbase     = op->d_tab_cbase;
    a.tab_gs        = op->tab_gs;
    a.old_stride    = op->n_cells * nq;
    a.cellwise      = (const T *)op->d_cellwise;
    a.n_cells       = op->n_cells;
    a.old_grad      = (const T *)op->d_old_grad;
    a.dst           = nullptr;
    a.src           = nullptr;
    a.cell_begin    = 0;
    a.cell_end      = op->n_cells;
    a.nu            = (T)op->prm.nu;
    a.w0            = (T)op->prm.w0;
    a.theta         = (T)op->prm.theta;
    a.td            = ((op->prm.flags & GLS_CONSIDER_TIME_DERIVATIVE) && op->prm.order > 0) ? 1 : 0;
    a.cw            = (op->prm.flags & GLS_CELL_WISE_STAB) ? 1 : 0;
    a.have_prev     = op->have_prev ? 1 : 0;
    a.have_old_grad = (op->have_old_grad && op->prm.theta != 1.0) ? 1 : 0;
    a.diag_ndof     = nq * (dim + 1);
    a.emat          = nullptr;
    a.sh            = make_shape<T, n>(op->basis);
    return a;
  }

  // element matrices of cells [b, e) into out (device, op precision), one
  // unit-vector cell apply per (cell, local dof) (k_apply<DIAG> with emat)
  static void
  element_matrices(const glsOp_ *op, int mode, void *out, int64_t b, int64_t e, hipStream_t s)
  {
    if (e <= b)
      return;
    auto a       = args(op);
    a.emat       = (T *)out;
    a.cell_begin = b;
    a.cell_end   = e;
    constexpr int CPB = (64 / nq > 0 ? 64 / nq : 1) * (BLOCK / 64);
    const int64_t nv  = (e - b) * (int64_t)nq * (dim + 1);
    const dim3    grid((unsigned)((nv + CPB - 1) / CPB));
    if (mode == MODE_NEWTON)
      hipLaunchKernelGGL((k_apply<dim, k, T, MODE_NEWTON, true>), grid, dim3(BLOCK), 0, s, a);
    else
      hipLaunchKernelGGL((k_apply<dim, k, T, MODE_FIXED, true>), grid, dim3(BLOCK), 0, s, a);
    HIP_THROW(hipGetLastError());
  }

  static void
  apply(const glsOp_ *op, int mode, bool diag, void *dst, const void *src, int64_t b, int64_t e,
        hipStream_t s)
  {
    if (e <= b)
      return;
    auto a       = args(op);
    a.dst        = (T *)dst;
    a.src        = (const T *)src;
    a.cell_begin = b;
    a.cell_end   = e;
    constexpr int CPB = (64 / nq > 0 ? 64 / nq : 1) * (BLOCK / 64);
    const int64_t nv  = (e - b) * (diag ? (int64_t)nq * (dim + 1) : 1);
    const dim3    grid((unsigned)((nv + CPB - 1) / CPB));
#define GLS_LAUNCH(M, DG) hipLaunchKernelGGL((k_apply<dim, k, T, M, DG>), grid, dim3(BLOCK), 0, s, a)
    if (diag)
      {
        if (mode == MODE_NEWTON)
          GLS_LAUNCH(MODE_NEWTON, true);
        else
          GLS_LAUNCH(MODE_FIXED, true);
      }
    else if (mode == MODE_NEWTON)
      GLS_LAUNCH(MODE_NEWTON, false);
    else if (mode == MODE_FIXED)
      GLS_LAUNCH(MODE_FIXED, false);
    else
      GLS_LAUNCH(MODE_RESIDUAL, false);
#undef GLS_LAUNCH
    HIP_THROW(hipGetLastError());
  }

  // the brick kernel over n_units work units of one geometry type, one
  // workgroup per unit
  template <int M, bool DET = false>
  static void
  launch_brick(int64_t n_units, size_t lds, int geo, hipStream_t s, const BrickArgs<T, dim, n> &a)
  {
    if constexpr (!DET)
      if (a.det) // the deterministic accumulation: its own instantiations
        return launch_brick<M, true>(n_units, lds, geo, s, a);
    // two-layer bricks (3D Q2, build_bricks): two lattice chunks per thread
    if constexpr (dim == 3 && k == 2)
      if (a.L > BrickLattice<dim, k, 1>::L)
        {
          if (geo == GEO_GEN)
            hipLaunchKernelGGL((k_brick<dim, k, T, M, GEO_GEN, 2, DET>), dim3((unsigned)n_units),
                               dim3(BLOCK), lds, s, a);
          else if (geo == GEO_CART)
            hipLaunchKernelGGL((k_brick<dim, k, T, M, GEO_CART, 2, DET>), dim3((unsigned)n_units),
                               dim3(BLOCK), lds, s, a);
          else
            hipLaunchKernelGGL((k_brick<dim, k, T, M, GEO_ANY, 2, DET>), dim3((unsigned)n_units),
                               dim3(BLOCK), lds, s, a);
          return;
        }
    if (geo == GEO_GEN)
      hipLaunchKernelGGL((k_brick<dim, k, T, M, GEO_GEN, 1, DET>), dim3((unsigned)n_units),
                         dim3(BLOCK), lds, s, a);
    else if (geo == GEO_CART)
      hipLaunchKernelGGL((k_brick<dim, k, T, M, GEO_CART, 1, DET>), dim3((unsigned)n_units),
                         dim3(BLOCK), lds, s, a);
    else
      hipLaunchKernelGGL((k_brick<dim, k, T, M, GEO_ANY, 1, DET>), dim3((unsigned)n_units),
                         dim3(BLOCK), lds, s, a);
  }

  // the brick kernels' arguments for one apply (dst, src; rx: the fused
  // relaxation / deferred reduction), bricks [0, 0)
  static BrickArgs<T, dim, n>
  brick_args(const glsOp_ *op, int mode, void *dst, const void *src, const RelaxStep *rx)
  {
    BrickArgs<T, dim, n> a;
    a.brick_nodes   = op->d_brick_nodes;
    a.brick_target  = op->d_brick_target;
    a.brick_geo     = op->d_brick_geo;
    a.brick_cell0   = op->d_brick_cell0;
    a.brick_chunk0  = op->d_brick_chunk0;
    a.tab_v         = (const typename Pack<T>::V *)op->d_tab;
    a.geo_cart      = (const T *)op->d_bgeo_cart; // cell-indexed
    a.geo_gen       = (const T *)op->d_bgeo_gen;  // cell-indexed
    a.n_cells       = op->n_cells;
    a.cellwise      = (const T *)op->d_cellwise;
    a.old_grad      = (const T *)op->d_old_grad;
    a.dst           = (T *)dst;
    a.src           = (const T *)src;
    a.partial       = (T *)(rx && rx->partial ? rx->partial : op->d_partial);
    a.rb            = rx ? (const T *)rx->b : nullptr;
    a.rd            = rx ? (const T *)rx->d : nullptr;
    a.romega        = rx ? (T)rx->omega : T(0);
    a.rkeep         = rx ? (rx->keep ? 1 : 0) : 1;
    a.qslots        = rx ? (const T *)rx->prev_partial : nullptr;
    a.qprev         = rx ? (const T *)rx->prev_src : nullptr;
    a.qb            = rx ? (const T *)rx->prev_b : nullptr;
    a.qd            = rx ? (const T *)rx->prev_d : nullptr;
    a.qomega        = rx ? (T)rx->prev_omega : T(0);
    a.qsrc_w        = (T *)src;
    a.out64         = rx ? rx->out64 : nullptr;
    if (a.out64 && (sizeof(T) != 4 || op->reduce_classes.n == 0 || mode == MODE_RESIDUAL))
      throw std::runtime_error("fused FP64 output: FP32 brick operators with class reductions");
    a.rc            = op->reduce_classes;
    if (a.qslots && !(sizeof(T) == 4 && dim == 3 && op->reduce_classes.n > 0))
      throw std::runtime_error("deferred shared-node reduction: FP32 3D brick levels only");
    a.brick_begin   = 0;
    a.brick_end     = 0;
    a.bx            = op->bx;
    a.by            = op->by;
    a.bz            = op->bz;
    a.L             = op->L;
    a.Lx            = op->Lx;
    a.Ly            = op->Ly;
    a.rLx           = 1.0f / (float)op->Lx;
    a.rLxy          = 1.0f / (float)(op->Lx * op->Ly);
    a.rbx           = 1.0f / (float)op->bx;
    a.rbxy          = 1.0f / (float)(op->bx * op->by);
    // LDS lattice strides of 3D Q2 bricks of 4x4 cells in x, y (9 x 9
    // nodes per layer): the widest padding the kernel's LDS budget takes
    // at its occupancy (160 KB / workgroups per CU, one wave per SIMD
    // each): 11 x 12 -- the x-sweep's ds_read_b128 conflict-free and the
    // lattice accumulation's ds_add_f64 at 7 instead of 12 LDS cycles
    // (bank model of MI355X_MICROARCH §LDS, scripts/lds_layout_search.py
    // --lattice) -- else 9 x 11 (the 4-wave FP64 kernels: reads 5 / adds 7
    // cycles, 297 of the 328 lattice positions their 40 KB allow), else
    // unpadded (reads 8 / adds 12)
    auto set_lattice = [&]() {
      const bool four  = mode != MODE_RESIDUAL && dim == 3 && k == 2 &&
                        op->L <= 243; // BrickOcc<...>::four (one-layer bricks)
      const int  waves = four ? BrickOcc<dim, k, T, MODE_NEWTON, GEO_ANY, 1>::waves :
                                BrickOcc<dim, k, T, MODE_RESIDUAL, GEO_ANY, 1>::waves;
      const int  nz    = op->L / (op->Lx * op->Ly);
      const size_t budget = (size_t)160 * 1024 / waves;
      a.PLx = op->Lx, a.PLy = op->Ly;
      if (dim == 3 && k == 2 && op->Lx == 9 && op->Ly == 9)
        {
          // x-line lane map (brick.h xline): each lane reads and adds its own
          // node only; 11 x 9 is the best model cost that fits both budgets
          // (reads 8 / adds 7 cycles, scripts/lds_layout_search.py --xdpp)
          static constexpr int pads_l[2][2] = {{11, 12}, {9, 11}};
          static constexpr int pads_x[2][2] = {{11, 9}, {11, 9}};
          const auto &pads = xdpp<dim, k, T>() ? pads_x : pads_l;
          for (const auto &pl : pads)
            if (BrickLDS<dim, k, T>::bytes(pl[0] * pl[1] * nz) <= budget)
              {
                a.PLx = pl[0], a.PLy = pl[1];
                break;
              }
        }
      a.LP = a.PLx * a.PLy * nz;
    };
    set_lattice();
    a.nu            = (T)op->prm.nu;
    a.w0            = (T)op->prm.w0;
    a.theta         = (T)op->prm.theta;
    a.stau          = (T)(op->prm.dt == 0.0 ? 0.0 : 1.0 / op->prm.dt);
    a.nu4           = T(4) * a.nu;
    a.stau2         = a.stau * a.stau;
    a.td            = ((op->prm.flags & GLS_CONSIDER_TIME_DERIVATIVE) && op->prm.order > 0);
    a.cw            = (op->prm.flags & GLS_CELL_WISE_STAB) ? 1 : 0;
    a.have_prev     = op->have_prev ? 1 : 0;
    a.have_old_grad = (op->have_old_grad && op->prm.theta != 1.0) ? 1 : 0;
    a.det           = (op->prm.flags & GLS_DETERMINISTIC) ? 1 : 0;
    a.sh            = make_shape<T, n>(op->basis);
    return a;
  }

  // T1 (Fields::T1) from the current tables and time weights, before a
  // Newton brick apply
  static void
  ensure_t1(const glsOp_ *op, const BrickArgs<T, dim, n> &a, hipStream_t s)
  {
    if (!op->t1_valid || op->t1_w0 != op->prm.w0 || op->t1_td != a.td)
      {
        const int64_t nqc = op->n_cells * nq;
        if (nqc > 0)
          hipLaunchKernelGGL((k_finalize_t1<dim, T>), dim3((unsigned)((nqc + 255) / 256)),
                             dim3(256), 0, s, (T *)op->d_tab, op->d_tab_cbase, op->tab_gs,
                             op->n_cells, nq, (T)op->prm.w0, a.td);
        HIP_THROW(hipGetLastError());
        op->t1_valid = true;
        op->t1_w0    = op->prm.w0;
        op->t1_td    = a.td;
      }
  }

  static int
  brick_geo(const glsOp_ *op)
  {
    return op->n_curved_bricks == 0            ? GEO_CART :
           op->n_curved_bricks == op->n_bricks ? GEO_GEN :
                                                 GEO_ANY;
  }

  // brick kernel over work units [b0, b1) (what & BRICK_RUN) and the
  // shared-node reduction (what & BRICK_REDUCE); both over all units: dst
  // fully (over)written
  static void
  brick(const glsOp_ *op, int mode, void *dst, const void *src, int64_t b0, int64_t b1,
        int what, hipStream_t s, const RelaxStep *rx)
  {
    if constexpr (BrickLattice<dim, k>::fits)
      {
        BrickArgs<T, dim, n> a = brick_args(op, mode, dst, src, rx);
        if (rx && rx->defer)
          what &= ~BRICK_REDUCE;
#ifdef GLS_EXP_NB
        // timing experiments only (variant builds): the first N bricks
        if (const char *e = getenv("GLS_EXP_NB"))
          b1 = std::min<int64_t>(b1, std::atoll(e));
#endif
        a.brick_begin = b0;
        a.brick_end   = b1;
        if ((what & BRICK_RUN) && b1 > b0 && mode == MODE_NEWTON)
          ensure_t1(op, a, s);
        if ((what & BRICK_RUN) && b1 > b0)
          {
            const int    geo = brick_geo(op);
            const size_t lds = BrickLDS<dim, k, T>::bytes(a.LP);
            if (mode == MODE_NEWTON)
              launch_brick<MODE_NEWTON>(b1 - b0, lds, geo, s, a);
            else if (mode == MODE_FIXED)
              launch_brick<MODE_FIXED>(b1 - b0, lds, geo, s, a);
            else
              launch_brick<MODE_RESIDUAL>(b1 - b0, lds, geo, s, a);
            HIP_THROW(hipGetLastError());
          }
        // the shared-node reduction over all shared nodes, or over the owned
        // / ghost part alone ([owned | ghost] order, build_bricks)
        int64_t              r0 = 0, r1 = 0;
        const ReduceClasses *rcp = &op->reduce_classes;
        if ((what & BRICK_REDUCE) == BRICK_REDUCE)
          r1 = op->n_shared;
        else if (what & BRICK_REDUCE_OWNED)
          r1 = op->n_shared_owned, rcp = &op->reduce_owned;
        else if (what & BRICK_REDUCE_GHOST)
          r0 = op->n_shared_owned, r1 = op->n_shared, rcp = &op->reduce_ghost;
        const int64_t nr = r1 - r0;
        if (nr > 0)
          {
            const dim3 g2((unsigned)((nr * (dim + 1) + 255) / 256));
            // the class kernel runs one thread per 16-byte pack when nc = 4
            const int  npk = (dim + 1) % (16 / (int)sizeof(T)) == 0 ?
                               (dim + 1) / (16 / (int)sizeof(T)) : dim + 1;
            const dim3 g3((unsigned)((nr * npk + 255) / 256));
            const ReduceClasses &rc   = *rcp;
            const uint32_t      *nods = op->d_shared_nodes + r0;
            const uint32_t      *offs = op->d_shared_off + r0;
            if (rc.n > 0 && mode == MODE_RESIDUAL)
              hipLaunchKernelGGL((k_shared_reduce_cls<T, dim + 1, true>), g3, dim3(256), 0, s,
                                 (T *)dst, (const T *)src, (const T *)a.partial, nods, rc,
                                 nr);
            else if (rc.n > 0)
              hipLaunchKernelGGL((k_shared_reduce_cls<T, dim + 1, false>), g3, dim3(256), 0, s,
                                 (T *)dst, (const T *)src, (const T *)a.partial, nods, rc,
                                 nr, a.rb, a.rd, a.romega, a.rkeep,
                                 (uint32_t)op->n_owned_nodes, a.out64);
            else if (mode == MODE_RESIDUAL)
              hipLaunchKernelGGL((k_shared_reduce<T, dim + 1, true>), g2, dim3(256), 0, s,
                                 (T *)dst, (const T *)src, (const T *)a.partial, nods, offs,
                                 nr);
            else
              hipLaunchKernelGGL((k_shared_reduce<T, dim + 1, false>), g2, dim3(256), 0, s,
                                 (T *)dst, (const T *)src, (const T *)a.partial, nods, offs,
                                 nr, a.rb, a.rd, a.romega, a.rkeep,
                                 (uint32_t)op->n_owned_nodes);
            HIP_THROW(hipGetLastError());
          }
      }
    else
      throw std::runtime_error("brick kernel not available for this (dim, degree)");
  }

  // element-matrix diagonal by direct evaluation (k_diag), assembled into
  // diag (zeroed by the caller)
  static void
  diag(const glsOp_ *op, int mode, double *diag_out, hipStream_t s)
  {
    DiagArgs<T, dim, n> da;
    da.a            = args(op);
    da.diag         = diag_out;
    da.a.cell_begin = 0;
    da.a.cell_end   = op->n_cells;
    for (int q = 0; q < n; ++q)
      for (int i = 0; i < n; ++i)
        da.D[q][i] = (T)op->basis.D[q * n + i];
    constexpr int CPB = (64 / nq > 0 ? 64 / nq : 1) * (BLOCK / 64);
    if (op->n_cells == 0)
      return;
    auto launch = [&](const DiagArgs<T, dim, n> &x, int64_t cells) {
      const dim3 grid((unsigned)((cells + CPB - 1) / CPB));
      if (mode == MODE_NEWTON)
        hipLaunchKernelGGL((k_diag<dim, k, T, MODE_NEWTON>), grid, dim3(BLOCK), 0, s, x);
      else
        hipLaunchKernelGGL((k_diag<dim, k, T, MODE_FIXED>), grid, dim3(BLOCK), 0, s, x);
      HIP_THROW(hipGetLastError());
    };
    if (!op_deterministic(op))
      launch(da, op->n_cells);
    else
      {
        // colour by colour: no two cells of a launch add to one node
        op_cell_colours(const_cast<glsOp_ *>(op));
        for (size_t c = 0; c + 1 < op->colour_off.size(); ++c)
          {
            DiagArgs<T, dim, n> x = da;
            x.cells               = op->d_colour_cells + op->colour_off[c];
            x.n_list              = op->colour_off[c + 1] - op->colour_off[c];
            launch(x, x.n_list);
          }
      }
  }

  static void
  produce(const glsOp_ *op, int what, const void *vec, hipStream_t s)
  {
    ProducerArgs<T, dim, n> a;
    a.nodes      = op->d_nodes;
    a.cell_geo   = op->d_cell_geo;
    a.geo_cart   = (const T *)op->d_geo_cart;
    a.n_cart     = op->n_cart;
    a.geo_gen    = (const T *)op->d_geo_gen;
    a.gen_stride = op->n_gen * nq;
    a.tab        = (T *)op->d_tab;
    a.tab_cbase  = op->d_tab_cbase;
    a.tab_gs     = op->tab_gs;
    a.old_stride = op->n_cells * nq;
    a.cellwise   = (T *)op->d_cellwise;
    a.n_cells    = op->n_cells;
    a.old_grad   = (T *)op->d_old_grad;
    a.vec        = (const T *)vec;
    a.h_q        = (const T *)op->d_hq;
    a.h_min      = (const T *)op->d_hmin;
    a.nu         = (T)op->prm.nu;
    a.c1         = (T)op->prm.c1;
    a.c2         = (T)op->prm.c2;
    a.stau       = (T)(op->prm.dt == 0.0 ? 0.0 : 1.0 / op->prm.dt);
    a.what       = what;
    a.sh         = make_shape<T, n>(op->basis);
    constexpr int CPB = BLOCK / nq;
    const dim3    grid((unsigned)((op->n_cells + CPB - 1) / CPB));
    hipLaunchKernelGGL((k_produce<dim, k, T>), grid, dim3(BLOCK), 0, s, a);
    HIP_THROW(hipGetLastError());
  }
};

using ApplyFn   = void (*)(const glsOp_ *, int, bool, void *, const void *, int64_t, int64_t,
                         hipStream_t);
using DiagFn    = void (*)(const glsOp_ *, int, double *, hipStream_t);

template <typename T>
DiagFn
select_diag_t(int dim, int k)
{
#define GLS_CASE(D, K)     \
  if (dim == D && k == K)  \
    return &Impl<D, K, T>::diag;
  GLS_CASE(2, 1)
  GLS_CASE(2, 2)
  GLS_CASE(2, 3)
  GLS_CASE(3, 1)
  GLS_CASE(3, 2)
  GLS_CASE(3, 3)
#undef GLS_CASE
  return nullptr;
}
using ProduceFn = void (*)(const glsOp_ *, int, const void *, hipStream_t);
using EmatFn    = void (*)(const glsOp_ *, int, void *, int64_t, int64_t, hipStream_t);

template <typename T>
EmatFn
select_emat_t(int dim, int k)
{
#define GLS_CASE(D, K)     \
  if (dim == D && k == K)  \
    return &Impl<D, K, T>::element_matrices;
  GLS_CASE(2, 1)
  GLS_CASE(2, 2)
  GLS_CASE(2, 3)
  GLS_CASE(3, 1)
  GLS_CASE(3, 2)
  GLS_CASE(3, 3)
#undef GLS_CASE
  return nullptr;
}

template <typename T>
void
select_t(int dim, int k, ApplyFn &af, ProduceFn &pf)
{
  af = nullptr;
  pf = nullptr;
#define GLS_CASE(D, K)                  \
  if (dim == D && k == K)               \
    {                                   \
      af = &Impl<D, K, T>::apply;       \
      pf = &Impl<D, K, T>::produce;     \
    }
  GLS_CASE(2, 1)
  GLS_CASE(2, 2)
  GLS_CASE(2, 3)
  GLS_CASE(3, 1)
  GLS_CASE(3, 2)
  GLS_CASE(3, 3)
#undef GLS_CASE
}

void
select(const glsOp_ *op, ApplyFn &af, ProduceFn &pf)
{
  if (op->prec == GLS_F64)
    select_t<double>(op->dim, op->degree, af, pf);
  else
    select_t<float>(op->dim, op->degree, af, pf);
  if (!af)
    throw std::runtime_error("no kernel instantiation for this (dim, degree)");
}

using BrickFn = void (*)(const glsOp_ *, int, void *, const void *, int64_t, int64_t, int,
                         hipStream_t, const RelaxStep *);

template <typename T>
BrickFn
select_brick_t(int dim, int k)
{
#define GLS_CASE(D, K)     \
  if (dim == D && k == K)  \
    return &Impl<D, K, T>::brick;
  GLS_CASE(2, 1)
  GLS_CASE(2, 2)
  GLS_CASE(2, 3)
  GLS_CASE(3, 1)
  GLS_CASE(3, 2)
  GLS_CASE(3, 3)
#undef GLS_CASE
  return nullptr;
}

BrickFn
select_brick(const glsOp_ *op)
{
  return op->prec == GLS_F64 ? select_brick_t<double>(op->dim, op->degree) :
                               select_brick_t<float>(op->dim, op->degree);
}

int
vmult_mode(const glsOp_ *op)
{
  return (op->prm.flags & GLS_INCREMENT_FORM) ? MODE_NEWTON : MODE_FIXED;
}

dim3
grid1d(int64_t n)
{
  return dim3((unsigned)((n + 255) / 256));
}

template <typename T>
void
launch_init(const glsOp_ *op, void *dst, const void *src, hipStream_t s)
{
  hipLaunchKernelGGL(k_init_dst<T>, grid1d(op->n_dofs), dim3(256), 0, s, (T *)dst,
                     (const T *)src, op->d_cbits, op->n_owned_dofs, op->n_dofs);
  HIP_THROW(hipGetLastError());
}

void
init_dst(const glsOp_ *op, void *dst, const void *src, hipStream_t s)
{
  if (op->prec == GLS_F64)
    launch_init<double>(op, dst, src, s);
  else
    launch_init<float>(op, dst, src, s);
}

} // namespace

namespace gls
{
void
op_vmult_device(glsOp op, void *dst, const void *src, hipStream_t s)
{
  if (!op->have_lin)
    throw std::runtime_error("vmult before set_linearization_point");
  ApplyFn   af;
  ProduceFn pf;
  select(op, af, pf);
  if (op->use_brick)
    select_brick(op)(op, vmult_mode(op), dst, src, 0, op->n_bricks, BRICK_RUN | BRICK_REDUCE, s,
                     nullptr);
  else
    {
      init_dst(op, dst, src, s);
      af(op, vmult_mode(op), false, dst, src, 0, op->n_cells, s);
    }
  faces_apply(op, false, dst, src, s);
}

// the pieces of vmult dist.hip orchestrates around the ghost exchange
void
brick_launch(const glsOp_ *op, int mode, void *dst, const void *src, int64_t b0, int64_t b1,
             int what, hipStream_t s, const RelaxStep *rx)
{
  BrickFn f = select_brick(op);
  if (!f)
    throw std::runtime_error("no brick kernel for this (dim, degree)");
  f(op, mode, dst, src, b0, b1, what, s, rx);
}

int
op_vmult_mode(const glsOp_ *op)
{
  return vmult_mode(op);
}

bool
sweep_stalled(const glsOp_ *op)
{
  if (!op || !op->h_sweep_flag || op->sweep_reported ||
      *(volatile const uint32_t *)op->h_sweep_flag == 0)
    return false;
  op->sweep_off      = true;
  op->sweep_reported = true;
  return true;
}

bool
brick_sweeps(const glsOp_ *op, int mode, void *v0, void *v1, void *slots0, void *slots1,
             int nsweep, const RelaxStep &rx, hipStream_t s)
{
  using I = Impl<3, 2, float>;
  // after a stall (a brick's neighbour was not resident: kernels of other
  // streams or processes held its CU) one launch per step for good
  if (op->sweep_off || (op->h_sweep_flag && *(volatile const uint32_t *)op->h_sweep_flag))
    {
      op->sweep_off = true;
      return false;
    }
  if (nsweep < 2 || !op->d_sweep_gran[0] || !deferred_reduce_ok(op) || op->degree != 2 ||
      op->L > SWEEP_MAX_L || !rx.b || (mode != MODE_NEWTON && mode != MODE_FIXED))
    return false;
  RelaxStep r     = rx;
  r.partial       = slots0;
  r.prev_partial  = nullptr;
  r.defer         = true;
  auto      a     = I::brick_args(op, mode, v1, v0, &r);
  a.brick_begin   = 0;
  a.brick_end     = op->n_bricks;
  const int    geo = I::brick_geo(op);
  const bool   det = a.det != 0;
  const size_t lds = BrickLDS<3, 2, float>::bytes(a.LP);
  // every brick resident at once (a brick waits for its neighbours)
  int64_t &cap = op->sweep_cap[mode == MODE_NEWTON ? 1 : 0][geo][det ? 1 : 0];
  if (cap < 0)
    cap = sweeps_capacity(mode, geo, det, lds, op->device);
  if (op->n_bricks > cap)
    return false;
  if (mode == MODE_NEWTON)
    I::ensure_t1(op, a, s);
  SweepArgs sw;
  sw.vec[0]     = (float *)v0;
  sw.vec[1]     = (float *)v1;
  sw.slots[0]   = (float *)slots0;
  sw.slots[1]   = (float *)slots1;
  sw.gran[0]    = op->d_sweep_gran[0];
  sw.gran[1]    = op->d_sweep_gran[1];
  sw.gran_bytes = (uint32_t)((uint64_t)op->n_slots * 32u);
  sw.err        = op->d_sweep_err;
  sw.flag       = op->d_sweep_flag;
  sw.epoch      = op->sweep_epoch;
  sw.nsweep     = nsweep;
  sw.spin_max   = op->sweep_spin_max;
  sw.timing     = nullptr;
#if GLS_SWEEP_TIMING
  // timing builds: per-phase clock stamps of every launch appended to the
  // file $GLS_SWEEP_TIMING_OUT (header n_bricks, nsweep; then the stamps)
  static uint64_t *d_tim = nullptr;
  const size_t     nst   = (size_t)op->n_bricks * nsweep * 6;
  if (!d_tim)
    HIP_THROW(hipMalloc(&d_tim, (size_t)4096 * 64 * 6 * sizeof(uint64_t)));
  sw.timing = nst <= (size_t)4096 * 64 * 6 ? d_tim : nullptr;
#endif
  launch_sweeps(a, sw, mode, geo, det, lds, s);
#if GLS_SWEEP_TIMING
  if (const char *fn = getenv("GLS_SWEEP_TIMING_OUT"); fn && sw.timing)
    {
      std::vector<uint64_t> h(nst + 2);
      h[0] = (uint64_t)op->n_bricks, h[1] = (uint64_t)nsweep;
      HIP_THROW(hipStreamSynchronize(s));
      HIP_THROW(hipMemcpy(h.data() + 2, d_tim, nst * sizeof(uint64_t), hipMemcpyDeviceToHost));
      if (FILE *f = fopen(fn, "ab"))
        {
          fwrite(h.data(), sizeof(uint64_t), h.size(), f);
          fclose(f);
        }
    }
#endif
  op->sweep_epoch += (uint32_t)(nsweep - 1);
  op->sweep_launches++;
  return true;
}
} // namespace gls


// ------------------------------------------------------------ caller layout
namespace
{
// op order <- caller order: out[map[i]] = in[i]
template <typename T>
__global__ void
k_permute_in(T *__restrict__ out, const T *__restrict__ in, const int64_t *__restrict__ map,
             int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    out[map[i]] = in[i];
}

// caller order <- op order: out[i] = in[map[i]]
template <typename T>
__global__ void
k_permute_out(T *__restrict__ out, const T *__restrict__ in, const int64_t *__restrict__ map,
              int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    out[i] = in[map[i]];
}

void
permute(bool in_dir, size_t ts, void *out, const void *in, const int64_t *map, int64_t n,
        hipStream_t s)
{
  const dim3 g((unsigned)((n + 255) / 256));
  if (ts == 8)
    {
      if (in_dir)
        hipLaunchKernelGGL(k_permute_in<double>, g, dim3(256), 0, s, (double *)out,
                           (const double *)in, map, n);
      else
        hipLaunchKernelGGL(k_permute_out<double>, g, dim3(256), 0, s, (double *)out,
                           (const double *)in, map, n);
    }
  else
    {
      if (in_dir)
        hipLaunchKernelGGL(k_permute_in<float>, g, dim3(256), 0, s, (float *)out,
                           (const float *)in, map, n);
      else
        hipLaunchKernelGGL(k_permute_out<float>, g, dim3(256), 0, s, (float *)out,
                           (const float *)in, map, n);
    }
  HIP_THROW(hipGetLastError());
}

void *
lazy(void *&p, size_t bytes)
{
  if (!p)
    HIP_THROW(hipMalloc(&p, std::max<size_t>(bytes, 16)));
  return p;
}
} // namespace

namespace gls
{
void
VecStage::release()
{
  for (void *p : {(void *)d_map, raw, in[0], in[1], in[2], in[3], out})
    if (p)
      (void)hipFree(p);
  d_map = nullptr;
  raw = out = nullptr;
  for (auto &p : in)
    p = nullptr;
}

void
VecStage::set(int mem, const int64_t *map, int64_t n_, size_t ts_)
{
  if (mem != GLS_MEM_DEVICE && mem != GLS_MEM_HOST)
    throw std::runtime_error("vector layout: memory must be GLS_MEM_DEVICE or GLS_MEM_HOST");
  if (map)
    {
      std::vector<char> seen((size_t)n_, 0);
      for (int64_t i = 0; i < n_; ++i)
        {
          if (map[i] < 0 || map[i] >= n_ || seen[map[i]])
            throw std::runtime_error("vector layout: dof_map is not a permutation of [0, m)");
          seen[map[i]] = 1;
        }
    }
  HIP_THROW(hipDeviceSynchronize());
  release();
  memory = mem;
  n      = n_;
  ts     = ts_;
  if (map)
    {
      HIP_THROW(hipMalloc((void **)&d_map, std::max<size_t>(16, (size_t)n * sizeof(int64_t))));
      HIP_THROW(hipMemcpy(d_map, map, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice));
    }
}

const void *
VecStage::in_vec(const void *v, int slot, hipStream_t s)
{
  if (!active() || !v)
    return v;
  const size_t bytes = (size_t)n * ts;
  void        *dst   = lazy(in[slot], bytes);
  const void  *from  = v;
  if (memory == GLS_MEM_HOST)
    {
      void *to = d_map ? lazy(raw, bytes) : dst;
      HIP_THROW(hipMemcpyAsync(to, v, bytes, hipMemcpyHostToDevice, s));
      from = to;
    }
  if (d_map)
    permute(true, ts, dst, from, d_map, n, s);
  return dst;
}

void *
VecStage::out_vec(void *v)
{
  if (!active())
    return v;
  return lazy(out, (size_t)n * ts);
}

void
VecStage::finish_out(void *v, hipStream_t s)
{
  if (!active())
    return;
  const size_t bytes = (size_t)n * ts;
  const void  *res   = out;
  if (d_map)
    {
      void *to = memory == GLS_MEM_HOST ? lazy(raw, bytes) : v;
      permute(false, ts, to, out, d_map, n, s);
      res = to;
    }
  if (memory == GLS_MEM_HOST)
    HIP_THROW(hipMemcpyAsync(v, res, bytes, hipMemcpyDeviceToHost, s));
}

void
VecStage::done(hipStream_t s)
{
  if (memory == GLS_MEM_HOST)
    HIP_THROW(hipStreamSynchronize(s));
}
} // namespace gls

// ------------------------------------------------------------ get_max_u
namespace
{
// NavierStokesOperator::get_max_u (operator_ns.cc:530-568): one lane per
// (cell, q point): velocity at x_q from the cell's plain nodal values
// (read_dof_values_plain + evaluate(values)), |u|, block max into part[]
template <int dim, int k, typename T>
__global__ void __launch_bounds__(256)
  k_max_u(const uint32_t *__restrict__ nodes, const T *__restrict__ vec, int64_t n_cells,
          Shape<T, k + 1> sh, double *__restrict__ part)
{
  constexpr int n = k + 1, nq = ipow(n, dim), nc = dim + 1;
  __shared__ double red[4];
  const int64_t     g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double            m = 0;
  if (g < n_cells * nq)
    {
      const int64_t c  = g / nq;
      const int     q  = (int)(g - c * nq);
      const int     qa[3] = {q % n, (q / n) % n, dim == 3 ? q / (n * n) : 0};
      T             u[dim];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        u[d] = 0;
      for (int i = 0; i < nq; ++i)
        {
          const int ia[3] = {i % n, (i / n) % n, dim == 3 ? i / (n * n) : 0};
          T         w     = sh.S[qa[0]][ia[0]] * sh.S[qa[1]][ia[1]];
          if (dim == 3)
            w *= sh.S[qa[2]][ia[2]];
          const size_t node = nodes[c * nq + i] & NODE_MASK;
#pragma unroll
          for (int d = 0; d < dim; ++d)
            u[d] += w * vec[node * nc + d];
        }
      T s2 = 0;
#pragma unroll
      for (int d = 0; d < dim; ++d)
        s2 += u[d] * u[d];
      m = (double)sqrt(s2);
    }
  for (int off = 32; off > 0; off >>= 1)
    m = fmax(m, __shfl_down(m, off));
  if ((threadIdx.x & 63) == 0)
    red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    part[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

__global__ void __launch_bounds__(256)
  k_max_finish(const double *__restrict__ part, int64_t nb, double *__restrict__ out)
{
  __shared__ double red[256];
  double            m = 0;
  for (int64_t b = threadIdx.x; b < nb; b += 256)
    m = fmax(m, part[b]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1)
    {
      if ((int)threadIdx.x < st)
        red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + st]);
      __syncthreads();
    }
  if (threadIdx.x == 0)
    out[0] = red[0];
}

template <int dim, int k, typename T>
double
max_u_t(const glsOp_ *op, const void *vec, hipStream_t s)
{
  constexpr int n = k + 1, nq = ipow(n, dim);
  const int64_t nb   = (op->n_cells * nq + 255) / 256;
  double       *part = nullptr;
  HIP_THROW(hipMallocAsync((void **)&part, (size_t)(nb + 1) * sizeof(double), s));
  if (nb > 0)
    hipLaunchKernelGGL((k_max_u<dim, k, T>), dim3((unsigned)nb), dim3(256), 0, s, op->d_nodes,
                       (const T *)vec, op->n_cells, make_shape<T, n>(op->basis), part);
  hipLaunchKernelGGL(k_max_finish, dim3(1), dim3(256), 0, s, (const double *)part, nb,
                     part + nb);
  HIP_THROW(hipGetLastError());
  double r = 0;
  HIP_THROW(hipMemcpyAsync(&r, part + nb, sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_THROW(hipFreeAsync(part, s));
  HIP_THROW(hipStreamSynchronize(s));
  return r;
}

template <typename T>
double
max_u_p(const glsOp_ *op, const void *vec, hipStream_t s)
{
#define GLS_CASE(D, K)              \
  if (op->dim == D && op->degree == K) \
    return max_u_t<D, K, T>(op, vec, s);
  GLS_CASE(2, 1)
  GLS_CASE(2, 2)
  GLS_CASE(2, 3)
  GLS_CASE(3, 1)
  GLS_CASE(3, 2)
  GLS_CASE(3, 3)
#undef GLS_CASE
  throw std::runtime_error("get_max_u: no instantiation for this (dim, degree)");
}
} // namespace

// ------------------------------------------------------------ C-ABI
extern "C" {

const char *
gls_last_error(void)
{
  return gls::g_err.c_str();
}

glsStatus
gls_op_create(const glsOpDesc *d, glsOp *out)
{
  GLS_TRY
  if (!d || !out)
    throw std::runtime_error("gls_op_create: null argument");
  if ((d->dim != 2 && d->dim != 3) || d->degree < 1 || d->degree > 3 ||
      (d->precision != GLS_F64 && d->precision != GLS_F32) || d->n_cells < 0 || d->n_nodes < 0 ||
      d->n_owned_nodes < 0 || d->n_owned_nodes > d->n_nodes || !d->cell_nodes ||
      !d->node_coords || !d->node_cmask || !d->cell_measure || !d->cell_hmin ||
      (d->mapping_points && (d->mapping_degree < 1 || d->mapping_degree > 3)))
    throw std::runtime_error("gls_op_create: invalid descriptor");
  if (d->mapping_points && d->n_outflow_faces > 0)
    throw std::runtime_error("gls_op_create: outflow faces with mapping_points are not supported");
  if (d->n_nodes >= (int64_t)NODE_MASK)
    throw std::runtime_error("gls_op_create: too many local nodes for 28-bit node indices");
  // an arbitrary cell order (brick[0] < 0, e.g. deal.II's MatrixFree cell
  // order): discover the bricks from the connectivity and run the cells in
  // brick order (brick_discovery.cc); every cell-indexed input is permuted
  // here, vectors are node-indexed and unaffected
  const glsOpDesc      *caller = d;
  glsOpDesc             dd     = *d;
  gls::BrickPlan        plan;
  std::vector<uint32_t> p_nodes;
  std::vector<double>   p_meas, p_hmin, p_map;
  if (d->brick[0] < 0)
    {
      dd.brick[0] = dd.brick[1] = dd.brick[2] = 0;
      for (int64_t i = 0; i < d->n_cells * (int64_t)(d->dim == 3 ? (d->degree + 1) * (d->degree + 1) * (d->degree + 1)
                                                                   : (d->degree + 1) * (d->degree + 1));
           ++i)
        if ((int64_t)d->cell_nodes[i] >= d->n_nodes)
          throw std::runtime_error("gls_op_create: node index out of range");
      if (gls::discover_bricks(d->dim, d->degree, d->n_cells, d->cell_nodes, plan))
        {
          const int nqc = d->dim == 3 ? (d->degree + 1) * (d->degree + 1) * (d->degree + 1)
                                      : (d->degree + 1) * (d->degree + 1);
          p_nodes.resize((size_t)d->n_cells * nqc);
          p_meas.resize((size_t)d->n_cells);
          p_hmin.resize((size_t)d->n_cells);
          for (int64_t c = 0; c < d->n_cells; ++c)
            {
              const int64_t e = plan.perm[(size_t)c];
              std::copy(d->cell_nodes + e * nqc, d->cell_nodes + (e + 1) * nqc,
                        p_nodes.begin() + c * nqc);
              p_meas[c] = d->cell_measure[e];
              p_hmin[c] = d->cell_hmin[e];
            }
          if (d->mapping_points)
            {
              const int nm  = d->mapping_degree + 1;
              const int nmq = (d->dim == 3 ? nm * nm * nm : nm * nm) * d->dim;
              p_map.resize((size_t)d->n_cells * nmq);
              for (int64_t c = 0; c < d->n_cells; ++c)
                {
                  const int64_t e = plan.perm[(size_t)c];
                  std::copy(d->mapping_points + e * nmq, d->mapping_points + (e + 1) * nmq,
                            p_map.begin() + c * nmq);
                }
              dd.mapping_points = p_map.data();
            }
          dd.cell_nodes   = p_nodes.data();
          dd.cell_measure = p_meas.data();
          dd.cell_hmin    = p_hmin.data();
          for (int a = 0; a < 3; ++a)
            dd.brick[a] = plan.shape[a];
        }
    }
  d = &dd;
  auto *op          = new glsOp_();
  // an invalid descriptor found below (bricks, outflow faces, allocation
  // failures) frees what was built so far
  struct CreateGuard
  {
    glsOp_ *p;
    ~CreateGuard()
    {
      if (p)
        gls_op_destroy(p);
    }
  } guard{op};
  if (!p_nodes.empty())
    op->cell_perm = std::move(plan.perm);
  op->dim           = d->dim;
  op->degree        = d->degree;
  op->prec          = d->precision;
  op->n_cells       = d->n_cells;
  op->n_nodes       = d->n_nodes;
  op->n_owned_nodes = d->n_owned_nodes;
  op->n_dofs        = d->n_nodes * (d->dim + 1);
  op->n_owned_dofs  = d->n_owned_nodes * (d->dim + 1);
  op->basis         = Basis1D(d->degree);
  const int dim = d->dim, n = d->degree + 1;
  op->nq            = dim == 3 ? n * n * n : n * n;
  op->nf            = 2 + 3 * dim + dim * dim;
  op->nf_store      = dim == 3 ? Fields<3>::N : Fields<2>::N;
  HIP_THROW(hipGetDevice(&op->device));
  const int nq = op->nq;

  // packed node indices with constrained-component bits (read_dof_values /
  // distribute_local_to_global resolve homogeneous Dirichlet constraints)
  std::vector<uint32_t> nodes((size_t)d->n_cells * nq);
  for (size_t i = 0; i < nodes.size(); ++i)
    {
      const uint32_t nd = d->cell_nodes[i];
      if ((int64_t)nd >= d->n_nodes)
        throw std::runtime_error("gls_op_create: node index out of range");
      nodes[i] = nd | ((uint32_t)(d->node_cmask[nd] & 0xF) << 28);
    }
  upload((void **)&op->d_nodes, nodes);
  op->h_cmask.assign(d->node_cmask, d->node_cmask + d->n_nodes);
  op->h_cell_nodes.assign(caller->cell_nodes, caller->cell_nodes + (size_t)d->n_cells * nq);

  // constrained dof bitmask on the owned range (identity rows)
  std::vector<uint32_t> cbits((size_t)(op->n_owned_dofs + 31) / 32 + 1, 0u);
  for (int64_t nd = 0; nd < d->n_owned_nodes; ++nd)
    for (int c = 0; c <= dim; ++c)
      if ((d->node_cmask[nd] >> c) & 1)
        {
          const int64_t i = nd * (dim + 1) + c;
          cbits[i >> 5] |= 1u << (i & 31);
        }
  upload((void **)&op->d_cbits, cbits);
  upload((void **)&op->d_node_cmask, op->h_cmask);

  // MatrixFree-style geometry: Cartesian cells (constant diagonal J) store
  // dim+1 numbers, all others JxW + J^{-1} per quadrature point
  std::vector<uint32_t> cell_geo((size_t)d->n_cells);
  std::vector<double>   cart, gen; // [field][index] filled below
  std::vector<double>   cart_rows, gen_rows;
  std::vector<double>   X((size_t)nq * dim), J;
  int64_t               n_cart = 0, n_gen = 0;
  // a mapping of its own degree (glsOpDesc.mapping_points): its basis at the
  // element's quadrature points
  Basis1D mb(d->mapping_points ? d->mapping_degree : op->degree);
  if (d->mapping_points)
    mb = mapping_basis(d->mapping_degree, op->basis.qp);
  const int nmq = d->mapping_points ? (dim == 3 ? mb.n * mb.n * mb.n : mb.n * mb.n) : nq;
  for (int64_t c = 0; c < d->n_cells; ++c)
    {
      if (d->mapping_points)
        cell_jacobians(dim, mb, d->mapping_points + (size_t)c * nmq * dim, J);
      else
        {
          for (int i = 0; i < nq; ++i)
            for (int e = 0; e < dim; ++e)
              X[i * dim + e] = d->node_coords[(size_t)d->cell_nodes[c * nq + i] * dim + e];
          cell_jacobians(dim, op->basis, X.data(), J);
        }
      double scale = 0;
      for (int e = 0; e < dim; ++e)
        scale = std::max(scale, std::abs(J[e * dim + e]));
      bool cartesian = true;
      for (int q = 0; q < nq && cartesian; ++q)
        for (int i = 0; i < dim * dim; ++i)
          {
            const double v  = J[q * dim * dim + i];
            const bool   dg = (i / dim) == (i % dim);
            if ((!dg && std::abs(v) > 1e-12 * scale) ||
                std::abs(v - J[i]) > 1e-12 * scale)
              {
                cartesian = false;
                break;
              }
          }
      if (cartesian)
        {
          cell_geo[c] = (uint32_t)n_cart++;
          double det  = 1;
          for (int e = 0; e < dim; ++e)
            {
              cart_rows.push_back(1.0 / J[e * dim + e]);
              det *= J[e * dim + e];
            }
          cart_rows.push_back(det);
        }
      else
        {
          cell_geo[c] = GEO_GENERAL | (uint32_t)n_gen++;
          for (int q = 0; q < nq; ++q)
            {
              double inv[9], det;
              invert(dim, &J[(size_t)q * dim * dim], inv, det);
              const int qa[3] = {q % n, (q / n) % n, dim == 3 ? q / (n * n) : 0};
              double    w     = 1;
              for (int a = 0; a < dim; ++a)
                w *= op->basis.qw[qa[a]];
              gen_rows.push_back(det * w);
              for (int i = 0; i < dim * dim; ++i)
                gen_rows.push_back(inv[i]);
            }
        }
    }
  op->n_cart = n_cart;
  op->n_gen  = n_gen;
  // transpose rows -> SoA [field][index]
  const int ncf = dim + 1, ngf = 1 + dim * dim;
  cart.resize((size_t)ncf * n_cart);
  for (int64_t i = 0; i < n_cart; ++i)
    for (int f = 0; f < ncf; ++f)
      cart[(size_t)f * n_cart + i] = cart_rows[(size_t)i * ncf + f];
  gen.resize((size_t)ngf * n_gen * nq);
  for (int64_t g = 0; g < n_gen; ++g)
    for (int q = 0; q < nq; ++q)
      for (int f = 0; f < ngf; ++f)
        gen[(size_t)f * n_gen * nq + host_qindex(dim, n, g, q, n_gen)] =
          gen_rows[((size_t)g * nq + q) * ngf + f];
  upload((void **)&op->d_cell_geo, cell_geo);
  // per-cell geometry type for the brick order (curved bricks balanced over
  // the XCDs, build_bricks)
  std::vector<char> cell_curved((size_t)d->n_cells);
  for (int64_t c = 0; c < d->n_cells; ++c)
    cell_curved[(size_t)c] = (cell_geo[(size_t)c] & GEO_GENERAL) ? 1 : 0;
  build_bricks(op, d, cell_curved.data());

  std::vector<double> hq((size_t)d->n_cells), hmin((size_t)d->n_cells);
  for (int64_t c = 0; c < d->n_cells; ++c)
    {
      const double hk = d->cell_measure[c];
      hq[c]   = dim == 2 ? std::sqrt(4. * hk / M_PI) / d->degree :
                           std::pow(6 * hk / M_PI, 1. / 3.) / d->degree;
      hmin[c] = d->cell_hmin[c];
    }
  // brick path: the same geometry indexed by CELL ([field][cell] Cartesian,
  // [field][plane][cell][line] curved; only the curved cells' entries of the
  // latter are ever read), so no geometry load waits for a cell_geo load
  // A brick with any curved cell is a curved brick: all its cells get per-q
  // geometry (a Cartesian cell's per-q JxW = det * w_q, J^{-1} = its
  // diagonal: the same numbers the Cartesian path forms), so the geometry
  // type is uniform per workgroup.
  std::vector<double>   bcart, bgen;
  std::vector<uint32_t> bgeo;
  if (op->use_brick)
    {
      const int64_t C = d->n_cells;
      bcart.assign((size_t)ncf * C, 0.0);
      bgen.assign((size_t)ngf * C * nq, 0.0);
      bgeo.assign((size_t)op->n_bricks, 0u);
      std::vector<int64_t> brick_of((size_t)C, -1);
      for (int64_t b = 0; b < op->n_bricks; ++b)
        for (uint32_t lc = 0; lc < op->brick_ncell[b]; ++lc)
          brick_of[op->brick_cell0[b] + lc] = b;
      for (int64_t c = 0; c < C; ++c)
        if (cell_geo[c] & GEO_GENERAL)
          bgeo[brick_of[c]] |= 1u;
      op->n_curved_bricks = 0;
      for (int64_t b = 0; b < op->n_bricks; ++b)
        {
          op->n_curved_bricks += bgeo[b] & 1u;
          bgeo[b] |= op->brick_ncell[b] << 8;
        }
      for (int64_t c = 0; c < C; ++c)
        {
          const uint32_t cg = cell_geo[c];
          if (!(bgeo[brick_of[c]] & 1u))
            {
              for (int f = 0; f < ncf; ++f)
                bcart[(size_t)f * C + c] = cart_rows[(size_t)cg * ncf + f];
              continue;
            }
          for (int q = 0; q < nq; ++q)
            {
              double vals[1 + 9] = {0};
              if (cg & GEO_GENERAL)
                {
                  const int64_t g = cg & ~GEO_GENERAL;
                  for (int f = 0; f < ngf; ++f)
                    vals[f] = gen_rows[((size_t)g * nq + q) * ngf + f];
                }
              else
                {
                  const int qa[3] = {q % n, (q / n) % n, dim == 3 ? q / (n * n) : 0};
                  double    w     = op->basis.qw[qa[0]] * op->basis.qw[qa[1]];
                  if (dim == 3)
                    w *= op->basis.qw[qa[2]];
                  vals[0] = cart_rows[(size_t)cg * ncf + dim] * w;
                  for (int e = 0; e < dim; ++e)
                    vals[1 + e * dim + e] = cart_rows[(size_t)cg * ncf + e];
                }
              for (int f = 0; f < ngf; ++f)
                bgen[(size_t)f * C * nq + host_qindex(dim, n, c, q, C)] = vals[f];
            }
        }
      upload((void **)&op->d_brick_geo, bgeo);
    }
  if (op->prec == GLS_F64)
    {
      if (op->use_brick)
        {
          upload(&op->d_bgeo_cart, bcart);
          upload(&op->d_bgeo_gen, bgen);
        }
      upload(&op->d_geo_cart, cart);
      upload(&op->d_geo_gen, gen);
      upload(&op->d_hq, hq);
      upload(&op->d_hmin, hmin);
    }
  else
    {
      if (op->use_brick)
        {
          upload(&op->d_bgeo_cart, convert<float>(bcart));
          upload(&op->d_bgeo_gen, convert<float>(bgen));
        }
      upload(&op->d_geo_cart, convert<float>(cart));
      upload(&op->d_geo_gen, convert<float>(gen));
      upload(&op->d_hq, convert<float>(hq));
      upload(&op->d_hmin, convert<float>(hmin));
    }
  const size_t ts = op->tsize();
  build_table_layout(op);
  HIP_THROW(hipMalloc(&op->d_tab, std::max<size_t>(1, (size_t)op->tab_elems * ts)));
  HIP_THROW(hipMemset(op->d_tab, 0, std::max<size_t>(1, (size_t)op->tab_elems * ts)));
  HIP_THROW(hipMalloc(&op->d_cellwise, std::max<size_t>(1, 2 * (size_t)d->n_cells * ts)));
  HIP_THROW(hipMemset(op->d_cellwise, 0, std::max<size_t>(1, 2 * (size_t)d->n_cells * ts)));
  HIP_THROW(hipMalloc(&op->d_tmp, std::max<size_t>(1, (size_t)op->n_dofs * ts)));
  op->prm.nu    = 1.0;
  op->prm.theta = 1.0;
  op->prm.dt    = 1.0;
  gls::faces_setup(op, caller);
  guard.p       = nullptr;
  *out          = op;
  GLS_CATCH
}

void
gls_op_destroy(glsOp op)
{
  if (!op)
    return;
  void *bufs[] = {op->d_nodes,        op->d_cell_geo,     op->d_geo_cart,     op->d_geo_gen,
                  op->d_tab,          op->d_cellwise,     op->d_old_grad,     op->d_hq,
                  op->d_hmin,         op->d_tmp,          op->d_cbits,        op->d_brick_nodes,
                  op->d_brick_target, op->d_shared_nodes, op->d_shared_off,
                  op->d_shared_index, op->d_partial,      op->d_bgeo_cart,    op->d_bgeo_gen,
                  op->d_brick_geo,    op->d_brick_cell0,  op->d_brick_chunk0, op->d_tab_cbase,
                  op->d_node_cmask,   op->d_inhom,        op->gmres_ws,
                  op->d_colour_cells, op->d_sweep_gran[0], op->d_sweep_gran[1],
                  op->d_sweep_err};
  for (void *b : bufs)
    if (b)
      (void)hipFree(b);
  if (op->gmres_host)
    (void)hipHostFree(op->gmres_host);
  if (op->h_sweep_flag)
    (void)hipHostFree(op->h_sweep_flag);
  op->stage.release();
  gls::faces_release(op);
  delete op;
}

glsStatus
gls_op_set_parameters(glsOp op, const glsOpParams *prm)
{
  GLS_TRY
  if (!op || !prm)
    throw std::runtime_error("gls_op_set_parameters: null argument");
  // operator_ns.cc:126-129: theta == 1 required with a stabilised time derivative
  const bool td = (prm->flags & GLS_CONSIDER_TIME_DERIVATIVE) && prm->order > 0;
  if (td && prm->theta != 1.0)
    throw std::runtime_error("consider_time_derivative requires theta == 1 "
                             "(operator_ns.cc:126-129)");
  op->prm = *prm;
  op->version++;
  GLS_CATCH
}

int64_t
gls_op_m(glsOp op)
{
  return op ? op->n_dofs : 0;
}

int
gls_op_precision(glsOp op)
{
  return op ? op->prec : -1;
}

glsStatus
gls_op_set_vector_layout(glsOp op, int memory, const int64_t *dof_map)
{
  GLS_TRY
  if (!op)
    throw std::runtime_error("gls_op_set_vector_layout: null operator");
  op->stage.set(memory, dof_map, op->n_dofs, op->tsize());
  GLS_CATCH
}

glsStatus
gls_op_set_linearization_point(glsOp op, const void *vec, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::set_linearization_point", (hipStream_t)stream);
  if (!op || !vec)
    throw std::runtime_error("gls_op_set_linearization_point: null argument");
  ApplyFn     af;
  ProduceFn   pf;
  hipStream_t s = (hipStream_t)stream;
  select(op, af, pf);
  const void *x = op->stage.in_vec(vec, 0, s);
  pf(op, 0, x, s);
  gls::faces_linearization(op, x, s);
  op->stage.done(s);
  op->have_lin = true;
  op->t1_valid = false;
  op->version++;
  GLS_CATCH
}

glsStatus
gls_op_set_previous_solution(glsOp op, const void *const *hist, int n_hist,
                             const double *weights, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::set_previous_solution", (hipStream_t)stream);
  if (!op)
    throw std::runtime_error("gls_op_set_previous_solution: null operator");
  const int order = op->prm.order;
  if (order == 0)
    return 0; // operator_ns.cc:243-244
  if (!hist || !weights || n_hist < order + 1 || order > 3)
    throw std::runtime_error("gls_op_set_previous_solution: need order+1 history vectors");
  ApplyFn     af;
  ProduceFn   pf;
  hipStream_t s = (hipStream_t)stream;
  select(op, af, pf);
  const void *x[4] = {nullptr, nullptr, nullptr, nullptr};
  double      w[4] = {0, 0, 0, 0};
  for (int i = 1; i <= order; ++i)
    {
      if (!hist[i])
        throw std::runtime_error("gls_op_set_previous_solution: null history vector");
      x[i - 1] = op->stage.in_vec(hist[i], i - 1, s);
      w[i - 1] = weights[i];
    }
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL(k_lincomb<double>, grid1d(op->n_dofs), dim3(256), 0, s,
                       (double *)op->d_tmp, (const double *)x[0], (const double *)x[1],
                       (const double *)x[2], (const double *)x[3], w[0], w[1], w[2], w[3],
                       op->n_dofs);
  else
    hipLaunchKernelGGL(k_lincomb<float>, grid1d(op->n_dofs), dim3(256), 0, s,
                       (float *)op->d_tmp, (const float *)x[0], (const float *)x[1],
                       (const float *)x[2], (const float *)x[3], w[0], w[1], w[2], w[3],
                       op->n_dofs);
  HIP_THROW(hipGetLastError());
  pf(op, 1, op->d_tmp, s);
  op->have_prev = true;
  op->t1_valid  = false;
  op->version++;
  if (op->prm.theta != 1.0)
    {
      if (!op->d_old_grad)
        {
          const size_t sz = (size_t)(op->dim * op->dim + op->dim) * op->n_cells * op->nq * op->tsize();
          HIP_THROW(hipMalloc(&op->d_old_grad, std::max<size_t>(1, sz)));
        }
      pf(op, 2, x[0], s);
      op->have_old_grad = true;
    }
  op->stage.done(s);
  GLS_CATCH
}

glsStatus
gls_op_vmult_init(glsOp op, void *dst, const void *src, void *stream)
{
  GLS_TRY
  if (!op || !dst || !src)
    throw std::runtime_error("gls_op_vmult_init: null argument");
  init_dst(op, dst, src, (hipStream_t)stream);
  GLS_CATCH
}

glsStatus
gls_op_apply_identity_rows(glsOp op, void *dst, const void *src, void *stream)
{
  GLS_TRY
  if (!op || !dst || !src)
    throw std::runtime_error("gls_op_apply_identity_rows: null argument");
  if (op->n_owned_dofs == 0)
    return 0;
  hipStream_t s = (hipStream_t)stream;
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL(k_identity_rows<double>, grid1d(op->n_owned_dofs), dim3(256), 0, s,
                       (double *)dst, (const double *)src, op->d_cbits, op->n_owned_dofs);
  else
    hipLaunchKernelGGL(k_identity_rows<float>, grid1d(op->n_owned_dofs), dim3(256), 0, s,
                       (float *)dst, (const float *)src, op->d_cbits, op->n_owned_dofs);
  HIP_THROW(hipGetLastError());
  GLS_CATCH
}

glsStatus
gls_op_vmult_cells(glsOp op, void *dst, const void *src, int64_t b, int64_t e, void *stream)
{
  GLS_TRY
  if (!op || !dst || !src)
    throw std::runtime_error("gls_op_vmult_cells: null argument");
  if (!op->have_lin)
    throw std::runtime_error("vmult before set_linearization_point");
  if (b < 0 || e > op->n_cells || b > e)
    throw std::runtime_error("gls_op_vmult_cells: bad cell range");
  if (op->faces.n)
    throw std::runtime_error("gls_op_vmult_cells: operators with outflow faces run gls_op_vmult");
  ApplyFn   af;
  ProduceFn pf;
  select(op, af, pf);
  af(op, vmult_mode(op), false, dst, src, b, e, (hipStream_t)stream);
  GLS_CATCH
}

glsStatus
gls_op_vmult(glsOp op, void *dst, const void *src, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::vmult", (hipStream_t)stream);
  if (!op || !dst || !src)
    throw std::runtime_error("gls_op_vmult: null argument");
  if (dst == src)
    throw std::runtime_error("gls_op_vmult: dst and src must not alias");
  hipStream_t s = (hipStream_t)stream;
  const void *x = op->stage.in_vec(src, 0, s);
  void       *y = op->stage.out_vec(dst);
  gls::op_vmult_device(op, y, x, s);
  op->stage.finish_out(dst, s);
  op->stage.done(s);
  GLS_CATCH
}

// NavierStokesOperator::vmult_interface_down (operator_ns.cc:734-753): the
// cell loop over src with dst zeroed, then dst = src on the constrained dofs.
// The refinement-edge dofs (edge_constrained_indices, .cc:131-152) exist only
// on locally refined level meshes; every mesh this library takes is a whole
// level of a globally refined hierarchy, so the set is empty and the result
// is the vmult's (whose edge save / restore, .cc:691-731, is then a no-op).
glsStatus
gls_op_vmult_interface_down(glsOp op, void *dst, const void *src, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::vmult_interface_down", (hipStream_t)stream);
  if (!op || !dst || !src)
    throw std::runtime_error("gls_op_vmult_interface_down: null argument");
  if (dst == src)
    throw std::runtime_error("gls_op_vmult_interface_down: dst and src must not alias");
  hipStream_t s = (hipStream_t)stream;
  const void *x = op->stage.in_vec(src, 0, s);
  void       *y = op->stage.out_vec(dst);
  gls::op_vmult_device(op, y, x, s);
  op->stage.finish_out(dst, s);
  op->stage.done(s);
  GLS_CATCH
}

// NavierStokesOperator::vmult_interface_up (operator_ns.cc:755-787): with no
// edge-constrained dofs (has_edge_constrained_indices == false, above) the
// reference sets dst = 0 and returns.
glsStatus
gls_op_vmult_interface_up(glsOp op, void *dst, const void *src, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::vmult_interface_up", (hipStream_t)stream);
  if (!op || !dst || !src)
    throw std::runtime_error("gls_op_vmult_interface_up: null argument");
  hipStream_t s = (hipStream_t)stream;
  void       *y = op->stage.out_vec(dst);
  HIP_THROW(hipMemsetAsync(y, 0, (size_t)op->n_dofs * op->tsize(), s));
  op->stage.finish_out(dst, s);
  op->stage.done(s);
  GLS_CATCH
}

} // extern "C"

// constraints_inhomogeneous.distribute(tmp) on a copy of src (src NULL: a
// zero vector, evaluate_rhs): constrained components take the inhomogeneity
// (zero for the homogeneous Dirichlet / slip / pressure rows it shares with
// constraints_copy, main.cc:879-891), all others src.  One lane per dof.
template <typename T>
__global__ void
k_distribute(T *__restrict__ tmp, const T *__restrict__ src, const uint8_t *__restrict__ cmask,
             const T *__restrict__ inhom, int64_t n_dofs, int nc)
{
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n_dofs)
    return;
  const int64_t node = i / nc;
  const int     c    = (int)(i - node * nc);
  T             v    = src ? src[i] : T(0);
  if ((cmask[node] >> c) & 1)
    v = inhom ? inhom[i] : T(0);
  tmp[i] = v;
}

static void
distribute(glsOp op, void *tmp, const void *src, hipStream_t s)
{
  const int nc = op->dim + 1;
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL(k_distribute<double>, grid1d(op->n_dofs), dim3(256), 0, s,
                       (double *)tmp, (const double *)src, op->d_node_cmask,
                       (const double *)op->d_inhom, op->n_dofs, nc);
  else
    hipLaunchKernelGGL(k_distribute<float>, grid1d(op->n_dofs), dim3(256), 0, s, (float *)tmp,
                       (const float *)src, op->d_node_cmask, (const float *)op->d_inhom,
                       op->n_dofs, nc);
  HIP_THROW(hipGetLastError());
}

extern "C" {

glsStatus
gls_op_set_constraint_values(glsOp op, const void *values, void *stream)
{
  GLS_TRY
  if (!op)
    throw std::runtime_error("gls_op_set_constraint_values: null operator");
  hipStream_t s = (hipStream_t)stream;
  if (!values)
    {
      if (op->d_inhom)
        {
          HIP_THROW(hipStreamSynchronize(s));
          HIP_THROW(hipFree(op->d_inhom));
        }
      op->d_inhom = nullptr;
    }
  else
    {
      if (!op->d_inhom)
        HIP_THROW(hipMalloc(&op->d_inhom, std::max<size_t>(1, (size_t)op->n_dofs * op->tsize())));
      // host or device pointer (hipMemcpyDefault); a caller numbering is
      // permuted through the staging buffers first
      const void *v = op->stage.d_map ? op->stage.in_vec(values, 1, s) : values;
      HIP_THROW(hipMemcpyAsync(op->d_inhom, v, (size_t)op->n_dofs * op->tsize(),
                               hipMemcpyDefault, s));
      op->stage.done(s);
    }
  GLS_CATCH
}

} // extern "C"

static void
residual_cells(glsOp op, void *dst, const void *src, hipStream_t s)
{
  ApplyFn   af;
  ProduceFn pf;
  select(op, af, pf);
  if (op->use_brick)
    select_brick(op)(op, MODE_RESIDUAL, dst, src, 0, op->n_bricks, BRICK_RUN | BRICK_REDUCE,
                     s, nullptr);
  else
    {
      HIP_THROW(hipMemsetAsync(dst, 0, (size_t)op->n_dofs * op->tsize(), s));
      af(op, MODE_RESIDUAL, false, dst, src, 0, op->n_cells, s);
    }
  gls::faces_apply(op, true, dst, src, s);
}

extern "C" {

glsStatus
gls_op_evaluate_rhs(glsOp op, void *dst, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::evaluate_rhs", (hipStream_t)stream);
  if (!op || !dst)
    throw std::runtime_error("gls_op_evaluate_rhs: null argument");
  if (!op->have_lin)
    throw std::runtime_error("evaluate_rhs before set_linearization_point");
  hipStream_t s = (hipStream_t)stream;
  void       *y = op->stage.out_vec(dst);
  distribute(op, op->d_tmp, nullptr, s);
  residual_cells(op, y, op->d_tmp, s);
  op->stage.finish_out(dst, s);
  op->stage.done(s);
  GLS_CATCH
}

glsStatus
gls_op_evaluate_residual(glsOp op, void *dst, const void *src, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::evaluate_residual", (hipStream_t)stream);
  if (!op || !dst || !src || dst == src)
    throw std::runtime_error("gls_op_evaluate_residual: bad arguments");
  if (!op->have_lin)
    throw std::runtime_error("evaluate_residual before set_linearization_point");
  hipStream_t s = (hipStream_t)stream;
  const void *x = op->stage.in_vec(src, 0, s);
  void       *y = op->stage.out_vec(dst);
  // operator_ns.cc:655-656: tmp = src; constraints_inhomogeneous.distribute(tmp)
  distribute(op, op->d_tmp, x, s);
  residual_cells(op, y, op->d_tmp, s);
  op->stage.finish_out(dst, s);
  op->stage.done(s);
  GLS_CATCH
}

glsStatus
gls_op_evaluate_residual_plain(glsOp op, void *dst, const void *src, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::evaluate_residual", (hipStream_t)stream);
  if (!op || !dst || !src || dst == src)
    throw std::runtime_error("gls_op_evaluate_residual_plain: bad arguments");
  if (!op->have_lin)
    throw std::runtime_error("evaluate_residual before set_linearization_point");
  hipStream_t s = (hipStream_t)stream;
  const void *x = op->stage.in_vec(src, 0, s);
  void       *y = op->stage.out_vec(dst);
  residual_cells(op, y, x, s);
  op->stage.finish_out(dst, s);
  op->stage.done(s);
  GLS_CATCH
}

glsStatus
gls_op_get_max_u(glsOp op, const void *vec, double *u_max, void *stream)
{
  GLS_TRY
  if (!op || !vec || !u_max)
    throw std::runtime_error("gls_op_get_max_u: null argument");
  hipStream_t s = (hipStream_t)stream;
  const void *x = op->stage.in_vec(vec, 0, s);
  *u_max        = op->prec == GLS_F64 ? max_u_p<double>(op, x, s) : max_u_p<float>(op, x, s);
  GLS_CATCH
}

glsStatus
gls_op_compute_diagonal(glsOp op, void *diag, void *stream)
{
  GLS_TRY
  if (!op || !diag)
    throw std::runtime_error("gls_op_compute_diagonal: null argument");
  if (!op->have_lin)
    throw std::runtime_error("compute_diagonal before set_linearization_point");
  hipStream_t s   = (hipStream_t)stream;
  double     *d64 = nullptr;
  HIP_THROW(hipMallocAsync((void **)&d64, (size_t)op->n_dofs * sizeof(double), s));
  HIP_THROW(hipMemsetAsync(d64, 0, (size_t)op->n_dofs * sizeof(double), s));
  (op->prec == GLS_F64 ? select_diag_t<double>(op->dim, op->degree) :
                         select_diag_t<float>(op->dim, op->degree))(op, vmult_mode(op), d64, s);
  gls::faces_diagonal(op, d64, true, s);
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL(k_diag_out<double>, grid1d(op->n_dofs), dim3(256), 0, s, (double *)diag,
                       (const double *)d64, op->d_cbits, op->n_owned_dofs, op->n_dofs);
  else
    hipLaunchKernelGGL(k_diag_out<float>, grid1d(op->n_dofs), dim3(256), 0, s, (float *)diag,
                       (const double *)d64, op->d_cbits, op->n_owned_dofs, op->n_dofs);
  HIP_THROW(hipGetLastError());
  HIP_THROW(hipFreeAsync(d64, s));
  GLS_CATCH
}

glsStatus
gls_op_invert_diagonal(glsOp op, void *diag, void *stream)
{
  GLS_TRY
  if (!op || !diag)
    throw std::runtime_error("gls_op_invert_diagonal: null argument");
  hipStream_t s = (hipStream_t)stream;
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL(k_invert_diag<double>, grid1d(op->n_dofs), dim3(256), 0, s,
                       (double *)diag, op->d_cbits, op->n_owned_dofs, op->n_dofs);
  else
    hipLaunchKernelGGL(k_invert_diag<float>, grid1d(op->n_dofs), dim3(256), 0, s, (float *)diag,
                       op->d_cbits, op->n_owned_dofs, op->n_dofs);
  HIP_THROW(hipGetLastError());
  GLS_CATCH
}

glsStatus
gls_op_compute_inverse_diagonal(glsOp op, void *diag_, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::compute_inverse_diagonal", (hipStream_t)stream);
  if (!op || !diag_)
    throw std::runtime_error("gls_op_compute_inverse_diagonal: null argument");
  hipStream_t s = (hipStream_t)stream;
  gls::op_inverse_diagonal_device(op, op->stage.out_vec(diag_), s);
  op->stage.finish_out(diag_, s);
  op->stage.done(s);
  GLS_CATCH
}

} // extern "C"

namespace gls
{
void
op_cell_colours(glsOp_ *op)
{
  if (op->d_colour_cells)
    return;
  const int64_t nc_ = op->n_cells;
  const int     nq  = op->nq;
  // per node, the colours of the cells already coloured that touch it
  std::vector<uint64_t> used((size_t)op->n_nodes, 0);
  std::vector<int>      colour((size_t)nc_, 0);
  int                   n_col = 0;
  for (int64_t c = 0; c < nc_; ++c)
    {
      const uint32_t *cn   = &op->h_cell_nodes[(size_t)ext_cell(op, c) * nq];
      uint64_t        mask = 0;
      for (int p = 0; p < nq; ++p)
        mask |= used[cn[p]];
      if (~mask == 0)
        throw std::runtime_error("deterministic assembly: more than 64 cell colours");
      const int k = __builtin_ctzll(~mask);
      colour[(size_t)c] = k;
      n_col             = std::max(n_col, k + 1);
      for (int p = 0; p < nq; ++p)
        used[cn[p]] |= 1ull << k;
    }
  std::vector<int32_t> list;
  list.reserve((size_t)nc_);
  op->colour_off.assign(1, 0);
  for (int k = 0; k < n_col; ++k)
    {
      for (int64_t c = 0; c < nc_; ++c)
        if (colour[(size_t)c] == k)
          list.push_back((int32_t)c);
      op->colour_off.push_back((int64_t)list.size());
    }
  upload((void **)&op->d_colour_cells, list);
}

void
op_inverse_diagonal_device(glsOp op, void *diag, hipStream_t s)
{
  if (!op->have_lin)
    throw std::runtime_error("compute_inverse_diagonal before set_linearization_point");
  // the element diagonals evaluated directly (k_diag) instead of
  // MatrixFreeTools::compute_diagonal's unit-vector cell applies (1.68 ms of
  // k_apply<DIAG> per level, round 1)
  {
      // direct element diagonals, assembled in FP64 (in place for FP64
      // operators), inverted into the operator's precision
      double *d64 = (double *)diag;
      if (op->prec != GLS_F64)
        HIP_THROW(hipMallocAsync((void **)&d64, (size_t)op->n_dofs * sizeof(double), s));
      HIP_THROW(hipMemsetAsync(d64, 0, (size_t)op->n_dofs * sizeof(double), s));
      (op->prec == GLS_F64 ? select_diag_t<double>(op->dim, op->degree) :
                             select_diag_t<float>(op->dim, op->degree))(op, vmult_mode(op), d64, s);
      faces_diagonal(op, d64, true, s);
      if (op->prec == GLS_F64)
        hipLaunchKernelGGL(k_invert_diag64<double>, grid1d(op->n_dofs), dim3(256), 0, s,
                           (double *)diag, (const double *)d64, op->d_cbits, op->n_owned_dofs,
                           op->n_dofs);
      else
        {
          hipLaunchKernelGGL(k_invert_diag64<float>, grid1d(op->n_dofs), dim3(256), 0, s,
                             (float *)diag, (const double *)d64, op->d_cbits, op->n_owned_dofs,
                             op->n_dofs);
          HIP_THROW(hipFreeAsync(d64, s));
        }
      HIP_THROW(hipGetLastError());
    }
}

void
op_element_matrices_device(const glsOp_ *op, void *emat, int64_t b, int64_t e, hipStream_t s)
{
  if (!op->have_lin)
    throw std::runtime_error("element matrices before set_linearization_point");
  EmatFn fn = op->prec == GLS_F64 ? select_emat_t<double>(op->dim, op->degree) :
                                    select_emat_t<float>(op->dim, op->degree);
  if (!fn)
    throw std::runtime_error("no kernel instantiation for this (dim, degree)");
  fn(op, vmult_mode(op), emat, b, e, s);
  faces_element_matrices(op, emat, b, e, s);
}
} // namespace gls

extern "C" {

glsStatus
gls_op_upload_tables(glsOp op, const double *tables, const double *cellwise)
{
  GLS_TRY
  if (!op || !tables)
    throw std::runtime_error("gls_op_upload_tables: null argument");
  std::vector<double> soa((size_t)op->tab_elems, 0.0);
  for (int64_t c = 0; c < op->n_cells; ++c)
    for (int q = 0; q < op->nq; ++q)
      for (int f = 0; f < op->nf; ++f)
        soa[host_tab_index(op, c, q, storage_field(op, f))] =
          tables[((size_t)ext_cell(op, c) * op->nq + q) * op->nf + f];
  std::vector<double> cw((size_t)2 * op->n_cells, 0.0);
  if (cellwise)
    for (int64_t c = 0; c < op->n_cells; ++c)
      {
        cw[c]               = cellwise[2 * ext_cell(op, c)];
        cw[op->n_cells + c] = cellwise[2 * ext_cell(op, c) + 1];
      }
  if (op->prec == GLS_F64)
    {
      HIP_THROW(hipMemcpy(op->d_tab, soa.data(), soa.size() * 8, hipMemcpyHostToDevice));
      HIP_THROW(hipMemcpy(op->d_cellwise, cw.data(), cw.size() * 8, hipMemcpyHostToDevice));
    }
  else
    {
      auto sf = convert<float>(soa);
      auto cf = convert<float>(cw);
      HIP_THROW(hipMemcpy(op->d_tab, sf.data(), sf.size() * 4, hipMemcpyHostToDevice));
      HIP_THROW(hipMemcpy(op->d_cellwise, cf.data(), cf.size() * 4, hipMemcpyHostToDevice));
    }
  op->have_lin  = true;
  op->have_prev = op->prm.order > 0;
  // the H field from the cell geometry (the uploaded tables carry delta only)
  {
    const int64_t nqc = op->n_cells * op->nq;
    const dim3    g((unsigned)((nqc + 255) / 256));
    if (nqc > 0)
      {
        if (op->prec == GLS_F64 && op->dim == 3)
          hipLaunchKernelGGL((k_fill_h<3, double>), g, dim3(256), 0, 0, (double *)op->d_tab,
                             op->d_tab_cbase, op->tab_gs, (const double *)op->d_hq, op->n_cells, op->nq);
        else if (op->prec == GLS_F64)
          hipLaunchKernelGGL((k_fill_h<2, double>), g, dim3(256), 0, 0, (double *)op->d_tab,
                             op->d_tab_cbase, op->tab_gs, (const double *)op->d_hq, op->n_cells, op->nq);
        else if (op->dim == 3)
          hipLaunchKernelGGL((k_fill_h<3, float>), g, dim3(256), 0, 0, (float *)op->d_tab,
                             op->d_tab_cbase, op->tab_gs, (const float *)op->d_hq, op->n_cells, op->nq);
        else
          hipLaunchKernelGGL((k_fill_h<2, float>), g, dim3(256), 0, 0, (float *)op->d_tab,
                             op->d_tab_cbase, op->tab_gs, (const float *)op->d_hq, op->n_cells, op->nq);
        HIP_THROW(hipGetLastError());
        HIP_THROW(hipDeviceSynchronize());
      }
  }
  op->t1_valid = false;
  op->version++;
  GLS_CATCH
}

glsStatus
gls_op_download_tables(glsOp op, double *tables, double *cellwise)
{
  GLS_TRY
  if (!op)
    throw std::runtime_error("gls_op_download_tables: null argument");
  HIP_THROW(hipDeviceSynchronize());
  std::vector<double> soa((size_t)op->tab_elems), cw((size_t)2 * op->n_cells);
  if (op->prec == GLS_F64)
    {
      HIP_THROW(hipMemcpy(soa.data(), op->d_tab, soa.size() * 8, hipMemcpyDeviceToHost));
      HIP_THROW(hipMemcpy(cw.data(), op->d_cellwise, cw.size() * 8, hipMemcpyDeviceToHost));
    }
  else
    {
      std::vector<float> sf(soa.size()), cf(cw.size());
      HIP_THROW(hipMemcpy(sf.data(), op->d_tab, sf.size() * 4, hipMemcpyDeviceToHost));
      HIP_THROW(hipMemcpy(cf.data(), op->d_cellwise, cf.size() * 4, hipMemcpyDeviceToHost));
      soa.assign(sf.begin(), sf.end());
      cw.assign(cf.begin(), cf.end());
    }
  if (tables)
    for (int64_t c = 0; c < op->n_cells; ++c)
      for (int q = 0; q < op->nq; ++q)
        for (int f = 0; f < op->nf; ++f)
          tables[((size_t)ext_cell(op, c) * op->nq + q) * op->nf + f] =
            soa[host_tab_index(op, c, q, storage_field(op, f))];
  if (cellwise)
    for (int64_t c = 0; c < op->n_cells; ++c)
      {
        cellwise[2 * ext_cell(op, c)]     = cw[c];
        cellwise[2 * ext_cell(op, c) + 1] = cw[op->n_cells + c];
      }
  GLS_CATCH
}

glsStatus
gls_discover_bricks(int dim, int degree, int64_t n_cells, const uint32_t *cell_nodes,
                    int *shape, int64_t *perm)
{
  GLS_TRY
  if (!cell_nodes || !shape || !perm || (dim != 2 && dim != 3) || degree < 1 || n_cells < 0)
    throw std::runtime_error("gls_discover_bricks: invalid argument");
  gls::BrickPlan plan;
  if (!gls::discover_bricks(dim, degree, n_cells, cell_nodes, plan))
    {
      shape[0] = shape[1] = shape[2] = 0;
      for (int64_t c = 0; c < n_cells; ++c)
        perm[c] = c;
    }
  else
    {
      for (int a = 0; a < 3; ++a)
        shape[a] = plan.shape[a];
      std::copy(plan.perm.begin(), plan.perm.end(), perm);
    }
  GLS_CATCH
}

// element matrices of every cell, FP64 host [cell][col j][row i], i, j =
// local dofs p * (dim + 1) + component (the caller's cell order); computed
// on the device in chunks of cells
static void
element_matrices_host(glsOp op, double *out)
{
  const int     ndof  = op->nq * (op->dim + 1);
  const size_t  per   = (size_t)ndof * ndof;
  const int64_t chunk = std::max<int64_t>(1, (int64_t)((256u << 20) / (per * op->tsize())));
  EmatFn        fn    = op->prec == GLS_F64 ? select_emat_t<double>(op->dim, op->degree) :
                                              select_emat_t<float>(op->dim, op->degree);
  if (!fn)
    throw std::runtime_error("no kernel instantiation for this (dim, degree)");
  void *buf = nullptr;
  HIP_THROW(hipMalloc(&buf, (size_t)std::min(chunk, op->n_cells) * per * op->tsize()));
  std::vector<double> tmp;
  std::vector<float>  tmpf;
  try
    {
      for (int64_t b = 0; b < op->n_cells; b += chunk)
        {
          const int64_t e = std::min(op->n_cells, b + chunk);
          fn(op, op_vmult_mode(op), buf, b, e, nullptr);
          faces_element_matrices(op, buf, b, e, nullptr);
          const size_t cnt = (size_t)(e - b) * per;
          if (op->prec == GLS_F64)
            {
              tmp.resize(cnt);
              HIP_THROW(hipMemcpy(tmp.data(), buf, cnt * 8, hipMemcpyDeviceToHost));
            }
          else
            {
              tmpf.resize(cnt);
              HIP_THROW(hipMemcpy(tmpf.data(), buf, cnt * 4, hipMemcpyDeviceToHost));
              tmp.assign(tmpf.begin(), tmpf.end());
            }
          for (int64_t c = b; c < e; ++c)
            std::copy(tmp.begin() + (size_t)(c - b) * per, tmp.begin() + (size_t)(c - b + 1) * per,
                      out + (size_t)ext_cell(op, c) * per);
        }
    }
  catch (...)
    {
      (void)hipFree(buf);
      throw;
    }
  HIP_THROW(hipFree(buf));
}

glsStatus
gls_op_element_matrices(glsOp op, double *out)
{
  GLS_TRY
  if (!op || !out)
    throw std::runtime_error("gls_op_element_matrices: null argument");
  if (!op->have_lin)
    throw std::runtime_error("gls_op_element_matrices before set_linearization_point");
  element_matrices_host(op, out);
  GLS_CATCH
}

glsStatus
gls_op_system_matrix(glsOp op, int64_t *nnz, int64_t *row_ptr, int64_t *cols, double *vals)
{
  GLS_TRY
  gls::Section sec_("ns::initialize_system_matrix", nullptr);
  if (!op || !nnz)
    throw std::runtime_error("gls_op_system_matrix: null argument");
  if (op->n_owned_nodes != op->n_nodes)
    throw std::runtime_error("gls_op_system_matrix: single-domain operators only");
  const int     nc = op->dim + 1, nq = op->nq, ndof = nq * nc;
  const int64_t N  = op->n_dofs;
  // sparsity: the node couplings of the cells, every component pair; rows
  // and columns of constrained dofs hold only their unit diagonal (the
  // identity rows of vmult, operator_ns.cc:719-721)
  std::vector<std::vector<uint32_t>> adj((size_t)op->n_nodes);
  for (int64_t c = 0; c < op->n_cells; ++c)
    for (int i = 0; i < nq; ++i)
      for (int j = 0; j < nq; ++j)
        adj[op->h_cell_nodes[(size_t)c * nq + i]].push_back(op->h_cell_nodes[(size_t)c * nq + j]);
  for (auto &a : adj)
    {
      std::sort(a.begin(), a.end());
      a.erase(std::unique(a.begin(), a.end()), a.end());
    }
  auto constrained = [&](int64_t dof) { return (op->h_cmask[dof / nc] >> (dof % nc)) & 1; };
  std::vector<int64_t> rp((size_t)N + 1, 0);
  for (int64_t r = 0; r < N; ++r)
    {
      int64_t cnt = 0;
      if (constrained(r))
        cnt = 1;
      else
        for (uint32_t m : adj[(size_t)(r / nc)])
          for (int cc = 0; cc < nc; ++cc)
            cnt += constrained((int64_t)m * nc + cc) ? 0 : 1;
      rp[(size_t)r + 1] = rp[(size_t)r] + cnt;
    }
  *nnz = rp.back();
  if (!row_ptr)
    return 0; // sizing call
  if (!cols || !vals)
    throw std::runtime_error("gls_op_system_matrix: null output arrays");
  std::copy(rp.begin(), rp.end(), row_ptr);
  for (int64_t r = 0; r < N; ++r)
    {
      int64_t k = rp[(size_t)r];
      if (constrained(r))
        {
          cols[k] = r;
          vals[k] = 1.0;
          continue;
        }
      for (uint32_t m : adj[(size_t)(r / nc)])
        for (int cc = 0; cc < nc; ++cc)
          {
            const int64_t col = (int64_t)m * nc + cc;
            if (constrained(col))
              continue;
            cols[k]   = col;
            vals[k++] = 0.0;
          }
    }
  std::vector<double> E((size_t)op->n_cells * ndof * ndof);
  element_matrices_host(op, E.data());
  for (int64_t c = 0; c < op->n_cells; ++c)
    {
      const uint32_t *cn = &op->h_cell_nodes[(size_t)c * nq];
      const double   *Ec = &E[(size_t)c * ndof * ndof];
      for (int i = 0; i < ndof; ++i)
        {
          const int64_t r = (int64_t)cn[i / nc] * nc + i % nc;
          if (constrained(r))
            continue;
          const int64_t *cb = cols + rp[(size_t)r], *ce = cols + rp[(size_t)r + 1];
          for (int j = 0; j < ndof; ++j)
            {
              const int64_t col = (int64_t)cn[j / nc] * nc + j % nc;
              if (constrained(col))
                continue;
              const int64_t *it = std::lower_bound(cb, ce, col);
              vals[it - cols] += Ec[(size_t)j * ndof + i];
            }
        }
    }
  GLS_CATCH
}

glsStatus
gls_op_brick_shape(glsOp op, int *dims)
{
  GLS_TRY
  if (!op || !dims)
    throw std::runtime_error("gls_op_brick_shape: null argument");
  dims[0] = op->use_brick ? op->bx : 0;
  dims[1] = op->use_brick ? op->by : 0;
  dims[2] = op->use_brick ? op->bz : 0;
  GLS_CATCH
}

glsStatus
gls_op_sweep_stats(glsOp op, uint64_t *launches, uint64_t *timeouts)
{
  GLS_TRY
  if (!op || !launches || !timeouts)
    throw std::runtime_error("gls_op_sweep_stats: null argument");
  uint32_t h = 0;
  if (op->d_sweep_err)
    {
      gls::DeviceScope dev(op->device);
      HIP_THROW(hipDeviceSynchronize());
      HIP_THROW(hipMemcpy(&h, op->d_sweep_err, sizeof(h), hipMemcpyDeviceToHost));
    }
  *launches = op->sweep_launches;
  *timeouts = h;
  GLS_CATCH
}

glsStatus
gls_op_set_sweep_spin_bound(glsOp op, int64_t polls)
{
  GLS_TRY
  if (!op || polls < 0 || polls > (int64_t)1 << 30)
    throw std::runtime_error("gls_op_set_sweep_spin_bound: bad arguments");
  op->sweep_spin_max = (int)polls;
  GLS_CATCH
}

glsStatus
gls_op_cell_permutation(glsOp op, int64_t *perm)
{
  GLS_TRY
  if (!op || !perm)
    throw std::runtime_error("gls_op_cell_permutation: null argument");
  for (int64_t c = 0; c < op->n_cells; ++c)
    perm[c] = ext_cell(op, c);
  GLS_CATCH
}

glsStatus
gls_op_geometry_counts(glsOp op, int64_t *n_general, int64_t *n_cartesian)
{
  GLS_TRY
  if (!op)
    throw std::runtime_error("gls_op_geometry_counts: null argument");
  if (n_general)
    *n_general = op->n_gen;
  if (n_cartesian)
    *n_cartesian = op->n_cart;
  GLS_CATCH
}

double
gls_op_vmult_bytes(glsOp op)
{
  if (!op)
    return 0;
  // B = s 2N + s C nq n_tab + s [n_gen nq (dim^2+1) +
  //                 n_cart (dim+1)] + 4 C nq,
  // with n_tab the table values per q this build streams, in whole 16-byte
  // groups (brick.h field_read): the reference's 20 in 3D (operator_ns.h:
  // 120-132) with the time derivative, the U_t-only group skipped without it
  // (18 in FP64); 16 for the brick Newton vmult (T1 tables, delta from U and
  // h); the per-cell path the reference's set
  const double s   = (double)op->tsize();
  const int    dim = op->dim;
  const bool   td  = (op->prm.flags & GLS_CONSIDER_TIME_DERIVATIVE) && op->prm.order > 0;
  const bool   nt  = (op->prm.flags & GLS_INCREMENT_FORM) != 0;
  int          n_tab;
  if (op->use_brick)
    {
      const int W = (int)(16 / op->tsize());
      n_tab       = 0;
      for (int g = 0; g * W < op->nf_store; ++g)
        {
          bool any = false;
          for (int w = 0; w < W; ++w)
            {
              const int f = g * W + w;
              const bool q2 = op->degree == 2;
              any = any || (dim == 3 ? (nt ? (q2 ? field_read<3, MODE_NEWTON, 2>(f)
                                                 : field_read<3, MODE_NEWTON, 1>(f))
                                            : field_read<3, MODE_FIXED>(f))
                                     : (nt ? (q2 ? field_read<2, MODE_NEWTON, 2>(f)
                                                 : field_read<2, MODE_NEWTON, 1>(f))
                                            : field_read<2, MODE_FIXED>(f)));
            }
          const bool ut_only = nt && (dim == 3 ? group_ut_only<3, MODE_NEWTON>(g, W)
                                               : group_ut_only<2, MODE_NEWTON>(g, W));
          n_tab += any && (!ut_only || td) ? W : 0;
        }
    }
  else if (nt)
    n_tab = 2 + dim + dim * dim + dim + (td ? dim : 0);
  else
    n_tab = 2 + dim;
  if (!op->use_brick && (op->prm.flags & GLS_CELL_WISE_STAB))
    n_tab -= 2;
  const double C = (double)op->n_cells, nq = (double)op->nq;
  double b = s * 2.0 * (double)op->n_dofs + s * C * nq * n_tab +
             s * ((double)op->n_gen * nq * (dim * dim + 1) + (double)op->n_cart * (dim + 1)) +
             4.0 * C * nq;
  if (op->prm.flags & GLS_CELL_WISE_STAB)
    b += s * 2.0 * C;
  return b;
}

} // extern "C"
