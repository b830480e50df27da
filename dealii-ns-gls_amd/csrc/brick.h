// brick.h — the production vmult / residual kernel (gfx950).
//
// Work decomposition: one 256-thread workgroup per BRICK, a block of
// bx*by*bz cells of one refined coarse cell (3D: 4x4x4 cells, Q2 -> a 9^3
// node lattice).  The workgroup
//   1. runs the brick's cells through the per-cell operator (sum
//      factorisation + GLS q-point physics, do_vmult_cell
//      operator_ns.cc:949-1182) in rounds of CPW cells per wavefront and adds
//      every cell's nodal result into an LDS accumulator lattice (LDS
//      atomics: cells of different wavefronts share lattice nodes);
//   2. writes the lattice out: nodes owned by this brick alone go straight to
//      dst (plain stores; dst is never zeroed), nodes on the brick boundary go
//      to a per-node-contiguous partial buffer that k_shared_reduce sums.  No
//      global atomics; bitwise reproducible up to the LDS-atomic order.
//      (distribute_local_to_global + compress(add) of the reference's
//      cell_loop and the identity rows of vmult, operator_ns.cc:702-721.)
//
// Thread map: one lane per (cell, quadrature point) = (cell, node) since
// FE_Q(k) and QGauss(k+1) both have (k+1)^dim points; a cell never straddles
// a wavefront (3D Q2: 2 cells = 54 of 64 lanes), so the LDS sum-factorisation
// sweeps are ordered by wavefront fences, not workgroup barriers.
// Occupancy is the lever (the kernel is LDS-latency bound at low wave
// counts): 3 waves/SIMD (FP64, <= 168 VGPRs, 37 KB LDS per workgroup).
// Software-pipelining the next round's loads was measured and gave nothing.
#pragma once

#include "kernels.h"

namespace gls
{
constexpr uint32_t SHARED_BIT = 0x80000000u;

template <int dim>
struct BrickMax
{
  static constexpr int cells = dim == 3 ? 4 : 8; // cells per direction
};

template <int dim, int k>
struct BrickLattice
{
  static constexpr int side = k * BrickMax<dim>::cells + 1;
  static constexpr int L    = dim == 3 ? side * side * side : side * side;
  // the brick kernel is used when the accumulator lattice fits in LDS
  static constexpr bool fits = L <= 729;
};

// workgroup-scope atomic add on an LDS address (ds_add_f64 / ds_add_f32)
template <typename T>
__device__ __forceinline__ void
lds_add(T *p, T v)
{
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <typename T, int dim, int n>
struct BrickArgs
{
  const uint32_t *brick_nodes;  // [n_bricks][L] node | cmask << 28
  const uint32_t *brick_target; // [n_bricks][L] node, or SHARED_BIT | slot
  const uint32_t *cell_geo;
  const T        *geo_cart;
  int64_t         n_cart;
  const T        *geo_gen; // [field][plane][g][line]
  int64_t         n_gen;
  const T        *tab;     // [field][plane][cell][line]
  int64_t         n_cells;
  const T        *cellwise;
  const T        *old_grad;
  T              *dst;
  const T        *src;
  T              *partial; // [slot][dim+1], slots of a node contiguous
  int64_t         brick_begin, brick_end;
  int             bx, by, bz;
  int             L, Lx, Ly;
  T               nu, w0, theta;
  int             td, cw, have_prev, have_old_grad;
  Shape<T, n>     sh;
};

// everything one lane needs from HBM for one (cell, q point)
template <int dim, typename T, int MODE>
struct LaneData
{
  static constexpr int NOLD = MODE == MODE_RESIDUAL ? dim * dim + dim : 1;
  T        u[dim + 1];
  T        inv[dim][dim];
  T        JxW;
  T        U[dim], GU[dim][dim], GP[dim], UT[dim], oldg[NOLD];
  T        d1, d2;
  uint32_t cm;
  int      li;
  bool     active;
};

template <int dim, int k, typename T, int MODE>
__device__ __forceinline__ void
load_lane(const BrickArgs<T, dim, k + 1> &a, int64_t brick, int lcell, bool in_wave, int p,
          const int (&pa)[3], LaneData<dim, T, MODE> &r)
{
  constexpr int n   = k + 1;
  constexpr int nq  = ipow(n, dim);
  constexpr int nc  = dim + 1;
  constexpr bool R  = MODE == MODE_RESIDUAL;
  using F           = Fields<dim>;
  const int     cpb = a.bx * a.by * a.bz;
  r.active          = in_wave && lcell < cpb;
  const int cx      = r.active ? lcell % a.bx : 0;
  const int cy      = r.active ? (lcell / a.bx) % a.by : 0;
  const int cz      = r.active ? lcell / (a.bx * a.by) : 0;
  r.li = (cx * k + pa[0]) + a.Lx * ((cy * k + pa[1]) + a.Ly * (cz * k + pa[2]));
  const int64_t cell = brick * cpb + lcell;
  const int64_t nqc  = a.n_cells * nq;
  r.cm               = 0;
  r.JxW = r.d1 = r.d2 = 0;
#pragma unroll
  for (int c = 0; c < nc; ++c)
    r.u[c] = 0;
#pragma unroll
  for (int i = 0; i < dim; ++i)
    {
#pragma unroll
      for (int e = 0; e < dim; ++e)
        {
          r.inv[i][e] = 0;
          r.GU[i][e]  = 0;
        }
      r.U[i] = r.GP[i] = r.UT[i] = 0;
    }
#pragma unroll
  for (int i = 0; i < LaneData<dim, T, MODE>::NOLD; ++i)
    r.oldg[i] = 0;
  if (!r.active)
    return;
  // node values (read_dof_values / read_dof_values_plain)
  const uint32_t packed = a.brick_nodes[brick * (int64_t)a.L + r.li];
  r.cm                  = packed >> 28;
  if (GLS_ABL & 8)
    {
#pragma unroll
      for (int c = 0; c < nc; ++c)
        r.u[c] = T(1e-3) * (r.li + c);
    }
  else
    load_node<T, nc>(a.src, packed & NODE_MASK, r.u);
  if (GLS_ABL & 4)
    {
      r.JxW = T(1e-6);
#pragma unroll
      for (int i = 0; i < dim; ++i)
        {
          r.inv[i][i] = T(10) + p;
          r.U[i]      = T(1) + i;
        }
      r.d1 = T(1e-4) * p;
      r.d2 = T(1e-3);
      return;
    }
  // geometry (MatrixFree-style compressed: Cartesian per cell, else per q)
  const uint32_t cg = a.cell_geo[cell];
  if (cg & GEO_GENERAL)
    {
      const int64_t gq  = qindex<dim, n>(cg & ~GEO_GENERAL, p, a.n_gen);
      const int64_t gst = a.n_gen * nq;
      r.JxW             = a.geo_gen[gq];
#pragma unroll
      for (int i = 0; i < dim; ++i)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          r.inv[i][e] = a.geo_gen[(1 + i * dim + e) * gst + gq];
    }
  else
    {
      T w = a.sh.w[pa[0]] * a.sh.w[pa[1]];
      if (dim == 3)
        w *= a.sh.w[pa[2]];
#pragma unroll
      for (int i = 0; i < dim; ++i)
        r.inv[i][i] = a.geo_cart[i * a.n_cart + cg];
      r.JxW = a.geo_cart[dim * a.n_cart + cg] * w;
    }
  // per-q tables (operator_ns.h:120-132)
  const int64_t tq = qindex<dim, n>(cell, p, a.n_cells);
#pragma unroll
  for (int d = 0; d < dim; ++d)
    {
      r.U[d] = a.tab[(F::U + d) * nqc + tq];
      if (MODE == MODE_NEWTON)
        {
#pragma unroll
          for (int e = 0; e < dim; ++e)
            r.GU[d][e] = a.tab[(F::GU + d * dim + e) * nqc + tq];
          r.GP[d] = a.tab[(F::GP + d) * nqc + tq];
        }
      if ((MODE == MODE_NEWTON && a.td) || (R && a.have_prev))
        r.UT[d] = a.tab[(F::UT + d) * nqc + tq];
    }
  if (R && a.have_old_grad)
#pragma unroll
    for (int i = 0; i < LaneData<dim, T, MODE>::NOLD; ++i)
      r.oldg[i] = a.old_grad[i * nqc + tq];
  if (a.cw)
    {
      r.d1 = a.cellwise[cell];
      r.d2 = a.cellwise[a.n_cells + cell];
    }
  else
    {
      r.d1 = a.tab[F::D1 * nqc + tq];
      r.d2 = a.tab[F::D2 * nqc + tq];
    }
}

template <int dim, int k, typename T, int MODE>
__global__ void __launch_bounds__(BLOCK, 3)
  k_brick(BrickArgs<T, dim, k + 1> a)
{
  constexpr int n    = k + 1;
  constexpr int nq   = ipow(n, dim);
  constexpr int nc   = dim + 1;
  constexpr int CPW  = 64 / nq > 0 ? 64 / nq : 1; // cells per wavefront
  constexpr int WPB  = BLOCK / 64;
  constexpr int LMAX = BrickLattice<dim, k>::L;
  constexpr int WB   = 2 * nc * nq; // per-cell ping-pong sweep buffer
  constexpr bool R   = MODE == MODE_RESIDUAL;
  static_assert(nq <= 64, "one cell must fit a wavefront");

  __shared__ T s_acc[nc * LMAX];
  // one sweep buffer per cell slot; left-over lanes (64 % nq) only read the
  // first slot's buffer, every LDS store is guarded by in_wave
  __shared__ T s_work[WPB * CPW * WB];
  __shared__ T sS[n][n], sD[n][n];

  const int64_t brick = a.brick_begin + blockIdx.x;
  if (brick >= a.brick_end)
    return;
  const int t   = threadIdx.x;
  const int L   = a.L;
  const int cpb = a.bx * a.by * a.bz;
  if (t < n * n)
    {
      sS[t / n][t % n] = a.sh.S[t / n][t % n];
      sD[t / n][t % n] = a.sh.Dq[t / n][t % n];
    }
  for (int i = t; i < L; i += BLOCK)
#pragma unroll
    for (int c = 0; c < nc; ++c)
      s_acc[c * LMAX + i] = T(0);

  const int  wave    = t >> 6, lane = t & 63;
  const int  slot    = lane / nq;
  const int  p       = lane - slot * nq;
  const bool in_wave = slot < CPW;
  T         *A       = s_work + (wave * CPW + (in_wave ? slot : 0)) * WB;
  T         *B       = A + nc * nq;
  const int  pa[3]   = {p % n, (p / n) % n, dim == 3 ? p / (n * n) : 0};
  const int  st[3]   = {1, n, n * n};
  const int  step    = CPW * WPB;
  __syncthreads();

  for (int base = 0; base < cpb; base += step)
    {
      LaneData<dim, T, MODE> cur;
      load_lane<dim, k, T, MODE>(a, brick, base + wave * CPW + slot, in_wave, p, pa, cur);

      if (in_wave)
#pragma unroll
        for (int c = 0; c < nc; ++c)
          A[c * nq + p] = (!R && ((cur.cm >> c) & 1)) ? T(0) : cur.u[c];
      wave_sync();

      // ---- evaluate: values at q (dim sweeps with S), gradients by Dq
      T *in = A, *out = B;
#pragma unroll
      for (int ax = 0; ax < dim; ++ax)
        {
          if (in_wave)
#pragma unroll
            for (int c = 0; c < nc; ++c)
              out[c * nq + p] =
                contract<n, false>(in + c * nq, sS, pa[ax], p - pa[ax] * st[ax], st[ax]);
          wave_sync();
          T *tmp = in;
          in     = out;
          out    = tmp;
        }
      T val[nc], gref[nc][dim];
#pragma unroll
      for (int c = 0; c < nc; ++c)
        {
          val[c] = in[c * nq + p];
#pragma unroll
          for (int ax = 0; ax < dim; ++ax)
            gref[c][ax] =
              contract<n, false>(in + c * nq, sD, pa[ax], p - pa[ax] * st[ax], st[ax]);
        }
      wave_sync();

      // ---- q-point physics (do_vmult_cell)
      T gu[dim][dim], gp[dim];
#pragma unroll
      for (int c = 0; c < nc; ++c)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          {
            T s = 0;
#pragma unroll
            for (int i = 0; i < dim; ++i)
              s += cur.inv[i][e] * gref[c][i];
            if (c < dim)
              gu[c][e] = s;
            else
              gp[e] = s;
          }
      T vr[nc], gr[nc][dim];
      qpoint_physics<dim, T, MODE>(val, val[dim], gu, gp, cur.U, cur.GU, cur.GP, cur.UT,
                                   cur.oldg, cur.d1, cur.d2, a.nu, a.w0, a.theta, a.td,
                                   a.have_prev, a.have_old_grad, vr, gr);
      // submit_value / submit_gradient (JxW, J^{-T}); inactive lanes: JxW 0
      T wq[nc], ghat[nc][dim];
#pragma unroll
      for (int c = 0; c < nc; ++c)
        {
          wq[c] = vr[c] * cur.JxW;
#pragma unroll
          for (int i = 0; i < dim; ++i)
            {
              T s = 0;
#pragma unroll
              for (int e = 0; e < dim; ++e)
                s += cur.inv[i][e] * gr[c][e];
              ghat[c][i] = s * cur.JxW;
            }
        }

      // ---- integrate: Dq^T on the gradient part (two axes per exchange
      // through the A/B halves), then S^T sweeps
#pragma unroll
      for (int ax0 = 0; ax0 < dim; ax0 += 2)
        {
          if (in_wave)
#pragma unroll
            for (int c = 0; c < nc; ++c)
              {
                A[c * nq + p] = ghat[c][ax0];
                if (ax0 + 1 < dim)
                  B[c * nq + p] = ghat[c][(ax0 + 1) % dim];
              }
          wave_sync();
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              wq[c] += contract<n, true>(A + c * nq, sD, pa[ax0], p - pa[ax0] * st[ax0], st[ax0]);
              if (ax0 + 1 < dim)
                {
                  const int ax1 = (ax0 + 1) % dim;
                  wq[c] += contract<n, true>(B + c * nq, sD, pa[ax1], p - pa[ax1] * st[ax1],
                                             st[ax1]);
                }
            }
          wave_sync();
        }
      if (in_wave)
#pragma unroll
        for (int c = 0; c < nc; ++c)
          A[c * nq + p] = wq[c];
      wave_sync();
      in  = A;
      out = B;
#pragma unroll
      for (int ax = dim - 1; ax >= 0; --ax)
        {
          if (in_wave)
#pragma unroll
            for (int c = 0; c < nc; ++c)
              out[c * nq + p] =
                contract<n, true>(in + c * nq, sS, pa[ax], p - pa[ax] * st[ax], st[ax]);
          wave_sync();
          T *tmp = in;
          in     = out;
          out    = tmp;
        }
      // ---- accumulate into the brick lattice
      if (cur.active)
#pragma unroll
        for (int c = 0; c < nc; ++c)
          lds_add(s_acc + c * LMAX + cur.li, in[c * nq + p]);
      wave_sync();
    }
  __syncthreads();

  // ---- write out: exclusive nodes -> dst, boundary nodes -> partials
  const uint32_t *bn = a.brick_nodes + brick * (int64_t)L;
  const uint32_t *bt = a.brick_target + brick * (int64_t)L;
  for (int i = t; i < L; i += BLOCK)
    {
      const uint32_t tg = bt[i];
      if (tg & SHARED_BIT)
        {
          T *pp = a.partial + (size_t)(tg & ~SHARED_BIT) * nc;
#pragma unroll
          for (int c = 0; c < nc; ++c)
            pp[c] = R ? -s_acc[c * LMAX + i] : s_acc[c * LMAX + i];
        }
      else
        {
          const uint32_t cm = bn[i] >> 28;
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              T v = R ? -s_acc[c * LMAX + i] : s_acc[c * LMAX + i];
              if ((cm >> c) & 1)
                v = R ? T(0) : a.src[(size_t)tg * nc + c];
              a.dst[(size_t)tg * nc + c] = v;
            }
        }
    }
}

// Sum the per-brick partials of every brick-boundary node (one contiguous
// slot run per node); constrained components get the identity row (vmult,
// operator_ns.cc:719-721) or zero (evaluate_residual's set_zero, :678).
// One thread per (shared node, component): consecutive threads touch
// consecutive doubles of a node's partials and of dst.
template <typename T, int nc, bool R>
__global__ void __launch_bounds__(256)
  k_shared_reduce(T *__restrict__ dst, const T *__restrict__ src,
                  const T *__restrict__ partial, const uint32_t *__restrict__ nodes,
                  const uint32_t *__restrict__ offsets, int64_t n_shared)
{
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n_shared * nc)
    return;
  const int64_t  s      = gid / nc;
  const int      c      = (int)(gid - s * nc);
  const uint32_t b      = offsets[s], e = offsets[s + 1];
  const uint32_t packed = nodes[s];
  T              sum    = 0;
  for (uint32_t i = b; i < e; ++i)
    sum += partial[(size_t)i * nc + c];
  const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
  if ((cm >> c) & 1)
    sum = R ? T(0) : src[(size_t)node * nc + c];
  dst[(size_t)node * nc + c] = sum;
}

} // namespace gls
