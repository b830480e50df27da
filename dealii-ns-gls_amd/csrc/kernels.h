// kernels.h — HIP/CDNA4 (gfx950) kernels of the matrix-free GLS
// Navier–Stokes operator.  Included by gls_op.hip only.
//
// Thread mapping: one thread per (cell, quadrature point); since FE_Q(k) has
// (k+1)^dim nodes and QGauss(k+1) has (k+1)^dim points, the same thread also
// owns the cell's node with the same lexicographic index.  A 256-thread
// workgroup holds CPB = 256 / (k+1)^dim cells (3D Q2: 9 cells, 243 lanes).
// Sum factorisation (deal.II's FEEvaluation::evaluate/integrate, called at
// operator_ns.cc:962-963,1064-1065,1074-1075,1179-1180) runs as 1D
// contractions through LDS: values by S (shape values at Gauss points),
// gradients by the collocation derivative Dq at the Gauss points, integrate
// by the transposes.  The q-point physics is do_vmult_cell,
// operator_ns.cc:949-1182 (Newton branch :1067-1181, fixed-point/residual
// branch :955-1066).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gls
{
constexpr uint32_t NODE_MASK  = 0x0FFFFFFFu;
constexpr int      BLOCK      = 256;
constexpr uint32_t GEO_GENERAL = 0x80000000u;

constexpr int
ipow(int n, int d)
{
  return d == 0 ? 1 : n * ipow(n, d - 1);
}

// Per-quadrature-point arrays (tables, general geometry) are stored
// [field][plane][cell][line]: q point p = line + LPC * plane with
// LPC = (k+1)^(dim-1), so the lanes that own one quadrature plane of
// consecutive cells read consecutive addresses (csrc/brick.h thread map).
template <int dim, int n>
__device__ __forceinline__ int64_t
qindex(int64_t cell, int p, int64_t ncell)
{
  constexpr int LPC = ipow(n, dim - 1);
  return ((int64_t)(p / LPC) * ncell + cell) * LPC + (p % LPC);
}

enum Mode
{
  MODE_NEWTON   = 0, // vmult, increment form (Newton Jacobian)
  MODE_FIXED    = 1, // vmult, fixed-point form (!increment_form)
  MODE_RESIDUAL = 2  // evaluate_residual (read plain, negate)
};

// table field offsets (SoA, [field][cell * nq + q])
template <int dim>
struct Fields
{
  // Table fields per (cell, q), in the order the brick kernel streams them:
  //   U = u_star_value, GU = u_star_gradient (operator_ns.h:126-127),
  //   T1 = the linearization-point part of the Newton SUPG residual R1
  //        (operator_ns.cc:1146-1151 without delta_1):
  //        (td ? w0 U + Ut_old : 0) + grad P* + (grad U) U, formed by
  //        k_finalize_t1 once the producers and the time weights are set,
  //   H  = the cell's q-wise h (operator_ns.cc:394-405), from which the
  //        brick kernel recomputes delta_1 / delta_2 (:407-420),
  //   D1, D2 = delta_1_q, delta_2_q, UT = u_time_derivative_old,
  //   GP = p_star_gradient (operator_ns.h:123-130).
  // A Newton vmult of the brick kernel reads U, GU, T1, H only (16 of the
  // reference's 20 values per q); D1, D2, GP, UT stay for the other paths.
  static constexpr int U = 0, GU = dim, T1 = dim + dim * dim, H = 2 * dim + dim * dim,
                       D1 = H + 1, D2 = H + 2, UT = H + 3, GP = H + 3 + dim,
                       N = H + 3 + 2 * dim;
  static constexpr int NEWTON = H + 1; // leading fields of a Newton brick vmult
};

// Per-q tables (set_linearization_point / set_previous_solution outputs,
// operator_ns.h:120-132) are stored in 16-byte field groups of W = 16 /
// sizeof(T) fields: element (cell, q, field f) at
//   cbase[cell] + (f / W) * gs + q * W + f % W.
// With the brick kernel, a cell's cbase places the cells of one wavefront
// round (csrc/brick.h: CPW cells) in one chunk, so every table load of the
// round is one contiguous 16-byte-per-lane wave load.
template <typename T>
__device__ __forceinline__ int64_t
tab_index(const int64_t *cbase, int64_t gs, int64_t cell, int p, int f)
{
  constexpr int W = 16 / sizeof(T);
  return cbase[cell] + (int64_t)(f / W) * gs + (int64_t)p * W + (f % W);
}

template <typename T, int n>
struct Shape
{
  T S[n][n];  // S[q][i]  = phi_i(x_q)          (nodal basis at Gauss points)
  T Dq[n][n]; // Dq[q][j] = l_j'(x_q)           (collocation derivative)
  T w[n];     // 1D Gauss weights on [0,1]
};

template <typename T, int dim, int n>
struct ApplyArgs
{
  const uint32_t *nodes;    // [cells][nq] node | cmask << 28
  const uint32_t *cell_geo; // GEO_GENERAL | index, or cartesian index
  const T        *geo_cart; // [dim + 1][n_cart]: invJ diagonal, det J
  int64_t         n_cart;
  const T        *geo_gen;  // [1 + dim*dim][n_gen * nq]: JxW, invJ[a][e]
  int64_t         gen_stride;
  const T        *tab;      // 16-byte field groups (tab_index)
  const int64_t  *tab_cbase;
  int64_t         tab_gs;
  int64_t         old_stride; // old_grad: [dim*dim + dim][plane][cell][line]
  const T        *cellwise; // [2][n_cells]
  int64_t         n_cells;
  const T        *old_grad; // [dim*dim + dim][n_cells * nq]
  T              *dst;
  const T        *src;
  int64_t         cell_begin, cell_end;
  T               nu, w0, theta;
  int             td, cw, have_prev, have_old_grad;
  int             diag_ndof;
  // DIAG with emat set: the whole column j of the element matrix instead of
  // its diagonal entry (MatrixFreeTools::compute_matrix, operator_ns.cc:
  // 1407-1430): emat[((cell - cell_begin) * ndof + j) * ndof + p * nc + c]
  T              *emat;
  Shape<T, n>     sh;
};

// ------------------------------------------------------------ helpers
template <typename T, int nc>
__device__ __forceinline__ void
load_node(const T *__restrict__ v, uint32_t node, T (&u)[nc])
{
#pragma unroll
  for (int c = 0; c < nc; ++c)
    u[c] = v[(size_t)node * nc + c];
}

template <>
__device__ __forceinline__ void
load_node<double, 4>(const double *__restrict__ v, uint32_t node, double (&u)[4])
{
  const double2 *p = reinterpret_cast<const double2 *>(v + (size_t)node * 4);
  const double2  a = p[0], b = p[1];
  u[0] = a.x, u[1] = a.y, u[2] = b.x, u[3] = b.y;
}

template <>
__device__ __forceinline__ void
load_node<float, 4>(const float *__restrict__ v, uint32_t node, float (&u)[4])
{
  const float4 a = *reinterpret_cast<const float4 *>(v + (size_t)node * 4);
  u[0] = a.x, u[1] = a.y, u[2] = a.z, u[3] = a.w;
}

template <typename T, int nc>
__device__ __forceinline__ void
store_node(T *__restrict__ v, uint32_t node, const T (&u)[nc])
{
#pragma unroll
  for (int c = 0; c < nc; ++c)
    v[(size_t)node * nc + c] = u[c];
}

template <>
__device__ __forceinline__ void
store_node<double, 4>(double *__restrict__ v, uint32_t node, const double (&u)[4])
{
  double2 *p = reinterpret_cast<double2 *>(v + (size_t)node * 4);
  p[0]       = make_double2(u[0], u[1]);
  p[1]       = make_double2(u[2], u[3]);
}

template <>
__device__ __forceinline__ void
store_node<float, 4>(float *__restrict__ v, uint32_t node, const float (&u)[4])
{
  *reinterpret_cast<float4 *>(v + (size_t)node * 4) = make_float4(u[0], u[1], u[2], u[3]);
}

// the same 4-value row as non-temporal 16-byte stores (the brick write-out
// under GLS_NT_STORE, an A/B build switch)
template <typename T>
__device__ __forceinline__ void
store_node_nt(T *__restrict__ v, uint32_t node, const T (&u)[4])
{
  typedef T V2 __attribute__((ext_vector_type(16 / sizeof(T))));
  V2 *p = reinterpret_cast<V2 *>(v + (size_t)node * 4);
  if constexpr (sizeof(T) == 8)
    {
      __builtin_nontemporal_store(V2{u[0], u[1]}, p);
      __builtin_nontemporal_store(V2{u[2], u[3]}, p + 1);
    }
  else
    __builtin_nontemporal_store(V2{u[0], u[1], u[2], u[3]}, p);
}

// 1D contraction along an axis with stride `s` (n points):
//   forward:   out[p] = sum_j M[pa][j] in[base + j s]
//   transpose: out[p] = sum_j M[j][pa] in[base + j s]
template <int n, bool TR, typename T>
__device__ __forceinline__ T
contract(const T *in, const T (*M)[n], int pa, int base, int s)
{
  T acc = 0;
#pragma unroll
  for (int j = 0; j < n; ++j)
    acc += (TR ? M[j][pa] : M[pa][j]) * in[base + j * s];
  return acc;
}

// q-wise stabilisation parameters, operator_ns.cc:407-420 (|U|^2 with the
// 1e-12 floor): the producer (tables) and the Newton brick kernel (on the
// fly from U and h) evaluate the same expression
template <typename T>
__device__ __forceinline__ void
delta_qwise(T u2, T h, T nu, T stau, T &d1, T &d2)
{
  const T umag2 = T(1e-12) + u2;
  const T fac   = T(4) * nu / (h * h);
  d1            = T(1) / sqrt(stau * stau + T(4) * umag2 / h / h + T(9) * fac * fac);
  d2            = sqrt(umag2) * h * T(0.5);
}

// the same delta_1 / delta_2 with hardware reciprocal / reciprocal square
// root estimates refined by Newton steps (two for FP64: ~1 ulp) instead of
// IEEE divisions and square roots: ~25 instead of ~55 VALU instructions per
// q point in the brick kernel; equal to delta_qwise to a few ulp
// (round 3: r2 FP64 -3.5 %, r3 FP64 -2 %, FP32 -2..3.5 % kernel time)
__device__ __forceinline__ double
nr_rcp(double x)
{
  double y = __builtin_amdgcn_rcp(x);
  y        = fma(y, fma(-x, y, 1.0), y);
  return fma(y, fma(-x, y, 1.0), y);
}
__device__ __forceinline__ double
nr_rsq(double x)
{
  double y = __builtin_amdgcn_rsq(x);
  double h = 0.5 * x;
  y        = y * fma(-h * y, y, 1.5);
  return y * fma(-h * y, y, 1.5);
}
__device__ __forceinline__ float
nr_rcp(float x)
{
  const float y = __builtin_amdgcn_rcpf(x);
  return fmaf(y, fmaf(-x, y, 1.0f), y);
}
__device__ __forceinline__ float
nr_rsq(float x)
{
  const float y = __builtin_amdgcn_rsqf(x);
  return y * fmaf(-0.5f * x * y, y, 1.5f);
}
// nu4 = 4 nu and stau2 = stau^2 come precomputed (bitwise the products the
// expression forms): as kernel arguments they stay scalar registers, where
// the products formed in the kernel became loop-invariant VGPRs that the
// 4-wave brick kernel had to spill
template <typename T>
__device__ __forceinline__ void
delta_qwise_fast(T u2, T h, T nu4, T stau2, T &d1, T &d2)
{
  const T umag2 = T(1e-12) + u2;
  const T ih    = nr_rcp(h);
  const T ih2   = ih * ih;
  const T fac   = nu4 * ih2;
  d1            = nr_rsq(stau2 + T(4) * umag2 * ih2 + T(9) * fac * fac);
  d2            = umag2 * nr_rsq(umag2) * h * T(0.5);
}

// ------------------------------------------------------------ q-point physics
// Newton increment branch (operator_ns.cc:1067-1181) with the
// linearization-point part of R1 precomputed: T1 = (td ? w0 U + Ut_old : 0)
// + grad P* + (grad U) U (k_finalize_t1), so R1 = delta_1 T1.  Same values as
// qpoint_physics<MODE_NEWTON>, fewer table loads and operations.
template <int dim, typename T>
__device__ __forceinline__ void
qpoint_newton_t1(const T *u, T p, const T (*gu)[dim], const T *gp, const T *U,
                 const T (*GU)[dim], const T *T1, T d1, T d2, T nu, T w0, int td, T *vr,
                 T (*gr)[dim])
{
  T ut[dim], sgu[dim], ugs[dim], divu = 0;
#pragma unroll
  for (int d = 0; d < dim; ++d)
    {
      ut[d] = u[d] * w0;
      divu += gu[d][d];
      sgu[d] = ugs[d] = 0;
#pragma unroll
      for (int e = 0; e < dim; ++e)
        {
          sgu[d] += gu[d][e] * U[e];
          ugs[d] += GU[d][e] * u[e];
        }
    }
#pragma unroll
  for (int d = 0; d < dim; ++d)
    {
      vr[d] = ut[d] + sgu[d] + ugs[d];
#pragma unroll
      for (int e = 0; e < dim; ++e)
        gr[d][e] = 0;
      gr[d][d] = gu[d][d] * (T(2) * nu) - p;
    }
#pragma unroll
  for (int e = 0; e < dim; ++e)
#pragma unroll
    for (int d = e + 1; d < dim; ++d)
      {
        const T tmp = (gu[d][e] + gu[e][d]) * nu; // symm_scalar_product_add :899-916
        gr[d][e] += tmp;
        gr[e][d] += tmp;
      }
  T r0[dim], r1[dim];
#pragma unroll
  for (int d = 0; d < dim; ++d)
    {
      r0[d] = d1 * ((td ? ut[d] : T(0)) + gp[d] + sgu[d] + ugs[d]);
      r1[d] = d1 * T1[d];
    }
#pragma unroll
  for (int d0 = 0; d0 < dim; ++d0)
#pragma unroll
    for (int e = 0; e < dim; ++e)
      gr[d0][e] += U[e] * r0[d0] + u[e] * r1[d0];
#pragma unroll
  for (int d = 0; d < dim; ++d)
    gr[d][d] += d2 * divu;
  vr[dim] = divu;
#pragma unroll
  for (int d = 0; d < dim; ++d)
    gr[dim][d] = r0[d];
}

// T1 = (td ? w0 U + Ut_old : 0) + grad P* + (grad U) U at every (cell, q)
// of the table (the linearization-point part of R1, operator_ns.cc:1146-1151)
template <int dim, typename T>
__global__ void __launch_bounds__(256)
  k_finalize_t1(T *__restrict__ tab, const int64_t *__restrict__ cbase, int64_t gs,
                int64_t n_cells, int nq, T w0, int td)
{
  using F         = Fields<dim>;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_cells * nq)
    return;
  const int64_t cell = g / nq;
  const int     p    = (int)(g - cell * nq);
  auto          TI   = [&](int f) { return tab_index<T>(cbase, gs, cell, p, f); };
  T             U[dim];
#pragma unroll
  for (int d = 0; d < dim; ++d)
    U[d] = tab[TI(F::U + d)];
#pragma unroll
  for (int d = 0; d < dim; ++d)
    {
      T s = tab[TI(F::GP + d)] + (td ? U[d] * w0 + tab[TI(F::UT + d)] : T(0));
#pragma unroll
      for (int e = 0; e < dim; ++e)
        s += tab[TI(F::GU + d * dim + e)] * U[e];
      tab[TI(F::T1 + d)] = s;
    }
}

// the H field (the cell's q-wise h) of every (cell, q): table uploads
template <int dim, typename T>
__global__ void __launch_bounds__(256)
  k_fill_h(T *__restrict__ tab, const int64_t *__restrict__ cbase, int64_t gs,
           const T *__restrict__ h_q, int64_t n_cells, int nq)
{
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_cells * nq)
    return;
  const int64_t cell = g / nq;
  const int     p    = (int)(g - cell * nq);
  tab[tab_index<T>(cbase, gs, cell, p, Fields<dim>::H)] = h_q[cell];
}

// do_vmult_cell, operator_ns.cc:949-1182; u/p/gu/gp are trial values and
// REAL-space gradients at the q point; output value / gradient coefficients
// (before JxW and J^{-T}).
template <int dim, typename T, int MODE>
__device__ __forceinline__ void
qpoint_physics(const T *u, T p, const T (*gu)[dim],
               const T *gp, const T *U, const T (*GU)[dim], const T *GP, const T *UT,
               const T *oldg, T d1, T d2, T nu, T w0, T theta, int td, int have_prev,
               int have_old_grad, T *vr, T (*gr)[dim])
{
#pragma unroll
  for (int c = 0; c <= dim; ++c)
    {
      vr[c] = 0;
#pragma unroll
      for (int e = 0; e < dim; ++e)
        gr[c][e] = 0;
    }
  if (MODE == MODE_NEWTON)
    {
      // Newton increment branch, operator_ns.cc:1067-1181
      T ut[dim], sgu[dim], ugs[dim], sgs[dim], divu = 0;
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          ut[d] = u[d] * w0;
          divu += gu[d][d];
          sgu[d] = ugs[d] = sgs[d] = 0;
#pragma unroll
          for (int e = 0; e < dim; ++e)
            {
              sgu[d] += gu[d][e] * U[e];
              ugs[d] += GU[d][e] * u[e];
              sgs[d] += GU[d][e] * U[e];
            }
        }
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          vr[d] = ut[d] + sgu[d] + ugs[d];
          gr[d][d] += gu[d][d] * (T(2) * nu) - p;
        }
#pragma unroll
      for (int e = 0; e < dim; ++e)
#pragma unroll
        for (int d = e + 1; d < dim; ++d)
          {
            const T tmp = (gu[d][e] + gu[e][d]) * nu;
            gr[d][e] += tmp;
            gr[e][d] += tmp;
          }
      T r0[dim], r1[dim];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          r0[d] = d1 * ((td ? ut[d] : T(0)) + gp[d] + sgu[d] + ugs[d]);
          r1[d] = d1 * ((td ? (U[d] * w0 + UT[d]) : T(0)) + GP[d] + sgs[d]);
        }
#pragma unroll
      for (int d0 = 0; d0 < dim; ++d0)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          gr[d0][e] += U[e] * r0[d0] + u[e] * r1[d0];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        gr[d][d] += d2 * divu;
      vr[dim] = divu;
#pragma unroll
      for (int d = 0; d < dim; ++d)
        gr[dim][d] = r0[d];
    }
  else
    {
      // fixed-point / residual branch, operator_ns.cc:955-1066
      const bool R = MODE == MODE_RESIDUAL;
      T          ut[dim], gb[dim][dim], gpb[dim];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          ut[d]  = u[d] * w0 + ((R && have_prev) ? UT[d] : T(0));
          gpb[d] = theta * gp[d];
#pragma unroll
          for (int e = 0; e < dim; ++e)
            gb[d][e] = theta * gu[d][e];
        }
      if (R && have_old_grad)
        {
#pragma unroll
          for (int d = 0; d < dim; ++d)
            {
#pragma unroll
              for (int e = 0; e < dim; ++e)
                gb[d][e] += (T(1) - theta) * oldg[d * dim + e];
              gpb[d] += (T(1) - theta) * oldg[dim * dim + d];
            }
        }
      T divb = 0, sgb[dim];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          divb += gb[d][d];
          sgb[d] = 0;
#pragma unroll
          for (int e = 0; e < dim; ++e)
            sgb[d] += gb[d][e] * U[e];
        }
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          vr[d] = ut[d] + sgb[d];
          gr[d][d] += gb[d][d] * (T(2) * nu) - p;
        }
#pragma unroll
      for (int e = 0; e < dim; ++e)
#pragma unroll
        for (int d = e + 1; d < dim; ++d)
          {
            const T tmp = (gb[d][e] + gb[e][d]) * nu;
            gr[d][e] += tmp;
            gr[e][d] += tmp;
          }
      T r0[dim];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        r0[d] = d1 * ((td ? ut[d] : T(0)) + gpb[d] + sgb[d]);
#pragma unroll
      for (int d0 = 0; d0 < dim; ++d0)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          gr[d0][e] += U[e] * r0[d0];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        gr[d][d] += d2 * divb;
      vr[dim] = divb;
#pragma unroll
      for (int d = 0; d < dim; ++d)
        gr[dim][d] = d1 * ((td ? ut[d] : T(0)) + gp[d] + sgb[d]);
    }
}

// ------------------------------------------------------------ geometry
template <int dim, int n, typename T>
struct QGeo
{
  T JxW;
  T inv[dim][dim]; // d xi_a / d x_e
};

template <int dim, int n, typename T, typename Args>
__device__ __forceinline__ void
load_geometry(const Args &a, int64_t cell, int p, int px, int py, int pz,
              const T *sw, QGeo<dim, n, T> &g)
{
  constexpr int  nq = ipow(n, dim);
  const uint32_t cg = a.cell_geo[cell];
  if (cg & GEO_GENERAL)
    {
      const int64_t idx = qindex<dim, n>(cg & ~GEO_GENERAL, p, a.gen_stride / nq);
      g.JxW             = a.geo_gen[idx];
#pragma unroll
      for (int i = 0; i < dim; ++i)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          g.inv[i][e] = a.geo_gen[(1 + i * dim + e) * a.gen_stride + idx];
    }
  else
    {
      const int64_t idx = cg;
#pragma unroll
      for (int i = 0; i < dim; ++i)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          g.inv[i][e] = (i == e) ? a.geo_cart[i * a.n_cart + idx] : T(0);
      T w = sw[px] * sw[py];
      if (dim == 3)
        w *= sw[pz];
      g.JxW = a.geo_cart[dim * a.n_cart + idx] * w;
    }
}

// ------------------------------------------------------------ apply kernel
// Wave-local cell packing: each wavefront owns CPW = 64 / (k+1)^dim whole
// cells (3D Q2: 2 cells = 54 lanes), so every sum-factorisation exchange is
// ordered by a wavefront-scope fence instead of a workgroup barrier.  The
// per-q tables and geometry are loaded into registers right after the
// gather, so their HBM latency overlaps the evaluate sweeps.
__device__ __forceinline__ void
wave_sync()
{
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// MODE: Newton / fixed-point vmult or residual.  DIAG: each virtual cell is
// (cell, local dof j) with a unit-vector input; only the diagonal entry is
// accumulated (MatrixFreeTools::compute_diagonal, operator_ns.cc:209-218).
template <int dim, int k, typename T, int MODE, bool DIAG>
__global__ void __launch_bounds__(BLOCK)
  k_apply(ApplyArgs<T, dim, k + 1> a)
{
  constexpr int n    = k + 1;
  constexpr int nq   = ipow(n, dim);
  constexpr int nc   = dim + 1;
  constexpr int CPW  = 64 / nq > 0 ? 64 / nq : 1;
  constexpr int WPB  = BLOCK / 64;
  constexpr int CPB  = CPW * WPB;
  constexpr int LDSC = nc * nq * (dim > 2 ? dim : 2);
  using F            = Fields<dim>;
  static_assert(nq <= 64, "one cell must fit a wavefront");

  __shared__ T smem[CPB * LDSC];
  __shared__ T sS[n][n], sD[n][n], sw[n];

  const int t = threadIdx.x;
  if (t < n * n)
    {
      sS[t / n][t % n] = a.sh.S[t / n][t % n];
      sD[t / n][t % n] = a.sh.Dq[t / n][t % n];
    }
  if (t < n)
    sw[t] = a.sh.w[t];

  const int     wave    = t >> 6;
  const int     lane    = t & 63;
  const int     slot    = lane / nq;
  const int     p       = lane - slot * nq;
  const bool    in_wave = slot < CPW;
  const int     lc      = wave * CPW + (in_wave ? slot : 0);
  const int64_t vcell   = (int64_t)blockIdx.x * CPB + lc;
  int64_t       cell;
  int           jdiag = 0;
  if (DIAG)
    {
      cell  = a.cell_begin + vcell / a.diag_ndof;
      jdiag = (int)(vcell % a.diag_ndof);
    }
  else
    cell = a.cell_begin + vcell;
  const bool active = in_wave && cell < a.cell_end;
  T         *A      = smem + lc * LDSC;
  T         *B      = A + nc * nq;
  const int  px     = p % n;
  const int  py     = (p / n) % n;
  const int  pz     = dim == 3 ? p / (n * n) : 0;
  const int  pa[3]  = {px, py, pz};
  const int  st[3]  = {1, n, n * n};

  // ---- gather (read_dof_values / read_dof_values_plain)
  uint32_t node = 0, cm = 0;
  T        u[nc];
#pragma unroll
  for (int c = 0; c < nc; ++c)
    u[c] = 0;
  if (active)
    {
      const uint32_t packed = a.nodes[cell * nq + p];
      node                  = packed & NODE_MASK;
      cm                    = packed >> 28;
      if (!DIAG)
        load_node<T, nc>(a.src, node, u);
    }

  // ---- prefetch geometry and per-q tables (consumed after evaluate)
  const int64_t   q  = qindex<dim, n>(cell, p, a.n_cells);
  const int64_t   ts = a.old_stride;
  const int64_t   tb = active ? a.tab_cbase[cell] + (int64_t)p * (16 / sizeof(T)) : 0;
  constexpr int   TW = 16 / sizeof(T);
  auto            TI = [&](int f) { return tb + (int64_t)(f / TW) * a.tab_gs + f % TW; };
  QGeo<dim, n, T> g;
  T               U[dim], GU[dim][dim], GP[dim], UT[dim], oldg[dim * dim + dim], d1 = 0, d2 = 0;
  g.JxW = 0;
#pragma unroll
  for (int i = 0; i < dim; ++i)
    {
#pragma unroll
      for (int e = 0; e < dim; ++e)
        {
          g.inv[i][e] = 0;
          GU[i][e]    = 0;
        }
      U[i] = GP[i] = UT[i] = 0;
    }
#pragma unroll
  for (int i = 0; i < dim * dim + dim; ++i)
    oldg[i] = 0;
  if (active)
    {
      const uint32_t cg = a.cell_geo[cell];
      if (cg & GEO_GENERAL)
        {
          const int64_t idx = qindex<dim, n>(cg & ~GEO_GENERAL, p, a.gen_stride / nq);
          g.JxW             = a.geo_gen[idx];
#pragma unroll
          for (int i = 0; i < dim; ++i)
#pragma unroll
            for (int e = 0; e < dim; ++e)
              g.inv[i][e] = a.geo_gen[(1 + i * dim + e) * a.gen_stride + idx];
        }
      else
        {
#pragma unroll
          for (int i = 0; i < dim; ++i)
            g.inv[i][i] = a.geo_cart[i * a.n_cart + cg];
          g.JxW = a.geo_cart[dim * a.n_cart + cg]; // det J, times weight below
        }
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          U[d] = a.tab[TI(F::U + d)];
          if (MODE == MODE_NEWTON)
            {
#pragma unroll
              for (int e = 0; e < dim; ++e)
                GU[d][e] = a.tab[TI(F::GU + d * dim + e)];
              GP[d] = a.tab[TI(F::GP + d)];
            }
          if ((MODE == MODE_NEWTON && a.td) || (MODE == MODE_RESIDUAL && a.have_prev))
            UT[d] = a.tab[TI(F::UT + d)];
        }
      if (MODE == MODE_RESIDUAL && a.have_old_grad)
#pragma unroll
        for (int i = 0; i < dim * dim + dim; ++i)
          oldg[i] = a.old_grad[i * ts + q];
      if (a.cw)
        {
          d1 = a.cellwise[cell];
          d2 = a.cellwise[a.n_cells + cell];
        }
      else
        {
          d1 = a.tab[TI(F::D1)];
          d2 = a.tab[TI(F::D2)];
        }
      if (!(cg & GEO_GENERAL))
        {
          T w = 1;
#pragma unroll
          for (int d = 0; d < dim; ++d)
            w *= a.sh.w[pa[d]];
          g.JxW *= w;
        }
    }
  if (DIAG)
    {
#pragma unroll
      for (int c = 0; c < nc; ++c)
        u[c] = (active && p == jdiag / nc && c == jdiag % nc) ? T(1) : T(0);
    }
  else if (MODE != MODE_RESIDUAL)
    {
#pragma unroll
      for (int c = 0; c < nc; ++c)
        if ((cm >> c) & 1)
          u[c] = 0;
    }
  __syncthreads(); // shape tables in LDS
  if (in_wave)
#pragma unroll
    for (int c = 0; c < nc; ++c)
      A[c * nq + p] = u[c];
  wave_sync();

  // ---- evaluate: values at q (dim sweeps with S)
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
        gref[c][ax] = contract<n, false>(in + c * nq, sD, pa[ax], p - pa[ax] * st[ax], st[ax]);
    }
  wave_sync();

  // ---- q-point physics
  T gu[dim][dim], gp[dim];
#pragma unroll
  for (int c = 0; c < nc; ++c)
#pragma unroll
    for (int e = 0; e < dim; ++e)
      {
        T s = 0;
#pragma unroll
        for (int i = 0; i < dim; ++i)
          s += g.inv[i][e] * gref[c][i];
        if (c < dim)
          gu[c][e] = s;
        else
          gp[e] = s;
      }
  T vr[nc], gr[nc][dim];
  qpoint_physics<dim, T, MODE>(val, val[dim], gu, gp, U, GU, GP, UT, oldg, d1, d2, a.nu, a.w0,
                               a.theta, a.td, a.have_prev, a.have_old_grad, vr, gr);
  // submit_value / submit_gradient (JxW, J^{-T}); inactive lanes have JxW 0
  T vhat[nc];
#pragma unroll
  for (int c = 0; c < nc; ++c)
    {
      vhat[c] = vr[c] * g.JxW;
#pragma unroll
      for (int i = 0; i < dim; ++i)
        {
          T s = 0;
#pragma unroll
          for (int e = 0; e < dim; ++e)
            s += g.inv[i][e] * gr[c][e];
          if (in_wave)
            A[(c * dim + i) * nq + p] = s * g.JxW;
        }
    }
  wave_sync();
  // ---- integrate: gradient part via Dq^T, then S^T sweeps
  T wq[nc];
#pragma unroll
  for (int c = 0; c < nc; ++c)
    {
      T s = vhat[c];
#pragma unroll
      for (int ax = 0; ax < dim; ++ax)
        s += contract<n, true>(A + (c * dim + ax) * nq, sD, pa[ax], p - pa[ax] * st[ax], st[ax]);
      wq[c] = s;
    }
  wave_sync();
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

  // ---- scatter (distribute_local_to_global, constrained dofs skipped)
  if (!active)
    return;
  if (DIAG && a.emat)
    {
      T *col = a.emat + ((size_t)(cell - a.cell_begin) * a.diag_ndof + jdiag) * a.diag_ndof;
#pragma unroll
      for (int c = 0; c < nc; ++c)
        col[p * nc + c] = in[c * nq + p];
    }
  else if (DIAG)
    {
      const int c = jdiag % nc;
      if (p == jdiag / nc && !((cm >> c) & 1))
        unsafeAtomicAdd(a.dst + (size_t)node * nc + c, in[c * nq + p]);
    }
  else
    {
#pragma unroll
      for (int c = 0; c < nc; ++c)
        if (!((cm >> c) & 1))
          {
            const T r = in[c * nq + p];
            unsafeAtomicAdd(a.dst + (size_t)node * nc + c, MODE == MODE_RESIDUAL ? -r : r);
          }
    }
}

// ------------------------------------------------------------ producers
// set_linearization_point (operator_ns.cc:570-620) fused with
// compute_penalty_parameters (:322-421): u*, grad u*, grad p* at q and the
// q-wise / cell-wise delta_1, delta_2.
template <typename T, int dim, int n>
struct ProducerArgs
{
  const uint32_t *nodes;
  const uint32_t *cell_geo;
  const T        *geo_cart;
  int64_t         n_cart;
  const T        *geo_gen;
  int64_t         gen_stride;
  T              *tab;
  const int64_t  *tab_cbase;
  int64_t         tab_gs;
  int64_t         old_stride;
  T              *cellwise;
  int64_t         n_cells;
  T              *old_grad;
  const T        *vec;
  const T        *h_q;   // [n_cells] (6|K|/pi)^(1/3)/k or sqrt(4|K|/pi)/k
  const T        *h_min; // [n_cells] minimum vertex distance
  T               nu, c1, c2, stau;
  int             what; // 0: linearization point, 1: Ut_old, 2: old gradients
  Shape<T, n>     sh;
};

template <int dim, int k, typename T>
__global__ void __launch_bounds__(BLOCK)
  k_produce(ProducerArgs<T, dim, k + 1> a)
{
  constexpr int n    = k + 1;
  constexpr int nq   = ipow(n, dim);
  constexpr int nc   = dim + 1;
  constexpr int CPB  = BLOCK / nq;
  constexpr int LDSC = 2 * nc * nq;
  using F            = Fields<dim>;

  __shared__ T smem[CPB * LDSC];
  __shared__ T sS[n][n], sD[n][n], sw[n];
  __shared__ T umax[CPB];

  const int t = threadIdx.x;
  if (t < n * n)
    {
      sS[t / n][t % n] = a.sh.S[t / n][t % n];
      sD[t / n][t % n] = a.sh.Dq[t / n][t % n];
    }
  if (t < n)
    sw[t] = a.sh.w[t];
  const int     lc       = t / nq;
  const int     p        = t - lc * nq;
  const bool    in_block = lc < CPB;
  const int64_t cell     = (int64_t)blockIdx.x * CPB + lc;
  const bool    active   = in_block && cell < a.n_cells;
  T            *A        = smem + (in_block ? lc : 0) * LDSC;
  T            *B        = A + nc * nq;
  const int     px = p % n, py = (p / n) % n, pz = dim == 3 ? p / (n * n) : 0;
  const int     pa[3] = {px, py, pz};
  const int     st[3] = {1, n, n * n};

  T u[nc];
#pragma unroll
  for (int c = 0; c < nc; ++c)
    u[c] = 0;
  if (active)
    load_node<T, nc>(a.vec, a.nodes[cell * nq + p] & NODE_MASK, u); // read plain
  if (in_block)
#pragma unroll
    for (int c = 0; c < nc; ++c)
      A[c * nq + p] = u[c];
  __syncthreads();
  T *in = A, *out = B;
#pragma unroll
  for (int ax = 0; ax < dim; ++ax)
    {
      if (in_block)
#pragma unroll
        for (int c = 0; c < nc; ++c)
          out[c * nq + p] =
            contract<n, false>(in + c * nq, sS, pa[ax], p - pa[ax] * st[ax], st[ax]);
      __syncthreads();
      T *tmp = in;
      in     = out;
      out    = tmp;
    }
  T val[nc], gref[nc][dim];
  if (in_block)
#pragma unroll
    for (int c = 0; c < nc; ++c)
      {
        val[c] = in[c * nq + p];
#pragma unroll
        for (int ax = 0; ax < dim; ++ax)
          gref[c][ax] = contract<n, false>(in + c * nq, sD, pa[ax], p - pa[ax] * st[ax], st[ax]);
      }
  const int64_t q  = qindex<dim, n>(cell, p, a.n_cells);
  const int64_t ts = a.old_stride;
  constexpr int TW = 16 / sizeof(T);
  const int64_t tb = active ? a.tab_cbase[cell] + (int64_t)p * TW : 0;
  auto          TI = [&](int f) { return tb + (int64_t)(f / TW) * a.tab_gs + f % TW; };
  T             unorm = 0;
  if (active)
    {
      if (a.what == 1)
        {
          // set_previous_solution: u_time_derivative_old (:262-271)
#pragma unroll
          for (int d = 0; d < dim; ++d)
            a.tab[TI(F::UT + d)] = val[d];
        }
      else
        {
          QGeo<dim, n, T> g;
          ApplyArgs<T, dim, n> ga;
          ga.cell_geo   = a.cell_geo;
          ga.geo_cart   = a.geo_cart;
          ga.n_cart     = a.n_cart;
          ga.geo_gen    = a.geo_gen;
          ga.gen_stride = a.gen_stride;
          load_geometry<dim, n, T>(ga, cell, p, px, py, pz, sw, g);
          T gr[nc][dim];
#pragma unroll
          for (int c = 0; c < nc; ++c)
#pragma unroll
            for (int e = 0; e < dim; ++e)
              {
                T s = 0;
#pragma unroll
                for (int i = 0; i < dim; ++i)
                  s += g.inv[i][e] * gref[c][i];
                gr[c][e] = s;
              }
          if (a.what == 2)
            {
              // theta != 1: u_old_gradient, p_old_gradient (:273-316)
#pragma unroll
              for (int d = 0; d < dim; ++d)
                {
#pragma unroll
                  for (int e = 0; e < dim; ++e)
                    a.old_grad[(d * dim + e) * ts + q] = gr[d][e];
                  a.old_grad[(dim * dim + d) * ts + q] = gr[dim][d];
                }
            }
          else
            {
              T u2 = 0;
#pragma unroll
              for (int d = 0; d < dim; ++d)
                {
                  a.tab[TI(F::U + d)] = val[d];
#pragma unroll
                  for (int e = 0; e < dim; ++e)
                    a.tab[TI(F::GU + d * dim + e)] = gr[d][e];
                  a.tab[TI(F::GP + d)] = gr[dim][d];
                  u2 += val[d] * val[d];
                }
              unorm = sqrt(u2);
              // q-wise stabilisation, operator_ns.cc:394-420
              const T h = a.h_q[cell];
              T       d1, d2;
              delta_qwise(u2, h, a.nu, a.stau, d1, d2);
              a.tab[TI(F::D1)] = d1;
              a.tab[TI(F::D2)] = d2;
              a.tab[TI(F::H)]  = h;
            }
        }
    }
  if (a.what != 0)
    return;
  // cell-wise stabilisation (:365-388): u_max over the cell's q points
  __syncthreads();
  if (in_block)
    A[p] = unorm;
  __syncthreads();
  if (active && p == 0)
    {
      T m = 0;
      for (int i = 0; i < nq; ++i)
        m = A[i] > m ? A[i] : m;
      umax[lc]  = m;
      const T h = a.h_min[cell];
      T       d1, d2;
      if (a.nu < h)
        {
          d1 = a.c1 / sqrt(a.stau * a.stau + m * m / (h * h));
          d2 = a.c2 * h;
        }
      else
        {
          d1 = a.c1 * h * h;
          d2 = a.c2 * h * h;
        }
      a.cellwise[cell]             = d1;
      a.cellwise[a.n_cells + cell] = d2;
    }
}

// ------------------------------------------------------------ vector kernels
// dst[i] = constrained(i) ? src[i] : 0 (owned), 0 (ghost)  — cell_loop's
// zero_dst plus the identity rows of vmult (operator_ns.cc:719-721)
template <typename T>
__global__ void
k_init_dst(T *__restrict__ dst, const T *__restrict__ src, const uint32_t *__restrict__ cbits,
           int64_t n_owned, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  T v = 0;
  if (i < n_owned && ((cbits[i >> 5] >> (i & 31)) & 1))
    v = src[i];
  dst[i] = v;
}

// dst[i] = src[i] on constrained owned dofs only (identity rows re-applied
// after the ghost export-add of a distributed vmult)
template <typename T>
__global__ void
k_identity_rows(T *__restrict__ dst, const T *__restrict__ src,
                const uint32_t *__restrict__ cbits, int64_t n_owned)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_owned && ((cbits[i >> 5] >> (i & 31)) & 1))
    dst[i] = src[i];
}

template <typename T>
__global__ void
k_fill(T *__restrict__ dst, T v, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    dst[i] = v;
}

// y = sum_j w_j x_j (j < 4)
template <typename T>
__global__ void
k_lincomb(T *__restrict__ y, const T *x0, const T *x1, const T *x2, const T *x3, double w0,
          double w1, double w2, double w3, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  T s = 0;
  if (x0)
    s += T(w0) * x0[i];
  if (x1)
    s += T(w1) * x1[i];
  if (x2)
    s += T(w2) * x2[i];
  if (x3)
    s += T(w3) * x3[i];
  y[i] = s;
}

// compute_inverse_diagonal finalisation (:220-224): constrained -> 1, then
// d <- |d| > 1e-10 ? 1/d : 1
// compute_inverse_diagonal (operator_ns.cc:195-225) by direct evaluation of
// the element-matrix diagonal: for the test/trial function phi_i e_c the cell
// operator (do_vmult_cell<false>, Newton :1067-1181 or fixed point
// :955-1066) is linear in the trial, and its c-th test row needs only the
// c-th output row, so
//   A_ii = sum_q JxW [V_c(phi_i e_c) phi_i + Gr_c(phi_i e_c) . grad phi_i]
// with (trial u = phi e_c, grad u = e_c (x) grad phi):
//   Newton  V_c = w0 phi + U.grad phi + phi dU_c/dx_c
//           Gr_c = nu (grad phi + e_c d_c phi) + U R0_c + e_c phi R1_c
//                  + e_c delta_2 d_c phi,
//           R0_c = delta_1 ((td ? w0 phi : 0) + U.grad phi + phi dU_c/dx_c)
//   fixed   V_c = w0 phi + theta U.grad phi
//           Gr_c = nu theta (grad phi + e_c d_c phi) + U R0_c
//                  + e_c delta_2 theta d_c phi,
//           R0_c = delta_1 ((td ? w0 phi : 0) + theta U.grad phi)
//   pressure (both): Gr_p = delta_1 grad phi, V_p = 0
// (R1 = delta_1 ((td ? w0 U + Ut_old : 0) + grad P* + (grad U) U), the
// trial-independent SUPG residual).  Instead of MatrixFreeTools::
// compute_diagonal's dpc unit-vector cell applies (and this library's former
// k_apply<DIAG>: one full q-point physics per (dof, q)): phase 1 stages the
// per-q data of the workgroup's cells in LDS (one lane per (cell, q)),
// phase 2 runs one lane per (cell, node) over the q points.  The result is
// assembled with atomics like distribute_local_to_global (constrained
// components skipped), then k_invert_diag.
template <typename T, int dim, int n>
struct DiagArgs
{
  ApplyArgs<T, dim, n> a;
  T                    D[n][n]; // D[q][i] = phi_i'(x_q) (nodal basis derivative)
  double              *diag;    // [n_dofs] FP64 accumulator (both precisions)
  // deterministic assembly: the cells of one colour (null: all cells)
  const int32_t       *cells  = nullptr;
  int64_t              n_list = 0;
};

template <int dim, int k, typename T, int MODE>
__global__ void __launch_bounds__(BLOCK)
  k_diag(DiagArgs<T, dim, k + 1> da)
{
  constexpr int n   = k + 1;
  constexpr int nq  = ipow(n, dim);
  constexpr int nc  = dim + 1;
  constexpr int CPW = 64 / nq > 0 ? 64 / nq : 1;
  constexpr int CPB = CPW * (BLOCK / 64);
  // per (cell, q): JxW, inv (dim^2), U (dim), diag grad U (dim), R1 (dim), d1, d2
  constexpr int QF = 1 + dim * dim + 3 * dim + 2;
  using F          = Fields<dim>;
  const auto &a    = da.a;
  __shared__ T sq[CPB][nq][QF];
  __shared__ T sS[n][n], sDn[n][n];

  const int t = threadIdx.x;
  if (t < n * n)
    {
      sS[t / n][t % n]  = a.sh.S[t / n][t % n];
      sDn[t / n][t % n] = da.D[t / n][t % n];
    }
  const int     wave    = t >> 6, lane = t & 63;
  const int     slot    = lane / nq;
  const int     p       = lane - slot * nq;
  const bool    in_wave = slot < CPW;
  const int     lc      = wave * CPW + (in_wave ? slot : 0);
  const int64_t idx     = (int64_t)blockIdx.x * CPB + lc;
  const int64_t cell    = da.cells ? (idx < da.n_list ? (int64_t)da.cells[idx] : 0) : idx;
  const bool    active  = in_wave && (da.cells ? idx < da.n_list : cell < a.cell_end);
  const int     pa[3]   = {p % n, (p / n) % n, dim == 3 ? p / (n * n) : 0};
  if (active)
    {
      // phase 1: the q point's data
      QGeo<dim, n, T> g;
      load_geometry<dim, n, T>(a, cell, p, pa[0], pa[1], pa[2], a.sh.w, g);
      constexpr int TW = 16 / sizeof(T);
      const int64_t tb = a.tab_cbase[cell] + (int64_t)p * TW;
      auto          TI = [&](int f) { return tb + (int64_t)(f / TW) * a.tab_gs + f % TW; };
      T             U[dim], d1, d2;
#pragma unroll
      for (int d = 0; d < dim; ++d)
        U[d] = a.tab[TI(F::U + d)];
      if (a.cw)
        {
          d1 = a.cellwise[cell];
          d2 = a.cellwise[a.n_cells + cell];
        }
      else
        {
          d1 = a.tab[TI(F::D1)];
          d2 = a.tab[TI(F::D2)];
        }
      T *qd = sq[lc][p];
      qd[0] = g.JxW;
#pragma unroll
      for (int i = 0; i < dim * dim; ++i)
        qd[1 + i] = g.inv[i / dim][i % dim];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          qd[1 + dim * dim + d] = U[d];
          T gdiag = 0, r1 = 0;
          if (MODE == MODE_NEWTON)
            {
              gdiag = a.tab[TI(F::GU + d * dim + d)];
              r1    = a.tab[TI(F::GP + d)] + (a.td ? U[d] * a.w0 + a.tab[TI(F::UT + d)] : T(0));
#pragma unroll
              for (int e = 0; e < dim; ++e)
                r1 += a.tab[TI(F::GU + d * dim + e)] * U[e];
              r1 *= d1;
            }
          qd[1 + dim * dim + dim + d]     = gdiag;
          qd[1 + dim * dim + 2 * dim + d] = r1;
        }
      qd[QF - 2] = d1;
      qd[QF - 1] = d2;
    }
  __syncthreads();
  if (!active)
    return;
  // phase 2: lane = (cell, node i); the diagonal entries of its nc dofs
  const int ia[3] = {pa[0], pa[1], pa[2]};
  // phase 2 in FP64 for both precisions (the FP32 level operators' diagonals
  // feed the smoother's D^{-1}: summed in FP64, rounded once)
  using R = double;
  R     acc[nc];
#pragma unroll
  for (int c = 0; c < nc; ++c)
    acc[c] = 0;
  const R nu = a.nu, w0 = a.w0, th = MODE == MODE_NEWTON ? R(1) : R(a.theta);
  for (int q = 0; q < nq; ++q)
    {
      const int qa[3] = {q % n, (q / n) % n, dim == 3 ? q / (n * n) : 0};
      R         phi = R(1), gref[dim];
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          phi *= sS[qa[d]][ia[d]];
          R gd = R(1);
#pragma unroll
          for (int e = 0; e < dim; ++e)
            gd *= e == d ? sDn[qa[e]][ia[e]] : sS[qa[e]][ia[e]];
          gref[d] = gd;
        }
      const T *qd = sq[lc][q];
      R        gp[dim]; // real-space grad phi = J^{-T} grad_ref phi
#pragma unroll
      for (int e = 0; e < dim; ++e)
        {
          R s = 0;
#pragma unroll
          for (int i = 0; i < dim; ++i)
            s += qd[1 + i * dim + e] * gref[i];
          gp[e] = s;
        }
      const R  JxW = qd[0], d1 = qd[QF - 2], d2 = qd[QF - 1];
      const T *U   = qd + 1 + dim * dim;
      R        ugp = 0, gg = 0;
#pragma unroll
      for (int e = 0; e < dim; ++e)
        {
          ugp += U[e] * gp[e];
          gg += gp[e] * gp[e];
        }
#pragma unroll
      for (int c = 0; c < dim; ++c)
        {
          const R gdiag = MODE == MODE_NEWTON ? R(qd[1 + dim * dim + dim + c]) : R(0);
          const R r1    = MODE == MODE_NEWTON ? R(qd[1 + dim * dim + 2 * dim + c]) : R(0);
          const R adv   = th * ugp + phi * gdiag; // (U.grad) u + (u.grad) U, c-th entry
          const R Vc    = w0 * phi + adv;
          const R R0c   = d1 * ((a.td ? w0 * phi : R(0)) + adv);
          // Gr_c . grad phi
          const R grc = nu * th * (gg + gp[c] * gp[c]) + R0c * ugp + phi * r1 * gp[c] +
                        d2 * th * gp[c] * gp[c];
          acc[c] += JxW * (Vc * phi + grc);
        }
      acc[dim] += JxW * d1 * gg;
    }
  // distribute_local_to_global of the diagonal (constrained components skipped)
  const uint32_t packed = a.nodes[cell * nq + p];
  const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
#pragma unroll
  for (int c = 0; c < nc; ++c)
    if (!((cm >> c) & 1))
      unsafeAtomicAdd(da.diag + (size_t)node * nc + c, acc[c]);
}

// the assembled (not inverted) diagonal in the operator's precision, the
// identity rows' 1 on constrained owned components (partitioned operators:
// the ghost partials are added to their owners before the inversion)
template <typename T>
__global__ void
k_diag_out(T *__restrict__ out, const double *__restrict__ d, const uint32_t *__restrict__ cbits,
           int64_t n_owned, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  double v = d[i];
  if (i < n_owned && ((cbits[i >> 5] >> (i & 31)) & 1))
    v = 1;
  out[i] = (T)v;
}

// inverse of an FP64-assembled diagonal into the operator's precision
template <typename T>
__global__ void
k_invert_diag64(T *__restrict__ out, const double *__restrict__ d, const uint32_t *__restrict__ cbits,
                int64_t n_owned, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  double v = d[i];
  if (i < n_owned && ((cbits[i >> 5] >> (i & 31)) & 1))
    v = 1;
  out[i] = (T)((fabs(v) > 1.0e-10) ? 1.0 / v : 1.0);
}

template <typename T>
__global__ void
k_invert_diag(T *__restrict__ d, const uint32_t *__restrict__ cbits, int64_t n_owned, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  T v = d[i];
  if (i < n_owned && ((cbits[i >> 5] >> (i & 31)) & 1))
    v = 1;
  d[i] = (fabs((double)v) > 1.0e-10) ? T(1) / v : T(1);
}

} // namespace gls
