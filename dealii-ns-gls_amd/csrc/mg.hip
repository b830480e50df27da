// mg.hip — geometric multigrid on the GPU: level transfer (MGTwoLevelTransfer
// semantics, main.cc:538-563), damped-Jacobi relaxation smoother with a
// power-iteration relaxation factor (PreconditionRelaxation with
// relaxation = 0, multigrid.cc:281-369 — NOT Chebyshev), and the
// V-cycle of PreconditionMG / Multigrid (multigrid.cc:202-220, 534-548).
//
// Transfer between level l-1 (coarse) and l (fine), per coarse cell, with
// P the 1D interpolation of the parent's Q_k basis to the (2k+1) child
// lattice points:
//   prolongate_add: dst_f += w_f * (P x P x P) (Z_c src_c)
//   restrict_add:   dst_c += Z_c (P x P x P)^T (w_f * src_f)
// Z_c zeroes constrained coarse dofs, w_f = 1/valence on unconstrained fine
// dofs and 0 on constrained ones; interpolate = nodal injection (nested GLL
// nodes, k <= 2).
#include "../../include/gls_op.h"
#include "common.h"
#include "kernels.h"
#include "op_internal.h"
#include "cgs.h"
#include "trace.h"

#include <chrono>
#include <string>

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

using namespace gls;

namespace
{
constexpr int MAXP = 2 * 3 + 1; // (2k+1) for k <= 3
constexpr int MAXN = 4;
constexpr uint32_t NOT_OWNER = 0x80000000u;

template <typename T>
struct TransferArgs
{
  const uint32_t *coarse_nodes; // [cells_c][nq] node | cmask << 28
  const uint32_t *child;        // [cells_c][nl] fine node ids | NOT_OWNER: every fine
                                // node is owned by one entry (its first coarse cell)
  const T        *weight;       // [n_dofs_f]
  int64_t         n_cells_c;
  T               P[MAXP][MAXN];
  // restriction of a residual whose shared-node reduction is still pending
  // (v_step, FP32 3D brick levels; null: src complete): the fine node's
  // shared index, the residual apply's slots and classes, its src x and b
  const int32_t  *q_index   = nullptr;
  const uint32_t *q_nodes   = nullptr; // shared node | cmask << 28
  const T        *q_slots   = nullptr;
  const T        *q_x       = nullptr;
  const T        *q_b       = nullptr;
  gls::ReduceClasses q_rc{};
  // prolongation of a coarse solution whose last smoothing step's reduction
  // is pending: the coarse node's shared index, that step's slots, its src
  // (the iterate before), b, d (null: 1) and omega
  const int32_t  *p_index   = nullptr;
  const T        *p_slots   = nullptr;
  const T        *p_prev    = nullptr;
  const T        *p_b       = nullptr;
  const T        *p_d       = nullptr;
  T               p_omega   = T(0);
  gls::ReduceClasses p_rc{};
  // deterministic restriction (GLS_DETERMINISTIC): the coarse cells of one
  // colour, one workgroup each (null: workgroup c = coarse cell c)
  const int32_t  *cells     = nullptr;
};

// the relaxation step x_prev + omega d (b - A x_prev) at shared coarse node s
// from the step's partial slots, in k_shared_reduce_cls's order and
// arithmetic (bitwise its result; constrained components keep x_prev)
template <typename T>
__device__ __forceinline__ typename gls::Pack<T>::V
rebuild_relax(const TransferArgs<T> &a, uint32_t s, uint32_t node, uint32_t cm)
{
  using V        = typename gls::Pack<T>::V;
  constexpr int W = gls::Pack<T>::W;
  int           k = 0;
#pragma unroll
  for (int j = 1; j < gls::ReduceClasses::MAX; ++j)
    if (j < a.p_rc.n && s >= a.p_rc.first[j])
      k = j;
  const uint32_t m   = a.p_rc.mult[k];
  const uint32_t b0  = a.p_rc.slot0[k] + (s - a.p_rc.first[k]) * m;
  const V       *pp  = reinterpret_cast<const V *>(a.p_slots);
  V              sum = {};
  uint32_t       i   = 0;
  for (; i + 4 <= m; i += 4)
    {
      const V x0 = pp[b0 + i], x1 = pp[b0 + i + 1], x2 = pp[b0 + i + 2], x3 = pp[b0 + i + 3];
      sum += (x0 + x1) + (x2 + x3);
    }
  if (i + 2 <= m)
    {
      const V x0 = pp[b0 + i], x1 = pp[b0 + i + 1];
      sum += x0 + x1;
      i += 2;
    }
  if (i < m)
    sum += pp[b0 + i];
  const V xs = reinterpret_cast<const V *>(a.p_prev)[node];
  if (cm)
#pragma unroll
    for (int w = 0; w < W; ++w)
      if ((cm >> w) & 1)
        sum[w] = xs[w];
  const V dj = a.p_d ? reinterpret_cast<const V *>(a.p_d)[node] : V{} + T(1);
  return xs + a.p_omega * dj * (reinterpret_cast<const V *>(a.p_b)[node] - sum);
}

// the residual b - A x of shared fine node s from the residual apply's
// partial slots, in k_shared_reduce_cls's order and arithmetic (bitwise its
// result: keep 0, omega 1, d 1; constrained components b - x)
template <typename T>
__device__ __forceinline__ typename gls::Pack<T>::V
rebuild_residual(const TransferArgs<T> &a, uint32_t s)
{
  using V        = typename gls::Pack<T>::V;
  constexpr int W = gls::Pack<T>::W;
  int           k = 0;
#pragma unroll
  for (int j = 1; j < gls::ReduceClasses::MAX; ++j)
    if (j < a.q_rc.n && s >= a.q_rc.first[j])
      k = j;
  const uint32_t m      = a.q_rc.mult[k];
  const uint32_t b0     = a.q_rc.slot0[k] + (s - a.q_rc.first[k]) * m;
  const uint32_t packed = a.q_nodes[s];
  const V       *pp     = reinterpret_cast<const V *>(a.q_slots);
  V              sum    = {};
  uint32_t       i      = 0;
  for (; i + 4 <= m; i += 4)
    {
      const V x0 = pp[b0 + i], x1 = pp[b0 + i + 1], x2 = pp[b0 + i + 2], x3 = pp[b0 + i + 3];
      sum += (x0 + x1) + (x2 + x3);
    }
  if (i + 2 <= m)
    {
      const V x0 = pp[b0 + i], x1 = pp[b0 + i + 1];
      sum += x0 + x1;
      i += 2;
    }
  if (i < m)
    sum += pp[b0 + i];
  const uint32_t node = packed & gls::NODE_MASK, cm = packed >> 28;
  const V        xs   = reinterpret_cast<const V *>(a.q_x)[node];
  if (cm)
#pragma unroll
    for (int w = 0; w < W; ++w)
      if ((cm >> w) & 1)
        sum[w] = xs[w];
  const V dj = V{} + T(1);
  return V{} + T(1) * dj * (reinterpret_cast<const V *>(a.q_b)[node] - sum);
}

// Transfers as sum factorisation over the (2k+1)^dim child lattice of one
// coarse cell: the 1-D interpolation matrix P [(2k+1) x (k+1)] is staged in
// LDS and each lane reads its rows into registers, so every tensor index is a
// compile-time constant of the unrolled sweeps (a dense (2k+1)^dim x
// (k+1)^dim loop indexing the kernel-argument array at run time went
// through scratch: 28.7 us per r2 -> r1 restriction).
// threads per transfer workgroup (one coarse cell): the fine lattice's
// (2k+1)^dim points rounded up to whole waves, at least the coarse cell's
// dofs, at most 256 (3D Q2: 125 points -> 128 threads, twice the resident
// workgroups of a 256-thread block that idles half its lanes)
template <int dim, int k>
constexpr int
transfer_block()
{
  constexpr int nl = ipow(2 * k + 1, dim), nd = ipow(k + 1, dim) * (dim + 1);
  constexpr int m  = nl > nd ? nl : nd;
  return m <= 64 ? 64 : m <= 128 ? 128 : 256;
}

template <int dim, int k, typename T>
__global__ void __launch_bounds__(256)
  k_prolongate(TransferArgs<T> a, T *__restrict__ dst_f, const T *__restrict__ src_c,
               const T *__restrict__ base = nullptr)
{
  constexpr int n = k + 1, nq = ipow(n, dim), nc = dim + 1, L = 2 * k + 1;
  constexpr int nl = ipow(L, dim);
  constexpr int TB  = transfer_block<dim, k>();
  constexpr int NIT = (nl + TB - 1) / TB; // lattice points per thread
  __shared__ T  u[nc][nq];
  __shared__ T  sP[L][n];
  const int64_t c = blockIdx.x;
  const int     t = threadIdx.x;
  // the lattice's fine node ids and their weights / base values do not
  // depend on the coarse gather: issued first, in flight together with it
  // (one memory round trip before the sweeps instead of two)
  uint32_t fe[NIT];
  T        wv[NIT][nc], bv[NIT][nc];
#pragma unroll
  for (int r = 0; r < NIT; ++r)
    {
      const int I = t + r * TB;
      fe[r]       = I < nl ? a.child[c * nl + I] : NOT_OWNER;
    }
#pragma unroll
  for (int r = 0; r < NIT; ++r)
#pragma unroll
    for (int comp = 0; comp < nc; ++comp)
      {
        const size_t j = (size_t)(fe[r] & ~NOT_OWNER) * nc + comp;
        const bool   o = !(fe[r] & NOT_OWNER);
        wv[r][comp]    = o ? a.weight[j] : T(0);
        bv[r][comp]    = o ? (base ? base[j] : dst_f[j]) : T(0);
      }
  if (t < L * n)
    sP[t / n][t % n] = a.P[t / n][t % n];
  if (t < nq)
    {
      const uint32_t packed = a.coarse_nodes[c * nq + t];
      const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
      bool           done = false;
      if constexpr (sizeof(T) == 4 && nc == 4)
        if (a.p_index)
          {
            // pending last smoothing step: shared coarse rows rebuilt
            using V          = typename gls::Pack<T>::V;
            const int32_t si = a.p_index[node];
            const V       x  = si >= 0 ? rebuild_relax(a, (uint32_t)si, node, cm) :
                                         reinterpret_cast<const V *>(src_c)[node];
#pragma unroll
            for (int comp = 0; comp < nc; ++comp)
              u[comp][t] = ((cm >> comp) & 1) ? T(0) : x[comp];
            done = true;
          }
      if (!done)
#pragma unroll
        for (int comp = 0; comp < nc; ++comp)
          u[comp][t] = ((cm >> comp) & 1) ? T(0) : src_c[(size_t)node * nc + comp];
    }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < NIT; ++r)
    {
      const int I = t + r * TB;
      if (I >= nl)
        break;
      const int Ix = I % L, Iy = (I / L) % L, Iz = dim == 3 ? I / (L * L) : 0;
      T         px[n], py[n], pz[n];
#pragma unroll
      for (int i = 0; i < n; ++i)
        {
          px[i] = sP[Ix][i];
          py[i] = sP[Iy][i];
          pz[i] = dim == 3 ? sP[Iz][i] : T(0);
        }
      // a fine node shared by several coarse cells is written by its owner
      // only (conforming interpolation: all give the same value), so the
      // update is a plain read-modify-write, no atomics
      if (fe[r] & NOT_OWNER)
        continue;
      const uint32_t fn = fe[r];
#pragma unroll
      for (int comp = 0; comp < nc; ++comp)
        {
          T s = 0;
#pragma unroll
          for (int iz = 0; iz < (dim == 3 ? n : 1); ++iz)
            {
              T sy = 0;
#pragma unroll
              for (int iy = 0; iy < n; ++iy)
                {
                  T sx = 0;
#pragma unroll
                  for (int ix = 0; ix < n; ++ix)
                    sx += px[ix] * u[comp][ix + n * (iy + n * iz)];
                  sy += py[iy] * sx;
                }
              s += (dim == 3 ? pz[iz] : T(1)) * sy;
            }
          const T      w = wv[r][comp];
          const size_t j = (size_t)fn * nc + comp;
          if (base) // out of place: dst = base + w P src
            dst_f[j] = bv[r][comp] + (w != T(0) ? w * s : T(0));
          else if (w != T(0))
            dst_f[j] = bv[r][comp] + w * s;
        }
    }
}

template <int dim, int k, typename T>
__global__ void __launch_bounds__(256)
  k_restrict(TransferArgs<T> a, T *__restrict__ dst_c, const T *__restrict__ src_f)
{
  constexpr int n = k + 1, nq = ipow(n, dim), nc = dim + 1, L = 2 * k + 1;
  constexpr int nl = ipow(L, dim);
  __shared__ T  v[nc][nl];
  __shared__ T  sP[L][n];
  const int64_t c = a.cells ? (int64_t)a.cells[blockIdx.x] : (int64_t)blockIdx.x;
  const int     t = threadIdx.x;
  // this thread's coarse dof (node id, constraint bits) is independent of
  // the fine gather: loaded up front (blockDim >= nq * nc, k <= 2 in 3D)
  constexpr bool ONE = nq * nc <= transfer_block<dim, k>();
  const uint32_t pk0 = ONE && t < nq * nc ? a.coarse_nodes[c * nq + t % nq] : 0u;
  if (t < L * n)
    sP[t / n][t % n] = a.P[t / n][t % n];
  for (int I = t; I < nl; I += blockDim.x)
    {
      // R = P^T of the owner-only prolongation: a shared fine node feeds its
      // owner's coarse dofs only (its other cells' shape functions that are
      // nonzero there are the same shared coarse dofs)
      const uint32_t fe    = a.child[c * nl + I];
      const bool     owner = !(fe & NOT_OWNER);
      const uint32_t fn    = fe & ~NOT_OWNER;
      if constexpr (sizeof(T) == 4 && nc == 4)
        if (a.q_index)
          {
            // pending residual: shared rows rebuilt from the slots
            using V     = typename gls::Pack<T>::V;
            const int32_t si = owner ? a.q_index[fn] : -1;
            const V       r  = si >= 0 ? rebuild_residual(a, (uint32_t)si) :
                               owner  ? reinterpret_cast<const V *>(src_f)[fn] : V{};
            const V       wv = owner ? reinterpret_cast<const V *>(a.weight)[fn] : V{};
#pragma unroll
            for (int comp = 0; comp < nc; ++comp)
              v[comp][I] = wv[comp] * r[comp];
            continue;
          }
#pragma unroll
      for (int comp = 0; comp < nc; ++comp)
        v[comp][I] = owner ? a.weight[(size_t)fn * nc + comp] * src_f[(size_t)fn * nc + comp]
                           : T(0);
    }
  __syncthreads();
  for (int i = t; i < nq * nc; i += blockDim.x)
    {
      const int      ii = i % nq, comp = i / nq;
      const uint32_t packed = ONE ? pk0 : a.coarse_nodes[c * nq + ii];
      const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
      if ((cm >> comp) & 1)
        continue;
      const int ix = ii % n, iy = (ii / n) % n, iz = dim == 3 ? ii / (n * n) : 0;
      T         px[L], py[L], pz[L];
#pragma unroll
      for (int I = 0; I < L; ++I)
        {
          px[I] = sP[I][ix];
          py[I] = sP[I][iy];
          pz[I] = dim == 3 ? sP[I][iz] : T(0);
        }
      const T *vc = v[comp];
      T        s  = 0;
#pragma unroll
      for (int Iz = 0; Iz < (dim == 3 ? L : 1); ++Iz)
        {
          T sy = 0;
#pragma unroll
          for (int Iy = 0; Iy < L; ++Iy)
            {
              T sx = 0;
#pragma unroll
              for (int Ix = 0; Ix < L; ++Ix)
                sx += px[Ix] * vc[Ix + L * (Iy + L * Iz)];
              sy += py[Iy] * sx;
            }
          s += (dim == 3 ? pz[Iz] : T(1)) * sy;
        }
      unsafeAtomicAdd(dst_c + (size_t)node * nc + comp, s);
    }
}

// interpolate_to_mg: coarse GLL node i sits at fine lattice point 2 i (k <= 2)
template <int dim, int k, typename T>
__global__ void
k_interpolate(TransferArgs<T> a, T *__restrict__ dst_c, const T *__restrict__ src_f)
{
  constexpr int n = k + 1, nq = ipow(n, dim), nc = dim + 1, L = 2 * k + 1;
  constexpr int nl = ipow(L, dim);
  const int64_t g  = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.n_cells_c * nq)
    return;
  const int64_t  c  = g / nq;
  const int      i  = (int)(g % nq);
  const int      ix = i % n, iy = (i / n) % n, iz = dim == 3 ? i / (n * n) : 0;
  const int      I  = 2 * ix + L * (2 * iy + L * (dim == 3 ? 2 * iz : 0));
  const uint32_t fn = a.child[c * nl + I] & ~NOT_OWNER;
  const uint32_t cn = a.coarse_nodes[c * nq + i] & NODE_MASK;
#pragma unroll
  for (int comp = 0; comp < nc; ++comp)
    dst_c[(size_t)cn * nc + comp] = src_f[(size_t)fn * nc + comp];
}

// ------------------------------------------------------------ vectors
// PreconditionRelaxation with a diagonal preconditioner:
//   first (zero start): x = omega d . b;  step: x += omega d . (b - t), t = A x
template <typename T>
__global__ void
k_relax(T *__restrict__ x, const T *__restrict__ b, const T *__restrict__ t,
        const T *__restrict__ d, T omega, int first, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  if (first)
    x[i] = omega * d[i] * b[i];
  else
    x[i] += omega * d[i] * (b[i] - t[i]);
}

// The zero-start relaxation of a level's pre-smoothing with two neighbours of
// the V-cycle folded in: the next coarser defect, which the restriction then
// accumulates into, is zeroed here (zero_words), and on the finest level the
// outer FP64 defect is converted here (copy_to_mg): b = (T) b64, written to
// bout.  One launch instead of three.
template <typename T>
__global__ void
k_relax_first(T *__restrict__ x, const T *__restrict__ b, const T *__restrict__ d, T omega,
              int64_t n, uint32_t *__restrict__ zero, int64_t zero_words,
              const double *__restrict__ b64, T *__restrict__ bout)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < zero_words)
    zero[i] = 0u;
  if (i >= n)
    return;
  T bi;
  if (b64)
    {
      bi      = (T)b64[i];
      bout[i] = bi;
    }
  else
    bi = b[i];
  x[i] = omega * d[i] * bi;
}

// t = b - t  (Multigrid residual step)
template <typename T>
__global__ void
k_residual(T *__restrict__ t, const T *__restrict__ b, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    t[i] = b[i] - t[i];
}

// zero fill / copy of the V-cycle's own buffers (kernels)
__global__ void
k_zero(uint32_t *__restrict__ x, int64_t n_words)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_words)
    x[i] = 0u;
}

__global__ void
k_copy(uint32_t *__restrict__ y, const uint32_t *__restrict__ x, int64_t n_words)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_words)
    y[i] = x[i];
}

template <typename Tin, typename Tout>
__global__ void
k_convert(Tout *__restrict__ dst, const Tin *__restrict__ src, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    dst[i] = (Tout)src[i];
}

// power iteration step (deal.II power_iteration, see power_iteration_t):
// y = D^{-1} (A x) in place; per-block partial sums of x.y and y.y into
// part[2 block], part[2 block + 1] (no atomics: k_power_finish adds the
// blocks in a fixed order)
template <typename T>
__global__ void __launch_bounds__(256)
  k_power_step(T *__restrict__ y, const T *__restrict__ x, const T *__restrict__ d,
               double *__restrict__ part, int64_t n)
{
  __shared__ double red[2][4];
  const int64_t     i  = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double            xy = 0, yy = 0;
  if (i < n)
    {
      const T v = d[i] * y[i];
      y[i]      = v;
      xy        = (double)x[i] * (double)v;
      yy        = (double)v * (double)v;
    }
  for (int off = 32; off > 0; off >>= 1)
    {
      xy += __shfl_down(xy, off);
      yy += __shfl_down(yy, off);
    }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    {
      red[0][w] = xy;
      red[1][w] = yy;
    }
  __syncthreads();
  if (threadIdx.x == 0)
    {
      part[2 * blockIdx.x]     = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
      part[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    }
}

// deal.II set_initial_guess + constraints.set_zero: x_i = i % 11 - mean,
// zero on constrained components; per-block partial sums of x.x for the
// normalisation (k_power_finish)
template <typename T>
__global__ void __launch_bounds__(256)
  k_power_start(T *__restrict__ x, const uint8_t *__restrict__ cmask, int nc, double mean,
                double *__restrict__ part, int64_t n)
{
  __shared__ double red[4];
  const int64_t     i  = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double            xx = 0;
  if (i < n)
    {
      const int64_t node = i / nc;
      const int     c    = (int)(i - node * nc);
      const double  v    = ((cmask[node] >> c) & 1) ? 0.0 : (double)(i % 11) - mean;
      x[i]               = (T)v;
      xx                 = v * v;
    }
  for (int off = 32; off > 0; off >>= 1)
    xx += __shfl_down(xx, off);
  if ((threadIdx.x & 63) == 0)
    red[threadIdx.x >> 6] = xx;
  __syncthreads();
  if (threadIdx.x == 0)
    {
      part[2 * blockIdx.x]     = 0.0;
      part[2 * blockIdx.x + 1] = (red[0] + red[1]) + (red[2] + red[3]);
    }
}

// one workgroup: scal[0] = x.y (the Rayleigh quotient of the normalised x),
// scal[1] = 1 / |y| (0 if y = 0)
__global__ void __launch_bounds__(256)
  k_power_finish(const double *__restrict__ part, int64_t n_blocks, double *__restrict__ scal)
{
  __shared__ double red[2][256];
  double            xy = 0, yy = 0;
  for (int64_t b = threadIdx.x; b < n_blocks; b += 256)
    {
      xy += part[2 * b];
      yy += part[2 * b + 1];
    }
  red[0][threadIdx.x] = xy;
  red[1][threadIdx.x] = yy;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1)
    {
      if ((int)threadIdx.x < s)
        {
          red[0][threadIdx.x] += red[0][threadIdx.x + s];
          red[1][threadIdx.x] += red[1][threadIdx.x + s];
        }
      __syncthreads();
    }
  if (threadIdx.x == 0)
    {
      scal[0] = red[0][0];
      scal[1] = red[1][0] > 0 ? 1.0 / sqrt(red[1][0]) : 0.0;
    }
}

// x = scal[1] * y (the scale factor stays on the device: no host round trip
// per power iteration)
template <typename T>
__global__ void
k_scale_dev(T *__restrict__ x, const T *__restrict__ y, const double *__restrict__ scal,
            int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    x[i] = (T)(scal[1] * (double)y[i]);
}

dim3
g1(int64_t n)
{
  return dim3((unsigned)((n + 255) / 256));
}

void
zero_words(void *x, int64_t n_words, hipStream_t s)
{
  hipLaunchKernelGGL(k_zero, g1(n_words), dim3(256), 0, s, (uint32_t *)x, n_words);
  HIP_THROW(hipGetLastError());
}

void
copy_words(void *y, const void *x, int64_t n_words, hipStream_t s)
{
  hipLaunchKernelGGL(k_copy, g1(n_words), dim3(256), 0, s, (uint32_t *)y, (const uint32_t *)x,
                     n_words);
  HIP_THROW(hipGetLastError());
}


} // namespace

struct glsMG_
{
  glsMGDesc          desc{};
  // timer-section names of the V-cycle phases per level (multigrid.cc:550-583:
  // gmg::vmult::level_<l>::<phase>; [l][5] = the coarse solve's plain name)
  std::vector<std::vector<std::string>> sec;
  std::vector<glsOp> ops;
  int                prec = GLS_F32, dim = 3, degree = 2, nc = 4;
  std::vector<uint32_t *> d_child;  // level l >= 1: [cells(l-1)][nl]
  std::vector<void *>     d_weight; // level l >= 1: [n_dofs(l)]
  std::vector<void *>     invdiag, sol, def, tmp;
  // deferred shared-node reductions of the smoother (smooth): per level two
  // partial-slot buffers the applies alternate between (beside the
  // operator's own, which the residual and the explicit reductions use);
  // GLS_MG_DEFER=0 reduces after every apply instead
  std::vector<void *>     qslot[2];
  std::vector<double>     omega, lambda;
  // power iteration: per level, block partials | 2 scalars (the levels'
  // estimates run concurrently, gls_mg_setup)
  double                 *d_acc = nullptr;
  std::vector<int64_t>    acc_off; // level l's partials start at d_acc + acc_off[l]
  std::vector<hipStream_t> side;   // setup: one stream per level, joined by events
  std::vector<hipEvent_t>  side_ev;
  double                  P[3][MAXP][MAXN]{}; // 1D prolongation per coarse degree (1, 2)
  bool                    setup_done = false;
  bool                    partitioned = false; // rank-local level operators
  gls::VecStage           stage; // caller layout of gls_mg_vcycle's vectors
  // dense LU coarse solver (coarse_n_iterations < 0): the substitute for the
  // reference's Trilinos direct solver (multigrid.cc:448-455, 477-481)
  rocblas_handle blas   = nullptr;
  double        *d_lu   = nullptr; // [nf][nf] column major: LU factors, then the inverse
  rocblas_int   *d_ipiv = nullptr;
  rocblas_int   *d_info = nullptr;
  double        *d_rhs  = nullptr; // [(2 + GEMV_CHUNKS) nf]: rhs | solution | partials
  int32_t       *d_free = nullptr; // [nf] the free (unconstrained) coarse dofs
  // [nf] the GEMV's input gather: the free dof whose entry multiplies column
  // i of the stored inverse (free[p[i]] for the unpermuted U^-1 L^-1 of the
  // trtri path, A^-1 = U^-1 L^-1 P^T; free[i] otherwise)
  int32_t       *d_free_in = nullptr;
  int64_t        n_free = 0, ld_free = 0; // ld_free: nf rounded up to 4
  // static condensation of the cells' interior dofs (coarse_lu_setup_t):
  // the dense inverse covers the remaining free dofs only; per cell
  // C = E_II^-1 [ni][ni], F = E_BI E_II^-1 [nb][ni], G = E_II^-1 E_IB [ni][nb]
  // (constrained boundary dofs: zero rows / columns), the interior / boundary
  // dofs' global indices (-1: constrained), y = C b_I per solve, and per GEMV
  // column i the (cell, boundary slot) pairs of its dof (CSR)
  bool           cond = false;
  bool           cond_failed = false; // a cell's E_II was (numerically) singular: no condensation
  int            cond_ni = 0, cond_nb = 0;
  std::vector<int32_t> cond_lint, cond_lbnd; // local interior / boundary dofs of a cell
  double        *d_cC = nullptr, *d_cF = nullptr, *d_cG = nullptr;
  int32_t       *d_cint = nullptr, *d_cbnd = nullptr, *d_rg_off = nullptr, *d_rg_ent = nullptr;
  float         *d_inv32 = nullptr; // [nf][nf] FP32 copy of the inverse (inv_f32)
  bool           inv_f32 = false;
  // last dense-coarse setup: assembly / getrf / getri wall ms, cell colours
  double         coarse_setup_ms[3] = {0, 0, 0};
  int            coarse_colors      = 0;
  // coarse GMRES (coarse_iterate): FP64 Krylov workspace, two level-
  // precision operand buffers, statistics of the last solve
  // finest-level FP64 defect for the fused copy_to_mg (mg_vcycle_device; null:
  // def[top] already holds the defect)
  const double *top_b64 = nullptr;
  // its FP64 result for the fused copy_from_mg (null: none), and whether the
  // last post-smoothing step wrote it
  double *top_out64      = nullptr;
  bool    top_out64_done = false;
  // the residual of level rq_level whose shared-node reduction the next
  // restriction rebuilds (v_step; rq_level < 0: none): its slots, x and b
  mutable int   rq_level = -1;
  mutable void *rq_slots = nullptr;
  mutable const void *rq_x = nullptr, *rq_b = nullptr;
  // the coarse solution of level pp_level - 1 whose last smoothing step's
  // reduction the next prolongation into level pp_level rebuilds
  mutable int         pp_level = -1;
  mutable const void *pp_slots = nullptr, *pp_prev = nullptr, *pp_b = nullptr,
                     *pp_d = nullptr;
  mutable double      pp_omega = 0.0;
  double *cg_ws    = nullptr;
  void   *cg_lvl   = nullptr;
  double *cg_host  = nullptr; // pinned: two Hessenberg columns (software pipeline)
  hipEvent_t cg_ev[2] = {nullptr, nullptr};
  int     cg_iters = 0, cg_conv = 0;
  // "gmg coarse grid solver": "AMG" (desc.coarse_amg): the smoothed-
  // aggregation AMG on the coarse level's system matrix (amg.hip), rebuilt by
  // every gls_mg_setup (PreconditionerGMG::initialize, multigrid.cc:372-433)
  glsAMG  amg      = nullptr;
  double *amg_io   = nullptr; // [2 n0] FP64 in / out of a direct AMG coarse solve
  double  amg_setup_ms = 0;

  size_t
  ts() const
  {
    return prec == GLS_F64 ? 8 : 4;
  }
};

namespace
{
template <typename T>
TransferArgs<T>
targs(const glsMG_ *mg, int level)
{
  TransferArgs<T> a;
  a.coarse_nodes = mg->ops[level - 1]->d_nodes;
  a.child        = mg->d_child[level];
  a.weight       = (const T *)mg->d_weight[level];
  a.n_cells_c    = mg->ops[level - 1]->n_cells;
  const int kc   = mg->ops[level - 1]->degree;
  for (int i = 0; i < MAXP; ++i)
    for (int j = 0; j < MAXN; ++j)
      a.P[i][j] = (T)mg->P[kc][i][j];
  if (mg->rq_level == level)
    {
      const glsOp op = mg->ops[level];
      a.q_index      = op->d_shared_index;
      a.q_nodes      = op->d_shared_nodes;
      a.q_slots      = (const T *)mg->rq_slots;
      a.q_x          = (const T *)mg->rq_x;
      a.q_b          = (const T *)mg->rq_b;
      a.q_rc         = op->reduce_classes;
    }
  if (mg->pp_level == level)
    {
      const glsOp oc = mg->ops[level - 1];
      a.p_index      = oc->d_shared_index;
      a.p_slots      = (const T *)mg->pp_slots;
      a.p_prev       = (const T *)mg->pp_prev;
      a.p_b          = (const T *)mg->pp_b;
      a.p_d          = (const T *)mg->pp_d;
      a.p_omega      = (T)mg->pp_omega;
      a.p_rc         = oc->reduce_classes;
    }
  return a;
}

// kind: 0 prolongate_add, 1 restrict_add, 2 interpolate; base (prolongate
// only): dst = base + P src instead of dst += P src
template <int dim, int k, typename T>
void
transfer_t(const glsMG_ *mg, int kind, int level, void *dst, const void *src, hipStream_t s,
           const void *base)
{
  constexpr int nq = ipow(k + 1, dim);
  const auto    a  = targs<T>(mg, level);
  const dim3    grid((unsigned)a.n_cells_c);
  const dim3    tb(transfer_block<dim, k>());
  if (kind == 0)
    hipLaunchKernelGGL((k_prolongate<dim, k, T>), grid, tb, 0, s, a, (T *)dst, (const T *)src,
                       (const T *)base);
  else if (kind == 1 && !gls::op_deterministic(mg->ops[level - 1]))
    hipLaunchKernelGGL((k_restrict<dim, k, T>), grid, tb, 0, s, a, (T *)dst, (const T *)src);
  else if (kind == 1)
    {
      // coarse cell colour by colour: no two workgroups of a launch add to
      // one coarse node, the sums in a fixed order
      glsOp_ *oc = const_cast<glsOp_ *>(mg->ops[level - 1]);
      gls::op_cell_colours(oc);
      for (size_t col = 0; col + 1 < oc->colour_off.size(); ++col)
        {
          auto ac  = a;
          ac.cells = oc->d_colour_cells + oc->colour_off[col];
          hipLaunchKernelGGL((k_restrict<dim, k, T>),
                             dim3((unsigned)(oc->colour_off[col + 1] - oc->colour_off[col])), tb, 0,
                             s, ac, (T *)dst, (const T *)src);
        }
    }
  else
    hipLaunchKernelGGL((k_interpolate<dim, k, T>), g1(a.n_cells_c * nq), dim3(256), 0, s, a,
                       (T *)dst, (const T *)src);
  HIP_THROW(hipGetLastError());
}

template <typename T>
void
transfer_p(const glsMG_ *mg, int kind, int level, void *dst, const void *src, hipStream_t s,
           const void *base)
{
  // the coarse level's degree: a FE_Q_iso_Q1 coarsest level is Q1 on the
  // sub-cells under Q_k levels (main.cc:436-446)
  const int d = mg->dim, k = mg->ops[level - 1]->degree;
  if (d == 2 && k == 1)
    transfer_t<2, 1, T>(mg, kind, level, dst, src, s, base);
  else if (d == 2 && k == 2)
    transfer_t<2, 2, T>(mg, kind, level, dst, src, s, base);
  else if (d == 3 && k == 1)
    transfer_t<3, 1, T>(mg, kind, level, dst, src, s, base);
  else if (d == 3 && k == 2)
    transfer_t<3, 2, T>(mg, kind, level, dst, src, s, base);
  else
    throw std::runtime_error("multigrid transfer: degree must be 1 or 2");
}

void
transfer(const glsMG_ *mg, int kind, int level, void *dst, const void *src, hipStream_t s,
         const void *base = nullptr)
{
  if (level < 1 || level >= (int)mg->ops.size())
    throw std::runtime_error("multigrid transfer: level out of range");
  if (mg->prec == GLS_F64)
    transfer_p<double>(mg, kind, level, dst, src, s, base);
  else
    transfer_p<float>(mg, kind, level, dst, src, s, base);
}

void
check(glsStatus st)
{
  if (st != 0)
    throw std::runtime_error(gls_last_error());
}

template <typename T>
void
relax_t(const glsMG_ *mg, int level, void *x, const void *b, int first, hipStream_t s)
{
  const int64_t n = mg->ops[level]->n_dofs;
  hipLaunchKernelGGL(k_relax<T>, g1(n), dim3(256), 0, s, (T *)x, (const T *)b,
                     (const T *)mg->tmp[level], (const T *)mg->invdiag[level],
                     (T)mg->omega[level], first, n);
  HIP_THROW(hipGetLastError());
}

// what the zero-start relaxation folds in (k_relax_first)
struct FirstRelax
{
  uint32_t     *zero       = nullptr;
  int64_t       zero_words = 0;
  const double *b64        = nullptr; // FP64 defect to convert into b
};

template <typename T>
void
relax_first_t(const glsMG_ *mg, int level, void *x, void *b, const FirstRelax &fr, hipStream_t s)
{
  const int64_t n = mg->ops[level]->n_dofs;
  hipLaunchKernelGGL(k_relax_first<T>, g1(std::max(n, fr.zero_words)), dim3(256), 0, s, (T *)x,
                     (const T *)b, (const T *)mg->invdiag[level], (T)mg->omega[level], n,
                     fr.zero, fr.zero_words, fr.b64, (T *)b);
  HIP_THROW(hipGetLastError());
}

// the last apply of a smoothing sequence whose shared-node reduction is
// still pending (deferred): its slots, its src (the iterate before) and its
// relaxation
struct PendingReduce
{
  const void *slots = nullptr, *src = nullptr, *b = nullptr, *d = nullptr;
  double      omega = 0.0;
  bool        valid = false;
};

bool
defer_reduce(const glsMG_ *mg, int level)
{
  static const bool on = [] {
    const char *e = getenv("GLS_MG_DEFER");
    return !e || std::atoi(e) != 0;
  }();
  return on && gls::deferred_reduce_ok(mg->ops[level]) && mg->qslot[0].size() > (size_t)level &&
         mg->qslot[0][(size_t)level];
}

// deferred smoothing sequences in one resident launch (k_brick_sweeps) where
// the level qualifies: GLS_MG_DEFER unset or >= 2; 1 keeps one launch per
// step (with deferred reductions), 0 reduces after every step
bool
defer_resident()
{
  static const bool on = [] {
    const char *e = getenv("GLS_MG_DEFER");
    return !e || std::atoi(e) >= 2;
  }();
  return on;
}

// PreconditionRelaxation::vmult (zero start) / step, `iters` iterations;
// the result in x.  x_in (step only): the starting iterate is in tmp[level]
// instead of x (the multigrid's out-of-place prolongation put it there).
// fr (zero start only): folded into the first relaxation; false when there
// was none (iters == 0), so the caller does that work itself
// out64 (deferred-reduction levels only): the last step's result also
// written as FP64 by its brick write-out and reduction (*wrote64 = true)
bool
smooth(const glsMG_ *mg, int level, void *x, const void *b, bool zero_start, int iters,
       hipStream_t s, bool start_in_tmp = false, const FirstRelax *fr = nullptr,
       PendingReduce *pend = nullptr, double *out64 = nullptr, bool *wrote64 = nullptr)
{
  auto  relax = mg->prec == GLS_F64 ? relax_t<double> : relax_t<float>;
  auto  first = [&](void *xx) {
    if (fr)
      (mg->prec == GLS_F64 ? relax_first_t<double> : relax_first_t<float>)(mg, level, xx,
                                                                          (void *)b, *fr, s);
    else
      relax(mg, level, xx, b, 1, s);
  };
  glsOp op    = mg->ops[level];
  void *tmp   = mg->tmp[level];
  if (!gls::fused_relax_ok(op))
    {
      int it = 0;
      if (start_in_tmp)
        {
          const int64_t w = (int64_t)((size_t)op->n_dofs * mg->ts() / 4);
          copy_words(x, tmp, w, s);
        }
      if (zero_start && iters > 0)
        {
          first(x);
          it = 1;
        }
      for (; it < iters; ++it)
        {
          gls::op_vmult_device(op, tmp, x, s);
          relax(mg, level, x, b, 0, s);
        }
      return zero_start && iters > 0;
    }
  // brick operators: the step x + omega D^{-1} (b - A x) is fused into the
  // vmult's write-out (k_brick, k_shared_reduce_cls), ping-ponging between x
  // and tmp; the start buffer is chosen so that the last step lands in x
  // (zero start: the first iterate omega D^{-1} b goes to tmp when the
  // remaining count is odd), a final copy otherwise
  int   it  = 0;
  void *cur = start_in_tmp ? tmp : x;
  if (zero_start && iters > 0)
    {
      cur = ((iters - 1) % 2 == 1) ? tmp : x;
      first(cur);
      it = 1;
    }
  gls::RelaxStep rx;
  rx.b     = b;
  rx.d     = mg->invdiag[level];
  rx.omega = mg->omega[level];
  // deferred reductions: apply j writes its boundary partials to slot
  // buffer j % 2 and skips its reduction; apply j + 1 rebuilds those rows in
  // its gather (and stores them into its src); the last apply's reduction
  // runs explicitly below, or is handed to the caller (pend), whose next
  // apply of the operator to x rebuilds it the same way
  const bool    defer = defer_reduce(mg, level);
  if (!defer || pend || it >= iters)
    out64 = nullptr;
  PendingReduce pr;
  // the steps in one resident launch (k_brick_sweeps) where the level
  // qualifies; the same iterates as the per-step launches below
  if (defer && defer_resident() && iters - it >= 2)
    {
      void          *oth = cur == x ? tmp : x;
      void          *s0  = mg->qslot[it % 2][(size_t)level];
      void          *s1  = mg->qslot[(it + 1) % 2][(size_t)level];
      gls::RelaxStep r   = rx;
      r.out64            = out64;
      const int      ns  = iters - it;
      if (gls::brick_sweeps(op, gls::op_vmult_mode(op), cur, oth, s0, s1, ns, r, s))
        {
          // the last sweep (ns - 1) read v[(ns - 1) % 2] and wrote the other
          const bool even = (ns - 1) % 2 == 0;
          pr  = PendingReduce{even ? s0 : s1, even ? cur : oth, rx.b, rx.d, rx.omega, true};
          cur = even ? oth : cur;
          it  = iters;
        }
    }
  for (; it < iters; ++it)
    {
      void          *oth = cur == x ? tmp : x;
      gls::RelaxStep r   = rx;
      if (it + 1 == iters)
        r.out64 = out64;
      if (defer)
        {
          r.defer   = true;
          r.partial = mg->qslot[it % 2][(size_t)level];
          if (pr.valid)
            {
              r.prev_partial = pr.slots, r.prev_src = pr.src;
              r.prev_b = pr.b, r.prev_d = pr.d, r.prev_omega = pr.omega;
            }
        }
      gls::brick_launch(op, gls::op_vmult_mode(op), oth, cur, 0, op->n_bricks,
                        gls::BRICK_RUN | gls::BRICK_REDUCE, s, &r);
      if (defer)
        pr = PendingReduce{r.partial, cur, rx.b, rx.d, rx.omega, true};
      cur = oth;
    }
  if (pr.valid)
    {
      if (pend && cur == x)
        *pend = pr;
      else
        {
          gls::RelaxStep r = rx;
          r.partial        = const_cast<void *>(pr.slots);
          r.out64          = out64;
          gls::brick_launch(op, gls::op_vmult_mode(op), cur, pr.src, 0, 0, gls::BRICK_REDUCE, s,
                            &r);
        }
    }
  if (cur != x)
    {
      const int64_t w = (int64_t)((size_t)op->n_dofs * mg->ts() / 4);
      copy_words(x, cur, w, s);
    }
  if (wrote64)
    *wrote64 = out64 != nullptr && pr.valid;
  return zero_start && iters > 0;
}

void
residual(const glsMG_ *mg, int level, void *t, const void *b, hipStream_t s)
{
  const int64_t n = mg->ops[level]->n_dofs;
  if (mg->prec == GLS_F64)
    hipLaunchKernelGGL(k_residual<double>, g1(n), dim3(256), 0, s, (double *)t,
                       (const double *)b, n);
  else
    hipLaunchKernelGGL(k_residual<float>, g1(n), dim3(256), 0, s, (float *)t,
                       (const float *)b, n);
  HIP_THROW(hipGetLastError());
}

void
check_blas(rocblas_status st, const char *what)
{
  if (st != rocblas_status_success)
    throw std::runtime_error(std::string(what) + " failed (rocblas status " +
                             std::to_string((int)st) + ")");
}

// X = the unit lower triangle of the LU factors (column major n x n):
// strictly lower entries copied, 1 on the diagonal, 0 above
__global__ void
k_unit_lower(double *__restrict__ X, const double *__restrict__ LU, int64_t n)
{
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n * n)
    return;
  const int64_t c = k / n, r = k - c * n;
  X[k]            = r > c ? LU[k] : (r == c ? 1.0 : 0.0);
}

// X[i][i] = 1 (column major n x n, X zeroed)
__global__ void
k_set_diag(double *X, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    X[(size_t)i * n + i] = 1.0;
}

template <typename T>
__global__ void
k_set_unit(T *x, int64_t j, int64_t n, int on)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && i == j)
    x[i] = on ? T(1) : T(0);
}

// y = M x for the dense coarse inverse (column major, n x n, FP64 or FP32
// storage, FP64 sums): the rows split over threads (coalesced column reads)
// and the columns over blockIdx.y chunks, partial sums reduced in a fixed
// order by k_gemv_sum; with ~64 chunks the launch has enough waves to stream
// the matrix at HBM rate (rocBLAS dgemv: 0.86 ms for the 2.2 GB inverse at
// n = 16,704)
constexpr int GEMV_CHUNKS = 64;
template <typename TM>
__global__ void __launch_bounds__(256)
  k_gemv_part(const TM *__restrict__ M, const double *__restrict__ x,
              double *__restrict__ part, int64_t n, int64_t ld)
{
  const int64_t i  = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t cw = (n + GEMV_CHUNKS - 1) / GEMV_CHUNKS;
  const int64_t j0 = blockIdx.y * cw, j1 = j0 + cw < n ? j0 + cw : n;
  if (i >= n)
    return;
  double  s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int64_t j  = j0;
  for (; j + 4 <= j1; j += 4)
    {
      s0 += (double)M[j * n + i] * x[j];
      s1 += (double)M[(j + 1) * n + i] * x[j + 1];
      s2 += (double)M[(j + 2) * n + i] * x[j + 2];
      s3 += (double)M[(j + 3) * n + i] * x[j + 3];
    }
  for (; j < j1; ++j)
    s0 += (double)M[j * n + i] * x[j];
  part[blockIdx.y * ld + i] = (s0 + s1) + (s2 + s3);
}

// The FP32-stored inverse, row major (row stride ld, a multiple of 4,
// padded columns zero): one wavefront per row streams the row as 16-byte
// loads (contiguous), x (FP32, the coarse defect's free entries: exact for
// FP32 levels) from L2, FP64 sums in a fixed order (lane partials, then a
// fixed shuffle tree), and writes y[free[row]] itself: no partial-sum pass.
typedef float gemv_f4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4
gemv_row_load(const float4 *p)
{
  if constexpr (NT)
    {
      const gemv_f4 t = __builtin_nontemporal_load(reinterpret_cast<const gemv_f4 *>(p));
      return make_float4(t.x, t.y, t.z, t.w);
    }
  else
    return *p;
}

template <typename T, bool NT>
__global__ void __launch_bounds__(256)
  k_gemv_rows_f32(const float4 *__restrict__ M, const float4 *__restrict__ x,
                  T *__restrict__ y, const int32_t *__restrict__ free, int64_t n, int64_t ld)
{
  const int64_t row  = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int     lane = threadIdx.x & 63;
  if (row >= n)
    return;
  const int64_t l4 = ld / 4;
  const float4 *mr = M + row * l4;
  double        a0 = 0, a1 = 0;
  int64_t       c  = lane;
  // four 16-byte row loads in flight per lane
  for (; c + 192 < l4; c += 256)
    {
      float4 m[4], xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        m[u] = gemv_row_load<NT>(mr + c + 64 * u);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        xv[u] = x[c + 64 * u];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        {
          a0 += (double)m[u].x * (double)xv[u].x + (double)m[u].y * (double)xv[u].y;
          a1 += (double)m[u].z * (double)xv[u].z + (double)m[u].w * (double)xv[u].w;
        }
    }
  for (; c < l4; c += 64)
    {
      const float4 m0 = gemv_row_load<NT>(mr + c), x0 = x[c];
      a0 += (double)m0.x * (double)x0.x + (double)m0.y * (double)x0.y;
      a1 += (double)m0.z * (double)x0.z + (double)m0.w * (double)x0.w;
    }
  double v = a0 + a1;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    v += __shfl_down(v, off);
  if (lane == 0)
    y[free[row]] = (T)v;
}

// coarse solve prologue for the row GEMV: sol = def on every dof (the
// constrained rows keep it), xf[i] = def[free[i]] in FP32 (padded to ld)
template <typename T>
__global__ void
k_coarse_prep(T *__restrict__ sol, const T *__restrict__ def, float *__restrict__ xf,
              const int32_t *__restrict__ free, int64_t n, int64_t nf, int64_t ld)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    sol[i] = def[i];
  if (i < ld)
    xf[i] = i < nf ? (float)def[free[i]] : 0.0f;
}

// y[free[i]] = sum of the chunk partials (leading dimension ld, fixed
// order), converted to the level precision
template <typename T>
__global__ void
k_gemv_sum(const double *__restrict__ part, T *__restrict__ y, const int32_t *__restrict__ free,
           int64_t n, int64_t ld)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  // eight independent partial loads per step, summed in a fixed order
  double s = 0;
  for (int c = 0; c < GEMV_CHUNKS; c += 8)
    {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = part[(c + u) * ld + i];
      s += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
  y[free[i]] = (T)s;
}

// out[i] = in[free[i]] (FP64): the free rows of an assembled column, or the
// free entries of the coarse right-hand side
template <typename T>
__global__ void
k_gather_free(double *__restrict__ out, const T *__restrict__ in, const int32_t *__restrict__ free,
              int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    out[i] = (double)in[free[i]];
}

// out = in^T rounded to FP32, row major with row stride ld >= n (padded
// columns zero): in is the n x n column-major inverse, so out's row i is
// in's row i (setup only; the strided reads do not matter)
__global__ void
k_narrow(float *__restrict__ out, const double *__restrict__ in, int64_t n, int64_t ld)
{
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * ld)
    return;
  const int64_t i = e / ld, j = e - i * ld; // row i, column j
  out[e] = j < n ? (float)in[j * n + i] : 0.0f;
}

// Static condensation of the cells' interior dofs, one workgroup per cell:
// from the element matrix E (column major per cell: E[c][j][i] = entry
// (i, j)) with interior local dofs lint[ni] and boundary local dofs
// lbnd[nb] (free[b] = 0: a constrained boundary dof, its couplings dropped
// as the assembly drops them), C = E_II^-1 (Gauss-Jordan with partial
// pivoting, FP64), F = E_BI C, G = C E_IB, and the element Schur complement
// S = E_BB - F E_IB (column major [c][b2][b1]), assembled like E.
constexpr int COND_MAXI = 32;
template <typename T>
__global__ void __launch_bounds__(256)
  k_condense(const T *__restrict__ E, int ndof, const int32_t *__restrict__ lint, int ni,
             const int32_t *__restrict__ lbnd, int nb, const int32_t *__restrict__ bfree,
             double *__restrict__ S, double *__restrict__ Cm, double *__restrict__ F,
             double *__restrict__ G, int32_t *__restrict__ bad)
{
  __shared__ double a[COND_MAXI][2 * COND_MAXI];
  __shared__ double f[128 * COND_MAXI / 4]; // F rows of this cell (nb <= 128, ni <= 8)
  const int64_t c   = blockIdx.x;
  const size_t  per = (size_t)ndof * ndof;
  const T      *Ec  = E + (size_t)c * per;
  auto          e   = [&](int row, int col) { return (double)Ec[(size_t)col * ndof + row]; };
  const int     t   = threadIdx.x;
  const int32_t *fr = bfree + (size_t)c * nb;
  // [E_II | I] in LDS, then Gauss-Jordan by one thread (ni <= COND_MAXI)
  for (int k = t; k < ni * 2 * ni; k += blockDim.x)
    {
      const int r = k / (2 * ni), q = k % (2 * ni);
      a[r][q] = q < ni ? e(lint[r], lint[q]) : (q - ni == r ? 1.0 : 0.0);
    }
  __syncthreads();
  if (t == 0)
    {
      // a pivot below 1e-12 of E_II's largest entry (or a non-finite one)
      // marks the cell: the host then assembles without condensation, where
      // getrf's info check covers a singular coarse matrix
      double scale = 0;
      for (int r = 0; r < ni; ++r)
        for (int q = 0; q < ni; ++q)
          scale = fmax(scale, fabs(a[r][q]));
      bool sing = !(scale > 0) || !isfinite(scale);
      for (int col = 0; col < ni && !sing; ++col)
        {
          int piv = col;
          for (int r = col + 1; r < ni; ++r)
            if (fabs(a[r][col]) > fabs(a[piv][col]))
              piv = r;
          if (!(fabs(a[piv][col]) > 1e-12 * scale))
            {
              sing = true;
              break;
            }
          if (piv != col)
            for (int q = 0; q < 2 * ni; ++q)
              {
                const double x = a[col][q];
                a[col][q]      = a[piv][q];
                a[piv][q]      = x;
              }
          const double d = 1.0 / a[col][col];
          for (int q = 0; q < 2 * ni; ++q)
            a[col][q] *= d;
          for (int r = 0; r < ni; ++r)
            if (r != col)
              {
                const double m = a[r][col];
                for (int q = 0; q < 2 * ni; ++q)
                  a[r][q] -= m * a[col][q];
              }
        }
      if (sing)
        bad[c] = 1;
    }
  __syncthreads();
  double *Cc = Cm + (size_t)c * ni * ni, *Fc = F + (size_t)c * nb * ni, *Gc = G + (size_t)c * ni * nb;
  for (int k = t; k < ni * ni; k += blockDim.x)
    Cc[k] = a[k / ni][ni + k % ni];
  // F[b][k] = sum_m E_BI(b, m) C(m, k); G[k][b] = sum_m C(k, m) E_IB(m, b)
  for (int k = t; k < nb * ni; k += blockDim.x)
    {
      const int b = k / ni, kk = k % ni;
      double    sf = 0, sg = 0;
      if (fr[b])
        for (int m = 0; m < ni; ++m)
          {
            sf += e(lbnd[b], lint[m]) * a[m][ni + kk];
            sg += a[kk][ni + m] * e(lint[m], lbnd[b]);
          }
      Fc[(size_t)b * ni + kk] = sf;
      f[b * ni + kk]          = sf;
      Gc[(size_t)kk * nb + b] = sg;
    }
  __syncthreads();
  // S[b2][b1] = E_BB(b1, b2) - sum_k F[b1][k] E_IB(k, b2)
  double *Sc = S + (size_t)c * nb * nb;
  for (int k = t; k < nb * nb; k += blockDim.x)
    {
      const int b2 = k / nb, b1 = k % nb;
      double    v  = e(lbnd[b1], lbnd[b2]);
      if (fr[b2])
        for (int m = 0; m < ni; ++m)
          v -= f[b1 * ni + m] * e(lint[m], lbnd[b2]);
      Sc[k] = v;
    }
}

// sum over the 64 lanes of a wavefront (butterfly, every lane gets it)
__device__ __forceinline__ double
cond_wave_sum(double v)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    v += __shfl_xor(v, o);
  return v;
}

// the condensed right-hand side of GEMV column i: b_S[rin[i]] = def[rin[i]]
// - sum over its (cell, slot) pairs of F[c][slot] . b_I[c] (F = E_BI C
// already holds C, so the cell's interior right-hand side enters as is).
// Eight lanes per column, one (cell, slot) pair each (a vertex of a hex mesh
// usually has at most 8 cells; more loop), summed by a butterfly; sol = def
// on every dof (the constrained rows keep it); out padded to ld with zeros
template <typename T, typename O>
__global__ void __launch_bounds__(256)
  k_cond_rhs(T *__restrict__ sol, const T *__restrict__ def, O *__restrict__ out,
             const int32_t *__restrict__ rin, const int32_t *__restrict__ off,
             const int32_t *__restrict__ ent, const double *__restrict__ F,
             const int32_t *__restrict__ cint, int ni, int nb, int64_t n, int64_t nr,
             int64_t ld)
{
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < n)
    sol[g] = def[g];
  const int64_t i  = g >> 3;
  const int     l8 = (int)(g & 7);
  double        v  = 0;
  if (i < nr)
    for (int32_t e = off[i] + l8; e < off[i + 1]; e += 8)
      {
        const int32_t  cs = ent[e]; // cell * nb + slot
        const int64_t  c  = cs / nb;
        const double  *f  = F + (size_t)cs * ni;
        const int32_t *ic = cint + (size_t)c * ni;
        for (int m = 0; m < ni; ++m)
          v += f[m] * (double)def[ic[m]];
      }
#pragma unroll
  for (int o = 4; o > 0; o >>= 1)
    v += __shfl_xor(v, o);
  if (l8 != 0 || i >= ld)
    return;
  out[i] = i < nr ? (O)((double)def[rin[i]] - v) : O(0);
}

// the interior dofs from the boundary solution: x_I = C b_I - G x_B, one
// wavefront per (cell, interior dof k): the lanes stride G's row (nb
// entries) and the first ni lanes add C's row times b_I
template <typename T>
__global__ void __launch_bounds__(256)
  k_cond_post(T *__restrict__ sol, const T *__restrict__ def, const double *__restrict__ Cm,
              const double *__restrict__ G, const int32_t *__restrict__ cint,
              const int32_t *__restrict__ cbnd, int ni, int nb, int64_t n_cells)
{
  const int64_t row  = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int     lane = threadIdx.x & 63;
  if (row >= n_cells * ni)
    return;
  const int64_t  c  = row / ni;
  const double  *gr = G + (size_t)row * nb;
  const int32_t *cb = cbnd + (size_t)c * nb;
  double         v  = 0;
  for (int b = lane; b < nb; b += 64)
    {
      const int32_t d = cb[b];
      if (d >= 0)
        v -= gr[b] * (double)sol[d];
    }
  if (lane < ni)
    v += Cm[(size_t)row * ni + lane] * (double)def[cint[(size_t)c * ni + lane]];
  v = cond_wave_sum(v);
  if (lane == 0)
    sol[cint[row]] = (T)v;
}

// A_ff[fj][fi] += E[c][j][i] over the cells of one colour (no two of them
// share a node, so no two threads of a launch touch the same entry): the
// element matrices scattered into the column-major free-dof block, the
// colours in a fixed order (deterministic sums)
template <typename T>
__global__ void
k_scatter_emat(double *__restrict__ A, int64_t nf, const T *__restrict__ E,
               const int32_t *__restrict__ cdof, const int32_t *__restrict__ cells,
               int64_t n_cells, int ndof)
{
  const int64_t per = (int64_t)ndof * ndof;
  const int64_t g   = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_cells * per)
    return;
  const int64_t ci = g / per;
  const int     r  = (int)(g - ci * per);
  const int     j = r / ndof, i = r - j * ndof;
  const int64_t c  = cells[ci];
  const int32_t fi = cdof[c * ndof + i], fj = cdof[c * ndof + j];
  if (fi < 0 || fj < 0)
    return;
  A[(size_t)fj * nf + fi] += (double)E[(size_t)c * per + r];
}

// A_ff from the element matrices of the coarse level operator (what the
// reference's coarse direct solver factorises: get_system_matrix ->
// MatrixFreeTools::compute_matrix, operator_ns.cc:1407-1430, assembled into
// the Trilinos matrix, multigrid.cc:448-455): one element-matrix launch over
// all coarse cells, then one scatter launch per cell colour (greedy colouring
// on the host, cells of a colour share no node), summed in FP64
template <typename T>
bool
assemble_free_block(glsMG_ *mg, const std::vector<int32_t> &freel, hipStream_t s)
{
  bool ok = true; // false: a condensed cell's interior block is singular
  glsOp         op   = mg->ops[0];
  const int64_t n    = op->n_dofs, nf = (int64_t)freel.size(), nc_ = op->n_cells;
  const int     nc   = op->dim + 1, nq = op->nq, ndof = nq * nc;
  std::vector<int32_t> fidx((size_t)n, -1);
  for (int64_t j = 0; j < nf; ++j)
    fidx[(size_t)freel[(size_t)j]] = (int32_t)j;
  // internal cell c -> free index of each local dof (-1: constrained)
  std::vector<int32_t> cdof((size_t)nc_ * ndof);
  std::vector<std::vector<int32_t>> node_cells((size_t)op->n_nodes);
  for (int64_t c = 0; c < nc_; ++c)
    {
      const uint32_t *cn = &op->h_cell_nodes[(size_t)gls::ext_cell(op, c) * nq];
      for (int p = 0; p < nq; ++p)
        {
          node_cells[cn[p]].push_back((int32_t)c);
          for (int k = 0; k < nc; ++k)
            cdof[(size_t)c * ndof + p * nc + k] = fidx[(size_t)cn[p] * nc + k];
        }
    }
  // greedy colouring: the smallest colour no node-sharing neighbour has
  std::vector<int> color((size_t)nc_, -1);
  int              n_colors = 0;
  std::vector<int> seen;
  for (int64_t c = 0; c < nc_; ++c)
    {
      seen.assign((size_t)n_colors + 1, 0);
      const uint32_t *cn = &op->h_cell_nodes[(size_t)gls::ext_cell(op, c) * nq];
      for (int p = 0; p < nq; ++p)
        for (int32_t o : node_cells[cn[p]])
          if (color[(size_t)o] >= 0)
            seen[(size_t)color[(size_t)o]] = 1;
      int k = 0;
      while (seen[(size_t)k])
        ++k;
      color[(size_t)c] = k;
      n_colors         = std::max(n_colors, k + 1);
    }
  std::vector<int32_t> order;
  std::vector<int64_t> cbeg(1, 0);
  for (int k = 0; k < n_colors; ++k)
    {
      for (int64_t c = 0; c < nc_; ++c)
        if (color[(size_t)c] == k)
          order.push_back((int32_t)c);
      cbeg.push_back((int64_t)order.size());
    }
  const size_t eb = (size_t)nc_ * ndof * ndof * sizeof(T);
  void        *E = nullptr, *d_cdof = nullptr, *d_order = nullptr;
  HIP_THROW(hipMallocAsync(&E, eb, s));
  HIP_THROW(hipMallocAsync(&d_cdof, cdof.size() * sizeof(int32_t), s));
  HIP_THROW(hipMallocAsync(&d_order, order.size() * sizeof(int32_t), s));
  HIP_THROW(hipMemcpyAsync(d_cdof, cdof.data(), cdof.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, s));
  HIP_THROW(hipMemcpyAsync(d_order, order.data(), order.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, s));
  gls::op_element_matrices_device(op, E, 0, nc_, s);
  HIP_THROW(hipMemsetAsync(mg->d_lu, 0, (size_t)nf * nf * sizeof(double), s));
  if (!mg->cond)
    {
      const int64_t per = (int64_t)ndof * ndof;
      for (int k = 0; k < n_colors; ++k)
        {
          const int64_t cnt = cbeg[(size_t)k + 1] - cbeg[(size_t)k];
          hipLaunchKernelGGL(k_scatter_emat<T>, g1(cnt * per), dim3(256), 0, s, mg->d_lu, nf,
                             (const T *)E, (const int32_t *)d_cdof,
                             (const int32_t *)d_order + cbeg[(size_t)k], cnt, ndof);
        }
      HIP_THROW(hipGetLastError());
    }
  else
    {
      // element Schur complements over the boundary dofs (k_condense), then
      // assembled like the element matrices
      const int ni = mg->cond_ni, nb = mg->cond_nb;
      std::vector<int32_t> cdb((size_t)nc_ * nb), bfree((size_t)nc_ * nb), cint((size_t)nc_ * ni),
        cbnd((size_t)nc_ * nb);
      for (int64_t c = 0; c < nc_; ++c)
        {
          const uint32_t *cn = &op->h_cell_nodes[(size_t)gls::ext_cell(op, c) * nq];
          for (int b = 0; b < nb; ++b)
            {
              const int     l = mg->cond_lbnd[(size_t)b];
              const int32_t f = cdof[(size_t)c * ndof + l];
              cdb[(size_t)c * nb + b]   = f;
              bfree[(size_t)c * nb + b] = f >= 0 ? 1 : 0;
              cbnd[(size_t)c * nb + b]  = f >= 0 ? (int32_t)(cn[l / nc] * nc + l % nc) : -1;
            }
          for (int m = 0; m < ni; ++m)
            {
              const int l = mg->cond_lint[(size_t)m];
              cint[(size_t)c * ni + m] = (int32_t)(cn[l / nc] * nc + l % nc);
            }
        }
      if (!mg->d_cC)
        {
          HIP_THROW(hipMalloc((void **)&mg->d_cC, (size_t)nc_ * ni * ni * 8));
          HIP_THROW(hipMalloc((void **)&mg->d_cF, (size_t)nc_ * nb * ni * 8));
          HIP_THROW(hipMalloc((void **)&mg->d_cG, (size_t)nc_ * ni * nb * 8));
          HIP_THROW(hipMalloc((void **)&mg->d_cint, (size_t)nc_ * ni * 4));
          HIP_THROW(hipMalloc((void **)&mg->d_cbnd, (size_t)nc_ * nb * 4));
        }
      HIP_THROW(hipMemcpyAsync(mg->d_cint, cint.data(), cint.size() * 4, hipMemcpyHostToDevice, s));
      HIP_THROW(hipMemcpyAsync(mg->d_cbnd, cbnd.data(), cbnd.size() * 4, hipMemcpyHostToDevice, s));
      void *Sd = nullptr, *d_lint = nullptr, *d_lbnd = nullptr, *d_bfree = nullptr, *d_cdb = nullptr;
      HIP_THROW(hipMallocAsync(&Sd, (size_t)nc_ * nb * nb * 8, s));
      HIP_THROW(hipMallocAsync(&d_lint, (size_t)ni * 4, s));
      HIP_THROW(hipMallocAsync(&d_lbnd, (size_t)nb * 4, s));
      HIP_THROW(hipMallocAsync(&d_bfree, bfree.size() * 4, s));
      HIP_THROW(hipMallocAsync(&d_cdb, cdb.size() * 4, s));
      HIP_THROW(hipMemcpyAsync(d_lint, mg->cond_lint.data(), (size_t)ni * 4, hipMemcpyHostToDevice, s));
      HIP_THROW(hipMemcpyAsync(d_lbnd, mg->cond_lbnd.data(), (size_t)nb * 4, hipMemcpyHostToDevice, s));
      HIP_THROW(hipMemcpyAsync(d_bfree, bfree.data(), bfree.size() * 4, hipMemcpyHostToDevice, s));
      HIP_THROW(hipMemcpyAsync(d_cdb, cdb.data(), cdb.size() * 4, hipMemcpyHostToDevice, s));
      int32_t *d_bad = nullptr;
      HIP_THROW(hipMallocAsync((void **)&d_bad, (size_t)nc_ * 4, s));
      HIP_THROW(hipMemsetAsync(d_bad, 0, (size_t)nc_ * 4, s));
      hipLaunchKernelGGL(k_condense<T>, dim3((unsigned)nc_), dim3(256), 0, s, (const T *)E, ndof,
                         (const int32_t *)d_lint, ni, (const int32_t *)d_lbnd, nb,
                         (const int32_t *)d_bfree, (double *)Sd, mg->d_cC, mg->d_cF, mg->d_cG,
                         d_bad);
      std::vector<int32_t> hbad((size_t)nc_);
      HIP_THROW(hipMemcpyAsync(hbad.data(), d_bad, (size_t)nc_ * 4, hipMemcpyDeviceToHost, s));
      HIP_THROW(hipStreamSynchronize(s));
      HIP_THROW(hipFreeAsync(d_bad, s));
      for (int32_t b : hbad)
        ok = ok && b == 0;
      const int64_t per = (int64_t)nb * nb;
      for (int k = 0; k < n_colors; ++k)
        {
          const int64_t cnt = cbeg[(size_t)k + 1] - cbeg[(size_t)k];
          hipLaunchKernelGGL(k_scatter_emat<double>, g1(cnt * per), dim3(256), 0, s, mg->d_lu, nf,
                             (const double *)Sd, (const int32_t *)d_cdb,
                             (const int32_t *)d_order + cbeg[(size_t)k], cnt, nb);
        }
      HIP_THROW(hipGetLastError());
      for (void *q : {Sd, d_lint, d_lbnd, d_bfree, d_cdb})
        HIP_THROW(hipFreeAsync(q, s));
    }
  HIP_THROW(hipFreeAsync(E, s));
  HIP_THROW(hipFreeAsync(d_cdof, s));
  HIP_THROW(hipFreeAsync(d_order, s));
  mg->coarse_colors = n_colors;
  // (the synchronised setup of the caller waits for these launches)
  return ok;
}

// GLS_COARSE_REFERENCE: a comma-separated list of reference forms of the
// dense coarse solver for tests -- "columns" (A_ff assembled column by
// column from unit-vector vmults instead of the element matrices), "getrs"
// / "getri" (the inverse by getrs with the identity / by getri instead of
// U^-1 L^-1), "nocond" (no static condensation)
bool
coarse_reference(const char *what)
{
  const char *e = getenv("GLS_COARSE_REFERENCE");
  if (!e)
    return false;
  const std::string list = std::string(",") + e + ",";
  return list.find(std::string(",") + what + ",") != std::string::npos;
}

// Assemble the coarse level operator into FP64 and LU-factorise it.  Only
// the free (unconstrained) dofs take part: a constrained dof's row and
// column of A are both the unit vector (identity rows of vmult, homogeneous
// constraints read as 0), so A = diag(A_ff, I) in free / constrained order
// and the direct solve is x_c = b_c, x_f = A_ff^{-1} b_f — the same solution
// as the full matrix, on nf^2 instead of n^2 entries (Re3900 r0: 14,206 of
// 16,704 dofs free, 1.61 instead of 2.23 GB).
template <typename T>
void
coarse_lu_setup_t(glsMG_ *mg, hipStream_t s)
{
  glsOp         op = mg->ops[0];
  const int64_t n  = op->n_dofs;
  const int     nc = op->dim + 1;
  if (n > 40000)
    throw std::runtime_error("dense LU coarse solver: coarse level too large");
  std::vector<int32_t> freel;
  freel.reserve((size_t)n);
  for (int64_t d = 0; d < n; ++d)
    if (!((op->h_cmask[(size_t)(d / nc)] >> (d % nc)) & 1))
      freel.push_back((int32_t)d);
  // static condensation of the cells' interior dofs (default with the
  // element-matrix assembly; GLS_COARSE_REFERENCE=nocond off): a node with every
  // lattice coordinate inside (0, k) belongs to one cell only, so its dofs
  // are eliminated cell by cell (Schur complement of the element matrix) and
  // the dense inverse covers the other free dofs (Re3900 r0: 12,606 of
  // 14,206, 0.70x the factorisation flops, 0.79x the GEMV's bytes); the
  // coarse solve adds the condensed right-hand side b_B - F b_I before the
  // GEMV and x_I = C b_I - G x_B after it (k_cond_rhs / k_cond_post)
  const bool columns = coarse_reference("columns");
  {
    const int   k  = op->degree, dim = op->dim, nq = op->nq;
    mg->cond_lint.clear(), mg->cond_lbnd.clear();
    for (int p = 0; p < nq; ++p)
      {
        const int  co[3] = {p % (k + 1), (p / (k + 1)) % (k + 1), dim == 3 ? p / ((k + 1) * (k + 1)) : 1};
        const bool in    = co[0] > 0 && co[0] < k && co[1] > 0 && co[1] < k && co[2] > 0 && co[2] < k;
        for (int q = 0; q < nc; ++q)
          (in ? mg->cond_lint : mg->cond_lbnd).push_back(p * nc + q);
      }
    const int ni = (int)mg->cond_lint.size(), nb = (int)mg->cond_lbnd.size();
    bool      cond = !columns && !coarse_reference("nocond") && !mg->cond_failed && ni > 0 && ni <= COND_MAXI &&
                nb <= 128 && nb * ni <= 1024;
    std::vector<char> is_int((size_t)n, 0);
    for (int64_t c = 0; cond && c < op->n_cells; ++c)
      {
        const uint32_t *cn = &op->h_cell_nodes[(size_t)gls::ext_cell(op, c) * nq];
        for (int m = 0; m < ni && cond; ++m)
          {
            const int     l = mg->cond_lint[(size_t)m];
            const int64_t d = (int64_t)cn[l / nc] * nc + l % nc;
            // every interior dof free and in this cell alone
            if (((op->h_cmask[(size_t)cn[l / nc]] >> (l % nc)) & 1) || is_int[(size_t)d])
              cond = false;
            is_int[(size_t)d] = 1;
          }
      }
    mg->cond = cond, mg->cond_ni = ni, mg->cond_nb = nb;
    if (cond)
      {
        std::vector<int32_t> rl;
        rl.reserve(freel.size());
        for (int32_t d : freel)
          if (!is_int[(size_t)d])
            rl.push_back(d);
        freel.swap(rl);
      }
  }
  const int64_t nf = (int64_t)freel.size();
  if (nf == 0)
    throw std::runtime_error("dense LU coarse solver: no free coarse dofs");
  if (!mg->blas)
    check_blas(rocblas_create_handle(&mg->blas), "rocblas_create_handle");
  check_blas(rocblas_set_stream(mg->blas, s), "rocblas_set_stream");
  if (mg->d_free && mg->n_free != nf)
    throw std::runtime_error("dense LU coarse solver: constrained dofs changed");
  // the FP64 factors are released after an FP32 setup (k_narrow below)
  if (!mg->d_lu)
    HIP_THROW(hipMalloc((void **)&mg->d_lu, (size_t)nf * nf * sizeof(double)));
  if (!mg->d_ipiv)
    HIP_THROW(hipMalloc((void **)&mg->d_ipiv, (size_t)nf * sizeof(rocblas_int)));
  if (!mg->d_free)
    {
      HIP_THROW(hipMalloc((void **)&mg->d_info, sizeof(rocblas_int)));
      mg->ld_free = (nf + 3) / 4 * 4;
      HIP_THROW(hipMalloc((void **)&mg->d_rhs,
                          (size_t)(2 + GEMV_CHUNKS) * mg->ld_free * sizeof(double)));
      HIP_THROW(hipMalloc((void **)&mg->d_free, (size_t)nf * sizeof(int32_t)));
      HIP_THROW(hipMalloc((void **)&mg->d_free_in, (size_t)nf * sizeof(int32_t)));
      mg->n_free = nf;
    }
  if (mg->n_free != nf)
    throw std::runtime_error("dense LU coarse solver: constrained dofs changed");
  HIP_THROW(hipMemcpyAsync(mg->d_free, freel.data(), (size_t)nf * sizeof(int32_t),
                           hipMemcpyHostToDevice, s));
  const auto  t0 = std::chrono::steady_clock::now();
  if (columns)
    {
      // reference path of the assembly test: A_ff column by column from
      // unit-vector vmults (nf vmults of the level operator)
      T *e = (T *)mg->sol[0], *col = (T *)mg->tmp[0];
      HIP_THROW(hipMemsetAsync(e, 0, n * sizeof(T), s));
      for (int64_t j = 0; j < nf; ++j)
        {
          const int64_t dj = freel[(size_t)j];
          hipLaunchKernelGGL(k_set_unit<T>, g1(n), dim3(256), 0, s, e, dj, n, 1);
          gls::op_vmult_device(op, col, e, s);
          hipLaunchKernelGGL(k_gather_free<T>, g1(nf), dim3(256), 0, s,
                             mg->d_lu + (size_t)j * nf, (const T *)col,
                             (const int32_t *)mg->d_free, nf);
          hipLaunchKernelGGL(k_set_unit<T>, g1(n), dim3(256), 0, s, e, dj, n, 0);
        }
      HIP_THROW(hipGetLastError());
    }
  else if (!assemble_free_block<T>(mg, freel, s))
    {
      // a cell's interior block E_II is singular: start over without the
      // static condensation (the free-dof buffers are sized for nf)
      HIP_THROW(hipStreamSynchronize(s));
      for (void **q : {(void **)&mg->d_lu, (void **)&mg->d_ipiv, (void **)&mg->d_info,
                       (void **)&mg->d_rhs, (void **)&mg->d_free, (void **)&mg->d_free_in})
        {
          HIP_THROW(hipFree(*q));
          *q = nullptr;
        }
      mg->n_free      = 0;
      mg->cond        = false;
      mg->cond_failed = true;
      fprintf(stderr, "[glsamd] coarse solver: singular interior block in a coarse cell, "
                      "assembling without static condensation\n");
      return coarse_lu_setup_t<T>(mg, s);
    }
  HIP_THROW(hipStreamSynchronize(s));
  const auto t1 = std::chrono::steady_clock::now();
  check_blas(rocsolver_dgetrf(mg->blas, (rocblas_int)nf, (rocblas_int)nf, mg->d_lu,
                              (rocblas_int)nf, mg->d_ipiv, mg->d_info),
             "rocsolver_dgetrf");
  rocblas_int info = 0;
  HIP_THROW(hipMemcpyAsync(&info, mg->d_info, sizeof(info), hipMemcpyDeviceToHost, s));
  HIP_THROW(hipStreamSynchronize(s));
  const auto t2 = std::chrono::steady_clock::now();
  if (info != 0)
    throw std::runtime_error("dense LU coarse solver: singular coarse matrix (info " +
                             std::to_string(info) + ")");
  // the inverse from the LU factors, once: every coarse solve is then one
  // GEMV streaming the nf x nf matrix at HBM rate (the two triangular solves
  // of getrs ran 33.7 ms per V-cycle at n = 16,704 on MI355X).  Default
  // Z = U^-1 L^-1 from the unit lower
  // factor inverted in place (rocsolver_dtrtri, n^3 / 3 flops) and one
  // triangular solve with U (rocblas_dtrsm, n^3): 4/3 n^3 instead of the
  // 2 n^3 of getrs with the identity, and A^-1 = Z P^T needs no column
  // permutation of the matrix: the GEMV gathers its input through free[p[i]]
  // (d_free_in).  Reference forms (GLS_COARSE_REFERENCE): "getrs", the
  // identity as right-hand side (rocsolver dgetrs); "getri", rocsolver_dgetri
  // in place.
  std::vector<int32_t> fin = freel; // the GEMV's input gather
  const std::string inv_mode = coarse_reference("getri") ? "getri" :
                               coarse_reference("getrs") ? "getrs" : "trtri";
  if (inv_mode == "getri")
    {
      check_blas(rocsolver_dgetri(mg->blas, (rocblas_int)nf, mg->d_lu, (rocblas_int)nf,
                                  mg->d_ipiv, mg->d_info),
                 "rocsolver_dgetri");
      HIP_THROW(hipMemcpyAsync(&info, mg->d_info, sizeof(info), hipMemcpyDeviceToHost, s));
      HIP_THROW(hipStreamSynchronize(s));
      if (info != 0)
        throw std::runtime_error("dense LU coarse solver: singular coarse matrix in getri "
                                 "(info " + std::to_string(info) + ")");
    }
  else
    {
      const bool trtri = inv_mode != "getrs";
      double    *X     = nullptr;
      HIP_THROW(hipMalloc((void **)&X, (size_t)nf * nf * sizeof(double)));
      try
        {
          if (trtri)
            {
              hipLaunchKernelGGL(k_unit_lower, g1(nf * nf), dim3(256), 0, s, X,
                                 (const double *)mg->d_lu, nf);
              HIP_THROW(hipGetLastError());
              check_blas(rocsolver_dtrtri(mg->blas, rocblas_fill_lower, rocblas_diagonal_unit,
                                          (rocblas_int)nf, X, (rocblas_int)nf, mg->d_info),
                         "rocsolver_dtrtri");
              const double one = 1.0;
              check_blas(rocblas_set_pointer_mode(mg->blas, rocblas_pointer_mode_host),
                         "pointer mode");
              check_blas(rocblas_dtrsm(mg->blas, rocblas_side_left, rocblas_fill_upper,
                                       rocblas_operation_none, rocblas_diagonal_non_unit,
                                       (rocblas_int)nf, (rocblas_int)nf, &one, mg->d_lu,
                                       (rocblas_int)nf, X, (rocblas_int)nf),
                         "rocblas_dtrsm");
              // P^T from the pivots (1-based row interchanges, in order)
              std::vector<rocblas_int> ip((size_t)nf);
              HIP_THROW(hipMemcpyAsync(ip.data(), mg->d_ipiv, (size_t)nf * sizeof(rocblas_int),
                                       hipMemcpyDeviceToHost, s));
              HIP_THROW(hipMemcpyAsync(&info, mg->d_info, sizeof(info), hipMemcpyDeviceToHost, s));
              HIP_THROW(hipStreamSynchronize(s));
              if (info != 0)
                throw std::runtime_error("dense LU coarse solver: singular unit factor (info " +
                                         std::to_string(info) + ")");
              std::vector<int32_t> p((size_t)nf);
              for (int64_t i = 0; i < nf; ++i)
                p[(size_t)i] = (int32_t)i;
              for (int64_t j = 0; j < nf; ++j)
                std::swap(p[(size_t)j], p[(size_t)ip[(size_t)j] - 1]);
              for (int64_t i = 0; i < nf; ++i)
                fin[(size_t)i] = freel[(size_t)p[(size_t)i]];
            }
          else
            {
              HIP_THROW(hipMemsetAsync(X, 0, (size_t)nf * nf * sizeof(double), s));
              hipLaunchKernelGGL(k_set_diag, g1(nf), dim3(256), 0, s, X, nf);
              HIP_THROW(hipGetLastError());
              check_blas(rocsolver_dgetrs(mg->blas, rocblas_operation_none, (rocblas_int)nf,
                                          (rocblas_int)nf, mg->d_lu, (rocblas_int)nf, mg->d_ipiv,
                                          X, (rocblas_int)nf),
                         "rocsolver_dgetrs");
            }
          HIP_THROW(hipStreamSynchronize(s));
        }
      catch (...)
        {
          (void)hipFree(X);
          throw;
        }
      HIP_THROW(hipFree(mg->d_lu));
      mg->d_lu = X;
    }
  HIP_THROW(hipMemcpyAsync(mg->d_free_in, fin.data(), (size_t)nf * sizeof(int32_t),
                           hipMemcpyHostToDevice, s));
  if (mg->cond)
    {
      // per GEMV column i: the (cell, boundary slot) pairs of dof fin[i]
      const int     nb = mg->cond_nb, nq = op->nq;
      std::vector<std::vector<int32_t>> at((size_t)n);
      for (int64_t c = 0; c < op->n_cells; ++c)
        {
          const uint32_t *cn = &op->h_cell_nodes[(size_t)gls::ext_cell(op, c) * nq];
          for (int b = 0; b < nb; ++b)
            {
              const int     l = mg->cond_lbnd[(size_t)b];
              const int64_t d = (int64_t)cn[l / nc] * nc + l % nc;
              if (!((op->h_cmask[(size_t)cn[l / nc]] >> (l % nc)) & 1))
                at[(size_t)d].push_back((int32_t)(c * nb + b));
            }
        }
      std::vector<int32_t> off(1, 0), ent;
      for (int64_t i = 0; i < nf; ++i)
        {
          for (int32_t e : at[(size_t)fin[(size_t)i]])
            ent.push_back(e);
          off.push_back((int32_t)ent.size());
        }
      for (int32_t **q : {&mg->d_rg_off, &mg->d_rg_ent})
        if (*q)
          {
            HIP_THROW(hipStreamSynchronize(s));
            HIP_THROW(hipFree(*q));
            *q = nullptr;
          }
      HIP_THROW(hipMalloc((void **)&mg->d_rg_off, off.size() * 4));
      HIP_THROW(hipMalloc((void **)&mg->d_rg_ent, std::max<size_t>(1, ent.size()) * 4));
      HIP_THROW(hipMemcpy(mg->d_rg_off, off.data(), off.size() * 4, hipMemcpyHostToDevice));
      if (!ent.empty())
        HIP_THROW(hipMemcpy(mg->d_rg_ent, ent.data(), ent.size() * 4, hipMemcpyHostToDevice));
    }
  const auto t3 = std::chrono::steady_clock::now();
  auto       ms = [](auto a, auto b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  mg->coarse_setup_ms[0] = ms(t0, t1);
  mg->coarse_setup_ms[1] = ms(t1, t2);
  mg->coarse_setup_ms[2] = ms(t2, t3);
  // FP32 levels keep an FP32 copy of the inverse (FP64 sums): half the bytes
  // per coarse solve; the Re3900 r0..r2 V-cycle differs from the FP64-stored
  // inverse's by 2.1e-7 (relative l2), the FP32 level arithmetic's own
  // round-off.  GLS_COARSE_INV_F32=0 keeps the FP64 inverse.
  const char *e32 = getenv("GLS_COARSE_INV_F32");
  mg->inv_f32     = !(e32 && e32[0] == '0') && mg->prec == GLS_F32;
  if (mg->inv_f32)
    {
      const int64_t ld = mg->ld_free;
      if (!mg->d_inv32)
        HIP_THROW(hipMalloc((void **)&mg->d_inv32, (size_t)nf * ld * sizeof(float)));
      hipLaunchKernelGGL(k_narrow, g1(nf * ld), dim3(256), 0, s, mg->d_inv32,
                         (const double *)mg->d_lu, nf, ld);
      HIP_THROW(hipGetLastError());
      // the FP32 solve reads d_inv32 only: release the nf x nf FP64 factors
      // (1.6 GB at Re3900 r0) and the pivots; a re-setup allocates them again
      HIP_THROW(hipStreamSynchronize(s));
      HIP_THROW(hipFree(mg->d_lu));
      HIP_THROW(hipFree(mg->d_ipiv));
      mg->d_lu   = nullptr;
      mg->d_ipiv = nullptr;
    }
}

// the condensed coarse right-hand side into out (GEMV column order, padded
// to ld_free) and sol = def; then, after the GEMV, the interior dofs
template <typename T, typename O>
void
cond_rhs_t(glsMG_ *mg, O *out, hipStream_t s)
{
  const int64_t n = mg->ops[0]->n_dofs;
  hipLaunchKernelGGL((k_cond_rhs<T, O>), g1(std::max(n, 8 * mg->ld_free)), dim3(256), 0, s,
                     (T *)mg->sol[0], (const T *)mg->def[0], out,
                     (const int32_t *)mg->d_free_in, (const int32_t *)mg->d_rg_off,
                     (const int32_t *)mg->d_rg_ent, (const double *)mg->d_cF,
                     (const int32_t *)mg->d_cint, mg->cond_ni, mg->cond_nb, n, mg->n_free,
                     mg->ld_free);
  HIP_THROW(hipGetLastError());
}

template <typename T>
void
cond_post_t(glsMG_ *mg, hipStream_t s)
{
  const int64_t nc_ = mg->ops[0]->n_cells;
  hipLaunchKernelGGL(k_cond_post<T>, g1(64 * nc_ * mg->cond_ni), dim3(256), 0, s,
                     (T *)mg->sol[0], (const T *)mg->def[0], (const double *)mg->d_cC,
                     (const double *)mg->d_cG, (const int32_t *)mg->d_cint,
                     (const int32_t *)mg->d_cbnd, mg->cond_ni, mg->cond_nb, nc_);
  HIP_THROW(hipGetLastError());
}

template <typename T>
void
coarse_lu_solve_t(glsMG_ *mg, hipStream_t s)
{
  const int64_t n = mg->ops[0]->n_dofs, nf = mg->n_free, ld = mg->ld_free;
  if (mg->inv_f32)
    {
      // sol = def (constrained dofs: x_c = b_c, their rows of A are the
      // identity), then sol[free] = A_ff^{-1} def[free], one wave per row
      float *xf = reinterpret_cast<float *>(mg->d_rhs);
      if (mg->cond)
        cond_rhs_t<T, float>(mg, xf, s);
      else
        hipLaunchKernelGGL(k_coarse_prep<T>, g1(std::max(n, ld)), dim3(256), 0, s,
                           (T *)mg->sol[0], (const T *)mg->def[0], xf,
                           (const int32_t *)mg->d_free_in, n, nf, ld);
      // the inverse is read once per solve and is larger than the MALL:
      // non-temporal row loads (132 against 146 us with the default policy,
      // round 3)
      hipLaunchKernelGGL((k_gemv_rows_f32<T, true>), dim3((unsigned)((nf + 3) / 4)), dim3(256), 0,
                         s, (const float4 *)mg->d_inv32, (const float4 *)xf, (T *)mg->sol[0],
                         (const int32_t *)mg->d_free, nf, ld);
      HIP_THROW(hipGetLastError());
      if (mg->cond)
        cond_post_t<T>(mg, s);
      return;
    }
  // constrained dofs: x_c = b_c (their rows of A are the identity)
  if (mg->cond)
    cond_rhs_t<T, double>(mg, mg->d_rhs, s);
  else
    {
      copy_words(mg->sol[0], mg->def[0], n * (int64_t)sizeof(T) / 4, s);
      hipLaunchKernelGGL(k_gather_free<T>, g1(nf), dim3(256), 0, s, mg->d_rhs,
                         (const T *)mg->def[0], (const int32_t *)mg->d_free_in, nf);
    }
  double *part = mg->d_rhs + 2 * ld;
  hipLaunchKernelGGL(k_gemv_part<double>, dim3((unsigned)((nf + 255) / 256), GEMV_CHUNKS),
                     dim3(256), 0, s, (const double *)mg->d_lu, (const double *)mg->d_rhs, part,
                     nf, ld);
  hipLaunchKernelGGL(k_gemv_sum<T>, g1(nf), dim3(256), 0, s, (const double *)part,
                     (T *)mg->sol[0], (const int32_t *)mg->d_free, nf, ld);
  HIP_THROW(hipGetLastError());
  if (mg->cond)
    cond_post_t<T>(mg, s);
}

void v_step(glsMG_ *mg, int l, hipStream_t s);

void
check_amg(glsStatus st)
{
  if (st != 0)
    throw std::runtime_error(std::string("coarse AMG: ") + gls_last_error());
}

// the coarse "preconditioner" once: sol[0] from def[0] (multigrid.cc:465-489):
// dense LU (< 0), identity (0) or relaxation sweeps (> 0)
void
coarse_apply(glsMG_ *mg, hipStream_t s, PendingReduce *pend = nullptr)
{
  const size_t bytes = (size_t)mg->ops[0]->n_dofs * mg->ts();
  if (mg->desc.coarse_amg)
    {
      // one AMG V-cycle as the coarse solver (coarse_iterate = 0): in FP64
      const int64_t n = mg->ops[0]->n_dofs;
      if (mg->prec == GLS_F64)
        check_amg(gls_amg_vmult(mg->amg, (double *)mg->sol[0], (const double *)mg->def[0], s));
      else
        {
          hipLaunchKernelGGL((k_convert<float, double>), g1(n), dim3(256), 0, s, mg->amg_io,
                             (const float *)mg->def[0], n);
          check_amg(gls_amg_vmult(mg->amg, mg->amg_io + n, mg->amg_io, s));
          hipLaunchKernelGGL((k_convert<double, float>), g1(n), dim3(256), 0, s,
                             (float *)mg->sol[0], mg->amg_io + n, n);
        }
      HIP_THROW(hipGetLastError());
    }
  else if (mg->desc.coarse_n_iterations < 0)
    {
      if (mg->prec == GLS_F64)
        coarse_lu_solve_t<double>(mg, s);
      else
        coarse_lu_solve_t<float>(mg, s);
    }
  else if (mg->desc.coarse_n_iterations == 0)
    {
      copy_words(mg->sol[0], mg->def[0], (int64_t)(bytes / 4), s);
    }
  else
    smooth(mg, 0, mg->sol[0], mg->def[0], true, mg->desc.coarse_n_iterations, s, false, nullptr,
           pend);
}

// r = b - r (the coarse GMRES restart residual)
__global__ void
k_sub(double *__restrict__ r, const double *__restrict__ b, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    r[i] = b[i] - r[i];
}

// coarse_grid_iterate (multigrid.cc:491-530, MGCoarseGridIterativeSolver):
// SolverGMRES<VectorType<double>> with deal.II's defaults (left
// preconditioning, max_n_tmp_vectors 30 -> restart after 28) under
// ReductionControl(maxiter, 1e-20, reltol) on the coarse level operator,
// preconditioned by coarse_apply (the substitute for Trilinos AMG / ILU:
// relaxation sweeps or the dense LU).  FP64 Krylov vectors, the level
// operator and preconditioner in the level precision (the reference solves
// with the FP64 system matrix assembled from the MGNumber operator).  Every
// vector stays on the device.  The Arnoldi step runs as the outer solver's
// (krylov.hip): fused CGS2 passes (cgs.h), |w| and v_{j+1} = w / |w| on the
// device, and step j + 1 enqueued before the host waits for step j's
// Hessenberg column (pinned, double-buffered), so the device never idles
// through the host round trip; a converged solve runs one discarded step.
template <typename T>
void
coarse_gmres_t(glsMG_ *mg, hipStream_t s)
{
  glsOp         op = mg->ops[0];
  const int64_t n  = op->n_dofs;
  const int     m  = 28;
  const int     HC = 2 * (m + 1) + 1; // both CGS passes' coefficients and |w|
  if (n > (int64_t)0x7fffffff)
    throw std::runtime_error("coarse GMRES: level too large for 32-bit rocBLAS sizes");
  if (!mg->blas)
    check_blas(rocblas_create_handle(&mg->blas), "rocblas_create_handle");
  check_blas(rocblas_set_stream(mg->blas, s), "rocblas_set_stream");
  check_blas(rocblas_set_pointer_mode(mg->blas, rocblas_pointer_mode_host), "pointer mode");
  rocblas_handle h = mg->blas;
  if (!mg->cg_ws)
    {
      HIP_THROW(hipMalloc((void **)&mg->cg_ws,
                          ((size_t)(m + 4) * n + HC + (size_t)CGS_PART) * 8));
      HIP_THROW(hipMalloc(&mg->cg_lvl, (size_t)2 * n * sizeof(T)));
      HIP_THROW(hipHostMalloc((void **)&mg->cg_host, (size_t)2 * HC * 8,
                              hipHostMallocMapped | hipHostMallocCoherent));
      for (hipEvent_t &e : mg->cg_ev)
        HIP_THROW(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
  double *V = mg->cg_ws, *w = V + (size_t)(m + 1) * n, *x = w + n, *b = x + n,
         *dh = b + n, *cpart = dh + HC;
  double *host_dev = nullptr; // cg_host as the device sees it (k_cgs_unit writes it)
  HIP_THROW(hipHostGetDevicePointer((void **)&host_dev, mg->cg_host, 0));
  T *la = (T *)mg->cg_lvl, *lb = la + n;
  auto cvt_in = [&](T *dst, const double *src) {
    hipLaunchKernelGGL((k_convert<double, T>), g1(n), dim3(256), 0, s, dst, src, n);
  };
  auto cvt_out = [&](double *dst, const T *src) {
    hipLaunchKernelGGL((k_convert<T, double>), g1(n), dim3(256), 0, s, dst, src, n);
  };
  // dst = P^{-1} src (through def[0] -> sol[0]); AMG: its V-cycle on the
  // FP64 vectors directly (the reference's Trilinos AMG on the FP64 matrix)
  auto prec = [&](double *dst, const double *src) {
    if (mg->desc.coarse_amg)
      {
        check_amg(gls_amg_vmult(mg->amg, dst, src, s));
        return;
      }
    cvt_in((T *)mg->def[0], src);
    coarse_apply(mg, s);
    cvt_out(dst, (const T *)mg->sol[0]);
  };
  // FP32 brick levels: the FP64 result written by the brick write-out and
  // the reduction themselves (RelaxStep.out64), no conversion pass
  const bool fused_out = std::is_same<T, float>::value && gls::deferred_reduce_ok(op);
  auto apply_A = [&](double *dst, const double *src) {
    cvt_in(la, src);
    if (fused_out)
      {
        gls::RelaxStep r;
        r.out64 = dst;
        gls::brick_launch(op, gls::op_vmult_mode(op), lb, la, 0, op->n_bricks,
                          gls::BRICK_RUN | gls::BRICK_REDUCE, s, &r);
      }
    else
      {
        gls::op_vmult_device(op, lb, la, s);
        cvt_out(dst, lb);
      }
  };
  auto nrm2 = [&](const double *v) {
    double r = 0;
    check_blas(rocblas_dnrm2(h, (rocblas_int)n, v, 1, &r), "rocblas_dnrm2");
    return r;
  };
  auto vc = [&](int j) { return V + (size_t)j * n; };
  // Arnoldi step j, enqueued only: v_{j+1} = P^{-1} A v_j orthogonalised
  // (CGS2) and normalised on the device, its Hessenberg column to pinned
  // host buffer j % 2 (event cg_ev[j % 2])
  auto arnoldi = [&](int j) {
    apply_A(w, vc(j));
    double *wv = vc(j + 1);
    prec(wv, w);
    double *hn = dh + 2 * (m + 1);
    const int J         = j + 1;
    bool      unit_done = false;
    if (J < CGS_MAXJ)
      {
        // CGS2 with the second update folded into the normalisation
        // (krylov.hip, cgs.h k_cgs_unit)
        hipLaunchKernelGGL(k_cgs_dots, dim3(CGS_BLOCKS), dim3(256), 0, s, (const double *)V, J,
                           (const double *)wv, cpart, n, n);
        hipLaunchKernelGGL(k_cgs_finish, dim3(J), dim3(256), 0, s, (const double *)cpart, dh, 0);
        hipLaunchKernelGGL(k_cgs_update, dim3(CGS_BLOCKS), dim3(256), 0, s, (const double *)V, J,
                           (const double *)dh, wv, cpart, n, n, n, 2);
        hipLaunchKernelGGL(k_cgs_finish, dim3(J + 1), dim3(256), 0, s, (const double *)cpart,
                           dh + (m + 1), 0);
        hipLaunchKernelGGL(k_cgs_unit, dim3(CGS_BLOCKS), dim3(256), 0, s, (const double *)V, J,
                           (const double *)(dh + (m + 1)), (const double *)wv, wv, hn, n, n,
                           (const double *)dh, host_dev + (j % 2) * HC, HC, 2 * (m + 1));
        HIP_THROW(hipGetLastError());
        unit_done = true;
      }
    else if (J <= CGS_MAXJ)
      {
        hipLaunchKernelGGL(k_cgs_dots, dim3(CGS_BLOCKS), dim3(256), 0, s, (const double *)V, J,
                           (const double *)wv, cpart, n, n);
        hipLaunchKernelGGL(k_cgs_finish, dim3(J), dim3(256), 0, s, (const double *)cpart, dh, 0);
        hipLaunchKernelGGL(k_cgs_update, dim3(CGS_BLOCKS), dim3(256), 0, s, (const double *)V, J,
                           (const double *)dh, wv, cpart, n, n, n, 0);
        hipLaunchKernelGGL(k_cgs_finish, dim3(J), dim3(256), 0, s, (const double *)cpart,
                           dh + (m + 1), 0);
        hipLaunchKernelGGL(k_cgs_update, dim3(CGS_BLOCKS), dim3(256), 0, s, (const double *)V, J,
                           (const double *)(dh + (m + 1)), wv, cpart, n, n, n, 1);
        hipLaunchKernelGGL(k_cgs_finish, dim3(1), dim3(256), 0, s, (const double *)cpart, hn, 1);
        HIP_THROW(hipGetLastError());
      }
    else
      {
        const double one = 1.0, zero = 0.0, mone = -1.0;
        for (int pass = 0; pass < 2; ++pass)
          {
            double *hp = dh + pass * (m + 1);
            check_blas(rocblas_dgemv(h, rocblas_operation_transpose, (rocblas_int)n, J, &one, V,
                                     (rocblas_int)n, wv, 1, &zero, hp, 1),
                       "rocblas_dgemv");
            check_blas(rocblas_dgemv(h, rocblas_operation_none, (rocblas_int)n, J, &mone, V,
                                     (rocblas_int)n, hp, 1, &one, wv, 1),
                       "rocblas_dgemv");
          }
        check_blas(rocblas_set_pointer_mode(h, rocblas_pointer_mode_device), "pointer mode");
        check_blas(rocblas_dnrm2(h, (rocblas_int)n, wv, 1, hn), "rocblas_dnrm2");
        check_blas(rocblas_set_pointer_mode(h, rocblas_pointer_mode_host), "pointer mode");
      }
    if (!unit_done)
      HIP_THROW(hipMemcpyAsync(mg->cg_host + (j % 2) * HC, dh, HC * 8, hipMemcpyDeviceToHost, s));
    HIP_THROW(hipEventRecord(mg->cg_ev[j % 2], s));
    if (!unit_done)
      hipLaunchKernelGGL(k_unit_col, g1(n), dim3(256), 0, s, wv, (const double *)wv,
                         (const double *)hn, n);
    HIP_THROW(hipGetLastError());
  };
  cvt_out(b, (const T *)mg->def[0]);
  HIP_THROW(hipMemsetAsync(x, 0, n * 8, s));
  // r0 = P^{-1} (b - A 0)
  prec(vc(0), b);
  double       res = nrm2(vc(0));
  const double tol = std::max(mg->desc.coarse_reltol * res, 1e-20);
  int          it  = 0;
  std::vector<double> H((size_t)(m + 1) * m), g(m + 1), cs(m), sn(m), y(m);
  while (res > tol && it < mg->desc.coarse_maxiter)
    {
      const double sc = 1.0 / res;
      check_blas(rocblas_dscal(h, (rocblas_int)n, &sc, vc(0), 1), "rocblas_dscal");
      std::fill(g.begin(), g.end(), 0.0);
      g[0]   = res;
      int jd = 0;
      arnoldi(0);
      for (int j = 0; j < m && it < mg->desc.coarse_maxiter; ++j)
        {
          if (j + 1 < m && it + 1 < mg->desc.coarse_maxiter)
            arnoldi(j + 1);
          HIP_THROW(hipEventSynchronize(mg->cg_ev[j % 2]));
          const double *hc = mg->cg_host + (j % 2) * HC;
          const double  hn = hc[2 * (m + 1)];
          double       *Hj = &H[(size_t)j * (m + 1)];
          for (int i = 0; i <= j; ++i)
            Hj[i] = hc[i] + hc[(m + 1) + i];
          Hj[j + 1] = hn;
          for (int i = 0; i < j; ++i)
            {
              const double t = cs[i] * Hj[i] + sn[i] * Hj[i + 1];
              Hj[i + 1]      = -sn[i] * Hj[i] + cs[i] * Hj[i + 1];
              Hj[i]          = t;
            }
          const double rr = std::hypot(Hj[j], Hj[j + 1]);
          cs[j]           = rr > 0 ? Hj[j] / rr : 1.0;
          sn[j]           = rr > 0 ? Hj[j + 1] / rr : 0.0;
          Hj[j]           = rr;
          Hj[j + 1]       = 0;
          g[j + 1]        = -sn[j] * g[j];
          g[j]            = cs[j] * g[j];
          ++it;
          ++jd;
          res = std::fabs(g[j + 1]);
          if (res <= tol || hn == 0)
            break;
        }
      // x += V y (left preconditioning: the update is in the Krylov space)
      for (int i = jd - 1; i >= 0; --i)
        {
          double t = g[i];
          for (int c = i + 1; c < jd; ++c)
            t -= H[(size_t)c * (m + 1) + i] * y[c];
          y[i] = t / H[(size_t)i * (m + 1) + i];
        }
      HIP_THROW(hipMemcpyAsync(dh, y.data(), jd * 8, hipMemcpyHostToDevice, s));
      {
        const double one = 1.0;
        check_blas(rocblas_dgemv(h, rocblas_operation_none, (rocblas_int)n, jd, &one, V,
                                 (rocblas_int)n, dh, 1, &one, x, 1),
                   "rocblas_dgemv");
      }
      HIP_THROW(hipStreamSynchronize(s)); // y is a host buffer reused below
      if (res <= tol || it >= mg->desc.coarse_maxiter)
        break;
      // restart: r = P^{-1} (b - A x)
      apply_A(w, x);
      hipLaunchKernelGGL(k_sub, g1(n), dim3(256), 0, s, w, b, n);
      prec(vc(0), w);
      res = nrm2(vc(0));
    }
  mg->cg_iters = it;
  mg->cg_conv  = res <= tol;
  // deal.II's SolverGMRES inside MGCoarseGridIterativeSolver throws
  // SolverControl::NoConvergence when maxiter is reached (multigrid.cc:
  // 494-530): the V-cycle fails the same way instead of continuing with an
  // unconverged coarse correction
  if (!mg->cg_conv)
    throw std::runtime_error("coarse GMRES: no convergence in " + std::to_string(it) +
                             " iterations (residual " + std::to_string(res) + ", tolerance " +
                             std::to_string(tol) + "; SolverControl::NoConvergence)");
  cvt_in((T *)mg->sol[0], x);
  HIP_THROW(hipGetLastError());
}

// Multigrid::level_v_step (deal.II default V-cycle): solution[l] from defect[l]
void v_step_body(glsMG_ *mg, int l, hipStream_t s);
void
v_step(glsMG_ *mg, int l, hipStream_t s)
{
  // a deferred reduction handed to the next transfer (rq_level / pp_level)
  // must not outlive a failed step: a later transfer of that level would read
  // stale slots and vectors
  try
    {
      v_step_body(mg, l, s);
    }
  catch (...)
    {
      mg->rq_level = -1;
      mg->pp_level = -1;
      throw;
    }
}

void
v_step_body(glsMG_ *mg, int l, hipStream_t s)
{
  const std::vector<std::string> &sec = mg->sec[(size_t)l];
  if (l == 0 && mg->desc.coarse_iterate)
    {
      gls::Section sc(sec[5], s);
      if (mg->prec == GLS_F64)
        coarse_gmres_t<double>(mg, s);
      else
        coarse_gmres_t<float>(mg, s);
      return;
    }
  // the last smoothing step's reduction of a level below the finest handed
  // to the prolongation that reads its result (GLS_MG_DEFER=0: off)
  auto hand_over = [&](int lc, const PendingReduce &p) {
    if (!p.valid)
      return;
    mg->pp_level = lc + 1, mg->pp_slots = p.slots, mg->pp_prev = p.src;
    mg->pp_b = p.b, mg->pp_d = p.d, mg->pp_omega = p.omega;
  };
  const bool pro_ok = [&](int lc) {
    return mg->prec == GLS_F32 && mg->dim == 3 && lc + 1 < (int)mg->ops.size() &&
           defer_reduce(mg, lc);
  }(l);
  if (l == 0)
    {
      gls::Section  sc(sec[5], s);
      PendingReduce pc;
      coarse_apply(mg, s, pro_ok ? &pc : nullptr);
      hand_over(0, pc);
      return;
    }
  const int nit = mg->desc.smoothing_n_iterations;
  // pre-smoothing from a zero initial guess (MGSmootherPrecondition::apply);
  // its first relaxation also zeroes the coarser defect for the restriction
  // (and on the finest level converts the outer defect, mg->top_b64)
  FirstRelax fr;
  fr.zero       = (uint32_t *)mg->def[l - 1];
  fr.zero_words = (int64_t)((size_t)mg->ops[l - 1]->n_dofs * mg->ts() / 4);
  fr.b64        = l == (int)mg->ops.size() - 1 ? mg->top_b64 : nullptr;
  PendingReduce pend;
  bool          folded;
  {
    gls::Section sc(sec[0], s);
    folded = smooth(mg, l, mg->sol[l], mg->def[l], true, nit, s, false, &fr, &pend);
    if (!folded && fr.b64)
      {
        const int64_t n = mg->ops[l]->n_dofs;
        hipLaunchKernelGGL((k_convert<double, float>), g1(n), dim3(256), 0, s,
                           (float *)mg->def[l], fr.b64, n);
        HIP_THROW(hipGetLastError());
      }
  }
  // residual t = defect - A solution (fused into the brick vmult's write-out
  // and shared-node reduction for brick operators)
  std::unique_ptr<gls::Section> sc_res(new gls::Section(sec[1], s));
  if (gls::fused_relax_ok(mg->ops[l]))
    {
      gls::RelaxStep rs;
      rs.b     = mg->def[l];
      rs.omega = 1.0;
      rs.keep  = false;
      if (pend.valid) // the pre-smoothing's last reduction, rebuilt in this gather
        {
          rs.prev_partial = pend.slots, rs.prev_src = pend.src;
          rs.prev_b = pend.b, rs.prev_d = pend.d, rs.prev_omega = pend.omega;
        }
      // the residual's own reduction deferred into the restriction's gather
      // (its only reader: the prolongation overwrites tmp afterwards), into
      // the slot buffer the pre-smoothing's pending slots do not occupy
      if (defer_reduce(mg, l) && mg->prec == GLS_F32 && mg->ops[l]->dim == 3)
        {
          void *q0   = mg->qslot[0][(size_t)l], *q1 = mg->qslot[1][(size_t)l];
          rs.defer   = true;
          rs.partial = pend.valid && pend.slots == q0 ? q1 : q0;
        }
      gls::brick_launch(mg->ops[l], gls::op_vmult_mode(mg->ops[l]), mg->tmp[l], mg->sol[l], 0,
                        mg->ops[l]->n_bricks, gls::BRICK_RUN | gls::BRICK_REDUCE, s, &rs);
      if (rs.defer) // (set only once the launch went through)
        mg->rq_level = l, mg->rq_slots = rs.partial, mg->rq_x = mg->sol[l], mg->rq_b = mg->def[l];
    }
  else
    {
      gls::op_vmult_device(mg->ops[l], mg->tmp[l], mg->sol[l], s);
      residual(mg, l, mg->tmp[l], mg->def[l], s);
    }
  sc_res.reset();
  // restrict
  {
    gls::Section sc(sec[2], s);
    if (!folded)
      {
        const int64_t w = (int64_t)((size_t)mg->ops[l - 1]->n_dofs * mg->ts() / 4);
        zero_words(mg->def[l - 1], w, s);
      }
    transfer(mg, 1, l, mg->def[l - 1], mg->tmp[l], s);
  }
  mg->rq_level = -1;
  v_step(mg, l - 1, s);
  // prolongate and add the coarse correction; with an odd number of fused
  // smoothing steps to follow it goes out of place into tmp, so the
  // ping-pong ends in sol without a copy
  const bool odd = gls::fused_relax_ok(mg->ops[l]) && nit % 2 == 1;
  {
    gls::Section sc(sec[3], s);
    if (odd)
      transfer(mg, 0, l, mg->tmp[l], mg->sol[l - 1], s, mg->sol[l]);
    else
      transfer(mg, 0, l, mg->sol[l], mg->sol[l - 1], s);
  }
  mg->pp_level = -1;
  // post-smoothing (MGSmootherPrecondition::smooth -> step); on the finest
  // level its last step also writes the FP64 result (copy_from_mg folded)
  bool          wrote = false;
  PendingReduce pp;
  {
    gls::Section sc(sec[4], s);
    smooth(mg, l, mg->sol[l], mg->def[l], false, nit, s, odd, nullptr, pro_ok ? &pp : nullptr,
           l == (int)mg->ops.size() - 1 ? mg->top_out64 : nullptr, &wrote);
  }
  if (l == (int)mg->ops.size() - 1)
    mg->top_out64_done = wrote;
  hand_over(l, pp);
}

// Relaxation-factor estimate of PreconditionRelaxation with relaxation = 0
// and EigenvalueAlgorithm::power_iteration (multigrid.cc:294-305, 353-369).
// Restates deal.II (>= 9.4, not vendored):
//   internal::PreconditionChebyshevImplementation::set_initial_guess:
//     x_i = i % 11 on the global index, minus the mean; then
//     AdditionalData::constraints.set_zero(x)
//   power_iteration(matrix, x, D^{-1}, eig_cg_n_iterations):
//     x /= |x|; repeat: y = D^{-1} A x; lambda = x . y; x = y / |y|;
//     return |lambda|
//   estimate_eigenvalues: max_eigenvalue_estimate = 1.2 * lambda (safety
//     factor), and PreconditionRelaxation::estimate_eigenvalues then sets
//     omega = 2 / (alpha + max), alpha = max / smoothing_range.
// The index i is this library's dof numbering (node-major), not deal.II's
// DoFHandler numbering, so the start vector is the same formula on a
// different numbering (deviation).  All reductions stay on the
// device; the host reads lambda once after the last iteration.
template <typename T>
void
power_iteration_t(glsMG_ *mg, int l, hipStream_t s)
{
  // enqueues the estimate on s; the Rayleigh quotient x.y of the last step
  // ends in d_acc[acc_off[l] + 2 nb] (gls_mg_setup collects it)
  glsOp         op = mg->ops[l];
  const int64_t n  = op->n_dofs;
  void         *x = mg->sol[l], *y = mg->tmp[l];
  const int64_t nb   = (n + 255) / 256;
  double       *part = mg->d_acc + mg->acc_off[l], *scal = part + 2 * nb;
  // start vector on the device: mean of i % 11 over [0, n) in closed form
  const int64_t q11  = n / 11, r11 = n % 11;
  const double  mean = n > 0 ? (double)(q11 * 55 + r11 * (r11 - 1) / 2) / (double)n : 0.0;
  hipLaunchKernelGGL(k_power_start<T>, g1(n), dim3(256), 0, s, (T *)x, op->d_node_cmask,
                     op->dim + 1, mean, part, n);
  hipLaunchKernelGGL(k_power_finish, dim3(1), dim3(256), 0, s, (const double *)part, nb, scal);
  hipLaunchKernelGGL(k_scale_dev<T>, g1(n), dim3(256), 0, s, (T *)x, (const T *)x,
                     (const double *)scal, n);
  HIP_THROW(hipGetLastError());
  HIP_THROW(hipMemsetAsync(scal, 0, 2 * sizeof(double), s));
  for (int it = 0; it < mg->desc.smoothing_eig_n_iterations; ++it)
    {
      gls::op_vmult_device(op, y, x, s);
      hipLaunchKernelGGL(k_power_step<T>, g1(n), dim3(256), 0, s, (T *)y, (const T *)x,
                         (const T *)mg->invdiag[l], part, n);
      hipLaunchKernelGGL(k_power_finish, dim3(1), dim3(256), 0, s, (const double *)part, nb,
                         scal);
      hipLaunchKernelGGL(k_scale_dev<T>, g1(n), dim3(256), 0, s, (T *)x, (const T *)y,
                         (const double *)scal, n);
      HIP_THROW(hipGetLastError());
    }
}

// v_step(top) on stream s.  (A hipGraph replay of the whole cycle, captured
// once per setup, measured slower than these direct launches -- 0.539 vs
// 0.484 ms: the cycle's launches run back to back, there is no launch
// overhead to remove -- and is on the git tag r4-graph-replay.)
void
run_v_step(glsMG_ *mg, int top, hipStream_t s)
{
  v_step(mg, top, s);
}

} // namespace

extern "C" {

glsStatus
gls_mg_create(const glsMGDesc *desc, const glsOp *levels, const uint32_t *const *child,
              glsMG *out)
{
  GLS_TRY
  if (!desc || !levels || !out || desc->n_levels < 1)
    throw std::runtime_error("gls_mg_create: invalid arguments");
  auto *mg   = new glsMG_();
  mg->desc   = *desc;
  mg->prec   = levels[0]->prec;
  mg->dim    = levels[0]->dim;
  mg->degree = levels[desc->n_levels - 1]->degree;
  mg->nc     = mg->dim + 1;
  const int nl_levels = desc->n_levels;
  for (int l = 0; l < nl_levels; ++l)
    {
      glsOp op = levels[l];
      // every level shares dim, precision and degree, except that the
      // coarsest may be of lower degree (FE_Q_iso_Q1: Q1 on the sub-cells)
      if (!op || op->prec != mg->prec || op->dim != mg->dim ||
          (l > 0 && op->degree != mg->degree) || op->degree > mg->degree)
        throw std::runtime_error("gls_mg_create: level operators must share dim, degree and "
                                 "precision (the coarsest may be of lower degree)");
      // partitioned (rank-local) level operators: the transfers
      // (prolongate_add / restrict_add / interpolate) and the relaxation
      // step serve the host-driven distributed multigrid (glsdist.py);
      // setup / V-cycle / smooth are single-domain and refuse them
      mg->partitioned = mg->partitioned || op->n_owned_nodes != op->n_nodes;
      mg->ops.push_back(op);
    }
  if (desc->coarse_amg && mg->partitioned)
    throw std::runtime_error("gls_mg_create: the AMG coarse solver is single-domain");
  if (nl_levels > 1 && (!child || mg->degree > 2))
    throw std::runtime_error("gls_mg_create: child lattices required (degree <= 2)");
  // 1D prolongation per coarse degree: parent GLL basis at the child
  // lattice points (for a Q1 coarse level under Q_k: the iso-Q1 embedding)
  for (int k = 1; k <= 2; ++k)
    {
      Basis1D b(k);
      for (int I = 0; I <= 2 * k; ++I)
        {
          const int    c = I / k > 1 ? 1 : I / k;
          const double x = 0.5 * (c + b.nodes[I - c * k]);
          for (int j = 0; j <= k; ++j)
            {
              double v = 1;
              for (int m = 0; m <= k; ++m)
                if (m != j)
                  v *= (x - b.nodes[m]) / (b.nodes[j] - b.nodes[m]);
              mg->P[k][I][j] = v;
            }
        }
    }
  mg->d_child.assign(nl_levels, nullptr);
  mg->d_weight.assign(nl_levels, nullptr);
  for (int l = 1; l < nl_levels; ++l)
    {
      glsOp         cop = mg->ops[l - 1], fop = mg->ops[l];
      const int     L   = 2 * cop->degree + 1;
      const int     nl  = mg->dim == 3 ? L * L * L : L * L;
      const int64_t nch = cop->n_cells * nl;
      std::vector<uint32_t> ch(child[l], child[l] + nch);
      std::vector<uint8_t>  seen((size_t)fop->n_nodes, 0);
      // ownership of the fine nodes: the first coarse cell touching a node
      // owns it; a lattice that already carries NOT_OWNER bits (bit 31,
      // e.g. the global-first owners of a partitioned hierarchy) is taken as
      // given
      bool flagged = false;
      for (uint32_t fn : ch)
        flagged = flagged || (fn & NOT_OWNER);
      for (uint32_t &fn : ch)
        {
          if ((int64_t)(fn & ~NOT_OWNER) >= fop->n_nodes)
            throw std::runtime_error("gls_mg_create: child lattice node out of range");
          if (!flagged && seen[fn])
            fn |= NOT_OWNER;
          seen[fn & ~NOT_OWNER] = 1;
        }
      // the transfer kernels walk the coarse operator's cells in its own
      // (possibly brick-discovered) order: rows follow it
      if (!cop->cell_perm.empty())
        {
          std::vector<uint32_t> pc(ch.size());
          for (int64_t c = 0; c < cop->n_cells; ++c)
            std::copy(ch.begin() + gls::ext_cell(cop, c) * nl,
                      ch.begin() + (gls::ext_cell(cop, c) + 1) * nl, pc.begin() + c * nl);
          ch.swap(pc);
        }
      std::vector<double> w((size_t)fop->n_dofs, 0.0);
      for (int64_t nd = 0; nd < fop->n_nodes; ++nd)
        for (int c = 0; c < mg->nc; ++c)
          w[nd * mg->nc + c] = (((fop->h_cmask[nd] >> c) & 1) || !seen[nd]) ? 0.0 : 1.0;
      HIP_THROW(hipMalloc((void **)&mg->d_child[l], nch * sizeof(uint32_t)));
      HIP_THROW(hipMemcpy(mg->d_child[l], ch.data(), nch * sizeof(uint32_t),
                          hipMemcpyHostToDevice));
      HIP_THROW(hipMalloc(&mg->d_weight[l], w.size() * mg->ts()));
      if (mg->prec == GLS_F64)
        HIP_THROW(hipMemcpy(mg->d_weight[l], w.data(), w.size() * 8, hipMemcpyHostToDevice));
      else
        {
          std::vector<float> wf(w.begin(), w.end());
          HIP_THROW(hipMemcpy(mg->d_weight[l], wf.data(), wf.size() * 4, hipMemcpyHostToDevice));
        }
    }
  for (int l = 0; l < nl_levels; ++l)
    {
      const size_t bytes = (size_t)mg->ops[l]->n_dofs * mg->ts();
      void        *p[4];
      for (auto &q : p)
        {
          HIP_THROW(hipMalloc(&q, std::max<size_t>(bytes, 1)));
          HIP_THROW(hipMemset(q, 0, std::max<size_t>(bytes, 1)));
        }
      mg->invdiag.push_back(p[0]);
      mg->sol.push_back(p[1]);
      mg->def.push_back(p[2]);
      mg->tmp.push_back(p[3]);
    }
  mg->omega.assign(nl_levels, 1.0);
  mg->lambda.assign(nl_levels, 0.0);
  for (int l = 0; l < nl_levels; ++l)
    {
      const std::string b = "gmg::vmult::level_" + std::to_string(l);
      mg->sec.push_back({b + "::0_pre_smoother_step", b + "::1_residual_step",
                         b + "::2_restriction", b + "::3_prolongation",
                         b + "::5_post_smoother_step", b});
    }
  int64_t acc_total = 0;
  for (int l = 0; l < nl_levels; ++l)
    {
      mg->acc_off.push_back(acc_total);
      acc_total += 2 * ((mg->ops[l]->n_dofs + 255) / 256) + 2;
    }
  HIP_THROW(hipMalloc((void **)&mg->d_acc, std::max<int64_t>(acc_total, 1) * sizeof(double)));
  *out = mg;
  GLS_CATCH
}

void
gls_mg_destroy(glsMG mg)
{
  if (!mg)
    return;
  for (auto *p : mg->d_child)
    if (p)
      (void)hipFree(p);
  for (auto *p : mg->d_weight)
    if (p)
      (void)hipFree(p);
  for (auto *v : {&mg->invdiag, &mg->sol, &mg->def, &mg->tmp, &mg->qslot[0], &mg->qslot[1]})
    for (void *p : *v)
      if (p)
        (void)hipFree(p);
  if (mg->d_acc)
    (void)hipFree(mg->d_acc);
  for (hipStream_t st : mg->side)
    (void)hipStreamDestroy(st);
  for (hipEvent_t ev : mg->side_ev)
    (void)hipEventDestroy(ev);
  for (void *p : {(void *)mg->d_lu, (void *)mg->d_ipiv, (void *)mg->d_info, (void *)mg->d_rhs,
                  (void *)mg->d_free, (void *)mg->d_free_in, (void *)mg->d_inv32,
                  (void *)mg->cg_ws, mg->cg_lvl, (void *)mg->d_cC, (void *)mg->d_cF,
                  (void *)mg->d_cG, (void *)mg->d_cint, (void *)mg->d_cbnd,
                  (void *)mg->d_rg_off, (void *)mg->d_rg_ent})
    if (p)
      (void)hipFree(p);
  if (mg->cg_host)
    (void)hipHostFree(mg->cg_host);
  for (hipEvent_t ev : mg->cg_ev)
    if (ev)
      (void)hipEventDestroy(ev);
  if (mg->blas)
    rocblas_destroy_handle(mg->blas);
  if (mg->amg)
    gls_amg_destroy(mg->amg);
  if (mg->amg_io)
    (void)hipFree(mg->amg_io);
  mg->stage.release();
  delete mg;
}

glsStatus
gls_mg_setup(glsMG mg, void *stream)
{
  GLS_TRY
  if (!mg)
    throw std::runtime_error("gls_mg_setup: null handle");
  if (mg->partitioned)
    throw std::runtime_error("gls_mg_setup: partitioned levels are set up by the host-driven "
                             "distributed multigrid (glsdist.py)");
  // every allocation and launch of the setup (the AMG hierarchy included)
  // on the levels' device; the caller's current device is restored
  gls::DeviceScope dev(mg->ops[0]->device);
  hipStream_t      s  = (hipStream_t)stream;
  gls::Section     sec_("gmg::initialize", s);
  const size_t     nl = mg->ops.size();
  // the smoother's slot buffers for deferred reductions (smooth)
  for (int q = 0; q < 2; ++q)
    {
      mg->qslot[q].resize(nl, nullptr);
      for (size_t l = 0; l < nl; ++l)
        if (!mg->qslot[q][l] && gls::deferred_reduce_ok(mg->ops[l]))
          HIP_THROW(hipMalloc(&mg->qslot[q][l], std::max<size_t>(16, (size_t)mg->ops[l]->n_slots *
                                                                        (mg->dim + 1) * mg->ts())));
    }
  // the levels are independent here: each level's diagonal and power
  // iteration run on a stream of its own (forked from and joined back into
  // s by events), so the small levels' launch-bound steps overlap the fine
  // level's instead of queueing behind them
  if (mg->side.empty())
    for (size_t l = 0; l < nl; ++l)
      {
        hipStream_t st;
        hipEvent_t  ev;
        HIP_THROW(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIP_THROW(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        mg->side.push_back(st);
        mg->side_ev.push_back(ev);
      }
  hipEvent_t fork;
  HIP_THROW(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  HIP_THROW(hipEventRecord(fork, s));
  std::vector<char> estimate(nl, 0);
  // enqueued finest level first: its kernels (the longest chain) start while
  // the host is still enqueueing the coarser levels' ~100 short launches each
  for (size_t li = nl; li-- > 0;)
    {
      const size_t l  = li;
      hipStream_t  ls = mg->side[l];
      HIP_THROW(hipStreamWaitEvent(ls, fork, 0));
      // compute_inverse_diagonal (multigrid.cc:290-293)
      {
        gls::Section sc("gmg::initialize::smoother::init0", ls);
        gls::op_inverse_diagonal_device(mg->ops[l], mg->invdiag[l], ls);
      }
      // relaxation = 0: omega from the power-iteration estimate of
      // lambda_max(D^-1 A) (power_iteration_t), estimated on the levels
      // above the coarsest one (multigrid.cc:355-358 with
      // compute_evs_n_levels = 0); the coarse level's smoother is used only
      // by the relaxation coarse solve (coarse_n_iterations > 0), which
      // then gets an estimate too
      if (l == 0 && mg->ops.size() > 1 && mg->desc.coarse_n_iterations <= 0 &&
          mg->desc.compute_evs_n_levels <= 0)
        {
          mg->lambda[l] = 0.0;
          mg->omega[l]  = 1.0;
        }
      else
        {
          gls::Section sc("gmg::initialize::smoother::init1", ls);
          if (mg->prec == GLS_F64)
            power_iteration_t<double>(mg, (int)l, ls);
          else
            power_iteration_t<float>(mg, (int)l, ls);
          estimate[l] = 1;
        }
      HIP_THROW(hipMemsetAsync(mg->sol[l], 0, (size_t)mg->ops[l]->n_dofs * mg->ts(), ls));
      HIP_THROW(hipEventRecord(mg->side_ev[l], ls));
      HIP_THROW(hipStreamWaitEvent(s, mg->side_ev[l], 0));
    }
  HIP_THROW(hipEventDestroy(fork));
  // collect the Rayleigh quotients (one host sync for all levels)
  std::vector<double> lam(nl, 0.0);
  for (size_t l = 0; l < nl; ++l)
    if (estimate[l])
      {
        const int64_t nb = (mg->ops[l]->n_dofs + 255) / 256;
        HIP_THROW(hipMemcpyAsync(&lam[l], mg->d_acc + mg->acc_off[l] + 2 * nb, sizeof(double),
                                 hipMemcpyDeviceToHost, s));
      }
  HIP_THROW(hipStreamSynchronize(s));
  for (size_t l = 0; l < nl; ++l)
    if (estimate[l])
      {
        const double ev_max = 1.2 * std::abs(lam[l]); // estimate_eigenvalues' safety factor
        mg->lambda[l]       = ev_max;
        if (ev_max > 0)
          {
            const double alpha = mg->desc.smoothing_range > 1.0 ?
                                   ev_max / mg->desc.smoothing_range :
                                   0.9 * ev_max;
            mg->omega[l] = 2.0 / (alpha + ev_max);
          }
        else
          mg->omega[l] = 1.0;
      }
  if (mg->desc.coarse_amg)
    {
      // the coarse level's system matrix (FP64, constrained rows / columns
      // identity) and the AMG hierarchy on it
      HIP_THROW(hipStreamSynchronize(s));
      gls::Section sc("gmg::initialize::amg", s);
      const auto t0   = std::chrono::steady_clock::now();
      glsOp      op0  = mg->ops[0];
      int64_t    nnz  = 0;
      if (gls_op_system_matrix(op0, &nnz, nullptr, nullptr, nullptr) != 0)
        throw std::runtime_error(std::string("coarse AMG: ") + gls_last_error());
      std::vector<int64_t> rp((size_t)op0->n_dofs + 1), ci((size_t)nnz);
      std::vector<double>  va((size_t)nnz);
      if (gls_op_system_matrix(op0, &nnz, rp.data(), ci.data(), va.data()) != 0)
        throw std::runtime_error(std::string("coarse AMG: ") + gls_last_error());
      if (mg->amg)
        gls_amg_destroy(mg->amg), mg->amg = nullptr;
      check_amg(gls_amg_create(op0->n_dofs, rp.data(), ci.data(), va.data(), &mg->desc.amg,
                               &mg->amg));
      if (!mg->amg_io)
        HIP_THROW(hipMalloc((void **)&mg->amg_io, (size_t)2 * op0->n_dofs * 8));
      mg->amg_setup_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
  else if (mg->desc.coarse_n_iterations < 0)
    {
      gls::Section sc("gmg::initialize::direct", s);
      if (mg->prec == GLS_F64)
        coarse_lu_setup_t<double>(mg, s);
      else
        coarse_lu_setup_t<float>(mg, s);
    }
  HIP_THROW(hipStreamSynchronize(s));
  mg->setup_done = true;
  GLS_CATCH
}

glsStatus
gls_mg_get_relaxation(glsMG mg, int level, double *omega, double *lambda_max)
{
  GLS_TRY
  if (!mg || level < 0 || level >= (int)mg->ops.size())
    throw std::runtime_error("gls_mg_get_relaxation: bad level");
  if (omega)
    *omega = mg->omega[level];
  if (lambda_max)
    *lambda_max = mg->lambda[level];
  GLS_CATCH
}

glsStatus
gls_mg_vcycle(glsMG mg, void *dst, const void *src, void *stream)
{
  GLS_TRY
  if (!mg || !dst || !src)
    throw std::runtime_error("gls_mg_vcycle: null argument");
  hipStream_t s = (hipStream_t)stream;
  gls::Section sec_("gmg::vmult", s);
  // a stall of an earlier (asynchronous) V-cycle is reported before this one
  // runs; a stall of this one as soon as its flag is visible (host-layout
  // vectors: at return)
  gls::mg_check_stall(mg, "gls_mg_vcycle");
  const void *x = mg->stage.in_vec(src, 0, s);
  void       *y = mg->stage.out_vec(dst);
  gls::mg_vcycle_device(mg, y, x, s);
  mg->stage.finish_out(dst, s);
  mg->stage.done(s);
  gls::mg_check_stall(mg, "gls_mg_vcycle");
  GLS_CATCH
}

glsStatus
gls_mg_relax(glsMG mg, int level, void *x, const void *b, const void *ax, const void *inv_diag,
             double omega, int zero_start, void *stream)
{
  GLS_TRY
  if (!mg || level < 0 || level >= (int)mg->ops.size() || !x || !b || !inv_diag ||
      (!zero_start && !ax))
    throw std::runtime_error("gls_mg_relax: bad arguments");
  const int64_t n = mg->ops[level]->n_dofs;
  hipStream_t   s = (hipStream_t)stream;
  if (mg->prec == GLS_F64)
    hipLaunchKernelGGL(k_relax<double>, g1(n), dim3(256), 0, s, (double *)x, (const double *)b,
                       (const double *)ax, (const double *)inv_diag, omega, zero_start ? 1 : 0,
                       n);
  else
    hipLaunchKernelGGL(k_relax<float>, g1(n), dim3(256), 0, s, (float *)x, (const float *)b,
                       (const float *)ax, (const float *)inv_diag, (float)omega,
                       zero_start ? 1 : 0, n);
  HIP_THROW(hipGetLastError());
  GLS_CATCH
}

glsStatus
gls_mg_set_vector_layout(glsMG mg, int memory, const int64_t *dof_map)
{
  GLS_TRY
  if (!mg)
    throw std::runtime_error("gls_mg_set_vector_layout: null handle");
  const size_t ts = mg->desc.outer_precision == GLS_F64 ? 8 : mg->ts();
  mg->stage.set(memory, dof_map, mg->ops.back()->n_dofs, ts);
  GLS_CATCH
}

} // extern "C"

namespace gls
{
void
mg_check_outer(glsMG mg, const glsOp_ *op)
{
  if (mg->desc.outer_precision != GLS_F64)
    throw std::runtime_error("gls_gmres_solve: the multigrid's outer_precision must be GLS_F64 "
                             "(PreconditionerGMG::vmult on VectorType<double>)");
  if (mg->ops.empty() || mg->ops.back()->n_dofs != op->n_dofs)
    throw std::runtime_error("gls_gmres_solve: the multigrid's finest level does not match the "
                             "operator's size");
  if (!mg->setup_done)
    throw std::runtime_error("gls_gmres_solve: the multigrid is not set up (gls_mg_setup)");
}

// a resident smoothing sweep of a level stalled since the last check (its
// neighbour brick was not resident: kernels of other streams held CUs): the
// level now runs one launch per step (gls::brick_sweeps); reported once
void
mg_check_stall(glsMG mg, const char *who)
{
  bool stalled = false;
  for (glsOp op : mg->ops)
    stalled = gls::sweep_stalled(op) || stalled;
  if (stalled)
    throw std::runtime_error(std::string(who) +
                             ": a resident smoothing sweep timed out (co-residency of the "
                             "level's bricks lost, INTEGRATION.md §5); the V-cycle it ran in "
                             "returned NaN, the multigrid now runs one launch per smoothing "
                             "step: repeat the computation");
}

bool
mg_is_linear(glsMG mg)
{
  return !mg->desc.coarse_iterate;
}

void
mg_vcycle_device(glsMG mg, void *dst, const void *src, hipStream_t s)
{
  if (!mg->setup_done)
    throw std::runtime_error("gls_mg_vcycle before gls_mg_setup");
  const int     top = (int)mg->ops.size() - 1;
  const int64_t n   = mg->ops[top]->n_dofs;
  const bool    cvt = mg->desc.outer_precision == GLS_F64 && mg->prec == GLS_F32;
  // copy_to_mg: folded into the finest level's first relaxation (v_step)
  // when the V-cycle has a smoothing level on top (the coarse-only hierarchy
  // has no relaxation to fold into)
  const bool folded = cvt && top > 0 && mg->desc.smoothing_n_iterations > 0;
  if (folded)
    {
      mg->top_b64   = (const double *)src;
      mg->top_out64 = (double *)dst;
    }
  else if (cvt)
    hipLaunchKernelGGL((k_convert<double, float>), g1(n), dim3(256), 0, s,
                       (float *)mg->def[top], (const double *)src, n);
  else
    HIP_THROW(hipMemcpyAsync(mg->def[top], src, n * mg->ts(), hipMemcpyDeviceToDevice, s));
  HIP_THROW(hipGetLastError());
  try
    {
      run_v_step(mg, top, s);
    }
  catch (...)
    {
      mg->top_b64   = nullptr;
      mg->top_out64 = nullptr;
      throw;
    }
  const bool done = mg->top_out64 != nullptr && mg->top_out64_done;
  mg->top_b64        = nullptr;
  mg->top_out64      = nullptr;
  mg->top_out64_done = false;
  // copy_from_mg (unless the last post-smoothing step wrote dst itself)
  if (done)
    ;
  else if (cvt)
    hipLaunchKernelGGL((k_convert<float, double>), g1(n), dim3(256), 0, s, (double *)dst,
                       (const float *)mg->sol[top], n);
  else
    HIP_THROW(hipMemcpyAsync(dst, mg->sol[top], n * mg->ts(), hipMemcpyDeviceToDevice, s));
  HIP_THROW(hipGetLastError());
}
} // namespace gls

extern "C" {

glsStatus
gls_mg_coarse_statistics(glsMG mg, int *n_iterations, int *converged)
{
  GLS_TRY
  if (!mg || !n_iterations || !converged)
    throw std::runtime_error("gls_mg_coarse_statistics: null argument");
  *n_iterations = mg->cg_iters;
  *converged    = mg->cg_conv;
  GLS_CATCH
}

glsStatus
gls_mg_coarse_amg(glsMG mg, glsAMG *amg, double *setup_ms)
{
  GLS_TRY
  if (!mg || !amg)
    throw std::runtime_error("gls_mg_coarse_amg: null argument");
  *amg = mg->amg;
  if (setup_ms)
    *setup_ms = mg->amg_setup_ms;
  GLS_CATCH
}

glsStatus
gls_mg_coarse_setup_times(glsMG mg, double *ms3, int *n_colors)
{
  GLS_TRY
  if (!mg || !ms3)
    throw std::runtime_error("gls_mg_coarse_setup_times: null argument");
  for (int i = 0; i < 3; ++i)
    ms3[i] = mg->coarse_setup_ms[i];
  if (n_colors)
    *n_colors = mg->coarse_colors;
  GLS_CATCH
}

glsStatus
gls_mg_prolongate_add(glsMG mg, int level, void *dst_fine, const void *src_coarse,
                      void *stream)
{
  GLS_TRY
  if (!mg)
    throw std::runtime_error("gls_mg_prolongate_add: null handle");
  transfer(mg, 0, level, dst_fine, src_coarse, (hipStream_t)stream);
  GLS_CATCH
}

glsStatus
gls_mg_restrict_add(glsMG mg, int level, void *dst_coarse, const void *src_fine, void *stream)
{
  GLS_TRY
  if (!mg)
    throw std::runtime_error("gls_mg_restrict_add: null handle");
  transfer(mg, 1, level, dst_coarse, src_fine, (hipStream_t)stream);
  GLS_CATCH
}

glsStatus
gls_mg_interpolate(glsMG mg, int level, void *dst_coarse, const void *src_fine, void *stream)
{
  GLS_TRY
  if (!mg)
    throw std::runtime_error("gls_mg_interpolate: null handle");
  transfer(mg, 2, level, dst_coarse, src_fine, (hipStream_t)stream);
  GLS_CATCH
}

glsStatus
gls_mg_smooth(glsMG mg, int level, void *x, const void *b, int zero_initial_guess,
              void *stream)
{
  GLS_TRY
  if (!mg || level < 0 || level >= (int)mg->ops.size())
    throw std::runtime_error("gls_mg_smooth: bad arguments");
  if (!mg->setup_done)
    throw std::runtime_error("gls_mg_smooth before gls_mg_setup");
  smooth(mg, level, x, b, zero_initial_guess != 0, mg->desc.smoothing_n_iterations,
         (hipStream_t)stream);
  GLS_CATCH
}

} // extern "C"
