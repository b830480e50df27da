// amg.hip — smoothed-aggregation algebraic multigrid on the coarse level's
// assembled system matrix: the substitute for TrilinosWrappers::
// PreconditionAMG (Trilinos ML) that the reference's coarse GMRES uses for
// "gmg coarse grid solver": "AMG" (multigrid.cc:372-433, 491-530; the sphere
// and Re20 decks).  ML is not available here; the algorithm restated is
// classical smoothed aggregation:
//   * strength of connection on the node graph (block_size dofs per node, the
//     "PDE equations" of ML; deal.II's constant modes per component give
//     block_size = dim+1, the default parameters one scalar mode):
//     ||A_IJ||_F >= threshold * sqrt(||A_II||_F ||A_JJ||_F);
//   * standard (uncoupled) aggregation in three passes over the nodes in
//     index order: a node whose strong neighbours are all free seeds an
//     aggregate with them; a remaining node joins the aggregate of its first
//     aggregated strong neighbour; the rest seed aggregates with their free
//     strong neighbours.  A node with no off-diagonal entry at all (the
//     identity rows / columns of constrained dofs: Dirichlet points) is left
//     out of every aggregate, its prolongator row zero, as ML and MueLu treat
//     Dirichlet rows, so the coarse levels carry only the coupled dofs;
//   * tentative prolongator from the near-null space (constant modes) by a
//     QR per aggregate and mode (per-mode disjoint supports: a scaling);
//   * prolongator smoothing P = (I - omega / lambda D^-1 A) P_tent, omega =
//     4/3, lambda from 15 power iterations on D^-1 A;
//   * Galerkin coarse operators R A P with R = P^T, until a level has at most
//     coarse_max_size dofs (deal.II's "coarse: max size" 2000), solved there
//     by a dense inverse (the reference: Amesos-KLU);
//   * Chebyshev smoothing of degree smoother_sweeps on D^-1 A over
//     [1.1 lambda / alpha, 1.1 lambda], alpha = chebyshev_alpha (deal.II's
//     10; ML's own default 30) -- ML's default smoother for the elliptic
//     defaults; the decks' ILU smoother is sequential and substituted by it.
// Setup on the host (as ML's); the V-cycle on the device: CSR SpMV kernels
// with the Chebyshev update fused, one launch per sweep.  tests/amg_ref.py
// restates the same algorithm with scipy for the parity tests.
#include "../../include/gls_op.h"
#include "common.h"

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

namespace gls
{
namespace
{
struct HostCSR
{
  int64_t              n = 0, m = 0; // rows, columns
  std::vector<int64_t> rp;
  std::vector<int32_t> ci;
  std::vector<double>  v;
};

HostCSR
transpose(const HostCSR &A)
{
  HostCSR T;
  T.n = A.m, T.m = A.n;
  T.rp.assign((size_t)T.n + 1, 0);
  for (int32_t c : A.ci)
    T.rp[(size_t)c + 1]++;
  for (int64_t i = 0; i < T.n; ++i)
    T.rp[(size_t)i + 1] += T.rp[(size_t)i];
  T.ci.resize(A.ci.size());
  T.v.resize(A.v.size());
  std::vector<int64_t> fill(T.rp.begin(), T.rp.end() - 1);
  for (int64_t r = 0; r < A.n; ++r) // rows in order: columns of T sorted
    for (int64_t k = A.rp[(size_t)r]; k < A.rp[(size_t)r + 1]; ++k)
      {
        const int64_t p = fill[(size_t)A.ci[(size_t)k]]++;
        T.ci[(size_t)p] = (int32_t)r;
        T.v[(size_t)p]  = A.v[(size_t)k];
      }
  return T;
}

// C = A B (Gustavson, columns sorted per row)
HostCSR
multiply(const HostCSR &A, const HostCSR &B)
{
  if (A.m != B.n)
    throw std::runtime_error("amg: inner dimensions differ");
  HostCSR C;
  C.n = A.n, C.m = B.m;
  C.rp.assign((size_t)C.n + 1, 0);
  std::vector<double>  acc((size_t)B.m, 0.0);
  std::vector<int32_t> mark((size_t)B.m, -1), cols;
  for (int64_t r = 0; r < A.n; ++r)
    {
      cols.clear();
      for (int64_t k = A.rp[(size_t)r]; k < A.rp[(size_t)r + 1]; ++k)
        {
          const int32_t j = A.ci[(size_t)k];
          const double  a = A.v[(size_t)k];
          for (int64_t l = B.rp[(size_t)j]; l < B.rp[(size_t)j + 1]; ++l)
            {
              const int32_t c = B.ci[(size_t)l];
              if (mark[(size_t)c] != (int32_t)r)
                {
                  mark[(size_t)c] = (int32_t)r;
                  acc[(size_t)c]  = 0.0;
                  cols.push_back(c);
                }
              acc[(size_t)c] += a * B.v[(size_t)l];
            }
        }
      std::sort(cols.begin(), cols.end());
      for (int32_t c : cols)
        {
          C.ci.push_back(c);
          C.v.push_back(acc[(size_t)c]);
        }
      C.rp[(size_t)r + 1] = (int64_t)C.ci.size();
    }
  return C;
}

std::vector<double>
diagonal(const HostCSR &A)
{
  std::vector<double> d((size_t)A.n, 0.0);
  for (int64_t r = 0; r < A.n; ++r)
    for (int64_t k = A.rp[(size_t)r]; k < A.rp[(size_t)r + 1]; ++k)
      if (A.ci[(size_t)k] == r)
        d[(size_t)r] = A.v[(size_t)k];
  return d;
}

// spectral-radius estimate of D^-1 A: 15 power iterations from a fixed start
// vector (tests/amg_ref.py runs the same sequence)
double
power_lambda(const HostCSR &A, const std::vector<double> &dinv)
{
  const int64_t       n = A.n;
  std::vector<double> x((size_t)n), y((size_t)n);
  double              nx = 0;
  for (int64_t i = 0; i < n; ++i)
    {
      x[(size_t)i] = 1.0 + (double)((i * 7919) % 97) / 97.0;
      nx += x[(size_t)i] * x[(size_t)i];
    }
  nx = std::sqrt(nx);
  for (auto &v : x)
    v /= nx;
  double lam = 0;
  for (int it = 0; it < 15; ++it)
    {
      double ny = 0;
      for (int64_t r = 0; r < n; ++r)
        {
          double s = 0;
          for (int64_t k = A.rp[(size_t)r]; k < A.rp[(size_t)r + 1]; ++k)
            s += A.v[(size_t)k] * x[(size_t)A.ci[(size_t)k]];
          y[(size_t)r] = dinv[(size_t)r] * s;
          ny += y[(size_t)r] * y[(size_t)r];
        }
      lam = std::sqrt(ny);
      if (lam == 0)
        break;
      for (int64_t i = 0; i < n; ++i)
        x[(size_t)i] = y[(size_t)i] / lam;
    }
  return lam;
}

// the node aggregates of one level: agg[node] (pyamg-style standard
// aggregation over the strong node graph)
std::vector<int32_t>
aggregate(const HostCSR &A, int b, double theta, int32_t &n_agg)
{
  const int64_t N = A.n / b;
  // node graph with squared block Frobenius norms (neighbours sorted)
  std::vector<std::vector<std::pair<int32_t, double>>> g((size_t)N);
  std::vector<double>  self((size_t)N, 0.0);
  std::vector<double>  acc((size_t)N, 0.0);
  std::vector<int32_t> mark((size_t)N, -1), cols;
  for (int64_t I = 0; I < N; ++I)
    {
      cols.clear();
      for (int c = 0; c < b; ++c)
        {
          const int64_t r = I * b + c;
          for (int64_t k = A.rp[(size_t)r]; k < A.rp[(size_t)r + 1]; ++k)
            {
              const int32_t J = A.ci[(size_t)k] / b;
              if (mark[(size_t)J] != (int32_t)I)
                {
                  mark[(size_t)J] = (int32_t)I;
                  acc[(size_t)J]  = 0.0;
                  cols.push_back(J);
                }
              acc[(size_t)J] += A.v[(size_t)k] * A.v[(size_t)k];
            }
        }
      std::sort(cols.begin(), cols.end());
      for (int32_t J : cols)
        {
          if (J == I)
            self[(size_t)I] = std::sqrt(acc[(size_t)J]);
          else
            g[(size_t)I].push_back({J, std::sqrt(acc[(size_t)J])});
        }
    }
  // strong neighbours
  std::vector<std::vector<int32_t>> S((size_t)N);
  for (int64_t I = 0; I < N; ++I)
    for (const auto &e : g[(size_t)I])
      if (e.second > 0 && e.second >= theta * std::sqrt(self[(size_t)I] * self[(size_t)e.first]))
        S[(size_t)I].push_back(e.first);
  std::vector<int32_t> agg((size_t)N, -1);
  n_agg = 0;
  // Dirichlet points: no off-diagonal entry (never aggregated; -2)
  for (int64_t I = 0; I < N; ++I)
    if (g[(size_t)I].empty())
      agg[(size_t)I] = -2;
  // pass 1: nodes whose strong neighbourhood is entirely free
  for (int64_t I = 0; I < N; ++I)
    {
      if (agg[(size_t)I] != -1)
        continue;
      bool free_nb = true;
      for (int32_t J : S[(size_t)I])
        if (agg[(size_t)J] >= 0)
          {
            free_nb = false;
            break;
          }
      if (!free_nb)
        continue;
      agg[(size_t)I] = n_agg;
      for (int32_t J : S[(size_t)I])
        agg[(size_t)J] = n_agg;
      ++n_agg;
    }
  // pass 2: join the first strong neighbour's pass-1 aggregate
  std::vector<int32_t> agg1 = agg;
  for (int64_t I = 0; I < N; ++I)
    if (agg1[(size_t)I] < 0)
      for (int32_t J : S[(size_t)I])
        if (agg1[(size_t)J] >= 0)
          {
            agg[(size_t)I] = agg1[(size_t)J];
            break;
          }
  // pass 3: the rest seed aggregates with their free strong neighbours
  for (int64_t I = 0; I < N; ++I)
    {
      if (agg[(size_t)I] != -1)
        continue;
      agg[(size_t)I] = n_agg;
      for (int32_t J : S[(size_t)I])
        if (agg[(size_t)J] < 0)
          agg[(size_t)J] = n_agg;
      ++n_agg;
    }
  return agg;
}

// ------------------------------------------------------------ device kernels
// G lanes per row (G = 64 / 32 / 16 / 8, chosen per matrix from its mean row
// length: rows of the iso-Q1 coarse levels hold ~90 entries, a full
// wavefront per row would idle 40 % of its lanes on the second pass):
// out_i = (f_i - sum_j A_ij (x_j + d_j)) and the Chebyshev update
// (cheb_step), or plain forms (below)
__device__ __forceinline__ double
wave_sum(double s)
{
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    s += __shfl_xor(s, o);
  return s;
}

template <int G>
__device__ __forceinline__ double
row_dot(const int32_t *__restrict__ rp, const int32_t *__restrict__ ci,
        const double *__restrict__ v, const double *__restrict__ x,
        const double *__restrict__ d, int64_t r, int lane)
{
  double s = 0;
  for (int32_t k = rp[r] + lane; k < rp[r + 1]; k += G)
    {
      const int32_t j = ci[k];
      s += v[k] * (d ? x[j] + d[j] : x[j]);
    }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1)
    s += __shfl_xor(s, o);
  return s;
}

// Chebyshev step: t = dinv (f - A (x + d)); xo = x + d; do = alpha d + beta t
template <int G>
__global__ void __launch_bounds__(256)
  k_cheb_step(const int32_t *__restrict__ rp, const int32_t *__restrict__ ci,
              const double *__restrict__ v, const double *__restrict__ x,
              const double *__restrict__ d, const double *__restrict__ f,
              const double *__restrict__ dinv, double *__restrict__ xo, double *__restrict__ dout,
              double alpha, double beta, int64_t n)
{
  const int64_t r    = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int     lane = threadIdx.x & (G - 1);
  if (r >= n)
    return;
  const double s = row_dot<G>(rp, ci, v, x, d, r, lane);
  if (lane == 0)
    {
      const double dr = d ? d[r] : 0.0;
      const double t  = dinv[r] * (f[r] - s);
      xo[r]           = x[r] + dr;
      dout[r]         = alpha * dr + beta * t;
    }
}

// zero start: x = 0, d = dinv f / theta
__global__ void
k_cheb_first(const double *__restrict__ f, const double *__restrict__ dinv, double *__restrict__ x,
             double *__restrict__ d, double inv_theta, int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    {
      x[i] = 0.0;
      d[i] = dinv[i] * f[i] * inv_theta;
    }
}

// residual of the pending iterate: xo = x + d, r = f - A (x + d)
template <int G>
__global__ void __launch_bounds__(256)
  k_residual(const int32_t *__restrict__ rp, const int32_t *__restrict__ ci,
             const double *__restrict__ v, const double *__restrict__ x,
             const double *__restrict__ d, const double *__restrict__ f, double *__restrict__ xo,
             double *__restrict__ res, int64_t n)
{
  const int64_t r    = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int     lane = threadIdx.x & (G - 1);
  if (r >= n)
    return;
  const double s = row_dot<G>(rp, ci, v, x, d, r, lane);
  if (lane == 0)
    {
      xo[r]  = x[r] + d[r];
      res[r] = f[r] - s;
    }
}

// y = M x (add = 0) or y += M x (add = 1)
template <int G>
__global__ void __launch_bounds__(256)
  k_spmv(const int32_t *__restrict__ rp, const int32_t *__restrict__ ci,
         const double *__restrict__ v, const double *__restrict__ x, double *__restrict__ y,
         int add, int64_t n)
{
  const int64_t r    = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int     lane = threadIdx.x & (G - 1);
  if (r >= n)
    return;
  const double s = row_dot<G>(rp, ci, v, x, nullptr, r, lane);
  if (lane == 0)
    y[r] = add ? y[r] + s : s;
}

// y = x + d
__global__ void
k_add2(const double *__restrict__ x, const double *__restrict__ d, double *__restrict__ y,
       int64_t n)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    y[i] = x[i] + d[i];
}

// dense coarse solve: x = Inv f, Inv row major [n][n], one wavefront per row
__global__ void __launch_bounds__(256)
  k_dense_gemv(const double *__restrict__ inv, const double *__restrict__ f,
               double *__restrict__ x, int64_t n)
{
  const int64_t r    = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int     lane = threadIdx.x & 63;
  if (r >= n)
    return;
  double s = 0;
  for (int64_t j = lane; j < n; j += 64)
    s += inv[r * n + j] * f[j];
  s = wave_sum(s);
  if (lane == 0)
    x[r] = s;
}

dim3
rows_grid(int64_t n, int G = 64)
{
  return dim3((unsigned)((n * G + 255) / 256));
}
dim3
elem_grid(int64_t n)
{
  return dim3((unsigned)((n + 255) / 256));
}

struct DevCSR
{
  int64_t  n = 0, nnz = 0;
  int32_t *rp = nullptr, *ci = nullptr;
  double  *v  = nullptr;
  int      g  = 64; // lanes per row of its row kernels
};

// launch a row kernel K<G>(args...) with the matrix's lanes per row
#define GLS_ROWS(K, M, st, ...)                                                               \
  do                                                                                         \
    {                                                                                        \
      const DevCSR &m_ = (M);                                                                \
      if (m_.g == 8)                                                                         \
        hipLaunchKernelGGL(K<8>, rows_grid(m_.n, 8), dim3(256), 0, st, __VA_ARGS__);         \
      else if (m_.g == 16)                                                                   \
        hipLaunchKernelGGL(K<16>, rows_grid(m_.n, 16), dim3(256), 0, st, __VA_ARGS__);       \
      else if (m_.g == 32)                                                                   \
        hipLaunchKernelGGL(K<32>, rows_grid(m_.n, 32), dim3(256), 0, st, __VA_ARGS__);       \
      else                                                                                   \
        hipLaunchKernelGGL(K<64>, rows_grid(m_.n, 64), dim3(256), 0, st, __VA_ARGS__);       \
    }                                                                                        \
  while (0)

template <typename T>
void
upload_vec(T **d, const std::vector<T> &h)
{
  HIP_THROW(hipMalloc((void **)d, std::max<size_t>(1, h.size() * sizeof(T))));
  if (!h.empty())
    HIP_THROW(hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
}

DevCSR
to_device(const HostCSR &A)
{
  if (A.rp.back() >= (int64_t)0x7fffffff)
    throw std::runtime_error("amg: matrix too large for 32-bit indices");
  DevCSR               D;
  D.n   = A.n;
  D.nnz = A.rp.back();
  // lanes per row: the smallest power of two >= 8 covering half a mean row
  const double mean = A.n > 0 ? (double)D.nnz / (double)A.n : 0.0;
  D.g               = mean > 96 ? 64 : mean > 48 ? 32 : mean > 24 ? 16 : 8;
  // (sphere r3 coarse level, 87 entries per row: 32 lanes 16.9-17.0 ms per
  // V-cycle, 8 / 16 / 64 lanes 20.0 / 18.1 / 18.0 ms;
  // profiles/r04/amg/ab_amg_rows_per_lane_group.txt)
  std::vector<int32_t> rp(A.rp.begin(), A.rp.end());
  upload_vec(&D.rp, rp);
  upload_vec(&D.ci, A.ci);
  upload_vec(&D.v, A.v);
  return D;
}

void
free_csr(DevCSR &D)
{
  (void)hipFree(D.rp), (void)hipFree(D.ci), (void)hipFree(D.v);
  D = DevCSR{};
}
} // namespace

// largest coarsest level that gets a dense inverse (n^2 doubles)
int64_t
amg_dense_limit(const glsAMGParams &prm)
{
  return std::max<int64_t>(4 * (int64_t)prm.coarse_max_size, 2048);
}

struct AmgLevel
{
  DevCSR  A, P, R; // P: n x n_coarse, R = P^T (none on the coarsest)
  double *dinv = nullptr, *x = nullptr, *d = nullptr, *f = nullptr, *r = nullptr,
         *x2 = nullptr, *d2 = nullptr;
  double  lambda = 0; // spectral radius estimate of D^-1 A
};
} // namespace gls

struct glsAMG_
{
  glsAMGParams                prm{};
  std::vector<gls::AmgLevel> lv;
  double                     *d_inv = nullptr; // coarsest: row-major dense inverse
  int64_t                     n_coarse = 0;
  int                         device   = 0;
};

namespace gls
{
namespace
{
// Chebyshev smoothing on level l (x, d: pending iterate x + d): s + 1
// Chebyshev steps in both cases.  The nonzero start forms its first
// correction from the residual f - A x (one matrix-vector product); the
// zero start skips that product (A 0 = 0), so pre-smoothing costs s and
// post-smoothing s + 1 products for the same polynomial (tests/amg_ref.py
// _cheb runs the same steps).
void
chebyshev(glsAMG_ *amg, AmgLevel &L, bool zero_start, hipStream_t st)
{
  const int    s   = std::max(1, amg->prm.smoother_sweeps);
  const double al  = amg->prm.chebyshev_alpha > 0 ? amg->prm.chebyshev_alpha : 10.0;
  const double b   = 1.1 * L.lambda, a = b / al;
  const double th  = 0.5 * (b + a), de = 0.5 * (b - a), sg = th / de;
  double       rho = 1.0 / sg;
  const int64_t n  = L.A.n;
  double *x = L.x, *d = L.d, *xo = L.x2, *dn = L.d2;
  if (zero_start)
    hipLaunchKernelGGL(k_cheb_first, elem_grid(n), dim3(256), 0, st, L.f, L.dinv, x, d, 1.0 / th,
                       n);
  else
    {
      // d = dinv (f - A x) / theta (pending part zero)
      GLS_ROWS(k_cheb_step, L.A, st, L.A.rp, L.A.ci, L.A.v, x, (const double *)nullptr, L.f,
               L.dinv, xo, dn, 0.0, 1.0 / th, n);
      std::swap(x, xo), std::swap(d, dn);
    }
  for (int k = 0; k < s; ++k) // s further steps, one matrix-vector product each
    {
      const double rn = 1.0 / (2.0 * sg - rho);
      GLS_ROWS(k_cheb_step, L.A, st, L.A.rp, L.A.ci, L.A.v, x, d, L.f, L.dinv, xo, dn,
               rn * rho, 2.0 * rn / de, n);
      std::swap(x, xo), std::swap(d, dn);
      rho = rn;
    }
  // the pending iterate x + d stays in (x, d); keep the level's canonical
  // buffers pointing at the current pair
  L.x = x, L.d = d, L.x2 = xo, L.d2 = dn;
  HIP_THROW(hipGetLastError());
}

// x_l = V(f_l), level l's x written as the pending pair (x, d) unless coarsest
void
vcycle_level(glsAMG_ *amg, size_t l, hipStream_t st)
{
  AmgLevel &L = amg->lv[l];
  if (l + 1 == amg->lv.size())
    {
      if (amg->d_inv)
        hipLaunchKernelGGL(k_dense_gemv, rows_grid(L.A.n), dim3(256), 0, st, amg->d_inv, L.f, L.x,
                           L.A.n);
      else
        {
          // coarsest level above the dense limit (aggregation stalled or
          // max_levels reached): smoothing sweeps as its solve, x = x + d
          chebyshev(amg, L, true, st);
          hipLaunchKernelGGL(k_add2, elem_grid(L.A.n), dim3(256), 0, st, L.x, L.d, L.x2, L.A.n);
          std::swap(L.x, L.x2);
        }
      HIP_THROW(hipGetLastError());
      return;
    }
  AmgLevel &C = amg->lv[l + 1];
  chebyshev(amg, L, true, st);
  // residual of x + d; x <- x + d
  GLS_ROWS(k_residual, L.A, st, L.A.rp, L.A.ci, L.A.v, L.x,
                     L.d, L.f, L.x2, L.r, L.A.n);
  std::swap(L.x, L.x2);
  GLS_ROWS(k_spmv, L.R, st, L.R.rp, L.R.ci, L.R.v, L.r, C.f,
                     0, L.R.n);
  vcycle_level(amg, l + 1, st);
  const double *xc = C.x;
  if (l + 2 < amg->lv.size())
    {
      // the coarser level's pending pair: x_c + d_c
      hipLaunchKernelGGL(k_add2, elem_grid(C.A.n), dim3(256), 0, st, C.x, C.d, C.x2, C.A.n);
      xc = C.x2;
    }
  GLS_ROWS(k_spmv, L.P, st, L.P.rp, L.P.ci, L.P.v, xc, L.x, 1,
                     L.P.n);
  chebyshev(amg, L, false, st);
  HIP_THROW(hipGetLastError());
}
} // namespace
} // namespace gls

extern "C" {

glsStatus
gls_amg_create(int64_t n, const int64_t *row_ptr, const int64_t *cols, const double *vals,
               const glsAMGParams *prm, glsAMG *out)
{
  GLS_TRY
  using namespace gls;
  if (!row_ptr || !cols || !vals || !prm || !out || n <= 0)
    throw std::runtime_error("gls_amg_create: invalid argument");
  const int b = prm->block_size;
  if (b < 1 || n % b != 0 || prm->smoother_sweeps < 1 || prm->coarse_max_size < 1 ||
      prm->max_levels < 1 || !(prm->threshold >= 0))
    throw std::runtime_error("gls_amg_create: invalid parameters");
  if (n >= 0x7fffffff)
    throw std::runtime_error("gls_amg_create: matrix too large for 32-bit indices");
  auto *amg = new glsAMG_();
  struct Guard
  {
    glsAMG_ *p;
    ~Guard()
    {
      if (p)
        gls_amg_destroy(p);
    }
  } guard{amg};
  amg->prm = *prm;
  HIP_THROW(hipGetDevice(&amg->device));
  HostCSR A;
  A.n = A.m = n;
  A.rp.assign(row_ptr, row_ptr + n + 1);
  A.ci.resize((size_t)A.rp.back());
  A.v.assign(vals, vals + A.rp.back());
  for (int64_t k = 0; k < A.rp.back(); ++k)
    {
      if (cols[k] < 0 || cols[k] >= n)
        throw std::runtime_error("gls_amg_create: column index out of range");
      A.ci[(size_t)k] = (int32_t)cols[k];
    }
  // near-null space per dof (constant modes: one per component when
  // block_size > 1, one overall otherwise)
  std::vector<double> beta((size_t)n, 1.0);
  std::vector<HostCSR> hA{A};
  for (int lev = 0;; ++lev)
    {
      HostCSR &Al = hA.back();
      // the level joins the hierarchy before any of its buffers exists, so
      // the guard frees whatever a failure below leaves allocated
      amg->lv.emplace_back();
      AmgLevel           &L = amg->lv.back();
      std::vector<double> d = diagonal(Al), dinv((size_t)Al.n);
      for (int64_t i = 0; i < Al.n; ++i)
        dinv[(size_t)i] = d[(size_t)i] != 0.0 ? 1.0 / d[(size_t)i] : 1.0;
      L.lambda = power_lambda(Al, dinv);
      L.A      = to_device(Al);
      upload_vec(&L.dinv, dinv);
      for (double **p : {&L.x, &L.d, &L.f, &L.r, &L.x2, &L.d2})
        {
          HIP_THROW(hipMalloc((void **)p, (size_t)Al.n * 8));
          HIP_THROW(hipMemset(*p, 0, (size_t)Al.n * 8));
        }
      const bool last = Al.n <= prm->coarse_max_size || lev + 1 >= prm->max_levels;
      if (!last)
        {
          int32_t                    n_agg = 0;
          const std::vector<int32_t> agg   = aggregate(Al, b, prm->threshold, n_agg);
          const int64_t              nc    = (int64_t)n_agg * b;
          if (nc >= Al.n)
            break; // no coarsening: this level is the coarsest
          // tentative prolongator: P[i, agg(i) b + comp(i)] = beta_i / |beta_(agg, comp)|
          // (rows of Dirichlet points empty)
          std::vector<double> nrm((size_t)nc, 0.0);
          for (int64_t i = 0; i < Al.n; ++i)
            if (agg[(size_t)(i / b)] >= 0)
              nrm[(size_t)(agg[(size_t)(i / b)] * (int64_t)b + i % b)] +=
                beta[(size_t)i] * beta[(size_t)i];
          for (auto &v : nrm)
            v = std::sqrt(v);
          HostCSR Pt;
          Pt.n = Al.n, Pt.m = nc;
          Pt.rp.resize((size_t)Al.n + 1);
          for (int64_t i = 0; i < Al.n; ++i)
            {
              Pt.rp[(size_t)i] = (int64_t)Pt.ci.size();
              if (agg[(size_t)(i / b)] < 0)
                continue;
              const int64_t c = agg[(size_t)(i / b)] * (int64_t)b + i % b;
              Pt.ci.push_back((int32_t)c);
              Pt.v.push_back(nrm[(size_t)c] > 0 ? beta[(size_t)i] / nrm[(size_t)c] : 0.0);
            }
          Pt.rp[(size_t)Al.n] = (int64_t)Pt.ci.size();
          // P = P_t - omega / lambda D^-1 A P_t (omega 4/3; elliptic = 0: P_t)
          HostCSR P = Pt;
          if (prm->elliptic && L.lambda > 0)
            {
              HostCSR      AP = multiply(Al, Pt);
              const double w  = (4.0 / 3.0) / L.lambda;
              HostCSR      S;
              S.n = Al.n, S.m = nc;
              S.rp.assign((size_t)Al.n + 1, 0);
              for (int64_t i = 0; i < Al.n; ++i)
                {
                  // merge row i of P_t (one entry, or none) with -w dinv_i (A P_t)_i
                  const bool    has = Pt.rp[(size_t)i + 1] > Pt.rp[(size_t)i];
                  const int32_t ct  = has ? Pt.ci[(size_t)Pt.rp[(size_t)i]] : -1;
                  const double  pv  = has ? Pt.v[(size_t)Pt.rp[(size_t)i]] : 0.0;
                  bool          put = !has;
                  for (int64_t k = AP.rp[(size_t)i]; k < AP.rp[(size_t)i + 1]; ++k)
                    {
                      const int32_t c = AP.ci[(size_t)k];
                      if (!put && ct < c)
                        {
                          S.ci.push_back(ct), S.v.push_back(pv);
                          put = true;
                        }
                      double v = -w * dinv[(size_t)i] * AP.v[(size_t)k];
                      if (c == ct)
                        {
                          v += pv;
                          put = true;
                        }
                      S.ci.push_back(c), S.v.push_back(v);
                    }
                  if (!put)
                    S.ci.push_back(ct), S.v.push_back(pv);
                  S.rp[(size_t)i + 1] = (int64_t)S.ci.size();
                }
              P = std::move(S);
            }
          HostCSR R  = transpose(P);
          HostCSR Ac = multiply(R, multiply(Al, P));
          L.P        = to_device(P);
          L.R        = to_device(R);
          beta.assign(nrm.begin(), nrm.end()); // coarse near-null space (the R of the QR)
          hA.push_back(std::move(Ac));
          continue;
        }
      break;
    }
  // coarsest: dense inverse (LU + inverse on the device) up to the dense
  // limit; a larger coarsest level (aggregation stalled or max_levels
  // reached) is smoothed instead of factorised (a dense matrix of it would
  // need n^2 doubles on the host and the device)
  amg->n_coarse = hA.back().n;
  if (hA.back().n <= amg_dense_limit(*prm))
  {
    const HostCSR &Ac = hA.back();
    const int64_t  nc = Ac.n;
    std::vector<double> dense((size_t)nc * nc, 0.0); // column major for rocSOLVER
    for (int64_t r = 0; r < nc; ++r)
      for (int64_t k = Ac.rp[(size_t)r]; k < Ac.rp[(size_t)r + 1]; ++k)
        dense[(size_t)Ac.ci[(size_t)k] * nc + r] = Ac.v[(size_t)k];
    double *d_a = nullptr;
    HIP_THROW(hipMalloc((void **)&d_a, dense.size() * 8));
    amg->d_inv = d_a; // owned by the guard from here on
    struct Scratch    // pivots, info and the rocBLAS handle, freed on every path
    {
      rocblas_int   *ipiv = nullptr, *info = nullptr;
      rocblas_handle h    = nullptr;
      ~Scratch()
      {
        (void)hipFree(ipiv), (void)hipFree(info);
        if (h)
          rocblas_destroy_handle(h);
      }
    } w;
    HIP_THROW(hipMalloc((void **)&w.ipiv, (size_t)nc * sizeof(rocblas_int)));
    HIP_THROW(hipMalloc((void **)&w.info, sizeof(rocblas_int)));
    HIP_THROW(hipMemcpy(d_a, dense.data(), dense.size() * 8, hipMemcpyHostToDevice));
    if (rocblas_create_handle(&w.h) != rocblas_status_success)
      throw std::runtime_error("gls_amg_create: rocblas_create_handle failed");
    rocblas_status st = rocsolver_dgetrf(w.h, (rocblas_int)nc, (rocblas_int)nc, d_a,
                                         (rocblas_int)nc, w.ipiv, w.info);
    rocblas_int    hinfo = 0;
    if (st == rocblas_status_success)
      {
        HIP_THROW(hipMemcpy(&hinfo, w.info, sizeof(hinfo), hipMemcpyDeviceToHost));
        if (hinfo == 0)
          st = rocsolver_dgetri(w.h, (rocblas_int)nc, d_a, (rocblas_int)nc, w.ipiv, w.info);
      }
    if (st == rocblas_status_success && hinfo == 0)
      HIP_THROW(hipMemcpy(&hinfo, w.info, sizeof(hinfo), hipMemcpyDeviceToHost));
    if (st != rocblas_status_success || hinfo != 0)
      throw std::runtime_error("gls_amg_create: singular coarsest AMG matrix");
    // column-major inverse -> row major for the wavefront-per-row GEMV
    std::vector<double> inv(dense.size());
    HIP_THROW(hipMemcpy(inv.data(), d_a, inv.size() * 8, hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < nc; ++r)
      for (int64_t c = 0; c < nc; ++c)
        dense[(size_t)r * nc + c] = inv[(size_t)c * nc + r];
    HIP_THROW(hipMemcpy(d_a, dense.data(), dense.size() * 8, hipMemcpyHostToDevice));
  }
  guard.p = nullptr;
  *out    = amg;
  GLS_CATCH
}

void
gls_amg_destroy(glsAMG amg)
{
  if (!amg)
    return;
  for (auto &L : amg->lv)
    {
      gls::free_csr(L.A), gls::free_csr(L.P), gls::free_csr(L.R);
      for (double *p : {L.dinv, L.x, L.d, L.f, L.r, L.x2, L.d2})
        (void)hipFree(p);
    }
  (void)hipFree(amg->d_inv);
  delete amg;
}

glsStatus
gls_amg_vmult(glsAMG amg, double *dst, const double *src, void *stream)
{
  GLS_TRY
  using namespace gls;
  if (!amg || !dst || !src)
    throw std::runtime_error("gls_amg_vmult: null argument");
  DeviceScope         ds(amg->device);
  const hipStream_t   st = (hipStream_t)stream;
  AmgLevel           &L0 = amg->lv[0];
  const int64_t       n  = L0.A.n;
  // the finest level reads its right-hand side only (Chebyshev steps,
  // residual): the caller's src serves as f for this cycle, no copy
  double *const f0 = L0.f;
  L0.f             = const_cast<double *>(src);
  try
    {
      vcycle_level(amg, 0, st);
    }
  catch (...)
    {
      L0.f = f0;
      throw;
    }
  L0.f = f0;
  if (amg->lv.size() > 1)
    hipLaunchKernelGGL(k_add2, elem_grid(n), dim3(256), 0, st, L0.x, L0.d, dst, n);
  else
    HIP_THROW(hipMemcpyAsync(dst, L0.x, (size_t)n * 8, hipMemcpyDeviceToDevice, st));
  HIP_THROW(hipGetLastError());
  GLS_CATCH
}

glsStatus
gls_amg_level_matrix(glsAMG amg, int level, int which, int64_t *n_rows, int64_t *nnz,
                     int32_t *row_ptr, int32_t *cols, double *vals)
{
  GLS_TRY
  if (!amg || !n_rows || !nnz || level < 0 || level >= (int)amg->lv.size() || which < 0 ||
      which > 2)
    throw std::runtime_error("gls_amg_level_matrix: bad argument");
  gls::DeviceScope ds(amg->device);
  const auto &L = amg->lv[(size_t)level];
  const auto &M = which == 0 ? L.A : which == 1 ? L.P : L.R;
  *n_rows       = M.n;
  *nnz          = M.nnz;
  if (row_ptr && M.rp)
    HIP_THROW(hipMemcpy(row_ptr, M.rp, (size_t)(M.n + 1) * 4, hipMemcpyDeviceToHost));
  if (cols && M.ci)
    HIP_THROW(hipMemcpy(cols, M.ci, (size_t)M.nnz * 4, hipMemcpyDeviceToHost));
  if (vals && M.v)
    HIP_THROW(hipMemcpy(vals, M.v, (size_t)M.nnz * 8, hipMemcpyDeviceToHost));
  GLS_CATCH
}

glsStatus
gls_amg_info(glsAMG amg, int *n_levels, int64_t *sizes, int64_t *nnz, double *lambda)
{
  GLS_TRY
  if (!amg || !n_levels)
    throw std::runtime_error("gls_amg_info: null argument");
  *n_levels = (int)amg->lv.size();
  for (size_t l = 0; l < amg->lv.size(); ++l)
    {
      if (sizes)
        sizes[l] = amg->lv[l].A.n;
      if (nnz)
        nnz[l] = amg->lv[l].A.nnz;
      if (lambda)
        lambda[l] = amg->lv[l].lambda;
    }
  GLS_CATCH
}

} // extern "C"
