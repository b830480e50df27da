// gls_vmult.hip — `gls-vmult dim n_global_refinements fe_degree`: the
// reference's benchmark program (performance.cc:12-182) on this library.
//
// Same setup as performance.cc:16-74: unit hyper cube refined n times
// (GridGenerator::hyper_cube + refine_global, here gls_mesh_hypercube),
// FESystem(FE_Q(k), dim+1), QGauss(k+1), MappingQ(1), no constraints,
// nu = 0.1, c1 = 4, c2 = 2, BDF2 after one update_dt(0.1) (weights 10, -10,
// 0), consider_time_derivative = false, increment_form, cell-wise
// stabilisation, zero history and zero linearisation point; then the three
// timed variants, 10 repetitions each, under the reference's section names:
//   ns::vmult::mf       NavierStokesOperator::vmult (gls_op_vmult)
//   ns::vmult::mb       get_system_matrix() + SparseMatrix::vmult (the CSR
//                       of gls_op_system_matrix, rocSPARSE SpMV)
//   poisson::vmult::mf  the trivial vector-valued mass + Laplace matrix-free
//                       cell loop (performance.cc:97-142; k_poisson below)
// and TimerCollection::print_all_wall_time_statistics (gls_timer_report).
// The reference never fills src (its run times only); --check instead fills
// src and the linearisation point with seeded values and checks mf against
// mb (the compute_matrix equivalence performance.cc relies on) and the
// Poisson kernel against a host loop of the same operator.
#include <hip/hip_runtime.h>
#include <rocsparse/rocsparse.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gls_mesh.h"
#include "gls_operator.hpp"

#define HIPCHK(x)                                                                        \
  do                                                                                     \
    {                                                                                    \
      const hipError_t e_ = (x);                                                         \
      if (e_ != hipSuccess)                                                              \
        {                                                                                \
          std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
          std::exit(2);                                                                  \
        }                                                                                \
    }                                                                                    \
  while (0)
#define SPCHK(x)                                                                         \
  do                                                                                     \
    {                                                                                    \
      const rocsparse_status s_ = (x);                                                   \
      if (s_ != rocsparse_status_success)                                                \
        {                                                                                \
          std::fprintf(stderr, "%s: rocsparse status %d\n", #x, (int)s_);                \
          std::exit(2);                                                                  \
        }                                                                                \
    }                                                                                    \
  while (0)

// ---- 1D data of FE_Q(k) on Gauss-Lobatto points at QGauss(k+1) on [0,1]
struct Tab1D
{
  int    n = 0;       // k + 1
  double S[4][4]{};   // S[q][i]  = phi_i(x_q)
  double Dq[4][4]{};  // Dq[q][j] = l_j'(x_q), l_j Lagrange on the Gauss points
  double w[4]{};      // Gauss weights
};

static double
lagrange(const double *x, int n, int i, double t)
{
  double v = 1;
  for (int j = 0; j < n; ++j)
    if (j != i)
      v *= (t - x[j]) / (x[i] - x[j]);
  return v;
}

static double
lagrange_d(const double *x, int n, int i, double t)
{
  double s = 0;
  for (int m = 0; m < n; ++m)
    if (m != i)
      {
        double p = 1 / (x[i] - x[m]);
        for (int j = 0; j < n; ++j)
          if (j != i && j != m)
            p *= (t - x[j]) / (x[i] - x[j]);
        s += p;
      }
  return s;
}

static Tab1D
tables(int k)
{
  Tab1D t;
  t.n = k + 1;
  double gll[4], gq[4], gw[4];
  if (k == 1)
    gll[0] = 0, gll[1] = 1;
  else if (k == 2)
    gll[0] = 0, gll[1] = 0.5, gll[2] = 1;
  else
    gll[0] = 0, gll[1] = 0.5 * (1 - 1 / std::sqrt(5.0)), gll[2] = 0.5 * (1 + 1 / std::sqrt(5.0)),
    gll[3] = 1;
  // Gauss-Legendre on [-1, 1], mapped to [0, 1]
  const double x2[2] = {-0.5773502691896257, 0.5773502691896257}, w2[2] = {1, 1};
  const double x3[3] = {-0.7745966692414834, 0, 0.7745966692414834},
               w3[3] = {5.0 / 9, 8.0 / 9, 5.0 / 9};
  const double x4[4] = {-0.8611363115940526, -0.3399810435848563, 0.3399810435848563,
                        0.8611363115940526},
               w4[4] = {0.3478548451374538, 0.6521451548625461, 0.6521451548625461,
                        0.3478548451374538};
  const double *xs = k == 1 ? x2 : k == 2 ? x3 : x4, *ws = k == 1 ? w2 : k == 2 ? w3 : w4;
  for (int q = 0; q < t.n; ++q)
    gq[q] = 0.5 * (1 + xs[q]), gw[q] = 0.5 * ws[q];
  for (int q = 0; q < t.n; ++q)
    {
      t.w[q] = gw[q];
      for (int i = 0; i < t.n; ++i)
        {
          t.S[q][i]  = lagrange(gll, t.n, i, gq[q]);
          t.Dq[q][i] = lagrange_d(gq, t.n, i, gq[q]);
        }
    }
  return t;
}

// ---- poisson::vmult::mf (performance.cc:97-142): per component
// dst += M u + K u on Cartesian cells of width h: gather, values at the
// Gauss points by sum factorisation (S along each axis), reference gradients
// by the collocation derivative Dq, submit value * JxW and gradient * JxW /
// h^2, integrate (Dq^T, then S^T along each axis), scatter-add.  One
// 64-lane wavefront per cell, (k+1)^dim <= 64 lanes busy; LDS per component.
template <int dim>
__global__ void __launch_bounds__(64)
  k_poisson(double *__restrict__ dst, const double *__restrict__ src,
            const uint32_t *__restrict__ cell_nodes, int64_t n_cells, Tab1D tb, double h)
{
  const int64_t cell = blockIdx.x;
  if (cell >= n_cells)
    return;
  const int n = tb.n, nq = dim == 3 ? n * n * n : n * n, nc = dim + 1;
  const int t = threadIdx.x;
  __shared__ double A[64], B[64], G[3][64];
  const bool act = t < nq;
  int        ix[3] = {0, 0, 0}, st[3] = {1, n, n * n};
  if (act)
    {
      ix[0] = t % n;
      ix[1] = (t / n) % n;
      ix[2] = dim == 3 ? t / (n * n) : 0;
    }
  double wq = 1;
  for (int d = 0; d < dim; ++d)
    wq *= tb.w[ix[d]];
  const double jxw  = wq * (dim == 3 ? h * h * h : h * h);
  const double gfac = jxw / (h * h);
  const uint32_t node = act ? cell_nodes[cell * nq + t] : 0u;
  for (int c = 0; c < nc; ++c)
    {
      A[t] = act ? src[(size_t)node * nc + c] : 0.0;
      __syncthreads();
      // values at the Gauss points
      for (int d = 0; d < dim; ++d)
        {
          double s = 0;
          if (act)
            for (int j = 0; j < n; ++j)
              s += tb.S[ix[d]][j] * A[t + (j - ix[d]) * st[d]];
          __syncthreads();
          B[t] = s;
          __syncthreads();
          A[t] = B[t];
          __syncthreads();
        }
      // reference gradients, submitted (J^{-1} = 1/h), and the value part
      for (int d = 0; d < dim; ++d)
        {
          double s = 0;
          if (act)
            for (int j = 0; j < n; ++j)
              s += tb.Dq[ix[d]][j] * A[t + (j - ix[d]) * st[d]];
          G[d][t] = s * gfac;
        }
      __syncthreads();
      double v = A[t] * jxw;
      for (int d = 0; d < dim; ++d)
        if (act)
          for (int j = 0; j < n; ++j)
            v += tb.Dq[j][ix[d]] * G[d][t + (j - ix[d]) * st[d]];
      __syncthreads();
      A[t] = v;
      __syncthreads();
      // S^T along each axis: back to the nodes
      for (int d = 0; d < dim; ++d)
        {
          double s = 0;
          if (act)
            for (int j = 0; j < n; ++j)
              s += tb.S[j][ix[d]] * A[t + (j - ix[d]) * st[d]];
          __syncthreads();
          B[t] = s;
          __syncthreads();
          A[t] = B[t];
          __syncthreads();
        }
      if (act)
        atomicAdd(dst + (size_t)node * nc + c, A[t]);
      __syncthreads();
    }
}

// the same operator on the host, element by element with full tensor loops
static void
poisson_host(int dim, const Tab1D &tb, double h, int64_t n_cells, const uint32_t *cn,
             const std::vector<double> &src, std::vector<double> &dst)
{
  const int n = tb.n, nq = dim == 3 ? n * n * n : n * n, nc = dim + 1;
  auto idx = [&](int i, int d) { return d == 0 ? i % n : d == 1 ? (i / n) % n : i / (n * n); };
  for (int64_t cell = 0; cell < n_cells; ++cell)
    for (int c = 0; c < nc; ++c)
      for (int q = 0; q < nq; ++q)
        {
          double wq = 1;
          for (int d = 0; d < dim; ++d)
            wq *= tb.w[idx(q, d)];
          const double jxw = wq * std::pow(h, dim);
          double       val = 0, g[3] = {0, 0, 0};
          std::vector<double> phi(nq), dphi((size_t)nq * 3);
          for (int i = 0; i < nq; ++i)
            {
              double p = 1;
              for (int d = 0; d < dim; ++d)
                p *= tb.S[idx(q, d)][idx(i, d)];
              phi[i] = p;
              for (int e = 0; e < dim; ++e)
                {
                  // d/dx_e of phi_i at q: the derivative of the 1D GLL basis
                  // at a Gauss point, = sum_j Dq[q_e][j] S[j][i_e]
                  double pe = 1;
                  for (int d = 0; d < dim; ++d)
                    if (d != e)
                      pe *= tb.S[idx(q, d)][idx(i, d)];
                  double de = 0;
                  for (int j = 0; j < n; ++j)
                    de += tb.Dq[idx(q, e)][j] * tb.S[j][idx(i, e)];
                  dphi[(size_t)i * 3 + e] = pe * de / h;
                }
              const double u = src[(size_t)cn[cell * nq + i] * nc + c];
              val += phi[i] * u;
              for (int e = 0; e < dim; ++e)
                g[e] += dphi[(size_t)i * 3 + e] * u;
            }
          for (int i = 0; i < nq; ++i)
            {
              double r = phi[i] * val;
              for (int e = 0; e < dim; ++e)
                r += dphi[(size_t)i * 3 + e] * g[e];
              dst[(size_t)cn[cell * nq + i] * nc + c] += r * jxw;
            }
        }
}

static double
rel_err(const std::vector<double> &a, const std::vector<double> &b)
{
  double d = 0, r = 0;
  for (size_t i = 0; i < a.size(); ++i)
    d += (a[i] - b[i]) * (a[i] - b[i]), r += b[i] * b[i];
  return std::sqrt(d / (r > 0 ? r : 1));
}

int
main(int argc, char **argv)
{
  // performance.cc:162-168: dim, n_global_refinements, fe_degree
  const int  dim   = argc >= 2 ? std::atoi(argv[1]) : 2;
  const int  n_ref = argc >= 3 ? std::atoi(argv[2]) : 5;
  const int  k     = argc >= 4 ? std::atoi(argv[3]) : 1;
  const bool check = argc >= 5 && std::strcmp(argv[4], "--check") == 0;
  const int  reps  = 10; // n_repetitions, performance.cc:24
  if ((dim != 2 && dim != 3) || k < 1 || k > 3)
    {
      std::fprintf(stderr, "usage: gls-vmult [dim(2|3) [n_global_refinements [fe_degree(1..3) "
                           "[--check]]]]\n");
      return 2;
    }
  gls::timer_enable(true);

  glsMesh *mesh = nullptr;
  if (gls_mesh_hypercube(dim, k, n_ref, &mesh))
    {
      std::fprintf(stderr, "mesh: %s\n", gls_mesh_last_error());
      return 2;
    }
  const int64_t nc = gls_mesh_n_cells(mesh), nn = gls_mesh_n_nodes(mesh);
  const int     ncomp = dim + 1;
  const int64_t ndof  = nn * ncomp;
  std::printf("Number of DoFs: %lld\n", (long long)ndof);
  std::vector<uint8_t> cmask((size_t)nn, 0); // AffineConstraints: empty
  std::vector<double>  meas((size_t)nc), hmin((size_t)nc);
  int                  brick[3] = {0, 0, 0};
  if (gls_mesh_cell_measure(mesh, meas.data(), hmin.data()) || gls_mesh_brick(mesh, brick))
    {
      std::fprintf(stderr, "mesh: %s\n", gls_mesh_last_error());
      return 2;
    }
  glsOpDesc d{};
  d.dim           = dim;
  d.degree        = k;
  d.precision     = GLS_F64;
  d.n_cells       = nc;
  d.n_nodes       = nn;
  d.n_owned_nodes = nn;
  d.cell_nodes    = gls_mesh_cell_nodes(mesh);
  d.node_coords   = gls_mesh_node_coords(mesh);
  d.node_cmask    = cmask.data();
  d.cell_measure  = meas.data();
  d.cell_hmin     = hmin.data();
  for (int i = 0; i < 3; ++i)
    d.brick[i] = brick[i];

  gls::Operator   op(d);
  gls::Parameters prm;
  prm.nu    = 0.1;
  prm.c1    = 4.0;
  prm.c2    = 2.0;
  prm.theta = 1.0;
  prm.dt    = 0.1;
  prm.order = 2;
  prm.w0    = 10.0; // BDF2 after one update_dt(0.1): 1/dt, -1/dt, 0
  prm.flags = GLS_INCREMENT_FORM | GLS_CELL_WISE_STAB;
  op.set_parameters(prm);

  // vectors: zero (performance.cc:65-79) or, with --check, seeded values
  std::vector<double> h_src((size_t)ndof, 0.0), h_u((size_t)ndof, 0.0);
  if (check)
    {
      uint64_t x = 0x9E3779B97F4A7C15ull;
      auto     rnd = [&]() {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        return (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
      };
      for (auto &v : h_src)
        v = rnd();
      for (auto &v : h_u)
        v = rnd();
    }
  double *src, *dst, *u, *zero;
  HIPCHK(hipMalloc(&src, ndof * 8));
  HIPCHK(hipMalloc(&dst, ndof * 8));
  HIPCHK(hipMalloc(&u, ndof * 8));
  HIPCHK(hipMalloc(&zero, ndof * 8));
  HIPCHK(hipMemcpy(src, h_src.data(), ndof * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(u, h_u.data(), ndof * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(zero, 0, ndof * 8));
  HIPCHK(hipMemset(dst, 0, ndof * 8));
  op.set_previous_solution({zero, zero, zero}, {10.0, -10.0, 0.0});
  op.set_linearization_point(u);
  op.vmult(dst, src); // first call: code objects, tables
  HIPCHK(hipDeviceSynchronize());

  auto timed = [&](const char *name, const auto &body) {
    gls::Scope s(name);
    for (int r = 0; r < reps; ++r)
      body();
    HIPCHK(hipDeviceSynchronize()); // the reference's calls are synchronous
  };

  // ns::vmult::mf
  timed("ns::vmult::mf", [&] { op.vmult(dst, src); });
  std::vector<double> y_mf((size_t)ndof);
  HIPCHK(hipMemcpy(y_mf.data(), dst, ndof * 8, hipMemcpyDeviceToHost));

  // ns::vmult::mb: get_system_matrix() (untimed, as the reference's) + SpMV
  const auto A = op.get_system_matrix();
  int64_t *rp, *ci;
  double  *va, *ymb;
  const int64_t nnz = (int64_t)A.vals.size();
  HIPCHK(hipMalloc(&rp, (ndof + 1) * 8));
  HIPCHK(hipMalloc(&ci, nnz * 8));
  HIPCHK(hipMalloc(&va, nnz * 8));
  HIPCHK(hipMalloc(&ymb, ndof * 8));
  HIPCHK(hipMemcpy(rp, A.row_ptr.data(), (ndof + 1) * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ci, A.cols.data(), nnz * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(va, A.vals.data(), nnz * 8, hipMemcpyHostToDevice));
  rocsparse_handle      sh;
  rocsparse_spmat_descr mat;
  rocsparse_dnvec_descr vx, vy;
  SPCHK(rocsparse_create_handle(&sh));
  SPCHK(rocsparse_create_csr_descr(&mat, ndof, ndof, nnz, rp, ci, va, rocsparse_indextype_i64,
                                   rocsparse_indextype_i64, rocsparse_index_base_zero,
                                   rocsparse_datatype_f64_r));
  SPCHK(rocsparse_create_dnvec_descr(&vx, ndof, src, rocsparse_datatype_f64_r));
  SPCHK(rocsparse_create_dnvec_descr(&vy, ndof, ymb, rocsparse_datatype_f64_r));
  const double one = 1.0, zro = 0.0;
  size_t       bsz = 0;
  void        *buf = nullptr;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wdeprecated-declarations"
  auto spmv = [&](rocsparse_spmv_stage stage) {
    SPCHK(rocsparse_spmv(sh, rocsparse_operation_none, &one, mat, vx, &zro, vy,
                         rocsparse_datatype_f64_r, rocsparse_spmv_alg_csr_adaptive, stage, &bsz,
                         buf));
  };
  spmv(rocsparse_spmv_stage_buffer_size);
  HIPCHK(hipMalloc(&buf, bsz > 0 ? bsz : 8));
  spmv(rocsparse_spmv_stage_preprocess);
  spmv(rocsparse_spmv_stage_compute);
  HIPCHK(hipDeviceSynchronize());
  timed("ns::vmult::mb", [&] { spmv(rocsparse_spmv_stage_compute); });
#pragma clang diagnostic pop
  std::vector<double> y_mb((size_t)ndof);
  HIPCHK(hipMemcpy(y_mb.data(), ymb, ndof * 8, hipMemcpyDeviceToHost));

  // poisson::vmult::mf (its own vectors, performance.cc:112-114)
  const Tab1D tb = tables(k);
  const double h  = 1.0 / (double)(1 << n_ref);
  uint32_t    *dcn;
  double      *pdst;
  const int    npc = dim == 3 ? (k + 1) * (k + 1) * (k + 1) : (k + 1) * (k + 1);
  HIPCHK(hipMalloc(&dcn, nc * npc * 4));
  HIPCHK(hipMalloc(&pdst, ndof * 8));
  HIPCHK(hipMemcpy(dcn, gls_mesh_cell_nodes(mesh), nc * npc * 4, hipMemcpyHostToDevice));
  auto poisson = [&] {
    HIPCHK(hipMemsetAsync(pdst, 0, ndof * 8, nullptr)); // cell_loop zeroes dst
    if (dim == 2)
      hipLaunchKernelGGL(k_poisson<2>, dim3((unsigned)nc), dim3(64), 0, nullptr, pdst, src, dcn,
                         nc, tb, h);
    else
      hipLaunchKernelGGL(k_poisson<3>, dim3((unsigned)nc), dim3(64), 0, nullptr, pdst, src, dcn,
                         nc, tb, h);
    HIPCHK(hipGetLastError());
  };
  poisson();
  HIPCHK(hipDeviceSynchronize());
  timed("poisson::vmult::mf", poisson);
  std::vector<double> y_p((size_t)ndof);
  HIPCHK(hipMemcpy(y_p.data(), pdst, ndof * 8, hipMemcpyDeviceToHost));

  // TimerCollection::print_all_wall_time_statistics
  std::printf("%s", gls::timer_report().c_str());
  int64_t calls = 0;
  double  hms = 0, gms = 0;
  char    name[256];
  for (int64_t i = 0; i < gls_timer_n_sections(); ++i)
    {
      gls_timer_section(i, name, sizeof name, &calls, &hms, &gms);
      if (std::strstr(name, "::vmult::"))
        std::printf("%-20s %9.3f us per vmult  %8.3f G DoF/s (host wall)\n", name,
                    hms * 1e3 / reps, (double)ndof * reps / (hms * 1e-3) / 1e9);
    }

  int rc = 0;
  if (check)
    {
      const double e_mb = rel_err(y_mb, y_mf);
      std::vector<double> y_ph((size_t)ndof, 0.0);
      poisson_host(dim, tb, h, nc, gls_mesh_cell_nodes(mesh), h_src, y_ph);
      const double e_p = rel_err(y_p, y_ph);
      std::printf("check: mf vs mb %.3e, poisson vs host %.3e\n", e_mb, e_p);
      rc = e_mb < 1e-12 && e_p < 1e-12 ? 0 : 1;
    }
  SPCHK(rocsparse_destroy_dnvec_descr(vx));
  SPCHK(rocsparse_destroy_dnvec_descr(vy));
  SPCHK(rocsparse_destroy_spmat_descr(mat));
  SPCHK(rocsparse_destroy_handle(sh));
  for (void *p : {(void *)src, (void *)dst, (void *)u, (void *)zero, (void *)rp, (void *)ci,
                  (void *)va, (void *)ymb, buf, (void *)dcn, (void *)pdst})
    HIPCHK(hipFree(p));
  gls_mesh_destroy(mesh);
  return rc;
}
