// TEST INFRASTRUCTURE: C++ parity check of the HIP operator through the
// header-only facade include/gls_operator.hpp (the host-side mirror of the
// reference's OperatorBase), against the CPU oracle (oracle/gls_oracle.h)
// on the same mesh and §8d synthetic inputs.  Driven by tests/test_cpp.py.
//
//   test_operator dim degree n_ref length height position diameter shift
//                 vel_bits p_bits slip_bits u_inf nu c1 c2 theta dt order
//                 flags w0 [w1 w2 w3]
// exit 0: relative l2 errors < 1e-12 (inverse diagonal 1e-11) and the
// error path throws.
#include "gls_mesh.h"
#include "gls_operator.hpp"
#include "../../oracle/gls_oracle.h"

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

static uint64_t
splitmix64(uint64_t x)
{
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z          = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z          = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// glsinputs.rnd: ((splitmix64(seed * 2^32 + i) >> 11) * 2^-53) * 2 - 1
static std::vector<double>
rnd(uint64_t seed, size_t n)
{
  std::vector<double> r(n);
  for (size_t i = 0; i < n; ++i)
    r[i] = (double)(splitmix64(seed * (1ull << 32) + i) >> 11) * 0x1.0p-53 * 2.0 - 1.0;
  return r;
}

static double
rel_err(const std::vector<double> &a, const std::vector<double> &b)
{
  double num = 0, den = 0;
  for (size_t i = 0; i < a.size(); ++i)
    {
      num += (a[i] - b[i]) * (a[i] - b[i]);
      den += b[i] * b[i];
    }
  return std::sqrt(num) / std::max(std::sqrt(den), 1e-300);
}

#define HIPCHK(x)                                                              \
  do                                                                           \
    {                                                                          \
      if ((x) != hipSuccess)                                                   \
        {                                                                      \
          std::fprintf(stderr, "HIP error %s line %d\n", #x, __LINE__);        \
          return 2;                                                            \
        }                                                                      \
    }                                                                          \
  while (0)

struct DevVec
{
  double *p = nullptr;
  size_t  n = 0;
  explicit DevVec(size_t n_) : n(n_) { (void)hipMalloc(&p, n * sizeof(double)); }
  ~DevVec() { (void)hipFree(p); }
  void up(const std::vector<double> &h) { (void)hipMemcpy(p, h.data(), n * 8, hipMemcpyHostToDevice); }
  std::vector<double>
  down() const
  {
    std::vector<double> h(n);
    (void)hipMemcpy(h.data(), p, n * 8, hipMemcpyDeviceToHost);
    return h;
  }
};

// the VectorType of the facade's nonlinear solvers (include/gls_operator.hpp)
// for a device-layout FP64 operator: the reductions and the update through
// host copies (test sizes only)
struct NewtonVec
{
  double *p = nullptr;
  size_t  n = 0;
  explicit NewtonVec(size_t n_) : n(n_) { (void)hipMalloc(&p, n * 8); }
  NewtonVec(const NewtonVec &o) : NewtonVec(o.n)
  {
    (void)hipMemcpy(p, o.p, n * 8, hipMemcpyDeviceToDevice);
  }
  NewtonVec &
  operator=(const NewtonVec &o)
  {
    (void)hipMemcpy(p, o.p, n * 8, hipMemcpyDeviceToDevice);
    return *this;
  }
  ~NewtonVec() { (void)hipFree(p); }
  void reinit(const NewtonVec &) { (void)hipMemset(p, 0, n * 8); }
  NewtonVec &
  operator=(double)
  {
    (void)hipMemset(p, 0, n * 8);
    return *this;
  }
  std::vector<double>
  down() const
  {
    std::vector<double> h(n);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h.data(), p, n * 8, hipMemcpyDeviceToHost);
    return h;
  }
  void
  add(double a, const NewtonVec &v)
  {
    std::vector<double> x = down(), y = v.down();
    for (size_t i = 0; i < n; ++i)
      x[i] += a * y[i];
    (void)hipMemcpy(p, x.data(), n * 8, hipMemcpyHostToDevice);
  }
  double
  l2_norm() const
  {
    double s = 0;
    for (double x : down())
      s += x * x;
    return std::sqrt(s);
  }
};

static int run(int argc, char **argv);

int
main(int argc, char **argv)
{
  try
    {
      return run(argc, argv);
    }
  catch (const std::exception &e)
    {
      std::printf("uncaught: %s\n", e.what());
      return 2;
    }
}

static int
run(int argc, char **argv)
{
  if (argc < 21)
    {
      std::fprintf(stderr, "usage: see header\n");
      return 2;
    }
  gls::timer_enable(true); // the library's timer sections, reported at the end
  int         a = 1;
  const int   dim = std::atoi(argv[a++]), degree = std::atoi(argv[a++]), n_ref = std::atoi(argv[a++]);
  const double length = std::atof(argv[a++]), height = std::atof(argv[a++]),
               position = std::atof(argv[a++]), diameter = std::atof(argv[a++]),
               shift = std::atof(argv[a++]);
  const uint32_t vel = (uint32_t)std::atol(argv[a++]), pb = (uint32_t)std::atol(argv[a++]),
                 slip = (uint32_t)std::atol(argv[a++]);
  const double u_inf = std::atof(argv[a++]);
  gls::Parameters prm;
  prm.nu    = std::atof(argv[a++]);
  prm.c1    = std::atof(argv[a++]);
  prm.c2    = std::atof(argv[a++]);
  prm.theta = std::atof(argv[a++]);
  prm.dt    = std::atof(argv[a++]);
  prm.order = std::atoi(argv[a++]);
  prm.flags = std::atoi(argv[a++]);
  std::vector<double> w;
  for (; a < argc; ++a)
    w.push_back(std::atof(argv[a]));
  prm.w0 = w.empty() ? 0.0 : w[0];

  glsMesh *mesh = nullptr;
  if (gls_mesh_cylinder(dim, degree, n_ref, length, height, position, diameter, shift, &mesh))
    {
      std::fprintf(stderr, "mesh: %s\n", gls_mesh_last_error());
      return 2;
    }
  const int64_t        nc = gls_mesh_n_cells(mesh), nn = gls_mesh_n_nodes(mesh);
  const int            ncomp = dim + 1;
  const size_t         ndof  = (size_t)nn * ncomp;
  std::vector<uint8_t> cmask((size_t)nn);
  std::vector<double>  meas((size_t)nc), hmin((size_t)nc);
  int                  brick[3] = {0, 0, 0};
  if (gls_mesh_constraint_mask(mesh, vel, pb, slip, cmask.data()) ||
      gls_mesh_cell_measure(mesh, meas.data(), hmin.data()) || gls_mesh_brick(mesh, brick))
    {
      std::fprintf(stderr, "mesh: %s\n", gls_mesh_last_error());
      return 2;
    }

  glsOpDesc d{};
  d.dim           = dim;
  d.degree        = degree;
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

  // error convention: an invalid descriptor throws gls::Error
  {
    glsOpDesc bad     = d;
    bad.n_owned_nodes = nn + 1;
    bool thrown       = false;
    try
      {
        gls::Operator op(bad);
      }
    catch (const gls::Error &e)
      {
        thrown = true;
        std::printf("error path ok: %s\n", e.what());
        std::fflush(stdout);
      }
    if (!thrown)
      {
        std::fprintf(stderr, "invalid descriptor did not throw\n");
        return 1;
      }
  }

  // §8d inputs (glsinputs.py)
  std::vector<double> src = rnd(1, ndof), r2 = rnd(2, ndof), u(ndof);
  for (int64_t i = 0; i < nn; ++i)
    {
      u[i * ncomp] = u_inf * (1.0 + 0.1 * r2[i * ncomp]);
      for (int c = 1; c < dim; ++c)
        u[i * ncomp + c] = 0.1 * u_inf * r2[i * ncomp + c];
      u[i * ncomp + dim] = r2[i * ncomp + dim];
    }
  std::vector<std::vector<double>> hist(1, u);
  for (int i = 1; i <= prm.order; ++i)
    {
      std::vector<double> h(u);
      for (double &x : h)
        x *= 1.0 - 0.01 * i;
      hist.push_back(h);
    }

  // HIP operator through the facade
  gls::Operator op(d);
  op.set_parameters(prm);
  DevVec dsrc(ndof), du(ndof), ddst(ndof), dres(ndof), ddiag(ndof);
  dsrc.up(src);
  du.up(u);
  op.set_linearization_point(du.p);
  std::vector<DevVec *> dh;
  std::vector<const void *> hp;
  for (auto &h : hist)
    {
      dh.push_back(new DevVec(ndof));
      dh.back()->up(h);
      hp.push_back(dh.back()->p);
    }
  if (prm.order > 0)
    op.set_previous_solution(hp, w);
  op.vmult(ddst.p, dsrc.p);
  op.evaluate_residual_plain(dres.p, dsrc.p);
  op.compute_inverse_diagonal(ddiag.p);
  HIPCHK(hipDeviceSynchronize());
  // get_system_matrix through the facade: CSR x == vmult x
  std::vector<double> g_spmv(ndof, 0.0);
  {
    const auto A = op.get_system_matrix();
    for (size_t r = 0; r < ndof; ++r)
      for (int64_t q = A.row_ptr[r]; q < A.row_ptr[r + 1]; ++q)
        g_spmv[r] += A.vals[(size_t)q] * src[(size_t)A.cols[(size_t)q]];
  }
  const std::vector<double> g_dst = ddst.down(), g_res = dres.down(), g_diag = ddiag.down();
  for (DevVec *p : dh)
    delete p;

  // oracle
  orc_mesh   om{dim, degree, nc, nn, d.cell_nodes, d.node_coords, cmask.data(), meas.data(),
              hmin.data()};
  orc_params oprm{prm.nu, prm.c1, prm.c2, prm.theta, prm.w0, prm.dt, prm.order,
                  (prm.flags & GLS_CONSIDER_TIME_DERIVATIVE) ? 1 : 0,
                  (prm.flags & GLS_INCREMENT_FORM) ? 1 : 0,
                  (prm.flags & GLS_CELL_WISE_STAB) ? 1 : 0};
  orc_op    *o = orc_create(&om, &oprm);
  orc_set_linearization_point(o, u.data());
  if (prm.order > 0)
    {
      std::vector<const double *> hh;
      for (auto &h : hist)
        hh.push_back(h.data());
      orc_set_previous_solution(o, hh.data(), (int)hh.size(), w.data());
    }
  std::vector<double> c_dst(ndof), c_res(ndof), c_diag(ndof);
  orc_vmult(o, c_dst.data(), src.data());
  orc_evaluate_residual(o, c_res.data(), src.data());
  orc_compute_inverse_diagonal(o, c_diag.data());
  orc_destroy(o);

  const double e0 = rel_err(g_dst, c_dst), e1 = rel_err(g_res, c_res), e2 = rel_err(g_diag, c_diag),
               e8 = rel_err(g_spmv, c_dst);
  std::printf("cells %lld dofs %zu  vmult %.3e  residual %.3e  inverse_diagonal %.3e  "
              "system matrix %.3e\n",
              (long long)nc, ndof, e0, e1, e2, e8);

  // ---- the reference's vector layout: host memory (LA::distributed::Vector
  // in host memory, config.h:9-10) in a non-node-major numbering (a
  // deal.II-like DoFHandler numbering: a fixed pseudo-random permutation
  // perm[i] = node-major dof of caller dof i)
  std::vector<int64_t> perm(ndof);
  for (size_t i = 0; i < ndof; ++i)
    perm[i] = (int64_t)i;
  for (size_t i = ndof - 1; i > 0; --i)
    std::swap(perm[i], perm[splitmix64(77 + i) % (i + 1)]);
  auto to_caller = [&](const std::vector<double> &x) {
    std::vector<double> y(ndof);
    for (size_t i = 0; i < ndof; ++i)
      y[i] = x[(size_t)perm[i]];
    return y;
  };
  gls::Operator hop(d);
  hop.set_vector_layout(GLS_MEM_HOST, perm);
  hop.set_parameters(prm);
  const std::vector<double> u_c = to_caller(u), src_c = to_caller(src);
  hop.set_linearization_point(u_c.data());
  std::vector<std::vector<double>> hist_c;
  std::vector<const void *>        hp_c;
  for (auto &hv : hist)
    hist_c.push_back(to_caller(hv));
  for (auto &hv : hist_c)
    hp_c.push_back(hv.data());
  if (prm.order > 0)
    hop.set_previous_solution(hp_c, w);
  std::vector<double> h_dst(ndof), h_res(ndof), h_diag(ndof);
  hop.vmult(h_dst.data(), src_c.data());
  hop.evaluate_residual_plain(h_res.data(), src_c.data());
  hop.compute_inverse_diagonal(h_diag.data());
  const double gmax = hop.get_max_u(u_c.data());
  orc_op *o2 = orc_create(&om, &oprm);
  const double cmax = orc_get_max_u(o2, u.data());
  orc_destroy(o2);
  // ---- LinearSolverGMRES with the GMG preconditioner through the facade
  // (3D, n_ref >= 1: levels r-1, r in FP32, coarse relaxation sweeps): the
  // solution's true residual, from the oracle, meets the tolerance.  (The
  // damped-Jacobi V-cycle does not precondition the stationary 2D
  // saddle-point decks; tests/test_gpu_krylov.py covers those.)
  double e7 = 0.0;
  int    gm_its = 0;
  int    n_newton = 0;          // Newton steps (3D, n_ref >= 1)
  double newton_res = 0.0;      // the oracle's residual of the Newton solution
  if (n_ref >= 1 && dim == 3)
    {
      glsMesh *cmesh = nullptr;
      if (gls_mesh_cylinder(dim, degree, n_ref - 1, length, height, position, diameter, shift,
                            &cmesh))
        {
          std::fprintf(stderr, "mesh: %s\n", gls_mesh_last_error());
          return 2;
        }
      const int64_t        cnc = gls_mesh_n_cells(cmesh), cnn = gls_mesh_n_nodes(cmesh);
      std::vector<uint8_t> ccm((size_t)cnn);
      std::vector<double>  cmeas((size_t)cnc), chmin((size_t)cnc);
      int                  cbrick[3] = {0, 0, 0};
      const int            Lc = 2 * degree + 1, nl = dim == 3 ? Lc * Lc * Lc : Lc * Lc;
      std::vector<uint32_t> child((size_t)cnc * nl);
      if (gls_mesh_constraint_mask(cmesh, vel, pb, slip, ccm.data()) ||
          gls_mesh_cell_measure(cmesh, cmeas.data(), chmin.data()) ||
          gls_mesh_brick(cmesh, cbrick) || gls_mesh_child_lattice(cmesh, mesh, child.data()))
        {
          std::fprintf(stderr, "mesh: %s\n", gls_mesh_last_error());
          return 2;
        }
      glsOpDesc cd = d;
      cd.precision = GLS_F32;
      cd.n_cells = cnc, cd.n_nodes = cnn, cd.n_owned_nodes = cnn;
      cd.cell_nodes   = gls_mesh_cell_nodes(cmesh);
      cd.node_coords  = gls_mesh_node_coords(cmesh);
      cd.node_cmask   = ccm.data();
      cd.cell_measure = cmeas.data();
      cd.cell_hmin    = chmin.data();
      for (int i = 0; i < 3; ++i)
        cd.brick[i] = cbrick[i];
      glsOpDesc fd = d;
      fd.precision = GLS_F32;
      gls::Operator l0(cd), l1(fd);
      l0.set_parameters(prm);
      l1.set_parameters(prm);
      glsMGDesc md{};
      md.n_levels = 2, md.smoothing_n_iterations = 5, md.smoothing_eig_n_iterations = 20;
      md.smoothing_range = 20.0, md.coarse_n_iterations = 10, md.outer_precision = GLS_F64;
      gls::Multigrid mg(md, {&l0, &l1}, {child.data()});
      // the linearization point on the levels (interpolate_to_mg, main.cc:772-803)
      const size_t cdof = (size_t)cnn * ncomp;
      float       *fu = nullptr, *cu = nullptr;
      std::vector<float> uf(u.begin(), u.end());
      HIPCHK(hipMalloc(&fu, ndof * 4));
      HIPCHK(hipMalloc(&cu, cdof * 4));
      HIPCHK(hipMemcpy(fu, uf.data(), ndof * 4, hipMemcpyHostToDevice));
      mg.interpolate(1, cu, fu);
      l1.set_linearization_point(fu);
      l0.set_linearization_point(cu);
      std::vector<std::vector<float>> hf;
      std::vector<float *>            dhf, dhc;
      std::vector<const void *>       pf, pc;
      if (prm.order > 0)
        for (auto &hv : hist)
          {
            hf.emplace_back(hv.begin(), hv.end());
            float *a1 = nullptr, *a0 = nullptr;
            HIPCHK(hipMalloc(&a1, ndof * 4));
            HIPCHK(hipMalloc(&a0, cdof * 4));
            HIPCHK(hipMemcpy(a1, hf.back().data(), ndof * 4, hipMemcpyHostToDevice));
            mg.interpolate(1, a0, a1);
            dhf.push_back(a1), dhc.push_back(a0), pf.push_back(a1), pc.push_back(a0);
          }
      if (prm.order > 0)
        {
          l1.set_previous_solution(pf, w);
          l0.set_previous_solution(pc, w);
        }
      mg.initialize();
      const double         rtol = 1e-6;
      gls::LinearSolverGMRES solver(op, &mg, 500, 1e-12, rtol);
      DevVec               dx(ndof);
      solver.solve(dx.p, dsrc.p);
      HIPCHK(hipDeviceSynchronize());
      gm_its                 = solver.last().n_iterations;
      const std::vector<double> x = dx.down();
      orc_op *o3 = orc_create(&om, &oprm);
      orc_set_linearization_point(o3, u.data());
      if (prm.order > 0)
        {
          std::vector<const double *> hh;
          for (auto &hv : hist)
            hh.push_back(hv.data());
          orc_set_previous_solution(o3, hh.data(), (int)hh.size(), w.data());
        }
      std::vector<double> ax(ndof);
      orc_vmult(o3, ax.data(), x.data());
      orc_destroy(o3);
      double rn = 0, bn = 0;
      for (size_t i = 0; i < ndof; ++i)
        {
          rn += (src[i] - ax[i]) * (src[i] - ax[i]);
          bn += src[i] * src[i];
        }
      e7 = std::sqrt(rn / bn) / rtol;
      // ---- NonLinearSolverNewton (solver_nl.cc:36-89) through the facade,
      // wired as main.cc:805-864: one implicit step of this operator from
      // the history, homogeneous Dirichlet values (the start value's
      // constrained entries zero), inexact Newton (the multigrid set up at
      // the first step), GMRES to 1e-2; the converged solution's residual
      // recomputed by the oracle
      {
        gls::LinearSolverGMRES                lin(op, &mg, 1000, 1e-12, 1e-2);
        gls::NonLinearSolverNewton<NewtonVec> newton(true);
        newton.setup_jacobian = [&](const NewtonVec &v) { op.set_linearization_point(v.p); };
        newton.setup_preconditioner = [&](const NewtonVec &) { mg.initialize(); };
        newton.evaluate_residual    = [&](NewtonVec &dst, const NewtonVec &src) {
          op.evaluate_residual(dst.p, src.p);
        };
        newton.solve_with_jacobian = [&](NewtonVec &dst, const NewtonVec &src) {
          lin.solve(dst.p, src.p);
        };
        std::vector<double> u0 = u;
        for (int64_t nd = 0; nd < nn; ++nd)
          for (int c = 0; c < ncomp; ++c)
            if ((cmask[(size_t)nd] >> c) & 1)
              u0[(size_t)nd * ncomp + c] = 0.0;
        NewtonVec sol(ndof);
        (void)hipMemcpy(sol.p, u0.data(), ndof * 8, hipMemcpyHostToDevice);
        n_newton = newton.solve(sol);
        const std::vector<double> xs = sol.down();
        orc_op *o4 = orc_create(&om, &oprm);
        orc_set_linearization_point(o4, xs.data());
        if (prm.order > 0)
          {
            std::vector<const double *> hh;
            for (auto &hv : hist)
              hh.push_back(hv.data());
            orc_set_previous_solution(o4, hh.data(), (int)hh.size(), w.data());
          }
        std::vector<double> r(ndof);
        orc_evaluate_residual(o4, r.data(), xs.data());
        orc_destroy(o4);
        double r2 = 0;
        for (double v : r)
          r2 += v * v;
        newton_res = std::sqrt(r2);
        std::printf("Newton (facade): %d steps, residuals", n_newton);
        for (double h : newton.history)
          std::printf(" %.3e", h);
        std::printf("; oracle residual of the solution %.3e\n", newton_res);
      }
      for (float *q : dhf)
        (void)hipFree(q);
      for (float *q : dhc)
        (void)hipFree(q);
      (void)hipFree(fu);
      (void)hipFree(cu);
      gls_mesh_destroy(cmesh);
      std::printf("GMRES + GMG (facade): %d iterations, true residual / tolerance %.3f\n", gm_its,
                  e7);
    }
  gls_mesh_destroy(mesh); // owns cell_nodes / node_coords of d and om
  const double e3 = rel_err(h_dst, to_caller(c_dst)), e4 = rel_err(h_res, to_caller(c_res)),
               e5 = rel_err(h_diag, to_caller(c_diag)), e6 = std::fabs(gmax - cmax) / cmax;
  std::printf("host memory, permuted numbering: vmult %.3e  residual %.3e  inverse_diagonal "
              "%.3e  get_max_u %.6f vs %.6f (%.1e)\n",
              e3, e4, e5, gmax, cmax, e6);
  const std::string rep = gls::timer_report();
  std::printf("%s", rep.c_str());
  // (the GMRES + GMG block runs on the 3D decks only)
  const bool timed = rep.find("ns::vmult ") != std::string::npos &&
                     (gm_its == 0 ||
                      (rep.find("gmres::solve ") != std::string::npos &&
                       rep.find("gmg::vmult::level_1::0_pre_smoother_step") != std::string::npos)) &&
                     (n_newton == 0 || rep.find("newton::solve ") != std::string::npos);
  // 1/d amplifies the round-off of near-cancelling diagonal entries:
  // 10x the FP64 bound, as tests/test_gpu_parity.py
  return (timed && e0 < 1e-12 && e1 < 1e-12 && e2 < 1e-11 && e3 < 1e-12 && e4 < 1e-12 && e5 < 1e-11 &&
          e6 < 1e-13 && e7 < 1.05 && e8 < 1e-12 && newton_res <= 1e-6 && n_newton <= 30) ?
           0 :
           1;
}
