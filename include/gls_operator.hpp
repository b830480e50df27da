// gls_operator.hpp — header-only C++17 facade over the C ABI of
// libglsamd.so (include/gls_op.h): the host-side mirror of the reference's
// OperatorBase<Number> (include/operator_base.h:13-73) and
// PreconditionerGMG (include/multigrid.h:61-141) for the matrix-free GLS
// Navier–Stokes operator on MI355X, with the Krylov and nonlinear solvers
// around them (solver_l.h, solver_nl.h).
//
// RAII handles; a nonzero status becomes gls::Error (std::runtime_error)
// carrying gls_last_error() — the reference's AssertThrow convention.
// Vectors are device pointers in the operator's precision, local layout
// [owned | ghost], dof = node * (dim+1) + component — or, after
// set_vector_layout(GLS_MEM_HOST, dof_map), host pointers in the caller's
// (deal.II DoFHandler) numbering, as the reference's
// LinearAlgebra::distributed::Vector<Number> (config.h:9-10).  Calls are
// stream-ordered (hipStream_t passed as void*, nullptr = default stream)
// and, like the reference's const-but-mutable operator, not reentrant per
// handle.
#pragma once

#include "gls_op.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace gls
{
class Error : public std::runtime_error
{
public:
  using std::runtime_error::runtime_error;
};

inline void
check(glsStatus s, const char *what)
{
  if (s != 0)
    throw Error(std::string(what) + ": " + gls_last_error());
}

// the library's timer sections (MyTimerOutput, timer.h:194-338): tally on /
// off (returns the previous state) and TimerOutput-style statistics
inline bool
timer_enable(bool on)
{
  int was = 0;
  check(gls_timer_enable(on ? 1 : 0, &was), "timer_enable");
  return was != 0;
}

// MyScope (timer.h:342-413) for the caller's code: a timer section for the
// lifetime of the object
class Scope
{
public:
  explicit Scope(const char *name, void *stream = nullptr)
  {
    check(gls_timer_begin(name, stream, &token), "timer Scope");
  }
  ~Scope() { (void)gls_timer_end(token); }
  Scope(const Scope &)            = delete;
  Scope &operator=(const Scope &) = delete;

private:
  void *token = nullptr;
};

inline std::string
timer_report()
{
  std::string s((size_t)gls_timer_report(nullptr, 0), '\0');
  gls_timer_report(&s[0], (int64_t)s.size());
  s.resize(s.size() - 1);
  return s;
}

// the scalars NavierStokesOperator / TimeIntegratorData feed the cell kernel
// (operator_ns.h:102-114, time_integration.h:10-36)
struct Parameters
{
  double nu = 1, c1 = 1, c2 = 1;
  double theta = 1;  // get_theta()
  double w0    = 0;  // get_primary_weight()
  double dt    = 1;  // get_current_dt()
  int    order = 0;  // get_order()
  int    flags = 0;  // GLS_INCREMENT_FORM | GLS_CONSIDER_TIME_DERIVATIVE | GLS_CELL_WISE_STAB
};

class Operator
{
public:
  Operator() = default;
  explicit Operator(const glsOpDesc &desc) { check(gls_op_create(&desc, &h), "gls_op_create"); }
  ~Operator()
  {
    if (h)
      gls_op_destroy(h);
  }
  Operator(const Operator &)            = delete;
  Operator &operator=(const Operator &) = delete;
  Operator(Operator &&o) noexcept : h(std::exchange(o.h, nullptr)) {}
  Operator &
  operator=(Operator &&o) noexcept
  {
    if (this != &o)
      {
        if (h)
          gls_op_destroy(h);
        h = std::exchange(o.h, nullptr);
      }
    return *this;
  }

  glsOp handle() const { return h; }

  // vector arguments: host or device memory, caller dof numbering
  // (dof_map[i] = node-major dof of caller dof i; empty = node-major)
  void
  set_vector_layout(int memory, const std::vector<int64_t> &dof_map = {})
  {
    check(gls_op_set_vector_layout(h, memory, dof_map.empty() ? nullptr : dof_map.data()),
          "set_vector_layout");
  }

  // OperatorBase::m()  operator_base.h:20-21
  int64_t m() const { return gls_op_m(h); }

  void
  set_parameters(const Parameters &p)
  {
    const glsOpParams q{p.nu, p.c1, p.c2, p.theta, p.w0, p.dt, p.order, p.flags};
    check(gls_op_set_parameters(h, &q), "gls_op_set_parameters");
  }

  // operator_base.h:35-36 (operator_ns.cc:570-620)
  void
  set_linearization_point(const void *src, void *stream = nullptr)
  {
    check(gls_op_set_linearization_point(h, src, stream), "set_linearization_point");
  }

  // operator_base.h:32-33 (operator_ns.cc:234-320): history[0] unused,
  // weights[i] the BDF weights of TimeIntegratorData::get_weights()
  void
  set_previous_solution(const std::vector<const void *> &history,
                        const std::vector<double> &weights, void *stream = nullptr)
  {
    check(gls_op_set_previous_solution(h, history.data(), (int)history.size(), weights.data(),
                                       stream),
          "set_previous_solution");
  }

  // operator_base.h:45-46 (operator_ns.cc:684-732)
  void
  vmult(void *dst, const void *src, void *stream = nullptr) const
  {
    check(gls_op_vmult(h, dst, src, stream), "vmult");
  }

  // operator_base.h:41-43 (operator_ns.cc:648-682)
  void
  evaluate_residual(void *dst, const void *src, void *stream = nullptr) const
  {
    check(gls_op_evaluate_residual(h, dst, src, stream), "evaluate_residual");
  }

  // operator_base.h:41-43 without the distribute step
  void
  evaluate_residual_plain(void *dst, const void *src, void *stream = nullptr) const
  {
    check(gls_op_evaluate_residual_plain(h, dst, src, stream), "evaluate_residual_plain");
  }

  // operator_base.h:38-39 (operator_ns.cc:622-646)
  void
  evaluate_rhs(void *dst, void *stream = nullptr) const
  {
    check(gls_op_evaluate_rhs(h, dst, stream), "evaluate_rhs");
  }

  // constraints_inhomogeneous (main.cc:879-891): values on constrained dofs
  void
  set_constraint_values(const void *values, void *stream = nullptr)
  {
    check(gls_op_set_constraint_values(h, values, stream), "set_constraint_values");
  }

  // operator_base.h:26-27 (operator_ns.cc:195-225)
  void
  compute_inverse_diagonal(void *diag, void *stream = nullptr) const
  {
    check(gls_op_compute_inverse_diagonal(h, diag, stream), "compute_inverse_diagonal");
  }

  // OperatorBase::get_max_u operator_base.h:71-72 (operator_ns.cc:530-568)
  double
  get_max_u(const void *src, void *stream = nullptr) const
  {
    double u = 0;
    check(gls_op_get_max_u(h, src, &u, stream), "get_max_u");
    return u;
  }

  // identity rows after a ghost export-add (distributed vmult)
  void
  apply_identity_rows(void *dst, const void *src, void *stream = nullptr) const
  {
    check(gls_op_apply_identity_rows(h, dst, src, stream), "apply_identity_rows");
  }

  double vmult_bytes() const { return gls_op_vmult_bytes(h); }

  // OperatorBase::Tvmult forwards to vmult (operator_base.cc:12-18)
  void
  Tvmult(void *dst, const void *src, void *stream = nullptr) const
  {
    vmult(dst, src, stream);
  }

  // OperatorBase::vmult_interface_down / _up (operator_ns.cc:734-787); on the
  // globally refined levels this library takes: the vmult / zero
  void
  vmult_interface_down(void *dst, const void *src, void *stream = nullptr) const
  {
    check(gls_op_vmult_interface_down(h, dst, src, stream), "vmult_interface_down");
  }

  void
  vmult_interface_up(void *dst, const void *src, void *stream = nullptr) const
  {
    check(gls_op_vmult_interface_up(h, dst, src, stream), "vmult_interface_up");
  }

  // OperatorBase::get_system_matrix (operator_ns.cc:1407-1430) as CSR over
  // the node-major dofs; constrained rows / columns carry their unit diagonal
  struct SparseMatrix
  {
    std::vector<int64_t> row_ptr, cols;
    std::vector<double>  vals;
  };
  SparseMatrix
  get_system_matrix() const
  {
    SparseMatrix A;
    int64_t      nnz = 0;
    check(gls_op_system_matrix(h, &nnz, nullptr, nullptr, nullptr), "get_system_matrix");
    A.row_ptr.resize((size_t)m() + 1);
    A.cols.resize((size_t)nnz);
    A.vals.resize((size_t)nnz);
    check(gls_op_system_matrix(h, &nnz, A.row_ptr.data(), A.cols.data(), A.vals.data()),
          "get_system_matrix");
    return A;
  }

private:
  glsOp h = nullptr;
};

// PreconditionerGMG: level operators (MGNumber precision), transfers,
// relaxation smoother, V-cycle
class Multigrid
{
public:
  Multigrid() = default;
  Multigrid(const glsMGDesc &desc, const std::vector<const Operator *> &levels,
            const std::vector<const uint32_t *> &child_lattices)
  {
    std::vector<glsOp> ops;
    for (const Operator *o : levels)
      ops.push_back(o->handle());
    std::vector<const uint32_t *> ch(levels.size(), nullptr);
    for (size_t l = 1; l < levels.size() && l - 1 < child_lattices.size(); ++l)
      ch[l] = child_lattices[l - 1];
    check(gls_mg_create(&desc, ops.data(), ch.data(), &h), "gls_mg_create");
  }
  ~Multigrid()
  {
    if (h)
      gls_mg_destroy(h);
  }
  Multigrid(const Multigrid &)            = delete;
  Multigrid &operator=(const Multigrid &) = delete;
  Multigrid(Multigrid &&o) noexcept : h(std::exchange(o.h, nullptr)) {}

  void
  set_vector_layout(int memory, const std::vector<int64_t> &dof_map = {})
  {
    check(gls_mg_set_vector_layout(h, memory, dof_map.empty() ? nullptr : dof_map.data()),
          "gls_mg_set_vector_layout");
  }

  // PreconditionerGMG::initialize (multigrid.cc:247-370)
  void initialize(void *stream = nullptr) { check(gls_mg_setup(h, stream), "gls_mg_setup"); }

  // PreconditionerGMG::vmult (multigrid.cc:202-220): one V-cycle
  void
  vmult(void *dst, const void *src, void *stream = nullptr) const
  {
    check(gls_mg_vcycle(h, dst, src, stream), "gls_mg_vcycle");
  }

  std::pair<double, double>
  relaxation(int level) const
  {
    double w = 0, lam = 0;
    check(gls_mg_get_relaxation(h, level, &w, &lam), "gls_mg_get_relaxation");
    return {w, lam};
  }

  void
  interpolate(int level, void *dst_coarse, const void *src_fine, void *stream = nullptr) const
  {
    check(gls_mg_interpolate(h, level, dst_coarse, src_fine, stream), "gls_mg_interpolate");
  }

  glsMG handle() const { return h; }

private:
  glsMG h = nullptr;
};

// LinearSolverGMRES (solver_l.h:60-82, solver_l.cc:26-74): right-
// preconditioned restarted GMRES on the device (gls_gmres_solve), the
// preconditioner a Multigrid (PreconditionerGMG::vmult, one V-cycle) or none;
// vectors in the operator's layout.  solve() throws gls::Error on no
// convergence (SolverControl::NoConvergence); last() holds the statistics.
class LinearSolverGMRES
{
public:
  LinearSolverGMRES(const Operator &op, const Multigrid *preconditioner = nullptr,
                    int n_max_iterations = 10000, double absolute_tolerance = 1e-12,
                    double relative_tolerance = 1e-8, int max_n_tmp_vectors = 30)
    : op(op), mg(preconditioner),
      desc{max_n_tmp_vectors, n_max_iterations, absolute_tolerance, relative_tolerance}
  {}

  void
  solve(void *dst, const void *src, void *stream = nullptr)
  {
    check(gls_gmres_solve(op.handle(), mg ? mg->handle() : nullptr, &desc, dst, src, &res,
                          stream),
          "gls_gmres_solve");
  }

  const glsGMRESResult &last() const { return res; }

private:
  const Operator   &op;
  const Multigrid  *mg;
  glsGMRESDesc      desc;
  glsGMRESResult    res{};
};

// ---- nonlinear solvers: NonLinearSolverLinearized / Newton / Picard
// (solver_nl.h:14-95, solver_nl.cc:4-140) over the caller's vector type with
// the reference's std::function hooks, which a driver wires as main.cc:805-864
// does (setup_jacobian = set_linearization_point, evaluate_residual /
// evaluate_rhs = the operator's, solve_with_jacobian = LinearSolverGMRES::
// solve, setup_preconditioner = Multigrid::initialize).  VectorType needs
// what deal.II's Vector offers here: reinit(const VectorType &) (same layout,
// zero), operator=(double) (0 only), add(double, const VectorType &),
// l2_norm() and copy construction; HostVector below is one for operators in
// the GLS_MEM_HOST layout.  A failed convergence throws gls::Error, as the
// reference's AssertThrow.
template <typename VectorType>
class NonLinearSolverBase
{
public:
  virtual ~NonLinearSolverBase() = default;
  virtual int solve(VectorType &solution) const = 0; // returns the iterations

  std::function<void(const VectorType &src)>                  setup_jacobian;
  std::function<void(const VectorType &src)>                  setup_preconditioner;
  std::function<void(VectorType &dst, const VectorType &src)> evaluate_residual;
  std::function<void(VectorType &dst)>                        evaluate_rhs;
  std::function<void(VectorType &dst, const VectorType &src)> solve_with_jacobian;
  std::function<void(const VectorType &dst)>                  postprocess;
  // the residual l2 norm of every step (the reference's "[N] step" lines)
  mutable std::vector<double> history;
};

// one linear solve around the current solution (solver_nl.cc:10-24)
template <typename VectorType>
class NonLinearSolverLinearized : public NonLinearSolverBase<VectorType>
{
public:
  int
  solve(VectorType &solution) const override
  {
    this->setup_jacobian(solution);
    VectorType rhs(solution);
    rhs.reinit(solution);
    this->evaluate_rhs(rhs);
    this->setup_preconditioner(solution);
    this->solve_with_jacobian(solution, rhs);
    return 1;
  }
};

// Newton on the residual, the preconditioner set up at the first step only
// when inexact (solver_nl.cc:26-89; tolerance 1e-7, at most 30 steps there)
template <typename VectorType>
class NonLinearSolverNewton : public NonLinearSolverBase<VectorType>
{
public:
  explicit NonLinearSolverNewton(bool inexact_newton, double newton_tolerance = 1.0e-7,
                                 int newton_max_iteration = 30)
    : inexact_newton(inexact_newton), tol(newton_tolerance), max_it(newton_max_iteration)
  {}

  int
  solve(VectorType &solution) const override
  {
    Scope      scope("newton::solve"); // solver_nl.cc:38
    VectorType rhs(solution), inc(solution);
    rhs.reinit(solution);
    inc.reinit(solution);
    this->setup_jacobian(solution);
    this->evaluate_residual(rhs, solution);
    double l2 = rhs.l2_norm();
    int    it = 0;
    this->history.assign(1, l2);
    while (l2 > tol)
      {
        inc = 0.0;
        if (it == 0 || !inexact_newton)
          this->setup_preconditioner(solution);
        this->solve_with_jacobian(inc, rhs);
        solution.add(1.0, inc);
        if (this->postprocess)
          this->postprocess(solution);
        this->setup_jacobian(solution);
        this->evaluate_residual(rhs, solution);
        l2 = rhs.l2_norm();
        ++it;
        this->history.push_back(l2);
        if (it > max_it)
          throw Error("Newton iteration did not converge. Final residual_0 is " +
                      std::to_string(l2) + ".");
      }
    return it;
  }

private:
  bool   inexact_newton;
  double tol;
  int    max_it;
};

// fixed-point iteration on the linearized operator, converged when the
// update's l2 norm drops below the tolerance (solver_nl.cc:91-140)
template <typename VectorType>
class NonLinearSolverPicard : public NonLinearSolverBase<VectorType>
{
public:
  explicit NonLinearSolverPicard(double picard_tolerance = 1.0e-7, int picard_max_iteration = 30)
    : tol(picard_tolerance), max_it(picard_max_iteration)
  {}

  int
  solve(VectorType &solution) const override
  {
    VectorType rhs(solution), tmp(solution);
    rhs.reinit(solution);
    double l2 = 1e10;
    int    it = 0;
    this->history.clear();
    while (l2 > tol)
      {
        tmp = solution;
        this->setup_jacobian(solution);
        this->evaluate_rhs(rhs);
        this->setup_preconditioner(solution);
        this->solve_with_jacobian(solution, rhs);
        tmp.add(-1.0, solution);
        l2 = tmp.l2_norm();
        ++it;
        this->history.push_back(l2);
        if (it > max_it)
          throw Error("Picard iteration did not converge. Final residual_0 is " +
                      std::to_string(l2) + ".");
      }
    return it;
  }

private:
  double tol;
  int    max_it;
};

// a host vector for operators in the GLS_MEM_HOST layout (the reference's
// LinearAlgebra::distributed::Vector<double> on one rank)
struct HostVector : std::vector<double>
{
  using std::vector<double>::vector;
  void
  reinit(const HostVector &like)
  {
    assign(like.size(), 0.0);
  }
  HostVector &
  operator=(double s)
  {
    std::fill(begin(), end(), s);
    return *this;
  }
  void
  add(double a, const HostVector &v)
  {
    for (size_t i = 0; i < size(); ++i)
      (*this)[i] += a * v[i];
  }
  double
  l2_norm() const
  {
    double s = 0;
    for (double x : *this)
      s += x * x;
    return std::sqrt(s);
  }
};
} // namespace gls
