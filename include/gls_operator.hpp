// gls_operator.hpp — header-only C++17 facade over the C ABI of
// libglsamd.so (include/gls_op.h): the host-side mirror of the reference's
// OperatorBase<Number> (include/operator_base.h:13-73) and
// PreconditionerGMG (include/multigrid.h:61-141) for the matrix-free GLS
// Navier–Stokes operator on MI355X.
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
} // namespace gls
