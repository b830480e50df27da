// op_internal.h — the operator handle's state, shared by gls_op.hip (the
// operator) and mg.hip (the multigrid that drives level operators).
#pragma once

#include "../../include/gls_op.h"
#include "common.h"

#include <cstdint>
#include <vector>

namespace gls
{
// Caller-side vector layout of the C-ABI (gls_op_set_vector_layout /
// gls_mg_set_vector_layout): vectors in host memory (the reference's
// LinearAlgebra::distributed::Vector<Number> lives in host memory,
// config.h:9-10) and/or in the caller's dof numbering (deal.II's DoFHandler
// numbering, dof_map[i] = this library's node-major dof of caller dof i).
// Inputs are staged into node-major device buffers, outputs written to a
// device buffer and permuted / copied back; host-memory calls return
// synchronised (host semantics).  Device memory in node-major order (the
// default) takes no staging at all.
struct VecStage
{
  int      memory = GLS_MEM_DEVICE;
  int64_t  n      = 0;
  size_t   ts     = 8;
  int64_t *d_map  = nullptr; // [n] or null
  void    *raw    = nullptr; // [n] caller-order device copy of a host vector
  void    *in[4]  = {nullptr, nullptr, nullptr, nullptr};
  void    *out    = nullptr;

  bool
  active() const
  {
    return memory == GLS_MEM_HOST || d_map;
  }
  void        set(int memory, const int64_t *map, int64_t n, size_t ts);
  const void *in_vec(const void *v, int slot, hipStream_t s);
  void       *out_vec(void *v);
  void        finish_out(void *v, hipStream_t s);
  void        done(hipStream_t s);
  void        release();
};

// outflow boundary faces (faces.hip): per face the internal cell, the kind
// (cut / Nitsche), effective_beta_face and the face geometry at the
// QGauss(k+1)^(dim-1) points, in the operator's precision
struct OutflowFaces
{
  int64_t             n   = 0;
  int                 nqf = 0;
  std::vector<double> h_points; // [n][nqf][dim] face quadrature points
  int64_t            *d_cell   = nullptr;
  int32_t            *d_kind   = nullptr;
  void               *d_beta   = nullptr; // [n]
  void               *d_jxw    = nullptr; // [n][nqf]
  void               *d_normal = nullptr; // [n][nqf][dim]
  void               *d_phi    = nullptr; // [n][nqf][nq] cell basis at the face points
  void               *d_dn     = nullptr; // [n][nqf][nq] its physical normal derivative
  void               *d_ustar  = nullptr; // [n][nqf][dim] face_velocity
  void               *d_target = nullptr; // [n][nqf][dim] face_target_velocity
};
} // namespace gls

struct glsOp_
{
  int     dim = 3, degree = 2, prec = GLS_F64;
  int64_t n_cells = 0, n_nodes = 0, n_owned_nodes = 0, n_dofs = 0, n_owned_dofs = 0;
  int     nq = 0, nf = 0; // nf: fields of the canonical host table layout (upload/download)
  int     nf_store = 0;    // fields stored per (cell, q) on the device (kernels.h Fields)
  // T1 (Fields::T1) is formed from the producers' tables and the time
  // weights; recomputed before a Newton brick vmult when either changed
  mutable bool   t1_valid = false;
  mutable double t1_w0    = 0.0;
  mutable int    t1_td    = -1;
  gls::Basis1D basis{1};

  glsOpParams prm{};
  bool        have_lin = false, have_prev = false, have_old_grad = false;
  // bumped by every call that changes what a launch captures by value
  // (parameters, table producers): a captured V-cycle graph of the
  // multigrid (csrc/mg.hip) is re-captured when a level's version moved
  uint64_t    version = 0;

  // host copies the multigrid transfer setup needs
  std::vector<uint8_t>  h_cmask;      // [n_nodes]
  std::vector<uint32_t> h_cell_nodes; // [n_cells][nq], caller cell order
  // discovered bricks (glsOpDesc::brick[0] < 0): the operator runs its cells
  // in brick order, cell_perm[internal cell] = caller cell (empty: identity)
  std::vector<int64_t>  cell_perm;

  int64_t n_gen = 0, n_cart = 0;
  // device buffers
  uint32_t *d_nodes    = nullptr; // [n_cells][nq] node | cmask << 28
  uint32_t *d_cell_geo = nullptr;
  void     *d_geo_cart = nullptr;
  void     *d_geo_gen  = nullptr;
  void     *d_tab      = nullptr;
  void     *d_cellwise = nullptr;
  void     *d_old_grad = nullptr;
  void     *d_hq       = nullptr;
  void     *d_hmin     = nullptr;
  void     *d_tmp      = nullptr;
  uint32_t *d_cbits    = nullptr; // constrained-dof bitmask (owned range)
  uint8_t  *d_node_cmask = nullptr; // [n_nodes] constrained components (owned + ghost)
  void     *d_inhom      = nullptr; // [n_dofs] inhomogeneity of constraints_inhomogeneous
                                    // (values on constrained dofs), or null = all zero
  int       device     = 0;
  gls::VecStage stage; // caller vector layout (host memory / dof permutation)
  gls::OutflowFaces faces; // weak outflow boundary faces (faces.hip)
  // gls_gmres_solve workspace (Krylov basis and vectors), grown on demand
  void     *gmres_ws       = nullptr;
  size_t    gmres_ws_bytes = 0;
  // pinned host staging of the per-iteration Hessenberg column (two buffers)
  double   *gmres_host       = nullptr;
  size_t    gmres_host_count = 0;

  // brick decomposition (csrc/brick.h)
  bool      use_brick = false;
  int       bx = 1, by = 1, bz = 1, L = 0, Lx = 0, Ly = 0;
  int64_t   n_bricks = 0, n_slots = 0, n_shared = 0;
  int64_t   n_interior_bricks = 0; // leading work units that read no ghost node
  uint32_t *d_brick_nodes  = nullptr;
  uint32_t *d_brick_target = nullptr;
  uint32_t *d_shared_nodes = nullptr;
  uint32_t *d_shared_off   = nullptr;
  int32_t  *d_shared_index = nullptr; // node -> shared index (-1: exclusive)
  // cells grouped by colour (no two cells of a colour share a node; internal
  // order): the deterministic (GLS_DETERMINISTIC) assembly of the diagonal
  // and of the multigrid restriction, colour by colour without atomics
  // (built on first use, op_cell_colours)
  int32_t             *d_colour_cells = nullptr;
  std::vector<int64_t> colour_off;
  gls::ReduceClasses reduce_classes{}; // multiplicity classes of the shared nodes
  // the shared nodes are ordered [owned | ghost]: the first n_shared_owned
  // are owned rows; classes of each part on its own (first[] relative to the
  // part's first node, slot0 absolute), so the ghost rows of a partitioned
  // vmult are reduced (and exported) before the rest of the cell loop
  int64_t            n_shared_owned = 0;
  gls::ReduceClasses reduce_owned{}, reduce_ghost{};
  void     *d_partial      = nullptr;
  void     *d_bgeo_cart    = nullptr; // brick path: cell-indexed geometry
  void     *d_bgeo_gen     = nullptr;
  uint32_t *d_brick_geo    = nullptr; // per brick: curved (bit 0) | cells << 8
  uint32_t *d_brick_cell0  = nullptr; // per brick: first cell
  uint32_t *d_brick_chunk0 = nullptr; // per brick: first table chunk
  // bricks with per-q geometry (any curved cell): none -> the launches run
  // k_brick<GEO_CART>, all -> <GEO_GEN>, some -> <GEO_ANY>
  int64_t   n_curved_bricks = 0;

  // per-q table layout (kernels.h tab_index): 16-byte field groups, one
  // chunk per wavefront round of the brick kernel
  std::vector<int64_t> h_tab_cbase; // [n_cells]
  int64_t  *d_tab_cbase = nullptr;
  int64_t   tab_gs = 0, tab_elems = 0;
  std::vector<uint32_t> brick_cell0, brick_ncell;
  // resident smoothing sweeps (brick.h k_brick_sweeps; FP32 3D operators with
  // few bricks): two tagged-granule slot buffers ([slot][4] {value, tag}),
  // the waits that hit the spin bound, the last tag used (tags grow across
  // launches; launches on one operator are stream-ordered) and the resident
  // capacity per instantiation [Newton][geometry][deterministic] (-1: not
  // asked yet)
  uint64_t        *d_sweep_gran[2] = {nullptr, nullptr};
  uint32_t        *d_sweep_err     = nullptr;
  // stall flag in host-mapped memory (set by a wait that hit the spin bound)
  // and its device address; after a stall the operator runs one launch per
  // step for the rest of its life (sweep_off) and the stall is reported once
  // through the next multigrid / GMRES status (sweep_stalled)
  uint32_t        *h_sweep_flag    = nullptr;
  uint32_t        *d_sweep_flag    = nullptr;
  mutable bool     sweep_off       = false;
  mutable bool     sweep_reported  = false;
  int              sweep_spin_max  = gls::SWEEP_SPIN_MAX_DEFAULT;
  mutable uint32_t sweep_epoch     = 0;
  mutable uint64_t sweep_launches  = 0;
  mutable int64_t  sweep_cap[2][3][2] = {{{-1, -1}, {-1, -1}, {-1, -1}}, {{-1, -1}, {-1, -1}, {-1, -1}}};

  size_t
  tsize() const
  {
    return prec == GLS_F64 ? 8 : 4;
  }
};

namespace gls
{
// brick discovery for an arbitrary cell order (brick_discovery.cc)
struct BrickPlan
{
  int                  shape[3] = {0, 0, 0};
  std::vector<int64_t> perm; // internal (brick-ordered) cell -> caller cell
};
bool discover_bricks(int dim, int degree, int64_t n_cells, const uint32_t *cell_nodes,
                     BrickPlan &plan);

// caller cell of internal cell c
inline int64_t
ext_cell(const glsOp_ *op, int64_t c)
{
  return op->cell_perm.empty() ? c : op->cell_perm[(size_t)c];
}

// the operator's cells by colour (greedy over the internal order; cells of a
// colour share no node): device list op->d_colour_cells, colour k at
// [colour_off[k], colour_off[k+1])
void op_cell_colours(glsOp_ *op);

inline bool
op_deterministic(const glsOp_ *op)
{
  return (op->prm.flags & GLS_DETERMINISTIC) != 0;
}

// fused damped-Jacobi step of the multigrid smoother (csrc/mg.hip): with it a
// brick vmult writes x + omega * d . (b - A x) instead of A x.  Passed per
// launch, never stored on the handle (a concurrent plain vmult on the same
// level operator stays a plain vmult).
struct RelaxStep
{
  const void *b     = nullptr;
  const void *d     = nullptr; // null: 1
  double      omega = 0.0;
  bool        keep  = true;    // false: omega d (b - A x) (with d null, omega 1: the
                               // multigrid residual b - A x)
  // deferred shared-node reduction (FP32 3D brick levels, mg.hip smooth):
  // partial: this apply's slot buffer (null: the operator's); prev_partial:
  // the previous apply's slots, whose reduction this apply's gather rebuilds
  // from prev_src (the iterate before src) with the previous step's b, d,
  // omega and writes into src; defer: skip this apply's own reduction
  void       *partial      = nullptr;
  const void *prev_partial = nullptr;
  const void *prev_src     = nullptr;
  const void *prev_b       = nullptr;
  const void *prev_d       = nullptr;
  double      prev_omega   = 0.0;
  bool        defer        = false;
  // the result also converted to FP64 here (the V-cycle's copy_from_mg fused
  // into its last apply; brick write-out and class reduce, FP32 levels)
  double     *out64        = nullptr;
};

// a brick operator whose smoother can defer its shared-node reductions
// (the gather rebuilds them: one 16-byte pack per node, FP32 3D)
inline bool
deferred_reduce_ok(const glsOp_ *op)
{
  return op->use_brick && op->n_owned_dofs == op->n_dofs && op->faces.n == 0 &&
         op->prec == GLS_F32 && op->dim == 3 && op->reduce_classes.n > 0;
}

// the pieces of vmult that dist.hip / mg.hip orchestrate (gls_op.hip):
// brick kernel over work units [b0, b1) (what & BRICK_RUN) and the
// shared-node reduction (what & BRICK_REDUCE)
void brick_launch(const glsOp_ *op, int mode, void *dst, const void *src, int64_t b0,
                  int64_t b1, int what, hipStream_t s, const RelaxStep *rx = nullptr);
int  op_vmult_mode(const glsOp_ *op);
// nsweep >= 2 fused damped-Jacobi steps (rx: b, d, omega, keep, out64 for the
// last) in one resident launch (k_brick_sweeps): sweep j reads v[j % 2] and
// writes v[(j + 1) % 2], its partial slots slots[j % 2]; the last sweep's
// reduction is left pending (its slots, its src) as after a deferred
// per-launch sequence.  False (nothing launched) where the operator or the
// device does not qualify: the caller launches the steps one by one.
// a resident sweep of op stalled (its stall flag is set) and this was not
// reported yet: marks it reported and turns the resident sweeps off for op
bool sweep_stalled(const glsOp_ *op);
bool brick_sweeps(const glsOp_ *op, int mode, void *v0, void *v1, void *slots0, void *slots1,
                  int nsweep, const RelaxStep &rx, hipStream_t s);
// one V-cycle on node-major device vectors of the multigrid's outer
// precision (gls_mg_vcycle without the caller-layout staging; GMRES calls it)
void mg_vcycle_device(glsMG mg, void *dst, const void *src, hipStream_t s);
// throws unless mg can precondition op's FP64 Krylov vectors in place: outer
// precision FP64, finest level of op's size, gls_mg_setup done
void mg_check_outer(glsMG mg, const glsOp_ *op);
// true when one V-cycle is a linear map of its input (no coarse solve
// iterated to a tolerance): GMRES may then keep M^{-1} v_j (krylov.hip)
bool mg_is_linear(glsMG mg);
// throws (once) when a level's resident smoothing sweeps stalled
void mg_check_stall(glsMG mg, const char *who);
// outflow boundary-face terms (faces.hip), launched after the cell kernels
void faces_setup(glsOp_ *op, const glsOpDesc *d);
void faces_release(glsOp_ *op);
void faces_linearization(const glsOp_ *op, const void *lin, hipStream_t s);
void faces_apply(const glsOp_ *op, bool residual, void *dst, const void *src, hipStream_t s);
void faces_diagonal(const glsOp_ *op, void *diag, bool f64_out, hipStream_t s);
void faces_element_matrices(const glsOp_ *op, void *emat, int64_t b, int64_t e, hipStream_t s);
// the brick vmult with the smoother step fused into its write-out needs the
// whole A x inside the kernel: single domain, no face terms
inline bool
fused_relax_ok(const glsOp_ *op)
{
  return op->use_brick && op->n_owned_dofs == op->n_dofs && op->faces.n == 0;
}

// team primitives of the partitioned multigrid / GMRES (dist.hip): the ranks
// one process drives in lockstep — one RCCL rank, or all members of an
// in-process group (rank order)
glsOp_ *dist_op(glsDist d);
// a member of an in-process group (several partitions on one device)
bool    dist_in_process(glsDist d);
int     dist_rank(glsDist d);
int     dist_world(glsDist d);
// rx: per member, the damped-Jacobi step / residual fused on the owned rows
void    team_vmult(glsDist const *m, void *const *dst, void *const *src, int n, hipStream_t s,
                   const RelaxStep *rx = nullptr);
void    team_update_ghosts(glsDist const *m, void *const *v, int n, hipStream_t s);
void    team_compress_add(glsDist const *m, void *const *v, int n, hipStream_t s);
// buf[r][0 .. count) <- the sum over the team's ranks (ncclAllReduce / member order)
void    team_allreduce_sum(glsDist const *m, double *const *buf, int64_t count, int n,
                           hipStream_t s);

// the same operator pieces without staging (GMRES, multigrid)
void op_vmult_device(glsOp op, void *dst, const void *src, hipStream_t s);
void op_inverse_diagonal_device(glsOp op, void *diag, hipStream_t s);
// element matrices of internal cells [b, e) into emat (device, the operator's
// precision, [cell][col j][row i], local dof = point * (dim+1) + component),
// outflow faces included (MatrixFreeTools::compute_matrix's cell + boundary
// lambdas, operator_ns.cc:1407-1430)
void op_element_matrices_device(const glsOp_ *op, void *emat, int64_t b, int64_t e,
                                hipStream_t s);
} // namespace gls
