/*
 * gls_op.h — C-ABI of the MI355X (gfx950) matrix-free GLS Navier–Stokes
 * operator and its geometric-multigrid pieces (libglsamd.so).
 *
 * This is the drop-in boundary for the reference's hot path.  Each entry
 * point replaces one member of the reference's operator / preconditioner
 * interface (peterrum/dealii-ns-gls @ 2025-05-23):
 *
 *   gls_op_create                    NavierStokesOperator ctor
 *                                      include/operator_ns.h:24-41, .cc:68-153
 *                                      (+ MatrixFree::reinit of the cell
 *                                      geometry, .cc:110-121)
 *   gls_op_set_parameters            the scalars the ctor / TimeIntegratorData
 *                                      feed the kernel (nu, c1, c2, theta,
 *                                      primary weight, dt, order, flags)
 *                                      operator_ns.h:102-114,
 *                                      time_integration.h:10-36
 *   gls_op_set_linearization_point   OperatorBase::set_linearization_point
 *                                      operator_base.h:35-36, operator_ns.cc:570-620
 *                                      (+ compute_penalty_parameters :322-421)
 *   gls_op_set_previous_solution     OperatorBase::set_previous_solution
 *                                      operator_base.h:32-33, operator_ns.cc:234-320
 *   gls_op_vmult                     OperatorBase::vmult
 *                                      operator_base.h:45-46, operator_ns.cc:684-732
 *   gls_op_vmult_interface_down /
 *   gls_op_vmult_interface_up        OperatorBase::vmult_interface_down / _up
 *                                      operator_base.h:51-58, operator_ns.cc:734-787
 *                                      (local-smoothing interface matrices;
 *                                      globally refined levels: down = vmult,
 *                                      up = 0)
 *   gls_op_vmult_init /
 *   gls_op_vmult_cells /
 *   gls_op_apply_identity_rows       the pieces of vmult around the ghost
 *                                      exchange (deal.II cell_loop with
 *                                      update_ghost_values / compress(add),
 *                                      .cc:702-721) for multi-GPU
 *   gls_op_evaluate_residual         OperatorBase::evaluate_residual
 *                                      operator_base.h:41-43, operator_ns.cc:648-682
 *   gls_op_evaluate_rhs              OperatorBase::evaluate_rhs
 *                                      operator_base.h:38-39, operator_ns.cc:622-646
 *   gls_op_set_constraint_values     the constraints_inhomogeneous the
 *                                      operator holds by reference
 *                                      (operator_ns.h:95, main.cc:879-891)
 *   gls_op_compute_inverse_diagonal  OperatorBase::compute_inverse_diagonal
 *                                      operator_base.h:26-27, operator_ns.cc:195-225
 *   gls_op_m                         OperatorBase::m  operator_base.h:20-21
 *   gls_op_upload_tables /
 *   gls_op_download_tables           host-produced / inspected per-q tables
 *                                      (u_star_value ... operator_ns.h:120-132)
 *   gls_gmres_solve                  LinearSolverGMRES::solve
 *                                      solver_l.cc:45-74 (device-resident)
 *   gls_mg_*                         PreconditionerGMG (multigrid.h:61-141):
 *                                      relaxation smoother (multigrid.cc:281-351),
 *                                      MGTwoLevelTransfer (main.cc:538-563),
 *                                      V-cycle apply (multigrid.cc:202-220)
 *   gls_timer_*                      MyTimerOutput / MyScope sections and
 *                                      TimerOutput wall-time statistics
 *                                      (timer.h:194-338, 342-413): the
 *                                      reference's section names as roctx
 *                                      ranges, optional per-section tally
 *
 * Conventions
 *   - Vectors are DEVICE pointers in the operator's precision (double for
 *     GLS_F64, float for GLS_F32), local layout [owned | ghost] with
 *     dof = node * (dim + 1) + component (component dim = pressure).
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  Calls are
 *     stream-ordered and not thread safe per handle (as the reference: one
 *     host thread per rank, mutable state, operator_ns.h:181-188).
 *   - Every function returns 0 on success; nonzero status = error, with a
 *     thread-local message from gls_last_error() (the C++ facade turns it
 *     into an exception, mirroring AssertThrow).
 */
#ifndef GLS_OP_H
#define GLS_OP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct glsOp_ *glsOp;
typedef struct glsMG_ *glsMG;
typedef struct glsAMG_ *glsAMG;
typedef int            glsStatus;

enum glsPrecision
{
  GLS_F64 = 0,
  GLS_F32 = 1
};

enum glsMemory
{
  GLS_MEM_DEVICE = 0, /* vectors are device pointers (default)             */
  GLS_MEM_HOST   = 1  /* vectors are host pointers, staged over PCIe       */
};

enum glsFlags
{
  GLS_INCREMENT_FORM           = 1, /* Newton: increment_form, main.cc:331    */
  GLS_CONSIDER_TIME_DERIVATIVE = 2, /* consider_time_derivative (ctor arg)    */
  GLS_CELL_WISE_STAB           = 4, /* cell_wise_stabilization (ctor arg)     */
  /* not a reference parameter: results bitwise reproducible run to run (the
   * brick kernels add a round's cells into the LDS lattice in cell order
   * instead of by LDS atomics; the diagonal and the multigrid restriction
   * assemble cell colour by colour instead of by global atomics), at some
   * cost in speed; debugging, SURVEY §7.2.2 */
  GLS_DETERMINISTIC            = 8
};

typedef struct
{
  int             dim;        /* 2 or 3                                       */
  int             degree;     /* Q_k, k in {1,2,3}                            */
  int             precision;  /* glsPrecision                                 */
  int64_t         n_cells;    /* locally processed cells                      */
  int64_t         n_nodes;    /* local nodes [owned | ghost]                  */
  int64_t         n_owned_nodes; /* owned prefix; identity rows only there    */
  const uint32_t *cell_nodes; /* host [n_cells][(k+1)^dim] lexicographic      */
  const double   *node_coords;/* host [n_nodes][dim] MappingQ_k support pts   */
  const uint8_t  *node_cmask; /* host [n_nodes] constrained component bits    */
  const double   *cell_measure;     /* host [n_cells] vertex measure |K|      */
  const double   *cell_hmin;        /* host [n_cells] min vertex distance     */
  int             brick[3];   /* structure hint: the cell list is a sequence
                                 of bricks of brick[0]*brick[1]*brick[2]
                                 cells, lexicographic inside a brick, sharing
                                 nodes like a structured block (as produced by
                                 gls_mesh_brick).  {-1,-1,-1}: any cell order
                                 (deal.II's MatrixFree order) — the bricks are
                                 discovered from the connectivity and the
                                 cells run in brick order internally
                                 (gls_op_cell_permutation).  {0,0,0}: no
                                 structure, per-cell kernel.                */
  /* weak outflow boundaries (constructor arguments all_outflow_bcs_cut /
   * all_outflow_bcs_nitsche, operator_ns.cc:79-95; needs_face_integrals):
   * the boundary faces on them, as (caller cell, face number 2*axis + side,
   * deal.II's face numbering of a hex / quad) with their kind
   * (glsOutflow).  0 faces: cell integrals only (cell_loop).  Single-domain
   * operators only (n_owned_nodes == n_nodes).                             */
  int64_t         n_outflow_faces;
  const int64_t  *outflow_cells;   /* host [n_outflow_faces]                 */
  const int32_t  *outflow_face_no; /* host [n_outflow_faces] 0 .. 2*dim-1    */
  const int32_t  *outflow_kind;    /* host [n_outflow_faces] glsOutflow      */
  /* optional cell mapping of its own degree (the level's
   * MappingQ(mapping_degree), main.cc:413-414, which maps the FE_Q_iso_Q1
   * coarse level too, where the element is Q1 on sub-cells, :437-446):
   * per cell the (m+1)^dim support points of its MappingQ_m, lexicographic
   * on the Gauss-Lobatto lattice.  NULL (zero-initialised descriptor): the
   * element's own support points node_coords.  Cell integrals only (no
   * outflow faces with it).                                                 */
  int             mapping_degree;  /* m, 1..3                                */
  const double   *mapping_points;  /* host [n_cells][(m+1)^dim][dim] or NULL */
} glsOpDesc;

enum glsOutflow
{
  GLS_OUTFLOW_CUT     = 1, /* beta min(0, u*.n) u on the face, :1201-1240    */
  GLS_OUTFLOW_NITSCHE = 2  /* Nitsche with target g, :1241-1287              */
};

typedef struct
{
  double nu, c1, c2;
  double theta;  /* TimeIntegratorData::get_theta()                          */
  double w0;     /* get_primary_weight()                                      */
  double dt;     /* get_current_dt()  (stau = dt == 0 ? 0 : 1/dt)             */
  int    order;  /* get_order()                                               */
  int    flags;  /* glsFlags                                                  */
} glsOpParams;

glsStatus gls_op_create(const glsOpDesc *desc, glsOp *out);
/* The brick shape the operator runs ({0,0,0}: per-cell kernel) and its
 * internal cell order: perm[internal cell] = caller cell, n_cells entries.
 * Only gls_op_vmult_cells ranges refer to the internal order; table
 * upload/download and every vector use the caller's numbering. */
glsStatus gls_op_brick_shape(glsOp op, int *dims);
/* Diagnostics of the multigrid's resident smoothing sweeps on this level
 * operator since its creation: *launches = smoothing
 * sequences run as one resident launch, *timeouts = slot waits that hit
 * their spin bound (0 on a healthy device; synchronises the device). */
glsStatus gls_op_sweep_stats(glsOp op, uint64_t *launches, uint64_t *timeouts);
/* Polls of a neighbour's partial-slot granule before a resident sweep's wait
 * gives up (default 2^18).  A wait that gives up poisons the brick's iterate
 * with NaN and raises the operator's stall flag; from then on the level runs
 * one launch per smoothing step, and the next gls_mg_vcycle or
 * gls_gmres_solve on the multigrid returns an error status once (the
 * co-residency precondition of INTEGRATION.md §5).  Test hook: 0 makes every
 * wait that is not satisfied at its first poll give up. */
glsStatus gls_op_set_sweep_spin_bound(glsOp op, int64_t polls);
/* The discovery gls_op_create runs for brick = {-1,-1,-1}, on its own (host
 * only, no device call): shape = the brick shape found ({0,0,0}: none),
 * perm[internal cell] = caller cell. */
glsStatus gls_discover_bricks(int dim, int degree, int64_t n_cells, const uint32_t *cell_nodes,
                              int *shape, int64_t *perm);
glsStatus gls_op_cell_permutation(glsOp op, int64_t *perm);
void      gls_op_destroy(glsOp op);
glsStatus gls_op_set_parameters(glsOp op, const glsOpParams *prm);
int64_t   gls_op_m(glsOp op); /* number of local dofs */
int       gls_op_precision(glsOp op);

/* Caller-side vector layout of every vector argument of the gls_op_* calls
 * below that take whole dof vectors (set_linearization_point,
 * set_previous_solution, vmult, evaluate_residual(_plain), evaluate_rhs,
 * set_constraint_values, compute_inverse_diagonal, get_max_u, and x / b of
 * gls_gmres_solve):
 *   memory   GLS_MEM_DEVICE (default) or GLS_MEM_HOST: host pointers, as the
 *            reference's LinearAlgebra::distributed::Vector<Number> in host
 *            memory (config.h:9-10); staged through device buffers, the
 *            call returns synchronised;
 *   dof_map  NULL (node-major: dof = node * (dim+1) + component) or a host
 *            array [gls_op_m] with dof_map[i] = the node-major dof of the
 *            caller's local dof i (deal.II DoFHandler numbering); a
 *            permutation, copied.
 * The multi-GPU pieces (vmult_cells / vmult_init / apply_identity_rows,
 * gls_dist_*) always take node-major device vectors. */
glsStatus gls_op_set_vector_layout(glsOp op, int memory, const int64_t *dof_map);

glsStatus gls_op_set_linearization_point(glsOp op, const void *vec, void *stream);
/* vec_old = sum_{i=1..order} weights[i] * history[i]  (history[0] unused) */
glsStatus gls_op_set_previous_solution(glsOp op, const void *const *history,
                                       int n_history, const double *weights,
                                       void *stream);

glsStatus gls_op_vmult(glsOp op, void *dst, const void *src, void *stream);
/* the local-smoothing interface matrices of OperatorBase (operator_ns.cc:
 * 734-787).  Their edge-constrained dofs (operator_ns.cc:131-152) sit on the
 * refinement edges of a locally refined level; the meshes this library takes
 * are whole levels of a globally refined hierarchy, where that set is empty:
 * interface_down is then the vmult (cell loop, dst = src on the constrained
 * dofs) and interface_up sets dst = 0 -- what the reference computes on such
 * a mesh.  Same vector layout and errors as gls_op_vmult. */
glsStatus gls_op_vmult_interface_down(glsOp op, void *dst, const void *src, void *stream);
glsStatus gls_op_vmult_interface_up(glsOp op, void *dst, const void *src, void *stream);
/* cells [cell_begin, cell_end): dst += cell contributions (no zeroing) */
glsStatus gls_op_vmult_cells(glsOp op, void *dst, const void *src,
                             int64_t cell_begin, int64_t cell_end,
                             void *stream);
/* dst[i] = constrained(i) ? src[i] : 0 on the owned dofs, 0 on ghosts */
glsStatus gls_op_vmult_init(glsOp op, void *dst, const void *src, void *stream);
/* dst[i] = src[i] on constrained owned dofs, others untouched: the identity
 * rows of vmult (operator_ns.cc:719-721) re-applied after the ghost
 * export-add (compress(add)) of a distributed vmult */
glsStatus gls_op_apply_identity_rows(glsOp op, void *dst, const void *src, void *stream);

/* evaluate_residual (operator_ns.cc:648-682): tmp = src;
 * constraints_inhomogeneous.distribute(tmp) (constrained components take the
 * values set by gls_op_set_constraint_values, zero if none are set); cell
 * loop with the residual kernel on tmp; set_zero on constrained rows;
 * dst *= -1. */
glsStatus gls_op_evaluate_residual(glsOp op, void *dst, const void *src,
                                   void *stream);
/* the same without the distribute step: constrained components of src are
 * read as they are (read_dof_values_plain on an already distributed vector,
 * which is what the Newton loop passes, main.cc:893) */
glsStatus gls_op_evaluate_residual_plain(glsOp op, void *dst, const void *src,
                                         void *stream);
/* evaluate_rhs (operator_ns.cc:622-646): the residual of the zero vector
 * with the inhomogeneous constraints distributed */
glsStatus gls_op_evaluate_rhs(glsOp op, void *dst, void *stream);
/* the inhomogeneity of constraints_inhomogeneous (main.cc:879-891,
 * 926-942: VectorTools::interpolate_boundary_values of the inflow function
 * on top of constraints_copy): a vector of the operator's size and
 * precision (host or device pointer) whose constrained components hold
 * the Dirichlet values; other components are ignored.  NULL clears it
 * (all constrained values zero).  Copied; call again when the time-dependent
 * boundary values change (every time step in the reference). */
glsStatus gls_op_set_constraint_values(glsOp op, const void *values, void *stream);
glsStatus gls_op_compute_inverse_diagonal(glsOp op, void *inv_diag,
                                          void *stream);
/* OperatorBase::get_max_u (operator_base.h:71-72; NavierStokesOperator
 * operator_ns.cc:530-568): max over the locally processed cells and their
 * quadrature points of |u(x_q)| of the velocity of `vec` (read plain, no
 * constraints), into *u_max (host).  Called every time step for the CFL dt
 * (main.cc:913-920).  Partitioned operators: gls_dist_get_max_u adds the
 * MPI max. */
glsStatus gls_op_get_max_u(glsOp op, const void *vec, double *u_max, void *stream);
/* the pieces of compute_inverse_diagonal for a partitioned operator: the
 * rank-local assembled diagonal (constrained owned components 1), then —
 * after the caller's compress(add) of the ghost partials (gls_dist_compress_
 * add) — d <- |d| > 1e-10 ? 1/d : 1 (operator_ns.cc:220-224) */
glsStatus gls_op_compute_diagonal(glsOp op, void *diag, void *stream);
glsStatus gls_op_invert_diagonal(glsOp op, void *diag, void *stream);

/* canonical host layout [cell][q][field] (fields: delta1, delta2, U(dim),
 * gradU(dim*dim), gradP(dim), Ut_old(dim)) + cellwise [cell][2] */
glsStatus gls_op_upload_tables(glsOp op, const double *tables,
                               const double *cellwise);
glsStatus gls_op_download_tables(glsOp op, double *tables, double *cellwise);

/* number of cells whose geometry is stored per quadrature point (general)
 * and per cell (Cartesian) — MatrixFree-style compressed geometry */
glsStatus gls_op_geometry_counts(glsOp op, int64_t *n_general,
                                 int64_t *n_cartesian);
/* algorithmic bytes of one vmult (SURVEY §8d B_tab) */
double gls_op_vmult_bytes(glsOp op);

/* Outflow faces (glsOpDesc.n_outflow_faces): the count and the face
 * quadrature points per face ((k+1)^(dim-1), QGauss(k+1) on the face, first
 * tangential axis fastest), the points [face][point][dim] in the
 * descriptor's face order; the caller evaluates the Nitsche target there
 * (face_target_velocity, operator_ns.cc:478-521: the boundary function of
 * all_outflow_bcs_nitsche at time t, main.cc:935-939) and hands the
 * velocity [face][point][dim] over, host memory.  Default target: zero. */
glsStatus gls_op_n_outflow_faces(glsOp op, int64_t *n_faces, int *n_face_points);
glsStatus gls_op_outflow_face_points(glsOp op, double *xyz);
glsStatus gls_op_set_outflow_target(glsOp op, const double *target, void *stream);

/* OperatorBase::get_system_matrix (operator_ns.cc:1407-1430,
 * MatrixFreeTools::compute_matrix): the element matrices, from one
 * unit-vector cell apply per (cell, local dof) on the device, FP64 host
 * [cell][col j][row i] with local dof = point * (dim+1) + component, cells in
 * the caller's order (n_cells * ((k+1)^dim (dim+1))^2 entries) ... */
glsStatus gls_op_element_matrices(glsOp op, double *out);
/* ... and assembled into CSR over the node-major dofs (single domain):
 * rows / columns of constrained dofs carry only their unit diagonal, as the
 * identity rows of vmult.  Call with row_ptr = NULL for *nnz first; then
 * row_ptr [n_dofs + 1], cols / vals [nnz] (columns sorted per row). */
glsStatus gls_op_system_matrix(glsOp op, int64_t *nnz, int64_t *row_ptr, int64_t *cols,
                               double *vals);

/* ------------------------------------------------- algebraic multigrid
 * Smoothed-aggregation AMG on an assembled CSR matrix: the substitute for
 * TrilinosWrappers::PreconditionAMG (Trilinos ML) of the coarse solver
 * "AMG" (multigrid.cc:372-433).  Algorithm: csrc/amg.hip, DESIGN.md §7. */
typedef struct
{
  int    block_size;      /* dofs per node ("PDE equations"): dim + 1 with
                             constant modes per component (deal.II's
                             extract_constant_modes, the decks' custom
                             parameters), 1 with the default parameters   */
  double threshold;       /* aggregation_threshold (1e-4 deal.II default)   */
  int    smoother_sweeps; /* smoother_sweeps: Chebyshev degree (2)           */
  int    coarse_max_size; /* "coarse: max size": dense direct solve below
                             (2000, deal.II's ML parameter)                */
  int    elliptic;        /* 1: smoothed prolongator (omega 4/3 / lambda);
                             0: tentative prolongator (non-elliptic)       */
  int    max_levels;      /* ML "max levels" (10)                            */
  double chebyshev_alpha; /* ML "smoother: Chebyshev alpha": the smoother
                             damps [lambda_max / alpha, lambda_max]; deal.II's
                             PreconditionAMG sets 10 (ML's own default 30);
                             <= 0: 10                                       */
} glsAMGParams;
/* PreconditionAMG::initialize(matrix, data): n x n CSR (host, int64
 * row_ptr[n + 1], cols / vals [nnz]); setup on the host, the hierarchy and
 * the V-cycle on the current device */
glsStatus gls_amg_create(int64_t n, const int64_t *row_ptr, const int64_t *cols,
                         const double *vals, const glsAMGParams *prm, glsAMG *out);
void      gls_amg_destroy(glsAMG amg);
/* PreconditionAMG::vmult: dst = one V-cycle on src (device FP64 vectors) */
glsStatus gls_amg_vmult(glsAMG amg, double *dst, const double *src, void *stream);
/* levels, per level its size, nonzeros and the D^-1 A spectral-radius
 * estimate (arrays of at least n_levels entries, or NULL) */
glsStatus gls_amg_info(glsAMG amg, int *n_levels, int64_t *sizes, int64_t *nnz,
                       double *lambda);
/* the device hierarchy of level `level` as built (which: 0 A, 1 P, 2 R;
 * none on the coarsest for P / R): rows, nonzeros, and with non-NULL
 * arrays the CSR (int32 row_ptr [rows + 1], cols / vals [nnz]) */
glsStatus gls_amg_level_matrix(glsAMG amg, int level, int which, int64_t *n_rows, int64_t *nnz,
                               int32_t *row_ptr, int32_t *cols, double *vals);

/* ------------------------------------------------------------ multigrid */
typedef struct
{
  int    n_levels;             /* levels 0 (coarse) .. n_levels-1 (fine)     */
  int    smoothing_n_iterations;       /* 5   multigrid.h:31                 */
  int    smoothing_eig_n_iterations;   /* 20  multigrid.h:32                 */
  double smoothing_range;              /* 20  multigrid.h:30                 */
  int    coarse_n_iterations;  /* coarse solver: relaxation sweeps (0 =
                                  identity); see DESIGN.md                   */
  int    outer_precision;      /* precision of the vectors gls_mg_vcycle
                                  takes (GLS_F64: copy_to_mg / copy_from_mg
                                  convert to the level precision, as
                                  PreconditionMG does for MGNumber = float)  */
  int    compute_evs_n_levels; /* "gmg compute evs n levels" (multigrid.cc:
                                  307, 355-358): > 0 also estimates the
                                  relaxation factor on the coarsest level    */
  int    coarse_iterate;       /* "gmg coarse grid iterate" (multigrid.cc:
                                  491-530): 1 = GMRES on the coarse level
                                  (FP64 vectors, left preconditioning, 30
                                  temporary vectors, deal.II SolverGMRES
                                  defaults) preconditioned by the coarse
                                  solver above; 0 = apply it once            */
  double coarse_reltol;        /* 1e-4  multigrid.h:41 (ReductionControl)    */
  int    coarse_maxiter;       /* 10000 multigrid.h:39                       */
  /* "gmg coarse grid solver": "AMG" (multigrid.cc:372-433): 1 = the coarse
   * preconditioner is one V-cycle of a smoothed-aggregation AMG built by
   * gls_mg_setup on the coarse level's assembled system matrix
   * (gls_op_system_matrix, as op[min_level]->get_system_matrix()), applied
   * to the FP64 coarse GMRES vectors (coarse_iterate = 1 needed);
   * coarse_n_iterations is then ignored.  0 = as above.                     */
  int    coarse_amg;
  glsAMGParams amg;            /* its parameters (gls_amg_create)            */
} glsMGDesc;

/* levels[l] are level operators (same precision); child[l] for l >= 1 is the
 * host child lattice of level l-1 cells into level l nodes
 * (gls_mesh_child_lattice), n_cells(l-1) * (2k+1)^dim entries. */
glsStatus gls_mg_create(const glsMGDesc *desc, const glsOp *levels,
                        const uint32_t *const *child, glsMG *out);
void      gls_mg_destroy(glsMG mg);
/* PreconditionerGMG::initialize (multigrid.cc:247-370): inverse diagonals
 * and power-iteration relaxation factors on every level */
glsStatus gls_mg_setup(glsMG mg, void *stream);
glsStatus gls_mg_get_relaxation(glsMG mg, int level, double *omega,
                                double *lambda_max);
/* GMRES iterations of the last coarse solve (coarse_iterate = 1), and
 * whether it reached the tolerance */
glsStatus gls_mg_coarse_statistics(glsMG mg, int *n_iterations, int *converged);
/* the AMG of the coarse solver (desc.coarse_amg; NULL before gls_mg_setup)
 * and the wall ms of its last setup (system matrix + hierarchy) */
glsStatus gls_mg_coarse_amg(glsMG mg, glsAMG *amg, double *setup_ms);
/* the last dense-coarse setup (coarse_n_iterations < 0): wall ms of the
 * free-block assembly (element matrices of the coarse level, the cells'
 * interior dofs statically condensed, scattered per cell colour), of getrf
 * and of the inverse (trtri + trsm), and the number of cell colours */
glsStatus gls_mg_coarse_setup_times(glsMG mg, double *ms3, int *n_colors);
/* one V-cycle on the finest level: dst = V(src) (PreconditionMG::vmult) */
glsStatus gls_mg_vcycle(glsMG mg, void *dst, const void *src, void *stream);
/* caller vector layout of gls_mg_vcycle's dst / src (as gls_op_set_vector_
 * layout; n = the finest level's dofs) */
glsStatus gls_mg_set_vector_layout(glsMG mg, int memory, const int64_t *dof_map);
/* transfer on level pair (l-1, l): prolongate_and_add / restrict_and_add */
glsStatus gls_mg_prolongate_add(glsMG mg, int level, void *dst_fine,
                                const void *src_coarse, void *stream);
glsStatus gls_mg_restrict_add(glsMG mg, int level, void *dst_coarse,
                              const void *src_fine, void *stream);
/* interpolate_to_mg: nodal injection level l -> l-1 */
glsStatus gls_mg_interpolate(glsMG mg, int level, void *dst_coarse,
                             const void *src_fine, void *stream);
/* PreconditionRelaxation::vmult (zero start) / step on one level */
glsStatus gls_mg_smooth(glsMG mg, int level, void *x, const void *b,
                        int zero_initial_guess, void *stream);
/* one damped-Jacobi update on level `level`'s vectors (the host-driven
 * distributed smoother, glsdist.py): zero_start: x = omega d b, else
 * x += omega d (b - ax), ax = A x from a partitioned vmult */
glsStatus gls_mg_relax(glsMG mg, int level, void *x, const void *b, const void *ax,
                       const void *inv_diag, double omega, int zero_start, void *stream);

/* ---- partitioned operator: one rank per GPU, ghost exchange over RCCL
 * (deal.II update_ghost_values / compress(add) inside
 * MatrixFree::cell_loop, operator_ns.cc:702-721).  The local operator is a
 * glsOp built on the rank-local mesh with n_owned_nodes < n_nodes, ghosts
 * grouped by owner ([owned | ghosts of owner q0 | ghosts of q1 | ...]). */
typedef struct glsDist_ *glsDist;
typedef struct
{
  int             rank, world;
  const void     *nccl_id;    /* 128-byte ncclUniqueId shared by all ranks
                                 (gls_dist_unique_id on one rank); NULL: an
                                 in-process group on one device (tests)      */
  glsDist         group;      /* in-process group: any member created before,
                                 NULL for the first                          */
  int             n_peers;
  const int      *peers;      /* [n_peers] peer ranks                        */
  const int64_t  *send_count; /* [n_peers] owned nodes that are ghosts on the
                                 peer                                        */
  const uint32_t *send_nodes; /* concatenated, per peer in the peer's ghost
                                 order (local node ids)                      */
  const int64_t  *recv_begin; /* [n_peers] first local node of the ghost
                                 block the peer owns                         */
  const int64_t  *recv_count; /* [n_peers] its length                        */
} glsDistDesc;

glsStatus gls_dist_unique_id(void *id_out /* 128 bytes */);
glsStatus gls_dist_create(glsOp op, const glsDistDesc *desc, glsDist *out);
void      gls_dist_destroy(glsDist d);
/* vmult of the partitioned operator on the rank-local [owned | ghost]
 * vectors: src's ghost block is overwritten by the import (as deal.II's
 * update_ghost_values), dst's ghost block is zero on return (compress).
 * An RCCL rank, or a member of an in-process group driven from its own host
 * thread (every member then makes the same sequence of rank calls, each on
 * its own stream; tests).  An in-process member waits for its peers at host
 * barriers: it fails after GLS_DIST_BARRIER_TIMEOUT seconds (default 120),
 * or after 10 s when every missing member was last driven by the waiting
 * thread itself (members driven one after another from one thread), and the
 * group is then broken for good. */
glsStatus gls_dist_vmult(glsDist d, void *dst, void *src, void *stream);
/* the same for all members of an in-process group, phases in lockstep */
glsStatus gls_dist_vmult_group(glsDist const *members, void *const *dsts,
                               void *const *srcs, int n, void *stream);
glsStatus gls_dist_interior_bricks(glsDist d, int64_t *n_interior,
                                   int64_t *n_total);
/* update_ghost_values of a rank-local [owned | ghost] vector (the import
 * half of gls_dist_vmult); rank calls as gls_dist_vmult */
glsStatus gls_dist_update_ghost_values(glsDist d, void *vec, void *stream);
/* compress(VectorOperation::add): the ghost block's partial sums added to
 * their owners (constrained components skipped), ghost block zeroed (the
 * export half of gls_dist_vmult); rank calls as gls_dist_vmult */
glsStatus gls_dist_compress_add(glsDist d, void *vec, void *stream);
/* get_max_u of the partitioned operator (operator_ns.cc:530-568): ghost
 * import, local max (gls_op_get_max_u), RCCL all-reduce max */
glsStatus gls_dist_get_max_u(glsDist d, void *vec, double *u_max, void *stream);

/* ---- device-resident Krylov solver:
 * LinearSolverGMRES::solve, solver_l.cc:45-74 — deal.II SolverGMRES with
 * max_n_tmp_vectors = 30 (restart after 28 iterations) and right
 * preconditioning; tolerance max(relative * |b|, absolute) (:52-53); x = 0
 * on entry (:66).  `mg` NULL = identity preconditioner (PreconditionIdentity),
 * else one V-cycle per application (PreconditionerGMG::vmult,
 * multigrid.cc:202-220; the MG must be set up with outer_precision F64).
 * op: FP64, single domain.  b and x are device vectors of op's size.
 * No convergence within max_iterations = status 1 (SolverControl::
 * NoConvergence), with *result filled. */
typedef struct
{
  int    max_n_tmp_vectors;  /* 30  solver_l.cc:62                         */
  int    max_iterations;     /* lin n max iterations  main.cc:97 (10000)   */
  double absolute_tolerance; /* lin absolute tolerance main.cc:98 (1e-12)  */
  double relative_tolerance; /* lin relative tolerance main.cc:99 (1e-8)   */
} glsGMRESDesc;
typedef struct
{
  int    n_iterations;       /* SolverControl::last_step()                 */
  int    n_restarts;
  int    converged;
  double initial_residual, final_residual, tolerance;
} glsGMRESResult;
glsStatus gls_gmres_solve(glsOp op, glsMG mg, const glsGMRESDesc *desc, void *x,
                          const void *b, glsGMRESResult *result, void *stream);

/* ---- partitioned multigrid preconditioner and GMRES:
 * PreconditionerGMG::initialize / vmult (multigrid.cc:247-370, 202-220) over
 * partitioned level operators and LinearSolverGMRES::solve (solver_l.cc:
 * 45-74) with all-reduced dots, on rank-local [owned | ghost] device vectors.
 * Every call takes a TEAM: the handles of the ranks this process drives —
 * n = 1 for a rank of an RCCL communicator (the production case, one process
 * per GPU), or all members of an in-process group in rank order (tests).
 * The levels are glsDist handles on the same coarse-cell partition
 * (main.cc:398-400); parameters are set on every level operator (and the
 * coarse operator) with gls_op_set_parameters before the linearization
 * point. */
typedef struct glsDistMG_ *glsDistMG;
typedef struct
{
  glsMGDesc              mg;   /* as gls_mg_create; coarse_iterate must be 0 */
  /* child[l] (l >= 1): the rank-local child lattice of the rank's level l-1
   * cells into level-l local nodes, bit 31 set where the cell is not the
   * GLOBAL first cell touching the node (the owner-only transfers) */
  const uint32_t *const *child;
  const int64_t *const  *owned_global_nodes; /* [n_levels][n_owned_nodes(l)]: global
                                                node ids (power-iteration start
                                                vector on the global dof index) */
  const int64_t         *n_global_nodes;     /* [n_levels] */
  /* coarse_n_iterations < 0 ("direct"): a single-domain operator on the whole
   * level-0 mesh (global node numbering, parameters set), solved redundantly
   * on every rank, and the map of the rank's level-0 local nodes (owned |
   * ghost) to global nodes; NULL otherwise */
  glsOp                  coarse_global;
  const int64_t         *coarse_local_global;
  /* Level agglomeration (deal.II builds every global-coarsening level with its
   * own partition, main.cc:398-400; here the levels below a threshold are
   * gathered whole onto every rank): n_redundant_levels > 0 makes this
   * hierarchy's level 0 the coarsest PARTITIONED level and runs the levels
   * below it, plus a copy of level 0, redundantly and single-domain on every
   * rank.  coarse_global is then the global operator of level 0 (with
   * coarse_local_global as for "direct"), redundant_ops[0 .. n-1] the global
   * operators of the n levels below it (coarsest first) and
   * redundant_child[l] (l = 1 .. n) the child lattice of global level l-1
   * into global level l (level n = coarse_global; entry 0 unused).  The
   * coarse solve of the partitioned V-cycle is one single-domain V-cycle over
   * those n + 1 global levels with mg's smoother and mg's coarse solver on
   * the lowest one: the same cycle as the whole hierarchy, with the small
   * levels' halo exchanges replaced by one all-reduce of level 0's
   * right-hand side (and the resident smoothing sweeps usable there).
   * 0: none (NULL arrays). */
  int                    n_redundant_levels;
  const glsOp           *redundant_ops;
  const uint32_t *const *redundant_child;
} glsDistMGDesc;
glsStatus gls_dist_mg_create(const glsDistMGDesc *desc, const glsDist *levels, glsDistMG *out);
void      gls_dist_mg_destroy(glsDistMG mg);
/* interpolate_to_mg (main.cc:772-803) of the finest level's linearization
 * point and history (level precision, rank-local) down the hierarchy, set on
 * every level operator (and the redundant coarse operator); hist_fine[r] is
 * rank r's SolutionHistory as gls_op_set_previous_solution takes it (n_hist
 * entries, entry 0 unused; n_hist 0: none) */
glsStatus gls_dist_mg_set_linearization_point(glsDistMG const *team, int n,
                                              const void *const *u_fine,
                                              const void *const *const *hist_fine, int n_hist,
                                              const double *weights, void *stream);
/* diagonals (compress(add) + inversion) and power-iteration relaxation
 * factors with all-reduced dots; the redundant coarse LU */
glsStatus gls_dist_mg_setup(glsDistMG const *team, int n, void *stream);
glsStatus gls_dist_mg_get_relaxation(glsDistMG mg, int level, double *omega, double *lambda_max);
/* one V-cycle on the finest level's rank-local vectors (outer precision) */
glsStatus gls_dist_mg_vcycle(glsDistMG const *team, int n, void *const *dst,
                             const void *const *src, void *stream);
/* GMRES on the FP64 partitioned operator A (the finest level's partition),
 * preconditioned by one V-cycle per application (mg NULL: identity);
 * x = 0 on entry; status 1 on no convergence with *result filled */
glsStatus gls_dist_gmres_solve(glsDist const *A, glsDistMG const *mg, int n,
                               const glsGMRESDesc *desc, void *const *x, const void *const *b,
                               glsGMRESResult *result, void *stream);


const char *gls_last_error(void);

/* ---- timer sections (timer.h:194-413 MyTimerOutput / MyScope).  Every
 * entry point and V-cycle phase opens a section named as the reference's
 * (ns::vmult, ns::compute_inverse_diagonal, ns::set_linearization_point,
 * ns::set_previous_solution, ns::evaluate_rhs, ns::evaluate_residual,
 * ns::vmult_interface_down / _up, ns::initialize_system_matrix,
 * gmres::solve, gmg::initialize, gmg::initialize::smoother::init0 / init1,
 * gmg::initialize::direct / amg, gmg::vmult, and per level
 * gmg::vmult::level_<l>::0_pre_smoother_step / 1_residual_step /
 * 2_restriction / 3_prolongation / 5_post_smoother_step, gmg::vmult::level_0
 * for the coarse solve: multigrid.cc:550-583).  A section is always a roctx
 * range (rocprofv3 --marker-trace shows them); with timing on (this call or
 * GLS_TIMING=1 in the environment) it also adds its host wall time and the
 * GPU time between two events on its stream to a process-wide tally.  The
 * events are read when the tally is (no synchronisation inside the timed
 * calls).  Sections nest: a V-cycle's time is also inside gmres::solve. */
glsStatus gls_timer_enable(int on, int *was_on);
/* a section around the caller's own code (MyScope in solver_nl.cc /
 * solver_l.cc: newton::solve, ...): begin returns a token, end closes it;
 * sections close in reverse order of opening (roctx ranges nest) */
glsStatus gls_timer_begin(const char *name, void *stream, void **token);
glsStatus gls_timer_end(void *token);
glsStatus gls_timer_reset(void);
int64_t   gls_timer_n_sections(void);
/* section i: its name (truncated to name_len - 1 characters), calls, host ms
 * and GPU ms summed over the calls (-1 when no call had events) */
glsStatus gls_timer_section(int64_t i, char *name, int64_t name_len, int64_t *calls,
                            double *host_ms, double *gpu_ms);
/* the tally as a text table (print_wall_time_statistics); returns the
 * length needed including the terminating NUL (snprintf semantics) */
int64_t   gls_timer_report(char *buf, int64_t len);

#ifdef __cplusplus
}
#endif

#endif
