/*
 * gls_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C99, optional OpenMP) of the reference's hot path,
 * used as the parity checker for the HIP product path and as the CPU
 * baseline ("kind": "port") in bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library never
 * links or calls it.
 *
 * Restated reference code (peterrum/dealii-ns-gls @ 2025-05-23):
 *   - NavierStokesOperator::do_vmult_cell, both branches
 *       include/operator_ns.cc:949-1182, symm_scalar_product_add :899-916
 *   - do_vmult_range / vmult loop + identity rows        :684-732, :806-830
 *   - set_linearization_point                            :570-620
 *   - compute_penalty_parameters (cell-wise + q-wise)    :322-421
 *   - set_previous_solution                              :234-320
 *   - evaluate_residual                                  :648-682
 *   - compute_inverse_diagonal                           :195-225
 *   - TimeIntegratorDataBDF/Theta/None weights           time_integration.cc:10-178
 *   - the deal.II pieces those call (FEEvaluation sum factorisation on
 *     Q_k GLL-Lagrange / QGauss(k+1), MatrixFreeTools::compute_diagonal,
 *     PreconditionRelaxation, MGTwoLevelTransfer, Multigrid V-cycle) are
 *     restated from their documented semantics (deal.II is not vendored).
 *
 * PARITY STATUS: the reference cannot be built here (deal.II + p4est +
 * Trilinos absent) and ships no golden data, so this oracle is pinned by the
 * known-answer tests KAT-1..6 of SURVEY §8c (tests/test_oracle_kat.py), not
 * by reference outputs: "parity unpinned" w.r.t. the reference binary.
 *
 * Vector layout: dof = node * (dim + 1) + component (component dim = p).
 */
#ifndef GLS_ORACLE_H
#define GLS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct
{
  int             dim, degree;
  int64_t         n_cells, n_nodes;
  const uint32_t *cell_nodes;   /* [n_cells][(k+1)^dim] lexicographic       */
  const double   *coords;       /* [n_nodes][dim] MappingQ_k support points */
  const uint8_t  *cmask;        /* [n_nodes] constrained component bits      */
  const double   *cell_measure; /* [n_cells] vertex-based measure (|K|)     */
  const double   *cell_hmin;    /* [n_cells] minimum vertex distance        */
  /* optional cell mapping of another degree (main.cc:413-414: the level's
   * MappingQ(mapping_degree) on every level, also on the FE_Q_iso_Q1 coarse
   * level where the element is Q1 on sub-cells): per cell the
   * (m+1)^dim support points of its MappingQ_m, lexicographic on the GLL
   * lattice.  NULL: the element's own support points (coords).           */
  int             mapping_degree;
  const double   *mapping_points; /* [n_cells][(m+1)^dim][dim] or NULL     */
} orc_mesh;

typedef struct
{
  double nu, c1, c2;
  double theta;        /* TimeIntegratorData::get_theta()                   */
  double w0;           /* get_primary_weight()                              */
  double dt;           /* get_current_dt(); stau = dt == 0 ? 0 : 1/dt      */
  int    order;        /* get_order(): BDF order, 1 (theta), 0 (none)       */
  int    consider_time_derivative; /* as passed to the constructor           */
  int    increment_form;
  int    cell_wise_stabilization;
} orc_params;

typedef struct orc_op orc_op;

orc_op *orc_create(const orc_mesh *mesh, const orc_params *prm);
void    orc_destroy(orc_op *op);
void    orc_set_threads(int n);

/* operator_ns.cc:570-620 (+ compute_penalty_parameters :322-421) */
void orc_set_linearization_point(orc_op *op, const double *vec);
/* operator_ns.cc:234-320: vec_old = sum_{i=1..order} weights[i] * hist[i] */
void orc_set_previous_solution(orc_op *op, const double *const *hist,
                               int n_hist, const double *weights);
/* operator_ns.cc:684-732 */
void orc_vmult(const orc_op *op, double *dst, const double *src);
/* operator_ns.cc:648-682 (src already carries the inhomogeneous values) */
void orc_evaluate_residual(const orc_op *op, double *dst, const double *src);
/* Outflow boundary faces (all_outflow_bcs_cut / all_outflow_bcs_nitsche,
 * operator_ns.cc:79-95, do_vmult_boundary :1195-1295): face_no = 2 * axis +
 * side of cells[f]; kind per face.  Their terms enter vmult, the residual,
 * the diagonal and orc_cell_matrix (the element matrix of a cell includes its
 * outflow faces).  Call before orc_set_linearization_point.  Returns 0. */
enum { ORC_OUTFLOW_CUT = 1, ORC_OUTFLOW_NITSCHE = 2 };
int  orc_set_outflow_faces(orc_op *op, int64_t n, const int64_t *cells, const int32_t *face_no,
                           const int32_t *kind);
/* [f][qf][dim] face quadrature points (QGauss(k+1)^(dim-1), first tangential
 * axis fastest) ... */
void orc_outflow_face_points(const orc_op *op, double *xyz);
/* ... and the Nitsche target velocity there (face_target_velocity,
 * :478-521), [f][qf][dim] */
void orc_set_outflow_target(orc_op *op, const double *target);
/* operator_ns.cc:195-225 */
void orc_compute_inverse_diagonal(const orc_op *op, double *inv_diag);
void orc_compute_diagonal(const orc_op *op, int64_t n_owned_nodes, double *diag);
/* get_max_u, operator_ns.cc:530-568 */
double orc_get_max_u(const orc_op *op, const double *vec);
/* element matrix of one cell, column j = cell operator applied to unit
 * vector j (what MatrixFreeTools::compute_matrix does), local dof order
 * (node, component) -> node * (dim+1) + c.  mat is [ndof][ndof] row major. */
void orc_cell_matrix(const orc_op *op, int64_t cell, double *mat);

/* Tables in canonical [cell][q][field] layout, fields:
 *   0 delta1_q, 1 delta2_q, 2.. U (dim), grad U (dim*dim, [d][e] = dU_d/dx_e),
 *   grad P* (dim), Ut_old (dim)      -> n = 2 + 3 dim + dim^2
 * plus per cell: delta1, delta2 (cell-wise) in cellwise[2*cell + {0,1}].
 * Returns the number of fields. */
int orc_get_tables(const orc_op *op, double *tables, double *cellwise);

/* quadrature geometry per cell and q: JxW and inverse Jacobian
 * ([a][e] = d xi_a / d x_e), layout [cell][q][1 + dim*dim] */
void orc_get_geometry(const orc_op *op, double *geo);

/* time integration weights, time_integration.cc:61-91 (BDF, variable step),
 * :100-107 (theta), :141-178 (none).  dt[0] newest.  Returns order. */
int orc_bdf_weights(int order, const double *dt, double *weights);

/* ----------------------------------------------------------- multigrid
 * Level transfer between consecutive geometric levels, MGTwoLevelTransfer
 * semantics (main.cc:538-563):
 *   prolongate_add: dst_f += sum_cells w_f * P_cell (Z_c src_c)
 *   restrict_add:   dst_c += Z_c sum_cells P_cell^T (w_f * src_f)
 * with Z zeroing constrained coarse dofs, w_f = 1/valence on unconstrained
 * fine dofs and 0 on constrained fine dofs.  child[cell][(2k+1)^dim] from
 * gls_mesh_child_lattice. */
void orc_prolongate_add(const orc_mesh *coarse, const orc_mesh *fine,
                        const uint32_t *child, double *dst_f,
                        const double *src_c);
void orc_restrict_add(const orc_mesh *coarse, const orc_mesh *fine,
                      const uint32_t *child, double *dst_c,
                      const double *src_f);
/* interpolate_to_mg: nodal injection fine -> coarse (no constraints) */
void orc_interpolate(const orc_mesh *coarse, const orc_mesh *fine,
                     const uint32_t *child, double *dst_c,
                     const double *src_f);

#ifdef __cplusplus
}
#endif

#endif
