/*
 * gls_oracle.c — TEST INFRASTRUCTURE ONLY (see gls_oracle.h header).
 *
 * CPU restatement of the reference's matrix-free GLS Navier-Stokes operator.
 * Evaluation is by tensor-product sum factorisation on the Q_k GLL-Lagrange
 * basis at QGauss(k+1) (as deal.II's FEEvaluation does); cells are processed
 * one at a time (optionally OpenMP-parallel with atomic scatter).
 * Parity status: pinned by KAT-1..6, not by reference outputs.
 */
#include "gls_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXK 4
#define MAXN (MAXK + 1)
#define MAXNQ (MAXN * MAXN * MAXN)

static int g_threads = 1;

void
orc_set_threads(int n)
{
  g_threads = n < 1 ? 1 : n;
}

/* ------------------------------------------------------------ 1D basis */
typedef struct
{
  int    n;                 /* k + 1                                         */
  double nodes[MAXN];       /* GLL support points of FE_Q(k) on [0,1]        */
  double qp[MAXN], qw[MAXN];/* QGauss(k+1) on [0,1]                          */
  double S[MAXN][MAXN];     /* S[q][i] = phi_i(x_q)                          */
  double D[MAXN][MAXN];     /* D[q][i] = phi_i'(x_q)                         */
} basis1d;

static void
gauss_legendre(int n, double *x, double *w)
{
  /* Newton on Legendre P_n in [-1,1], mapped to [0,1] */
  for (int i = 0; i < n; ++i)
    {
      double z = cos(M_PI * (i + 0.75) / (n + 0.5)), pp = 0;
      for (int it = 0; it < 100; ++it)
        {
          double p1 = 1, p2 = 0;
          for (int j = 1; j <= n; ++j)
            {
              double p3 = p2;
              p2        = p1;
              p1        = ((2.0 * j - 1.0) * z * p2 - (j - 1.0) * p3) / j;
            }
          pp        = n * (z * p1 - p2) / (z * z - 1.0);
          double z1 = z;
          z         = z1 - p1 / pp;
          if (fabs(z - z1) < 1e-16)
            break;
        }
      x[n - 1 - i] = 0.5 * (1.0 + z); /* ascending */
      w[n - 1 - i] = 1.0 / ((1.0 - z * z) * pp * pp);
    }
}

static void
make_basis(int k, basis1d *b)
{
  b->n = k + 1;
  if (k == 1)
    {
      b->nodes[0] = 0, b->nodes[1] = 1;
    }
  else if (k == 2)
    {
      b->nodes[0] = 0, b->nodes[1] = 0.5, b->nodes[2] = 1;
    }
  else if (k == 3)
    {
      b->nodes[0] = 0, b->nodes[1] = 0.5 - sqrt(5.0) / 10.0,
      b->nodes[2] = 0.5 + sqrt(5.0) / 10.0, b->nodes[3] = 1;
    }
  else
    {
      b->nodes[0] = 0, b->nodes[1] = 0.5 - sqrt(21.0) / 14.0, b->nodes[2] = 0.5,
      b->nodes[3] = 0.5 + sqrt(21.0) / 14.0, b->nodes[4] = 1;
    }
  gauss_legendre(b->n, b->qp, b->qw);
  for (int q = 0; q < b->n; ++q)
    for (int i = 0; i < b->n; ++i)
      {
        const double x = b->qp[q];
        double       v = 1, d = 0;
        for (int j = 0; j < b->n; ++j)
          if (j != i)
            {
              double prod = 1.0 / (b->nodes[i] - b->nodes[j]);
              for (int m = 0; m < b->n; ++m)
                if (m != i && m != j)
                  prod *= (x - b->nodes[m]) / (b->nodes[i] - b->nodes[m]);
              d += prod;
              v *= (x - b->nodes[j]) / (b->nodes[i] - b->nodes[j]);
            }
        b->S[q][i] = v;
        b->D[q][i] = d;
      }
}

/* apply a 1D matrix M (n x n, M[q][i]) along axis `ax` of a dim-tensor with
 * n points per direction: out[.. q ..] = sum_i M[q][i] in[.. i ..]
 * (transpose: out[.. i ..] = sum_q M[q][i] in[.. q ..]) */
static void
apply1d(int dim, int n, const double M[MAXN][MAXN], int ax, int transpose,
        const double *in, double *out)
{
  const int s  = ax == 0 ? 1 : (ax == 1 ? n : n * n);
  const int nt = dim == 3 ? n * n * n : n * n;
  for (int p = 0; p < nt; ++p)
    {
      const int pi   = (p / s) % n;
      const int base = p - pi * s;
      double    acc  = 0;
      for (int j = 0; j < n; ++j)
        acc += (transpose ? M[j][pi] : M[pi][j]) * in[base + j * s];
      out[p] = acc;
    }
}

/* evaluate value and reference gradient of a scalar field at all q */
static void
eval_scalar(int dim, const basis1d *b, const double *u, double *val,
            double *grad /* [dim][MAXNQ] */)
{
  const int n = b->n;
  double    t1[MAXNQ], t2[MAXNQ];
  if (dim == 2)
    {
      apply1d(2, n, b->S, 0, 0, u, t1);
      apply1d(2, n, b->S, 1, 0, t1, val);
      apply1d(2, n, b->D, 1, 0, t1, grad + MAXNQ);
      apply1d(2, n, b->D, 0, 0, u, t1);
      apply1d(2, n, b->S, 1, 0, t1, grad);
    }
  else
    {
      apply1d(3, n, b->S, 0, 0, u, t1);
      apply1d(3, n, b->S, 1, 0, t1, t2);
      apply1d(3, n, b->S, 2, 0, t2, val);
      apply1d(3, n, b->D, 2, 0, t2, grad + 2 * MAXNQ);
      apply1d(3, n, b->D, 1, 0, t1, t2);
      apply1d(3, n, b->S, 2, 0, t2, grad + MAXNQ);
      apply1d(3, n, b->D, 0, 0, u, t1);
      apply1d(3, n, b->S, 1, 0, t1, t2);
      apply1d(3, n, b->S, 2, 0, t2, grad);
    }
}

/* transpose of eval_scalar: out_i = sum_q (val_q phi_i + sum_a grad_aq dphi_i/dxi_a) */
static void
integrate_scalar(int dim, const basis1d *b, const double *val,
                 const double *grad, double *out)
{
  const int n = b->n, nq = dim == 3 ? n * n * n : n * n;
  double    t1[MAXNQ], t2[MAXNQ], acc[MAXNQ];
  if (dim == 2)
    {
      apply1d(2, n, b->S, 1, 1, val, t1);
      apply1d(2, n, b->D, 1, 1, grad + MAXNQ, t2);
      for (int p = 0; p < nq; ++p)
        t1[p] += t2[p];
      apply1d(2, n, b->S, 0, 1, t1, out);
      apply1d(2, n, b->S, 1, 1, grad, t1);
      apply1d(2, n, b->D, 0, 1, t1, t2);
      for (int p = 0; p < nq; ++p)
        out[p] += t2[p];
    }
  else
    {
      /* value + z-gradient share the (S_x, S_y) path */
      apply1d(3, n, b->S, 2, 1, val, t1);
      apply1d(3, n, b->D, 2, 1, grad + 2 * MAXNQ, t2);
      for (int p = 0; p < nq; ++p)
        t1[p] += t2[p];
      apply1d(3, n, b->S, 1, 1, t1, t2);
      apply1d(3, n, b->S, 2, 1, grad + MAXNQ, t1);
      apply1d(3, n, b->D, 1, 1, t1, acc);
      for (int p = 0; p < nq; ++p)
        t2[p] += acc[p];
      apply1d(3, n, b->S, 0, 1, t2, out);
      apply1d(3, n, b->S, 2, 1, grad, t1);
      apply1d(3, n, b->S, 1, 1, t1, t2);
      apply1d(3, n, b->D, 0, 1, t2, t1);
      for (int p = 0; p < nq; ++p)
        out[p] += t1[p];
    }
}

/* ------------------------------------------------------------ operator */
struct orc_op
{
  orc_mesh   m;
  orc_params prm;
  basis1d    b;
  int        nq, nf;
  double    *geo;      /* [cell][q][1 + dim*dim] JxW, invJ[a][e]          */
  double    *tab;      /* [cell][q][nf] canonical tables                   */
  double    *cellwise; /* [cell][2]                                        */
  int        have_prev;
  int        have_old_grad;
  double    *old_grad; /* [cell][q][dim*dim + dim] grad u_old, grad p_old  */
  /* outflow boundary faces (orc_set_outflow_faces) */
  int64_t    n_faces;
  int        nqf;
  int64_t   *fcell;    /* [f] cell                                          */
  int       *fkind;    /* [f] ORC_OUTFLOW_CUT / ORC_OUTFLOW_NITSCHE          */
  double    *fbeta;    /* [f] effective_beta_face                           */
  double    *fjxw;     /* [f][qf] face JxW                                  */
  double    *fnormal;  /* [f][qf][dim] outward unit normal                  */
  double    *fphi;     /* [f][qf][nq] cell basis values at the face points  */
  double    *fdn;      /* [f][qf][nq] normal derivatives of the cell basis  */
  double    *fpts;     /* [f][qf][dim] face quadrature points               */
  double    *fustar;   /* [f][qf][dim] face_velocity (linearization point)  */
  double    *ftarget;  /* [f][qf][dim] face_target_velocity                 */
};

static void faces_linearization(orc_op *op, const double *vec);

static int
nfields(int dim)
{
  return 2 + 3 * dim + dim * dim;
}
#define F_D1 0
#define F_D2 1
#define F_U(dim) 2
#define F_GU(dim) (2 + (dim))
#define F_GP(dim) (2 + (dim) + (dim) * (dim))
#define F_UT(dim) (2 + 2 * (dim) + (dim) * (dim))

static void lagrange1d(const basis1d *b, int i, double x, double *v, double *d);

/* reference-space gradient of the MappingQ_m map of cell c at the element's
 * quadrature points (QGauss(k+1)^dim): g[d][a][q] = dx_d / dxi_a, from the
 * cell's (m+1)^dim mapping support points (mapping_points) */
static void
mapping_gradients(const orc_op *op, int64_t c, double g[3][3][MAXNQ])
{
  const int dim = op->m.dim, n = op->b.n, nq = op->nq;
  const int m = op->m.mapping_degree, nm = m + 1;
  const int nmq = dim == 3 ? nm * nm * nm : nm * nm;
  basis1d   bm;
  make_basis(m, &bm);
  double S[MAXN][MAXN], D[MAXN][MAXN]; /* [q][i]: mapping basis at the FE points */
  for (int q = 0; q < n; ++q)
    for (int i = 0; i < nm; ++i)
      lagrange1d(&bm, i, op->b.qp[q], &S[q][i], &D[q][i]);
  const double *X = op->m.mapping_points + (size_t)c * nmq * dim;
  for (int d = 0; d < dim; ++d)
    for (int a = 0; a < dim; ++a)
      for (int q = 0; q < nq; ++q)
        g[d][a][q] = 0;
  for (int q = 0; q < nq; ++q)
    {
      const int qa[3] = {q % n, (q / n) % n, dim == 3 ? q / (n * n) : 0};
      for (int i = 0; i < nmq; ++i)
        {
          const int ia[3] = {i % nm, (i / nm) % nm, dim == 3 ? i / (nm * nm) : 0};
          for (int a = 0; a < dim; ++a)
            {
              double w = 1;
              for (int e = 0; e < dim; ++e)
                w *= e == a ? D[qa[e]][ia[e]] : S[qa[e]][ia[e]];
              for (int d = 0; d < dim; ++d)
                g[d][a][q] += X[i * dim + d] * w;
            }
        }
    }
}

static void
compute_geometry(orc_op *op)
{
  const int dim = op->m.dim, nq = op->nq, nloc = nq;
  const int ng  = 1 + dim * dim;
  op->geo       = (double *)calloc((size_t)op->m.n_cells * nq * ng, sizeof(double));
  for (int64_t c = 0; c < op->m.n_cells; ++c)
    {
      double X[3][MAXNQ], val[MAXNQ], g[3][3][MAXNQ];
      if (op->m.mapping_points)
        mapping_gradients(op, c, g);
      else
        {
          for (int d = 0; d < dim; ++d)
            for (int i = 0; i < nloc; ++i)
              X[d][i] = op->m.coords[(size_t)op->m.cell_nodes[c * nloc + i] * dim + d];
          for (int d = 0; d < dim; ++d)
            eval_scalar(dim, &op->b, X[d], val, &g[d][0][0]);
        }
      for (int q = 0; q < nq; ++q)
        {
          double J[3][3] = {{0}}, inv[3][3] = {{0}}, det;
          for (int d = 0; d < dim; ++d)
            for (int a = 0; a < dim; ++a)
              J[d][a] = g[d][a][q]; /* dx_d / dxi_a */
          if (dim == 2)
            {
              det       = J[0][0] * J[1][1] - J[0][1] * J[1][0];
              inv[0][0] = J[1][1] / det, inv[0][1] = -J[0][1] / det;
              inv[1][0] = -J[1][0] / det, inv[1][1] = J[0][0] / det;
            }
          else
            {
              det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                    J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                    J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
              inv[0][0] = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) / det;
              inv[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
              inv[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
              inv[1][0] = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) / det;
              inv[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
              inv[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
              inv[2][0] = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) / det;
              inv[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
              inv[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
            }
          const int qx = q % op->b.n, qy = (q / op->b.n) % op->b.n,
                    qz = q / (op->b.n * op->b.n);
          double w = op->b.qw[qx] * op->b.qw[qy] * (dim == 3 ? op->b.qw[qz] : 1.0);
          double *G = op->geo + ((size_t)c * nq + q) * ng;
          G[0]      = det * w;
          for (int a = 0; a < dim; ++a)
            for (int e = 0; e < dim; ++e)
              G[1 + a * dim + e] = inv[a][e]; /* dxi_a / dx_e */
        }
    }
}

orc_op *
orc_create(const orc_mesh *mesh, const orc_params *prm)
{
  if (!mesh || !prm || mesh->degree < 1 || mesh->degree > MAXK ||
      (mesh->dim != 2 && mesh->dim != 3) ||
      (mesh->mapping_points && (mesh->mapping_degree < 1 || mesh->mapping_degree > MAXK)))
    return NULL;
  orc_op *op = (orc_op *)calloc(1, sizeof(orc_op));
  op->m      = *mesh;
  op->prm    = *prm;
  make_basis(mesh->degree, &op->b);
  op->nq       = mesh->dim == 3 ? op->b.n * op->b.n * op->b.n : op->b.n * op->b.n;
  op->nf       = nfields(mesh->dim);
  op->tab      = (double *)calloc((size_t)mesh->n_cells * op->nq * op->nf, sizeof(double));
  op->cellwise = (double *)calloc((size_t)mesh->n_cells * 2, sizeof(double));
  compute_geometry(op);
  return op;
}

void
orc_destroy(orc_op *op)
{
  if (!op)
    return;
  free(op->geo);
  free(op->tab);
  free(op->cellwise);
  free(op->old_grad);
  free(op->fcell), free(op->fkind), free(op->fbeta), free(op->fjxw), free(op->fnormal);
  free(op->fphi), free(op->fdn), free(op->fpts), free(op->fustar), free(op->ftarget);
  free(op);
}

/* values + real-space gradients of `ncomp` components starting at `c0` of a
 * global vector at all q of a cell (read_dof_values_plain) */
static void
eval_cell(const orc_op *op, int64_t c, const double *vec, int c0, int ncomp,
          double val[][MAXNQ], double grad[][3][MAXNQ])
{
  const int dim = op->m.dim, nq = op->nq, ng = 1 + dim * dim, nc = dim + 1;
  for (int comp = 0; comp < ncomp; ++comp)
    {
      double u[MAXNQ], gr[3][MAXNQ];
      for (int i = 0; i < nq; ++i)
        u[i] = vec[(size_t)op->m.cell_nodes[c * nq + i] * nc + c0 + comp];
      eval_scalar(dim, &op->b, u, val[comp], &gr[0][0]);
      for (int q = 0; q < nq; ++q)
        {
          const double *G = op->geo + ((size_t)c * nq + q) * ng;
          for (int e = 0; e < dim; ++e)
            {
              double s = 0;
              for (int a = 0; a < dim; ++a)
                s += G[1 + a * dim + e] * gr[a][q];
              grad[comp][e][q] = s;
            }
        }
    }
}

void
orc_set_linearization_point(orc_op *op, const double *vec)
{
  const int    dim = op->m.dim, nq = op->nq, nf = op->nf, k = op->m.degree;
  const double tau  = op->prm.dt;
  const double stau = tau == 0.0 ? 0.0 : 1.0 / tau;
  const double nu   = op->prm.nu;
  for (int64_t c = 0; c < op->m.n_cells; ++c)
    {
      double val[4][MAXNQ], grad[4][3][MAXNQ];
      eval_cell(op, c, vec, 0, dim + 1, val, grad);
      double *T = op->tab + (size_t)c * nq * nf;
      for (int q = 0; q < nq; ++q)
        {
          double *t = T + q * nf;
          for (int d = 0; d < dim; ++d)
            {
              t[F_U(dim) + d] = val[d][q];
              for (int e = 0; e < dim; ++e)
                t[F_GU(dim) + d * dim + e] = grad[d][e][q];
              t[F_GP(dim) + d] = grad[dim][d][q];
            }
        }
      /* compute_penalty_parameters, operator_ns.cc:357-421 */
      double u_max = 0.0;
      for (int q = 0; q < nq; ++q)
        {
          double s = 0;
          for (int d = 0; d < dim; ++d)
            s += val[d][q] * val[d][q];
          if (sqrt(s) > u_max)
            u_max = sqrt(s);
        }
      {
        const double h = op->m.cell_hmin[c];
        if (nu < h)
          {
            op->cellwise[2 * c] =
              op->prm.c1 / sqrt(stau * stau + u_max * u_max / (h * h));
            op->cellwise[2 * c + 1] = op->prm.c2 * h;
          }
        else
          {
            op->cellwise[2 * c]     = op->prm.c1 * h * h;
            op->cellwise[2 * c + 1] = op->prm.c2 * h * h;
          }
      }
      const double hk = op->m.cell_measure[c];
      const double h  = dim == 2 ? sqrt(4. * hk / M_PI) / k : pow(6 * hk / M_PI, 1. / 3.) / k;
      for (int q = 0; q < nq; ++q)
        {
          double u2 = 1e-12;
          for (int d = 0; d < dim; ++d)
            u2 += val[d][q] * val[d][q];
          const double a = 4. * nu / (h * h);
          T[q * nf + F_D1] = 1. / sqrt(stau * stau + 4. * u2 / h / h + 9. * a * a);
          T[q * nf + F_D2] = sqrt(u2) * h * 0.5;
        }
    }  faces_linearization(op, vec);
}

void
orc_set_previous_solution(orc_op *op, const double *const *hist, int n_hist,
                          const double *weights)
{
  const int dim = op->m.dim, nq = op->nq, nf = op->nf;
  const int order = op->prm.order;
  if (order == 0)
    return;
  const int64_t n   = op->m.n_nodes * (dim + 1);
  double       *old = (double *)calloc((size_t)n, sizeof(double));
  for (int i = 1; i <= order && i < n_hist; ++i)
    for (int64_t j = 0; j < n; ++j)
      old[j] += weights[i] * hist[i][j];
  for (int64_t c = 0; c < op->m.n_cells; ++c)
    {
      double val[4][MAXNQ], grad[4][3][MAXNQ];
      eval_cell(op, c, old, 0, dim, val, grad);
      for (int q = 0; q < nq; ++q)
        for (int d = 0; d < dim; ++d)
          op->tab[((size_t)c * nq + q) * nf + F_UT(dim) + d] = val[d][q];
    }
  op->have_prev = 1;
  free(old);
  if (op->prm.theta != 1.0)
    {
      const int ng = dim * dim + dim;
      free(op->old_grad);
      op->old_grad = (double *)calloc((size_t)op->m.n_cells * nq * ng, sizeof(double));
      for (int64_t c = 0; c < op->m.n_cells; ++c)
        {
          double val[4][MAXNQ], grad[4][3][MAXNQ];
          eval_cell(op, c, hist[1], 0, dim + 1, val, grad);
          for (int q = 0; q < nq; ++q)
            {
              double *o = op->old_grad + ((size_t)c * nq + q) * ng;
              for (int d = 0; d < dim; ++d)
                {
                  for (int e = 0; e < dim; ++e)
                    o[d * dim + e] = grad[d][e][q];
                  o[dim * dim + d] = grad[dim][d][q];
                }
            }
        }
      op->have_old_grad = 1;
    }
}

/* do_vmult_cell, operator_ns.cc:949-1182.  uloc/out: [comp][node] */
static void
cell_apply(const orc_op *op, int64_t c, const double uloc[][MAXNQ],
           double out[][MAXNQ], int residual)
{
  const int dim = op->m.dim, nq = op->nq, nf = op->nf, ng = 1 + dim * dim;
  const int nc  = dim + 1;
  const double nu = op->prm.nu, w0 = op->prm.w0, theta = op->prm.theta;
  const int td = op->prm.consider_time_derivative && op->prm.order > 0;
  const int cw = op->prm.cell_wise_stabilization;
  double    val[4][MAXNQ], rg[4][3][MAXNQ];
  double    V[4][MAXNQ], Gq[4][3][MAXNQ]; /* reference-space test coeffs */

  for (int comp = 0; comp < nc; ++comp)
    eval_scalar(dim, &op->b, uloc[comp], val[comp], &rg[comp][0][0]);

  for (int q = 0; q < nq; ++q)
    {
      const double *G   = op->geo + ((size_t)c * nq + q) * ng;
      const double *t   = op->tab + ((size_t)c * nq + q) * nf;
      const double  JxW = G[0];
      double        u[3], p, gu[3][3], gp[3];
      for (int d = 0; d < dim; ++d)
        u[d] = val[d][q];
      p = val[dim][q];
      for (int comp = 0; comp < nc; ++comp)
        for (int e = 0; e < dim; ++e)
          {
            double s = 0;
            for (int a = 0; a < dim; ++a)
              s += G[1 + a * dim + e] * rg[comp][a][q];
            if (comp < dim)
              gu[comp][e] = s;
            else
              gp[e] = s;
          }
      const double d1 = cw ? op->cellwise[2 * c] : t[F_D1];
      const double d2 = cw ? op->cellwise[2 * c + 1] : t[F_D2];
      const double *U  = t + F_U(dim);
      const double *GU = t + F_GU(dim);
      double        vr[4] = {0, 0, 0, 0}, gr[4][3] = {{0}};

      if (residual || !op->prm.increment_form)
        {
          /* fixed-point / residual branch, :955-1066 */
          double ut[3], gb[3][3], gpb[3];
          for (int d = 0; d < dim; ++d)
            {
              ut[d]  = u[d] * w0;
              gpb[d] = theta * gp[d];
              for (int e = 0; e < dim; ++e)
                gb[d][e] = theta * gu[d][e];
            }
          if (residual && op->have_prev)
            for (int d = 0; d < dim; ++d)
              ut[d] += t[F_UT(dim) + d];
          if (residual && theta != 1.0 && op->have_old_grad)
            {
              const double *o = op->old_grad + ((size_t)c * nq + q) * (dim * dim + dim);
              for (int d = 0; d < dim; ++d)
                {
                  for (int e = 0; e < dim; ++e)
                    gb[d][e] += (1.0 - theta) * o[d * dim + e];
                  gpb[d] += (1.0 - theta) * o[dim * dim + d];
                }
            }
          double divb = 0, sgb[3];
          for (int d = 0; d < dim; ++d)
            divb += gb[d][d];
          for (int d = 0; d < dim; ++d)
            {
              sgb[d] = 0;
              for (int e = 0; e < dim; ++e)
                sgb[d] += gb[d][e] * U[e];
            }
          for (int d = 0; d < dim; ++d)
            vr[d] = ut[d] + sgb[d];
          for (int d = 0; d < dim; ++d)
            gr[d][d] -= p;
          /* symm_scalar_product_add(gr, gb, 2 nu) :899-916 */
          for (int d = 0; d < dim; ++d)
            gr[d][d] += gb[d][d] * (2.0 * nu);
          for (int e = 0; e < dim; ++e)
            for (int d = e + 1; d < dim; ++d)
              {
                const double tmp = (gb[d][e] + gb[e][d]) * nu;
                gr[d][e] += tmp;
                gr[e][d] += tmp;
              }
          double r0[3];
          for (int d = 0; d < dim; ++d)
            r0[d] = d1 * ((td ? ut[d] : 0.0) + gpb[d] + sgb[d]);
          for (int d0 = 0; d0 < dim; ++d0)
            for (int d1i = 0; d1i < dim; ++d1i)
              gr[d0][d1i] += U[d1i] * r0[d0];
          for (int d = 0; d < dim; ++d)
            gr[d][d] += d2 * divb;
          vr[dim] = divb;
          for (int d = 0; d < dim; ++d)
            gr[dim][d] = d1 * ((td ? ut[d] : 0.0) + gp[d] + sgb[d]);
        }
      else
        {
          /* Newton increment branch, :1067-1181 */
          const double *GP = t + F_GP(dim);
          const double *UT = t + F_UT(dim);
          double        ut[3], divu = 0, sgu[3], ugs[3], sgs[3];
          for (int d = 0; d < dim; ++d)
            ut[d] = u[d] * w0;
          for (int d = 0; d < dim; ++d)
            divu += gu[d][d];
          for (int d = 0; d < dim; ++d)
            {
              sgu[d] = ugs[d] = sgs[d] = 0;
              for (int e = 0; e < dim; ++e)
                {
                  sgu[d] += gu[d][e] * U[e];
                  ugs[d] += GU[d * dim + e] * u[e];
                  sgs[d] += GU[d * dim + e] * U[e];
                }
            }
          for (int d = 0; d < dim; ++d)
            vr[d] = ut[d] + sgu[d] + ugs[d];
          for (int d = 0; d < dim; ++d)
            gr[d][d] -= p;
          for (int d = 0; d < dim; ++d)
            gr[d][d] += gu[d][d] * (2.0 * nu);
          for (int e = 0; e < dim; ++e)
            for (int d = e + 1; d < dim; ++d)
              {
                const double tmp = (gu[d][e] + gu[e][d]) * nu;
                gr[d][e] += tmp;
                gr[e][d] += tmp;
              }
          double r0[3], r1[3];
          for (int d = 0; d < dim; ++d)
            {
              r0[d] = d1 * ((td ? ut[d] : 0.0) + gp[d] + sgu[d] + ugs[d]);
              r1[d] = d1 * ((td ? (U[d] * w0 + UT[d]) : 0.0) + GP[d] + sgs[d]);
            }
          for (int d0 = 0; d0 < dim; ++d0)
            for (int e = 0; e < dim; ++e)
              gr[d0][e] += U[e] * r0[d0] + u[e] * r1[d0];
          for (int d = 0; d < dim; ++d)
            gr[d][d] += d2 * divu;
          vr[dim] = divu;
          for (int d = 0; d < dim; ++d)
            gr[dim][d] = d1 * ((td ? ut[d] : 0.0) + gp[d] + sgu[d] + ugs[d]);
        }
      /* submit_value / submit_gradient: multiply by JxW and J^{-T} */
      for (int comp = 0; comp < nc; ++comp)
        {
          V[comp][q] = vr[comp] * JxW;
          for (int a = 0; a < dim; ++a)
            {
              double s = 0;
              for (int e = 0; e < dim; ++e)
                s += G[1 + a * dim + e] * gr[comp][e];
              Gq[comp][a][q] = s * JxW;
            }
        }
    }
  for (int comp = 0; comp < nc; ++comp)
    integrate_scalar(dim, &op->b, V[comp], &Gq[comp][0][0], out[comp]);
}

/* ------------------------------------------------------------ outflow faces
 * Boundary-face terms of the outflow boundaries, do_vmult_boundary
 * operator_ns.cc:1195-1295: "cut" (:1201-1240) submits
 *   beta_F min(0, u* . n) u                        (velocity components)
 * with u* = face_velocity (the linearization point, :459-477) in vmult and the
 * current value in evaluate_residual; "Nitsche" (:1241-1287) submits
 *   value    beta_F (u - g) - nu (grad u) n
 *   gradient -nu (u - g) (x) n
 * with g = face_target_velocity (:478-521) in the residual only.
 * beta_F = 1 / h^(k+1), h = (4|K|/pi)^(1/2) / k (2D), (6|K|/pi)^(1/3) / k
 * (3D) of the face's cell (:423-457).  FEFaceEvaluation on QGauss(k+1)^(dim-1)
 * is restated as direct sums of the cell basis at the face points; faces are
 * identified by (cell, face number 2 * axis + side) as deal.II numbers them. */

/* 1D Lagrange basis function i on the GLL nodes and its derivative at x */
static void
lagrange1d(const basis1d *b, int i, double x, double *v, double *d)
{
  double vv = 1, dd = 0;
  for (int j = 0; j < b->n; ++j)
    if (j != i)
      {
        double prod = 1.0 / (b->nodes[i] - b->nodes[j]);
        for (int m = 0; m < b->n; ++m)
          if (m != i && m != j)
            prod *= (x - b->nodes[m]) / (b->nodes[i] - b->nodes[m]);
        dd += prod;
        vv *= (x - b->nodes[j]) / (b->nodes[i] - b->nodes[j]);
      }
  *v = vv;
  *d = dd;
}

int
orc_set_outflow_faces(orc_op *op, int64_t n, const int64_t *cells, const int32_t *face_no,
                      const int32_t *kind)
{
  const int dim = op->m.dim, nq = op->nq, n1 = op->b.n, k = op->m.degree;
  const int nqf = dim == 3 ? n1 * n1 : n1;
  if (op->m.mapping_points && n > 0)
    return 1; /* face geometry from the element's support points only */
  for (int64_t f = 0; f < n; ++f)
    if (cells[f] < 0 || cells[f] >= op->m.n_cells || face_no[f] < 0 || face_no[f] >= 2 * dim ||
        (kind[f] != ORC_OUTFLOW_CUT && kind[f] != ORC_OUTFLOW_NITSCHE))
      return -1;
  op->n_faces = n;
  op->nqf     = nqf;
#define ORC_REALLOC(p, cnt) p = realloc(p, sizeof(*p) * (size_t)((cnt) > 0 ? (cnt) : 1))
  ORC_REALLOC(op->fcell, n);
  ORC_REALLOC(op->fkind, n);
  ORC_REALLOC(op->fbeta, n);
  ORC_REALLOC(op->fjxw, n * nqf);
  ORC_REALLOC(op->fnormal, n * nqf * dim);
  ORC_REALLOC(op->fphi, n * nqf * nq);
  ORC_REALLOC(op->fdn, n * nqf * nq);
  ORC_REALLOC(op->fpts, n * nqf * dim);
  ORC_REALLOC(op->fustar, n * nqf * dim);
  ORC_REALLOC(op->ftarget, n * nqf * dim);
#undef ORC_REALLOC
  memset(op->fustar, 0, sizeof(double) * (size_t)(n * nqf * dim));
  memset(op->ftarget, 0, sizeof(double) * (size_t)(n * nqf * dim));
  for (int64_t f = 0; f < n; ++f)
    {
      const int64_t c = cells[f];
      const int     a = face_no[f] / 2, side = face_no[f] % 2;
      int           tang[2] = {0, 0}, nt = 0;
      for (int e = 0; e < dim; ++e)
        if (e != a)
          tang[nt++] = e;
      op->fcell[f] = c;
      op->fkind[f] = kind[f];
      {
        const double meas = op->m.cell_measure[c];
        const double h    = dim == 2 ? sqrt(4. * meas / M_PI) / k : pow(6. * meas / M_PI, 1. / 3.) / k;
        op->fbeta[f]      = 1.0 / pow(h, (double)(k + 1));
      }
      for (int qf = 0; qf < nqf; ++qf)
        {
          double xi[3] = {0, 0, 0}, w = 1;
          xi[a] = side;
          const int qt[2] = {qf % n1, qf / n1};
          for (int t = 0; t < nt; ++t)
            {
              xi[tang[t]] = op->b.qp[qt[t]];
              w *= op->b.qw[qt[t]];
            }
          double phi[MAXNQ], gref[MAXNQ][3], J[3][3] = {{0}}, x[3] = {0, 0, 0};
          for (int i = 0; i < nq; ++i)
            {
              const int ia[3] = {i % n1, (i / n1) % n1, dim == 3 ? i / (n1 * n1) : 0};
              double    v[3] = {1, 1, 1}, d[3] = {0, 0, 0};
              for (int e = 0; e < dim; ++e)
                lagrange1d(&op->b, ia[e], xi[e], &v[e], &d[e]);
              phi[i] = v[0] * v[1] * v[2];
              for (int e = 0; e < dim; ++e)
                {
                  double g = d[e];
                  for (int e2 = 0; e2 < dim; ++e2)
                    if (e2 != e)
                      g *= v[e2];
                  gref[i][e] = g;
                }
              const double *X = op->m.coords + (size_t)op->m.cell_nodes[c * nq + i] * dim;
              for (int dd = 0; dd < dim; ++dd)
                {
                  x[dd] += X[dd] * phi[i];
                  for (int e = 0; e < dim; ++e)
                    J[dd][e] += X[dd] * gref[i][e];
                }
            }
          double inv[3][3] = {{0}}, det;
          if (dim == 2)
            {
              det       = J[0][0] * J[1][1] - J[0][1] * J[1][0];
              inv[0][0] = J[1][1] / det, inv[0][1] = -J[0][1] / det;
              inv[1][0] = -J[1][0] / det, inv[1][1] = J[0][0] / det;
            }
          else
            {
              det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                    J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                    J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
              inv[0][0] = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) / det;
              inv[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
              inv[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
              inv[1][0] = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) / det;
              inv[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
              inv[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
              inv[2][0] = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) / det;
              inv[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
              inv[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
            }
          /* J^{-T} n_ref with n_ref = (2 side - 1) e_a: its length is the
           * face area element over |det J|, its direction the normal */
          double m[3] = {0, 0, 0}, mn = 0;
          for (int e = 0; e < dim; ++e)
            {
              m[e] = (2 * side - 1) * inv[a][e];
              mn += m[e] * m[e];
            }
          mn                          = sqrt(mn);
          const size_t fq             = (size_t)f * nqf + qf;
          op->fjxw[fq]                = fabs(det) * mn * w;
          for (int e = 0; e < dim; ++e)
            {
              op->fnormal[fq * dim + e] = m[e] / mn;
              op->fpts[fq * dim + e]    = x[e];
            }
          for (int i = 0; i < nq; ++i)
            {
              double dn = 0;
              for (int e = 0; e < dim; ++e)
                {
                  double gx = 0;
                  for (int b2 = 0; b2 < dim; ++b2)
                    gx += inv[b2][e] * gref[i][b2];
                  dn += gx * m[e] / mn;
                }
              op->fphi[fq * nq + i] = phi[i];
              op->fdn[fq * nq + i]  = dn;
            }
        }
    }
  return 0;
}

void
orc_outflow_face_points(const orc_op *op, double *xyz)
{
  memcpy(xyz, op->fpts, sizeof(double) * (size_t)(op->n_faces * op->nqf * op->m.dim));
}

void
orc_set_outflow_target(orc_op *op, const double *target)
{
  memcpy(op->ftarget, target, sizeof(double) * (size_t)(op->n_faces * op->nqf * op->m.dim));
}

/* face_velocity: the linearization point's velocity at the face points
 * (read_dof_values_plain + evaluate(values), operator_ns.cc:465-476) */
static void
faces_linearization(orc_op *op, const double *vec)
{
  const int dim = op->m.dim, nq = op->nq, nc = dim + 1, nqf = op->nqf;
  for (int64_t f = 0; f < op->n_faces; ++f)
    for (int qf = 0; qf < nqf; ++qf)
      for (int d = 0; d < dim; ++d)
        {
          double        u   = 0;
          const double *phi = op->fphi + ((size_t)f * nqf + qf) * nq;
          for (int i = 0; i < nq; ++i)
            u += phi[i] * vec[(size_t)op->m.cell_nodes[op->fcell[f] * nq + i] * nc + d];
          op->fustar[((size_t)f * nqf + qf) * dim + d] = u;
        }
}

/* do_vmult_boundary on face f for the cell-local dof values uloc (velocity
 * components; the pressure takes no face term): out += face integrals */
static void
face_apply(const orc_op *op, int64_t f, const double uloc[][MAXNQ], double out[][MAXNQ],
           int residual)
{
  const int    dim = op->m.dim, nq = op->nq, nqf = op->nqf;
  const double beta = op->fbeta[f], nu = op->prm.nu;
  for (int qf = 0; qf < nqf; ++qf)
    {
      const size_t  fq  = (size_t)f * nqf + qf;
      const double *phi = op->fphi + fq * nq, *dn = op->fdn + fq * nq, *nrm = op->fnormal + fq * dim;
      double        u[3] = {0, 0, 0}, un[3] = {0, 0, 0}, vr[3] = {0, 0, 0}, gc[3] = {0, 0, 0};
      for (int d = 0; d < dim; ++d)
        for (int i = 0; i < nq; ++i)
          {
            u[d] += phi[i] * uloc[d][i];
            un[d] += dn[i] * uloc[d][i];
          }
      if (op->fkind[f] == ORC_OUTFLOW_CUT)
        {
          const double *star = residual ? u : op->fustar + fq * dim;
          double        on   = 0;
          for (int d = 0; d < dim; ++d)
            on += star[d] * nrm[d];
          on = on < 0 ? on : 0.0;
          for (int d = 0; d < dim; ++d)
            vr[d] = beta * on * u[d];
        }
      else
        {
          if (residual)
            for (int d = 0; d < dim; ++d)
              u[d] -= op->ftarget[fq * dim + d];
          for (int d = 0; d < dim; ++d)
            {
              vr[d] = beta * u[d] - nu * un[d];
              gc[d] = -nu * u[d]; /* gradient_result = gc (x) n, tested: gc dn */
            }
        }
      const double jxw = op->fjxw[fq];
      for (int d = 0; d < dim; ++d)
        for (int i = 0; i < nq; ++i)
          out[d][i] += jxw * (vr[d] * phi[i] + gc[d] * dn[i]);
    }
}

/* the face loop of MatrixFree::loop (boundary faces, do_vmult_boundary_range
 * operator_ns.cc:849-879): read_dof_values(_plain), distribute_local_to_global */
static void
face_loop(const orc_op *op, double *dst, const double *src, int residual)
{
  const int dim = op->m.dim, nq = op->nq, nc = dim + 1;
  for (int64_t f = 0; f < op->n_faces; ++f)
    {
      const int64_t c = op->fcell[f];
      double        uloc[4][MAXNQ], out[4][MAXNQ];
      memset(out, 0, sizeof(out));
      for (int i = 0; i < nq; ++i)
        {
          const uint32_t node = op->m.cell_nodes[c * nq + i];
          const uint8_t  cm   = op->m.cmask[node];
          for (int comp = 0; comp < nc; ++comp)
            uloc[comp][i] = (!residual && ((cm >> comp) & 1)) ? 0.0 : src[(size_t)node * nc + comp];
        }
      face_apply(op, f, (const double(*)[MAXNQ])uloc, out, residual);
      for (int i = 0; i < nq; ++i)
        {
          const uint32_t node = op->m.cell_nodes[c * nq + i];
          const uint8_t  cm   = op->m.cmask[node];
          for (int comp = 0; comp < dim; ++comp)
            if (!((cm >> comp) & 1))
              dst[(size_t)node * nc + comp] += out[comp][i];
        }
    }
}

/* face part of the element matrix of cell c (compute_matrix with a
 * boundary worker, operator_ns.cc:1380-1400) and of the diagonal
 * (compute_diagonal's boundary_function, :202-218) */
static void
face_cell_matrix_add(const orc_op *op, int64_t c, double *mat)
{
  const int nq = op->nq, nc = op->m.dim + 1, nd = nq * nc;
  for (int64_t f = 0; f < op->n_faces; ++f)
    {
      if (op->fcell[f] != c)
        continue;
      for (int j = 0; j < nd; ++j)
        {
          double uloc[4][MAXNQ] = {{0}}, out[4][MAXNQ];
          memset(out, 0, sizeof(out));
          uloc[j % nc][j / nc] = 1.0;
          face_apply(op, f, (const double(*)[MAXNQ])uloc, out, 0);
          for (int i = 0; i < nd; ++i)
            mat[(size_t)i * nd + j] += out[i % nc][i / nc];
        }
    }
}

static void
face_diagonal_add(const orc_op *op, double *diag)
{
  const int nq = op->nq, dim = op->m.dim, nc = dim + 1;
  for (int64_t f = 0; f < op->n_faces; ++f)
    {
      const int64_t c = op->fcell[f];
      for (int i = 0; i < nq; ++i)
        for (int comp = 0; comp < dim; ++comp)
          {
            const uint32_t node = op->m.cell_nodes[c * nq + i];
            if ((op->m.cmask[node] >> comp) & 1)
              continue;
            double uloc[4][MAXNQ] = {{0}}, out[4][MAXNQ];
            memset(out, 0, sizeof(out));
            uloc[comp][i] = 1.0;
            face_apply(op, f, (const double(*)[MAXNQ])uloc, out, 0);
            diag[(size_t)node * nc + comp] += out[comp][i];
          }
    }
}

static inline void
atomic_add(double *p, double v)
{
#ifdef _OPENMP
#pragma omp atomic
#endif
  *p += v;
}

static void
cell_loop(const orc_op *op, double *dst, const double *src, int residual)
{
  const int     dim = op->m.dim, nq = op->nq, nc = dim + 1;
  const int64_t n   = op->m.n_nodes * nc;
  memset(dst, 0, sizeof(double) * (size_t)n);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
#endif
  for (int64_t c = 0; c < op->m.n_cells; ++c)
    {
      double uloc[4][MAXNQ], out[4][MAXNQ];
      for (int i = 0; i < nq; ++i)
        {
          const uint32_t node = op->m.cell_nodes[c * nq + i];
          const uint8_t  cm   = op->m.cmask[node];
          for (int comp = 0; comp < nc; ++comp)
            uloc[comp][i] = (!residual && ((cm >> comp) & 1)) ?
                              0.0 : /* read_dof_values: homogeneous constraints */
                              src[(size_t)node * nc + comp];
        }
      cell_apply(op, c, (const double(*)[MAXNQ])uloc, out, residual);
      for (int i = 0; i < nq; ++i)
        {
          const uint32_t node = op->m.cell_nodes[c * nq + i];
          const uint8_t  cm   = op->m.cmask[node];
          for (int comp = 0; comp < nc; ++comp)
            if (!((cm >> comp) & 1)) /* distribute_local_to_global skips constrained */
              {
                if (g_threads > 1)
                  atomic_add(&dst[(size_t)node * nc + comp], out[comp][i]);
                else
                  dst[(size_t)node * nc + comp] += out[comp][i];
              }
        }
    }  face_loop(op, dst, src, residual);
}

void
orc_vmult(const orc_op *op, double *dst, const double *src)
{
  const int nc = op->m.dim + 1;
  cell_loop(op, dst, src, 0);
  /* identity rows, operator_ns.cc:719-721 */
  for (int64_t node = 0; node < op->m.n_nodes; ++node)
    for (int comp = 0; comp < nc; ++comp)
      if ((op->m.cmask[node] >> comp) & 1)
        dst[node * nc + comp] = src[node * nc + comp];
}

void
orc_evaluate_residual(const orc_op *op, double *dst, const double *src)
{
  const int     nc = op->m.dim + 1;
  const int64_t n  = op->m.n_nodes * nc;
  cell_loop(op, dst, src, 1);
  for (int64_t node = 0; node < op->m.n_nodes; ++node)
    for (int comp = 0; comp < nc; ++comp)
      if ((op->m.cmask[node] >> comp) & 1)
        dst[node * nc + comp] = 0.0; /* set_zero */
  for (int64_t i = 0; i < n; ++i)
    dst[i] = -dst[i];
}

void
orc_cell_matrix(const orc_op *op, int64_t c, double *mat)
{
  const int nq = op->nq, nc = op->m.dim + 1, nd = nq * nc;
  for (int j = 0; j < nd; ++j)
    {
      double uloc[4][MAXNQ] = {{0}}, out[4][MAXNQ];
      uloc[j % nc][j / nc]  = 1.0;
      cell_apply(op, c, (const double(*)[MAXNQ])uloc, out, 0);
      for (int i = 0; i < nd; ++i)
        mat[(size_t)i * nd + j] = out[i % nc][i / nc];
    }  face_cell_matrix_add(op, c, mat);
}

/* the assembled diagonal before the inversion (constrained components: 1 on
 * the owned range [0, n_owned_nodes), 0 elsewhere): the rank-local half of a
 * partitioned compute_inverse_diagonal (the caller adds the ghost partials
 * to their owners, then inverts) */
void
orc_compute_diagonal(const orc_op *op, int64_t n_owned_nodes, double *diag)
{
  const int     nq = op->nq, nc = op->m.dim + 1, nd = nq * nc;
  const int64_t n  = op->m.n_nodes * nc;
  memset(diag, 0, sizeof(double) * (size_t)n);
  for (int64_t c = 0; c < op->m.n_cells; ++c)
    for (int j = 0; j < nd; ++j)
      {
        const uint32_t node = op->m.cell_nodes[c * nq + j / nc];
        const int      comp = j % nc;
        if ((op->m.cmask[node] >> comp) & 1)
          continue;
        double uloc[4][MAXNQ] = {{0}}, out[4][MAXNQ];
        uloc[comp][j / nc]    = 1.0;
        cell_apply(op, c, (const double(*)[MAXNQ])uloc, out, 0);
        diag[(size_t)node * nc + comp] += out[comp][j / nc];
      }
  face_diagonal_add(op, diag);
  for (int64_t node = 0; node < n_owned_nodes; ++node)
    for (int comp = 0; comp < nc; ++comp)
      if ((op->m.cmask[node] >> comp) & 1)
        diag[node * nc + comp] = 1.0;
}

void
orc_compute_inverse_diagonal(const orc_op *op, double *diag)
{
  const int     nq = op->nq, nc = op->m.dim + 1, nd = nq * nc;
  const int64_t n  = op->m.n_nodes * nc;
  memset(diag, 0, sizeof(double) * (size_t)n);
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)
#endif
  for (int64_t c = 0; c < op->m.n_cells; ++c)
    for (int j = 0; j < nd; ++j)
      {
        const uint32_t node = op->m.cell_nodes[c * nq + j / nc];
        const int      comp = j % nc;
        if ((op->m.cmask[node] >> comp) & 1)
          continue;
        double uloc[4][MAXNQ] = {{0}}, out[4][MAXNQ];
        uloc[comp][j / nc]    = 1.0;
        cell_apply(op, c, (const double(*)[MAXNQ])uloc, out, 0);
        if (g_threads > 1)
          atomic_add(&diag[(size_t)node * nc + comp], out[comp][j / nc]);
        else
          diag[(size_t)node * nc + comp] += out[comp][j / nc];
      }
  face_diagonal_add(op, diag);
  for (int64_t node = 0; node < op->m.n_nodes; ++node)
    for (int comp = 0; comp < nc; ++comp)
      if ((op->m.cmask[node] >> comp) & 1)
        diag[node * nc + comp] = 1.0; /* constrained rows are identity */
  for (int64_t i = 0; i < n; ++i)
    diag[i] = fabs(diag[i]) > 1.0e-10 ? 1.0 / diag[i] : 1.0;
}

/* NavierStokesOperator::get_max_u, operator_ns.cc:530-568: read_dof_values_plain,
 * evaluate(values), max over cells and q points of |u(x_q)| (velocity only) */
double
orc_get_max_u(const orc_op *op, const double *vec)
{
  const int dim = op->m.dim, nq = op->nq, nc = dim + 1;
  double    m   = 0.0;
  for (int64_t c = 0; c < op->m.n_cells; ++c)
    {
      double val[3][MAXNQ], gr[3][MAXNQ];
      for (int d = 0; d < dim; ++d)
        {
          double u[MAXNQ];
          for (int i = 0; i < nq; ++i)
            u[i] = vec[(size_t)op->m.cell_nodes[c * nq + i] * nc + d];
          eval_scalar(dim, &op->b, u, val[d], &gr[0][0]);
        }
      for (int q = 0; q < nq; ++q)
        {
          double s = 0;
          for (int d = 0; d < dim; ++d)
            s += val[d][q] * val[d][q];
          if (sqrt(s) > m)
            m = sqrt(s);
        }
    }
  return m;
}

int
orc_get_tables(const orc_op *op, double *tables, double *cellwise)
{
  const size_t n = (size_t)op->m.n_cells * op->nq * op->nf;
  if (tables)
    memcpy(tables, op->tab, n * sizeof(double));
  if (cellwise)
    memcpy(cellwise, op->cellwise, (size_t)op->m.n_cells * 2 * sizeof(double));
  return op->nf;
}

void
orc_get_geometry(const orc_op *op, double *geo)
{
  const int dim = op->m.dim;
  memcpy(geo, op->geo, (size_t)op->m.n_cells * op->nq * (1 + dim * dim) * sizeof(double));
}

int
orc_bdf_weights(int order, const double *dt, double *w)
{
  /* TimeIntegratorDataBDF::update_weights, time_integration.cc:61-91;
   * effective order = number of positive dt entries */
  int eff = 0;
  for (int i = 0; i < order; ++i)
    eff += dt[i] > 0;
  for (int i = 0; i <= order; ++i)
    w[i] = 0;
  if (eff == 3)
    {
      w[1] = -(dt[0] + dt[1]) * (dt[0] + dt[1] + dt[2]) / (dt[0] * dt[1] * (dt[1] + dt[2]));
      w[2] = dt[0] * (dt[0] + dt[1] + dt[2]) / (dt[1] * dt[2] * (dt[0] + dt[1]));
      w[3] = -dt[0] * (dt[0] + dt[1]) / (dt[2] * (dt[1] + dt[2]) * (dt[0] + dt[1] + dt[2]));
      w[0] = -(w[1] + w[2] + w[3]);
    }
  else if (eff == 2)
    {
      w[0] = (2 * dt[0] + dt[1]) / (dt[0] * (dt[0] + dt[1]));
      w[1] = -(dt[0] + dt[1]) / (dt[0] * dt[1]);
      w[2] = dt[0] / (dt[1] * (dt[0] + dt[1]));
    }
  else if (eff == 1)
    {
      w[0] = 1.0 / dt[0];
      w[1] = -1.0 / dt[0];
    }
  return eff;
}

/* ------------------------------------------------------------ transfer */
static void
lattice_prolongation_1d(int k, double P[2 * MAXK + 1][MAXN])
{
  /* P[I][j] = phi_j(I / (2k)) on the parent's GLL basis (equispaced k<=2) */
  basis1d b;
  make_basis(k, &b);
  for (int I = 0; I <= 2 * k; ++I)
    {
      /* fine lattice coordinate: child c = I / k (clipped), local i */
      const int    c = I / k > 1 ? 1 : I / k;
      const int    i = I - c * k;
      const double x = 0.5 * (c + b.nodes[i]);
      for (int j = 0; j <= k; ++j)
        {
          double v = 1;
          for (int m = 0; m <= k; ++m)
            if (m != j)
              v *= (x - b.nodes[m]) / (b.nodes[j] - b.nodes[m]);
          P[I][j] = v;
        }
    }
}

static double *
fine_weights(const orc_mesh *coarse, const orc_mesh *fine, const uint32_t *child)
{
  const int dim = fine->dim, k = coarse->degree, nc = dim + 1;
  const int L = 2 * k + 1, nl = dim == 3 ? L * L * L : L * L;
  double   *val = (double *)calloc((size_t)fine->n_nodes, sizeof(double));
  for (int64_t c = 0; c < coarse->n_cells; ++c)
    for (int i = 0; i < nl; ++i)
      val[child[c * nl + i]] += 1.0;
  double *w = (double *)calloc((size_t)fine->n_nodes * nc, sizeof(double));
  for (int64_t n = 0; n < fine->n_nodes; ++n)
    for (int comp = 0; comp < nc; ++comp)
      w[n * nc + comp] = ((fine->cmask[n] >> comp) & 1) ? 0.0 : 1.0 / val[n];
  free(val);
  return w;
}

void
orc_prolongate_add(const orc_mesh *coarse, const orc_mesh *fine,
                   const uint32_t *child, double *dst_f, const double *src_c)
{
  /* the coarse level's degree (FE_Q_iso_Q1 coarse levels are Q1 on the
     sub-cells below a Q_k level, main.cc:436-446) */
  const int dim = fine->dim, k = coarse->degree, nc = dim + 1, n = k + 1;
  const int L = 2 * k + 1, nl = dim == 3 ? L * L * L : L * L;
  const int nloc = dim == 3 ? n * n * n : n * n;
  double    P[2 * MAXK + 1][MAXN];
  lattice_prolongation_1d(k, P);
  double *w = fine_weights(coarse, fine, child);
  for (int64_t c = 0; c < coarse->n_cells; ++c)
    for (int comp = 0; comp < nc; ++comp)
      {
        double u[MAXNQ];
        for (int i = 0; i < nloc; ++i)
          {
            const uint32_t node = coarse->cell_nodes[c * nloc + i];
            u[i] = ((coarse->cmask[node] >> comp) & 1) ? 0.0 : src_c[(size_t)node * nc + comp];
          }
        for (int I = 0; I < nl; ++I)
          {
            const int Ix = I % L, Iy = (I / L) % L, Iz = dim == 3 ? I / (L * L) : 0;
            double    s  = 0;
            for (int i = 0; i < nloc; ++i)
              {
                const int ix = i % n, iy = (i / n) % n, iz = dim == 3 ? i / (n * n) : 0;
                s += P[Ix][ix] * P[Iy][iy] * (dim == 3 ? P[Iz][iz] : 1.0) * u[i];
              }
            const uint32_t fn = child[c * nl + I];
            dst_f[(size_t)fn * nc + comp] += w[(size_t)fn * nc + comp] * s;
          }
      }
  free(w);
}

void
orc_restrict_add(const orc_mesh *coarse, const orc_mesh *fine,
                 const uint32_t *child, double *dst_c, const double *src_f)
{
  /* the coarse level's degree (FE_Q_iso_Q1 coarse levels are Q1 on the
     sub-cells below a Q_k level, main.cc:436-446) */
  const int dim = fine->dim, k = coarse->degree, nc = dim + 1, n = k + 1;
  const int L = 2 * k + 1, nl = dim == 3 ? L * L * L : L * L;
  const int nloc = dim == 3 ? n * n * n : n * n;
  double    P[2 * MAXK + 1][MAXN];
  lattice_prolongation_1d(k, P);
  double *w = fine_weights(coarse, fine, child);
  for (int64_t c = 0; c < coarse->n_cells; ++c)
    for (int comp = 0; comp < nc; ++comp)
      {
        double v[(2 * MAXK + 1) * (2 * MAXK + 1) * (2 * MAXK + 1)];
        for (int I = 0; I < nl; ++I)
          {
            const uint32_t fn = child[c * nl + I];
            v[I] = w[(size_t)fn * nc + comp] * src_f[(size_t)fn * nc + comp];
          }
        for (int i = 0; i < nloc; ++i)
          {
            const uint32_t node = coarse->cell_nodes[c * nloc + i];
            if ((coarse->cmask[node] >> comp) & 1)
              continue;
            const int ix = i % n, iy = (i / n) % n, iz = dim == 3 ? i / (n * n) : 0;
            double    s  = 0;
            for (int I = 0; I < nl; ++I)
              {
                const int Ix = I % L, Iy = (I / L) % L, Iz = dim == 3 ? I / (L * L) : 0;
                s += P[Ix][ix] * P[Iy][iy] * (dim == 3 ? P[Iz][iz] : 1.0) * v[I];
              }
            dst_c[(size_t)node * nc + comp] += s;
          }
      }
  free(w);
}

void
orc_interpolate(const orc_mesh *coarse, const orc_mesh *fine,
                const uint32_t *child, double *dst_c, const double *src_f)
{
  /* the coarse level's degree (FE_Q_iso_Q1 coarse levels are Q1 on the
     sub-cells below a Q_k level, main.cc:436-446) */
  const int dim = fine->dim, k = coarse->degree, nc = dim + 1, n = k + 1;
  const int L = 2 * k + 1, nl = dim == 3 ? L * L * L : L * L;
  const int nloc = dim == 3 ? n * n * n : n * n;
  (void)nl;
  for (int64_t c = 0; c < coarse->n_cells; ++c)
    for (int i = 0; i < nloc; ++i)
      {
        const int ix = i % n, iy = (i / n) % n, iz = dim == 3 ? i / (n * n) : 0;
        /* coarse GLL node i sits at fine lattice point 2*i (k <= 2) */
        const int I = 2 * ix + L * (2 * iy + L * (dim == 3 ? 2 * iz : 0));
        const uint32_t fn = child[c * nl + I];
        const uint32_t cn = coarse->cell_nodes[c * nloc + i];
        for (int comp = 0; comp < nc; ++comp)
          dst_c[(size_t)cn * nc + comp] = src_f[(size_t)fn * nc + comp];
      }
}
