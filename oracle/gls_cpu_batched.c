/*
 * gls_cpu_batched.c — TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py
 * (cpu_baseline, "kind": "port").
 *
 * A cell-batched, SIMD-vectorised CPU restatement of the headline workload:
 * the Newton-Jacobian (increment-form) GLS operator apply of
 * NavierStokesOperator::vmult (operator_ns.cc:684-732, do_vmult_cell
 * :1067-1181) for 3D Q2/Q2, organised the way deal.II's MatrixFree runs it on
 * a CPU: batches of W = 8 cells, one cell per SIMD lane (VectorizedArray<
 * double, 8> with AVX-512, 2 x 4 with AVX2), per-q tables stored per batch
 * [batch][q][field][lane], MatrixFree-style compressed geometry (Cartesian
 * batches: J^{-1} diagonal and det J per lane; others J^{-1} and JxW per q),
 * sum factorisation with 1-D 3x3 kernels, gather/scatter per lane, and the
 * batches coloured so that batches of one colour share no node: the threads
 * of a colour scatter without atomics (deal.II's partition_partition
 * colouring for thread-parallel loops).
 *
 * Same numbers as oracle/gls_oracle.c (the scalar restatement, which checks
 * this file: tests/test_cpu_batched.py) up to the summation order.
 *
 * Compiled twice (oracle/Makefile): -mavx512f (W = 8 doubles per vector) and
 * -mavx2 -mfma (the same vector type, lowered to two 256-bit halves); the
 * caller picks by CPU flags.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define W 8
#define N 3   /* Q2: 3 points per direction */
#define NQ 27 /* (k+1)^3 */
#define NC 4  /* dim + 1 */
#define NF 20 /* delta1, delta2, U(3), gradU(9), gradP(3), Ut_old(3) */

typedef double vd __attribute__((vector_size(8 * W), aligned(8 * W)));

typedef struct
{
  int64_t   n_batches, n_nodes;
  int       threads;
  double    nu, w0;
  int       td;
  uint32_t *node;   /* [nb][NQ][W] node of lane cell (empty lane: 0) */
  uint8_t  *cmask;  /* [n_nodes] constrained component bits */
  uint8_t  *lanes;  /* [nb] active lanes */
  uint8_t  *cart;   /* [nb] 1: Cartesian batch */
  int64_t  *goff;   /* [nb] offset into geo (in vd) */
  vd       *geo;    /* Cartesian: 4 vd (invJ_xx, invJ_yy, invJ_zz, det); else NQ * 10 */
  vd       *tab;    /* [nb][NQ][NF] */
  int       n_colors;
  int64_t  *color_off;   /* [n_colors + 1] */
  int64_t  *color_batch; /* batches by colour */
  double    S[N][N], D[N][N], w[N];
} cpu_op;

static void
basis(cpu_op *op)
{
  const double x[N] = {0.0, 0.5, 1.0};
  const double g    = sqrt(3.0 / 5.0) / 2.0;
  const double q[N] = {0.5 - g, 0.5, 0.5 + g};
  const double w[N] = {5.0 / 18.0, 8.0 / 18.0, 5.0 / 18.0};
  for (int a = 0; a < N; ++a)
    {
      op->w[a] = w[a];
      for (int i = 0; i < N; ++i)
        {
          double v = 1, d = 0;
          for (int j = 0; j < N; ++j)
            if (j != i)
              {
                double p = 1.0 / (x[i] - x[j]);
                for (int l = 0; l < N; ++l)
                  if (l != i && l != j)
                    p *= (q[a] - x[l]) / (x[i] - x[l]);
                d += p;
                v *= (q[a] - x[j]) / (x[i] - x[j]);
              }
          op->S[a][i] = v;
          op->D[a][i] = d;
        }
    }
}

/* geo: [cell][q][1 + 9] (JxW, J^{-1} row-major, oracle orc_get_geometry);
 * tables: [cell][q][NF] (oracle orc_get_tables); cells batched in order */
cpu_op *
cpu_create(int64_t n_cells, int64_t n_nodes, const uint32_t *cell_nodes, const uint8_t *cmask,
           const double *geo, const double *tables, double nu, double w0, int td, int threads)
{
  cpu_op *op = calloc(1, sizeof(cpu_op));
  basis(op);
  op->threads   = threads > 0 ? threads : 1;
  op->nu        = nu;
  op->w0        = w0;
  op->td        = td;
  op->n_nodes   = n_nodes;
  const int64_t nb = (n_cells + W - 1) / W;
  op->n_batches = nb;
  op->node      = aligned_alloc(64, (size_t)nb * NQ * W * sizeof(uint32_t) + 64);
  op->cmask     = malloc((size_t)n_nodes);
  memcpy(op->cmask, cmask, (size_t)n_nodes);
  op->lanes = calloc((size_t)nb, 1);
  op->cart  = calloc((size_t)nb, 1);
  op->goff  = calloc((size_t)nb, sizeof(int64_t));
  op->tab   = aligned_alloc(64, (size_t)nb * NQ * NF * sizeof(vd) + 64);
  /* geometry: classify batches */
  int64_t ng = 0;
  for (int64_t b = 0; b < nb; ++b)
    {
      int cart = 1;
      for (int l = 0; l < W && cart; ++l)
        {
          const int64_t c = b * W + l;
          if (c >= n_cells)
            break;
          const double *G0 = geo + (size_t)c * NQ * 10;
          for (int q = 0; q < NQ && cart; ++q)
            {
              const double *G = G0 + q * 10;
              for (int i = 0; i < 9; ++i)
                {
                  const int diag = i == 0 || i == 4 || i == 8;
                  if ((!diag && G[1 + i] != 0.0) || fabs(G[1 + i] - G0[1 + i]) > 1e-14 * fabs(G0[1 + i]))
                    cart = 0;
                }
            }
        }
      op->cart[b] = (uint8_t)cart;
      op->goff[b] = ng;
      ng += cart ? 4 : NQ * 10;
    }
  op->geo = aligned_alloc(64, (size_t)ng * sizeof(vd) + 64);
  for (int64_t b = 0; b < nb; ++b)
    {
      int nl = 0;
      for (int l = 0; l < W; ++l)
        {
          const int64_t c  = b * W + l;
          const int     on = c < n_cells;
          const int64_t cc = on ? c : b * W; /* empty lanes: copy of lane 0, never scattered */
          nl += on;
          for (int q = 0; q < NQ; ++q)
            {
              op->node[((size_t)b * NQ + q) * W + l] = cell_nodes[(size_t)cc * NQ + q];
              for (int f = 0; f < NF; ++f)
                op->tab[((size_t)b * NQ + q) * NF + f][l] = tables[((size_t)cc * NQ + q) * NF + f];
            }
          const double *G0 = geo + (size_t)cc * NQ * 10;
          vd           *g  = op->geo + op->goff[b];
          if (op->cart[b])
            {
              g[0][l] = G0[1];
              g[1][l] = G0[5];
              g[2][l] = G0[9];
              /* JxW_q = det * w_x w_y w_z */
              g[3][l] = G0[0] / (op->w[0] * op->w[0] * op->w[0]);
            }
          else
            for (int q = 0; q < NQ; ++q)
              for (int i = 0; i < 10; ++i)
                g[q * 10 + i][l] = G0[q * 10 + i];
        }
      op->lanes[b] = (uint8_t)nl;
    }
  /* greedy colouring of the batches: no two batches of one colour share a
   * node (node -> batches adjacency, colours as 64-bit masks) */
  int64_t *nb_cnt = calloc((size_t)n_nodes + 1, sizeof(int64_t));
  for (int64_t b = 0; b < nb; ++b)
    for (int i = 0; i < NQ * W; ++i)
      if (i % W < op->lanes[b])
        nb_cnt[op->node[(size_t)b * NQ * W + i] + 1]++;
  for (int64_t v = 0; v < n_nodes; ++v)
    nb_cnt[v + 1] += nb_cnt[v];
  int64_t *adj  = malloc((size_t)nb_cnt[n_nodes] * sizeof(int64_t));
  int64_t *fill = calloc((size_t)n_nodes, sizeof(int64_t));
  for (int64_t b = 0; b < nb; ++b)
    for (int i = 0; i < NQ * W; ++i)
      if (i % W < op->lanes[b])
        {
          const uint32_t v = op->node[(size_t)b * NQ * W + i];
          adj[nb_cnt[v] + fill[v]++] = b;
        }
  int *color = malloc((size_t)nb * sizeof(int));
  for (int64_t b = 0; b < nb; ++b)
    color[b] = -1;
  int max_color = 0;
  for (int64_t b = 0; b < nb; ++b)
    {
      uint64_t used = 0;
      for (int i = 0; i < NQ * W; ++i)
        if (i % W < op->lanes[b])
          {
            const uint32_t v = op->node[(size_t)b * NQ * W + i];
            for (int64_t j = nb_cnt[v]; j < nb_cnt[v + 1]; ++j)
              if (color[adj[j]] >= 0)
                used |= 1ull << color[adj[j]];
          }
      int c = 0;
      while (c < 63 && ((used >> c) & 1))
        ++c;
      color[b] = c;
      if (c + 1 > max_color)
        max_color = c + 1;
    }
  op->n_colors    = max_color;
  op->color_off   = calloc((size_t)max_color + 1, sizeof(int64_t));
  op->color_batch = malloc((size_t)nb * sizeof(int64_t));
  for (int64_t b = 0; b < nb; ++b)
    op->color_off[color[b] + 1]++;
  for (int c = 0; c < max_color; ++c)
    op->color_off[c + 1] += op->color_off[c];
  int64_t *cf = calloc((size_t)max_color, sizeof(int64_t));
  for (int64_t b = 0; b < nb; ++b)
    op->color_batch[op->color_off[color[b]] + cf[color[b]]++] = b;
  free(cf);
  free(color);
  free(adj);
  free(fill);
  free(nb_cnt);
  return op;
}

int
cpu_n_colors(const cpu_op *op)
{
  return op->n_colors;
}

void
cpu_destroy(cpu_op *op)
{
  if (!op)
    return;
  free(op->node);
  free(op->cmask);
  free(op->lanes);
  free(op->cart);
  free(op->goff);
  free(op->geo);
  free(op->tab);
  free(op->color_off);
  free(op->color_batch);
  free(op);
}

/* 1-D sweep along axis ax (stride st) of a 3x3x3 vd block: out = M in */
static inline void
sweep(const double M[N][N], int ax, const vd *in, vd *out)
{
  const int st = ax == 0 ? 1 : ax == 1 ? N : N * N;
  for (int p = 0; p < NQ; ++p)
    {
      const int pa = (p / st) % N, base = p - pa * st;
      out[p]       = M[pa][0] * in[base] + M[pa][1] * in[base + st] + M[pa][2] * in[base + 2 * st];
    }
}

/* transpose: out = M^T in */
static inline void
sweep_t(const double M[N][N], int ax, const vd *in, vd *out)
{
  const int st = ax == 0 ? 1 : ax == 1 ? N : N * N;
  for (int p = 0; p < NQ; ++p)
    {
      const int pa = (p / st) % N, base = p - pa * st;
      out[p]       = M[0][pa] * in[base] + M[1][pa] * in[base + st] + M[2][pa] * in[base + 2 * st];
    }
}

static void
batch_apply(const cpu_op *op, int64_t b, double *dst, const double *src)
{
  vd u[NC][NQ], val[NC][NQ], gr[NC][3][NQ], t1[NQ], t2[NQ];
  const uint32_t *nd = op->node + (size_t)b * NQ * W;
  /* read_dof_values: homogeneous constraints read as 0 */
  for (int i = 0; i < NQ; ++i)
    for (int l = 0; l < W; ++l)
      {
        const uint32_t v  = nd[i * W + l];
        const uint8_t  cm = op->cmask[v];
        for (int c = 0; c < NC; ++c)
          u[c][i][l] = ((cm >> c) & 1) ? 0.0 : src[(size_t)v * NC + c];
      }
  /* evaluate: values and reference gradients */
  for (int c = 0; c < NC; ++c)
    {
      sweep(op->S, 0, u[c], t1);
      sweep(op->S, 1, t1, t2);
      sweep(op->S, 2, t2, val[c]);
      sweep(op->D, 2, t2, gr[c][2]);
      sweep(op->D, 1, t1, t2);
      sweep(op->S, 2, t2, gr[c][1]);
      sweep(op->D, 0, u[c], t1);
      sweep(op->S, 1, t1, t2);
      sweep(op->S, 2, t2, gr[c][0]);
    }
  const vd *G    = op->geo + op->goff[b];
  const int cart = op->cart[b];
  const vd  vzero = {0};
  const double vnu = op->nu, w0 = op->w0;
  for (int q = 0; q < NQ; ++q)
    {
      const vd *t = op->tab + ((size_t)b * NQ + q) * NF;
      vd        inv[3][3], JxW;
      if (cart)
        {
          const int qa[3] = {q % N, (q / N) % N, q / (N * N)};
          for (int a = 0; a < 3; ++a)
            for (int e = 0; e < 3; ++e)
              inv[a][e] = vzero;
          inv[0][0] = G[0];
          inv[1][1] = G[1];
          inv[2][2] = G[2];
          JxW       = G[3] * (op->w[qa[0]] * op->w[qa[1]] * op->w[qa[2]]);
        }
      else
        {
          JxW = G[q * 10];
          for (int a = 0; a < 3; ++a)
            for (int e = 0; e < 3; ++e)
              inv[a][e] = G[q * 10 + 1 + a * 3 + e];
        }
      vd uq[3], p = val[3][q], gu[3][3], gp[3];
      for (int d = 0; d < 3; ++d)
        uq[d] = val[d][q];
      for (int c = 0; c < NC; ++c)
        for (int e = 0; e < 3; ++e)
          {
            vd s = inv[0][e] * gr[c][0][q] + inv[1][e] * gr[c][1][q] + inv[2][e] * gr[c][2][q];
            if (c < 3)
              gu[c][e] = s;
            else
              gp[e] = s;
          }
      const vd d1 = t[0], d2 = t[1];
      const vd *U = t + 2, *GU = t + 5, *GP = t + 14, *UT = t + 17;
      /* Newton increment branch, operator_ns.cc:1067-1181 */
      vd ut[3], divu = gu[0][0] + gu[1][1] + gu[2][2], sgu[3], ugs[3], sgs[3];
      for (int d = 0; d < 3; ++d)
        {
          ut[d]  = uq[d] * w0;
          sgu[d] = gu[d][0] * U[0] + gu[d][1] * U[1] + gu[d][2] * U[2];
          ugs[d] = GU[d * 3] * uq[0] + GU[d * 3 + 1] * uq[1] + GU[d * 3 + 2] * uq[2];
          sgs[d] = GU[d * 3] * U[0] + GU[d * 3 + 1] * U[1] + GU[d * 3 + 2] * U[2];
        }
      vd vr[NC], g[NC][3];
      for (int d = 0; d < 3; ++d)
        vr[d] = ut[d] + sgu[d] + ugs[d];
      for (int d = 0; d < 3; ++d)
        for (int e = 0; e < 3; ++e)
          g[d][e] = (gu[d][e] + gu[e][d]) * vnu; /* symm_scalar_product_add :899-916 */
      for (int d = 0; d < 3; ++d)
        g[d][d] -= p;
      vd r0[3], r1[3];
      for (int d = 0; d < 3; ++d)
        {
          const vd a = gp[d] + sgu[d] + ugs[d];
          const vd c = GP[d] + sgs[d];
          r0[d]      = d1 * (op->td ? ut[d] + a : a);
          r1[d]      = d1 * (op->td ? U[d] * w0 + UT[d] + c : c);
        }
      for (int d0 = 0; d0 < 3; ++d0)
        for (int e = 0; e < 3; ++e)
          g[d0][e] += U[e] * r0[d0] + uq[e] * r1[d0];
      for (int d = 0; d < 3; ++d)
        g[d][d] += d2 * divu;
      vr[3] = divu;
      for (int d = 0; d < 3; ++d)
        g[3][d] = r0[d];
      /* submit_value / submit_gradient (JxW, J^{-T}) */
      for (int c = 0; c < NC; ++c)
        {
          val[c][q] = vr[c] * JxW;
          for (int a = 0; a < 3; ++a)
            gr[c][a][q] = (inv[a][0] * g[c][0] + inv[a][1] * g[c][1] + inv[a][2] * g[c][2]) * JxW;
        }
    }
  /* integrate (transpose of evaluate), into u:
   * out = Sx^T (Sy^T (Sz^T val + Dz^T g2) + Dy^T Sz^T g1) + Dx^T Sy^T Sz^T g0 */
  for (int c = 0; c < NC; ++c)
    {
      vd z3[NQ], z[NQ], y[NQ], y1[NQ];
      sweep_t(op->S, 2, val[c], z3);
      sweep_t(op->D, 2, gr[c][2], z);
      for (int i = 0; i < NQ; ++i)
        z3[i] += z[i];
      sweep_t(op->S, 1, z3, y);
      sweep_t(op->S, 2, gr[c][1], z);
      sweep_t(op->D, 1, z, t1);
      for (int i = 0; i < NQ; ++i)
        y[i] += t1[i];
      sweep_t(op->S, 2, gr[c][0], z);
      sweep_t(op->S, 1, z, y1);
      sweep_t(op->S, 0, y, t1);
      sweep_t(op->D, 0, y1, t2);
      for (int i = 0; i < NQ; ++i)
        u[c][i] = t1[i] + t2[i];
    }
  /* distribute_local_to_global: skip constrained components */
  const int nl = op->lanes[b];
  for (int l = 0; l < nl; ++l)
    for (int i = 0; i < NQ; ++i)
      {
        const uint32_t v  = nd[i * W + l];
        const uint8_t  cm = op->cmask[v];
        for (int c = 0; c < NC; ++c)
          if (!((cm >> c) & 1))
            dst[(size_t)v * NC + c] += u[c][i][l];
      }
}

void
cpu_vmult(const cpu_op *op, double *dst, const double *src)
{
  const int64_t n = op->n_nodes * NC;
#pragma omp parallel num_threads(op->threads)
  {
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i)
      dst[i] = 0.0;
    for (int c = 0; c < op->n_colors; ++c)
      {
#pragma omp for schedule(static)
        for (int64_t j = op->color_off[c]; j < op->color_off[c + 1]; ++j)
          batch_apply(op, op->color_batch[j], dst, src);
      }
    /* identity rows, operator_ns.cc:719-721 */
#pragma omp for schedule(static)
    for (int64_t v = 0; v < op->n_nodes; ++v)
      for (int c = 0; c < NC; ++c)
        if ((op->cmask[v] >> c) & 1)
          dst[v * NC + c] = src[v * NC + c];
  }
}
