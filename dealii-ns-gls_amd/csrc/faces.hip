// faces.hip — outflow boundary-face terms of the operator.
//
// NavierStokesOperator runs MatrixFree::loop instead of cell_loop as soon as
// an outflow boundary is weak (needs_face_integrals, operator_ns.cc:94-95,
// 660-680, 702-716): do_vmult_boundary (:1195-1295) adds, on the faces of
// all_outflow_bcs_cut,
//   ( beta_F min(0, u* . n) u, v )_F                     (velocity only)
// with u* = face_velocity (the linearization point, :459-477) in vmult and
// the current value in evaluate_residual, and on those of
// all_outflow_bcs_nitsche
//   ( beta_F (u - g) - nu (grad u) n, v )_F - ( nu (u - g) (x) n, grad v )_F
// with g = face_target_velocity (:478-521) in the residual only;
// beta_F = 1 / h^(k+1) of the face's cell (:423-457).  compute_diagonal and
// compute_matrix take the same boundary worker (:202-218, 1380-1400).
//
// The outflow faces are a few hundred to a few thousand of the mesh's cells'
// faces, so this is a side path: one workgroup per face after the cell
// kernels on the same stream, with the face geometry (JxW, normal, the cell
// basis and its physical normal derivative at the QGauss(k+1)^(dim-1) face
// points) precomputed on the host at gls_op_create and atomically added
// contributions (a face's nodes are shared with the cell kernel's output).
#include "kernels.h"
#include "op_internal.h"

#include <cmath>
#include <stdexcept>

namespace gls
{
namespace
{
constexpr int FACE_BLOCK = 128;
constexpr int MAX_NQF    = 16; // (k+1)^(dim-1), k <= 3
constexpr int MAX_NQ     = 64;

template <typename T>
struct FaceArgs
{
  int             dim, nq, nqf;
  const uint32_t *nodes; // op->d_nodes, internal cell order
  const int64_t  *cell;  // [f] internal cell
  const int32_t  *kind;  // [f] GLS_OUTFLOW_CUT / GLS_OUTFLOW_NITSCHE
  const T        *beta;  // [f]
  const T        *jxw;   // [f][qf]
  const T        *normal;// [f][qf][dim]
  const T        *phi;   // [f][qf][nq]
  const T        *dn;    // [f][qf][nq]
  const T        *ustar; // [f][qf][dim]
  const T        *target;// [f][qf][dim]
  T               nu;
};

// vmult (R = false: read_dof_values, homogeneous constraints) or residual
// (R = true: read_dof_values_plain, negated like the cell residual)
template <typename T, bool R>
__global__ void __launch_bounds__(FACE_BLOCK)
  k_face_apply(FaceArgs<T> a, T *__restrict__ dst, const T *__restrict__ src)
{
  __shared__ T        sU[3][MAX_NQ];
  __shared__ T        sVR[MAX_NQF][3], sGC[MAX_NQF][3];
  __shared__ uint32_t sPk[MAX_NQ];
  const int64_t f = blockIdx.x;
  const int     t = threadIdx.x, dim = a.dim, nq = a.nq, nqf = a.nqf, nc = dim + 1;
  const int64_t c = a.cell[f];
  for (int i = t; i < nq; i += FACE_BLOCK)
    {
      const uint32_t pk = a.nodes[c * nq + i], node = pk & NODE_MASK, cm = pk >> 28;
      sPk[i] = pk;
      for (int d = 0; d < dim; ++d)
        sU[d][i] = (!R && ((cm >> d) & 1)) ? T(0) : src[(size_t)node * nc + d];
    }
  __syncthreads();
  if (t < nqf)
    {
      const size_t fq  = (size_t)f * nqf + t;
      const T     *phi = a.phi + fq * nq, *dn = a.dn + fq * nq, *nrm = a.normal + fq * dim;
      T            u[3] = {0, 0, 0}, un[3] = {0, 0, 0}, vr[3] = {0, 0, 0}, gc[3] = {0, 0, 0};
      for (int i = 0; i < nq; ++i)
        for (int d = 0; d < dim; ++d)
          {
            u[d] += phi[i] * sU[d][i];
            un[d] += dn[i] * sU[d][i];
          }
      const T beta = a.beta[f];
      if (a.kind[f] == GLS_OUTFLOW_CUT)
        {
          T on = 0;
          for (int d = 0; d < dim; ++d)
            on += (R ? u[d] : a.ustar[fq * dim + d]) * nrm[d];
          on = on < T(0) ? on : T(0);
          for (int d = 0; d < dim; ++d)
            vr[d] = beta * on * u[d];
        }
      else
        {
          if (R)
            for (int d = 0; d < dim; ++d)
              u[d] -= a.target[fq * dim + d];
          for (int d = 0; d < dim; ++d)
            {
              vr[d] = beta * u[d] - a.nu * un[d];
              gc[d] = -a.nu * u[d];
            }
        }
      const T w = a.jxw[fq];
      for (int d = 0; d < 3; ++d)
        {
          sVR[t][d] = w * vr[d];
          sGC[t][d] = w * gc[d];
        }
    }
  __syncthreads();
  for (int i = t; i < nq; i += FACE_BLOCK)
    {
      const uint32_t node = sPk[i] & NODE_MASK, cm = sPk[i] >> 28;
      for (int d = 0; d < dim; ++d)
        {
          if ((cm >> d) & 1)
            continue;
          T r = 0;
          for (int q = 0; q < nqf; ++q)
            {
              const size_t fq = (size_t)f * nqf + q;
              r += sVR[q][d] * a.phi[fq * nq + i] + sGC[q][d] * a.dn[fq * nq + i];
            }
          unsafeAtomicAdd(dst + (size_t)node * nc + d, R ? -r : r);
        }
    }
}

// diagonal: the unit-vector face apply at (node i, component d) has the
// self-entry sum_q JxW (beta min(0, u*.n) phi_i^2) (cut) or
// sum_q JxW (beta phi_i^2 - 2 nu phi_i dn_i) (Nitsche), the same for every
// velocity component
template <typename T, typename OutT>
__global__ void __launch_bounds__(FACE_BLOCK)
  k_face_diag(FaceArgs<T> a, OutT *__restrict__ diag)
{
  const int64_t f = blockIdx.x;
  const int     dim = a.dim, nq = a.nq, nqf = a.nqf, nc = dim + 1;
  const int64_t c = a.cell[f];
  for (int i = threadIdx.x; i < nq; i += FACE_BLOCK)
    {
      T acc = 0;
      for (int q = 0; q < nqf; ++q)
        {
          const size_t fq = (size_t)f * nqf + q;
          const T      ph = a.phi[fq * nq + i], dn = a.dn[fq * nq + i];
          T            v;
          if (a.kind[f] == GLS_OUTFLOW_CUT)
            {
              T on = 0;
              for (int d = 0; d < dim; ++d)
                on += a.ustar[fq * dim + d] * a.normal[fq * dim + d];
              on = on < T(0) ? on : T(0);
              v  = a.beta[f] * on * ph * ph;
            }
          else
            v = a.beta[f] * ph * ph - T(2) * a.nu * ph * dn;
          acc += a.jxw[fq] * v;
        }
      const uint32_t pk = a.nodes[c * nq + i], node = pk & NODE_MASK, cm = pk >> 28;
      for (int d = 0; d < dim; ++d)
        if (!((cm >> d) & 1))
          unsafeAtomicAdd(diag + (size_t)node * nc + d, (OutT)acc);
    }
}

// element matrices of cells [b, e): the face block couples (node j, d) to
// (node i, d) with the same entry for every velocity component d
template <typename T>
__global__ void __launch_bounds__(FACE_BLOCK)
  k_face_emat(FaceArgs<T> a, T *__restrict__ emat, int64_t b, int64_t e)
{
  const int64_t f = blockIdx.x;
  const int64_t c = a.cell[f];
  if (c < b || c >= e)
    return;
  const int dim = a.dim, nq = a.nq, nqf = a.nqf, nc = dim + 1, ndof = nq * nc;
  for (int p = threadIdx.x; p < nq * nq; p += FACE_BLOCK)
    {
      const int i = p % nq, j = p / nq; // row node i, column node j
      T         m = 0;
      for (int q = 0; q < nqf; ++q)
        {
          const size_t fq = (size_t)f * nqf + q;
          const T      pi = a.phi[fq * nq + i], pj = a.phi[fq * nq + j];
          T            v;
          if (a.kind[f] == GLS_OUTFLOW_CUT)
            {
              T on = 0;
              for (int d = 0; d < dim; ++d)
                on += a.ustar[fq * dim + d] * a.normal[fq * dim + d];
              on = on < T(0) ? on : T(0);
              v  = a.beta[f] * on * pj * pi;
            }
          else
            v = (a.beta[f] * pj - a.nu * a.dn[fq * nq + j]) * pi - a.nu * pj * a.dn[fq * nq + i];
          m += a.jxw[fq] * v;
        }
      for (int d = 0; d < dim; ++d)
        unsafeAtomicAdd(emat + ((size_t)(c - b) * ndof + j * nc + d) * ndof + i * nc + d, m);
    }
}

// face_velocity: the linearization point's velocity at the face points
template <typename T>
__global__ void
k_face_ustar(FaceArgs<T> a, int64_t n, T *__restrict__ ustar, const T *__restrict__ lin)
{
  const int64_t fq = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (fq >= n * a.nqf)
    return;
  const int64_t f = fq / a.nqf;
  const int     nc = a.dim + 1;
  const int64_t c  = a.cell[f];
  for (int d = 0; d < a.dim; ++d)
    {
      T u = 0;
      for (int i = 0; i < a.nq; ++i)
        u += a.phi[fq * a.nq + i] * lin[(size_t)(a.nodes[c * a.nq + i] & NODE_MASK) * nc + d];
      ustar[fq * a.dim + d] = u;
    }
}

template <typename T>
FaceArgs<T>
face_args(const glsOp_ *op)
{
  const OutflowFaces &F = op->faces;
  FaceArgs<T>         a;
  a.dim    = op->dim;
  a.nq     = op->nq;
  a.nqf    = F.nqf;
  a.nodes  = op->d_nodes;
  a.cell   = F.d_cell;
  a.kind   = F.d_kind;
  a.beta   = (const T *)F.d_beta;
  a.jxw    = (const T *)F.d_jxw;
  a.normal = (const T *)F.d_normal;
  a.phi    = (const T *)F.d_phi;
  a.dn     = (const T *)F.d_dn;
  a.ustar  = (const T *)F.d_ustar;
  a.target = (const T *)F.d_target;
  a.nu     = (T)op->prm.nu;
  return a;
}

// 1D Lagrange basis function i on the GLL nodes and its derivative at x
void
lagrange(const Basis1D &b, int i, double x, double &v, double &dv)
{
  v  = 1;
  dv = 0;
  for (int j = 0; j < b.n; ++j)
    if (j != i)
      {
        double prod = 1.0 / (b.nodes[i] - b.nodes[j]);
        for (int m = 0; m < b.n; ++m)
          if (m != i && m != j)
            prod *= (x - b.nodes[m]) / (b.nodes[i] - b.nodes[m]);
        dv += prod;
        v *= (x - b.nodes[j]) / (b.nodes[i] - b.nodes[j]);
      }
}

// inverse and determinant of the dim x dim Jacobian J[d][a] (row-major)
void
invert_jacobian(int dim, const double *J, double *inv, double &det)
{
  if (dim == 2)
    {
      det    = J[0] * J[3] - J[1] * J[2];
      inv[0] = J[3] / det, inv[1] = -J[1] / det, inv[2] = -J[2] / det, inv[3] = J[0] / det;
      return;
    }
  const double c00 = J[4] * J[8] - J[5] * J[7], c01 = J[5] * J[6] - J[3] * J[8],
               c02 = J[3] * J[7] - J[4] * J[6];
  det    = J[0] * c00 + J[1] * c01 + J[2] * c02;
  inv[0] = c00 / det, inv[1] = (J[2] * J[7] - J[1] * J[8]) / det;
  inv[2] = (J[1] * J[5] - J[2] * J[4]) / det;
  inv[3] = c01 / det, inv[4] = (J[0] * J[8] - J[2] * J[6]) / det;
  inv[5] = (J[2] * J[3] - J[0] * J[5]) / det;
  inv[6] = c02 / det, inv[7] = (J[1] * J[6] - J[0] * J[7]) / det;
  inv[8] = (J[0] * J[4] - J[1] * J[3]) / det;
}

template <typename T>
void
upload_as(void **d, const std::vector<double> &h)
{
  std::vector<T> t(h.begin(), h.end());
  HIP_THROW(hipMalloc(d, std::max<size_t>(1, t.size() * sizeof(T))));
  if (!t.empty())
    HIP_THROW(hipMemcpy(*d, t.data(), t.size() * sizeof(T), hipMemcpyHostToDevice));
}
} // namespace

void
faces_setup(glsOp_ *op, const glsOpDesc *d)
{
  OutflowFaces &F = op->faces;
  F.n             = d->n_outflow_faces;
  if (F.n <= 0)
    {
      F.n = 0;
      return;
    }
  if (!d->outflow_cells || !d->outflow_face_no || !d->outflow_kind)
    throw std::runtime_error("gls_op_create: outflow faces without cells / face_no / kind");
  if (op->n_owned_nodes != op->n_nodes)
    throw std::runtime_error("gls_op_create: outflow faces on a partitioned operator are not "
                             "supported (single domain only)");
  const int dim = op->dim, k = op->degree, n = k + 1, nq = op->nq;
  const int nqf = dim == 3 ? n * n : n;
  F.nqf         = nqf;
  // caller cell -> internal cell
  std::vector<int64_t> internal((size_t)op->n_cells);
  for (int64_t c = 0; c < op->n_cells; ++c)
    internal[(size_t)ext_cell(op, c)] = c;
  std::vector<int64_t> cell((size_t)F.n);
  std::vector<int32_t> kind((size_t)F.n);
  std::vector<double>  beta((size_t)F.n), jxw((size_t)F.n * nqf), nrm((size_t)F.n * nqf * dim),
    phi((size_t)F.n * nqf * nq), dnv((size_t)F.n * nqf * nq);
  F.h_points.assign((size_t)F.n * nqf * dim, 0.0);
  const Basis1D &b = op->basis;
  for (int64_t f = 0; f < F.n; ++f)
    {
      const int64_t cc = d->outflow_cells[f];
      const int     fn = d->outflow_face_no[f];
      if (cc < 0 || cc >= op->n_cells || fn < 0 || fn >= 2 * dim ||
          (d->outflow_kind[f] != GLS_OUTFLOW_CUT && d->outflow_kind[f] != GLS_OUTFLOW_NITSCHE))
        throw std::runtime_error("gls_op_create: bad outflow face");
      cell[(size_t)f] = internal[(size_t)cc];
      kind[(size_t)f] = d->outflow_kind[f];
      const int ax = fn / 2, side = fn % 2;
      int       tang[2] = {0, 0}, nt = 0;
      for (int e = 0; e < dim; ++e)
        if (e != ax)
          tang[nt++] = e;
      {
        // effective_beta_face, operator_ns.cc:437-456 (beta = 1)
        const double meas = d->cell_measure[cc];
        const double h    = dim == 2 ? std::sqrt(4. * meas / M_PI) / k :
                                       std::pow(6. * meas / M_PI, 1. / 3.) / k;
        beta[(size_t)f]   = 1.0 / std::pow(h, (double)(k + 1));
      }
      for (int qf = 0; qf < nqf; ++qf)
        {
          double    xi[3] = {0, 0, 0}, w = 1;
          const int qt[2] = {qf % n, qf / n};
          xi[ax]          = side;
          for (int t = 0; t < nt; ++t)
            {
              xi[tang[t]] = b.qp[(size_t)qt[t]];
              w *= b.qw[(size_t)qt[t]];
            }
          std::vector<double> ph((size_t)nq), gr((size_t)nq * 3);
          double              J[9] = {0}, x[3] = {0, 0, 0};
          for (int i = 0; i < nq; ++i)
            {
              const int ia[3] = {i % n, (i / n) % n, dim == 3 ? i / (n * n) : 0};
              double    v[3] = {1, 1, 1}, dv[3] = {0, 0, 0};
              for (int e = 0; e < dim; ++e)
                lagrange(b, ia[e], xi[e], v[e], dv[e]);
              ph[(size_t)i] = v[0] * v[1] * v[2];
              for (int e = 0; e < dim; ++e)
                {
                  double g = dv[e];
                  for (int e2 = 0; e2 < dim; ++e2)
                    if (e2 != e)
                      g *= v[e2];
                  gr[(size_t)i * 3 + e] = g;
                }
              const double *X = d->node_coords + (size_t)d->cell_nodes[(size_t)cc * nq + i] * dim;
              for (int dd = 0; dd < dim; ++dd)
                {
                  x[dd] += X[dd] * ph[(size_t)i];
                  for (int e = 0; e < dim; ++e)
                    J[dd * dim + e] += X[dd] * gr[(size_t)i * 3 + e];
                }
            }
          double inv[9], det;
          invert_jacobian(dim, J, inv, det);
          // J^{-T} n_ref, n_ref = (2 side - 1) e_ax: length = face area
          // element / |det J|, direction = outward normal
          double m[3] = {0, 0, 0}, mn = 0;
          for (int e = 0; e < dim; ++e)
            {
              m[e] = (2 * side - 1) * inv[ax * dim + e];
              mn += m[e] * m[e];
            }
          mn              = std::sqrt(mn);
          const size_t fq = (size_t)f * nqf + qf;
          jxw[fq]         = std::fabs(det) * mn * w;
          for (int e = 0; e < dim; ++e)
            {
              nrm[fq * dim + e]        = m[e] / mn;
              F.h_points[fq * dim + e] = x[e];
            }
          for (int i = 0; i < nq; ++i)
            {
              double dn = 0;
              for (int e = 0; e < dim; ++e)
                {
                  double gx = 0;
                  for (int a = 0; a < dim; ++a)
                    gx += inv[a * dim + e] * gr[(size_t)i * 3 + a];
                  dn += gx * m[e] / mn;
                }
              phi[fq * nq + i] = ph[(size_t)i];
              dnv[fq * nq + i] = dn;
            }
        }
    }
  HIP_THROW(hipMalloc((void **)&F.d_cell, cell.size() * sizeof(int64_t)));
  HIP_THROW(hipMemcpy(F.d_cell, cell.data(), cell.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  HIP_THROW(hipMalloc((void **)&F.d_kind, kind.size() * sizeof(int32_t)));
  HIP_THROW(hipMemcpy(F.d_kind, kind.data(), kind.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  const std::vector<double> zero((size_t)F.n * nqf * dim, 0.0);
  if (op->prec == GLS_F64)
    {
      upload_as<double>(&F.d_beta, beta);
      upload_as<double>(&F.d_jxw, jxw);
      upload_as<double>(&F.d_normal, nrm);
      upload_as<double>(&F.d_phi, phi);
      upload_as<double>(&F.d_dn, dnv);
      upload_as<double>(&F.d_ustar, zero);
      upload_as<double>(&F.d_target, zero);
    }
  else
    {
      upload_as<float>(&F.d_beta, beta);
      upload_as<float>(&F.d_jxw, jxw);
      upload_as<float>(&F.d_normal, nrm);
      upload_as<float>(&F.d_phi, phi);
      upload_as<float>(&F.d_dn, dnv);
      upload_as<float>(&F.d_ustar, zero);
      upload_as<float>(&F.d_target, zero);
    }
}

void
faces_release(glsOp_ *op)
{
  OutflowFaces &F      = op->faces;
  void         *bufs[] = {F.d_cell, F.d_kind, F.d_beta,  F.d_jxw,   F.d_normal,
                          F.d_phi,  F.d_dn,   F.d_ustar, F.d_target};
  for (void *p : bufs)
    if (p)
      (void)hipFree(p);
  F = OutflowFaces{};
}

void
faces_linearization(const glsOp_ *op, const void *lin, hipStream_t s)
{
  const OutflowFaces &F = op->faces;
  if (!F.n)
    return;
  const int64_t m = F.n * F.nqf;
  const dim3    g((unsigned)((m + 127) / 128));
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL(k_face_ustar<double>, g, dim3(128), 0, s, face_args<double>(op), F.n,
                       (double *)F.d_ustar, (const double *)lin);
  else
    hipLaunchKernelGGL(k_face_ustar<float>, g, dim3(128), 0, s, face_args<float>(op), F.n,
                       (float *)F.d_ustar, (const float *)lin);
  HIP_THROW(hipGetLastError());
}

void
faces_apply(const glsOp_ *op, bool residual, void *dst, const void *src, hipStream_t s)
{
  const OutflowFaces &F = op->faces;
  if (!F.n)
    return;
  const dim3 g((unsigned)F.n);
  if (op->prec == GLS_F64)
    {
      if (residual)
        hipLaunchKernelGGL((k_face_apply<double, true>), g, dim3(FACE_BLOCK), 0, s,
                           face_args<double>(op), (double *)dst, (const double *)src);
      else
        hipLaunchKernelGGL((k_face_apply<double, false>), g, dim3(FACE_BLOCK), 0, s,
                           face_args<double>(op), (double *)dst, (const double *)src);
    }
  else
    {
      if (residual)
        hipLaunchKernelGGL((k_face_apply<float, true>), g, dim3(FACE_BLOCK), 0, s,
                           face_args<float>(op), (float *)dst, (const float *)src);
      else
        hipLaunchKernelGGL((k_face_apply<float, false>), g, dim3(FACE_BLOCK), 0, s,
                           face_args<float>(op), (float *)dst, (const float *)src);
    }
  HIP_THROW(hipGetLastError());
}

void
faces_diagonal(const glsOp_ *op, void *diag, bool f64_out, hipStream_t s)
{
  const OutflowFaces &F = op->faces;
  if (!F.n)
    return;
  const dim3 g((unsigned)F.n);
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL((k_face_diag<double, double>), g, dim3(FACE_BLOCK), 0, s,
                       face_args<double>(op), (double *)diag);
  else if (f64_out)
    hipLaunchKernelGGL((k_face_diag<float, double>), g, dim3(FACE_BLOCK), 0, s,
                       face_args<float>(op), (double *)diag);
  else
    hipLaunchKernelGGL((k_face_diag<float, float>), g, dim3(FACE_BLOCK), 0, s,
                       face_args<float>(op), (float *)diag);
  HIP_THROW(hipGetLastError());
}

void
faces_element_matrices(const glsOp_ *op, void *emat, int64_t b, int64_t e, hipStream_t s)
{
  const OutflowFaces &F = op->faces;
  if (!F.n)
    return;
  const dim3 g((unsigned)F.n);
  if (op->prec == GLS_F64)
    hipLaunchKernelGGL(k_face_emat<double>, g, dim3(FACE_BLOCK), 0, s, face_args<double>(op),
                       (double *)emat, b, e);
  else
    hipLaunchKernelGGL(k_face_emat<float>, g, dim3(FACE_BLOCK), 0, s, face_args<float>(op),
                       (float *)emat, b, e);
  HIP_THROW(hipGetLastError());
}
} // namespace gls

extern "C" {

glsStatus
gls_op_n_outflow_faces(glsOp op, int64_t *n_faces, int *n_face_points)
{
  GLS_TRY
  if (!op || !n_faces || !n_face_points)
    throw std::runtime_error("gls_op_n_outflow_faces: null argument");
  *n_faces       = op->faces.n;
  *n_face_points = op->faces.nqf;
  GLS_CATCH
}

glsStatus
gls_op_outflow_face_points(glsOp op, double *xyz)
{
  GLS_TRY
  if (!op || !xyz)
    throw std::runtime_error("gls_op_outflow_face_points: null argument");
  std::copy(op->faces.h_points.begin(), op->faces.h_points.end(), xyz);
  GLS_CATCH
}

glsStatus
gls_op_set_outflow_target(glsOp op, const double *target, void *stream)
{
  GLS_TRY
  if (!op || !target)
    throw std::runtime_error("gls_op_set_outflow_target: null argument");
  const gls::OutflowFaces &F = op->faces;
  const size_t             m = (size_t)F.n * F.nqf * op->dim;
  if (!m)
    return 0;
  // pageable host source: copied and waited for (a per-time-step update)
  hipStream_t s = (hipStream_t)stream;
  if (op->prec == GLS_F64)
    HIP_THROW(hipMemcpyAsync(F.d_target, target, m * sizeof(double), hipMemcpyHostToDevice, s));
  else
    {
      std::vector<float> t(target, target + m);
      HIP_THROW(hipMemcpyAsync(F.d_target, t.data(), m * sizeof(float), hipMemcpyHostToDevice, s));
      HIP_THROW(hipStreamSynchronize(s));
    }
  HIP_THROW(hipStreamSynchronize(s));
  GLS_CATCH
}

} // extern "C"
