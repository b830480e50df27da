// cgs.h — Gram-Schmidt kernels of the device GMRES (krylov.hip, single
// domain) and of the partitioned GMRES (dist_mg.hip): fused CGS2 passes over
// the Krylov basis with per-block partials summed in a fixed order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace
{
// v = w / |w| with the norm read on the device (|w| = 0, the lucky
// breakdown: v = 0, never used); the same 1/hn multiply as a host dscal
__global__ void
k_unit_col(double *__restrict__ v, const double *__restrict__ w, const double *__restrict__ hn,
           int64_t n)
{
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const double  h = *hn;
  if (i < n)
    v[i] = h > 0 ? w[i] * (1.0 / h) : 0.0;
}

// Fused CGS2 for the restart lengths GMRES runs by default (j + 1 <= 32
// basis columns): three streaming passes over the basis instead of four
// rocBLAS GEMVs plus a norm, each thread holding its rows' basis entries in
// registers between the update and the next dots.
//   k_cgs_dots:   part = V^T w                         (pass 1)
//   k_cgs_update: w -= V h; part = V^T w  (or |w|^2)   (passes 2, 3)
// Per-block partials (fixed row ranges) are summed in a fixed order by
// k_cgs_finish: the result does not depend on scheduling.
constexpr int CGS_MAXJ   = 32;
constexpr int CGS_BLOCKS = 512; // 1024 measured slower (update 24.1 -> 27.4 us)
constexpr int CGS_PART   = CGS_BLOCKS * CGS_MAXJ; // partials buffer (doubles)

__device__ __forceinline__ void
cgs_block_store(double (&acc)[CGS_MAXJ], int J, double *__restrict__ part)
{
  __shared__ double red[4][CGS_MAXJ];
  const int         lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < CGS_MAXJ; ++c)
    if (c < J) // uniform: a skipped column costs a branch, not its shuffles
      {
        double v = acc[c];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
          v += __shfl_down(v, off);
        if (lane == 0)
          red[wv][c] = v;
      }
  __syncthreads();
  if (threadIdx.x < J)
    {
      const int c = threadIdx.x;
      part[(size_t)blockIdx.x * CGS_MAXJ + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    }
}

__global__ void __launch_bounds__(256)
  k_cgs_dots(const double *__restrict__ V, int J, const double *__restrict__ w,
             double *__restrict__ part, int64_t n, int64_t ld)
{
  double acc[CGS_MAXJ];
#pragma unroll
  for (int c = 0; c < CGS_MAXJ; ++c)
    acc[c] = 0;
  const int64_t per = (n + CGS_BLOCKS - 1) / CGS_BLOCKS;
  const int64_t r0 = blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x)
    {
      // all of the row's basis loads issued before the first FMA
      double v[CGS_MAXJ];
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        v[c] = c < J ? V[(size_t)c * ld + i] : 0.0;
      const double wi = w[i];
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        acc[c] += v[c] * wi;
    }
  cgs_block_store(acc, J, part);
}

// w -= V h (h on the device) over rows [0, n); then the dots of the updated w
// with the basis (norm = 0), its squared norm into partial 0 (norm = 1), or
// both: the dots into partials [0, J) and the squared norm into partial J
// (norm = 2, J < CGS_MAXJ), over rows [0, n_dot) (a partitioned vector: its
// owned rows)
__global__ void __launch_bounds__(256)
  k_cgs_update(const double *__restrict__ V, int J, const double *__restrict__ h,
               double *__restrict__ w, double *__restrict__ part, int64_t n, int64_t n_dot,
               int64_t ld, int norm)
{
  double acc[CGS_MAXJ], hc[CGS_MAXJ], nrm = 0;
#pragma unroll
  for (int c = 0; c < CGS_MAXJ; ++c)
    {
      acc[c] = 0;
      hc[c]  = c < J ? h[c] : 0.0;
    }
  const int64_t per = (n + CGS_BLOCKS - 1) / CGS_BLOCKS;
  const int64_t r0 = blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x)
    {
      double v[CGS_MAXJ];
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        v[c] = c < J ? V[(size_t)c * ld + i] : 0.0;
      double wi = w[i], t = 0;
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        t += v[c] * hc[c];
      wi -= t;
      w[i] = wi;
      if (i >= n_dot)
        continue;
      if (norm == 1)
        acc[0] += wi * wi;
      else
        {
#pragma unroll
          for (int c = 0; c < CGS_MAXJ; ++c)
            acc[c] += v[c] * wi; // v[c] = 0 for c >= J
          if (norm == 2)
            nrm += wi * wi;
        }
    }
  if (norm == 2)
#pragma unroll
    for (int c = 0; c < CGS_MAXJ; ++c)
      if (c == J)
        acc[c] = nrm;
  cgs_block_store(acc, norm == 1 ? 1 : norm == 2 ? J + 1 : J, part);
}

// The second CGS pass's update folded into the normalisation: v = (w - V h)
// / |w - V h| with h = V^T w (the re-orthogonalisation coefficients) and the
// norm from Pythagoras, |w - V h|^2 = |w|^2 - |h|^2 (V orthonormal; h is
// O(eps |w|), so the subtraction loses nothing): one pass over the basis
// instead of an update pass, a norm reduction and a scaling pass.  h[0, J)
// and |w|^2 = h[J] on the device (k_cgs_update norm = 2 + k_cgs_finish);
// block 0 writes the norm to *hn for the Hessenberg column.
__global__ void __launch_bounds__(256)
  k_cgs_unit(const double *__restrict__ V, int J, const double *__restrict__ h, const double *w,
             double *v, double *__restrict__ hn, int64_t n, int64_t ld, // v may be w
             const double *__restrict__ col = nullptr, double *__restrict__ host = nullptr,
             int n_col = 0, int hn_at = 0)
{
  double hc[CGS_MAXJ];
  double h2 = 0;
#pragma unroll
  for (int c = 0; c < CGS_MAXJ; ++c)
    {
      hc[c] = c < J ? h[c] : 0.0;
      h2 += hc[c] * hc[c];
    }
  const double nw = h[J] - h2;
  const double nn = sqrt(nw > 0 ? nw : 0.0);
  if (blockIdx.x == 0 && threadIdx.x == 0)
    *hn = nn;
  // the Hessenberg column (col[0, n_col), the norm at hn_at) stored straight
  // into mapped pinned host memory: no device-to-host copy on the stream
  if (host && blockIdx.x == 0)
    for (int i = threadIdx.x; i < n_col; i += blockDim.x)
      host[i] = i == hn_at ? nn : col[i];
  const double  sc  = nn > 0 ? 1.0 / nn : 0.0;
  const int64_t per = (n + CGS_BLOCKS - 1) / CGS_BLOCKS;
  const int64_t r0 = blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x)
    {
      double vr[CGS_MAXJ];
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        vr[c] = c < J ? V[(size_t)c * ld + i] : 0.0;
      double t = 0;
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        t += vr[c] * hc[c];
      v[i] = (w[i] - t) * sc;
    }
}

// out[c] = sum over blocks of part[b][c] in a fixed order: one workgroup
// per column c = blockIdx.x (two partials per thread, fixed shuffle tree);
// sqrt_out: out[0] = sqrt(sum) (the norm)
__global__ void __launch_bounds__(256)
  k_cgs_finish(const double *__restrict__ part, double *__restrict__ out, int sqrt_out)
{
  static_assert(CGS_BLOCKS == 512, "two partials per thread");
  __shared__ double red[4];
  const int    c = blockIdx.x, t = threadIdx.x;
  double       s = part[(size_t)t * CGS_MAXJ + c] + part[(size_t)(t + 256) * CGS_MAXJ + c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    s += __shfl_down(s, off);
  if ((t & 63) == 0)
    red[t >> 6] = s;
  __syncthreads();
  if (t == 0)
    {
      const double v = (red[0] + red[1]) + (red[2] + red[3]);
      out[c]         = sqrt_out ? sqrt(v) : v;
    }
}

// ---- delayed CGS2 (DCGS2; Bielich, Langou, Thomas, Swirydowicz, Yamazaki,
// Boman, "Low-synch Gram-Schmidt with delayed reorthogonalization for
// Krylov solvers", Parallel Computing 2022): the re-orthogonalisation of the
// tentative basis vector u_j is delayed into the next Arnoldi step and merged
// with the projection of w_j = A M^{-1} u_j, one reduction and two basis
// passes per step instead of three passes (krylov.hip derives the Hessenberg
// entries).  Dots of step j, stride DCGS_W per block:
//   [0, 32): s = Q^T u_j   [32, 64): z = Q^T w_j   64: u_j.u_j   65: u_j.w_j
// and, on the device after the update: 66 alpha_j  67 h_jj  68 |u_{j+1}|^2.
constexpr int DCGS_W   = 2 * CGS_MAXJ + 2;
constexpr int DCGS_D   = DCGS_W + 3; // dots + alpha, h_jj, nu
constexpr int DCGS_PART = CGS_BLOCKS * DCGS_W;

__device__ __forceinline__ bool
dcgs_col_used(int c, int J)
{
  return c >= 2 * CGS_MAXJ || (c & (CGS_MAXJ - 1)) < J;
}

// pass 1: s = Q^T u, z = Q^T w (J columns of Q), u.u, u.w (w null: only
// s and u.u, the end of a cycle)
__global__ void __launch_bounds__(256)
  k_dcgs_dots(const double *__restrict__ V, int J, const double *__restrict__ u,
              const double *__restrict__ w, double *__restrict__ part, int64_t n, int64_t ld)
{
  double as[CGS_MAXJ], az[CGS_MAXJ], b = 0, g = 0;
#pragma unroll
  for (int c = 0; c < CGS_MAXJ; ++c)
    as[c] = az[c] = 0;
  const int64_t per = (n + CGS_BLOCKS - 1) / CGS_BLOCKS;
  const int64_t r0 = blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x)
    {
      double v[CGS_MAXJ];
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        v[c] = c < J ? V[(size_t)c * ld + i] : 0.0;
      const double ui = u[i], wi = w ? w[i] : 0.0;
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        {
          as[c] += v[c] * ui;
          az[c] += v[c] * wi;
        }
      b += ui * ui;
      g += ui * wi;
    }
  __shared__ double red[4][DCGS_W];
  const int         lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < DCGS_W; ++c)
    if (dcgs_col_used(c, J))
      {
        double x = c < CGS_MAXJ ? as[c] : c < 2 * CGS_MAXJ ? az[c - CGS_MAXJ] : c == 2 * CGS_MAXJ ? b : g;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
          x += __shfl_down(x, off);
        if (lane == 0)
          red[wv][c] = x;
      }
  __syncthreads();
  for (int c = threadIdx.x; c < DCGS_W; c += blockDim.x)
    if (dcgs_col_used(c, J))
      part[(size_t)blockIdx.x * DCGS_W + c] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}

// d[c] = sum over the blocks of part[b][c] (stride `stride`) in a fixed
// order, one workgroup per column c = blockIdx.x (unused DCGS columns: 0)
// (J < 0: every column used.)  host: a one-column launch (the norm of the
// new tentative vector, out at d[out]) also stores d[0, DCGS_D) into mapped
// pinned host memory, the step's record for the host
__global__ void __launch_bounds__(256)
  k_dcgs_finish(const double *__restrict__ part, double *__restrict__ d, int J, int out = -1,
                double *__restrict__ host = nullptr)
{
  static_assert(CGS_BLOCKS == 512, "two partials per thread");
  __shared__ double red[4];
  const int c = blockIdx.x, t = threadIdx.x, o = out >= 0 ? out : c;
  if (J >= 0 && !dcgs_col_used(c, J))
    {
      if (t == 0)
        d[o] = 0;
      return;
    }
  double s = part[(size_t)t * DCGS_W + c] + part[(size_t)(t + 256) * DCGS_W + c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    s += __shfl_down(s, off);
  if ((t & 63) == 0)
    red[t >> 6] = s;
  __syncthreads();
  const double v = (red[0] + red[1]) + (red[2] + red[3]);
  if (t == 0)
    d[o] = v;
  if (host)
    for (int i = t; i < DCGS_D; i += blockDim.x)
      host[i] = i == o ? v : d[i];
}

// pass 2: q_j = (u_j - Q s) / alpha_j, alpha_j = sqrt(u_j.u_j - |s|^2)
// (Pythagoras), written over u_j; the next tentative vector
// u_{j+1} = (w_j - Q z - q_j h_jj) / alpha_j with h_jj = (u_j.w_j - s.z) /
// alpha_j, and the partials of |u_{j+1}|^2.  Block 0 stores alpha_j, h_jj
// (d[66], d[67]).  J = 0: q_0 = u_0 / |u_0|.
__global__ void __launch_bounds__(256)
  k_dcgs_update(const double *__restrict__ V, int J, double *__restrict__ d, double *q,
                const double *__restrict__ w, double *__restrict__ un,
                double *__restrict__ part, int64_t n, int64_t ld)
{
  double sc[CGS_MAXJ], zc[CGS_MAXJ], s2 = 0, sz = 0;
#pragma unroll
  for (int c = 0; c < CGS_MAXJ; ++c)
    {
      sc[c] = c < J ? d[c] : 0.0;
      zc[c] = c < J ? d[CGS_MAXJ + c] : 0.0;
      s2 += sc[c] * sc[c];
      sz += sc[c] * zc[c];
    }
  const double a2    = d[2 * CGS_MAXJ] - s2;
  const double alpha = sqrt(a2 > 0 ? a2 : 0.0);
  const double ia    = alpha > 0 ? 1.0 / alpha : 0.0;
  const double hjj   = (d[2 * CGS_MAXJ + 1] - sz) * ia;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    {
      d[DCGS_W]     = alpha;
      d[DCGS_W + 1] = hjj;
    }
  double        nu  = 0;
  const int64_t per = (n + CGS_BLOCKS - 1) / CGS_BLOCKS;
  const int64_t r0 = blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x)
    {
      double vr[CGS_MAXJ];
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        vr[c] = c < J ? V[(size_t)c * ld + i] : 0.0;
      double ts = 0, tz = 0;
#pragma unroll
      for (int c = 0; c < CGS_MAXJ; ++c)
        {
          ts += vr[c] * sc[c];
          tz += vr[c] * zc[c];
        }
      const double qi = (q[i] - ts) * ia;
      const double ui = (w[i] - tz - qi * hjj) * ia;
      q[i]            = qi;
      un[i]           = ui;
      nu += ui * ui;
    }
  __shared__ double red[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    nu += __shfl_down(nu, off);
  if ((threadIdx.x & 63) == 0)
    red[threadIdx.x >> 6] = nu;
  __syncthreads();
  if (threadIdx.x == 0)
    part[(size_t)blockIdx.x * DCGS_W] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- wide forms of the two DCGS2 basis passes (round 6): 512-thread
// blocks (8 waves; CGS_BLOCKS of them, the partial layout of k_dcgs_dots /
// k_dcgs_update, so k_dcgs_finish is unchanged) and 16-byte loads, a lane
// holding two consecutive rows.  Valid for an even row count and leading
// dimension (16-byte aligned columns); krylov.hip takes the narrow forms
// otherwise.
constexpr int DCGS_WIDE = 512;

// rows [r0, r1) of block b, r0 even
__device__ __forceinline__ void
dcgs_rows(int64_t n, int64_t &r0, int64_t &r1)
{
  const int64_t per = (((n + CGS_BLOCKS - 1) / CGS_BLOCKS) + 1) & ~(int64_t)1;
  r0                = blockIdx.x * per;
  r1                = r0 + per < n ? r0 + per : n;
}

// pass 1 (k_dcgs_dots), wide: the 8 waves of a block split its rows in two
// halves and the columns in four groups (wave v: row half v / 4, columns
// c = v % 4 + 4 k, k < 8), each keeping 2 x 8 accumulators (the narrow form
// kept all 64 in every thread: 2 waves per SIMD) and streaming u and w over
// its half (each read by 4 waves, the re-reads L2 hits), the basis once, in
// 16-byte loads; the two halves' sums of a column meet in LDS.  u.u and u.w
// from the column-group-0 waves.
__global__ void __launch_bounds__(DCGS_WIDE)
  k_dcgs_dots_wide(const double *__restrict__ V, int J, const double *__restrict__ u,
                   const double *__restrict__ w, double *__restrict__ part, int64_t n, int64_t ld)
{
  using D2         = __attribute__((ext_vector_type(2))) double;
  constexpr int NG = 4, NK = CGS_MAXJ / NG; // column groups, columns per group
  __shared__ double red[2][DCGS_W];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cg = wv % NG, half = wv / NG;
  double    as[NK], az[NK], b = 0, g = 0;
#pragma unroll
  for (int k = 0; k < NK; ++k)
    as[k] = az[k] = 0;
  int64_t r0, r1;
  dcgs_rows(n, r0, r1);
  // the block's row pairs split in two contiguous halves
  const int64_t np = (r1 - r0 + 1) / 2, hp = (np + 1) / 2;
  const int64_t h0 = r0 + 2 * (half * hp), h1 = half ? r1 : (r0 + 2 * hp < r1 ? r0 + 2 * hp : r1);
  for (int64_t i = h0 + 2 * lane; i < h1; i += 128)
    {
      const D2 u2 = *reinterpret_cast<const D2 *>(u + i);
      const D2 w2 = w ? *reinterpret_cast<const D2 *>(w + i) : D2{0.0, 0.0};
      D2       v2[NK];
#pragma unroll
      for (int k = 0; k < NK; ++k)
        {
          const int c = cg + NG * k;
          v2[k]       = c < J ? *reinterpret_cast<const D2 *>(V + (size_t)c * ld + i) : D2{0.0, 0.0};
        }
#pragma unroll
      for (int k = 0; k < NK; ++k)
        {
          as[k] += v2[k][0] * u2[0];
          as[k] += v2[k][1] * u2[1];
          az[k] += v2[k][0] * w2[0];
          az[k] += v2[k][1] * w2[1];
        }
      if (cg == 0)
        {
          b += u2[0] * u2[0];
          b += u2[1] * u2[1];
          g += u2[0] * w2[0];
          g += u2[1] * w2[1];
        }
    }
#pragma unroll
  for (int k = 0; k < NK; ++k)
    {
      const int c = cg + NG * k;
      if (c >= J)
        continue; // wave-uniform
      double xs = as[k], xz = az[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1)
        {
          xs += __shfl_down(xs, off);
          xz += __shfl_down(xz, off);
        }
      if (lane == 0)
        {
          red[half][c]            = xs;
          red[half][CGS_MAXJ + c] = xz;
        }
    }
  if (cg == 0)
    {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1)
        {
          b += __shfl_down(b, off);
          g += __shfl_down(g, off);
        }
      if (lane == 0)
        {
          red[half][2 * CGS_MAXJ]     = b;
          red[half][2 * CGS_MAXJ + 1] = g;
        }
    }
  __syncthreads();
  double *pb = part + (size_t)blockIdx.x * DCGS_W;
  for (int c = threadIdx.x; c < DCGS_W; c += blockDim.x)
    if (dcgs_col_used(c, J))
      pb[c] = red[0][c] + red[1][c];
}

// pass 2 (k_dcgs_update), wide: the step's coefficients s, z in LDS (one
// broadcast ds_read_b128 per column instead of 64 registers), rows
// interleaved over the 8 waves in 16-byte pairs, columns in groups of 8
// loads in flight
__global__ void __launch_bounds__(DCGS_WIDE)
  k_dcgs_update_wide(const double *__restrict__ V, int J, double *__restrict__ d, double *q,
                     const double *__restrict__ w, double *__restrict__ un,
                     double *__restrict__ part, int64_t n, int64_t ld)
{
  using D2 = __attribute__((ext_vector_type(2))) double;
  __shared__ D2     coef[CGS_MAXJ]; // {s_c, z_c}
  __shared__ double red[DCGS_WIDE / 64];
  __shared__ double scal[3];        // 1 / alpha, h_jj
  if (threadIdx.x < CGS_MAXJ)
    {
      const int c    = threadIdx.x;
      coef[c]        = c < J ? D2{d[c], d[CGS_MAXJ + c]} : D2{0.0, 0.0};
    }
  if (threadIdx.x == 0)
    {
      // the same arithmetic (and order) as k_dcgs_update
      double s2 = 0, sz = 0;
      for (int c = 0; c < CGS_MAXJ; ++c)
        {
          const double sc = c < J ? d[c] : 0.0, zc = c < J ? d[CGS_MAXJ + c] : 0.0;
          s2 += sc * sc;
          sz += sc * zc;
        }
      const double a2    = d[2 * CGS_MAXJ] - s2;
      const double alpha = sqrt(a2 > 0 ? a2 : 0.0);
      const double ia    = alpha > 0 ? 1.0 / alpha : 0.0;
      scal[0]            = ia;
      scal[1]            = (d[2 * CGS_MAXJ + 1] - sz) * ia;
      if (blockIdx.x == 0)
        {
          d[DCGS_W]     = alpha;
          d[DCGS_W + 1] = scal[1];
        }
    }
  __syncthreads();
  const double ia = scal[0], hjj = scal[1];
  const int    wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double       nu = 0;
  int64_t      r0, r1;
  dcgs_rows(n, r0, r1);
  for (int64_t i = r0 + 2 * (lane + 64 * wv); i < r1; i += 2 * DCGS_WIDE)
    {
      D2 ts = {0.0, 0.0}, tz = {0.0, 0.0};
#pragma unroll 1
      for (int c0 = 0; c0 < J; c0 += 8)
        {
          D2 v2[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            v2[k] = c0 + k < J ? *reinterpret_cast<const D2 *>(V + (size_t)(c0 + k) * ld + i)
                               : D2{0.0, 0.0};
#pragma unroll
          for (int k = 0; k < 8; ++k)
            {
              const D2 cf = coef[c0 + k < CGS_MAXJ ? c0 + k : 0];
              const double s = c0 + k < J ? cf[0] : 0.0, z = c0 + k < J ? cf[1] : 0.0;
              ts += v2[k] * s;
              tz += v2[k] * z;
            }
        }
      const D2 q2 = *reinterpret_cast<const D2 *>(q + i);
      const D2 w2 = *reinterpret_cast<const D2 *>(w + i);
      const D2 qi = (q2 - ts) * ia;
      const D2 ui = (w2 - tz - qi * hjj) * ia;
      *reinterpret_cast<D2 *>(q + i)  = qi;
      *reinterpret_cast<D2 *>(un + i) = ui;
      nu += ui[0] * ui[0];
      nu += ui[1] * ui[1];
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    nu += __shfl_down(nu, off);
  if (lane == 0)
    red[wv] = nu;
  __syncthreads();
  if (threadIdx.x == 0)
    {
      double t = 0;
      for (int k = 0; k < DCGS_WIDE / 64; ++k)
        t += red[k];
      part[(size_t)blockIdx.x * DCGS_W] = t;
    }
}

// v = w / sqrt(|w|^2) with the squared norm read on the device (the
// partitioned GMRES all-reduces |w|^2 before the root)
__global__ void
k_unit_col_sq(double *__restrict__ v, const double *__restrict__ w,
              const double *__restrict__ hn2, int64_t n)
{
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const double  h = sqrt(*hn2 > 0 ? *hn2 : 0.0);
  if (i < n)
    v[i] = h > 0 ? w[i] * (1.0 / h) : 0.0;
}
} // namespace
