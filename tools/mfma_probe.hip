// mfma_probe.hip — does the sum-factorisation of k_brick belong on MFMA?
// (SURVEY §7.1 step 4).  A measurement tool, not part of
// the product library.
//
// Workload: the evaluate step of the Q2 cell loop (values and the three
// collocation gradients of 4 components at the 27 points of each cell,
// FEEvaluation::evaluate(values | gradients)), for N cells read from HBM,
// reduced to a per-lane checksum so that no output stream hides the compute.
//
//  k_sumfac<T> : what k_brick does — one lane per (cell, point), 2 cells per
//                wavefront, three 1-D sweeps through LDS for the values and
//                three collocation sweeps for the gradients (VALU FMAs).
//  k_dense_f32 : MFMA — the 108 x 27 dense cell operator [S⊗S⊗S; D⊗S⊗S;
//                S⊗D⊗S; S⊗S⊗D] times a 27 x 32 block of 8 cells x 4
//                components, v_mfma_f32_32x32x2_f32 (3x the flops of the
//                sum factorisation, no LDS sweeps).
//  k_dense_f64 : the same with v_mfma_f64_16x16x4_f64.
//
// The 1-D sum factorisation itself (3 x 3 contractions) cannot use MFMA
// usefully: K = 3 pads to 4 and one of M / N to 16, 14 % of the issued MACs.
//
// Build: make -C tools; run: tools/build/mfma_probe [n_cells] — prints one
// JSON line per kernel (median of 20 event-timed launches, checksums).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do                                                                                         \
    {                                                                                        \
      hipError_t e_ = (x);                                                                   \
      if (e_ != hipSuccess)                                                                  \
        {                                                                                    \
          std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
          std::exit(1);                                                                      \
        }                                                                                    \
    }                                                                                        \
  while (0)

// Gauss-Lobatto Q2 on [0,1] evaluated at 3-point Gauss: S[q][i]; collocation
// derivative at the Gauss points: D[q][p]
struct Basis
{
  double S[3][3], D[3][3];
  Basis()
  {
    const double x[3] = {0.0, 0.5, 1.0};
    const double g[3] = {0.5 - std::sqrt(0.15), 0.5, 0.5 + std::sqrt(0.15)};
    for (int q = 0; q < 3; ++q)
      for (int i = 0; i < 3; ++i)
        {
          double v = 1;
          for (int m = 0; m < 3; ++m)
            if (m != i)
              v *= (g[q] - x[m]) / (x[i] - x[m]);
          S[q][i] = v;
        }
    for (int q = 0; q < 3; ++q)
      for (int p = 0; p < 3; ++p)
        {
          // d/dx of the Lagrange polynomial through the Gauss points
          double s = 0;
          for (int m = 0; m < 3; ++m)
            {
              if (m == p)
                continue;
              double t = 1 / (g[p] - g[m]);
              for (int r = 0; r < 3; ++r)
                if (r != p && r != m)
                  t *= (g[q] - g[r]) / (g[p] - g[r]);
              s += t;
            }
          D[q][p] = s;
        }
  }
};

__constant__ double cS[3][3], cD[3][3];

// ---------------------------------------------------------------- sum factorisation
template <typename T>
__global__ void __launch_bounds__(256)
  k_sumfac(const T *__restrict__ u, T *__restrict__ out, int n_cells)
{
  __shared__ T buf[4][2][4][27 + 5]; // [wave][cell][comp][point] (+pad)
  __shared__ T tmp[4][2][4][27 + 5];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lc = lane / 27, p = lane % 27;
  const int cell = (blockIdx.x * 4 + wave) * 2 + lc;
  const bool act = lane < 54 && cell < n_cells;
  const int i = p % 3, j = (p / 3) % 3, l = p / 9;
  T S[3][3], D[3][3];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b)
      S[a][b] = (T)cS[a][b], D[a][b] = (T)cD[a][b];
  T acc = 0;
  if (lane < 54)
    for (int c = 0; c < 4; ++c)
      buf[wave][lc][c][p] = act ? u[((size_t)cell * 4 + c) * 27 + p] : T(0);
  __builtin_amdgcn_wave_barrier();
  auto sweep = [&](T (*src)[27 + 5], T (*dst)[27 + 5], const T (&M)[3][3], int dir) {
    if (lane < 54)
      for (int c = 0; c < 4; ++c)
        {
          T s = 0;
          for (int m = 0; m < 3; ++m)
            {
              const int pm = dir == 0 ? m + 3 * j + 9 * l : dir == 1 ? i + 3 * m + 9 * l : i + 3 * j + 9 * m;
              const int qa = dir == 0 ? i : dir == 1 ? j : l;
              s += M[qa][m] * src[c][pm];
            }
          dst[c][p] = s;
        }
    __builtin_amdgcn_wave_barrier();
  };
  // values: x, y, z sweeps (buf -> tmp -> buf -> tmp)
  sweep(buf[wave][lc], tmp[wave][lc], S, 0);
  sweep(tmp[wave][lc], buf[wave][lc], S, 1);
  sweep(buf[wave][lc], tmp[wave][lc], S, 2);
  if (act)
    for (int c = 0; c < 4; ++c)
      acc += tmp[wave][lc][c][p];
  // collocation gradients from the values in tmp
  for (int d = 0; d < 3; ++d)
    {
      sweep(tmp[wave][lc], buf[wave][lc], D, d);
      if (act)
        for (int c = 0; c < 4; ++c)
          acc += buf[wave][lc][c][p];
      __builtin_amdgcn_wave_barrier();
    }
  if (act)
    out[(size_t)cell * 27 + p] = acc;
}

// ---------------------------------------------------------------- dense MFMA f32
// A (the dense operator, 4 blocks of 32 rows x 28 k) in registers, loaded
// from a [blk][s][lane] table; B = 28 x 32 (k = point, column = cell * 4 + comp)
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void __launch_bounds__(256)
  k_dense_f32(const float *__restrict__ u, const float *__restrict__ Atab, float *__restrict__ out,
              int n_cells)
{
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 31, kh = lane >> 5;
  const int cell0 = (blockIdx.x * 4 + wave) * 8;
  const int cell  = cell0 + col / 4, comp = col % 4;
  float A[4][14];
  for (int b = 0; b < 4; ++b)
    for (int s = 0; s < 14; ++s)
      A[b][s] = Atab[(b * 14 + s) * 64 + lane];
  float B[14];
  for (int s = 0; s < 14; ++s)
    {
      const int k = 2 * s + kh;
      B[s] = (cell < n_cells && k < 27) ? u[((size_t)cell * 4 + comp) * 27 + k] : 0.f;
    }
  float acc = 0;
  for (int b = 0; b < 4; ++b)
    {
      f32x16 c = {};
      for (int s = 0; s < 14; ++s)
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(A[b][s], B[s], c, 0, 0, 0);
      for (int r = 0; r < 16; ++r)
        acc += c[r];
    }
  if (cell0 < n_cells)
    out[(size_t)(blockIdx.x * 4 + wave) * 64 + lane] = acc;
}

// ---------------------------------------------------------------- dense MFMA f64
typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256)
  k_dense_f64(const double *__restrict__ u, const double *__restrict__ Atab,
              double *__restrict__ out, int n_cells)
{
  // 16 x 16 x 4: rows = 16 points of one operator block (7 row tiles cover
  // 108 rows), k = 4 nodes (7 steps cover 28), columns = 4 cells x 4 comps
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 15, kq = lane >> 4;
  const int cell0 = (blockIdx.x * 4 + wave) * 4;
  const int cell  = cell0 + col / 4, comp = col % 4;
  double B[7];
  for (int s = 0; s < 7; ++s)
    {
      const int k = 4 * s + kq;
      B[s] = (cell < n_cells && k < 27) ? u[((size_t)cell * 4 + comp) * 27 + k] : 0.0;
    }
  double acc = 0;
  for (int t = 0; t < 7; ++t)
    {
      f64x4 c = {};
      for (int s = 0; s < 7; ++s)
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(Atab[(t * 7 + s) * 64 + lane], B[s], c, 0, 0, 0);
      for (int r = 0; r < 4; ++r)
        acc += c[r];
    }
  if (cell0 < n_cells)
    out[(size_t)(blockIdx.x * 4 + wave) * 64 + lane] = acc;
}

// dense operator rows: block b (0 values, 1..3 gradient d) at point q, node k
static double
dense(const Basis &B, int b, int q, int k)
{
  const int qi = q % 3, qj = (q / 3) % 3, ql = q / 9;
  const int ki = k % 3, kj = (k / 3) % 3, kl = k / 9;
  const double sx = B.S[qi][ki], sy = B.S[qj][kj], sz = B.S[ql][kl];
  if (b == 0)
    return sx * sy * sz;
  // collocation derivative of the interpolated values: sum_p D[q][p] S[p][k]
  double dx = 0, dy = 0, dz = 0;
  for (int m = 0; m < 3; ++m)
    {
      dx += B.D[qi][m] * B.S[m][ki];
      dy += B.D[qj][m] * B.S[m][kj];
      dz += B.D[ql][m] * B.S[m][kl];
    }
  return b == 1 ? dx * sy * sz : b == 2 ? sx * dy * sz : sx * sy * dz;
}

template <typename F>
static float
time_ms(F &&launch)
{
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w)
    launch();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < 20; ++r)
    {
      CK(hipEventRecord(a, 0));
      launch();
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      t.push_back(ms);
    }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return t[t.size() / 2];
}

template <typename T>
static double
sum_dev(const T *d, size_t n)
{
  std::vector<T> h(n);
  CK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
  double s = 0;
  for (T v : h)
    s += (double)v;
  return s;
}

int
main(int argc, char **argv)
{
  const int n_cells = argc > 1 ? std::atoi(argv[1]) : 204800;
  if (n_cells <= 0 || n_cells % 32 != 0)
    {
      std::fprintf(stderr, "n_cells must be a positive multiple of 32\n");
      return 2;
    }
  Basis B;
  CK(hipMemcpyToSymbol(HIP_SYMBOL(cS), B.S, sizeof(B.S)));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(cD), B.D, sizeof(B.D)));
  const size_t nu = (size_t)n_cells * 4 * 27;
  std::vector<double> uh(nu);
  uint64_t st = 0x9e3779b97f4a7c15ULL;
  for (auto &v : uh)
    {
      st ^= st << 13, st ^= st >> 7, st ^= st << 17;
      v = (double)(st >> 11) / 9007199254740992.0 - 0.5;
    }
  std::vector<float> uf(uh.begin(), uh.end());
  // dense tables in the MFMA A layouts
  std::vector<float> A32(4 * 14 * 64);
  for (int b = 0; b < 4; ++b)
    for (int s = 0; s < 14; ++s)
      for (int l = 0; l < 64; ++l)
        {
          const int row = l & 31, k = 2 * s + (l >> 5);
          A32[(b * 14 + s) * 64 + l] = (row < 27 && k < 27) ? (float)dense(B, b, row, k) : 0.f;
        }
  std::vector<double> A64(7 * 7 * 64);
  for (int t = 0; t < 7; ++t)
    for (int s = 0; s < 7; ++s)
      for (int l = 0; l < 64; ++l)
        {
          const int r = t * 16 + (l & 15), k = 4 * s + (l >> 4);
          const int b = r / 27, q = r % 27;
          A64[(t * 7 + s) * 64 + l] = (r < 108 && k < 27) ? dense(B, b, q, k) : 0.0;
        }
  float *du32, *dA32, *do32;
  double *du64, *dA64, *do64;
  const size_t nout = (size_t)n_cells * 27;
  CK(hipMalloc(&du32, nu * 4));
  CK(hipMalloc(&du64, nu * 8));
  CK(hipMalloc(&dA32, A32.size() * 4));
  CK(hipMalloc(&dA64, A64.size() * 8));
  CK(hipMalloc(&do32, nout * 4));
  CK(hipMalloc(&do64, nout * 8));
  CK(hipMemcpy(du32, uf.data(), nu * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(du64, uh.data(), nu * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA32, A32.data(), A32.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA64, A64.data(), A64.size() * 8, hipMemcpyHostToDevice));

  const double bytes32 = (double)nu * 4, bytes64 = (double)nu * 8;
  // flops: sum factorisation 3 value sweeps + 3 gradient sweeps of 27 x 3
  // MACs per component; dense 108 x 27 MACs per component
  const double f_sf = (double)n_cells * 4 * 6 * 27 * 3 * 2, f_dn = (double)n_cells * 4 * 108 * 27 * 2;
  auto report = [&](const char *name, const char *dtype, float ms, double flops, double bytes,
                    double checksum) {
    std::printf("{\"kernel\": \"%s\", \"dtype\": \"%s\", \"n_cells\": %d, \"us\": %.2f, "
                "\"ns_per_cell\": %.4f, \"useful_flops\": %.4g, \"tflops\": %.2f, "
                "\"input_GBps\": %.0f, \"checksum\": %.10g}\n",
                name, dtype, n_cells, ms * 1e3, ms * 1e6 / n_cells, flops, flops / (ms * 1e-3) / 1e12,
                bytes / (ms * 1e-3) / 1e9, checksum);
  };
  {
    CK(hipMemset(do32, 0, nout * 4));
    const dim3 g((unsigned)((n_cells + 7) / 8));
    const float ms = time_ms([&] { hipLaunchKernelGGL(k_sumfac<float>, g, dim3(256), 0, 0, du32, do32, n_cells); });
    CK(hipGetLastError());
    report("sumfac_lds_valu", "f32", ms, f_sf, bytes32, sum_dev(do32, nout));
  }
  {
    CK(hipMemset(do32, 0, nout * 4));
    const dim3 g((unsigned)(n_cells / 32));
    const float ms = time_ms([&] { hipLaunchKernelGGL(k_dense_f32, g, dim3(256), 0, 0, du32, dA32, do32, n_cells); });
    CK(hipGetLastError());
    report("dense_mfma_32x32x2_f32", "f32", ms, f_dn, bytes32, sum_dev(do32, (size_t)n_cells / 8 * 64));
  }
  {
    CK(hipMemset(do64, 0, nout * 8));
    const dim3 g((unsigned)((n_cells + 7) / 8));
    const float ms = time_ms([&] { hipLaunchKernelGGL(k_sumfac<double>, g, dim3(256), 0, 0, du64, do64, n_cells); });
    CK(hipGetLastError());
    report("sumfac_lds_valu", "f64", ms, f_sf, bytes64, sum_dev(do64, nout));
  }
  {
    CK(hipMemset(do64, 0, nout * 8));
    const dim3 g((unsigned)(n_cells / 16));
    const float ms = time_ms([&] { hipLaunchKernelGGL(k_dense_f64, g, dim3(256), 0, 0, du64, dA64, do64, n_cells); });
    CK(hipGetLastError());
    report("dense_mfma_16x16x4_f64", "f64", ms, f_dn, bytes64, sum_dev(do64, (size_t)n_cells / 4 * 64));
  }
  CK(hipFree(du32));
  CK(hipFree(du64));
  CK(hipFree(dA32));
  CK(hipFree(dA64));
  CK(hipFree(do32));
  CK(hipFree(do64));
  return 0;
}
