// common.h — shared host helpers of libglsamd.so (error handling, 1D basis).
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace gls
{
void set_error(const std::string &s);

#define HIP_THROW(expr)                                                                      \
  do                                                                                         \
    {                                                                                        \
      const hipError_t e_ = (expr);                                                          \
      if (e_ != hipSuccess)                                                                  \
        throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_));         \
    }                                                                                        \
  while (0)

// every C-ABI function body is wrapped in these: exceptions -> status 1 +
// thread-local message (the reference's AssertThrow becomes a status code)
#define GLS_TRY \
  try           \
    {
#define GLS_CATCH                                 \
  }                                               \
  catch (const std::exception &ex_)               \
    {                                             \
      gls::set_error(ex_.what());                 \
      return 1;                                   \
    }                                             \
  return 0;

// the caller's current device switched to `device` for a scope and restored
// on every exit path (C-ABI calls that allocate or launch on an operator's
// device leave the caller's device as they found it)
struct DeviceScope
{
  int prev = -1;
  explicit DeviceScope(int device)
  {
    HIP_THROW(hipGetDevice(&prev));
    if (prev != device)
      HIP_THROW(hipSetDevice(device));
  }
  ~DeviceScope()
  {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev)
      (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope &)            = delete;
  DeviceScope &operator=(const DeviceScope &) = delete;
};

// what a brick launch runs: the brick kernel, and the shared-node reduction
// of the owned rows, of the ghost rows (a partitioned operator's export
// block), or of both
enum
{
  BRICK_RUN          = 1,
  BRICK_REDUCE_OWNED = 2,
  BRICK_REDUCE_GHOST = 4,
  BRICK_REDUCE       = BRICK_REDUCE_OWNED | BRICK_REDUCE_GHOST
};

// polls of a partial-slot granule before a resident sweep's wait gives up
// (brick.h k_brick_sweeps; gls_op_set_sweep_spin_bound changes it per operator)
constexpr int SWEEP_SPIN_MAX_DEFAULT = 1 << 18;

// multiplicity classes of the brick-boundary nodes (k_shared_reduce_cls)
struct ReduceClasses
{
  static constexpr int MAX = 16;
  int                  n   = 0; // classes; -1: too many (offset-table kernel)
  uint32_t             first[MAX + 1];
  uint32_t             mult[MAX];
  uint32_t             slot0[MAX];
};

// FE_Q(k) on Gauss-Lobatto points, QGauss(k+1), on [0,1]
struct Basis1D
{
  int                 n = 0;
  std::vector<double> nodes, qp, qw;
  std::vector<double> S;  // S[q*n+i]  = phi_i(x_q)
  std::vector<double> D;  // D[q*n+i]  = phi_i'(x_q)
  std::vector<double> Dq; // Dq[q*n+j] = l_j'(x_q), l_j Lagrange on Gauss points
  explicit Basis1D(int k);
};

// 16-byte vector of solution components (4 FP32 or 2 FP64): the brick
// kernels' LDS packs and node loads, the reduction's slot sums
template <typename T>
struct Pack;
template <>
struct Pack<double>
{
  typedef double V __attribute__((ext_vector_type(2)));
  static constexpr int W = 2;
};
template <>
struct Pack<float>
{
  typedef float V __attribute__((ext_vector_type(4)));
  static constexpr int W = 4;
};

} // namespace gls
