// sweeps.hip — launches of the resident smoothing-sweep kernel
// (gls::k_brick_sweeps, csrc/brick.h): FP32 3D Q2 levels, vmult modes
// Newton / fixed point, per brick geometry, default or deterministic
// lattice accumulation.  Its own translation unit so that gls_op.hip's
// instantiations and these compile in parallel.
#include "brick.h"

namespace gls
{
namespace
{
using SweepKernel = void (*)(BrickArgs<float, 3, 3>, SweepArgs);

template <int MODE, bool DET>
SweepKernel
sweep_kernel_m(int geo)
{
  if (geo == GEO_GEN)
    return &k_brick_sweeps<3, 2, float, MODE, GEO_GEN, DET>;
  if (geo == GEO_CART)
    return &k_brick_sweeps<3, 2, float, MODE, GEO_CART, DET>;
  return &k_brick_sweeps<3, 2, float, MODE, GEO_ANY, DET>;
}

SweepKernel
sweep_kernel(int mode, int geo, bool det)
{
  if (mode == MODE_NEWTON)
    return det ? sweep_kernel_m<MODE_NEWTON, true>(geo) : sweep_kernel_m<MODE_NEWTON, false>(geo);
  if (mode == MODE_FIXED)
    return det ? sweep_kernel_m<MODE_FIXED, true>(geo) : sweep_kernel_m<MODE_FIXED, false>(geo);
  return nullptr;
}
} // namespace

// workgroups of the sweep kernel resident at once on the device (every
// brick of a launch must be: a brick waits for its neighbours' sweeps).
// One workgroup per CU below the occupancy API's answer (which can admit one
// more than the hardware at high SGPR counts, MI355X_MICROARCH.md
// § Residency and cooperative launch).
int64_t
sweeps_capacity(int mode, int geo, bool det, size_t lds, int device)
{
  SweepKernel f = sweep_kernel(mode, geo, det);
  if (!f)
    return 0;
  int per_cu = 0, n_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(f),
                                                   BLOCK, lds) != hipSuccess)
    return 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return 0;
  return (int64_t)std::max(0, per_cu - 1) * n_cu;
}

void
launch_sweeps(const BrickArgs<float, 3, 3> &a, const SweepArgs &sw, int mode, int geo, bool det,
              size_t lds, hipStream_t s)
{
  SweepKernel f = sweep_kernel(mode, geo, det);
  if (!f)
    throw std::runtime_error("resident sweeps: no kernel for this mode");
  hipLaunchKernelGGL(f, dim3((unsigned)(a.brick_end - a.brick_begin)), dim3(BLOCK), lds, s, a,
                     sw);
  HIP_THROW(hipGetLastError());
}
} // namespace gls
