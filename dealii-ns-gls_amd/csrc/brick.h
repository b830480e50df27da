// brick.h — the production vmult / residual kernel (gfx950).
//
// Work decomposition: one 256-thread workgroup per BRICK, a block of
// bx*by*bz cells of one refined coarse cell (3D: 4x4x4 cells, Q2 -> a 9^3
// node lattice).  The workgroup
//   1. runs the brick's cells through the per-cell operator (sum
//      factorisation + GLS q-point physics, do_vmult_cell
//      operator_ns.cc:949-1182) in rounds of CPW cells per wavefront and adds
//      every cell's nodal result into an LDS accumulator lattice (LDS
//      atomics: cells of different wavefronts share lattice nodes);
//   2. writes the lattice out: nodes owned by this brick alone go straight to
//      dst (plain stores; dst is never zeroed), nodes on the brick boundary go
//      to a per-node-contiguous partial buffer that k_shared_reduce sums.  No
//      global atomics; bitwise reproducible up to the LDS-atomic order.
//      (distribute_local_to_global + compress(add) of the reference's
//      cell_loop and the identity rows of vmult, operator_ns.cc:702-721.)
//
// Thread map: one lane per (cell, quadrature point) = (cell, node) since
// FE_Q(k) and QGauss(k+1) both have (k+1)^dim points; a cell never straddles
// a wavefront (3D Q2: 2 cells = 54 of 64 lanes), so the LDS sum-factorisation
// sweeps are ordered by wavefront fences, not workgroup barriers.
// Occupancy: 3 waves/SIMD for the FP64 kernels with curved bricks (164
// VGPRs, 44 KB LDS per workgroup), 4 for the Cartesian FP64 and the FP32
// ones (BrickOcc).  Variants measured and not kept (persistent pipelined
// bricks, fused last-arriver reduction, ablation builds) are on the git tag
// r3-variants.
#pragma once

#include "common.h"
#include "kernels.h"


namespace gls
{
constexpr uint32_t SHARED_BIT  = 0x80000000u;
constexpr uint32_t UNUSED_NODE = 0x0FFFFFFFu; // lattice node outside a split brick

template <int dim>
struct BrickMax
{
  static constexpr int cells = dim == 3 ? 4 : 8; // cells per direction
};

template <int dim, int k, int ZL = 1>
struct BrickLattice
{
  // largest lattice the brick kernel takes: 3D bricks of up to 4x4xZL cells
  // (build_bricks runs 3D bricks as one-cell layers, ZL = 1, except the
  // two-layer FP32 bricks, ZL = 2), 2D up to 8x8 cells
  static constexpr int side = k * BrickMax<dim>::cells + 1;
  static constexpr int L    = dim == 3 ? side * side * (ZL * k + 1) : side * side;
  static constexpr bool fits = L <= 729;
};

// floor(i / d) for 0 <= i < 4096 and 1 <= d <= 729 from r = 1/d rounded to
// float: (i + 1/2) / d stays >= 0.5 / 729 away from an integer, more than
// the product's rounding error (< 4096 * 2^-23), so the truncation is exact.
// Three VALU operations instead of the ~18 of an integer division by a
// runtime divisor.
__device__ __forceinline__ int
idiv_f(int i, float r)
{
  return (int)(((float)i + 0.5f) * r);
}

// workgroup-scope atomic add on an LDS address (ds_add_f64 / ds_add_f32)
template <typename T>
__device__ __forceinline__ void
lds_add(T *p, T v)
{
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// multiplicity class of partial slot `slot` (the shared nodes are ordered by
// class, build_bricks): the node's slots are slot0 + j m + [0, m)
__device__ __forceinline__ int
slot_class(const ReduceClasses &rc, uint32_t slot)
{
  int kc = 0;
#pragma unroll
  for (int j = 1; j < ReduceClasses::MAX; ++j)
    if (j < rc.n && slot >= rc.slot0[j])
      kc = j;
  return kc;
}

// 16-byte LDS packs of solution components: the sum-factorisation sweeps
// move (dim+1) components as ceil((dim+1)/W) ds_read_b128 / ds_write_b128
// instead of one 8-byte access per component (and no ds_read2_b64, which
// moves 16 B at a quarter of ds_read_b128's rate, MI355X_MICROARCH §LDS).
// (Pack<T>: common.h)

template <typename T, int dim, int n>
struct BrickArgs
{
  const uint32_t *brick_nodes;  // [n_bricks][L] node | cmask << 28
  const uint32_t *brick_target; // [n_bricks][L] node, or SHARED_BIT | slot
  const uint32_t *brick_geo; // per brick: bit 0 curved (per-q geometry for all its
                             // cells) | number of cells << 8
  const uint32_t *brick_cell0;  // per brick: first cell
  const uint32_t *brick_chunk0; // per brick: first table chunk
  const T        *geo_cart;  // [dim+1][cell]               (cells of Cartesian bricks)
  const T        *geo_gen;   // [1+dim^2][plane][cell][line] (cells of curved bricks)
  const typename Pack<T>::V *tab_v; // tables: 16-byte field groups, a chunk per
                                    // wavefront round (group stride CPW * nq)
  int64_t         n_cells;
  const T        *cellwise;
  const T        *old_grad;
  T              *dst;
  const T        *src;
  T              *partial; // [slot][dim+1], slots of a node contiguous
  // fused damped-Jacobi step (PreconditionRelaxation::step of the multigrid
  // smoother): with rb set, dst = src + omega * rd * (rb - A src) instead of
  // A src (the smoother's separate k_relax pass over n dofs disappears)
  const T        *rb;
  const T        *rd;
  T               romega;
  int             rkeep; // 1: src + omega rd (rb - A src); 0: omega rd (rb - A src)
                         // (rd null: 1) — the multigrid residual b - A x
  // deferred shared-node reduction (FP32 3D smoothing levels):
  // with qslots set, src's brick-boundary rows are not in memory: each is
  // the previous apply's reduction, rebuilt in the gather exactly as
  // k_shared_reduce_cls would have written it -- its partial slots (qslots,
  // slot ranges from rc), the iterate before it (qprev) and that step's
  // relaxation (qb, qd, qomega, keep 1) -- and stored into src (qsrc_w)
  const T        *qslots;
  const T        *qprev;
  const T        *qb;
  const T        *qd;
  T               qomega;
  T              *qsrc_w;
  double         *out64; // FP32: the written rows also as FP64 (null: none)
  ReduceClasses   rc;
  int64_t         brick_begin, brick_end;
  int             bx, by, bz;
  int             L, Lx, Ly;
  int             PLx, PLy, LP; // padded LDS lattice strides / size (>= L)
  // reciprocals of Lx, Lx Ly, bx, bx by for exact float quotients (idiv_f)
  float           rLx, rLxy, rbx, rbxy;
  T               nu, w0, theta, stau;
  T               nu4, stau2; // 4 nu, stau^2 (delta_qwise_fast)
  int             td, cw, have_prev, have_old_grad;
  int             det; // deterministic lattice accumulation (GLS_DETERMINISTIC): k_brick<..., DET>
  Shape<T, n>     sh;
};

// 1D coefficient tables in LDS: S, S^T, Dq, Dq^T, each row padded to whole
// 16-byte packs (RP values) so that a lane's row M[pa][*] (or M[*][pa]) is
// one ds_read_b128 (+ one ds_read_b64 for Q2 FP64) instead of
// ds_read2_b64 + ds_read_b64 on 24-byte rows
template <typename T, int n>
struct CoefRow
{
  static constexpr int W  = 16 / (int)sizeof(T);
  static constexpr int RP = (n + W - 1) / W * W; // padded row length
};
enum
{
  TAB_S = 0,
  TAB_ST,
  TAB_D,
  TAB_DT
};

// coefficient row of a lane, read once into registers and applied to every
// component pack (the LDS stores of a sweep may alias the tables, so
// reading M inside the pack loop would re-read it after every store)
template <int n, typename T>
__device__ __forceinline__ void
coefs(const T *tab, int pa, T (&c)[n])
{
  using CR         = CoefRow<T, n>;
  using V          = typename Pack<T>::V;
  const V *row     = reinterpret_cast<const V *>(tab + pa * CR::RP);
#pragma unroll
  for (int g = 0; g < CR::RP / CR::W; ++g)
    {
      V v = row[g];
      // FP32 rows are one 16-byte pack of which n = 3 values are used: keep
      // the load a ds_read_b128 (4 LDS cycles) instead of the ds_read_b96 the
      // compiler narrows it to (8 cycles, MI355X_MICROARCH §LDS)
      if constexpr (sizeof(T) == 4)
        asm volatile("" : "+v"(v));
#pragma unroll
      for (int w = 0; w < CR::W; ++w)
        if (g * CR::W + w < n)
          c[g * CR::W + w] = v[w];
    }
}

template <int n, typename T, typename V>
__device__ __forceinline__ V
contract_c(const V *in, const T (&c)[n], int base, int s)
{
  V acc = c[0] * in[base];
#pragma unroll
  for (int j = 1; j < n; ++j)
    acc += c[j] * in[base + j * s];
  return acc;
}

template <int n, typename T, typename V>
__device__ __forceinline__ V
contract_v(const V *in, const T *tab, int pa, int base, int s)
{
  T c[n];
  coefs<n>(tab, pa, c);
  return contract_c<n>(in, c, base, s);
}

// x contractions across lanes (3D Q2, round 6).  The lanes of a wavefront
// hold 18 x-lines of 3 quadrature points (2 cells x 9 lines), five lines per
// 16-lane DPP row (lane 16 r + 3 s + x; the 16th lane of every row and the
// last 6 lanes of the wave idle: 54 of 64 busy, as before).  A contraction
// along x, out(x) = sum_j M[x][j] in(j), then reads the line's other points
// from the neighbouring lanes by DPP row shifts (row_shr / row_shl by 1 and
// 2: never across a row, so never across a line's row) instead of from the
// LDS sweep buffer: five taps k_d = M[x][x+d] (zero where x+d leaves the
// line), applied in the order d = -2..2, which is the order j = 0..2 of the
// LDS form -- the same FMA chain, bitwise, since the zero taps add +-0.  The
// x sweeps of evaluate (from the src lattice), of the collocation gradient,
// of the Dq^T test-function sweep and of the S^T sweep that feeds the
// lattice accumulation leave LDS: per round 3 fewer dependent LDS round
// trips and a quarter fewer LDS instructions.  Measured and NOT adopted
// (profiles/r06/explore/ab_xline_dpp.txt): the DPP shifts cost what the LDS
// traffic saved (FP32: 27.3 us at 4 waves, spill-free, against 26.2 us for
// the LDS sweeps at 5 waves; FP64 needs 3 waves to avoid spills, -7 %), so
// the kernels are not bound by LDS throughput.  GLS_XDPP_F32 / _F64 = 1
// build the x-line kernels (parity-tested: tests/test_gpu_parity.py,
// tests/test_a_gpu_configs.py, 44 passed).
#ifndef GLS_XDPP_F32
#define GLS_XDPP_F32 0
#endif
#ifndef GLS_XDPP_F64
#define GLS_XDPP_F64 0
#endif
// L2 prefetch of the next round's tables (round 6 experiment): in the
// prologue every wave of a FOUR kernel pulls the cache lines of its round-1
// Newton table chunk into the L2 with one LDS-DMA dword load per line
// (global_load_lds_dword into a 256-byte landing area nobody reads: no
// registers held), so the round's LATE loads hit the L2 instead of the MALL /
// HBM.  Measured and NOT adopted: 6-13 % slower, FP64 and FP32
// (profiles/r06/explore/ab_l2_prefetch.txt): round 1's tables are not the
// critical path.  GLS_TAB_PREFETCH=1 builds it.
#ifndef GLS_TAB_PREFETCH
#define GLS_TAB_PREFETCH 0
#endif
// Non-temporal stores of the brick write-out (dst rows and partial slots;
// round 6 experiment): the 20 MB an r2 FP64 vmult writes stream out instead of
// staying dirty in the L2s until the kernel's end.  Measured and NOT adopted
// (profiles/r06/explore/ab_nt_store.txt): r2 FP64 33.0 -> 36.9 us, r3 FP64
// 238 -> 345 us, FP32 r2 23.0 -> 24.0 us.  GLS_NT_STORE=1 builds it.
#ifndef GLS_NT_STORE
#define GLS_NT_STORE 0
#endif

template <int dim, int k, typename T>
__host__ __device__ constexpr bool
xdpp()
{
  return dim == 3 && k == 2 && (sizeof(T) == 4 ? GLS_XDPP_F32 : GLS_XDPP_F64);
}

// value of lane + D (D = -2, -1, 1, 2) within the lane's 16-lane row, 0 past
// the row's ends (DPP row_shr / row_shl, bound_ctrl: zero)
template <int D>
__device__ __forceinline__ float
row_shift(float v)
{
  constexpr int ctrl = D < 0 ? 0x110 - D : 0x100 + D;
  return __builtin_bit_cast(
    float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, 0xF, 0xF, true));
}
template <int D>
__device__ __forceinline__ double
row_shift(double v)
{
  typedef int I2 __attribute__((ext_vector_type(2)));
  constexpr int ctrl = D < 0 ? 0x110 - D : 0x100 + D;
  I2            u    = __builtin_bit_cast(I2, v);
  u.x                = __builtin_amdgcn_update_dpp(0, u.x, ctrl, 0xF, 0xF, true);
  u.y                = __builtin_amdgcn_update_dpp(0, u.y, ctrl, 0xF, 0xF, true);
  return __builtin_bit_cast(double, u);
}

// out(x) = sum_d k[d + 2] v(x + d) over the lane's x-line, every component of
// a pack; executed by every lane of the wavefront (idle lanes hold finite
// values: they only ever meet zero taps)
template <typename T, typename V, int W>
__device__ __forceinline__ V
xline(const V &v, const T (&kk)[5])
{
  V r;
#pragma unroll
  for (int w = 0; w < W; ++w)
    {
      T a = kk[0] * row_shift<-2>(v[w]);
      a += kk[1] * row_shift<-1>(v[w]);
      a += kk[2] * v[w];
      a += kk[3] * row_shift<1>(v[w]);
      a += kk[4] * row_shift<2>(v[w]);
      r[w] = a;
    }
  return r;
}

// the five taps of table `tab` for a lane at x (LDS rows of 8 values: one
// ds_read_b128 + one ds_read_b32 for FP32, two b128 + one b64 for FP64)
constexpr int TAPS = 8;
template <int n, typename T>
__device__ __forceinline__ void
taps5(const T *s_tap, int tab, int x, T (&kk)[5])
{
  using V      = typename Pack<T>::V;
  constexpr int W = Pack<T>::W;
  const T *row = s_tap + (tab * n + x) * TAPS;
#pragma unroll
  for (int g = 0; g < 4 / W; ++g)
    {
      const V v = reinterpret_cast<const V *>(row)[g];
#pragma unroll
      for (int w = 0; w < W; ++w)
        kk[g * W + w] = v[w];
    }
  kk[4] = row[4];
}

// Sweep-buffer layout of one cell (in packs): point (x, y, z) at
// x + PY y + PZ z, component pack kp at + kp KS, ping-pong halves A | B,
// cells WB apart.  3D Q2 is padded (FP64: PY 4, PZ 13, KS 37, WB 151): with the
// ds_read_b128 lane groups of MI355X_MICROARCH §LDS this takes the sweep
// reads from 7.0 to 4.3 LDS cycles per instruction (4 = conflict free;
// exhaustive search over PY, PZ, KS, WB of the exact lane/address map).
// With the x-line lane map (X) only the y and z sweeps read the buffers:
// PY 3, PZ 10, KS 29 is conflict free for both precisions in the same model
// (scripts/lds_layout_search.py --xdpp), 40 % less LDS for FP32.
template <int dim, int n, int NP, bool X = false>
struct BufLayout
{
  static constexpr bool pad  = dim == 3 && n == 3 && NP == 2 && !X;
  // FP32 (one pack per point): same search, 6.0 -> 4.3 modelled cycles per
  // sweep read (scripts/lds_layout_search.py)
  static constexpr bool pad1 = dim == 3 && n == 3 && NP == 1 && !X;
  static constexpr int  PY   = X ? 3 : pad ? 4 : pad1 ? 3 : n;
  static constexpr int  PZ   = X ? 10 : pad ? 13 : pad1 ? 20 : n * n;
  static constexpr int  KS   = X ? 29 : pad ? 37 : pad1 ? 49 : ipow(n, dim);
  static constexpr int  WB   = X ? (NP == 1 ? 61 : 125) : pad ? 151 : pad1 ? 107 : 2 * NP * ipow(n, dim);
};

// dynamic LDS of one workgroup: src lattice packs | sweep buffers |
// accumulator lattice | coefficient tables (S, S^T, Dq, Dq^T; padded rows)
template <int dim, int k, typename T>
struct BrickLDS
{
  static constexpr int n   = k + 1;
  static constexpr int nq  = ipow(n, dim);
  static constexpr int nc  = dim + 1;
  static constexpr int W   = Pack<T>::W;
  static constexpr int NP  = (nc + W - 1) / W;
  static constexpr int CPW = 64 / nq > 0 ? 64 / nq : 1;
  static constexpr bool X  = xdpp<dim, k, T>();
  static constexpr int WB  = BufLayout<dim, n, NP, X>::WB; // per-cell sweep buffer (packs)
  static constexpr int WPB = BLOCK / 64;
  static constexpr int ORG = 64; // cell-origin table entries (cells per brick)
  static constexpr int NTAP = X ? 4 * n * TAPS : 0; // x-line taps (values)
  static constexpr int PF   = GLS_TAB_PREFETCH ? 256 : 0; // L2-prefetch landing bytes
  static size_t
  bytes(int L) // L: padded LDS lattice size
  {
    return 16 * ((size_t)NP * L + (size_t)WPB * CPW * WB) + tab_offset(L) +
           sizeof(T) * (NTAP + 4 * n * CoefRow<T, n>::RP) + sizeof(int) * ORG + PF;
  }
  __host__ __device__ static size_t
  tab_offset(int L) // accumulator bytes (FP64 for both precisions) rounded up to 16
  {
    return (sizeof(double) * (size_t)nc * L + 15) / 16 * 16;
  }
};

// Table formulation of the brick kernel (the tables hold
// the reference's per-q fields, operator_ns.h:120-132, plus T1 and h): the
// Newton vmult streams T1 (Fields::T1, the linearization-point part of R1,
// formed once per linearization point and time weights by k_finalize_t1)
// instead of grad P* and Ut_old, and recomputes the q-wise delta_1 /
// delta_2 from U and h at the q point (delta_qwise_fast, the producer's
// expression) instead of streaming them: 16 instead of the reference's 20
// values per q (round 2: r3 283 -> 272 us), and the register budget that
// lets the Cartesian kernel run 4 waves per SIMD (round 3).
// q-wise delta_1 / delta_2 recomputed in the kernel: the Q2 Newton vmult
// only (its sqrt / division temporaries push other instantiations over their
// register budget)
template <int k, int MODE>
__host__ __device__ constexpr bool
delta_otf()
{
  return MODE == MODE_NEWTON && k == 2;
}

// the table fields a brick vmult / residual of MODE streams: Newton U, grad U,
// T1 and h (or delta_1/2); fixed-point U and delta_1/2; residual also
// Ut_old.  Groups of 16 bytes with none of these are not loaded.
// (GLS_EXP_NO_UGU: timing-only build that skips U and grad U -- wrong
// results; the bound on what recomputing them in the kernel could gain)
#ifndef GLS_EXP_NO_UGU
#define GLS_EXP_NO_UGU 0
#endif
template <int dim, int MODE, int k = 2>
__host__ __device__ constexpr bool
field_read(int f)
{
  using F         = Fields<dim>;
  const bool d12  = f == F::D1 || f == F::D2;
  const bool u    = !GLS_EXP_NO_UGU && f >= F::U && f < F::U + dim;
  const bool h    = f == F::H;
  const bool ut   = f >= F::UT && f < F::UT + dim;
  const bool gu   = !GLS_EXP_NO_UGU && f >= F::GU && f < F::GU + dim * dim;
  const bool t1   = f >= F::T1 && f < F::T1 + dim;
  return (delta_otf<k, MODE>() ? h : d12) || u || (MODE == MODE_NEWTON && (gu || t1)) ||
         (MODE == MODE_RESIDUAL && ut);
}

// a 16-byte group whose only Newton fields are U_t (read when the time
// derivative is considered): loaded only when the runtime flag td says so
template <int dim, int MODE, int k = 2>
__host__ __device__ constexpr bool
group_ut_only(int g, int W)
{
  using F  = Fields<dim>;
  bool any = false, other = false;
  for (int w = 0; w < W; ++w)
    {
      const int f = g * W + w;
      if (!field_read<dim, MODE, k>(f))
        continue;
      any = true;
      other = other || !(f >= F::UT && f < F::UT + dim);
    }
  return MODE == MODE_NEWTON && any && !other;
}

// Geometry of a launch's bricks (build_bricks spreads the curved bricks
// evenly over the XCD runs of each segment): GEO_CART bricks hold
// one diagonal J^{-1} and det J per cell, GEO_GEN bricks J^{-1} and JxW per
// q point, GEO_ANY reads the type per brick (brick_geo bit 0).
enum
{
  GEO_ANY  = 0,
  GEO_CART = 1,
  GEO_GEN  = 2
};

// everything one lane needs from HBM for one (cell, q point)
template <int dim, typename T, int MODE>
struct LaneData
{
  static constexpr int NOLD = MODE == MODE_RESIDUAL ? dim * dim + dim : 1;
  T    inv[dim][dim];
  T    JxW; // as loaded: JxW (curved) or det J (Cartesian); see jxw()
  T    U[dim], GU[dim][dim], T1[dim], UT[dim], oldg[NOLD];
  T    h, d1, d2; // h: q-wise delta from U on the fly (delta_otf)
  bool active;
};

// Every load here is independent of every other and of the lane's other
// loads in flight (no data-dependent branch: the geometry type is per brick,
// read in the prologue), so the whole set issues back to back and is waited
// for once, at the q-point physics.
template <int dim, int k, typename T, int MODE, int GEO>
__device__ __forceinline__ void
load_lane(const BrickArgs<T, dim, k + 1> &a, int64_t cell0, int64_t chunk0, int ncell,
          bool general, int lcell, bool in_wave, int p, const int (&pa)[3],
          LaneData<dim, T, MODE> &r)
{
  constexpr int  n   = k + 1;
  constexpr int  nq  = ipow(n, dim);
  constexpr int  CPW = 64 / nq > 0 ? 64 / nq : 1;
  constexpr bool R   = MODE == MODE_RESIDUAL;
  constexpr int  W   = Pack<T>::W;
  using V            = typename Pack<T>::V;
  using F            = Fields<dim>;
  constexpr int NG   = (F::N + W - 1) / W;
  r.active           = in_wave && lcell < ncell;
  // inactive lanes (the 64 % nq left-over lanes, cells past the brick's
  // end) load the brick's first cell instead of zero-filling ~30 registers
  // per round: finite values, and JxW = 0 below keeps them out of the sums
  if (!r.active)
    lcell = 0;
  const int64_t cell = cell0 + lcell;
  const int64_t nqc  = a.n_cells * nq;
  if (GEO == GEO_CART) // (the Cartesian path reads the diagonal only)
#pragma unroll
    for (int i = 0; i < dim; ++i)
#pragma unroll
      for (int e = 0; e < dim; ++e)
        r.inv[i][e] = 0;
  // geometry (MatrixFree-style compressed: Cartesian per cell, else per q).
  // loaded values stay untouched here: any arithmetic on them (the
  // quadrature weight, the inactive-lane mask) would make the compiler wait
  // for the loads at the prefetch point (an s_waitcnt vmcnt(0) in the middle
  // of the round); jxw() applies both at the point of use
  if (GEO == GEO_ANY)
    {
      // mixed meshes: one load per entry whatever the brick's type, only the
      // address selected, and no branch around a load: a VALU write into a
      // register that the other branch loads makes the waitcnt pass wait
      // for every load issued before it -- the src gather among them --
      // before this round's tables are even issued.  Cartesian bricks read
      // their off-diagonal entries (never used) from distinct fixed
      // addresses (identical addresses would be merged into one load and a
      // copy, which waits for it).
      const int64_t gq = qindex<dim, n>(cell, p, a.n_cells);
      r.JxW            = *(general ? a.geo_gen + gq : a.geo_cart + dim * a.n_cells + cell);
#pragma unroll
      for (int i = 0; i < dim; ++i)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          r.inv[i][e] = *(general ? a.geo_gen + (1 + i * dim + e) * nqc + gq :
                          i == e  ? a.geo_cart + i * a.n_cells + cell :
                                    a.geo_cart + (i * dim + e));
    }
  else if (GEO == GEO_GEN)
    {
      const int64_t gq = qindex<dim, n>(cell, p, a.n_cells);
      r.JxW            = a.geo_gen[gq];
#pragma unroll
      for (int i = 0; i < dim; ++i)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          r.inv[i][e] = a.geo_gen[(1 + i * dim + e) * nqc + gq];
    }
  else
    {
#pragma unroll
      for (int i = 0; i < dim; ++i)
        r.inv[i][i] = a.geo_cart[i * a.n_cells + cell];
      r.JxW = a.geo_cart[dim * a.n_cells + cell];
    }
  // per-q tables (operator_ns.h:120-132): the round's CPW cells form one
  // chunk, each 16-byte field group of it one contiguous wave load; the
  // groups a mode reads are fixed at compile time, except that a group of
  // U_t values only is skipped (uniform branch) without the time derivative
  // (other fields a runtime flag switches off are loaded and ignored)
  constexpr int GS = CPW * nq; // group stride in packs
  const V *tv = a.tab_v + (chunk0 + lcell / CPW) * (NG * GS) + (lcell % CPW) * nq + p;
  T        tf[NG * W];
#pragma unroll
  for (int g = 0; g < NG; ++g)
    {
      bool any = false;
#pragma unroll
      for (int w = 0; w < W; ++w)
        any = any || field_read<dim, MODE, k>(g * W + w);
      V v = {};
      if (any && (!group_ut_only<dim, MODE, k>(g, W) || a.td))
        v = tv[g * GS];
#pragma unroll
      for (int w = 0; w < W; ++w)
        tf[g * W + w] = v[w];
    }
#pragma unroll
  for (int d = 0; d < dim; ++d)
    {
      r.U[d]  = tf[F::U + d];
      r.T1[d] = tf[F::T1 + d];
      r.UT[d] = tf[F::UT + d];
#pragma unroll
      for (int e = 0; e < dim; ++e)
        r.GU[d][e] = tf[F::GU + d * dim + e];
    }
#pragma unroll
  for (int i = 0; i < LaneData<dim, T, MODE>::NOLD; ++i)
    r.oldg[i] = 0;
  if (R && a.have_old_grad)
    {
      const int64_t tq = qindex<dim, n>(cell, p, a.n_cells);
#pragma unroll
      for (int i = 0; i < LaneData<dim, T, MODE>::NOLD; ++i)
        r.oldg[i] = a.old_grad[i * nqc + tq];
    }
  if (a.cw)
    {
      r.d1 = a.cellwise[cell];
      r.d2 = a.cellwise[a.n_cells + cell];
    }
  else
    {
      r.d1 = tf[F::D1];
      r.d2 = tf[F::D2];
    }
  r.h = tf[F::H];
}

// JxW of a lane at its quadrature point: the loaded JxW (curved bricks) or
// det J times the tensor quadrature weight (Cartesian), zero on inactive
// lanes (they stay out of every sum)
template <int dim, int k, typename T, int MODE>
__device__ __forceinline__ T
jxw(const LaneData<dim, T, MODE> &r, bool general, const Shape<T, k + 1> &sh, const int (&pa)[3])
{
  T w = sh.w[pa[0]] * sh.w[pa[1]];
  if (dim == 3)
    w *= sh.w[pa[2]];
  const T j = general ? r.JxW : r.JxW * w;
  return r.active ? j : T(0);
}

template <typename V, typename T, int nc, int NP, int W>
__device__ __forceinline__ void
to_packs(const T (&x)[nc], V (&v)[NP])
{
#pragma unroll
  for (int kp = 0; kp < NP; ++kp)
#pragma unroll
    for (int w = 0; w < W; ++w)
      v[kp][w] = kp * W + w < nc ? x[kp * W + w] : T(0);
}

// Occupancy.  The FP64 3D Q2 vmult kernels (Newton, fixed point) with
// one-layer bricks run 4 waves/SIMD (<= 128 VGPRs, unpadded 34 KB lattice: 4
// workgroups per CU) for Cartesian AND curved bricks: the round loop is
// compiled once per brick geometry (a GEO_ANY launch branches per brick,
// wave-uniformly), and
//  * a Cartesian brick issues a round's tables and its diagonal J^{-1} / det J
//    at the start of that round (LATE: in flight during the evaluate sweeps);
//  * a curved brick issues its tables and per-q J^{-1} / JxW after the
//    evaluate sweeps (AT_USE: nothing in flight across them) and parks J^{-1}
//    in its own sweep-buffer slots (free between the evaluate and the
//    integrate sweeps) from the real-space gradients to the test-function
//    transform, so the physics holds no more registers than the Cartesian
//    one's.  Scheduling barriers keep the compiler from hoisting those loads
//    and the LDS reload back into the evaluate sweeps / the physics.
// (Round 4 had one mixed-geometry body: 164 VGPRs, 3 waves; forced to 4 it
// spilled 140 B/lane and took 63.7 instead of 40.2 us at r2.)  The other
// instantiations (FP64 residual, two-layer bricks, other degrees) keep the
// earlier prefetch (issued behind the previous round's Dq^T sweeps) at 3
// waves; the FP32 kernels fit 4 waves with it.
// (GLS_XD_WAVES_F32 / _F64: the occupancy of the x-line kernels, brick.h
// xline, for A/B builds)
#ifndef GLS_XD_WAVES_F32
#define GLS_XD_WAVES_F32 4
#endif
#ifndef GLS_XD_WAVES_F64
#define GLS_XD_WAVES_F64 3
#endif
template <int dim, int k, typename T, int MODE, int GEO, int ZL = 1>
struct BrickOcc
{
  static constexpr bool four  = dim == 3 && k == 2 && MODE != MODE_RESIDUAL && ZL == 1;
  static constexpr bool X     = xdpp<dim, k, T>();
  static constexpr int  waves = four ? (sizeof(T) == 4 ? (X ? GLS_XD_WAVES_F32 : 5) :
                                                         (X ? GLS_XD_WAVES_F64 : 4)) :
                                       (sizeof(T) == 4 ? 4 : 3);
};

// DET: the deterministic lattice accumulation (GLS_DETERMINISTIC: the cells
// of a round add in cell order between barriers instead of by LDS atomics;
// its own instantiation, so the default kernels keep their registers)
template <int dim, int k, typename T, int MODE, int GEO = GEO_ANY, int ZL = 1, bool DET = false>
__global__ void __launch_bounds__(BLOCK, (BrickOcc<dim, k, T, MODE, GEO, ZL>::waves))
  k_brick(BrickArgs<T, dim, k + 1> a)
{
  if constexpr (GEO == GEO_ANY && BrickOcc<dim, k, T, MODE, GEO, ZL>::four)
    {
      // the round loop compiled once per brick geometry (BrickOcc)
      const int brick = (int)a.brick_begin + (int)blockIdx.x;
      if (brick >= (int)a.brick_end)
        return;
      if (a.brick_geo[brick] & 1u) // (wave-uniform: per brick)
        {
          constexpr int G = GEO_GEN;
#include "brick_body.inc"
        }
      else
        {
          constexpr int G = GEO_CART;
#include "brick_body.inc"
        }
    }
  else
    {
      constexpr int G = GEO;
#include "brick_body.inc"
    }
}

// Resident smoothing sweeps (mg.hip smooth; FP32 3D levels with deferred
// reductions whose bricks are all resident at once, csrc/sweeps.hip): the
// damped-Jacobi steps of one smoothing sequence in ONE launch, one
// workgroup per brick for all of them.  A workgroup keeps its brick's node
// ids and the iterate, b and D^{-1} at its lattice nodes in registers across
// the sweeps.  Between sweeps no kernel boundary and no counter: a brick
// publishes its shared nodes' partial sums as tagged granules and its
// neighbours rebuild those nodes as soon as the tags of their slots read
// the previous sweep.
struct SweepArgs
{
  float          *vec[2];   // sweep j reads vec[j & 1], writes vec[(j + 1) & 1] (last sweep only)
  float          *slots[2]; // the last sweep's partial slots: slots[j & 1] (plain)
  uint64_t       *gran[2];  // the other sweeps': gran[j & 1], [slot][component] {value, tag}
  uint32_t        gran_bytes;
  uint32_t       *err;      // granule waits that hit the spin bound
  uint32_t       *flag;     // host-mapped word set to 1 on such a wait (the host
                            // reads it without a synchronisation, gls::sweep_stalled)
  uint32_t        epoch;    // tags before this launch (sweep j tags epoch + j + 1)
  int             nsweep;
  int             spin_max; // polls of a slot before the wait gives up
  uint64_t       *timing;   // GLS_SWEEP_TIMING builds: [brick][sweep][6] clock stamps
};
#ifndef GLS_SWEEP_TIMING
#define GLS_SWEEP_TIMING 0
#endif
constexpr int SWEEP_MAX_MULT = 11;      // bricks per shared node (two groups of 4 + 3)
constexpr int SWEEP_MAX_L    = 128;     // lattice nodes per brick (a thread pair per node)
// a slot that never arrives: counted, not waited for (SweepArgs.spin_max,
// by default SWEEP_SPIN_MAX_DEFAULT of common.h; gls_op_set_sweep_spin_bound)

// one node's partial sums as 8-byte {value, tag} granules, two per 16-byte
// write-through (sc1) store (each 8-byte half is written whole)
__device__ __forceinline__ void
store_granules(uint64_t *base, uint32_t bytes, uint32_t slot, uint32_t tag, const float (&u)[4])
{
  using U4 = __attribute__((ext_vector_type(4))) unsigned int;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000);
  const U4   g0   = {__float_as_uint(u[0]), tag, __float_as_uint(u[1]), tag};
  const U4   g1   = {__float_as_uint(u[2]), tag, __float_as_uint(u[3]), tag};
  __builtin_amdgcn_raw_buffer_store_b128(g0, rsrc, (int)(slot * 32u), 0, 16);
  __builtin_amdgcn_raw_buffer_store_b128(g1, rsrc, (int)(slot * 32u + 16u), 0, 16);
}

// 3 waves/SIMD (<= 168 VGPRs): the sweep loop keeps its uniform kernel
// arguments in SGPRs across iterations (SGPR spills go to VGPR lanes); at 4
// waves the mixed-geometry kernels spilled to scratch.  The levels it runs
// (a few hundred bricks) fill fewer slots than 3 workgroups per CU give.
template <int dim, int k, typename T, int MODE, int GEO = GEO_ANY, bool DET = false>
__global__ void __launch_bounds__(BLOCK, 3)
  k_brick_sweeps(BrickArgs<T, dim, k + 1> a, SweepArgs sw)
{
  constexpr int ZL = 1;
  if constexpr (GEO == GEO_ANY && BrickOcc<dim, k, T, MODE, GEO, ZL>::four)
    {
      // one body per brick geometry, as k_brick's (the same arithmetic)
      if (a.brick_geo[(int)a.brick_begin + (int)blockIdx.x] & 1u)
        {
          constexpr int G = GEO_GEN;
#include "brick_sweeps.inc"
        }
      else
        {
          constexpr int G = GEO_CART;
#include "brick_sweeps.inc"
        }
    }
  else
    {
      constexpr int G = GEO;
#include "brick_sweeps.inc"
    }
}

// Sum the per-brick partials of every brick-boundary node (one contiguous
// slot run per node); constrained components get the identity row (vmult,
// operator_ns.cc:719-721) or zero (evaluate_residual's set_zero, :678).
// One thread per (shared node, component): consecutive threads touch
// consecutive doubles of a node's partials and of dst.
template <typename T, int nc, bool R>
__global__ void __launch_bounds__(256)
  k_shared_reduce(T *__restrict__ dst, const T *__restrict__ src,
                  const T *__restrict__ partial, const uint32_t *__restrict__ nodes,
                  const uint32_t *__restrict__ offsets, int64_t n_shared,
                  const T *__restrict__ rb = nullptr, const T *__restrict__ rd = nullptr,
                  T romega = T(0), int keep = 1, uint32_t n_relax = 0xFFFFFFFFu)
{
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n_shared * nc)
    return;
  const int64_t  s      = gid / nc;
  const int      c      = (int)(gid - s * nc);
  const uint32_t b      = offsets[s], e = offsets[s + 1];
  const uint32_t packed = nodes[s];
  // the slot loads of a node are independent: issue them four at a time
  // (a plain loop waits one memory latency per slot)
  const T *pp = partial + c;
  T        sum = 0;
  uint32_t i   = b;
  for (; i + 4 <= e; i += 4)
    {
      const T x0 = pp[(size_t)i * nc], x1 = pp[(size_t)(i + 1) * nc];
      const T x2 = pp[(size_t)(i + 2) * nc], x3 = pp[(size_t)(i + 3) * nc];
      sum += (x0 + x1) + (x2 + x3);
    }
  if (i + 2 <= e)
    {
      const T x0 = pp[(size_t)i * nc], x1 = pp[(size_t)(i + 1) * nc];
      sum += x0 + x1;
      i += 2;
    }
  if (i < e)
    sum += pp[(size_t)i * nc];
  const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
  if ((cm >> c) & 1)
    sum = R ? T(0) : src[(size_t)node * nc + c];
  if (!R && rb && node < n_relax)
    {
      const size_t j = (size_t)node * nc + c;
      sum            = (keep ? src[j] : T(0)) + romega * (rd ? rd[j] : T(1)) * (rb[j] - sum);
    }
  dst[(size_t)node * nc + c] = sum;
}

// Same reduction with the shared nodes ordered by brick multiplicity
// (build_bricks): the slots of node s of class (first, m, slot0) are
// slot0 + (s - first) * m + [0, m), computed, not loaded, so the slot loads
// issue together with the node id load (one memory round trip, not two).
template <typename T, int nc, bool R>
__global__ void __launch_bounds__(256)
  k_shared_reduce_cls(T *__restrict__ dst, const T *__restrict__ src,
                      const T *__restrict__ partial, const uint32_t *__restrict__ nodes,
                      const ReduceClasses rc, int64_t n_shared,
                      const T *__restrict__ rb = nullptr, const T *__restrict__ rd = nullptr,
                      T romega = T(0), int keep = 1, uint32_t n_relax = 0xFFFFFFFFu,
                      double *__restrict__ out64 = nullptr)
{
  // 16-byte packs when a node's row is whole packs (nc = 4): one thread per
  // (node, pack), vector loads and stores
  using V            = typename Pack<T>::V;
  constexpr int W    = Pack<T>::W;
  constexpr int NPK  = nc % W == 0 ? nc / W : 0;
  if constexpr (NPK > 0)
    {
      const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
      if (gid >= n_shared * NPK)
        return;
      const uint32_t s  = (uint32_t)(gid / NPK);
      const int      kp = (int)(gid - (int64_t)s * NPK);
      int            k  = 0;
#pragma unroll
      for (int j = 1; j < ReduceClasses::MAX; ++j)
        if (j < rc.n && s >= rc.first[j])
          k = j;
      const uint32_t m      = rc.mult[k];
      const uint32_t b      = rc.slot0[k] + (s - rc.first[k]) * m;
      const uint32_t packed = nodes[s];
      const V       *pp     = reinterpret_cast<const V *>(partial) + kp;
      V              sum    = {};
      uint32_t       i      = 0;
      for (; i + 4 <= m; i += 4)
        {
          const V x0 = pp[(size_t)(b + i) * NPK], x1 = pp[(size_t)(b + i + 1) * NPK];
          const V x2 = pp[(size_t)(b + i + 2) * NPK], x3 = pp[(size_t)(b + i + 3) * NPK];
          sum += (x0 + x1) + (x2 + x3);
        }
      if (i + 2 <= m)
        {
          const V x0 = pp[(size_t)(b + i) * NPK], x1 = pp[(size_t)(b + i + 1) * NPK];
          sum += x0 + x1;
          i += 2;
        }
      if (i < m)
        sum += pp[(size_t)(b + i) * NPK];
      const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
      if (cm)
#pragma unroll
        for (int w = 0; w < W; ++w)
          if ((cm >> (kp * W + w)) & 1)
            sum[w] = R ? T(0) : src[(size_t)node * nc + kp * W + w];
      if (!R && rb && node < n_relax)
        {
          const size_t j  = (size_t)node * NPK + kp;
          const V      xs = keep ? reinterpret_cast<const V *>(src)[j] : V{};
          const V      dj = rd ? reinterpret_cast<const V *>(rd)[j] : V{} + T(1);
          sum = xs + romega * dj * (reinterpret_cast<const V *>(rb)[j] - sum);
        }
      reinterpret_cast<V *>(dst)[(size_t)node * NPK + kp] = sum;
      if (out64)
#pragma unroll
        for (int w = 0; w < W; ++w)
          out64[(size_t)node * nc + kp * W + w] = (double)sum[w];
      return;
    }
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n_shared * nc)
    return;
  const uint32_t s = (uint32_t)(gid / nc);
  const int      c = (int)(gid - (int64_t)s * nc);
  int            k = 0;
#pragma unroll
  for (int j = 1; j < ReduceClasses::MAX; ++j)
    if (j < rc.n && s >= rc.first[j])
      k = j;
  const uint32_t m      = rc.mult[k];
  const uint32_t b      = rc.slot0[k] + (s - rc.first[k]) * m;
  const uint32_t packed = nodes[s];
  const T       *pp     = partial + c;
  T              sum    = 0;
  uint32_t       i      = 0;
  for (; i + 4 <= m; i += 4)
    {
      const T x0 = pp[(size_t)(b + i) * nc], x1 = pp[(size_t)(b + i + 1) * nc];
      const T x2 = pp[(size_t)(b + i + 2) * nc], x3 = pp[(size_t)(b + i + 3) * nc];
      sum += (x0 + x1) + (x2 + x3);
    }
  if (i + 2 <= m)
    {
      const T x0 = pp[(size_t)(b + i) * nc], x1 = pp[(size_t)(b + i + 1) * nc];
      sum += x0 + x1;
      i += 2;
    }
  if (i < m)
    sum += pp[(size_t)(b + i) * nc];
  const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
  if ((cm >> c) & 1)
    sum = R ? T(0) : src[(size_t)node * nc + c];
  if (!R && rb && node < n_relax)
    {
      const size_t j = (size_t)node * nc + c;
      sum            = (keep ? src[j] : T(0)) + romega * (rd ? rd[j] : T(1)) * (rb[j] - sum);
    }
  dst[(size_t)node * nc + c] = sum;
  if (out64)
    out64[(size_t)node * nc + c] = (double)sum;
}

// resident smoothing sweeps (csrc/sweeps.hip): workgroups resident at once,
// and one launch over bricks [a.brick_begin, a.brick_end)
int64_t sweeps_capacity(int mode, int geo, bool det, size_t lds, int device);
void    launch_sweeps(const BrickArgs<float, 3, 3> &a, const SweepArgs &sw, int mode, int geo,
                      bool det, size_t lds, hipStream_t s);

} // namespace gls
