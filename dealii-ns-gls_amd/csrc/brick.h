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
// Occupancy is the lever (the kernel is LDS-latency bound at low wave
// counts): 3 waves/SIMD (FP64, 162 VGPRs, 44 KB LDS per workgroup).
// Software-pipelining the next round's loads was measured and gave nothing.
#pragma once

#include "common.h"
#include "kernels.h"


namespace gls
{
constexpr uint32_t SHARED_BIT  = 0x80000000u;
constexpr uint32_t UNUSED_NODE = 0x0FFFFFFFu; // lattice node outside a split brick

// GLS_STAMPS: diagnostic timeline build (never the product library): lane 0
// of every wave records s_memrealtime (100 MHz) at phase boundaries of each
// brick into g_stamps[brick][wave][8].
#ifdef GLS_STAMPS
constexpr size_t GLS_STAMP_MAX = 16384 * 4 * 8;
__device__ unsigned long long g_stamps[GLS_STAMP_MAX];
#define GLS_STAMP(brick, i)                                                                   \
  do                                                                                         \
    {                                                                                        \
      const size_t si_ = ((size_t)(brick) * (BLOCK / 64) + (threadIdx.x >> 6)) * 8 + (i);    \
      if ((threadIdx.x & 63) == 0 && si_ < GLS_STAMP_MAX)                                    \
        g_stamps[si_] = __builtin_amdgcn_s_memrealtime();                                    \
    }                                                                                        \
  while (0)
#else
#define GLS_STAMP(brick, i)                                                                   \
  do                                                                                         \
    {                                                                                        \
    }                                                                                        \
  while (0)
#endif

template <int dim>
struct BrickMax
{
  static constexpr int cells = dim == 3 ? 4 : 8; // cells per direction
};

#ifndef GLS_BRICK_MAXZ
#define GLS_BRICK_MAXZ 1
#endif
template <int dim, int k>
struct BrickLattice
{
  // largest lattice the brick kernel takes: 3D bricks of up to 4x4x1 cells
  // (build_bricks runs 3D bricks as one-cell layers; GLS_BRICK_MAXZ layers in
  // variant builds), 2D up to 8x8 cells
  static constexpr int side = k * BrickMax<dim>::cells + 1;
  static constexpr int L    = dim == 3 ? side * side * (k * GLS_BRICK_MAXZ + 1) : side * side;
  static constexpr bool fits = L <= 729;
};

// workgroup-scope atomic add on an LDS address (ds_add_f64 / ds_add_f32)
template <typename T>
__device__ __forceinline__ void
lds_add(T *p, T v)
{
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// 16-byte LDS packs of solution components: the sum-factorisation sweeps
// move (dim+1) components as ceil((dim+1)/W) ds_read_b128 / ds_write_b128
// instead of one 8-byte access per component (and no ds_read2_b64, which
// moves 16 B at a quarter of ds_read_b128's rate, MI355X_MICROARCH §LDS).
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
  int64_t         brick_begin, brick_end;
  int             bx, by, bz;
  int             L, Lx, Ly;
  int             PLx, PLy, LP; // padded LDS lattice strides / size (>= L)
  T               nu, w0, theta, stau;
  int             td, cw, have_prev, have_old_grad;
  // fused shared-node reduction (single-domain full vmult): per shared node
  // an arrival counter (zero between launches); the brick whose arrival
  // completes a node sums its partial slots and writes dst there, instead of
  // k_shared_reduce_cls.  null: partial slots only.
  uint32_t       *counters;
  uint32_t        partial_bytes;
  ReduceClasses   rc;
  Shape<T, n>     sh;
};

// partial slots of the fused reduction: written through to memory (sc1) and
// read back the same way, so a brick on another XCD sees them once the
// writer's arrival is counted (MI355X_MICROARCH.md, inter-workgroup
// visibility: sc1 stores, vmcnt(0) + barrier before the counter add, sc1
// loads by the last arriver after its add returned)
typedef unsigned int U4 __attribute__((ext_vector_type(4)));

template <typename T, int nc>
__device__ __forceinline__ void
store_slot_wt(__amdgpu_buffer_rsrc_t rs, uint32_t slot, const T (&r)[nc])
{
  constexpr int NB = nc * sizeof(T) / 16; // the fused path runs whole 16-byte slots only
#pragma unroll
  for (int b = 0; b < NB; ++b)
    {
      U4 v;
      __builtin_memcpy(&v, reinterpret_cast<const char *>(r) + 16 * b, 16);
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(slot * (uint32_t)(nc * sizeof(T)) + 16 * b),
                                             0, 16);
    }
}

template <typename T, int nc>
__device__ __forceinline__ void
load_slot_wt(__amdgpu_buffer_rsrc_t rs, uint32_t slot, T (&r)[nc])
{
  constexpr int NB = nc * sizeof(T) / 16;
#pragma unroll
  for (int b = 0; b < NB; ++b)
    {
      const U4 v = __builtin_amdgcn_raw_buffer_load_b128(
        rs, (int)(slot * (uint32_t)(nc * sizeof(T)) + 16 * b), 0, 16);
      __builtin_memcpy(reinterpret_cast<char *>(r) + 16 * b, &v, 16);
    }
}

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

// Sweep-buffer layout of one cell (in packs): point (x, y, z) at
// x + PY y + PZ z, component pack kp at + kp KS, ping-pong halves A | B,
// cells WB apart.  3D Q2 is padded (FP64: PY 4, PZ 13, KS 37, WB 151): with the
// ds_read_b128 lane groups of MI355X_MICROARCH §LDS this takes the sweep
// reads from 7.0 to 4.3 LDS cycles per instruction (4 = conflict free;
// exhaustive search over PY, PZ, KS, WB of the exact lane/address map).
template <int dim, int n, int NP>
struct BufLayout
{
  static constexpr bool pad  = dim == 3 && n == 3 && NP == 2;
  // FP32 (one pack per point): same search, 6.0 -> 4.3 modelled cycles per
  // sweep read (scripts/lds_layout_search.py)
  static constexpr bool pad1 = dim == 3 && n == 3 && NP == 1;
  static constexpr int  PY   = pad ? 4 : pad1 ? 3 : n;
  static constexpr int  PZ   = pad ? 13 : pad1 ? 20 : n * n;
  static constexpr int  KS   = pad ? 37 : pad1 ? 49 : ipow(n, dim);
  static constexpr int  WB   = pad ? 151 : pad1 ? 107 : 2 * NP * ipow(n, dim);
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
  static constexpr int WB  = BufLayout<dim, n, NP>::WB; // per-cell sweep buffer (packs)
  static constexpr int WPB = BLOCK / 64;
  static constexpr int ORG = 64; // cell-origin table entries (cells per brick)
  static size_t
  bytes(int L, bool pipe = false) // L: padded LDS lattice size; pipe: two src lattices
  {
    return 16 * ((size_t)(pipe ? 2 : 1) * NP * L + (size_t)WPB * CPW * WB) + tab_offset(L) +
           sizeof(T) * 4 * n * CoefRow<T, n>::RP + sizeof(int) * ORG;
  }
  __host__ __device__ static size_t
  tab_offset(int L) // accumulator bytes (FP64 for both precisions) rounded up to 16
  {
    return (sizeof(double) * (size_t)nc * L + 15) / 16 * 16;
  }
};

#ifndef GLS_INV_ZERO
#define GLS_INV_ZERO 1
#endif
// GLS_BABL: diagnostic-only ablation builds of k_brick (timing only, wrong
// results by design; never the product library): 1 no cell rounds (prologue
// + write-out), 2 no table / geometry loads, 4 no LDS sweeps, 8 no q-point
// physics
#ifndef GLS_BABL
#define GLS_BABL 0
#endif
// Table formulation of the brick kernel (the tables hold
// the reference's per-q fields, operator_ns.h:120-132, plus T1 and h):
//   GLS_NEWTON_T1: the Newton vmult streams T1 (Fields::T1, the
//     linearization-point part of R1, formed once per linearization point
//     and time weights by k_finalize_t1) instead of grad P* and Ut_old;
//   GLS_DELTA_OTF: q-wise delta_1 / delta_2 recomputed from U and h at the
//     q point (delta_qwise, the producer's expression) instead of streamed.
// Together: 16 instead of the reference's 20 values per q (round 2: r3
// 283 -> 272 us), and the register budget that lets the Cartesian kernel
// run 4 waves per SIMD (round 3).
#ifndef GLS_NEWTON_T1
#define GLS_NEWTON_T1 1
#endif
#ifndef GLS_DELTA_OTF
#define GLS_DELTA_OTF 1
#endif
#ifndef GLS_LATE_PREFETCH
#define GLS_LATE_PREFETCH 0
#endif
// q-wise delta_1 / delta_2 recomputed in the kernel: the Q2 Newton vmult
// only (its sqrt / division temporaries push other instantiations over their
// register budget)
template <int k, int MODE>
__host__ __device__ constexpr bool
delta_otf()
{
  return GLS_DELTA_OTF && MODE == MODE_NEWTON && k == 2;
}

// the table fields a brick vmult / residual of MODE streams: Newton U, grad U,
// T1 and h (or delta_1/2); fixed-point U and delta_1/2; residual also
// Ut_old.  Groups of 16 bytes with none of these are not loaded.
template <int dim, int MODE, int k = 2>
__host__ __device__ constexpr bool
field_read(int f)
{
  using F         = Fields<dim>;
  const bool d12  = f == F::D1 || f == F::D2;
  const bool u    = f >= F::U && f < F::U + dim;
  const bool h    = f == F::H;
  const bool ut   = f >= F::UT && f < F::UT + dim;
  const bool gu   = f >= F::GU && f < F::GU + dim * dim;
  const bool gp   = f >= F::GP && f < F::GP + dim;
  const bool t1   = f >= F::T1 && f < F::T1 + dim;
  const bool newt = GLS_NEWTON_T1 ? (gu || t1) : (gu || gp || ut);
  return (delta_otf<k, MODE>() ? h : d12) || u || (MODE == MODE_NEWTON && newt) ||
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

// everything one lane needs from HBM for one (cell, q point)
template <int dim, typename T, int MODE>
struct LaneData
{
  static constexpr int NOLD = MODE == MODE_RESIDUAL ? dim * dim + dim : 1;
  T    inv[dim][dim];
  T    JxW; // as loaded: JxW (curved) or det J (Cartesian); see jxw()
  T    U[dim], GU[dim][dim], T1[dim], UT[dim], oldg[NOLD];
  T    h, d1, d2; // h: q-wise delta from U on the fly (GLS_DELTA_OTF)
  bool active;
};

// Every load here is independent of every other and of the lane's other
// loads in flight (no data-dependent branch: the geometry type is per brick,
// read in the prologue), so the whole set issues back to back and is waited
// for once, at the q-point physics.
template <int dim, int k, typename T, int MODE>
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
#if GLS_INV_ZERO
#pragma unroll
  for (int i = 0; i < dim; ++i)
#pragma unroll
    for (int e = 0; e < dim; ++e)
      r.inv[i][e] = 0;
#endif
  // geometry (MatrixFree-style compressed: Cartesian per cell, else per q).
  // (GLS_INV_ZERO 0: the off-diagonal inv entries are not written on
  // Cartesian bricks: that path reads the diagonal only.)
  // loaded values stay untouched here: any arithmetic on them (the
  // quadrature weight, the inactive-lane mask) would make the compiler wait
  // for the loads at the prefetch point (an s_waitcnt vmcnt(0) in the middle
  // of the round); jxw() applies both at the point of use
  if (GLS_BABL & 2)
    {
#pragma unroll
      for (int i = 0; i < dim; ++i)
#pragma unroll
        for (int e = 0; e < dim; ++e)
          r.inv[i][e] = i == e ? T(1) + T(0.01) * p : T(0);
      r.JxW = T(1) + T(0.001) * lcell;
#pragma unroll
      for (int d = 0; d < dim; ++d)
        {
          r.U[d] = T(0.1) * d + T(0.01) * p, r.T1[d] = T(0.2), r.UT[d] = T(0.3);
#pragma unroll
          for (int e = 0; e < dim; ++e)
            r.GU[d][e] = T(0.05) * (d + e);
        }
#pragma unroll
      for (int i = 0; i < LaneData<dim, T, MODE>::NOLD; ++i)
        r.oldg[i] = 0;
      r.d1 = T(0.5), r.d2 = T(0.25), r.h = T(1);
      return;
    }
  if (general)
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
      r.T1[d] = tf[(GLS_NEWTON_T1 ? F::T1 : F::GP) + d]; // T1, or grad P*
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

// a shared node's final value from its summed partials (constraints, then
// the fused relaxation), as k_shared_reduce_cls writes it
template <typename T, int nc, bool R, typename Args>
__device__ __forceinline__ void
finish_shared(const Args &a, uint32_t packed, T (&r)[nc])
{
  const uint32_t node = packed & NODE_MASK, cm = packed >> 28;
#pragma unroll
  for (int c = 0; c < nc; ++c)
    if ((cm >> c) & 1)
      r[c] = R ? T(0) : a.src[(size_t)node * nc + c];
  if (!R && a.rb)
#pragma unroll
    for (int c = 0; c < nc; ++c)
      {
        const size_t j = (size_t)node * nc + c;
        r[c]           = (a.rkeep ? a.src[j] : T(0)) + a.romega * (a.rd ? a.rd[j] : T(1)) *
                                                       (a.rb[j] - r[c]);
      }
  store_node<T, nc>(a.dst, node, r);
}

#ifndef GLS_BRICK_OCC
#define GLS_BRICK_OCC 3
#endif
#ifndef GLS_BRICK_OCC32
#define GLS_BRICK_OCC32 3
#endif
#ifndef GLS_BRICK_OCC_CART
#define GLS_BRICK_OCC_CART 4
#endif

// Geometry of a launch's bricks (build_bricks orders the Cartesian and the
// curved bricks of each segment into separate runs): GEO_CART bricks hold
// one diagonal J^{-1} and det J per cell, GEO_GEN bricks J^{-1} and JxW per
// q point, GEO_ANY reads the type per brick (brick_geo bit 0).
enum
{
  GEO_ANY  = 0,
  GEO_CART = 1,
  GEO_GEN  = 2
};
// The Cartesian FP64 3D Q2 vmult kernel (Newton, fixed point) fits 128
// VGPRs (4 waves/SIMD) with its tables issued at the start of each round (in
// flight during the evaluate sweeps) and an unpadded lattice (4 workgroups
// per CU in LDS); the per-q geometry of curved bricks keeps 3 waves/SIMD and
// the earlier prefetch (issued behind the previous round's Dq^T sweeps), as
// do the other instantiations.
// (A GEO_ANY kernel whose curved bricks load J^{-1} at its two points of
// use instead of with the tables still needs 162 VGPRs: measured round 3.)
template <int dim, int k, typename T, int MODE, int GEO>
struct BrickOcc
{
  static constexpr bool cart4 = GEO == GEO_CART && sizeof(T) == 8 && dim == 3 && k == 2 &&
                                MODE != MODE_RESIDUAL;
  static constexpr int  waves = cart4 ? GLS_BRICK_OCC_CART :
                                sizeof(T) == 4 ? GLS_BRICK_OCC32 :
                                                 GLS_BRICK_OCC;
  static constexpr bool late  = GLS_LATE_PREFETCH || cart4;
};
// PIPE: persistent pipelined variant.  The grid is at most the resident
// workgroup slots; workgroup g runs the work units brick_begin + g + j *
// gridDim.x (gridDim.x a multiple of 8 keeps every unit of a workgroup on
// its XCD's run of bricks, build_bricks).  While a brick's cells run, the
// next brick's lattice node ids and write targets (issued with the brick's
// first round), its src gather and its first round's tables (both issued in
// the brick's last round, behind the Dq^T sweeps, when the q-point tables
// are dead) are in flight, so a brick switch costs the write-out and one
// barrier instead of the dependent id -> gather round trips of a
// workgroup's prologue.  The gather is an LDS-DMA
// (global_load_lds_dwordx4, one 16-byte pack per lane) straight into a
// second, unpadded src lattice: lattice node i of the next brick lands at
// pack i, lane-linear, and occupies no registers while in flight.
#ifndef GLS_FUSED_BUILD
#define GLS_FUSED_BUILD 0
#endif
// GLS_PIPE_TAB: the next brick's first-round tables are prefetched in the
// last round (1) or issued at the brick switch (0)
#ifndef GLS_PIPE_TAB
#define GLS_PIPE_TAB 1
#endif
template <int dim, int k, typename T, int MODE, bool PIPE = false, int GEO = GEO_ANY>
__global__ void __launch_bounds__(BLOCK, (BrickOcc<dim, k, T, MODE, GEO>::waves))
  k_brick(BrickArgs<T, dim, k + 1> a)
{
  using LDS          = BrickLDS<dim, k, T>;
  using V            = typename Pack<T>::V;
  constexpr int n    = k + 1;
  constexpr int nq   = LDS::nq;
  constexpr int nc   = LDS::nc;
  constexpr int W    = LDS::W;
  constexpr int NP   = LDS::NP;
  constexpr int CPW  = LDS::CPW;
  constexpr int WPB  = LDS::WPB;
  constexpr int WB   = LDS::WB;
  constexpr bool R   = MODE == MODE_RESIDUAL;
  static_assert(nq <= 64, "one cell must fit a wavefront");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int L      = a.L;  // lattice nodes (global order of brick_nodes)
  const int LP     = a.LP; // padded LDS lattice (bank-conflict-free x sweep)
  V        *s_src  = reinterpret_cast<V *>(smem);   // [NP][LP] brick src values
  // PIPE: the next brick's lattice (LDS-DMA target; LP == L, unpadded)
  V        *s_alt  = s_src + NP * LP;
  V        *s_work = s_src + (PIPE ? 2 : 1) * NP * LP; // [WPB*CPW][WB]
  // the accumulator lattice is FP64 for both precisions: ds_add_f32 costs
  // ~10 us per FP32 vmult on gfx950 (ablation GLS_ABL_NOATOMIC: 38.1 -> 28.2
  // us), ds_add_f64 next to nothing (40.1 -> 39.7 us)
  double   *s_acc  = reinterpret_cast<double *>(s_work + WPB * CPW * WB); // [nc][LP]
  constexpr int RP = CoefRow<T, n>::RP;
  T        *s_tab  = reinterpret_cast<T *>(reinterpret_cast<unsigned char *>(s_acc) +
                                     LDS::tab_offset(LP)); // [4][n][RP]
  const T  *sS     = s_tab + TAB_S * n * RP;
  const T  *sST    = s_tab + TAB_ST * n * RP;
  const T  *sD     = s_tab + TAB_D * n * RP;
  const T  *sDT    = s_tab + TAB_DT * n * RP;
  // lattice position of each brick cell's first node (cell-major order
  // x, y, z): one LDS read per round instead of per-lane divisions by the
  // runtime brick shape, which the compiler would hoist into registers
  int      *s_org  = reinterpret_cast<int *>(s_tab + 4 * n * RP); // [ORG]

  // 32-bit brick indices and cell / chunk offsets (uniform values: fewer
  // SGPRs live across the persistent variant's brick loop)
  int brick = (int)a.brick_begin + (int)blockIdx.x;
  const int brick_end = (int)a.brick_end;
  if (brick >= brick_end)
    return;
  const int bstride = PIPE ? (int)gridDim.x : 0;
  const int t   = threadIdx.x;
  GLS_STAMP(brick, 0);
  if (t < n * RP)
    {
      const int  r = t / RP, j = t % RP;
      const bool v = j < n;
      s_tab[TAB_S * n * RP + t]  = v ? a.sh.S[r][j] : T(0);
      s_tab[TAB_ST * n * RP + t] = v ? a.sh.S[j][r] : T(0);
      s_tab[TAB_D * n * RP + t]  = v ? a.sh.Dq[r][j] : T(0);
      s_tab[TAB_DT * n * RP + t] = v ? a.sh.Dq[j][r] : T(0);
    }
  if (t < a.bx * a.by * a.bz && t < LDS::ORG)
    {
      const int cx = t % a.bx, cy = (t / a.bx) % a.by, cz = t / (a.bx * a.by);
      s_org[t]     = cx * k + a.PLx * (cy * k + a.PLy * cz * k);
    }
  const int  wave    = t >> 6, lane = t & 63;
  const int  slot    = lane / nq;
  const int  p       = lane - slot * nq;
  const bool in_wave = slot < CPW;
  // left-over lanes (64 % nq) only read the first slot's buffer; every LDS
  // store of the sweeps is guarded by in_wave
  V         *A       = s_work + (wave * CPW + (in_wave ? slot : 0)) * WB;
  using BL           = BufLayout<dim, n, NP>;
  V         *B       = A + NP * BL::KS;
  const int  pa[3]   = {p % n, (p / n) % n, dim == 3 ? p / (n * n) : 0};
  const int  st[3]   = {1, BL::PY, BL::PZ};               // buffer strides
  const int  q       = pa[0] + BL::PY * pa[1] + BL::PZ * pa[2]; // own slot
  const int  lpa     = pa[0] + a.PLx * (pa[1] + a.PLy * pa[2]);  // lattice offset in a cell
  const int  step    = CPW * WPB;

  // ---- prologue: every load that does not depend on another is issued
  // up front (lattice node ids, write-out targets, round 0's geometry and
  // tables), so the block pays one HBM latency before its first sweep
  constexpr int   NI = (BrickLattice<dim, k>::L + BLOCK - 1) / BLOCK;
  const uint32_t *bn = a.brick_nodes + brick * (int64_t)L;
  const uint32_t *bt = a.brick_target + brick * (int64_t)L;
  uint32_t        pk[NI], tg[NI];
#pragma unroll
  for (int it = 0; it < NI; ++it)
    {
      const int i = t + it * BLOCK;
      pk[it]      = i < L ? bn[i] : 0u;
      tg[it]      = i < L ? bt[i] : 0u;
    }
  uint32_t binfo   = a.brick_geo[brick];
#ifndef GLS_FORCE_CART
#define GLS_FORCE_CART 0
#endif
  constexpr bool LATE = BrickOcc<dim, k, T, MODE, GEO>::late;
  bool     general = GEO == GEO_GEN || (GEO == GEO_ANY && !GLS_FORCE_CART && (binfo & 1u) != 0);
  int      ncell   = (int)(binfo >> 8);
  uint32_t cell0   = a.brick_cell0[brick];
  uint32_t chunk0  = a.brick_chunk0[brick];

  // ---- stage the brick's src values once per node (read_dof_values:
  // homogeneous constraints read as 0; the residual reads plain values).
  // The gather is issued before round 0's loads: vmcnt retires in order, so
  // the staging then waits for the gather only.
  const int Lxy = a.Lx * a.Ly;
  T         u[NI][nc];
#pragma unroll
  for (int it = 0; it < NI; ++it)
    {
      const int i = t + it * BLOCK;
      if (i < L && (pk[it] & NODE_MASK) != UNUSED_NODE)
        load_node<T, nc>(a.src, pk[it] & NODE_MASK, u[it]);
      else
#pragma unroll
        for (int c = 0; c < nc; ++c)
          u[it][c] = T(0);
    }
  // FP32 (multigrid levels): the fused relaxation's operands b, d and the
  // unmodified src of the exclusive nodes are loaded here, behind the
  // gather, instead of after the cell rounds (one memory round trip less at
  // the end of every brick; FP64 has no registers to spare for them)
#ifndef GLS_RELAX_PREFETCH
#define GLS_RELAX_PREFETCH 1
#endif
  constexpr bool PRE = GLS_RELAX_PREFETCH && sizeof(T) == 4 && !R;
  constexpr int  NPR = PRE ? NI : 1;
  T              xb[NPR][nc], xd[NPR][nc], xs[NPR][nc];
  if constexpr (PRE)
    {
#pragma unroll
      for (int it = 0; it < NI; ++it)
        {
          const int  i    = t + it * BLOCK;
          const bool excl = i < L && tg[it] != UNUSED_NODE && !(tg[it] & SHARED_BIT);
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              xs[it][c] = u[it][c];
              xb[it][c] = T(0);
              xd[it][c] = T(1);
            }
          if (excl && a.rb)
            {
              load_node<T, nc>(a.rb, tg[it], xb[it]);
              if (a.rd)
                load_node<T, nc>(a.rd, tg[it], xd[it]);
            }
        }
    }
  LaneData<dim, T, MODE> cur;
  load_lane<dim, k, T, MODE>(a, cell0, chunk0, ncell, general, wave * CPW + slot, in_wave, p, pa,
                             cur);
#pragma unroll
  for (int it = 0; it < NI; ++it)
    {
      const int i = t + it * BLOCK;
      if (i >= L)
        break;
      // PIPE runs the unpadded lattice (the LDS-DMA lands lane-linearly)
      const int      iz = PIPE ? 0 : i / Lxy, iy = PIPE ? 0 : (i - iz * Lxy) / a.Lx;
      const int      ip = PIPE ? i : (i - iz * Lxy - iy * a.Lx) + a.PLx * (iy + a.PLy * iz);
      const uint32_t cm = pk[it] >> 28;
#pragma unroll
      for (int c = 0; c < nc; ++c)
        {
          if (!R && ((cm >> c) & 1))
            u[it][c] = T(0);
          s_acc[c * LP + ip] = 0.0;
        }
      V v[NP];
      to_packs<V, T, nc, NP, W>(u[it], v);
#pragma unroll
      for (int kp = 0; kp < NP; ++kp)
        s_src[kp * LP + ip] = v[kp];
    }
  __syncthreads();
  GLS_STAMP(brick, 1);

  // the lane's tensor quadrature weight (Cartesian bricks: JxW = det J w_q)
  T wq_lane = a.sh.w[pa[0]] * a.sh.w[pa[1]];
  if (dim == 3)
    wq_lane *= a.sh.w[pa[2]];
  for (;;) // the workgroup's bricks (one pass unless PIPE)
  {
  // PIPE: the thread index made opaque per brick (and again before the
  // write-out) so that index arithmetic of the write-out / staging passes is
  // recomputed there instead of being hoisted out of the brick loop and held
  // in registers through the cell rounds
  int tl = t;
  if (PIPE)
    asm volatile("" : "+v"(tl));
  const int     next     = brick + bstride;
  const bool    has_next = PIPE && next < brick_end;
  constexpr int NIP      = PIPE ? NI : 1;
  uint32_t      pk_n[NIP], tg_n[NIP];
  uint32_t      binfo_n  = 0;
  uint32_t      cell0_n = 0, chunk0_n = 0;
  if (PIPE && has_next)
    {
      // the next brick's ids and write targets: in flight during this
      // brick's rounds (the next brick's gather depends on them)
      const uint32_t *bnn = a.brick_nodes + next * (int64_t)L;
      const uint32_t *btn = a.brick_target + next * (int64_t)L;
#pragma unroll
      for (int it = 0; it < NIP; ++it)
        {
          const int i = tl + it * BLOCK;
          pk_n[it]    = i < L ? bnn[i] : 0u;
          tg_n[it]    = i < L ? btn[i] : 0u;
        }
      binfo_n  = a.brick_geo[next];
      cell0_n  = a.brick_cell0[next];
      chunk0_n = a.brick_chunk0[next];
    }
  for (int base = 0; base < ((GLS_BABL & 1) ? 0 : ncell); base += step)
    {
      // GLS_LATE_PREFETCH: a round's geometry and tables are issued at the
      // start of that round (in flight during its evaluate sweeps) instead
      // of before the previous round's integrate sweeps: fewer registers
      // live across the integrate sweeps
      if (LATE && base > 0)
        load_lane<dim, k, T, MODE>(a, cell0, chunk0, ncell, general, base + wave * CPW + slot,
                                   in_wave, p, pa, cur);

      // the lane's lattice node this round (inactive lanes: the first cell's)
      const int li = (cur.active ? s_org[base + wave * CPW + slot] : 0) + lpa;
      // ---- evaluate: x sweep straight from the src lattice, then y (, z)
      if (!(GLS_BABL & 4))
      {
        const int lb = li - pa[0];
        if (in_wave)
#pragma unroll
          for (int kp = 0; kp < NP; ++kp)
            A[kp * BL::KS + q] = contract_v<n>(s_src + kp * LP, sS, pa[0], lb, 1);
      }
      wave_sync();
      V *in = A, *out = B;
#pragma unroll
      for (int ax = 1; ax < ((GLS_BABL & 4) ? 1 : dim); ++ax)
        {
          if (in_wave)
#pragma unroll
            for (int kp = 0; kp < NP; ++kp)
              out[kp * BL::KS + q] =
                contract_v<n>(in + kp * BL::KS, sS, pa[ax], q - pa[ax] * st[ax], st[ax]);
          wave_sync();
          V *tmp = in;
          in     = out;
          out    = tmp;
        }
      // values and reference-space gradients (collocation derivative)
      T val[nc], gref[nc][dim];
#pragma unroll
      for (int c = 0; c < nc; ++c)
        {
          val[c] = T(0);
#pragma unroll
          for (int ax = 0; ax < dim; ++ax)
            gref[c][ax] = T(0);
        }
      // left-over lanes stay out of the reads (they would only add bank
      // conflicts in their ds_read_b128 lane groups)
      if (GLS_BABL & 4)
        {
#pragma unroll
          for (int kp = 0; kp < NP; ++kp)
            {
              const V v = s_src[kp * LP + li];
#pragma unroll
              for (int w = 0; w < W; ++w)
                if (kp * W + w < nc)
                  {
                    val[kp * W + w] = v[w];
#pragma unroll
                    for (int ax = 0; ax < dim; ++ax)
                      gref[kp * W + w][ax] = v[w] * sS[ax];
                  }
            }
        }
      else if (in_wave)
#pragma unroll
      for (int kp = 0; kp < NP; ++kp)
        {
          const V v = in[kp * BL::KS + q];
          V       g[dim];
#pragma unroll
          for (int ax = 0; ax < dim; ++ax)
            g[ax] = contract_v<n>(in + kp * BL::KS, sD, pa[ax], q - pa[ax] * st[ax], st[ax]);
#pragma unroll
          for (int w = 0; w < W; ++w)
            if (kp * W + w < nc)
              {
                val[kp * W + w] = v[w];
#pragma unroll
                for (int ax = 0; ax < dim; ++ax)
                  gref[kp * W + w][ax] = g[ax][w];
              }
        }
      wave_sync();

      GLS_STAMP(brick, base == 0 ? 2 : 4);
      // ---- q-point physics (do_vmult_cell)
      // real-space gradients J^{-T} grad_ref: Cartesian bricks (wave-uniform
      // branch) have a diagonal J^{-1}
      T gu[dim][dim], gp[dim];
      if (general)
        {
#pragma unroll
          for (int c = 0; c < nc; ++c)
#pragma unroll
            for (int e = 0; e < dim; ++e)
              {
                T s = 0;
#pragma unroll
                for (int i = 0; i < dim; ++i)
                  s += cur.inv[i][e] * gref[c][i];
                if (c < dim)
                  gu[c][e] = s;
                else
                  gp[e] = s;
              }
        }
      else
        {
#pragma unroll
          for (int c = 0; c < nc; ++c)
#pragma unroll
            for (int e = 0; e < dim; ++e)
              {
                const T s = cur.inv[e][e] * gref[c][e];
                if (c < dim)
                  gu[c][e] = s;
                else
                  gp[e] = s;
              }
        }
      T vr[nc], gr[nc][dim];
      T d1 = cur.d1, d2 = cur.d2;
      if (delta_otf<k, MODE>() && !a.cw)
        {
          T u2 = 0;
#pragma unroll
          for (int d = 0; d < dim; ++d)
            u2 += cur.U[d] * cur.U[d];
          if (GLS_FAST_DELTA)
            delta_qwise_fast(u2, cur.h, a.nu, a.stau, d1, d2);
          else
            delta_qwise(u2, cur.h, a.nu, a.stau, d1, d2);
        }
      if constexpr ((GLS_BABL & 8) != 0)
        {
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              vr[c] = val[c] * cur.U[c % dim] + cur.d1;
#pragma unroll
              for (int e = 0; e < dim; ++e)
                gr[c][e] = (c < dim ? gu[c][e] : gp[e]) * cur.GU[c % dim][e] + cur.d2 * cur.T1[e] + cur.UT[e];
            }
        }
      else if constexpr (MODE == MODE_NEWTON && GLS_NEWTON_T1)
        qpoint_newton_t1<dim, T>(val, val[dim], gu, gp, cur.U, cur.GU, cur.T1, d1, d2, a.nu,
                                 a.w0, a.td, vr, gr);
      else
        qpoint_physics<dim, T, MODE>(val, val[dim], gu, gp, cur.U, cur.GU, cur.T1, cur.UT,
                                     cur.oldg, d1, d2, a.nu, a.w0, a.theta, a.td,
                                     a.have_prev, a.have_old_grad, vr, gr);
      // submit_value / submit_gradient (JxW, J^{-T}); inactive lanes: JxW 0
      const T JxW = general ? (cur.active ? cur.JxW : T(0))
                            : (cur.active ? cur.JxW * wq_lane : T(0));
      T       wq[nc], ghat[dim][nc];
      if (general)
        {
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              wq[c] = vr[c] * JxW;
#pragma unroll
              for (int i = 0; i < dim; ++i)
                {
                  T s = 0;
#pragma unroll
                  for (int e = 0; e < dim; ++e)
                    s += cur.inv[i][e] * gr[c][e];
                  ghat[i][c] = s * JxW;
                }
            }
        }
      else
        {
          T sc[dim];
#pragma unroll
          for (int i = 0; i < dim; ++i)
            sc[i] = cur.inv[i][i] * JxW;
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              wq[c] = vr[c] * JxW;
#pragma unroll
              for (int i = 0; i < dim; ++i)
                ghat[i][c] = gr[c][i] * sc[i];
            }
        }

      // ---- integrate: Dq^T on the gradient part (two axes per exchange
      // through the A/B halves), then S^T sweeps z (, y); the x sweep is
      // fused with the accumulation into the brick lattice
      V wv[NP];
      to_packs<V, T, nc, NP, W>(wq, wv);
      if (GLS_BABL & 4)
        {
#pragma unroll
          for (int kp = 0; kp < NP; ++kp)
#pragma unroll
            for (int ax = 0; ax < dim; ++ax)
              {
                V g0[NP];
                to_packs<V, T, nc, NP, W>(ghat[ax], g0);
                wv[kp] += g0[kp];
              }
        }
#pragma unroll
      for (int ax0 = 0; ax0 < ((GLS_BABL & 4) ? 0 : dim); ax0 += 2)
        {
          if (in_wave)
            {
              V g0[NP];
              to_packs<V, T, nc, NP, W>(ghat[ax0], g0);
#pragma unroll
              for (int kp = 0; kp < NP; ++kp)
                A[kp * BL::KS + q] = g0[kp];
              if (ax0 + 1 < dim)
                {
                  V g1[NP];
                  to_packs<V, T, nc, NP, W>(ghat[(ax0 + 1) % dim], g1);
#pragma unroll
                  for (int kp = 0; kp < NP; ++kp)
                    B[kp * BL::KS + q] = g1[kp];
                }
            }
          wave_sync();
          if (in_wave)
#pragma unroll
          for (int kp = 0; kp < NP; ++kp)
            {
              wv[kp] += contract_v<n>(A + kp * BL::KS, sDT, pa[ax0], q - pa[ax0] * st[ax0],
                                            st[ax0]);
              if (ax0 + 1 < dim)
                {
                  const int ax1 = (ax0 + 1) % dim;
                  wv[kp] += contract_v<n>(B + kp * BL::KS, sDT, pa[ax1],
                                                q - pa[ax1] * st[ax1], st[ax1]);
                }
            }
          wave_sync();
        }
      if (in_wave)
#pragma unroll
        for (int kp = 0; kp < NP; ++kp)
          A[kp * BL::KS + q] = wv[kp];
      // the next round's geometry and tables: issued here (few registers
      // live), in flight during the S^T sweeps and the next evaluate (this
      // round's lattice position is kept: the prefetch overwrites cur)
      GLS_STAMP(brick, base == 0 ? 3 : 5);
      const int  li_now     = li;
      const bool active_now = cur.active;
      if (!LATE && base + step < ncell)
        load_lane<dim, k, T, MODE>(a, cell0, chunk0, ncell, general, base + step + wave * CPW + slot,
                                   in_wave, p, pa, cur);
      else if (!LATE && PIPE && GLS_PIPE_TAB && has_next)
        load_lane<dim, k, T, MODE>(a, cell0_n, chunk0_n, (int)(binfo_n >> 8), (binfo_n & 1u) != 0,
                                   wave * CPW + slot, in_wave, p, pa, cur);
      if constexpr (PIPE && nc * sizeof(T) % 16 == 0)
      if (has_next && base + step >= ncell)
        {
          // last round: the next brick's src gather (read_dof_values of its
          // lattice) by LDS-DMA into the other lattice, one 16-byte pack per
          // lane and instruction; lattice positions outside the next brick's
          // cells (UNUSED_NODE) read node 0 (never read back)
#pragma unroll
          for (int it = 0; it < NIP; ++it)
            {
              const int i = tl + it * BLOCK;
              if (i < L)
                {
                  uint32_t node = pk_n[it] & NODE_MASK;
                  if (node == UNUSED_NODE)
                    node = 0;
                  const V *g = reinterpret_cast<const V *>(a.src) + (size_t)node * NP;
#pragma unroll
                  for (int kp = 0; kp < NP; ++kp)
                    __builtin_amdgcn_global_load_lds(
                      (const void *)(g + kp),
                      (__attribute__((address_space(3))) void *)(s_alt + kp * LP + it * BLOCK +
                                                                 wave * 64),
                      16, 0, 0);
                }
            }
        }
      wave_sync();
      in  = A;
      out = B;
#pragma unroll
      for (int ax = dim - 1; ax >= ((GLS_BABL & 4) ? dim : 1); --ax)
        {
          if (in_wave)
#pragma unroll
            for (int kp = 0; kp < NP; ++kp)
              out[kp * BL::KS + q] =
                contract_v<n>(in + kp * BL::KS, sST, pa[ax], q - pa[ax] * st[ax], st[ax]);
          wave_sync();
          V *tmp = in;
          in     = out;
          out    = tmp;
        }
      T cx[n];
      coefs<n>(sST, pa[0], cx);
      if (active_now)
#pragma unroll
        for (int kp = 0; kp < NP; ++kp)
          {
            const V r = (GLS_BABL & 4) ? wv[kp] : contract_c<n>(in + kp * BL::KS, cx, q - pa[0], 1);
#pragma unroll
            for (int w = 0; w < W; ++w)
              if (kp * W + w < nc)
#ifdef GLS_ABL_NOATOMIC // diagnostic timing build only: racy plain adds
                s_acc[(kp * W + w) * LP + li_now] += (double)r[w];
#else
                lds_add(s_acc + (kp * W + w) * LP + li_now, (double)r[w]);
#endif
          }
      wave_sync();
    }
  if constexpr (PIPE)
    // a bare barrier: __syncthreads() would also wait for the next brick's
    // LDS-DMA gather (a pending LDS write on the VM counter)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else
    __syncthreads();
  GLS_STAMP(brick, 6);

  if (PIPE)
    asm volatile("" : "+v"(tl));
  // ---- write out: exclusive nodes -> dst, boundary nodes -> partials
  // the fused last-arriver reduction (measured slower) is only
  // compiled into GLS_FUSED_BUILD=1 diagnostic builds
  constexpr bool FUSE = GLS_FUSED_BUILD && nc * sizeof(T) % 16 == 0; // 3D: 4 comps per slot
  const __amdgpu_buffer_rsrc_t prs =
    __builtin_amdgcn_make_buffer_rsrc(a.partial, 0, (int)a.partial_bytes, 0x00020000);
#pragma unroll
  for (int it = 0; it < NI; ++it)
    {
      const int i = tl + it * BLOCK;
      if (i >= L)
        break;
      // PIPE runs the unpadded lattice (the LDS-DMA lands lane-linearly)
      const int      iz = PIPE ? 0 : i / Lxy, iy = PIPE ? 0 : (i - iz * Lxy) / a.Lx;
      const int      ip = PIPE ? i : (i - iz * Lxy - iy * a.Lx) + a.PLx * (iy + a.PLy * iz);
      const uint32_t tgt = tg[it];
      double         acc[nc];
#pragma unroll
      for (int c = 0; c < nc; ++c)
        {
          acc[c] = s_acc[c * LP + ip];
          if (PIPE)
            s_acc[c * LP + ip] = 0.0; // the next brick's accumulator
        }
      if (tgt == UNUSED_NODE)
        continue;
      if (tgt & SHARED_BIT)
        {
          T r[nc];
#pragma unroll
          for (int c = 0; c < nc; ++c)
            r[c] = (T)(R ? -acc[c] : acc[c]);
          bool done = false;
          if constexpr (FUSE)
            if (a.counters)
              {
                const uint32_t slot = tgt & ~SHARED_BIT;
                if (a.rc.mult[slot_class(a.rc, slot)] == 1)
                  finish_shared<T, nc, R>(a, pk[it], r); // the node's only brick
                else
                  store_slot_wt<T, nc>(prs, slot, r);
                done = true;
              }
          if (!done)
            store_node<T, nc>(a.partial, tgt & ~SHARED_BIT, r);
        }
      else
        {
          const uint32_t cm = pk[it] >> 28;
          T              r[nc];
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              r[c] = (T)(R ? -acc[c] : acc[c]);
              if ((cm >> c) & 1)
                r[c] = R ? T(0) : (PRE ? xs[PRE ? it : 0][c] : a.src[(size_t)tgt * nc + c]);
            }
          if constexpr (PRE)
            {
              if (a.rb)
#pragma unroll
                for (int c = 0; c < nc; ++c)
                  {
                    const T base = a.rkeep ? xs[it][c] : T(0);
                    r[c]         = base + a.romega * xd[it][c] * (xb[it][c] - r[c]);
                  }
            }
          else if constexpr (!R)
            if (a.rb)
#pragma unroll
              for (int c = 0; c < nc; ++c)
                {
                  const size_t j = (size_t)tgt * nc + c;
                  const T  base  = a.rkeep ? a.src[j] : T(0);
                  r[c]           = base + a.romega * (a.rd ? a.rd[j] : T(1)) * (a.rb[j] - r[c]);
                }
          store_node<T, nc>(a.dst, tgt, r);
        }
    }
  if constexpr (FUSE)
  if (a.counters)
    {
      // every wave's slot stores have reached memory before any arrival of
      // this brick is counted
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#pragma unroll
      for (int it = 0; it < NI; ++it)
        {
          const int i = tl + it * BLOCK;
          if (i >= L)
            break;
          const uint32_t tgt = tg[it];
          if (tgt == UNUSED_NODE || !(tgt & SHARED_BIT))
            continue;
          const uint32_t slot = tgt & ~SHARED_BIT;
          const int      kc   = slot_class(a.rc, slot);
          const uint32_t m    = a.rc.mult[kc];
          if (m == 1)
            continue;
          const uint32_t sn  = a.rc.first[kc] + (slot - a.rc.slot0[kc]) / m;
          const uint32_t b0s = a.rc.slot0[kc] + (sn - a.rc.first[kc]) * m;
          const uint32_t old = __hip_atomic_fetch_add(a.counters + sn, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
          if (old != m - 1)
            continue;
          // last arrival: the node's slots in slot order, summed as
          // k_shared_reduce_cls sums them
          T        sum[nc] = {};
          uint32_t j       = 0;
          for (; j + 4 <= m; j += 4)
            {
              T x0[nc], x1[nc], x2[nc], x3[nc];
              load_slot_wt<T, nc>(prs, b0s + j, x0);
              load_slot_wt<T, nc>(prs, b0s + j + 1, x1);
              load_slot_wt<T, nc>(prs, b0s + j + 2, x2);
              load_slot_wt<T, nc>(prs, b0s + j + 3, x3);
#pragma unroll
              for (int c = 0; c < nc; ++c)
                sum[c] += (x0[c] + x1[c]) + (x2[c] + x3[c]);
            }
          if (j + 2 <= m)
            {
              T x0[nc], x1[nc];
              load_slot_wt<T, nc>(prs, b0s + j, x0);
              load_slot_wt<T, nc>(prs, b0s + j + 1, x1);
#pragma unroll
              for (int c = 0; c < nc; ++c)
                sum[c] += x0[c] + x1[c];
              j += 2;
            }
          if (j < m)
            {
              T x0[nc];
              load_slot_wt<T, nc>(prs, b0s + j, x0);
#pragma unroll
              for (int c = 0; c < nc; ++c)
                sum[c] += x0[c];
            }
          finish_shared<T, nc, R>(a, pk[it], sum);
          __hip_atomic_store(a.counters + sn, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
  GLS_STAMP(brick, 7);
  if (!has_next)
    break;
  // ---- switch to the next brick: its lattice has landed in s_alt (the
  // accumulator was zeroed by the write-out), its ids / targets / scalars
  // come from this brick's prefetch
  brick   = next;
  binfo   = binfo_n;
  general = GEO == GEO_GEN || (GEO == GEO_ANY && !GLS_FORCE_CART && (binfo & 1u) != 0);
  ncell   = (int)(binfo >> 8);
  cell0   = cell0_n;
  chunk0  = chunk0_n;
#pragma unroll
  for (int it = 0; it < NIP; ++it)
    {
      pk[it] = pk_n[it];
      tg[it] = tg_n[it];
    }
  // the DMA (and the next round's tables issued before it) complete
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  {
    V *tmp = s_src;
    s_src  = s_alt;
    s_alt  = tmp;
  }
#pragma unroll
  for (int it = 0; it < NIP; ++it)
    {
      const int i = tl + it * BLOCK;
      if (i >= L)
        break;
      const uint32_t cm = pk[it] >> 28;
      if constexpr (PRE)
        {
          // the fused relaxation's operands of the exclusive nodes: the raw
          // src values from the landed lattice, b and d from memory
          const bool excl = tg[it] != UNUSED_NODE && !(tg[it] & SHARED_BIT);
#pragma unroll
          for (int kp = 0; kp < NP; ++kp)
            {
              const V v = s_src[kp * LP + i];
#pragma unroll
              for (int w = 0; w < W; ++w)
                if (kp * W + w < nc)
                  xs[it][kp * W + w] = v[w];
            }
#pragma unroll
          for (int c = 0; c < nc; ++c)
            {
              xb[it][c] = T(0);
              xd[it][c] = T(1);
            }
          if (excl && a.rb)
            {
              load_node<T, nc>(a.rb, tg[it], xb[it]);
              if (a.rd)
                load_node<T, nc>(a.rd, tg[it], xd[it]);
            }
        }
      // homogeneous constraints read as 0 (read_dof_values)
      if (!R && cm)
        {
          T *sv = reinterpret_cast<T *>(s_src);
#pragma unroll
          for (int c = 0; c < nc; ++c)
            if ((cm >> c) & 1)
              sv[((c / W) * LP + i) * W + c % W] = T(0);
        }
    }
  if (LATE || !GLS_PIPE_TAB)
    load_lane<dim, k, T, MODE>(a, cell0, chunk0, ncell, general, wave * CPW + slot, in_wave, p,
                               pa, cur);
  __syncthreads();
  } // brick loop
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
                      T romega = T(0), int keep = 1, uint32_t n_relax = 0xFFFFFFFFu)
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
}

} // namespace gls
