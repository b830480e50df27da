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
  T               nu, w0, theta, stau;
  int             td, cw, have_prev, have_old_grad;
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
  bytes(int L) // L: padded LDS lattice size
  {
    return 16 * ((size_t)NP * L + (size_t)WPB * CPW * WB) + tab_offset(L) +
           sizeof(T) * 4 * n * CoefRow<T, n>::RP + sizeof(int) * ORG;
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
  else if (general)
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

// The Cartesian FP64 3D Q2 vmult kernel (Newton, fixed point) fits 128
// VGPRs (4 waves/SIMD) with its tables issued at the start of each round (in
// flight during the evaluate sweeps) and an unpadded lattice (4 workgroups
// per CU in LDS); the per-q geometry of curved bricks keeps 3 waves/SIMD and
// the earlier prefetch (issued behind the previous round's Dq^T sweeps), as
// do the other instantiations.
// (A GEO_ANY kernel whose curved bricks load J^{-1} at its two points of
// use instead of with the tables still needs 162 VGPRs: measured round 3;
// forced to 4 waves it spills 140 B/lane inside the round loop and takes
// 63.7 instead of 40.2 us at r2, 517 instead of 276 us at r3: round 4,
// profiles/r04/explore/ab_any4_spill.txt.)
template <int dim, int k, typename T, int MODE, int GEO, int ZL = 1>
struct BrickOcc
{
  static constexpr bool cart4 = GEO == GEO_CART && sizeof(T) == 8 && dim == 3 && k == 2 &&
                                MODE != MODE_RESIDUAL && ZL == 1;
  static constexpr int  waves = cart4 || sizeof(T) == 4 ? 4 : 3;
  static constexpr bool late  = cart4; // tables issued at the start of each round
};

template <int dim, int k, typename T, int MODE, int GEO = GEO_ANY, int ZL = 1>
__global__ void __launch_bounds__(BLOCK, (BrickOcc<dim, k, T, MODE, GEO, ZL>::waves))
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
  constexpr bool LATE = BrickOcc<dim, k, T, MODE, GEO, ZL>::late;
  static_assert(nq <= 64, "one cell must fit a wavefront");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int L      = a.L;  // lattice nodes (global order of brick_nodes)
  const int LP     = a.LP; // padded LDS lattice (bank-conflict-free x sweep)
  V        *s_src  = reinterpret_cast<V *>(smem);   // [NP][LP] brick src values
  V        *s_work = s_src + NP * LP;               // [WPB*CPW][WB]
  // the accumulator lattice is FP64 for both precisions: ds_add_f32 costs
  // ~10 us per FP32 vmult on gfx950 (racy plain-add ablation: 38.1 -> 28.2
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

  const int brick = (int)a.brick_begin + (int)blockIdx.x;
  if (brick >= (int)a.brick_end)
    return;
  const int t = threadIdx.x;
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
  constexpr int   NI = (BrickLattice<dim, k, ZL>::L + BLOCK - 1) / BLOCK;
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
  const uint32_t binfo   = a.brick_geo[brick];
  const bool     general = GEO == GEO_GEN || (GEO == GEO_ANY && (binfo & 1u) != 0);
  const int      ncell   = (int)(binfo >> 8);
  const uint32_t cell0   = a.brick_cell0[brick];
  const uint32_t chunk0  = a.brick_chunk0[brick];

  // ---- stage the brick's src values once per node (read_dof_values:
  // homogeneous constraints read as 0; the residual reads plain values).
  // The gather is issued before round 0's loads: vmcnt retires in order, so
  // the staging then waits for the gather only.
  const int Lxy = a.Lx * a.Ly;
  T         u[NI][nc];
  // deferred reduction of the previous apply (one 16-byte pack per node)
  constexpr bool QREC = sizeof(T) == 4 && !R && nc * sizeof(T) == 16;
#pragma unroll
  for (int it = 0; it < NI; ++it)
    {
      const int      i    = t + it * BLOCK;
      const uint32_t node = pk[it] & NODE_MASK;
      if (QREC && i < L && node != UNUSED_NODE && a.qslots && (tg[it] & SHARED_BIT))
        {
          // the previous apply's shared-node reduction of this node, in
          // k_shared_reduce_cls's order and arithmetic (bitwise the same)
          const uint32_t slt = tg[it] & ~SHARED_BIT;
          const int      kc  = slot_class(a.rc, slt);
          const uint32_t m   = a.rc.mult[kc];
          const uint32_t b0  = a.rc.slot0[kc] + (slt - a.rc.slot0[kc]) / m * m;
          const V       *pp  = reinterpret_cast<const V *>(a.qslots);
          V              sum = {};
          uint32_t       j   = 0;
          for (; j + 4 <= m; j += 4)
            {
              const V x0 = pp[b0 + j], x1 = pp[b0 + j + 1], x2 = pp[b0 + j + 2],
                      x3 = pp[b0 + j + 3];
              sum += (x0 + x1) + (x2 + x3);
            }
          if (j + 2 <= m)
            {
              const V x0 = pp[b0 + j], x1 = pp[b0 + j + 1];
              sum += x0 + x1;
              j += 2;
            }
          if (j < m)
            sum += pp[b0 + j];
          const V        xs = reinterpret_cast<const V *>(a.qprev)[node];
          const V        bb = reinterpret_cast<const V *>(a.qb)[node];
          const V        dd = a.qd ? reinterpret_cast<const V *>(a.qd)[node] : V{} + T(1);
          const uint32_t cm = pk[it] >> 28;
#pragma unroll
          for (int w = 0; w < W; ++w)
            if ((cm >> w) & 1)
              sum[w] = xs[w];
          const V v = xs + a.qomega * dd * (bb - sum);
          reinterpret_cast<V *>(a.qsrc_w)[node] = v;
#pragma unroll
          for (int c = 0; c < nc; ++c)
            u[it][c] = v[c % W];
        }
      else if (i < L && node != UNUSED_NODE)
        load_node<T, nc>(a.src, node, u[it]);
      else
#pragma unroll
        for (int c = 0; c < nc; ++c)
          u[it][c] = T(0);
    }
  // FP32 (multigrid levels): the fused relaxation's operands b, d and the
  // unmodified src of the exclusive nodes are loaded here, behind the
  // gather, instead of after the cell rounds (one memory round trip less at
  // the end of every brick; FP64 has no registers to spare for them)
  // (two-layer bricks: two lattice chunks per thread; the operands' 24
  // registers would spill, so they are read at the write-out)
  constexpr bool PRE = sizeof(T) == 4 && !R && ZL == 1;
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
  load_lane<dim, k, T, MODE, GEO>(a, cell0, chunk0, ncell, general, wave * CPW + slot, in_wave, p,
                                  pa, cur);
#pragma unroll
  for (int it = 0; it < NI; ++it)
    {
      const int i = t + it * BLOCK;
      if (i >= L)
        break;
      const int      iz = i / Lxy, iy = (i - iz * Lxy) / a.Lx;
      const int      ip = (i - iz * Lxy - iy * a.Lx) + a.PLx * (iy + a.PLy * iz);
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

  // the lane's tensor quadrature weight (Cartesian bricks: JxW = det J w_q)
  T wq_lane = a.sh.w[pa[0]] * a.sh.w[pa[1]];
  if (dim == 3)
    wq_lane *= a.sh.w[pa[2]];
  for (int base = 0; base < ncell; base += step)
    {
      // LATE: a round's geometry and tables are issued at the start of that
      // round (in flight during its evaluate sweeps) instead of before the
      // previous round's integrate sweeps: fewer registers live across the
      // integrate sweeps
      if (LATE && base > 0)
        load_lane<dim, k, T, MODE, GEO>(a, cell0, chunk0, ncell, general,
                                        base + wave * CPW + slot, in_wave, p, pa, cur);

      // the lane's lattice node this round (inactive lanes: the first cell's)
      const int li = (cur.active ? s_org[base + wave * CPW + slot] : 0) + lpa;
      // ---- evaluate: x sweep straight from the src lattice, then y (, z).
      // Each sweep reads its coefficient row once for every pack and issues
      // every pack's reads before the first store (a store could alias the
      // tables or the next pack's reads: interleaved, each pack would wait
      // one LDS round trip of its own)
      if (in_wave)
        {
          T c[n];
          coefs<n>(sS, pa[0], c);
          V r[NP];
#pragma unroll
          for (int kp = 0; kp < NP; ++kp)
            r[kp] = contract_c<n>(s_src + kp * LP, c, li - pa[0], 1);
#pragma unroll
          for (int kp = 0; kp < NP; ++kp)
            A[kp * BL::KS + q] = r[kp];
        }
      wave_sync();
      V *in = A, *out = B;
#pragma unroll
      for (int ax = 1; ax < dim; ++ax)
        {
          if (in_wave)
            {
              T c[n];
              coefs<n>(sS, pa[ax], c);
              V r[NP];
#pragma unroll
              for (int kp = 0; kp < NP; ++kp)
                r[kp] = contract_c<n>(in + kp * BL::KS, c, q - pa[ax] * st[ax], st[ax]);
#pragma unroll
              for (int kp = 0; kp < NP; ++kp)
                out[kp * BL::KS + q] = r[kp];
            }
          wave_sync();
          V *tmp = in;
          in     = out;
          out    = tmp;
        }
      // values and reference-space gradients (collocation derivative);
      // left-over lanes stay out of the reads (they would only add bank
      // conflicts in their ds_read_b128 lane groups)
      T val[nc], gref[nc][dim];
#pragma unroll
      for (int c = 0; c < nc; ++c)
        {
          val[c] = T(0);
#pragma unroll
          for (int ax = 0; ax < dim; ++ax)
            gref[c][ax] = T(0);
        }
      if (in_wave)
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
          delta_qwise_fast(u2, cur.h, a.nu, a.stau, d1, d2);
        }
      if constexpr (MODE == MODE_NEWTON)
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
#pragma unroll
      for (int ax0 = 0; ax0 < dim; ax0 += 2)
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
      const int  li_now     = li;
      const bool active_now = cur.active;
      if (!LATE && base + step < ncell)
        load_lane<dim, k, T, MODE, GEO>(a, cell0, chunk0, ncell, general,
                                        base + step + wave * CPW + slot, in_wave, p, pa, cur);
      wave_sync();
      in  = A;
      out = B;
#pragma unroll
      for (int ax = dim - 1; ax >= 1; --ax)
        {
          if (in_wave)
            {
              T c[n];
              coefs<n>(sST, pa[ax], c);
              V r[NP];
#pragma unroll
              for (int kp = 0; kp < NP; ++kp)
                r[kp] = contract_c<n>(in + kp * BL::KS, c, q - pa[ax] * st[ax], st[ax]);
#pragma unroll
              for (int kp = 0; kp < NP; ++kp)
                out[kp * BL::KS + q] = r[kp];
            }
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
            const V r = contract_c<n>(in + kp * BL::KS, cx, q - pa[0], 1);
#pragma unroll
            for (int w = 0; w < W; ++w)
              if (kp * W + w < nc)
                lds_add(s_acc + (kp * W + w) * LP + li_now, (double)r[w]);
          }
      wave_sync();
    }
  __syncthreads();

  // ---- write out: exclusive nodes -> dst, boundary nodes -> partials
#pragma unroll
  for (int it = 0; it < NI; ++it)
    {
      const int i = t + it * BLOCK;
      if (i >= L)
        break;
      const int      iz  = i / Lxy, iy = (i - iz * Lxy) / a.Lx;
      const int      ip  = (i - iz * Lxy - iy * a.Lx) + a.PLx * (iy + a.PLy * iz);
      const uint32_t tgt = tg[it];
      if (tgt == UNUSED_NODE)
        continue;
      double acc[nc];
#pragma unroll
      for (int c = 0; c < nc; ++c)
        acc[c] = s_acc[c * LP + ip];
      T r[nc];
      if (tgt & SHARED_BIT)
        {
#pragma unroll
          for (int c = 0; c < nc; ++c)
            r[c] = (T)(R ? -acc[c] : acc[c]);
          store_node<T, nc>(a.partial, tgt & ~SHARED_BIT, r);
          continue;
        }
      const uint32_t cm = pk[it] >> 28;
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
              const size_t j    = (size_t)tgt * nc + c;
              const T      base = a.rkeep ? a.src[j] : T(0);
              r[c]              = base + a.romega * (a.rd ? a.rd[j] : T(1)) * (a.rb[j] - r[c]);
            }
      store_node<T, nc>(a.dst, tgt, r);
      if constexpr (sizeof(T) == 4 && !R)
        if (a.out64)
          {
            double r64[nc];
#pragma unroll
            for (int c = 0; c < nc; ++c)
              r64[c] = (double)r[c];
            store_node<double, nc>(a.out64, tgt, r64);
          }
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

} // namespace gls
