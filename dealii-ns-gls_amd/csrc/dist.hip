// dist.hip — partitioned (one rank per GPU) vmult of the GLS operator with
// the ghost exchange over RCCL (xGMI), overlapped with the interior bricks.
//
// Reference behaviour (deal.II distributed vectors inside
// MatrixFree::cell_loop, operator_ns.cc:702-721):
//   src.update_ghost_values()            owner -> ghost copies   (import)
//   dst = cell loop (ghost rows collect partial sums)
//   dst.compress(VectorOperation::add)   ghost partials -> owner, added;
//                                        ghost entries zeroed   (export-add)
//   dst[c] = src[c] on constrained owned dofs        (identity rows)
//
// One gls_dist_vmult on stream s (deal.II's overlapped cell_loop: ghost
// import behind the first interior cells, export-add behind the rest):
//   pack      k_pack: send buffer <- src[send nodes]                  (s)
//   import    ncclSend/ncclRecv per peer, the receives land directly in
//             src's ghost block of that owner                          (comm stream)
//   interior1 k_brick over the first half of the work units that read no
//             ghost node                                               (s, overlaps the import)
//   boundary  k_brick over the units that read ghost nodes, after the
//             import event, then the reduction of the GHOST rows only
//             (their partial sums come from these units alone)         (s)
//   export    ncclSend of each owner's ghost block of dst, ncclRecv into
//             the export buffer, after the ghost-reduce event          (comm stream)
//   interior2 k_brick over the other interior units, then the reduction of
//             the owned rows (brick boundaries, identity rows)         (s, overlaps the export)
//   unpack    after the export event, k_unpack_add: owned rows +=
//             received partials (fixed order per node, constrained
//             components skipped: their identity value stands), then the
//             ghost block of dst is zeroed.
// The exchanges go through a Transport: RCCL send/recv for the ranks of a
// communicator, device copies for the members of an in-process group
// (gls_dist_create with nccl_id NULL: tests on one GPU).  A member of an
// in-process group driven from its own host thread (team calls with n = 1,
// like an RCCL rank) runs THIS function, with its own compute stream and
// communication stream: its import copies a peer's send buffer on d->cs once
// the peer's ev_packed has passed, its export copies a peer's ghost rows once
// the peer's ev_ghosts has passed, and two fences keep a member from
// rewriting its send buffer or zeroing its ghost rows before the peers'
// copies of them are done (host barriers order the event records with the
// waits).  gls_dist_vmult_group runs the same phases for all members of a
// group from one thread in lockstep on one stream.
#include "../../include/gls_op.h"
#include "common.h"
#include "trace.h"
#include "kernels.h"
#include "op_internal.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace gls
{
// send buffer <- src rows of the send nodes (plain values)
template <typename T, int nc>
__global__ void __launch_bounds__(256)
  k_pack(T *__restrict__ buf, const T *__restrict__ src, const uint32_t *__restrict__ nodes,
         int64_t n)
{
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * nc)
    return;
  const int64_t j = gid / nc;
  const int     c = (int)(gid - j * nc);
  buf[gid]        = src[(size_t)(nodes[j] & NODE_MASK) * nc + c];
}

// owned rows += the partial sums the peers computed for them (compress(add));
// one thread per (receiving node, component), contributions summed in a fixed
// order, constrained components keep their identity-row value.  With a fused
// relaxation / residual on the local part (dst = x + omega d (b - A_loc x),
// or omega d (b - A_loc x)), the peers' part of A x enters as
// dst -= omega d (sum): rd the inverse diagonal (null: 1), scale = omega
// (0: plain compress(add))
template <typename T, int nc>
__global__ void __launch_bounds__(256)
  k_unpack_add(T *__restrict__ dst, const T *__restrict__ xrecv,
               const uint32_t *__restrict__ nodes, const uint32_t *__restrict__ off,
               const uint32_t *__restrict__ entry, int64_t n, const T *__restrict__ rd,
               T scale)
{
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n * nc)
    return;
  const int64_t  u      = gid / nc;
  const int      c      = (int)(gid - u * nc);
  const uint32_t packed = nodes[u];
  if ((packed >> 28 >> c) & 1)
    return;
  T s = 0;
  for (uint32_t e = off[u]; e < off[u + 1]; ++e)
    s += xrecv[(size_t)entry[e] * nc + c];
  const size_t j = (size_t)(packed & NODE_MASK) * nc + c;
  if (scale != T(0))
    s *= -scale * (rd ? rd[j] : T(1));
  dst[j] += s;
}
} // namespace gls

namespace
{
#define NCCL_THROW(x)                                                                          \
  do                                                                                           \
    {                                                                                          \
      ncclResult_t r_ = (x);                                                                   \
      if (r_ != ncclSuccess)                                                                   \
        throw std::runtime_error(std::string("RCCL: ") + ncclGetErrorString(r_) + " at " +   \
                                 #x);                                                          \
    }                                                                                          \
  while (0)

struct Peer
{
  int     rank;
  int64_t send_off, send_cnt;    // in the send / export-receive buffers (nodes)
  int64_t recv_begin, recv_cnt;  // ghost block of this owner (local nodes)
};

struct Group; // in-process group (tests)

// the data movement of one rank's exchanges (dist_vmult, update_ghost_values,
// compress(add)) and its all-reduces
struct Transport
{
  virtual ~Transport() = default;
  // the owners' rows into this rank's ghost block of src (update_ghost_values),
  // on d->cs behind d->ev_packed
  virtual void import_ghosts(glsDist_ *d, void *src) = 0;
  // this rank's ghost partial sums of dst to their owners' export buffers
  // (compress(add)), on d->cs behind d->ev_ghosts
  virtual void export_ghosts(glsDist_ *d, const void *dst) = 0;
  // on s, before this rank rewrites its send buffer / zeroes its ghost rows:
  // the peers' reads of them are done
  virtual void fence_send(glsDist_ *, hipStream_t) {}
  virtual void fence_ghosts(glsDist_ *, hipStream_t) {}
  // buf[0, count) <- the sum (max) over the ranks, on s
  virtual void allreduce(glsDist_ *d, double *buf, int64_t count, bool max, hipStream_t s) = 0;
};
} // namespace

struct glsDist_
{
  glsOp_           *op = nullptr;
  int               rank = 0, world = 1;
  ncclComm_t        comm = nullptr;
  Group            *group = nullptr;
  // the host thread that last drove this member in rank mode (creation: the
  // creating thread); Group::barrier tells a lockstep misuse from slow peers
  std::thread::id   driver = std::this_thread::get_id();
  std::unique_ptr<Transport> tx;
  // in-process all-reduce: this member's staged operand (peers read it)
  double           *red_stage = nullptr;
  int64_t           red_cap   = 0;
  hipEvent_t        ev_red_staged = nullptr, ev_red_done = nullptr;
  hipStream_t       cs   = nullptr;
  hipEvent_t        ev_packed = nullptr, ev_imported = nullptr;
  hipEvent_t        ev_ghosts = nullptr, ev_exported = nullptr;
  std::vector<Peer> peers;
  int64_t           n_send = 0, n_recv_nodes = 0;
  uint32_t         *d_send_nodes = nullptr; // [n_send] node | cmask << 28
  void             *d_send_buf   = nullptr; // [n_send][nc]
  void             *d_xrecv_buf  = nullptr; // [n_send][nc]
  uint32_t         *d_un_nodes = nullptr, *d_un_off = nullptr, *d_un_entry = nullptr;
  int64_t           n_un = 0;
  // vectors of the current call (in-process group: peers read them)
  void             *cur_dst = nullptr, *cur_src = nullptr;
};

namespace
{
struct Group
{
  std::vector<glsDist_ *> members; // by rank
  // host barrier of the members driven from their own threads
  std::mutex              mu;
  std::condition_variable cv;
  int                     arrived = 0;
  uint64_t                gen     = 0;
  bool                    broken  = false;

  // per rank: the barrier generation it last arrived at
  std::vector<uint64_t>   arrived_at;

  // host barrier of the members driven one thread per member.  Fails fast
  // (after a 10 s grace for first-launch code-object loads) when every member
  // still missing was last driven -- or created -- by the very thread that is
  // blocked here: the members are being driven one after another from one
  // thread, which can never complete a rank-mode call; otherwise fails after
  // GLS_DIST_BARRIER_TIMEOUT seconds (default 120).  Either way the group is
  // broken for good (its members' events are mid-call).
  void
  barrier(glsDist_ *self);
};

double
barrier_timeout_s()
{
  static const double t = [] {
    const char *e = getenv("GLS_DIST_BARRIER_TIMEOUT");
    const double v = e ? std::atof(e) : 0.0;
    return v > 0 ? v : 120.0;
  }();
  return t;
}

void
Group::barrier(glsDist_ *self)
{
  const int world = self->world;
  std::unique_lock<std::mutex> lk(mu);
  if (broken)
    throw std::runtime_error("gls_dist: in-process group broken by an earlier failure");
  const std::thread::id me = std::this_thread::get_id();
  self->driver             = me;
  const uint64_t g         = gen;
  if (arrived_at.size() < (size_t)world)
    arrived_at.resize((size_t)world, UINT64_MAX);
  arrived_at[(size_t)self->rank] = g;
  if (++arrived == world)
    {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
  const auto   t0    = std::chrono::steady_clock::now();
  const double limit = barrier_timeout_s();
  for (;;)
    {
      if (cv.wait_for(lk, std::chrono::milliseconds(250), [&] { return gen != g || broken; }))
        {
          if (broken)
            throw std::runtime_error("gls_dist: in-process group broken by an earlier failure");
          return;
        }
      const double el =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      bool lockstep = el > 10.0;
      for (size_t r = 0; lockstep && r < members.size(); ++r)
        if (r < arrived_at.size() && arrived_at[r] != g && members[r] && members[r]->driver != me)
          lockstep = false;
      if (lockstep || el > limit)
        {
          broken = true;
          cv.notify_all();
          throw std::runtime_error(
            lockstep ? "gls_dist: rank-mode call on an in-process group driven from one thread "
                       "(every missing member was last driven by this blocked thread); drive "
                       "each member from its own thread, or use the *_group entry points" :
                       "gls_dist: an in-process group member waited " + std::to_string(limit) +
                         " s for its peers (GLS_DIST_BARRIER_TIMEOUT; each member driven from "
                         "its own thread makes the same sequence of rank calls)");
        }
    }
}

size_t
row_bytes(const glsOp_ *op)
{
  return (size_t)(op->dim + 1) * op->tsize();
}

const Peer *
find_peer(const glsDist_ *d, int rank)
{
  for (const Peer &p : d->peers)
    if (p.rank == rank)
      return &p;
  return nullptr;
}

template <typename T>
void
launch_pack(glsDist_ *d, const void *src, hipStream_t s)
{
  const int nc = d->op->dim + 1;
  if (d->n_send == 0)
    return;
  const dim3 g((unsigned)((d->n_send * nc + 255) / 256));
  if (nc == 4)
    hipLaunchKernelGGL((gls::k_pack<T, 4>), g, dim3(256), 0, s, (T *)d->d_send_buf,
                       (const T *)src, d->d_send_nodes, d->n_send);
  else
    hipLaunchKernelGGL((gls::k_pack<T, 3>), g, dim3(256), 0, s, (T *)d->d_send_buf,
                       (const T *)src, d->d_send_nodes, d->n_send);
  HIP_THROW(hipGetLastError());
}

template <typename T>
void
launch_unpack(glsDist_ *d, void *dst, hipStream_t s, const gls::RelaxStep *rx)
{
  const T *rd    = rx ? (const T *)rx->d : nullptr;
  const T  scale = rx ? (T)rx->omega : T(0);
  const int nc = d->op->dim + 1;
  if (d->n_un == 0)
    return;
  const dim3 g((unsigned)((d->n_un * nc + 255) / 256));
  if (nc == 4)
    hipLaunchKernelGGL((gls::k_unpack_add<T, 4>), g, dim3(256), 0, s, (T *)dst,
                       (const T *)d->d_xrecv_buf, d->d_un_nodes, d->d_un_off, d->d_un_entry,
                       d->n_un, rd, scale);
  else
    hipLaunchKernelGGL((gls::k_unpack_add<T, 3>), g, dim3(256), 0, s, (T *)dst,
                       (const T *)d->d_xrecv_buf, d->d_un_nodes, d->d_un_off, d->d_un_entry,
                       d->n_un, rd, scale);
  HIP_THROW(hipGetLastError());
}

void
pack(glsDist_ *d, const void *src, hipStream_t s)
{
  if (d->op->prec == GLS_F64)
    launch_pack<double>(d, src, s);
  else
    launch_pack<float>(d, src, s);
}

void
unpack(glsDist_ *d, void *dst, hipStream_t s, const gls::RelaxStep *rx = nullptr)
{
  if (d->op->prec == GLS_F64)
    launch_unpack<double>(d, dst, s, rx);
  else
    launch_unpack<float>(d, dst, s, rx);
}

ncclDataType_t
nccl_type(const glsOp_ *op)
{
  return op->prec == GLS_F64 ? ncclDouble : ncclFloat;
}

// ---- RCCL transport
void
nccl_import(glsDist_ *d, void *src)
{
  const size_t rb = row_bytes(d->op);
  const int    nc = d->op->dim + 1;
  NCCL_THROW(ncclGroupStart());
  for (const Peer &p : d->peers)
    {
      if (p.recv_cnt > 0)
        NCCL_THROW(ncclRecv((char *)src + p.recv_begin * rb, (size_t)p.recv_cnt * nc,
                            nccl_type(d->op), p.rank, d->comm, d->cs));
      if (p.send_cnt > 0)
        NCCL_THROW(ncclSend((const char *)d->d_send_buf + p.send_off * rb,
                            (size_t)p.send_cnt * nc, nccl_type(d->op), p.rank, d->comm, d->cs));
    }
  NCCL_THROW(ncclGroupEnd());
}

void
nccl_export(glsDist_ *d, const void *dst, hipStream_t s)
{
  const size_t rb = row_bytes(d->op);
  const int    nc = d->op->dim + 1;
  NCCL_THROW(ncclGroupStart());
  for (const Peer &p : d->peers)
    {
      if (p.send_cnt > 0)
        NCCL_THROW(ncclRecv((char *)d->d_xrecv_buf + p.send_off * rb, (size_t)p.send_cnt * nc,
                            nccl_type(d->op), p.rank, d->comm, s));
      if (p.recv_cnt > 0)
        NCCL_THROW(ncclSend((const char *)dst + p.recv_begin * rb, (size_t)p.recv_cnt * nc,
                            nccl_type(d->op), p.rank, d->comm, s));
    }
  NCCL_THROW(ncclGroupEnd());
}

// ---- in-process transport: the same data movement as device copies (all
// members of the group share one device and run the phases in lockstep)
void
local_import(glsDist_ *d, hipStream_t s)
{
  const size_t rb = row_bytes(d->op);
  for (const Peer &p : d->peers)
    {
      if (p.recv_cnt == 0)
        continue;
      const glsDist_ *q  = d->group->members.at(p.rank);
      const Peer     *qp = find_peer(q, d->rank);
      if (!qp || qp->send_cnt != p.recv_cnt)
        throw std::runtime_error("gls_dist: inconsistent exchange lists");
      HIP_THROW(hipMemcpyAsync((char *)d->cur_src + p.recv_begin * rb,
                               (const char *)q->d_send_buf + qp->send_off * rb,
                               (size_t)p.recv_cnt * rb, hipMemcpyDeviceToDevice, s));
    }
}

void
local_export(glsDist_ *d, hipStream_t s)
{
  const size_t rb = row_bytes(d->op);
  for (const Peer &p : d->peers)
    {
      if (p.send_cnt == 0)
        continue;
      const glsDist_ *q  = d->group->members.at(p.rank);
      const Peer     *qp = find_peer(q, d->rank);
      if (!qp || qp->recv_cnt != p.send_cnt)
        throw std::runtime_error("gls_dist: inconsistent exchange lists");
      HIP_THROW(hipMemcpyAsync((char *)d->d_xrecv_buf + p.send_off * rb,
                               (const char *)q->cur_dst + qp->recv_begin * rb,
                               (size_t)p.send_cnt * rb, hipMemcpyDeviceToDevice, s));
    }
}

// every member's buf[i] <- the sum (or max) of the members' staged operands,
// in rank order
struct StageArgs
{
  const double *stage[16];
};
__global__ void
k_stage_reduce(double *buf, StageArgs a, int n, int64_t count, int max)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count)
    return;
  double v = a.stage[0][i];
  for (int r = 1; r < n; ++r)
    v = max ? fmax(v, a.stage[r][i]) : v + a.stage[r][i];
  buf[i] = v;
}

struct RcclTransport : Transport
{
  void
  import_ghosts(glsDist_ *d, void *src) override
  {
    nccl_import(d, src);
  }
  void
  export_ghosts(glsDist_ *d, const void *dst) override
  {
    nccl_export(d, dst, d->cs);
  }
  void
  allreduce(glsDist_ *d, double *buf, int64_t count, bool max, hipStream_t s) override
  {
    if (d->world > 1 && count > 0)
      NCCL_THROW(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, max ? ncclMax : ncclSum,
                               d->comm, s));
  }
};

// a member of an in-process group driven from its own host thread: the
// peers' buffers read by device copies on this member's streams, gated by
// the peers' events; the barriers make every member's record of an event
// precede the peers' waits on it (a wait on a not-yet-recorded event would
// not wait)
struct GroupTransport : Transport
{
  static void
  wait_peers(glsDist_ *d, hipStream_t s, hipEvent_t glsDist_::*ev)
  {
    for (const Peer &p : d->peers)
      HIP_THROW(hipStreamWaitEvent(s, d->group->members.at(p.rank)->*ev, 0));
  }
  void
  import_ghosts(glsDist_ *d, void *src) override
  {
    d->group->barrier(d); // every member's ev_packed recorded
    const size_t rb = row_bytes(d->op);
    for (const Peer &p : d->peers)
      {
        if (p.recv_cnt == 0)
          continue;
        const glsDist_ *q  = d->group->members.at(p.rank);
        const Peer     *qp = find_peer(q, d->rank);
        if (!qp || qp->send_cnt != p.recv_cnt)
          throw std::runtime_error("gls_dist: inconsistent exchange lists");
        HIP_THROW(hipStreamWaitEvent(d->cs, q->ev_packed, 0));
        HIP_THROW(hipMemcpyAsync((char *)src + p.recv_begin * rb,
                                 (const char *)q->d_send_buf + qp->send_off * rb,
                                 (size_t)p.recv_cnt * rb, hipMemcpyDeviceToDevice, d->cs));
      }
  }
  void
  export_ghosts(glsDist_ *d, const void *dst) override
  {
    d->cur_dst = const_cast<void *>(dst);
    d->group->barrier(d); // every member's ev_ghosts recorded, cur_dst set
    const size_t rb = row_bytes(d->op);
    for (const Peer &p : d->peers)
      {
        if (p.send_cnt == 0)
          continue;
        const glsDist_ *q  = d->group->members.at(p.rank);
        const Peer     *qp = find_peer(q, d->rank);
        if (!qp || qp->recv_cnt != p.send_cnt)
          throw std::runtime_error("gls_dist: inconsistent exchange lists");
        HIP_THROW(hipStreamWaitEvent(d->cs, q->ev_ghosts, 0));
        HIP_THROW(hipMemcpyAsync((char *)d->d_xrecv_buf + p.send_off * rb,
                                 (const char *)q->cur_dst + qp->recv_begin * rb,
                                 (size_t)p.send_cnt * rb, hipMemcpyDeviceToDevice, d->cs));
      }
  }
  void
  fence_send(glsDist_ *d, hipStream_t s) override
  {
    d->group->barrier(d); // the peers' last imports from this send buffer recorded
    wait_peers(d, s, &glsDist_::ev_imported);
  }
  void
  fence_ghosts(glsDist_ *d, hipStream_t s) override
  {
    d->group->barrier(d); // the peers' exports from these ghost rows recorded
    wait_peers(d, s, &glsDist_::ev_exported);
  }
  void
  allreduce(glsDist_ *d, double *buf, int64_t count, bool max, hipStream_t s) override
  {
    Group *g = d->group;
    g->barrier(d); // the last all-reduce's ev_red_done recorded everywhere
    for (glsDist_ *q : g->members)
      HIP_THROW(hipStreamWaitEvent(s, q->ev_red_done, 0));
    if (d->red_cap < count)
      {
        HIP_THROW(hipStreamSynchronize(s));
        if (d->red_stage)
          HIP_THROW(hipFree(d->red_stage));
        HIP_THROW(hipMalloc((void **)&d->red_stage, (size_t)count * sizeof(double)));
        d->red_cap = count;
      }
    if (count > 0)
      HIP_THROW(hipMemcpyAsync(d->red_stage, buf, (size_t)count * sizeof(double),
                               hipMemcpyDeviceToDevice, s));
    HIP_THROW(hipEventRecord(d->ev_red_staged, s));
    g->barrier(d); // every member's operand staged (and its pointer set)
    StageArgs a{};
    const int n = (int)g->members.size();
    if (n > 16)
      throw std::runtime_error("gls_dist: in-process groups of at most 16 members");
    for (int r = 0; r < n; ++r)
      {
        HIP_THROW(hipStreamWaitEvent(s, g->members[r]->ev_red_staged, 0));
        a.stage[r] = g->members[r]->red_stage;
      }
    if (count > 0)
      {
        hipLaunchKernelGGL(k_stage_reduce, dim3((unsigned)((count + 255) / 256)), dim3(256), 0,
                           s, buf, a, n, count, max ? 1 : 0);
        HIP_THROW(hipGetLastError());
      }
    HIP_THROW(hipEventRecord(d->ev_red_done, s));
  }
};

void
zero_ghosts(glsDist_ *d, void *dst, hipStream_t s)
{
  const glsOp_ *op = d->op;
  const size_t  g  = (size_t)(op->n_dofs - op->n_owned_dofs) * op->tsize();
  if (g)
    HIP_THROW(hipMemsetAsync((char *)dst + (size_t)op->n_owned_dofs * op->tsize(), 0, g, s));
}

void
check_vectors(glsDist_ *d, void *dst, void *src)
{
  if (!d || !dst || !src || dst == src)
    throw std::runtime_error("gls_dist_vmult: bad arguments");
  if (!d->op->have_lin)
    throw std::runtime_error("gls_dist_vmult before set_linearization_point");
  if (!d->op->use_brick)
    throw std::runtime_error("gls_dist_vmult needs the brick decomposition (glsOpDesc.brick)");
}
} // namespace

extern "C" {

glsStatus
gls_dist_unique_id(void *id_out)
{
  GLS_TRY
  if (!id_out)
    throw std::runtime_error("gls_dist_unique_id: null argument");
  ncclUniqueId id;
  NCCL_THROW(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  GLS_CATCH
}

glsStatus
gls_dist_create(glsOp op, const glsDistDesc *desc, glsDist *out)
{
  GLS_TRY
  if (!op || !desc || !out)
    throw std::runtime_error("gls_dist_create: null argument");
  if (op->faces.n)
    throw std::runtime_error("gls_dist_create: outflow faces are single-domain only");
  if (desc->world < 1 || desc->rank < 0 || desc->rank >= desc->world)
    throw std::runtime_error("gls_dist_create: bad rank / world");
  HIP_THROW(hipSetDevice(op->device));
  auto d   = std::make_unique<glsDist_>();
  d->op    = op;
  d->rank  = desc->rank;
  d->world = desc->world;
  int64_t off = 0;
  for (int i = 0; i < desc->n_peers; ++i)
    {
      Peer p;
      p.rank       = desc->peers[i];
      p.send_off   = off;
      p.send_cnt   = desc->send_count[i];
      p.recv_begin = desc->recv_begin[i];
      p.recv_cnt   = desc->recv_count[i];
      if (p.rank < 0 || p.rank >= d->world || p.rank == d->rank)
        throw std::runtime_error("gls_dist_create: bad peer rank");
      if (p.recv_cnt > 0 && (p.recv_begin < op->n_owned_nodes ||
                             p.recv_begin + p.recv_cnt > op->n_nodes))
        throw std::runtime_error("gls_dist_create: ghost block outside the ghost range");
      off += p.send_cnt;
      d->n_recv_nodes += p.recv_cnt;
      d->peers.push_back(p);
    }
  d->n_send = off;
  // send nodes (cmask bits attached) and the per-node CSR of the export-add
  std::vector<uint32_t> sn((size_t)d->n_send);
  for (int64_t j = 0; j < d->n_send; ++j)
    {
      const uint32_t node = desc->send_nodes[j];
      if ((int64_t)node >= op->n_owned_nodes)
        throw std::runtime_error("gls_dist_create: send node is not owned");
      sn[j] = node | (uint32_t)(op->h_cmask[node] & 0xF) << 28;
    }
  std::vector<uint32_t> idx((size_t)d->n_send);
  for (int64_t j = 0; j < d->n_send; ++j)
    idx[j] = (uint32_t)j;
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) {
    return (sn[x] & gls::NODE_MASK) < (sn[y] & gls::NODE_MASK);
  });
  std::vector<uint32_t> un, uoff{0}, uent;
  for (int64_t j = 0; j < d->n_send; ++j)
    {
      const uint32_t e = idx[j];
      if (un.empty() || (un.back() & gls::NODE_MASK) != (sn[e] & gls::NODE_MASK))
        {
          if (!un.empty())
            uoff.push_back((uint32_t)uent.size());
          un.push_back(sn[e]);
        }
      uent.push_back(e);
    }
  if (!un.empty())
    uoff.push_back((uint32_t)uent.size());
  d->n_un      = (int64_t)un.size();
  const size_t rb = row_bytes(op);
  auto up = [](void **p, const void *h, size_t bytes) {
    HIP_THROW(hipMalloc(p, std::max<size_t>(bytes, 16)));
    if (bytes)
      HIP_THROW(hipMemcpy(*p, h, bytes, hipMemcpyHostToDevice));
  };
  up((void **)&d->d_send_nodes, sn.data(), sn.size() * 4);
  up((void **)&d->d_un_nodes, un.data(), un.size() * 4);
  up((void **)&d->d_un_off, uoff.data(), uoff.size() * 4);
  up((void **)&d->d_un_entry, uent.data(), uent.size() * 4);
  HIP_THROW(hipMalloc(&d->d_send_buf, std::max<size_t>(16, (size_t)d->n_send * rb)));
  HIP_THROW(hipMalloc(&d->d_xrecv_buf, std::max<size_t>(16, (size_t)d->n_send * rb)));
  HIP_THROW(hipStreamCreateWithFlags(&d->cs, hipStreamNonBlocking));
  HIP_THROW(hipEventCreateWithFlags(&d->ev_packed, hipEventDisableTiming));
  HIP_THROW(hipEventCreateWithFlags(&d->ev_imported, hipEventDisableTiming));
  HIP_THROW(hipEventCreateWithFlags(&d->ev_ghosts, hipEventDisableTiming));
  HIP_THROW(hipEventCreateWithFlags(&d->ev_exported, hipEventDisableTiming));
  HIP_THROW(hipEventCreateWithFlags(&d->ev_red_staged, hipEventDisableTiming));
  HIP_THROW(hipEventCreateWithFlags(&d->ev_red_done, hipEventDisableTiming));
  if (desc->nccl_id)
    {
      ncclUniqueId id;
      std::memcpy(&id, desc->nccl_id, sizeof(id));
      NCCL_THROW(ncclCommInitRank(&d->comm, d->world, id, d->rank));
      d->tx = std::make_unique<RcclTransport>();
    }
  else
    {
      // in-process group: the members find each other through the group
      // handle passed as desc->group (NULL for the first member)
      Group *g = desc->group ? reinterpret_cast<glsDist_ *>(desc->group)->group : new Group;
      if ((int)g->members.size() < d->world)
        g->members.resize((size_t)d->world, nullptr);
      if (g->members[d->rank])
        throw std::runtime_error("gls_dist_create: rank already in the group");
      g->members[d->rank] = d.get();
      d->group            = g;
      d->tx               = std::make_unique<GroupTransport>();
    }
  *out = d.release();
  GLS_CATCH
}

void
gls_dist_destroy(glsDist d)
{
  if (!d)
    return;
  if (d->comm)
    (void)ncclCommDestroy(d->comm);
  if (d->group)
    {
      d->group->members[d->rank] = nullptr;
      bool empty                 = true;
      for (auto *m : d->group->members)
        empty = empty && !m;
      if (empty)
        delete d->group;
    }
  (void)hipFree(d->d_send_nodes);
  (void)hipFree(d->d_un_nodes);
  (void)hipFree(d->d_un_off);
  (void)hipFree(d->d_un_entry);
  (void)hipFree(d->d_send_buf);
  (void)hipFree(d->d_xrecv_buf);
  if (d->ev_packed)
    (void)hipEventDestroy(d->ev_packed);
  if (d->ev_imported)
    (void)hipEventDestroy(d->ev_imported);
  for (hipEvent_t e : {d->ev_ghosts, d->ev_exported, d->ev_red_staged, d->ev_red_done})
    if (e)
      (void)hipEventDestroy(e);
  if (d->red_stage)
    (void)hipFree(d->red_stage);
  if (d->cs)
    (void)hipStreamDestroy(d->cs);
  delete d;
}

namespace
{
// the partitioned vmult of one rank (RCCL, or a threaded in-process member);
// rx: the damped-Jacobi step (or the
// residual) fused into the local bricks and reduce on the owned rows, the
// peers' contributions entering through the unpack (k_unpack_add)
void
dist_vmult(glsDist d, void *dst, void *src, hipStream_t s, const gls::RelaxStep *rx)
{
  check_vectors(d, dst, src);
  glsOp_       *op   = d->op;
  const int     mode = gls::op_vmult_mode(op);
  if (d->comm && d->peers.empty()) // one RCCL rank: nothing to exchange
    {
      gls::brick_launch(op, mode, dst, src, 0, op->n_bricks, gls::BRICK_RUN | gls::BRICK_REDUCE,
                        s, rx);
      zero_ghosts(d, dst, s);
      return;
    }
  const int64_t ni = op->n_interior_bricks, nh = ni / 2;
  // import (comm stream) || first interior half (s)
  d->tx->fence_send(d, s);
  pack(d, src, s);
  HIP_THROW(hipEventRecord(d->ev_packed, s));
  HIP_THROW(hipStreamWaitEvent(d->cs, d->ev_packed, 0));
  d->tx->import_ghosts(d, src);
  HIP_THROW(hipEventRecord(d->ev_imported, d->cs));
  gls::brick_launch(op, mode, dst, src, 0, nh, gls::BRICK_RUN, s, rx);
  // boundary units and the ghost rows they complete
  HIP_THROW(hipStreamWaitEvent(s, d->ev_imported, 0));
  gls::brick_launch(op, mode, dst, src, ni, op->n_bricks,
                    gls::BRICK_RUN | gls::BRICK_REDUCE_GHOST, s, rx);
  HIP_THROW(hipEventRecord(d->ev_ghosts, s));
  // compress(add) of the ghost rows (comm stream) || second interior half
  // and the owned rows' reduction (s)
  HIP_THROW(hipStreamWaitEvent(d->cs, d->ev_ghosts, 0));
  d->tx->export_ghosts(d, dst);
  HIP_THROW(hipEventRecord(d->ev_exported, d->cs));
  gls::brick_launch(op, mode, dst, src, nh, ni, gls::BRICK_RUN | gls::BRICK_REDUCE_OWNED, s, rx);
  HIP_THROW(hipStreamWaitEvent(s, d->ev_exported, 0));
  unpack(d, dst, s, rx);
  d->tx->fence_ghosts(d, s);
  zero_ghosts(d, dst, s);
}

// the in-process group's vmult; rx: per member, or null
void
dist_vmult_group(glsDist const *members, void *const *dsts, void *const *srcs, int n,
                 hipStream_t s, const gls::RelaxStep *rx)
{
  if (!members || !dsts || !srcs || n < 1)
    throw std::runtime_error("gls_dist_vmult_group: bad arguments");
  for (int r = 0; r < n; ++r)
    {
      check_vectors(members[r], dsts[r], srcs[r]);
      if (!members[r]->group)
        throw std::runtime_error("gls_dist_vmult_group: not an in-process group");
      members[r]->cur_dst = dsts[r];
      members[r]->cur_src = srcs[r];
    }
  // the phases of dist_vmult, member by member in lockstep on one stream
  for (int r = 0; r < n; ++r)
    pack(members[r], srcs[r], s);
  for (int r = 0; r < n; ++r)
    {
      glsOp_ *op = members[r]->op;
      gls::brick_launch(op, gls::op_vmult_mode(op), dsts[r], srcs[r], 0,
                        op->n_interior_bricks / 2, gls::BRICK_RUN, s, rx ? rx + r : nullptr);
    }
  for (int r = 0; r < n; ++r)
    local_import(members[r], s);
  for (int r = 0; r < n; ++r)
    {
      glsOp_ *op = members[r]->op;
      gls::brick_launch(op, gls::op_vmult_mode(op), dsts[r], srcs[r], op->n_interior_bricks,
                        op->n_bricks, gls::BRICK_RUN | gls::BRICK_REDUCE_GHOST, s,
                        rx ? rx + r : nullptr);
    }
  for (int r = 0; r < n; ++r)
    local_export(members[r], s);
  for (int r = 0; r < n; ++r)
    {
      glsOp_ *op = members[r]->op;
      gls::brick_launch(op, gls::op_vmult_mode(op), dsts[r], srcs[r], op->n_interior_bricks / 2,
                        op->n_interior_bricks, gls::BRICK_RUN | gls::BRICK_REDUCE_OWNED, s,
                        rx ? rx + r : nullptr);
    }
  for (int r = 0; r < n; ++r)
    unpack(members[r], dsts[r], s, rx ? rx + r : nullptr);
  for (int r = 0; r < n; ++r)
    zero_ghosts(members[r], dsts[r], s);
}
} // namespace

glsStatus
gls_dist_vmult(glsDist d, void *dst, void *src, void *stream)
{
  GLS_TRY
  gls::Section sec_("ns::vmult", (hipStream_t)stream);
  dist_vmult(d, dst, src, (hipStream_t)stream, nullptr);
  GLS_CATCH
}

glsStatus
gls_dist_vmult_group(glsDist const *members, void *const *dsts, void *const *srcs, int n,
                     void *stream)
{
  GLS_TRY
  dist_vmult_group(members, dsts, srcs, n, (hipStream_t)stream, nullptr);
  GLS_CATCH
}

glsStatus
gls_dist_update_ghost_values(glsDist d, void *vec, void *stream)
{
  GLS_TRY
  if (!d || !vec)
    throw std::runtime_error("gls_dist_update_ghost_values: null argument");
  hipStream_t s = (hipStream_t)stream;
  if (!(d->comm && d->peers.empty()))
    {
      d->tx->fence_send(d, s);
      pack(d, vec, s);
      HIP_THROW(hipEventRecord(d->ev_packed, s));
      HIP_THROW(hipStreamWaitEvent(d->cs, d->ev_packed, 0));
      d->tx->import_ghosts(d, vec);
      HIP_THROW(hipEventRecord(d->ev_imported, d->cs));
      HIP_THROW(hipStreamWaitEvent(s, d->ev_imported, 0));
    }
  GLS_CATCH
}

glsStatus
gls_dist_compress_add(glsDist d, void *vec, void *stream)
{
  GLS_TRY
  if (!d || !vec)
    throw std::runtime_error("gls_dist_compress_add: null argument");
  hipStream_t s = (hipStream_t)stream;
  if (!(d->comm && d->peers.empty()))
    {
      HIP_THROW(hipEventRecord(d->ev_ghosts, s));
      HIP_THROW(hipStreamWaitEvent(d->cs, d->ev_ghosts, 0));
      d->tx->export_ghosts(d, vec);
      HIP_THROW(hipEventRecord(d->ev_exported, d->cs));
      HIP_THROW(hipStreamWaitEvent(s, d->ev_exported, 0));
      unpack(d, vec, s);
      d->tx->fence_ghosts(d, s);
    }
  zero_ghosts(d, vec, s);
  GLS_CATCH
}

glsStatus
gls_dist_get_max_u(glsDist d, void *vec, double *u_max, void *stream)
{
  GLS_TRY
  if (!d || !vec || !u_max)
    throw std::runtime_error("gls_dist_get_max_u: null argument");
  // operator_ns.cc:540-567: vec.update_ghost_values(); local max over the
  // locally owned cells; Utilities::MPI::max
  if (gls_dist_update_ghost_values(d, vec, stream) != 0)
    throw std::runtime_error(gls_last_error());
  double local = 0;
  if (gls_op_get_max_u(d->op, vec, &local, stream) != 0)
    throw std::runtime_error(gls_last_error());
  hipStream_t s   = (hipStream_t)stream;
  double     *buf = nullptr;
  HIP_THROW(hipMallocAsync((void **)&buf, sizeof(double), s));
  HIP_THROW(hipMemcpyAsync(buf, &local, sizeof(double), hipMemcpyHostToDevice, s));
  d->tx->allreduce(d, buf, 1, true, s);
  HIP_THROW(hipMemcpyAsync(u_max, buf, sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_THROW(hipFreeAsync(buf, s));
  HIP_THROW(hipStreamSynchronize(s));
  GLS_CATCH
}

glsStatus
gls_dist_interior_bricks(glsDist d, int64_t *n_interior, int64_t *n_total)
{
  GLS_TRY
  if (!d)
    throw std::runtime_error("gls_dist_interior_bricks: null argument");
  if (n_interior)
    *n_interior = d->op->n_interior_bricks;
  if (n_total)
    *n_total = d->op->n_bricks;
  GLS_CATCH
}

} // extern "C"

// ---- team primitives of the partitioned multigrid and GMRES (dist_mg.hip):
// a "team" is the set of ranks this process drives in lockstep — one RCCL
// rank (n = 1, members[0]->comm), or every member of an in-process group
namespace gls
{
namespace
{
constexpr int TEAM_MAX = 16;
struct SumArgs
{
  double *buf[TEAM_MAX];
};
// every member's buf[i] <- the sum over the members in member order
__global__ void
k_team_sum(SumArgs a, int n, int64_t count)
{
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count)
    return;
  double s = 0;
  for (int r = 0; r < n; ++r)
    s += a.buf[r][i];
  for (int r = 0; r < n; ++r)
    a.buf[r][i] = s;
}

// a team of one: an RCCL rank, or a member of an in-process group driven
// from its own host thread (both through the member's Transport)
bool
rank_mode(glsDist const *m, int n)
{
  return n == 1 && m[0] && (m[0]->comm || (m[0]->group && m[0]->world > 1));
}

void
check_team(glsDist const *m, int n)
{
  if (!m || n < 1 || n > TEAM_MAX)
    throw std::runtime_error("gls_dist team: bad member list");
  if (rank_mode(m, n))
    return;
  for (int r = 0; r < n; ++r)
    if (!m[r] || m[r]->comm || !m[r]->group || m[r]->rank != r || m[r]->world != n)
      throw std::runtime_error("gls_dist team: an in-process group is driven with all its "
                               "members in rank order (lockstep) or one member per host thread; "
                               "RCCL ranks one at a time");
}
} // namespace

glsOp_ *
dist_op(glsDist d)
{
  return d->op;
}

// a member of an in-process group (several partitions on one device)
bool
dist_in_process(glsDist d)
{
  return d && d->group != nullptr;
}

int
dist_rank(glsDist d)
{
  return d->rank;
}

int
dist_world(glsDist d)
{
  return d->world;
}

void
team_vmult(glsDist const *m, void *const *dst, void *const *src, int n, hipStream_t s,
           const RelaxStep *rx)
{
  check_team(m, n);
  if (rank_mode(m, n))
    dist_vmult(m[0], dst[0], src[0], s, rx);
  else
    dist_vmult_group(m, dst, src, n, s, rx);
}

void
team_update_ghosts(glsDist const *m, void *const *v, int n, hipStream_t s)
{
  check_team(m, n);
  if (rank_mode(m, n))
    {
      if (gls_dist_update_ghost_values(m[0], v[0], s))
        throw std::runtime_error(gls_last_error());
      return;
    }
  for (int r = 0; r < n; ++r)
    {
      m[r]->cur_src = v[r];
      pack(m[r], v[r], s);
    }
  for (int r = 0; r < n; ++r)
    local_import(m[r], s);
}

void
team_compress_add(glsDist const *m, void *const *v, int n, hipStream_t s)
{
  check_team(m, n);
  if (rank_mode(m, n))
    {
      if (gls_dist_compress_add(m[0], v[0], s))
        throw std::runtime_error(gls_last_error());
      return;
    }
  for (int r = 0; r < n; ++r)
    m[r]->cur_dst = v[r];
  for (int r = 0; r < n; ++r)
    local_export(m[r], s);
  for (int r = 0; r < n; ++r)
    unpack(m[r], v[r], s);
  for (int r = 0; r < n; ++r)
    zero_ghosts(m[r], v[r], s);
}

void
team_allreduce_sum(glsDist const *m, double *const *buf, int64_t count, int n, hipStream_t s)
{
  check_team(m, n);
  if (count <= 0)
    return;
  if (rank_mode(m, n))
    {
      m[0]->tx->allreduce(m[0], buf[0], count, false, s);
      return;
    }
  SumArgs a{};
  for (int r = 0; r < n; ++r)
    a.buf[r] = buf[r];
  hipLaunchKernelGGL(k_team_sum, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, a, n,
                     count);
  HIP_THROW(hipGetLastError());
}
} // namespace gls

