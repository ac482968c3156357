// dmf_comm.hip — multi-GPU merge of the fusion counters and visibility flags over a
// caller's RCCL communicator.
//
// Poses shard across ranks; every rank holds a full grid replica.  The reference has no
// multi-GPU path: these entry points are what a C++ caller of the reference API adds to
// run configs 4/5.  The communicator is an ncclComm_t passed as
// void* (e.g. torch's ProcessGroupNCCL._comm_ptr(), or dmf_comm_init_rank below); all
// collectives are enqueued on the volume's stream and nothing synchronises the host.
//
// Merge-and-finalize moves 10 B/cell instead of the all-reduce's 16 (2 x 8 B int32 x 2):
// reduce-scatter of hits and of misses over whole tile rows, the rank finalizes its slab
// of tile rows into int16 log-odds, all-gather of the int16 slabs.
#include <algorithm>
#include <cstring>

#include <rccl/rccl.h>

#include "dmf_host.hpp"

namespace dmf {

#define DMF_NCCL(expr)                                                                        \
  do {                                                                                        \
    ncclResult_t r_ = (expr);                                                                 \
    if (r_ != ncclSuccess)                                                                    \
      return ::dmf::fail(DMF_ERR_HIP, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), \
                         __FILE__, __LINE__);                                                 \
  } while (0)

static int comm_shape(void* comm, int* nranks, int* rank) {
  if (!comm) return fail(DMF_ERR_INVALID, "null communicator");
  DMF_NCCL(ncclCommCount((ncclComm_t)comm, nranks));
  DMF_NCCL(ncclCommUserRank((ncclComm_t)comm, rank));
  return DMF_OK;
}

// The merge's slab arithmetic for `rank` of `nranks` (rank = -1: the whole grid, as one
// rank that holds every slab) on a grid of dims (x, y, z), shared by the collective merge
// and the exported plans.  Tile rows (2 x-rows of 2x2x4-cell tiles) per rank:
// whole rows, equal counts per rank, the counter arrays padded to nranks * rows rows.
static dmf_merge_plan merge_plan_dims(int64_t xd, int64_t yd, int64_t zd, int nranks, int rank) {
  const int64_t ntx = (xd + 1) >> 1, tpr = ((yd + 1) >> 1) * ((zd + 3) >> 2);
  const int64_t rows = (ntx + nranks - 1) / nranks;
  dmf_merge_plan p{};
  p.n_padded = rows * nranks * tpr * 16;
  p.chunk = rows * tpr * 16;
  p.logodds_padded = rows * nranks * 2 * yd * zd;
  p.slab_bytes = rows * 2 * yd * zd * (int64_t)sizeof(int16_t);
  if (rank < 0) {
    p.chunk_offset = 0;
    p.tile_begin = 0;
    p.tile_end = ntx * tpr;
    p.slab_offset = 0;
  } else {
    p.chunk_offset = rank * p.chunk;
    // the rank's slab: tile rows [rank*rows, (rank+1)*rows) clipped to the grid (the last
    // ranks of a grid with fewer tile rows than ranks * rows hold padding only)
    p.tile_begin = std::min<int64_t>(ntx, rank * rows) * tpr;
    p.tile_end = std::min<int64_t>(ntx, (rank + 1) * rows) * tpr;
    p.slab_offset = rank * p.slab_bytes;
  }
  return p;
}

static dmf_merge_plan merge_plan(const dmf_volume* v, int nranks, int rank) {
  return merge_plan_dims(v->xdim, v->ydim, v->zdim, nranks, rank);
}

// ncclGroupStart / ncclGroupEnd as a scope: an early error return between them still
// closes the group (a group left open would absorb the caller's later collectives).
struct NcclGroup {
  bool open = false;
  ncclResult_t start() {
    const ncclResult_t r = ncclGroupStart();
    open = r == ncclSuccess;
    return r;
  }
  ncclResult_t end() {
    open = false;
    return ncclGroupEnd();
  }
  ~NcclGroup() {
    if (open) ncclGroupEnd();
  }
};

// Voxel::view merge: the smallest non-zero id over the ranks (0 = never viewed).
__global__ void k_view_zero_to_max(int32_t* view, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && view[i] == 0) view[i] = INT32_MAX;
}
__global__ void k_view_max_to_zero(int32_t* view, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && view[i] == INT32_MAX) view[i] = 0;
}

}  // namespace dmf

using namespace dmf;

extern "C" {

int dmf_rccl_version(int32_t* version) {
  DMF_API_BEGIN
  if (!version) return fail(DMF_ERR_INVALID, "null argument");
  int v = 0;
  DMF_NCCL(ncclGetVersion(&v));
  *version = v;
  return DMF_OK;
  DMF_API_END
}

int dmf_comm_unique_id(void* id) {
  DMF_API_BEGIN
  if (!id) return fail(DMF_ERR_INVALID, "null argument");
  static_assert(sizeof(ncclUniqueId) == DMF_COMM_ID_BYTES, "ncclUniqueId size");
  DMF_NCCL(ncclGetUniqueId((ncclUniqueId*)id));
  return DMF_OK;
  DMF_API_END
}

int dmf_comm_init_rank(void** comm, int32_t nranks, const void* id, int32_t rank, int32_t device) {
  DMF_API_BEGIN
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(DMF_ERR_INVALID, "bad communicator arguments");
  DMF_HIP(hipSetDevice(device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  DMF_NCCL(ncclCommInitRank(&c, nranks, uid, rank));
  *comm = (void*)c;
  return DMF_OK;
  DMF_API_END
}

int dmf_comm_shape(void* comm, int32_t* nranks, int32_t* rank) {
  DMF_API_BEGIN
  if (!nranks || !rank) return fail(DMF_ERR_INVALID, "null argument");
  int nr = 0, rk = 0;
  DMF_TRY(comm_shape(comm, &nr, &rk));
  *nranks = nr;
  *rank = rk;
  return DMF_OK;
  DMF_API_END
}

int dmf_comm_destroy(void* comm) {
  DMF_API_BEGIN
  if (!comm) return DMF_OK;
  DMF_NCCL(ncclCommDestroy((ncclComm_t)comm));
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_counter_cells_padded(const dmf_volume* v, int32_t nranks, int64_t* n) {
  DMF_API_BEGIN
  if (!n || nranks < 1) return fail(DMF_ERR_INVALID, "bad argument");
  DMF_TRY(require_constructed(v));
  *n = merge_plan(v, nranks, 0).n_padded;
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_logodds_cells_padded(const dmf_volume* v, int32_t nranks, int64_t* n) {
  DMF_API_BEGIN
  if (!n || nranks < 1) return fail(DMF_ERR_INVALID, "bad argument");
  DMF_TRY(require_constructed(v));
  *n = merge_plan(v, nranks, 0).logodds_padded;
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_merge_plan(const dmf_volume* v, int32_t nranks, int32_t rank, dmf_merge_plan* out) {
  DMF_API_BEGIN
  if (!out || nranks < 1 || rank < -1 || rank >= nranks) return fail(DMF_ERR_INVALID, "bad argument");
  DMF_TRY(require_constructed(v));
  *out = merge_plan(v, nranks, rank);
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_merge_plan_dims(int32_t xdim, int32_t ydim, int32_t zdim, int32_t nranks, int32_t rank,
                             dmf_merge_plan* out) {
  DMF_API_BEGIN
  if (!out || nranks < 1 || rank < -1 || rank >= nranks || xdim < 1 || ydim < 1 || zdim < 1)
    return fail(DMF_ERR_INVALID, "bad argument");
  *out = merge_plan_dims(xdim, ydim, zdim, nranks, rank);
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_finalize_slab_device(dmf_volume* v, const int32_t* d_counters, const dmf_fuse_params* prm,
                                  int16_t* d_logodds, int32_t nranks, int32_t rank, void* stream) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!d_counters || !prm || !d_logodds) return fail(DMF_ERR_INVALID, "null argument");
  if (nranks < 1 || rank < -1 || rank >= nranks) return fail(DMF_ERR_INVALID, "bad rank %d of %d", rank, nranks);
  const hipStream_t st = stream ? (hipStream_t)stream : v->stream;
  const dmf_merge_plan p = merge_plan(v, nranks, rank);
  return finalize_tiles(v, d_counters, d_counters + p.n_padded, prm, d_logodds, p.tile_begin, p.tile_end, st);
  DMF_API_END
}

int dmf_fuse_allreduce_device(dmf_volume* v, int32_t* d_counters, int64_t n_per_array, void* comm, void* stream) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  const hipStream_t st = stream ? (hipStream_t)stream : v->stream;
  if (!d_counters || n_per_array <= 0) return fail(DMF_ERR_INVALID, "bad counter buffer");
  int nr, rk;
  DMF_TRY(comm_shape(comm, &nr, &rk));
  DMF_NCCL(ncclAllReduce(d_counters, d_counters, (size_t)(2 * n_per_array), ncclInt32, ncclSum, (ncclComm_t)comm,
                         st));
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_merge_finalize_device(dmf_volume* v, int32_t* d_counters, const dmf_fuse_params* prm,
                                   int16_t* d_logodds, void* comm, void* stream) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  const hipStream_t st = stream ? (hipStream_t)stream : v->stream;
  if (!d_counters || !prm || !d_logodds) return fail(DMF_ERR_INVALID, "null argument");
  int nr = 1, rk = 0;
  if (comm) DMF_TRY(comm_shape(comm, &nr, &rk));  // NULL: one rank, no collective
  const dmf_merge_plan p = merge_plan(v, nr, rk);
  int32_t* d_hits = d_counters;
  int32_t* d_miss = d_counters + p.n_padded;
  if (comm) {  // in place: this rank's reduced slab lands at its own offset of each array
    NcclGroup grp;
    DMF_NCCL(grp.start());
    DMF_NCCL(ncclReduceScatter(d_hits, d_hits + p.chunk_offset, (size_t)p.chunk, ncclInt32, ncclSum,
                               (ncclComm_t)comm, st));
    DMF_NCCL(ncclReduceScatter(d_miss, d_miss + p.chunk_offset, (size_t)p.chunk, ncclInt32, ncclSum,
                               (ncclComm_t)comm, st));
    DMF_NCCL(grp.end());
  }
  DMF_TRY(finalize_tiles(v, d_hits, d_miss, prm, d_logodds, p.tile_begin, p.tile_end, st));
  // int16 slabs of 2*rows x-rows each, gathered in rank order (bytes: RCCL has no int16)
  if (comm)
    DMF_NCCL(ncclAllGather((const char*)d_logodds + p.slab_offset, d_logodds, (size_t)p.slab_bytes, ncclUint8,
                           (ncclComm_t)comm, st));
  return DMF_OK;
  DMF_API_END
}

int dmf_flags_allreduce(dmf_volume* v, void* comm, void* stream) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  const hipStream_t st = stream ? (hipStream_t)stream : v->stream;
  int nr, rk;
  DMF_TRY(comm_shape(comm, &nr, &rk));
  if (v->V == 0) return DMF_OK;
  const int64_t n = (int64_t)v->V;
  const unsigned nb = (unsigned)((n + 255) / 256);
  // view: the smallest non-zero id (0 -> INT32_MAX, min, back); good: max (a flag).  The
  // restore runs on every exit path once the rewrite is enqueued: a failed
  // collective leaves the view ids as they were on this rank, never INT32_MAX.
  hipLaunchKernelGGL(k_view_zero_to_max, dim3(nb), dim3(256), 0, st, v->d_view, n);
  DMF_LAUNCH_CHECK();
  // the guard restores on error / exception exits only; the success path launches the restore
  // itself and checks that launch
  struct Restore {
    int32_t* view;
    int64_t n;
    unsigned nb;
    hipStream_t st;
    bool armed = true;
    ~Restore() {
      if (armed) hipLaunchKernelGGL(k_view_max_to_zero, dim3(nb), dim3(256), 0, st, view, n);
    }
  } restore{v->d_view, n, nb, st};
  {
    NcclGroup grp;
    DMF_NCCL(grp.start());
    DMF_NCCL(ncclAllReduce(v->d_view, v->d_view, (size_t)n, ncclInt32, ncclMin, (ncclComm_t)comm, st));
    DMF_NCCL(ncclAllReduce(v->d_good, v->d_good, (size_t)n, ncclUint8, ncclMax, (ncclComm_t)comm, st));
    DMF_NCCL(grp.end());
  }
  restore.armed = false;
  hipLaunchKernelGGL(k_view_max_to_zero, dim3(nb), dim3(256), 0, st, v->d_view, n);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"
