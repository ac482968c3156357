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

// Tile rows per rank of the padded counter layout (whole rows, equal counts per rank).
static int64_t rows_per_rank(const dmf_volume* v, int nranks) {
  int64_t ntx, tpr;
  tile_rows(v, &ntx, &tpr);
  return (ntx + nranks - 1) / nranks;
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
  int64_t ntx, tpr;
  tile_rows(v, &ntx, &tpr);
  *n = rows_per_rank(v, nranks) * nranks * tpr * 16;
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_logodds_cells_padded(const dmf_volume* v, int32_t nranks, int64_t* n) {
  DMF_API_BEGIN
  if (!n || nranks < 1) return fail(DMF_ERR_INVALID, "bad argument");
  DMF_TRY(require_constructed(v));
  *n = rows_per_rank(v, nranks) * nranks * 2 * (int64_t)v->ydim * v->zdim;
  return DMF_OK;
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
  int64_t ntx, tpr;
  tile_rows(v, &ntx, &tpr);
  const int64_t rows = rows_per_rank(v, nr);
  const int64_t n_pad = rows * nr * tpr * 16;      // elements per counter array
  const size_t chunk = (size_t)(rows * tpr * 16);  // this rank's reduced slab of each
  int32_t* d_hits = d_counters;
  int32_t* d_miss = d_counters + n_pad;
  if (comm) {
    DMF_NCCL(ncclGroupStart());
    DMF_NCCL(ncclReduceScatter(d_hits, d_hits + rk * chunk, chunk, ncclInt32, ncclSum, (ncclComm_t)comm, st));
    DMF_NCCL(ncclReduceScatter(d_miss, d_miss + rk * chunk, chunk, ncclInt32, ncclSum, (ncclComm_t)comm, st));
    DMF_NCCL(ncclGroupEnd());
  }
  // the rank's slab: tile rows [rk*rows, (rk+1)*rows) clipped to the grid
  const int64_t r0 = std::min<int64_t>(ntx, rk * rows), r1 = std::min<int64_t>(ntx, (rk + 1) * rows);
  DMF_TRY(finalize_tiles(v, d_hits, d_miss, prm, d_logodds, r0 * tpr, r1 * tpr, st));
  // int16 slabs of 2*rows x-rows each, gathered in rank order (bytes: RCCL has no int16)
  const size_t slab = (size_t)(rows * 2 * (int64_t)v->ydim * v->zdim) * sizeof(int16_t);
  if (comm) DMF_NCCL(ncclAllGather((const char*)d_logodds + rk * slab, d_logodds, slab, ncclUint8, (ncclComm_t)comm, st));
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
  DMF_NCCL(ncclGroupStart());
  DMF_NCCL(ncclAllReduce(v->d_view, v->d_view, (size_t)v->V, ncclInt32, ncclMax, (ncclComm_t)comm, st));
  DMF_NCCL(ncclAllReduce(v->d_good, v->d_good, (size_t)v->V, ncclUint8, ncclMax, (ncclComm_t)comm, st));
  DMF_NCCL(ncclGroupEnd());
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"
