// dmf_host.hpp — host-side plumbing shared by the C-ABI translation units:
// status/error reporting, HIP error checks, the per-volume scratch arena and the
// pose-table upload.  No compute lives here.
#pragma once
#include <cstdarg>
#include <cstdio>
#include <new>

#include "dmf_internal.hpp"

namespace dmf {

void set_error(const char* fmt, ...);
int fail(int status, const char* fmt, ...);

#define DMF_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return ::dmf::fail(DMF_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                         __FILE__, __LINE__);                                           \
  } while (0)

#define DMF_TRY(expr)            \
  do {                           \
    int s_ = (expr);             \
    if (s_ != DMF_OK) return s_; \
  } while (0)

#define DMF_LAUNCH_CHECK() DMF_HIP(hipGetLastError())

// Guard every C entry point: no C++ exception crosses the ABI.
#define DMF_API_BEGIN try {
#define DMF_API_END                                                        \
  }                                                                        \
  catch (const std::bad_alloc&) {                                          \
    return ::dmf::fail(DMF_ERR_NOMEM, "host allocation failed");           \
  }                                                                        \
  catch (...) {                                                            \
    return ::dmf::fail(DMF_ERR_INVALID, "unexpected C++ exception");       \
  }

// Make v's device current (HIP device state is per host thread).
int activate(const dmf_volume* v);
inline dmf_volume* v_mut(const dmf_volume* v) { return const_cast<dmf_volume*>(v); }
int require_constructed(const dmf_volume* v);

// Scratch arena: slot k is a device buffer grown on demand, reused across calls.
int scratch(dmf_volume* v, int k, size_t bytes, void** out);
enum ScratchSlot {
  kScPoses = 0, kScHost0, kScHost1, kScHost2, kScOut0, kScOut1, kScOut2, kScOut3, kScTmp, kScSort0,
  kScSort1, kScSort2, kScSort3, kScCount, kScStats,
  // brick-owned fusion (dmf_fuse.hip)
  kScBkRays, kScBkPairs, kScBkPairsB, kScBkBricks, kScBkWgBase, kScBkCtl, kScBkPoseCnt, kScBkPoseBase, kScBkBatch,
  kScBkWgList,
  // the second staging slot of pipelined fusion (dmf_fuse_set_input_stream) and the
  // per-slot pose tables / pass-A statistics
  kScBkRays1, kScBkWgBase1, kScBkWgList1, kScBkPoseCnt1, kScBkBatch1, kScStPoses0, kScStPoses1, kScStStats0,
  kScStStats1,
  // ... and, when pass B is staged as well, the second slot's brick layout and pair records
  kScBkBricks1, kScBkCtl1, kScBkPairs1, kScBkPairsB1, kScBkPoseBase1,
  kScOgP0, kScOgP1, kScOgFinal, kScOgOcc,  // OccupancyGrid reorganization (dmf_ogrid.hip)
  kScRevItems,  // reverseRayTraceFast's item-ordered (spatial order) result masks (dmf_trace.hip)
  kScBkOvf, kScBkOvf1  // pass A's hashed-histogram overflow lists, per staging slot (dmf_fuse.hip)
};

// Striped statistics: kernels add into slot (block % kStatSlots) of a zeroed buffer
// of kStatSlots x kStatWidth counters (one hot address per counter serialises at the
// memory side); stats_end() sums the slots into the caller's counters.
#if defined(DMF_EXP_STATS)
constexpr int kStatSlots = 256, kStatWidth = 20;  // diagnostic builds: extra counters 7..19
#else
constexpr int kStatSlots = 256, kStatWidth = 8;
#endif
int stats_begin(dmf_volume* v, unsigned long long** striped);
// (on `stream`, the volume's stream by default; the sums are atomic: a pipelined call's
// pass-A statistics are summed on the staging stream while the previous call's are on the
// volume's)
int stats_end(dmf_volume* v, const unsigned long long* striped, uint64_t* d_user, int ncounters,
              uint32_t* fault = nullptr, hipStream_t stream = nullptr);
__device__ inline unsigned long long* stat_slot(unsigned long long* base) {
  return base ? base + kStatWidth * ((blockIdx.x + blockIdx.y * gridDim.x) & (kStatSlots - 1)) : nullptr;
}

// Upload P host poses (or take device poses) and build the PoseX table on device.
int pose_table(dmf_volume* v, const float* poses, int P, bool poses_on_device, PoseX** d_table);
// The same table from P device poses into d_out, on stream s (the staging stream of a
// pipelined fusion call).
int pose_table_into(const float* d_poses, int P, PoseX* d_out, hipStream_t s);

CamP cam_params(const dmf_camera* c);

// Fusion finalize over tiled counters, tiles [t0, t1) (dmf_fuse.hip); the tiled layout's
// x extent in 2-cell tile rows and tiles per row (a contiguous tile range of whole rows is
// an x slab of the grid).
int finalize_tiles(dmf_volume* v, const int32_t* d_hits, const int32_t* d_misses, const dmf_fuse_params* prm,
                   int16_t* d_out, int64_t t0, int64_t t1, hipStream_t stream);
int tile_rows(const dmf_volume* v, int64_t* ntx, int64_t* tiles_per_row);
int check_camera(const dmf_camera* c);

// Lazily (re)build the float-accumulated enumeration list (reverseRayTrace / rayTraceVolume).
int ensure_enumeration(dmf_volume* v);
int ensure_brick_dist(dmf_volume* v);

// Device-wide helpers implemented with rocPRIM in dmf_core.hip.
int exclusive_scan_i64(dmf_volume* v, const int64_t* in, int64_t* out, size_t n);
int exclusive_scan_i32(dmf_volume* v, const int32_t* in, int32_t* out, size_t n);
int sort_pairs_u64(dmf_volume* v, uint64_t* keys, uint64_t* vals, size_t n, int end_bit);
int sort_pairs_u32(dmf_volume* v, uint32_t* keys, uint32_t* vals, size_t n, int end_bit);

// Order-preserving compaction of per-pose bitmasks (P x words) into concatenated
// lists: element e of pose p with bit set -> out[base[p] + rank] = value(e).
// value source: hash[e] (slot lists) or a callback kernel (enumeration lists).
int compact_masks(dmf_volume* v, const uint64_t* d_masks, int P, int64_t words, int64_t nelem,
                  int64_t* counts_h, uint64_t** d_out_lists, int64_t* total, int value_kind);
enum { kValueSlotHash = 0, kValueEnumCentroidHash = 1 };

}  // namespace dmf
