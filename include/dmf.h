/*
 * dmf.h — C ABI of the MI355X-native voxel ray-tracing / depth-fusion engine.
 *
 * The reference (REXJJ/depth-map-fusion-utils) has no FFI layer: its boundary is the
 * header-only C++ class API of include/Camera.hpp, include/Volume.hpp and
 * include/RayTracingEngine.hpp.  Every entry point below names the
 * reference member it replaces (file:line in the reference tree).  The C++ drop-in
 * classes in depth-map-fusion-utils_amd/compat/ and the Python mirror in dmf_amd/
 * are thin layers over this ABI; see INTEGRATION.md for the bindings.
 *
 * Conventions
 *  - All calls return an int status (DMF_OK == 0); nothing throws across the ABI.
 *    dmf_last_error() returns a thread-local message for the last failure.
 *  - A dmf_volume is one device-resident VoxelVolume plus its HIP stream; use one
 *    handle per host thread (the reference hot path is single-threaded).
 *  - Poses are float[12], row-major 3x4 [R|t] (rows 0..2 of Eigen::Affine3f), camera
 *    -> world, exactly the `transformation` argument of the reference.
 *  - Voxel ids are the reference hash (x<<40) ^ (y<<20) ^ z (Volume.hpp:143-148).
 *    "slot" = position of a voxel in occupied_cells_ (first-touch order).
 *  - Functions without a _device suffix take HOST pointers and synchronise the
 *    stream before returning; *_device functions take DEVICE pointers, only enqueue
 *    work on the volume's stream and never synchronise.
 *  - The engine needs a gfx950 GPU.  There is no CPU fallback: with no usable
 *    device every compute call fails with DMF_ERR_NO_DEVICE.
 */
#ifndef DMF_H_
#define DMF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMF_ABI_VERSION 1

enum dmf_status {
  DMF_OK = 0,
  DMF_ERR_INVALID = 1,   /* bad argument (null pointer, bad size, bad pose count ...) */
  DMF_ERR_STATE = 2,     /* volume not constructed / wrong call order              */
  DMF_ERR_HIP = 3,       /* HIP runtime error (message in dmf_last_error)          */
  DMF_ERR_NOMEM = 4,     /* device or host allocation failed                       */
  DMF_ERR_CAPACITY = 5,  /* output buffer too small: required size returned        */
  DMF_ERR_RANGE = 6,     /* grid too large for a packed field (hash / fixed point) */
  DMF_ERR_NO_DEVICE = 7, /* no usable GPU                                          */
  DMF_ERR_DEVICE_CHECK = 8 /* a device-side consistency check failed: the results of the
                              calls it covers are invalid (dmf_fuse_status)               */
};

typedef struct dmf_volume dmf_volume;

/* Camera(vector<float>& K, int height=480, int width=640)  Camera.hpp:23
 * K row-major 3x3: fx=K[0], cx=K[2], fy=K[4], cy=K[5]  (Camera.hpp:26). */
typedef struct dmf_camera {
  float K[9];
  int32_t height;
  int32_t width;
} dmf_camera;

/* VoxelVolume public fields (Volume.hpp:54-60) + engine bookkeeping. */
typedef struct dmf_volume_info {
  double xmin, xmax, ymin, ymax, zmin, zmax;
  double xcenter, ycenter, zcenter;
  double xdelta, ydelta, zdelta;
  double voxel_size;
  int32_t xdim, ydim, zdim;
  int32_t constructed;
  uint64_t hsize;
  int64_t num_occupied;  /* occupied_cells_.size() */
  int64_t num_points;    /* points binned so far   */
  int64_t hazards;       /* unguarded out-of-range accesses the reference would make */
} dmf_volume_info;

/* 3D-DDA log-odds fusion parameters (not in the reference). */
typedef struct dmf_fuse_params {
  int32_t dmin_mm;  /* depth accepted iff dmin_mm <= d < dmax_mm */
  int32_t dmax_mm;
  int32_t l_hit;    /* milli-logit per hit   (OctoMap default p=0.7  ->  847) */
  int32_t l_miss;   /* milli-logit per miss  (OctoMap default p=0.4  -> -405) */
  int32_t l_min;    /* clamp                 (p=0.1192 -> -2000)              */
  int32_t l_max;    /*                       (p=0.971  ->  3511)              */
} dmf_fuse_params;

/* ---- library ------------------------------------------------------------ */
int dmf_abi_version(void);
const char* dmf_status_string(int status);
const char* dmf_last_error(void);
int dmf_device_count(int32_t* count);
void dmf_fuse_params_default(dmf_fuse_params* p);
/* The normal test degree(acos(n.v)) in [0,90] (CommonUtilities.hpp:17,
 * RayTracingEngine.hpp:207-219) is evaluated on the GPU as dstar <= n.v <= 1, with
 * dstar the smallest float whose host-libm acosf passes (the function the reference
 * binary calls).  Host-only; no GPU needed. */
int dmf_angle_threshold(float* dstar);
/* The fusion implementation, its kernel name and the tuning / test knobs of a volume are
 * diagnostics, declared in include/dmf_diag.h (results never depend on them). */

/* ---- VoxelVolume  (Volume.hpp:50-255) ------------------------------------ */
/* VoxelVolume::VoxelVolume()  Volume.hpp:63 — device = HIP device ordinal. */
int dmf_volume_create(dmf_volume** out, int32_t device);
/* VoxelVolume::~VoxelVolume()  Volume.hpp:80-87 */
int dmf_volume_destroy(dmf_volume* v);
/* All work of this handle is enqueued on `stream` (hipStream_t; NULL = default).  The
 * switch does not block the host: the new stream waits for the work already enqueued on
 * the old one (skipped when either stream is capturing a graph). */
int dmf_volume_set_stream(dmf_volume* v, void* hip_stream);
int dmf_volume_synchronize(dmf_volume* v);
/* setDimensions  Volume.hpp:89-100 */
int dmf_volume_set_dimensions(dmf_volume* v, double xmin, double xmax, double ymin, double ymax,
                              double zmin, double zmax);
/* setResolution  Volume.hpp:102-107 */
int dmf_volume_set_resolution(dmf_volume* v, double xdelta, double ydelta, double zdelta);
/* setVolumeSize  Volume.hpp:109-117 */
int dmf_volume_set_volume_size(dmf_volume* v, int32_t xdim, int32_t ydim, int32_t zdim);
/* constructVolume  Volume.hpp:119-128 (dims recomputed by truncation, as the reference) */
int dmf_volume_construct(dmf_volume* v);
int dmf_volume_get_info(const dmf_volume* v, dmf_volume_info* out);

/* integratePointCloud(cloud [, normals])  Volume.hpp:172-197 / :199-228.
 * xyz: n*3 floats (PointXYZRGB x,y,z); normals: n*3 floats or NULL.  Points
 * outside the grid are skipped (the no-normals reference overload indexes out of
 * range there — counted in *n_hazard). */
int dmf_volume_integrate(dmf_volume* v, const float* xyz, const float* normals, int64_t n,
                         int64_t* n_binned, int64_t* n_hazard);
int dmf_volume_integrate_device(dmf_volume* v, const float* d_xyz, const float* d_normals, int64_t n);

/* occupied_cells_ (Volume.hpp:54) in insertion order. */
int dmf_volume_occupied(const dmf_volume* v, uint64_t* hashes, int64_t cap, int64_t* n);
/* Voxel::view / Voxel::good (Volume.hpp:29-48) per slot. */
int dmf_volume_voxel_flags(const dmf_volume* v, int32_t* view, uint8_t* good, int64_t cap);
int dmf_volume_reset_flags(dmf_volume* v);
/* Voxel::pts.size() / normals.size() per slot. */
int dmf_volume_voxel_counts(const dmf_volume* v, int64_t* npts, int64_t* nnormals, int64_t cap);
/* Voxel::pts / Voxel::normals of one voxel (insertion order); *n = #points, -1 if empty. */
int dmf_volume_voxel_points(const dmf_volume* v, uint64_t hash, float* pts, float* normals, int64_t cap,
                            int64_t* n);
/* Bulk export of every voxel's points/normals (host mirror of voxels_[x][y][z]->pts /
 * ->normals): offsets[V+1] (points of slot s are [offsets[s], offsets[s+1])), pts
 * 3 floats per point, normals4 4 floats per point (w = 1 if the point carried a
 * normal), in occupied_cells_ order and insertion order within a voxel.  cap_points
 * must be >= num_points (dmf_volume_get_info); any output may be NULL. */
int dmf_volume_export(const dmf_volume* v, int32_t* offsets, float* pts, float* normals4, int64_t cap_points);
/* voxels_[x][y][z] != nullptr as a dense x-major byte grid (xdim*ydim*zdim). */
int dmf_volume_occupancy(const dmf_volume* v, uint8_t* dense);

/* ---- Camera back-projection  (Camera.hpp:24-31 projectPoint + :39-45 transformPoints) */
/* depth: H*W uint16 mm, pose: 12 floats -> xyz: H*W*3 floats (world). */
int dmf_backproject(dmf_volume* v, const dmf_camera* cam, const uint16_t* depth, const float* pose,
                    float* xyz);
int dmf_backproject_device(dmf_volume* v, const dmf_camera* cam, const uint16_t* d_depth,
                           const float* d_poses, int32_t P, float* d_xyz);

/* ---- RayTracingEngine  (RayTracingEngine.hpp:27-564) ---------------------- */
/* reverseRayTraceFast  RayTracingEngine.hpp:136-226, batched over P poses.
 * found[P]; counts[P]; hashes = the P good lists concatenated in pose order, each in
 * occupied_cells_ order.  DMF_ERR_CAPACITY (counts filled) if sum(counts) > cap. */
int dmf_reverse_ray_trace_fast(dmf_volume* v, const dmf_camera* cam, const float* poses, int32_t P,
                               int32_t viz, uint8_t* found, int64_t* counts, uint64_t* hashes,
                               int64_t cap);
/* Device form: per-pose bitmasks over slots, words = ceil(num_occupied/64) per pose,
 * d_visible / d_good: P*words uint64 (either may be NULL).  d_poses: P*12 floats. */
int dmf_reverse_visibility_device(dmf_volume* v, const dmf_camera* cam, const float* d_poses, int32_t P,
                                  int32_t viz, uint64_t* d_visible, uint64_t* d_good,
                                          uint64_t* d_stats /* 2 counters += {march samples, voxel rays}; may be NULL */);
/* reverseRayTrace  RayTracingEngine.hpp:45-134 (float-accumulated grid enumeration). */
int dmf_reverse_ray_trace(dmf_volume* v, const dmf_camera* cam, const float* poses, int32_t P, int32_t viz,
                          uint8_t* found, int64_t* counts, uint64_t* hashes, int64_t cap);
/* Set-cover consumer: Algorithms.hpp:38-86 greedySetCover over the reverseRayTraceFast
 * good sets of P candidate poses (the loop of tests/SetCover.cpp:218-240).  selected[P]
 * receives the chosen pose indices in selection order; the reference stops when no set
 * adds anything or the best adds fewer than min_gain (5) voxels. */
int dmf_greedy_set_cover(dmf_volume* v, const dmf_camera* cam, const float* poses, int32_t P, int32_t min_gain,
                         int32_t* selected, int32_t* nselected);
/* Same over caller bitmasks (P x words uint64, e.g. d_good of dmf_reverse_visibility_device). */
int dmf_greedy_set_cover_masks_device(dmf_volume* v, const uint64_t* d_masks, int32_t P, int64_t words,
                                      int32_t min_gain, int32_t* selected, int32_t* nselected);
/* rayTrace  RayTracingEngine.hpp:268-309 */
int dmf_ray_trace(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta, int32_t sparse);
/* rayTraceAndClassify  RayTracingEngine.hpp:311-375 */
int dmf_ray_trace_and_classify(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta,
                               int32_t view, int32_t sparse);
/* rayTraceAndGetMinimum  RayTracingEngine.hpp:229-264 (-1 if nothing hit) */
int dmf_ray_trace_and_get_minimum(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta,
                                  int32_t sparse, int32_t* minimum);
/* rayTraceAndGetPoints  RayTracingEngine.hpp:447-494 */
int dmf_ray_trace_and_get_points(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta,
                                 int32_t sparse, uint8_t* found, uint64_t* hashes, int64_t cap, int64_t* n);
/* rayTraceAndGetGoodPoints  RayTracingEngine.hpp:377-445 */
int dmf_ray_trace_and_get_good_points(dmf_volume* v, const dmf_camera* cam, const float* pose,
                                      int32_t zdelta, int32_t sparse, uint8_t* found, uint64_t* hashes,
                                      int64_t cap, int64_t* n);
/* Per-pixel first hit of the forward march on the (rdelta, cdelta) lattice:
 * k_out[R*C] depth-plane index (-1 = none), hash_out[R*C]. */
int dmf_forward_first_hits(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zstart,
                           int32_t zdelta, int32_t rdelta, int32_t cdelta, int32_t* k_out,
                           uint64_t* hash_out);
/* Batched device form for P poses: d_k / d_slot P*R*C int32 (first-hit depth-plane index
 * and occupied slot, -1 = none); d_stats (may be NULL) += {march samples}. */
int dmf_forward_first_hits_device(dmf_volume* v, const dmf_camera* cam, const float* d_poses, int32_t P,
                                  int32_t zstart, int32_t zdelta, int32_t rdelta, int32_t cdelta, int32_t* d_k,
                                  int32_t* d_slot, uint64_t* d_stats);
/* rayTraceVolume  RayTracingEngine.hpp:498-564 (depth_out: H*W int32 z-buffer or NULL). */
int dmf_ray_trace_volume(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t* depth_out);
/* willCollide  tests/CameraPathGen.cpp:128-156, for n segment pairs a[i] -> b[i]. */
int dmf_will_collide(dmf_volume* v, const float* a, const float* b, int64_t n, uint8_t* collided);
/* Planner::run_tsp cost map  tests/CameraPathGen.cpp:310-331 (also CameraMotionTSP.cpp:
 * 291-306): for all V*V ordered pairs of camera centres (translation of poses[i], P*12
 * floats) map[i*V+j] = INT_MAX if willCollide(c_i, c_j) else int(|c_i - c_j| * 1000).
 * V <= 46340.  Device form: a pair the reference cannot march (non-finite centre, or a
 * segment over INT_MAX mm) gets -1; the host form rejects non-finite centres. */
int dmf_collision_cost_map(dmf_volume* v, const float* poses, int32_t V, int32_t* map);
int dmf_collision_cost_map_device(dmf_volume* v, const float* d_poses, int32_t V, int32_t* d_map);

/* ---- 3D-DDA log-odds fusion (new capability) ------------------ */
/* Host form: depth P*H*W uint16 mm, poses P*12; hits/misses: xdim*ydim*zdim int32 in
 * the reference's x-major voxel order, ACCUMULATED (caller zeroes).
 * stats[3] += {cell updates, rays, hits}. */
int dmf_fuse_depth(dmf_volume* v, const dmf_camera* cam, const uint16_t* depth, const float* poses,
                   int32_t P, const dmf_fuse_params* prm, int32_t* hits, int32_t* misses, int64_t* stats);
/* Device form.  d_hits / d_misses are fusion counters in the TILED layout (2x2x4-cell
 * tiles of 16 int32 = one 64-B line, tiles x-major) of
 * dmf_fuse_counter_cells() elements each, ACCUMULATED; any elementwise sum of them
 * (e.g. an all-reduce across ranks) stays valid.  d_stats (may be NULL): 8 uint64
 * counters += {cell updates, rays, hits, layout faults, LDS rounds | pairs, direct rounds |
 * parts, flushed cell atomics, 0}; layout faults (must stay 0) = the device-side check of
 * the brick pipeline's pair layout (dmf_fuse_status) -- a non-zero count means the counters
 * of that call are invalid. */
int dmf_fuse_depth_device(dmf_volume* v, const dmf_camera* cam, const uint16_t* d_depth,
                          const float* d_poses, int32_t P, const dmf_fuse_params* prm, int32_t* d_hits,
                          int32_t* d_misses, uint64_t* d_stats);
/* Pre-allocate the fusion scratch for calls of up to P frames of `cam`'s size on this
 * volume, so that dmf_fuse_depth_device then neither allocates nor synchronises (e.g. for
 * hipGraph capture).  The brick pipeline fits its ray records, brick tables and (ray,
 * brick) pair records into max_scratch_bytes (0 = keep the current budget; default 45 % of
 * the device's memory, ~130 GB on MI355X): serial calls use one slot of the whole budget,
 * pipelined calls (dmf_fuse_set_input_stream) two staging slots of half each.  A call whose
 * pairs exceed a slot's pair capacity is cut into pose batches on the device
 * (dmf_fuse_plan).  A new budget frees and re-plans the slots.  Synchronises the stream.
 * The budget is PER VOLUME: several volumes fusing on one device (or several processes
 * sharing it) should each reserve their share explicitly, e.g. 0.9 x free memory / volumes;
 * a call whose pairs exceed the share runs in more pose batches (dmf_fuse_batches_used),
 * with identical results. */
int dmf_fuse_reserve(dmf_volume* v, const dmf_camera* cam, int32_t P, uint64_t max_scratch_bytes);
/* Pipelined fusion (an extension, the reference fuses one frame at a time,
 * tests/Raytracing.cpp:70-76).  Declares that the device inputs (d_depth, d_poses) of later
 * dmf_fuse_depth_device calls on this volume are ordered on `stream` (a hipStream_t the
 * caller writes them on) instead of on the volume's stream.  The brick pipeline then runs
 * each call's per-frame pass (pose table + pass A: back-projection, ray records, brick
 * counts) on a staging stream of the volume that waits only for `stream`, for its staging
 * slot's previous reader and (pass A itself) for the previous call's pass B, so that it
 * overlaps the previous call's phase F; the device-side batch cut, brick layout, pass B
 * (pair records) and phase F run on the volume's stream after pass A.  Two staging slots
 * alternate between super-batches, each with its
 * own pair records and half of the fusion budget (dmf_fuse_reserve).  `stream` is made to
 * wait until the call's pass A has read the inputs, so inputs rewritten there afterwards
 * stay ordered.  Results are identical to the serial order, and serial and pipelined calls
 * may be mixed on one volume without synchronising (a pipelined call waits for the serial
 * calls before it that used its slot).  Switching the mode frees the fusion scratch (after
 * synchronising the volume's streams) so that it is re-planned.  stream = NULL restores
 * the serial order (the default); a volume stream that is capturing a graph always runs
 * serially, and so does the host form dmf_fuse_depth (a captured graph must not be launched
 * while pipelined calls of the same volume are in flight: it reads the serial slot). */
int dmf_fuse_set_input_stream(dmf_volume* v, void* stream);
/* Phase-F event: `event` (a hipEvent_t the caller created; NULL = off) is recorded on the
 * volume's stream of every later fusion call right before its (first) phase F launch -- on
 * the brick pipeline after the call's pass B, on k_fuse_l before that kernel.  A caller that
 * pipelines its own steps makes the previous step's merge / finalize wait for it, so that
 * this HBM-bound work runs beside the issue-bound phase F instead of beside the next call's
 * passes A / B (bench.py).  The event is re-recorded by each call: wait on
 * it after the call returns and before the next call.  It must stay valid until it is
 * unregistered (event = NULL) or the volume is destroyed.  A call enqueued while the volume's
 * stream is capturing a graph does not record it (a record inside a graph would not re-record
 * the caller's event when the graph is launched): order captured work by the graph itself. */
int dmf_fuse_set_phase_event(dmf_volume* v, void* event);
/* How a fusion call of P frames of `cam`'s size on this volume is executed (no GPU work,
 * no allocation): brick = 1 for the brick-owned pipeline (k_bk_*), 0 for k_fuse_l.  The
 * brick pipeline runs pass A over super-batches of super_batch_poses frames; the DEVICE cuts
 * each into pose batches by the (ray, brick) pairs they really make against pair_capacity
 * records of record_bytes (no host synchronisation); at most max_batches batches, each of at
 * least poses_per_batch frames (the geometric bound rays x (1 + brick boundaries));
 * scratch_bytes = the pipeline's device scratch over its `slots` staging slots (2 when the
 * calls are pipelined). */
typedef struct dmf_fuse_plan_info {
  int32_t brick;
  int32_t max_batches;
  int32_t poses_per_batch;
  int32_t record_bytes;
  uint64_t pair_capacity;
  uint64_t scratch_bytes;
  int32_t super_batch_poses;
  int32_t slots;
} dmf_fuse_plan_info;
int dmf_fuse_plan(const dmf_volume* v, const dmf_camera* cam, int32_t P, dmf_fuse_plan_info* out);
/* Diagnostic (synchronises the stream): the pose batches the device cut the latest
 * brick-pipeline super-batch of this volume into (0 before any brick-pipeline call). */
int dmf_fuse_batches_used(dmf_volume* v, int32_t* batches);
/* Device-side check of the brick pipeline (synchronises the volume's streams): pass B
 * writes each (ray, brick) pair record into the slot range pass A counted for it; a store
 * outside the call's pair records is dropped, and every workgroup compares the slots it took
 * per brick with pass A's counts.  Returns DMF_ERR_DEVICE_CHECK (and clears the count) when
 * any fusion call since the last dmf_fuse_status disagreed -- their counters are invalid --
 * else DMF_OK; *faults (may be NULL) = the workgroup-brick disagreements seen.  The host
 * form dmf_fuse_depth runs this check itself. */
int dmf_fuse_status(dmf_volume* v, uint64_t* faults);
/* Elements of one tiled counter array (>= xdim*ydim*zdim: dims padded to 2, 2, 4). */
int dmf_fuse_counter_cells(const dmf_volume* v, int64_t* n);
/* Tiled counters -> x-major int32 (xdim*ydim*zdim). */
int dmf_fuse_counters_to_linear_device(dmf_volume* v, const int32_t* d_tiled, int32_t* d_linear);
/* clamp(hits*l_hit + misses*l_miss, l_min, l_max) -> int16 log-odds grid, x-major.
 * Host form: linear counters; device form: tiled counters. */
int dmf_fuse_finalize(dmf_volume* v, const int32_t* hits, const int32_t* misses, const dmf_fuse_params* prm,
                      int16_t* logodds);
int dmf_fuse_finalize_device(dmf_volume* v, const int32_t* d_hits, const int32_t* d_misses,
                             const dmf_fuse_params* prm, int16_t* d_logodds);

/* ---- multi-GPU merge over RCCL ------------------------
 * Poses shard across ranks, each rank fuses into its own replica of the counters, and
 * the replicas merge with integer collectives (bit-identical to one rank fusing all
 * poses).  `comm` is an ncclComm_t (RCCL) as void*: torch's ProcessGroupNCCL._comm_ptr()
 * or one made with dmf_comm_init_rank.  Collectives (and the slab finalize) run on
 * `stream` (hipStream_t; NULL = the volume's stream), e.g. a communication stream that
 * overlaps the next fusion call on the volume's stream. */
#define DMF_COMM_ID_BYTES 128
int dmf_rccl_version(int32_t* version);
/* ncclGetUniqueId into id[DMF_COMM_ID_BYTES] (rank 0; share it with the other ranks). */
int dmf_comm_unique_id(void* id);
int dmf_comm_init_rank(void** comm, int32_t nranks, const void* id, int32_t rank, int32_t device);
int dmf_comm_destroy(void* comm);
/* ncclCommCount / ncclCommUserRank of a communicator (e.g. torch's, to report the ranks the
 * merge's collectives span). */
int dmf_comm_shape(void* comm, int32_t* nranks, int32_t* rank);
/* Tiled counter elements per array padded to whole tile rows per rank (>= the unpadded
 * dmf_fuse_counter_cells), and the padded int16 log-odds grid (>= xdim*ydim*zdim) used by
 * dmf_fuse_merge_finalize_device.  Counters = [hits | misses], each n_padded elements. */
int dmf_fuse_counter_cells_padded(const dmf_volume* v, int32_t nranks, int64_t* n_padded);
int dmf_fuse_logodds_cells_padded(const dmf_volume* v, int32_t nranks, int64_t* n_padded);
/* The merge's slab arithmetic for `rank` of `nranks` (rank = -1: the whole grid), so a
 * caller with its own collectives (MPI, gloo, a test emulating ranks on one GPU) can
 * reproduce dmf_fuse_merge_finalize_device exactly: each counter array holds n_padded
 * elements; the reduce-scatter gives rank r the sums of elements [chunk_offset,
 * chunk_offset + chunk) of each array (in place); rank r finalizes counter tiles
 * [tile_begin, tile_end) (tile rows of 2 x-rows, clipped to the grid); the all-gather moves
 * slab_bytes of int16 log-odds from byte slab_offset of each rank's padded grid
 * (logodds_padded elements). */
typedef struct dmf_merge_plan {
  int64_t n_padded;
  int64_t chunk;
  int64_t chunk_offset;
  int64_t tile_begin;
  int64_t tile_end;
  int64_t logodds_padded;
  int64_t slab_bytes;
  int64_t slab_offset;
} dmf_merge_plan;
int dmf_fuse_merge_plan(const dmf_volume* v, int32_t nranks, int32_t rank, dmf_merge_plan* out);
/* The same for a grid of xdim x ydim x zdim cells (host only: no volume, no GPU). */
int dmf_fuse_merge_plan_dims(int32_t xdim, int32_t ydim, int32_t zdim, int32_t nranks, int32_t rank,
                             dmf_merge_plan* out);
/* Finalize rank `rank`'s slab (rank = -1: every slab) of the padded [hits | misses]
 * counters (n_padded per array for nranks) into the padded int16 log-odds grid, on
 * `stream` (NULL = the volume's).  The merge's own finalize step. */
int dmf_fuse_finalize_slab_device(dmf_volume* v, const int32_t* d_counters, const dmf_fuse_params* prm,
                                  int16_t* d_logodds, int32_t nranks, int32_t rank, void* stream);
/* In-place all-reduce(sum) of [hits | misses] (2*n_per_array int32). */
int dmf_fuse_allreduce_device(dmf_volume* v, int32_t* d_counters, int64_t n_per_array, void* comm, void* stream);
/* Merge + finalize: reduce-scatter(sum) of hits and of misses over whole tile rows, this
 * rank finalizes its slab, all-gather of the int16 slabs: every rank ends with the full
 * log-odds grid in d_logodds (x-major; the first xdim*ydim*zdim of the padded buffer).
 * d_counters: padded [hits | misses]; afterwards only this rank's slab holds sums.
 * comm = NULL: a single rank (no collective): the whole grid is finalized on `stream`. */
int dmf_fuse_merge_finalize_device(dmf_volume* v, int32_t* d_counters, const dmf_fuse_params* prm,
                                   int16_t* d_logodds, void* comm, void* stream);
/* Voxel::view / Voxel::good of the replicated occupied list after pose-sharded queries:
 * good = all-reduce(max); view = the smallest non-zero id over the ranks (classify sets
 * view only while it is 0, RayTracingEngine.hpp:354, so a single rank keeps the first
 * pose's id: the same when view ids grow with pose order, as in the reference's loops). */
int dmf_flags_allreduce(dmf_volume* v, void* comm, void* stream);

/* ---- persistent fused grid (checkpoint / resume; host only, no GPU needed) ------
 * The clamped int16 log-odds grid (x-major, dims[0]*dims[1]*dims[2] cells) with its
 * geometry and fusion parameters, little-endian, CRC-32 checked (csrc/dmf_io.hip).  The
 * reference's only persistent outputs are text (FileRoutines.hpp:98-112
 * writeCameraLocations); this is the fusion engine's counterpart.  dmf_grid_load with
 * logodds = NULL reads the header only; DMF_ERR_CAPACITY if cap < the grid's cells; a bad
 * magic, version, size or checksum is DMF_ERR_INVALID. */
typedef struct dmf_grid_header {
  int32_t dims[3];
  int32_t reserved;
  double bounds[6]; /* xmin, xmax, ymin, ymax, zmin, zmax (setDimensions) */
  dmf_fuse_params params;
} dmf_grid_header;
int dmf_grid_save(const char* path, const dmf_grid_header* h, const int16_t* logodds);
int dmf_grid_load(const char* path, dmf_grid_header* h, int16_t* logodds, int64_t cap);

/* ---- OccupancyGrid  (include/OccupancyGrid.hpp:50-318) ----------------------- */
/* The reference's second fusion path.  updateStates is computed in the deterministic
 * single-threaded order (the reference's OpenMP loops race); state is dense, x-major,
 * persistent across calls. */
typedef struct dmf_ogrid dmf_ogrid;
int dmf_ogrid_create(dmf_ogrid** out, int32_t device);
int dmf_ogrid_destroy(dmf_ogrid* g);
int dmf_ogrid_set_stream(dmf_ogrid* g, void* hip_stream);
/* setDimensions(bounds[6]) + setResolution(float x3) + setK + construct (:323-352). */
int dmf_ogrid_setup(dmf_ogrid* g, const double* bounds, float xres, float yres, float zres, int32_t k);
int dmf_ogrid_get_dims(const dmf_ogrid* g, int32_t* dims);
/* updateStates(cloud, normals) (:99-164): cloud n_cloud x 3 floats, normals n_normals x 6
 * floats (x, y, z, nx, ny, nz).  Host and device-pointer forms. */
int dmf_ogrid_update_states(dmf_ogrid* g, const float* cloud, int64_t n_cloud, const float* normals,
                            int64_t n_normals);
int dmf_ogrid_update_states_device(dmf_ogrid* g, const float* d_cloud, int64_t n_cloud, const float* d_normals,
                                   int64_t n_normals);
/* Dense state copies (any may be NULL): normal / centroid 3 floats per voxel, count,
 * flags (bit 0 occupied, bit 1 normal_found). */
int dmf_ogrid_state(const dmf_ogrid* g, float* normal, float* centroid, int32_t* count, uint8_t* flags);
/* Write the dense state (the reference's public voxels_ fields; any may be NULL). */
int dmf_ogrid_set_state(dmf_ogrid* g, const float* normal, const float* centroid, const int32_t* count,
                        const uint8_t* flags);
/* mode 0 downloadCloud (:166-193), 1 downloadHQCloud (count > 100, :283-318): occupied
 * voxels in x-major order as (cx, cy, cz, nx, ny, nz).  Modes 2 / 3 downloadReorganizedCloud
 * (:200-286) with clean = false / true: every occupied voxel (clean: count >= 100 at its
 * turn) merges into the voxel holding its centroid, in the single-threaded x-major order
 * the reference's OpenMP loop races over; the merged voxels, x-major.  DMF_ERR_CAPACITY
 * (n set) if n > cap. */
int dmf_ogrid_download(dmf_ogrid* g, int32_t mode, float* out, int64_t cap, int64_t* n);

/* ---- device memory helpers for callers without their own allocator ---------- */
int dmf_device_malloc(dmf_volume* v, void** d_ptr, size_t bytes);
int dmf_device_free(dmf_volume* v, void* d_ptr);
int dmf_memcpy_h2d(dmf_volume* v, void* d_dst, const void* h_src, size_t bytes);
int dmf_memcpy_d2h(dmf_volume* v, void* h_dst, const void* d_src, size_t bytes);
int dmf_memset_device(dmf_volume* v, void* d_ptr, int value, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* DMF_H_ */
