// dmf_core.hip — library plumbing, VoxelVolume lifecycle, point-cloud integration
// (Volume.hpp:172-228) and depth back-projection (Camera.hpp:24-45) on gfx950.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "dmf_host.hpp"

namespace dmf {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int fail(int status, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return status;
}

int activate(const dmf_volume* v) {
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  DMF_HIP(hipSetDevice(v->device));
  return DMF_OK;
}

int require_constructed(const dmf_volume* v) {
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  if (!v->constructed) return fail(DMF_ERR_STATE, "constructVolume() has not been called");
  return activate(v);
}

int scratch(dmf_volume* v, int k, size_t bytes, void** out) {
  if ((int)v->scratch.size() <= k) v->scratch.resize(k + 1, {nullptr, 0});
  auto& s = v->scratch[k];
  if (s.second < bytes) {
    // forget the old slot before allocating: a failed hipMalloc must leave the slot
    // empty (size 0), never a stale size with a freed or null pointer
    void* old = s.first;
    s.first = nullptr;
    s.second = 0;
    if (old) DMF_HIP(hipFree(old));
    const size_t nb = std::max<size_t>(bytes + bytes / 4, 256);
    void* p = nullptr;
    DMF_HIP(hipMalloc(&p, nb));
    s.first = p;
    s.second = nb;
  }
  *out = s.first;
  return DMF_OK;
}

CamP cam_params(const dmf_camera* c) {
  CamP p;
  p.fx = c->K[0]; p.cx = c->K[2]; p.fy = c->K[4]; p.cy = c->K[5];
  p.rfx = 1.0 / p.fx;
  p.rfy = 1.0 / p.fy;
  p.H = c->height; p.W = c->width;
  return p;
}

int check_camera(const dmf_camera* c) {
  if (!c) return fail(DMF_ERR_INVALID, "null camera");
  if (c->height <= 0 || c->width <= 0 || c->height > 65536 || c->width > 65536)
    return fail(DMF_ERR_INVALID, "bad image size %dx%d", c->width, c->height);
  return DMF_OK;
}

__global__ void k_pose_table(const float* __restrict__ poses, int P, PoseX* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  PoseX x;
  for (int k = 0; k < 12; ++k) x.f[k] = poses[12 * p + k];
  inverse_pose(x.f, x.i);
  out[p] = x;
}

int pose_table(dmf_volume* v, const float* poses, int P, bool on_device, PoseX** d_table) {
  if (P <= 0) return fail(DMF_ERR_INVALID, "pose count must be > 0");
  if (!poses) return fail(DMF_ERR_INVALID, "null poses");
  const float* src = poses;
  if (!on_device) {
    void* buf;
    DMF_TRY(scratch(v, kScHost0, sizeof(float) * 12 * (size_t)P, &buf));
    DMF_HIP(hipMemcpyAsync(buf, poses, sizeof(float) * 12 * (size_t)P, hipMemcpyHostToDevice, v->stream));
    src = (const float*)buf;
  }
  void* tab;
  DMF_TRY(scratch(v, kScPoses, sizeof(PoseX) * (size_t)P, &tab));
  hipLaunchKernelGGL(k_pose_table, dim3((P + 63) / 64), dim3(64), 0, v->stream, src, P, (PoseX*)tab);
  DMF_LAUNCH_CHECK();
  *d_table = (PoseX*)tab;
  return DMF_OK;
}

int pose_table_into(const float* d_poses, int P, PoseX* d_out, hipStream_t s) {
  hipLaunchKernelGGL(k_pose_table, dim3((P + 63) / 64), dim3(64), 0, s, d_poses, P, d_out);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
}

// ---------------------------------------------------------------- striped stats
int stats_begin(dmf_volume* v, unsigned long long** striped) {
  void* b;
  DMF_TRY(scratch(v, kScStats, sizeof(unsigned long long) * kStatSlots * kStatWidth, &b));
  DMF_HIP(hipMemsetAsync(b, 0, sizeof(unsigned long long) * kStatSlots * kStatWidth, v->stream));
  *striped = (unsigned long long*)b;
  return DMF_OK;
}

// fault (may be null): the volume's fault words; word 1 (faults not yet reported in a call's
// statistics) is taken atomically into counter 3
__global__ void k_stats_reduce(const unsigned long long* __restrict__ s, int n, unsigned long long* __restrict__ out,
                               uint32_t* fault) {
  const int c = threadIdx.x;
  if (c >= n) return;
  unsigned long long t = 0;
  for (int k = 0; k < kStatSlots; ++k) t += s[k * kStatWidth + c];
  if (c == 3 && fault) t += atomicExch(&fault[1], 0u);
  if (t) atomicAdd(&out[c], t);
}

int stats_end(dmf_volume* v, const unsigned long long* striped, uint64_t* d_user, int n, uint32_t* fault,
              hipStream_t stream) {
  if (!d_user) return DMF_OK;
  hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(64), 0, stream ? stream : v->stream, striped, n,
                     (unsigned long long*)d_user, fault);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
}

// ---------------------------------------------------------------- rocPRIM glue
int exclusive_scan_i64(dmf_volume* v, const int64_t* in, int64_t* out, size_t n) {
  size_t bytes = 0;
  DMF_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, (int64_t)0, n, rocprim::plus<int64_t>(), v->stream));
  void* tmp;
  DMF_TRY(scratch(v, kScTmp, bytes, &tmp));
  DMF_HIP(rocprim::exclusive_scan(tmp, bytes, in, out, (int64_t)0, n, rocprim::plus<int64_t>(), v->stream));
  return DMF_OK;
}

int exclusive_scan_i32(dmf_volume* v, const int32_t* in, int32_t* out, size_t n) {
  size_t bytes = 0;
  DMF_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, (int32_t)0, n, rocprim::plus<int32_t>(), v->stream));
  void* tmp;
  DMF_TRY(scratch(v, kScTmp, bytes, &tmp));
  DMF_HIP(rocprim::exclusive_scan(tmp, bytes, in, out, (int32_t)0, n, rocprim::plus<int32_t>(), v->stream));
  return DMF_OK;
}

template <class K, class Vv>
static int sort_pairs_impl(dmf_volume* v, K* keys, Vv* vals, size_t n, int end_bit, int slot_k, int slot_v) {
  if (n == 0) return DMF_OK;
  void *kb, *vb;
  DMF_TRY(scratch(v, slot_k, sizeof(K) * n, &kb));
  DMF_TRY(scratch(v, slot_v, sizeof(Vv) * n, &vb));
  size_t bytes = 0;
  DMF_HIP(rocprim::radix_sort_pairs(nullptr, bytes, keys, (K*)kb, vals, (Vv*)vb, n, 0, end_bit, v->stream));
  void* tmp;
  DMF_TRY(scratch(v, kScTmp, bytes, &tmp));
  DMF_HIP(rocprim::radix_sort_pairs(tmp, bytes, keys, (K*)kb, vals, (Vv*)vb, n, 0, end_bit, v->stream));
  DMF_HIP(hipMemcpyAsync(keys, kb, sizeof(K) * n, hipMemcpyDeviceToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(vals, vb, sizeof(Vv) * n, hipMemcpyDeviceToDevice, v->stream));
  return DMF_OK;
}

int sort_pairs_u64(dmf_volume* v, uint64_t* keys, uint64_t* vals, size_t n, int end_bit) {
  return sort_pairs_impl(v, keys, vals, n, end_bit, kScSort0, kScSort1);
}
int sort_pairs_u32(dmf_volume* v, uint32_t* keys, uint32_t* vals, size_t n, int end_bit) {
  return sort_pairs_impl(v, keys, vals, n, end_bit, kScSort2, kScSort3);
}

// ---------------------------------------------------------------- mask compaction
__global__ void k_mask_popc(const uint64_t* __restrict__ m, int64_t n, int64_t* __restrict__ c) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = __popcll(m[i]);
}

// centroid hash of enumeration entry e (RayTracingEngine.hpp:66,74): getHash(x+dx/2, ...)
__device__ inline uint64_t enum_centroid_hash(const Geom& g, const float* axes, const int32_t* nax, uint32_t e) {
  const uint32_t nyz = (uint32_t)nax[1] * (uint32_t)nax[2];
  const uint32_t i = e / nyz, j = (e / nax[2]) % nax[1], k = e % nax[2];
  const float x = axes[i], y = axes[nax[0] + j], z = axes[nax[0] + nax[1] + k];
  const float cx = (float)((double)x + g.hdl[0]);
  const float cy = (float)((double)y + g.hdl[1]);
  const float cz = (float)((double)z + g.hdl[2]);
  return hash_id(bin_axis(g, 0, cx), bin_axis(g, 1, cy), bin_axis(g, 2, cz));
}

struct EnumCtx {
  const float* axes;
  int32_t nax[3];
  const uint32_t* list;
};

__global__ void k_mask_scatter(const uint64_t* __restrict__ m, int64_t words, int64_t total_words,
                               int64_t nelem, const int64_t* __restrict__ pos, const uint64_t* __restrict__ hash,
                               Geom g, EnumCtx ec, int value_kind, uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total_words) return;
  uint64_t bits = m[i];
  int64_t o = pos[i];
  const int64_t e0 = (i % words) * 64;
  while (bits) {
    const int b = __ffsll((unsigned long long)bits) - 1;
    bits &= bits - 1;
    const int64_t e = e0 + b;
    if (e >= nelem) break;
    uint64_t val;
    if (value_kind == kValueSlotHash) {
      val = hash[e];
    } else {
      val = enum_centroid_hash(g, ec.axes, ec.nax, ec.list[e]);
    }
    out[o++] = val;
  }
}

__global__ void k_gather_bases(const int64_t* __restrict__ s, int64_t words, int P, int64_t* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p <= P) out[p] = s[(int64_t)p * words];
}

int compact_masks(dmf_volume* v, const uint64_t* d_masks, int P, int64_t words, int64_t nelem,
                  int64_t* counts_h, uint64_t** d_out, int64_t* total, int value_kind) {
  const int64_t tw = (int64_t)P * words;
  void *pc, *ps;
  DMF_TRY(scratch(v, kScOut2, sizeof(int64_t) * (tw + 1), &pc));
  DMF_TRY(scratch(v, kScOut3, sizeof(int64_t) * (tw + 1), &ps));
  int64_t* c = (int64_t*)pc;
  int64_t* s = (int64_t*)ps;
  DMF_HIP(hipMemsetAsync(c + tw, 0, sizeof(int64_t), v->stream));
  if (tw > 0) {
    hipLaunchKernelGGL(k_mask_popc, dim3((unsigned)((tw + 255) / 256)), dim3(256), 0, v->stream, d_masks, tw, c);
    DMF_LAUNCH_CHECK();
  }
  DMF_TRY(exclusive_scan_i64(v, c, s, (size_t)tw + 1));
  std::vector<int64_t> base((size_t)P + 1);
  void* pb;
  DMF_TRY(scratch(v, kScCount, sizeof(int64_t) * (P + 1), &pb));
  hipLaunchKernelGGL(k_gather_bases, dim3((P + 1 + 255) / 256), dim3(256), 0, v->stream, s, words, P, (int64_t*)pb);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(base.data(), pb, sizeof(int64_t) * (P + 1), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  for (int p = 0; p < P; ++p) counts_h[p] = base[p + 1] - base[p];
  *total = base[P];
  void* ob;
  DMF_TRY(scratch(v, kScOut1, sizeof(uint64_t) * std::max<int64_t>(*total, 1), &ob));
  Geom g = v->geom();
  EnumCtx ec{v->d_axes, {v->nax[0], v->nax[1], v->nax[2]}, v->d_enum};
  if (tw > 0 && *total > 0) {
    hipLaunchKernelGGL(k_mask_scatter, dim3((unsigned)((tw + 255) / 256)), dim3(256), 0, v->stream, d_masks, words,
                       tw, nelem, s, v->d_hash, g, ec, value_kind, (uint64_t*)ob);
    DMF_LAUNCH_CHECK();
  }
  *d_out = (uint64_t*)ob;
  return DMF_OK;
}

// ---------------------------------------------------------------- enumeration
// `for(float x=xmin_; x<xmax_; x+=xdelta_)` (RayTracingEngine.hpp:54-56): a serial
// float recurrence, evaluated by one lane per axis.
__global__ void k_float_axes(Geom g, int cap, float* __restrict__ axes, int32_t* __restrict__ counts) {
  const int a = threadIdx.x;
  if (a >= 3) return;
  float* out = axes + a * cap;
  int n = 0;
  for (float x = (float)g.mn[a]; (double)x < g.mx[a]; x = (float)((double)x + g.dl[a])) {
    if (n < cap) out[n] = x;
    ++n;
    if (n > cap) break;
  }
  counts[a] = n;
}

__global__ void k_enum_flags(Geom g, const uint32_t* __restrict__ occ, const float* __restrict__ axes, int32_t nx,
                             int32_t ny, int32_t nz, uint64_t total, uint8_t* __restrict__ flags,
                             unsigned long long* __restrict__ hazards) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const uint32_t i = (uint32_t)(e / ((uint64_t)ny * nz)), j = (uint32_t)((e / nz) % ny), k = (uint32_t)(e % nz);
  const int a = bin_axis(g, 0, axes[i]), b = bin_axis(g, 1, axes[nx + j]), c = bin_axis(g, 2, axes[nx + ny + k]);
  uint8_t f = 0;
  if (!valid_coords(g, a, b, c)) {
    atomicAdd(hazards, 1ull);  // reference indexes voxels_ out of range here (UB)
  } else {
    f = occ_test(occ, occ_bit(g, a, b, c)) ? 1 : 0;
  }
  flags[e] = f;
}

int ensure_enumeration(dmf_volume* v) {
  if (v->enum_valid) return DMF_OK;
  Geom g = v->geom();
  const int cap = std::max({v->xdim, v->ydim, v->zdim}) * 2 + 8;
  if (!v->d_axes) DMF_HIP(hipMalloc((void**)&v->d_axes, sizeof(float) * 3 * cap + 16));
  void* cnt;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * 4 + sizeof(unsigned long long), &cnt));
  hipLaunchKernelGGL(k_float_axes, dim3(1), dim3(64), 0, v->stream, g, cap, v->d_axes, (int32_t*)cnt);
  DMF_LAUNCH_CHECK();
  int32_t nax[3];
  DMF_HIP(hipMemcpyAsync(nax, cnt, sizeof(nax), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  for (int a = 0; a < 3; ++a)
    if (nax[a] > cap) return fail(DMF_ERR_RANGE, "float enumeration axis %d longer than %d", a, cap);
  // compact x/y/z axes into one array [xs|ys|zs]
  std::vector<float> h((size_t)3 * cap);
  DMF_HIP(hipMemcpyAsync(h.data(), v->d_axes, sizeof(float) * 3 * cap, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  std::vector<float> packed;
  for (int a = 0; a < 3; ++a) packed.insert(packed.end(), h.begin() + (size_t)a * cap, h.begin() + (size_t)a * cap + nax[a]);
  DMF_HIP(hipMemcpyAsync(v->d_axes, packed.data(), sizeof(float) * packed.size(), hipMemcpyHostToDevice, v->stream));
  for (int a = 0; a < 3; ++a) v->nax[a] = nax[a];
  const uint64_t total = (uint64_t)nax[0] * nax[1] * nax[2];
  if (total >= (1ull << 32)) return fail(DMF_ERR_RANGE, "enumeration too large");
  void *fl, *cnt2;
  DMF_TRY(scratch(v, kScOut1, total + 16, &fl));
  DMF_TRY(scratch(v, kScOut2, 2 * sizeof(unsigned long long), &cnt2));
  DMF_HIP(hipMemsetAsync(cnt2, 0, 2 * sizeof(unsigned long long), v->stream));
  if (total > 0) {
    hipLaunchKernelGGL(k_enum_flags, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, v->stream, g, v->d_occ,
                       v->d_axes, nax[0], nax[1], nax[2], total, (uint8_t*)fl, (unsigned long long*)cnt2 + 1);
    DMF_LAUNCH_CHECK();
  }
  if ((int64_t)total > v->enum_cap) {
    if (v->d_enum) DMF_HIP(hipFree(v->d_enum));
    DMF_HIP(hipMalloc((void**)&v->d_enum, sizeof(uint32_t) * std::max<uint64_t>(total, 1)));
    v->enum_cap = (int64_t)total;
  }
  size_t bytes = 0;
  auto it = rocprim::counting_iterator<uint32_t>(0);
  unsigned long long* nsel = (unsigned long long*)cnt2;
  DMF_HIP(rocprim::select(nullptr, bytes, it, (uint8_t*)fl, v->d_enum, nsel, total, v->stream));
  void* tmp;
  DMF_TRY(scratch(v, kScTmp, bytes, &tmp));
  DMF_HIP(rocprim::select(tmp, bytes, it, (uint8_t*)fl, v->d_enum, nsel, total, v->stream));
  unsigned long long hc[2];
  DMF_HIP(hipMemcpyAsync(hc, cnt2, sizeof(hc), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  v->nenum = (int64_t)hc[0];
  v->enum_hazards = (int64_t)hc[1];
  v->enum_valid = true;
  return DMF_OK;
}

// ---------------------------------------------------------------- integration
// Volume.hpp:199-228: per point validPoints -> getVoxel -> validCoords -> first
// touch allocates the voxel and appends its hash to occupied_cells_.  On the GPU
// the first toucher of a cell is the smallest point index (atomicMin on a pending
// code), and the new slots are ranked by an order-preserving scan over points, so
// occupied_cells_ comes out in exactly the reference insertion order.
__global__ void k_bin_points(Geom g, const float* __restrict__ xyz, int64_t n, int32_t* __restrict__ slot_of,
                             int32_t* __restrict__ plin, unsigned long long* __restrict__ hazards, int unguarded) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
  int32_t lin = -1;
  if (valid_points(g, x, y, z)) {
    const int a = bin_axis(g, 0, x), b = bin_axis(g, 1, y), c = bin_axis(g, 2, z);
    if (valid_coords(g, a, b, c)) {
      lin = (int32_t)lin_index(g, a, b, c);
      const int32_t cur = slot_of[lin];
      if (cur < 0 || cur == kEmpty) atomicMin(&slot_of[lin], kPendBase + (int32_t)i);
    } else if (unguarded) {
      atomicAdd(hazards, 1ull);  // Volume.hpp:184 indexes voxels_ without validCoords (UB)
    }
  }
  plin[i] = lin;
}

__global__ void k_first_flags(const int32_t* __restrict__ plin, int64_t n, const int32_t* __restrict__ slot_of,
                              int32_t* __restrict__ flag) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t lin = plin[i];
  flag[i] = (lin >= 0 && slot_of[lin] == kPendBase + (int32_t)i) ? 1 : 0;
}

__global__ void k_assign_slots(Geom g, const int32_t* __restrict__ plin, const int32_t* __restrict__ flag,
                               const int32_t* __restrict__ rank, int64_t n, int64_t V0, int32_t* __restrict__ slot_of,
                               uint64_t* __restrict__ hash, int32_t* __restrict__ view, uint8_t* __restrict__ good,
                               uint32_t* __restrict__ occ, uint32_t* __restrict__ brick, int nby, int nbz,
                               int bsh) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !flag[i]) return;
  const int32_t lin = plin[i];
  const int32_t slot = (int32_t)(V0 + rank[i]);
  slot_of[lin] = slot;
  const uint32_t nyz = (uint32_t)g.n[1] * (uint32_t)g.n[2];
  const int x = (int)((uint32_t)lin / nyz), y = (int)(((uint32_t)lin / g.n[2]) % g.n[1]), z = (int)((uint32_t)lin % g.n[2]);
  hash[slot] = hash_id(x, y, z);
  view[slot] = 0;
  good[slot] = 0;
  const uint32_t ob = occ_bit(g, x, y, z);
  atomicOr(&occ[ob >> 5], 1u << (ob & 31));
  const uint32_t bl = ((uint32_t)(x >> bsh) * (uint32_t)nby + (uint32_t)(y >> bsh)) * (uint32_t)nbz + (uint32_t)(z >> bsh);
  atomicOr(&brick[bl >> 5], 1u << (bl & 31));
}

__global__ void k_point_slots(const int32_t* __restrict__ plin, int64_t n, const int32_t* __restrict__ slot_of,
                              int32_t* __restrict__ pslot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t lin = plin[i];
  pslot[i] = lin >= 0 ? slot_of[lin] : -1;
}

__global__ void k_store_points(const float* __restrict__ xyz, const float* __restrict__ nrm, int64_t n,
                               float* __restrict__ pts, float4* __restrict__ pnrm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pts[3 * i] = xyz[3 * i];
  pts[3 * i + 1] = xyz[3 * i + 1];
  pts[3 * i + 2] = xyz[3 * i + 2];
  pnrm[i] = nrm ? make_float4(nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2], 1.0f) : make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ void k_csr_keys(const int32_t* __restrict__ pslot, int64_t n, uint32_t V, uint32_t* __restrict__ keys,
                           uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t s = pslot[i];
  keys[i] = s >= 0 ? (uint32_t)s : V;
  vals[i] = (uint32_t)i;
}

__global__ void k_csr_build(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, int64_t n,
                            uint32_t V, const float* __restrict__ pts, const float4* __restrict__ pnrm,
                            int32_t* __restrict__ off, float* __restrict__ cpts, float4* __restrict__ cnrm) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t k = keys[j];
  if (k >= V) {
    if (j == 0 || keys[j - 1] < V) off[V] = (int32_t)j;
    return;
  }
  if (j == 0 || keys[j - 1] != k) off[k] = (int32_t)j;
  if (j == n - 1) off[V] = (int32_t)n;
  const uint32_t p = vals[j];
  cpts[3 * j] = pts[3 * p];
  cpts[3 * j + 1] = pts[3 * p + 1];
  cpts[3 * j + 2] = pts[3 * p + 2];
  cnrm[j] = pnrm[p];
}

template <class T>
static int grow(dmf_volume* v, T** p, int64_t old_n, int64_t new_cap) {
  T* q = nullptr;
  DMF_HIP(hipMalloc((void**)&q, sizeof(T) * (size_t)std::max<int64_t>(new_cap, 1)));
  if (*p) {
    if (old_n > 0) DMF_HIP(hipMemcpyAsync(q, *p, sizeof(T) * (size_t)old_n, hipMemcpyDeviceToDevice, v->stream));
    DMF_HIP(hipFree(*p));
  }
  *p = q;
  return DMF_OK;
}

static int integrate_impl(dmf_volume* v, const float* d_xyz, const float* d_nrm, int64_t n, int64_t* binned,
                          int64_t* hazard) {
  if (n < 0) return fail(DMF_ERR_INVALID, "negative point count");
  if (n == 0) { if (binned) *binned = 0; if (hazard) *hazard = 0; return DMF_OK; }
  if (v->npts + n >= (int64_t)0x7fffffff) return fail(DMF_ERR_RANGE, "more than 2^31 points");
  const Geom g = v->geom();
  const int64_t P0 = v->npts;
  if (P0 + n > v->pcap) {
    const int64_t cap = std::max<int64_t>(P0 + n, v->pcap * 2);
    DMF_TRY(grow(v, &v->d_pts, 3 * P0, 3 * cap));
    DMF_TRY(grow(v, &v->d_pnrm, P0, cap));
    DMF_TRY(grow(v, &v->d_pslot, P0, cap));
    v->pcap = cap;
  }
  void *plin, *flag, *rank, *cnt;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * n, &plin));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * (n + 1), &flag));
  DMF_TRY(scratch(v, kScOut2, sizeof(int32_t) * (n + 1), &rank));
  DMF_TRY(scratch(v, kScOut3, sizeof(unsigned long long) * 2, &cnt));
  DMF_HIP(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * 2, v->stream));
  const dim3 blk(256), grd((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(k_store_points, grd, blk, 0, v->stream, d_xyz, d_nrm, n, v->d_pts + 3 * P0, v->d_pnrm + P0);
  DMF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bin_points, grd, blk, 0, v->stream, g, d_xyz, n, v->d_slot_of, (int32_t*)plin,
                     (unsigned long long*)cnt, d_nrm == nullptr ? 1 : 0);
  DMF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_first_flags, grd, blk, 0, v->stream, (const int32_t*)plin, n, v->d_slot_of, (int32_t*)flag);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemsetAsync((int32_t*)flag + n, 0, sizeof(int32_t), v->stream));
  DMF_TRY(exclusive_scan_i32(v, (const int32_t*)flag, (int32_t*)rank, (size_t)n + 1));
  int32_t nnew = 0;
  unsigned long long hz = 0;
  DMF_HIP(hipMemcpyAsync(&nnew, (int32_t*)rank + n, sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipMemcpyAsync(&hz, cnt, sizeof(hz), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  const int64_t V0 = v->V, V1 = v->V + nnew;
  if (V1 > v->Vcap) {
    const int64_t cap = std::max<int64_t>(V1, v->Vcap * 2);
    DMF_TRY(grow(v, &v->d_hash, V0, cap));
    DMF_TRY(grow(v, &v->d_view, V0, cap));
    DMF_TRY(grow(v, &v->d_good, V0, cap));
    v->Vcap = cap;
  }
  hipLaunchKernelGGL(k_assign_slots, grd, blk, 0, v->stream, g, (const int32_t*)plin, (const int32_t*)flag,
                     (const int32_t*)rank, n, V0, v->d_slot_of, v->d_hash, v->d_view, v->d_good, v->d_occ, v->d_brick, v->nb[1], v->nb[2], v->brick_shift);
  DMF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_point_slots, grd, blk, 0, v->stream, (const int32_t*)plin, n, v->d_slot_of, v->d_pslot + P0);
  DMF_LAUNCH_CHECK();
  v->V = V1;
  v->npts = P0 + n;
  v->hazards += (int64_t)hz;
  v->enum_valid = false;
  v->bdist_valid = false;
  v->sorder_valid = false;
  // CSR over all points, stable in point order within each slot.
  const int64_t N = v->npts;
  void *keys, *vals;
  DMF_TRY(scratch(v, kScOut0, sizeof(uint32_t) * N, &keys));
  DMF_TRY(scratch(v, kScOut1, sizeof(uint32_t) * N, &vals));
  const dim3 g2((unsigned)((N + 255) / 256));
  hipLaunchKernelGGL(k_csr_keys, g2, blk, 0, v->stream, v->d_pslot, N, (uint32_t)v->V, (uint32_t*)keys,
                     (uint32_t*)vals);
  DMF_LAUNCH_CHECK();
  int end_bit = 1;
  while ((1ll << end_bit) <= v->V) ++end_bit;
  DMF_TRY(sort_pairs_u32(v, (uint32_t*)keys, (uint32_t*)vals, (size_t)N, end_bit));
  if (v->csr_cap < N || !v->d_off) {
    if (v->d_csr_nrm) DMF_HIP(hipFree(v->d_csr_nrm));
    if (v->d_csr_pts) DMF_HIP(hipFree(v->d_csr_pts));
    const int64_t cap = std::max<int64_t>(N, v->csr_cap * 2);
    DMF_HIP(hipMalloc((void**)&v->d_csr_nrm, sizeof(float4) * cap));
    DMF_HIP(hipMalloc((void**)&v->d_csr_pts, sizeof(float) * 3 * cap));
    v->csr_cap = cap;
  }
  if (v->d_off) DMF_HIP(hipFree(v->d_off));
  DMF_HIP(hipMalloc((void**)&v->d_off, sizeof(int32_t) * (v->V + 1)));
  DMF_HIP(hipMemsetAsync(v->d_off, 0, sizeof(int32_t) * (v->V + 1), v->stream));
  hipLaunchKernelGGL(k_csr_build, g2, blk, 0, v->stream, (const uint32_t*)keys, (const uint32_t*)vals, N,
                     (uint32_t)v->V, v->d_pts, v->d_pnrm, v->d_off, v->d_csr_pts, v->d_csr_nrm);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipStreamSynchronize(v->stream));
  int32_t nb = 0;
  DMF_HIP(hipMemcpy(&nb, v->d_off + v->V, sizeof(int32_t), hipMemcpyDeviceToHost));
  const int64_t newly = (int64_t)nb - v->nbinned;
  v->nbinned = nb;
  if (binned) *binned = newly;
  if (hazard) *hazard = (int64_t)hz;
  return DMF_OK;
}

// ---------------------------------------------------------------- back-projection
// Camera.hpp:24-31 projectPoint then :39-45 transformPoints, one lane per pixel.
__global__ void k_backproject(CamP cam, const uint16_t* __restrict__ depth, const PoseX* __restrict__ poses, int P,
                              float* __restrict__ xyz) {
  const int64_t HW = (int64_t)cam.H * cam.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int p = blockIdx.y;
  if (i >= HW || p >= P) return;
  const int r = (int)(i / cam.W), c = (int)(i % cam.W);
  float pc[3], w[3];
  project(cam, r, c, depth[(int64_t)p * HW + i], pc);
  xform(poses[p].f, pc[0], pc[1], pc[2], w);
  float* o = xyz + 3 * ((int64_t)p * HW + i);
  o[0] = w[0];
  o[1] = w[1];
  o[2] = w[2];
}

// Smallest float d with degree(acosf(d)) in [k_AngleMin, k_AngleMax] (host libm,
// as the reference binary), verified over every float of the transition window.
static float angle_threshold() {
  auto ok = [](float d) {
    const int a = to_int_x86(((double)std::acos(d) * 180) / 3.14159);
    return a >= 0 && a <= 90;
  };
  float lo = -0.03f, hi = -0.005f;  // ok(lo) false, ok(hi) true
  uint32_t ulo, uhi;
  std::memcpy(&ulo, &lo, 4);
  std::memcpy(&uhi, &hi, 4);
  // negative floats: larger bit pattern = more negative
  while (ulo - uhi > 1) {
    const uint32_t mid = uhi + (ulo - uhi) / 2;
    float m;
    std::memcpy(&m, &mid, 4);
    if (ok(m)) uhi = mid; else ulo = mid;
  }
  float dstar;
  std::memcpy(&dstar, &uhi, 4);
  return dstar;
}


// ---- brick distance field (empty-space skipping in the reverse march) ---------
// d(b) = min over occupied bricks q of max_axis |b - q| (L-inf, in bricks), capped.
// L-inf distance is separable: three 1-D passes d' = min_t max(|t|, d(b + t e_axis)).
__global__ void k_bdist_init(const uint32_t* __restrict__ brick, int64_t nbr, int cap, uint8_t* __restrict__ d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nbr) d[i] = ((brick[i >> 5] >> (i & 31)) & 1u) ? 0 : (uint8_t)cap;
}
__global__ void k_bdist_pass(int nbx, int nby, int nbz, int axis, int cap, const uint8_t* __restrict__ src,
                             uint8_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nbr = (int64_t)nbx * nby * nbz;
  if (i >= nbr) return;
  const int z = (int)(i % nbz), y = (int)((i / nbz) % nby), x = (int)(i / ((int64_t)nbz * nby));
  const int c = axis == 0 ? x : (axis == 1 ? y : z), n = axis == 0 ? nbx : (axis == 1 ? nby : nbz);
  const int64_t stride = axis == 0 ? (int64_t)nby * nbz : (axis == 1 ? nbz : 1);
  int best = src[i];
  for (int t = 1; t < best && t < cap; ++t) {
    if (c - t >= 0) best = min(best, max(t, (int)src[i - t * stride]));
    if (c + t < n) best = min(best, max(t, (int)src[i + t * stride]));
  }
  dst[i] = (uint8_t)best;
}

int ensure_brick_dist(dmf_volume* v) {
  if (v->bdist_valid) return DMF_OK;
  const int64_t nbr = (int64_t)v->nb[0] * v->nb[1] * v->nb[2];
  uint8_t* a = v->d_bdist;
  uint8_t* b = v->d_bdist + nbr + 64;
  const dim3 blk(256), grd((unsigned)((nbr + 255) / 256));
  hipLaunchKernelGGL(k_bdist_init, grd, blk, 0, v->stream, v->d_brick, nbr, v->brick_cap, a);
  DMF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bdist_pass, grd, blk, 0, v->stream, v->nb[0], v->nb[1], v->nb[2], 2, v->brick_cap, a, b);
  DMF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bdist_pass, grd, blk, 0, v->stream, v->nb[0], v->nb[1], v->nb[2], 1, v->brick_cap, b, a);
  DMF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bdist_pass, grd, blk, 0, v->stream, v->nb[0], v->nb[1], v->nb[2], 0, v->brick_cap, a, b);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(a, b, (size_t)nbr, hipMemcpyDeviceToDevice, v->stream));
  v->bdist_valid = true;
  return DMF_OK;
}

}  // namespace dmf

using namespace dmf;

dmf::Geom dmf_volume::geom() const {
  Geom g;
  const double mn[3] = {xmin, ymin, zmin}, mx[3] = {xmax, ymax, zmax}, dl[3] = {xdelta, ydelta, zdelta};
  const int n[3] = {xdim, ydim, zdim};
  g.pow2 = 1;
  for (int a = 0; a < 3; ++a) {
    g.mn[a] = mn[a]; g.mx[a] = mx[a]; g.dl[a] = dl[a]; g.hdl[a] = dl[a] / 2.0; g.n[a] = n[a];
    int e;
    const double m = std::frexp(dl[a], &e);
    const bool p2 = (m == 0.5) && std::isfinite(dl[a]) && dl[a] > 0;
    g.inv[a] = p2 ? 1.0 / dl[a] : 0.0;
    if (!p2) g.pow2 = 0;
    float lo = (float)mn[a], hi = (float)mx[a];
    if (!((double)lo > mn[a])) lo = std::nextafter(lo, INFINITY);
    if (!((double)hi < mx[a])) hi = std::nextafter(hi, -INFINITY);
    g.vlo[a] = lo;
    g.vhi[a] = hi;
  }
  fbin_setup(g);
  jump_margin_setup(g);
  return g;
}

dmf::DevVol dmf_volume::dev() const {
  DevVol d;
  d.occ = d_occ; d.bdist = d_bdist; d.bsh = brick_shift;
  d.brick = d_brick; d.nb[0] = nb[0]; d.nb[1] = nb[1]; d.nb[2] = nb[2]; d.slot_of = d_slot_of; d.hash = d_hash; d.off = d_off; d.nrm = d_csr_nrm;
  d.view = d_view; d.good = d_good; d.V = V;
  return d;
}

static void free_state(dmf_volume* v) {
  auto f = [&](void* p) { if (p) (void)hipFree(p); };
  f(v->d_occ); f(v->d_brick); f(v->d_bdist); f(v->d_slot_of); f(v->d_hash); f(v->d_view); f(v->d_good);
  f(v->d_pts); f(v->d_pnrm); f(v->d_pslot); f(v->d_off); f(v->d_csr_nrm); f(v->d_csr_pts);
  f(v->d_axes); f(v->d_enum); f(v->d_sorder); f(v->d_fault);
  v->d_fault = nullptr;
  v->d_sorder = nullptr;
  v->sorder_cap = 0;
  v->sorder_valid = false;
  for (auto& s : v->scratch) f(s.first);
  v->scratch.clear();
  v->d_occ = nullptr; v->d_brick = nullptr; v->d_bdist = nullptr; v->bdist_valid = false; v->d_slot_of = nullptr; v->d_hash = nullptr; v->d_view = nullptr; v->d_good = nullptr;
  v->d_pts = nullptr; v->d_pnrm = nullptr; v->d_pslot = nullptr; v->d_off = nullptr; v->d_csr_nrm = nullptr;
  v->d_csr_pts = nullptr; v->d_axes = nullptr; v->d_enum = nullptr;
  v->V = v->Vcap = v->npts = v->pcap = v->nbinned = v->csr_cap = v->nenum = v->enum_cap = 0;
  v->enum_valid = false;
  v->bdist_valid = false;
  v->constructed = false;
}

extern "C" {

int dmf_abi_version(void) { return DMF_ABI_VERSION; }

const char* dmf_status_string(int s) {
  switch (s) {
    case DMF_OK: return "ok";
    case DMF_ERR_INVALID: return "invalid argument";
    case DMF_ERR_STATE: return "invalid state";
    case DMF_ERR_HIP: return "HIP runtime error";
    case DMF_ERR_NOMEM: return "out of memory";
    case DMF_ERR_CAPACITY: return "output buffer too small";
    case DMF_ERR_RANGE: return "size out of range";
    case DMF_ERR_NO_DEVICE: return "no usable GPU";
    case DMF_ERR_DEVICE_CHECK: return "device-side consistency check failed";
    default: return "unknown status";
  }
}

const char* dmf_last_error(void) { return g_err; }

int dmf_device_count(int32_t* count) {
  if (!count) return fail(DMF_ERR_INVALID, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = (e == hipSuccess) ? n : 0;
  return DMF_OK;
}

void dmf_fuse_params_default(dmf_fuse_params* p) {
  if (!p) return;
  p->dmin_mm = 1;
  p->dmax_mm = 65535;
  p->l_hit = 847;
  p->l_miss = -405;
  p->l_min = -2000;
  p->l_max = 3511;
}

int dmf_angle_threshold(float* dstar) {
  if (!dstar) return fail(DMF_ERR_INVALID, "null output");
  *dstar = angle_threshold();
  return DMF_OK;
}

int dmf_volume_create(dmf_volume** out, int32_t device) {
  DMF_API_BEGIN
  if (!out) return fail(DMF_ERR_INVALID, "null out");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(DMF_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return fail(DMF_ERR_INVALID, "device %d out of range [0,%d)", device, n);
  hipDeviceProp_t prop;
  DMF_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(DMF_ERR_NO_DEVICE, "device %d is %s, this build targets gfx950", device, prop.gcnArchName);
  auto* v = new dmf_volume();
  v->device = device;
  v->dstar = angle_threshold();
  // brick-fusion scratch budget: 45 % of the device's HBM (~130 GB of MI355X's 288 GB; the
  // two staging slots of pipelined calls get half each), at least 8 GiB -- every pose batch a
  // smaller pair capacity forces costs its own passes and counter flushes (the device cuts
  // the batches by the pairs a call really makes).  Config 5's 1024^3 shard (2.85G pairs +
  // the per-pose tables) runs as two batches per pipelined call at 45 %, in the same time as
  // one batch at 55 % (round 5: 68.6 ms either way); the rest of the device
  // stays free for a second volume or the caller.  A volume only allocates what
  // its plan uses (dmf_fuse_plan); dmf_fuse_reserve sets another budget.
  v->bk_budget = std::max<uint64_t>(8ull << 30, (uint64_t)prop.totalGlobalMem / 20 * 9);
  *out = v;
  return DMF_OK;
  DMF_API_END
}

int dmf_volume_destroy(dmf_volume* v) {
  DMF_API_BEGIN
  if (!v) return DMF_OK;
  (void)hipSetDevice(v->device);
  if (v->stream) (void)hipStreamSynchronize(v->stream);
  (void)hipDeviceSynchronize();
  free_state(v);
  if (v->switch_ev) (void)hipEventDestroy(v->switch_ev);
  for (hipEvent_t e : {v->st_in, v->st_done[0], v->st_done[1], v->st_free[0], v->st_free[1], v->st_b[0], v->st_b[1], v->st_a[0], v->st_a[1]})
    if (e) (void)hipEventDestroy(e);
  if (v->stage) (void)hipStreamDestroy(v->stage);
  delete v;
  return DMF_OK;
  DMF_API_END
}

// Switching streams never blocks the host: the new stream waits (hipStreamWaitEvent) for
// the work already enqueued on the old one, so scratch buffers in flight stay ordered.
// A new stream that is capturing a graph is not made to wait on a non-captured event
// (not permitted during capture): the capturing caller orders it (torch.cuda.graph
// does, wait_stream before capture).
int dmf_volume_set_stream(dmf_volume* v, void* s) {
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  DMF_TRY(activate(v));
  const hipStream_t ns = (hipStream_t)s;
  if (v->stream == ns) return DMF_OK;
  hipStreamCaptureStatus cs_old = hipStreamCaptureStatusNone, cs_new = hipStreamCaptureStatusNone;
  DMF_HIP(hipStreamIsCapturing(v->stream, &cs_old));
  DMF_HIP(hipStreamIsCapturing(ns, &cs_new));
  if (cs_new == hipStreamCaptureStatusNone && cs_old == hipStreamCaptureStatusNone) {
    if (!v->switch_ev) DMF_HIP(hipEventCreateWithFlags(&v->switch_ev, hipEventDisableTiming));
    DMF_HIP(hipEventRecord(v->switch_ev, v->stream));
    DMF_HIP(hipStreamWaitEvent(ns, v->switch_ev, 0));
  }
  v->stream = ns;
  return DMF_OK;
}

int dmf_volume_synchronize(dmf_volume* v) {
  DMF_TRY(activate(v));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
}

int dmf_volume_set_dimensions(dmf_volume* v, double xmin, double xmax, double ymin, double ymax, double zmin,
                              double zmax) {
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  v->xmin = xmin; v->xmax = xmax; v->ymin = ymin; v->ymax = ymax; v->zmin = zmin; v->zmax = zmax;
  v->xcenter = v->xmin + (v->xmax - v->xmin) / 2.0;
  v->ycenter = v->ymin + (v->ymax - v->ymin) / 2.0;
  v->zcenter = v->zmin + (v->zmax - v->zmin) / 2.0;
  return DMF_OK;
}

int dmf_volume_set_resolution(dmf_volume* v, double dx, double dy, double dz) {
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  v->xdelta = dx; v->ydelta = dy; v->zdelta = dz;
  return DMF_OK;
}

int dmf_volume_set_volume_size(dmf_volume* v, int32_t nx, int32_t ny, int32_t nz) {
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  v->xdim = nx; v->ydim = ny; v->zdim = nz;
  v->xdelta = (v->xmax - v->xmin) / nx;
  v->ydelta = (v->ymax - v->ymin) / ny;
  v->zdelta = (v->zmax - v->zmin) / nz;
  return DMF_OK;
}

int dmf_volume_construct(dmf_volume* v) {
  DMF_API_BEGIN
  DMF_TRY(activate(v));
  const double ex = (v->xmax - v->xmin) / v->xdelta, ey = (v->ymax - v->ymin) / v->ydelta,
               ez = (v->zmax - v->zmin) / v->zdelta;
  if (!(ex >= 1 && ey >= 1 && ez >= 1) || !(ex < 1048576 && ey < 1048576 && ez < 1048576))
    return fail(DMF_ERR_RANGE, "volume dims must be in [1, 2^20) (got %g x %g x %g)", ex, ey, ez);
  DMF_HIP(hipStreamSynchronize(v->stream));
  free_state(v);
  // Volume.hpp:121-125 truncating recompute; hsize_ is an int product
  v->xdim = (int)ex; v->ydim = (int)ey; v->zdim = (int)ez;
  v->hsize = (uint64_t)(int64_t)(int32_t)((uint32_t)v->xdim * (uint32_t)v->ydim * (uint32_t)v->zdim);
  v->voxel_size = v->xdelta * v->ydelta * v->zdelta;
  v->ncell = (size_t)v->xdim * v->ydim * v->zdim;
  if (v->ncell >= (size_t)0x7fffffff) return fail(DMF_ERR_RANGE, "more than 2^31-1 cells");
  const uint64_t nocc = occ_words(v->geom().n);
  if (nocc * 32u > (uint64_t)UINT32_MAX)
    return fail(DMF_ERR_RANGE, "occupancy bitmask over 2^32 bits (grid padded to 8-cell tiles)");
  DMF_HIP(hipMalloc((void**)&v->d_occ, sizeof(uint32_t) * (nocc + 1)));
  DMF_HIP(hipMemsetAsync(v->d_occ, 0, sizeof(uint32_t) * (nocc + 1), v->stream));
  v->brick_shift = kBrickShiftDefault;
  v->brick_cap = kBrickDistCapDefault;
  const int bs = 1 << v->brick_shift;
  v->nb[0] = (v->xdim + bs - 1) / bs; v->nb[1] = (v->ydim + bs - 1) / bs; v->nb[2] = (v->zdim + bs - 1) / bs;
  const size_t bwords = ((size_t)v->nb[0] * v->nb[1] * v->nb[2] + 31) / 32 + 1;
  DMF_HIP(hipMalloc((void**)&v->d_brick, sizeof(uint32_t) * bwords));
  DMF_HIP(hipMemsetAsync(v->d_brick, 0, sizeof(uint32_t) * bwords, v->stream));
  // brick distance field + one scratch copy for the separable passes
  DMF_HIP(hipMalloc((void**)&v->d_bdist, 2 * ((size_t)v->nb[0] * v->nb[1] * v->nb[2] + 64)));
  v->bdist_valid = false;
  DMF_HIP(hipMalloc((void**)&v->d_slot_of, sizeof(int32_t) * v->ncell));
  DMF_HIP(hipMemsetD32Async((hipDeviceptr_t)v->d_slot_of, kEmpty, v->ncell, v->stream));
  DMF_HIP(hipMalloc((void**)&v->d_off, sizeof(int32_t)));
  DMF_HIP(hipMemsetAsync(v->d_off, 0, sizeof(int32_t), v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  v->constructed = true;
  v->hazards = 0;
  return DMF_OK;
  DMF_API_END
}

int dmf_volume_get_info(const dmf_volume* v, dmf_volume_info* o) {
  if (!v || !o) return fail(DMF_ERR_INVALID, "null argument");
  o->xmin = v->xmin; o->xmax = v->xmax; o->ymin = v->ymin; o->ymax = v->ymax; o->zmin = v->zmin; o->zmax = v->zmax;
  o->xcenter = v->xcenter; o->ycenter = v->ycenter; o->zcenter = v->zcenter;
  o->xdelta = v->xdelta; o->ydelta = v->ydelta; o->zdelta = v->zdelta;
  o->voxel_size = v->voxel_size;
  o->xdim = v->xdim; o->ydim = v->ydim; o->zdim = v->zdim;
  o->constructed = v->constructed ? 1 : 0;
  o->hsize = v->hsize;
  o->num_occupied = v->V;
  o->num_points = v->nbinned;
  o->hazards = v->hazards;
  return DMF_OK;
}

int dmf_volume_integrate_device(dmf_volume* v, const float* d_xyz, const float* d_nrm, int64_t n) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (n > 0 && !d_xyz) return fail(DMF_ERR_INVALID, "null points");
  return integrate_impl(v, d_xyz, d_nrm, n, nullptr, nullptr);
  DMF_API_END
}

int dmf_volume_integrate(dmf_volume* v, const float* xyz, const float* nrm, int64_t n, int64_t* binned,
                         int64_t* hazard) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (n < 0 || (n > 0 && !xyz)) return fail(DMF_ERR_INVALID, "bad points");
  if (n == 0) { if (binned) *binned = 0; if (hazard) *hazard = 0; return DMF_OK; }
  void *dx, *dn = nullptr;
  DMF_TRY(scratch(v, kScHost1, sizeof(float) * 3 * n, &dx));
  DMF_HIP(hipMemcpyAsync(dx, xyz, sizeof(float) * 3 * n, hipMemcpyHostToDevice, v->stream));
  if (nrm) {
    DMF_TRY(scratch(v, kScHost2, sizeof(float) * 3 * n, &dn));
    DMF_HIP(hipMemcpyAsync(dn, nrm, sizeof(float) * 3 * n, hipMemcpyHostToDevice, v->stream));
  }
  return integrate_impl(v, (const float*)dx, (const float*)dn, n, binned, hazard);
  DMF_API_END
}

int dmf_volume_occupied(const dmf_volume* v, uint64_t* hashes, int64_t cap, int64_t* n) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (n) *n = v->V;
  if (cap < v->V) return hashes ? fail(DMF_ERR_CAPACITY, "need %lld entries", (long long)v->V) : DMF_OK;
  if (v->V > 0) {
    if (!hashes) return fail(DMF_ERR_INVALID, "null output");
    DMF_HIP(hipMemcpyAsync(hashes, v->d_hash, sizeof(uint64_t) * v->V, hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
  }
  return DMF_OK;
  DMF_API_END
}

int dmf_volume_voxel_flags(const dmf_volume* v, int32_t* view, uint8_t* good, int64_t cap) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (cap < v->V) return fail(DMF_ERR_CAPACITY, "need %lld entries", (long long)v->V);
  if (v->V > 0) {
    if (view) DMF_HIP(hipMemcpyAsync(view, v->d_view, sizeof(int32_t) * v->V, hipMemcpyDeviceToHost, v->stream));
    if (good) DMF_HIP(hipMemcpyAsync(good, v->d_good, v->V, hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
  }
  return DMF_OK;
  DMF_API_END
}

int dmf_volume_reset_flags(dmf_volume* v) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (v->V > 0) {
    DMF_HIP(hipMemsetAsync(v->d_view, 0, sizeof(int32_t) * v->V, v->stream));
    DMF_HIP(hipMemsetAsync(v->d_good, 0, v->V, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
  }
  return DMF_OK;
  DMF_API_END
}

__global__ void k_voxel_counts(const int32_t* __restrict__ off, const float4* __restrict__ nrm, int64_t V,
                               int64_t* __restrict__ npts, int64_t* __restrict__ nn) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= V) return;
  const int32_t a = off[s], b = off[s + 1];
  npts[s] = b - a;
  int64_t c = 0;
  for (int32_t j = a; j < b; ++j) c += nrm[j].w != 0.0f;
  nn[s] = c;
}

int dmf_volume_voxel_counts(const dmf_volume* v, int64_t* npts, int64_t* nnormals, int64_t cap) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (cap < v->V) return fail(DMF_ERR_CAPACITY, "need %lld entries", (long long)v->V);
  if (v->V == 0) return DMF_OK;
  void *a, *b;
  DMF_TRY(scratch(v_mut(v), kScOut0, sizeof(int64_t) * v->V, &a));
  DMF_TRY(scratch(v_mut(v), kScOut1, sizeof(int64_t) * v->V, &b));
  hipLaunchKernelGGL(k_voxel_counts, dim3((unsigned)((v->V + 255) / 256)), dim3(256), 0, v->stream, v->d_off,
                     v->d_csr_nrm, v->V, (int64_t*)a, (int64_t*)b);
  DMF_LAUNCH_CHECK();
  if (npts) DMF_HIP(hipMemcpyAsync(npts, a, sizeof(int64_t) * v->V, hipMemcpyDeviceToHost, v->stream));
  if (nnormals) DMF_HIP(hipMemcpyAsync(nnormals, b, sizeof(int64_t) * v->V, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_volume_voxel_points(const dmf_volume* v, uint64_t hash, float* pts, float* nrm, int64_t cap, int64_t* n) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!n) return fail(DMF_ERR_INVALID, "null n");
  const int x = (int)(hash >> 40), y = (int)((hash >> 20) & 0xFFFFF), z = (int)(hash & 0xFFFFF);
  *n = -1;
  if (x >= v->xdim || y >= v->ydim || z >= v->zdim) return DMF_OK;
  const size_t lin = ((size_t)x * v->ydim + y) * v->zdim + z;
  int32_t slot = kEmpty;
  DMF_HIP(hipMemcpyAsync(&slot, v->d_slot_of + lin, sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  if (slot < 0 || slot == kEmpty) return DMF_OK;
  int32_t ab[2];
  DMF_HIP(hipMemcpy(ab, v->d_off + slot, sizeof(ab), hipMemcpyDeviceToHost));
  const int64_t cnt = ab[1] - ab[0];
  *n = cnt;
  if (cap < cnt) return (pts || nrm) ? fail(DMF_ERR_CAPACITY, "need %lld points", (long long)cnt) : DMF_OK;
  if (cnt == 0) return DMF_OK;
  if (pts) DMF_HIP(hipMemcpy(pts, v->d_csr_pts + 3 * (size_t)ab[0], sizeof(float) * 3 * cnt, hipMemcpyDeviceToHost));
  if (nrm) {
    std::vector<float4> tmp(cnt);
    DMF_HIP(hipMemcpy(tmp.data(), v->d_csr_nrm + ab[0], sizeof(float4) * cnt, hipMemcpyDeviceToHost));
    int64_t k = 0;
    for (int64_t i = 0; i < cnt; ++i)
      if (tmp[i].w != 0.0f) { nrm[3 * k] = tmp[i].x; nrm[3 * k + 1] = tmp[i].y; nrm[3 * k + 2] = tmp[i].z; ++k; }
    for (; k < cnt; ++k) nrm[3 * k] = nrm[3 * k + 1] = nrm[3 * k + 2] = 0.0f;
  }
  return DMF_OK;
  DMF_API_END
}

int dmf_volume_export(const dmf_volume* v, int32_t* offsets, float* pts, float* normals4, int64_t cap) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (cap < v->nbinned && (pts || normals4)) return fail(DMF_ERR_CAPACITY, "need %lld points", (long long)v->nbinned);
  if (offsets) DMF_HIP(hipMemcpyAsync(offsets, v->d_off, sizeof(int32_t) * (v->V + 1), hipMemcpyDeviceToHost, v->stream));
  if (v->nbinned > 0) {
    if (pts)
      DMF_HIP(hipMemcpyAsync(pts, v->d_csr_pts, sizeof(float) * 3 * v->nbinned, hipMemcpyDeviceToHost, v->stream));
    if (normals4)
      DMF_HIP(hipMemcpyAsync(normals4, v->d_csr_nrm, sizeof(float4) * v->nbinned, hipMemcpyDeviceToHost, v->stream));
  }
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

__global__ void k_occupancy_dense(Geom g, const uint32_t* __restrict__ occ, size_t n, uint8_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t nyz = (uint32_t)g.n[1] * (uint32_t)g.n[2];
  const int x = (int)((uint32_t)i / nyz), y = (int)(((uint32_t)i / g.n[2]) % g.n[1]), z = (int)((uint32_t)i % g.n[2]);
  out[i] = occ_test(occ, occ_bit(g, x, y, z)) ? 1 : 0;
}

int dmf_volume_occupancy(const dmf_volume* v, uint8_t* dense) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!dense) return fail(DMF_ERR_INVALID, "null output");
  void* d;
  DMF_TRY(scratch(v_mut(v), kScOut0, v->ncell, &d));
  hipLaunchKernelGGL(k_occupancy_dense, dim3((unsigned)((v->ncell + 255) / 256)), dim3(256), 0, v->stream, v->geom(), v->d_occ,
                     v->ncell, (uint8_t*)d);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(dense, d, v->ncell, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_backproject_device(dmf_volume* v, const dmf_camera* cam, const uint16_t* d_depth, const float* d_poses,
                           int32_t P, float* d_xyz) {
  DMF_API_BEGIN
  DMF_TRY(activate(v));
  DMF_TRY(check_camera(cam));
  if (!d_depth || !d_xyz) return fail(DMF_ERR_INVALID, "null buffer");
  PoseX* tab;
  DMF_TRY(pose_table(v, d_poses, P, true, &tab));
  const CamP cp = cam_params(cam);
  const int64_t HW = (int64_t)cp.H * cp.W;
  hipLaunchKernelGGL(k_backproject, dim3((unsigned)((HW + 255) / 256), P), dim3(256), 0, v->stream, cp, d_depth, tab,
                     P, d_xyz);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
  DMF_API_END
}

int dmf_backproject(dmf_volume* v, const dmf_camera* cam, const uint16_t* depth, const float* pose, float* xyz) {
  DMF_API_BEGIN
  DMF_TRY(activate(v));
  DMF_TRY(check_camera(cam));
  if (!depth || !pose || !xyz) return fail(DMF_ERR_INVALID, "null buffer");
  const int64_t HW = (int64_t)cam->height * cam->width;
  void *dd, *dp, *dx;
  DMF_TRY(scratch(v, kScHost1, sizeof(uint16_t) * HW, &dd));
  DMF_TRY(scratch(v, kScHost2, sizeof(float) * 12, &dp));
  DMF_TRY(scratch(v, kScOut0, sizeof(float) * 3 * HW, &dx));
  DMF_HIP(hipMemcpyAsync(dd, depth, sizeof(uint16_t) * HW, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dp, pose, sizeof(float) * 12, hipMemcpyHostToDevice, v->stream));
  DMF_TRY(dmf_backproject_device(v, cam, (const uint16_t*)dd, (const float*)dp, 1, (float*)dx));
  DMF_HIP(hipMemcpyAsync(xyz, dx, sizeof(float) * 3 * HW, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_device_malloc(dmf_volume* v, void** p, size_t bytes) {
  DMF_TRY(activate(v));
  if (!p) return fail(DMF_ERR_INVALID, "null out");
  DMF_HIP(hipMalloc(p, std::max<size_t>(bytes, 1)));
  return DMF_OK;
}
int dmf_device_free(dmf_volume* v, void* p) {
  DMF_TRY(activate(v));
  if (p) DMF_HIP(hipFree(p));
  return DMF_OK;
}
int dmf_memcpy_h2d(dmf_volume* v, void* d, const void* h, size_t bytes) {
  DMF_TRY(activate(v));
  DMF_HIP(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
}
int dmf_memcpy_d2h(dmf_volume* v, void* h, const void* d, size_t bytes) {
  DMF_TRY(activate(v));
  DMF_HIP(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
}
int dmf_memset_device(dmf_volume* v, void* d, int value, size_t bytes) {
  DMF_TRY(activate(v));
  DMF_HIP(hipMemsetAsync(d, value, bytes, v->stream));
  return DMF_OK;
}

}  // extern "C"
