// dmf_ogrid.hip — OccupancyGrid (include/OccupancyGrid.hpp:50-318) on gfx950.
//
// The reference's other fusion path: updateStates folds, per voxel, a running
// normalised normal sum (pass 1, over the normal cloud) and then a running centroid
// mean of point projections onto that normal (pass 2, over the point cloud) for every
// voxel within K of each point, under `#pragma omp parallel for` with racy
// read-modify-writes.  Here the result is the deterministic one — the single-threaded
// order (points in cloud order; for one voxel the contributing points are distinct and
// arrive in point order) — computed race-free: every (voxel, point) event becomes a
// 64-bit key voxel << 32 | point, keys are radix-sorted, and one lane folds each
// voxel's events in order with the reference's float arithmetic (no FMA contraction).
// Dense per-voxel state in the reference's x-major order, persistent across calls.
#include <algorithm>
#include <cmath>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "dmf_host.hpp"

struct dmf_ogrid {
  dmf_volume* ctx = nullptr;  // device, stream and scratch arena (never constructed)
  double bounds[6] = {0, 0, 0, 0, 0, 0};
  double res[3] = {0, 0, 0};
  int dims[3] = {0, 0, 0};
  int k = 0;
  size_t ncell = 0;
  float* d_normal = nullptr;    // 3 per voxel
  float* d_centroid = nullptr;  // 3 per voxel
  int32_t* d_count = nullptr;
  uint8_t* d_flags = nullptr;   // bit 0 occupied, bit 1 normal_found
};

namespace dmf {

struct OGeom {
  double mn[3], res[3];
  int n[3], k;
};

__device__ inline bool og_valid(const OGeom& g, int x, int y, int z) {  // OccupancyGrid.hpp:399-402
  return x < g.n[0] && y < g.n[1] && z < g.n[2] && x >= 0 && y >= 0 && z >= 0;
}
__device__ inline int og_coord(const OGeom& g, int a, float p) {  // :373-379
  return (int)floor(((double)p - g.mn[a]) / g.res[a]);
}

// Events (voxel << 32 | point) of points [0, n), stride = floats per point; the order
// of emission is irrelevant (sorted next).
__global__ void k_og_events(OGeom g, const float* __restrict__ pts, int stride, int64_t n,
                            unsigned long long* __restrict__ keys, unsigned long long* __restrict__ count) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float* q = pts + stride * p;
  const int x = og_coord(g, 0, q[0]), y = og_coord(g, 1, q[1]), z = og_coord(g, 2, q[2]);
  const int K = g.k;
  for (int i = -K; i <= K; ++i)
    for (int j = -K; j <= K; ++j)
      for (int k = -K; k <= K; ++k) {
        if (!og_valid(g, x + i, y + j, z + k)) continue;
        const uint64_t v = ((uint64_t)(x + i) * g.n[1] + (y + j)) * g.n[2] + (z + k);
        keys[atomicAdd(count, 1ull)] = (v << 32) | (uint64_t)p;
      }
}

// Pass 1 (:101-123): normal = normalized(normal + n_p) over the voxel's points in order.
__global__ void k_og_fold_normals(const unsigned long long* __restrict__ keys, int64_t ne,
                                  const float* __restrict__ pn, float* __restrict__ normal,
                                  uint8_t* __restrict__ flags) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ne) return;
  const uint64_t v = keys[e] >> 32;
  if (e > 0 && (keys[e - 1] >> 32) == v) return;  // not the first event of its voxel
  float n[3] = {normal[3 * v], normal[3 * v + 1], normal[3 * v + 2]};
  for (int64_t f = e; f < ne && (keys[f] >> 32) == v; ++f) {
    const float* q = pn + 6 * (keys[f] & 0xffffffffull);
    const float s[3] = {n[0] + q[3], n[1] + q[4], n[2] + q[5]};
    normalized(s, n);
  }
  normal[3 * v] = n[0]; normal[3 * v + 1] = n[1]; normal[3 * v + 2] = n[2];
  flags[v] |= 2;
}

// :88-98 projectPointToVector, float (the double ball_radius applied as float).
__device__ inline void og_project(const float pt[3], const float np[3], const float n[3], float out[3]) {
  const float br = (float)0.015;
  float a[3], ap[3], ab[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float d = n[i] * br;
    a[i] = np[i] - d;
    const float b = np[i] + d;
    ap[i] = a[i] - pt[i];
    ab[i] = a[i] - b;
  }
  const float s = sum3(ap[0] * ab[0], ap[1] * ab[1], ap[2] * ab[2]) / sum3(ab[0] * ab[0], ab[1] * ab[1], ab[2] * ab[2]);
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = a[i] - s * ab[i];
}

// Pass 2 (:125-163): for voxels with a normal, fold the running centroid of the point
// projections lying within cylinder_radius of the point.
__global__ void k_og_fold_centroids(OGeom g, const unsigned long long* __restrict__ keys, int64_t ne,
                                    const float* __restrict__ cloud, const float* __restrict__ normal,
                                    float* __restrict__ centroid, int32_t* __restrict__ count,
                                    const uint8_t* __restrict__ flags) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ne) return;
  const uint64_t v = keys[e] >> 32;
  if (e > 0 && (keys[e - 1] >> 32) == v) return;
  if (!(flags[v] & 2)) return;
  const int nyz = g.n[1] * g.n[2];
  const int x = (int)(v / nyz), y = (int)((v / g.n[2]) % g.n[1]), z = (int)(v % g.n[2]);
  const float c[3] = {(float)(g.mn[0] + g.res[0] * x + g.res[0] / 2.0), (float)(g.mn[1] + g.res[1] * y + g.res[1] / 2.0),
                      (float)(g.mn[2] + g.res[2] * z + g.res[2] / 2.0)};
  const float nv[3] = {normal[3 * v], normal[3 * v + 1], normal[3 * v + 2]};
  float cen[3] = {centroid[3 * v], centroid[3 * v + 1], centroid[3 * v + 2]};
  int cnt = count[v];
  for (int64_t f = e; f < ne && (keys[f] >> 32) == v; ++f) {
    const float* pt = cloud + 3 * (keys[f] & 0xffffffffull);
    float pr[3];
    og_project(pt, c, nv, pr);
    const float d[3] = {pt[0] - pr[0], pt[1] - pr[1], pt[2] - pr[2]};
    const float dist = sqrtf(sum3(d[0] * d[0], d[1] * d[1], d[2] * d[2]));
    if ((double)dist < 0.001) {
      ++cnt;
#pragma unroll
      for (int a = 0; a < 3; ++a) cen[a] = cen[a] + (pr[a] - cen[a]) / (float)cnt;
    }
  }
  centroid[3 * v] = cen[0]; centroid[3 * v + 1] = cen[1]; centroid[3 * v + 2] = cen[2];
  count[v] = cnt;
}

// :159-162: the point's own voxel becomes occupied.
__global__ void k_og_occupy(OGeom g, const float* __restrict__ cloud, int64_t n, uint8_t* __restrict__ flags) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float* q = cloud + 3 * p;
  const int x = og_coord(g, 0, q[0]), y = og_coord(g, 1, q[1]), z = og_coord(g, 2, q[2]);
  if (og_valid(g, x, y, z)) atomicOr((unsigned int*)&flags[(((size_t)x * g.n[1] + y) * g.n[2] + z) & ~(size_t)3],
                                     1u << (8 * ((((size_t)x * g.n[1] + y) * g.n[2] + z) & 3)));
}

__global__ void k_og_select(const uint8_t* __restrict__ flags, const int32_t* __restrict__ count, int64_t n,
                            int mode, int32_t* __restrict__ sel) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sel[i] = (flags[i] & 1) && (mode != 1 || count[i] > 100) ? 1 : 0;
}

__global__ void k_og_gather(const int32_t* __restrict__ sel, const int32_t* __restrict__ pos, int64_t n,
                            const float* __restrict__ centroid, const float* __restrict__ normal, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !sel[i]) return;
  float* o = out + 6 * (int64_t)pos[i];
#pragma unroll
  for (int a = 0; a < 3; ++a) { o[a] = centroid[3 * i + a]; o[3 + a] = normal[3 * i + a]; }
}

static OGeom og_geom(const dmf_ogrid* g) {
  OGeom o;
  for (int a = 0; a < 3; ++a) {
    o.mn[a] = g->bounds[2 * a];
    o.res[a] = g->res[a];
    o.n[a] = g->dims[a];
  }
  o.k = g->k;
  return o;
}

static void og_free(dmf_ogrid* g) {
  auto f = [](void* p) { if (p) (void)hipFree(p); };
  f(g->d_normal); f(g->d_centroid); f(g->d_count); f(g->d_flags);
  g->d_normal = g->d_centroid = nullptr;
  g->d_count = nullptr;
  g->d_flags = nullptr;
  g->ncell = 0;
}

// Sort the events of one pass; returns the number of events.
static int og_events(dmf_ogrid* g, const float* d_pts, int stride, int64_t n, unsigned long long** keys_out,
                     int64_t* ne_out) {
  dmf_volume* v = g->ctx;
  const int64_t per = (int64_t)(2 * g->k + 1) * (2 * g->k + 1) * (2 * g->k + 1);
  const size_t cap = (size_t)std::max<int64_t>(n * per, 1);
  void *kb, *cnt;
  DMF_TRY(scratch(v, kScSort0, sizeof(unsigned long long) * cap, &kb));
  DMF_TRY(scratch(v, kScCount, 64, &cnt));
  DMF_HIP(hipMemsetAsync(cnt, 0, 8, v->stream));
  if (n > 0)
    hipLaunchKernelGGL(k_og_events, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream, og_geom(g), d_pts, stride,
                       n, (unsigned long long*)kb, (unsigned long long*)cnt);
  DMF_LAUNCH_CHECK();
  unsigned long long ne = 0;
  DMF_HIP(hipMemcpyAsync(&ne, cnt, 8, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  if (ne > 1) {
    void* ob;
    DMF_TRY(scratch(v, kScSort1, sizeof(unsigned long long) * ne, &ob));
    int vbits = 1;
    while ((1ull << vbits) < (unsigned long long)g->ncell) ++vbits;
    size_t bytes = 0;
    DMF_HIP(rocprim::radix_sort_keys(nullptr, bytes, (unsigned long long*)kb, (unsigned long long*)ob, (size_t)ne, 0,
                                     32 + vbits, v->stream));
    void* tmp;
    DMF_TRY(scratch(v, kScTmp, bytes, &tmp));
    DMF_HIP(rocprim::radix_sort_keys(tmp, bytes, (unsigned long long*)kb, (unsigned long long*)ob, (size_t)ne, 0,
                                     32 + vbits, v->stream));
    *keys_out = (unsigned long long*)ob;
  } else {
    *keys_out = (unsigned long long*)kb;
  }
  *ne_out = (int64_t)ne;
  return DMF_OK;
}

static int og_update(dmf_ogrid* g, const float* d_cloud, int64_t n_cloud, const float* d_pn, int64_t n_nrm) {
  dmf_volume* v = g->ctx;
  const OGeom og = og_geom(g);
  unsigned long long* keys;
  int64_t ne;
  DMF_TRY(og_events(g, d_pn, 6, n_nrm, &keys, &ne));
  if (ne > 0)
    hipLaunchKernelGGL(k_og_fold_normals, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, v->stream, keys, ne, d_pn,
                       g->d_normal, g->d_flags);
  DMF_LAUNCH_CHECK();
  DMF_TRY(og_events(g, d_cloud, 3, n_cloud, &keys, &ne));
  if (ne > 0)
    hipLaunchKernelGGL(k_og_fold_centroids, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, v->stream, og, keys, ne,
                       d_cloud, g->d_normal, g->d_centroid, g->d_count, g->d_flags);
  DMF_LAUNCH_CHECK();
  if (n_cloud > 0)
    hipLaunchKernelGGL(k_og_occupy, dim3((unsigned)((n_cloud + 255) / 256)), dim3(256), 0, v->stream, og, d_cloud,
                       n_cloud, g->d_flags);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
}

static int og_ready(const dmf_ogrid* g) {
  if (!g) return fail(DMF_ERR_INVALID, "null grid");
  if (!g->ncell) return fail(DMF_ERR_STATE, "grid not constructed (dmf_ogrid_setup)");
  return activate(g->ctx);
}

}  // namespace dmf

using namespace dmf;

extern "C" {

int dmf_ogrid_create(dmf_ogrid** out, int32_t device) {
  DMF_API_BEGIN
  if (!out) return fail(DMF_ERR_INVALID, "null argument");
  dmf_ogrid* g = new dmf_ogrid();
  const int st = dmf_volume_create(&g->ctx, device);
  if (st != DMF_OK) { delete g; return st; }
  *out = g;
  return DMF_OK;
  DMF_API_END
}

int dmf_ogrid_destroy(dmf_ogrid* g) {
  DMF_API_BEGIN
  if (!g) return DMF_OK;
  if (g->ctx) {
    (void)activate(g->ctx);
    (void)hipStreamSynchronize(g->ctx->stream);
  }
  og_free(g);
  if (g->ctx) dmf_volume_destroy(g->ctx);
  delete g;
  return DMF_OK;
  DMF_API_END
}

int dmf_ogrid_set_stream(dmf_ogrid* g, void* hip_stream) {
  if (!g) return fail(DMF_ERR_INVALID, "null grid");
  return dmf_volume_set_stream(g->ctx, hip_stream);
}

int dmf_ogrid_setup(dmf_ogrid* g, const double* bounds, float xres, float yres, float zres, int32_t k) {
  DMF_API_BEGIN
  if (!g || !bounds) return fail(DMF_ERR_INVALID, "null argument");
  DMF_TRY(activate(g->ctx));
  if (k < 0 || k > 8) return fail(DMF_ERR_RANGE, "K must be in [0, 8]");
  if (!(xres > 0 && yres > 0 && zres > 0)) return fail(DMF_ERR_INVALID, "resolution must be > 0");
  // setDimensions (:323-336), setResolution(float) (:338-343), setK, construct (:345-352)
  std::memcpy(g->bounds, bounds, sizeof(g->bounds));
  g->res[0] = xres; g->res[1] = yres; g->res[2] = zres;
  g->k = k;
  int d[3];
  for (int a = 0; a < 3; ++a) {
    const double e = (bounds[2 * a + 1] - bounds[2 * a]) / g->res[a];
    if (!(e >= 1 && e < 1048576)) return fail(DMF_ERR_RANGE, "grid dims must be in [1, 2^20)");
    d[a] = (int)e;
  }
  const size_t n = (size_t)d[0] * d[1] * d[2];
  if (n >= (size_t)0x7fffffff) return fail(DMF_ERR_RANGE, "more than 2^31-1 cells");
  DMF_HIP(hipStreamSynchronize(g->ctx->stream));
  og_free(g);
  g->dims[0] = d[0]; g->dims[1] = d[1]; g->dims[2] = d[2];
  DMF_HIP(hipMalloc((void**)&g->d_normal, sizeof(float) * 3 * n));
  DMF_HIP(hipMalloc((void**)&g->d_centroid, sizeof(float) * 3 * n));
  DMF_HIP(hipMalloc((void**)&g->d_count, sizeof(int32_t) * n));
  DMF_HIP(hipMalloc((void**)&g->d_flags, (n + 3) / 4 * 4));
  DMF_HIP(hipMemsetAsync(g->d_normal, 0, sizeof(float) * 3 * n, g->ctx->stream));
  DMF_HIP(hipMemsetAsync(g->d_centroid, 0, sizeof(float) * 3 * n, g->ctx->stream));
  DMF_HIP(hipMemsetAsync(g->d_count, 0, sizeof(int32_t) * n, g->ctx->stream));
  DMF_HIP(hipMemsetAsync(g->d_flags, 0, (n + 3) / 4 * 4, g->ctx->stream));
  g->ncell = n;
  return DMF_OK;
  DMF_API_END
}

int dmf_ogrid_get_dims(const dmf_ogrid* g, int32_t* dims) {
  if (!g || !dims) return fail(DMF_ERR_INVALID, "null argument");
  dims[0] = g->dims[0]; dims[1] = g->dims[1]; dims[2] = g->dims[2];
  return DMF_OK;
}

int dmf_ogrid_update_states_device(dmf_ogrid* g, const float* d_cloud, int64_t n_cloud, const float* d_normals,
                                   int64_t n_normals) {
  DMF_API_BEGIN
  DMF_TRY(og_ready(g));
  if (n_cloud < 0 || n_normals < 0 || n_cloud >= 0x7fffffff || n_normals >= 0x7fffffff)
    return fail(DMF_ERR_RANGE, "point counts must be in [0, 2^31)");
  if ((n_cloud && !d_cloud) || (n_normals && !d_normals)) return fail(DMF_ERR_INVALID, "null point buffer");
  return og_update(g, d_cloud, n_cloud, d_normals, n_normals);
  DMF_API_END
}

int dmf_ogrid_update_states(dmf_ogrid* g, const float* cloud, int64_t n_cloud, const float* normals,
                            int64_t n_normals) {
  DMF_API_BEGIN
  DMF_TRY(og_ready(g));
  if (n_cloud < 0 || n_normals < 0 || n_cloud >= 0x7fffffff || n_normals >= 0x7fffffff)
    return fail(DMF_ERR_RANGE, "point counts must be in [0, 2^31)");
  if ((n_cloud && !cloud) || (n_normals && !normals)) return fail(DMF_ERR_INVALID, "null point buffer");
  void *dc, *dn;
  DMF_TRY(scratch(g->ctx, kScHost0, sizeof(float) * 3 * std::max<int64_t>(n_cloud, 1), &dc));
  DMF_TRY(scratch(g->ctx, kScHost1, sizeof(float) * 6 * std::max<int64_t>(n_normals, 1), &dn));
  if (n_cloud)
    DMF_HIP(hipMemcpyAsync(dc, cloud, sizeof(float) * 3 * n_cloud, hipMemcpyHostToDevice, g->ctx->stream));
  if (n_normals)
    DMF_HIP(hipMemcpyAsync(dn, normals, sizeof(float) * 6 * n_normals, hipMemcpyHostToDevice, g->ctx->stream));
  DMF_TRY(og_update(g, (const float*)dc, n_cloud, (const float*)dn, n_normals));
  DMF_HIP(hipStreamSynchronize(g->ctx->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_ogrid_state(const dmf_ogrid* g, float* normal, float* centroid, int32_t* count, uint8_t* flags) {
  DMF_API_BEGIN
  DMF_TRY(og_ready(g));
  hipStream_t s = g->ctx->stream;
  if (normal) DMF_HIP(hipMemcpyAsync(normal, g->d_normal, sizeof(float) * 3 * g->ncell, hipMemcpyDeviceToHost, s));
  if (centroid) DMF_HIP(hipMemcpyAsync(centroid, g->d_centroid, sizeof(float) * 3 * g->ncell, hipMemcpyDeviceToHost, s));
  if (count) DMF_HIP(hipMemcpyAsync(count, g->d_count, sizeof(int32_t) * g->ncell, hipMemcpyDeviceToHost, s));
  if (flags) DMF_HIP(hipMemcpyAsync(flags, g->d_flags, g->ncell, hipMemcpyDeviceToHost, s));
  DMF_HIP(hipStreamSynchronize(s));
  return DMF_OK;
  DMF_API_END
}

int dmf_ogrid_download(dmf_ogrid* g, int32_t mode, float* out, int64_t cap, int64_t* n) {
  DMF_API_BEGIN
  DMF_TRY(og_ready(g));
  if (!n || (cap > 0 && !out)) return fail(DMF_ERR_INVALID, "null argument");
  if (mode != 0 && mode != 1) return fail(DMF_ERR_INVALID, "mode must be 0 (downloadCloud) or 1 (downloadHQCloud)");
  dmf_volume* v = g->ctx;
  const int64_t nc = (int64_t)g->ncell;
  void *sel, *pos, *buf;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * (nc + 1), &sel));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * (nc + 1), &pos));
  const dim3 grd((unsigned)((nc + 255) / 256));
  hipLaunchKernelGGL(k_og_select, grd, dim3(256), 0, v->stream, g->d_flags, g->d_count, nc, mode, (int32_t*)sel);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemsetAsync((int32_t*)sel + nc, 0, sizeof(int32_t), v->stream));
  DMF_TRY(exclusive_scan_i32(v, (const int32_t*)sel, (int32_t*)pos, (size_t)nc + 1));
  int32_t total = 0;
  DMF_HIP(hipMemcpyAsync(&total, (int32_t*)pos + nc, sizeof(int32_t), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  *n = total;
  if (total > cap) return fail(DMF_ERR_CAPACITY, "download needs %d points, capacity %lld", total, (long long)cap);
  if (total == 0) return DMF_OK;
  DMF_TRY(scratch(v, kScOut2, sizeof(float) * 6 * (size_t)total, &buf));
  hipLaunchKernelGGL(k_og_gather, grd, dim3(256), 0, v->stream, (const int32_t*)sel, (const int32_t*)pos, nc,
                     g->d_centroid, g->d_normal, (float*)buf);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(out, buf, sizeof(float) * 6 * (size_t)total, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"
