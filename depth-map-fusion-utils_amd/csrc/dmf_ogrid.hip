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
// downloadReorganizedCloud (:200-286) is the same kind of racy loop: its sequential
// result is computed by fixed-point rounds over sorted (target, source) keys (below).
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

// ---- downloadReorganizedCloud (:200-286) ----------------------------------------
// Sequential semantics (the reference's OpenMP loops race): voxels are visited x-major;
// an occupied voxel s (with clean: count >= 100 at its turn) merges its CURRENT
// reorganized state into the voxel t(s) holding its centroid.  Its current state P(s) is
// its initial state folded with the merges of the voxels before it that targeted it, so
// P depends only on lower indices.  Parallel form: iterate
//   targets t_r(s) from P_r;  P_{r+1}(T) = init(T) folded with [P_r(s) : s < T, t_r(s) = T]
// (sorted (T, s) keys, one lane per T, sources in index order) until P stops changing;
// round r makes every voxel of dependency depth < r exact, so the fixed point is the
// sequential result.  Then one final fold per target over ALL its sources in order gives
// the reorganized grid (a source equal to its target reads P(T), which is exactly the
// aliased state the reference reads: n + n, (c + c) / 2).
struct OgS {
  float n[3], c[3];
  int32_t k;
};

__device__ inline void og_merge(OgS& d, const OgS& s) {  // :242-255
  const float sum[3] = {d.n[0] + s.n[0], d.n[1] + s.n[1], d.n[2] + s.n[2]};
  normalized(sum, d.n);
  if (d.k == 0) {
    d.c[0] = s.c[0]; d.c[1] = s.c[1]; d.c[2] = s.c[2];
  } else {
#pragma unroll
    for (int a = 0; a < 3; ++a) d.c[a] = (d.c[a] + s.c[a]) / 2.0f;
    ++d.k;
  }
}

__global__ void k_og_reorg_seed(int64_t n, const float* __restrict__ normal, const float* __restrict__ centroid,
                                const int32_t* __restrict__ count, OgS* __restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  OgS s;
#pragma unroll
  for (int a = 0; a < 3; ++a) { s.n[a] = normal[3 * i + a]; s.c[a] = centroid[3 * i + a]; }
  s.k = count[i];
  P[i] = s;
}

// Keys (t(s) << 32 | s) of the voxels that merge, from their current estimate P(s).
__global__ void k_og_reorg_keys(OGeom g, int64_t n, const uint8_t* __restrict__ flags, const OgS* __restrict__ P,
                                int clean, unsigned long long* __restrict__ keys, unsigned long long* __restrict__ cnt) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n || !(flags[s] & 1)) return;
  const OgS st = P[s];
  if (clean && st.k < 100) return;
  int t[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) t[a] = to_int_x86(floor(((double)st.c[a] - g.mn[a]) / g.res[a]));  // :373-379
  if (!og_valid(g, t[0], t[1], t[2])) return;
  const uint64_t T = ((uint64_t)t[0] * g.n[1] + t[1]) * g.n[2] + t[2];
  keys[atomicAdd(cnt, 1ull)] = (T << 32) | (uint64_t)s;
}

// One lane per target segment of the sorted keys.  FINAL = 0: the target's current state
// (sources before it only) -> Pn; FINAL = 1: every source in order -> F, and occ[T] = 1.
template <int FINAL>
__global__ void k_og_reorg_fold(const unsigned long long* __restrict__ keys, int64_t ne, const OgS* __restrict__ init,
                                const OgS* __restrict__ P, OgS* __restrict__ out, uint8_t* __restrict__ occ) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= ne) return;
  const uint64_t T = keys[e] >> 32;
  if (e > 0 && (keys[e - 1] >> 32) == T) return;  // not the first key of its target
  OgS d = init[T];
  for (int64_t f = e; f < ne && (keys[f] >> 32) == T; ++f) {
    const uint64_t s = keys[f] & 0xffffffffull;
    if (!FINAL && s >= T) break;
    og_merge(d, P[s]);
  }
  out[T] = d;
  if (FINAL) occ[T] = 1;
}

__global__ void k_og_reorg_diff(int64_t n, const OgS* __restrict__ a, const OgS* __restrict__ b,
                                unsigned int* __restrict__ changed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* x = (const uint32_t*)&a[i];
  const uint32_t* y = (const uint32_t*)&b[i];
  bool d = false;
#pragma unroll
  for (int w = 0; w < 7; ++w) d |= x[w] != y[w];
  if (d) *changed = 1u;
}

// Fallback when the rounds do not settle (a dependency chain longer than the round
// cap): the sequential loop itself, one lane.
__global__ void k_og_reorg_serial(OGeom g, int64_t n, const uint8_t* __restrict__ flags, int clean,
                                  OgS* __restrict__ R, uint8_t* __restrict__ occ) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (int64_t s = 0; s < n; ++s) {
    if (!(flags[s] & 1)) continue;
    const OgS st = R[s];
    if (clean && st.k < 100) continue;
    int t[3];
    for (int a = 0; a < 3; ++a) t[a] = to_int_x86(floor(((double)st.c[a] - g.mn[a]) / g.res[a]));
    if (!og_valid(g, t[0], t[1], t[2])) continue;
    const int64_t T = ((int64_t)t[0] * g.n[1] + t[1]) * g.n[2] + t[2];
    OgS d = R[T];
    og_merge(d, st);
    R[T] = d;
    occ[T] = 1;
  }
}

__global__ void k_og_select_reorg(const uint8_t* __restrict__ occ, int64_t n, int32_t* __restrict__ sel) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sel[i] = occ[i] ? 1 : 0;
}

__global__ void k_og_gather_state(const int32_t* __restrict__ sel, const int32_t* __restrict__ pos, int64_t n,
                                  const OgS* __restrict__ F, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !sel[i]) return;
  float* o = out + 6 * (int64_t)pos[i];
  const OgS f = F[i];
#pragma unroll
  for (int a = 0; a < 3; ++a) { o[a] = f.c[a]; o[3 + a] = f.n[a]; }
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

static int og_sort_keys(dmf_volume* v, unsigned long long* kb, size_t ne, size_t ncell, unsigned long long** out) {
  if (ne <= 1) { *out = kb; return DMF_OK; }
  void* ob;
  DMF_TRY(scratch(v, kScSort1, sizeof(unsigned long long) * ne, &ob));
  int vbits = 1;
  while ((1ull << vbits) < (unsigned long long)ncell) ++vbits;
  size_t bytes = 0;
  DMF_HIP(rocprim::radix_sort_keys(nullptr, bytes, kb, (unsigned long long*)ob, ne, 0, 32 + vbits, v->stream));
  void* tmp;
  DMF_TRY(scratch(v, kScTmp, bytes, &tmp));
  DMF_HIP(rocprim::radix_sort_keys(tmp, bytes, kb, (unsigned long long*)ob, ne, 0, 32 + vbits, v->stream));
  *out = (unsigned long long*)ob;
  return DMF_OK;
}

// Reorganized grid (F, occ) of downloadReorganizedCloud(clean); see the kernels above.
static int og_reorganize(dmf_ogrid* g, int clean, OgS** F_out, uint8_t** occ_out, int* rounds_out) {
  dmf_volume* v = g->ctx;
  const int64_t n = (int64_t)g->ncell;
  const OGeom og = og_geom(g);
  const dim3 grd((unsigned)((n + 255) / 256)), blk(256);
  void *p0, *p1, *pf, *po, *kb, *cnt;
  DMF_TRY(scratch(v, kScOgP0, sizeof(OgS) * n, &p0));
  DMF_TRY(scratch(v, kScOgP1, sizeof(OgS) * n, &p1));
  DMF_TRY(scratch(v, kScOgFinal, sizeof(OgS) * n, &pf));
  DMF_TRY(scratch(v, kScOgOcc, (size_t)n + 8, &po));
  DMF_TRY(scratch(v, kScSort0, sizeof(unsigned long long) * n, &kb));
  DMF_TRY(scratch(v, kScCount, 64, &cnt));
  OgS* init = (OgS*)pf;  // the initial state (stage 1 copy), kept until the final fold
  OgS* cur = (OgS*)p0;
  OgS* nxt = (OgS*)p1;
  uint8_t* occ = (uint8_t*)po;
  unsigned int* changed = (unsigned int*)((char*)cnt + 8);
  hipLaunchKernelGGL(k_og_reorg_seed, grd, blk, 0, v->stream, n, g->d_normal, g->d_centroid, g->d_count, init);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(cur, init, sizeof(OgS) * n, hipMemcpyDeviceToDevice, v->stream));
  constexpr int kMaxRounds = 64;
  unsigned long long* keys = nullptr;
  unsigned long long ne = 0;
  int r = 0;
  bool settled = false;
  for (; r < kMaxRounds && !settled; ++r) {
    DMF_HIP(hipMemsetAsync(cnt, 0, 16, v->stream));
    hipLaunchKernelGGL(k_og_reorg_keys, grd, blk, 0, v->stream, og, n, g->d_flags, cur, clean,
                       (unsigned long long*)kb, (unsigned long long*)cnt);
    DMF_LAUNCH_CHECK();
    DMF_HIP(hipMemcpyAsync(&ne, cnt, 8, hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
    DMF_TRY(og_sort_keys(v, (unsigned long long*)kb, (size_t)ne, (size_t)n, &keys));
    DMF_HIP(hipMemcpyAsync(nxt, init, sizeof(OgS) * n, hipMemcpyDeviceToDevice, v->stream));
    if (ne)
      hipLaunchKernelGGL(k_og_reorg_fold<0>, dim3((unsigned)((ne + 255) / 256)), blk, 0, v->stream, keys,
                         (int64_t)ne, init, cur, nxt, occ);
    DMF_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_og_reorg_diff, grd, blk, 0, v->stream, n, cur, nxt, changed);
    DMF_LAUNCH_CHECK();
    unsigned int ch = 0;
    DMF_HIP(hipMemcpyAsync(&ch, changed, 4, hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
    std::swap(cur, nxt);
    settled = ch == 0;  // cur == previous estimate: the targets (keys) are those of cur too
  }
  DMF_HIP(hipMemsetAsync(occ, 0, (size_t)n, v->stream));
  if (settled) {
    // final fold of every source into its target, from the initial state
    DMF_HIP(hipMemcpyAsync(nxt, init, sizeof(OgS) * n, hipMemcpyDeviceToDevice, v->stream));
    if (ne)
      hipLaunchKernelGGL(k_og_reorg_fold<1>, dim3((unsigned)((ne + 255) / 256)), blk, 0, v->stream, keys,
                         (int64_t)ne, init, cur, nxt, occ);
    DMF_LAUNCH_CHECK();
    *F_out = nxt;
  } else {
    DMF_HIP(hipMemcpyAsync(nxt, init, sizeof(OgS) * n, hipMemcpyDeviceToDevice, v->stream));
    hipLaunchKernelGGL(k_og_reorg_serial, dim3(1), dim3(64), 0, v->stream, og, n, g->d_flags, clean, nxt, occ);
    DMF_LAUNCH_CHECK();
    *F_out = nxt;
  }
  *occ_out = occ;
  if (rounds_out) *rounds_out = settled ? r : -1;
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

int dmf_ogrid_set_state(dmf_ogrid* g, const float* normal, const float* centroid, const int32_t* count,
                        const uint8_t* flags) {
  DMF_API_BEGIN
  DMF_TRY(og_ready(g));
  hipStream_t s = g->ctx->stream;
  if (normal) DMF_HIP(hipMemcpyAsync(g->d_normal, normal, sizeof(float) * 3 * g->ncell, hipMemcpyHostToDevice, s));
  if (centroid) DMF_HIP(hipMemcpyAsync(g->d_centroid, centroid, sizeof(float) * 3 * g->ncell, hipMemcpyHostToDevice, s));
  if (count) DMF_HIP(hipMemcpyAsync(g->d_count, count, sizeof(int32_t) * g->ncell, hipMemcpyHostToDevice, s));
  if (flags) DMF_HIP(hipMemcpyAsync(g->d_flags, flags, g->ncell, hipMemcpyHostToDevice, s));
  DMF_HIP(hipStreamSynchronize(s));
  return DMF_OK;
  DMF_API_END
}

int dmf_ogrid_download(dmf_ogrid* g, int32_t mode, float* out, int64_t cap, int64_t* n) {
  DMF_API_BEGIN
  DMF_TRY(og_ready(g));
  if (!n || (cap > 0 && !out)) return fail(DMF_ERR_INVALID, "null argument");
  if (mode < 0 || mode > 3)
    return fail(DMF_ERR_INVALID, "mode must be 0 (downloadCloud), 1 (downloadHQCloud), 2/3 (downloadReorganizedCloud "
                                 "clean=false/true)");
  dmf_volume* v = g->ctx;
  const int64_t nc = (int64_t)g->ncell;
  void *sel, *pos, *buf;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * (nc + 1), &sel));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * (nc + 1), &pos));
  const dim3 grd((unsigned)((nc + 255) / 256));
  OgS* F = nullptr;
  if (mode >= 2) {
    uint8_t* occ;
    DMF_TRY(og_reorganize(g, mode == 3, &F, &occ, nullptr));
    hipLaunchKernelGGL(k_og_select_reorg, grd, dim3(256), 0, v->stream, occ, nc, (int32_t*)sel);
  } else {
    hipLaunchKernelGGL(k_og_select, grd, dim3(256), 0, v->stream, g->d_flags, g->d_count, nc, mode, (int32_t*)sel);
  }
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
  if (F)
    hipLaunchKernelGGL(k_og_gather_state, grd, dim3(256), 0, v->stream, (const int32_t*)sel, (const int32_t*)pos, nc,
                       (const OgS*)F, (float*)buf);
  else
    hipLaunchKernelGGL(k_og_gather, grd, dim3(256), 0, v->stream, (const int32_t*)sel, (const int32_t*)pos, nc,
                       g->d_centroid, g->d_normal, (float*)buf);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(out, buf, sizeof(float) * 6 * (size_t)total, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"
