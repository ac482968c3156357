// dmf_fuse.hip — per-ray 3D-DDA log-odds depth fusion on gfx950.
//
// Not in the reference: the ray endpoint is the reference's own
// back-projection (Camera.hpp:24-45 projectPoint + transformPoints, bit-exact) and
// its cell is the reference binning (Volume.hpp:150-156, 199-228); the traversal
// between camera centre and endpoint is an exact integer 3D-DDA (fixed-point
// endpoints, crossing times compared by cross-multiplication), so GPU and CPU
// oracle visit the same cells and the int32 hit/miss counts are bit-identical.
//
// Launch shape: a 256-lane workgroup owns a 16x16 pixel tile of one frame, each
// 64-lane wave an 8x8 packet, so the rays of a workgroup start at one camera centre
// and stay spatially coherent; the production kernel aggregates their cell updates
// in LDS before touching HBM (k_fuse_lds).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "dmf_host.hpp"

namespace dmf {

constexpr int64_t kQ = 256;  // fixed-point sub-cell resolution (1/256 cell)

__device__ inline int64_t clampi(int64_t v, int64_t lo, int64_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ inline void atomic_add_dev(int32_t* p, int32_t v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-ray DDA state after setup (exact integer walk).
struct Ray {
  int c[3];        // current cell
  int st[3];       // step direction per axis (-1, 0, +1)
  int32_t lin;     // linear index of c
  int32_t dl[3];   // linear-index delta per axis step
  uint64_t T[3];   // next crossing time per axis (scaled, half units)
  uint64_t In[3];  // crossing-time increment per axis
  int left;        // remaining cell updates (misses + final), 0 = inactive
  bool end_inside;
};

// Clip O->E to the grid and set up the walk.  Mirrors oracle.cpp dda_ray()
// operation for operation.  Returns false when the ray misses the grid.
__device__ inline bool dda_setup(const Geom& g, const float O[3], const float E[3], bool end_inside, Ray& R) {
  double go[3], ge[3], D[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    go[a] = ((double)O[a] - g.mn[a]) / g.dl[a];
    ge[a] = ((double)E[a] - g.mn[a]) / g.dl[a];
    D[a] = ge[a] - go[a];
  }
  double t0 = 0.0, t1 = 1.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (D[a] == 0.0) {
      if (go[a] < 0.0 || go[a] >= (double)g.n[a]) return false;
    } else {
      double ta = (0.0 - go[a]) / D[a];
      double tb = ((double)g.n[a] - go[a]) / D[a];
      if (ta > tb) { const double tt = ta; ta = tb; tb = tt; }
      if (ta > t0) t0 = ta;
      if (tb < t1) t1 = tb;
    }
  }
  if (end_inside) { t1 = 1.0; if (t0 > 1.0) t0 = 1.0; }
  if (t0 > t1) return false;
  int64_t cs[3], ce[3], qs[3], qe[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double gs = go[a] + t0 * D[a];
    const double gx = end_inside ? ge[a] : go[a] + t1 * D[a];
    cs[a] = clampi((int64_t)floor(gs), 0, g.n[a] - 1);
    ce[a] = end_inside ? (int64_t)floor(ge[a]) : clampi((int64_t)floor(gx), 0, g.n[a] - 1);
    qs[a] = clampi((int64_t)floor(gs * (double)kQ), cs[a] * kQ, cs[a] * kQ + kQ - 1);
    qe[a] = clampi((int64_t)floor(gx * (double)kQ), ce[a] * kQ, ce[a] * kQ + kQ - 1);
  }
  uint64_t adq[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int64_t dq = qe[a] - qs[a];
    adq[a] = (uint64_t)(dq < 0 ? -dq : dq);
    R.st[a] = ce[a] > cs[a] ? 1 : (ce[a] < cs[a] ? -1 : 0);
  }
  // crossing times in half fixed-point units scaled by the other axes' |dq|
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const uint64_t M = (a != 0 && adq[0] ? adq[0] : 1) * (a != 1 && adq[1] ? adq[1] : 1) * (a != 2 && adq[2] ? adq[2] : 1);
    const int64_t h = R.st[a] > 0 ? 2 * ((cs[a] + 1) * kQ - qs[a]) : 2 * (qs[a] - cs[a] * kQ) + 1;
    R.T[a] = R.st[a] == 0 ? ~0ull : (uint64_t)h * M;
    R.In[a] = (uint64_t)(2 * kQ) * M;
  }
  const int nsteps = (int)((ce[0] > cs[0] ? ce[0] - cs[0] : cs[0] - ce[0]) + (ce[1] > cs[1] ? ce[1] - cs[1] : cs[1] - ce[1]) +
                           (ce[2] > cs[2] ? ce[2] - cs[2] : cs[2] - ce[2]));
  const int32_t sx = g.n[1] * g.n[2], sy = g.n[2];
  R.dl[0] = R.st[0] * sx;
  R.dl[1] = R.st[1] * sy;
  R.dl[2] = R.st[2];
  R.c[0] = (int)cs[0];
  R.c[1] = (int)cs[1];
  R.c[2] = (int)cs[2];
  R.lin = (int32_t)(cs[0] * sx + cs[1] * sy + cs[2]);
  R.left = nsteps + 1;
  R.end_inside = end_inside;
  return true;
}

// Advance one cell (earliest crossing; ties x before y before z).
__device__ inline void dda_advance(Ray& R) {
  const bool b10 = R.T[1] < R.T[0];
  const uint64_t m01 = b10 ? R.T[1] : R.T[0];
  const bool b2 = R.T[2] < m01;
  if (b2) {
    R.T[2] += R.In[2]; R.lin += R.dl[2]; R.c[2] += R.st[2];
  } else if (b10) {
    R.T[1] += R.In[1]; R.lin += R.dl[1]; R.c[1] += R.st[1];
  } else {
    R.T[0] += R.In[0]; R.lin += R.dl[0]; R.c[0] += R.st[0];
  }
}

// Per-pixel ray: back-projection (Camera.hpp:24-45) + binning of the endpoint
// (Volume.hpp:150-156, 199-228) + DDA setup.  Returns the update count (0 = no ray).
__device__ inline int pixel_ray(const Geom& g, const CamP& cam, const uint16_t* __restrict__ depth,
                                const PoseX* __restrict__ poses, int p, int r, int c, int dmin, int dmax, Ray& R,
                                bool& valid) {
  R.left = 0;
  valid = false;
  if (r >= cam.H || c >= cam.W) return 0;
  const int d = depth[((int64_t)p * cam.H + r) * cam.W + c];
  if (!(d >= dmin && d < dmax)) return 0;
  valid = true;
  const PoseX& T = poses[p];
  float pc[3], E[3];
  project(cam, r, c, d, pc);
  xform(T.f, pc[0], pc[1], pc[2], E);
  bool inside = valid_points(g, E[0], E[1], E[2]);
  if (inside) inside = valid_coords(g, bin_axis(g, 0, E[0]), bin_axis(g, 1, E[1]), bin_axis(g, 2, E[2]));
  const float O[3] = {T.f[3], T.f[7], T.f[11]};
  if (!dda_setup(g, O, E, inside, R)) { R.left = 0; return 0; }
  return R.left;
}

__device__ inline void wave_stats(unsigned long long* stats, unsigned long long upd, unsigned long long ray,
                                  unsigned long long hit) {
  for (int o = 32; o > 0; o >>= 1) {
    upd += __shfl_down(upd, o, 64);
    ray += __shfl_down(ray, o, 64);
    hit += __shfl_down(hit, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (upd) atomicAdd(&stats[0], upd);
    if (ray) atomicAdd(&stats[1], ray);
    if (hit) atomicAdd(&stats[2], hit);
  }
}

// 16x16 tile of pixels per 256-lane workgroup; each wave an 8x8 packet.
__device__ inline void tile_pixel(int tile, int tiles_x, int& r, int& c) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  c = (tile % tiles_x) * 16 + (w & 1) * 8 + (l & 7);
  r = (tile / tiles_x) * 16 + (w >> 1) * 8 + (l >> 3);
}

// Reference variant: one device-scope atomic per cell update.  Bound by the
// memory-side atomic request rate (profiles/r01_baseline_atomic); kept for A/B.
__global__ __launch_bounds__(256) void k_fuse_direct(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                                     const PoseX* __restrict__ poses, int dmin, int dmax, int tiles_x,
                                                     int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                     unsigned long long* __restrict__ stats) {
  int r, c;
  tile_pixel(blockIdx.x, tiles_x, r, c);
  Ray R;
  bool valid;
  const int upd = pixel_ray(g, cam, depth, poses, blockIdx.y, r, c, dmin, dmax, R, valid);
  const bool hit = R.left > 0 && R.end_inside;
  while (R.left > 1) {
    atomic_add_dev(&misses[R.lin], 1);
    dda_advance(R);
    --R.left;
  }
  if (R.left == 1) atomic_add_dev(R.end_inside ? &hits[R.lin] : &misses[R.lin], 1);
  if (stats) wave_stats(stats, (unsigned long long)upd, valid ? 1ull : 0ull, hit ? 1ull : 0ull);
}

// LDS-aggregated variant (the production kernel).  The 256 rays of a tile walk in
// lockstep rounds of kS cell updates.  Each round the workgroup reduces the
// bounding box of the cells its rays can reach (the packet's slab), counts misses
// into a dense LDS box with LDS atomics, records every first-touched cell in an LDS
// list, then flushes ONE device-scope atomic per distinct cell: the global atomic
// request count drops by the packet's rays-per-cell reuse.  A round
// whose box exceeds kBox cells falls back to direct atomics.  Counts are exact
// integers, so the result is bit-identical to k_fuse_direct and to the oracle.
template <int kS, int kBox>
__global__ __launch_bounds__(256) void k_fuse_lds(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                                  const PoseX* __restrict__ poses, int dmin, int dmax, int tiles_x,
                                                  int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                  unsigned long long* __restrict__ stats) {
  constexpr int kList = 256 * kS;
  __shared__ int box[kBox];
  __shared__ int list_loc[kList];
  __shared__ int32_t list_lin[kList];
  __shared__ int red[4][6];
  __shared__ int nlist;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  for (int i = tid; i < kBox; i += 256) box[i] = 0;
  int r, c;
  tile_pixel(blockIdx.x, tiles_x, r, c);
  Ray R;
  bool valid;
  const int upd = pixel_ray(g, cam, depth, poses, blockIdx.y, r, c, dmin, dmax, R, valid);
  const bool hit = R.left > 0 && R.end_inside;
  while (true) {
    // bounding box of the cells this lane can reach in the next kS updates
    const int rem = R.left < kS ? R.left : kS;
    int lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      if (rem > 0) {
        const int reach = rem - 1;
        lo[a] = R.c[a] - (R.st[a] < 0 ? reach : 0);
        hi[a] = R.c[a] + (R.st[a] > 0 ? reach : 0);
        lo[a] = lo[a] < 0 ? 0 : lo[a];
        hi[a] = hi[a] >= g.n[a] ? g.n[a] - 1 : hi[a];
      } else {
        lo[a] = 0x7fffffff;
        hi[a] = -1;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        lo[a] = min(lo[a], __shfl_xor(lo[a], o, 64));
        hi[a] = max(hi[a], __shfl_xor(hi[a], o, 64));
      }
    }
    if (l == 0) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        red[w][a] = lo[a];
        red[w][3 + a] = hi[a];
      }
    }
    if (tid == 0) nlist = 0;
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      lo[a] = min(min(red[0][a], red[1][a]), min(red[2][a], red[3][a]));
      hi[a] = max(max(red[0][3 + a], red[1][3 + a]), max(red[2][3 + a], red[3][3 + a]));
    }
    if (hi[0] < lo[0]) break;  // no active ray left in the tile (uniform)
    const int e1 = hi[1] - lo[1] + 1, e2 = hi[2] - lo[2] + 1;
    const int64_t vol = (int64_t)(hi[0] - lo[0] + 1) * e1 * e2;
    const bool use_lds = vol <= kBox;
    for (int k = 0; k < rem; ++k) {
      if (R.left == 1 && R.end_inside) {
        atomic_add_dev(&hits[R.lin], 1);
      } else if (use_lds) {
        const int loc = ((R.c[0] - lo[0]) * e1 + (R.c[1] - lo[1])) * e2 + (R.c[2] - lo[2]);
        if (atomicAdd(&box[loc], 1) == 0) {
          const int j = atomicAdd(&nlist, 1);
          list_loc[j] = loc;
          list_lin[j] = R.lin;
        }
      } else {
        atomic_add_dev(&misses[R.lin], 1);
      }
      if (R.left > 1) dda_advance(R);
      --R.left;
    }
    __syncthreads();
    if (use_lds) {
      const int n = nlist;
      for (int j = tid; j < n; j += 256) {
        const int loc = list_loc[j];
        const int cnt = box[loc];
        box[loc] = 0;
        atomic_add_dev(&misses[list_lin[j]], cnt);
      }
    }
    __syncthreads();
  }
  if (stats) wave_stats(stats, (unsigned long long)upd, valid ? 1ull : 0ull, hit ? 1ull : 0ull);
}

// clamp(hits*l_hit + misses*l_miss, l_min, l_max) -> int16, 8 cells per lane
// (2 x 32 B loads, one 16 B store: a pure HBM stream).
__global__ __launch_bounds__(256) void k_finalize(const int32_t* __restrict__ hits, const int32_t* __restrict__ misses,
                                                  int64_t n, int l_hit, int l_miss, int l_min, int l_max,
                                                  int16_t* __restrict__ out) {
  const int64_t i8 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i8 >= n) return;
  auto f = [&](int32_t h, int32_t m) -> int16_t {
    int64_t L = (int64_t)h * l_hit + (int64_t)m * l_miss;
    L = L < l_min ? l_min : (L > l_max ? l_max : L);
    return (int16_t)L;
  };
  if (i8 + 8 <= n) {
    const int4 h0 = *(const int4*)(hits + i8), h1 = *(const int4*)(hits + i8 + 4);
    const int4 m0 = *(const int4*)(misses + i8), m1 = *(const int4*)(misses + i8 + 4);
    union { int16_t s[8]; int4 v; } o;
    o.s[0] = f(h0.x, m0.x); o.s[1] = f(h0.y, m0.y); o.s[2] = f(h0.z, m0.z); o.s[3] = f(h0.w, m0.w);
    o.s[4] = f(h1.x, m1.x); o.s[5] = f(h1.y, m1.y); o.s[6] = f(h1.z, m1.z); o.s[7] = f(h1.w, m1.w);
    *(int4*)(out + i8) = o.v;
  } else {
    for (int64_t i = i8; i < n; ++i) out[i] = f(hits[i], misses[i]);
  }
}

constexpr int kRoundCells = 8;   // cell updates per ray per aggregation round
constexpr int kBoxCells = 8192;  // LDS box capacity (32 KiB)

// DMF_FUSE_MODE=direct selects the one-atomic-per-update kernel (A/B measurements).
static int fuse_mode() {
  static const int mode = [] {
    const char* e = getenv("DMF_FUSE_MODE");
    return (e && std::string(e) == "direct") ? 1 : 0;
  }();
  return mode;
}

static int check_fuse(const dmf_volume* v, const dmf_camera* cam, int P, const dmf_fuse_params* prm) {
  DMF_TRY(require_constructed(v));
  DMF_TRY(check_camera(cam));
  if (!prm) return fail(DMF_ERR_INVALID, "null params");
  if (P <= 0 || P > 65535) return fail(DMF_ERR_INVALID, "pose count %d out of range [1,65535]", P);
  if (v->xdim > 2048 || v->ydim > 2048 || v->zdim > 2048)
    return fail(DMF_ERR_RANGE, "fusion grid is limited to 2048 cells per axis (fixed-point DDA)");
  return DMF_OK;
}

}  // namespace dmf

using namespace dmf;

extern "C" {

int dmf_fuse_depth_device(dmf_volume* v, const dmf_camera* cam, const uint16_t* d_depth, const float* d_poses,
                          int32_t P, const dmf_fuse_params* prm, int32_t* d_hits, int32_t* d_misses,
                          uint64_t* d_stats) {
  DMF_API_BEGIN
  DMF_TRY(check_fuse(v, cam, P, prm));
  if (!d_depth || !d_poses || !d_hits || !d_misses) return fail(DMF_ERR_INVALID, "null device buffer");
  PoseX* tab;
  DMF_TRY(pose_table(v, d_poses, P, true, &tab));
  const CamP cp = cam_params(cam);
  const int tx = (cp.W + 15) / 16, ty = (cp.H + 15) / 16;
  const dim3 grid((unsigned)(tx * ty), (unsigned)P);
  if (fuse_mode() == 1)
    hipLaunchKernelGGL(k_fuse_direct, grid, dim3(256), 0, v->stream, v->geom(), cp, d_depth, tab, prm->dmin_mm,
                       prm->dmax_mm, tx, d_hits, d_misses, (unsigned long long*)d_stats);
  else
    hipLaunchKernelGGL((k_fuse_lds<kRoundCells, kBoxCells>), grid, dim3(256), 0, v->stream, v->geom(), cp, d_depth,
                       tab, prm->dmin_mm, prm->dmax_mm, tx, d_hits, d_misses, (unsigned long long*)d_stats);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_depth(dmf_volume* v, const dmf_camera* cam, const uint16_t* depth, const float* poses, int32_t P,
                   const dmf_fuse_params* prm, int32_t* hits, int32_t* misses, int64_t* stats) {
  DMF_API_BEGIN
  DMF_TRY(check_fuse(v, cam, P, prm));
  if (!depth || !poses || !hits || !misses) return fail(DMF_ERR_INVALID, "null buffer");
  const size_t HW = (size_t)cam->height * cam->width;
  void *dd, *dp, *dh, *dm, *ds;
  DMF_TRY(scratch(v, kScHost1, sizeof(uint16_t) * HW * P, &dd));
  DMF_TRY(scratch(v, kScHost2, sizeof(float) * 12 * P, &dp));
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * v->ncell, &dh));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * v->ncell, &dm));
  DMF_TRY(scratch(v, kScOut2, sizeof(uint64_t) * 4, &ds));
  DMF_HIP(hipMemcpyAsync(dd, depth, sizeof(uint16_t) * HW * P, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dp, poses, sizeof(float) * 12 * P, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dh, hits, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dm, misses, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemsetAsync(ds, 0, sizeof(uint64_t) * 4, v->stream));
  DMF_TRY(dmf_fuse_depth_device(v, cam, (const uint16_t*)dd, (const float*)dp, P, prm, (int32_t*)dh, (int32_t*)dm,
                                (uint64_t*)ds));
  uint64_t st[4];
  DMF_HIP(hipMemcpyAsync(hits, dh, sizeof(int32_t) * v->ncell, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipMemcpyAsync(misses, dm, sizeof(int32_t) * v->ncell, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipMemcpyAsync(st, ds, sizeof(st), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  if (stats)
    for (int k = 0; k < 3; ++k) stats[k] += (int64_t)st[k];
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_finalize_device(dmf_volume* v, const int32_t* d_hits, const int32_t* d_misses,
                             const dmf_fuse_params* prm, int16_t* d_out) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!prm || !d_hits || !d_misses || !d_out) return fail(DMF_ERR_INVALID, "null argument");
  const int64_t n = (int64_t)v->ncell;
  const int64_t lanes = (n + 7) / 8;
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, v->stream, d_hits, d_misses, n,
                     prm->l_hit, prm->l_miss, prm->l_min, prm->l_max, d_out);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_finalize(dmf_volume* v, const int32_t* hits, const int32_t* misses, const dmf_fuse_params* prm,
                      int16_t* out) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!prm || !hits || !misses || !out) return fail(DMF_ERR_INVALID, "null argument");
  void *dh, *dm, *dout;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * v->ncell + 32, &dh));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * v->ncell + 32, &dm));
  DMF_TRY(scratch(v, kScOut2, sizeof(int16_t) * v->ncell + 32, &dout));
  DMF_HIP(hipMemcpyAsync(dh, hits, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dm, misses, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  DMF_TRY(dmf_fuse_finalize_device(v, (const int32_t*)dh, (const int32_t*)dm, prm, (int16_t*)dout));
  DMF_HIP(hipMemcpyAsync(out, dout, sizeof(int16_t) * v->ncell, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"
