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
// 64-lane wave an 8x8 packet, so the 64 rays of a wave start at one camera centre
// and stay spatially coherent (neighbouring cells, shared L2 lines).
#include <algorithm>
#include <cmath>

#include "dmf_host.hpp"

namespace dmf {

constexpr int64_t kQ = 256;  // fixed-point sub-cell resolution (1/256 cell)

__device__ inline int64_t clampi(int64_t v, int64_t lo, int64_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ inline void atomic_inc(int32_t* p) {
  __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One ray: clip O->E to the grid, walk the cells, count misses / hit.  Mirrors
// oracle.cpp dda_ray() operation for operation.  Returns the number of cell updates.
__device__ inline int dda_ray(const Geom& g, const float O[3], const float E[3], bool end_inside,
                              int32_t* __restrict__ hits, int32_t* __restrict__ misses, uint32_t ncell) {
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
      if (go[a] < 0.0 || go[a] >= (double)g.n[a]) return 0;
    } else {
      double ta = (0.0 - go[a]) / D[a];
      double tb = ((double)g.n[a] - go[a]) / D[a];
      if (ta > tb) { const double tt = ta; ta = tb; tb = tt; }
      if (ta > t0) t0 = ta;
      if (tb < t1) t1 = tb;
    }
  }
  if (end_inside) { t1 = 1.0; if (t0 > 1.0) t0 = 1.0; }
  if (t0 > t1) return 0;
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
  int st[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int64_t dq = qe[a] - qs[a];
    adq[a] = (uint64_t)(dq < 0 ? -dq : dq);
    st[a] = ce[a] > cs[a] ? 1 : (ce[a] < cs[a] ? -1 : 0);
  }
  // crossing times in half fixed-point units scaled by the other axes' |dq|
  uint64_t Tm[3], In[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const uint64_t M = (a != 0 && adq[0] ? adq[0] : 1) * (a != 1 && adq[1] ? adq[1] : 1) * (a != 2 && adq[2] ? adq[2] : 1);
    const int64_t h = st[a] > 0 ? 2 * ((cs[a] + 1) * kQ - qs[a]) : 2 * (qs[a] - cs[a] * kQ) + 1;
    Tm[a] = st[a] == 0 ? ~0ull : (uint64_t)h * M;
    In[a] = (uint64_t)(2 * kQ) * M;
  }
  const int nsteps = (int)((ce[0] > cs[0] ? ce[0] - cs[0] : cs[0] - ce[0]) + (ce[1] > cs[1] ? ce[1] - cs[1] : cs[1] - ce[1]) +
                           (ce[2] > cs[2] ? ce[2] - cs[2] : cs[2] - ce[2]));
  const int32_t sx = g.n[1] * g.n[2], sy = g.n[2];
  const int32_t d0 = st[0] * sx, d1 = st[1] * sy, d2 = st[2];
  int32_t lin = (int32_t)(cs[0] * sx + cs[1] * sy + cs[2]);
  uint64_t T0 = Tm[0], T1 = Tm[1], T2 = Tm[2];
  if ((uint32_t)lin >= ncell) return -1;  // cannot happen by construction; never fault
  for (int s = 0; s < nsteps; ++s) {
    atomic_inc(&misses[lin]);
    const bool b10 = T1 < T0;
    const uint64_t m01 = b10 ? T1 : T0;
    const bool b2 = T2 < m01;
    if (b2) {
      T2 += In[2];
      lin += d2;
    } else if (b10) {
      T1 += In[1];
      lin += d1;
    } else {
      T0 += In[0];
      lin += d0;
    }
  }
  if ((uint32_t)lin >= ncell) return -1;
  if (end_inside) atomic_inc(&hits[lin]);
  else atomic_inc(&misses[lin]);
  return nsteps + 1;
}

__global__ __launch_bounds__(256) void k_fuse(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                              const PoseX* __restrict__ poses, int dmin, int dmax, int tiles_x,
                                              int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                              unsigned long long* __restrict__ stats) {
  const int p = blockIdx.y;
  const int tile = blockIdx.x;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int c = (tile % tiles_x) * 16 + (w & 1) * 8 + (l & 7);
  const int r = (tile / tiles_x) * 16 + (w >> 1) * 8 + (l >> 3);
  unsigned long long upd = 0, ray = 0, hit = 0, bad = 0;
  if (r < cam.H && c < cam.W) {
    const int d = depth[((int64_t)p * cam.H + r) * cam.W + c];
    if (d >= dmin && d < dmax) {
      const PoseX& T = poses[p];
      float pc[3], E[3];
      project(cam, r, c, d, pc);
      xform(T.f, pc[0], pc[1], pc[2], E);
      bool inside = valid_points(g, E[0], E[1], E[2]);
      if (inside) inside = valid_coords(g, bin_axis(g, 0, E[0]), bin_axis(g, 1, E[1]), bin_axis(g, 2, E[2]));
      const float O[3] = {T.f[3], T.f[7], T.f[11]};
      const uint32_t ncell = (uint32_t)g.n[0] * (uint32_t)g.n[1] * (uint32_t)g.n[2];
      const int u = dda_ray(g, O, E, inside, hits, misses, ncell);
      if (u < 0) {
        bad = 1;
      } else {
        upd = (unsigned long long)u;
        hit = (inside && u > 0) ? 1 : 0;
      }
      ray = 1;
    }
  }
  if (stats) {
    for (int o = 32; o > 0; o >>= 1) {
      upd += __shfl_down(upd, o, 64);
      ray += __shfl_down(ray, o, 64);
      hit += __shfl_down(hit, o, 64);
      bad += __shfl_down(bad, o, 64);
    }
    if (l == 0) {
      if (upd) atomicAdd(&stats[0], upd);
      if (ray) atomicAdd(&stats[1], ray);
      if (hit) atomicAdd(&stats[2], hit);
      if (bad) atomicAdd(&stats[3], bad);
    }
  }
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
  hipLaunchKernelGGL(k_fuse, dim3((unsigned)(tx * ty), (unsigned)P), dim3(256), 0, v->stream, v->geom(), cp, d_depth,
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
