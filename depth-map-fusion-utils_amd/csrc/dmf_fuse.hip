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

// Wave-wide min / max through DPP (row_shr 1,2,4,8 then row_bcast 15/31) and a
// readlane: no LDS traffic, unlike __shfl_xor (ds_bpermute).
__device__ inline int wave_min(int v) {
  constexpr int kId = 0x7fffffff;
  v = min(v, __builtin_amdgcn_update_dpp(kId, v, 0x111, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(kId, v, 0x112, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(kId, v, 0x114, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(kId, v, 0x118, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(kId, v, 0x142, 0xa, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(kId, v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ inline int wave_max(int v) {
  constexpr int kId = (int)0x80000000;
  v = max(v, __builtin_amdgcn_update_dpp(kId, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(kId, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(kId, v, 0x114, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(kId, v, 0x118, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(kId, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(kId, v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
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
  stats = stat_slot(stats);
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
template <int kS, int kBox, int kFlush, bool kDpp = false, bool kVec = false, bool kExact = false, int kAblate = 0>
__global__ __launch_bounds__(256) void k_fuse_lds(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                                  const PoseX* __restrict__ poses, int dmin, int dmax, int tiles_x,
                                                  int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                  unsigned long long* __restrict__ stats) {
  stats = stat_slot(stats);
  constexpr bool kScan = kFlush == 1, kRows = kFlush == 2;
  constexpr int kList = kFlush == 1 ? 1 : 256 * kS;
  __shared__ __attribute__((aligned(16))) int box[kBox];
  __shared__ int list_loc[kList];                  // list: cell loc   | rows: row index
  __shared__ int32_t list_lin[kList];              // list: global lin | rows: global row base
  __shared__ uint32_t rowbits[kRows ? kBox / 32 : 1];
  __shared__ int red[4][6];
  __shared__ int nlist;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  for (int i = tid; i < kBox; i += 256) box[i] = 0;
  if (kRows)
    for (int i = tid; i < kBox / 32; i += 256) rowbits[i] = 0;
  int r, c;
  tile_pixel(blockIdx.x, tiles_x, r, c);
  Ray R;
  bool valid;
  const int upd = pixel_ray(g, cam, depth, poses, blockIdx.y, r, c, dmin, dmax, R, valid);
  const bool hit = R.left > 0 && R.end_inside;
  unsigned long long nflush = 0, nround_lds = 0, nround_direct = 0;
  while (true) {
    // bounding box of the cells this lane can reach in the next kS updates
    const int rem = R.left < kS ? R.left : kS;
    int lo[3], hi[3];
    if (kExact && rem > 0) {
      // exact extent: pre-walk the round on a copy of the DDA state (VALU is cheap here)
      Ray P = R;
      for (int k = 1; k < rem; ++k) dda_advance(P);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        lo[a] = min(R.c[a], P.c[a]);
        hi[a] = max(R.c[a], P.c[a]);
      }
    } else {
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
    }
    if (kDpp) {
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        lo[a] = wave_min(lo[a]);
        hi[a] = wave_max(hi[a]);
      }
    } else {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          lo[a] = min(lo[a], __shfl_xor(lo[a], o, 64));
          hi[a] = max(hi[a], __shfl_xor(hi[a], o, 64));
        }
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
    if (tid == 0) ++(use_lds ? nround_lds : nround_direct);
    for (int k = 0; k < rem; ++k) {
      if (R.left == 1 && R.end_inside) {
        atomic_add_dev(&hits[R.lin], 1);
      } else if (use_lds) {
        const int row = (R.c[0] - lo[0]) * e1 + (R.c[1] - lo[1]);
        const int loc = row * e2 + (R.c[2] - lo[2]);
        if (kAblate & 2) {
          nflush += (unsigned)loc;  // timing ablation: no LDS atomic
        } else if (kScan) {
          atomicAdd(&box[loc], 1);
        } else if (kRows) {
          if (atomicAdd(&box[loc], 1) == 0) {
            const uint32_t bit = 1u << (row & 31);
            if ((atomicOr(&rowbits[row >> 5], bit) & bit) == 0) {
              const int j = atomicAdd(&nlist, 1);
              list_loc[j] = row;
              list_lin[j] = R.lin - R.c[2];
            }
          }
        } else if (atomicAdd(&box[loc], 1) == 0) {
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
      if (kRows) {
        // touched rows only; consecutive lanes -> consecutive z of a row -> contiguous atomics
        const int nr = nlist;
        const int total = nr * e2;
        // k = i / e2 by a 33-bit reciprocal: ceil(2^32/e2) (2^32 for e2 = 1); exact for i, e2 <= 2^13
        const uint64_t magic = (0x100000000ull + (uint64_t)e2 - 1) / (uint64_t)e2;
        for (int i = tid; i < total; i += 256) {
          const int k = (int)(((uint64_t)i * magic) >> 32);
          const int iz = i - k * e2;
          const int loc = list_loc[k] * e2 + iz;
          const int cnt = box[loc];
          if (cnt) {
            ++nflush;
            box[loc] = 0;
            atomic_add_dev(&misses[list_lin[k] + lo[2] + iz], cnt);
          }
        }
        for (int k = tid; k < nr; k += 256) rowbits[list_loc[k] >> 5] = 0;
      } else if (kScan) {
        if (kVec) {
        // in-order box scan, 4 cells per 128-bit LDS read: consecutive lanes -> consecutive
        // z of a box row -> contiguous device atomics
        const int nyz = g.n[1] * g.n[2];
        const int e12 = e1 * e2;
        const uint64_t m12 = (0x100000000ull + (uint64_t)e12 - 1) / (uint64_t)e12;  // exact /e12, /e2
        const uint64_t m2 = (0x100000000ull + (uint64_t)e2 - 1) / (uint64_t)e2;     // for i, e <= 2^13
        int4* box4 = reinterpret_cast<int4*>(box);
        const int nvec = ((int)vol + 3) >> 2;
        for (int j = tid; j < nvec; j += 256) {
          const int4 q = box4[j];
          if ((q.x | q.y | q.z | q.w) == 0) continue;
          box4[j] = make_int4(0, 0, 0, 0);
          const int i0 = 4 * j;
          int ix = (int)(((uint64_t)i0 * m12) >> 32);
          const int r2 = i0 - ix * e12;
          int iy = (int)(((uint64_t)r2 * m2) >> 32);
          int iz = r2 - iy * e2;
          const int cnts[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (cnts[t]) {
              ++nflush;
              atomic_add_dev(&misses[(lo[0] + ix) * nyz + (lo[1] + iy) * g.n[2] + lo[2] + iz], cnts[t]);
            }
            if (++iz == e2) { iz = 0; if (++iy == e1) { iy = 0; ++ix; } }
          }
        }
        } else {
          const int nyz = g.n[1] * g.n[2];
          const int e12 = e1 * e2;
          for (int i = tid; i < (int)vol; i += 256) {
            const int cnt = box[i];
            if (cnt) {
              ++nflush;
              box[i] = 0;
                  const int ix = i / e12, rem2 = i - ix * e12, iy = rem2 / e2, iz = rem2 - iy * e2;
              if (!(kAblate & 1))  // timing ablation: no device atomics in the flush
                atomic_add_dev(&misses[(lo[0] + ix) * nyz + (lo[1] + iy) * g.n[2] + lo[2] + iz], cnt);
              else
                nflush += (unsigned)(ix + iy + iz);
            }
          }
        }
      } else {
        const int n = nlist;
        for (int j = tid; j < n; j += 256) {
          const int loc = list_loc[j];
          const int cnt = box[loc];
          box[loc] = 0;
          ++nflush;
          atomic_add_dev(&misses[list_lin[j]], cnt);
        }
      }
    }
    __syncthreads();
  }
  if (stats) {
    wave_stats(stats, (unsigned long long)upd, valid ? 1ull : 0ull, hit ? 1ull : 0ull);
    // aggregation diagnostics: [4] LDS rounds, [5] fallback rounds, [6] flushed cells
    for (int o = 32; o > 0; o >>= 1) nflush += __shfl_down(nflush, o, 64);
    if (l == 0 && nflush) atomicAdd(&stats[6], nflush);
    if (tid == 0) {
      if (nround_lds) atomicAdd(&stats[4], nround_lds);
      if (nround_direct) atomicAdd(&stats[5], nround_direct);
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

// Branch-free DDA step over the crossing times only; returns the axis taken
// (ties x before y before z) as the three selector masks.
__device__ inline void dda_pick(uint64_t& T0, uint64_t& T1, uint64_t& T2, uint64_t I0, uint64_t I1, uint64_t I2,
                                bool& s0, bool& s1, bool& s2) {
  const bool b10 = T1 < T0;
  const uint64_t m = b10 ? T1 : T0;
  s2 = T2 < m;
  s1 = !s2 && b10;
  s0 = !s2 && !b10;
  T0 = s0 ? T0 + I0 : T0;
  T1 = s1 ? T1 + I1 : T1;
  T2 = s2 ? T2 + I2 : T2;
}

// Lean LDS-aggregated fusion kernel.  Same rounds / LDS slab box / in-order flush as
// k_fuse_lds, but inside an LDS round a lane only advances its crossing times and
// its box-local index (branch-free); the cell coordinates and the grid index are
// recovered once per round by exact reciprocal division.  Bit-identical counts.
template <int kS, int kBox>
__global__ __launch_bounds__(256) void k_fuse_lean(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                                   const PoseX* __restrict__ poses, int dmin, int dmax, int tiles_x,
                                                   int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                   unsigned long long* __restrict__ stats) {
  stats = stat_slot(stats);
  __shared__ __attribute__((aligned(16))) int box[kBox];
  __shared__ int red[4][6];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  for (int i = tid; i < kBox; i += 256) box[i] = 0;
  int r, c;
  tile_pixel(blockIdx.x, tiles_x, r, c);
  Ray R;
  bool valid;
  const int upd = pixel_ray(g, cam, depth, poses, blockIdx.y, r, c, dmin, dmax, R, valid);
  const bool hit = R.left > 0 && R.end_inside;
  const int nyz = g.n[1] * g.n[2], nz = g.n[2];
  uint64_t T0 = R.T[0], T1 = R.T[1], T2 = R.T[2];
  const uint64_t I0 = R.In[0], I1 = R.In[1], I2 = R.In[2];
  int c0 = R.c[0], c1 = R.c[1], c2 = R.c[2];
  int lin = R.lin, left = R.left;
  unsigned long long nflush = 0, nround_lds = 0, nround_direct = 0;
  while (true) {
    const int rem = left < kS ? left : kS;
    int lo0, lo1, lo2, hi0, hi1, hi2;
    {
      const int reach = rem - 1;
      const bool act = rem > 0;
      lo0 = act ? max(c0 - (R.st[0] < 0 ? reach : 0), 0) : 0x7fffffff;
      lo1 = act ? max(c1 - (R.st[1] < 0 ? reach : 0), 0) : 0x7fffffff;
      lo2 = act ? max(c2 - (R.st[2] < 0 ? reach : 0), 0) : 0x7fffffff;
      hi0 = act ? min(c0 + (R.st[0] > 0 ? reach : 0), g.n[0] - 1) : -1;
      hi1 = act ? min(c1 + (R.st[1] > 0 ? reach : 0), g.n[1] - 1) : -1;
      hi2 = act ? min(c2 + (R.st[2] > 0 ? reach : 0), g.n[2] - 1) : -1;
    }
    lo0 = wave_min(lo0); lo1 = wave_min(lo1); lo2 = wave_min(lo2);
    hi0 = wave_max(hi0); hi1 = wave_max(hi1); hi2 = wave_max(hi2);
    if (l == 0) {
      red[w][0] = lo0; red[w][1] = lo1; red[w][2] = lo2;
      red[w][3] = hi0; red[w][4] = hi1; red[w][5] = hi2;
    }
    __syncthreads();
    lo0 = min(min(red[0][0], red[1][0]), min(red[2][0], red[3][0]));
    lo1 = min(min(red[0][1], red[1][1]), min(red[2][1], red[3][1]));
    lo2 = min(min(red[0][2], red[1][2]), min(red[2][2], red[3][2]));
    hi0 = max(max(red[0][3], red[1][3]), max(red[2][3], red[3][3]));
    hi1 = max(max(red[0][4], red[1][4]), max(red[2][4], red[3][4]));
    hi2 = max(max(red[0][5], red[1][5]), max(red[2][5], red[3][5]));
    if (hi0 < lo0) break;  // no active ray left in the tile (uniform)
    const int e1 = hi1 - lo1 + 1, e2 = hi2 - lo2 + 1, e12 = e1 * e2;
    const int64_t vol = (int64_t)(hi0 - lo0 + 1) * e12;
    const bool use_lds = vol <= kBox;
    const int nf = rem < left ? rem : rem - 1;  // updates followed by an advance
    const bool fin = rem == left && rem > 0;    // this round holds the final update
    if (use_lds) {
      if (tid == 0) ++nround_lds;
      const int b0 = R.st[0] * e12, b1 = R.st[1] * e2, b2 = R.st[2];
      int loc = ((c0 - lo0) * e1 + (c1 - lo1)) * e2 + (c2 - lo2);
      int ploc = loc;  // last updated (in-box) cell
      bool s0 = false, s1 = false, s2 = false;
      for (int k = 0; k < nf; ++k) {
        atomicAdd(&box[loc], 1);
        dda_pick(T0, T1, T2, I0, I1, I2, s0, s1, s2);
        ploc = loc;
        loc += s2 ? b2 : (s1 ? b1 : b0);
      }
      if (rem > 0) {
        // Recover the cell from an in-box index (exact reciprocal division for loc,
        // e <= 2^13).  A non-final round ends one advance past its box: decode the
        // last updated cell and apply that advance to the coordinates.
        const int dloc = fin ? loc : ploc;
        const uint64_t m12 = (0x100000000ull + (uint64_t)e12 - 1) / (uint64_t)e12;
        const uint64_t m2 = (0x100000000ull + (uint64_t)e2 - 1) / (uint64_t)e2;
        const int ix = (int)(((uint64_t)dloc * m12) >> 32);
        const int rr = dloc - ix * e12;
        const int iy = (int)(((uint64_t)rr * m2) >> 32);
        c0 = lo0 + ix;
        c1 = lo1 + iy;
        c2 = lo2 + (rr - iy * e2);
        if (!fin) {
          c0 += s0 ? R.st[0] : 0;
          c1 += s1 ? R.st[1] : 0;
          c2 += s2 ? R.st[2] : 0;
        }
        lin = c0 * nyz + c1 * nz + c2;
        if (fin) {
          if (R.end_inside) atomic_add_dev(&hits[lin], 1);
          else atomicAdd(&box[loc], 1);
        }
      }
    } else {
      if (tid == 0) ++nround_direct;
      for (int k = 0; k < nf; ++k) {
        atomic_add_dev(&misses[lin], 1);
        bool s0, s1, s2;
        dda_pick(T0, T1, T2, I0, I1, I2, s0, s1, s2);
        lin += s2 ? R.dl[2] : (s1 ? R.dl[1] : R.dl[0]);
        c0 += s0 ? R.st[0] : 0;
        c1 += s1 ? R.st[1] : 0;
        c2 += s2 ? R.st[2] : 0;
      }
      if (fin) atomic_add_dev(R.end_inside ? &hits[lin] : &misses[lin], 1);
    }
    left -= rem;
    __syncthreads();
    if (use_lds) {
      // in-order box scan: consecutive lanes -> consecutive z -> contiguous device atomics
      for (int i = tid; i < (int)vol; i += 256) {
        const int cnt = box[i];
        if (cnt) {
          ++nflush;
          box[i] = 0;
          const int ix = i / e12, rr = i - ix * e12, iy = rr / e2, iz = rr - iy * e2;
          atomic_add_dev(&misses[(lo0 + ix) * nyz + (lo1 + iy) * nz + lo2 + iz], cnt);
        }
      }
    }
    __syncthreads();
  }
  if (stats) {
    wave_stats(stats, (unsigned long long)upd, valid ? 1ull : 0ull, hit ? 1ull : 0ull);
    for (int o = 32; o > 0; o >>= 1) nflush += __shfl_down(nflush, o, 64);
    if (l == 0 && nflush) atomicAdd(&stats[6], nflush);
    if (tid == 0) {
      if (nround_lds) atomicAdd(&stats[4], nround_lds);
      if (nround_direct) atomicAdd(&stats[5], nround_direct);
    }
  }
}

// Single-walk LDS-aggregated fusion kernel (production).  Per round each lane walks
// its DDA once for up to kS updates, recording the axis of every step as a 2-bit
// code; the tile's exact slab box is reduced (DPP + LDS); the codes are replayed into
// box indices held in registers, and the LDS atomics are issued forward on even
// lanes and backward on odd lanes so that neighbouring rays, which share cells at
// the same step, rarely hit the same LDS address in one instruction.  In-order box
// scan flush (contiguous device atomics).  Bit-identical counts.
template <int kS, int kBox>
__global__ __launch_bounds__(256) void k_fuse_v2(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                                 const PoseX* __restrict__ poses, int dmin, int dmax, int tiles_x,
                                                 int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                 unsigned long long* __restrict__ stats) {
  stats = stat_slot(stats);
  static_assert(kS <= 16, "2-bit step codes are packed into one 32-bit register");
  __shared__ __attribute__((aligned(16))) int box[kBox];
  __shared__ int red[4][6];
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  for (int i = tid; i < kBox; i += 256) box[i] = 0;
  int r, c;
  tile_pixel(blockIdx.x, tiles_x, r, c);
  Ray R;
  bool valid;
  const int upd = pixel_ray(g, cam, depth, poses, blockIdx.y, r, c, dmin, dmax, R, valid);
  const bool hit = R.left > 0 && R.end_inside;
  const int nyz = g.n[1] * g.n[2], nz = g.n[2];
  uint64_t T0 = R.T[0], T1 = R.T[1], T2 = R.T[2];
  const uint64_t I0 = R.In[0], I1 = R.In[1], I2 = R.In[2];
  int c0 = R.c[0], c1 = R.c[1], c2 = R.c[2];
  int left = R.left;
  const bool odd = (l & 1) != 0;
  unsigned long long nflush = 0, nround_lds = 0, nround_direct = 0;
  while (true) {
    const int rem = left < kS ? left : kS;
    const bool fin = rem == left && rem > 0;  // this round holds the ray's final update
    const int nadv = fin ? rem - 1 : rem;      // DDA advances this round
    // walk once: 2-bit axis code per advance, end cell of the round
    uint32_t codes = 0;
    int e0 = c0, e1c = c1, e2c = c2;
#pragma unroll
    for (int k = 0; k < kS; ++k) {
      if (k < nadv) {
        bool s0, s1, s2;
        dda_pick(T0, T1, T2, I0, I1, I2, s0, s1, s2);
        codes |= (s2 ? 2u : (s1 ? 1u : 0u)) << (2 * k);
        e0 += s0 ? R.st[0] : 0;
        e1c += s1 ? R.st[1] : 0;
        e2c += s2 ? R.st[2] : 0;
      }
    }
    // exact extent per axis: monotone walk -> [min, max] of start and last updated cell;
    // the last advance of a non-final round leaves the round, so use the cell before it
    int l0 = c0, l1 = c1, l2 = c2;
    if (!fin && nadv > 0) {
      const uint32_t last = (codes >> (2 * (nadv - 1))) & 3u;
      l0 = e0 - (last == 0u ? R.st[0] : 0);
      l1 = e1c - (last == 1u ? R.st[1] : 0);
      l2 = e2c - (last == 2u ? R.st[2] : 0);
    } else {
      l0 = e0; l1 = e1c; l2 = e2c;
    }
    const bool act = rem > 0;
    int lo0 = act ? min(c0, l0) : 0x7fffffff, hi0 = act ? max(c0, l0) : -1;
    int lo1 = act ? min(c1, l1) : 0x7fffffff, hi1 = act ? max(c1, l1) : -1;
    int lo2 = act ? min(c2, l2) : 0x7fffffff, hi2 = act ? max(c2, l2) : -1;
    lo0 = wave_min(lo0); lo1 = wave_min(lo1); lo2 = wave_min(lo2);
    hi0 = wave_max(hi0); hi1 = wave_max(hi1); hi2 = wave_max(hi2);
    if (l == 0) {
      red[w][0] = lo0; red[w][1] = lo1; red[w][2] = lo2;
      red[w][3] = hi0; red[w][4] = hi1; red[w][5] = hi2;
    }
    __syncthreads();
    lo0 = min(min(red[0][0], red[1][0]), min(red[2][0], red[3][0]));
    lo1 = min(min(red[0][1], red[1][1]), min(red[2][1], red[3][1]));
    lo2 = min(min(red[0][2], red[1][2]), min(red[2][2], red[3][2]));
    hi0 = max(max(red[0][3], red[1][3]), max(red[2][3], red[3][3]));
    hi1 = max(max(red[0][4], red[1][4]), max(red[2][4], red[3][4]));
    hi2 = max(max(red[0][5], red[1][5]), max(red[2][5], red[3][5]));
    if (hi0 < lo0) break;  // no active ray left in the tile (uniform)
    const int bx1 = hi1 - lo1 + 1, bx2 = hi2 - lo2 + 1, b12 = bx1 * bx2;
    const int64_t vol = (int64_t)(hi0 - lo0 + 1) * b12;
    const bool use_lds = vol <= kBox;
    const int nmiss = (fin && R.end_inside) ? rem - 1 : rem;  // LDS/miss updates this round
    if (use_lds) {
      if (tid == 0) ++nround_lds;
      const int sx = R.st[0] * b12, sy = R.st[1] * bx2, sz = R.st[2];
      int loc[kS];
      int cur = ((c0 - lo0) * bx1 + (c1 - lo1)) * bx2 + (c2 - lo2);
#pragma unroll
      for (int k = 0; k < kS; ++k) {
        loc[k] = cur;
        const uint32_t cd = (codes >> (2 * k)) & 3u;
        cur += cd == 2u ? sz : (cd == 1u ? sy : sx);
      }
#pragma unroll
      for (int k = 0; k < kS; ++k) {
        const int kk = odd ? kS - 1 - k : k;
        if (kk < nmiss) atomicAdd(&box[loc[kk]], 1);
      }
    } else {
      if (tid == 0) ++nround_direct;
      int lin = c0 * nyz + c1 * nz + c2;
      const int d0 = R.st[0] * nyz, d1 = R.st[1] * nz, d2 = R.st[2];
#pragma unroll
      for (int k = 0; k < kS; ++k) {
        if (k < nmiss) atomic_add_dev(&misses[lin], 1);
        const uint32_t cd = (codes >> (2 * k)) & 3u;
        lin += cd == 2u ? d2 : (cd == 1u ? d1 : d0);
      }
    }
    if (fin && R.end_inside) atomic_add_dev(&hits[e0 * nyz + e1c * nz + e2c], 1);
    c0 = e0; c1 = e1c; c2 = e2c;
    left -= rem;
    __syncthreads();
    if (use_lds) {
      // in-order box scan: consecutive lanes -> consecutive z -> contiguous device atomics
      for (int i = tid; i < (int)vol; i += 256) {
        const int cnt = box[i];
        if (cnt) {
          ++nflush;
          box[i] = 0;
          const int ix = i / b12, rr = i - ix * b12, iy = rr / bx2, iz = rr - iy * bx2;
          atomic_add_dev(&misses[(lo0 + ix) * nyz + (lo1 + iy) * nz + lo2 + iz], cnt);
        }
      }
    }
    __syncthreads();
  }
  if (stats) {
    wave_stats(stats, (unsigned long long)upd, valid ? 1ull : 0ull, hit ? 1ull : 0ull);
    for (int o = 32; o > 0; o >>= 1) nflush += __shfl_down(nflush, o, 64);
    if (l == 0 && nflush) atomicAdd(&stats[6], nflush);
    if (tid == 0) {
      if (nround_lds) atomicAdd(&stats[4], nround_lds);
      if (nround_direct) atomicAdd(&stats[5], nround_direct);
    }
  }
}

// Timing-only probes (wrong results, DMF_FUSE_VARIANT >= 94): 94 = setup only,
// 95 = setup + register-only DDA walk (no LDS, no barriers, no atomics).
template <int kMode>
__global__ __launch_bounds__(256) void k_fuse_probe(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                                    const PoseX* __restrict__ poses, int dmin, int dmax, int tiles_x,
                                                    int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                    unsigned long long* __restrict__ stats) {
  stats = stat_slot(stats);
  int r, c;
  tile_pixel(blockIdx.x, tiles_x, r, c);
  Ray R;
  bool valid;
  const int upd = pixel_ray(g, cam, depth, poses, blockIdx.y, r, c, dmin, dmax, R, valid);
  uint64_t T0 = R.T[0], T1 = R.T[1], T2 = R.T[2];
  int lin = R.lin;
  if (kMode == 1) {
    for (int k = 1; k < R.left; ++k) {
      bool s0, s1, s2;
      dda_pick(T0, T1, T2, R.In[0], R.In[1], R.In[2], s0, s1, s2);
      lin += s2 ? R.dl[2] : (s1 ? R.dl[1] : R.dl[0]);
    }
  }
  if (lin == -12345 && T0 == 7) hits[0] = 1;  // keep the walk alive
  if (stats) wave_stats(stats, (unsigned long long)upd, valid ? 1ull : 0ull, 0ull);
}

// Kernel variant: DMF_FUSE_VARIANT=<n> selects a (round length, LDS box, flush)
// instantiation for A/B measurements; 1 = one atomic per update (k_fuse_direct).
static int fuse_variant() {
  static const int v = [] {
    const char* e = getenv("DMF_FUSE_VARIANT");
    return e ? atoi(e) : 0;
  }();
  return v;
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
  const Geom g = v->geom();
  unsigned long long* st = nullptr;
  if (d_stats) DMF_TRY(stats_begin(v, &st));
#define DMF_FUSE_LAUNCH(K)                                                                                     \
  hipLaunchKernelGGL(K, grid, dim3(256), 0, v->stream, g, cp, d_depth, tab, prm->dmin_mm, prm->dmax_mm, tx, d_hits, \
                     d_misses, st)
  switch (fuse_variant()) {
    case 1: DMF_FUSE_LAUNCH(k_fuse_direct); break;
    case 2: DMF_FUSE_LAUNCH((k_fuse_lds<8, 8192, 0>)); break;
    case 3: DMF_FUSE_LAUNCH((k_fuse_lds<8, 8192, 1>)); break;
    case 4: DMF_FUSE_LAUNCH((k_fuse_lds<8, 8192, 2>)); break;
    case 9: DMF_FUSE_LAUNCH((k_fuse_lds<8, 8192, 1, true, false>)); break;
    case 10: DMF_FUSE_LAUNCH((k_fuse_lds<8, 8192, 1, false, true>)); break;
    case 11: DMF_FUSE_LAUNCH((k_fuse_lds<8, 8192, 1, true, true>)); break;
    case 12: DMF_FUSE_LAUNCH((k_fuse_lds<8, 8192, 1, true, false, true>)); break;
    case 13: DMF_FUSE_LAUNCH((k_fuse_lds<16, 8192, 1, true, false, true>)); break;
    case 14: DMF_FUSE_LAUNCH((k_fuse_lds<24, 12288, 1, true, false, true>)); break;
    case 15: DMF_FUSE_LAUNCH((k_fuse_lds<12, 8192, 1, true, false, true>)); break;
    case 16: DMF_FUSE_LAUNCH((k_fuse_lean<8, 8192>)); break;
    case 17: DMF_FUSE_LAUNCH((k_fuse_lean<12, 8192>)); break;
    case 18: DMF_FUSE_LAUNCH((k_fuse_lean<16, 12288>)); break;
    case 19: DMF_FUSE_LAUNCH((k_fuse_lean<6, 6144>)); break;
    case 20: DMF_FUSE_LAUNCH((k_fuse_v2<16, 8192>)); break;
    case 21: DMF_FUSE_LAUNCH((k_fuse_v2<12, 8192>)); break;
    case 22: DMF_FUSE_LAUNCH((k_fuse_v2<16, 12288>)); break;
    case 23: DMF_FUSE_LAUNCH((k_fuse_v2<8, 6144>)); break;
    case 24: DMF_FUSE_LAUNCH((k_fuse_v2<8, 4096>)); break;
    case 25: DMF_FUSE_LAUNCH((k_fuse_v2<6, 4096>)); break;
    case 26: DMF_FUSE_LAUNCH((k_fuse_v2<10, 6144>)); break;
    case 27: DMF_FUSE_LAUNCH((k_fuse_v2<6, 3072>)); break;
    case 28: DMF_FUSE_LAUNCH((k_fuse_v2<8, 5120>)); break;
    case 94: DMF_FUSE_LAUNCH((k_fuse_probe<0>)); break;
    case 95: DMF_FUSE_LAUNCH((k_fuse_probe<1>)); break;
    // timing-only ablations (wrong results): 91 no flush atomics, 92 no LDS atomics, 93 neither
    case 91: DMF_FUSE_LAUNCH((k_fuse_lds<16, 8192, 1, true, false, true, 1>)); break;
    case 92: DMF_FUSE_LAUNCH((k_fuse_lds<16, 8192, 1, true, false, true, 2>)); break;
    case 93: DMF_FUSE_LAUNCH((k_fuse_lds<16, 8192, 1, true, false, true, 3>)); break;
    case 5: DMF_FUSE_LAUNCH((k_fuse_lds<12, 8192, 2>)); break;
    case 6: DMF_FUSE_LAUNCH((k_fuse_lds<6, 6144, 2>)); break;
    case 7: DMF_FUSE_LAUNCH((k_fuse_lds<16, 12288, 2>)); break;
    case 8: DMF_FUSE_LAUNCH((k_fuse_lds<10, 10240, 2>)); break;
    default: DMF_FUSE_LAUNCH((k_fuse_v2<10, 6144>)); break;
  }
#undef DMF_FUSE_LAUNCH
  DMF_LAUNCH_CHECK();
  if (d_stats) DMF_TRY(stats_end(v, st, d_stats, kStatWidth));
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
  DMF_TRY(scratch(v, kScOut2, sizeof(uint64_t) * 8, &ds));
  DMF_HIP(hipMemcpyAsync(dd, depth, sizeof(uint16_t) * HW * P, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dp, poses, sizeof(float) * 12 * P, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dh, hits, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dm, misses, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemsetAsync(ds, 0, sizeof(uint64_t) * 8, v->stream));
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
