// dmf_trace.hip — RayTracingEngine (RayTracingEngine.hpp:27-564) on gfx950.
//
//  * reverse visibility (reverseRayTraceFast :136-226, reverseRayTrace :45-134):
//    one lane per (occupied voxel, pose), the reference 1 mm march toward the
//    camera over the N-bit occupancy mask; results are per-pose ballot bitmasks in
//    occupied_cells_ order, compacted order-preservingly into the good lists.
//  * forward depth-plane march (rayTrace* :229-494): one lane per lattice pixel,
//    first occupied sample per pixel; list outputs are ordered by the reference
//    loop key (z_depth, r, c) through a per-voxel atomicMin + radix sort.
//  * z-buffer splat rayTraceVolume (:498-564) and the willCollide segment march
//    (tests/CameraPathGen.cpp:128-156).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include <rocprim/rocprim.hpp>

#include "dmf_host.hpp"

namespace dmf {

// Register budgets of the march kernels: DMF_EXP_REV_WAVES / DMF_EXP_FWD_WAVES = n keeps their
// registers for n waves per SIMD (experiment builds override them)
// k_reverse_x at 6 waves per SIMD (round 6: the next sample computed while a sample's loads are
// in flight needs 4 more VGPRs; at 7 waves 2 spill: 4.49-4.51 ms at 6 waves vs 4.56 at 7 with
// the spill and 4.54-4.56 without the precompute at 7; round 5: 7 waves, 72
// VGPRs, 5.19 vs 5.21 ms at 6; 8 waves spilled and lost)
#if !defined(DMF_EXP_REV_WAVES)
#define DMF_EXP_REV_WAVES 6
#endif
#define DMF_REV_OCC __attribute__((amdgpu_waves_per_eu(DMF_EXP_REV_WAVES)))
// The queue marches' empty-space jumps: 0 (default) = the target is computed from the cube's
// faces moved in by Geom::jmarg and needs no check (round 6: 5.19 -> 4.77 ms per 128 poses,
// samples 937M -> 649M, DESIGN.md §5.5, profiles/r06y); 1 = the landing sample is evaluated and
// checked against the cube before the jump is taken (experiment builds)
#ifndef DMF_REV_VERIFY_JUMPS
#define DMF_REV_VERIFY_JUMPS 0
#endif
// The forward marches' jumps: 0 (default) = the line's point at the landing is checked against
// the cube shrunk by twice the rounding margin, and the entry jump's target is taken as computed
// (round 6: 6.16 -> 5.51 ms per 128 poses, samples 1.10G -> 0.77G, DESIGN.md §5.6,
// profiles/r06z); 1 = the landing sample is evaluated and checked (experiment builds)
#ifndef DMF_FWD_VERIFY_JUMPS
#define DMF_FWD_VERIFY_JUMPS 0
#endif
// The reverse march computes sample s + 1 while sample s's occupancy and distance loads are in
// flight (used when the step is a plain step; a jump or the centroid's cell recomputes): 1 (the
// default, round 6); 0 = one sample computed per step (experiment builds)
#ifndef DMF_EXP_REV_PRECOMP
#define DMF_EXP_REV_PRECOMP 1
#endif
#if defined(DMF_EXP_FWD_WAVES)
#define DMF_FWD_OCC __attribute__((amdgpu_waves_per_eu(DMF_EXP_FWD_WAVES)))
#else
#define DMF_FWD_OCC
#endif
#if defined(DMF_EXP_FWDQ_WAVES)
#define DMF_FWDQ_OCC __attribute__((amdgpu_waves_per_eu(DMF_EXP_FWDQ_WAVES)))
#else
#define DMF_FWDQ_OCC
#endif

struct EnumList {
  const float* axes;  // xs | ys | zs (float-accumulated, RayTracingEngine.hpp:54-56)
  int32_t nax[3];
  const uint32_t* list;  // occupied enumeration indices (i*ny+j)*nz+k, enumeration order
};

__device__ inline void wave_add_u64(unsigned long long* dst, unsigned long long x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
  if ((threadIdx.x & 63) == 0 && x) atomicAdd(dst, x);
}

// One sample of the reverse march: pt = c + (v * (float)depth) / 1000.0f per axis
// (Eigen evaluates the double depth as float; RayTracingEngine.hpp:82, :173).
__device__ inline void march_sample(const float cen[3], const float v[3], int depth, float p[3]) {
  const float fd = (float)depth;
  p[0] = cen[0] + div_rn(v[0] * fd, 1000.0f, 1.0f / 1000.0f);
  p[1] = cen[1] + div_rn(v[1] * fd, 1000.0f, 1.0f / 1000.0f);
  p[2] = cen[2] + div_rn(v[2] * fd, 1000.0f, 1.0f / 1000.0f);
}

// The reverse 1 mm march (RayTracingEngine.hpp:81-103 / :172-200).  Returns true if
// an occupied voxel other than the centroid's is hit before leaving the volume.
// `capped` reports a march that never left (v == 0 or NaN: the reference loops
// forever there) — treated as occluded and counted as a hazard.
//
// kSkip: empty-space skipping over 8^3 bricks, exact.  Each sample coordinate is a
// monotone function of the step index (RN(v*fd), /1000 and + cen are monotone), so
// if samples s and j both lie inside one empty brick and inside the volume, every
// sample between them does too: none can hit an occupied cell, leave the volume or
// be the centroid cell (an occupied cell).  j is estimated from the brick faces and
// then verified by evaluating sample j exactly; on failure the march steps normally.
template <bool kSkip>
__device__ inline bool reverse_march(const Geom& g, const DevVol& vd, const float cen[3], const float v[3], int cx,
                                     int cy, int cz, int depth0, int max_steps, int64_t& samples, bool& capped) {
  capped = false;
  float rv[3] = {0.f, 0.f, 0.f};  // 1000 / v (estimate only)
  if (kSkip) {
#pragma unroll
    for (int a = 0; a < 3; ++a) rv[a] = v[a] != 0.0f ? 1000.0f / v[a] : 0.0f;
  }
  uint32_t known_full = 0xffffffffu;  // last brick found occupied (or not skippable)
  for (int s = 0; s < max_steps; ++s) {
    float p[3];
    march_sample(cen, v, depth0 + s, p);
    ++samples;
    if (!valid_points(g, p[0], p[1], p[2])) return false;
    const int a = bin_axis(g, 0, p[0]), b = bin_axis(g, 1, p[1]), c = bin_axis(g, 2, p[2]);
    if (a == cx && b == cy && c == cz) continue;  // hash == centroid_hash
    if (!valid_coords(g, a, b, c)) return false;
    if (occ_test(vd.occ, occ_bit(g, a, b, c))) return true;
    if (kSkip) {
      const uint32_t bl = ((uint32_t)(a >> vd.bsh) * (uint32_t)vd.nb[1] + (uint32_t)(b >> vd.bsh)) *
                              (uint32_t)vd.nb[2] + (uint32_t)(c >> vd.bsh);
      if (bl == known_full) continue;
      if (((vd.brick[bl >> 5] >> (bl & 31)) & 1u) == 0u) {
        // last depth still inside the brick along each moving axis (estimate)
        const int cell[3] = {a, b, c};
        float fdmax = 3.0e38f;
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
          if (v[ax] == 0.0f) continue;
          const int lo = (cell[ax] >> vd.bsh) << vd.bsh;
          const int hi = min(lo + (1 << vd.bsh), g.n[ax]);  // exclusive
          const float face = (float)(g.mn[ax] + (double)(v[ax] > 0.0f ? hi : lo) * g.dl[ax]);
          fdmax = fminf(fdmax, (face - cen[ax]) * rv[ax]);
        }
        const float jf = floorf(fdmax) - (float)depth0 - 2.0f;
        if (jf > (float)(s + 1) && jf < (float)max_steps) {
          const int j = (int)jf;
          float q[3];
          march_sample(cen, v, depth0 + j, q);
          ++samples;
          if (valid_points(g, q[0], q[1], q[2])) {
            const int qa = bin_axis(g, 0, q[0]), qb = bin_axis(g, 1, q[1]), qc = bin_axis(g, 2, q[2]);
            if ((qa >> vd.bsh) == (a >> vd.bsh) && (qb >> vd.bsh) == (b >> vd.bsh) &&
                (qc >> vd.bsh) == (c >> vd.bsh) && valid_coords(g, qa, qb, qc)) {
              s = j;  // samples s+1 .. j lie inside the empty brick
              continue;
            }
          }
        }
      }
      known_full = bl;  // occupied brick, or estimate failed: step through it
    }
  }
  capped = true;
  return true;
}

// kEnum = false: reverseRayTraceFast over occupied_cells_ (element = slot)
// kEnum = true : reverseRayTrace over the float-accumulated enumeration list
template <bool kEnum, bool kSkip>
__global__ __launch_bounds__(256) void k_reverse(Geom g, DevVol vd, CamP cam, const PoseX* __restrict__ poses,
                                                 int64_t nelem, EnumList el, int depth0, int max_steps, float dstar,
                                                 int viz, int normal_test, uint64_t* __restrict__ vis_mask,
                                                 uint64_t* __restrict__ good_mask, int64_t words,
                                                 unsigned long long* __restrict__ stats, int* __restrict__ found,
                                                 unsigned long long* __restrict__ hazards) {
  stats = stat_slot(stats);
  const int p = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool vis = false, good = false;
  int64_t samples = 0;
  if (e < nelem) {
    float cen[3];
    int64_t slot;
    if (!kEnum) {
      slot = e;
      const uint64_t h = vd.hash[e];
      const int xid = (int)(h >> 40), yid = (int)((h >> 20) & 0xFFFFF), zid = (int)(h & 0xFFFFF);
      // :151-153 x = xid*xdelta_ + xmin_ (float); :157 centroid = x + xdelta_/2.0 (float)
      const float x = (float)((double)xid * g.dl[0] + g.mn[0]);
      const float y = (float)((double)yid * g.dl[1] + g.mn[1]);
      const float z = (float)((double)zid * g.dl[2] + g.mn[2]);
      cen[0] = (float)((double)x + g.hdl[0]);
      cen[1] = (float)((double)y + g.hdl[1]);
      cen[2] = (float)((double)z + g.hdl[2]);
    } else {
      const uint32_t en = el.list[e];
      const uint32_t nyz = (uint32_t)el.nax[1] * (uint32_t)el.nax[2];
      const uint32_t i = en / nyz, j = (en / el.nax[2]) % el.nax[1], k = en % el.nax[2];
      const float x = el.axes[i], y = el.axes[el.nax[0] + j], z = el.axes[el.nax[0] + el.nax[1] + k];
      slot = vd.slot_of[lin_index(g, bin_axis(g, 0, x), bin_axis(g, 1, y), bin_axis(g, 2, z))];
      cen[0] = (float)((double)x + g.hdl[0]);
      cen[1] = (float)((double)y + g.hdl[1]);
      cen[2] = (float)((double)z + g.hdl[2]);
    }
    const PoseX& T = poses[p];
    float t[3];
    xform(T.i, cen[0], cen[1], cen[2], t);
    int r, c;
    if (deproject_valid(cam, t[0], t[1], t[2], r, c)) {
      const float d[3] = {T.f[3] - cen[0], T.f[7] - cen[1], T.f[11] - cen[2]};
      float v[3];
      normalized(d, v);
      bool capped;
      const bool collided = reverse_march<kSkip>(g, vd, cen, v, bin_axis(g, 0, cen[0]), bin_axis(g, 1, cen[1]),
                                          bin_axis(g, 2, cen[2]), depth0, max_steps, samples, capped);
      if (capped) atomicAdd(hazards, 1ull);
      if (!collided) {
        vis = true;
        const double zz = (double)t[2];
        if (zz >= kZMin && zz <= kZMax) {
          if (normal_test) {
            const int32_t a = vd.off[slot], b = vd.off[slot + 1];
            for (int32_t j = a; j < b; ++j) {
              const float4 n = vd.nrm[j];
              if (n.w != 0.0f && angle_ok(n.x, n.y, n.z, v, dstar)) { good = true; break; }
            }
          } else {
            good = true;
          }
        }
      }
    }
    if (viz) {
      if (vis) vd.view[slot] = 1;
      if (good) vd.good[slot] = 1;
    }
  }
  const uint64_t vb = __ballot(vis), gb = __ballot(good);
  const int64_t w = e >> 6;
  if ((threadIdx.x & 63) == 0 && w < words) {
    if (vis_mask) vis_mask[(int64_t)p * words + w] = vb;
    if (good_mask) good_mask[(int64_t)p * words + w] = gb;
    if (vb) atomicOr(&found[p], 1);
  }
  if (stats) {
    wave_add_u64(&stats[0], (unsigned long long)samples);
    wave_add_u64(&stats[1], (unsigned long long)(e < nelem ? 1 : 0));
  }
}

// ---- persistent reverse visibility (work queue per wave) -----------------------
// Same per-(voxel, pose) semantics as k_reverse<kEnum, true>; the march lengths of
// neighbouring voxels differ by orders of magnitude (outside the frustum: 0 samples,
// occluded: tens, visible: hundreds), so one lane per voxel leaves most lanes of a
// wave idle.  Here each wave owns kItems consecutive voxels of one pose and keeps
// its lanes busy: a lane that finishes records its result bits in LDS and takes the
// next voxel; refills run when at least kRefill lanes are idle (the setup is
// divergent code, so it is batched).
struct RevLane {
  float cen[3], v[3], rv[3];
  uint32_t cob;         // occupancy bit of the centroid's cell (0xffffffff: outside the grid)
  int s;                // next sample index
  uint32_t known_full;  // last brick found occupied / not skippable
  int item;             // local item index, -1 = idle
  int32_t slot;
  float tz;             // camera-frame z of the centroid (z-range test)
  uint32_t occi, occw;  // cached occupancy word
#if DMF_EXP_REV_PRECOMP
  float pn[3];          // sample pns, computed ahead
  int pns;
#endif
};

__device__ inline bool valid_points_f(const Geom& g, const float p[3]) {
  // one combined mask (no per-axis branches)
  return (p[0] >= g.vlo[0]) & (p[0] <= g.vhi[0]) & (p[1] >= g.vlo[1]) & (p[1] <= g.vhi[1]) & (p[2] >= g.vlo[2]) &
         (p[2] <= g.vhi[2]);
}

// getVoxel of a point inside the volume in the reference's double arithmetic (bin_axis).
// (The certified float bins of dmf_geom.hpp bin_axis_f, exact by tools/binning_selftest.cpp,
// measured SLOWER in the reverse march: 8.35 vs 7.57 ms per 128-pose batch -- gfx950 runs
// the fp64 add / mul / floor / converts at the non-packed fp32 rate)
__device__ inline void bin_point(const Geom& g, const float p[3], int& a, int& b, int& c) {
  a = bin_axis(g, 0, p[0]);
  b = bin_axis(g, 1, p[1]);
  c = bin_axis(g, 2, p[2]);
}

// Diagnostic build (DMF_EXP_STATS): sample categories into stats[2..12]
#if defined(DMF_EXP_STATS)
#define DMF_RS(i, x) (rst[(i) - 2] += (unsigned long long)(x))
#else
#define DMF_RS(i, x) ((void)0)
#endif
constexpr int kRevStatN = 11;

// One sample of the reverse march (RayTracingEngine.hpp:172-200): 0 = continue,
// 1 = collided, 2 = left the volume (visible), 3 = capped (collided, hazard).
//
// validPoints (x > min and x < max in double) is the exact float test
// vlo <= x <= vhi.  Empty-space skipping: the brick distance field d gives an empty
// cube of bricks of radius d - 1 around the current brick; every sample coordinate is
// a monotone function of the step index, so if samples s and j both lie in that cube
// (and inside the volume) so does every sample between them — none can hit an
// occupied cell, the centroid's cell (occupied) or leave the volume.  j is computed from the
// cube's faces moved in by Geom::jmarg, which puts sample j inside the cube without evaluating
// it (DMF_REV_VERIFY_JUMPS = 0, the default), or estimated from the faces themselves and
// verified by evaluating sample j exactly (= 1).
__device__ inline int rev_step(const Geom& g, const DevVol& vd, RevLane& L, int depth0, int max_steps,
                               int64_t& samples, unsigned long long* rst) {
  (void)rst;
  if (L.s >= max_steps) return 3;
  float p[3];
#if DMF_EXP_REV_PRECOMP
  // sample s was computed by the previous step while that step's loads were in flight
  if (L.pns == L.s) {
    p[0] = L.pn[0];
    p[1] = L.pn[1];
    p[2] = L.pn[2];
  } else {
    march_sample(L.cen, L.v, depth0 + L.s, p);
  }
#else
  march_sample(L.cen, L.v, depth0 + L.s, p);
#endif
  ++samples;
  int a, b, c;
  if (!valid_points_f(g, p)) return 2;
  bin_point(g, p, a, b, c);
  // (the reference tests the centroid's hash before validCoords; the centroid's cell is inside
  // the grid, so testing validCoords first and then the cell by its occupancy bit, which is
  // one-to-one on the grid, takes the same branches with one compare instead of three)
  if (!valid_coords(g, a, b, c)) return 2;
  const uint32_t ob = occ_bit(g, a, b, c);
  if (ob == L.cob) { DMF_RS(2, 1); ++L.s; return 0; }
  // the brick's distance is loaded together with the occupancy word, before the occupancy test:
  // one memory latency per empty sample instead of two (round 6: 4.67 -> 4.56 ms per 128 poses,
  // DESIGN.md §5.5; the load is wasted on occupied samples and in known-full bricks)
  const int ba = a >> vd.bsh, bb = b >> vd.bsh, bc = c >> vd.bsh;
  const uint32_t bl = ((uint32_t)ba * (uint32_t)vd.nb[1] + (uint32_t)bb) * (uint32_t)vd.nb[2] + (uint32_t)bc;
  const int dpre = vd.bdist[bl];
  if ((ob >> 5) != L.occi) { L.occi = ob >> 5; L.occw = vd.occ[L.occi]; }
#if DMF_EXP_REV_PRECOMP
  march_sample(L.cen, L.v, depth0 + L.s + 1, L.pn);  // the next sample, while the loads are in flight
  L.pns = L.s + 1;
#endif
  if ((L.occw >> (ob & 31)) & 1u) return 1;
  if (bl != L.known_full) {
    const int d = dpre;
#if !DMF_REV_VERIFY_JUMPS
    if (d > 0) {
      // the jump target from the cube's exit faces moved toward the sample by g.jmarg: no
      // sample of the jump is evaluated here; the target j is the next one marched, and the
      // samples s+1 .. j-1 lie inside the empty cube (the moved face is
      // farther inside than every rounding of the face, the samples and their bins, so sample
      // j is inside the cube; the samples before it follow by monotonicity)
      const int R = d - 1;  // bricks within R of this one are empty
      const int bx[3] = {ba, bb, bc};
      float fdmax = 3.0e38f;
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        if (L.v[ax] == 0.0f) continue;
        const int cf = L.v[ax] > 0.0f ? min((bx[ax] + R + 1) << vd.bsh, g.n[ax]) : max(bx[ax] - R, 0) << vd.bsh;
        const float face = (float)(g.mn[ax] + (double)cf * g.dl[ax]);
        const float fin = L.v[ax] > 0.0f ? face - g.jmarg[ax] : face + g.jmarg[ax];
        fdmax = fminf(fdmax, (fin - L.cen[ax]) * L.rv[ax]);
      }
      const float jf = floorf(fdmax) - (float)depth0 - 2.0f;
      if (jf > (float)(L.s + 1) && jf < (float)max_steps && jf < 4194304.0f) {
        DMF_RS(4, 1);
        DMF_RS(5, 1);
        DMF_RS(6, (int)jf - L.s);
        L.s = (int)jf;
        return 0;
      }
    } else {
      DMF_RS(12, 1);
    }
#else
    if (d > 0) {
      const int R = d - 1;  // bricks within R of this one are empty
      const int bx[3] = {ba, bb, bc};
      int clo[3], chi[3];   // cell range of the empty cube, [clo, chi)
      float fdmax = 3.0e38f;
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        clo[ax] = max(bx[ax] - R, 0) << vd.bsh;
        chi[ax] = min((bx[ax] + R + 1) << vd.bsh, g.n[ax]);
        if (L.v[ax] == 0.0f) continue;
        const float face = (float)(g.mn[ax] + (double)(L.v[ax] > 0.0f ? chi[ax] : clo[ax]) * g.dl[ax]);
        fdmax = fminf(fdmax, (face - L.cen[ax]) * L.rv[ax]);
      }
      const float jf = floorf(fdmax) - (float)depth0 - 2.0f;
      if (jf > (float)(L.s + 1) && jf < (float)max_steps) {
        const int j = (int)jf;
        DMF_RS(4, 1);
        float q[3];
        march_sample(L.cen, L.v, depth0 + j, q);
        ++samples;
        if (valid_points_f(g, q)) {
          int qa, qb, qc;
          bin_point(g, q, qa, qb, qc);
          if (qa >= clo[0] && qa < chi[0] && qb >= clo[1] && qb < chi[1] && qc >= clo[2] && qc < chi[2]) {
            DMF_RS(5, 1);
            DMF_RS(6, j - L.s);
            L.s = j + 1;  // samples s+1 .. j lie inside the empty cube
            return 0;
          }
        }
      }
    } else {
      DMF_RS(12, 1);
    }
#endif
    L.known_full = bl;  // occupied brick, or the jump failed: step through it
  }
  DMF_RS(3, 1);
  ++L.s;
  return 0;
}

// kOrder (reverseRayTraceFast only): the wave's items are the occupied voxels in SPATIAL
// order (order[k] = the slot of the k-th voxel along a 3D Morton curve of its cell,
// ensure_spatial_order), so that a wave's 64 lanes start in neighbouring voxels: their rays
// toward the camera are near-parallel, cross the same bricks and end alike (all occluded or
// all visible).  The result bits are then in item order: vis_mask / good_mask receive
// item-ordered words, which k_mask_to_slots permutes into occupied_cells_ order (the output
// is a per-slot bitmask, so the processing order is free).
// One wave's work queue over items [base, base + nitems) of pose T: result bits into the
// wave's LDS words lvis / lgood (item-indexed, zeroed by the caller); returns the lane's "some
// item visible".  Shared by k_reverse_q (a grid of (item chunk, pose)) and k_reverse_x (per-XCD
// unit queues).
template <bool kEnum, int kItems, int kRefill, int kBurst, bool kOrder>
__device__ inline bool rev_wave(const Geom& g, const DevVol& vd, const CamP& cam, const PoseX& T, const EnumList& el,
                                const uint32_t* __restrict__ order, int64_t base, int nitems, int depth0,
                                int max_steps, float dstar, int viz, int normal_test, uint32_t* lvis, uint32_t* lgood,
                                int64_t& samples, int64_t& rays, unsigned long long& ncap, unsigned long long* rst) {
  [[maybe_unused]] const int l = threadIdx.x & 63;  // (diagnostic-build statistics)
  bool any_vis = false;
  RevLane L;
  L.item = -1;
  int next = 0;  // wave-uniform queue head
  while (true) {
    const uint64_t idle = __builtin_amdgcn_ballot_w64(L.item < 0);
    const int nidle = __builtin_popcountll(idle);
    if (next < nitems && (nidle >= kRefill || nidle == 64)) {
      if (L.item < 0) {
        const int it = next + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        if (it < nitems) {
          const int64_t e = base + it;
          ++rays;
          float cen[3];
          int32_t slot;
          if (!kEnum) {
            slot = kOrder ? (int32_t)order[e] : (int32_t)e;
            const uint64_t h = vd.hash[slot];
            const int xid = (int)(h >> 40), yid = (int)((h >> 20) & 0xFFFFF), zid = (int)(h & 0xFFFFF);
            const float x = (float)((double)xid * g.dl[0] + g.mn[0]);
            const float y = (float)((double)yid * g.dl[1] + g.mn[1]);
            const float z = (float)((double)zid * g.dl[2] + g.mn[2]);
            cen[0] = (float)((double)x + g.hdl[0]);
            cen[1] = (float)((double)y + g.hdl[1]);
            cen[2] = (float)((double)z + g.hdl[2]);
          } else {
            const uint32_t en = el.list[e];
            const uint32_t nyz = (uint32_t)el.nax[1] * (uint32_t)el.nax[2];
            const uint32_t i = en / nyz, j = (en / el.nax[2]) % el.nax[1], k = en % el.nax[2];
            const float x = el.axes[i], y = el.axes[el.nax[0] + j], z = el.axes[el.nax[0] + el.nax[1] + k];
            slot = vd.slot_of[lin_index(g, bin_axis(g, 0, x), bin_axis(g, 1, y), bin_axis(g, 2, z))];
            cen[0] = (float)((double)x + g.hdl[0]);
            cen[1] = (float)((double)y + g.hdl[1]);
            cen[2] = (float)((double)z + g.hdl[2]);
          }
          float t[3];
          xform(T.i, cen[0], cen[1], cen[2], t);
          int r, c;
          if (deproject_valid(cam, t[0], t[1], t[2], r, c)) {
            const float d[3] = {T.f[3] - cen[0], T.f[7] - cen[1], T.f[11] - cen[2]};
            normalized(d, L.v);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
              L.cen[a] = cen[a];
              L.rv[a] = L.v[a] != 0.0f ? 1000.0f / L.v[a] : 0.0f;
            }
            {
              const int cx = bin_axis(g, 0, cen[0]), cy = bin_axis(g, 1, cen[1]), cz = bin_axis(g, 2, cen[2]);
              L.cob = valid_coords(g, cx, cy, cz) ? occ_bit(g, cx, cy, cz) : 0xffffffffu;
            }
            L.s = 0;
            L.known_full = 0xffffffffu;
            L.occi = 0xffffffffu;
#if DMF_EXP_REV_PRECOMP
            L.pns = -1;
#endif
            L.item = it;
            L.slot = slot;
            L.tz = t[2];
            DMF_RS(9, 1);
          }
        }
      }
      next += nidle;
    }
    if (__builtin_amdgcn_ballot_w64(L.item >= 0) == 0) {
      if (next >= nitems) break;
      continue;
    }
    // march: up to kBurst samples per busy lane
    int st = 0;
#pragma unroll 1
    for (int b = 0; b < kBurst; ++b) {
      DMF_RS(10, l == 0);
      DMF_RS(11, L.item >= 0 && st == 0);
      if (L.item >= 0 && st == 0) st = rev_step(g, vd, L, depth0, max_steps, samples, rst);
      if (__builtin_amdgcn_ballot_w64(L.item >= 0 && st == 0) == 0) break;
    }
    if (L.item >= 0 && st != 0) {
      DMF_RS(7, st == 1);
      DMF_RS(8, st == 2);
      if (st == 3) ++ncap;
      if (st == 2) {
        any_vis = true;
        bool good = false;
        const double zz = (double)L.tz;
        if (zz >= kZMin && zz <= kZMax) {
          if (normal_test) {
            const int32_t a = vd.off[L.slot], b = vd.off[L.slot + 1];
            for (int32_t j = a; j < b; ++j) {
              const float4 n = vd.nrm[j];
              if (n.w != 0.0f && angle_ok(n.x, n.y, n.z, L.v, dstar)) { good = true; break; }
            }
          } else {
            good = true;
          }
        }
        atomicOr(&lvis[L.item >> 5], 1u << (L.item & 31));
        if (good) atomicOr(&lgood[L.item >> 5], 1u << (L.item & 31));
        if (viz) {
          vd.view[L.slot] = 1;
          if (good) vd.good[L.slot] = 1;
        }
      }
      L.item = -1;
    }
  }
  return any_vis;
}

template <bool kEnum, int kItems, int kRefill, int kBurst, bool kOrder = false>
__global__ __launch_bounds__(256) void k_reverse_q(Geom g, DevVol vd, CamP cam, const PoseX* __restrict__ poses,
                                                   int64_t nelem, EnumList el, const uint32_t* __restrict__ order,
                                                   int depth0, int max_steps, float dstar, int viz, int normal_test,
                                                   uint64_t* __restrict__ vis_mask, uint64_t* __restrict__ good_mask,
                                                   int64_t words, unsigned long long* __restrict__ stats,
                                                   int* __restrict__ found, unsigned long long* __restrict__ hazards) {
  static_assert(kItems % 64 == 0, "whole mask words per wave");
  static_assert(!(kEnum && kOrder), "spatial order: occupied_cells_ items only");
  stats = stat_slot(stats);
  __shared__ uint32_t lvis[4][kItems / 32], lgood[4][kItems / 32];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int i = l; i < kItems / 32; i += 64) { lvis[w][i] = 0; lgood[w][i] = 0; }
  const int p = blockIdx.y;
  const int64_t base = ((int64_t)blockIdx.x * 4 + w) * kItems;
  const int nitems = (int)max<int64_t>(0, min<int64_t>(kItems, nelem - base));
  int64_t samples = 0, rays = 0;
  unsigned long long ncap = 0;
  unsigned long long rst[kRevStatN] = {};
  __syncthreads();
  const bool any_vis = rev_wave<kEnum, kItems, kRefill, kBurst, kOrder>(
      g, vd, cam, poses[p], el, order, base, nitems, depth0, max_steps, dstar, viz, normal_test, lvis[w], lgood[w],
      samples, rays, ncap, rst);
  __syncthreads();
  const int64_t w0 = base >> 6;
  for (int i = l; i < kItems / 64; i += 64) {
    if (w0 + i < words) {
      const uint64_t vb = (uint64_t)lvis[w][2 * i] | ((uint64_t)lvis[w][2 * i + 1] << 32);
      const uint64_t gb = (uint64_t)lgood[w][2 * i] | ((uint64_t)lgood[w][2 * i + 1] << 32);
      if (vis_mask) vis_mask[(int64_t)p * words + w0 + i] = vb;
      if (good_mask) good_mask[(int64_t)p * words + w0 + i] = gb;
    }
  }
  if (__builtin_amdgcn_ballot_w64(any_vis) != 0 && l == 0) atomicOr(&found[p], 1);
  for (int o = 32; o > 0; o >>= 1) ncap += __shfl_down(ncap, o, 64);
  if (l == 0 && ncap) atomicAdd(hazards, ncap);
  if (stats) {
    wave_add_u64(&stats[0], (unsigned long long)samples);
    wave_add_u64(&stats[1], (unsigned long long)rays);
#if defined(DMF_EXP_STATS)
#pragma unroll
    for (int i = 0; i < kRevStatN; ++i) wave_add_u64(&stats[2 + i], rst[i]);
#endif
  }
}

// reverseRayTraceFast with per-XCD work queues (spatial order only).  A unit is one wave's
// 64 consecutive items of the Morton order for one pose.  The Morton range is cut into 8
// contiguous eighths, one queue per eighth, units pose-major inside it; workgroup b serves the
// queue of its XCD group b % 8 (blocks b and b + 8 share an XCD's L2 under the observed
// round-robin placement -- a speed choice only, any placement gives the same bits), so the
// waves resident on one XCD march rays from one region of the surface toward one camera at a
// time and share its L2 lines of the occupancy bitmask and distance field.  A wave whose queue
// is empty takes units from the next groups' queues (work stealing at the tail), so uneven
// march work per eighth cannot idle an XCD; every wave exits once all 8 queues are drained.
// heads[8]: the queues' unit counters (zeroed before the launch).
// kWg: a unit is the workgroup's 4 consecutive waves' worth of items (256, as one workgroup of
// k_reverse_q), taken by the workgroup together: its waves share the CU's L1 lines as in
// k_reverse_q, at the price of a barrier per unit; else one wave's 64 items per unit.
template <int kItems, int kRefill, int kBurst, bool kWg>
__global__ __launch_bounds__(256) DMF_REV_OCC void k_reverse_x(Geom g, DevVol vd, CamP cam, const PoseX* __restrict__ poses, int P,
                                                   int64_t nelem, const uint32_t* __restrict__ order, int depth0,
                                                   int max_steps, float dstar, int viz, uint64_t* __restrict__ vis_mask,
                                                   uint64_t* __restrict__ good_mask, int64_t words,
                                                   unsigned int* __restrict__ heads,
                                                   unsigned long long* __restrict__ stats, int* __restrict__ found,
                                                   unsigned long long* __restrict__ hazards) {
  static_assert(kItems == 64, "one mask word per wave and unit");
  stats = stat_slot(stats);
  __shared__ uint32_t lvis[4][2], lgood[4][2];
  __shared__ uint32_t s_unit;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int grp = (int)(blockIdx.x & 7u);
  const EnumList el{};
  int64_t samples = 0, rays = 0;
  unsigned long long ncap = 0;
  unsigned long long rst[kRevStatN] = {};
  constexpr int kPer = kWg ? 4 : 1;  // mask words per unit
  const int64_t nwu = (words + kPer - 1) / kPer;
  for (int q = 0; q < 8; ++q) {
    const int gq = (grp + q) & 7;
    const int64_t c0 = nwu * gq / 8, nch = nwu * (gq + 1) / 8 - c0;
    const uint32_t nunits = (uint32_t)(nch * P);
    for (;;) {
      uint32_t u = 0;
      if (kWg) {
        if (threadIdx.x == 0) s_unit = atomicAdd(&heads[gq], 1u);
        __syncthreads();
        u = s_unit;
        __syncthreads();  // every wave has read it before the next unit's write
      } else {
        if (l == 0) u = atomicAdd(&heads[gq], 1u);
        u = (uint32_t)__builtin_amdgcn_readfirstlane((int)u);
      }
      if (u >= nunits) break;
      const int p = (int)(u / (uint32_t)nch);
      const int64_t c = (c0 + (int64_t)(u - (uint32_t)p * (uint32_t)nch)) * kPer + (kWg ? w : 0);
      if (l < 2) { lvis[w][l] = 0; lgood[w][l] = 0; }
      __builtin_amdgcn_wave_barrier();
      const int64_t base = c * kItems;
      const int nitems = (int)max<int64_t>(0, min<int64_t>(kItems, nelem - base));
      const bool any_vis = rev_wave<false, kItems, kRefill, kBurst, true>(
          g, vd, cam, poses[p], el, order, base, nitems, depth0, max_steps, dstar, viz, 1, lvis[w], lgood[w],
          samples, rays, ncap, rst);
      __builtin_amdgcn_wave_barrier();
      if (l == 0 && c < words) {
        const uint64_t vb = (uint64_t)lvis[w][0] | ((uint64_t)lvis[w][1] << 32);
        const uint64_t gb = (uint64_t)lgood[w][0] | ((uint64_t)lgood[w][1] << 32);
        if (vis_mask) vis_mask[(int64_t)p * words + c] = vb;
        if (good_mask) good_mask[(int64_t)p * words + c] = gb;
      }
      if (__builtin_amdgcn_ballot_w64(any_vis) != 0 && l == 0) atomicOr(&found[p], 1);
    }
  }
  for (int o = 32; o > 0; o >>= 1) ncap += __shfl_down(ncap, o, 64);
  if (l == 0 && ncap) atomicAdd(hazards, ncap);
  if (stats) {
    wave_add_u64(&stats[0], (unsigned long long)samples);
    wave_add_u64(&stats[1], (unsigned long long)rays);
#if defined(DMF_EXP_STATS)
#pragma unroll
    for (int i = 0; i < kRevStatN; ++i) wave_add_u64(&stats[2 + i], rst[i]);
#endif
  }
}

// Item-ordered result bits (k_reverse_q<*, kOrder>) -> occupied_cells_ order: one wave per
// output word of 64 slots, all P poses; lane l takes slot 64 w + l, whose item is rank[slot].
__global__ __launch_bounds__(256) void k_mask_to_slots(const uint64_t* __restrict__ vis_items,
                                                       const uint64_t* __restrict__ good_items,
                                                       const uint32_t* __restrict__ rank, int64_t V, int64_t words,
                                                       int P, uint64_t* __restrict__ vis, uint64_t* __restrict__ good) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int l = threadIdx.x & 63;
  if (w >= words) return;
  const int64_t s = w * 64 + l;
  const uint32_t k = s < V ? rank[s] : 0u;
  for (int p = 0; p < P; ++p) {
    const int64_t row = (int64_t)p * words;
    bool bv = false, bg = false;
    if (s < V) {
      bv = (vis_items[row + (k >> 6)] >> (k & 63)) & 1ull;
      bg = (good_items[row + (k >> 6)] >> (k & 63)) & 1ull;
    }
    const uint64_t mv = __builtin_amdgcn_ballot_w64(bv), mg = __builtin_amdgcn_ballot_w64(bg);
    if (l == 0) {
      vis[row + w] = mv;
      good[row + w] = mg;
    }
  }
}

// 3D Morton key of an occupied voxel (21 bits per axis; the hash holds 20) and the slot as value.
__device__ inline uint64_t morton_spread(uint64_t x) {
  x &= 0x1fffffull;
  x = (x | x << 32) & 0x1f00000000ffffull;
  x = (x | x << 16) & 0x1f0000ff0000ffull;
  x = (x | x << 8) & 0x100f00f00f00f00full;
  x = (x | x << 4) & 0x10c30c30c30c30c3ull;
  x = (x | x << 2) & 0x1249249249249249ull;
  return x;
}
__global__ void k_morton_keys(const uint64_t* __restrict__ hash, int64_t V, uint64_t* __restrict__ keys,
                              uint64_t* __restrict__ vals) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= V) return;
  const uint64_t h = hash[s];
  keys[s] = morton_spread(h >> 40) << 2 | morton_spread((h >> 20) & 0xFFFFF) << 1 | morton_spread(h & 0xFFFFF);
  vals[s] = (uint64_t)s;
}
__global__ void k_order_store(const uint64_t* __restrict__ vals, int64_t V, uint32_t* __restrict__ order,
                              uint32_t* __restrict__ rank) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= V) return;
  const uint32_t s = (uint32_t)vals[k];
  order[k] = s;
  rank[s] = (uint32_t)k;
}

// The occupied voxels in spatial (3D Morton) order, rebuilt after an integration changed them.
static int ensure_spatial_order(dmf_volume* v) {
  if (v->sorder_valid) return DMF_OK;
  const int64_t V = v->V;
  if (V > v->sorder_cap) {
    if (v->d_sorder) DMF_HIP(hipFree(v->d_sorder));
    v->d_sorder = nullptr;
    v->sorder_cap = 0;
    DMF_HIP(hipMalloc((void**)&v->d_sorder, sizeof(uint32_t) * 2 * (size_t)V));
    v->sorder_cap = V;
  }
  void *keys, *vals;
  DMF_TRY(scratch(v, kScOut2, sizeof(uint64_t) * (size_t)V, &keys));
  DMF_TRY(scratch(v, kScOut3, sizeof(uint64_t) * (size_t)V, &vals));
  const dim3 blk(256), grd((unsigned)((V + 255) / 256));
  hipLaunchKernelGGL(k_morton_keys, grd, blk, 0, v->stream, v->d_hash, V, (uint64_t*)keys, (uint64_t*)vals);
  DMF_LAUNCH_CHECK();
  DMF_TRY(sort_pairs_u64(v, (uint64_t*)keys, (uint64_t*)vals, (size_t)V, 63));
  hipLaunchKernelGGL(k_order_store, grd, blk, 0, v->stream, (const uint64_t*)vals, V, v->d_sorder,
                     v->d_sorder + v->sorder_cap);
  DMF_LAUNCH_CHECK();
  v->sorder_valid = true;
  return DMF_OK;
}

// ---- greedy set cover over per-pose good bitmasks (Algorithms.hpp:38-86) ---------
// The reference scans the remaining set ids in increasing order and keeps the
// strictly largest |set \ covered|; with sets as bitmasks over occupied slots that
// difference size is popcount(good[p] & ~covered).  One iteration = gain, pick,
// merge; every kernel returns at once after the stop condition.
struct CoverCtl {
  int done;
  int sel;
  int nsel;
};

__global__ __launch_bounds__(256) void k_cover_gain(const uint64_t* __restrict__ masks, int64_t words,
                                                    const uint64_t* __restrict__ covered,
                                                    const uint8_t* __restrict__ removed,
                                                    unsigned long long* __restrict__ gain,
                                                    const CoverCtl* __restrict__ ctl) {
  if (ctl->done) return;
  const int p = blockIdx.x;
  if (removed[p]) {
    if (threadIdx.x == 0) gain[p] = 0;
    return;
  }
  const uint64_t* m = masks + (int64_t)p * words;
  unsigned long long c = 0;
  for (int64_t w = threadIdx.x; w < words; w += blockDim.x) c += __popcll(m[w] & ~covered[w]);
  __shared__ unsigned long long part[4];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) gain[p] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(256) void k_cover_pick(const unsigned long long* __restrict__ gain, int P, int min_gain,
                                                    uint8_t* __restrict__ removed, int32_t* __restrict__ selected,
                                                    CoverCtl* __restrict__ ctl) {
  if (ctl->done) return;
  // argmax with ties to the smallest index: key = gain << 32 | (2^32 - 1 - p)
  unsigned long long best = 0;
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const unsigned long long k = (gain[p] << 32) | (unsigned long long)(0xffffffffu - (uint32_t)p);
    best = k > best ? k : best;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_down(best, o, 64);
    best = t > best ? t : best;
  }
  __shared__ unsigned long long part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) best = part[i] > best ? part[i] : best;
    const unsigned long long g = best >> 32;
    if (g == 0 || g < (unsigned long long)min_gain) {  // selected == -1, or max_points < 5
      ctl->done = 1;
    } else {
      const int p = (int)(0xffffffffu - (uint32_t)(best & 0xffffffffu));
      ctl->sel = p;
      selected[ctl->nsel++] = p;
      removed[p] = 1;
    }
  }
}

__global__ __launch_bounds__(256) void k_cover_merge(const uint64_t* __restrict__ masks, int64_t words,
                                                     uint64_t* __restrict__ covered, const CoverCtl* __restrict__ ctl) {
  if (ctl->done) return;
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w < words) covered[w] |= masks[(int64_t)ctl->sel * words + w];
}

static int greedy_cover(dmf_volume* v, const uint64_t* d_masks, int P, int64_t words, int min_gain,
                        int32_t* selected, int32_t* nselected) {
  if (P <= 0) { *nselected = 0; return DMF_OK; }
  void *cov, *aux;
  const size_t cov_bytes = sizeof(uint64_t) * (size_t)std::max<int64_t>(words, 1);
  DMF_TRY(scratch(v, kScTmp, cov_bytes, &cov));
  const size_t gain_off = 64, rem_off = gain_off + sizeof(unsigned long long) * P,
               sel_off = rem_off + ((size_t)P + 7) / 8 * 8;
  DMF_TRY(scratch(v, kScCount, sel_off + sizeof(int32_t) * P, &aux));
  CoverCtl* ctl = (CoverCtl*)aux;
  unsigned long long* gain = (unsigned long long*)((char*)aux + gain_off);
  uint8_t* removed = (uint8_t*)aux + rem_off;
  int32_t* sel = (int32_t*)((char*)aux + sel_off);
  DMF_HIP(hipMemsetAsync(cov, 0, cov_bytes, v->stream));
  DMF_HIP(hipMemsetAsync(aux, 0, sel_off, v->stream));
  const unsigned mb = (unsigned)((words + 255) / 256);
  for (int it = 0; it < P; it += 8) {
    for (int k = it; k < std::min(P, it + 8); ++k) {
      hipLaunchKernelGGL(k_cover_gain, dim3((unsigned)P), dim3(256), 0, v->stream, d_masks, words,
                         (const uint64_t*)cov, removed, gain, ctl);
      hipLaunchKernelGGL(k_cover_pick, dim3(1), dim3(256), 0, v->stream, gain, P, min_gain, removed, sel, ctl);
      if (mb) hipLaunchKernelGGL(k_cover_merge, dim3(mb), dim3(256), 0, v->stream, d_masks, words, (uint64_t*)cov, ctl);
    }
    DMF_LAUNCH_CHECK();
    CoverCtl h;
    DMF_HIP(hipMemcpyAsync(&h, ctl, sizeof(h), hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
    if (h.done) break;
  }
  CoverCtl h;
  DMF_HIP(hipMemcpyAsync(&h, ctl, sizeof(h), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  if (h.nsel) DMF_HIP(hipMemcpy(selected, sel, sizeof(int32_t) * h.nsel, hipMemcpyDeviceToHost));
  *nselected = h.nsel;
  return DMF_OK;
}

static int max_march_steps(const dmf_volume* v) {
  const double dx = v->xmax - v->xmin, dy = v->ymax - v->ymin, dz = v->zmax - v->zmin;
  const double diag_mm = std::sqrt(dx * dx + dy * dy + dz * dz) * 1000.0;
  const double s = std::ceil(diag_mm * 1.01) + 64;
  return s > 2e9 ? 2000000000 : (int)s;
}

// Runs k_reverse for P poses; masks land in scratch kScOut0 (vis | good).
static int run_reverse(dmf_volume* v, const dmf_camera* cam, const float* poses, int P, bool poses_on_device,
                       int viz, bool enumerate, uint64_t** d_vis, uint64_t** d_good, int64_t* words_out,
                       int64_t* nelem_out, std::vector<int>* found_h, uint64_t* d_stats) {
  DMF_TRY(require_constructed(v));
  DMF_TRY(check_camera(cam));
  if (P <= 0 || P > 65535) return fail(DMF_ERR_INVALID, "pose count %d out of range [1,65535]", P);
  if (enumerate) DMF_TRY(ensure_enumeration(v));
  PoseX* tab;
  DMF_TRY(pose_table(v, poses, P, poses_on_device, &tab));
  const int64_t nelem = enumerate ? v->nenum : v->V;
  const int64_t words = (nelem + 63) / 64;
  void *masks, *aux;
  DMF_TRY(scratch(v, kScOut0, sizeof(uint64_t) * (size_t)std::max<int64_t>(2 * P * words, 1), &masks));
  const size_t found_bytes = ((sizeof(int) * P + 7) / 8) * 8;
  DMF_TRY(scratch(v, kScHost2, found_bytes + 2 * sizeof(unsigned long long), &aux));
  int* found = (int*)aux;
  unsigned long long* hz = (unsigned long long*)((char*)aux + found_bytes);
  DMF_HIP(hipMemsetAsync(aux, 0, found_bytes + 2 * sizeof(unsigned long long), v->stream));
  uint64_t* vis = (uint64_t*)masks;
  uint64_t* good = vis + P * words;
  unsigned long long* st = nullptr;
  if (d_stats) DMF_TRY(stats_begin(v, &st));
  if (nelem > 0) {
    EnumList el{v->d_axes, {v->nax[0], v->nax[1], v->nax[2]}, v->d_enum};
    const dim3 grid((unsigned)((nelem + 255) / 256), (unsigned)P);
    const int depth0 = enumerate ? 1 : 50;  // :81 vs :172
    // DMF_KNOB_REVERSE_KERNEL (dmf_diag.h): 0 = default (the work-queue march with the brick
    // distance field, items in spatial order for reverseRayTraceFast, per-XCD unit queues),
    // 1 = lane per (voxel, pose), 2 = the same with brick skipping, 3 = the work queue in
    // occupied_cells_ order, 4 = per-XCD queues of per-wave units, 5 = the spatial-order work
    // queue on a (chunk, pose) grid (the default until round 5)
    const int64_t kr = v->knob[DMF_KNOB_REVERSE_KERNEL];
    // work-queue shape (items per wave, refill threshold, burst): 512 / 8 / 8 in enumeration
    // or insertion order; in spatial order smaller queues pay (neighbouring lanes agree, so
    // the per-wave tail is the cost): 64 / 8 / 16 measured 5.54 ms vs 5.94 at 128 / 8 / 16 and
    // 6.51 at 512 / 8 / 8 (profiles/r04/reverse_queue_sweep.json)
    constexpr int kRevItems = 512, kRevRefill = 8, kRevBurst = 8;
#if defined(DMF_EXP_REV_ITEMS)  // experiment builds: the spatial-order queue's shape
    constexpr int kSpItems = DMF_EXP_REV_ITEMS, kSpRefill = DMF_EXP_REV_REFILL, kSpBurst = DMF_EXP_REV_BURST;
#else
    // (round 5, per-XCD queues: burst 32 5.24-5.25 ms vs 16 5.29-5.32, 24 5.25-5.26, 8 5.39-5.41;
    // refill 4 / 12 / 16 at burst 16 within +-0.5 %: profiles/r05j/.  Round 6, after the
    // unchecked jumps: burst 64 4.67-4.69 ms vs 32 4.71-4.72, 48 4.71-4.74, 96 4.68-4.70, 128 4.68;
    // refill 4 / 16 at burst 32 +-0.2 %: profiles/r06ab/, r06ac/)
    constexpr int kSpItems = 64, kSpRefill = 8, kSpBurst = 64;
#endif
    const dim3 gridq((unsigned)((nelem + 4 * kRevItems - 1) / (4 * kRevItems)), (unsigned)P);
    const dim3 gridqs((unsigned)((nelem + 4 * kSpItems - 1) / (4 * kSpItems)), (unsigned)P);
    const Geom g = v->geom();
    const DevVol dv = v->dev();
    const CamP cp = cam_params(cam);
    const int ms = max_march_steps(v);
    if (kr == 1 || kr == 2) {
      const bool skip = kr == 2;
      if (enumerate) {
        if (skip) hipLaunchKernelGGL((k_reverse<true, true>), grid, dim3(256), 0, v->stream, g, dv, cp, tab, nelem, el,
                                     depth0, ms, v->dstar, viz, 0, vis, good, words, st, found, hz);
        else hipLaunchKernelGGL((k_reverse<true, false>), grid, dim3(256), 0, v->stream, g, dv, cp, tab, nelem, el,
                                depth0, ms, v->dstar, viz, 0, vis, good, words, st, found, hz);
      } else {
        if (skip) hipLaunchKernelGGL((k_reverse<false, true>), grid, dim3(256), 0, v->stream, g, dv, cp, tab, nelem,
                                     el, depth0, ms, v->dstar, viz, 1, vis, good, words, st, found, hz);
        else hipLaunchKernelGGL((k_reverse<false, false>), grid, dim3(256), 0, v->stream, g, dv, cp, tab, nelem, el,
                                depth0, ms, v->dstar, viz, 1, vis, good, words, st, found, hz);
      }
    } else {
      DMF_TRY(ensure_brick_dist(v));
      // the queue kernel writes every mask word it owns; words past the last wave stay 0
      if (enumerate) {
        hipLaunchKernelGGL((k_reverse_q<true, kRevItems, kRevRefill, kRevBurst>), gridq, dim3(256), 0, v->stream, g, dv, cp, tab, nelem,
                           el, nullptr, depth0, ms, v->dstar, viz, 0, vis, good, words, st, found, hz);
      } else if (kr == 3) {
        hipLaunchKernelGGL((k_reverse_q<false, kRevItems, kRevRefill, kRevBurst>), gridq, dim3(256), 0, v->stream, g, dv, cp, tab,
                           nelem, el, nullptr, depth0, ms, v->dstar, viz, 1, vis, good, words, st, found, hz);
      } else {
        DMF_TRY(ensure_spatial_order(v));
        void* items;
        // item-ordered masks, then 8 queue heads (k_reverse_x)
        DMF_TRY(scratch(v, kScRevItems, sizeof(uint64_t) * (size_t)(2 * P * words) + 64, &items));
        uint64_t* vis_i = (uint64_t*)items;
        uint64_t* good_i = vis_i + P * words;
        if (kr != 5) {
          // default: per-XCD unit queues (persistent: as many workgroups as the device holds at
          // once), a unit = the workgroup's 256 items (kr 4: a wave's 64) -- 5.30 vs 5.56 ms per
          // 128 poses (k_reverse_q's (chunk, pose) grid, kr 5), L2 hit rate 0.56 -> 0.83, beyond-L2
          // bytes 8.1 -> 3.3 GB; per-wave units 10.3 ms (the CU's waves no longer share L1 lines:
          // L2 requests x1.6).  DESIGN.md §5.5, profiles/r05b/
          unsigned int* heads = (unsigned int*)(good_i + P * words);
          DMF_HIP(hipMemsetAsync(heads, 0, 8 * sizeof(unsigned int), v->stream));
          const bool wg_units = kr != 4;
          const void* kfn = wg_units ? (const void*)k_reverse_x<kSpItems, kSpRefill, kSpBurst, true>
                                     : (const void*)k_reverse_x<kSpItems, kSpRefill, kSpBurst, false>;
          int per_cu = 0;
          DMF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 256, 0));
          int ncu = 0;
          DMF_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, v->device));
          const unsigned nwg = (unsigned)(std::max(ncu, 8) * std::max(per_cu, 1));
          if (wg_units)
            hipLaunchKernelGGL((k_reverse_x<kSpItems, kSpRefill, kSpBurst, true>), dim3(nwg), dim3(256), 0, v->stream, g,
                               dv, cp, tab, P, nelem, (const uint32_t*)v->d_sorder, depth0, ms, v->dstar, viz, vis_i,
                               good_i, words, heads, st, found, hz);
          else
            hipLaunchKernelGGL((k_reverse_x<kSpItems, kSpRefill, kSpBurst, false>), dim3(nwg), dim3(256), 0, v->stream,
                               g, dv, cp, tab, P, nelem, (const uint32_t*)v->d_sorder, depth0, ms, v->dstar, viz, vis_i,
                               good_i, words, heads, st, found, hz);
        } else {
          hipLaunchKernelGGL((k_reverse_q<false, kSpItems, kSpRefill, kSpBurst, true>), gridqs, dim3(256), 0, v->stream, g,
                             dv, cp, tab, nelem, el, (const uint32_t*)v->d_sorder, depth0, ms, v->dstar, viz, 1, vis_i,
                             good_i, words, st, found, hz);
        }
        DMF_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_mask_to_slots, dim3((unsigned)((words * 64 + 255) / 256)), dim3(256), 0, v->stream,
                           (const uint64_t*)vis_i, (const uint64_t*)good_i, (const uint32_t*)(v->d_sorder + v->sorder_cap),
                           nelem, words, P, vis, good);
      }
    }
    DMF_LAUNCH_CHECK();
  }
#if defined(DMF_EXP_STATS)
  if (d_stats) DMF_TRY(stats_end(v, st, d_stats, 2 + kRevStatN));
#else
  if (d_stats) DMF_TRY(stats_end(v, st, d_stats, 2));
#endif
  if (found_h) {
    found_h->assign(P, 0);
    unsigned long long hzh = 0;
    DMF_HIP(hipMemcpyAsync(found_h->data(), found, sizeof(int) * P, hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipMemcpyAsync(&hzh, hz, sizeof(hzh), hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
    v->hazards += (int64_t)hzh;
  }
  *d_vis = vis;
  *d_good = good;
  *words_out = words;
  *nelem_out = nelem;
  return DMF_OK;
}

static int reverse_lists(dmf_volume* v, const dmf_camera* cam, const float* poses, int32_t P, int32_t viz,
                         bool enumerate, uint8_t* found, int64_t* counts, uint64_t* hashes, int64_t cap) {
  if (!poses || !counts) return fail(DMF_ERR_INVALID, "null argument");
  uint64_t *vis, *good;
  int64_t words, nelem;
  std::vector<int> fh;
  DMF_TRY(run_reverse(v, cam, poses, P, false, viz, enumerate, &vis, &good, &words, &nelem, &fh, nullptr));
  if (found)
    for (int p = 0; p < P; ++p) found[p] = fh[p] ? 1 : 0;
  uint64_t* d_list;
  int64_t total = 0;
  DMF_TRY(compact_masks(v, good, P, words, nelem, counts, &d_list, &total,
                        enumerate ? kValueEnumCentroidHash : kValueSlotHash));
  if (total > cap) return fail(DMF_ERR_CAPACITY, "need %lld hashes", (long long)total);
  if (total > 0) {
    if (!hashes) return fail(DMF_ERR_INVALID, "null hashes");
    DMF_HIP(hipMemcpyAsync(hashes, d_list, sizeof(uint64_t) * total, hipMemcpyDeviceToHost, v->stream));
  }
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
}

// ---------------------------------------------------------------- forward march
// First occupied sample per lattice pixel (RayTracingEngine.hpp:280-308 loop body).
//
// Empty-space skipping (kSkip), exact.  Sample k is w_k = T * project(r, c, zd_k) in the
// reference's float/double arithmetic; the same expression in exact arithmetic is the
// line L(zd) = t + zd * dir (project is linear in zd).  A rounding-error bound
// eps_a(zd) = 8u (|t_a| + zd * 0.001 (|m_a0 ux| + |m_a1 uy| + |m_a2|)), u = 2^-24, covers
// |w_k - L(zd_k)| on each axis (5 roundings of float terms on inputs within u of exact;
// 8u leaves room).  Hence, with every margin delta = 2 eps(zd_j) + 1e-9 m:
//  * entry: samples whose exact point lies before the line enters the volume box grown by
//    delta are outside the volume (validPoints false, the reference `continue`s) — jump to
//    the last of them;
//  * bricks: if samples s and j both lie inside an empty cube of bricks (L-inf brick
//    distance field, as the reverse march) shrunk by delta, their exact points lie inside it
//    shrunk by eps and, the cube being convex, so do the exact points of every sample in
//    between; those samples are therefore inside the cube: no hit, no hazard — jump to j.
// j is estimated from the line and then verified by evaluating sample j exactly.
// The march of lattice pixel (ri, ci) of one pose: k_out / slot_out [ri * C + ci].
template <bool kSkip>
__device__ inline void fwd_ray(const Geom& g, const DevVol& vd, const CamP& cam, const PoseX* __restrict__ pose,
                               int zstart, int zdelta, int rdelta, int cdelta, int R, int C, int ri, int ci,
                               int32_t* __restrict__ k_out, int32_t* __restrict__ slot_out,
                               unsigned long long* __restrict__ hazards, int64_t& samples) {
  const int64_t idx = (int64_t)ri * C + ci;
  if (ri < R && ci < C) {
    const int r = ri * rdelta, c = ci * cdelta;
    int32_t kk = -1, sl = -1;
    const float* m = pose->f;
    // the exact line (double estimates) and the error-bound coefficients
    double dir[3], eA[3], eB[3];
    float fdir[3], frd[3];  // float copies for the jump estimates (verified exactly)
    int dmin_jump = 1 << 30;  // smallest brick distance d whose cube holds >= 2 more samples
    if (kSkip) {
      const double ux = ((double)c - cam.cx) / cam.fx, uy = ((double)r - cam.cy) / cam.fy;
      double step = 0.0;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const double m0 = m[4 * a], m1 = m[4 * a + 1], m2 = m[4 * a + 2];
        dir[a] = 0.001 * (m0 * ux + m1 * uy + m2);
        eA[a] = 0x1p-21 * fabs((double)m[4 * a + 3]);
        eB[a] = 0x1p-21 * 0.001 * (fabs(m0 * ux) + fabs(m1 * uy) + fabs(m2));
        fdir[a] = (float)dir[a];
        frd[a] = dir[a] != 0.0 ? (float)(1.0 / dir[a]) : 0.0f;
        step = fmax(step, fabs(dir[a]) * zdelta / g.dl[a]);  // cells per sample along axis a
      }
      // the cube reaches (d - 1) bricks of 2^bsh cells beyond the current brick on every side
      dmin_jump = 1 + (int)ceil(2.0 * step / (double)(1 << vd.bsh)) + 1;
    }
    auto margin = [&](int a, double zd) { return 2.0 * (eA[a] + zd * eB[a]) + 1e-9; };
    const int last_k = (int)((kZMax * 1000 - 1 - zstart) / zdelta);  // samples k = 0..last_k
    uint32_t known_full = 0xffffffffu;  // last brick found occupied (or not skippable)
    bool entered = false;
    int k = 0;
    for (int zd = zstart; (double)zd < kZMax * 1000; zd += zdelta, ++k) {
      float pc[3], w[3];
      project(cam, r, c, zd, pc);
      xform(m, pc[0], pc[1], pc[2], w);
      ++samples;
      if (!valid_points_f(g, w)) {
        if (kSkip && !entered) {
          // jump to the last sample before the line enters the volume grown by the margin
          entered = true;  // (once: after the entry the march proceeds normally)
          double tin = -1e300, tout = 1e300;
          const double zmax = kZMax * 1000;
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            const double dm = margin(a, zmax);
            const double lo = g.mn[a] - dm, hi = g.mx[a] + dm, t0 = (double)m[4 * a + 3];
            if (dir[a] == 0.0) {
              if (t0 <= lo || t0 >= hi) tout = -1e300;  // never enters
            } else {
              const double ta = (lo - t0) / dir[a], tb = (hi - t0) / dir[a];
              tin = fmax(tin, fmin(ta, tb));
              tout = fmin(tout, fmax(ta, tb));
            }
          }
          int kj = tout < tin ? last_k : (int)floor((tin - (double)zstart) / zdelta) - 1;
          kj = min(kj, last_k);
          if (kj > k) {
            const int zj = zstart + kj * zdelta;
#if DMF_FWD_VERIFY_JUMPS
            float qc[3], q[3];
            project(cam, r, c, zj, qc);
            xform(m, qc[0], qc[1], qc[2], q);
            ++samples;
            if (!valid_points_f(g, q)) {  // verified: still outside
              k = kj;
              zd = zj;
            }
#else
            // zj is a whole step before the line enters the volume grown by the margin, so every
            // sample up to it is outside the volume: no sample is evaluated to check it
            k = kj;
            zd = zj;
#endif
          }
        }
        continue;
      }
      entered = true;
      int a, b, cc;
      bin_point(g, w, a, b, cc);
      if (!valid_coords(g, a, b, cc)) {  // reference indexes voxels_ unguarded here (UB)
        atomicAdd(hazards, 1ull);
        continue;
      }
      if (occ_test(vd.occ, occ_bit(g, a, b, cc))) {
        kk = k;
        sl = vd.slot_of[lin_index(g, a, b, cc)];
        break;
      }
      if (!kSkip) continue;
      const int ba = a >> vd.bsh, bb = b >> vd.bsh, bc = cc >> vd.bsh;
      const uint32_t bl = ((uint32_t)ba * (uint32_t)vd.nb[1] + (uint32_t)bb) * (uint32_t)vd.nb[2] + (uint32_t)bc;
      if (bl == known_full) continue;
      const int d = vd.bdist[bl];
      if (d >= dmin_jump) {  // (smaller cubes cannot hold two more samples: not worth a try)
        const int Rb = d - 1;  // bricks within Rb of this one are empty
        const int bx[3] = {ba, bb, bc};
        double lo[3], hi[3];
        float zexit = 3.0e38f;
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
          lo[ax] = g.mn[ax] + (double)(max(bx[ax] - Rb, 0) << vd.bsh) * g.dl[ax];
          hi[ax] = g.mn[ax] + (double)min((bx[ax] + Rb + 1) << vd.bsh, g.n[ax]) * g.dl[ax];
          if (fdir[ax] != 0.0f)
            zexit = fminf(zexit, ((float)(fdir[ax] > 0.0f ? hi[ax] : lo[ax]) - m[4 * ax + 3]) * frd[ax]);
        }
        int kj = min((int)floorf((zexit - (float)zstart) / (float)zdelta) - 1, last_k);
        if (kj > k + 1) {
          const int zj = zstart + kj * zdelta;
          bool ok = true;
#if DMF_FWD_VERIFY_JUMPS
          float qc[3], q[3];
          project(cam, r, c, zj, qc);
          xform(m, qc[0], qc[1], qc[2], q);
          ++samples;
#pragma unroll
          for (int ax = 0; ax < 3; ++ax) {
            const double dm = margin(ax, (double)zj);
            ok = ok && (double)w[ax] >= lo[ax] + dm && (double)w[ax] <= hi[ax] - dm && (double)q[ax] >= lo[ax] + dm &&
                 (double)q[ax] <= hi[ax] - dm;
          }
#else
          // sample j is not evaluated: the line's point at zj inside the cube shrunk by 2 delta
          // puts sample j inside it shrunk by delta (its rounding is within eps of the line)
#pragma unroll
          for (int ax = 0; ax < 3; ++ax) {
            const double dm = margin(ax, (double)zj), lq = (double)m[4 * ax + 3] + (double)zj * dir[ax];
            ok = ok && (double)w[ax] >= lo[ax] + dm && (double)w[ax] <= hi[ax] - dm && lq >= lo[ax] + 2.0 * dm &&
                 lq <= hi[ax] - 2.0 * dm;
          }
#endif
          if (ok) {  // samples k+1 .. kj lie inside the empty cube
            k = kj;
            zd = zj;
            continue;
          }
        }
      }
      known_full = bl;  // occupied brick, or the jump failed: step through it
    }
    k_out[idx] = kk;
    slot_out[idx] = sl;
  }
}

template <bool kSkip>
__global__ __launch_bounds__(256) DMF_FWD_OCC void k_forward(Geom g, DevVol vd, CamP cam, const PoseX* __restrict__ pose,
                                                 int zstart, int zdelta, int rdelta, int cdelta, int R, int C,
                                                 int32_t* __restrict__ k_out, int32_t* __restrict__ slot_out,
                                                 unsigned long long* __restrict__ hazards,
                                                 unsigned long long* __restrict__ stats) {
  stats = stat_slot(stats);
  // a wave marches an 8x8 tile of lattice pixels (fwd_threads): neighbouring rays in both
  // directions reach similar depths and read the same bitmask tiles (a row of 64 pixels
  // spans 8x the angle); outputs stay row-major (idx)
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int tpr = (C + 7) >> 3, ln = (int)(t & 63);
  const int64_t tile = t >> 6;
  const int ri = (int)(tile / tpr) * 8 + (ln >> 3), ci = (int)(tile % tpr) * 8 + (ln & 7);
  // grid.y = pose index of a batched launch (one pose: grid.y = 1)
  int64_t samples = 0;
  fwd_ray<kSkip>(g, vd, cam, pose + blockIdx.y, zstart, zdelta, rdelta, cdelta, R, C, ri, ci,
                 k_out + (int64_t)blockIdx.y * R * C, slot_out + (int64_t)blockIdx.y * R * C, hazards, samples);
  if (stats) wave_add_u64(&stats[0], (unsigned long long)samples);
#if defined(DMF_EXP_STATS)
  // diagnostic build: 64 x the wave's longest march (lane-samples the wave occupies), so that
  // stats[0] / stats[1] is the march's lane utilisation
  if (stats) {
    unsigned long long mx = (unsigned long long)samples;
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned long long)__shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) atomicAdd(&stats[1], 64ull * mx);
  }
#endif
}

// ---- forward march with per-wave lane refill (fwd_kernel knob 2) -----------------------
// fwd_ray's loop, split into a per-pixel setup and one loop iteration (fwd_step), so that a lane
// whose ray has ended takes the next pixel of its wave's queue while the others march on: the
// k_reverse_q pattern on the forward march.  Same arithmetic, same outputs.
struct FwdLane {
  double dir[3], eA[3], eB[3];
  float fdir[3], frd[3];
  int k, zd, dmin_jump;
  uint32_t known_full;
  bool entered;
};

template <bool kSkip>
__device__ inline void fwd_setup(const Geom& g, const DevVol& vd, const CamP& cam, const float* m, int zstart,
                                 int zdelta, int r, int c, FwdLane& L) {
  L.dmin_jump = 1 << 30;
  if (kSkip) {
    const double ux = ((double)c - cam.cx) / cam.fx, uy = ((double)r - cam.cy) / cam.fy;
    double step = 0.0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const double m0 = m[4 * a], m1 = m[4 * a + 1], m2 = m[4 * a + 2];
      L.dir[a] = 0.001 * (m0 * ux + m1 * uy + m2);
      L.eA[a] = 0x1p-21 * fabs((double)m[4 * a + 3]);
      L.eB[a] = 0x1p-21 * 0.001 * (fabs(m0 * ux) + fabs(m1 * uy) + fabs(m2));
      L.fdir[a] = (float)L.dir[a];
      L.frd[a] = L.dir[a] != 0.0 ? (float)(1.0 / L.dir[a]) : 0.0f;
      step = fmax(step, fabs(L.dir[a]) * zdelta / g.dl[a]);
    }
    L.dmin_jump = 1 + (int)ceil(2.0 * step / (double)(1 << vd.bsh)) + 1;
  }
  L.known_full = 0xffffffffu;
  L.entered = false;
  L.k = 0;
  L.zd = zstart;
}

// One iteration of fwd_ray's loop for pixel (r, c): 0 = march on, 1 = hit (kk, sl), 2 = the
// march left the depth range without a hit.
template <bool kSkip>
__device__ inline int fwd_step(const Geom& g, const DevVol& vd, const CamP& cam, const float* m, int zstart, int zdelta,
                               int last_k, int r, int c, FwdLane& L, int32_t& kk, int32_t& sl,
                               unsigned long long* __restrict__ hazards, int64_t& samples) {
  if (!((double)L.zd < kZMax * 1000)) return 2;
  auto margin = [&](int a, double zd) { return 2.0 * (L.eA[a] + zd * L.eB[a]) + 1e-9; };
  float pc[3], w[3];
  project(cam, r, c, L.zd, pc);
  xform(m, pc[0], pc[1], pc[2], w);
  ++samples;
  if (!valid_points_f(g, w)) {
    if (kSkip && !L.entered) {
      L.entered = true;
      double tin = -1e300, tout = 1e300;
      const double zmax = kZMax * 1000;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const double dm = margin(a, zmax);
        const double lo = g.mn[a] - dm, hi = g.mx[a] + dm, t0 = (double)m[4 * a + 3];
        if (L.dir[a] == 0.0) {
          if (t0 <= lo || t0 >= hi) tout = -1e300;
        } else {
          const double ta = (lo - t0) / L.dir[a], tb = (hi - t0) / L.dir[a];
          tin = fmax(tin, fmin(ta, tb));
          tout = fmin(tout, fmax(ta, tb));
        }
      }
      int kj = tout < tin ? last_k : (int)floor((tin - (double)zstart) / zdelta) - 1;
      kj = min(kj, last_k);
      if (kj > L.k) {
        const int zj = zstart + kj * zdelta;
#if DMF_FWD_VERIFY_JUMPS
        float qc[3], q[3];
        project(cam, r, c, zj, qc);
        xform(m, qc[0], qc[1], qc[2], q);
        ++samples;
        if (!valid_points_f(g, q)) {
          L.k = kj;
          L.zd = zj;
        }
#else
        L.k = kj;  // (as fwd_ray)
        L.zd = zj;
#endif
      }
    }
    L.zd += zdelta;
    ++L.k;
    return 0;
  }
  L.entered = true;
  int a, b, cc;
  bin_point(g, w, a, b, cc);
  if (!valid_coords(g, a, b, cc)) {
    atomicAdd(hazards, 1ull);
    L.zd += zdelta;
    ++L.k;
    return 0;
  }
  if (occ_test(vd.occ, occ_bit(g, a, b, cc))) {
    kk = L.k;
    sl = vd.slot_of[lin_index(g, a, b, cc)];
    return 1;
  }
  if (kSkip) {
    const int ba = a >> vd.bsh, bb = b >> vd.bsh, bc = cc >> vd.bsh;
    const uint32_t bl = ((uint32_t)ba * (uint32_t)vd.nb[1] + (uint32_t)bb) * (uint32_t)vd.nb[2] + (uint32_t)bc;
    if (bl != L.known_full) {
      bool jumped = false;
      const int d = vd.bdist[bl];
      if (d >= L.dmin_jump) {
        const int Rb = d - 1;
        const int bx[3] = {ba, bb, bc};
        double lo[3], hi[3];
        float zexit = 3.0e38f;
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) {
          lo[ax] = g.mn[ax] + (double)(max(bx[ax] - Rb, 0) << vd.bsh) * g.dl[ax];
          hi[ax] = g.mn[ax] + (double)min((bx[ax] + Rb + 1) << vd.bsh, g.n[ax]) * g.dl[ax];
          if (L.fdir[ax] != 0.0f)
            zexit = fminf(zexit, ((float)(L.fdir[ax] > 0.0f ? hi[ax] : lo[ax]) - m[4 * ax + 3]) * L.frd[ax]);
        }
        int kj = min((int)floorf((zexit - (float)zstart) / (float)zdelta) - 1, last_k);
        if (kj > L.k + 1) {
          const int zj = zstart + kj * zdelta;
          bool ok = true;
#if DMF_FWD_VERIFY_JUMPS
          float qc[3], q[3];
          project(cam, r, c, zj, qc);
          xform(m, qc[0], qc[1], qc[2], q);
          ++samples;
#pragma unroll
          for (int ax = 0; ax < 3; ++ax) {
            const double dm = margin(ax, (double)zj);
            ok = ok && (double)w[ax] >= lo[ax] + dm && (double)w[ax] <= hi[ax] - dm && (double)q[ax] >= lo[ax] + dm &&
                 (double)q[ax] <= hi[ax] - dm;
          }
#else
#pragma unroll
          for (int ax = 0; ax < 3; ++ax) {  // (as fwd_ray)
            const double dm = margin(ax, (double)zj), lq = (double)m[4 * ax + 3] + (double)zj * L.dir[ax];
            ok = ok && (double)w[ax] >= lo[ax] + dm && (double)w[ax] <= hi[ax] - dm && lq >= lo[ax] + 2.0 * dm &&
                 lq <= hi[ax] - 2.0 * dm;
          }
#endif
          if (ok) {
            L.k = kj;
            L.zd = zj;
            jumped = true;
          }
        }
      }
      if (!jumped) L.known_full = bl;
    }
  }
  L.zd += zdelta;
  ++L.k;
  return 0;
}

// Each wave owns kUnit consecutive 8x8 tiles of one pose (grid.y) and keeps its lanes busy:
// a lane whose ray has ended writes its outputs and takes the next pixel of the unit (tile
// order: neighbouring rays together) when at least kRefill lanes are idle; between refills
// every busy lane marches up to kBurst samples.
template <bool kSkip, int kUnit, int kRefill, int kBurst>
__global__ __launch_bounds__(256) DMF_FWDQ_OCC void k_forward_q(Geom g, DevVol vd, CamP cam,
                                                                const PoseX* __restrict__ pose, int zstart, int zdelta,
                                                                int rdelta, int cdelta, int R, int C,
                                                                int32_t* __restrict__ k_out, int32_t* __restrict__ slot_out,
                                                                unsigned long long* __restrict__ hazards,
                                                                unsigned long long* __restrict__ stats) {
  stats = stat_slot(stats);
  const int w = threadIdx.x >> 6;
  const int tpr = (C + 7) >> 3;
  const int64_t ntiles = (int64_t)((R + 7) >> 3) * tpr;
  const int64_t t0 = ((int64_t)blockIdx.x * 4 + w) * kUnit;
  if (t0 >= ntiles) return;
  const int nitems = (int)min<int64_t>(ntiles - t0, kUnit) * 64;
  const float* m = pose[blockIdx.y].f;
  int32_t* const ko = k_out + (int64_t)blockIdx.y * R * C;
  int32_t* const so = slot_out + (int64_t)blockIdx.y * R * C;
  const int last_k = (int)((kZMax * 1000 - 1 - zstart) / zdelta);
  int64_t samples = 0;
  [[maybe_unused]] unsigned long long busy = 0, slots = 0;  // (diagnostic build: lane utilisation)
  FwdLane L;
  int item = -1, r = 0, c = 0;
  int64_t idx = 0;
  int next = 0;  // wave-uniform queue head
  while (true) {
    const uint64_t idle = __builtin_amdgcn_ballot_w64(item < 0);
    const int nidle = __builtin_popcountll(idle);
    if (next < nitems && (nidle >= kRefill || nidle == 64)) {
      if (item < 0) {
        const int it = next + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        if (it < nitems) {
          const int64_t tile = t0 + (it >> 6);
          const int ln = it & 63;
          const int ri = (int)(tile / tpr) * 8 + (ln >> 3), ci = (int)(tile % tpr) * 8 + (ln & 7);
          if (ri < R && ci < C) {
            item = it;
            idx = (int64_t)ri * C + ci;
            r = ri * rdelta;
            c = ci * cdelta;
            fwd_setup<kSkip>(g, vd, cam, m, zstart, zdelta, r, c, L);
          }
        }
      }
      next += nidle;
    }
    if (__builtin_amdgcn_ballot_w64(item >= 0) == 0) {
      if (next >= nitems) break;
      continue;
    }
    int st = 0;
    int32_t kk = -1, sl = -1;
#pragma unroll 1
    for (int b = 0; b < kBurst; ++b) {
#if defined(DMF_EXP_STATS)
      if ((threadIdx.x & 63) == 0) slots += 64;
      if (item >= 0 && st == 0) ++busy;
#endif
      if (item >= 0 && st == 0) st = fwd_step<kSkip>(g, vd, cam, m, zstart, zdelta, last_k, r, c, L, kk, sl, hazards, samples);
      if (__builtin_amdgcn_ballot_w64(item >= 0 && st == 0) == 0) break;
    }
    if (item >= 0 && st != 0) {
      ko[idx] = kk;
      so[idx] = sl;
      item = -1;
    }
  }
  if (stats) wave_add_u64(&stats[0], (unsigned long long)samples);
#if defined(DMF_EXP_STATS)
  // diagnostic build: busy lane-iterations against 64 x burst iterations (stats[0] / stats[1]
  // of k_forward is the same utilisation of its lane-per-pixel march)
  if (stats) {
    wave_add_u64(&stats[2], busy);
    wave_add_u64(&stats[3], slots);
  }
#endif
}

// The batched forward march with per-XCD unit queues (as k_reverse_x): a unit is one
// workgroup's 4 consecutive 8x8 tiles (row-major tile order) of one pose; the tile range is
// cut into 8 contiguous bands of rows, one queue per band, units pose-major inside it, and
// workgroup b serves the queue of its XCD group b % 8 first (a speed choice: the waves of one
// XCD then march one slab of one frustum at a time and share its L2 lines of the occupancy
// bitmask and distance field), then steals from the other queues.  heads[8] zeroed before.
template <bool kSkip>
__global__ __launch_bounds__(256) void k_forward_x(Geom g, DevVol vd, CamP cam, const PoseX* __restrict__ pose, int P,
                                                   int zstart, int zdelta, int rdelta, int cdelta, int R, int C,
                                                   int32_t* __restrict__ k_out, int32_t* __restrict__ slot_out,
                                                   unsigned int* __restrict__ heads,
                                                   unsigned long long* __restrict__ hazards,
                                                   unsigned long long* __restrict__ stats) {
  stats = stat_slot(stats);
  __shared__ uint32_t s_unit;
  const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int tpr = (C + 7) >> 3;
  const int64_t ntiles = (int64_t)((R + 7) >> 3) * tpr, nwu = (ntiles + 3) / 4;
  const int grp = (int)(blockIdx.x & 7u);
  int64_t samples = 0;
  for (int q = 0; q < 8; ++q) {
    const int gq = (grp + q) & 7;
    const int64_t u0 = nwu * gq / 8, nch = nwu * (gq + 1) / 8 - u0;
    const uint32_t nunits = (uint32_t)(nch * P);
    for (;;) {
      if (threadIdx.x == 0) s_unit = atomicAdd(&heads[gq], 1u);
      __syncthreads();
      const uint32_t u = s_unit;
      __syncthreads();  // every wave has read it before the next unit's write
      if (u >= nunits) break;
      const int p = (int)(u / (uint32_t)nch);
      const int64_t tile = (u0 + (int64_t)(u - (uint32_t)p * (uint32_t)nch)) * 4 + w;
      if (tile < ntiles) {
        const int ri = (int)(tile / tpr) * 8 + (ln >> 3), ci = (int)(tile % tpr) * 8 + (ln & 7);
        fwd_ray<kSkip>(g, vd, cam, pose + p, zstart, zdelta, rdelta, cdelta, R, C, ri, ci,
                       k_out + (int64_t)p * R * C, slot_out + (int64_t)p * R * C, hazards, samples);
      }
    }
  }
  if (stats) wave_add_u64(&stats[0], (unsigned long long)samples);
}

// k_forward_q's shape: tiles per wave unit, refill threshold, samples per burst
#if defined(DMF_EXP_FWDQ_UNIT)
constexpr int kFwdUnit = DMF_EXP_FWDQ_UNIT, kFwdRefill = DMF_EXP_FWDQ_REFILL, kFwdBurst = DMF_EXP_FWDQ_BURST;
#else
constexpr int kFwdUnit = 4, kFwdRefill = 16, kFwdBurst = 8;
#endif

// threads of a k_forward launch per pose: whole 8x8 tiles of the R x C lattice
static unsigned fwd_blocks(int R, int C) {
  const int64_t threads = (int64_t)((R + 7) / 8) * ((C + 7) / 8) * 64;
  return (unsigned)((threads + 255) / 256);
}

// DMF_KNOB_FWD_SKIP = -1 (dmf_diag.h) disables the forward march's empty-space skipping (A/B)
static bool fwd_skip(const dmf_volume* v) { return v->knob[DMF_KNOB_FWD_SKIP] >= 0; }

#define DMF_LAUNCH_FORWARD(GRID, ...)                                                                          \
  do {                                                                                                        \
    if (fwd_skip(v)) {                                                                                         \
      DMF_TRY(ensure_brick_dist(v));                                                                          \
      hipLaunchKernelGGL(k_forward<true>, GRID, dim3(256), 0, v->stream, __VA_ARGS__);                         \
    } else {                                                                                                  \
      hipLaunchKernelGGL(k_forward<false>, GRID, dim3(256), 0, v->stream, __VA_ARGS__);                        \
    }                                                                                                         \
  } while (0)

enum FwdMode { kTrace = 0, kClassify = 1, kGoodPoints = 2, kPoints = 3, kMinimum = 4 };

// Side effects of the first hit per pixel (RayTracingEngine.hpp:299-305, 351-371,
// 420-440, 480-489, 256-259).
__global__ void k_forward_post(Geom g, DevVol vd, CamP cam, const PoseX* __restrict__ pose, int mode, int zstart,
                               int zdelta, int rdelta, int cdelta, int R, int C, int view_arg, float dstar,
                               const int32_t* __restrict__ k_in, const int32_t* __restrict__ slot_in,
                               unsigned long long* __restrict__ minkey, int* __restrict__ kmin,
                               int* __restrict__ found) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)R * C) return;
  const int32_t kk = k_in[idx];
  if (kk < 0) return;
  const int32_t slot = slot_in[idx];
  *found = 1;
  if (mode == kMinimum) {
    atomicMin(kmin, kk);
    return;
  }
  if (mode == kTrace) {
    vd.view[slot] = 1;
    return;
  }
  const unsigned long long key = (unsigned long long)kk * (unsigned long long)((int64_t)R * C) + (unsigned long long)idx;
  if (mode == kPoints) {
    atomicMin(&minkey[slot], key);
    return;
  }
  // classify / good points: pseudo-centroid = sample + delta/2, v toward the camera
  const int zd = zstart + kk * zdelta;
  const int r = (int)(idx / C) * rdelta, c = (int)(idx % C) * cdelta;
  float pc[3], w[3];
  project(cam, r, c, zd, pc);
  xform(pose->f, pc[0], pc[1], pc[2], w);
  const float cen[3] = {(float)((double)w[0] + g.hdl[0]), (float)((double)w[1] + g.hdl[1]),
                        (float)((double)w[2] + g.hdl[2])};
  const float d[3] = {pose->f[3] - cen[0], pose->f[7] - cen[1], pose->f[11] - cen[2]};
  float v[3];
  normalized(d, v);
  bool ok = false;
  if (zd >= 250 && zd <= 600) {
    const int32_t a = vd.off[slot], b = vd.off[slot + 1];
    for (int32_t j = a; j < b; ++j) {
      const float4 n = vd.nrm[j];
      if (n.w != 0.0f && angle_ok(n.x, n.y, n.z, v, dstar)) { ok = true; break; }
    }
  }
  if (mode == kClassify) {
    if (vd.view[slot] == 0) vd.view[slot] = view_arg;
    if (ok) vd.good[slot] = 1;
  } else if (ok) {
    atomicMin(&minkey[slot], key);
  }
}

__global__ void k_minkey_flags(const unsigned long long* __restrict__ minkey, int64_t V, uint8_t* __restrict__ flags) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < V) flags[s] = minkey[s] != ~0ull;
}

__global__ void k_minkey_pairs(const uint32_t* __restrict__ slots, const unsigned long long* __restrict__ nsel,
                               const unsigned long long* __restrict__ minkey, const uint64_t* __restrict__ hash,
                               uint64_t* __restrict__ keys, uint64_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((unsigned long long)i >= *nsel) return;
  const uint32_t s = slots[i];
  keys[i] = minkey[s];
  vals[i] = hash[s];
}

struct FwdResult {
  int found = 0;
  int minimum = -1;
  int64_t n = 0;
  uint64_t* d_list = nullptr;
};

static int run_forward(dmf_volume* v, const dmf_camera* cam, const float* pose, int mode, int zstart, int zdelta,
                       int rdelta, int cdelta, int view_arg, FwdResult* res) {
  DMF_TRY(require_constructed(v));
  DMF_TRY(check_camera(cam));
  if (!pose) return fail(DMF_ERR_INVALID, "null pose");
  if (zdelta <= 0) return fail(DMF_ERR_INVALID, "zdelta must be > 0 (the reference loops forever)");
  if (rdelta <= 0 || cdelta <= 0) return fail(DMF_ERR_INVALID, "bad pixel stride");
  PoseX* tab;
  DMF_TRY(pose_table(v, pose, 1, false, &tab));
  const int R = (cam->height + rdelta - 1) / rdelta, C = (cam->width + cdelta - 1) / cdelta;
  const int64_t RC = (int64_t)R * C;
  void *kb, *sb, *aux;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * RC, &kb));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * RC, &sb));
  DMF_TRY(scratch(v, kScHost2, 64, &aux));
  int* found = (int*)aux;
  int* kmin = found + 1;
  unsigned long long* hz = (unsigned long long*)((char*)aux + 16);
  DMF_HIP(hipMemsetAsync(aux, 0, 64, v->stream));
  DMF_HIP(hipMemsetAsync(kmin, 0x7f, sizeof(int), v->stream));
  const CamP cp = cam_params(cam);
  const Geom g = v->geom();
  const dim3 grid((unsigned)((RC + 255) / 256));
  DMF_LAUNCH_FORWARD(dim3(fwd_blocks(R, C)), g, v->dev(), cp, tab, zstart, zdelta, rdelta, cdelta, R, C, (int32_t*)kb, (int32_t*)sb, hz,
                     nullptr);
  DMF_LAUNCH_CHECK();
  unsigned long long* minkey = nullptr;
  if ((mode == kPoints || mode == kGoodPoints) && v->V > 0) {
    void* mk;
    DMF_TRY(scratch(v, kScOut2, sizeof(unsigned long long) * v->V, &mk));
    minkey = (unsigned long long*)mk;
    DMF_HIP(hipMemsetAsync(minkey, 0xff, sizeof(unsigned long long) * v->V, v->stream));
  }
  hipLaunchKernelGGL(k_forward_post, grid, dim3(256), 0, v->stream, g, v->dev(), cp, tab, mode, zstart, zdelta,
                     rdelta, cdelta, R, C, view_arg, v->dstar, (const int32_t*)kb, (const int32_t*)sb, minkey, kmin,
                     found);
  DMF_LAUNCH_CHECK();
  int hf[2];
  unsigned long long hzh = 0;
  DMF_HIP(hipMemcpyAsync(hf, aux, sizeof(hf), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipMemcpyAsync(&hzh, hz, sizeof(hzh), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  v->hazards += (int64_t)hzh;
  res->found = hf[0];
  res->minimum = (hf[1] == 0x7f7f7f7f) ? -1 : zstart + hf[1] * zdelta;
  res->n = 0;
  if (minkey) {
    // slots with a key, ordered by the reference loop key (k, r, c)
    void *fl, *sel, *ns, *kk2;
    DMF_TRY(scratch(v, kScOut3, v->V + 16, &fl));
    DMF_TRY(scratch(v, kScOut0, sizeof(uint32_t) * v->V, &sel));
    DMF_TRY(scratch(v, kScHost1, 16, &ns));
    hipLaunchKernelGGL(k_minkey_flags, dim3((unsigned)((v->V + 255) / 256)), dim3(256), 0, v->stream, minkey, v->V,
                       (uint8_t*)fl);
    DMF_LAUNCH_CHECK();
    size_t bytes = 0;
    auto it = rocprim::counting_iterator<uint32_t>(0);
    DMF_HIP(rocprim::select(nullptr, bytes, it, (uint8_t*)fl, (uint32_t*)sel, (unsigned long long*)ns, (size_t)v->V,
                            v->stream));
    void* tmp;
    DMF_TRY(scratch(v, kScTmp, bytes, &tmp));
    DMF_HIP(rocprim::select(tmp, bytes, it, (uint8_t*)fl, (uint32_t*)sel, (unsigned long long*)ns, (size_t)v->V,
                            v->stream));
    unsigned long long n = 0;
    DMF_HIP(hipMemcpyAsync(&n, ns, sizeof(n), hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
    if (n > 0) {
      DMF_TRY(scratch(v, kScOut1, sizeof(uint64_t) * n, &kk2));
      void* vals;
      DMF_TRY(scratch(v, kScHost0, sizeof(uint64_t) * n, &vals));
      hipLaunchKernelGGL(k_minkey_pairs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream,
                         (const uint32_t*)sel, (const unsigned long long*)ns, minkey, v->d_hash, (uint64_t*)kk2,
                         (uint64_t*)vals);
      DMF_LAUNCH_CHECK();
      int end_bit = 1;
      const unsigned long long maxkey = (unsigned long long)((1000 - zstart) / zdelta + 2) * (unsigned long long)RC;
      while (end_bit < 64 && (1ull << end_bit) <= maxkey) ++end_bit;
      DMF_TRY(sort_pairs_u64(v, (uint64_t*)kk2, (uint64_t*)vals, n, end_bit));
      res->d_list = (uint64_t*)vals;
      res->n = (int64_t)n;
    }
  }
  return DMF_OK;
}

static int forward_list_api(dmf_volume* v, const dmf_camera* cam, const float* pose, int mode, int zdelta, int sparse,
                            uint8_t* found, uint64_t* hashes, int64_t cap, int64_t* n) {
  const int s = sparse ? 5 : 1;  // RayTracingEngine.hpp:387-392 / 452-457
  FwdResult res;
  DMF_TRY(run_forward(v, cam, pose, mode, 10, zdelta, s, s, 1, &res));
  if (found) *found = res.found ? 1 : 0;
  if (n) *n = res.n;
  if (res.n > cap) return fail(DMF_ERR_CAPACITY, "need %lld hashes", (long long)res.n);
  if (res.n > 0) {
    if (!hashes) return fail(DMF_ERR_INVALID, "null hashes");
    DMF_HIP(hipMemcpyAsync(hashes, res.d_list, sizeof(uint64_t) * res.n, hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
  }
  return DMF_OK;
}

// ---------------------------------------------------------------- rayTraceVolume
// z-buffer over the float-accumulated enumeration (RayTracingEngine.hpp:509-536),
// then view marking where the voxel's depth equals the pixel minimum (:540-563).
__global__ void k_zbuffer(Geom g, DevVol vd, CamP cam, const PoseX* __restrict__ pose, EnumList el, int64_t n,
                          int pass, int* __restrict__ zbuf, unsigned long long* __restrict__ hazards) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint32_t en = el.list[e];
  const uint32_t nyz = (uint32_t)el.nax[1] * (uint32_t)el.nax[2];
  const uint32_t i = en / nyz, j = (en / el.nax[2]) % el.nax[1], k = en % el.nax[2];
  const float x = el.axes[i], y = el.axes[el.nax[0] + j], z = el.axes[el.nax[0] + el.nax[1] + k];
  float t[3];
  xform(pose->i, (float)((double)x + g.hdl[0]), (float)((double)y + g.hdl[1]), (float)((double)z + g.hdl[2]), t);
  int r, c;
  if (!deproject_valid(cam, t[0], t[1], t[2], r, c)) return;
  const int d = to_int_x86((double)roundf(t[2] * 1000.0f));
  int* px = &zbuf[(int64_t)r * cam.W + c];
  if (pass == 0) {
    if (d == -1) atomicAdd(hazards, 1ull);  // collides with the reference's -1 "unset" marker (:529)
    atomicMin(px, d);
  } else if (*px == d) {
    vd.view[vd.slot_of[lin_index(g, bin_axis(g, 0, x), bin_axis(g, 1, y), bin_axis(g, 2, z))]] = 1;
  }
}

__global__ void k_zbuf_out(const int* __restrict__ z, int64_t n, int* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = z[i] == 0x7fffffff ? -1 : z[i];
}

// ---------------------------------------------------------------- willCollide
// tests/CameraPathGen.cpp:128-156, one lane per segment.
__global__ void k_will_collide(Geom g, const uint32_t* __restrict__ occ, const float* __restrict__ A,
                               const float* __restrict__ B, int64_t n, uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a[3] = {A[3 * i], A[3 * i + 1], A[3 * i + 2]};
  const float b[3] = {B[3 * i], B[3 * i + 1], B[3 * i + 2]};
  const float ab[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  const double distance = (double)sqrtf(sum3(ab[0] * ab[0], ab[1] * ab[1], ab[2] * ab[2]));
  const float ba[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  float v[3];
  normalized(ba, v);
  bool collided = false;
  const double lim = distance * 1000;
  for (int depth = 1; !collided; depth++) {
    if ((double)depth > lim) break;
    const float fd = (float)depth;
    const float px = a[0] + div_rn(v[0] * fd, 1000.0f, 1.0f / 1000.0f);
    const float py = a[1] + div_rn(v[1] * fd, 1000.0f, 1.0f / 1000.0f);
    const float pz = a[2] + div_rn(v[2] * fd, 1000.0f, 1.0f / 1000.0f);
    const float pp[3] = {px, py, pz};
    if (!valid_points_f(g, pp)) continue;
    int x, y, z;
    bin_point(g, pp, x, y, z);
    if (!valid_coords(g, x, y, z)) continue;
    if (occ_test(occ, occ_bit(g, x, y, z))) collided = true;
  }
  out[i] = collided ? 1 : 0;
}

// Planner::run_tsp cost map (tests/CameraPathGen.cpp:310-331): all V*V ordered pairs
// of camera centres, map = INT_MAX if willCollide(a, b) else int(|a-b| * 1000).
// willCollide's loop only ever sets `collided`, so its result is the OR over depths
// 1..floor(distance*1000) of "sample valid and occupied": one wave per pair, lane l
// tests depth base+l, a ballot ends the pair at the first occupied 64-depth group.
// Every lane evaluates the same float expressions as the scalar loop, so the OR is
// bit-identical to the sequential march and there is no per-lane length divergence.
// Pairs whose segment the reference cannot march (non-finite, or more than INT_MAX
// depths: the int counter overflows) get -1.
constexpr int kCostWaves = 4;
constexpr int32_t kMaxCostPoses = 46340;  // V*V int32 entries < 2^31
__global__ __launch_bounds__(64 * kCostWaves) void k_cost_map(Geom g, const uint32_t* __restrict__ occ,
                                                              const float* __restrict__ poses, int32_t V,
                                                              int32_t* __restrict__ map) {
  const int64_t pair = (int64_t)blockIdx.x * kCostWaves + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (pair >= (int64_t)V * V) return;
  const int64_t i = pair / V, j = pair - i * V;
  const float a[3] = {poses[12 * i + 3], poses[12 * i + 7], poses[12 * i + 11]};
  const float b[3] = {poses[12 * j + 3], poses[12 * j + 7], poses[12 * j + 11]};
  const float ab[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  const double distance = (double)sqrtf(sum3(ab[0] * ab[0], ab[1] * ab[1], ab[2] * ab[2]));
  const double lim = distance * 1000;
  if (!(lim < 2147483647.0)) {  // NaN or an overflowing depth counter
    if (lane == 0) map[pair] = -1;
    return;
  }
  const float ba[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  float v[3];
  normalized(ba, v);
  bool collided = false;
  for (int64_t base = 1; (double)base <= lim; base += 64) {
    const int64_t depth = base + lane;
    bool hit = false;
    if ((double)depth <= lim) {
      const float fd = (float)depth;
      const float px = a[0] + div_rn(v[0] * fd, 1000.0f, 1.0f / 1000.0f);
      const float py = a[1] + div_rn(v[1] * fd, 1000.0f, 1.0f / 1000.0f);
      const float pz = a[2] + div_rn(v[2] * fd, 1000.0f, 1.0f / 1000.0f);
      const float pp[3] = {px, py, pz};
      if (valid_points_f(g, pp)) {
        int x, y, z;
        bin_point(g, pp, x, y, z);
        hit = valid_coords(g, x, y, z) && occ_test(occ, occ_bit(g, x, y, z));
      }
    }
    if (__builtin_amdgcn_ballot_w64(hit)) {
      collided = true;
      break;
    }
  }
  if (lane == 0) map[pair] = collided ? 0x7fffffff : to_int_x86(distance * 1000);
}

static int cost_map(dmf_volume* v, const float* d_poses, int32_t V, int32_t* d_map) {
  const int64_t pairs = (int64_t)V * V;
  if (pairs == 0) return DMF_OK;
  hipLaunchKernelGGL(k_cost_map, dim3((unsigned)((pairs + kCostWaves - 1) / kCostWaves)), dim3(64 * kCostWaves), 0,
                     v->stream, v->geom(), v->d_occ, d_poses, V, d_map);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
}

}  // namespace dmf

using namespace dmf;

extern "C" {

int dmf_reverse_ray_trace_fast(dmf_volume* v, const dmf_camera* cam, const float* poses, int32_t P, int32_t viz,
                               uint8_t* found, int64_t* counts, uint64_t* hashes, int64_t cap) {
  DMF_API_BEGIN
  return reverse_lists(v, cam, poses, P, viz, false, found, counts, hashes, cap);
  DMF_API_END
}

int dmf_reverse_ray_trace(dmf_volume* v, const dmf_camera* cam, const float* poses, int32_t P, int32_t viz,
                          uint8_t* found, int64_t* counts, uint64_t* hashes, int64_t cap) {
  DMF_API_BEGIN
  return reverse_lists(v, cam, poses, P, viz, true, found, counts, hashes, cap);
  DMF_API_END
}

int dmf_reverse_visibility_device(dmf_volume* v, const dmf_camera* cam, const float* d_poses, int32_t P, int32_t viz,
                                  uint64_t* d_visible, uint64_t* d_good, uint64_t* d_stats) {
  DMF_API_BEGIN
  uint64_t *vis, *good;
  int64_t words, nelem;
  DMF_TRY(run_reverse(v, cam, d_poses, P, true, viz, false, &vis, &good, &words, &nelem, nullptr, d_stats));
  const size_t bytes = sizeof(uint64_t) * (size_t)P * words;
  if (bytes) {
    if (d_visible) DMF_HIP(hipMemcpyAsync(d_visible, vis, bytes, hipMemcpyDeviceToDevice, v->stream));
    if (d_good) DMF_HIP(hipMemcpyAsync(d_good, good, bytes, hipMemcpyDeviceToDevice, v->stream));
  }
  return DMF_OK;
  DMF_API_END
}

int dmf_greedy_set_cover_masks_device(dmf_volume* v, const uint64_t* d_masks, int32_t P, int64_t words,
                                      int32_t min_gain, int32_t* selected, int32_t* nselected) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!selected || !nselected || (P > 0 && !d_masks)) return fail(DMF_ERR_INVALID, "null argument");
  if (P < 0 || P > 65535 || words < 0) return fail(DMF_ERR_INVALID, "bad set count / width");
  return greedy_cover(v, d_masks, P, words, min_gain, selected, nselected);
  DMF_API_END
}

int dmf_greedy_set_cover(dmf_volume* v, const dmf_camera* cam, const float* poses, int32_t P, int32_t min_gain,
                         int32_t* selected, int32_t* nselected) {
  DMF_API_BEGIN
  if (!poses || !selected || !nselected) return fail(DMF_ERR_INVALID, "null argument");
  uint64_t *vis, *good;
  int64_t words, nelem;
  DMF_TRY(run_reverse(v, cam, poses, P, false, 0, false, &vis, &good, &words, &nelem, nullptr, nullptr));
  return greedy_cover(v, good, P, words, min_gain, selected, nselected);
  DMF_API_END
}

int dmf_ray_trace(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta, int32_t sparse) {
  DMF_API_BEGIN
  const int s = sparse ? 5 : 1;  // RayTracingEngine.hpp:274-279
  FwdResult res;
  return run_forward(v, cam, pose, kTrace, 10, zdelta, s, s, 1, &res);
  DMF_API_END
}

int dmf_ray_trace_and_classify(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta, int32_t view,
                               int32_t sparse) {
  DMF_API_BEGIN
  const int s = sparse ? 5 : 1;  // :321-326
  FwdResult res;
  return run_forward(v, cam, pose, kClassify, 10, zdelta, s, s, view, &res);
  DMF_API_END
}

int dmf_ray_trace_and_get_minimum(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta,
                                  int32_t sparse, int32_t* minimum) {
  DMF_API_BEGIN
  if (!minimum) return fail(DMF_ERR_INVALID, "null output");
  const int s = sparse ? 10 : 1;  // :233-238
  FwdResult res;
  DMF_TRY(run_forward(v, cam, pose, kMinimum, 5, zdelta, s, s, 1, &res));
  *minimum = res.minimum;
  return DMF_OK;
  DMF_API_END
}

int dmf_ray_trace_and_get_points(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta,
                                 int32_t sparse, uint8_t* found, uint64_t* hashes, int64_t cap, int64_t* n) {
  DMF_API_BEGIN
  return forward_list_api(v, cam, pose, kPoints, zdelta, sparse, found, hashes, cap, n);
  DMF_API_END
}

int dmf_ray_trace_and_get_good_points(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zdelta,
                                      int32_t sparse, uint8_t* found, uint64_t* hashes, int64_t cap, int64_t* n) {
  DMF_API_BEGIN
  return forward_list_api(v, cam, pose, kGoodPoints, zdelta, sparse, found, hashes, cap, n);
  DMF_API_END
}

__global__ void k_first_hit_hash(const int32_t* __restrict__ slot, const uint64_t* __restrict__ hash, int64_t n,
                                 uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = slot[i] >= 0 ? hash[slot[i]] : 0;
}

int dmf_forward_first_hits_device(dmf_volume* v, const dmf_camera* cam, const float* d_poses, int32_t P,
                                  int32_t zstart, int32_t zdelta, int32_t rdelta, int32_t cdelta, int32_t* d_k,
                                  int32_t* d_slot, uint64_t* d_stats) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  DMF_TRY(check_camera(cam));
  if (!d_poses || !d_k || !d_slot) return fail(DMF_ERR_INVALID, "null argument");
  if (P <= 0 || P > 65535) return fail(DMF_ERR_INVALID, "pose count %d out of range [1,65535]", P);
  if (zdelta <= 0 || rdelta <= 0 || cdelta <= 0) return fail(DMF_ERR_INVALID, "bad strides");
  PoseX* tab;
  DMF_TRY(pose_table(v, d_poses, P, true, &tab));
  const int R = (cam->height + rdelta - 1) / rdelta, C = (cam->width + cdelta - 1) / cdelta;
  void* aux;
  DMF_TRY(scratch(v, kScHost2, 64, &aux));
  DMF_HIP(hipMemsetAsync(aux, 0, 64, v->stream));
  unsigned long long* st = nullptr;
  if (d_stats) DMF_TRY(stats_begin(v, &st));
  if (v->knob[DMF_KNOB_FWD_KERNEL] == 1) {
    // per-XCD unit queues (k_forward_x; persistent: the workgroups the device holds at once)
    unsigned int* heads = (unsigned int*)aux + 8;
    const bool skip = fwd_skip(v);
    if (skip) DMF_TRY(ensure_brick_dist(v));
    const void* kfn = skip ? (const void*)k_forward_x<true> : (const void*)k_forward_x<false>;
    int per_cu = 0, ncu = 0;
    DMF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, 256, 0));
    DMF_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, v->device));
    const dim3 grid((unsigned)(std::max(ncu, 8) * std::max(per_cu, 1)));
    if (skip)
      hipLaunchKernelGGL(k_forward_x<true>, grid, dim3(256), 0, v->stream, v->geom(), v->dev(), cam_params(cam), tab, P,
                         zstart, zdelta, rdelta, cdelta, R, C, d_k, d_slot, heads, (unsigned long long*)aux, st);
    else
      hipLaunchKernelGGL(k_forward_x<false>, grid, dim3(256), 0, v->stream, v->geom(), v->dev(), cam_params(cam), tab,
                         P, zstart, zdelta, rdelta, cdelta, R, C, d_k, d_slot, heads, (unsigned long long*)aux, st);
  } else if (v->knob[DMF_KNOB_FWD_KERNEL] == 2) {
    // per-wave lane refill over units of kFwdUnit tiles (k_forward_q)
    const int64_t ntiles = (int64_t)((R + 7) / 8) * ((C + 7) / 8), nunits = (ntiles + kFwdUnit - 1) / kFwdUnit;
    const dim3 grid((unsigned)((nunits + 3) / 4), (unsigned)P);
    if (fwd_skip(v)) {
      DMF_TRY(ensure_brick_dist(v));
      hipLaunchKernelGGL((k_forward_q<true, kFwdUnit, kFwdRefill, kFwdBurst>), grid, dim3(256), 0, v->stream, v->geom(),
                         v->dev(), cam_params(cam), tab, zstart, zdelta, rdelta, cdelta, R, C, d_k, d_slot,
                         (unsigned long long*)aux, st);
    } else {
      hipLaunchKernelGGL((k_forward_q<false, kFwdUnit, kFwdRefill, kFwdBurst>), grid, dim3(256), 0, v->stream,
                         v->geom(), v->dev(), cam_params(cam), tab, zstart, zdelta, rdelta, cdelta, R, C, d_k, d_slot,
                         (unsigned long long*)aux, st);
    }
  } else {
    DMF_LAUNCH_FORWARD(dim3(fwd_blocks(R, C), (unsigned)P), v->geom(), v->dev(), cam_params(cam), tab,
                       zstart, zdelta, rdelta, cdelta, R, C, d_k, d_slot, (unsigned long long*)aux, st);
  }
  DMF_LAUNCH_CHECK();
#if defined(DMF_EXP_STATS)
  if (d_stats) DMF_TRY(stats_end(v, st, d_stats, 4));
#else
  if (d_stats) DMF_TRY(stats_end(v, st, d_stats, 1));
#endif
  return DMF_OK;
  DMF_API_END
}

int dmf_forward_first_hits(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t zstart, int32_t zdelta,
                           int32_t rdelta, int32_t cdelta, int32_t* k_out, uint64_t* hash_out) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  DMF_TRY(check_camera(cam));
  if (!pose || !k_out || !hash_out) return fail(DMF_ERR_INVALID, "null argument");
  if (zdelta <= 0 || rdelta <= 0 || cdelta <= 0) return fail(DMF_ERR_INVALID, "bad strides");
  PoseX* tab;
  DMF_TRY(pose_table(v, pose, 1, false, &tab));
  const int R = (cam->height + rdelta - 1) / rdelta, C = (cam->width + cdelta - 1) / cdelta;
  const int64_t RC = (int64_t)R * C;
  void *kb, *sb, *hb, *aux;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * RC, &kb));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * RC, &sb));
  DMF_TRY(scratch(v, kScOut2, sizeof(uint64_t) * RC, &hb));
  DMF_TRY(scratch(v, kScHost2, 64, &aux));
  DMF_HIP(hipMemsetAsync(aux, 0, 64, v->stream));
  const dim3 grid((unsigned)((RC + 255) / 256));
  DMF_LAUNCH_FORWARD(dim3(fwd_blocks(R, C)), v->geom(), v->dev(), cam_params(cam), tab, zstart, zdelta, rdelta, cdelta, R, C,
                     (int32_t*)kb, (int32_t*)sb, (unsigned long long*)aux, nullptr);
  DMF_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_first_hit_hash, grid, dim3(256), 0, v->stream, (const int32_t*)sb, v->d_hash, RC,
                     (uint64_t*)hb);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(k_out, kb, sizeof(int32_t) * RC, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipMemcpyAsync(hash_out, hb, sizeof(uint64_t) * RC, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_ray_trace_volume(dmf_volume* v, const dmf_camera* cam, const float* pose, int32_t* depth_out) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  DMF_TRY(check_camera(cam));
  if (!pose) return fail(DMF_ERR_INVALID, "null pose");
  DMF_TRY(ensure_enumeration(v));
  PoseX* tab;
  DMF_TRY(pose_table(v, pose, 1, false, &tab));
  const int64_t HW = (int64_t)cam->height * cam->width;
  void *zb, *aux;
  DMF_TRY(scratch(v, kScOut0, sizeof(int) * HW, &zb));
  DMF_TRY(scratch(v, kScHost2, 64, &aux));
  DMF_HIP(hipMemsetD32Async((hipDeviceptr_t)zb, 0x7fffffff, HW, v->stream));
  DMF_HIP(hipMemsetAsync(aux, 0, 64, v->stream));
  EnumList el{v->d_axes, {v->nax[0], v->nax[1], v->nax[2]}, v->d_enum};
  const int64_t n = v->nenum;
  if (n > 0) {
    const dim3 grid((unsigned)((n + 255) / 256));
    for (int pass = 0; pass < 2; ++pass) {
      hipLaunchKernelGGL(k_zbuffer, grid, dim3(256), 0, v->stream, v->geom(), v->dev(), cam_params(cam), tab, el, n,
                         pass, (int*)zb, (unsigned long long*)aux);
      DMF_LAUNCH_CHECK();
    }
  }
  unsigned long long hz = 0;
  DMF_HIP(hipMemcpyAsync(&hz, aux, sizeof(hz), hipMemcpyDeviceToHost, v->stream));
  if (depth_out) {
    void* ob;
    DMF_TRY(scratch(v, kScOut1, sizeof(int) * HW, &ob));
    hipLaunchKernelGGL(k_zbuf_out, dim3((unsigned)((HW + 255) / 256)), dim3(256), 0, v->stream, (const int*)zb, HW,
                       (int*)ob);
    DMF_LAUNCH_CHECK();
    DMF_HIP(hipMemcpyAsync(depth_out, ob, sizeof(int) * HW, hipMemcpyDeviceToHost, v->stream));
  }
  DMF_HIP(hipStreamSynchronize(v->stream));
  v->hazards += (int64_t)hz + v->enum_hazards;
  return DMF_OK;
  DMF_API_END
}

int dmf_will_collide(dmf_volume* v, const float* a, const float* b, int64_t n, uint8_t* collided) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (n < 0 || (n > 0 && (!a || !b || !collided))) return fail(DMF_ERR_INVALID, "bad arguments");
  if (n == 0) return DMF_OK;
  for (int64_t i = 0; i < 3 * n; ++i)
    if (!std::isfinite(a[i]) || !std::isfinite(b[i]))
      return fail(DMF_ERR_INVALID, "non-finite segment endpoint (the reference never terminates)");
  void *da, *db, *dout;
  DMF_TRY(scratch(v, kScHost0, sizeof(float) * 3 * n, &da));
  DMF_TRY(scratch(v, kScHost1, sizeof(float) * 3 * n, &db));
  DMF_TRY(scratch(v, kScOut0, n, &dout));
  DMF_HIP(hipMemcpyAsync(da, a, sizeof(float) * 3 * n, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(db, b, sizeof(float) * 3 * n, hipMemcpyHostToDevice, v->stream));
  hipLaunchKernelGGL(k_will_collide, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream, v->geom(), v->d_occ,
                     (const float*)da, (const float*)db, n, (uint8_t*)dout);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(collided, dout, n, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_collision_cost_map(dmf_volume* v, const float* poses, int32_t V, int32_t* map) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (V < 0 || V > kMaxCostPoses || (V > 0 && (!poses || !map))) return fail(DMF_ERR_INVALID, "bad arguments");
  if (V == 0) return DMF_OK;
  for (int64_t i = 0; i < V; ++i)
    for (int k = 3; k < 12; k += 4)
      if (!std::isfinite(poses[12 * i + k]))
        return fail(DMF_ERR_INVALID, "non-finite camera centre (the reference never terminates)");
  const int64_t pairs = (int64_t)V * V;
  void *dp, *dm;
  DMF_TRY(scratch(v, kScPoses, sizeof(float) * 12 * V, &dp));
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * pairs, &dm));
  DMF_HIP(hipMemcpyAsync(dp, poses, sizeof(float) * 12 * V, hipMemcpyHostToDevice, v->stream));
  DMF_TRY(cost_map(v, (const float*)dp, V, (int32_t*)dm));
  DMF_HIP(hipMemcpyAsync(map, dm, sizeof(int32_t) * pairs, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_collision_cost_map_device(dmf_volume* v, const float* d_poses, int32_t V, int32_t* d_map) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (V < 0 || V > kMaxCostPoses || (V > 0 && (!d_poses || !d_map))) return fail(DMF_ERR_INVALID, "bad arguments");
  return cost_map(v, d_poses, V, d_map);
  DMF_API_END
}

}  // extern "C"
