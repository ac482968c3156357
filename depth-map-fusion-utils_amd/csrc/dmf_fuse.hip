// dmf_fuse.hip — per-ray 3D-DDA log-odds depth fusion on gfx950.
//
// Not in the reference: the ray endpoint is the reference's own
// back-projection (Camera.hpp:24-45 projectPoint + transformPoints, bit-exact) and
// its cell is the reference binning (Volume.hpp:150-156, 199-228); the traversal
// between camera centre and endpoint is an exact integer 3D-DDA (fixed-point
// endpoints, crossing times compared by cross-multiplication), so GPU and CPU
// oracle visit the same cells and the int32 hit/miss counts are bit-identical.
//
// Device atomics execute at the memory side, one request per distinct 64-B line per
// wave instruction (≈2e10 requests/s chip-wide, MI355X_MICROARCH.md §Global float
// atomics), so one atomic per cell update costs ~320 ms per launch.  LDS aggregation
// of each 8x8 ray packet's updates (≈8.2 rays share a cell per round) and a tiled
// counter layout (2x2x4-cell tiles = one 64-B line) bring that to 2.3e8 requests;
// what remains binding is instruction issue.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "dmf_brick.hpp"
#include "dmf_host.hpp"

namespace dmf {

constexpr int64_t kQ = 256;  // fixed-point sub-cell resolution (1/256 cell)

__device__ inline int64_t clampi(int64_t v, int64_t lo, int64_t hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ inline int32_t clamp32(int32_t v, int32_t lo, int32_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

// (int64_t) floor(x) as the oracle's x86 conversion gives it (cvttsd2si: NaN and |x| >= 2^63
// -> INT64_MIN), saturated to +-2^30: a v_cvt_i32_f64 and a select instead of the int64
// conversion sequence.  Every use clamps the result into [0, n * kQ) with n * kQ <= 2^19
// (fusion grids <= 2048 cells per axis, check_fuse), so the clamped values are identical.
__device__ inline int32_t floor_sat32(double x) {
  const double f = floor(x);
  return fabs(f) < 9223372036854775808.0 ? (int32_t)fmin(fmax(f, -1073741824.0), 1073741824.0) : -(1 << 30);
}

__device__ inline void atomic_add_dev(int32_t* p, int32_t v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Tiled counter layout: 2x2x4-cell tiles (x, y, z), 16 int32 = one 64-B line, tiles
// x-major over the padded grid; inside a tile ((x&1)*2 + (y&1))*4 + (z&3).
struct Tiles {
  uint32_t ny, nz;  // tiles along y and z
};
__host__ __device__ inline Tiles tiles_of(const int n[3]) {
  return Tiles{(uint32_t)(n[1] + 1) >> 1, (uint32_t)(n[2] + 3) >> 2};
}
__host__ __device__ inline uint32_t tile_base(const Tiles& t, int tx, int ty, int tz) {
  return (((uint32_t)tx * t.ny + (uint32_t)ty) * t.nz + (uint32_t)tz) << 4;
}
__host__ __device__ inline uint32_t tiled_index(const Tiles& t, int x, int y, int z) {
  return tile_base(t, x >> 1, y >> 1, z >> 2) | (uint32_t)(((x & 1) << 3) | ((y & 1) << 2) | (z & 3));
}
inline size_t tiled_cells(const int n[3]) {
  return (size_t)((n[0] + 1) >> 1) * (size_t)((n[1] + 1) >> 1) * (size_t)((n[2] + 3) >> 2) * 16;
}

// Per-ray DDA state after setup (exact integer walk).
//
// The oracle compares next-crossing times T_a = h_a * prod_{b != a} |dq_b| in 64 bits.
// For a pair of moving axes, sign(T_a - T_b) = sign(E_ab) with
// E_ab = h_a |dq_b| - h_b |dq_a| (T_a - T_b divided by the third axis' |dq|), and
// because both next crossings lie within one cell interval of the current time,
// |E_ab| < (2Q + 1) max|dq| <= 2^29 for grids up to 2048 cells per axis: the walk
// runs on three int32 differences.  A step along axis a adds 2Q|dq_b| to E_ab (and
// subtracts 2Q|dq_a| from E_ba).  A pair with a non-moving axis holds a constant that
// never lets that axis win.
struct Ray {
  int c[3];        // current cell
  int st[3];       // step direction per axis (-1, 0, +1)
  int32_t E01, E02, E12;  // crossing-time differences (see above)
  int32_t K[3];    // 2Q |dq_a|
  int left;        // remaining cell updates (misses + final), 0 = inactive
  bool end_inside;
};
constexpr int32_t kNever = 1 << 30;  // |E| of a pair with a non-moving axis

// One DDA selection (earliest crossing; ties x before y before z): s2 = z, s1 = y, else x.
__device__ inline void dda_select(int32_t& E01, int32_t& E02, int32_t& E12, int32_t K0, int32_t K1, int32_t K2,
                                  bool& s0, bool& s1, bool& s2) {
  const bool b10 = E01 > 0;             // T1 < T0
  s2 = (b10 ? E12 : E02) > 0;            // T2 < min(T0, T1)
  s1 = !s2 && b10;
  s0 = !s2 && !b10;
  E01 += s0 ? K1 : (s1 ? -K0 : 0);
  E02 += s0 ? K2 : (s2 ? -K0 : 0);
  E12 += s1 ? K2 : (s2 ? -K1 : 0);
}

// (x - min) / delta in double (oracle.cpp dda_ray); a power-of-two delta divides exactly
// as a multiplication by its (exact) reciprocal, as in bin_axis
__device__ inline double grid_coord(const Geom& g, int a, float x) {
  const double t = (double)x - g.mn[a];
  return g.pow2 ? t * g.inv[a] : t / g.dl[a];
}

// Grid coordinates of the ray origin.
__device__ inline void grid_origin(const Geom& g, const float O[3], double go[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) go[a] = grid_coord(g, a, O[a]);
}

// Clip O->E to the grid and quantise the clipped endpoints to 1/256 cell (clamped
// into their cells).  Mirrors oracle.cpp dda_ray() lines 752-780 operation for
// operation; go = grid_origin(O) (one per pose: callers hoist it).  Returns false when
// the ray misses the grid.
// A ray that ends inside the grid has t1 overwritten by 1, so of each axis' two slab
// quotients only the entry one, min(ta, tb), matters, and only when it can exceed t0 >= 0:
// (0 - go) / D for D > 0, which is <= 0 unless go < 0, and (n - go) / D for D < 0, which is
// <= 0 unless go > n (division is monotone and keeps the sign) -- so the other divisions
// are skipped with identical t0 and t1.
__device__ inline bool dda_quantize_go(const Geom& g, const double go[3], const float E[3], bool end_inside,
                                       int64_t qs[3], int64_t qe[3]) {
  double ge[3], D[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    ge[a] = grid_coord(g, a, E[a]);
    D[a] = ge[a] - go[a];
  }
  double t0 = 0.0, t1 = 1.0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (D[a] == 0.0) {
      if (go[a] < 0.0 || go[a] >= (double)g.n[a]) return false;
    } else if (end_inside) {
      if (D[a] > 0.0 ? go[a] < 0.0 : go[a] > (double)g.n[a]) {
        const double lo = (D[a] > 0.0 ? 0.0 - go[a] : (double)g.n[a] - go[a]) / D[a];
        if (lo > t0) t0 = lo;
      }
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
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const double gs = go[a] + t0 * D[a];
    const double gx = end_inside ? ge[a] : go[a] + t1 * D[a];
    const int32_t n = (int32_t)g.n[a], Q = (int32_t)kQ;
    const int32_t cs = clamp32(floor_sat32(gs), 0, n - 1);
    const int32_t ce = end_inside ? floor_sat32(ge[a]) : clamp32(floor_sat32(gx), 0, n - 1);
    qs[a] = clamp32(floor_sat32(gs * (double)kQ), cs * Q, cs * Q + Q - 1);
    qe[a] = clamp32(floor_sat32(gx * (double)kQ), ce * Q, ce * Q + Q - 1);
  }
  return true;
}

__device__ inline bool dda_quantize(const Geom& g, const float O[3], const float E[3], bool end_inside, int64_t qs[3],
                                    int64_t qe[3]) {
  double go[3];
  grid_origin(g, O, go);
  return dda_quantize_go(g, go, E, end_inside, qs, qe);
}

// Clip/quantise, then set up the walk state (oracle.cpp dda_ray lines 781-806).
__device__ inline bool dda_setup(const Geom& g, const float O[3], const float E[3], bool end_inside, Ray& R) {
  int64_t qs[3], qe[3];
  if (!dda_quantize(g, O, E, end_inside, qs, qe)) return false;
  int64_t cs[3], ce[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    cs[a] = qs[a] / kQ;  // qs, qe >= 0 and clamped into their cells
    ce[a] = qe[a] / kQ;
  }
  int64_t adq[3], h[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int64_t dq = qe[a] - qs[a];
    adq[a] = dq < 0 ? -dq : dq;
    R.st[a] = ce[a] > cs[a] ? 1 : (ce[a] < cs[a] ? -1 : 0);
    // next crossing numerator in half fixed-point units (oracle.cpp dda_ray)
    h[a] = R.st[a] > 0 ? 2 * ((cs[a] + 1) * kQ - qs[a]) : 2 * (qs[a] - cs[a] * kQ) + 1;
    R.K[a] = (int32_t)(2 * kQ * adq[a]);
  }
  auto pair = [&](int a, int b) -> int32_t {
    if (R.st[a] && R.st[b]) return (int32_t)(h[a] * adq[b] - h[b] * adq[a]);
    return R.st[a] ? -kNever : (R.st[b] ? kNever : 0);
  };
  R.E01 = pair(0, 1);
  R.E02 = pair(0, 2);
  R.E12 = pair(1, 2);
  const int nsteps = (int)((ce[0] > cs[0] ? ce[0] - cs[0] : cs[0] - ce[0]) + (ce[1] > cs[1] ? ce[1] - cs[1] : cs[1] - ce[1]) +
                           (ce[2] > cs[2] ? ce[2] - cs[2] : cs[2] - ce[2]));
  R.c[0] = (int)cs[0];
  R.c[1] = (int)cs[1];
  R.c[2] = (int)cs[2];
  R.left = nsteps + 1;
  R.end_inside = end_inside;
  return true;
}

// The acceptance of integratePointCloud(cloud, normals) (Volume.hpp:199-228):
// validPoints(E) && validCoords(getVoxel(E)).  validPoints as float compares (vlo / vhi,
// dmf_geom.hpp; a NaN endpoint, from a non-finite pose, is outside: the reference's getVoxel
// gives INT_MIN for it, which validCoords rejects), then getVoxel in double.
__device__ inline bool endpoint_inside(const Geom& g, const float E[3]) {
  const bool in = (E[0] >= g.vlo[0]) & (E[0] <= g.vhi[0]) & (E[1] >= g.vlo[1]) & (E[1] <= g.vhi[1]) &
                  (E[2] >= g.vlo[2]) & (E[2] <= g.vhi[2]);
  if (!in) return false;
  return valid_coords(g, bin_axis(g, 0, E[0]), bin_axis(g, 1, E[1]), bin_axis(g, 2, E[2]));
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
  const bool inside = endpoint_inside(g, E);
  const float O[3] = {T.f[3], T.f[7], T.f[11]};
  if (!dda_setup(g, O, E, inside, R)) { R.left = 0; return 0; }
  return R.left;
}

// The brick path's ray record: pixel_ray up to the quantised endpoints, with the pose's grid
// origin already computed (go = grid_origin of poses[p]'s translation; d < 0: outside the frame).
__device__ inline bool pixel_quant_go(const Geom& g, const CamP& cam, int d, const float Tf[12], const double go[3],
                                      int r, int c, int dmin, int dmax, int64_t qs[3], int64_t qe[3], bool& inside,
                                      bool& valid) {
  valid = false;
  inside = false;
  if (d < 0 || !(d >= dmin && d < dmax)) return false;
  valid = true;
  float pc[3], E[3];
  project(cam, r, c, d, pc);
  xform(Tf, pc[0], pc[1], pc[2], E);
  inside = endpoint_inside(g, E);
  return dda_quantize_go(g, go, E, inside, qs, qe);
}

__device__ inline int pixel_depth(const CamP& cam, const uint16_t* __restrict__ depth, int p, int r, int c) {
  return (r >= cam.H || c >= cam.W) ? -1 : (int)depth[((int64_t)p * cam.H + r) * cam.W + c];
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


// Packed (hi | (0xffff - lo) << 16) extent reduction over the wave: one DPP max
// chain of v_pk_max_u16 per axis gives both max(hi) and min(lo).  0 = no lane.
typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ inline uint32_t pkmax(uint32_t a, uint32_t b) {
  us2 x = __builtin_bit_cast(us2, a), y = __builtin_bit_cast(us2, b);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}
__device__ inline uint32_t wave_pkmax(uint32_t v) {
  v = pkmax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = pkmax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = pkmax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = pkmax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = pkmax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = pkmax(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ inline int lane_prefix(uint64_t mask) {  // set lanes of mask below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// q = i / b for 0 <= i < 2^20, 1 <= b < 2^16 from a float reciprocal plus one
// correction step (the float quotient is within 1 of the true one).
__device__ inline int small_div(int i, int b, float rb, int& rem) {
  int q = (int)((float)i * rb);
  int r = i - q * b;
  if (r < 0) { --q; r += b; }
  if (r >= b) { ++q; r -= b; }
  rem = r;
  return q;
}

__device__ inline int popc(uint32_t v) { return __builtin_popcount(v); }
__device__ inline int popc(uint64_t v) { return __builtin_popcountll(v); }

// Production fusion kernel.  One 64-lane workgroup per 8x8 pixel
// packet of one frame; the wave runs its own rounds (no cross-wave barriers).  Per
// round of kS cell updates per ray:
//  1. walk: kS unconditional exact-DDA steps (dda_select, ties x < y < z), recording
//     2-bit axis codes.  A lane with fewer advances finishes in this round (or has
//     finished): its walk state is never read again, codes past its advance count
//     are masked off, and the crossing-time invariants keep |E| bounded past the
//     ray's end, so no per-step predication is needed;
//  2. box: exact extents of the round's miss cells (per-axis advance counts from
//     popcounts of the codes), wave-reduced with packed DPP maxima; the LDS box is
//     stored LINEARLY over those extents (x-major, z fastest, no padding);
//  3. replay: each lane replays its miss cells into LDS adds, ROTATED to start at a
//     lane-dependent cell P_o: moves o..nm-2, then code 3 = jump P_{nm-1} -> P_0, then
//     moves 0..o-2.  Neighbouring rays of a packet sit in one cell at the same step;
//     rotation puts them in different cells, cutting same-bank LDS atomics from ~9.6x
//     to ~3.7x the conflict-free cycles (tools/sim_fusion_lds.py; SQ_LDS_BANK_CONFLICT
//     1.89e9 -> 0.69e9 per launch);
//  4. flush: an in-order scan compacts the non-zero cells (ballot + mbcnt) into a list
//     kept in the box's own LDS; one device atomic per listed cell.  Box order puts
//     ~4.4 cells of one 64-B tiled counter line into each wave instruction
//     (tools/sim_fusion_flush_order.py; tile order: 4.85), which is one memory-side request.
// A round whose box exceeds kBox cells adds its misses to HBM directly.  Hits (one per
// ray) go straight to HBM.  Counts are exact integers: bit-identical to the oracle.
template <int kS, int kBox>
__global__ __launch_bounds__(64) void k_fuse_l(Geom g, CamP cam, const uint16_t* __restrict__ depth,
                                               const PoseX* __restrict__ poses, int dmin, int dmax, int packets_x,
                                               int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                               unsigned long long* __restrict__ stats) {
  static_assert(kS <= 31, "2-bit codes of up to 31 advances with a 64-bit field mask");
  using CodeT = typename std::conditional<(kS <= 15), uint32_t, uint64_t>::type;
  constexpr CodeT kOne = 1, kOdd = (CodeT)0x5555555555555555ull, kEven = (CodeT)0xAAAAAAAAAAAAAAAAull;
  static_assert(kBox % 256 == 0 && kBox <= 65536, "box scanned 256 cells per iteration, 16-bit indices");
  static_assert(kBox >= 64 * kS, "the non-zero list lives in the box");
  stats = stat_slot(stats);
  __shared__ __attribute__((aligned(16))) int box[kBox];
  uint32_t* nzl = (uint32_t*)box;
  const int l = threadIdx.x;
  for (int i = l; i < kBox; i += 64) box[i] = 0;
  const Tiles tl = tiles_of(g.n);
  const int pr = (blockIdx.x / packets_x) * 8 + (l >> 3), pc = (blockIdx.x % packets_x) * 8 + (l & 7);
  Ray R;
  bool valid;
  const unsigned long long upd = (unsigned long long)pixel_ray(g, cam, depth, poses, blockIdx.y, pr, pc, dmin, dmax,
                                                               R, valid);
  const unsigned long long nvalid = valid ? 1 : 0, nhit = (R.left > 0 && R.end_inside) ? 1 : 0;
  int32_t E01 = R.E01, E02 = R.E02, E12 = R.E12;
  const int32_t K0 = R.K[0], K1 = R.K[1], K2 = R.K[2];
  const int st0 = R.st[0], st1 = R.st[1], st2 = R.st[2];
  int c0 = R.c[0], c1 = R.c[1], c2 = R.c[2], left = R.left;
  const bool end_inside = R.end_inside;
  const int rot = ((l & 7) + 3 * (l >> 3)) % kS;  // replay start offset in a full round
  unsigned long long nflush = 0, nround_lds = 0, nround_direct = 0;
  while (__builtin_amdgcn_ballot_w64(left > 0)) {
    const int rem = left < kS ? left : kS;
    const bool fin = rem == left && rem > 0;
    const int nadv = fin ? rem - 1 : rem;
    CodeT codes = 0;
#pragma unroll
    for (int k = 0; k < kS; ++k) {
      bool s0, s1, s2;
      dda_select(E01, E02, E12, K0, K1, K2, s0, s1, s2);
      codes |= (CodeT)(s2 ? 2u : (s1 ? 1u : 0u)) << (2 * k);
    }
    const CodeT fmask = (kOne << (2 * nadv)) - 1u;
    const int n2 = popc(codes & fmask & kEven);
    const int n1 = popc(codes & fmask & kOdd);
    const int n0 = nadv - n1 - n2;
    const int e0 = c0 + st0 * n0, e1 = c1 + st1 * n1, e2 = c2 + st2 * n2;
    const int nm = (fin && end_inside) ? rem - 1 : rem;  // miss cells of this round
    int m0 = e0, m1 = e1, m2 = e2;                       // last miss cell
    if (nm > 0 && nadv > 0 && (!fin || end_inside)) {
      const uint32_t lc = (uint32_t)(codes >> (2 * (nadv - 1))) & 3u;
      m0 -= lc == 0u ? st0 : 0;
      m1 -= lc == 1u ? st1 : 0;
      m2 -= lc == 2u ? st2 : 0;
    }
    uint32_t px = 0, py = 0, pz = 0;
    if (nm > 0) {
      px = (uint32_t)max(c0, m0) | ((0xffffu - (uint32_t)min(c0, m0)) << 16);
      py = (uint32_t)max(c1, m1) | ((0xffffu - (uint32_t)min(c1, m1)) << 16);
      pz = (uint32_t)max(c2, m2) | ((0xffffu - (uint32_t)min(c2, m2)) << 16);
    }
    const uint32_t rx = wave_pkmax(px), ry = wave_pkmax(py), rz = wave_pkmax(pz);
    if (rx != 0u) {
      const int ax = 0xffff - (int)(rx >> 16), ay = 0xffff - (int)(ry >> 16), az = 0xffff - (int)(rz >> 16);
      const int bx = (int)(rx & 0xffffu) - ax + 1, by = (int)(ry & 0xffffu) - ay + 1, bz = (int)(rz & 0xffffu) - az + 1;
      const int byz = by * bz;
      const int64_t ncell_box = (int64_t)bx * byz;
      if (ncell_box <= kBox) {
        ++nround_lds;
        // byte offsets into the box; per-axis byte strides along this ray
        const int dX = st0 * byz * 4, dY = st1 * bz * 4, dZ = st2 * 4;
        const int cur0 = (((c0 - ax) * by + (c1 - ay)) * bz + (c2 - az)) * 4;
        int cur = cur0, dJ = 0;
        CodeT rc = codes;
        if (nm > 1) {
          int o = rot;
          if (o >= nm) small_div(o, nm, __builtin_amdgcn_rcpf((float)nm), o);
          const CodeT lo = (kOne << (2 * o)) - 1u;
          const int q2 = popc(codes & lo & kEven);
          const int q1 = popc(codes & lo & kOdd);
          cur += ((o - q1 - q2) * st0 * byz + q1 * st1 * bz + q2 * st2) * 4;
          dJ = cur0 - (((m0 - ax) * by + (m1 - ay)) * bz + (m2 - az)) * 4;
          const CodeT a = (codes >> (2 * o)) & ((kOne << (2 * (nm - 1 - o))) - 1u);
          const CodeT b = o > 1 ? (codes & ((kOne << (2 * (o - 1))) - 1u)) << (2 * (nm - o)) : (CodeT)0;
          rc = a | ((CodeT)3 << (2 * (nm - 1 - o))) | b;
        }
        const bool full = __builtin_amdgcn_ballot_w64(nm != kS) == 0;
        char* const b8 = (char*)box;
#pragma unroll
        for (int k = 0; k < kS; ++k) {
          if (full || k < nm) atomicAdd((int*)(b8 + cur), 1);
          if (k + 1 < kS) {
            const uint32_t cd = (uint32_t)(rc >> (2 * k)) & 3u;
            cur += cd == 3u ? dJ : (cd == 2u ? dZ : (cd == 1u ? dY : dX));
          }
        }
        __syncthreads();  // single-wave workgroup: orders the LDS adds before the scan
        const int nb = (int)ncell_box;
        int nnz = 0;
        for (int i0 = 0; i0 < nb; i0 += 256) {
          int v[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int i = i0 + 64 * u + l;
            v[u] = i < nb ? box[i] : 0;
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int i = i0 + 64 * u + l;
            const uint64_t b = __builtin_amdgcn_ballot_w64(v[u] != 0);
            if (i < nb) box[i] = 0;
            if (v[u]) nzl[nnz + lane_prefix(b)] = (uint32_t)i | ((uint32_t)v[u] << 16);
            nnz += __builtin_popcountll(b);
          }
        }
        __syncthreads();
        const float ryz = __builtin_amdgcn_rcpf((float)byz), rz1 = __builtin_amdgcn_rcpf((float)bz);
        for (int e = l; e < nnz; e += 64) {
          const uint32_t en = nzl[e];
          int rr, qz;
          const int qx = small_div((int)(en & 0xffffu), byz, ryz, rr);
          const int qy = small_div(rr, bz, rz1, qz);
          ++nflush;
          atomic_add_dev(&misses[tiled_index(tl, ax + qx, ay + qy, az + qz)], (int)(en >> 16));
        }
        __syncthreads();
        for (int e = l; e < nnz; e += 64) box[e] = 0;
        __syncthreads();
      } else {
        ++nround_direct;
        int x = c0, y = c1, z = c2;
#pragma unroll
        for (int k = 0; k < kS; ++k) {
          if (k < nm) atomic_add_dev(&misses[tiled_index(tl, x, y, z)], 1);
          const uint32_t cd = (uint32_t)(codes >> (2 * k)) & 3u;
          x += cd == 0u ? st0 : 0;
          y += cd == 1u ? st1 : 0;
          z += cd == 2u ? st2 : 0;
        }
      }
    }
    if (fin && end_inside) atomic_add_dev(&hits[tiled_index(tl, e0, e1, e2)], 1);
    c0 = e0; c1 = e1; c2 = e2;
    left -= rem;
  }
  if (stats) {
    wave_stats(stats, upd, nvalid, nhit);
    for (int o = 32; o > 0; o >>= 1) nflush += __shfl_down(nflush, o, 64);
    if (l == 0) {
      if (nflush) atomicAdd(&stats[6], nflush);
      if (nround_lds) atomicAdd(&stats[4], nround_lds);
      if (nround_direct) atomicAdd(&stats[5], nround_direct);
    }
  }
}

// ------------------------------------------------------------ brick-owned fusion
// (exact decomposition in dmf_brick.hpp, checked on the CPU by
// tools/brick_selftest.cpp).  The grid is cut into 32^3-cell bricks.  One fusion
// batch runs four kernels:
//  A  k_bk_rays   — per pixel: back-projection, clip, quantised ray record (16 B);
//                   the coarse walk over brick boundaries counts (ray, brick) pairs per
//                   brick (LDS histogram, one device atomic per brick per workgroup);
//  S  k_bk_scan   — brick offsets and the part table (parts of <= 65535 pairs);
//  B  k_bk_pairs  — the coarse walk again: per pair a self-contained 24-B record (the
//                   fine walk's int32 state at the brick entry, entry cell, cells in
//                   the brick), written into the brick's list (ranges reserved per
//                   workgroup);
//  F  k_bk_fuse   — persistent, one 1024-lane workgroup per CU, 128 KiB of LDS
//                   counters (16-bit misses | 16-bit hits per cell) for the brick of
//                   its part: each lane restarts the exact int32 walk at its pair's
//                   entry event and adds one LDS count per cell; the part's counters
//                   are then added to HBM once (one device atomic per non-zero cell and
//                   counter).  No device atomic per update.
namespace bk = dmf::brick;

struct BkGeom {
  int nb[3];    // bricks per axis
  int nbricks;
};

// phase F's workgroup: 1024 lanes over a 32^3 brick (one per CU by LDS); an experiment build
// with 16^3 bricks (DMF_EXP_BRICK_LOG = 4) runs 256-lane workgroups, several per CU
constexpr int kBkThreads = bk::kLog == 5 ? 1024 : 256;
// passes A/B: 256-lane workgroups (several per CU) while the LDS brick histogram is small;
// 1024 lanes when it is large (over 8192 bricks: one workgroup per CU by LDS)
constexpr int kBkPassThreads = 256, kBkPassThreadsBig = 1024, kBkBigHist = 8192;
constexpr int kBkScanMax = 32768;  // bricks the scan holds in LDS (the brick path: <= 1024 cells per axis)
constexpr uint32_t kBkPartMax = 65535;  // pairs per part: 16-bit miss / hit fields never carry
// LDS box of phase F: cell (x, y, z) of the brick at word x*kSx + y*kSy + z.  The skew
// (kSy = 33, kSx = 32*33 + 1) puts the cell in bank (x + y + z) mod 32 instead of z alone,
// so lanes on different rows/columns of one z-plane do not collide.
constexpr int kBkSy = bk::kB + 1, kBkSx = bk::kB * kBkSy + 1;
constexpr int kBkBoxWords = bk::kB * kBkSx;               // 33824 words
// (k_bk_fuse declares the box statically: 135,312 B of the CU's 160 KiB)

// LDS byte offset of brick-local cell (x, y, z) in phase F's skewed box (< 2^18)
__host__ __device__ constexpr uint32_t bk_lds_off(uint32_t x, uint32_t y, uint32_t z) {
  return (x * kBkSx + y * kBkSy + z) * 4u;
}

// word index of the same cell (< 33824: 16 bits in the pair record)
__host__ __device__ constexpr uint32_t bk_lds_word(uint32_t x, uint32_t y, uint32_t z) { return x * kBkSx + y * kBkSy + z; }

__device__ inline int bk_index(const BkGeom& bg, int x, int y, int z) {
  return bk::mul24(bk::mul24(x, bg.nb[1]) + y, bg.nb[2]) + z;  // (24-bit multiplies, dmf_brick.hpp mul24)
}

// Coarse walk of one ray: calls f(brick index, axis of the boundary crossed to enter it
// (-1 for the first brick), brick coordinates) for every brick it passes, in order.
template <class F>
__device__ inline void bk_coarse(const BkGeom& bg, const bk::QRay& R, F&& f) {
  int b0 = R.cs[0] >> bk::kLog, b1 = R.cs[1] >> bk::kLog, b2 = R.cs[2] >> bk::kLog;
  f(bk_index(bg, b0, b1, b2), -1, b0, b1, b2);
  bk::Coarse cw;
  bk::coarse_init(R, cw);
  for (int t = 0; t < cw.total; ++t) {
    const int a = bk::coarse_next(cw);
    b0 += a == 0 ? R.st[0] : 0;
    b1 += a == 1 ? R.st[1] : 0;
    b2 += a == 2 ? R.st[2] : 0;
    f(bk_index(bg, b0, b1, b2), a, b0, b1, b2);
  }
}

// Wave-aggregated LDS histogram add: the lanes of a packet walk near-parallel rays and
// name the same brick at the same coarse step, so one atomic per distinct brick among
// the active lanes replaces a same-address atomic per lane (which the LDS serialises).
// Callable from divergent code: the loop runs over the currently active lanes.
template <bool H16 = false>
__device__ inline void hist_add_agg(uint32_t* hist, int b) {
  uint64_t rem = __builtin_amdgcn_ballot_w64(true);
  const int l = (int)(threadIdx.x & 63);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const int bl = __builtin_amdgcn_readlane(b, leader);
    const uint64_t same = __builtin_amdgcn_ballot_w64(b == bl) & rem;
    if (l == leader) {
      if constexpr (H16) atomicAdd(&hist[bl >> 1], (uint32_t)__builtin_popcountll(same) << ((bl & 1) << 4));
      else atomicAdd(&hist[bl], (uint32_t)__builtin_popcountll(same));
    }
    rem &= ~same;
  }
}

// hist_add_agg's common case in one step: the lanes naming the first active lane's brick add
// with one atomic of that lane, the rest (rare: a packet's near-parallel rays cross the same
// bricks at the same step) each with their own -- no loop over the distinct bricks.
template <bool H16 = false>
__device__ inline void hist_add_first(uint32_t* hist, int b) {
  const int b0 = __builtin_amdgcn_readfirstlane(b);
  const uint64_t same = __builtin_amdgcn_ballot_w64(b == b0);
  const int l = (int)(threadIdx.x & 63);
  uint32_t* w;
  uint32_t n;
  if (b == b0) {
    if (l != __builtin_ctzll(same)) return;
    w = H16 ? &hist[b0 >> 1] : &hist[b0];
    n = (uint32_t)__builtin_popcountll(same);
  } else {
    w = H16 ? &hist[b >> 1] : &hist[b];
    n = 1u;
  }
  const int bb = b == b0 ? b0 : b;
  atomicAdd(w, H16 ? n << ((bb & 1) << 4) : n);
}

// Pass A's hashed histogram (grids over kBkBigHist bricks): open addressing
// over `mask + 1` words of (brick << 16 | 16-bit count); a workgroup touches a few hundred of
// the up to 32768 bricks, so 8 KB of LDS replace the 64-KB direct table and pass A fits beside
// phase F's box.  Returns false when the table is full (the workgroup is then redone with the
// direct table by k_bk_rays_recover).
constexpr uint32_t kHashEmpty = 0xffff0000u;  // key 0xffff: no brick (bricks < 32768)
__device__ inline bool hash_add(uint32_t* tab, uint32_t mask, int shift, uint32_t b, uint32_t n) {
  uint32_t h = (b * 2654435761u) >> shift;
  for (uint32_t k = 0; k <= mask; ++k) {
    const uint32_t old = atomicCAS(&tab[h], kHashEmpty, b << 16 | n);
    if (old == kHashEmpty) return true;
    if ((old >> 16) == b) {
      atomicAdd(&tab[h], n);
      return true;
    }
    h = (h + 1) & mask;
  }
  return false;
}

// hist_add_agg into the hashed histogram; sets *ovf when an insert finds the table full
__device__ inline void hash_add_agg(uint32_t* tab, uint32_t mask, int shift, int b, uint32_t* ovf) {
  uint64_t rem = __builtin_amdgcn_ballot_w64(true);
  const int l = (int)(threadIdx.x & 63);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const int bl = __builtin_amdgcn_readlane(b, leader);
    const uint64_t same = __builtin_amdgcn_ballot_w64(b == bl) & rem;
    if (l == leader && !hash_add(tab, mask, shift, (uint32_t)bl, (uint32_t)__builtin_popcountll(same))) *ovf = 1u;
    rem &= ~same;
  }
}

// hash_add_agg in one step, as hist_add_first
__device__ inline void hash_add_first(uint32_t* tab, uint32_t mask, int shift, int b, uint32_t* ovf) {
  const int b0 = __builtin_amdgcn_readfirstlane(b);
  const uint64_t same = __builtin_amdgcn_ballot_w64(b == b0);
  const int l = (int)(threadIdx.x & 63);
  if (b == b0 && l != __builtin_ctzll(same)) return;
  const uint32_t n = b == b0 ? (uint32_t)__builtin_popcountll(same) : 1u;
  if (!hash_add(tab, mask, shift, (uint32_t)b, n)) *ovf = 1u;
}

struct BkRaysArgs {
  Geom g;
  CamP cam;
  const uint16_t* depth;
  const PoseX* poses;
  int dmin, dmax, packets_x, packets_pose, wg_pose, span;
  BkGeom bg;
  ulonglong2* rays;
  uint64_t* paths;
  uint32_t* pose_cnt;
  uint32_t* wg_base;
  uint32_t* wg_list;
  int wgl_stride;
  unsigned long long* pose_pairs;
  unsigned long long* stats;
  uint32_t* ovl;   // [count | workgroups whose hashed histogram overflowed]
  int hash_log;    // log2 of the hashed histogram's words (HASH)
};

// Pass A for workgroup wg.  Workgroup = 4 (or 16) waves over a span of 8x8 packets of ONE
// pose (wg_pose workgroups per pose, the last one of a pose shorter); ray index = packet * 64
// + lane.  Counts are kept per (pose, brick): pose_cnt[p][b] (the workgroup's base inside
// that count is wg_base[wg][b]) and per pose: pose_pairs[p], so that the device can cut the
// call into pose batches by the pairs they really make (k_bk_batches) and any batch's
// per-brick lists can be laid out (k_bk_batch_counts) without re-running this pass.
// H16: the histogram holds two 16-bit counts per word (brick b in half b & 1 of word b >> 1:
// a workgroup's rays make at most span * 64 <= 65535 pairs in one brick).  Half the LDS, so
// that two pass-A workgroups fit beside phase F's box on a CU when calls are pipelined
// (DESIGN.md §5.10).  HASH: the hashed histogram above; a workgroup whose table overflows
// writes only its ray records, lists itself in ovl and leaves counts and statistics to
// k_bk_rays_recover.  sh: two shared words (touched-list count, overflow flag).
template <bool H16, bool HASH>
__device__ inline void bk_rays_wg(const BkRaysArgs& A_, unsigned wg, uint32_t* hist, uint32_t* sh) {
  const Geom& g = A_.g;
  const BkGeom& bg = A_.bg;
  unsigned long long* const stats = stat_slot(A_.stats);
  const uint32_t hmask = (1u << A_.hash_log) - 1u;
  const int hshift = 32 - A_.hash_log;
  if (threadIdx.x == 0) {
    sh[0] = 0;
    sh[1] = 0;
  }
  const int nwords = HASH ? (int)hmask + 1 : (H16 ? (bg.nbricks + 1) >> 1 : bg.nbricks);
  for (int i = threadIdx.x; i < nwords; i += blockDim.x) hist[i] = HASH ? kHashEmpty : 0u;
  __syncthreads();
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
#if defined(DMF_EXP_A_PRIO)  // experiment builds: pass A's waves at a raised issue priority
  __builtin_amdgcn_s_setprio(DMF_EXP_A_PRIO);
#endif
  const int pw = (int)(wg / (unsigned)A_.wg_pose);
  const int q0 = (int)(wg - (unsigned)pw * (unsigned)A_.wg_pose) * A_.span;
  const int64_t pk0 = (int64_t)pw * A_.packets_pose + q0,
                pk1 = (int64_t)pw * A_.packets_pose + min(A_.packets_pose, q0 + A_.span);
  unsigned long long upd = 0, nvalid = 0, nhit = 0;
  // (loading the next packet's depth one packet ahead measured slower: 0.79 -> 0.84 ms)
  double go[3];
  // the workgroup's pose, held in registers (read in the packet loop, it was reloaded after
  // every packet's record stores, which might alias it: ±0, profiles/r06i -- as the next
  // packet's depth loaded a packet ahead, +5 % A, pass A is not waiting on its stores)
  float Tf[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) Tf[i] = A_.poses[pw].f[i];
  {
    const float O[3] = {Tf[3], Tf[7], Tf[11]};
    grid_origin(g, O, go);
  }
  for (int64_t pk = pk0 + w; pk < pk1; pk += nw) {
    const int p = pw;
    const int q = (int)(pk - (int64_t)p * A_.packets_pose);
    const int r = (q / A_.packets_x) * 8 + (l >> 3), c = (q % A_.packets_x) * 8 + (l & 7);
    const int d = pixel_depth(A_.cam, A_.depth, p, r, c);
    int64_t qs[3], qe[3];
    bool inside, valid;
    ulonglong2 rec;
    rec.x = 0;
    rec.y = 0;
    uint64_t path = 0;  // the crossing axes of the coarse walk (pass B replays them)
    if (pixel_quant_go(g, A_.cam, d, Tf, go, r, c, A_.dmin, A_.dmax, qs, qe, inside, valid)) {
      uint64_t A, B;
      bk::pack_ray(qs, qe, inside, A, B);
      rec.x = A;
      rec.y = B;
      bk::QRay R;
      const int32_t qs32[3] = {(int32_t)qs[0], (int32_t)qs[1], (int32_t)qs[2]},
                    qe32[3] = {(int32_t)qe[0], (int32_t)qe[1], (int32_t)qe[2]};
      bk::qray_from(qs32, qe32, inside, R);  // = decode_ray(A, B), without the round trip
      upd += (unsigned long long)(R.nsteps + 1);
      nhit += inside ? 1 : 0;
      int t = 0;
      bk_coarse(bg, R, [&](int b, int a, int, int, int) {
#if defined(DMF_EXP_A_AGG_LOOP)  // experiment builds: the loop over every distinct brick
        if constexpr (HASH) hash_add_agg(hist, hmask, hshift, b, &sh[1]);
        else hist_add_agg<H16>(hist, b);
#else
        // (pass A 0.72 -> 0.67 ms at 512^3: one aggregation step instead of a loop)
        if constexpr (HASH) hash_add_first(hist, hmask, hshift, b, &sh[1]);
        else hist_add_first<H16>(hist, b);
#endif
        if (a >= 0) path = bk::path_put(path, t++, a);
      });
    }
    nvalid += valid ? 1 : 0;
    A_.rays[pk * 64 + l] = rec;
    A_.paths[pk * 64 + l] = path;
  }
  __syncthreads();
  if (HASH && sh[1]) {  // table full: k_bk_rays_recover redoes this workgroup
    if (threadIdx.x == 0) A_.ovl[1 + atomicAdd(&A_.ovl[0], 1u)] = wg;
    return;
  }
  uint32_t* const pc = A_.pose_cnt + (size_t)pw * bg.nbricks;
  // the workgroup's touched bricks: [count | (brick id | pair count << 16) per brick] (pass B
  // initialises only these, and checks the slots it took per brick against the counts; a
  // workgroup makes at most span * 64 <= 65535 pairs in one brick, bk_plan)
  uint32_t* const row = A_.wg_list + (size_t)wg * (size_t)A_.wgl_stride;
  unsigned long long mine = 0;
  for (int i = threadIdx.x; i < nwords; i += blockDim.x) {
    uint32_t b, n;
    if constexpr (HASH) {
      const uint32_t e = hist[i];
      b = e >> 16;
      n = e == kHashEmpty ? 0u : (e & 0xffffu);
    } else {
      // direct table: word i holds brick i (or bricks 2i, 2i + 1 when H16)
      b = (uint32_t)i;
      n = hist[i];
    }
    if (!HASH && H16) {
      for (int hh = 0; hh < 2; ++hh) {
        const uint32_t bb = 2u * (uint32_t)i + (uint32_t)hh, nn = (n >> (16 * hh)) & 0xffffu;
        if (nn) {
          A_.wg_base[(size_t)wg * bg.nbricks + bb] = atomicAdd(&pc[bb], nn);
          const uint32_t k = atomicAdd(&sh[0], 1u);
          row[1 + k] = bb | nn << 16;
          mine += nn;
        }
      }
    } else if (n) {
      A_.wg_base[(size_t)wg * bg.nbricks + b] = atomicAdd(&pc[b], n);
      const uint32_t k = atomicAdd(&sh[0], 1u);
      row[1 + k] = b | n << 16;
      mine += n;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) row[0] = sh[0];
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_down(mine, o, 64);
  if (l == 0 && mine) atomicAdd(&A_.pose_pairs[pw], mine);
  if (stats) wave_stats(stats, upd, nvalid, nhit);
}

template <bool H16>
__global__ __launch_bounds__(kBkPassThreadsBig) void k_bk_rays(BkRaysArgs a) {
  extern __shared__ uint32_t hist[];
  __shared__ uint32_t sh[2];
  bk_rays_wg<H16, false>(a, blockIdx.x, hist, sh);
}

// Pass A with the hashed histogram (256-lane workgroups, 8 KB of LDS by default).
__global__ __launch_bounds__(kBkPassThreads) void k_bk_rays_hash(BkRaysArgs a) {
  extern __shared__ uint32_t tab[];
  __shared__ uint32_t sh[2];
  bk_rays_wg<true, true>(a, blockIdx.x, tab, sh);
}

// The workgroups whose hashed histogram overflowed, redone with the direct 16-bit table
// (persistent: the grid strides over the list; exits at once when it is empty).
__global__ __launch_bounds__(kBkPassThreadsBig) void k_bk_rays_recover(BkRaysArgs a) {
  extern __shared__ uint32_t hist[];
  __shared__ uint32_t sh[2];
  const uint32_t n = a.ovl[0];
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    bk_rays_wg<true, false>(a, a.ovl[1 + i], hist, sh);
    __syncthreads();  // the next workgroup's table reset follows this one's flush
  }
}

// Pose batches of a call by the pairs pass A counted (one workgroup): greedy over the poses
// in order, a batch closes before a pose that would take it past `cap` pairs or
// `max_poses` poses (every pose alone fits: cap >= one pose's geometric bound, bk_plan).
// bt[0] = batches J, bt[1 + j] = first pose of batch j, bt[1 + J] = P.
__global__ __launch_bounds__(1024) void k_bk_batches(int P, const unsigned long long* __restrict__ pose_pairs,
                                                     unsigned long long cap, int max_poses,
                                                     uint32_t* __restrict__ bt) {
  // pose counts staged in LDS per round (8 KiB: with pipelined calls this kernel runs beside
  // phase F, whose box leaves ~25 KiB of the CU's LDS)
  constexpr int kChunk = 1024;
  __shared__ unsigned long long spp[kChunk];
  __shared__ unsigned long long s_tot;
  // the common case, every pose in one batch: a parallel sum decides it (the greedy cut below
  // is a serial loop of dependent LDS reads, ~10 us for 128 poses)
  if (P <= max_poses) {
    if (threadIdx.x == 0) s_tot = 0;
    __syncthreads();
    unsigned long long part = 0;
    for (int i = (int)threadIdx.x; i < P; i += blockDim.x) part += pose_pairs[i];
    for (int o = 32; o > 0; o >>= 1) part += __shfl_down(part, o, 64);
    if ((threadIdx.x & 63) == 0 && part) atomicAdd(&s_tot, part);
    __syncthreads();
    if (s_tot <= cap) {
      if (threadIdx.x == 0) {
        bt[0] = P > 0 ? 1u : 0u;
        bt[1] = 0;
        bt[2] = (uint32_t)P;
      }
      return;
    }
  }
  uint32_t J = 0;
  unsigned long long sum = 0;
  int n = 0;
  for (int c0 = 0; c0 < P; c0 += kChunk) {
    const int c1 = min(P, c0 + kChunk);
    __syncthreads();
    for (int i = c0 + (int)threadIdx.x; i < c1; i += blockDim.x) spp[i - c0] = pose_pairs[i];
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int p = c0; p < c1; ++p) {
        const unsigned long long c = spp[p - c0];
        if (n == 0 || sum + c > cap || n >= max_poses) {
          bt[1 + J] = (uint32_t)p;
          ++J;
          sum = 0;
          n = 0;
        }
        sum += c;
        ++n;
      }
    }
  }
  if (threadIdx.x == 0) {
    bt[1 + J] = (uint32_t)P;
    bt[0] = J;
  }
}

// pose_base[p][b] = brick b's pairs of poses p0 .. p-1 for p in [p0, p1); returns the total.
// The loads of a brick's counts are independent: 16 in flight per round (the chain between
// pass A and pass B is exposed in pipelined calls; 4 in flight took 21 us at 128 poses).
__device__ inline uint32_t bk_pose_prefix(const uint32_t* __restrict__ pose_cnt, uint32_t* __restrict__ pose_base,
                                          int nbricks, int b, int p0, int p1) {
  constexpr int kF = 16;
  uint32_t acc = 0;
  int p = p0;
  for (; p + kF <= p1; p += kF) {
    uint32_t c[kF];
#pragma unroll
    for (int k = 0; k < kF; ++k) c[k] = pose_cnt[(size_t)(p + k) * nbricks + b];
#pragma unroll
    for (int k = 0; k < kF; ++k) {
      pose_base[(size_t)(p + k) * nbricks + b] = acc;
      acc += c[k];
    }
  }
  for (; p < p1; ++p) {
    pose_base[(size_t)p * nbricks + b] = acc;
    acc += pose_cnt[(size_t)p * nbricks + b];
  }
  return acc;
}

// Brick lists of batch j (grid over bricks): cnt[b] = the batch's pairs in brick b, and
// pose_base[p][b] = pairs of the batch's earlier poses in brick b (pass B places pose p's
// pairs of brick b at off[b] + pose_base[p][b] + wg_base[wg][b] + slot).  Batches past
// bt[0] leave everything untouched (k_bk_scan empties them).
__global__ __launch_bounds__(256) void k_bk_batch_counts(int nbricks, int j, const uint32_t* __restrict__ bt,
                                                         const uint32_t* __restrict__ pose_cnt,
                                                         uint32_t* __restrict__ pose_base,
                                                         uint32_t* __restrict__ cnt) {
  const int b = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (b >= nbricks || (uint32_t)j >= bt[0]) return;
  const int p0 = (int)bt[1 + j], p1 = (int)bt[2 + j];
  cnt[b] = bk_pose_prefix(pose_cnt, pose_base, nbricks, b, p0, p1);
}

// Scan of the brick counts (one workgroup): list offsets, write cursors, and the part
// table part_pref[b] = parts of bricks < b (a brick of n pairs has ceil(n / 65535)
// parts).  ctl[0] = pairs, ctl[1] = parts.  order[] = the parts as (brick, index in the
// brick), largest first (counting sort into 64 size classes of 1024 pairs): phase F's
// queue hands out the big parts first, so the parts left when the queue runs dry are the
// small ones (the CUs finish together; counter sums do not depend on the order), and F
// needs no search of part_pref for the brick of a part.
// BIG (over 4096 bricks): the counts are staged in LDS (128 KiB); otherwise they are read
// from memory (4 per lane at 512^3) and the kernel's ~12 KiB of LDS fit beside phase F's box
// (pipelined calls).
// The scan's body (one 1024-lane workgroup): `cnt` = the batch's pair counts per brick, in
// memory or in LDS (s_cnt_in non-null).  Also zeroes ctl[2] / ctl[3] (phase F's queue head),
// so no memset precedes it.
template <bool BIG>
__device__ inline void bk_scan_body(int nbricks, const uint32_t* __restrict__ cnt, const uint32_t* s_cnt_in,
                                    uint32_t* __restrict__ off, uint32_t* __restrict__ part_pref,
                                    unsigned long long* __restrict__ ctl, uint2* __restrict__ order, uint32_t part_max,
                                    int split_cu) {
  __shared__ unsigned long long s_pairs[1024];
  __shared__ uint32_t s_parts[1024];
  __shared__ uint32_t s_cls[64];
  // the counts, loaded once with coalesced reads (the brick path has <= 32^3 bricks): the
  // per-thread brick ranges below then read LDS, not dependent HBM loads (1024^3: 0.18 ms)
  __shared__ uint32_t s_cnt_lds[BIG ? kBkScanMax : 1];
  const uint32_t* const s_cnt = BIG ? s_cnt_lds : (s_cnt_in ? s_cnt_in : cnt);
  const int t = threadIdx.x;
  if (t < 64) s_cls[t] = 0;
  if constexpr (BIG)
    for (int i = t; i < nbricks; i += 1024) s_cnt_lds[i] = cnt[i];
  __syncthreads();
  const int per = (nbricks + 1023) / 1024;
  const int i0 = min(nbricks, t * per), i1 = min(nbricks, i0 + per);
  // !BIG (<= 4096 bricks, <= 4 per lane): the lane's counts in registers, read once (the
  // three passes below re-read them)
  constexpr int kPer = 4;
  uint32_t rc[kPer];
  if constexpr (!BIG) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) rc[k] = i0 + k < i1 ? s_cnt[i0 + k] : 0u;
  }
  auto cnt_of = [&](int i) -> uint32_t {
    if constexpr (BIG) return s_cnt[i];
    else {
      uint32_t r = rc[0];
#pragma unroll
      for (int k = 1; k < kPer; ++k) r = i - i0 == k ? rc[k] : r;
      return r;
    }
  };
  unsigned long long sp = 0;
  uint32_t spt = 0;
  for (int i = i0; i < i1; ++i) {
    sp += cnt_of(i);
    spt += (cnt_of(i) + part_max - 1) / part_max;
  }
  s_pairs[t] = sp;
  s_parts[t] = spt;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const unsigned long long a = t >= o ? s_pairs[t - o] : 0ull;
    const uint32_t b = t >= o ? s_parts[t - o] : 0u;
    __syncthreads();
    s_pairs[t] += a;
    s_parts[t] += b;
    __syncthreads();
  }
  unsigned long long base = t ? s_pairs[t - 1] : 0ull;
  const uint32_t pbase0 = t ? s_parts[t - 1] : 0u;
  uint32_t pbase = pbase0;
  auto size_class = [](uint32_t n, uint32_t np) { return min(63u, ((n + np - 1) / np) >> 10); };
  for (int i = i0; i < i1; ++i) {
    off[i] = (uint32_t)base;
    part_pref[i] = pbase;
    base += cnt_of(i);
    const uint32_t np = (cnt_of(i) + part_max - 1) / part_max;
    pbase += np;
    if (np) atomicAdd(&s_cls[size_class(cnt_of(i), np)], np);
  }
  __syncthreads();
  if (t == 0) {  // class starts, largest class first
    uint32_t acc = 0;
    for (int c = 63; c >= 0; --c) {
      const uint32_t v = s_cls[c];
      s_cls[c] = acc;
      acc += v;
    }
  }
  __syncthreads();
  pbase = pbase0;
  for (int i = i0; i < i1; ++i) {
    const uint32_t np = (cnt_of(i) + part_max - 1) / part_max;
    if (np) {
      const uint32_t pos = atomicAdd(&s_cls[size_class(cnt_of(i), np)], np);
      for (uint32_t k = 0; k < np; ++k) order[pos + k] = make_uint2((uint32_t)i, k);  // (brick, part of it)
    }
    pbase += np;
  }
  // Tail split (split_cu = phase F's workgroups | k << 16, 0 = off): with fewer than 8 parts
  // per workgroup the parts are near equal (dense bricks at 256^3 all reach part_max), so
  // the last round of the queue leaves most CUs idle.  The last k * workgroups entries of
  // the order (k = 2: config 2 1.996 -> 1.961 ms; 1 and 4 slower) are cut into quarters
  // (entry .y = 4j + s with bit 31 set: quarter s of part j), so the queue ends in parts a
  // quarter of the size.  Only the largest-first order carries them.
  const uint32_t NP = s_parts[1023];
  uint32_t S = 0;
  if (split_cu > 0 && NP < 8u * (uint32_t)(split_cu & 0xffff))
    S = min(min(NP, 1024u), (uint32_t)(split_cu >> 16) * (uint32_t)(split_cu & 0xffff));
  __syncthreads();  // every order entry written
  uint2 e = make_uint2(0, 0);
  if ((uint32_t)t < S) e = order[NP - S + t];
  __syncthreads();
  if ((uint32_t)t < S)
    for (uint32_t sq = 0; sq < 4; ++sq) order[NP - S + 4 * t + sq] = make_uint2(e.x, (4u * e.y + sq) | 0x80000000u);
  if (t == 1023) {
    part_pref[nbricks] = NP;
    ctl[0] = s_pairs[1023];
    ctl[1] = NP + 3 * S;
    ctl[2] = 0;
    ctl[3] = 0;
  }
}

template <bool BIG>
__global__ __launch_bounds__(1024) void k_bk_scan(int nbricks, const uint32_t* __restrict__ cnt,
                                                  uint32_t* __restrict__ off,
                                                  uint32_t* __restrict__ part_pref,
                                                  unsigned long long* __restrict__ ctl,
                                                  uint2* __restrict__ order, uint32_t part_max,
                                                  const uint32_t* __restrict__ bt, int j, int split_cu) {
  if ((uint32_t)j >= bt[0]) {  // a batch the call does not need: no pairs, no parts
    if (threadIdx.x == 0) ctl[0] = ctl[1] = ctl[2] = ctl[3] = 0;
    return;
  }
  bk_scan_body<BIG>(nbricks, cnt, nullptr, off, part_pref, ctl, order, part_max, split_cu);
}

// Small grids (nbricks <= kBkLayout1Bricks, super-batch <= kBkLayout1Poses): the batch cut
// (k_bk_batches, batch 0's launch only), the batch's brick counts (k_bk_batch_counts) and the
// scan (k_bk_scan) in ONE workgroup: one launch instead of three on the chain between pass A
// and pass B of a pipelined call (config 2: 512 bricks, 64 poses; the chain's launch gaps
// and three kernels ~47 us of a 1.7-ms call).
constexpr int kBkLayout1Bricks = 1024, kBkLayout1Poses = 256;
__global__ __launch_bounds__(1024) void k_bk_layout1(int P, const unsigned long long* __restrict__ pose_pairs,
                                                     unsigned long long cap, int max_poses, uint32_t* __restrict__ bt,
                                                     int nbricks, int j, const uint32_t* __restrict__ pose_cnt,
                                                     uint32_t* __restrict__ pose_base, uint32_t* __restrict__ cnt,
                                                     uint32_t* __restrict__ off, uint32_t* __restrict__ part_pref,
                                                     unsigned long long* __restrict__ ctl, uint2* __restrict__ order,
                                                     uint32_t part_max, int split_cu) {
  __shared__ uint32_t s_bt[kBkLayout1Poses + 2];
  __shared__ uint32_t s_cnt[kBkLayout1Bricks];
  __shared__ unsigned long long s_pp[kBkLayout1Poses];
  const int t = threadIdx.x;
  __shared__ unsigned long long s_tot;
  bool one = false;  // every pose in one batch (decided by a parallel sum, as k_bk_batches)
  if (j == 0) {  // pose pair counts staged in LDS (one coalesced load; the cut below is serial)
    if (t == 0) s_tot = 0;
    __syncthreads();
    unsigned long long part = 0;
    for (int p = t; p < P; p += blockDim.x) {
      s_pp[p] = pose_pairs[p];
      part += s_pp[p];
    }
    for (int o = 32; o > 0; o >>= 1) part += __shfl_down(part, o, 64);
    if ((t & 63) == 0 && part) atomicAdd(&s_tot, part);
    __syncthreads();
    one = P <= max_poses && s_tot <= cap;
    if (one && t == 0) {
      s_bt[0] = P > 0 ? 1u : 0u;
      s_bt[1] = 0;
      s_bt[2] = (uint32_t)P;
      bt[0] = s_bt[0];
      bt[1] = 0;
      bt[2] = (uint32_t)P;
    }
  }
  if (t == 0 && !one) {
    if (j == 0) {  // the batch cut of k_bk_batches (serial over <= 256 poses)
      uint32_t J = 0;
      unsigned long long sum = 0;
      int n = 0;
      for (int p = 0; p < P; ++p) {
        const unsigned long long c = s_pp[p];
        if (n == 0 || sum + c > cap || n >= max_poses) {
          s_bt[1 + J] = (uint32_t)p;
          ++J;
          sum = 0;
          n = 0;
        }
        sum += c;
        ++n;
      }
      s_bt[1 + J] = (uint32_t)P;
      s_bt[0] = J;
      for (uint32_t k = 0; k <= J + 1; ++k) bt[k] = s_bt[k];
    }
  }
  if (j > 0) {  // the table batch 0's launch wrote (same stream, earlier)
    const uint32_t J = bt[0];
    for (uint32_t k = t; k <= J + 1 && k < kBkLayout1Poses + 2; k += blockDim.x) s_bt[k] = bt[k];
  }
  __syncthreads();
  if ((uint32_t)j >= s_bt[0]) {
    if (t == 0) ctl[0] = ctl[1] = ctl[2] = ctl[3] = 0;
    return;
  }
  const int p0 = (int)s_bt[1 + j], p1 = (int)s_bt[2 + j];
  for (int b = t; b < nbricks; b += blockDim.x) {  // k_bk_batch_counts
    const uint32_t acc = bk_pose_prefix(pose_cnt, pose_base, nbricks, b, p0, p1);
    cnt[b] = acc;
    s_cnt[b] = acc;
  }
  __syncthreads();
  bk_scan_body<false>(nbricks, cnt, s_cnt, off, part_pref, ctl, order, part_max, split_cu);
}

// Pass B.  Same spans as pass A; the workgroup's range in each brick was laid out by pass A
// and k_bk_batch_counts / k_bk_scan; every lane writes one self-contained record per (ray,
// brick) pair (the fine walk's state at the brick entry, so phase F makes ONE coalesced
// load per pair and never touches the ray records).
// Entry crossing counts at a brick boundary event (axis a, fine crossing k) come from
// bk::counts_at; E = E(0) + c_a K_b - c_b K_a (exact mod 2^32).
// SLAB (the default, phase F k_bk_fuse_s): the 20-byte record of
// dmf_brick.hpp pack20 (slab state on beta = b >> 9, |dq| in (major, minor1, minor2) order,
// the slab ownership code as the walk bound), pa = words 0-3, pb = word 4 (uint32).
// !SLAB (the per-cell walk of k_bk_fuse, kept as an independent exact check): a 24-B record
// (s = steps inside the brick = cells - 1, 0..93; word offsets into phase F's skewed box)
//   pa = {E01 | s[0:2) << 30, E02 | s[2:4) << 30, E12 | s[4:6) << 30, entry word | last word << 16}
//   pb = {adq0 | adq2[0:14) << 18, adq1 | adq2[14:18) << 18 | neg x,y,z << 22 | s[6] << 25 | ends << 26}
// with each E as a 30-bit two's-complement field (|E| < 2^28 for a moving pair of a grid
// <= 1024 cells/axis; a pair with a non-moving axis keeps a constant E of which only the
// sign is used, stored as +-(2^29 - 1)).
// Slots: one LDS atomic per lane, whose return is consumed only by the pair's store at the
// next brick boundary (its latency hides behind that boundary's count_at; B 1.92 -> 1.88 ms;
// wave-aggregated and run-aggregated takes measured slower).
// Pass B's store guard (experiment builds: 0 none, 1 a branch around the stores); the
// default 2 clamps the slot onto a spare record
#ifndef DMF_B_GUARD
#define DMF_B_GUARD 2
#endif
// pass B's slot cursor of a brick pass A did not count for the workgroup: every slot taken
// from it lies at or past any batch's records (pair capacity < the sentinel, bk_plan)
constexpr uint32_t kBkSlotSentinel = 0xF0000000u;
__device__ inline uint32_t bk_e30(int32_t e) {
  const int32_t lim = (1 << 29) - 1;
  return (uint32_t)(e > lim ? lim : (e < -lim ? -lim : e)) & 0x3fffffffu;
}


// (experiment builds DMF_EXP_B_WAVES = n: the compiler keeps B's registers for n waves per SIMD)
#if defined(DMF_EXP_B_WAVES)
#define DMF_B_OCC __attribute__((amdgpu_waves_per_eu(DMF_EXP_B_WAVES)))
#else
#define DMF_B_OCC
#endif
template <bool SLAB>
__global__ __launch_bounds__(kBkPassThreadsBig) DMF_B_OCC void k_bk_pairs(int packets_pose, int wg_pose, int span, BkGeom bg,
                                                         const ulonglong2* __restrict__ rays,
                                                         const uint64_t* __restrict__ paths,
                                                         const uint32_t* __restrict__ off,
                                                         const uint32_t* __restrict__ pose_base,
                                                         const uint32_t* __restrict__ wg_base,
                                                         const uint32_t* __restrict__ bt, int j,
                                                         const uint32_t* __restrict__ wg_list, int wgl_stride,
                                                         uint4* __restrict__ pa, void* __restrict__ pbv,
                                                         unsigned long long* __restrict__ ctl,
                                                         uint32_t* __restrict__ fault, int inject,
                                                         unsigned long long* __restrict__ stats) {
  uint2* const pb = (uint2*)pbv;
  uint32_t* const pw = (uint32_t*)pbv;
  extern __shared__ uint32_t hist[];
  // the workgroups of pass A (one pose each); only those of batch j's poses run
  const int pz = (int)(blockIdx.x / (unsigned)wg_pose);
  if ((uint32_t)j >= bt[0] || (uint32_t)pz < bt[1 + j] || (uint32_t)pz >= bt[2 + j]) return;
  // the batch's pair records: a slot at or past `total` (passes A and B disagree) never
  // stores outside them, and the end of the kernel checks the slots taken per brick against
  // pass A
  const uint32_t total = (uint32_t)ctl[0];
  // DMF_KNOB_FAULT_INJECT: the first pair of thread 0 of the first pose's workgroups takes
  // `inject` extra slots (a register, not LDS: nothing is read per pair for the test hook)
  uint32_t extra = (inject > 0 && j == 0 && (uint32_t)pz == bt[1] && threadIdx.x == 0) ? (uint32_t)inject : 0u;
  // this workgroup's range in brick i starts at off[i] + pose_base[p][i] + wg_base[wg][i]
  // (k_bk_scan, k_bk_batch_counts, pass A); only the bricks pass A counted for this
  // workgroup are initialised (1024^3: 32768 bricks, ~300 touched)
  const uint32_t* wb = wg_base + (size_t)blockIdx.x * bg.nbricks;
  const uint32_t* pbz = pose_base + (size_t)pz * bg.nbricks;
  {
    const uint32_t* row = wg_list + (size_t)blockIdx.x * (size_t)wgl_stride;
    const uint32_t nl = row[0];
#if DMF_B_GUARD != 0
    // bricks pass A did not count here: any slot taken from them is out of range (checked)
    for (int i = threadIdx.x; i < bg.nbricks; i += blockDim.x) hist[i] = kBkSlotSentinel;
    __syncthreads();
#endif
    for (uint32_t k = threadIdx.x; k < nl; k += blockDim.x) {
      const int i = (int)(row[1 + k] & 0xffffu);
      hist[i] = off[i] + pbz[i] + wb[i];
    }
  }
  __syncthreads();
  uint32_t over = 0;  // one past the lane's largest slot (the layout check; 0 = no pair)
#if defined(DMF_EXP_B_NOSLOT)
  uint32_t dslot = blockIdx.x * blockDim.x + threadIdx.x, dmask = 1u;
  while (dmask * 2u <= total && dmask < 0x80000000u) dmask *= 2u;
  dmask -= 1u;
#endif
#if defined(DMF_EXP_STATS)
  unsigned long long b_iters = 0, b_lanes = 0;
#endif
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int q0 = (int)(blockIdx.x - (unsigned)pz * (unsigned)wg_pose) * span;
  const int64_t pk0 = (int64_t)pz * packets_pose + q0, pk1 = (int64_t)pz * packets_pose + min(packets_pose, q0 + span);
  constexpr uint32_t m5 = bk::kB - 1;
  // the next packet's ray record is loaded one packet ahead: its HBM latency hides behind
  // this packet's coarse walk (B 2.03 -> 1.92 ms) instead of stalling the wave per packet
  ulonglong2 rnext = make_ulonglong2(0, 0);
  uint64_t pnext = 0;
  if (pk0 + w < pk1) {
    rnext = rays[(pk0 + w) * 64 + l];
    pnext = paths[(pk0 + w) * 64 + l];
  }
  for (int64_t pk = pk0 + w; pk < pk1; pk += nw) {
    const ulonglong2 rec = rnext;
    const uint64_t path = pnext;
    if (pk + nw < pk1) {
      rnext = rays[(pk + nw) * 64 + l];
      pnext = paths[(pk + nw) * 64 + l];
    }
    if ((rec.y >> 63) == 0) continue;  // no ray
    bk::QRay R;
    bk::decode_ray(rec.x, rec.y, R);
    const uint32_t K0 = (uint32_t)(2 * bk::kQ) * (uint32_t)R.adq[0], K1 = (uint32_t)(2 * bk::kQ) * (uint32_t)R.adq[1],
                   K2 = (uint32_t)(2 * bk::kQ) * (uint32_t)R.adq[2];
    const uint32_t e01 = (uint32_t)bk::e0_pair(R, 0, 1), e02 = (uint32_t)bk::e0_pair(R, 0, 2),
                   e12 = (uint32_t)bk::e0_pair(R, 1, 2);
    const uint32_t signs = (R.st[0] < 0 ? 1u << 22 : 0u) | (R.st[1] < 0 ? 1u << 23 : 0u) | (R.st[2] < 0 ? 1u << 24 : 0u);
    // SLAB: major axis M, minors m1 < m2; state and |dq| in (M, m1, m2) order
    const int M = SLAB ? bk::major_axis(R) : 0;
    const int m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
    const uint32_t aM = (uint32_t)bk::pick3(R.adq[0], R.adq[1], R.adq[2], M),
                   a1 = (uint32_t)bk::pick3(R.adq[0], R.adq[1], R.adq[2], m1),
                   a2 = (uint32_t)bk::pick3(R.adq[0], R.adq[1], R.adq[2], m2);
    const uint32_t KM = (uint32_t)(2 * bk::kQ) * aM, Km1 = (uint32_t)(2 * bk::kQ) * a1, Km2 = (uint32_t)(2 * bk::kQ) * a2;
    int32_t sb1 = 0, sb2 = 0, sb12 = 0;
    if (SLAB) bk::slab_from_pairwise(M, (int32_t)e01, (int32_t)e02, (int32_t)e12, sb1, sb2, sb12);
    const uint2 wb0 = make_uint2((uint32_t)R.adq[0] | (((uint32_t)R.adq[2] & 0x3fffu) << 18),
                                 (uint32_t)R.adq[1] | (((uint32_t)R.adq[2] >> 14) << 18) | signs);
    // entry state of the pair being built (the exact int32 state; put() formats it)
    auto entry = [&](const int32_t c[3]) {
      uint4 e;
      if (SLAB) {  // b = b(0) + c_M K_m - c_m K_M;  b12 = b12(0) + c_1 K_2 - c_2 K_1
        const uint32_t cM = (uint32_t)bk::pick3(c[0], c[1], c[2], M), c1 = (uint32_t)bk::pick3(c[0], c[1], c[2], m1),
                       c2 = (uint32_t)bk::pick3(c[0], c[1], c[2], m2);
        // c K = 2 kQ c |dq| mod 2^32: 24-bit multiplies (counts <= 1024, |dq| < 2^18)
        constexpr uint32_t k2 = (uint32_t)(2 * bk::kQ);
        auto m = [](uint32_t c, uint32_t a) { return (uint32_t)bk::mul24((int32_t)c, (int32_t)a); };
        e.x = (uint32_t)sb1 + (m(cM, a1) - m(c1, aM)) * k2;
        e.y = (uint32_t)sb2 + (m(cM, a2) - m(c2, aM)) * k2;
        e.z = (uint32_t)sb12 + (m(c1, a2) - m(c2, a1)) * k2;
      } else {
        e.x = e01 + (uint32_t)c[0] * K1 - (uint32_t)c[1] * K0;
        e.y = e02 + (uint32_t)c[0] * K2 - (uint32_t)c[2] * K0;
        e.z = e12 + (uint32_t)c[1] * K2 - (uint32_t)c[2] * K1;
      }
      const uint32_t x = (uint32_t)(R.cs[0] + bk::mul24(R.st[0], c[0])) & m5,
                     y = (uint32_t)(R.cs[1] + bk::mul24(R.st[1], c[1])) & m5,
                     z = (uint32_t)(R.cs[2] + bk::mul24(R.st[2], c[2])) & m5;
      e.w = bk_lds_word(x, y, z);
      return e;
    };
    // brick-local word of the cell before the crossing (axis a) that produced counts c
    auto last_before = [&](const int32_t c[3], int a) {
      const uint32_t x = (uint32_t)(R.cs[0] + bk::mul24(R.st[0], c[0] - (a == 0))) & m5,
                     y = (uint32_t)(R.cs[1] + bk::mul24(R.st[1], c[1] - (a == 1))) & m5,
                     z = (uint32_t)(R.cs[2] + bk::mul24(R.st[2], c[2] - (a == 2))) & m5;
      return bk_lds_word(x, y, z);
    };
    auto put = [&](uint32_t slot, uint4 e, uint32_t last, uint32_t steps, bool ends) {
#if DMF_B_GUARD == 1
      if (slot >= total) {  // only when A and B disagree (reported by the check below)
        over = slot + 1u;
        return;
      }
#elif DMF_B_GUARD == 2
      // a slot at or past the batch's records (only when A and B disagree, reported by the
      // check below) goes to the spare record at index `total` (pair_cap + 1 are reserved),
      // which phase F never reads: a v_max and a v_min instead of a branch around the stores
      over = max(over, slot + 1u);
      slot = min(slot, total);
#endif
      if constexpr (SLAB) {
        uint32_t w[5];
        bk::pack20((int32_t)e.x, (int32_t)e.y, (int32_t)e.z, aM, a1, a2, e.w, last, steps, signs >> 22, (uint32_t)M,
                   ends, w);
        pa[slot] = make_uint4(w[0], w[1], w[2], w[3]);
        pw[slot] = w[4];
      } else {
        e.x = bk_e30((int32_t)e.x) | (steps & 3u) << 30;
        e.y = bk_e30((int32_t)e.y) | ((steps >> 2) & 3u) << 30;
        e.z = bk_e30((int32_t)e.z) | ((steps >> 4) & 3u) << 30;
        e.w |= last << 16;
        pa[slot] = e;
        pb[slot] = make_uint2(wb0.x, wb0.y | ((steps >> 6) << 25) | (ends ? 1u << 26 : 0u));
      }
    };
    // the end cell (brick-local): the last cell of the ray's last pair
    const uint32_t endc = bk_lds_word((uint32_t)R.ce[0] & m5, (uint32_t)R.ce[1] & m5, (uint32_t)R.ce[2] & m5);
    // per axis, the fine-crossing index of the boundary into the next brick along it
    // (dmf_brick.hpp next_boundary_k): a boundary event on axis a takes P_a, which then grows by
    // kB -- selects, not per-axis branches: the compiler merged branch-wise updates into a
    // stack array indexed by the axis (scratch, as an axis-indexed array in round 4)
    const int cb0 = R.cs[0] >> bk::kLog, cb1 = R.cs[1] >> bk::kLog, cb2 = R.cs[2] >> bk::kLog;
    int32_t P0 = bk::next_boundary_k(R, 0, cb0), P1 = bk::next_boundary_k(R, 1, cb1), P2 = bk::next_boundary_k(R, 2, cb2);
    const int32_t c00[3] = {0, 0, 0};
    uint4 cur = entry(c00);
    int32_t idx = 0;                    // crossings before the current pair's first cell
    int32_t ci0 = 0, ci1 = 0, ci2 = 0;  // SLAB: their counts per axis
    // count field: SLAB = the slab code of dmf_brick.hpp slab_code (S | s << 5 | e << 7: F's
    // walk bound and its adoption of L's slab), else the pair's cells - 1; cL = crossing counts
    // at the pair's last cell
    auto count_field = [&](int32_t L0, int32_t L1, int32_t L2) -> uint32_t {
      if (!SLAB) return (uint32_t)(L0 + L1 + L2 - idx);
      const int32_t cin[3] = {ci0, ci1, ci2}, cL[3] = {L0, L1, L2};
      return bk::slab_code(M, sb1, sb2, sb12, KM, Km1, Km2, cin, cL);
    };
    // crossing counts per axis at the boundary event of axis a (fine crossing P_a)
    // the boundary counts in double arithmetic (dmf_brick.hpp counts_at_f64, exact by fma;
    // B 1.41 -> 1.37 ms): per ray three reciprocals, per event two fma
    // quotients instead of 64-bit products and float quotient estimates.  Constant axis in each
    // call: no dynamically indexed (scratch) arrays.
#if defined(DMF_EXP_B_INT_COUNTS)  // experiment builds: the integer counts_at
    auto counts = [&](int a, int32_t k, int32_t c[3]) {
      if (a == 0) bk::counts_at(R, 0, k, c);
      else if (a == 1) bk::counts_at(R, 1, k, c);
      else bk::counts_at(R, 2, k, c);
    };
#else
    bk::QRayF64 F64;
    bk::qray_f64(R, F64);
    auto counts = [&](int a, int32_t k, int32_t c[3]) {
      if (a == 0) bk::counts_at_f64<0>(R, F64, k, c);
      else if (a == 1) bk::counts_at_f64<1>(R, F64, k, c);
      else bk::counts_at_f64<2>(R, F64, k, c);
    };
#endif
    // the replay of the brick sequence (bk_coarse's order): the crossing axes pass A recorded
    // (path), past its kPathSteps boundaries the stateless next axis from the P's; the brick
    // index moves by a per-axis step
    const int total = bk::coarse_total(R);
    const int32_t nb12 = bg.nb[1] * bg.nb[2];
    const int32_t D0 = bk::mul24(R.st[0], nb12), D1 = bk::mul24(R.st[1], bg.nb[2]), D2 = R.st[2];
    int b = bk_index(bg, cb0, cb1, cb2);
#if defined(DMF_EXP_B_NOSLOT)  // diagnostic (wrong layout: the check fails, F skips): no slot atomics,
    // each lane's stores to distinct records, lanes of a wave adjacent (an ideal store stream)
#define DMF_B_SLOT(b) ((dslot += gridDim.x * blockDim.x) & dmask)
#else
#define DMF_B_SLOT(b) atomicAdd(&hist[b], 1u + extra)
#endif
    uint32_t slot = DMF_B_SLOT(b);
    extra = 0;
    for (int t = 0; t < total; ++t) {
#if defined(DMF_EXP_STATS)
      {  // diagnostic build: the replay loop's wave iterations and the lanes active in them
        const uint64_t am = __builtin_amdgcn_ballot_w64(true);
        if (l == __builtin_ctzll(am)) {
          ++b_iters;
          b_lanes += (unsigned long long)__builtin_popcountll(am);
        }
      }
#endif
      int a;
      if (t < bk::kPathSteps) a = bk::path_axis(path, t);
      else a = bk::coarse_next_k(R, P0, P1, P2);  // (branch: skipped by the waves whose lanes all replay)
      b += a == 0 ? D0 : (a == 1 ? D1 : D2);
      const int32_t k = a == 0 ? P0 : (a == 1 ? P1 : P2);
      P0 += a == 0 ? bk::kB : 0;
      P1 += a == 1 ? bk::kB : 0;
      P2 += a == 2 ? bk::kB : 0;
      int32_t c[3];
      counts(a, k, c);
      put(slot, cur, last_before(c, a), count_field(c[0] - (a == 0), c[1] - (a == 1), c[2] - (a == 2)), false);
      cur = entry(c);
      idx = c[0] + c[1] + c[2];
      ci0 = c[0];
      ci1 = c[1];
      ci2 = c[2];
      slot = DMF_B_SLOT(b);
      extra = 0;
    }
#undef DMF_B_SLOT
    put(slot, cur, endc, count_field(R.n[0], R.n[1], R.n[2]), R.end_inside);
  }
#if defined(DMF_EXP_STATS)
  if (stats && b_iters) {
    unsigned long long* const sl = stat_slot(stats);
    atomicAdd(&sl[18], b_iters);
    atomicAdd(&sl[19], b_lanes);
  }
#endif
  // layout check: the slots taken in each touched brick must be pass A's count for it
#if DMF_B_GUARD != 0
  __syncthreads();
  {
    const uint32_t* row = wg_list + (size_t)blockIdx.x * (size_t)wgl_stride;
    const uint32_t nl = row[0];
    uint32_t bad = over > total ? 1u : 0u;  // a slot past the records (or from an uncounted brick)
#if defined(DMF_EXP_LAYOUT_DEBUG)
    if (bad) printf("B over: wg %u j %d lane %u over %u total %u\n", blockIdx.x, j, threadIdx.x, over, total);
#endif
    for (uint32_t k = threadIdx.x; k < nl; k += blockDim.x) {
      const uint32_t e = row[1 + k];
      const int i = (int)(e & 0xffffu);
      bad += hist[i] != off[i] + pbz[i] + wb[i] + (e >> 16) ? 1u : 0u;
#if defined(DMF_EXP_LAYOUT_DEBUG)
      if (hist[i] != off[i] + pbz[i] + wb[i] + (e >> 16))
        printf("B count: wg %u j %d brick %d hist %u off %u pbz %u wb %u cnt %u total %u\n", blockIdx.x, j, i, hist[i],
               off[i], pbz[i], wb[i], e >> 16, total);
#endif
    }
#if defined(DMF_EXP_B_NOSLOT)  // (the diagnostic's layout is wrong: one flag per workgroup, F skips)
    if (threadIdx.x == 0) atomicOr(&ctl[3], 1ull);
#else
    if (bad) {
      atomicAdd(&fault[0], bad);
      atomicAdd(&fault[1], bad);
      atomicOr(&ctl[3], 1ull);  // phase F skips this batch: its records are not all in place
    }
#endif
  }
#endif
}

// Pair order inside a part: lane-adjacent picks come from S_ORDER far-apart regions of
// the brick's list (neighbouring rays sit in the same cells at the same step, so taking
// them together serialises the LDS adds), while each region is still read in order
// (coalesced record loads).  A bijection on [0, n).
template <int S_ORDER>
__device__ inline uint32_t bk_order(uint32_t k, uint32_t n) {
  if (S_ORDER <= 1) return k;
  const uint32_t per = n / S_ORDER, n1 = per * S_ORDER;
  // (24-bit multiply: per < 2^16 for parts of <= 65535 pairs; a 32-bit one became v_mad_u64_u32)
  return k < n1 ? (uint32_t)bk::mul24((int32_t)(k % S_ORDER), (int32_t)per) + k / S_ORDER : k;
}

// Phase F, per-cell walk (variant DMF_FUSE_CELL_WALK = 40: an independent exact walk kept for
// cross-checks; the default is k_bk_fuse_s below).  Persistent: a work queue of parts, every
// workgroup exits when it is empty.  Each lane walks one pair at a time, one DDA selection
// per cell; a wave refills its idle lanes when >= REFILL are idle, from per-lane records
// prefetched one refill ahead (their load latency is hidden behind the walk of the current
// pairs).  The E fields are kept biased by -1 so that E >= 0 tests E > 0.
template <int REFILL, int S_ORDER, int UNROLL>
__global__ __launch_bounds__(kBkThreads) void k_bk_fuse(Geom g, BkGeom bg, const uint4* __restrict__ pa,
                                                        const uint2* __restrict__ pb,
                                                        const uint32_t* __restrict__ off,
                                                        const uint32_t* __restrict__ cnt,
                                                        const uint32_t* __restrict__ part_pref,
                                                        unsigned long long* __restrict__ ctl,
                                                        int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                        unsigned long long* __restrict__ stats) {
  // counters (skewed), then 4 control words
  __shared__ uint32_t box[kBkBoxWords + 4];
  uint32_t* sh = box + kBkBoxWords;
  stats = stat_slot(stats);
  const int tid = threadIdx.x, l = tid & 63;
  if (ctl[3] != 0) return;  // pass B's layout check failed for this batch (as k_bk_fuse_s)
  for (int i = tid; i < kBkBoxWords; i += blockDim.x) box[i] = 0;
  const uint32_t nparts = (uint32_t)ctl[1];
  const Tiles tl = tiles_of(g.n);
  unsigned long long npairs = 0, nparts_done = 0, nflush = 0;
  for (;;) {
    if (tid == 0) {
      sh[0] = (uint32_t)atomicAdd(&ctl[2], 1ull);
      sh[1] = 0;
    }
    __syncthreads();
    const uint32_t t = sh[0];
    if (t >= nparts) break;
    int lo = 0, hi = bg.nbricks - 1;  // last brick b with part_pref[b] <= t
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (part_pref[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    const int b = lo;
    const uint32_t np = part_pref[b + 1] - part_pref[b], j = t - part_pref[b], nb_pairs = cnt[b];
    const uint32_t p0 = off[b] + (uint32_t)(((uint64_t)nb_pairs * j) / np);
    const uint32_t n = (uint32_t)(((uint64_t)nb_pairs * (j + 1)) / np) - (uint32_t)(((uint64_t)nb_pairs * j) / np);
    const int bz = b % bg.nb[2], by = (b / bg.nb[2]) % bg.nb[1], bx = b / (bg.nb[2] * bg.nb[1]);
    const int lo0 = bx << bk::kLog, lo1 = by << bk::kLog, lo2 = bz << bk::kLog;
    if (tid == 0) {
      npairs += n;
      ++nparts_done;
    }
    // walk state (biased E, K negated once per pair: the step is adds and bit selects); a
    // lane is active while cur != cend (its last cell, added at adoption)
    int32_t E01 = 0, E02 = 0, E12 = 0, K1 = 0, K2 = 0, nK0 = 0, nK1 = 0;
    int cur = 0, cend = 0, dX = 0, dY = 0, dZ = 0;
    uint4 ca = make_uint4(0, 0, 0, 0);
    uint2 cb = make_uint2(0, 0);
    bool fok = false;
    auto decode = [&]() {
      E01 = __builtin_amdgcn_sbfe((int32_t)ca.x, 0, 30) - 1;
      E02 = __builtin_amdgcn_sbfe((int32_t)ca.y, 0, 30) - 1;
      E12 = __builtin_amdgcn_sbfe((int32_t)ca.z, 0, 30) - 1;
      const uint32_t a0 = cb.x & 0x3ffffu, a1 = cb.y & 0x3ffffu, a2 = (cb.x >> 18) | (((cb.y >> 18) & 15u) << 14);
      nK0 = -(int32_t)(a0 << 9);
      K1 = (int32_t)(a1 << 9);
      K2 = (int32_t)(a2 << 9);
      nK1 = -K1;
      cur = (int)(ca.w & 0xffffu) * 4;
      cend = (int)(ca.w >> 16) * 4;
      dX = (cb.y >> 22) & 1u ? -(4 * kBkSx) : 4 * kBkSx;
      dY = (cb.y >> 23) & 1u ? -(4 * kBkSy) : 4 * kBkSy;
      dZ = (cb.y >> 24) & 1u ? -4 : 4;
      // the pair's last cell: a hit when the ray ends there inside the grid, else a miss
      atomicAdd(&box[ca.w >> 16], (cb.y >> 26) & 1u ? 0x10000u : 1u);
    };
    bool more = true;
    // lanes in `need` take the next pair indices (one LDS allocation) and load their records
    auto prefetch = [&](uint64_t need) {
      const uint32_t nn = (uint32_t)__builtin_popcountll(need);
      uint32_t base0 = 0;
      if (l == 0) base0 = atomicAdd(&sh[1], nn);
      const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base0);
      if (base + nn >= n) more = false;
      if ((need >> l) & 1ull) {
        const uint32_t k = base + (uint32_t)lane_prefix(need);
        fok = k < n;
        if (fok) {
          const uint32_t i = p0 + bk_order<S_ORDER>(k, n);
          ca = pa[i];
          cb = pb[i];
        }
      }
    };
    prefetch(~0ull);
    for (;;) {
      const uint64_t act = __builtin_amdgcn_ballot_w64(cur != cend);
      bool any_act = act != 0;
      if ((int)__builtin_popcountll(act) <= 64 - REFILL) {
        const uint64_t take = __builtin_amdgcn_ballot_w64(cur == cend && fok);
        if (take) {
          if (cur == cend && fok) {
            decode();
            fok = false;
          }
          if (more) prefetch(take);
          any_act = __builtin_amdgcn_ballot_w64(cur != cend) != 0;
        }
      }
      if (!any_act) {
        if (__builtin_amdgcn_ballot_w64(fok) == 0) break;
        continue;
      }
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        if (cur == cend) continue;
        atomicAdd((uint32_t*)((char*)box + cur), 1u);
        const bool b10 = E01 >= 0;              // E01 > 0 (biased): T1 < T0
        const bool s2 = (b10 ? E12 : E02) >= 0;  // T2 first
        const bool s1 = !s2 && b10, s0 = !s2 && !b10;
        E01 += s0 ? K1 : (s1 ? nK0 : 0);
        E02 += s0 ? K2 : (s2 ? nK0 : 0);
        E12 += s1 ? K2 : (s2 ? nK1 : 0);
        cur += s2 ? dZ : (s1 ? dY : dX);
      }
    }
    __syncthreads();
    // flush: e -> 2x2x4 tile (e >> 4) of the brick, cell (e & 15) as in the tiled layout,
    // so 16 lanes cover one 64-B counter line; device atomics for every part
    for (int e = tid; e < bk::kCells; e += blockDim.x) {
      const int tile = e >> 4, w16 = e & 15;
      const int tx = tile >> (2 * bk::kLog - 3), ty = (tile >> (bk::kLog - 2)) & ((bk::kB >> 1) - 1),
                tz = tile & ((bk::kB >> 2) - 1);
      const int lx = tx * 2 + (w16 >> 3), ly = ty * 2 + ((w16 >> 2) & 1), lz = tz * 4 + (w16 & 3);
      const int li = lx * kBkSx + ly * kBkSy + lz;
      const uint32_t v = box[li];
      if (v) {
        box[li] = 0;
        const uint32_t ti = tiled_index(tl, lo0 + lx, lo1 + ly, lo2 + lz);
        const int32_t mi = (int32_t)(v & 0xffffu), hv = (int32_t)(v >> 16);
        if (mi) atomic_add_dev(&misses[ti], mi);
        if (hv) atomic_add_dev(&hits[ti], hv);
        ++nflush;
      }
    }
    __syncthreads();
  }
  if (stats) {
    for (int o = 32; o > 0; o >>= 1) nflush += __shfl_down(nflush, o, 64);
    if (l == 0 && nflush) atomicAdd(&stats[6], nflush);
    if (tid == 0) {
      if (npairs) atomicAdd(&stats[4], npairs);
      if (nparts_done) atomicAdd(&stats[5], nparts_done);
    }
  }
}

// Phase F, slab walk (the default).  Same part queue, LDS box and
// flush as k_bk_fuse, but a lane advances one SLAB per step (dmf_brick.hpp slab_walk): the
// cells between two major-axis crossings, 1 + c1 + c2 of them, with one compare per minor
// axis instead of a three-way DDA selection per cell, on the 20-byte record's scaled state
// beta = b >> 9 with increments |dq| (exactly the decisions of b with K = 512 |dq|).  The
// pair's slab code (dmf_brick.hpp slab_code) bounds the walk: the S slabs before the last
// cell L's are taken whole, their LDS adds predicated on ONE test per slab (r > k); the
// state keeps moving harmlessly past them (unsigned arithmetic; refilled or ignored).  L and
// the s cells of L's slab before it are added at adoption, from L: L - d_e (s >= 1) and
// L - d_1 - d_2 (s = 2).  (Round 5 and before: the code R = 3 S + s and three thresholds per
// slab, r - 3k > j for cell j.)  A wave refills when >= REFILL of its lanes are idle, from
// per-lane records prefetched one refill ahead through buffer resources over the part.
// Parts are taken from k_bk_scan's largest-first order (entries (brick, part index); bit 31
// of the index marks a quarter of a part from the scan's tail split).
#if defined(DMF_EXP_STATS)
#define DMF_T(x) const unsigned long long x = __builtin_amdgcn_s_memtime()
#define DMF_TACC(acc, x) acc += __builtin_amdgcn_s_memtime() - (x)
#else
#define DMF_T(x)
#define DMF_TACC(acc, x)
#endif
template <int REFILL, int S_ORDER, int UNROLL>
__global__ __launch_bounds__(kBkThreads) void k_bk_fuse_s(Geom g, BkGeom bg, const uint4* __restrict__ pa,
                                                          const uint32_t* __restrict__ pw,
                                                          const uint32_t* __restrict__ off,
                                                          const uint32_t* __restrict__ cnt,
                                                          const uint2* __restrict__ order, uint32_t part_max,
                                                          unsigned long long* __restrict__ ctl,
                                                          int32_t* __restrict__ hits, int32_t* __restrict__ misses,
                                                          unsigned long long* __restrict__ stats,
                                                          const ulonglong2* __restrict__ xrays, uint32_t xnrays,
                                                          uint32_t xnpairs) {
  __shared__ uint32_t box[kBkBoxWords + 4];  // counters (skewed), control words
  uint32_t* sh = box + kBkBoxWords;
  // (xrays / xnrays / xnpairs: used only by the DMF_EXP_F_REBUILD experiment build below)
  // F's stride table, indexed by a record's T = w4 >> 24 (dmf_brick.hpp pack20: the slab code's
  // s and e, the step signs, the major axis M): (dM, d1, d2) the LDS byte strides of the pair's
  // major and minor axes, and the byte offsets from L of the cells of L's slab the code adopts
  // (low 16 bits, signed: L - d_e when s >= 1; high 16: L - d1 - d2 when s == 2; 0 = none).
  // (dmf_brick.hpp slab_table_entry).  One ds_read per refill instead of ~25 VALU of selects;
  // written before the first part's barrier
  __shared__ uint4 slut[256];
  if (threadIdx.x < 256) {
    uint32_t e[4];
    bk::slab_table_entry(threadIdx.x, 4u * kBkSx, 4u * kBkSy, 4u, e);
    slut[threadIdx.x] = make_uint4(e[0], e[1], e[2], e[3]);
  }
  stats = stat_slot(stats);
  const int tid = threadIdx.x, l = tid & 63;
  // pass B's layout check failed for this batch (dmf_fuse_status reports it): its pair
  // records are not all in place, so none is walked
  if (ctl[3] != 0) return;
#if defined(DMF_EXP_F_PRIO)  // experiment builds: phase F's waves at a raised issue priority
  __builtin_amdgcn_s_setprio(DMF_EXP_F_PRIO);
#endif
#if defined(DMF_EXP_F_REBUILD)
  xnpairs = (uint32_t)ctl[0];  // the batch's pairs (the stand-in ray ids spread over them)
  uint32_t sink = 0;           // the proxy's result
#endif
  for (int i = tid; i < kBkBoxWords; i += blockDim.x) box[i] = 0;
  const uint32_t nparts = (uint32_t)ctl[1];
  const Tiles tl = tiles_of(g.n);
  unsigned long long npairs = 0, nparts_done = 0, nflush = 0;
#if defined(DMF_EXP_STATS)
  // diagnostic build: wave blocks, lanes active at block start, refills, and s_memtime
  // cycles per phase (refill = decode + index allocation / prefetch, walk, flush incl. its
  // barriers, wait at the part-start barrier)
  unsigned long long nblocks = 0, nlanes = 0, nrefill = 0, t_refill = 0, t_walk = 0, t_flush = 0, t_bar = 0;
  unsigned long long t_dec = 0, t_pf = 0;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
  char* const lds = (char*)box;
  for (;;) {
    if (tid == 0) {
      sh[0] = (uint32_t)atomicAdd(&ctl[2], 1ull);
      sh[1] = 0;
    }
    DMF_T(tb0);
    __syncthreads();
    DMF_TACC(t_bar, tb0);
    if (sh[0] >= nparts) break;
    const uint2 o = order[sh[0]];
    const int b = (int)o.x;
    const uint32_t j = o.y & 0x7fffffffu, q4 = o.y >> 31 ? 4u : 1u;  // quarters of the tail split
    const uint32_t nb_pairs = cnt[b], np = q4 * ((nb_pairs + part_max - 1) / part_max);
    const uint32_t p0 = off[b] + (uint32_t)(((uint64_t)nb_pairs * j) / np);
    const uint32_t n = (uint32_t)(((uint64_t)nb_pairs * (j + 1)) / np) - (uint32_t)(((uint64_t)nb_pairs * j) / np);
    // buffer resources over the part's records (32-bit offsets < 2^21, no 64-bit address
    // math per load; a load past the part returns zeros)
    const __amdgpu_buffer_rsrc_t rs_a = __builtin_amdgcn_make_buffer_rsrc((void*)(pa + p0), (short)0, (int)(n * 16u),
                                                                         0x00020000);
    const __amdgpu_buffer_rsrc_t rs_w = __builtin_amdgcn_make_buffer_rsrc((void*)(pw + p0), (short)0, (int)(n * 4u),
                                                                         0x00020000);
    const int bz = b % bg.nb[2], by = (b / bg.nb[2]) % bg.nb[1], bx = b / (bg.nb[2] * bg.nb[1]);
    const int lo0 = bx << bk::kLog, lo1 = by << bk::kLog, lo2 = bz << bk::kLog;
    if (tid == 0) {
      npairs += n;
      ++nparts_done;
    }
    // slab state (unsigned: it may run past the pair's end), LDS byte offset and strides,
    // ownership code (r), the prefetched record (ca, cw) and whether it is valid
    uint32_t b1 = 0, b2 = 0, b12 = 0, K1 = 0, K2 = 0, K1mM = 0, K2mM = 0, nK1 = 0;
    uint32_t cur = 0, dM = 0, d1 = 0, d2 = 0;
    int r = 0;
    uint4 ca = make_uint4(0, 0, 0, 0);
    uint32_t cw = 0;
    bool fok = false;

#if defined(DMF_EXP_F_REBUILD)
    uint32_t kid = 0;  // the prefetched pair's index in the batch
#endif
    auto decode = [&]() {
      const uint32_t w[5] = {ca.x, ca.y, ca.z, ca.w, cw};
      bk::Slab20 sd;
      bk::unpack20(w, sd);
      b1 = (uint32_t)sd.b1;
      b2 = (uint32_t)sd.b2;
      b12 = (uint32_t)sd.b12;
      K1 = sd.a1;
      K2 = sd.a2;
      K1mM = sd.a1 - sd.aM;
      K2mM = sd.a2 - sd.aM;
      nK1 = 0u - sd.a1;
      cur = sd.entry * 4u;
      r = (int)sd.S;
      // (the strides computed from the record bits in VALU instead measured slower: F 3.39 ->
      // 3.50 ms, profiles/r06f -- the table read's latency is not what the refill waits on)
      const uint4 st3 = slut[cw >> 24];
      dM = st3.x;
      d1 = st3.y;
      d2 = st3.z;
      // the pair's last cell: a hit when the ray ends there inside the grid, else a miss
      const uint32_t Lb = sd.last * 4u;
      atomicAdd((uint32_t*)(lds + Lb), sd.ends ? 0x10000u : 1u);
      // the cells of L's slab before L (misses), at the table's offsets: L - d_e (s >= 1) and
      // the slab's first cell L - d_1 - d_2 (s == 2)
      if (st3.w != 0u) atomicAdd((uint32_t*)(lds + Lb + (uint32_t)(int32_t)(int16_t)(uint16_t)st3.w), 1u);
      if (st3.w > 0xffffu) atomicAdd((uint32_t*)(lds + Lb + (uint32_t)((int32_t)st3.w >> 16)), 1u);
#if defined(DMF_EXP_F_REBUILD)
      {
        // Cost proxy of a compact pair record (B stores <= 8 B, F rebuilds the
        // slab state): per adopted pair, pass B's per-pair arithmetic on a ray record -- its
        // 16-B load (a stand-in ray, monotone in the pair index as B's slot order is), the
        // decode, the f64 reciprocals, the boundary counts at entry and at exit, the entry
        // state and the slab code.  The records stay the product's (exact results); the
        // proxy's values only feed a test that is never true.
        const uint32_t rid = (uint32_t)(((uint64_t)kid * xnrays) / (xnpairs ? xnpairs : 1u));
        const ulonglong2 rr = xrays[rid];
        bk::QRay R;
        bk::decode_ray(rr.x, rr.y, R);
        bk::QRayF64 F64;
        bk::qray_f64(R, F64);
        const int Mx = bk::major_axis(R), m1x = Mx == 0 ? 1 : 0, m2x = Mx == 2 ? 1 : 2;
        int32_t c0[3], c1[3];
        const int32_t ka = (int32_t)(kid & 15u), kb = ka + 1;
        if (Mx == 0) bk::counts_at_f64<0>(R, F64, min(ka, max(R.n[0] - 1, 0)), c0);
        else if (Mx == 1) bk::counts_at_f64<1>(R, F64, min(ka, max(R.n[1] - 1, 0)), c0);
        else bk::counts_at_f64<2>(R, F64, min(ka, max(R.n[2] - 1, 0)), c0);
        if (m1x == 0) bk::counts_at_f64<0>(R, F64, min(kb, max(R.n[0] - 1, 0)), c1);
        else bk::counts_at_f64<1>(R, F64, min(kb, max(R.n[1] - 1, 0)), c1);
        const int32_t aMx = bk::pick3(R.adq[0], R.adq[1], R.adq[2], Mx), a1x = bk::pick3(R.adq[0], R.adq[1], R.adq[2], m1x),
                      a2x = bk::pick3(R.adq[0], R.adq[1], R.adq[2], m2x);
        const uint32_t KMx = 512u * (uint32_t)aMx, K1x = 512u * (uint32_t)a1x, K2x = 512u * (uint32_t)a2x;
        int32_t sb1, sb2, sb12;
        bk::slab_from_pairwise(Mx, bk::e0_pair(R, 0, 1), bk::e0_pair(R, 0, 2), bk::e0_pair(R, 1, 2), sb1, sb2, sb12);
        const uint32_t eb1 = (uint32_t)sb1 + ((uint32_t)bk::mul24(bk::pick3(c0[0], c0[1], c0[2], Mx), a1x) -
                                              (uint32_t)bk::mul24(bk::pick3(c0[0], c0[1], c0[2], m1x), aMx)) * 512u;
        const uint32_t code = bk::slab_code(Mx, sb1, sb2, sb12, KMx, K1x, K2x, c0, c1);
        const uint32_t xw = (uint32_t)(R.cs[0] + bk::mul24(R.st[0], c0[0])) & 31u,
                       yw = (uint32_t)(R.cs[1] + bk::mul24(R.st[1], c0[1])) & 31u,
                       zw = (uint32_t)(R.cs[2] + bk::mul24(R.st[2], c0[2])) & 31u;
        sink ^= code ^ eb1 ^ bk_lds_word(xw, yw, zw);
      }
#endif
    };
    bool more = true;
#if defined(DMF_EXP_F_XVALU)
    uint32_t xv = 0;
#endif
    // lanes in `need` take the next pair indices (one LDS counter atomic, issued by alloc()
    // before the refill's decode so that its return latency hides behind it) and load their
    // records (fetch())
    auto alloc = [&](uint64_t need) -> uint32_t {
      uint32_t base0 = 0;
      if (l == 0) base0 = atomicAdd(&sh[1], (uint32_t)__builtin_popcountll(need));
      return base0;
    };
    auto fetch = [&](uint64_t need, uint32_t base0) {
      const uint32_t nn = (uint32_t)__builtin_popcountll(need);
      const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base0);
      if (base + nn >= n) more = false;
      if ((need >> l) & 1ull) {
        const uint32_t k = base + (uint32_t)lane_prefix(need);
        fok = k < n;
        const uint32_t ob = bk_order<S_ORDER>(k, n);
#if defined(DMF_EXP_F_REBUILD)
        kid = p0 + ob;
#endif
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_a, ob * 16u, 0, 0);
        ca = make_uint4(v[0], v[1], v[2], v[3]);
        cw = __builtin_amdgcn_raw_buffer_load_b32(rs_w, ob * 4u, 0, 0);
      }
    };
    fetch(~0ull, alloc(~0ull));
    for (;;) {
      const uint64_t act = __builtin_amdgcn_ballot_w64(r > 0);
      bool any_act = act != 0;
      DMF_T(tr0);
      // (active lanes counted on 32-bit halves: the 64-bit popcount's compare became a VALU op)
      if (__builtin_popcount((uint32_t)act) + __builtin_popcount((uint32_t)(act >> 32)) <= 64 - REFILL) {
        const uint64_t take = __builtin_amdgcn_ballot_w64(r <= 0 && fok);
        if (take) {
#if defined(DMF_EXP_STATS)
          if (l == 0) ++nrefill;
#endif
          DMF_T(td0);
          const bool pf = more;
          const uint32_t base0 = pf ? alloc(take) : 0u;
          // the lanes of `take`, as a lane mask (their next records are loaded under the same
          // mask: no lane test of `take` in the fetch)
          const bool tk = r <= 0 && fok;
          if (tk) {
            decode();
            fok = false;
          }
#if defined(DMF_EXP_STATS)
          __builtin_amdgcn_s_waitcnt(0);  // close the decode interval on its loads and LDS adds
#endif
          DMF_TACC(t_dec, td0);
          DMF_T(tp0);
          // (read on every path, so that no path leaves the allocation's LDS return pending
          // into the walk block: the compiler's wait for it there drained the LDS queue at every
          // block's end)
          const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base0);
          if (pf) {
            if (base + (uint32_t)__builtin_popcountll(take) >= n) more = false;
            if (tk) {
              const uint32_t k = base + (uint32_t)lane_prefix(take);
              fok = k < n;
              const uint32_t ob = bk_order<S_ORDER>(k, n);
#if defined(DMF_EXP_F_REBUILD)
              kid = p0 + ob;
#endif
              const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_a, ob * 16u, 0, 0);
              ca = make_uint4(v[0], v[1], v[2], v[3]);
              cw = __builtin_amdgcn_raw_buffer_load_b32(rs_w, ob * 4u, 0, 0);
            }
          }
          DMF_TACC(t_pf, tp0);
          any_act = __builtin_amdgcn_ballot_w64(r > 0) != 0;
        }
      }
      DMF_TACC(t_refill, tr0);
      // (no `continue` when no lane walks but records wait -- rare: every decoded pair had no
      // whole slab -- the block below then adds nothing; one loop latch, so that the compiler
      // keeps the walk state in place instead of copying it at every block's end)
      if (!any_act && __builtin_amdgcn_ballot_w64(fok) == 0) break;
      DMF_T(tw0);
#if defined(DMF_EXP_STATS)
      if (l == 0) ++nblocks;
      nlanes += (unsigned long long)__builtin_popcountll(__builtin_amdgcn_ballot_w64(r > 0));
#endif
      // the k-th slab from here is walked iff r > k: inside the block the threshold moves
      // (u) and r drops by UNROLL once at its end
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const bool c1 = (int32_t)b1 >= 0, c2 = (int32_t)b2 >= 0, o2 = (int32_t)b12 >= 0;
        const uint32_t x1 = c1 ? d1 : 0u, x2 = c2 ? d2 : 0u;
        // the slab's cells: cur, then p1 if a minor crosses (on m2 iff o2, also when only
        // one does: dmf_brick.hpp slab_walk_owned), then p2 if both do
        const uint32_t p1 = cur + (o2 ? x2 : x1), p2 = cur + x1 + x2;
        if (r > u) {
          atomicAdd((uint32_t*)(lds + cur), 1u);
          if (c1 || c2) atomicAdd((uint32_t*)(lds + p1), 1u);
          if (c1 && c2) atomicAdd((uint32_t*)(lds + p2), 1u);
#if defined(DMF_EXP_F_XLDS)  // diagnostic (wrong counts): every walk atomic twice
          atomicAdd((uint32_t*)(lds + cur), 1u);
          if (c1 || c2) atomicAdd((uint32_t*)(lds + p1), 1u);
          if (c1 && c2) atomicAdd((uint32_t*)(lds + p2), 1u);
#endif
        }
#if defined(DMF_EXP_F_XVALU)  // diagnostic: independent VALU per slab, kept by a never-true test
        xv = ((xv ^ cur) + b1) ^ (b2 << 1);
        xv = ((xv ^ b12) + p1) ^ (p2 << 2);
#endif
        cur = p2 + dM;
        b1 += c1 ? K1mM : K1;
        b2 += c2 ? K2mM : K2;
        b12 += (c1 ? K2 : 0u) + (c2 ? nK1 : 0u);
      }
      r -= UNROLL;
      DMF_TACC(t_walk, tw0);
    }
#if defined(DMF_EXP_F_XVALU)
    if (xv == 0x9e3779b9u + n) atomicAdd(&hits[0], 0);
#endif
    DMF_T(tf0);
    __syncthreads();
    if constexpr (bk::kLog != 5) {
      // (experiment builds with another brick edge: the generic mapping of k_bk_fuse)
      for (int e = tid; e < bk::kCells; e += blockDim.x) {
        const int tile = e >> 4, w16 = e & 15;
        const int tx = tile >> (2 * bk::kLog - 3), ty = (tile >> (bk::kLog - 2)) & ((bk::kB >> 1) - 1),
                  tz = tile & ((bk::kB >> 2) - 1);
        const int lx = tx * 2 + (w16 >> 3), ly = ty * 2 + ((w16 >> 2) & 1), lz = tz * 4 + (w16 & 3);
        const int li = lx * kBkSx + ly * kBkSy + lz;
        const uint32_t v = box[li];
        if (v) {
          box[li] = 0;
          const uint32_t ti = tiled_index(tl, lo0 + lx, lo1 + ly, lo2 + lz);
          const int32_t mi = (int32_t)(v & 0xffffu), hv = (int32_t)(v >> 16);
          if (mi) atomic_add_dev(&misses[ti], mi);
          if (hv) atomic_add_dev(&hits[ti], hv);
          ++nflush;
        }
      }
    } else
    // flush (one device atomic per non-zero cell and counter): lane tid takes cells
    // e = tid + 1024 k of the brick in the tiled order (16 lanes per 64-B counter line).  The
    // cell's box word and its counter index inside the brick move by per-k constants, so
    // the index math is done once per part, not per cell (cell e: tile e >> 4 = (tx, ty, tz)
    // with tx = k >> 1, ty = 8 (k & 1) + (t0 >> 3), tz = t0 & 7 for t0 = tid >> 4).
    {
      static_assert(bk::kLog != 5 || kBkThreads == 1024, "flush strides: 32^3-cell bricks, 1024 lanes");
      const int t0 = tid >> 4, w16 = tid & 15;
      const int li0 = (w16 >> 3) * kBkSx + (2 * (t0 >> 3) + ((w16 >> 2) & 1)) * kBkSy + 4 * (t0 & 7) + (w16 & 3);
      const uint32_t ti0 = tile_base(tl, lo0 >> 1, lo1 >> 1, lo2 >> 2) +
                           ((((uint32_t)(t0 >> 3)) * tl.nz + (uint32_t)(t0 & 7)) << 4) + (uint32_t)w16;
      const uint32_t sA = (tl.ny * tl.nz) << 4, sB = (8u * tl.nz) << 4;  // tx + 1, ty + 8
#pragma unroll 4
      for (int k = 0; k < bk::kCells / kBkThreads; ++k) {
        const int li = li0 + (k >> 1) * (2 * kBkSx) + (k & 1) * (16 * kBkSy);
        const uint32_t v = box[li];
        if (v) {
          box[li] = 0;
          const uint32_t ti = ti0 + (uint32_t)(k >> 1) * sA + (uint32_t)(k & 1) * sB;
          const int32_t mi = (int32_t)(v & 0xffffu), hv = (int32_t)(v >> 16);
          if (mi) atomic_add_dev(&misses[ti], mi);
          if (hv) atomic_add_dev(&hits[ti], hv);
          ++nflush;
        }
      }
    }
    __syncthreads();
    DMF_TACC(t_flush, tf0);
  }
#if defined(DMF_EXP_F_REBUILD)
  if (sink == 0x9e3779b9u + xnrays) atomicAdd(&hits[0], 0);  // never true in practice: keeps the proxy
#endif
  if (stats) {
    for (int o = 32; o > 0; o >>= 1) nflush += __shfl_down(nflush, o, 64);
    if (l == 0 && nflush) atomicAdd(&stats[6], nflush);
#if defined(DMF_EXP_STATS)
    if (l == 0) {
      atomicAdd(&stats[7], nblocks);
      atomicAdd(&stats[8], nlanes);
      atomicAdd(&stats[9], nrefill);
      atomicAdd(&stats[10], t_refill);
      atomicAdd(&stats[11], t_walk);
      atomicAdd(&stats[12], t_flush);
      atomicAdd(&stats[15], t_bar);
      atomicAdd(&stats[16], t_dec);
      atomicAdd(&stats[17], t_pf);
      const unsigned long long t_end = __builtin_amdgcn_s_memtime();
      atomicMax(&stats[13], t_end - t_start);
      atomicAdd(&stats[14], t_end - t_start);
    }
#endif
    if (tid == 0) {
      if (npairs) atomicAdd(&stats[4], npairs);
      if (nparts_done) atomicAdd(&stats[5], nparts_done);
    }
  }
}
#undef DMF_T
#undef DMF_TACC

// Tiled counters -> clamped int16 log-odds in the reference's x-major voxel order.
// Four lanes per 2x2x4 tile: lane q of the tile reads int4 q of each counter line (the
// 4 z-cells of row (x, y) = (2tx + q/2, 2ty + q%2); a wave's loads are 1 KB contiguous)
// and writes them as one 8-B store; a wave covers 16 tiles along z, so each of its 4 rows
// gets a contiguous 128-B run.  (One lane per 4 z-cells of a row read a quarter of each
// 64-B line per wave and relied on L2 for the rest: 3.7 ms at 1024^3.)
// Tiles [t0, t1) only (a rank's slab after a reduce-scatter).
__global__ __launch_bounds__(256) void k_finalize(Geom g, const int32_t* __restrict__ hits,
                                                  const int32_t* __restrict__ misses, int l_hit, int l_miss,
                                                  int l_min, int l_max, int16_t* __restrict__ out, int64_t t0,
                                                  int64_t t1) {
  const Tiles tl = tiles_of(g.n);
  const int64_t i = t0 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // int4 index
  const int64_t t = i >> 2;
  if (t >= t1) return;
  const int q = (int)(i & 3);
  const int tz = (int)(t % tl.nz);
  const int64_t r = t / tl.nz;
  const int ty = (int)(r % tl.ny), tx = (int)(r / tl.ny);
  const int x = tx * 2 + (q >> 1), y = ty * 2 + (q & 1), z = tz * 4;
  const int4 h = ((const int4*)hits)[i], m = ((const int4*)misses)[i];
  if (x >= g.n[0] || y >= g.n[1]) return;
  auto f = [&](int32_t hv, int32_t mv) -> int16_t {
    int64_t L = (int64_t)hv * l_hit + (int64_t)mv * l_miss;
    L = L < l_min ? l_min : (L > l_max ? l_max : L);
    return (int16_t)L;
  };
  const int16_t o[4] = {f(h.x, m.x), f(h.y, m.y), f(h.z, m.z), f(h.w, m.w)};
  int16_t* dst = out + (((int64_t)x * g.n[1] + y) * g.n[2] + z);
  if (z + 4 <= g.n[2] && ((uintptr_t)dst & 7) == 0) {
    *(uint2*)dst = *(const uint2*)o;
  } else {
    for (int k = 0; k < 4 && z + k < g.n[2]; ++k) dst[k] = o[k];
  }
}

// Linear (x-major) <-> tiled counter copies for the host-pointer API and tests.
template <bool kToLinear>
__global__ __launch_bounds__(256) void k_counter_layout(Geom g, const int32_t* __restrict__ src,
                                                        int32_t* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t nyz = (int64_t)g.n[1] * g.n[2];
  const int x = (int)(i / nyz);
  const int64_t rr = i - x * nyz;
  const int y = (int)(rr / g.n[2]), z = (int)(rr - (int64_t)y * g.n[2]);
  const uint32_t ti = tiled_index(tiles_of(g.n), x, y, z);
  if (kToLinear) dst[i] = src[ti];
  else dst[ti] = src[i];
}

// Fusion implementation of a volume (dmf_diag.h dmf_fuse_set_variant; 0 = by grid size).
static bool is_known_variant(int v) {
  return v == DMF_FUSE_DEFAULT || v == DMF_FUSE_LDS_BOX || v == DMF_FUSE_CELL_WALK || v == DMF_FUSE_SLAB;
}

static BkGeom brick_geom(const Geom& g) {
  BkGeom bg;
  for (int a = 0; a < 3; ++a) bg.nb[a] = (g.n[a] + bk::kB - 1) >> bk::kLog;
  bg.nbricks = bg.nb[0] * bg.nb[1] * bg.nb[2];
  return bg;
}

// The brick path covers grids up to 1024 cells per axis (18-bit |dq| fields in the
// pair record) and <= 32768 bricks (LDS histogram of passes A/B).
static bool brick_path_ok(const Geom& g) {
  const BkGeom bg = brick_geom(g);
  return g.n[0] <= 1024 && g.n[1] <= 1024 && g.n[2] <= 1024 && bg.nbricks <= kBkScanMax;
}

// Default choice: the brick pipeline pays a per-ray cost (passes A/B) that the shorter rays
// of small grids do not amortise.  Measured on MI355X (640x480 frames, slab walk): 256^3 (64
// frames) brick 2.43 ms vs k_fuse_l 2.50; 320^3 2.91 vs 3.08; 384^3 3.30 vs 3.62; 512^3 (128
// frames) 7.6 vs 10.2; 1024^3 (32 frames) brick ahead by 2x.
static bool brick_preferred(const Geom& g) {
  return std::max(g.n[0], std::max(g.n[1], g.n[2])) >= 256;
}

static bool use_bricks(const dmf_volume* v, const Geom& g) {
  if (!brick_path_ok(g)) return false;
  const int fv = v->fuse_variant;
  return fv == DMF_FUSE_SLAB || fv == DMF_FUSE_CELL_WALK || (fv == DMF_FUSE_DEFAULT && brick_preferred(g));
}

// slabs per walk block of phase F: 8 (round 4 sweep 4/5/6/8/10/12 with pipelined calls: 8 is
// 1 % faster than 4 at 512^3 and at config 2, the others slower); with 8-slab blocks a wave
// refills at >= 16 idle lanes (sweep 16/20/24/32, picks over 16/32/64 regions: serial -1 %,
// config 2 -0.5 %, pipelined within the box's drift)
#if defined(DMF_EXP_F_UNROLL)  // experiment builds: slabs per walk block
constexpr int kBkUnroll = DMF_EXP_F_UNROLL;
#else
constexpr int kBkUnroll = 8;
#endif
#if defined(DMF_EXP_F_REFILL)  // experiment builds: refill threshold / pick spread of phase F
constexpr int kBkRefill = DMF_EXP_F_REFILL, kBkSpread = DMF_EXP_F_SPREAD;
#else
constexpr int kBkRefill = 16, kBkSpread = 32;
#endif
constexpr const char* kNameSlab = "dmf::k_bk_fuse_s<16, 32, 8>";
constexpr const char* kNameCell = "dmf::k_bk_fuse<16, 8, 8>";
constexpr const char* kNameLds = "dmf::k_fuse_l<12, 1280>";

static int cu_count(int device) {
  static std::atomic<int> cached{0};
  int n = cached.load();
  if (n <= 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n <= 0) n = 256;
    cached.store(n);
  }
  return n;
}

// Batching of the brick pipeline.  The (ray, brick) pairs a call makes are known only on
// the device (pass A), and the fusion call never reads anything back (no host sync, no
// allocation once reserved: dmf_fuse_reserve).  So the host plans by bounds and the device
// decides: pass A runs once over a super-batch of poses (all P when their ray records fit
// half the slot's budget), counting pairs per (pose, brick); k_bk_batches cuts the poses
// into batches by the pairs they really make against the pair capacity (the rest of the
// slot's budget, at most the geometric bound of the super-batch); the host launches jmax =
// the batches the geometric bound rays x (1 + brick boundaries) would need, and the launches
// past the device's batch count exit at once.  Budget (dmf_fuse_reserve): 55 % of the
// device's HBM by default (~158 GB of MI355X's 288 GB), all of it for the one slot of serial
// calls, half of it for each of the two staging slots of pipelined calls: the 1024-pose
// 512^3 anchor and the 256-pose 1024^3 shard each run as one batch either way.

struct BkPlan {
  BkGeom bg;
  int pkx = 0, pky = 0;
  int64_t ppose = 0;          // 8x8 packets per pose
  int64_t max_pairs_ray = 0;  // geometric bound of (ray, brick) pairs per ray
  int64_t PS = 0;             // poses per super-batch (one pass A over all of them)
  int64_t PBg = 0;            // poses per batch under the geometric bound (>= 1)
  int max_poses = 0;          // cap of poses per batch (DMF_KNOB_BATCH_POSES test hook; else PS)
  int ab_threads = 0, span = 0, wg_pose = 0, wgl_stride = 0;
  int hash_log = 0;  // pass A's hashed histogram: log2 of its words (0 = the direct table)
  uint32_t part_max = kBkPartMax;  // pairs per part of phase F (DMF_KNOB_PART_MAX)
  size_t rec_bytes = 20;           // bytes per pair record: 16 (pa) + 4 (slab walk) or 16 + 8 (per-cell walk)
  size_t hist_bytes = 0;
  uint64_t pair_cap = 0;  // pair records reserved per slot (shared by the batches of a call)
  uint64_t per_pose_bytes = 0;
  uint64_t slot_bytes = 0;  // device scratch of one slot
  int slots = 1;            // 2 when the calls are pipelined
  int64_t jmax(int64_t ps) const { return (ps + PBg - 1) / PBg; }
  int64_t max_batches(int64_t P) const { return (P / PS) * jmax(PS) + (P % PS ? jmax(P % PS) : 0); }
  int split_cu = 0;  // k_bk_scan's tail split: F's workgroups | entries split per CU << 16 (0 = off)
  size_t max_parts() const { return (size_t)bg.nbricks + pair_cap / part_max + 1 + 3 * 1024; }
};

static int bk_plan(const dmf_volume* v, const CamP& cp, const Geom& g, int P, BkPlan& pl) {
  const int64_t* kn = v->knob;
  pl.bg = brick_geom(g);
  pl.pkx = (cp.W + 7) / 8;
  pl.pky = (cp.H + 7) / 8;
  pl.ppose = (int64_t)pl.pkx * pl.pky;
  pl.max_pairs_ray = 1 + (pl.bg.nb[0] - 1) + (pl.bg.nb[1] - 1) + (pl.bg.nb[2] - 1);
  pl.rec_bytes = v->fuse_variant == DMF_FUSE_CELL_WALK ? 24 : 20;
  const int64_t rays_pose = pl.ppose * 64;
  const uint64_t one_pose = (uint64_t)rays_pose * (uint64_t)pl.max_pairs_ray;  // pairs of one pose, at most
  if (one_pose > (uint64_t)UINT32_MAX) return fail(DMF_ERR_RANGE, "one frame exceeds the 32-bit pair offsets");
  pl.ab_threads = pl.bg.nbricks > kBkBigHist ? kBkPassThreadsBig : kBkPassThreads;
#if defined(DMF_EXP_AB_THREADS)  // experiment builds: passes A/B workgroup size below kBkBigHist bricks
  if (pl.bg.nbricks <= kBkBigHist) pl.ab_threads = DMF_EXP_AB_THREADS;
#endif
  // packets per workgroup of passes A/B (>= 16 per wave; the histogram's zero + flush
  // amortised over >= 64 packets per 1k bricks).  Up to 512 bricks (grids <= 256^3) the
  // histogram is small enough for 8 per wave: config 2 fusion 2.05 -> 2.02 ms, while 384^3
  // and 512^3 measured slower at 32 packets than at 64
  pl.span = std::max((pl.bg.nbricks <= 512 ? 8 : 16) * (pl.ab_threads / 64), (pl.bg.nbricks + 63) / 64);
  // over kBkBigHist bricks pass A counts into a hashed histogram of 2048 words (8 KB: it runs
  // beside phase F's box when calls are pipelined; the 64-KB direct table cannot) over spans
  // of 128 packets (a few hundred touched bricks per workgroup at 1024^3)
  if (kn[DMF_KNOB_A_HASH] > 0) {
    int lg = 4;
    while (lg < 14 && (1ll << lg) < kn[DMF_KNOB_A_HASH]) ++lg;  // 16 .. 16384 words (64 KB)
    pl.hash_log = lg;
  } else if (kn[DMF_KNOB_A_HASH] == 0 && pl.bg.nbricks > kBkBigHist) {
    pl.hash_log = 11;
    pl.span = 128;
  }
  // (at most 1023 packets: a workgroup's pairs per brick, <= span * 64, fit the 16-bit counts
  // of pass A's histogram and of its touched-brick list)
  if (kn[DMF_KNOB_SPAN] > 0) pl.span = (int)std::max<int64_t>(4, std::min<int64_t>(kn[DMF_KNOB_SPAN], 1023));
  if (kn[DMF_KNOB_PART_MAX] > 0)
    pl.part_max = (uint32_t)std::max<int64_t>(1024, std::min<int64_t>(kn[DMF_KNOB_PART_MAX], kBkPartMax));
  pl.wg_pose = (int)((pl.ppose + pl.span - 1) / pl.span);
  pl.hist_bytes = sizeof(uint32_t) * (size_t)pl.bg.nbricks;
  // per pose: ray records, per-workgroup brick bases, pose counts and bases, pose pairs + batch table
  // touched-brick list per workgroup: count + one word per touched brick (uint16 id | uint16
  // pair count: pass B's layout check; ADVICE r5 -- 1.5 words per brick before)
  pl.wgl_stride = 1 + pl.bg.nbricks;
  pl.per_pose_bytes = (uint64_t)rays_pose * (sizeof(ulonglong2) + sizeof(uint64_t)) + (uint64_t)pl.wg_pose * pl.hist_bytes +
                      (uint64_t)pl.wg_pose * sizeof(uint32_t) * (uint64_t)pl.wgl_stride + 2 * (uint64_t)pl.hist_bytes +
                      sizeof(unsigned long long) + sizeof(uint32_t);
  // pipelined calls: two staging slots, each with its own pair records, share the budget
  pl.slots = v->pipelined ? 2 : 1;
  const uint64_t budget = v->bk_budget / (uint64_t)pl.slots;
  pl.PS = std::min<int64_t>(P, (int64_t)(budget / 2 / pl.per_pose_bytes));
  if (kn[DMF_KNOB_SUPER_POSES] > 0) pl.PS = std::min<int64_t>(pl.PS, kn[DMF_KNOB_SUPER_POSES]);
  if (pl.PS < 1) return fail(DMF_ERR_RANGE, "one frame exceeds the brick fusion budget (dmf_fuse_reserve)");
  // (below pass B's slot sentinel: a slot taken from an uncounted brick is never in range)
  pl.pair_cap = std::min<uint64_t>({(budget - (uint64_t)pl.PS * pl.per_pose_bytes) / pl.rec_bytes,
                                    (uint64_t)pl.PS * one_pose, (uint64_t)kBkSlotSentinel - 1});
  if (pl.pair_cap < one_pose) return fail(DMF_ERR_RANGE, "one frame exceeds the brick fusion pair budget (dmf_fuse_reserve)");
  if (kn[DMF_KNOB_PAIR_CAP] > 0)  // test hook: the caller guarantees it holds any one pose's pairs
    pl.pair_cap = std::min<uint64_t>(pl.pair_cap, (uint64_t)kn[DMF_KNOB_PAIR_CAP]);
  pl.max_poses = (int)pl.PS;
  if (kn[DMF_KNOB_BATCH_POSES] > 0) pl.max_poses = (int)std::min<int64_t>(pl.PS, kn[DMF_KNOB_BATCH_POSES]);
  pl.PBg = std::max<int64_t>(1, std::min<int64_t>(pl.max_poses, (int64_t)(pl.pair_cap / one_pose)));
  // tail split of the part queue (k_bk_scan, slab walk only): on for serial calls; pipelined
  // calls skip it (the next call's pass A fills the queue's last round there: config 2 1.78
  // -> 1.74 ms per call without the split)
  const int64_t ts = kn[DMF_KNOB_TAIL_SPLIT];
  if (v->fuse_variant != DMF_FUSE_CELL_WALK && ts >= 0 && (ts > 0 || !v->pipelined)) {
    const int k = ts > 0 ? (int)std::min<int64_t>(ts, 8) : 2;  // entries split: k per CU
    pl.split_cu = std::min(512, cu_count(v->device)) | (k << 16);
  }
  pl.slot_bytes = pl.pair_cap * pl.rec_bytes + (uint64_t)pl.PS * pl.per_pose_bytes +
                  sizeof(uint32_t) * (3 * (uint64_t)pl.bg.nbricks + 6 + 2 * pl.max_parts()) +
                  sizeof(unsigned long long) * 4;
  return DMF_OK;
}

// A/B histograms above 48 KiB of dynamic LDS need the attribute (once per process).
static int bk_attributes() {
  static std::atomic<bool> attr_set{false};
  if (!attr_set.load()) {
    const int lds = (int)(sizeof(uint32_t) * 32768);
    DMF_HIP(hipFuncSetAttribute((const void*)k_bk_rays<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    DMF_HIP(hipFuncSetAttribute((const void*)k_bk_rays_recover, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    DMF_HIP(hipFuncSetAttribute((const void*)k_bk_rays_hash, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    DMF_HIP(hipFuncSetAttribute((const void*)k_bk_pairs<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    DMF_HIP(hipFuncSetAttribute((const void*)k_bk_pairs<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set.store(true);
  }
  return DMF_OK;
}

// The scratch of a plan: ray records, brick counts / offsets / part table / part order,
// queue control words, per-workgroup and per-pose brick bases, pose pair counts and the
// batch table, pair records.
struct BkBufs {
  ulonglong2* rays = nullptr;
  uint64_t* paths = nullptr;
  uint32_t *cnt = nullptr, *off = nullptr, *part_pref = nullptr, *wgb = nullptr, *wgl = nullptr;
  uint32_t *pose_cnt = nullptr, *pose_base = nullptr, *bt = nullptr;
  unsigned long long* pose_pairs = nullptr;
  uint2* order = nullptr;
  unsigned long long* ctl = nullptr;
  uint4* pra = nullptr;
  void* prb = nullptr;  // uint32 per pair (20-B records) or uint2 (24-B records)
  uint32_t* ovl = nullptr;  // pass A's overflow list [count | workgroups]
};

// Allocates only when a slot is too small.  `slot` = 0 or 1: the two staging slots of
// pipelined fusion (serial calls use slot 0).
static int bk_scratch(dmf_volume* v, const BkPlan& pl, BkBufs& b, int slot) {
  const size_t PS = (size_t)pl.PS, nb = (size_t)pl.bg.nbricks;
  void *rays, *bricks, *ctl, *wgb, *wgl, *pra, *prb, *pcnt, *pbase, *batch;
  const size_t nrays = (size_t)(pl.PS * pl.ppose * 64);  // ray records, then the crossing paths
  DMF_TRY(scratch(v, slot ? kScBkRays1 : kScBkRays, (sizeof(ulonglong2) + sizeof(uint64_t)) * nrays, &rays));
  // cnt | off | part_pref (nbricks + 1) | order (uint2 per part)
  DMF_TRY(scratch(v, slot ? kScBkBricks1 : kScBkBricks, sizeof(uint32_t) * (3 * nb + 6 + 2 * pl.max_parts()), &bricks));
  DMF_TRY(scratch(v, slot ? kScBkCtl1 : kScBkCtl, sizeof(unsigned long long) * 4, &ctl));
  DMF_TRY(scratch(v, slot ? kScBkWgBase1 : kScBkWgBase, pl.hist_bytes * (size_t)pl.wg_pose * PS, &wgb));
  DMF_TRY(scratch(v, slot ? kScBkWgList1 : kScBkWgList,
                  sizeof(uint32_t) * (size_t)pl.wgl_stride * (size_t)pl.wg_pose * PS, &wgl));
  // pair records: pair_cap, plus the spare record pass B's store guard writes to
  DMF_TRY(scratch(v, slot ? kScBkPairs1 : kScBkPairs, sizeof(uint4) * ((size_t)pl.pair_cap + 1), &pra));
  DMF_TRY(scratch(v, slot ? kScBkPairsB1 : kScBkPairsB, (pl.rec_bytes - sizeof(uint4)) * ((size_t)pl.pair_cap + 1),
                  &prb));
  DMF_TRY(scratch(v, slot ? kScBkPoseCnt1 : kScBkPoseCnt, pl.hist_bytes * PS, &pcnt));
  DMF_TRY(scratch(v, slot ? kScBkPoseBase1 : kScBkPoseBase, pl.hist_bytes * PS, &pbase));
  DMF_TRY(scratch(v, slot ? kScBkBatch1 : kScBkBatch, sizeof(unsigned long long) * PS + sizeof(uint32_t) * (PS + 4),
                  &batch));
  void* ovl;
  DMF_TRY(scratch(v, slot ? kScBkOvf1 : kScBkOvf, sizeof(uint32_t) * (1 + (size_t)pl.wg_pose * PS), &ovl));
  b.ovl = (uint32_t*)ovl;
  b.rays = (ulonglong2*)rays;
  b.paths = (uint64_t*)(b.rays + nrays);
  b.cnt = (uint32_t*)bricks;
  b.off = b.cnt + nb;
  b.part_pref = b.off + nb;  // nbricks + 1
  b.order = (uint2*)(b.part_pref + nb + 4 + (nb & 1));  // 8-B aligned
  b.wgb = (uint32_t*)wgb;
  b.wgl = (uint32_t*)wgl;
  b.ctl = (unsigned long long*)ctl;
  b.pra = (uint4*)pra;
  b.prb = prb;
  b.pose_cnt = (uint32_t*)pcnt;
  b.pose_base = (uint32_t*)pbase;
  b.pose_pairs = (unsigned long long*)batch;
  b.bt = (uint32_t*)(b.pose_pairs + PS);
  return DMF_OK;
}

// Frees the brick pipeline's scratch (both slots), after the work in flight that may read
// it: a volume switching between serial and pipelined calls re-plans its slots against the
// budget (one slot of the whole budget, or two of half).
static int bk_release(dmf_volume* v) {
  static const int kSlots[] = {kScBkRays, kScBkPairs, kScBkPairsB, kScBkBricks, kScBkWgBase, kScBkCtl, kScBkPoseCnt,
                               kScBkPoseBase, kScBkBatch, kScBkWgList, kScBkRays1, kScBkWgBase1, kScBkWgList1,
                               kScBkPoseCnt1, kScBkBatch1, kScBkBricks1, kScBkCtl1, kScBkPairs1, kScBkPairsB1,
                               kScBkPoseBase1, kScBkOvf, kScBkOvf1};
  if (v->stream) DMF_HIP(hipStreamSynchronize(v->stream));
  if (v->stage) DMF_HIP(hipStreamSynchronize(v->stage));
  for (int k : kSlots) {
    if (k < (int)v->scratch.size() && v->scratch[k].first) {
      DMF_HIP(hipFree(v->scratch[k].first));
      v->scratch[k] = {nullptr, 0};
    }
  }
  v->bk_last_bt = nullptr;
  return DMF_OK;
}

// Brick-owned fusion of P frames (kernels above).  Only enqueues work: per super-batch,
// pass A over all its poses, the device's batch cut, then per batch the brick layout
// (k_bk_batch_counts, k_bk_scan), pass B and phase F; a launch past the device's batch
// count exits at once.  Phase F reads its part count itself (its persistent workgroups exit
// when the queue is empty).
// Pipelined (staged): the pose table and pass A of each super-batch run on
// the volume's staging stream into staging slot s (alternating), after the caller's input
// stream and after the slot's previous reader (event st_free[s]), beside the previous call's
// phase F; the batch cut, the brick layout, pass B and phase F run on the volume's stream
// after pass A's event; the input stream waits for pass A (the inputs stay ordered before the
// caller's next writes).  Pass A's statistics go to the slot's own striped buffer, summed into
// d_user on the staging stream.  Serial calls use slot 0 on the volume's stream; once the staging stream exists
// they record st_free[0] too, so that a later pipelined call on slot 0 waits for them.
static int stage_init(dmf_volume* v) {
  if (v->stage) return DMF_OK;
  DMF_HIP(hipStreamCreateWithFlags(&v->stage, hipStreamNonBlocking));
  DMF_HIP(hipEventCreateWithFlags(&v->st_in, hipEventDisableTiming));
  for (int k = 0; k < 2; ++k) {
    DMF_HIP(hipEventCreateWithFlags(&v->st_done[k], hipEventDisableTiming));
    DMF_HIP(hipEventCreateWithFlags(&v->st_free[k], hipEventDisableTiming));
    DMF_HIP(hipEventCreateWithFlags(&v->st_b[k], hipEventDisableTiming));
    DMF_HIP(hipEventCreateWithFlags(&v->st_a[k], hipEventDisableTiming));
    v->st_b_set[k] = false;
    v->st_free_set[k] = false;
  }
  // work already enqueued on the volume's stream (a serial call's slot 0 readers) precedes
  // the first staged use of slot 0
  DMF_HIP(hipEventRecord(v->st_free[0], v->stream));
  v->st_free_set[0] = true;
  return DMF_OK;
}

// The volume's two fault words (dmf_fuse_status), zeroed once when first needed (the volume's
// stream is synchronised then: every stream that later reads them is ordered after it).
static int fault_words(dmf_volume* v) {
  if (v->d_fault) return DMF_OK;
  void* p = nullptr;
  DMF_HIP(hipMalloc(&p, 2 * sizeof(uint32_t)));
  v->d_fault = (uint32_t*)p;
  DMF_HIP(hipMemsetAsync(p, 0, 2 * sizeof(uint32_t), v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
}

static int fuse_bricks(dmf_volume* v, const CamP& cp, const Geom& g, const uint16_t* d_depth, const PoseX* tab,
                       const float* d_poses, int P, const dmf_fuse_params* prm, int32_t* d_hits, int32_t* d_misses,
                       unsigned long long* st, uint64_t* d_user, bool staged, bool capturing) {
  BkPlan pl;
  DMF_TRY(bk_plan(v, cp, g, P, pl));
  const BkGeom& bg = pl.bg;
  DMF_TRY(bk_attributes());
  DMF_TRY(fault_words(v));
  BkBufs b;
  if (staged) DMF_TRY(stage_init(v));
  const bool slab = v->fuse_variant != DMF_FUSE_CELL_WALK;
  // pass A with 16-bit histogram counts (a workgroup's pairs per brick <= span * 64 rays; the
  // plan holds span <= 1023)
  if ((int64_t)pl.span * 64 > 65535) return fail(DMF_ERR_RANGE, "pass A span %d exceeds 16-bit counts", pl.span);
  const unsigned nf = (unsigned)cu_count(v->device);
  // phase F's persistent workgroups: one per CU (32^3 bricks); an experiment build with
  // smaller bricks holds as many per CU as fit
  unsigned nfF = nf;
  if constexpr (bk::kLog != 5) {
    int per = 0;
    DMF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per, (const void*)k_bk_fuse_s<kBkRefill, kBkSpread, kBkUnroll>, kBkThreads, 0));
    nfF = nf * (unsigned)std::max(per, 1);
  }
  for (int64_t s0 = 0; s0 < P; s0 += pl.PS) {
    const int64_t ps = std::min<int64_t>(pl.PS, P - s0);
    const unsigned nwg = (unsigned)(ps * pl.wg_pose);
    const int slot = staged ? v->st_slot : 0;
    DMF_TRY(bk_scratch(v, pl, b, slot));
    // everything but phase F: the staging stream (pipelined) or the volume's stream
    const hipStream_t sa = staged ? v->stage : v->stream;
    const PoseX* tab_a = staged ? nullptr : tab + s0;
    unsigned long long* st_a = st;
    if (staged) {
      v->st_slot ^= 1;
      DMF_HIP(hipEventRecord(v->st_in, v->in_stream));
      DMF_HIP(hipStreamWaitEvent(sa, v->st_in, 0));
      if (v->st_free_set[slot]) DMF_HIP(hipStreamWaitEvent(sa, v->st_free[slot], 0));
      void* t;
      DMF_TRY(scratch(v, slot ? kScStPoses1 : kScStPoses0, sizeof(PoseX) * (size_t)pl.PS, &t));
      DMF_TRY(pose_table_into(d_poses + (size_t)s0 * 12, (int)ps, (PoseX*)t, sa));
      tab_a = (const PoseX*)t;
      if (st) {
        void* sbuf;
        DMF_TRY(scratch(v, slot ? kScStStats1 : kScStStats0, sizeof(unsigned long long) * kStatSlots * kStatWidth, &sbuf));
        DMF_HIP(hipMemsetAsync(sbuf, 0, sizeof(unsigned long long) * kStatSlots * kStatWidth, sa));
        st_a = (unsigned long long*)sbuf;
      }
    }
    DMF_HIP(hipMemsetAsync(b.pose_cnt, 0, pl.hist_bytes * (size_t)ps, sa));
    DMF_HIP(hipMemsetAsync(b.pose_pairs, 0, sizeof(unsigned long long) * (size_t)ps, sa));
    // pass A after the previous super-batch's pass B: it then runs beside that super-batch's
    // phase F (launched at once, it would run beside pass B instead, and phase F alone); the
    // pose table and the zeroing above may run beside pass B
    if (staged && v->st_b_set[slot ^ 1]) DMF_HIP(hipStreamWaitEvent(sa, v->st_b_ev[slot ^ 1], 0));
    BkRaysArgs ra{g, cp, d_depth + (size_t)s0 * cp.H * cp.W, tab_a, prm->dmin_mm, prm->dmax_mm, pl.pkx, (int)pl.ppose,
                  pl.wg_pose, pl.span, bg, b.rays, b.paths, b.pose_cnt, b.wgb, b.wgl, pl.wgl_stride, b.pose_pairs,
                  st_a, b.ovl, 0};
    if (pl.hash_log > 0) {
      // hashed histogram (8 KB: beside phase F's box), then the overflowed workgroups (if any)
      // with the direct table
      ra.hash_log = pl.hash_log;
      DMF_HIP(hipMemsetAsync(b.ovl, 0, sizeof(uint32_t), sa));
      hipLaunchKernelGGL(k_bk_rays_hash, dim3(nwg), dim3(kBkPassThreads), sizeof(uint32_t) << pl.hash_log, sa, ra);
      DMF_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_bk_rays_recover, dim3(nf), dim3(kBkPassThreadsBig), sizeof(uint32_t) * ((bg.nbricks + 1) / 2),
                         sa, ra);
    } else {
      hipLaunchKernelGGL(k_bk_rays<true>, dim3(nwg), dim3(pl.ab_threads), sizeof(uint32_t) * ((bg.nbricks + 1) / 2), sa,
                         ra);
    }
    DMF_LAUNCH_CHECK();
    if (staged) {
      // the layout, pass B and phase F on the volume's stream after pass A (event st_a): pass
      // B follows the previous call's phase F in stream order (it never ran beside it: pass
      // A's tail outlasts F), and phase F follows pass B with no cross-stream event (13 -> 7
      // us per call).  Pass A's statistics are then summed here, on the staging stream
      // (atomic sums: the previous call's are summed on the volume's stream meanwhile), off
      // the chain to pass B; st_done (after them) orders the input stream, and the volume's
      // stream after this call's phase F.
      DMF_HIP(hipEventRecord(v->st_a[slot], sa));
      DMF_HIP(hipStreamWaitEvent(v->stream, v->st_a[slot], 0));
      if (st) DMF_TRY(stats_end(v, st_a, d_user, kStatWidth, nullptr, sa));
      DMF_HIP(hipEventRecord(v->st_done[slot], sa));
      DMF_HIP(hipStreamWaitEvent(v->in_stream, v->st_done[slot], 0));
    }
    // everything after pass A: the volume's stream
    const hipStream_t sl = v->stream;
    // small grids: batch cut, brick counts and scan in one launch per batch (k_bk_layout1)
    const bool layout1 = bg.nbricks <= kBkLayout1Bricks && ps <= kBkLayout1Poses;
    if (!layout1) {
      hipLaunchKernelGGL(k_bk_batches, dim3(1), dim3(1024), 0, sl, (int)ps, (const unsigned long long*)b.pose_pairs,
                         (unsigned long long)pl.pair_cap, pl.max_poses, b.bt);
      DMF_LAUNCH_CHECK();
    }
    v->bk_last_bt = b.bt;
    const int64_t jm = pl.jmax(ps);
    for (int64_t j = 0; j < jm; ++j) {
      // batch j > 0 reuses the slot's pair records and part queue, so it follows batch j-1's
      // phase F in stream order.  The host launches jmax triples from the one-pose bound;
      // those past the device's batch count exit at once (1024^3: jmax 7, one batch).
      const hipStream_t sj = sl;
      // (the scan zeroes phase F's queue head: no memset of ctl)
      if (layout1) {
        hipLaunchKernelGGL(k_bk_layout1, dim3(1), dim3(1024), 0, sj, (int)ps, (const unsigned long long*)b.pose_pairs,
                           (unsigned long long)pl.pair_cap, pl.max_poses, b.bt, bg.nbricks, (int)j,
                           (const uint32_t*)b.pose_cnt, b.pose_base, b.cnt, b.off, b.part_pref, b.ctl, b.order,
                           pl.part_max, pl.split_cu);
      } else {
        hipLaunchKernelGGL(k_bk_batch_counts, dim3((unsigned)((bg.nbricks + 255) / 256)), dim3(256), 0, sj,
                           bg.nbricks, (int)j, (const uint32_t*)b.bt, (const uint32_t*)b.pose_cnt, b.pose_base, b.cnt);
        DMF_LAUNCH_CHECK();
      }
      if (layout1) {
      } else if (bg.nbricks > 4096)
        hipLaunchKernelGGL(k_bk_scan<true>, dim3(1), dim3(1024), 0, sj, bg.nbricks, (const uint32_t*)b.cnt, b.off,
                           b.part_pref, b.ctl, b.order, pl.part_max, (const uint32_t*)b.bt, (int)j, pl.split_cu);
      else
        hipLaunchKernelGGL(k_bk_scan<false>, dim3(1), dim3(1024), 0, sj, bg.nbricks, (const uint32_t*)b.cnt, b.off,
                           b.part_pref, b.ctl, b.order, pl.part_max, (const uint32_t*)b.bt, (int)j, pl.split_cu);
      DMF_LAUNCH_CHECK();
      if (slab)
        hipLaunchKernelGGL(k_bk_pairs<true>, dim3(nwg), dim3(pl.ab_threads), pl.hist_bytes, sj, (int)pl.ppose,
                           pl.wg_pose, pl.span, bg, (const ulonglong2*)b.rays, (const uint64_t*)b.paths, (const uint32_t*)b.off,
                           (const uint32_t*)b.pose_base, (const uint32_t*)b.wgb, (const uint32_t*)b.bt, (int)j,
                           (const uint32_t*)b.wgl, pl.wgl_stride, b.pra, b.prb, b.ctl,
                           v->d_fault, (int)std::min<int64_t>(v->knob[DMF_KNOB_FAULT_INJECT], 1 << 20), st);
      else
        hipLaunchKernelGGL(k_bk_pairs<false>, dim3(nwg), dim3(pl.ab_threads), pl.hist_bytes, sj, (int)pl.ppose,
                           pl.wg_pose, pl.span, bg, (const ulonglong2*)b.rays, (const uint64_t*)b.paths, (const uint32_t*)b.off,
                           (const uint32_t*)b.pose_base, (const uint32_t*)b.wgb, (const uint32_t*)b.bt, (int)j,
                           (const uint32_t*)b.wgl, pl.wgl_stride, b.pra, b.prb, b.ctl,
                           v->d_fault, (int)std::min<int64_t>(v->knob[DMF_KNOB_FAULT_INJECT], 1 << 20), st);
      DMF_LAUNCH_CHECK();
      // the call's phase F begins (not while capturing: the record would become a graph node
      // and the caller's event would never be re-recorded by the graph's launches)
      const bool fev = v->f_event && !capturing && s0 == 0 && j == 0;
      if (fev) DMF_HIP(hipEventRecord(v->f_event, v->stream));
      if (staged && j == 0) {
        // pass B done: the next super-batch's pass A waits for it (the caller's phase event,
        // recorded at the same point, serves when there is one: each record costs the chain
        // to phase F a few us)
        if (!fev) DMF_HIP(hipEventRecord(v->st_b[slot], sl));
        v->st_b_ev[slot] = fev ? v->f_event : v->st_b[slot];
        v->st_b_set[slot] = true;
      }
      if (slab)
        hipLaunchKernelGGL((k_bk_fuse_s<kBkRefill, kBkSpread, kBkUnroll>), dim3(nfF), dim3(kBkThreads), 0, v->stream, g, bg,
                           (const uint4*)b.pra, (const uint32_t*)b.prb, (const uint32_t*)b.off, (const uint32_t*)b.cnt,
                           (const uint2*)b.order, pl.part_max, b.ctl, d_hits, d_misses, st, (const ulonglong2*)b.rays,
                           (uint32_t)(ps * pl.ppose * 64), (uint32_t)std::min<uint64_t>(pl.pair_cap, UINT32_MAX));
      else
        hipLaunchKernelGGL((k_bk_fuse<16, 8, 8>), dim3(nf), dim3(kBkThreads), 0, v->stream, g, bg, (const uint4*)b.pra,
                           (const uint2*)b.prb, (const uint32_t*)b.off, (const uint32_t*)b.cnt,
                           (const uint32_t*)b.part_pref, b.ctl, d_hits, d_misses, st);
      DMF_LAUNCH_CHECK();
      if (staged) DMF_HIP(hipEventRecord(v->st_free[slot], v->stream));  // batch j's phase F
    }
    // pass A's statistics summed before the call's own (after phase F: off the chain)
    if (staged) DMF_HIP(hipStreamWaitEvent(v->stream, v->st_done[slot], 0));
    if (staged || (v->stage && !capturing)) {  // the slot's last reader (phase F) is enqueued
      DMF_HIP(hipEventRecord(v->st_free[slot], v->stream));
      v->st_free_set[slot] = true;
    }
  }
  return DMF_OK;
}

int finalize_tiles(dmf_volume* v, const int32_t* d_hits, const int32_t* d_misses, const dmf_fuse_params* prm,
                   int16_t* d_out, int64_t t0, int64_t t1, hipStream_t stream) {
  if (t1 <= t0) return DMF_OK;
  const int64_t lanes = (t1 - t0) * 4;  // four lanes per 2x2x4 tile
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, stream, v->geom(), d_hits,
                     d_misses, prm->l_hit, prm->l_miss, prm->l_min, prm->l_max, d_out, t0, t1);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
}

int tile_rows(const dmf_volume* v, int64_t* ntx, int64_t* tiles_per_row) {
  const Geom g = v->geom();
  const Tiles tl = tiles_of(g.n);
  *ntx = (g.n[0] + 1) >> 1;
  *tiles_per_row = (int64_t)tl.ny * tl.nz;
  return DMF_OK;
}

static const dmf_fuse_params kDefaultParamsForCheck = {200, 1000, 847, -405, -2000, 3511};

static int check_fuse(const dmf_volume* v, const dmf_camera* cam, int P, const dmf_fuse_params* prm) {
  DMF_TRY(require_constructed(v));
  DMF_TRY(check_camera(cam));
  if (!prm) return fail(DMF_ERR_INVALID, "null params");
  if (P <= 0 || P > 65535) return fail(DMF_ERR_INVALID, "pose count %d out of range [1,65535]", P);
  if (v->xdim > 2048 || v->ydim > 2048 || v->zdim > 2048)
    return fail(DMF_ERR_RANGE, "fusion grid is limited to 2048 cells per axis (fixed-point DDA)");
  if (tiled_cells(v->geom().n) > (size_t)UINT32_MAX)
    return fail(DMF_ERR_RANGE, "fusion grid is limited to 2^32 tiled counter cells");
  return DMF_OK;
}

static const char* variant_kernel(int fv) {
  return fv == DMF_FUSE_LDS_BOX ? kNameLds : (fv == DMF_FUSE_CELL_WALK ? kNameCell : kNameSlab);
}

}  // namespace dmf

using namespace dmf;

extern "C" {

const char* dmf_fuse_kernel_name(const dmf_volume* v) {
  if (!v) return "";
  return v->last_kernel ? v->last_kernel : variant_kernel(v->fuse_variant);
}

int dmf_fuse_set_variant(dmf_volume* v, int32_t variant) {
  DMF_API_BEGIN
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  if (!is_known_variant(variant)) return fail(DMF_ERR_INVALID, "unknown fusion variant %d", variant);
  v->fuse_variant = variant;
  v->last_kernel = nullptr;
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_get_variant(const dmf_volume* v, int32_t* variant) {
  if (!v || !variant) return fail(DMF_ERR_INVALID, "null argument");
  *variant = v->fuse_variant;
  return DMF_OK;
}

int dmf_volume_set_knob(dmf_volume* v, int32_t knob, int64_t value) {
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  if (knob < 1 || knob >= DMF_KNOB_COUNT) return fail(DMF_ERR_INVALID, "unknown knob %d", knob);
  if (knob == DMF_KNOB_BDIST_CAP) {
    if (value < 0 || value > 255) return fail(DMF_ERR_INVALID, "brick distance cap %lld not in 0..255 (0 = default)", (long long)value);
    const int cap = value ? (int)value : kBrickDistCapDefault;
    if (cap != v->brick_cap) {
      v->brick_cap = cap;
      v->bdist_valid = false;  // rebuilt at the next march
    }
  }
  v->knob[knob] = value;
  return DMF_OK;
}

int dmf_volume_get_knob(const dmf_volume* v, int32_t knob, int64_t* value) {
  if (!v || !value) return fail(DMF_ERR_INVALID, "null argument");
  if (knob < 1 || knob >= DMF_KNOB_COUNT) return fail(DMF_ERR_INVALID, "unknown knob %d", knob);
  *value = v->knob[knob];
  return DMF_OK;
}

int dmf_fuse_reserve(dmf_volume* v, const dmf_camera* cam, int32_t P, uint64_t max_scratch_bytes) {
  DMF_API_BEGIN
  DMF_TRY(check_fuse(v, cam, P, &kDefaultParamsForCheck));
  if (max_scratch_bytes && max_scratch_bytes != v->bk_budget) {
    DMF_TRY(bk_release(v));  // the slots are re-planned against the new budget
    v->bk_budget = max_scratch_bytes;
  }
  const CamP cp = cam_params(cam);
  const Geom g = v->geom();
  void* tab;
  DMF_TRY(scratch(v, kScPoses, sizeof(PoseX) * (size_t)P, &tab));
  unsigned long long* st;
  DMF_TRY(stats_begin(v, &st));
  if (use_bricks(v, g)) {
    BkPlan pl;
    DMF_TRY(bk_plan(v, cp, g, P, pl));
    DMF_TRY(bk_attributes());
    DMF_TRY(fault_words(v));
    BkBufs set;
    DMF_TRY(bk_scratch(v, pl, set, 0));
    if (v->pipelined) {  // the second staging slot, the staging stream, slot pose tables and statistics
      DMF_TRY(bk_scratch(v, pl, set, 1));
      DMF_TRY(stage_init(v));
      void* t;
      for (int k = 0; k < 2; ++k) {
        DMF_TRY(scratch(v, k ? kScStPoses1 : kScStPoses0, sizeof(PoseX) * (size_t)pl.PS, &t));
        DMF_TRY(scratch(v, k ? kScStStats1 : kScStStats0, sizeof(unsigned long long) * kStatSlots * kStatWidth, &t));
      }
    }
  }
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_plan(const dmf_volume* v, const dmf_camera* cam, int32_t P, dmf_fuse_plan_info* out) {
  DMF_API_BEGIN
  if (!out) return fail(DMF_ERR_INVALID, "null argument");
  DMF_TRY(check_fuse(v, cam, P, &kDefaultParamsForCheck));
  *out = dmf_fuse_plan_info{};
  const Geom g = v->geom();
  out->max_batches = 1;
  out->poses_per_batch = P;
  if (use_bricks(v, g)) {
    BkPlan pl;
    DMF_TRY(bk_plan(v, cam_params(cam), g, P, pl));
    out->brick = 1;
    out->poses_per_batch = (int32_t)pl.PBg;
    out->max_batches = (int32_t)pl.max_batches(P);
    out->record_bytes = (int32_t)pl.rec_bytes;
    out->pair_capacity = (uint64_t)pl.pair_cap;
    out->scratch_bytes = pl.slot_bytes * (uint64_t)pl.slots;  // both staging slots when pipelined
    out->super_batch_poses = (int32_t)pl.PS;
    out->slots = pl.slots;
  }
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_batches_used(dmf_volume* v, int32_t* batches) {
  DMF_API_BEGIN
  if (!batches) return fail(DMF_ERR_INVALID, "null argument");
  DMF_TRY(require_constructed(v));
  *batches = 0;
  if (!v->bk_last_bt) return DMF_OK;
  uint32_t J = 0;
  if (v->stage) DMF_HIP(hipStreamSynchronize(v->stage));  // the table of a staged call
  DMF_HIP(hipMemcpyAsync(&J, v->bk_last_bt, sizeof(J), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  *batches = (int32_t)J;
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_counter_cells(const dmf_volume* v, int64_t* n) {
  DMF_API_BEGIN
  if (!n) return fail(DMF_ERR_INVALID, "null argument");
  DMF_TRY(require_constructed(v));
  *n = (int64_t)tiled_cells(v->geom().n);
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_counters_to_linear_device(dmf_volume* v, const int32_t* d_tiled, int32_t* d_linear) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!d_tiled || !d_linear) return fail(DMF_ERR_INVALID, "null device buffer");
  const int64_t n = (int64_t)v->ncell;
  hipLaunchKernelGGL(k_counter_layout<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, v->stream, v->geom(),
                     d_tiled, d_linear, n);
  DMF_LAUNCH_CHECK();
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_set_phase_event(dmf_volume* v, void* event) {
  DMF_API_BEGIN
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  // the next pass A no longer waits on the caller's old event (the wait only schedules it
  // beside phase F: nothing depends on it, and the event may be destroyed after this)
  for (int k = 0; k < 2; ++k)
    if (v->st_b_ev[k] == v->f_event) v->st_b_set[k] = false;
  v->f_event = (hipEvent_t)event;
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_set_input_stream(dmf_volume* v, void* stream) {
  DMF_API_BEGIN
  if (!v) return fail(DMF_ERR_INVALID, "null volume");
  DMF_TRY(activate(v));
  const bool pipelined = stream != nullptr;
  if (pipelined != v->pipelined) DMF_TRY(bk_release(v));  // one slot of the budget, or two of half
  v->in_stream = (hipStream_t)stream;
  v->pipelined = pipelined;
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"

namespace dmf {
// dmf_fuse_depth_device; allow_stage = false for the host form (its inputs are uploaded on
// the volume's stream)
static int fuse_device(dmf_volume* v, const dmf_camera* cam, const uint16_t* d_depth, const float* d_poses, int32_t P,
                       const dmf_fuse_params* prm, int32_t* d_hits, int32_t* d_misses, uint64_t* d_stats,
                       bool allow_stage) {
  DMF_TRY(check_fuse(v, cam, P, prm));
  if (!d_depth || !d_poses || !d_hits || !d_misses) return fail(DMF_ERR_INVALID, "null device buffer");
  const CamP cp = cam_params(cam);
  const Geom g = v->geom();
  const bool brick = use_bricks(v, g);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  DMF_HIP(hipStreamIsCapturing(v->stream, &cs));
  const bool capturing = cs != hipStreamCaptureStatusNone;
  const bool staged = brick && allow_stage && v->pipelined && !capturing;
  PoseX* tab = nullptr;
  if (!staged) DMF_TRY(pose_table(v, d_poses, P, true, &tab));
  unsigned long long* st = nullptr;
  if (d_stats) DMF_TRY(stats_begin(v, &st));
  if (brick) {
    v->last_kernel = variant_kernel(v->fuse_variant);
    DMF_TRY(fuse_bricks(v, cp, g, d_depth, tab, d_poses, P, prm, d_hits, d_misses, st, d_stats, staged, capturing));
  } else {
    const int pkx = (cp.W + 7) / 8;
    if (v->f_event && !capturing) DMF_HIP(hipEventRecord(v->f_event, v->stream));
    hipLaunchKernelGGL((k_fuse_l<12, 1280>), dim3((unsigned)(pkx * ((cp.H + 7) / 8)), (unsigned)P), dim3(64), 0,
                       v->stream, g, cp, d_depth, tab, prm->dmin_mm, prm->dmax_mm, pkx, d_hits, d_misses, st);
    DMF_LAUNCH_CHECK();
    v->last_kernel = kNameLds;
  }
  // (brick pipeline: the layout faults not yet reported go to d_stats[3])
  if (d_stats) DMF_TRY(stats_end(v, st, d_stats, kStatWidth, brick ? v->d_fault : nullptr));
  DMF_LAUNCH_CHECK();
  return DMF_OK;
}

// Reads and clears the volume's layout-fault count (synchronises the volume's streams).
static int take_faults(dmf_volume* v, uint64_t* faults) {
  uint32_t f = 0;
  if (v->d_fault) {
    if (v->stage) DMF_HIP(hipStreamSynchronize(v->stage));
    DMF_HIP(hipMemcpyAsync(&f, v->d_fault, sizeof(f), hipMemcpyDeviceToHost, v->stream));
    DMF_HIP(hipStreamSynchronize(v->stream));
    if (f) {
      DMF_HIP(hipMemsetAsync(v->d_fault, 0, sizeof(uint32_t), v->stream));
      DMF_HIP(hipStreamSynchronize(v->stream));
    }
  }
  if (faults) *faults = f;
  return f ? fail(DMF_ERR_DEVICE_CHECK,
                  "brick pipeline layout check: %u workgroup-brick slot ranges disagreed with pass A (the fusion "
                  "counters of the calls since the last check are invalid)", f)
           : DMF_OK;
}
}  // namespace dmf

extern "C" {

int dmf_fuse_depth_device(dmf_volume* v, const dmf_camera* cam, const uint16_t* d_depth, const float* d_poses,
                          int32_t P, const dmf_fuse_params* prm, int32_t* d_hits, int32_t* d_misses,
                          uint64_t* d_stats) {
  DMF_API_BEGIN
  return fuse_device(v, cam, d_depth, d_poses, P, prm, d_hits, d_misses, d_stats, true);
  DMF_API_END
}

int dmf_fuse_depth(dmf_volume* v, const dmf_camera* cam, const uint16_t* depth, const float* poses, int32_t P,
                   const dmf_fuse_params* prm, int32_t* hits, int32_t* misses, int64_t* stats) {
  DMF_API_BEGIN
  DMF_TRY(check_fuse(v, cam, P, prm));
  if (!depth || !poses || !hits || !misses) return fail(DMF_ERR_INVALID, "null buffer");
  const size_t HW = (size_t)cam->height * cam->width;
  const Geom g = v->geom();
  const size_t nt = tiled_cells(g.n);
  const int64_t n = (int64_t)v->ncell;
  void *dd, *dp, *dh, *dm, *ds, *lin;
  DMF_TRY(scratch(v, kScHost1, sizeof(uint16_t) * HW * P, &dd));
  DMF_TRY(scratch(v, kScHost2, sizeof(float) * 12 * P, &dp));
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * nt, &dh));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * nt, &dm));
  DMF_TRY(scratch(v, kScOut2, sizeof(uint64_t) * 8, &ds));
  DMF_TRY(scratch(v, kScOut3, sizeof(int32_t) * v->ncell, &lin));
  DMF_HIP(hipMemcpyAsync(dd, depth, sizeof(uint16_t) * HW * P, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemcpyAsync(dp, poses, sizeof(float) * 12 * P, hipMemcpyHostToDevice, v->stream));
  DMF_HIP(hipMemsetAsync(dh, 0, sizeof(int32_t) * nt, v->stream));
  DMF_HIP(hipMemsetAsync(dm, 0, sizeof(int32_t) * nt, v->stream));
  const dim3 lg((unsigned)((n + 255) / 256));
  // accumulate onto the caller's linear counters
  DMF_HIP(hipMemcpyAsync(lin, hits, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  hipLaunchKernelGGL(k_counter_layout<false>, lg, dim3(256), 0, v->stream, g, (const int32_t*)lin, (int32_t*)dh, n);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(lin, misses, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  hipLaunchKernelGGL(k_counter_layout<false>, lg, dim3(256), 0, v->stream, g, (const int32_t*)lin, (int32_t*)dm, n);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemsetAsync(ds, 0, sizeof(uint64_t) * 8, v->stream));
  DMF_TRY(fuse_device(v, cam, (const uint16_t*)dd, (const float*)dp, P, prm, (int32_t*)dh, (int32_t*)dm,
                      (uint64_t*)ds, false));
  uint64_t st[4];
  hipLaunchKernelGGL(k_counter_layout<true>, lg, dim3(256), 0, v->stream, g, (const int32_t*)dh, (int32_t*)lin, n);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(hits, lin, sizeof(int32_t) * v->ncell, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  hipLaunchKernelGGL(k_counter_layout<true>, lg, dim3(256), 0, v->stream, g, (const int32_t*)dm, (int32_t*)lin, n);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipMemcpyAsync(misses, lin, sizeof(int32_t) * v->ncell, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipMemcpyAsync(st, ds, sizeof(st), hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  DMF_TRY(take_faults(v, nullptr));
  if (stats)
    for (int k = 0; k < 3; ++k) stats[k] += (int64_t)st[k];
  return DMF_OK;
  DMF_API_END
}

int dmf_fuse_status(dmf_volume* v, uint64_t* faults) {
  DMF_API_BEGIN
  if (faults) *faults = 0;
  DMF_TRY(require_constructed(v));
  DMF_TRY(activate(v));
  return take_faults(v, faults);
  DMF_API_END
}

int dmf_fuse_finalize_device(dmf_volume* v, const int32_t* d_hits, const int32_t* d_misses,
                             const dmf_fuse_params* prm, int16_t* d_out) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!prm || !d_hits || !d_misses || !d_out) return fail(DMF_ERR_INVALID, "null argument");
  return finalize_tiles(v, d_hits, d_misses, prm, d_out, 0, (int64_t)tiled_cells(v->geom().n) / 16, v->stream);
  DMF_API_END
}

int dmf_fuse_finalize(dmf_volume* v, const int32_t* hits, const int32_t* misses, const dmf_fuse_params* prm,
                      int16_t* out) {
  DMF_API_BEGIN
  DMF_TRY(require_constructed(v));
  if (!prm || !hits || !misses || !out) return fail(DMF_ERR_INVALID, "null argument");
  const Geom g = v->geom();
  const size_t nt = tiled_cells(g.n);
  const int64_t n = (int64_t)v->ncell;
  void *dh, *dm, *dout, *lin;
  DMF_TRY(scratch(v, kScOut0, sizeof(int32_t) * nt, &dh));
  DMF_TRY(scratch(v, kScOut1, sizeof(int32_t) * nt, &dm));
  DMF_TRY(scratch(v, kScOut2, sizeof(int16_t) * v->ncell + 32, &dout));
  DMF_TRY(scratch(v, kScOut3, sizeof(int32_t) * v->ncell, &lin));
  const dim3 lg((unsigned)((n + 255) / 256));
  DMF_HIP(hipMemsetAsync(dh, 0, sizeof(int32_t) * nt, v->stream));
  DMF_HIP(hipMemsetAsync(dm, 0, sizeof(int32_t) * nt, v->stream));
  DMF_HIP(hipMemcpyAsync(lin, hits, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  hipLaunchKernelGGL(k_counter_layout<false>, lg, dim3(256), 0, v->stream, g, (const int32_t*)lin, (int32_t*)dh, n);
  DMF_LAUNCH_CHECK();
  DMF_HIP(hipStreamSynchronize(v->stream));
  DMF_HIP(hipMemcpyAsync(lin, misses, sizeof(int32_t) * v->ncell, hipMemcpyHostToDevice, v->stream));
  hipLaunchKernelGGL(k_counter_layout<false>, lg, dim3(256), 0, v->stream, g, (const int32_t*)lin, (int32_t*)dm, n);
  DMF_LAUNCH_CHECK();
  DMF_TRY(dmf_fuse_finalize_device(v, (const int32_t*)dh, (const int32_t*)dm, prm, (int16_t*)dout));
  DMF_HIP(hipMemcpyAsync(out, dout, sizeof(int16_t) * v->ncell, hipMemcpyDeviceToHost, v->stream));
  DMF_HIP(hipStreamSynchronize(v->stream));
  return DMF_OK;
  DMF_API_END
}

}  // extern "C"
