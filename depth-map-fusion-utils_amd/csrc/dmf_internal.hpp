// dmf_internal.hpp — shared state and device math of the MI355X engine.
//
// Device functions restate the reference arithmetic with the exact IEEE operation
// sequence: fp64 where the reference uses double, fp32 where Eigen
// uses float, the Eigen 3-term reduction order a0 + (a1 + a2), and no FMA
// contraction (every TU is built with -ffp-contract=off; the pragma below repeats it).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "dmf.h"
#include "dmf_diag.h"
#include "dmf_geom.hpp"

namespace dmf {

constexpr int32_t kEmpty = 0x7fffffff;         // slot_of[] value of an empty cell
constexpr int32_t kPendBase = (int32_t)0x80000000;  // slot_of[] = kPendBase + i while binning
constexpr double kZMin = 0.20, kZMax = 1.0;    // RayTracingEngine.hpp:24-25
constexpr int kWave = 64;

// ---------------------------------------------------------------- geometry
// Camera.hpp:26 fx=K[0], cx=K[2], fy=K[4], cy=K[5] promoted to double.
struct CamP {
  double fx, cx, fy, cy;
  double rfx, rfy;  // RN(1/fx), RN(1/fy) (host division) for div_rn
  int H, W;
};

// Correctly rounded n / d from y = RN(1/d) (d > 0 normal): Markstein's final step
// q0 = RN(n*y), r = n - d*q0 (exact by fma), q = RN(q0 + r*y).  Bit-identical to n / d in
// the checked magnitude ranges (tools/fastdiv_selftest.cpp: 2.7e9 quotients over the
// projection and reverse-march domains, 0 mismatches); outside them (and for NaN) it
// divides; +-0 keeps its sign through q0.  Replaces the ~10-instruction IEEE division
// sequence by one multiply and two fmas per sample.
__device__ inline double div_rn(double n, double d, double y) {
  const double q0 = n * y;
  const double an = fabs(n);
  if (!(an >= 0x1p-900 && an <= 0x1p900)) return n == 0.0 ? q0 : n / d;
  const double r = fma(-d, q0, n);
  return fma(r, y, q0);
}
__device__ inline float div_rn(float n, float d, float y) {
  const float q0 = n * y;
  const float an = fabsf(n);
  if (!(an >= 0x1p-40f && an <= 0x1p40f)) return n == 0.0f ? q0 : n / d;
  const float r = fmaf(-d, q0, n);
  return fmaf(r, y, q0);
}

// Forward (camera->world) pose and its Eigen Affine inverse, row-major 3x4.
struct PoseX {
  float f[12];
  float i[12];
};

__host__ __device__ inline float sum3(float a0, float a1, float a2) { return a0 + (a1 + a2); }

// Camera.hpp:39-45 transformPoints (Eigen Transform*Vector3f, Affine)
__device__ inline void xform(const float* m, float x, float y, float z, float o[3]) {
  o[0] = m[3] + sum3(m[0] * x, m[1] * y, m[2] * z);
  o[1] = m[7] + sum3(m[4] * x, m[5] * y, m[6] * z);
  o[2] = m[11] + sum3(m[8] * x, m[9] * y, m[10] * z);
}

// Eigen Affine3f::inverse() (Mode Affine): 3x3 cofactor inverse + t' = -(R^-1 t).
__host__ __device__ inline void inverse_pose(const float* T, float* R) {
#define M_(i, j) T[(i)*4 + (j)]
  auto cof = [&](int i, int j) -> float {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return M_(i1, j1) * M_(i2, j2) - M_(i1, j2) * M_(i2, j1);
  };
  const float c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
  const float det = sum3(c0 * M_(0, 0), c1 * M_(1, 0), c2 * M_(2, 0));
  const float invdet = 1.0f / det;
  R[0] = c0 * invdet; R[1] = c1 * invdet; R[2] = c2 * invdet;
  R[4] = cof(0, 1) * invdet; R[5] = cof(1, 1) * invdet; R[6] = cof(2, 1) * invdet;
  R[8] = cof(0, 2) * invdet; R[9] = cof(1, 2) * invdet; R[10] = cof(2, 2) * invdet;
  for (int i = 0; i < 3; ++i)
    R[i * 4 + 3] = -sum3(R[i * 4 + 0] * M_(0, 3), R[i * 4 + 1] * M_(1, 3), R[i * 4 + 2] * M_(2, 3));
#undef M_
}

// Camera.hpp:24-31 projectPoint: double math, narrowed to float.
__device__ inline void project(const CamP& c, int r, int col, int depth_mm, float o[3]) {
  const double z = depth_mm * 0.001;
  const double x = div_rn(z * ((double)col - c.cx), c.fx, c.rfx);  // (z * (col - cx)) / fx
  const double y = div_rn(z * ((double)r - c.cy), c.fy, c.rfy);
  o[0] = (float)x;
  o[1] = (float)y;
  o[2] = (float)z;
}

// int(v) with the x86 cvttsd2si result for NaN / out of range (INT_MIN), so that
// validPixel() rejects exactly what the reference binary rejects.
__host__ __device__ inline int to_int_x86(double v) {
  return (v >= -2147483648.0 && v < 2147483648.0) ? (int)v : (int)0x80000000;
}

// Camera.hpp:32-38 deProjectPoint + :65-68 validPixel
__device__ inline bool deproject_valid(const CamP& c, float x, float y, float z, int& r, int& col) {
  col = to_int_x86(round(((double)x * c.fx) / (double)z + c.cx));
  r = to_int_x86(round(((double)y * c.fy) / (double)z + c.cy));
  return r >= 0 && r < c.H && col >= 0 && col < c.W;
}

// Volume.hpp:230-233 validPoints (strict interior, float promoted to double)
__device__ inline bool valid_points(const Geom& g, float x, float y, float z) {
  return !((double)x >= g.mx[0] || (double)y >= g.mx[1] || (double)z >= g.mx[2] ||
           (double)x <= g.mn[0] || (double)y <= g.mn[1] || (double)z <= g.mn[2]);
}

// Volume.hpp:167-170 validCoords
__device__ inline bool valid_coords(const Geom& g, int x, int y, int z) {
  return x < g.n[0] && y < g.n[1] && z < g.n[2] && x >= 0 && y >= 0 && z >= 0;
}

__device__ inline uint32_t lin_index(const Geom& g, int x, int y, int z) {
  return ((uint32_t)x * (uint32_t)g.n[1] + (uint32_t)y) * (uint32_t)g.n[2] + (uint32_t)z;
}

// Volume.hpp:143-148 getHashId (y<<20 is an int shift, sign-extended into the xor)
__host__ __device__ inline uint64_t hash_id(int x, int y, int z) {
  return ((uint64_t)(int64_t)x << 40) ^ (uint64_t)(int64_t)(y << 20) ^ (uint64_t)(int64_t)z;
}

// Occupancy bitmask layout: 8x8x8-cell tiles of 512 bits (16 words = 64 B), tiles x-major
// over the grid padded to whole tiles, bit (x&7)*64 + (y&7)*8 + (z&7) inside a tile.  A
// march sample stays in one tile for several samples whatever the ray direction; with
// x-major bits (one 128-B line = 1024 z-cells of one (x, y) column) a reverse march left
// the line at nearly every sample: L2 hit rate 0.50 and 43 GB beyond L2 per 128-pose
// reverseRayTraceFast launch at 512^3.
__host__ __device__ inline uint32_t occ_bit(const Geom& g, int x, int y, int z) {
  const uint32_t nty = ((uint32_t)g.n[1] + 7u) >> 3, ntz = ((uint32_t)g.n[2] + 7u) >> 3;
  const uint32_t t = (((uint32_t)x >> 3) * nty + ((uint32_t)y >> 3)) * ntz + ((uint32_t)z >> 3);
  return (t << 9) | (((uint32_t)x & 7u) << 6) | (((uint32_t)y & 7u) << 3) | ((uint32_t)z & 7u);
}
// 32-bit words of the tiled bitmask (bit indices must fit 32 bits: checked at construction)
inline uint64_t occ_words(const int n[3]) {
  return (uint64_t)((n[0] + 7) >> 3) * (uint64_t)((n[1] + 7) >> 3) * (uint64_t)((n[2] + 7) >> 3) * 16u;
}

__device__ inline bool occ_test(const uint32_t* occ, uint32_t bit) {
  return (occ[bit >> 5] >> (bit & 31)) & 1u;
}

// Eigen normalized()
__device__ inline void normalized(const float d[3], float v[3]) {
  const float s = sum3(d[0] * d[0], d[1] * d[1], d[2] * d[2]);
  if (s > 0.0f) {
    const float q = sqrtf(s);
    v[0] = d[0] / q; v[1] = d[1] / q; v[2] = d[2] / q;
  } else {
    v[0] = d[0]; v[1] = d[1]; v[2] = d[2];
  }
}

// degree(acos(n.v)) in [0,90] (CommonUtilities.hpp:17, RayTracingEngine.hpp:211-212)
// <=> dstar <= dot <= 1, where dstar is derived on the host from the host libm acosf
// (the function the reference binary calls) and verified over every float in the
// transition window (see dmf_core.hip angle_threshold()).
__device__ inline bool angle_ok(float nx, float ny, float nz, const float v[3], float dstar) {
  const float d = sum3(nx * v[0], ny * v[1], nz * v[2]);
  return d >= dstar && d <= 1.0f;
}

// ---------------------------------------------------------------- device state
// Coarse occupancy: one bit per 8x8x8-cell brick (empty-space skipping in the marches).
constexpr int kBrickShiftDefault = 1;    // 2^3-cell bricks (reverse batch: 8.1 ms; 4^3 9.1, 8^3 11.3, cells 9.6)
constexpr int kBrickDistCapDefault = 63;  // brick distance field saturates here (in bricks)

struct DevVol {
  const uint32_t* occ;     // occupancy bitmask (occ_bit tiles)
  const uint8_t* bdist;    // per brick: L-inf distance in bricks to the nearest occupied brick (0 = occupied), capped
  int bsh;                 // brick edge = 1 << bsh cells
  const uint32_t* brick;   // one bit per brick, x-major over nb[]
  int nb[3];               // bricks per axis = ceil(n / 8)
  const int32_t* slot_of;  // N: slot or kEmpty
  const uint64_t* hash;    // V: occupied_cells_
  const int32_t* off;      // V+1: CSR offsets into nrm
  const float4* nrm;       // CSR normals (w = 1 if the point carried a normal)
  int32_t* view;           // V
  uint8_t* good;           // V
  int64_t V;
};

}  // namespace dmf

// ---------------------------------------------------------------- host handle
struct dmf_volume {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t switch_ev = nullptr;  // orders a new stream after the old one (dmf_volume_set_stream)
  // reference fields (Volume.hpp:54-60)
  double xmin = 0, xmax = 0, ymin = 0, ymax = 0, zmin = 0, zmax = 0;
  double xcenter = 0, ycenter = 0, zcenter = 0;
  double xdelta = 0, ydelta = 0, zdelta = 0;
  double voxel_size = 0;
  int32_t xdim = 0, ydim = 0, zdim = 0;
  uint64_t hsize = 0;
  bool constructed = false;
  int64_t hazards = 0;
  float dstar = 0.0f;

  // device grid
  size_t ncell = 0;
  uint32_t* d_occ = nullptr;
  uint32_t* d_brick = nullptr;  // one bit per 8^3 brick
  uint8_t* d_bdist = nullptr;   // brick distance field (DevVol::bdist), valid when bdist_valid
  bool bdist_valid = false;
  // occupied voxels in spatial (3D Morton) order: d_sorder[k] = slot of the k-th, followed by
  // the inverse rank[slot] (sorder_cap entries each); reverseRayTraceFast's work order
  uint32_t* d_sorder = nullptr;
  int64_t sorder_cap = 0;
  bool sorder_valid = false;
  int brick_shift = dmf::kBrickShiftDefault, brick_cap = dmf::kBrickDistCapDefault;
  int32_t nb[3] = {0, 0, 0};
  int32_t* d_slot_of = nullptr;
  // occupied list
  int64_t V = 0, Vcap = 0;
  uint64_t* d_hash = nullptr;
  int32_t* d_view = nullptr;
  uint8_t* d_good = nullptr;
  // points (all integrated points; slot -1 = not binned)
  int64_t npts = 0, pcap = 0, nbinned = 0;
  float* d_pts = nullptr;     // 3*pcap
  float4* d_pnrm = nullptr;   // pcap (w = has normal)
  int32_t* d_pslot = nullptr; // pcap
  // CSR by slot
  int32_t* d_off = nullptr;      // V+1
  float4* d_csr_nrm = nullptr;   // nbinned
  float* d_csr_pts = nullptr;    // 3*nbinned
  int64_t csr_cap = 0;
  // float-accumulated enumeration axes (RayTracingEngine.hpp:54-56) + occupied list
  bool enum_valid = false;
  float* d_axes = nullptr;  // xs | ys | zs
  int32_t nax[3] = {0, 0, 0};
  uint32_t* d_enum = nullptr;  // occupied enumeration indices, enumeration order
  int64_t nenum = 0, enum_cap = 0, enum_hazards = 0;
  // brick fusion scratch budget (dmf_fuse_reserve)
  uint64_t bk_budget = 48ull << 30;  // set from the device's memory by dmf_volume_create
  uint32_t* bk_last_bt = nullptr;     // the batch table of the latest brick-pipeline super-batch (diagnostic)
  // pipelined fusion (dmf_fuse_set_input_stream): pass A of a super-batch
  // on the staging stream, into one of two slots
  bool pipelined = false;
  hipStream_t in_stream = nullptr;  // the caller's input stream
  hipStream_t stage = nullptr;      // staging stream (created on first use)
  hipEvent_t st_in = nullptr, st_done[2] = {nullptr, nullptr}, st_free[2] = {nullptr, nullptr};
  bool st_free_set[2] = {false, false};
  // pass B of the slot's call launched (the next call's pass A waits for it: it then runs beside
  // that call's phase F)
  hipEvent_t st_b[2] = {nullptr, nullptr};
  hipEvent_t st_b_ev[2] = {nullptr, nullptr};  // the event that marks it (st_b, or the caller's phase event)
  hipEvent_t st_a[2] = {nullptr, nullptr};  // the slot's pass A done (before its statistics' sum)
  bool st_b_set[2] = {false, false};
  hipEvent_t f_event = nullptr;  // caller's phase-F event (dmf_fuse_set_phase_event)
  int st_slot = 0;
  // device-side layout check of the brick pipeline (dmf_fuse_status): [0] disagreements since
  // the last dmf_fuse_status, [1] those not yet added to a call's d_stats[3]
  uint32_t* d_fault = nullptr;
  // diagnostic / A-B controls (include/dmf_diag.h): fusion implementation and knobs
  int fuse_variant = 0;
  const char* last_kernel = nullptr;  // the fusion kernel of the latest call
  int64_t knob[DMF_KNOB_COUNT] = {};
  // scratch arena
  std::vector<std::pair<void*, size_t>> scratch;

  dmf::Geom geom() const;
  dmf::DevVol dev() const;
};
