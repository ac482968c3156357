// dmf_geom.hpp — the grid geometry of a volume on the device (Volume.hpp:54-60) and the
// reference's binning getVoxel (Volume.hpp:150-156), exact, plus its certified float
// shortcut.  No HIP dependency: the CPU self-test tools/binning_selftest.cpp compiles
// this same code with g++ and checks bin_axis_f against bin_axis.
#pragma once
#include <cmath>
#include <cstdint>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace dmf {

// Volume.hpp:54-60 fields needed on device.
struct Geom {
  double mn[3];   // xmin_, ymin_, zmin_
  double mx[3];   // xmax_, ymax_, zmax_
  double dl[3];   // xdelta_, ...
  double hdl[3];  // xdelta_/2.0 (exact halving)
  double inv[3];  // 1/delta when delta is a power of two (then x*inv == x/delta exactly)
  int pow2;       // all three deltas are powers of two
  int n[3];       // xdim_, ydim_, zdim_ after constructVolume truncation
  float vlo[3];   // smallest float x with (double)x > mn  (validPoints as float compares)
  float vhi[3];   // largest float x with (double)x < mx
  // certified float binning (bin_axis_f): x in [vlo, vhi] bins to floor((x - fmn) * finv)
  // unless that float estimate lies within feps of a cell boundary (fbin_setup)
  float fmn[3], finv[3], feps[3];
  int fbin;       // 1: the float estimate is usable on every axis
  // reverse march: the distance by which an empty cube's exit face is moved toward the sample
  // before a jump is computed from it, 32 * 2^-24 * max(|min|, |max|) per axis -- more than
  // the float rounding of the face, of the sample coordinates and of the bins together, so a
  // jump target computed from the moved face lies inside the cube without evaluating it
  // (jump_margin_setup)
  float jmarg[3];
};

inline void jump_margin_setup(Geom& g) {
  for (int a = 0; a < 3; ++a) {
    const double b = std::fmax(std::fabs(g.mn[a]), std::fabs(g.mx[a]));
    // (non-finite bounds: an infinite margin, so no jump is ever taken -- a NaN would drop the
    // axis from the jump's fminf instead)
    g.jmarg[a] = b < INFINITY ? (float)(32.0 * 0x1p-24 * b) + 1e-30f : INFINITY;
  }
}

// Error bound of the float estimate qf = RN(RN(x - fmn) * finv) of Q = (x - mn) / dl and of
// the double getVoxel value Qd (bin_axis) for |Q| <= n + 2, in cells: with
// d = |mn - fmn| / dl, |qf - Q| <= d + (n + 2 + d) * 3.0001 * 2^-24 (three float roundings:
// the subtraction, finv, the product) and |Qd - Q| <= (n + 2) * 2^-51 (two double roundings).
// If the estimate's fraction lies in (eps, 1 - eps) with eps > both bounds (+ 2^-22 for the
// rounding of the fraction of a negative estimate), floor(qf) == floor(Qd).
// tools/binning_selftest.cpp checks this against bin_axis over billions of floats.
inline void fbin_setup(Geom& g) {
  g.fbin = 1;
  for (int a = 0; a < 3; ++a) {
    g.fmn[a] = (float)g.mn[a];
    g.finv[a] = (float)(1.0 / g.dl[a]);
    const double d = std::fabs(g.mn[a] - (double)g.fmn[a]) / g.dl[a];
    const double q = (double)g.n[a] + 2.0;
    const double eps = 1.25 * (d + (q + d) * 3.0001 * 0x1p-24 + q * 0x1p-51) + 0x1p-22;
    g.feps[a] = (float)eps;
    if (!(eps < 0.125) || !std::isfinite(g.finv[a]) || !(g.finv[a] > 0.0f) || !(q < 0x1p23)) g.fbin = 0;
  }
}

// Volume.hpp:150-156 getVoxel: floor((x - min)/delta) in double.  For power-of-two
// deltas the multiply by the exact reciprocal gives the identical double.
__host__ __device__ inline int bin_axis(const Geom& g, int a, float x) {
  const double t = (double)x - g.mn[a];
  const double q = g.pow2 ? t * g.inv[a] : t / g.dl[a];
  return (int)floor(q);
}

// bin_axis from the float estimate: true (and *out = the bin) when certified (fbin_setup);
// false when the estimate is too close to a cell boundary -- then bin_axis decides.
__host__ __device__ inline bool bin_axis_f(const Geom& g, int a, float x, int* out) {
  const float q = (x - g.fmn[a]) * g.finv[a];
  const float f = floorf(q);
  const float fr = q - f;
  *out = (int)f;
  return fr > g.feps[a] && fr < 1.0f - g.feps[a];
}

}  // namespace dmf
