// CPU self-test of the certified float binning of the marches (csrc/dmf_geom.hpp
// bin_axis_f): whenever it certifies its float estimate, the bin must equal the reference
// getVoxel binning bin_axis (Volume.hpp:150-156: floor((x - min) / delta) in double) --
// including the tiny-|x| points where x - min rounds in double.  Grids: the bench's
// [-0.5, 0.5] at 256 / 512 / 1024 cells (power-of-two deltas), non-power-of-two deltas,
// bounds that are not floats, the cloud-derived bounds of tests/Raytracing.cpp:62-69 (float
// min/max, 125 cells per metre) and an off-origin grid.  Per grid: every float in a window
// around each of the first / last cell boundaries and around 0, every stride-th float of
// [vlo, vhi], and random floats.  Reports the fraction the float path leaves to bin_axis.
// Build: g++ -O2 -ffp-contract=off -I depth-map-fusion-utils_amd/csrc tools/binning_selftest.cpp
// run: ./a.out [stride] (the exhaustive run is stride 1: every float of each grid's range)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "dmf_geom.hpp"

using dmf::Geom;

static Geom make_geom(const double mn[3], const double mx[3], const int n[3]) {
  Geom g{};
  g.pow2 = 1;
  for (int a = 0; a < 3; ++a) {
    g.mn[a] = mn[a];
    g.mx[a] = mx[a];
    g.n[a] = n[a];
    g.dl[a] = (mx[a] - mn[a]) / n[a];  // setVolumeSize (Volume.hpp:109-117)
    int e;
    const double m = std::frexp(g.dl[a], &e);
    const bool p2 = m == 0.5;
    g.inv[a] = p2 ? 1.0 / g.dl[a] : 0.0;
    if (!p2) g.pow2 = 0;
    float lo = (float)mn[a], hi = (float)mx[a];
    if (!((double)lo > mn[a])) lo = std::nextafter(lo, INFINITY);
    if (!((double)hi < mx[a])) hi = std::nextafter(hi, -INFINITY);
    g.vlo[a] = lo;
    g.vhi[a] = hi;
  }
  dmf::fbin_setup(g);
  return g;
}

static uint32_t fbits(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  return u;
}
static float ffrom(uint32_t u) {
  float x;
  std::memcpy(&x, &u, 4);
  return x;
}
// order-preserving integer key of a float (for stepping through [lo, hi])
static int64_t fkey(float x) {
  const uint32_t u = fbits(x);
  return (u >> 31) ? -(int64_t)(u & 0x7fffffffu) : (int64_t)u;
}
static float funkey(int64_t k) { return k < 0 ? ffrom((uint32_t)(-k) | 0x80000000u) : ffrom((uint32_t)k); }

struct Counts {
  long checked = 0, certified = 0, bad = 0;
};

static void check(const Geom& g, int a, float x, Counts& c) {
  if (!(x >= g.vlo[a] && x <= g.vhi[a])) return;
  ++c.checked;
  int fb = 0;
  if (!dmf::bin_axis_f(g, a, x, &fb)) return;
  ++c.certified;
  const int ref = dmf::bin_axis(g, a, x);
  if (fb != ref) {
    if (c.bad < 10) std::printf("  MISMATCH axis %d x=%.9g (%08x): float %d, getVoxel %d\n", a, x, fbits(x), fb, ref);
    ++c.bad;
  }
}

int main(int argc, char** argv) {
  const long stride = argc > 1 ? std::atol(argv[1]) : 1;
  struct G {
    double mn[3], mx[3];
    int n[3];
  };
  const float cmin[3] = {-0.4837f, -0.3012f, 0.1123f}, cmax[3] = {0.5219f, 0.4471f, 0.9377f};
  G grids[] = {
      {{-0.5, -0.5, -0.5}, {0.5, 0.5, 0.5}, {512, 256, 1024}},
      {{-0.5, -0.5, -0.5}, {0.5, 0.5, 0.5}, {300, 61, 1000}},                       // non-power-of-two deltas
      {{-0.3, -1.0 / 3, 0.1}, {0.7, 0.2, 1.3}, {384, 200, 600}},                    // bounds that are not floats
      {{cmin[0], cmin[1], cmin[2]}, {cmax[0], cmax[1], cmax[2]},                    // tests/Raytracing.cpp:62-69
       {(int)((cmax[0] - cmin[0]) * 125), (int)((cmax[1] - cmin[1]) * 125), (int)((cmax[2] - cmin[2]) * 125)}},
      {{100.25, -7.5, 3.0}, {101.25, -6.5, 4.0}, {1024, 512, 2048}},                // off-origin, 2048 cells
  };
  std::mt19937_64 rng(99);
  long bad = 0, checked = 0, certified = 0;
  for (const G& gg : grids) {
    const Geom g = make_geom(gg.mn, gg.mx, gg.n);
    for (int a = 0; a < 3; ++a) {
      Counts c;
      const int64_t k0 = fkey(g.vlo[a]), k1 = fkey(g.vhi[a]);
      // windows of 4096 floats around the first / last few cell boundaries and 0
      for (int i = 0; i <= 3; ++i)
        for (int side = 0; side < 2; ++side) {
          const int cell = side ? g.n[a] - i : i;
          const float b = (float)(g.mn[a] + cell * g.dl[a]);
          for (int64_t k = fkey(b) - 2048; k <= fkey(b) + 2048; ++k) check(g, a, funkey(k), c);
        }
      for (int64_t k = -4096; k <= 4096; ++k) check(g, a, funkey(k), c);
      for (int64_t k = k0; k <= k1; k += stride) check(g, a, funkey(k), c);
      std::uniform_int_distribution<int64_t> U(k0, k1);
      for (int i = 0; i < 200000; ++i) check(g, a, funkey(U(rng)), c);
      std::printf("grid n=%d dl=%.6g mn=%.9g eps=%.3g fbin=%d axis %d: %ld floats, certified %.5f, %ld mismatches\n",
                  g.n[a], g.dl[a], g.mn[a], (double)g.feps[a], g.fbin, a, c.checked,
                  c.checked ? (double)c.certified / c.checked : 0.0, c.bad);
      bad += c.bad;
      checked += c.checked;
      certified += c.certified;
      if (!g.fbin) ++bad;  // every grid here must take the float path
    }
  }
  std::printf("binning selftest: %ld floats, %ld certified, %ld mismatches\n", checked, certified, bad);
  return bad ? 1 : 0;
}
