// CPU self-test of the reverse march's unchecked empty-space jumps (csrc/dmf_trace.hip rev_step
// with DMF_REV_VERIFY_JUMPS = 0): from a sample s inside an empty cube of bricks
// (radius R around the sample's brick, clipped to the grid), the target j is computed from the
// cube's exit faces moved toward the sample by Geom::jmarg, in the kernel's float arithmetic;
// the march then continues at j without evaluating it first.  Exactness needs sample j inside
// the cube on every axis (its bins in [clo, chi)) and inside the volume (validPoints); the
// samples between s and j then follow by monotonicity (each coordinate c + RN(RN(v fd)/1000)
// is monotone in fd), which the test also checks directly on short jumps.  Grids: the bench's
// [-0.5, 0.5] (power-of-two deltas), non-power-of-two deltas, bounds that are not floats, an
// off-origin grid far from 0 and a large one; directions with components of every magnitude
// down to 1e-9 and exact zeros; brick edges 2, 4, 8 cells; cube radii 0..63 and samples placed
// just before a face.  Reports the jumps tried and taken and the failures (must be 0).
// Build: g++ -O2 -ffp-contract=off -I depth-map-fusion-utils_amd/csrc tools/jump_selftest.cpp
// run: ./a.out [trials per grid] [seed]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
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
    g.hdl[a] = g.dl[a] / 2.0;
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
  dmf::jump_margin_setup(g);
  return g;
}

// the march sample of RayTracingEngine.hpp:172-200: c + (v * (float)depth) / 1000 in float
static void sample(const float cen[3], const float v[3], int fd, float p[3]) {
  const float f = (float)fd;
  for (int a = 0; a < 3; ++a) {
    const float m = v[a] * f;
    const float q = m / 1000.0f;
    p[a] = cen[a] + q;
  }
}

static bool valid_f(const Geom& g, const float p[3]) {
  for (int a = 0; a < 3; ++a)
    if (!(p[a] >= g.vlo[a] && p[a] <= g.vhi[a])) return false;
  return true;
}

// ---- forward march (csrc/dmf_trace.hip fwd_ray / fwd_step, DMF_FWD_VERIFY_JUMPS = 0) ------
// Sample k of lattice pixel (r, c): w = T * projectPoint(r, c, zd_k) in the reference's
// arithmetic (Camera.hpp:24-31 in double, narrowed to float; Eigen's Affine3f product with the
// a0 + (a1 + a2) reduction).  A brick jump to sample j is taken without evaluating it when the
// double line t + zd_j dir lies inside the cube shrunk by twice the margin; the test evaluates
// sample j and checks the condition the kernel used to verify (inside the cube shrunk by the
// margin), and on short jumps every sample in between inside the cube's bins.  The entry jump:
// every sample up to the target lies outside the volume.
struct Cam {
  double fx, cx, fy, cy;
};
static void fwd_sample(const Cam& cam, const float m[12], int r, int c, int zd, float w[3]) {
  const double z = zd * 0.001;
  const float pc[3] = {(float)((z * ((double)c - cam.cx)) / cam.fx), (float)((z * ((double)r - cam.cy)) / cam.fy),
                       (float)z};
  for (int a = 0; a < 3; ++a) w[a] = m[4 * a + 3] + (m[4 * a] * pc[0] + (m[4 * a + 1] * pc[1] + m[4 * a + 2] * pc[2]));
}

static long forward_part(long trials, unsigned seed) {
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  struct G {
    double mn[3], mx[3];
    int n[3];
  };
  const G grids[] = {
      {{-0.5, -0.5, -0.5}, {0.5, 0.5, 0.5}, {512, 512, 512}},
      {{-0.37, -0.61, -0.5}, {0.63, 0.52, 0.41}, {300, 333, 257}},
      {{1000.0, -2000.5, 333.3}, {1001.0, -1999.5, 334.3}, {512, 512, 512}},
  };
  const Cam cam{525.0, 319.5, 525.0, 239.5};
  long tried = 0, taken = 0, fails = 0, between = 0, entries = 0;
  for (const G& gg : grids) {
    const Geom g = make_geom(gg.mn, gg.mx, gg.n);
    double ctr[3];
    for (int a = 0; a < 3; ++a) ctr[a] = 0.5 * (gg.mn[a] + gg.mx[a]);
    for (int bsh = 1; bsh <= 3; ++bsh) {
      for (long t = 0; t < trials / 4; ++t) {
        // a camera 0.5-1.1 m from the centre looking near it, random roll (or a random pose)
        double pos[3], f[3], up[3], rt[3], dn[3];
        double nrm = 0;
        for (int a = 0; a < 3; ++a) { pos[a] = 2.0 * U(rng) - 1.0; nrm += pos[a] * pos[a]; }
        nrm = std::sqrt(nrm);
        const double rad = 0.5 + 0.6 * U(rng);
        for (int a = 0; a < 3; ++a) pos[a] = ctr[a] + pos[a] / nrm * rad;
        nrm = 0;
        for (int a = 0; a < 3; ++a) { f[a] = ctr[a] + 0.3 * (U(rng) - 0.5) - pos[a]; nrm += f[a] * f[a]; }
        nrm = std::sqrt(nrm);
        for (int a = 0; a < 3; ++a) { f[a] /= nrm; up[a] = 2.0 * U(rng) - 1.0; }
        rt[0] = up[1] * f[2] - up[2] * f[1]; rt[1] = up[2] * f[0] - up[0] * f[2]; rt[2] = up[0] * f[1] - up[1] * f[0];
        nrm = std::sqrt(rt[0] * rt[0] + rt[1] * rt[1] + rt[2] * rt[2]);
        if (!(nrm > 1e-6)) continue;
        for (int a = 0; a < 3; ++a) rt[a] /= nrm;
        dn[0] = f[1] * rt[2] - f[2] * rt[1]; dn[1] = f[2] * rt[0] - f[0] * rt[2]; dn[2] = f[0] * rt[1] - f[1] * rt[0];
        float m[12];
        for (int a = 0; a < 3; ++a) {
          m[4 * a] = (float)rt[a]; m[4 * a + 1] = (float)dn[a]; m[4 * a + 2] = (float)f[a]; m[4 * a + 3] = (float)pos[a];
        }
        const int r = (int)(U(rng) * 480), c = (int)(U(rng) * 640);
        const int zstart = 100 + (int)(U(rng) * 300), zdelta = 1 + (int)(U(rng) * 9);
        // fwd_ray's per-pixel setup
        double dir[3], eA[3], eB[3];
        float fdir[3], frd[3];
        const double ux = ((double)c - cam.cx) / cam.fx, uy = ((double)r - cam.cy) / cam.fy;
        for (int a = 0; a < 3; ++a) {
          const double m0 = m[4 * a], m1 = m[4 * a + 1], m2 = m[4 * a + 2];
          dir[a] = 0.001 * (m0 * ux + m1 * uy + m2);
          eA[a] = 0x1p-21 * std::fabs((double)m[4 * a + 3]);
          eB[a] = 0x1p-21 * 0.001 * (std::fabs(m0 * ux) + std::fabs(m1 * uy) + std::fabs(m2));
          fdir[a] = (float)dir[a];
          frd[a] = dir[a] != 0.0 ? (float)(1.0 / dir[a]) : 0.0f;
        }
        auto margin = [&](int a, double zd) { return 2.0 * (eA[a] + zd * eB[a]) + 1e-9; };
        const int last_k = (int)((1000.0 - 1 - zstart) / zdelta);
        // the entry jump (the first sample outside the volume)
        float w[3];
        fwd_sample(cam, m, r, c, zstart, w);
        if (!valid_f(g, w)) {
          double tin = -1e300, tout = 1e300;
          for (int a = 0; a < 3; ++a) {
            const double dm = margin(a, 1000.0);
            const double lo = g.mn[a] - dm, hi = g.mx[a] + dm, t0 = (double)m[4 * a + 3];
            if (dir[a] == 0.0) {
              if (t0 <= lo || t0 >= hi) tout = -1e300;
            } else {
              const double ta = (lo - t0) / dir[a], tb = (hi - t0) / dir[a];
              tin = std::fmax(tin, std::fmin(ta, tb));
              tout = std::fmin(tout, std::fmax(ta, tb));
            }
          }
          int kj = tout < tin ? last_k : (int)std::floor((tin - (double)zstart) / zdelta) - 1;
          kj = std::min(kj, last_k);
          for (int k = 1; k <= kj; ++k) {
            ++entries;
            float q[3];
            fwd_sample(cam, m, r, c, zstart + k * zdelta, q);
            if (valid_f(g, q)) {
              if (++fails <= 10) std::printf("FAIL entry: k %d kj %d\n", k, kj);
              break;
            }
          }
        }
        // a brick jump from a sample inside the volume
        const int k = (int)(U(rng) * (last_k + 1));
        fwd_sample(cam, m, r, c, zstart + k * zdelta, w);
        if (!valid_f(g, w)) continue;
        int bx[3];
        bool inb = true;
        for (int a = 0; a < 3; ++a) {
          const int cc = dmf::bin_axis(g, a, w[a]);
          if (cc < 0 || cc >= g.n[a]) inb = false;
          bx[a] = cc >> bsh;
        }
        if (!inb) continue;
        const int Rb = U(rng) < 0.5 ? (int)(U(rng) * 4) : (int)(U(rng) * 64);
        double lo[3], hi[3];
        int clo[3], chi[3];
        float zexit = 3.0e38f;
        for (int ax = 0; ax < 3; ++ax) {
          clo[ax] = std::max(bx[ax] - Rb, 0) << bsh;
          chi[ax] = std::min((bx[ax] + Rb + 1) << bsh, g.n[ax]);
          lo[ax] = g.mn[ax] + (double)clo[ax] * g.dl[ax];
          hi[ax] = g.mn[ax] + (double)chi[ax] * g.dl[ax];
          if (fdir[ax] != 0.0f) zexit = std::fmin(zexit, ((float)(fdir[ax] > 0.0f ? hi[ax] : lo[ax]) - m[4 * ax + 3]) * frd[ax]);
        }
        const int kj = std::min((int)std::floor((zexit - (float)zstart) / (float)zdelta) - 1, last_k);
        if (!(kj > k + 1)) continue;
        ++tried;
        const int zj = zstart + kj * zdelta;
        bool ok = true;
        for (int ax = 0; ax < 3; ++ax) {
          const double dm = margin(ax, (double)zj), lq = (double)m[4 * ax + 3] + (double)zj * dir[ax];
          ok = ok && (double)w[ax] >= lo[ax] + dm && (double)w[ax] <= hi[ax] - dm && lq >= lo[ax] + 2.0 * dm &&
               lq <= hi[ax] - 2.0 * dm;
        }
        if (!ok) continue;
        ++taken;
        float q[3];
        fwd_sample(cam, m, r, c, zj, q);
        bool vok = true;
        for (int ax = 0; ax < 3; ++ax) {
          const double dm = margin(ax, (double)zj);
          vok = vok && (double)q[ax] >= lo[ax] + dm && (double)q[ax] <= hi[ax] - dm;
        }
        if (!vok) {
          if (++fails <= 10) std::printf("FAIL forward jump: k %d kj %d Rb %d bsh %d\n", k, kj, Rb, bsh);
          continue;
        }
        for (int kk = k + 1; kk <= kj && kk - k < 64; ++kk) {
          ++between;
          fwd_sample(cam, m, r, c, zstart + kk * zdelta, q);
          bool in = valid_f(g, q);
          for (int a = 0; a < 3 && in; ++a) {
            const int cc = dmf::bin_axis(g, a, q[a]);
            in = cc >= clo[a] && cc < chi[a];
          }
          if (!in) {
            if (++fails <= 10) std::printf("FAIL forward between: k %d kk %d kj %d\n", k, kk, kj);
            break;
          }
        }
      }
    }
  }
  std::printf("forward: entry samples checked %ld, jumps tried %ld taken %ld, samples between checked %ld, %ld failures\n",
              entries, tried, taken, between, fails);
  return fails;
}

int main(int argc, char** argv) {
  const long trials = argc > 1 ? std::atol(argv[1]) : 200000;
  const unsigned seed = argc > 2 ? (unsigned)std::atol(argv[2]) : 7u;
  struct G {
    double mn[3], mx[3];
    int n[3];
  };
  const G grids[] = {
      {{-0.5, -0.5, -0.5}, {0.5, 0.5, 0.5}, {512, 512, 512}},
      {{-0.5, -0.5, -0.5}, {0.5, 0.5, 0.5}, {256, 256, 256}},
      {{-0.37, -0.61, -0.5}, {0.63, 0.52, 0.41}, {300, 333, 257}},
      {{0.1, 0.2, 0.3}, {1.1, 1.3, 1.7}, {125, 137, 175}},
      {{1000.0, -2000.5, 333.3}, {1001.0, -1999.5, 334.3}, {512, 512, 512}},
      {{-40.0, -40.0, -8.0}, {40.0, 40.0, 8.0}, {1024, 1024, 256}},
  };
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  long tried = 0, taken = 0, fails = 0, between = 0;
  const int depth0 = 50;
  for (const G& gg : grids) {
    const Geom g = make_geom(gg.mn, gg.mx, gg.n);
    double diag = 0;
    for (int a = 0; a < 3; ++a) diag += (gg.mx[a] - gg.mn[a]) * (gg.mx[a] - gg.mn[a]);
    const double ms_d = std::ceil(std::sqrt(diag) * 1000.0 * 1.01) + 64;
    const int max_steps = ms_d > 2e9 ? 2000000000 : (int)ms_d;
    for (int bsh = 1; bsh <= 3; ++bsh) {
      for (long t = 0; t < trials; ++t) {
        // a voxel centroid (rev_wave: hash id -> float corner -> + delta / 2)
        float cen[3];
        for (int a = 0; a < 3; ++a) {
          const int id = (int)(U(rng) * g.n[a]) % g.n[a];
          const float x = (float)((double)id * g.dl[a] + g.mn[a]);
          cen[a] = (float)((double)x + g.hdl[a]);
        }
        // a direction: every magnitude, some exact zeros, normalised as Eigen does
        float d[3];
        for (int a = 0; a < 3; ++a) {
          const double r = U(rng);
          double m = 2.0 * U(rng) - 1.0;
          if (r < 0.15) m *= std::pow(10.0, -3.0 - 6.0 * U(rng));
          else if (r < 0.2) m = 0.0;
          d[a] = (float)m;
        }
        const float s2 = d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]);
        if (!(s2 > 0.0f)) continue;
        const float q = std::sqrt(s2);
        float v[3], rv[3];
        for (int a = 0; a < 3; ++a) {
          v[a] = d[a] / q;
          rv[a] = v[a] != 0.0f ? 1000.0f / v[a] : 0.0f;
        }
        // a sample s inside the volume
        int s = (int)(U(rng) * U(rng) * 4000.0);
        float p[3];
        sample(cen, v, depth0 + s, p);
        if (!valid_f(g, p)) continue;
        int bx[3];
        for (int a = 0; a < 3; ++a) {
          const int c = dmf::bin_axis(g, a, p[a]);
          if (c < 0 || c >= g.n[a]) goto next;
          bx[a] = c >> bsh;
        }
        {
          const int R = U(rng) < 0.5 ? (int)(U(rng) * 4) : (int)(U(rng) * 64);
          int clo[3], chi[3];
          float fdmax = 3.0e38f;
          for (int a = 0; a < 3; ++a) {
            clo[a] = std::max(bx[a] - R, 0) << bsh;
            chi[a] = std::min((bx[a] + R + 1) << bsh, g.n[a]);
            if (v[a] == 0.0f) continue;
            // rev_step (DMF_REV_VERIFY_JUMPS = 0): the exit face moved in by jmarg
            const int cf = v[a] > 0.0f ? chi[a] : clo[a];
            const float face = (float)(g.mn[a] + (double)cf * g.dl[a]);
            const float fin = v[a] > 0.0f ? face - g.jmarg[a] : face + g.jmarg[a];
            fdmax = std::fmin(fdmax, (fin - cen[a]) * rv[a]);
          }
          const float jf = std::floor(fdmax) - (float)depth0 - 2.0f;
          ++tried;
          if (!(jf > (float)(s + 1) && jf < (float)max_steps && jf < 4194304.0f)) goto next;
          ++taken;
          const int j = (int)jf;
          auto inside = [&](int k) {
            float x[3];
            sample(cen, v, depth0 + k, x);
            if (!valid_f(g, x)) return false;
            for (int a = 0; a < 3; ++a) {
              const int c = dmf::bin_axis(g, a, x[a]);
              if (c < clo[a] || c >= chi[a]) return false;
            }
            return true;
          };
          if (!inside(j)) {
            if (++fails <= 10)
              std::printf("FAIL grid n=%d,%d,%d bsh %d R %d s %d j %d v %.9g %.9g %.9g cen %.9g %.9g %.9g\n", g.n[0],
                          g.n[1], g.n[2], bsh, R, s, j, v[0], v[1], v[2], cen[0], cen[1], cen[2]);
            goto next;
          }
          if (j - s < 64) {
            for (int k = s + 1; k < j; ++k) {
              ++between;
              if (!inside(k)) {
                if (++fails <= 10) std::printf("FAIL between: s %d k %d j %d\n", s, k, j);
                break;
              }
            }
          }
        }
      next:;
      }
    }
  }
  std::printf("reverse: jumps tried %ld taken %ld, samples between checked %ld, %ld failures\n", tried, taken, between,
              fails);
  const long rfails = fails;
  fails = forward_part(trials, seed + 1);
  std::printf("total %ld failures\n", rfails + fails);
  return rfails + fails ? 1 : 0;
}
