// CPU self-test of the exact reciprocal division used by the marches (dmf_internal.hpp
// div_rn): for a divisor d with y = RN(1/d) (host division, correctly rounded),
//   q0 = RN(n * y);  r = fma(-d, q0, n) (exact);  q = fma(r, y, q0)
// must equal the correctly rounded quotient RN(n / d) for every n in the domains the
// kernels use (Markstein's final-step theorem; no overflow or underflow there).  Checks:
//   1. double, projectPoint (Camera.hpp:24-31): n = RN(RN(mm * 0.001) * ((double)col - c)),
//      mm in [0, 1100] x col in [0, 2048) and mm in [1101, 65535] x every 7th column, for
//      the K values of the tests / bench and
//      random focal lengths and principal points;
//   2. float, the reverse march's (v * depth) / 1000.0f (RayTracingEngine.hpp:166-176):
//      every float n with |n| in [2^-40, 2^40], and +-0.
// Build: g++ -O2 -ffp-contract=off tools/fastdiv_selftest.cpp ; run: ./a.out [stride]
// (stride > 1 subsamples depths and float bit patterns: the sanitizer build of
// tests/test_selftests.py; the exhaustive run is stride 1)
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

// (n = +-0: the fma step would lose the sign of zero; q0 = n * y carries it)
static double div_rn(double n, double d, double y) {
  const double q0 = n * y;
  const double r = std::fma(-d, q0, n);
  const double q = std::fma(r, y, q0);
  return n == 0.0 ? q0 : q;
}
static float div_rn(float n, float d, float y) {
  const float q0 = n * y;
  const float r = std::fmaf(-d, q0, n);
  const float q = std::fmaf(r, y, q0);
  return n == 0.0f ? q0 : q;
}

int main(int argc, char** argv) {
  const int stride = argc > 1 ? std::atoi(argv[1]) : 1;
  long bad = 0, checked = 0;
  // 1. double projection quotients
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> uf(50.0, 5000.0), uc(0.0, 2048.0);
  double cams[64][2];
  const double fixed[][2] = {{602.3930664062500, 314.6370849609375},  // reference K (Raytracing.cpp:61) fx, cx
                             {602.3930664062500, 245.0496215820312},  // fy, cy
                             {1204.7861328125, 629.274169921875},     // 1280x720
                             {1204.7861328125, 370.0992431640625}};
  int nc = 0;
  for (auto& f : fixed) { cams[nc][0] = f[0]; cams[nc][1] = f[1]; ++nc; }
  while (nc < 64) { cams[nc][0] = (double)(float)uf(rng); cams[nc][1] = (double)(float)uc(rng); ++nc; }
  for (int k = 0; k < nc; ++k) {
    const double d = cams[k][0], c = cams[k][1], y = 1.0 / d;
    for (int mm = 0; mm <= 1100; mm += stride) {
      const double z = mm * 0.001;
      for (int col = 0; col < 2048; ++col) {
        const double n = z * ((double)col - c);
        const double q = div_rn(n, d, y), e = n / d;
        ++checked;
        if (std::memcmp(&q, &e, 8) != 0) {
          if (bad < 10) std::printf("double mismatch d=%.17g n=%.17g: %.17g vs %.17g\n", d, n, q, e);
          ++bad;
        }
      }
    }
  }
  // 1b. the whole uint16 depth range, every 7th column
  for (int k = 0; k < nc; ++k) {
    const double d = cams[k][0], c = cams[k][1], y = 1.0 / d;
    for (int mm = 1101; mm <= 65535; mm += stride) {
      const double z = mm * 0.001;
      for (int col = mm % 7; col < 2048; col += 7) {
        const double n = z * ((double)col - c);
        const double q = div_rn(n, d, y), e = n / d;
        ++checked;
        if (std::memcmp(&q, &e, 8) != 0) {
          if (bad < 10) std::printf("double mismatch d=%.17g n=%.17g: %.17g vs %.17g\n", d, n, q, e);
          ++bad;
        }
      }
    }
  }
  // 2. float n / 1000.0f over every float with |n| in [2^-40, 2^40] (the kernels' fast
  //    range; outside it they divide: near the subnormal range the identity fails, e.g.
  //    n = 2.17e-41)
  const float d = 1000.0f, y = 1.0f / 1000.0f;
  for (uint32_t bits = ((127u - 40u) << 23); bits < ((127u + 40u) << 23); bits += (uint32_t)stride) {
    for (int s = 0; s < 2; ++s) {
      float n;
      const uint32_t b = bits | (s ? 0x80000000u : 0u);
      std::memcpy(&n, &b, 4);
      const float q = div_rn(n, d, y), e = n / d;
      ++checked;
      if (std::memcmp(&q, &e, 4) != 0) {
        if (bad < 20) std::printf("float mismatch n=%.9g: %.9g vs %.9g\n", n, q, e);
        ++bad;
      }
    }
  }
  for (float n : {0.0f, -0.0f}) {
    const float q = div_rn(n, d, y), e = n / d;
    ++checked;
    if (std::memcmp(&q, &e, 4) != 0) ++bad;
  }
  std::printf("fastdiv selftest: %ld quotients, %ld mismatches\n", checked, bad);
  return bad != 0;
}
