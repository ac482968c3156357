// Microbenchmark: issue rate of the fusion walk's integer VALU mix (bit selects, shifts,
// adds, compare+cndmask) on gfx950, with 1..8 waves per SIMD.  Prints instructions per
// cycle per SIMD from the kernel time (clock from hipDeviceAttributeClockRate).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ inline int bsel(int m, int a, int b) { return (a & m) | (b & ~m); }

template <int MODE>
__global__ void k_step(int iters, int* out) {
  int E01 = threadIdx.x * 7 - 100, E02 = threadIdx.x * 3 - 50, E12 = threadIdx.x - 20;
  const int K1 = 13 + (threadIdx.x & 3), K2 = 17, nK0 = -19, nK1 = -K1;
  int cur = threadIdx.x, dX = 1057, dY = 33, dZ = 1;
  const int rem = 5 + (threadIdx.x & 7), dummy = 4096 + threadIdx.x;
  unsigned long long P1 = ((unsigned long long)(unsigned)(E01 + (int)0x80000000) << 32) | (unsigned)cur;
  unsigned long long P2 = ((unsigned long long)(unsigned)(E12 + (int)0x80000000) << 32) | (unsigned)(E02 + (int)0x80000000);
  const unsigned long long Dx1 = ((unsigned long long)(long long)K1 << 32) + (long long)dX,
                           Dy1 = ((unsigned long long)(long long)nK0 << 32) + (long long)dY, Dz1 = (long long)dZ,
                           Dx2 = (unsigned long long)(long long)K2, Dy2 = (unsigned long long)(long long)K2 << 32,
                           Dz2 = ((unsigned long long)(long long)nK1 << 32) + (long long)nK0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (MODE == 0) {  // bit-select form
        const int m0 = E01 >> 31;
        const int m1 = bsel(m0, E02, E12) >> 31;
        E01 += bsel(m1, bsel(m0, K1, nK0), 0);
        E02 += bsel(m1, bsel(m0, K2, 0), nK0);
        E12 += bsel(m1, bsel(m0, 0, K2), nK1);
        cur += bsel(m1, bsel(m0, dX, dY), dZ);
      } else if (MODE == 1) {  // plain adds (independent chains): raw VALU rate
        E01 += K1; E02 += K2; E12 += nK1; cur += dX;
        E01 ^= dY; E02 ^= dZ; E12 ^= nK0; cur ^= K2;
      } else if (MODE == 3 || MODE == 5) {  // 64-bit packed (E01+2^31, cur) and (E12+2^31, E02+2^31)
        const unsigned h1 = (unsigned)(P1 >> 32), lo2 = (unsigned)P2, hi2 = (unsigned)(P2 >> 32);
        const bool A = h1 > 0x80000000u;
        const bool B = (A ? hi2 : lo2) > 0x80000000u;
        const unsigned long long d1 = B ? Dz1 : (A ? Dy1 : Dx1);
        const unsigned long long d2 = B ? Dz2 : (A ? Dy2 : Dx2);
        if (MODE == 5) asm volatile("" ::"v"(u < rem ? (int)(unsigned)P1 : dummy));
        P1 += d1;
        P2 += d2;
      } else if (MODE == 4) {  // compare + cndmask + dummy-address predication
        asm volatile("" ::"v"(u < rem ? cur : dummy));
        const bool b10 = E01 > 0;
        const bool s2 = (b10 ? E12 : E02) > 0;
        const bool s1 = !s2 && b10, s0 = !s2 && !b10;
        E01 += s0 ? K1 : (s1 ? nK0 : 0);
        E02 += s0 ? K2 : (s2 ? nK0 : 0);
        E12 += s1 ? K2 : (s2 ? nK1 : 0);
        cur += s2 ? dZ : (s1 ? dY : dX);
      } else {  // compare + cndmask form
        const bool b10 = E01 > 0;
        const bool s2 = (b10 ? E12 : E02) > 0;
        const bool s1 = !s2 && b10, s0 = !s2 && !b10;
        E01 += s0 ? K1 : (s1 ? nK0 : 0);
        E02 += s0 ? K2 : (s2 ? nK0 : 0);
        E12 += s1 ? K2 : (s2 ? nK1 : 0);
        cur += s2 ? dZ : (s1 ? dY : dX);
      }
    }
  }
  if ((E01 ^ E02 ^ E12 ^ cur ^ (int)P1 ^ (int)(P2 >> 7)) == 0x12345678) out[0] = 1;
}

int main() {
  int dev = 0, clk = 0, ncu = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int* out;
  hipMalloc(&out, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4000;
  for (int mode = 0; mode < 6; ++mode) {
    for (int wps = 1; wps <= 8; wps *= 2) {  // waves per SIMD
      const int threads = 256 * wps > 1024 ? 1024 : 256 * wps, blocks = ncu * (256 * wps / threads);
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(k_step<0>, dim3(blocks), dim3(threads), 0, 0, iters, out);
        else if (mode == 1) hipLaunchKernelGGL(k_step<1>, dim3(blocks), dim3(threads), 0, 0, iters, out);
        else if (mode == 2) hipLaunchKernelGGL(k_step<2>, dim3(blocks), dim3(threads), 0, 0, iters, out);
        else if (mode == 3) hipLaunchKernelGGL(k_step<3>, dim3(blocks), dim3(threads), 0, 0, iters, out);
        else if (mode == 4) hipLaunchKernelGGL(k_step<4>, dim3(blocks), dim3(threads), 0, 0, iters, out);
        else hipLaunchKernelGGL(k_step<5>, dim3(blocks), dim3(threads), 0, 0, iters, out);
      };
      launch();
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double waves_per_simd = wps, steps = 8.0 * iters;
      const double cycles = ms * 1e-3 * clk * 1e3;
      printf("mode %d  waves/SIMD %d  %.3f ms  cycles per step per SIMD-wave-step %.2f (clock %d MHz)\n", mode, wps, ms,
             cycles / (steps * waves_per_simd), clk / 1000);
    }
  }
  return 0;
}
