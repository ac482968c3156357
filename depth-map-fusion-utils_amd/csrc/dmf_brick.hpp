// dmf_brick.hpp — exact brick decomposition of the fusion DDA.
//
// The fusion walk (oracle.cpp dda_ray) visits the cells of a ray in
// the order of its crossing EVENTS: axis a's k-th crossing happens at time
// T_a(k) = (h_a + 2Qk) * prod_{b != a, |dq_b| > 0} |dq_b|, and events are taken in
// lexicographic (T, axis) order (ties x < y < z).  Everything here follows from that
// one ordering, in exact integer arithmetic:
//
//  * comparing two events (a, k_a), (b, k_b) divides out the common factor:
//      (h_a + 2Q k_a) |dq_b|  vs  (h_b + 2Q k_b) |dq_a|        (< 2^40, 64-bit)
//  * the number of b-events at or before event (a*, H*) [H* = h_a* + 2Q k*] is
//      #{k >= 0 : k Y < X}  (b > a*)   or   #{k >= 0 : k Y <= X}  (b < a*)
//      with X = H* |dq_b| - h_b |dq_a*|, Y = 2Q |dq_a*|  (an integer division);
//  * the fine walk's int32 state after c_a crossings per axis is
//      E_ab = E_ab(0) + c_a K_b - c_b K_a  (K = 2Q|dq|; exact mod 2^32, |E| < 2^29);
//  * brick boundaries are a subset of the crossings, so the sequence of 32^3 bricks
//    the walk passes through is a coarse walk over those events with the same order.
//
// Pass A/B (k_bk_count / k_bk_scatter) run the coarse walk per ray to build per-brick
// ray lists; phase 2 (k_bk_fuse) restarts the fine walk at each (ray, brick) pair's
// entry event and stops at its exit event, so every cell update of the fine walk is
// made exactly once, inside the workgroup that owns the brick (LDS counters, no
// device atomics per update).  All functions are __host__ __device__: the CPU
// self-test (tools/brick_selftest.cpp) checks them against the plain fine walk.
#pragma once
#include <cmath>
#include <cstdint>

#ifndef __HIPCC__
#define __host__
#define __device__
#endif

namespace dmf {
namespace brick {

#if defined(DMF_EXP_BRICK_LOG)  // experiment builds (tools/build_exp.sh): another brick edge, e.g. 4 = 16^3
constexpr int kLog = DMF_EXP_BRICK_LOG;
#else
constexpr int kLog = 5;                 // bricks of 32^3 cells
#endif
constexpr int kB = 1 << kLog;
constexpr int kCells = kB * kB * kB;    // 32768 LDS counters (128 KiB)
constexpr int kMaxBricks = 32768;       // per-WG LDS histograms of pass A/B (grids <= 1024^3)
constexpr int64_t kQ = 256;             // sub-cell fixed point (oracle.cpp kQ)
constexpr int32_t kNever = 1 << 30;     // fine-walk E of a pair with a non-moving axis
constexpr int64_t kNever64 = (int64_t)1 << 62;  // coarse-walk equivalent

// Ray after clipping/quantisation: start/end fixed-point positions (1/256 cell).
struct QRay {
  int32_t cs[3], ce[3];  // start / end cell
  int32_t st[3];         // step per axis (-1, 0, +1)
  int32_t n[3];          // crossings per axis |ce - cs|
  int32_t adq[3];        // |qe - qs|
  int32_t h0[3];         // first-crossing numerator (half fixed-point units)
  int32_t nsteps;        // n[0] + n[1] + n[2]
  bool end_inside;
};

// 16-byte ray record: 19 bits per fixed-point coordinate (grids <= 2048 cells/axis).
//   A = qs0 | qs1 << 19 | qs2 << 38 | end_inside << 63
//   B = qe0 | qe1 << 19 | qe2 << 38 | valid << 63
__host__ __device__ inline void pack_ray(const int64_t qs[3], const int64_t qe[3], bool end_inside, uint64_t& A,
                                         uint64_t& B) {
  A = (uint64_t)qs[0] | ((uint64_t)qs[1] << 19) | ((uint64_t)qs[2] << 38) | ((uint64_t)(end_inside ? 1 : 0) << 63);
  B = (uint64_t)qe[0] | ((uint64_t)qe[1] << 19) | ((uint64_t)qe[2] << 38) | ((uint64_t)1 << 63);
}

// The QRay of quantised endpoints qs, qe (what decode_ray gives for their record).
__host__ __device__ inline void qray_from(const int32_t qs[3], const int32_t qe[3], bool end_inside, QRay& r) {
  r.end_inside = end_inside;
  r.nsteps = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    r.cs[a] = qs[a] >> 8;
    r.ce[a] = qe[a] >> 8;
    const int32_t dq = qe[a] - qs[a];
    r.adq[a] = dq < 0 ? -dq : dq;
    r.st[a] = r.ce[a] > r.cs[a] ? 1 : (r.ce[a] < r.cs[a] ? -1 : 0);
    r.n[a] = r.ce[a] > r.cs[a] ? r.ce[a] - r.cs[a] : r.cs[a] - r.ce[a];
    // oracle.cpp dda_ray: moving up 2((cs+1)Q - qs), moving down 2(qs - cs Q) + 1
    r.h0[a] = r.st[a] > 0 ? 2 * ((r.cs[a] + 1) * (int32_t)kQ - qs[a]) : 2 * (qs[a] - r.cs[a] * (int32_t)kQ) + 1;
    r.nsteps += r.n[a];
  }
}

__host__ __device__ inline void decode_ray(uint64_t A, uint64_t B, QRay& r) {
  constexpr uint64_t m = (1u << 19) - 1;
  const int32_t qs[3] = {(int32_t)(A & m), (int32_t)((A >> 19) & m), (int32_t)((A >> 38) & m)};
  const int32_t qe[3] = {(int32_t)(B & m), (int32_t)((B >> 19) & m), (int32_t)((B >> 38) & m)};
  qray_from(qs, qe, (A >> 63) != 0, r);
}

// Fine-walk E of the pair (a, b) at the ray start (dmf_fuse.hip dda_setup).
__host__ __device__ inline int32_t e0_pair(const QRay& r, int a, int b) {
  if (r.st[a] && r.st[b]) return (int32_t)((int64_t)r.h0[a] * r.adq[b] - (int64_t)r.h0[b] * r.adq[a]);
  return r.st[a] ? -kNever : (r.st[b] ? kNever : 0);
}

// Event (a, H_a) strictly before event (b, H_b) in (T, axis) order; both axes moving.
__host__ __device__ inline bool ev_before(const QRay& r, int a, int64_t Ha, int b, int64_t Hb) {
  const int64_t L = Ha * (int64_t)r.adq[b], R = Hb * (int64_t)r.adq[a];
  return L < R || (L == R && a < b);
}

// floor(X / Y) for 0 <= X < 2^41, 0 < Y < 2^28 with a small quotient: count_at's quotient
// counts b-crossings up to a crossing event of the same ray, so it is <= n_b + 1 <= 2^11.
// Float estimate (relative error < 2^-21, so within 1 of the floor) and one exact
// correction in either direction.  The remainder is taken in 32 bits: with q within 1 of
// floor(X / Y) it lies in (-Y, 2Y), |.| < 2^29, so the wrapped difference of the low words
// is exact.
__host__ __device__ inline int32_t quot_small32(int64_t X, int32_t Y) {
  const float xf = (float)(int32_t)(X >> 20) * 1048576.0f + (float)(int32_t)(X & 0xfffff);
  const float yf = (float)Y;
#if defined(__HIP_DEVICE_COMPILE__)
  int32_t q = (int32_t)(xf * __builtin_amdgcn_rcpf(yf));  // v_rcp_f32: 1 ulp
#else
  int32_t q = (int32_t)(xf / yf);
#endif
  const int32_t rm = (int32_t)((uint32_t)X - (uint32_t)q * (uint32_t)Y);
  q += rm < 0 ? -1 : (rm >= Y ? 1 : 0);
  return q;
}

// Number of b-crossings taken at or before the event (a, Ha) (a's own crossings are
// the caller's: k + 1).  b != a.  Ha = h0_a + 2Qk < 2^21 and |dq| < 2^19 (grids <= 2048
// cells per axis): X is a difference of two 32x32-bit products, Y = 2Q|dq_a| < 2^28.
__host__ __device__ inline int32_t count_at(const QRay& r, int b, int a, int32_t Ha) {
  if (r.st[b] == 0) return 0;
  const int64_t X = (int64_t)Ha * (int64_t)r.adq[b] - (int64_t)r.h0[b] * (int64_t)r.adq[a];
  const int32_t Y = (int32_t)(2 * kQ) * r.adq[a];
  int32_t c;
  if (b < a) c = X < 0 ? 0 : quot_small32(X, Y) + 1;
  else c = X <= 0 ? 0 : quot_small32(X - 1, Y) + 1;
  return c < r.n[b] ? c : r.n[b];
}

// Crossing counts per axis at (and including) event (a, k); a < 0 = the ray start.
__host__ __device__ inline void counts_at(const QRay& r, int a, int32_t k, int32_t c[3]) {
  if (a < 0) { c[0] = c[1] = c[2] = 0; return; }
  const int32_t Ha = r.h0[a] + (int32_t)(2 * kQ) * k;
#pragma unroll
  for (int b = 0; b < 3; ++b) c[b] = (b == a) ? k + 1 : count_at(r, b, a, Ha);
}

// The value of x, opaque to the optimiser: a select between struct fields must stay a
// register select (folded into a select of addresses, the fields go to scratch memory).
__host__ __device__ inline int32_t opaque(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm("" : "+v"(x));
#endif
  return x;
}

// a * b for |a|, |b| < 2^23: the low 32 bits of the product, as the plain 32-bit product gives
// them.  On the device one v_mul_i32_i24 / v_mad_i32_i24, where the compiler's 32-bit integer
// multiply is a v_mul_lo_u32 / v_mad_u64_u32 (passes A / B: step -0.2 %; the
// experiment build -DDMF_EXP_MUL32 restores the 32-bit multiply).  The brick path's
// operands are in range: brick coordinates and counts <= 1024, |dq| < 2^18 (<= 1024 cells per
// axis, dmf_fuse.hip brick_path_ok).
#if defined(__HIP_DEVICE_COMPILE__)
// the LLVM intrinsic itself: HIP's __mul24 sign-extends its operands in IR, and when only some
// low bits of a product are used (a cell coordinate & 31, a count times 2 kQ) the optimiser
// drops that extension and selects the 32-bit multiply again
extern "C" __device__ int32_t dmf_llvm_mul_i24(int32_t, int32_t) __asm("llvm.amdgcn.mul.i24");
#endif
__host__ __device__ inline int32_t mul24(int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(DMF_EXP_MUL32)
  return dmf_llvm_mul_i24(a, b);
#else
  return (int32_t)((uint32_t)a * (uint32_t)b);
#endif
}

__host__ __device__ inline int32_t sel3(bool a0, bool a1, int32_t v0, int32_t v1, int32_t v2) {
  return a0 ? opaque(v0) : (a1 ? opaque(v1) : opaque(v2));
}

// counts_at for an axis a that differs between the lanes of a wave (pass B's boundary
// events): one straight code path of selects.  counts_at's constant-axis branches run
// once per distinct axis among a wave's lanes; here the two other axes (ascending:
// o1 = a == 0 ? 1 : 0, o2 = a == 2 ? 1 : 2) are picked and counted by the same code, with
// count_at's tie rule as a bias (b > a: X - 1).  The quotient's remainder is taken in 32
// bits: with q within 1 of floor(X / Y) it lies in (-Y, 2Y), |.| < 2^28 (Y = 2Q|dq_a| <
// 2^27), so the wrapped difference of the low words is exact (quot_small32).  A non-moving
// axis (n = 0) is clamped to 0 whatever its quotient.  Checked against counts_at by the brick
// self-test.
__host__ __device__ inline void counts_at_sel(const QRay& r, int a, int32_t k, int32_t c[3]) {
  const bool a0 = a == 0, a1 = a == 1, a2 = a == 2;
  const int32_t ha = sel3(a0, a1, r.h0[0], r.h0[1], r.h0[2]);
  const int32_t da = sel3(a0, a1, r.adq[0], r.adq[1], r.adq[2]);
  const int64_t Ha = (int64_t)ha + 2 * kQ * (int64_t)k;
  const int32_t Y = (int32_t)(2 * kQ) * da;
  auto cnt = [&](int32_t adb, int32_t hb, int32_t nb, bool after) -> int32_t {
    const int64_t X = Ha * (int64_t)adb - (int64_t)hb * (int64_t)da - (after ? 1 : 0);
    const int32_t q = quot_small32(X < 0 ? 0 : X, Y) + 1;
    return X < 0 ? 0 : (q < 0 ? 0 : (q > nb ? nb : q));
  };
  const int32_t c1 = cnt(a0 ? opaque(r.adq[1]) : opaque(r.adq[0]), a0 ? opaque(r.h0[1]) : opaque(r.h0[0]),
                         a0 ? opaque(r.n[1]) : opaque(r.n[0]), a0);
  const int32_t c2 = cnt(a2 ? opaque(r.adq[1]) : opaque(r.adq[2]), a2 ? opaque(r.h0[1]) : opaque(r.h0[2]),
                         a2 ? opaque(r.n[1]) : opaque(r.n[2]), !a2);
  c[0] = a0 ? k + 1 : c1;
  c[1] = a1 ? k + 1 : (a0 ? c1 : c2);
  c[2] = a2 ? k + 1 : c2;
}

// counts_at in double arithmetic (pass B's boundary counts).  Every quantity of count_at is
// an integer below 2^41 -- Ha < 2^20, |dq| < 2^19 on grids <= 2048 cells per axis -- so
// X = Ha |dq_b| - h_b |dq_a| is exact as fma(Ha, |dq_b|, -(h_b |dq_a|)) (the product h_b |dq_a|
// and the fma's exact result both fit 53 bits).  q = floor(X * RN(1/Y)) is within one of
// floor(X / Y) (X / Y < 2^12, relative error < 2^-51), and the remainder X - qY, exact by fma,
// corrects it.  The tie rule of count_at (b > a: X - 1) is the same bias.  Checked against
// counts_at by the brick self-test (check 7).
// The reciprocal need not be correctly rounded: with X / Y < 2^12, an inv of relative error
// eps puts X * inv within 2^12 eps of X / Y, so q stays within one of the floor -- which the
// remainder step corrects -- while eps < 2^-12.  The device takes v_rcp_f64, whose documented
// precision (2^29 ulps of a double) is a relative error near 2^-23; the self-test (check 7b)
// runs the counts with inv perturbed by +-2 ulps and by relative errors of +-2^-22 and +-2^-14.
struct QRayF64 {
  double adq[3], h[3], inv[3];  // |dq|, first-crossing numerator h0, ~1 / (2Q |dq|) (0: non-moving)
  double hx[3][3];              // [A][b], b != A: -(h_b |dq_A|) - (b > A), count_at's tie rule folded in
};
__host__ __device__ inline void qray_f64(const QRay& r, QRayF64& f) {
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    f.adq[a] = (double)r.adq[a];
    f.h[a] = (double)r.h0[a];
#if defined(__HIP_DEVICE_COMPILE__)
    f.inv[a] = r.adq[a] ? __builtin_amdgcn_rcp(2.0 * (double)kQ * (double)r.adq[a]) : 0.0;
#else
    f.inv[a] = r.adq[a] ? 1.0 / (2.0 * (double)kQ * (double)r.adq[a]) : 0.0;
#endif
  }
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) f.hx[a][b] = -(f.h[b] * f.adq[a]) - (b > a ? 1.0 : 0.0);  // exact: < 2^53
}
template <int A>
__host__ __device__ inline void counts_at_f64(const QRay& r, const QRayF64& f, int32_t k, int32_t c[3]) {
  const double Ha = fma(2.0 * (double)kQ, (double)k, f.h[A]);
  const double Y = 2.0 * (double)kQ * f.adq[A];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    if (b == A) {
      c[b] = k + 1;
      continue;
    }
    const double X = fma(Ha, f.adq[b], f.hx[A][b]);
    const double q = floor(X * f.inv[A]);
    const double rm = fma(-q, Y, X);
    // floor(X / Y) + 1 = q + 1, corrected by the exact remainder (one of the two terms at most)
    const int32_t cq = (int32_t)q + (rm < 0.0 ? 0 : 1) + (rm >= Y ? 1 : 0);
    c[b] = (r.st[b] == 0 || X < 0.0) ? 0 : (cq < r.n[b] ? cq : r.n[b]);
  }
}

// One (ray, brick) pair: where the fine walk enters brick (bx, by, bz), how many
// cells it visits there, and whether the last of them is the ray's end cell.
struct Pair {
  int32_t cin[3];  // crossings taken before the first cell in the brick
  int32_t cells;   // cells visited in the brick (>= 1 for a visited brick)
  bool ends;       // the ray's end cell is the last of them
};

__host__ __device__ inline void pair_in_brick(const QRay& r, const int32_t bb[3], const int32_t ng[3], Pair& p) {
  int ai = -1, ao = -1;
  int32_t ki = 0, ko = 0;
  int64_t Hi = 0, Ho = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int32_t lo = bb[a] << kLog;
    const int32_t hi = (lo + kB - 1 < ng[a] - 1) ? lo + kB - 1 : ng[a] - 1;
    // entry along a: the crossing that brings c_a into [lo, hi]
    int32_t k = -1;
    if (r.st[a] > 0 && r.cs[a] < lo) k = lo - r.cs[a] - 1;
    if (r.st[a] < 0 && r.cs[a] > hi) k = r.cs[a] - hi - 1;
    if (k >= 0) {
      const int64_t H = (int64_t)r.h0[a] + 2 * kQ * (int64_t)k;
      if (ai < 0 || ev_before(r, ai, Hi, a, H)) { ai = a; ki = k; Hi = H; }  // latest entry
    }
    // exit along a: the crossing that takes c_a out of [lo, hi]
    k = -1;
    if (r.st[a] > 0 && r.ce[a] > hi) k = hi - r.cs[a];
    if (r.st[a] < 0 && r.ce[a] < lo) k = r.cs[a] - lo;
    if (k >= 0) {
      const int64_t H = (int64_t)r.h0[a] + 2 * kQ * (int64_t)k;
      if (ao < 0 || ev_before(r, a, H, ao, Ho)) { ao = a; ko = k; Ho = H; }  // earliest exit
    }
  }
  counts_at(r, ai, ki, p.cin);
  const int32_t idx_in = p.cin[0] + p.cin[1] + p.cin[2];
  if (ao >= 0) {
    int32_t co[3];
    counts_at(r, ao, ko, co);
    p.cells = co[0] + co[1] + co[2] - idx_in;
    p.ends = false;
  } else {
    p.cells = r.nsteps - idx_in + 1;
    p.ends = true;
  }
}

// Coarse walk over brick-boundary crossings: the bricks the fine walk passes
// through, in order.  init() then `total` calls of next().
struct Coarse {
  int64_t E01, E02, E12, K0, K1, K2;  // E at the next boundary crossings; K = 32 * 2Q|dq|
  int32_t total;                      // boundary crossings of the whole ray
};

// Brick boundaries the ray crosses (the coarse walk's step count).
__host__ __device__ inline int32_t coarse_total(const QRay& r) {
  int32_t total = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int32_t off = r.cs[a] & (kB - 1);
    const int32_t k0 = r.st[a] > 0 ? kB - 1 - off : off;  // first boundary crossing
    if (r.st[a] != 0 && r.n[a] > k0) total += (r.n[a] - 1 - k0) / kB + 1;
  }
  return total;
}

__host__ __device__ inline void coarse_init(const QRay& r, Coarse& w) {
  int32_t H[3];  // < 2Q (kB + 1): 32x32-bit products below
  w.total = coarse_total(r);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int32_t off = r.cs[a] & (kB - 1);
    const int32_t k0 = r.st[a] > 0 ? kB - 1 - off : off;  // first boundary crossing
    H[a] = r.h0[a] + (int32_t)(2 * kQ) * k0;
  }
  auto pr = [&](int a, int b) -> int64_t {
    if (r.st[a] && r.st[b]) return (int64_t)H[a] * (int64_t)r.adq[b] - (int64_t)H[b] * (int64_t)r.adq[a];
    return r.st[a] ? -kNever64 : (r.st[b] ? kNever64 : 0);
  };
  w.E01 = pr(0, 1);
  w.E02 = pr(0, 2);
  w.E12 = pr(1, 2);
  w.K0 = (int64_t)kB * 2 * kQ * r.adq[0];
  w.K1 = (int64_t)kB * 2 * kQ * r.adq[1];
  w.K2 = (int64_t)kB * 2 * kQ * r.adq[2];
}

// Next boundary crossing: returns its axis (ties x < y < z, as the fine walk).
__host__ __device__ inline int coarse_next(Coarse& w) {
  const bool b10 = w.E01 > 0;
  const bool s2 = (b10 ? w.E12 : w.E02) > 0;
  const bool s1 = !s2 && b10, s0 = !s2 && !b10;
  w.E01 += s0 ? w.K1 : (s1 ? -w.K0 : 0);
  w.E02 += s0 ? w.K2 : (s2 ? -w.K0 : 0);
  w.E12 += s1 ? w.K2 : (s2 ? -w.K1 : 0);
  return s2 ? 2 : (s1 ? 1 : 0);
}

// coarse_next without its state: the axis of the next brick-boundary crossing of a ray now in
// brick coordinates (b0, b1, b2).  On each moving axis the next boundary is fine crossing
// k_a (into brick b_a + st_a); the earliest of those events in (T, axis) order (ev_before:
// H_a |dq_b| against H_b |dq_a|, ties x < y < z) is the one coarse_next takes.  An axis
// whose boundaries are all behind the ray's end never wins while crossings remain, so the
// caller takes exactly coarse_total steps, as with coarse_next.  For pass B's rays past the
// recorded path: no 64-bit walk state held across the replay.
// (kept from being hoisted out of the replay loop: its operands are loop-invariant, and as
// hoisted 64-bit values they would stay live across every ray's replay)
__host__ __device__ inline int32_t pinned(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#endif
  return x;
}
// coarse_next_at from the three next-boundary crossing indices k_a themselves (pass B carries
// them per axis: k_a grows by kB per brick step along a)
__host__ __device__ inline int coarse_next_k(const QRay& r, int32_t k0, int32_t k1, int32_t k2) {
  int best = -1;
  int64_t Hb = 0;
  int32_t db = 0;
  const int32_t ks[3] = {k0, k1, k2};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int32_t st = pinned(r.st[a]);
    if (st == 0) continue;
    const int32_t da = pinned(r.adq[a]);
    const int64_t H = (int64_t)pinned(r.h0[a]) + 2 * kQ * (int64_t)ks[a];
    // ev_before(r, a, H, best, Hb): H |dq_best| < Hb |dq_a| (a > best: ties keep best)
    if (best < 0 || H * (int64_t)db < Hb * (int64_t)da) {
      best = a;
      Hb = H;
      db = da;
    }
  }
  return best;
}
// the fine-crossing index of the boundary into brick coordinate b + st along axis a (moving up,
// cell nb*kB is reached by crossing nb*kB - cs - 1; moving down, cell nb*kB + kB - 1 by crossing
// cs - nb*kB - kB; nb may be -1: past the grid)
__host__ __device__ inline int32_t next_boundary_k(const QRay& r, int a, int b) {
  const int32_t st = r.st[a], nb = b + st;
  return st > 0 ? nb * kB - r.cs[a] - 1 : r.cs[a] - nb * kB - kB;
}
__host__ __device__ inline int coarse_next_at(const QRay& r, int b0, int b1, int b2) {
  return coarse_next_k(r, next_boundary_k(r, 0, b0), next_boundary_k(r, 1, b1), next_boundary_k(r, 2, b2));
}

// The coarse walk's crossing axes, 2 bits per brick boundary (step t at bits 2t, 2t + 1), for
// the first kPathSteps boundaries: pass A records them with its walk so that pass B replays
// the brick sequence without the 64-bit comparisons (a ray with more boundaries walks again).
constexpr int kPathSteps = 32;
__host__ __device__ inline uint64_t path_put(uint64_t path, int t, int a) {
  return t < kPathSteps ? path | (uint64_t)a << (2 * t) : path;
}
__host__ __device__ inline int path_axis(uint64_t path, int t) { return (int)(path >> (2 * t)) & 3; }

// ---- Major-axis ("slab") form of the fine walk (phase F) ----
//
// Let M be an axis with the largest |dq| (its crossings are the most frequent: interval
// 2Q/|dq_M| in tau = T / prod|dq|), m1 < m2 the other two.  Between two consecutive
// M-crossings (a "slab") each minor axis crosses AT MOST ONCE: its interval 2Q/|dq_m| is
// no shorter, and the half-open window (previous M-crossing, next M-crossing] holds one
// point of any arithmetic sequence with that step (ties keep the x < y < z order).  So the
// walk advances one slab at a time: minor m crosses in this slab iff its next crossing
// comes before the next M-crossing, the two minors (if both cross) in their own order,
// then M.  With pairwise E as in the fine walk, e_m = E_{M m} (sign-flipped when m < M)
// and e_12 = E_{m1 m2}; the biased forms below make every test "b >= 0":
//   b_m  = e_m + [m < M] - 1   >= 0  <=>  minor m crosses before the next M-crossing
//   b_12 = e_12 - 1            >= 0  <=>  m2 crosses before m1 (m1 < m2: ties go to m1)
// Updates per slab: b_m += K_m - (c_m ? K_M : 0);  b_12 += (c_1 ? K_2 : 0) - (c_2 ? K_1 : 0).
// A non-moving minor keeps b_m = -(never); the b_12 of a pair with one is never consulted.

// An axis with the largest |dq| (the lowest such index).
__host__ __device__ inline int major_axis(const QRay& r) {
  return r.adq[0] >= r.adq[1] ? (r.adq[0] >= r.adq[2] ? 0 : 2) : (r.adq[1] >= r.adq[2] ? 1 : 2);
}

__host__ __device__ inline int32_t pick3(int32_t v0, int32_t v1, int32_t v2, int a) {
  return a == 0 ? v0 : (a == 1 ? v1 : v2);
}

// Slab state (b1, b2, b12) from the fine walk's pairwise E (exact int32 values, or the
// +-kNever of a non-moving axis), major axis M.  No dynamic indexing (device scratch).
__host__ __device__ inline void slab_from_pairwise(int M, int32_t E01, int32_t E02, int32_t E12, int32_t& b1,
                                                   int32_t& b2, int32_t& b12) {
  // M = 0: minors 1, 2;  M = 1: minors 0, 2;  M = 2: minors 0, 1
  b1 = M == 0 ? (int32_t)((uint32_t)E01 - 1u) : (M == 1 ? (int32_t)(0u - (uint32_t)E01) : (int32_t)(0u - (uint32_t)E02));
  b2 = M == 0 ? (int32_t)((uint32_t)E02 - 1u) : (M == 1 ? (int32_t)((uint32_t)E12 - 1u) : (int32_t)(0u - (uint32_t)E12));
  b12 = (int32_t)((uint32_t)(M == 0 ? E12 : (M == 1 ? E02 : E01)) - 1u);
}

// Reference slab walk (CPU self-test and documentation of phase F's step): emits `cells`
// cells starting at cell p[] with state (b1, b2, b12); K* = 2Q|dq| of the major / minors,
// s* = their steps.  emit(x, y, z) per cell, in walk order.
template <class F>
__host__ __device__ inline void slab_walk(int M, int32_t b1, int32_t b2, int32_t b12, uint32_t KM, uint32_t K1,
                                          uint32_t K2, const int32_t st[3], const int32_t p0[3], int cells, F&& emit) {
  const int m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  int32_t p[3] = {p0[0], p0[1], p0[2]};
  int rem = cells;
  while (rem > 0) {
    const bool c1 = b1 >= 0, c2 = b2 >= 0, o = b12 >= 0;
    emit(p[0], p[1], p[2]);
    --rem;
    if (c1 && c2) {
      const int f = o ? m2 : m1, s = o ? m1 : m2;
      p[f] += st[f];
      if (rem > 0) { emit(p[0], p[1], p[2]); --rem; }
      p[s] += st[s];
      if (rem > 0) { emit(p[0], p[1], p[2]); --rem; }
    } else if (c1 || c2) {
      const int f = c1 ? m1 : m2;
      p[f] += st[f];
      if (rem > 0) { emit(p[0], p[1], p[2]); --rem; }
    }
    p[M] += st[M];
    b1 = (int32_t)((uint32_t)b1 + K1 - (c1 ? KM : 0u));
    b2 = (int32_t)((uint32_t)b2 + K2 - (c2 ? KM : 0u));
    b12 = (int32_t)((uint32_t)b12 + (c1 ? K2 : 0u) - (c2 ? K1 : 0u));
  }
}

// Slab ownership code of a pair (phase F's walk bound, the record's 7-bit count field):
// R = 3 S + s, where S = slabs walked before the one holding the pair's last cell L and
// s = cells of L's slab before L.  Cell j (0, 1, 2) of slab k is then owned by the walk
// (before L) iff R - 3k > j, so F tests three constant thresholds per slab instead of
// counting cells.  cin = crossing counts at the pair's first cell, cL = at L (counts
// since the ray's start); sb1, sb2 = slab state (b1, b2) at the ray's start (counts 0).
// Minor m crossed inside L's slab iff its latest crossing (number cL_m) comes after the
// major axis's crossing number cL_M that opened the slab, i.e. iff at counts
// (cL_M - 1, cL_m - 1), where both are the next crossings, b_m < 0 (the slab state's
// "m crosses before M" test with its tie order).  Evaluated in 64 bits: that state need
// not be one the walk passes through (m's latest crossing may lie far back), so its b can
// leave the int32 range.  S = 0: R = the pair's cells - 1 (all in its first slab).
__host__ __device__ inline uint32_t slab_rcode(int M, int32_t sb1, int32_t sb2, uint32_t KM, uint32_t K1, uint32_t K2,
                                               const int32_t cin[3], const int32_t cL[3]) {
  const int m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  const int32_t LM = pick3(cL[0], cL[1], cL[2], M), L1 = pick3(cL[0], cL[1], cL[2], m1),
                L2 = pick3(cL[0], cL[1], cL[2], m2);
  const int32_t S = LM - pick3(cin[0], cin[1], cin[2], M);
  const uint32_t steps = (uint32_t)((cL[0] - cin[0]) + (cL[1] - cin[1]) + (cL[2] - cin[2]));
  // e = the state one M- and one minor crossing before the last cell's: within K_1 + K_M of a
  // walk state (|b| < 2^29), so |e| < 2^30 and the wrapped 32-bit sum is exact; (L - 1) K =
  // 2 kQ (L - 1) |dq| mod 2^32 with 24-bit multiplies (K = 2 kQ |dq|)
  const uint32_t k2 = (uint32_t)(2 * kQ);
  const int32_t aM = (int32_t)(KM / k2), a1 = (int32_t)(K1 / k2), a2 = (int32_t)(K2 / k2);
  const int32_t e1 = (int32_t)((uint32_t)sb1 + ((uint32_t)mul24(LM - 1, a1) - (uint32_t)mul24(L1 - 1, aM)) * k2);
  const int32_t e2 = (int32_t)((uint32_t)sb2 + ((uint32_t)mul24(LM - 1, a2) - (uint32_t)mul24(L2 - 1, aM)) * k2);
  const uint32_t s = (L1 >= 1 && e1 < 0 ? 1u : 0u) + (L2 >= 1 && e2 < 0 ? 1u : 0u);
  return S == 0 ? steps : 3u * (uint32_t)S + s;
}

// Slab code of a pair (round 6: the record's 8-bit walk field, phase F's walk bound):
//   code = S | s << 5 | e << 7
// S = slabs the walk takes whole (the M-crossings between the pair's first cell and its last
// cell L, <= 31 inside a 32-cell brick), s = cells of L's slab before L (0..2), and e = the
// minor whose crossing entered L when s >= 1 (0: m1, 1: m2).  Phase F walks S whole slabs
// with ONE ownership test per slab (every cell of slab k < S lies before L) and adds L's slab
// at adoption from L itself: L - d_e (s >= 1) and L - d_1 - d_2 (s = 2, the slab's first
// cell) -- instead of three per-cell thresholds in every slab (R = 3 S + s, slab_rcode).
// e for s = 2: the later of the two minor crossings of L's slab; m1's (L1-th) and m2's
// (L2-th) crossings are the next crossings at counts (L1 - 1, L2 - 1), where b_12 >= 0 says
// m2's comes first (ties to m1): then m1 entered L (e = 0), else m2 (e = 1).  That b_12 is
// a state the walk passes through (its start of L's slab), so the wrapped int32 sum is exact.
__host__ __device__ inline uint32_t slab_code(int M, int32_t sb1, int32_t sb2, int32_t sb12, uint32_t KM, uint32_t K1,
                                              uint32_t K2, const int32_t cin[3], const int32_t cL[3]) {
  const int m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  const int32_t LM = pick3(cL[0], cL[1], cL[2], M), L1 = pick3(cL[0], cL[1], cL[2], m1),
                L2 = pick3(cL[0], cL[1], cL[2], m2);
  const int32_t S = LM - pick3(cin[0], cin[1], cin[2], M);
  const uint32_t k2 = (uint32_t)(2 * kQ);
  const int32_t aM = (int32_t)(KM / k2), a1 = (int32_t)(K1 / k2), a2 = (int32_t)(K2 / k2);
  uint32_t sc, e;
  if (S == 0) {  // L in the pair's first slab: every minor crossing since the entry is in it
    const int32_t n1 = L1 - pick3(cin[0], cin[1], cin[2], m1), n2 = L2 - pick3(cin[0], cin[1], cin[2], m2);
    sc = (uint32_t)(n1 + n2);
    e = n1 ? 0u : 1u;
  } else {  // as slab_rcode: minor m crossed in L's slab iff b_m < 0 at (cL_M - 1, cL_m - 1)
    const int32_t e1 = (int32_t)((uint32_t)sb1 + ((uint32_t)mul24(LM - 1, a1) - (uint32_t)mul24(L1 - 1, aM)) * k2);
    const int32_t e2 = (int32_t)((uint32_t)sb2 + ((uint32_t)mul24(LM - 1, a2) - (uint32_t)mul24(L2 - 1, aM)) * k2);
    const uint32_t t1 = L1 >= 1 && e1 < 0 ? 1u : 0u, t2 = L2 >= 1 && e2 < 0 ? 1u : 0u;
    sc = t1 + t2;
    e = t1 ? 0u : 1u;
  }
  if (sc == 2) {
    const int32_t e12 = (int32_t)((uint32_t)sb12 + ((uint32_t)mul24(L1 - 1, a2) - (uint32_t)mul24(L2 - 1, a1)) * k2);
    e = e12 >= 0 ? 0u : 1u;
  }
  if (sc == 0) e = 0;
  return (uint32_t)S | sc << 5 | e << 7;
}

// Phase F's walk from a slab code (CPU self-test): S whole slabs, then the cells of L's slab
// before L, derived from L (coordinates Lc) as phase F does at adoption: L - st_1 - st_2 when
// s = 2 (its first cell), then L - st_e (s >= 1).  emit(x, y, z) per cell, in walk order.
template <class F>
__host__ __device__ inline void slab_walk_code(int M, int32_t b1, int32_t b2, int32_t b12, uint32_t KM, uint32_t K1,
                                               uint32_t K2, const int32_t st[3], const int32_t p0[3], uint32_t code,
                                               const int32_t Lc[3], F&& emit) {
  const int m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  const int S = (int)(code & 31u), sc = (int)((code >> 5) & 3u), e = (int)(code >> 7);
  int32_t p[3] = {p0[0], p0[1], p0[2]};
  for (int k = 0; k < S; ++k) {
    const bool c1 = b1 >= 0, c2 = b2 >= 0, o = b12 >= 0;
    emit(p[0], p[1], p[2]);
    if (c1 || c2) {
      const int f = o ? m2 : m1, s2 = o ? m1 : m2;
      p[f] += st[f];
      emit(p[0], p[1], p[2]);
      if (c1 && c2) {
        p[s2] += st[s2];
        emit(p[0], p[1], p[2]);
      }
    }
    p[M] += st[M];
    b1 = (int32_t)((uint32_t)b1 + K1 - (c1 ? KM : 0u));
    b2 = (int32_t)((uint32_t)b2 + K2 - (c2 ? KM : 0u));
    b12 = (int32_t)((uint32_t)b12 + (c1 ? K2 : 0u) - (c2 ? K1 : 0u));
  }
  const int ea = e ? m2 : m1;
  if (sc == 2) {
    int32_t q[3] = {Lc[0], Lc[1], Lc[2]};
    q[m1] -= st[m1];
    q[m2] -= st[m2];
    emit(q[0], q[1], q[2]);
  }
  if (sc >= 1) {
    int32_t q[3] = {Lc[0], Lc[1], Lc[2]};
    q[ea] -= st[ea];
    emit(q[0], q[1], q[2]);
  }
}

// Phase F's walk bounded by a slab ownership code R (CPU self-test): slab by slab, cell j
// of slab k is emitted iff R - 3k > j; stops when R - 3k <= 0.
template <class F>
__host__ __device__ inline void slab_walk_owned(int M, int32_t b1, int32_t b2, int32_t b12, uint32_t KM, uint32_t K1,
                                                uint32_t K2, const int32_t st[3], const int32_t p0[3], int R,
                                                F&& emit) {
  const int m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  int32_t p[3] = {p0[0], p0[1], p0[2]};
  for (int t = R; t > 0; t -= 3) {
    const bool c1 = b1 >= 0, c2 = b2 >= 0, o = b12 >= 0;
    emit(p[0], p[1], p[2]);
    // the first minor step is on m2 iff o, also when only one minor crosses: m2 alone
    // crossing means m2 < next M < m1 in crossing order (and a non-moving m1 / m2 keeps
    // b12 at +- kNever), so F picks it with one select on o
    if (c1 || c2) {
      const int f = o ? m2 : m1, s = o ? m1 : m2;
      p[f] += st[f];
      if (t > 1) emit(p[0], p[1], p[2]);
      if (c1 && c2) {
        p[s] += st[s];
        if (t > 2) emit(p[0], p[1], p[2]);
      }
    }
    p[M] += st[M];
    b1 = (int32_t)((uint32_t)b1 + K1 - (c1 ? KM : 0u));
    b2 = (int32_t)((uint32_t)b2 + K2 - (c2 ? KM : 0u));
    b12 = (int32_t)((uint32_t)b12 + (c1 ? K2 : 0u) - (c2 ? K1 : 0u));
  }
}

// ---- 20-byte pair record: the slab walk on scaled state ----
//
// Every K is 2Q|dq| = 512 |dq|, and every update of the slab state (b1, b2, b12) adds a
// sum of K's, so b mod 512 never changes along a walk, and b >= 0 <=> floor(b / 512) >= 0.
// Hence the walk runs EXACTLY on beta = b >> 9 (arithmetic shift = floor division) with
// increments |dq| instead of K: the low 9 bits of b never influence a decision.  Range:
// |b| < (2Q + 1) max|dq| gives |beta| < 2^18 + 2^9 for grids <= 1024 cells per axis
// (|dq| < 2^18), a 20-bit two's-complement field; the +-never constant of a non-moving
// axis (only its sign is ever used) is stored as +-(2^19 - 1).
//   w0 = beta1 | aM[0:12) << 20          w1 = beta2 | aM[12:18) << 20 | S << 26 | ends << 31
//   w2 = beta12 | a1[0:12) << 20         w3 = entry word | last word << 16
//   w4 = a2 | a1[12:18) << 18 | T << 24,  T = s | e << 2 | step signs (x, y, z) << 3 | M << 6
// (a = |dq| of the major / minor axes, (S, s, e) = the slab code of slab_code (S | s << 5 |
// e << 7), entry / last = word offsets of the pair's first / last cell in phase F's LDS box).
// T = w[4] >> 24 is the index of phase F's stride table: one LDS read gives the pair's three
// strides and the offsets from L of the cells of L's slab that the code adopts (k_bk_fuse_s).
__host__ __device__ inline uint32_t beta20(int32_t b) {
  const int32_t lim = (1 << 19) - 1;
  const int32_t s = b >> 9;  // arithmetic shift: floor(b / 512)
  return (uint32_t)(s > lim ? lim : (s < -lim ? -lim : s)) & 0xfffffu;
}

__host__ __device__ inline void pack20(int32_t b1, int32_t b2, int32_t b12, uint32_t aM, uint32_t a1, uint32_t a2,
                                       uint32_t entry, uint32_t last, uint32_t code, uint32_t signs, uint32_t M,
                                       bool ends, uint32_t w[5]) {
  w[0] = beta20(b1) | (aM & 0xfffu) << 20;
  w[1] = beta20(b2) | ((aM >> 12) & 0x3fu) << 20 | (code & 31u) << 26 | (ends ? 1u << 31 : 0u);
  w[2] = beta20(b12) | (a1 & 0xfffu) << 20;
  w[3] = entry | last << 16;
  w[4] = a2 | ((a1 >> 12) & 0x3fu) << 18 | ((code >> 5) & 7u) << 24 | signs << 27 | M << 30;
}

// Phase F's stride-table entry for T = w[4] >> 24 (k_bk_fuse_s reads one per refill): e[0..2] =
// (dM, d1, d2), the signed steps of the major and minor axes in units of the box strides bx, by,
// bz of +x, +y, +z (mod 2^32); e[3] = the offsets from L of the cells of L's slab that the slab
// code adopts: L - d_e in the low 16 bits (signed; s >= 1) and L - d1 - d2 in the high 16 bits
// (s == 2), 0 = none (needs |d1| + |d2| < 2^15).  Entries with M = 3 are never read.
__host__ __device__ inline void slab_table_entry(uint32_t T, uint32_t bx, uint32_t by, uint32_t bz, uint32_t e[4]) {
  const uint32_t s = T & 3u, ee = (T >> 2) & 1u, sg = (T >> 3) & 7u, M = T >> 6;
  const uint32_t sx = sg & 1u ? 0u - bx : bx, sy = sg & 2u ? 0u - by : by, sz = sg & 4u ? 0u - bz : bz;
  e[0] = M == 0 ? sx : (M == 1 ? sy : sz);
  e[1] = M == 0 ? sy : sx;
  e[2] = M == 2 ? sy : sz;
  const uint32_t o1 = s >= 1 ? 0u - (ee ? e[2] : e[1]) : 0u, o2 = s == 2 ? 0u - e[1] - e[2] : 0u;
  e[3] = (o1 & 0xffffu) | o2 << 16;
}

struct Slab20 {
  int32_t b1, b2, b12;  // beta state
  uint32_t aM, a1, a2;  // |dq| of the major / minor axes (the beta walk's K)
  uint32_t entry, last, code, signs, M;
  uint32_t S, s, e;     // the code's fields (slab_code)
  bool ends;
};

__host__ __device__ inline int32_t sext20(uint32_t w) { return (int32_t)(w << 12) >> 12; }

__host__ __device__ inline void unpack20(const uint32_t w[5], Slab20& s) {
  s.b1 = sext20(w[0]);
  s.b2 = sext20(w[1]);
  s.b12 = sext20(w[2]);
  s.aM = (w[0] >> 20) | ((w[1] >> 20) & 0x3fu) << 12;
  s.a1 = (w[2] >> 20) | ((w[4] >> 18) & 0x3fu) << 12;
  s.a2 = w[4] & 0x3ffffu;
  s.entry = w[3] & 0xffffu;
  s.last = w[3] >> 16;
  s.S = (w[1] >> 26) & 31u;
  s.s = (w[4] >> 24) & 3u;
  s.e = (w[4] >> 26) & 1u;
  s.code = s.S | s.s << 5 | s.e << 7;
  s.signs = (w[4] >> 27) & 7u;
  s.M = w[4] >> 30;
  s.ends = (w[1] >> 31) != 0;
}

}  // namespace brick
}  // namespace dmf
