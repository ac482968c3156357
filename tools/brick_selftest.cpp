// CPU self-test of the exact brick decomposition (csrc/dmf_brick.hpp) against the
// plain fine walk of oracle.cpp dda_ray (64-bit crossing times, ties x < y < z).
// For random and adversarial fixed-point rays on grids that are and are not
// multiples of 32 cells it checks that
//   1. the coarse walk lists exactly the bricks the fine walk passes through, in order;
//   2. for every such brick, pair_in_brick's entry counts, cell count and end flag
//      restart the int32 fine walk (E = E0 + c_a K_b - c_b K_a) on exactly the cells
//      the fine walk visits there;
//   3. phase F's major-axis slab walk (slab_walk) restarted from the same counts visits
//      the same cells in the same order;
//   4. the slab walk bounded by the pair's ownership code (slab_rcode: R = 3 S + s) visits
//      exactly the pair's cells before its last cell, and R fits 7 bits; so does phase F's
//      walk from the slab code (slab_code: S whole slabs, then L's slab before L derived from
//      L, slab_walk_code), with S <= 31;
//   5. the slab-code walk from the 20-byte record (pack20 -> unpack20, scaled state beta), and
//      phase F's stride-table entry for it (slab_table_entry: strides and adopted cells);
//   6. pass B's select-based counts_at_sel equals counts_at at the ray's crossing events;
//   7. so does the double-arithmetic counts_at_f64 (also with its reciprocals 2 ulps and a
//      relative 2^-22 / 2^-14 off);
//   8. pass B's replay of pass A's recorded crossing path (path_put / path_axis, the first
//      kPathSteps boundaries; coarse_total = the walk's step count) lists the same bricks,
//      and so does its replay past them by the stateless coarse_next_at (also over whole rays),
//      and by the incremental per-axis boundary indices pass B carries (check 8c).
// Build: make -C depth-map-fusion-utils_amd build/brick_selftest ; run: <exe> [rays] [seed]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "dmf_brick.hpp"

using namespace dmf::brick;

struct Cell {
  int x, y, z;
  bool operator==(const Cell& o) const { return x == o.x && y == o.y && z == o.z; }
};

// oracle.cpp dda_ray lines 781-818, from quantised endpoints
static void fine_walk(const int64_t qs[3], const int64_t qe[3], std::vector<Cell>& out) {
  int64_t cs[3], ce[3], adq[3], step[3];
  for (int a = 0; a < 3; ++a) {
    cs[a] = qs[a] / kQ;
    ce[a] = qe[a] / kQ;
    const int64_t dq = qe[a] - qs[a];
    adq[a] = dq < 0 ? -dq : dq;
    step[a] = ce[a] > cs[a] ? 1 : (ce[a] < cs[a] ? -1 : 0);
  }
  uint64_t Tm[3], In[3];
  for (int a = 0; a < 3; ++a) {
    if (step[a] == 0) { Tm[a] = UINT64_MAX; In[a] = 0; continue; }
    uint64_t M = 1;
    for (int b = 0; b < 3; ++b)
      if (b != a && adq[b] > 0) M *= (uint64_t)adq[b];
    const int64_t h = step[a] > 0 ? 2 * ((cs[a] + 1) * kQ - qs[a]) : 2 * (qs[a] - cs[a] * kQ) + 1;
    Tm[a] = (uint64_t)h * M;
    In[a] = (uint64_t)(2 * kQ) * M;
  }
  int64_t nsteps = 0;
  for (int a = 0; a < 3; ++a) nsteps += ce[a] > cs[a] ? ce[a] - cs[a] : cs[a] - ce[a];
  int64_t cur[3] = {cs[0], cs[1], cs[2]};
  out.clear();
  for (int64_t s = 0; s < nsteps; ++s) {
    out.push_back({(int)cur[0], (int)cur[1], (int)cur[2]});
    int a = 0;
    if (Tm[1] < Tm[a]) a = 1;
    if (Tm[2] < Tm[a]) a = 2;
    cur[a] += step[a];
    Tm[a] += In[a];
  }
  out.push_back({(int)cur[0], (int)cur[1], (int)cur[2]});
}

// The kernels' int32 walk (dmf_fuse.hip dda_select) restarted from crossing counts c.
static void restart_walk(const QRay& r, const int32_t c[3], int cells, std::vector<Cell>& out) {
  const uint32_t K[3] = {(uint32_t)(2 * kQ * r.adq[0]), (uint32_t)(2 * kQ * r.adq[1]), (uint32_t)(2 * kQ * r.adq[2])};
  int32_t E01 = (int32_t)((uint32_t)e0_pair(r, 0, 1) + (uint32_t)c[0] * K[1] - (uint32_t)c[1] * K[0]);
  int32_t E02 = (int32_t)((uint32_t)e0_pair(r, 0, 2) + (uint32_t)c[0] * K[2] - (uint32_t)c[2] * K[0]);
  int32_t E12 = (int32_t)((uint32_t)e0_pair(r, 1, 2) + (uint32_t)c[1] * K[2] - (uint32_t)c[2] * K[1]);
  int x = r.cs[0] + r.st[0] * c[0], y = r.cs[1] + r.st[1] * c[1], z = r.cs[2] + r.st[2] * c[2];
  out.clear();
  for (int k = 0; k < cells; ++k) {
    out.push_back({x, y, z});
    const bool b10 = E01 > 0;
    const bool s2 = (b10 ? E12 : E02) > 0;
    const bool s1 = !s2 && b10, s0 = !s2 && !b10;
    E01 = (int32_t)((uint32_t)E01 + (s0 ? K[1] : (s1 ? (uint32_t)-K[0] : 0u)));
    E02 = (int32_t)((uint32_t)E02 + (s0 ? K[2] : (s2 ? (uint32_t)-K[0] : 0u)));
    E12 = (int32_t)((uint32_t)E12 + (s1 ? K[2] : (s2 ? (uint32_t)-K[1] : 0u)));
    x += s0 ? r.st[0] : 0;
    y += s1 ? r.st[1] : 0;
    z += s2 ? r.st[2] : 0;
  }
}

// Phase F's slab walk (dmf_brick.hpp slab_walk) restarted from the same crossing counts.
static void restart_slab(const QRay& r, const int32_t c[3], int cells, std::vector<Cell>& out) {
  const uint32_t K[3] = {(uint32_t)(2 * kQ * r.adq[0]), (uint32_t)(2 * kQ * r.adq[1]), (uint32_t)(2 * kQ * r.adq[2])};
  const int32_t E01 = (int32_t)((uint32_t)e0_pair(r, 0, 1) + (uint32_t)c[0] * K[1] - (uint32_t)c[1] * K[0]);
  const int32_t E02 = (int32_t)((uint32_t)e0_pair(r, 0, 2) + (uint32_t)c[0] * K[2] - (uint32_t)c[2] * K[0]);
  const int32_t E12 = (int32_t)((uint32_t)e0_pair(r, 1, 2) + (uint32_t)c[1] * K[2] - (uint32_t)c[2] * K[1]);
  const int M = major_axis(r), m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  int32_t b1, b2, b12;
  slab_from_pairwise(M, E01, E02, E12, b1, b2, b12);
  const int32_t p0[3] = {r.cs[0] + r.st[0] * c[0], r.cs[1] + r.st[1] * c[1], r.cs[2] + r.st[2] * c[2]};
  out.clear();
  slab_walk(M, b1, b2, b12, K[M], K[m1], K[m2], r.st, p0, cells, [&](int x, int y, int z) { out.push_back({x, y, z}); });
}

// Check 4: slab_walk_owned from the pair's entry counts, bounded by slab_rcode; or (code) the
// slab-code walk of phase F (slab_code, slab_walk_code from the last cell's coordinates Lc).
static void restart_owned(const QRay& r, const int32_t c[3], const int32_t cL[3], uint32_t& R,
                          std::vector<Cell>& out, const int32_t* Lc = nullptr) {
  const uint32_t K[3] = {(uint32_t)(2 * kQ * r.adq[0]), (uint32_t)(2 * kQ * r.adq[1]), (uint32_t)(2 * kQ * r.adq[2])};
  const int M = major_axis(r), m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  int32_t s1, s2, s12;  // slab state at the ray's start (counts 0), as pass B keeps it
  slab_from_pairwise(M, e0_pair(r, 0, 1), e0_pair(r, 0, 2), e0_pair(r, 1, 2), s1, s2, s12);
  R = Lc ? slab_code(M, s1, s2, s12, K[M], K[m1], K[m2], c, cL) : slab_rcode(M, s1, s2, K[M], K[m1], K[m2], c, cL);
  const int32_t E01 = (int32_t)((uint32_t)e0_pair(r, 0, 1) + (uint32_t)c[0] * K[1] - (uint32_t)c[1] * K[0]);
  const int32_t E02 = (int32_t)((uint32_t)e0_pair(r, 0, 2) + (uint32_t)c[0] * K[2] - (uint32_t)c[2] * K[0]);
  const int32_t E12 = (int32_t)((uint32_t)e0_pair(r, 1, 2) + (uint32_t)c[1] * K[2] - (uint32_t)c[2] * K[1]);
  int32_t b1, b2, b12;
  slab_from_pairwise(M, E01, E02, E12, b1, b2, b12);
  const int32_t p0[3] = {r.cs[0] + r.st[0] * c[0], r.cs[1] + r.st[1] * c[1], r.cs[2] + r.st[2] * c[2]};
  out.clear();
  if (Lc)
    slab_walk_code(M, b1, b2, b12, K[M], K[m1], K[m2], r.st, p0, R, Lc,
                   [&](int x, int y, int z) { out.push_back({x, y, z}); });
  else
    slab_walk_owned(M, b1, b2, b12, K[M], K[m1], K[m2], r.st, p0, (int)R,
                    [&](int x, int y, int z) { out.push_back({x, y, z}); });
}

// Check 5: the same walk from the 20-byte pair record (pack20 / unpack20): scaled state
// beta = b >> 9 with increments |dq| instead of K = 512 |dq|.
static void restart_owned20(const QRay& r, const int32_t c[3], const int32_t cL[3], const int32_t Lc[3], bool ends,
                            std::vector<Cell>& out) {
  const uint32_t K[3] = {(uint32_t)(2 * kQ * r.adq[0]), (uint32_t)(2 * kQ * r.adq[1]), (uint32_t)(2 * kQ * r.adq[2])};
  const int M = major_axis(r), m1 = M == 0 ? 1 : 0, m2 = M == 2 ? 1 : 2;
  int32_t s1, s2, s12;
  slab_from_pairwise(M, e0_pair(r, 0, 1), e0_pair(r, 0, 2), e0_pair(r, 1, 2), s1, s2, s12);
  const uint32_t R = slab_code(M, s1, s2, s12, K[M], K[m1], K[m2], c, cL);
  int32_t b1, b2, b12;
  slab_from_pairwise(M, (int32_t)((uint32_t)e0_pair(r, 0, 1) + (uint32_t)c[0] * K[1] - (uint32_t)c[1] * K[0]),
                     (int32_t)((uint32_t)e0_pair(r, 0, 2) + (uint32_t)c[0] * K[2] - (uint32_t)c[2] * K[0]),
                     (int32_t)((uint32_t)e0_pair(r, 1, 2) + (uint32_t)c[1] * K[2] - (uint32_t)c[2] * K[1]), b1, b2,
                     b12);
  const uint32_t signs = (r.st[0] < 0 ? 1u : 0u) | (r.st[1] < 0 ? 2u : 0u) | (r.st[2] < 0 ? 4u : 0u);
  uint32_t w[5];
  pack20(b1, b2, b12, (uint32_t)r.adq[M], (uint32_t)r.adq[m1], (uint32_t)r.adq[m2], 12345u, 54321u, R, signs,
         (uint32_t)M, ends, w);
  Slab20 s;
  unpack20(w, s);
  out.clear();
  if (s.aM != (uint32_t)r.adq[M] || s.a1 != (uint32_t)r.adq[m1] || s.a2 != (uint32_t)r.adq[m2] || s.code != R ||
      s.S != (R & 31u) || s.s != ((R >> 5) & 3u) || s.e != (R >> 7) ||
      s.signs != signs || s.M != (uint32_t)M || s.ends != ends || s.entry != 12345u || s.last != 54321u) {
    out.push_back({-1, -1, -1});  // a field did not round-trip
    return;
  }
  const int32_t st[3] = {s.signs & 1u ? -1 : 1, s.signs & 2u ? -1 : 1, s.signs & 4u ? -1 : 1};
  const int32_t p0[3] = {r.cs[0] + r.st[0] * c[0], r.cs[1] + r.st[1] * c[1], r.cs[2] + r.st[2] * c[2]};
  // a non-moving axis has sign bit 0 (+1) but never steps (its b stays negative / b12 never flips it)
  const int32_t stw[3] = {r.st[0] ? st[0] : 0, r.st[1] ? st[1] : 0, r.st[2] ? st[2] : 0};
  slab_walk_code((int)s.M, s.b1, s.b2, s.b12, s.aM, s.a1, s.a2, stw, p0, s.code, Lc,
                 [&](int x, int y, int z) { out.push_back({x, y, z}); });
  // phase F adopts L's slab through its stride table (slab_table_entry at T = w[4] >> 24, in
  // the LDS box's byte strides): the offsets must land on the cells slab_walk_code adopted
  uint32_t te[4];
  const int64_t bx = 4 * 1057, by = 4 * 33, bz = 4;
  slab_table_entry(w[4] >> 24, (uint32_t)bx, (uint32_t)by, (uint32_t)bz, te);
  auto lin = [&](int64_t x, int64_t y, int64_t z) { return x * bx + y * by + z * bz; };
  const int64_t L = lin(Lc[0], Lc[1], Lc[2]);
  const int64_t sb[3] = {bx, by, bz};
  const int64_t o1 = (int16_t)(te[3] & 0xffffu), o2 = (int16_t)(te[3] >> 16);
  const int64_t want1 = s.s >= 1 ? -st[s.e ? m2 : m1] * sb[s.e ? m2 : m1] : 0;
  const int64_t want2 = s.s == 2 ? -st[m1] * sb[m1] - st[m2] * sb[m2] : 0;
  const int64_t dM = (int32_t)te[0], d1 = (int32_t)te[1], d2 = (int32_t)te[2];
  if (o1 != want1 || o2 != want2 || dM != st[s.M] * sb[s.M] || d1 != st[m1] * sb[m1] || d2 != st[m2] * sb[m2] ||
      (L + o1 == L) != (s.s == 0))
    out.push_back({-2, -2, -2});  // the table disagrees with the record's adoption
}

int main(int argc, char** argv) {
  const long nrays = argc > 1 ? atol(argv[1]) : 200000;
  const unsigned seed = argc > 2 ? (unsigned)atol(argv[2]) : 1234u;
  std::mt19937_64 rng(seed);
  auto U = [&](int64_t lo, int64_t hi) { return lo + (int64_t)(rng() % (uint64_t)(hi - lo + 1)); };
  const int grids[][3] = {{64, 64, 64}, {96, 40, 33}, {128, 128, 128}, {200, 31, 77}, {512, 512, 512},
                          {37, 300, 65}, {1024, 1024, 1024}, {1, 90, 5}};
  std::vector<Cell> fine, seg;
  long checked = 0, pairs = 0, bad = 0, events = 0, paths_replayed = 0, long_replayed = 0;
  for (long i = 0; i < nrays && bad < 10; ++i) {
    const int* ng = grids[i % 8];
    int64_t qs[3], qe[3];
    const int mode = (int)(i % 7);
    for (int a = 0; a < 3; ++a) {
      const int64_t span = (int64_t)ng[a] * kQ - 1;
      qs[a] = U(0, span);
      qe[a] = U(0, span);
    }
    if (mode == 1) {  // shared fractions: exact ties between axes
      const int64_t f = U(0, kQ - 1);
      for (int a = 0; a < 3; ++a) { qs[a] = qs[a] / kQ * kQ + f; qe[a] = qe[a] / kQ * kQ + f; }
    } else if (mode == 2) {  // equal |dq| on two or three axes (exact diagonals)
      const int64_t d = U(1, 40 * kQ);
      for (int a = 0; a < 3; ++a) {
        const int64_t span = (int64_t)ng[a] * kQ - 1;
        qs[a] = U(0, span);
        qe[a] = qs[a] + ((a + i) % 2 ? d : -d);
        if (qe[a] < 0 || qe[a] > span) qe[a] = qs[a];
      }
    } else if (mode == 3) {  // axis-aligned / planar rays
      const int a = (int)(i / 7 % 3);
      for (int b = 0; b < 3; ++b)
        if (b != a && (i / 21) % 2) qe[b] = qs[b];
      qe[(a + 1) % 3] = qs[(a + 1) % 3];
    } else if (mode == 4) {  // endpoints on brick boundaries and cell corners
      for (int a = 0; a < 3; ++a) {
        const int64_t nb = (ng[a] + kB - 1) / kB;
        qs[a] = std::min<int64_t>(U(0, nb) * kB * kQ, (int64_t)ng[a] * kQ - 1);
        qe[a] = std::min<int64_t>(U(0, nb) * kB * kQ + U(-1, 0) * kQ, (int64_t)ng[a] * kQ - 1);
        if (qe[a] < 0) qe[a] = 0;
      }
    } else if (mode == 5) {  // short rays inside one or two bricks
      for (int a = 0; a < 3; ++a) {
        const int64_t span = (int64_t)ng[a] * kQ - 1;
        qe[a] = std::max<int64_t>(0, std::min<int64_t>(span, qs[a] + U(-40 * kQ, 40 * kQ)));
      }
    }
    const bool end_inside = (rng() & 1) != 0;
    uint64_t A, B;
    pack_ray(qs, qe, end_inside, A, B);
    QRay r;
    decode_ray(A, B, r);
    fine_walk(qs, qe, fine);
    if ((int)fine.size() != r.nsteps + 1) { printf("nsteps mismatch\n"); ++bad; continue; }
    // 1. brick sequence
    std::vector<int> fb;  // brick ids of fine cells, consecutive duplicates removed
    const int nbx = (ng[0] + kB - 1) / kB, nby = (ng[1] + kB - 1) / kB, nbz = (ng[2] + kB - 1) / kB;
    auto bid = [&](const Cell& c) { return ((c.x >> kLog) * nby + (c.y >> kLog)) * nbz + (c.z >> kLog); };
    for (const Cell& c : fine)
      if (fb.empty() || fb.back() != bid(c)) fb.push_back(bid(c));
    Coarse w;
    coarse_init(r, w);
    std::vector<int> cb;
    int bx = r.cs[0] >> kLog, by = r.cs[1] >> kLog, bz = r.cs[2] >> kLog;
    cb.push_back((bx * nby + by) * nbz + bz);
    for (int s = 0; s < w.total; ++s) {
      const int a = coarse_next(w);
      if (a == 0) bx += r.st[0];
      if (a == 1) by += r.st[1];
      if (a == 2) bz += r.st[2];
      cb.push_back((bx * nby + by) * nbz + bz);
    }
    if (cb != fb) {
      printf("ray %ld: coarse bricks differ (%zu vs %zu)\n", i, cb.size(), fb.size());
      ++bad;
      continue;
    }
    // 8. the recorded crossing path replays the same bricks
    {
      Coarse w2;
      coarse_init(r, w2);
      uint64_t path = 0;
      for (int s = 0; s < w2.total; ++s) path = path_put(path, s, coarse_next(w2));
      bool okp = coarse_total(r) == w2.total;
      if (okp && w2.total <= kPathSteps) {
        std::vector<int> rb;
        int px = r.cs[0] >> kLog, py = r.cs[1] >> kLog, pz = r.cs[2] >> kLog;
        rb.push_back((px * nby + py) * nbz + pz);
        for (int s = 0; s < w2.total; ++s) {
          const int a = path_axis(path, s);
          if (a == 0) px += r.st[0];
          if (a == 1) py += r.st[1];
          if (a == 2) pz += r.st[2];
          rb.push_back((px * nby + py) * nbz + pz);
        }
        okp = rb == cb;
        ++paths_replayed;
      }
      if (!okp) { printf("ray %ld: path replay differs (%d boundaries)\n", i, w2.total); ++bad; continue; }
      // 8b. pass B's replay of every ray: the path's axes, then coarse_next_at from the
      //     current brick past kPathSteps boundaries (and from the start, for a check of it
      //     over the whole ray)
      for (int from = 0; from < 2 && okp; ++from) {
        std::vector<int> rb;
        int px = r.cs[0] >> kLog, py = r.cs[1] >> kLog, pz = r.cs[2] >> kLog;
        rb.push_back((px * nby + py) * nbz + pz);
        const int lim = from == 0 ? kPathSteps : 0;
        for (int s = 0; s < w2.total; ++s) {
          const int a = s < lim ? path_axis(path, s) : coarse_next_at(r, px, py, pz);
          if (a == 0) px += r.st[0];
          if (a == 1) py += r.st[1];
          if (a == 2) pz += r.st[2];
          rb.push_back((px * nby + py) * nbz + pz);
        }
        okp = rb == cb;
        if (w2.total > kPathSteps && from == 0) ++long_replayed;
      }
      if (!okp) { printf("ray %ld: stateless replay differs (%d boundaries)\n", i, w2.total); ++bad; continue; }
      // 8c. pass B's replay as k_bk_pairs runs it: per axis the crossing index of the boundary
      //     into the next brick (next_boundary_k, +kB per step along it), the next axis past
      //     the path from those (coarse_next_k), the brick index moved by a per-axis step; the
      //     bricks and every event's crossing index equal the coordinate-based ones
      {
        std::vector<int> rb;
        const int c0 = r.cs[0] >> kLog, c1 = r.cs[1] >> kLog, c2 = r.cs[2] >> kLog;
        int32_t P[3] = {next_boundary_k(r, 0, c0), next_boundary_k(r, 1, c1), next_boundary_k(r, 2, c2)};
        const int D[3] = {r.st[0] * nby * nbz, r.st[1] * nbz, r.st[2]};
        int b = (c0 * nby + c1) * nbz + c2, pc[3] = {c0, c1, c2};
        rb.push_back(b);
        for (int s = 0; s < w2.total && okp; ++s) {
          const int a = s < kPathSteps ? path_axis(path, s) : coarse_next_k(r, P[0], P[1], P[2]);
          b += D[a];
          const int32_t k = P[a];
          P[a] += kB;
          pc[a] += r.st[a];
          const int32_t kc = r.st[a] > 0 ? (pc[a] << kLog) - r.cs[a] - 1 : r.cs[a] - (pc[a] << kLog) - kB;
          okp = k == kc;
          rb.push_back(b);
        }
        okp = okp && rb == cb;
      }
      if (!okp) { printf("ray %ld: incremental replay differs (%d boundaries)\n", i, w2.total); ++bad; continue; }
    }
    // 6. pass B's select-based counts_at_sel equals counts_at at every crossing event
    //    (every k for short axes, 97 spread k's for long ones)
    {
      bool okc = true;
      for (int a = 0; a < 3 && okc; ++a) {
        if (r.st[a] == 0) continue;
        const int32_t stride = r.n[a] > 97 ? r.n[a] / 97 : 1;
        for (int32_t k = 0; k < r.n[a] && okc; k += stride) {
          int32_t c0[3], c1[3], c2[3];
          counts_at(r, a, k, c0);
          counts_at_sel(r, a, k, c1);
          QRayF64 fd;
          qray_f64(r, fd);
          if (a == 0) counts_at_f64<0>(r, fd, k, c2);
          else if (a == 1) counts_at_f64<1>(r, fd, k, c2);
          else counts_at_f64<2>(r, fd, k, c2);
          okc = c0[0] == c1[0] && c0[1] == c1[1] && c0[2] == c1[2] && c0[0] == c2[0] && c0[1] == c2[1] &&
                c0[2] == c2[2];
          // 7b. the same with the reciprocals off either way, by 2 ulps and by a relative error
          //     of 2^-22 (v_rcp_f64's documented precision is 2^29 ulps of a double, i.e. a
          //     relative error near 2^-23) and of 2^-14 (the margin: the +-1 remainder step
          //     holds while X / Y * eps < 1, X / Y < 2^12)
          for (int pert = 0; pert < 6 && okc; ++pert) {
            const int dir = pert & 1 ? 1 : -1;
            QRayF64 fp = fd;
            for (int b = 0; b < 3; ++b) {
              if (fp.inv[b] == 0.0) continue;
              if (pert < 2) {
                for (int u = 0; u < 2; ++u) fp.inv[b] = std::nextafter(fp.inv[b], dir < 0 ? 0.0 : 1.0);
              } else {
                fp.inv[b] *= 1.0 + dir * std::ldexp(1.0, pert < 4 ? -22 : -14);
              }
            }
            int32_t c3[3];
            if (a == 0) counts_at_f64<0>(r, fp, k, c3);
            else if (a == 1) counts_at_f64<1>(r, fp, k, c3);
            else counts_at_f64<2>(r, fp, k, c3);
            okc = c0[0] == c3[0] && c0[1] == c3[1] && c0[2] == c3[2];
            if (!okc) printf("ray %ld: counts_at_f64 with perturbed inv (%d) (%d, %d) differs\n", i, pert, a, k);
          }
          if (!okc) printf("ray %ld: counts_at_sel / _f64(%d, %d) = %d %d %d / %d %d %d vs %d %d %d\n", i, a, k, c1[0],
                           c1[1], c1[2], c2[0], c2[1], c2[2], c0[0], c0[1], c0[2]);
          ++events;
        }
      }
      if (!okc) { ++bad; continue; }
    }
    // 2. per-brick restart
    size_t pos = 0;
    for (int b : cb) {
      const int32_t bb[3] = {b / (nby * nbz), (b / nbz) % nby, b % nbz};
      Pair p;
      pair_in_brick(r, bb, ng, p);
      restart_walk(r, p.cin, p.cells, seg);
      size_t len = 0;
      while (pos + len < fine.size() && bid(fine[pos + len]) == b) ++len;
      bool ok = p.cells == (int)len && p.ends == (pos + len == fine.size());
      for (size_t k = 0; ok && k < len; ++k) ok = seg[k] == fine[pos + k];
      restart_slab(r, p.cin, p.cells, seg);
      ok = ok && seg.size() == len;
      for (size_t k = 0; ok && k < len; ++k) ok = seg[k] == fine[pos + k];
      if (ok) {  // 4. the ownership-bounded slab walk: the cells before the last one
        const Cell& Lc = fine[pos + len - 1];
        const int32_t cL[3] = {(Lc.x - r.cs[0]) * r.st[0], (Lc.y - r.cs[1]) * r.st[1], (Lc.z - r.cs[2]) * r.st[2]};
        uint32_t R = 0;
        restart_owned(r, p.cin, cL, R, seg);
        ok = R < 128 && seg.size() == len - 1;
        for (size_t k = 0; ok && k + 1 < len; ++k) ok = seg[k] == fine[pos + k];
        if (!ok) printf("ownership code %u: %zu cells vs %zu\n", R, seg.size(), len - 1);
        const int32_t Lxyz[3] = {Lc.x, Lc.y, Lc.z};
        if (ok) {  // 4b. phase F's slab-code walk
          uint32_t code = 0;
          restart_owned(r, p.cin, cL, code, seg, Lxyz);
          const int Mx = major_axis(r);
          const int32_t Sx = pick3(cL[0], cL[1], cL[2], Mx) - pick3(p.cin[0], p.cin[1], p.cin[2], Mx);
          ok = code < 256 && Sx >= 0 && Sx <= 31 && (code & 31u) == (uint32_t)Sx && ((code >> 5) & 3u) <= 2u &&
               seg.size() == len - 1;
          for (size_t k = 0; ok && k + 1 < len; ++k) ok = seg[k] == fine[pos + k];
          if (!ok) printf("slab code %u: %zu cells vs %zu\n", code, seg.size(), len - 1);
        }
        if (ok) {  // 5. the same from the 20-byte record (beta state)
          restart_owned20(r, p.cin, cL, Lxyz, p.ends && end_inside, seg);
          ok = seg.size() == len - 1;
          for (size_t k = 0; ok && k + 1 < len; ++k) ok = seg[k] == fine[pos + k];
          if (!ok) printf("20-byte record walk: %zu cells vs %zu\n", seg.size(), len - 1);
        }
      }
      if (!ok) {
        printf("ray %ld (mode %d) brick %d: cells %d vs %zu, ends %d\n", i, mode, b, p.cells, len, (int)p.ends);
        ++bad;
        break;
      }
      pos += len;
      ++pairs;
    }
    ++checked;
  }
  printf("brick selftest: %ld rays, %ld (ray, brick) pairs, %ld crossing events, %ld paths replayed (%ld past the "
         "path), %ld failures\n",
         checked, pairs, events, paths_replayed, long_replayed, bad);
  return bad ? 1 : 0;
}
