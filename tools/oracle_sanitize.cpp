// ASan/UBSan driver for the CPU oracle (oracle/oracle.cpp, test infrastructure) and the
// host-side arithmetic the exactness claims rest on.  Built with
//   g++ -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -fopenmp
//       tools/oracle_sanitize.cpp oracle/oracle.cpp
// by tests/test_selftests.py: every oracle entry point runs once on a small synthetic scene
// (a sphere cloud with normals, a camera ring, synthetic depth frames) so that any
// out-of-bounds access, overflow or other undefined behaviour in the checker fails the
// CPU suite.  Prints "oracle sanitize ok" and the counts it saw.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

struct orc_volume;
struct orc_ogrid;
extern "C" {
orc_volume* orc_volume_new(void);
void orc_volume_free(orc_volume* v);
void orc_set_dimensions(orc_volume* v, double xmin, double xmax, double ymin, double ymax, double zmin, double zmax);
void orc_set_volume_size(orc_volume* v, int nx, int ny, int nz);
int orc_construct(orc_volume* v);
int64_t orc_integrate(orc_volume* v, const float* xyz, const float* normals, int64_t n);
int64_t orc_num_occupied(const orc_volume* v);
int64_t orc_occupied(const orc_volume* v, uint64_t* out, int64_t cap);
void orc_occupancy_dense(const orc_volume* v, uint8_t* out);
void orc_backproject(const float* K, int H, int W, const uint16_t* depth, const float* T, float* xyz);
int64_t orc_reverse_ray_trace_fast(orc_volume* vol, const float* K, int H, int W, const float* T, int viz,
                                   int dead_work, int* found_out, uint64_t* out, int64_t cap);
int64_t orc_reverse_ray_trace(orc_volume* vol, const float* K, int H, int W, const float* T, int viz, int* found_out,
                              uint64_t* out, int64_t cap);
void orc_ray_trace(orc_volume* vol, const float* K, int H, int W, const float* T, int zdelta, int sparse);
void orc_ray_trace_and_classify(orc_volume* vol, const float* K, int H, int W, const float* T, int zdelta, int view,
                                int sparse);
int64_t orc_ray_trace_and_get_good_points(orc_volume* vol, const float* K, int H, int W, const float* T, int zdelta,
                                          int sparse, int* found, uint64_t* out, int64_t cap);
int64_t orc_ray_trace_and_get_points(orc_volume* vol, const float* K, int H, int W, const float* T, int zdelta,
                                     int sparse, int* found, uint64_t* out, int64_t cap);
int orc_ray_trace_and_get_minimum(orc_volume* vol, const float* K, int H, int W, const float* T, int zdelta,
                                  int sparse);
void orc_forward_first_hits(orc_volume* vol, const float* K, int H, int W, const float* T, int zstart, int zdelta,
                            int rdelta, int cdelta, int32_t* k_out, uint64_t* hash_out);
void orc_ray_trace_volume(orc_volume* vol, const float* K, int H, int W, const float* T, int32_t* depth_out);
int orc_will_collide(orc_volume* vol, const float* a, const float* b);
void orc_collision_cost_map(orc_volume* vol, const float* poses, int V, int32_t* map);
void orc_fuse_depth(const orc_volume* vol, const float* K, int H, int W, const uint16_t* depth, const float* poses,
                    int P, int dmin, int dmax, int32_t* hits, int32_t* misses, int64_t* stats);
void orc_fuse_depth_mt(const orc_volume* vol, const float* K, int H, int W, const uint16_t* depth, const float* poses,
                       int P, int dmin, int dmax, int32_t* hits, int32_t* misses, int64_t* stats, int nthreads);
void orc_fuse_finalize(int64_t n, const int32_t* hits, const int32_t* misses, int l_hit, int l_miss, int l_min,
                       int l_max, int16_t* out);
int32_t orc_greedy_set_cover(const uint64_t* hashes, const int64_t* counts, int32_t nsets, int32_t min_gain,
                             int32_t* selected);
orc_ogrid* orc_ogrid_new();
void orc_ogrid_free(orc_ogrid* g);
void orc_ogrid_setup(orc_ogrid* g, const double* bounds, float xr, float yr, float zr, int k);
void orc_ogrid_dims(const orc_ogrid* g, int32_t* d);
void orc_ogrid_update(orc_ogrid* g, const float* cloud, int64_t n_cloud, const float* pn, int64_t n_nrm);
int64_t orc_ogrid_download(const orc_ogrid* g, int mode, float* out, int64_t cap);
int64_t orc_ogrid_download_reorganized(const orc_ogrid* g, int clean, float* out, int64_t cap);
}

static void look_at(float cx, float cy, float cz, float T[12]) {
  // camera z axis towards the origin, x/y completing a right-handed frame; T = [R | c]
  float z[3] = {-cx, -cy, -cz};
  const float nz = std::sqrt(z[0] * z[0] + z[1] * z[1] + z[2] * z[2]);
  for (float& e : z) e /= nz;
  float up[3] = {0.f, 0.f, 1.f};
  if (std::fabs(z[2]) > 0.9f) { up[0] = 1.f; up[2] = 0.f; }
  float x[3] = {up[1] * z[2] - up[2] * z[1], up[2] * z[0] - up[0] * z[2], up[0] * z[1] - up[1] * z[0]};
  const float nx = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  for (float& e : x) e /= nx;
  const float y[3] = {z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0]};
  const float c[3] = {cx, cy, cz};
  for (int r = 0; r < 3; ++r) {
    T[4 * r + 0] = x[r];
    T[4 * r + 1] = y[r];
    T[4 * r + 2] = z[r];
    T[4 * r + 3] = c[r];
  }
}

int main() {
  const int H = 48, W = 64, N = 40, P = 6;
  const float K[9] = {60.f, 0.f, 32.f, 0.f, 60.f, 24.f, 0.f, 0.f, 1.f};
  orc_volume* v = orc_volume_new();
  orc_set_dimensions(v, -0.5, 0.5, -0.5, 0.5, -0.5, 0.5);
  orc_set_volume_size(v, N, N, N);
  orc_construct(v);
  // sphere cloud (r = 0.2 m) with outward normals, plus points outside the volume
  std::vector<float> pts, nrm;
  for (int i = 0; i < 4000; ++i) {
    const float th = 0.0031f * (float)i * 7.f, ph = std::acos(1.f - 2.f * ((float)i + 0.5f) / 4000.f);
    const float d[3] = {std::sin(ph) * std::cos(th), std::sin(ph) * std::sin(th), std::cos(ph)};
    for (int a = 0; a < 3; ++a) {
      pts.push_back(0.2f * d[a]);
      nrm.push_back(d[a]);
    }
  }
  for (int a = 0; a < 3; ++a) { pts.push_back(0.7f); nrm.push_back(0.f); }
  const int64_t np = (int64_t)pts.size() / 3;
  orc_integrate(v, pts.data(), nrm.data(), np);
  const int64_t V = orc_num_occupied(v);
  std::vector<uint64_t> occ(V > 0 ? V : 1);
  orc_occupied(v, occ.data(), V);
  std::vector<uint8_t> dense((size_t)N * N * N);
  orc_occupancy_dense(v, dense.data());
  // camera ring at 0.45 m (inside the volume, as the reference's sphere path) and depth
  // frames: a plane 0.6 m ahead with a hole
  std::vector<float> poses(12 * P);
  for (int p = 0; p < P; ++p) {
    const float a = 6.2831853f * (float)p / (float)P;
    look_at(0.45f * std::cos(a), 0.45f * std::sin(a), 0.1f * (float)(p % 3 - 1), &poses[12 * p]);
  }
  std::vector<uint16_t> depth((size_t)P * H * W);
  for (size_t i = 0; i < depth.size(); ++i) depth[i] = (uint16_t)((i % 97) == 0 ? 0 : 300 + (i % 400));
  std::vector<float> xyz((size_t)H * W * 3);
  orc_backproject(K, H, W, depth.data(), &poses[0], xyz.data());
  std::vector<uint64_t> lst(V + 16);
  int found = 0;
  int64_t ng = 0;
  for (int p = 0; p < P; ++p) {
    const float* T = &poses[12 * p];
    ng += orc_reverse_ray_trace_fast(v, K, H, W, T, 1, 1, &found, lst.data(), V + 16);
    ng += orc_reverse_ray_trace(v, K, H, W, T, 1, &found, lst.data(), V + 16);
    orc_ray_trace(v, K, H, W, T, 10, p & 1);
    orc_ray_trace_and_classify(v, K, H, W, T, 10, 1, p & 1);
    ng += orc_ray_trace_and_get_good_points(v, K, H, W, T, 10, p & 1, &found, lst.data(), V + 16);
    ng += orc_ray_trace_and_get_points(v, K, H, W, T, 10, p & 1, &found, lst.data(), V + 16);
    ng += orc_ray_trace_and_get_minimum(v, K, H, W, T, 10, p & 1);
  }
  std::vector<int32_t> kk((size_t)H * W);
  std::vector<uint64_t> hh((size_t)H * W);
  orc_forward_first_hits(v, K, H, W, &poses[0], 10, 10, 1, 1, kk.data(), hh.data());
  std::vector<int32_t> zb((size_t)H * W);
  orc_ray_trace_volume(v, K, H, W, &poses[0], zb.data());
  const float a0[3] = {-0.45f, 0.f, 0.f}, a1[3] = {0.45f, 0.01f, 0.02f};
  const int col = orc_will_collide(v, a0, a1);
  std::vector<int32_t> cmap((size_t)P * P);
  orc_collision_cost_map(v, poses.data(), P, cmap.data());
  // fusion (single-threaded and OpenMP) and finalize
  const size_t nc = (size_t)N * N * N;
  std::vector<int32_t> h1(nc), m1(nc), h2(nc), m2(nc);
  int64_t s1[3] = {0, 0, 0}, s2[3] = {0, 0, 0};
  orc_fuse_depth(v, K, H, W, depth.data(), poses.data(), P, 200, 1000, h1.data(), m1.data(), s1);
  orc_fuse_depth_mt(v, K, H, W, depth.data(), poses.data(), P, 200, 1000, h2.data(), m2.data(), s2, 4);
  std::vector<int16_t> lo(nc);
  orc_fuse_finalize((int64_t)nc, h1.data(), m1.data(), 847, -405, -2000, 3511, lo.data());
  if (s1[0] != s2[0] || h1 != h2 || m1 != m2) {
    printf("oracle sanitize: single-threaded and OpenMP fusion differ\n");
    return 1;
  }
  // set cover over per-pose good lists (two synthetic sets)
  std::vector<uint64_t> sets = {1, 2, 3, 4, 5, 6, 7, 3, 4, 5, 6, 7, 8, 9, 10, 11};
  const int64_t counts[2] = {7, 9};
  int32_t sel[2];
  const int32_t nsel = orc_greedy_set_cover(sets.data(), counts, 2, 1, sel);
  // OccupancyGrid: update with K = 1 and the downloads (plain, HQ, reorganized)
  orc_ogrid* g = orc_ogrid_new();
  const double b[6] = {-0.5, 0.5, -0.5, 0.5, -0.5, 0.5};
  orc_ogrid_setup(g, b, 0.05f, 0.05f, 0.05f, 1);
  int32_t gd[3];
  orc_ogrid_dims(g, gd);
  std::vector<float> pn;  // updateStates' normals cloud: (x, y, z, nx, ny, nz) per entry
  for (int64_t i = 0; i < np; ++i)
    for (int a = 0; a < 6; ++a) pn.push_back(a < 3 ? pts[3 * i + a] : nrm[3 * i + a - 3]);
  orc_ogrid_update(g, pts.data(), np, pn.data(), np);
  std::vector<float> dl(3 * (size_t)gd[0] * gd[1] * gd[2] + 3);
  const int64_t cap = (int64_t)dl.size() / 3;
  int64_t nd = 0;
  for (int mode = 0; mode < 2; ++mode) nd += orc_ogrid_download(g, mode, dl.data(), cap);
  for (int clean = 0; clean < 2; ++clean) nd += orc_ogrid_download_reorganized(g, clean, dl.data(), cap);
  orc_ogrid_free(g);
  orc_volume_free(v);
  printf("oracle sanitize ok: %lld voxels, %lld list entries, collide %d, %lld updates, %d selected, %lld downloads\n",
         (long long)V, (long long)ng, col, (long long)s1[0], nsel, (long long)nd);
  return 0;
}
