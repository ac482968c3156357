// =============================================================================
// oracle/oracle.cpp — CPU restatement of the reference hot path.
//
// TEST INFRASTRUCTURE ONLY.  Nothing in the product (libdmf.so, compat/, dmf_amd)
// links, loads or calls this file.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
//
// PARITY UNPINNED: the reference (REXJJ/depth-map-fusion-utils) ships no golden
// vectors, fixtures or assertions for this path, and it cannot be
// built here (Eigen3/PCL/OpenCV/Boost/octomap/nlopt absent).  This
// restatement follows the reference source line by line (file:line cited at every
// function) with the evaluation-order spec of DESIGN.md §3; a second, independent
// pure-Python restatement (oracle/py_oracle.py) cross-checks it on small cases.
//
// Data layout is the REFERENCE layout on purpose (vector<vector<vector<Voxel*>>>
// with per-voxel point/normal vectors, Volume.hpp:29-61) so that timing it is an
// honest CPU baseline.  Built with -O3 -ffp-contract=off (no FMA contraction; the
// reference is x86-64 SSE2 -O3 which emits no FMAs either).
//
// The 3D-DDA log-odds fusion (orc_fuse_*) is NOT in the reference:
// its semantics are this repository's own spec, anchored to the
// reference only through projectPoint/transformPoints (Camera.hpp:24-45) and the
// integratePointCloud binning (Volume.hpp:199-228) of the ray endpoint.
// =============================================================================
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <iterator>
#include <unordered_set>
#include <vector>

namespace {

struct Pt { float x, y, z; };
struct Nrm { float n[3]; };

// Volume.hpp:29-48  struct Voxel {pts, normals, view, good}
struct Voxel {
  std::vector<Pt> pts;
  std::vector<Nrm> normals;
  int view = 0;
  bool good = false;
};

// Eigen::Affine3f restricted to the 3x4 part (row 3 is 0 0 0 1).
struct Aff { float m[3][4]; };

// Eigen 3.3/3.4 fixed-size-3 reduction (redux_novec_unroller, HalfLength split):
// sum(a0,a1,a2) = a0 + (a1 + a2).  Used by Transform*Vector3f (lazy coeff-based
// product), dot(), squaredNorm() and the 3x3 cofactor determinant.
static inline float sum3(float a0, float a1, float a2) { return a0 + (a1 + a2); }

static inline Aff load_aff(const float* T) {
  Aff a;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) a.m[i][j] = T[i * 4 + j];
  return a;
}

// Camera.hpp:39-45  transformPoints: p1 << x,y,z (double->float); p2 = T*p1.
// Eigen Transform*Vector (Affine): res = translation; res += linear*p.
static inline void xform(const Aff& T, float x, float y, float z, float out[3]) {
  for (int i = 0; i < 3; ++i)
    out[i] = T.m[i][3] + sum3(T.m[i][0] * x, T.m[i][1] * y, T.m[i][2] * z);
}

// Eigen Transform::inverse() with Mode=Affine: linear().inverse() (InverseImpl.h
// compute_inverse<3>: cofactors of column 0, det, invdet = 1/det, adjugate*invdet),
// translation = -(Rinv * t).  Called at RayTracingEngine.hpp:49,140,317,383,506.
static Aff inverse_aff(const Aff& T) {
  auto m = [&](int i, int j) { return T.m[i][j]; };
  auto cof = [&](int i, int j) -> float {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m(i1, j1) * m(i2, j2) - m(i1, j2) * m(i2, j1);
  };
  const float c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
  const float det = sum3(c0 * m(0, 0), c1 * m(1, 0), c2 * m(2, 0));
  const float invdet = 1.0f / det;
  Aff r;
  r.m[0][0] = c0 * invdet; r.m[0][1] = c1 * invdet; r.m[0][2] = c2 * invdet;
  r.m[1][0] = cof(0, 1) * invdet; r.m[1][1] = cof(1, 1) * invdet; r.m[1][2] = cof(2, 1) * invdet;
  r.m[2][0] = cof(0, 2) * invdet; r.m[2][1] = cof(1, 2) * invdet; r.m[2][2] = cof(2, 2) * invdet;
  for (int i = 0; i < 3; ++i)
    r.m[i][3] = -sum3(r.m[i][0] * T.m[0][3], r.m[i][1] * T.m[1][3], r.m[i][2] * T.m[2][3]);
  return r;
}

// Camera.hpp:17-86
struct Cam {
  float K[9];
  int height, width;
  // Camera.hpp:24-31  projectPoint (double math, tuple<double> narrowed to float)
  void project(int r, int c, int depth_mm, float out[3]) const {
    const double fx = K[0], cx = K[2], fy = K[4], cy = K[5];
    const double z = depth_mm * 0.001;
    const double x = z * ((double)c - cx) / (fx);
    const double y = z * ((double)r - cy) / (fy);
    out[0] = (float)x; out[1] = (float)y; out[2] = (float)z;
  }
  // Camera.hpp:32-38  deProjectPoint: int(round(...)).  x86 cvttsd2si yields INT_MIN
  // for NaN/out-of-range; restated explicitly so validPixel() rejects those.
  static int to_int_x86(double v) {
    if (!(v >= -2147483648.0 && v < 2147483648.0)) return INT32_MIN;
    return (int)v;
  }
  void deproject(double x, double y, double z, int& r, int& c) const {
    const double fx = K[0], cx = K[2], fy = K[4], cy = K[5];
    c = to_int_x86(std::round((x * fx) / z + cx));
    r = to_int_x86(std::round((y * fy) / z + cy));
  }
  // Camera.hpp:65-68
  bool valid_pixel(int r, int c) const { return r >= 0 && r < height && c >= 0 && c < width; }
};

// CommonUtilities.hpp:17  degree(): int((radian*180)/3.14159); NaN/overflow -> INT_MIN (x86).
static inline int degree_x86(double radian) { return Cam::to_int_x86((radian * 180) / 3.14159); }

// RayTracingEngine.hpp:22-25
constexpr double k_AngleMin = 0;
constexpr double k_AngleMax = 90;
constexpr double k_ZMin = 0.20;
constexpr double k_ZMax = 1.0;

// normal test used at RayTracingEngine.hpp:207-219,358-369,424-439:
// angle_z = degree(acos(normals.dot(v))) with std::acos(float) == acosf.
static inline bool angle_ok(const Nrm& n, const float v[3]) {
  const float d = sum3(n.n[0] * v[0], n.n[1] * v[1], n.n[2] * v[2]);
  const int a = degree_x86((double)std::acos(d));
  return a >= k_AngleMin && a <= k_AngleMax;
}

// Eigen normalized(): z = squaredNorm(); z > 0 ? v / sqrt(z) : v
static inline void normalized(const float d[3], float v[3]) {
  const float s = sum3(d[0] * d[0], d[1] * d[1], d[2] * d[2]);
  if (s > 0.0f) {
    const float q = std::sqrt(s);
    v[0] = d[0] / q; v[1] = d[1] / q; v[2] = d[2] / q;
  } else {
    v[0] = d[0]; v[1] = d[1]; v[2] = d[2];
  }
}

}  // namespace

// Volume.hpp:50-255 (VoxelVolume) in the reference layout.
struct orc_volume {
  std::vector<uint64_t> occupied_cells_;
  double xmin_ = 0, xmax_ = 0, ymin_ = 0, ymax_ = 0, zmin_ = 0, zmax_ = 0;
  double xcenter_ = 0, ycenter_ = 0, zcenter_ = 0;
  double xdelta_ = 0, ydelta_ = 0, zdelta_ = 0;
  double voxel_size_ = 0;
  int xdim_ = 0, ydim_ = 0, zdim_ = 0;
  uint64_t hsize_ = 0;
  std::vector<std::vector<std::vector<Voxel*>>> voxels_;
  int64_t hazards = 0;  // unguarded out-of-range accesses in the reference

  ~orc_volume() { clear(); }
  void clear() {
    for (auto& a : voxels_)
      for (auto& b : a)
        for (auto* v : b) delete v;
    voxels_.clear();
    occupied_cells_.clear();
  }
  // Volume.hpp:143-148 getHash / getHashId (y<<20 is an int shift)
  uint64_t hash_id(int x, int y, int z) const {
    uint64_t h = (uint64_t)(int64_t)x;
    return (h << 40) ^ (uint64_t)(int64_t)(y << 20) ^ (uint64_t)(int64_t)z;
  }
  // Volume.hpp:150-156 getVoxel: floor((x - min)/delta) in double
  void get_voxel(float x, float y, float z, int& xv, int& yv, int& zv) const {
    xv = (int)std::floor((x - xmin_) / xdelta_);
    yv = (int)std::floor((y - ymin_) / ydelta_);
    zv = (int)std::floor((z - zmin_) / zdelta_);
  }
  uint64_t get_hash(float x, float y, float z) const {
    int a, b, c;
    get_voxel(x, y, z, a, b, c);
    return hash_id(a, b, c);
  }
  // Volume.hpp:158-165
  static void voxel_coords(uint64_t id, int& x, int& y, int& z) {
    const uint64_t mask = (1 << 20) - 1;
    x = (int)(id >> 40);
    y = (int)(id >> 20 & mask);
    z = (int)(id & mask);
  }
  // Volume.hpp:167-170
  bool valid_coords(int x, int y, int z) const {
    return x < xdim_ && y < ydim_ && z < zdim_ && x >= 0 && y >= 0 && z >= 0;
  }
  // Volume.hpp:230-233 (strict interior)
  bool valid_points(float x, float y, float z) const {
    return !(x >= xmax_ || y >= ymax_ || z >= zmax_ || x <= xmin_ || y <= ymin_ || z <= zmin_);
  }
  // voxels_[x][y][z] where the reference indexes without a validCoords guard:
  // out-of-range is UB there; counted as a hazard and treated as empty here.
  Voxel* at_unguarded(int x, int y, int z) {
    if (!valid_coords(x, y, z)) { ++hazards; return nullptr; }
    return voxels_[x][y][z];
  }
  // Volume.hpp:235-255 getNeighborHashes (dead work inside reverseRayTraceFast;
  // kept for honest CPU timing, including the `i==j==k==0` expression).
  std::vector<uint64_t> neighbor_hashes(uint64_t hash, int K) const {
    int xi, yi, zi;
    voxel_coords(hash, xi, yi, zi);
    const double x = xi, y = yi, z = zi;
    std::vector<uint64_t> out;
    for (int i = -K; i <= K; i++)
      for (int j = -K; j <= K; j++)
        for (int k = -K; k <= K; k++) {
          if (((i == j) == k) == 0) continue;
          const int a = (int)(x + i), b = (int)(y + j), c = (int)(z + k);
          if (valid_coords(a, b, c))
            if (voxels_[a][b][c] != nullptr) out.push_back(hash_id(a, b, c));
        }
    return out;
  }
};

extern "C" {

orc_volume* orc_volume_new(void) { return new orc_volume(); }
void orc_volume_free(orc_volume* v) { delete v; }

// Volume.hpp:89-100
void orc_set_dimensions(orc_volume* v, double xmin, double xmax, double ymin, double ymax,
                        double zmin, double zmax) {
  v->xmin_ = xmin; v->xmax_ = xmax; v->ymin_ = ymin; v->ymax_ = ymax; v->zmin_ = zmin; v->zmax_ = zmax;
  v->xcenter_ = v->xmin_ + (v->xmax_ - v->xmin_) / 2.0;
  v->ycenter_ = v->ymin_ + (v->ymax_ - v->ymin_) / 2.0;
  v->zcenter_ = v->zmin_ + (v->zmax_ - v->zmin_) / 2.0;
}
// Volume.hpp:102-107
void orc_set_resolution(orc_volume* v, double dx, double dy, double dz) {
  v->xdelta_ = dx; v->ydelta_ = dy; v->zdelta_ = dz;
}
// Volume.hpp:109-117
void orc_set_volume_size(orc_volume* v, int nx, int ny, int nz) {
  v->xdim_ = nx; v->ydim_ = ny; v->zdim_ = nz;
  v->xdelta_ = (v->xmax_ - v->xmin_) / nx;
  v->ydelta_ = (v->ymax_ - v->ymin_) / ny;
  v->zdelta_ = (v->zmax_ - v->zmin_) / nz;
}
// Volume.hpp:119-128 (dims recomputed by truncation; hsize_ is an int product)
int orc_construct(orc_volume* v) {
  v->clear();
  v->xdim_ = (int)((v->xmax_ - v->xmin_) / v->xdelta_);
  v->ydim_ = (int)((v->ymax_ - v->ymin_) / v->ydelta_);
  v->zdim_ = (int)((v->zmax_ - v->zmin_) / v->zdelta_);
  v->hsize_ = (uint64_t)(int64_t)(v->xdim_ * v->ydim_ * v->zdim_);
  v->voxel_size_ = v->xdelta_ * v->ydelta_ * v->zdelta_;
  v->voxels_ = std::vector<std::vector<std::vector<Voxel*>>>(
      v->xdim_, std::vector<std::vector<Voxel*>>(v->ydim_, std::vector<Voxel*>(v->zdim_, nullptr)));
  return 1;
}

// d[13] = xmin,xmax,ymin,ymax,zmin,zmax,xcenter,ycenter,zcenter,xdelta,ydelta,zdelta,voxel_size
void orc_get_info(const orc_volume* v, double* d, int* dims, uint64_t* hsize) {
  const double vals[13] = {v->xmin_, v->xmax_, v->ymin_, v->ymax_, v->zmin_, v->zmax_,
                           v->xcenter_, v->ycenter_, v->zcenter_, v->xdelta_, v->ydelta_,
                           v->zdelta_, v->voxel_size_};
  std::memcpy(d, vals, sizeof(vals));
  dims[0] = v->xdim_; dims[1] = v->ydim_; dims[2] = v->zdim_;
  *hsize = v->hsize_;
}

int64_t orc_hazards(const orc_volume* v) { return v->hazards; }

// Volume.hpp:172-197 (no normals: NO validCoords guard -> hazard) and
// Volume.hpp:199-228 (with normals: guarded).  Returns the number of points binned.
int64_t orc_integrate(orc_volume* v, const float* xyz, const float* normals, int64_t n) {
  int64_t binned = 0;
  for (int64_t i = 0; i < n; i++) {
    const Pt pt{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
    if (v->valid_points(pt.x, pt.y, pt.z) == false) continue;
    int x, y, z;
    v->get_voxel(pt.x, pt.y, pt.z, x, y, z);
    if (normals) {
      if (v->valid_coords(x, y, z) == false) continue;
    } else if (!v->valid_coords(x, y, z)) {
      ++v->hazards;  // reference indexes voxels_ out of range here (UB)
      continue;
    }
    const uint64_t hash = v->hash_id(x, y, z);
    Voxel*& slot = v->voxels_[x][y][z];
    if (slot == nullptr) {
      v->occupied_cells_.push_back(hash);
      slot = new Voxel();
    }
    slot->pts.push_back(pt);
    if (normals) slot->normals.push_back(Nrm{{normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]}});
    ++binned;
  }
  return binned;
}

int64_t orc_num_occupied(const orc_volume* v) { return (int64_t)v->occupied_cells_.size(); }
int64_t orc_occupied(const orc_volume* v, uint64_t* out, int64_t cap) {
  const int64_t n = (int64_t)v->occupied_cells_.size();
  for (int64_t i = 0; i < n && i < cap; ++i) out[i] = v->occupied_cells_[i];
  return n;
}
// Per-voxel state in occupied_cells_ order: view, good, #points, #normals.
void orc_voxel_table(const orc_volume* v, int32_t* view, uint8_t* good, int64_t* npts, int64_t* nnrm) {
  for (size_t s = 0; s < v->occupied_cells_.size(); ++s) {
    int x, y, z;
    orc_volume::voxel_coords(v->occupied_cells_[s], x, y, z);
    const Voxel* vx = v->voxels_[x][y][z];
    if (view) view[s] = vx->view;
    if (good) good[s] = vx->good ? 1 : 0;
    if (npts) npts[s] = (int64_t)vx->pts.size();
    if (nnrm) nnrm[s] = (int64_t)vx->normals.size();
  }
}
// Points (xyz) and normals of one voxel, in insertion order.
int64_t orc_voxel_points(const orc_volume* v, int x, int y, int z, float* pts, float* nrm, int64_t cap) {
  if (!v->valid_coords(x, y, z) || !v->voxels_[x][y][z]) return -1;
  const Voxel* vx = v->voxels_[x][y][z];
  const int64_t n = (int64_t)vx->pts.size();
  for (int64_t i = 0; i < n && i < cap; ++i) {
    if (pts) { pts[3 * i] = vx->pts[i].x; pts[3 * i + 1] = vx->pts[i].y; pts[3 * i + 2] = vx->pts[i].z; }
    if (nrm && i < (int64_t)vx->normals.size())
      for (int k = 0; k < 3; ++k) nrm[3 * i + k] = vx->normals[i].n[k];
  }
  return n;
}
void orc_reset_flags(orc_volume* v) {
  for (uint64_t h : v->occupied_cells_) {
    int x, y, z;
    orc_volume::voxel_coords(h, x, y, z);
    v->voxels_[x][y][z]->view = 0;
    v->voxels_[x][y][z]->good = false;
  }
}
// Dense occupancy (1 byte per cell, x-major like voxels_[x][y][z]).
void orc_occupancy_dense(const orc_volume* v, uint8_t* out) {
  size_t i = 0;
  for (int x = 0; x < v->xdim_; ++x)
    for (int y = 0; y < v->ydim_; ++y)
      for (int z = 0; z < v->zdim_; ++z) out[i++] = v->voxels_[x][y][z] ? 1 : 0;
}

// ---- Camera helpers (Camera.hpp) -----------------------------------------
void orc_project_point(const float* K, int r, int c, int d, float* out) {
  Cam cam; std::memcpy(cam.K, K, sizeof(cam.K)); cam.project(r, c, d, out);
}
void orc_deproject_point(const float* K, double x, double y, double z, int* rc) {
  Cam cam; std::memcpy(cam.K, K, sizeof(cam.K)); cam.deproject(x, y, z, rc[0], rc[1]);
}
void orc_transform_point(const float* T, double x, double y, double z, float* out) {
  xform(load_aff(T), (float)x, (float)y, (float)z, out);
}
void orc_inverse_pose(const float* T, float* out) {
  const Aff r = inverse_aff(load_aff(T));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) out[i * 4 + j] = r.m[i][j];
}
int orc_degree(double radian) { return degree_x86(radian); }
int orc_angle_ok(const float* n, const float* v) { return angle_ok(Nrm{{n[0], n[1], n[2]}}, v) ? 1 : 0; }

// Per-pixel depth -> world point: projectPoint (Camera.hpp:24-31) then
// transformPoints (Camera.hpp:39-45) — the composition the depth-fusion path
// feeds into integratePointCloud.  Pixels with depth 0 give (0,0,0)->T.
void orc_backproject(const float* K, int H, int W, const uint16_t* depth, const float* T, float* xyz) {
  Cam cam; std::memcpy(cam.K, K, sizeof(cam.K)); cam.height = H; cam.width = W;
  const Aff A = load_aff(T);
  for (int r = 0; r < H; ++r)
    for (int c = 0; c < W; ++c) {
      float p[3];
      cam.project(r, c, depth[(size_t)r * W + c], p);
      xform(A, p[0], p[1], p[2], &xyz[3 * ((size_t)r * W + c)]);
    }
}

// ---- RayTracingEngine ------------------------------------------------------
static Cam make_cam(const float* K, int H, int W) {
  Cam c; std::memcpy(c.K, K, sizeof(c.K)); c.height = H; c.width = W; return c;
}

// Shared body of the reverse 1 mm march (RayTracingEngine.hpp:81-103 and 172-200).
static bool reverse_march_collides(orc_volume& vol, const float centroid[3], const float v[3],
                                   uint64_t centroid_hash, int depth0) {
  for (int depth = depth0;; depth++) {
    float pt[3];
    const float fd = (float)(double)depth;
    for (int i = 0; i < 3; ++i) pt[i] = centroid[i] + ((v[i] * fd) / 1000.0f);
    const double xx = pt[0], yy = pt[1], zz = pt[2];
    if (vol.valid_points(xx, yy, zz) == false) return false;
    const uint64_t hash = vol.get_hash(xx, yy, zz);
    if (hash == centroid_hash) continue;
    int a, b, c;
    vol.get_voxel(xx, yy, zz, a, b, c);
    if (vol.valid_coords(a, b, c) == false) return false;
    if (vol.voxels_[a][b][c] != nullptr) return true;
  }
}

// RayTracingEngine.hpp:136-226 reverseRayTraceFast.  Returns #good hashes (may exceed cap).
int64_t orc_reverse_ray_trace_fast(orc_volume* vol, const float* K, int H, int W, const float* T,
                                   int viz, int dead_work, int* found_out, uint64_t* out, int64_t cap) {
  const Cam cam = make_cam(K, H, W);
  const Aff transformation = load_aff(T);
  const Aff inverseT = inverse_aff(transformation);
  double found = false;
  std::vector<uint64_t> good_points;
  for (uint64_t hashes : vol->occupied_cells_) {
    int xid, yid, zid;
    orc_volume::voxel_coords(hashes, xid, yid, zid);
    const float x = (float)(xid * vol->xdelta_ + vol->xmin_);
    const float y = (float)(yid * vol->ydelta_ + vol->ymin_);
    const float z = (float)(zid * vol->zdelta_ + vol->zmin_);
    Voxel* voxel = vol->voxels_[xid][yid][zid];
    float centroid[3] = {(float)(x + vol->xdelta_ / 2.0), (float)(y + vol->ydelta_ / 2.0),
                         (float)(z + vol->zdelta_ / 2.0)};
    float t[3];
    xform(inverseT, centroid[0], centroid[1], centroid[2], t);
    const float zzz = t[2];
    int r, c;
    cam.deproject(t[0], t[1], t[2], r, c);
    const uint64_t centroid_hash = vol->get_hash(centroid[0], centroid[1], centroid[2]);
    if (cam.valid_pixel(r, c) == false) continue;
    const float cc[3] = {transformation.m[0][3], transformation.m[1][3], transformation.m[2][3]};
    const float d[3] = {cc[0] - centroid[0], cc[1] - centroid[1], cc[2] - centroid[2]};
    float v[3];
    normalized(d, v);
    if (dead_work) {  // :170-171 result unused
      auto neighbors = vol->neighbor_hashes(vol->get_hash(x, y, z), 5);
      std::unordered_set<uint64_t> n_set(neighbors.begin(), neighbors.end());
      if (n_set.size() == (size_t)-1) return -2;  // keep the set alive
    }
    const bool collided = reverse_march_collides(*vol, centroid, v, centroid_hash, 50);
    if (collided == false) {
      found = true;
      if (viz) voxel->view = 1;
      if (zzz >= k_ZMin && zzz <= k_ZMax) {
        for (const Nrm& n : voxel->normals) {
          if (angle_ok(n, v)) {
            if (viz) voxel->good = true;
            good_points.push_back(centroid_hash);
            break;
          }
        }
      }
    }
  }
  if (found_out) *found_out = found != 0.0;
  for (size_t i = 0; i < good_points.size() && (int64_t)i < cap; ++i) out[i] = good_points[i];
  return (int64_t)good_points.size();
}

// The float-accumulated grid enumeration `for(float x=xmin_; x<xmax_; x+=xdelta_)`
// (RayTracingEngine.hpp:54-56,509-511,540-542).
static std::vector<float> float_axis(double lo, double hi, double delta) {
  std::vector<float> xs;
  for (float x = (float)lo; x < hi; x += delta) xs.push_back(x);
  return xs;
}
int64_t orc_float_axis(double lo, double hi, double delta, float* out, int64_t cap) {
  auto xs = float_axis(lo, hi, delta);
  for (size_t i = 0; i < xs.size() && (int64_t)i < cap; ++i) out[i] = xs[i];
  return (int64_t)xs.size();
}

// RayTracingEngine.hpp:45-134 reverseRayTrace (whole-grid enumeration, depth from 1,
// z-window only: the normal test sits under `if(false)`, :115).
int64_t orc_reverse_ray_trace(orc_volume* vol, const float* K, int H, int W, const float* T, int viz,
                              int* found_out, uint64_t* out, int64_t cap) {
  const Cam cam = make_cam(K, H, W);
  const Aff transformation = load_aff(T);
  const Aff inverseT = inverse_aff(transformation);
  double found = false;
  std::vector<uint64_t> good_points;
  const auto xs = float_axis(vol->xmin_, vol->xmax_, vol->xdelta_);
  const auto ys = float_axis(vol->ymin_, vol->ymax_, vol->ydelta_);
  const auto zs = float_axis(vol->zmin_, vol->zmax_, vol->zdelta_);
  for (float x : xs)
    for (float y : ys)
      for (float z : zs) {
        int xid, yid, zid;
        vol->get_voxel(x, y, z, xid, yid, zid);
        Voxel* voxel = vol->at_unguarded(xid, yid, zid);
        if (voxel == nullptr) continue;
        float centroid[3] = {(float)(x + vol->xdelta_ / 2.0), (float)(y + vol->ydelta_ / 2.0),
                             (float)(z + vol->zdelta_ / 2.0)};
        float t[3];
        xform(inverseT, centroid[0], centroid[1], centroid[2], t);
        const float zz = t[2];
        int r, c;
        cam.deproject(t[0], t[1], t[2], r, c);
        const uint64_t centroid_hash = vol->get_hash(centroid[0], centroid[1], centroid[2]);
        if (cam.valid_pixel(r, c) == false) continue;
        const float cc[3] = {transformation.m[0][3], transformation.m[1][3], transformation.m[2][3]};
        const float d[3] = {cc[0] - centroid[0], cc[1] - centroid[1], cc[2] - centroid[2]};
        float v[3];
        normalized(d, v);
        const bool collided = reverse_march_collides(*vol, centroid, v, centroid_hash, 1);
        if (collided == false) {
          found = true;
          if (viz) voxel->view = 1;
          if (zz >= k_ZMin && zz <= k_ZMax) {
            if (viz) voxel->good = true;
            good_points.push_back(centroid_hash);
          }
        }
      }
  if (found_out) *found_out = found != 0.0;
  for (size_t i = 0; i < good_points.size() && (int64_t)i < cap; ++i) out[i] = good_points[i];
  return (int64_t)good_points.size();
}

// Forward depth-plane march, shared by RayTracingEngine.hpp:229-494.
// mode 0 rayTrace, 1 rayTraceAndClassify, 2 rayTraceAndGetGoodPoints, 3 rayTraceAndGetPoints,
// 4 rayTraceAndGetMinimum.  Loop order (z_depth, r, c) exactly as the reference.
static int64_t forward(orc_volume* vol, const float* K, int H, int W, const float* T, int mode,
                       int zstart, int zdelta, int rdelta, int cdelta, int view, int* found_out,
                       uint64_t* out, int64_t cap, int* minimum) {
  const Cam cam = make_cam(K, H, W);
  const Aff transformation = load_aff(T);
  std::vector<char> found((size_t)H * W, 0);
  std::unordered_set<uint64_t> checked;
  std::vector<uint64_t> list;
  bool point_found = false;
  for (int z_depth = zstart; z_depth < k_ZMax * 1000; z_depth += zdelta) {
    for (int r = 0; r < H; r += rdelta) {
      for (int c = 0; c < W; c += cdelta) {
        if (mode != 4 && found[(size_t)r * W + c]) continue;
        float p[3], w[3];
        cam.project(r, c, z_depth, p);
        xform(transformation, p[0], p[1], p[2], w);
        const double x = w[0], y = w[1], z = w[2];
        if (vol->valid_points(x, y, z) == false) continue;
        int xid, yid, zid;
        vol->get_voxel(x, y, z, xid, yid, zid);
        const uint64_t id = vol->hash_id(xid, yid, zid);
        Voxel* voxel = vol->at_unguarded(xid, yid, zid);  // reference: no validCoords guard
        if (voxel == nullptr) continue;
        if (mode == 4) {  // :256-259 early return
          *minimum = z_depth;
          return 0;
        }
        found[(size_t)r * W + c] = 1;
        point_found = true;
        if (mode == 0) {  // :299-305
          voxel->view = 1;
          checked.insert(id);
        } else if (mode == 3) {  // :480-489
          if (checked.find(id) == checked.end()) { checked.insert(id); list.push_back(id); }
        } else {  // classify (:345-370) / good points (:415-439)
          const float centroid[3] = {(float)(x + vol->xdelta_ / 2.0), (float)(y + vol->ydelta_ / 2.0),
                                     (float)(z + vol->zdelta_ / 2.0)};
          const float cc[3] = {transformation.m[0][3], transformation.m[1][3], transformation.m[2][3]};
          const float d[3] = {cc[0] - centroid[0], cc[1] - centroid[1], cc[2] - centroid[2]};
          float v[3];
          normalized(d, v);
          if (mode == 1) {
            if (voxel->view == 0) voxel->view = view;
            if (voxel->good == false) {
              for (const Nrm& n : voxel->normals) {
                const bool ok = angle_ok(n, v);
                if (z_depth >= 250 && z_depth <= 600)
                  if (ok) { voxel->good = true; break; }
              }
            }
          } else {
            for (const Nrm& n : voxel->normals) {
              const bool ok = angle_ok(n, v);
              if (z_depth >= 250 && z_depth <= 600)
                if (ok) {
                  if (checked.find(id) == checked.end()) { checked.insert(id); list.push_back(id); }
                  break;
                }
            }
          }
        }
      }
    }
  }
  if (mode == 4) { *minimum = -1; return 0; }
  if (found_out) *found_out = point_found ? 1 : 0;
  for (size_t i = 0; i < list.size() && (int64_t)i < cap; ++i) out[i] = list[i];
  return (int64_t)list.size();
}

// RayTracingEngine.hpp:268-309 (zdelta default 10, sparse default true -> stride 5)
void orc_ray_trace(orc_volume* vol, const float* K, int H, int W, const float* T, int zdelta, int sparse) {
  const int s = sparse ? 5 : 1;
  forward(vol, K, H, W, T, 0, 10, zdelta, s, s, 1, nullptr, nullptr, 0, nullptr);
}
// RayTracingEngine.hpp:311-375
void orc_ray_trace_and_classify(orc_volume* vol, const float* K, int H, int W, const float* T, int zdelta,
                                int view, int sparse) {
  const int s = sparse ? 5 : 1;
  forward(vol, K, H, W, T, 1, 10, zdelta, s, s, view, nullptr, nullptr, 0, nullptr);
}
// RayTracingEngine.hpp:377-445
int64_t orc_ray_trace_and_get_good_points(orc_volume* vol, const float* K, int H, int W, const float* T,
                                          int zdelta, int sparse, int* found, uint64_t* out, int64_t cap) {
  const int s = sparse ? 5 : 1;
  return forward(vol, K, H, W, T, 2, 10, zdelta, s, s, 1, found, out, cap, nullptr);
}
// RayTracingEngine.hpp:447-494
int64_t orc_ray_trace_and_get_points(orc_volume* vol, const float* K, int H, int W, const float* T,
                                     int zdelta, int sparse, int* found, uint64_t* out, int64_t cap) {
  const int s = sparse ? 5 : 1;
  return forward(vol, K, H, W, T, 3, 10, zdelta, s, s, 1, found, out, cap, nullptr);
}
// RayTracingEngine.hpp:229-264 (zdelta default 1, sparse default true -> stride 10)
int orc_ray_trace_and_get_minimum(orc_volume* vol, const float* K, int H, int W, const float* T,
                                  int zdelta, int sparse) {
  const int s = sparse ? 10 : 1;
  int m = -1;
  forward(vol, K, H, W, T, 4, 5, zdelta, s, s, 1, nullptr, nullptr, 0, &m);
  return m;
}

// Per-pixel first hit of the forward march on the (rdelta,cdelta) lattice:
// k_out = depth-plane index of the first occupied sample (or -1), hash_out = its voxel.
void orc_forward_first_hits(orc_volume* vol, const float* K, int H, int W, const float* T, int zstart,
                            int zdelta, int rdelta, int cdelta, int32_t* k_out, uint64_t* hash_out) {
  const Cam cam = make_cam(K, H, W);
  const Aff A = load_aff(T);
  const int R = (H + rdelta - 1) / rdelta, C = (W + cdelta - 1) / cdelta;
  for (int ri = 0; ri < R; ++ri)
    for (int ci = 0; ci < C; ++ci) {
      const int r = ri * rdelta, c = ci * cdelta;
      int32_t kk = -1; uint64_t hh = 0;
      int k = 0;
      for (int z_depth = zstart; z_depth < k_ZMax * 1000; z_depth += zdelta, ++k) {
        float p[3], w[3];
        cam.project(r, c, z_depth, p);
        xform(A, p[0], p[1], p[2], w);
        if (!vol->valid_points(w[0], w[1], w[2])) continue;
        int a, b, cc;
        vol->get_voxel(w[0], w[1], w[2], a, b, cc);
        if (!vol->valid_coords(a, b, cc)) continue;
        if (vol->voxels_[a][b][cc]) { kk = k; hh = vol->hash_id(a, b, cc); break; }
      }
      k_out[(size_t)ri * C + ci] = kk;
      hash_out[(size_t)ri * C + ci] = hh;
    }
}

// RayTracingEngine.hpp:498-564 rayTraceVolume (z-buffer splat then view marking).
void orc_ray_trace_volume(orc_volume* vol, const float* K, int H, int W, const float* T, int32_t* depth_out) {
  const Cam cam = make_cam(K, H, W);
  const Aff inverse_transformation = inverse_aff(load_aff(T));
  std::vector<int> depth((size_t)H * W, -1);
  const auto xs = float_axis(vol->xmin_, vol->xmax_, vol->xdelta_);
  const auto ys = float_axis(vol->ymin_, vol->ymax_, vol->ydelta_);
  const auto zs = float_axis(vol->zmin_, vol->zmax_, vol->zdelta_);
  for (int pass = 0; pass < 2; ++pass)
    for (float x : xs)
      for (float y : ys)
        for (float z : zs) {
          int xid, yid, zid;
          vol->get_voxel(x, y, z, xid, yid, zid);
          Voxel* voxel = vol->at_unguarded(xid, yid, zid);
          if (voxel == nullptr) continue;
          float t[3];
          xform(inverse_transformation, (float)(x + vol->xdelta_ / 2.0), (float)(y + vol->ydelta_ / 2.0),
                (float)(z + vol->zdelta_ / 2.0), t);
          int r, c;
          cam.deproject(t[0], t[1], t[2], r, c);
          if (cam.valid_pixel(r, c) == false) continue;
          const int d = Cam::to_int_x86((double)std::round(t[2] * 1000));
          int& px = depth[(size_t)r * W + c];
          if (pass == 0) {
            px = (px == -1) ? d : std::min(px, d);
          } else if (px == d) {
            voxel->view = 1;
          }
        }
  if (depth_out)
    for (size_t i = 0; i < depth.size(); ++i) depth_out[i] = depth[i];
}

// tests/CameraPathGen.cpp:128-156 willCollide (1 mm segment march between two points).
int orc_will_collide(orc_volume* vol, const float* a, const float* b) {
  const float ab[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
  const double distance = std::sqrt(sum3(ab[0] * ab[0], ab[1] * ab[1], ab[2] * ab[2]));
  const float ba[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  float v[3];
  normalized(ba, v);
  bool collided = false;
  for (int depth = 1; collided == false; depth++) {
    float pt[3];
    const float fd = (float)(double)depth;
    for (int i = 0; i < 3; ++i) pt[i] = a[i] + ((v[i] * fd) / 1000.0f);
    if (depth > distance * 1000) break;
    if (vol->valid_points(pt[0], pt[1], pt[2]) == false) continue;
    int x, y, z;
    vol->get_voxel(pt[0], pt[1], pt[2], x, y, z);
    if (vol->valid_coords(x, y, z) == false) continue;
    if (vol->voxels_[x][y][z] != nullptr) collided = true;
  }
  return collided ? 1 : 0;
}

// tests/CameraPathGen.cpp:310-331 Planner::run_tsp cost map over all V*V ordered pairs
// of camera centres (pose translations); euclideanDistance is CameraPathGen.cpp:56-59.
void orc_collision_cost_map(orc_volume* vol, const float* poses, int V, int32_t* map) {
  for (int i = 0; i < V; i++)
    for (int j = 0; j < V; j++) {
      const float a[3] = {poses[12 * i + 3], poses[12 * i + 7], poses[12 * i + 11]};
      const float b[3] = {poses[12 * j + 3], poses[12 * j + 7], poses[12 * j + 11]};
      if (orc_will_collide(vol, a, b)) {
        map[(int64_t)i * V + j] = INT_MAX;
      } else {
        const float ab[3] = {a[0] - b[0], a[1] - b[1], a[2] - b[2]};
        const double d = std::sqrt(sum3(ab[0] * ab[0], ab[1] * ab[1], ab[2] * ab[2]));
        map[(int64_t)i * V + j] = (int)(d * 1000);
      }
    }
}

// ============================================================================
// 3D-DDA log-odds depth fusion — this repository's own spec.
// Not in the reference.  Per pixel with dmin <= depth < dmax:
//   E = transformPoints(projectPoint(r,c,d), T)  (Camera.hpp:24-45, bit-exact)
//   O = camera centre (T translation)
//   grid coordinates g = ((double)p - min)/delta   (the Volume.hpp:150-156 expression)
//   end cell = getVoxel(E), inside iff validPoints && validCoords (Volume.hpp:206-213)
//   clip O->E to the box [0,n)^3 (slab test, double), quantise start/end to 1/256
//   cell (clamped into their cells), then an exact integer DDA from start cell to
//   end cell: every cell before the end cell gets a miss, the end cell a hit (or a
//   miss when the endpoint lies outside the grid).  Ties: x before y before z.
// ============================================================================
static const int64_t kQ = 256;  // fixed-point sub-cell resolution

struct FuseGeom {
  double mn[3], dl[3];
  int n[3];
};

static inline int64_t clampi(int64_t v, int64_t lo, int64_t hi) { return v < lo ? lo : (v > hi ? hi : v); }

extern "C++" {
template <bool kAtomic>
static inline void bump(int32_t* p) {
  if (kAtomic) __atomic_fetch_add(p, 1, __ATOMIC_RELAXED);
  else *p += 1;
}

// Returns number of cell updates (misses + hit) applied for this ray.
// kAtomic: the counters are shared by threads (orc_fuse_depth_mt).
template <bool kAtomic = false>
static int64_t dda_ray(const FuseGeom& g, const float O[3], const float E[3], bool end_inside,
                       int32_t* hits, int32_t* misses, int64_t* nhit) {
  double go[3], ge[3], D[3];
  for (int a = 0; a < 3; ++a) {
    go[a] = ((double)O[a] - g.mn[a]) / g.dl[a];
    ge[a] = ((double)E[a] - g.mn[a]) / g.dl[a];
    D[a] = ge[a] - go[a];
  }
  double t0 = 0.0, t1 = 1.0;
  for (int a = 0; a < 3; ++a) {
    if (D[a] == 0.0) {
      if (go[a] < 0.0 || go[a] >= (double)g.n[a]) return 0;
    } else {
      double ta = (0.0 - go[a]) / D[a];
      double tb = ((double)g.n[a] - go[a]) / D[a];
      if (ta > tb) { const double tt = ta; ta = tb; tb = tt; }
      if (ta > t0) t0 = ta;
      if (tb < t1) t1 = tb;
    }
  }
  if (end_inside) { t1 = 1.0; if (t0 > 1.0) t0 = 1.0; }
  if (t0 > t1) return 0;
  int64_t cs[3], ce[3], qs[3], qe[3];
  for (int a = 0; a < 3; ++a) {
    const double gs = go[a] + t0 * D[a];
    const double gx = end_inside ? ge[a] : go[a] + t1 * D[a];
    cs[a] = clampi((int64_t)std::floor(gs), 0, g.n[a] - 1);
    ce[a] = end_inside ? (int64_t)std::floor(ge[a]) : clampi((int64_t)std::floor(gx), 0, g.n[a] - 1);
    qs[a] = clampi((int64_t)std::floor(gs * (double)kQ), cs[a] * kQ, cs[a] * kQ + kQ - 1);
    qe[a] = clampi((int64_t)std::floor(gx * (double)kQ), ce[a] * kQ, ce[a] * kQ + kQ - 1);
  }
  int64_t adq[3], step[3];
  for (int a = 0; a < 3; ++a) {
    const int64_t dq = qe[a] - qs[a];
    adq[a] = dq < 0 ? -dq : dq;
    step[a] = ce[a] > cs[a] ? 1 : (ce[a] < cs[a] ? -1 : 0);
  }
  // Crossing times in half fixed-point units, scaled by the product of the other
  // axes' |dq| (common denominator):  T_a = h_a * prod_{b!=a, adq_b>0} adq_b with
  //   h_a = 2*((cs+1)*Q - qs)      moving up   (boundary reached exactly)
  //   h_a = 2*(qs - cs*Q) + 1      moving down (boundary left just after)
  // so every crossing the walk needs has t <= 1 and every other one t > 1 strictly.
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
  const int64_t nsteps = (ce[0] > cs[0] ? ce[0] - cs[0] : cs[0] - ce[0]) +
                         (ce[1] > cs[1] ? ce[1] - cs[1] : cs[1] - ce[1]) +
                         (ce[2] > cs[2] ? ce[2] - cs[2] : cs[2] - ce[2]);
  int64_t cur[3] = {cs[0], cs[1], cs[2]};
  const int64_t sx = (int64_t)g.n[1] * g.n[2], sy = g.n[2];
  for (int64_t s = 0; s < nsteps; ++s) {
    bump<kAtomic>(&misses[cur[0] * sx + cur[1] * sy + cur[2]]);
    int a = 0;
    if (Tm[1] < Tm[a]) a = 1;
    if (Tm[2] < Tm[a]) a = 2;
    cur[a] += step[a];
    Tm[a] += In[a];
  }
  const int64_t lin = cur[0] * sx + cur[1] * sy + cur[2];
  if (end_inside) { bump<kAtomic>(&hits[lin]); ++*nhit; }
  else bump<kAtomic>(&misses[lin]);
  return nsteps + 1;
}
}  // extern "C++"

// stats[0] = cell updates, stats[1] = rays traced (valid depth), stats[2] = hits
void orc_fuse_depth(const orc_volume* vol, const float* K, int H, int W, const uint16_t* depth,
                    const float* poses, int P, int dmin, int dmax, int32_t* hits, int32_t* misses,
                    int64_t* stats) {
  FuseGeom g;
  g.mn[0] = vol->xmin_; g.mn[1] = vol->ymin_; g.mn[2] = vol->zmin_;
  g.dl[0] = vol->xdelta_; g.dl[1] = vol->ydelta_; g.dl[2] = vol->zdelta_;
  g.n[0] = vol->xdim_; g.n[1] = vol->ydim_; g.n[2] = vol->zdim_;
  const Cam cam = make_cam(K, H, W);
  int64_t upd = 0, rays = 0, nhit = 0;
  for (int p = 0; p < P; ++p) {
    const Aff A = load_aff(poses + 12 * p);
    const float O[3] = {A.m[0][3], A.m[1][3], A.m[2][3]};
    const uint16_t* dp = depth + (size_t)p * H * W;
    for (int r = 0; r < H; ++r)
      for (int c = 0; c < W; ++c) {
        const int d = dp[(size_t)r * W + c];
        if (!(d >= dmin && d < dmax)) continue;
        float pc[3], E[3];
        cam.project(r, c, d, pc);
        xform(A, pc[0], pc[1], pc[2], E);
        bool inside = vol->valid_points(E[0], E[1], E[2]);
        if (inside) {
          int a, b, cc;
          vol->get_voxel(E[0], E[1], E[2], a, b, cc);
          inside = vol->valid_coords(a, b, cc);
        }
        ++rays;
        upd += dda_ray(g, O, E, inside, hits, misses, &nhit);
      }
  }
  if (stats) { stats[0] += upd; stats[1] += rays; stats[2] += nhit; }
}

// Same computation, pose/row-parallel over nthreads OpenMP threads with relaxed
// atomic counter increments (the CPU baseline on all host cores).
// Counts are integers, so the result equals orc_fuse_depth exactly.
void orc_fuse_depth_mt(const orc_volume* vol, const float* K, int H, int W, const uint16_t* depth,
                       const float* poses, int P, int dmin, int dmax, int32_t* hits, int32_t* misses,
                       int64_t* stats, int nthreads) {
  FuseGeom g;
  g.mn[0] = vol->xmin_; g.mn[1] = vol->ymin_; g.mn[2] = vol->zmin_;
  g.dl[0] = vol->xdelta_; g.dl[1] = vol->ydelta_; g.dl[2] = vol->zdelta_;
  g.n[0] = vol->xdim_; g.n[1] = vol->ydim_; g.n[2] = vol->zdim_;
  const Cam cam = make_cam(K, H, W);
  int64_t upd = 0, rays = 0, nhit = 0;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 4) reduction(+ : upd, rays, nhit)
  for (int64_t pr = 0; pr < (int64_t)P * H; ++pr) {
    const int p = (int)(pr / H), r = (int)(pr % H);
    const Aff A = load_aff(poses + 12 * p);
    const float O[3] = {A.m[0][3], A.m[1][3], A.m[2][3]};
    const uint16_t* dp = depth + (size_t)p * H * W;
    for (int c = 0; c < W; ++c) {
      const int d = dp[(size_t)r * W + c];
      if (!(d >= dmin && d < dmax)) continue;
      float pc[3], E[3];
      cam.project(r, c, d, pc);
      xform(A, pc[0], pc[1], pc[2], E);
      bool inside = vol->valid_points(E[0], E[1], E[2]);
      if (inside) {
        int a, b, cc;
        vol->get_voxel(E[0], E[1], E[2], a, b, cc);
        inside = vol->valid_coords(a, b, cc);
      }
      ++rays;
      int64_t h = 0;
      upd += dda_ray<true>(g, O, E, inside, hits, misses, &h);
      nhit += h;
    }
  }
  if (stats) { stats[0] += upd; stats[1] += rays; stats[2] += nhit; }
}

// Algorithms.hpp:38-86 greedySetCover (the set-cover consumer of reverseRayTraceFast,
// tests/SetCover.cpp:218-240): candidate sets given as concatenated SORTED hash
// lists with per-set counts.  Each iteration scans the remaining ids in increasing
// order, keeps the strictly largest |set \ covered| (std::set_difference), stops when
// none is positive (selected == -1) or the best is below min_gain (5 in the
// reference), merges the difference into the sorted `covered`, removes the id.
// Returns the number of selected ids written to `selected` (selection order).
int32_t orc_greedy_set_cover(const uint64_t* hashes, const int64_t* counts, int32_t nsets, int32_t min_gain,
                             int32_t* selected) {
  std::vector<std::vector<uint64_t>> sets(nsets);
  int64_t off = 0;
  for (int32_t i = 0; i < nsets; ++i) {
    sets[i].assign(hashes + off, hashes + off + counts[i]);
    off += counts[i];
  }
  std::vector<uint64_t> covered;
  std::vector<int32_t> ids(nsets);
  for (int32_t i = 0; i < nsets; ++i) ids[i] = i;
  int32_t nsel = 0;
  while (true) {
    int64_t sel = -1;
    size_t max_points = 0;
    for (int32_t x : ids) {
      std::vector<uint64_t> diff;
      std::set_difference(sets[x].begin(), sets[x].end(), covered.begin(), covered.end(),
                          std::inserter(diff, diff.begin()));
      if (diff.size() > max_points) {
        max_points = diff.size();
        sel = x;
      }
    }
    if (sel == -1) break;
    if ((int64_t)max_points < min_gain) break;
    std::vector<uint64_t> diff;
    std::set_difference(sets[sel].begin(), sets[sel].end(), covered.begin(), covered.end(),
                        std::inserter(diff, diff.begin()));
    for (uint64_t h : diff) covered.push_back(h);
    std::sort(covered.begin(), covered.end());
    selected[nsel++] = (int32_t)sel;
    ids.erase(std::remove(ids.begin(), ids.end(), (int32_t)sel), ids.end());
  }
  return nsel;
}

// ---- OccupancyGrid (include/OccupancyGrid.hpp:50-318), sequential semantics -------
// The reference runs updateStates' loops under OpenMP with racy read-modify-writes;
// the deterministic result it approximates is the single-threaded order restated here
// (points in cloud order, offsets i, j, k from -K..K).  Dense per-voxel state in the
// reference's x-major order.
struct orc_ogrid {
  double xmin_ = 0, xmax_ = 0, ymin_ = 0, ymax_ = 0, zmin_ = 0, zmax_ = 0;
  double xres_ = 0, yres_ = 0, zres_ = 0;
  int xdim_ = 0, ydim_ = 0, zdim_ = 0, k_ = 0;
  std::vector<float> normal, centroid;  // 3 per voxel
  std::vector<int32_t> count;
  std::vector<uint8_t> occupied, normal_found;
  size_t idx(int x, int y, int z) const { return ((size_t)x * ydim_ + y) * zdim_ + z; }
  bool valid_coords(int x, int y, int z) const {  // :399-402
    return x < xdim_ && y < ydim_ && z < zdim_ && x >= 0 && y >= 0 && z >= 0;
  }
  void coords(const float p[3], int& x, int& y, int& z) const {  // :373-379
    x = (int)std::floor(((double)p[0] - xmin_) / xres_);
    y = (int)std::floor(((double)p[1] - ymin_) / yres_);
    z = (int)std::floor(((double)p[2] - zmin_) / zres_);
  }
};

orc_ogrid* orc_ogrid_new() { return new orc_ogrid(); }
void orc_ogrid_free(orc_ogrid* g) { delete g; }
void orc_ogrid_setup(orc_ogrid* g, const double* bounds, float xr, float yr, float zr, int k) {
  g->xmin_ = bounds[0]; g->xmax_ = bounds[1]; g->ymin_ = bounds[2];  // :323-336
  g->ymax_ = bounds[3]; g->zmin_ = bounds[4]; g->zmax_ = bounds[5];
  g->xres_ = xr; g->yres_ = yr; g->zres_ = zr;                       // :338-343 (float params)
  g->k_ = k;                                                          // setK
  g->xdim_ = (int)((g->xmax_ - g->xmin_) / g->xres_);                 // :345-352 construct
  g->ydim_ = (int)((g->ymax_ - g->ymin_) / g->yres_);
  g->zdim_ = (int)((g->zmax_ - g->zmin_) / g->zres_);
  const size_t n = (size_t)g->xdim_ * g->ydim_ * g->zdim_;
  g->normal.assign(3 * n, 0.f); g->centroid.assign(3 * n, 0.f);
  g->count.assign(n, 0); g->occupied.assign(n, 0); g->normal_found.assign(n, 0);
}
void orc_ogrid_dims(const orc_ogrid* g, int32_t* d) { d[0] = g->xdim_; d[1] = g->ydim_; d[2] = g->zdim_; }

// :88-98 projectPointToVector (float; the double ball_radius is applied as float)
static void project_to_vector(const float pt[3], const float np[3], const float n[3], float out[3]) {
  const float br = (float)0.015;
  float a[3], b[3], ap[3], ab[3];
  for (int i = 0; i < 3; ++i) {
    const float d = n[i] * br;
    a[i] = np[i] - d;
    b[i] = np[i] + d;
  }
  for (int i = 0; i < 3; ++i) { ap[i] = a[i] - pt[i]; ab[i] = a[i] - b[i]; }
  const float s = sum3(ap[0] * ab[0], ap[1] * ab[1], ap[2] * ab[2]) / sum3(ab[0] * ab[0], ab[1] * ab[1], ab[2] * ab[2]);
  for (int i = 0; i < 3; ++i) out[i] = a[i] - s * ab[i];
}

// :99-164 updateStates(cloud, normals): cloud = n_cloud x 3 floats, normals = n_nrm x 6
// floats (x, y, z, nx, ny, nz).
void orc_ogrid_update(orc_ogrid* g, const float* cloud, int64_t n_cloud, const float* pn, int64_t n_nrm) {
  const int K = g->k_;
  for (int64_t p = 0; p < n_nrm; ++p) {
    const float* q = pn + 6 * p;
    int x, y, z;
    g->coords(q, x, y, z);
    for (int i = -K; i <= K; ++i)
      for (int j = -K; j <= K; ++j)
        for (int k = -K; k <= K; ++k) {
          if (!g->valid_coords(x + i, y + j, z + k)) continue;
          const size_t v = g->idx(x + i, y + j, z + k);
          float s[3] = {g->normal[3 * v] + q[3], g->normal[3 * v + 1] + q[4], g->normal[3 * v + 2] + q[5]};
          normalized(s, &g->normal[3 * v]);
          g->normal_found[v] = 1;
        }
  }
  for (int64_t p = 0; p < n_cloud; ++p) {
    const float* pt = cloud + 3 * p;
    int x, y, z;
    g->coords(pt, x, y, z);
    for (int i = -K; i <= K; ++i)
      for (int j = -K; j <= K; ++j)
        for (int k = -K; k <= K; ++k) {
          if (!g->valid_coords(x + i, y + j, z + k)) continue;
          const size_t v = g->idx(x + i, y + j, z + k);
          if (!g->normal_found[v]) continue;
          const float c[3] = {(float)(g->xmin_ + g->xres_ * (x + i) + g->xres_ / 2.0),
                              (float)(g->ymin_ + g->yres_ * (y + j) + g->yres_ / 2.0),
                              (float)(g->zmin_ + g->zres_ * (z + k) + g->zres_ / 2.0)};
          float pr[3];
          project_to_vector(pt, c, &g->normal[3 * v], pr);
          const float d[3] = {pt[0] - pr[0], pt[1] - pr[1], pt[2] - pr[2]};
          const float dist = std::sqrt(sum3(d[0] * d[0], d[1] * d[1], d[2] * d[2]));
          if ((double)dist < 0.001) {
            const int cnt = ++g->count[v];
            for (int a = 0; a < 3; ++a) g->centroid[3 * v + a] += (pr[a] - g->centroid[3 * v + a]) / (float)cnt;
          }
        }
    if (g->valid_coords(x, y, z)) g->occupied[g->idx(x, y, z)] = 1;
  }
}

// Dense state copy (normal, centroid: 3 floats; count; occupied | normal_found << 1).
void orc_ogrid_state(const orc_ogrid* g, float* normal, float* centroid, int32_t* count, uint8_t* flags) {
  const size_t n = g->count.size();
  std::memcpy(normal, g->normal.data(), sizeof(float) * 3 * n);
  std::memcpy(centroid, g->centroid.data(), sizeof(float) * 3 * n);
  std::memcpy(count, g->count.data(), sizeof(int32_t) * n);
  for (size_t i = 0; i < n; ++i) flags[i] = (uint8_t)(g->occupied[i] | (g->normal_found[i] << 1));
}

// :166-193 downloadCloud (mode 0) / :283-318 downloadHQCloud (mode 1): occupied voxels
// in x-major order as (cx, cy, cz, nx, ny, nz).  Returns the count (writes <= cap).
int64_t orc_ogrid_download(const orc_ogrid* g, int mode, float* out, int64_t cap) {
  int64_t n = 0;
  for (size_t v = 0; v < g->count.size(); ++v) {
    if (!g->occupied[v]) continue;
    if (mode == 1 && !(g->count[v] > 100)) continue;
    if (n < cap)
      for (int a = 0; a < 3; ++a) { out[6 * n + a] = g->centroid[3 * v + a]; out[6 * n + 3 + a] = g->normal[3 * v + a]; }
    ++n;
  }
  return n;
}

// Dense state upload (the reference's voxels_ fields are public; callers may write them).
void orc_ogrid_set_state(orc_ogrid* g, const float* normal, const float* centroid, const int32_t* count,
                         const uint8_t* flags) {
  const size_t n = g->count.size();
  std::memcpy(g->normal.data(), normal, sizeof(float) * 3 * n);
  std::memcpy(g->centroid.data(), centroid, sizeof(float) * 3 * n);
  std::memcpy(g->count.data(), count, sizeof(int32_t) * n);
  for (size_t i = 0; i < n; ++i) {
    g->occupied[i] = flags[i] & 1;
    g->normal_found[i] = (flags[i] >> 1) & 1;
  }
}

// :200-286 downloadReorganizedCloud(cloud, clean), in the single-threaded order its
// OpenMP loops race over.  Stage 1 copies normal / centroid / count / normal_found into
// voxels_reorganized_ (occupied stays false).  Stage 2, x-major: every voxel occupied in
// voxels_ (and, with clean, whose reorganized count is >= 100 at its turn) merges its
// CURRENT reorganized state into the reorganized voxel holding its centroid (the same
// object when that is itself: n + n, (c + c) / 2).  Stage 3 emits the reorganized voxels
// marked occupied, x-major, as (cx, cy, cz, nx, ny, nz).  Returns the count (writes <= cap).
int64_t orc_ogrid_download_reorganized(const orc_ogrid* g, int clean, float* out, int64_t cap) {
  const size_t n = g->count.size();
  std::vector<float> nr(g->normal), cr(g->centroid);
  std::vector<int32_t> kr(g->count);
  std::vector<uint8_t> occ(n, 0);
  for (int x = 0; x < g->xdim_; ++x)
    for (int y = 0; y < g->ydim_; ++y)
      for (int z = 0; z < g->zdim_; ++z) {
        const size_t s = g->idx(x, y, z);
        if (!g->occupied[s]) continue;
        if (clean && kr[s] < 100) continue;
        // getVoxelCoords(Vector3f) (:373-379): floor of the double quotient, int via cvttsd2si
        const float c[3] = {cr[3 * s], cr[3 * s + 1], cr[3 * s + 2]};
        const double q[3] = {std::floor(((double)c[0] - g->xmin_) / g->xres_),
                             std::floor(((double)c[1] - g->ymin_) / g->yres_),
                             std::floor(((double)c[2] - g->zmin_) / g->zres_)};
        int t[3];
        for (int a = 0; a < 3; ++a) t[a] = (q[a] >= -2147483648.0 && q[a] < 2147483648.0) ? (int)q[a] : INT32_MIN;
        if (!g->valid_coords(t[0], t[1], t[2])) continue;
        const size_t d = g->idx(t[0], t[1], t[2]);
        const float sn[3] = {nr[3 * s], nr[3 * s + 1], nr[3 * s + 2]};  // source state (read first: may alias d)
        occ[d] = 1;
        const float sum[3] = {nr[3 * d] + sn[0], nr[3 * d + 1] + sn[1], nr[3 * d + 2] + sn[2]};
        normalized(sum, &nr[3 * d]);
        if (kr[d] == 0) {
          for (int a = 0; a < 3; ++a) cr[3 * d + a] = c[a];
        } else {
          for (int a = 0; a < 3; ++a) cr[3 * d + a] = (cr[3 * d + a] + c[a]) / 2.0f;
          ++kr[d];
        }
      }
  int64_t m = 0;
  for (size_t v = 0; v < n; ++v) {
    if (!occ[v]) continue;
    if (m < cap)
      for (int a = 0; a < 3; ++a) { out[6 * m + a] = cr[3 * v + a]; out[6 * m + 3 + a] = nr[3 * v + a]; }
    ++m;
  }
  return m;
}

// Clamped fixed-point log-odds (milli-logit units) from the exact counts.
void orc_fuse_finalize(int64_t n, const int32_t* hits, const int32_t* misses, int l_hit, int l_miss,
                       int l_min, int l_max, int16_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t L = (int64_t)hits[i] * l_hit + (int64_t)misses[i] * l_miss;
    if (L < l_min) L = l_min;
    if (L > l_max) L = l_max;
    out[i] = (int16_t)L;
  }
}

}  // extern "C"
