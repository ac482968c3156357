// dmf_types.hpp — the minimal Eigen / PCL vocabulary the reference hot path uses
// (Affine3f, Vector3f with comma initialiser, PointXYZRGB, Normal, PointCloud::Ptr),
// so code written against include/Camera.hpp, Volume.hpp and RayTracingEngine.hpp of
// the reference compiles against the MI355X engine without Eigen or PCL installed.
//
// Arithmetic follows Eigen 3.3 for fixed-size 3-vectors: a 3-term sum is a0 + (a1 + a2)
// (redux_novec_unroller), Transform * Vector = t + linear * p, Affine inverse by 3x3
// cofactors.  Define DMF_COMPAT_REAL_EIGEN / DMF_COMPAT_REAL_PCL to use
// the real libraries' types instead (the engine only needs the 3x4 pose floats); the
// third-party shims live in compat/shims/ and go on the include path only without them.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

namespace dmf_compat {

inline float sum3(float a0, float a1, float a2) { return a0 + (a1 + a2); }

struct Vector3f {
  float v[3] = {0.f, 0.f, 0.f};
  Vector3f() = default;
  explicit Vector3f(int) {}  // Eigen's Vector3f p1(3) idiom
  Vector3f(float a, float b, float c) : v{a, b, c} {}
  float& operator()(int i) { return v[i]; }
  float operator()(int i) const { return v[i]; }
  float& operator[](int i) { return v[i]; }
  float operator[](int i) const { return v[i]; }
  struct CommaInit {
    Vector3f& t;
    int i;
    CommaInit& operator,(double x) { t.v[i++] = (float)x; return *this; }
  };
  CommaInit operator<<(double x) { v[0] = (float)x; return CommaInit{*this, 1}; }
  Vector3f operator+(const Vector3f& o) const { return {v[0] + o.v[0], v[1] + o.v[1], v[2] + o.v[2]}; }
  Vector3f operator-(const Vector3f& o) const { return {v[0] - o.v[0], v[1] - o.v[1], v[2] - o.v[2]}; }
  // Eigen promotes a double scalar to the float Scalar before the coefficient-wise op
  Vector3f operator*(double s) const { const float f = (float)s; return {v[0] * f, v[1] * f, v[2] * f}; }
  Vector3f operator/(double s) const { const float f = (float)s; return {v[0] / f, v[1] / f, v[2] / f}; }
  float dot(const Vector3f& o) const { return sum3(v[0] * o.v[0], v[1] * o.v[1], v[2] * o.v[2]); }
  // Eigen cross(): (a1 b2 - a2 b1, a2 b0 - a0 b2, a0 b1 - a1 b0)
  Vector3f cross(const Vector3f& o) const {
    return {v[1] * o.v[2] - v[2] * o.v[1], v[2] * o.v[0] - v[0] * o.v[2], v[0] * o.v[1] - v[1] * o.v[0]};
  }
  float squaredNorm() const { return dot(*this); }
  float norm() const { return std::sqrt(squaredNorm()); }
  Vector3f normalized() const {
    const float z = squaredNorm();
    if (z > 0.f) { const float q = std::sqrt(z); return {v[0] / q, v[1] / q, v[2] / q}; }
    return *this;
  }
};

struct Affine3f {
  float m[3][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}};
  static Affine3f Identity() { return Affine3f(); }
  float& operator()(int i, int j) { return m[i][j]; }
  float operator()(int i, int j) const { return (i == 3) ? (j == 3 ? 1.f : 0.f) : m[i][j]; }
  // Transform * Vector3f (Affine): res = translation; res += linear * p
  Vector3f operator*(const Vector3f& p) const {
    Vector3f r;
    for (int i = 0; i < 3; ++i) r.v[i] = m[i][3] + sum3(m[i][0] * p.v[0], m[i][1] * p.v[1], m[i][2] * p.v[2]);
    return r;
  }
  // Transform::inverse() with Mode=Affine (InverseImpl.h compute_inverse<3>)
  Affine3f inverse() const {
    auto M = [&](int i, int j) { return m[i][j]; };
    auto cof = [&](int i, int j) -> float {
      const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
    };
    const float c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const float det = sum3(c0 * M(0, 0), c1 * M(1, 0), c2 * M(2, 0));
    const float inv = 1.0f / det;
    Affine3f r;
    r.m[0][0] = c0 * inv; r.m[0][1] = c1 * inv; r.m[0][2] = c2 * inv;
    r.m[1][0] = cof(0, 1) * inv; r.m[1][1] = cof(1, 1) * inv; r.m[1][2] = cof(2, 1) * inv;
    r.m[2][0] = cof(0, 2) * inv; r.m[2][1] = cof(1, 2) * inv; r.m[2][2] = cof(2, 2) * inv;
    for (int i = 0; i < 3; ++i) r.m[i][3] = -sum3(r.m[i][0] * m[0][3], r.m[i][1] * m[1][3], r.m[i][2] * m[2][3]);
    return r;
  }
  // rows 0..2 as the C ABI's float[12]
  void to12(float* out) const {
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 4; ++j) out[4 * i + j] = m[i][j];
  }
};

struct PointXYZ {
  float x = 0, y = 0, z = 0;
};

struct PointXYZRGB {
  float x = 0, y = 0, z = 0;
  uint8_t r = 0, g = 0, b = 0;
};

// PCL's normal[3] aliases normal_x, normal_y, normal_z
#define DMF_COMPAT_NORMAL_FIELDS                   \
  union {                                          \
    float normal[3];                               \
    struct {                                       \
      float normal_x, normal_y, normal_z;          \
    };                                             \
  };

struct Normal {
  DMF_COMPAT_NORMAL_FIELDS
  float curvature = 0;
  Normal() : normal{0, 0, 0} {}
};

struct PointNormal {
  float x = 0, y = 0, z = 0;
  DMF_COMPAT_NORMAL_FIELDS
  float curvature = 0;
  PointNormal() : normal{0, 0, 0} {}
};

struct PointXYZRGBNormal {
  float x = 0, y = 0, z = 0;
  uint8_t r = 0, g = 0, b = 0;
  DMF_COMPAT_NORMAL_FIELDS
  float curvature = 0;
  PointXYZRGBNormal() : normal{0, 0, 0} {}
};

template <class T>
struct PointCloud {
  std::vector<T> points;
  uint32_t width = 0, height = 1;
  bool is_dense = true;
  using Ptr = std::shared_ptr<PointCloud<T>>;
  size_t size() const { return points.size(); }
  bool empty() const { return points.empty(); }
  void push_back(const T& p) { points.push_back(p); width = (uint32_t)points.size(); height = 1; }
  T& operator[](size_t i) { return points[i]; }
  const T& operator[](size_t i) const { return points[i]; }
  typename std::vector<T>::iterator begin() { return points.begin(); }
  typename std::vector<T>::iterator end() { return points.end(); }
};

// PCD field setters (pcl/io/pcd_io.h): rgb arrives as the packed 0x00RRGGBB integer
inline void set_xyz(float* p, const std::string& n, double v) {
  if (n == "x") p[0] = (float)v;
  else if (n == "y") p[1] = (float)v;
  else if (n == "z") p[2] = (float)v;
}
inline void set_rgb(uint8_t& r, uint8_t& g, uint8_t& b, const std::string& n, double v) {
  if (n != "rgb" && n != "rgba") return;
  const uint32_t u = (uint32_t)v;
  r = (uint8_t)(u >> 16); g = (uint8_t)(u >> 8); b = (uint8_t)u;
}
inline void set_nrm(float* nr, float& curv, const std::string& n, double v) {
  if (n == "normal_x") nr[0] = (float)v;
  else if (n == "normal_y") nr[1] = (float)v;
  else if (n == "normal_z") nr[2] = (float)v;
  else if (n == "curvature") curv = (float)v;
}
inline void set_field(PointXYZ& p, const std::string& n, double v) { float t[3] = {p.x, p.y, p.z}; set_xyz(t, n, v); p.x = t[0]; p.y = t[1]; p.z = t[2]; }
inline void set_field(PointXYZRGB& p, const std::string& n, double v) {
  float t[3] = {p.x, p.y, p.z}; set_xyz(t, n, v); p.x = t[0]; p.y = t[1]; p.z = t[2];
  set_rgb(p.r, p.g, p.b, n, v);
}
inline void set_field(Normal& p, const std::string& n, double v) { set_nrm(p.normal, p.curvature, n, v); }
inline void set_field(PointNormal& p, const std::string& n, double v) {
  float t[3] = {p.x, p.y, p.z}; set_xyz(t, n, v); p.x = t[0]; p.y = t[1]; p.z = t[2];
  set_nrm(p.normal, p.curvature, n, v);
}
inline void set_field(PointXYZRGBNormal& p, const std::string& n, double v) {
  float t[3] = {p.x, p.y, p.z}; set_xyz(t, n, v); p.x = t[0]; p.y = t[1]; p.z = t[2];
  set_rgb(p.r, p.g, p.b, n, v);
  set_nrm(p.normal, p.curvature, n, v);
}

// Float mean of every field of points idx[s..e) (pcl/filters/voxel_grid.h)
template <class T>
inline T mean_point(const std::vector<T>& pts, const std::vector<std::pair<int64_t, size_t>>& idx, size_t s, size_t e) {
  float acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  T out = pts[idx[s].second];
  for (size_t i = s; i < e; ++i) {
    const T& p = pts[idx[i].second];
    acc[0] += p.x; acc[1] += p.y; acc[2] += p.z;
    if constexpr (std::is_same<T, PointXYZRGB>::value || std::is_same<T, PointXYZRGBNormal>::value) {
      acc[3] += p.r; acc[4] += p.g; acc[5] += p.b;
    }
    if constexpr (std::is_same<T, PointXYZRGBNormal>::value) {
      acc[6] += p.normal[0]; acc[7] += p.normal[1]; acc[8] += p.normal[2]; acc[9] += p.curvature;
    }
  }
  const float n = (float)(e - s);
  out.x = acc[0] / n; out.y = acc[1] / n; out.z = acc[2] / n;
  if constexpr (std::is_same<T, PointXYZRGB>::value || std::is_same<T, PointXYZRGBNormal>::value) {
    out.r = (uint8_t)(acc[3] / n); out.g = (uint8_t)(acc[4] / n); out.b = (uint8_t)(acc[5] / n);
  }
  if constexpr (std::is_same<T, PointXYZRGBNormal>::value) {
    out.normal[0] = acc[6] / n; out.normal[1] = acc[7] / n; out.normal[2] = acc[8] / n; out.curvature = acc[9] / n;
  }
  return out;
}

// rows 0..2 of any Affine3f-like transform (the lite type or real Eigen) as float[12]
template <class T>
inline void pose12(const T& t, float* out) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = t(i, j);
}

}  // namespace dmf_compat

// The vocabulary's source: the real Eigen / PCL when the caller defines
// DMF_COMPAT_REAL_EIGEN / DMF_COMPAT_REAL_PCL (their headers first on the include path, and
// compat/shims NOT on it: INTEGRATION.md §2), else the lite types above (the shims in
// compat/shims/ forward <Eigen/Dense>, <pcl/point_types.h>, ... here).
#ifdef DMF_COMPAT_REAL_EIGEN
#include <Eigen/Dense>
#else
namespace Eigen {
using Affine3f = dmf_compat::Affine3f;
using Vector3f = dmf_compat::Vector3f;
}  // namespace Eigen
#endif

#ifdef DMF_COMPAT_REAL_PCL
#include <pcl/point_cloud.h>
#include <pcl/point_types.h>
#else
namespace pcl {
using PointXYZ = dmf_compat::PointXYZ;
using PointXYZRGB = dmf_compat::PointXYZRGB;
using PointXYZRGBNormal = dmf_compat::PointXYZRGBNormal;
using PointNormal = dmf_compat::PointNormal;
using Normal = dmf_compat::Normal;
template <class T>
using PointCloud = dmf_compat::PointCloud<T>;
}  // namespace pcl
#endif
