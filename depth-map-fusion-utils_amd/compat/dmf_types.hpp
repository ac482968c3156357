// dmf_types.hpp — the minimal Eigen / PCL vocabulary the reference hot path uses
// (Affine3f, Vector3f with comma initialiser, PointXYZRGB, Normal, PointCloud::Ptr),
// so code written against include/Camera.hpp, Volume.hpp and RayTracingEngine.hpp of
// the reference compiles against the MI355X engine without Eigen or PCL installed.
//
// Arithmetic follows Eigen 3.3 for fixed-size 3-vectors: a 3-term sum is a0 + (a1 + a2)
// (redux_novec_unroller), Transform * Vector = t + linear * p, Affine inverse by 3x3
// cofactors.  Define DMF_COMPAT_REAL_EIGEN / DMF_COMPAT_REAL_PCL to use
// the real libraries' types instead (the engine only needs the 3x4 pose floats).
#pragma once
#include <cmath>
#include <cstdint>
#include <memory>
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

struct PointXYZRGB {
  float x = 0, y = 0, z = 0;
  uint8_t r = 0, g = 0, b = 0;
};

struct Normal {
  float normal[3] = {0, 0, 0};
  float curvature = 0;
};

template <class T>
struct PointCloud {
  std::vector<T> points;
  using Ptr = std::shared_ptr<PointCloud<T>>;
  size_t size() const { return points.size(); }
  void push_back(const T& p) { points.push_back(p); }
};

// rows 0..2 of any Affine3f-like transform (the lite type or real Eigen) as float[12]
template <class T>
inline void pose12(const T& t, float* out) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = t(i, j);
}

}  // namespace dmf_compat

#ifndef DMF_COMPAT_REAL_EIGEN
namespace Eigen {
using Affine3f = dmf_compat::Affine3f;
using Vector3f = dmf_compat::Vector3f;
}  // namespace Eigen
#endif

#ifndef DMF_COMPAT_REAL_PCL
namespace pcl {
using PointXYZRGB = dmf_compat::PointXYZRGB;
using Normal = dmf_compat::Normal;
template <class T>
using PointCloud = dmf_compat::PointCloud<T>;
}  // namespace pcl
#endif
