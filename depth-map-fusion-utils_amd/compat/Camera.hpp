// Camera.hpp — drop-in for the reference include/Camera.hpp:17-86 (same class, same
// member signatures).  The scalar helpers are the reference formulas on the host;
// whole-frame back-projection runs on the GPU (RayTracingEngine::backproject /
// dmf_backproject in include/dmf.h).
#pragma once
#include <cmath>
#include <tuple>
#include <vector>

#include "dmf.h"
#include "dmf_types.hpp"

class Camera {
  std::vector<float> K_;
  int height_ = 480, width_ = 640;

 public:
  Camera() : K_(9, 0.f) {}
  Camera(std::vector<float>& K, int height = 480, int width = 640) : K_(K), height_(height), width_(width) {}

  // Camera.hpp:24-31
  std::tuple<float, float, float> projectPoint(int r, int c, int depth_mm) {
    const double fx = K_[0], cx = K_[2], fy = K_[4], cy = K_[5];
    const double z = depth_mm * 0.001;
    const double x = z * ((double)c - cx) / (fx);
    const double y = z * ((double)r - cy) / (fy);
    return std::make_tuple((float)x, (float)y, (float)z);
  }
  // Camera.hpp:32-38
  std::tuple<int, int> deProjectPoint(double x, double y, double z) {
    const double fx = K_[0], cx = K_[2], fy = K_[4], cy = K_[5];
    const int c = int(std::round((x * fx) / z + cx));
    const int r = int(std::round((y * fy) / z + cy));
    return std::make_tuple(r, c);
  }
  // Camera.hpp:39-45
  std::tuple<float, float, float> transformPoints(double x, double y, double z, Eigen::Affine3f& T) {
    Eigen::Vector3f p1(3);
    p1 << x, y, z;
    const Eigen::Vector3f p2 = T * p1;
    return std::make_tuple(p2(0), p2(1), p2(2));
  }
  std::tuple<float, float, float> getPoint(int r, int c, int depth_mm) { return projectPoint(r, c, depth_mm); }
  std::tuple<int, int> getPixel(double x, double y, double z, Eigen::Affine3f T = Eigen::Affine3f::Identity()) {
    float a, b, cc;
    std::tie(a, b, cc) = transformPoints(x, y, z, T);
    return deProjectPoint(a, b, cc);
  }
  int getHeight() { return height_; }
  int getWidth() { return width_; }
  bool validPixel(int r, int c) { return (r >= 0 && r < height_ && c >= 0 && c < width_); }
  float getAreaCovered(int depth_mm) {
    double x1, y1, x2, y2, x3, y3, z;
    std::tie(x1, y1, z) = getPoint(0, 0, depth_mm);
    std::tie(x2, y2, z) = getPoint(0, height_, depth_mm);
    std::tie(x3, y3, z) = getPoint(width_, 0, depth_mm);
    auto d = [](double a, double b, double c, double e) { return std::sqrt((a - c) * (a - c) + (b - e) * (b - e)); };
    return d(x1, y1, x2, y2) * d(x1, y1, x3, y3);
  }
  float getDistance(int depth_mm) {
    double x1, x2, y1, y2, z;
    std::tie(x1, y1, z) = getPoint(100, 100, depth_mm);
    std::tie(x2, y2, z) = getPoint(101, 101, depth_mm);
    return std::sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2));
  }

  // C-ABI view of this camera.
  dmf_camera abi() const {
    dmf_camera c;
    for (int i = 0; i < 9; ++i) c.K[i] = K_[i];
    c.height = height_;
    c.width = width_;
    return c;
  }
};
