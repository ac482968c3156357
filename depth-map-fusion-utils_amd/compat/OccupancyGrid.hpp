// OccupancyGrid.hpp — drop-in for the reference include/OccupancyGrid.hpp:50-318 class
// API (setDimensions, setResolution, setK, construct, updateStates, downloadCloud,
// downloadHQCloud, downloadReorganizedCloud) backed by dmf_ogrid_* on the MI355X.
// updateStates returns the deterministic single-threaded result of the reference's OpenMP
// loops.  The dense per-voxel state is on the device (state() copies it); the reference's
// public voxels_ / voxels_reorganized_ containers are not mirrored.  (The per-voxel struct is not named Voxel here: the reference's two
// headers cannot be included together, this compat set can.)
#pragma once
#include <vector>

#include "dmf.h"
#include "dmf_types.hpp"
#include "Volume.hpp"  // dmf_check

class OccupancyGrid {
 public:
  double xmin_ = 0, xmax_ = 0, ymin_ = 0, ymax_ = 0, zmin_ = 0, zmax_ = 0;
  double xres_ = 0, yres_ = 0, zres_ = 0;
  double xcenter_ = 0, ycenter_ = 0, zcenter_ = 0;
  int xdim_ = 0, ydim_ = 0, zdim_ = 0;
  int k_ = 0;

  explicit OccupancyGrid(int device = 0) { dmf_check(dmf_ogrid_create(&h_, device)); }
  ~OccupancyGrid() { dmf_ogrid_destroy(h_); }
  OccupancyGrid(const OccupancyGrid&) = delete;
  OccupancyGrid& operator=(const OccupancyGrid&) = delete;

  // :323-336
  void setDimensions(double xmin, double xmax, double ymin, double ymax, double zmin, double zmax) {
    xmin_ = xmin; xmax_ = xmax; ymin_ = ymin; ymax_ = ymax; zmin_ = zmin; zmax_ = zmax;
    xcenter_ = xmin_ + (xmax_ - xmin_) / 2.0;
    ycenter_ = ymin_ + (ymax_ - ymin_) / 2.0;
    zcenter_ = zmin_ + (zmax_ - zmin_) / 2.0;
  }
  // :338-343 (float parameters, stored as double)
  void setResolution(float x, float y, float z) { xres_ = x; yres_ = y; zres_ = z; }
  void setK(int k) { k_ = k; }
  // :345-352
  bool construct() {
    const double b[6] = {xmin_, xmax_, ymin_, ymax_, zmin_, zmax_};
    dmf_check(dmf_ogrid_setup(h_, b, (float)xres_, (float)yres_, (float)zres_, k_));
    int32_t d[3];
    dmf_check(dmf_ogrid_get_dims(h_, d));
    xdim_ = d[0]; ydim_ = d[1]; zdim_ = d[2];
    return true;
  }
  // :99-164
  template <class CloudPtr, class NormalPtr>
  bool updateStates(CloudPtr cloud, NormalPtr normals) {
    std::vector<float> c(3 * cloud->points.size()), n(6 * normals->points.size());
    for (size_t i = 0; i < cloud->points.size(); ++i) {
      c[3 * i] = cloud->points[i].x; c[3 * i + 1] = cloud->points[i].y; c[3 * i + 2] = cloud->points[i].z;
    }
    for (size_t i = 0; i < normals->points.size(); ++i) {
      const auto& p = normals->points[i];
      n[6 * i] = p.x; n[6 * i + 1] = p.y; n[6 * i + 2] = p.z;
      n[6 * i + 3] = p.normal[0]; n[6 * i + 4] = p.normal[1]; n[6 * i + 5] = p.normal[2];
    }
    dmf_check(dmf_ogrid_update_states(h_, c.data(), (int64_t)cloud->points.size(), n.data(),
                                      (int64_t)normals->points.size()));
    return true;
  }
  // :166-193 / :283-318
  template <class OutPtr>
  bool downloadCloud(OutPtr cloud) { return download(cloud, 0); }
  template <class OutPtr>
  bool downloadHQCloud(OutPtr cloud) { return download(cloud, 1); }
  // :200-286 (modes 2 / 3 of dmf_ogrid_download: the merged voxels, x-major)
  template <class OutPtr>
  bool downloadReorganizedCloud(OutPtr cloud, bool clean = false) { return download(cloud, clean ? 3 : 2); }

  dmf_ogrid* handle() { return h_; }

 private:
  template <class OutPtr>
  bool download(OutPtr cloud, int mode) {
    if (!cloud) return false;
    int64_t n = 0;
    const int st = dmf_ogrid_download(h_, mode, nullptr, 0, &n);
    if (st != DMF_OK && st != DMF_ERR_CAPACITY) dmf_check(st);
    std::vector<float> buf(6 * (size_t)n);
    if (n) dmf_check(dmf_ogrid_download(h_, mode, buf.data(), n, &n));
    for (int64_t i = 0; i < n; ++i) {
      typename std::decay<decltype(cloud->points[0])>::type pt;
      pt.x = buf[6 * i]; pt.y = buf[6 * i + 1]; pt.z = buf[6 * i + 2];
      pt.r = 0; pt.g = 0; pt.b = 0;
      pt.normal[0] = buf[6 * i + 3]; pt.normal[1] = buf[6 * i + 4]; pt.normal[2] = buf[6 * i + 5];
      cloud->points.push_back(pt);
    }
    return true;
  }
  dmf_ogrid* h_ = nullptr;
};
