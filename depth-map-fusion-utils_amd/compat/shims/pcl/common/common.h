// pcl/common/common.h for the drop-in build: getMinMax3D (pcl/common/impl/common.hpp),
// the per-axis float min / max over the cloud, skipping non-finite points when the cloud
// is not dense.
#pragma once
#include <cfloat>
#include <cmath>

#include "../../../dmf_types.hpp"

namespace pcl {
template <typename PointT>
inline void getMinMax3D(const PointCloud<PointT>& cloud, PointT& min_pt, PointT& max_pt) {
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (const PointT& p : cloud.points) {
    const float v[3] = {p.x, p.y, p.z};
    if (!cloud.is_dense && !(std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]))) continue;
    for (int a = 0; a < 3; ++a) {
      mn[a] = std::fmin(mn[a], v[a]);
      mx[a] = std::fmax(mx[a], v[a]);
    }
  }
  min_pt.x = mn[0]; min_pt.y = mn[1]; min_pt.z = mn[2];
  max_pt.x = mx[0]; max_pt.y = mx[1]; max_pt.z = mx[2];
}
}  // namespace pcl
