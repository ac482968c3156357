// pcl/filters/voxel_grid.h for the drop-in build: VoxelGrid<PointT> restated from PCL
// (filters/impl/voxel_grid.hpp applyFilter): float inverse leaf size, leaf coordinates
// floor(p * inv) - min_b over the cloud's finite bounding box, points ordered by leaf
// index (stable for equal indices), one output point per non-empty leaf, in increasing
// leaf order, holding the float mean of every field (downsample_all_data_).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../common/common.h"

namespace pcl {
template <typename PointT>
class VoxelGrid {
  float leaf_[3] = {1.f, 1.f, 1.f};
  typename PointCloud<PointT>::Ptr in_;

 public:
  void setLeafSize(float lx, float ly, float lz) { leaf_[0] = lx; leaf_[1] = ly; leaf_[2] = lz; }
  void setInputCloud(const typename PointCloud<PointT>::Ptr& c) { in_ = c; }
  void filter(PointCloud<PointT>& out) {
    out.points.clear();
    if (!in_ || in_->points.empty()) { out.width = 0; out.height = 1; return; }
    const float inv[3] = {1.0f / leaf_[0], 1.0f / leaf_[1], 1.0f / leaf_[2]};
    PointT mnp, mxp;
    getMinMax3D(*in_, mnp, mxp);
    const int min_b[3] = {(int)std::floor(mnp.x * inv[0]), (int)std::floor(mnp.y * inv[1]), (int)std::floor(mnp.z * inv[2])};
    const int max_b[3] = {(int)std::floor(mxp.x * inv[0]), (int)std::floor(mxp.y * inv[1]), (int)std::floor(mxp.z * inv[2])};
    const int64_t div0 = max_b[0] - min_b[0] + 1, div1 = max_b[1] - min_b[1] + 1;
    std::vector<std::pair<int64_t, size_t>> idx;
    idx.reserve(in_->points.size());
    for (size_t i = 0; i < in_->points.size(); ++i) {
      const PointT& p = in_->points[i];
      if (!(std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z))) continue;
      const int64_t i0 = (int64_t)std::floor(p.x * inv[0]) - min_b[0];
      const int64_t i1 = (int64_t)std::floor(p.y * inv[1]) - min_b[1];
      const int64_t i2 = (int64_t)std::floor(p.z * inv[2]) - min_b[2];
      idx.emplace_back(i0 + i1 * div0 + i2 * div0 * div1, i);
    }
    std::stable_sort(idx.begin(), idx.end(),
                     [](const std::pair<int64_t, size_t>& a, const std::pair<int64_t, size_t>& b) { return a.first < b.first; });
    for (size_t s = 0; s < idx.size();) {
      size_t e = s;
      while (e < idx.size() && idx[e].first == idx[s].first) ++e;
      out.points.push_back(dmf_compat::mean_point(in_->points, idx, s, e));
      s = e;
    }
    out.width = (uint32_t)out.points.size();
    out.height = 1;
  }
};
}  // namespace pcl
