// PointCloudProcessing.hpp — drop-in for the reference include/PointCloudProcessing.hpp:34-40
// downsample (pcl::VoxelGrid with a cubic leaf; compat pcl/filters/voxel_grid.h).
#pragma once
#include <pcl/filters/voxel_grid.h>
#include <pcl/point_cloud.h>

namespace PointCloudProcessing {
template <typename PointT>
void downsample(typename pcl::PointCloud<PointT>::Ptr cloud, typename pcl::PointCloud<PointT>::Ptr cloud_filtered,
                double leaf) {
  pcl::VoxelGrid<PointT> sor;
  sor.setLeafSize((float)leaf, (float)leaf, (float)leaf);
  sor.setInputCloud(cloud);
  sor.filter(*cloud_filtered);
}
}  // namespace PointCloudProcessing
