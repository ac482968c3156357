// pcl/point_cloud.h for the drop-in build: PointCloud<T> of dmf_types.hpp.
#pragma once
#include "../../dmf_types.hpp"
