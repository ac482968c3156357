// pcl/point_types.h for the drop-in build: point types of dmf_types.hpp.
#pragma once
#include "../../dmf_types.hpp"
