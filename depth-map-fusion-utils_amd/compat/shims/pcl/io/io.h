// pcl/io/io.h for the drop-in build.
#pragma once
#include "pcd_io.h"
