// pcl/visualization/cloud_viewer.h for the drop-in build (headless).
#pragma once
#include "pcl_visualizer.h"
