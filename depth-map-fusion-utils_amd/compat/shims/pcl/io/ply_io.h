// pcl/io/ply_io.h for the drop-in build: the reference drivers include it but read PCD
// (FileRoutines.hpp:36-47 keeps the PLY path under #if 0); PLYReader reports failure.
#pragma once
#include <string>

#include "../../../dmf_types.hpp"

namespace pcl {
struct PLYReader {
  template <class T>
  int read(const std::string&, PointCloud<T>&) { return -1; }
};
}  // namespace pcl
