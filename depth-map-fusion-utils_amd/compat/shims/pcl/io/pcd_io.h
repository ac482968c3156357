// pcl/io/pcd_io.h for the drop-in build: loadPCDFile for the PCD v0.7 files the reference
// drivers read (FileRoutines.hpp:33-67): DATA ascii or binary, any field order among
// x y z rgb/rgba normal_x normal_y normal_z curvature (other fields are skipped; binary
// fields of TYPE F/U/I and SIZE 1/2/4/8).  binary_compressed is not supported (returns -1).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../../dmf_types.hpp"

namespace pcl {
namespace io {
namespace detail {
struct PcdField {
  std::string name;
  int size = 4, count = 1;
  char type = 'F';
};
inline double pcd_value(const char* p, const PcdField& f) {
  switch (f.type) {
    case 'F': if (f.size == 8) { double d; std::memcpy(&d, p, 8); return d; } else { float v; std::memcpy(&v, p, 4); return v; }
    case 'U': {
      uint64_t v = 0;
      std::memcpy(&v, p, (size_t)f.size);
      return (double)v;
    }
    default: {
      int64_t v = 0;
      std::memcpy(&v, p, (size_t)f.size);
      const int sh = 64 - 8 * f.size;
      return (double)((v << sh) >> sh);
    }
  }
}
}  // namespace detail

template <typename PointT>
int loadPCDFile(const std::string& file, PointCloud<PointT>& cloud) {
  std::ifstream in(file, std::ios::binary);
  if (!in) return -1;
  std::vector<detail::PcdField> fields;
  size_t points = 0;
  std::string line, data;
  while (std::getline(in, line)) {
    if (line.empty() || line[0] == '#') continue;
    std::istringstream ss(line);
    std::string key;
    ss >> key;
    if (key == "FIELDS") {
      std::string n;
      while (ss >> n) fields.push_back(detail::PcdField{n});
    } else if (key == "SIZE") {
      for (auto& f : fields) ss >> f.size;
    } else if (key == "TYPE") {
      for (auto& f : fields) ss >> f.type;
    } else if (key == "COUNT") {
      for (auto& f : fields) ss >> f.count;
    } else if (key == "POINTS") {
      ss >> points;
    } else if (key == "DATA") {
      ss >> data;
      break;
    }
  }
  if (fields.empty() || (data != "ascii" && data != "binary")) return -1;
  // untrusted header: TYPE F is 4 or 8 bytes, U / I 1, 2, 4 or 8; COUNT >= 1 (and bounded,
  // so the record stride cannot overflow)
  for (const auto& f : fields) {
    const bool ok_size = f.type == 'F' ? (f.size == 4 || f.size == 8)
                                       : ((f.type == 'U' || f.type == 'I') &&
                                          (f.size == 1 || f.size == 2 || f.size == 4 || f.size == 8));
    if (!ok_size || f.count < 1 || f.count > (1 << 20)) return -1;
  }
  cloud.points.assign(points, PointT());
  cloud.is_dense = true;
  size_t stride = 0;
  for (auto& f : fields) stride += (size_t)f.size * f.count;
  std::vector<char> rec(stride);
  for (size_t i = 0; i < points; ++i) {
    std::vector<double> vals;
    if (data == "ascii") {
      if (!std::getline(in, line)) return -1;
      std::istringstream ss(line);
      for (auto& f : fields)
        for (int c = 0; c < f.count; ++c) {
          std::string tok;
          ss >> tok;
          double v;
          if (f.name == "rgb" || f.name == "rgba") {  // packed colour: float bits or integer
            if (tok.find_first_of(".eE") != std::string::npos || f.type == 'F') {
              float fv = std::strtof(tok.c_str(), nullptr);
              uint32_t u;
              std::memcpy(&u, &fv, 4);
              v = (double)u;
            } else {
              v = (double)std::strtoull(tok.c_str(), nullptr, 10);
            }
          } else {
            v = std::strtod(tok.c_str(), nullptr);
          }
          vals.push_back(v);
        }
    } else {
      if (!in.read(rec.data(), (std::streamsize)stride)) return -1;
      size_t off = 0;
      for (auto& f : fields)
        for (int c = 0; c < f.count; ++c, off += (size_t)f.size) {
          if ((f.name == "rgb" || f.name == "rgba") && f.size == 4) {
            uint32_t u;
            std::memcpy(&u, rec.data() + off, 4);
            vals.push_back((double)u);
          } else {
            vals.push_back(detail::pcd_value(rec.data() + off, f));
          }
        }
    }
    size_t k = 0;
    PointT& p = cloud.points[i];
    for (auto& f : fields)
      for (int c = 0; c < f.count; ++c, ++k) dmf_compat::set_field(p, f.name, vals[k]);
    if (!(std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z))) cloud.is_dense = false;
  }
  cloud.width = (uint32_t)points;
  cloud.height = 1;
  return 0;
}
}  // namespace io
}  // namespace pcl
