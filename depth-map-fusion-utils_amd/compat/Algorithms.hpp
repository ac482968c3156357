// Algorithms.hpp — drop-in for the set-cover consumer of the reference hot path:
// Algorithms::greedySetCover (include/Algorithms.hpp:38-86; the driver loop of
// tests/SetCover.cpp:218-240 batched as dmf_compat::setCoverBatched), and the camera
// placement the reference drivers call (positionCameras, :114-122, 189-298).  The greedy runs on the MI355X over bitmask
// sets (popcount of good & ~covered per candidate); the host only maps set elements
// to bit positions.  Same selection rule as the reference: remaining ids scanned in
// increasing order, strictly largest new-element count wins, stop when nothing is
// new or the best adds fewer than 5.  (The reference's console prints are dropped.)
#pragma once
#include <algorithm>
#include <cassert>
#include <memory>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "RayTracingEngine.hpp"
#include "Volume.hpp"
#include "dmf.h"

namespace dmf_compat {
// A constructed 1-cell volume on device 0 for engine calls that the reference makes
// without a volume (greedySetCover): it only supplies the device and stream.
inline dmf_volume* service_volume() {
  static std::unique_ptr<dmf_volume, int (*)(dmf_volume*)> h(
      [] {
        dmf_volume* v = nullptr;
        dmf_check(dmf_volume_create(&v, 0));
        dmf_check(dmf_volume_set_dimensions(v, 0, 1, 0, 1, 0, 1));
        dmf_check(dmf_volume_set_volume_size(v, 1, 1, 1));
        dmf_check(dmf_volume_construct(v));
        return v;
      }(),
      dmf_volume_destroy);
  return h.get();
}
}  // namespace dmf_compat

namespace Algorithms {

// greedySetCover over arbitrary host sets on the device of `v`.
inline std::vector<unsigned long long int> greedySetCoverOn(dmf_volume* v,
                                                            std::vector<std::vector<unsigned long long int>>& candidate_sets) {
  std::unordered_map<unsigned long long int, int64_t> bit;
  for (auto& s : candidate_sets)
    for (auto h : s) bit.emplace(h, (int64_t)bit.size());
  const int32_t P = (int32_t)candidate_sets.size();
  const int64_t words = ((int64_t)bit.size() + 63) / 64;
  std::vector<uint64_t> masks((size_t)P * std::max<int64_t>(words, 1), 0);
  for (int32_t p = 0; p < P; ++p)
    for (auto h : candidate_sets[p]) {
      const int64_t i = bit[h];
      masks[(size_t)p * words + i / 64] |= 1ull << (i % 64);
    }
  void* d = nullptr;
  dmf_check(dmf_device_malloc(v, &d, sizeof(uint64_t) * masks.size()));
  std::vector<int32_t> sel(std::max(P, 1));
  int32_t n = 0;
  int st = dmf_memcpy_h2d(v, d, masks.data(), sizeof(uint64_t) * masks.size());
  if (st == DMF_OK) st = dmf_greedy_set_cover_masks_device(v, (const uint64_t*)d, P, words, 5, sel.data(), &n);
  dmf_device_free(v, d);
  dmf_check(st);
  return std::vector<unsigned long long int>(sel.begin(), sel.begin() + n);
}

// Algorithms.hpp:38-86, the reference signature (device 0)
inline std::vector<unsigned long long int> greedySetCover(std::vector<std::vector<unsigned long long int>>& candidate_sets,
                                                          double resolution = 0.000008) {
  (void)resolution;  // only feeds the reference's commented-out volume threshold
  return greedySetCoverOn(dmf_compat::service_volume(), candidate_sets);
}

// Extension: the same on `volume`'s device and stream.
inline std::vector<unsigned long long int> greedySetCover(VoxelVolume& volume,
                                                          std::vector<std::vector<unsigned long long int>>& candidate_sets,
                                                          double resolution = 0.000008) {
  (void)resolution;
  return greedySetCoverOn(volume.handle(), candidate_sets);
}

// ---- camera placement used by the reference drivers (Algorithms.hpp:114-122, 189-298) ----
// Not on the hot path; restated so tests/Raytracing.cpp:80-81 builds and runs unchanged.

// :114-122 movePointAway: pi + (float)distance * nor, summed in double
inline std::vector<double> movePointAway(std::vector<double> pi, std::vector<double> nor, double distance) {
  Eigen::Vector3f n(3);
  n << nor[0], nor[1], nor[2];
  n = n * distance;
  return {n(0) + pi[0], n(1) + pi[1], n(2) + pi[2]};
}

// :189-234 positionCamera(locations, id, distance): the camera `distance` mm out along the
// location's normal, looking back along it (z = -normal), with the reference's fixed
// x = (0, -1, 0), y = (1, 0, 0) columns (its computed orthogonal x, y are overwritten).
inline Eigen::Affine3f positionCamera(pcl::PointCloud<pcl::PointXYZRGBNormal>::Ptr locations, int id,
                                      unsigned int distance = 300) {
  const pcl::PointXYZRGBNormal pt = locations->points[id];
  Eigen::Vector3f nor(3);
  nor << pt.normal[0], pt.normal[1], pt.normal[2];
  const std::vector<double> normals = {nor(0), nor(1), nor(2)};
  nor = nor * -1;
  const std::vector<double> np = movePointAway({pt.x, pt.y, pt.z}, normals, double(distance) / 1000.0);
  const Eigen::Vector3f x(0, -1, 0), y(1, 0, 0);
  Eigen::Affine3f Q = Eigen::Affine3f::Identity();
  for (int i = 0; i < 3; i++) {
    Q(i, 0) = x(i);
    Q(i, 1) = y(i);
    Q(i, 2) = nor(i);
    Q(i, 3) = (float)np[i];
  }
  return Q;
}

// :236-279 positionCamera(location): camera AT the location, z = -normal, x orthogonal to
// it from the first non-zero normal component, y = z x x
inline Eigen::Affine3f positionCamera(pcl::PointXYZRGBNormal location) {
  Eigen::Vector3f nor(3);
  nor << location.normal[0], location.normal[1], location.normal[2];
  nor = nor * -1;
  Eigen::Vector3f x(3);
  if (nor(2) != 0.0) {
    x << 1, 1, 0;
    x(2) = -(nor(0) + nor(1)) / nor(2);
  } else if (nor(1) != 0) {
    x << 1, 0, 1;
    x(1) = -(nor(0) + nor(2)) / nor(1);
  } else if (nor(0) != 0) {
    x << 0, 1, 1;
    x(0) = -(nor(1) + nor(2)) / nor(0);
  }
  x = x.normalized();
  const Eigen::Vector3f y = nor.cross(x);
  Eigen::Affine3f Q = Eigen::Affine3f::Identity();
  for (int i = 0; i < 3; i++) {
    Q(i, 0) = x(i);
    Q(i, 1) = y(i);
    Q(i, 2) = nor(i);
  }
  Q(0, 3) = location.x;
  Q(1, 3) = location.y;
  Q(2, 3) = location.z;
  return Q;
}

// :281-298 positionCameras: normals with z <= 0 are flipped IN the locations cloud first
inline std::vector<Eigen::Affine3f> positionCameras(pcl::PointCloud<pcl::PointXYZRGBNormal>::Ptr locations,
                                                    unsigned int distance = 300) {
  std::vector<Eigen::Affine3f> cameras;
  for (size_t i = 0; i < locations->points.size(); i++) {
    if (locations->points[i].normal[2] <= 0)
      for (int a = 0; a < 3; ++a) locations->points[i].normal[a] *= -1;
    cameras.push_back(positionCamera(locations, (int)i, distance));
  }
  return cameras;
}
}  // namespace Algorithms

// The loop of tests/SetCover.cpp:218-240 (reverseRayTraceFast good sets of every
// candidate pose, then greedySetCover) as ONE batched visibility launch plus the GPU
// greedy.  (The reference defines setCover in its driver, so the drop-in does not.)
namespace dmf_compat {
inline std::vector<unsigned long long int> setCoverBatched(RayTracingEngine engine, VoxelVolume& volume,
                                                    std::vector<Eigen::Affine3f> camera_locations,
                                                    int resolution_single_dimension = 0, bool sparse = true) {
  (void)resolution_single_dimension;
  (void)sparse;
  std::vector<float> poses(12 * camera_locations.size());
  for (size_t i = 0; i < camera_locations.size(); ++i) dmf_compat::pose12(camera_locations[i], &poses[12 * i]);
  const dmf_camera c = engine.cam_.abi();
  std::vector<int32_t> sel(std::max<size_t>(camera_locations.size(), 1));
  int32_t n = 0;
  dmf_check(dmf_greedy_set_cover(volume.handle(), &c, poses.data(), (int32_t)camera_locations.size(), 5, sel.data(),
                                 &n));
  volume.touch();
  return std::vector<unsigned long long int>(sel.begin(), sel.begin() + n);
}
}  // namespace dmf_compat
