// PathPlanning.hpp — drop-in for the collision queries of the reference's camera path
// planners: willCollide (tests/CameraPathGen.cpp:128-156, CameraMotionTSP.cpp:236-261)
// and the V x V TSP cost map built in Planner::run_tsp (tests/CameraPathGen.cpp:310-331,
// CameraMotionTSP.cpp:291-306).  The reference marches 1 mm steps on the host, one
// segment at a time, V*V times; here the whole map is one GPU launch
// (dmf_collision_cost_map).  The reference's console prints are dropped.
#pragma once
#include <climits>
#include <vector>

#include "Volume.hpp"
#include "dmf.h"

namespace PathPlanning {

// tests/CameraPathGen.cpp:56-59
template <class V3>
inline double euclideanDistance(const V3& a, const V3& b) {
  const float d[3] = {a(0) - b(0), a(1) - b(1), a(2) - b(2)};
  return std::sqrt(d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]));
}

// tests/CameraPathGen.cpp:128-156 for one segment a -> b.
template <class V3>
inline bool willCollide(VoxelVolume& volume, const V3& a, const V3& b) {
  const float fa[3] = {a(0), a(1), a(2)}, fb[3] = {b(0), b(1), b(2)};
  uint8_t out = 0;
  dmf_check(dmf_will_collide(volume.handle(), fa, fb, 1, &out));
  return out != 0;
}

// The run_tsp loop: map[i][j] = INT_MAX if willCollide(c_i, c_j) else
// int(euclideanDistance(c_i, c_j) * 1000), c = camera_locations[k] translation.
template <class Pose>
inline std::vector<std::vector<int>> collisionCostMap(VoxelVolume& volume, const std::vector<Pose>& camera_locations) {
  const int32_t V = (int32_t)camera_locations.size();
  std::vector<float> poses(12 * (size_t)V);
  for (int32_t i = 0; i < V; ++i) dmf_compat::pose12(camera_locations[i], &poses[12 * (size_t)i]);
  std::vector<int32_t> flat((size_t)V * V);
  dmf_check(dmf_collision_cost_map(volume.handle(), poses.data(), V, flat.data()));
  std::vector<std::vector<int>> map(V, std::vector<int>(V, 0));
  for (int32_t i = 0; i < V; ++i)
    for (int32_t j = 0; j < V; ++j) map[i][j] = flat[(size_t)i * V + j];
  return map;
}

}  // namespace PathPlanning
