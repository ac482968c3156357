// Algorithms.hpp — drop-in for the set-cover consumer of the reference hot path:
// Algorithms::greedySetCover (include/Algorithms.hpp:38-86) and the driver loop
// setCover (tests/SetCover.cpp:218-240).  The greedy runs on the MI355X over bitmask
// sets (popcount of good & ~covered per candidate); the host only maps set elements
// to bit positions.  Same selection rule as the reference: remaining ids scanned in
// increasing order, strictly largest new-element count wins, stop when nothing is
// new or the best adds fewer than 5.  (The reference's console prints are dropped.)
#pragma once
#include <algorithm>
#include <unordered_map>
#include <vector>

#include "RayTracingEngine.hpp"
#include "Volume.hpp"
#include "dmf.h"

namespace Algorithms {

// greedySetCover over arbitrary host sets; `volume` provides the device and stream.
inline std::vector<unsigned long long int> greedySetCover(VoxelVolume& volume,
                                                          std::vector<std::vector<unsigned long long int>>& candidate_sets,
                                                          double resolution = 0.000008) {
  (void)resolution;  // only feeds the reference's commented-out volume threshold
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
  dmf_volume* v = volume.handle();
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

}  // namespace Algorithms

// tests/SetCover.cpp:218-240: reverseRayTraceFast good sets of every candidate pose,
// then greedySetCover — one batched visibility launch plus the GPU greedy.
inline std::vector<unsigned long long int> setCover(RayTracingEngine engine, VoxelVolume& volume,
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
