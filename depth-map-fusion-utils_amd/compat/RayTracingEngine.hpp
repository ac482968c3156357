// RayTracingEngine.hpp — drop-in for the reference include/RayTracingEngine.hpp:27-564:
// same class, same eight methods, same default arguments; every trace runs on the
// MI355X through include/dmf.h.  Cheap to copy (holds only the camera), as the
// reference's callers pass it by value (Algorithms.hpp:364, tests/SetCover.cpp:218).
#pragma once
#include <cstdint>
#include <stdexcept>
#include <utility>
#include <vector>

#include "Camera.hpp"
#include "CommonUtilities.hpp"
#include "Volume.hpp"
#include "dmf.h"

constexpr double k_AngleMin = 0;
constexpr double k_AngleMax = 90;
constexpr double k_ZMin = 0.20;
constexpr double k_ZMax = 1.0;

class RayTracingEngine {
 public:
  Camera cam_;
  explicit RayTracingEngine(Camera& cam) : cam_(cam) {}

  // RayTracingEngine.hpp:45-134
  std::pair<bool, std::vector<unsigned long long int>> reverseRayTrace(VoxelVolume& volume, Eigen::Affine3f T,
                                                                       bool viz, int zdelta = 1) {
    return reverse(volume, T, viz, false);
  }
  // RayTracingEngine.hpp:136-226
  std::pair<bool, std::vector<unsigned long long int>> reverseRayTraceFast(VoxelVolume& volume, Eigen::Affine3f T,
                                                                           bool viz, int zdelta = 1) {
    return reverse(volume, T, viz, true);
  }
  // Batched extension: P poses in one launch (the set-cover loop of tests/SetCover.cpp:218-240).
  std::vector<std::pair<bool, std::vector<unsigned long long int>>> reverseRayTraceFastBatch(
      VoxelVolume& volume, const std::vector<Eigen::Affine3f>& poses, bool viz) {
    std::vector<float> p(12 * poses.size());
    for (size_t i = 0; i < poses.size(); ++i) dmf_compat::pose12(poses[i], &p[12 * i]);
    const int P = (int)poses.size();
    std::vector<uint8_t> found(P);
    std::vector<int64_t> counts(P);
    std::vector<uint64_t> out(volume.occupied_cells_.size() * (size_t)P / 2 + 64);
    const dmf_camera c = cam_.abi();
    int st = dmf_reverse_ray_trace_fast(volume.handle(), &c, p.data(), P, viz, found.data(), counts.data(),
                                        out.data(), (int64_t)out.size());
    if (st == DMF_ERR_CAPACITY) {
      int64_t tot = 0;
      for (auto n : counts) tot += n;
      out.resize((size_t)tot);
      st = dmf_reverse_ray_trace_fast(volume.handle(), &c, p.data(), P, viz, found.data(), counts.data(), out.data(),
                                      tot);
    }
    dmf_check(st);
    if (viz) volume.touch();
    std::vector<std::pair<bool, std::vector<unsigned long long int>>> res(P);
    size_t o = 0;
    for (int i = 0; i < P; ++i) {
      res[i].first = found[i] != 0;
      res[i].second.assign(out.begin() + o, out.begin() + o + counts[i]);
      o += counts[i];
    }
    return res;
  }
  // Extension (BASELINE.json north_star; no reference counterpart): 3D-DDA
  // log-odds fusion of P depth frames -- the per-frame back-project + integrate loop of
  // tests/Raytracing.cpp:70-76 / Volume.hpp:199-228 as one GPU call.  depth: P frames of
  // cam_ height x width uint16 millimetres (row-major), poses: the frames' camera -> world
  // transforms; hit / miss counts accumulate into `acc` (x-major over the volume's grid,
  // sized on first use).  dmf_fuse_depth in include/dmf.h.
  struct FusionCounts {
    std::vector<int32_t> hits, misses;  // per voxel, x-major (the reference's voxel order)
    int64_t updates = 0, rays = 0, hit_rays = 0;
  };
  FusionCounts& fuseDepth(VoxelVolume& volume, const std::vector<uint16_t>& depth,
                          const std::vector<Eigen::Affine3f>& poses, FusionCounts& acc,
                          const dmf_fuse_params* params = nullptr) {
    const size_t P = poses.size(), HW = (size_t)cam_.getHeight() * (size_t)cam_.getWidth();
    if (depth.size() != P * HW) throw std::invalid_argument("fuseDepth: depth must hold P frames of height x width");
    const size_t n = (size_t)volume.xdim_ * volume.ydim_ * volume.zdim_;
    if (acc.hits.size() != n) acc.hits.assign(n, 0);
    if (acc.misses.size() != n) acc.misses.assign(n, 0);
    std::vector<float> p(12 * P);
    for (size_t i = 0; i < P; ++i) dmf_compat::pose12(poses[i], &p[12 * i]);
    dmf_fuse_params prm;
    dmf_fuse_params_default(&prm);
    if (params) prm = *params;
    const dmf_camera c = cam_.abi();
    int64_t st[3] = {0, 0, 0};
    dmf_check(dmf_fuse_depth(volume.handle(), &c, depth.data(), p.data(), (int32_t)P, &prm, acc.hits.data(),
                             acc.misses.data(), st));
    acc.updates += st[0];
    acc.rays += st[1];
    acc.hit_rays += st[2];
    return acc;
  }
  // The clamped int16 log-odds grid of fused counts (x-major): clamp(hits * l_hit + misses *
  // l_miss, l_min, l_max) milli-logit (dmf_fuse_finalize).
  std::vector<int16_t> logOdds(VoxelVolume& volume, const FusionCounts& acc, const dmf_fuse_params* params = nullptr) {
    dmf_fuse_params prm;
    dmf_fuse_params_default(&prm);
    if (params) prm = *params;
    std::vector<int16_t> out(acc.hits.size());
    dmf_check(dmf_fuse_finalize(volume.handle(), acc.hits.data(), acc.misses.data(), &prm, out.data()));
    return out;
  }

  // RayTracingEngine.hpp:229-264
  int rayTraceAndGetMinimum(VoxelVolume& volume, Eigen::Affine3f& T, int zdelta = 1, bool sparse = true) {
    float p[12];
    dmf_compat::pose12(T, p);
    const dmf_camera c = cam_.abi();
    int32_t m = -1;
    dmf_check(dmf_ray_trace_and_get_minimum(volume.handle(), &c, p, zdelta, sparse, &m));
    return m;
  }
  // RayTracingEngine.hpp:268-309
  void rayTrace(VoxelVolume& volume, Eigen::Affine3f& T, int zdelta = 10, bool sparse = true) {
    float p[12];
    dmf_compat::pose12(T, p);
    const dmf_camera c = cam_.abi();
    dmf_check(dmf_ray_trace(volume.handle(), &c, p, zdelta, sparse));
    volume.touch();
  }
  // RayTracingEngine.hpp:311-375
  void rayTraceAndClassify(VoxelVolume& volume, Eigen::Affine3f& T, int zdelta = 10, int view = 1,
                           bool sparse = true) {
    float p[12];
    dmf_compat::pose12(T, p);
    const dmf_camera c = cam_.abi();
    dmf_check(dmf_ray_trace_and_classify(volume.handle(), &c, p, zdelta, view, sparse));
    volume.touch();
  }
  // RayTracingEngine.hpp:377-445
  std::pair<bool, std::vector<unsigned long long int>> rayTraceAndGetGoodPoints(VoxelVolume& volume,
                                                                                Eigen::Affine3f& T, int zdelta = 10,
                                                                                bool sparse = true) {
    return fwd_list(volume, T, zdelta, sparse, true);
  }
  // RayTracingEngine.hpp:447-494
  std::pair<bool, std::vector<unsigned long long int>> rayTraceAndGetPoints(VoxelVolume& volume, Eigen::Affine3f& T,
                                                                            int zdelta = 10, bool sparse = true) {
    return fwd_list(volume, T, zdelta, sparse, false);
  }
  // RayTracingEngine.hpp:498-564
  void rayTraceVolume(VoxelVolume& volume, Eigen::Affine3f& T) {
    float p[12];
    dmf_compat::pose12(T, p);
    const dmf_camera c = cam_.abi();
    dmf_check(dmf_ray_trace_volume(volume.handle(), &c, p, nullptr));
    volume.touch();
  }

 private:
  std::pair<bool, std::vector<unsigned long long int>> reverse(VoxelVolume& volume, const Eigen::Affine3f& T, bool viz,
                                                               bool fast) {
    float p[12];
    dmf_compat::pose12(T, p);
    const dmf_camera c = cam_.abi();
    uint8_t found = 0;
    int64_t count = 0;
    std::vector<uint64_t> out(volume.occupied_cells_.size() + 64);
    auto call = [&](int64_t cap) {
      return fast ? dmf_reverse_ray_trace_fast(volume.handle(), &c, p, 1, viz, &found, &count, out.data(), cap)
                  : dmf_reverse_ray_trace(volume.handle(), &c, p, 1, viz, &found, &count, out.data(), cap);
    };
    int st = call((int64_t)out.size());
    if (st == DMF_ERR_CAPACITY) {
      out.resize((size_t)count);
      st = call(count);
    }
    dmf_check(st);
    if (viz) volume.touch();
    return {found != 0, std::vector<unsigned long long int>(out.begin(), out.begin() + count)};
  }
  std::pair<bool, std::vector<unsigned long long int>> fwd_list(VoxelVolume& volume, Eigen::Affine3f& T, int zdelta,
                                                                bool sparse, bool good) {
    float p[12];
    dmf_compat::pose12(T, p);
    const dmf_camera c = cam_.abi();
    uint8_t found = 0;
    int64_t n = 0;
    std::vector<uint64_t> out(1 << 16);
    auto call = [&](int64_t cap) {
      return good ? dmf_ray_trace_and_get_good_points(volume.handle(), &c, p, zdelta, sparse, &found, out.data(), cap, &n)
                  : dmf_ray_trace_and_get_points(volume.handle(), &c, p, zdelta, sparse, &found, out.data(), cap, &n);
    };
    int st = call((int64_t)out.size());
    if (st == DMF_ERR_CAPACITY) {
      out.resize((size_t)n);
      st = call(n);
    }
    dmf_check(st);
    return {found != 0, std::vector<unsigned long long int>(out.begin(), out.begin() + n)};
  }
};
