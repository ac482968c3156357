// Volume.hpp — drop-in for the reference include/Volume.hpp:29-255 over the MI355X
// engine.  Same struct Voxel, same VoxelVolume member functions and public fields.
//
// The grid lives on the GPU (flat occupancy bitmask + slot map + CSR points/normals,
// DESIGN.md §6).  The public fields the reference's callers read directly are kept in
// sync: the geometry fields after every setup call, occupied_cells_ after every
// integration, and voxels_[x][y][z] (Voxel*) through a host mirror that is rebuilt
// lazily from the device whenever the device state changed (engine calls with viz
// flags, integration).  Copying is disabled, as a copy of the reference double-frees.
#pragma once
#include <cmath>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "dmf.h"
#include "dmf_types.hpp"

// Volume.hpp:29-48
struct Voxel {
  std::vector<pcl::PointXYZRGB> pts;
  std::vector<pcl::Normal> normals;
  int view = 0;
  bool good = false;
  Voxel() = default;
  explicit Voxel(pcl::PointXYZRGB pt) { pts.push_back(pt); }
  Voxel(pcl::PointXYZRGB pt, pcl::Normal n) { pts.push_back(pt); normals.push_back(n); }
};

inline void dmf_check(int status) {
  if (status != DMF_OK) throw std::runtime_error(std::string("dmf: ") + dmf_status_string(status) + ": " + dmf_last_error());
}

class VoxelVolume {
 public:
  // Volume.hpp:54-61 public fields
  std::vector<unsigned long long int> occupied_cells_;
  double xmin_ = 0, xmax_ = 0, ymin_ = 0, ymax_ = 0, zmin_ = 0, zmax_ = 0;
  double xcenter_ = 0, ycenter_ = 0, zcenter_ = 0;
  double xdelta_ = 0, ydelta_ = 0, zdelta_ = 0;
  double voxel_size_ = 0;
  int xdim_ = 0, ydim_ = 0, zdim_ = 0;
  unsigned long long int hsize_ = 0;

  // voxels_[x][y][z] -> Voxel* (nullptr if empty), served from the lazily rebuilt mirror
  struct ZRow {
    VoxelVolume* v;
    int x, y;
    Voxel* operator[](int z) const { return v->mirror_at(x, y, z); }
  };
  struct YRow {
    VoxelVolume* v;
    int x;
    ZRow operator[](int y) const { return ZRow{v, x, y}; }
  };
  struct Grid {
    VoxelVolume* v;
    YRow operator[](int x) const { return YRow{v, x}; }
  } voxels_{this};

  explicit VoxelVolume(int device = 0) { dmf_check(dmf_volume_create(&h_, device)); }
  ~VoxelVolume() { dmf_volume_destroy(h_); }
  VoxelVolume(const VoxelVolume&) = delete;
  VoxelVolume& operator=(const VoxelVolume&) = delete;

  // Volume.hpp:89-128
  void setDimensions(double xmin, double xmax, double ymin, double ymax, double zmin, double zmax) {
    dmf_check(dmf_volume_set_dimensions(h_, xmin, xmax, ymin, ymax, zmin, zmax));
    pull_info();
  }
  void setResolution(double xdelta, double ydelta, double zdelta) {
    dmf_check(dmf_volume_set_resolution(h_, xdelta, ydelta, zdelta));
    pull_info();
  }
  void setVolumeSize(int xdim, int ydim, int zdim) {
    dmf_check(dmf_volume_set_volume_size(h_, xdim, ydim, zdim));
    pull_info();
  }
  bool constructVolume() {
    dmf_check(dmf_volume_construct(h_));
    pull_info();
    occupied_cells_.clear();
    touch();
    return true;
  }
  template <typename PointT>
  bool addPointCloud(typename pcl::PointCloud<PointT>::Ptr) { return true; }  // Volume.hpp:130-133 stub

  // Volume.hpp:135-170 helpers (host formulas)
  unsigned long long int getHash(float x, float y, float z) {
    int a, b, c;
    std::tie(a, b, c) = getVoxel(x, y, z);
    return getHashId(a, b, c);
  }
  unsigned long long int getHashId(int x, int y, int z) {
    unsigned long long int hash = x;
    return (hash << 40) ^ (unsigned long long int)(long long)(y << 20) ^ (unsigned long long int)(long long)z;
  }
  std::tuple<int, int, int> getVoxel(float x, float y, float z) {
    return std::make_tuple((int)std::floor((x - xmin_) / xdelta_), (int)std::floor((y - ymin_) / ydelta_),
                           (int)std::floor((z - zmin_) / zdelta_));
  }
  std::tuple<int, int, int> getVoxelCoords(unsigned long long int id) {
    const unsigned long long int mask = (1 << 20) - 1;
    return std::make_tuple((int)(id >> 40), (int)(id >> 20 & mask), (int)(id & mask));
  }
  bool validCoords(int x, int y, int z) { return x < xdim_ && y < ydim_ && z < zdim_ && x >= 0 && y >= 0 && z >= 0; }
  bool validPoints(float x, float y, float z) {
    return !(x >= xmax_ || y >= ymax_ || z >= zmax_ || x <= xmin_ || y <= ymin_ || z <= zmin_);
  }

  // Volume.hpp:172-197 / 199-228 — binning on the GPU
  bool integratePointCloud(pcl::PointCloud<pcl::PointXYZRGB>::Ptr cloud) { return integrate(cloud, nullptr); }
  bool integratePointCloud(pcl::PointCloud<pcl::PointXYZRGB>::Ptr cloud, pcl::PointCloud<pcl::Normal>::Ptr normals) {
    return integrate(cloud, normals.get());
  }

  // Volume.hpp:235-255 (with the reference's `i==j==k==0` test)
  std::vector<unsigned long long int> getNeighborHashes(unsigned long long int hash, int K = 1) {
    int x, y, z;
    std::tie(x, y, z) = getVoxelCoords(hash);
    std::vector<unsigned long long int> out;
    for (int i = -K; i <= K; i++)
      for (int j = -K; j <= K; j++)
        for (int k = -K; k <= K; k++) {
          if (((i == j) == k) == 0) continue;
          if (validCoords(x + i, y + j, z + k) && voxels_[x + i][y + j][z + k] != nullptr)
            out.push_back(getHashId(x + i, y + j, z + k));
        }
    return out;
  }

  dmf_volume* handle() { return h_; }
  // Called by the engine after GPU calls that may change per-voxel flags.
  void touch() { ++version_; }

 private:
  dmf_volume* h_ = nullptr;
  uint64_t version_ = 1, mirror_version_ = 0;
  std::vector<std::unique_ptr<Voxel>> store_;
  std::vector<int32_t> slot_of_;  // dense x-major -> slot index or -1

  void pull_info() {
    dmf_volume_info i;
    dmf_check(dmf_volume_get_info(h_, &i));
    xmin_ = i.xmin; xmax_ = i.xmax; ymin_ = i.ymin; ymax_ = i.ymax; zmin_ = i.zmin; zmax_ = i.zmax;
    xcenter_ = i.xcenter; ycenter_ = i.ycenter; zcenter_ = i.zcenter;
    xdelta_ = i.xdelta; ydelta_ = i.ydelta; zdelta_ = i.zdelta;
    voxel_size_ = i.voxel_size;
    xdim_ = i.xdim; ydim_ = i.ydim; zdim_ = i.zdim;
    hsize_ = i.hsize;
  }

  bool integrate(const pcl::PointCloud<pcl::PointXYZRGB>::Ptr& cloud, const pcl::PointCloud<pcl::Normal>* normals) {
    const size_t n = cloud->points.size();
    std::vector<float> xyz(3 * n), nrm(normals ? 3 * n : 0);
    for (size_t i = 0; i < n; ++i) {
      xyz[3 * i] = cloud->points[i].x;
      xyz[3 * i + 1] = cloud->points[i].y;
      xyz[3 * i + 2] = cloud->points[i].z;
      if (normals)
        for (int k = 0; k < 3; ++k) nrm[3 * i + k] = normals->points[i].normal[k];
    }
    int64_t binned = 0, hazard = 0;
    dmf_check(dmf_volume_integrate(h_, xyz.data(), normals ? nrm.data() : nullptr, (int64_t)n, &binned, &hazard));
    int64_t V = 0;
    dmf_check(dmf_volume_occupied(h_, nullptr, 0, &V));
    occupied_cells_.resize((size_t)V);
    if (V) dmf_check(dmf_volume_occupied(h_, reinterpret_cast<uint64_t*>(occupied_cells_.data()), V, &V));
    touch();
    return true;
  }

  void rebuild_mirror() {
    const size_t V = occupied_cells_.size();
    dmf_volume_info info;
    dmf_check(dmf_volume_get_info(h_, &info));
    const int64_t np = info.num_points;
    std::vector<int32_t> view(V), off(V + 1);
    std::vector<uint8_t> good(V);
    std::vector<float> pts(3 * (size_t)np), nrm4(4 * (size_t)np);
    if (V) {
      dmf_check(dmf_volume_voxel_flags(h_, view.data(), good.data(), (int64_t)V));
      dmf_check(dmf_volume_export(h_, off.data(), pts.data(), nrm4.data(), np));
    }
    store_.clear();
    store_.reserve(V);
    slot_of_.assign((size_t)xdim_ * ydim_ * zdim_, -1);
    for (size_t s = 0; s < V; ++s) {
      std::unique_ptr<Voxel> vx(new Voxel());
      for (int32_t i = off[s]; i < off[s + 1]; ++i) {
        pcl::PointXYZRGB pt;
        pt.x = pts[3 * (size_t)i]; pt.y = pts[3 * (size_t)i + 1]; pt.z = pts[3 * (size_t)i + 2];
        vx->pts.push_back(pt);
        if (nrm4[4 * (size_t)i + 3] != 0.f) {  // only points integrated with a normal carry one
          pcl::Normal nm;
          for (int k = 0; k < 3; ++k) nm.normal[k] = nrm4[4 * (size_t)i + k];
          vx->normals.push_back(nm);
        }
      }
      vx->view = view[s];
      vx->good = good[s] != 0;
      store_.push_back(std::move(vx));
      int x, y, z;
      std::tie(x, y, z) = getVoxelCoords(occupied_cells_[s]);
      slot_of_[((size_t)x * ydim_ + y) * zdim_ + z] = (int32_t)s;
    }
    mirror_version_ = version_;
  }

  Voxel* mirror_at(int x, int y, int z) {
    if (mirror_version_ != version_) rebuild_mirror();
    if (!validCoords(x, y, z)) return nullptr;
    const int32_t s = slot_of_[((size_t)x * ydim_ + y) * zdim_ + z];
    return s < 0 ? nullptr : store_[(size_t)s].get();
  }
};
