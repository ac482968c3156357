// VisualizationUtilities.hpp — headless drop-in for the reference
// include/VisualizationUtilities.hpp:70-107 PCLVisualizerWrapper (visualisation is out of
// scope).  Every call is accepted; instead of drawing, the wrapper records
// the camera poses it was given and, when the environment variable DMF_COMPAT_VIZ_DUMP
// names a file, addVolumeWithVoxelsClassified writes what the reference would have shown
// there: the volume geometry, the cameras, and (hash, view, good) of every occupied voxel
// (the test of the unchanged tests/Raytracing.cpp checks that file against the oracle).
#pragma once
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <pcl/visualization/pcl_visualizer.h>

#include "Camera.hpp"
#include "Volume.hpp"
#include "dmf_types.hpp"

namespace VisualizationUtilities {
class PCLVisualizerWrapper {
  std::vector<std::pair<std::string, Eigen::Affine3f>> cameras_;

 public:
  pcl::visualization::PCLVisualizer::Ptr viewer_;
  PCLVisualizerWrapper() : viewer_(std::make_shared<pcl::visualization::PCLVisualizer>()) {}
  PCLVisualizerWrapper(double r, double g, double b) : PCLVisualizerWrapper() { viewer_->setBackgroundColor(r, g, b); }
  template <typename PointT>
  void addPointCloud(typename pcl::PointCloud<PointT>::Ptr, std::string = "cloud") {}
  template <typename PointT>
  void addPointCloudNormals(typename pcl::PointCloud<PointT>::Ptr, typename pcl::PointCloud<pcl::Normal>::Ptr) {}
  void spinViewerOnce() {}
  void spinViewer() {}
  bool viewerGood() const { return false; }  // headless: there is no window to keep open
  void addSphere(pcl::PointXYZ, std::string) {}
  void addCoordinateSystem() {}
  void addVolume(VoxelVolume&) {}
  void addPointCloudInVolume(VoxelVolume&) {}
  void addLine(std::vector<double>&, std::vector<double>&, std::string, std::vector<int> = {255, 0, 0}) {}
  void addPolygon(std::vector<std::vector<double>>&, std::string) {}
  void addPyramid(std::vector<std::vector<double>>&, std::vector<double>, std::string) {}
  void addNewCoordinateAxes(Eigen::Affine3f&, std::string) {}
  void addCamera(std::vector<float>&, int, int, Eigen::Affine3f& t, std::string id, int = 1000) { cameras_.emplace_back(id, t); }
  void addCamera(Camera&, Eigen::Affine3f& t, std::string id, int = 1000) { cameras_.emplace_back(id, t); }
  void addPointCloudInVolumeRayTraced(VoxelVolume& volume) { addVolumeWithVoxelsClassified(volume); }
  void addVolumeWithVoxelsClassified(VoxelVolume& volume) {
    const char* path = std::getenv("DMF_COMPAT_VIZ_DUMP");
    if (!path || !*path) return;
    FILE* f = std::fopen(path, "w");
    if (!f) return;
    std::fprintf(f, "bounds %.17g %.17g %.17g %.17g %.17g %.17g\n", volume.xmin_, volume.xmax_, volume.ymin_,
                 volume.ymax_, volume.zmin_, volume.zmax_);
    std::fprintf(f, "dims %d %d %d\n", volume.xdim_, volume.ydim_, volume.zdim_);
    for (auto& c : cameras_) {
      std::fprintf(f, "camera %s", c.first.c_str());
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) std::fprintf(f, " %.9g", c.second(i, j));
      std::fprintf(f, "\n");
    }
    for (unsigned long long h : volume.occupied_cells_) {
      int x, y, z;
      std::tie(x, y, z) = volume.getVoxelCoords(h);
      const Voxel* v = volume.voxels_[x][y][z];
      std::fprintf(f, "voxel %llu %d %d\n", h, v ? v->view : -1, v ? (int)v->good : -1);
    }
    std::fclose(f);
  }
};
}  // namespace VisualizationUtilities

// :432-471 VizThread: a viewer thread spinning the wrapper and an input thread; headless,
// the viewer loop ends at once (viewerGood() is false) and input() runs to completion.
class VizThread {
  std::vector<std::thread> threads_;
  std::mutex mtx_;
  bool changed_ = false;
  virtual void input() {}
  virtual void process(VisualizationUtilities::PCLVisualizerWrapper&) {}

 public:
  virtual ~VizThread() = default;
  bool updateViewer() {
    std::lock_guard<std::mutex> g(mtx_);
    changed_ = true;
    return false;
  }
  void makeThreads() {
    threads_.push_back(std::thread(&VizThread::spin, this));
    threads_.push_back(std::thread(&VizThread::input, this));
    for (auto& t : threads_) t.join();
  }
  void spin() {
    VisualizationUtilities::PCLVisualizerWrapper viz;
    viz.addCoordinateSystem();
    while (viz.viewerGood()) {
      {
        std::lock_guard<std::mutex> g(mtx_);
        if (changed_) process(viz);
        changed_ = false;
      }
      viz.spinViewerOnce();
    }
  }
};
