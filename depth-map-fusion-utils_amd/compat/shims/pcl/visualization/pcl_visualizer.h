// pcl/visualization/pcl_visualizer.h for the drop-in build: a headless PCLVisualizer whose
// calls are accepted and ignored (visualisation is out of scope; the
// compat VisualizationUtilities wrapper reports what it was asked to draw instead).
#pragma once
#include <memory>
#include <string>

#include "../../../dmf_types.hpp"

#define PCL_ERROR(...) std::fprintf(stderr, __VA_ARGS__)

namespace pcl {
namespace visualization {
enum RenderingProperties {
  PCL_VISUALIZER_POINT_SIZE,
  PCL_VISUALIZER_OPACITY,
  PCL_VISUALIZER_LINE_WIDTH,
  PCL_VISUALIZER_FONT_SIZE,
  PCL_VISUALIZER_COLOR,
  PCL_VISUALIZER_REPRESENTATION,
  PCL_VISUALIZER_IMMEDIATE_RENDERING,
  PCL_VISUALIZER_SHADING
};
class PCLVisualizer {
 public:
  using Ptr = std::shared_ptr<PCLVisualizer>;
  PCLVisualizer() = default;
  explicit PCLVisualizer(const std::string&) {}
  void setBackgroundColor(double, double, double) {}
  void initCameraParameters() {}
  void addCoordinateSystem(double = 1.0) {}
  bool removeCoordinateSystem() { return true; }
  bool removeAllCoordinateSystems() { return true; }
  void removeAllShapes() {}
  void removeAllPointClouds() {}
  template <class PointT>
  bool addSphere(const PointT&, double, double, double, double, const std::string& = "sphere") { return true; }
  template <class PointT>
  bool addSphere(const PointT&, double, const std::string& = "sphere") { return true; }
  template <class... A>
  bool setPointCloudRenderingProperties(int, A...) { return true; }
  bool wasStopped() const { return true; }
  void spin() {}
  void spinOnce(int = 1, bool = false) {}
};
}  // namespace visualization
}  // namespace pcl
