// Headless counterpart of the reference driver tests/Raytracing.cpp:55-105 (and of the
// per-pose visibility loop of tests/SetCover.cpp:218-240), written against the
// drop-in headers in compat/ exactly as the reference code is written against
// include/: same classes, same calls, same order.  Differences, all I/O:
//   - the cloud is read from a float32 file (x y z nx ny nz per point) instead of a
//     PCD (FileRoutines.hpp:33-67, PCL io is out of scope);
//   - camera poses come from a pose file in the FileRoutines.hpp:69-96 format instead
//     of positionCameras(downsample(cloud)) (Algorithms/PCL, out of scope);
//   - instead of the GUI (addVolumeWithVoxelsClassified + spinViewer) the classified
//     voxels are printed.
//   - (extension, BASELINE.json north_star) with depth.bin: the first P poses' 640x480
//     uint16 depth frames fused by RayTracingEngine::fuseDepth (3D-DDA log-odds), the
//     counts and log-odds written to out.bin (int32 hits | int32 misses | int16 log-odds).
// usage: raytracing_headless cloud.bin poses.txt [depth.bin P out.bin]
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "Algorithms.hpp"
#include "Camera.hpp"
#include "PathPlanning.hpp"
#include "RayTracingEngine.hpp"
#include "Volume.hpp"

using namespace std;

static vector<Eigen::Affine3f> readCameraLocations(const string& filename) {  // FileRoutines.hpp:69-96
  vector<Eigen::Affine3f> out;
  ifstream file(filename);
  string line;
  getline(file, line);
  const int length = stoi(line);
  for (int i = 0; i < length; i++) {
    Eigen::Affine3f temp = Eigen::Affine3f::Identity();
    for (int j = 0; j < 3; j++) {
      getline(file, line);
      stringstream ss(line);
      string tok;
      for (int k = 0; k < 4 && getline(ss, tok, ','); k++) temp(j, k) = stof(tok);
    }
    out.push_back(temp);
  }
  return out;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    cerr << "usage: " << argv[0] << " cloud.bin poses.txt\n";
    return 2;
  }
  pcl::PointCloud<pcl::PointXYZRGB>::Ptr cloud(new pcl::PointCloud<pcl::PointXYZRGB>);
  pcl::PointCloud<pcl::Normal>::Ptr normals(new pcl::PointCloud<pcl::Normal>);
  {
    ifstream f(argv[1], ios::binary);
    float rec[6];
    while (f.read(reinterpret_cast<char*>(rec), sizeof(rec))) {
      pcl::PointXYZRGB p;
      p.x = rec[0]; p.y = rec[1]; p.z = rec[2];
      pcl::Normal n;
      n.normal[0] = rec[3]; n.normal[1] = rec[4]; n.normal[2] = rec[5];
      cloud->points.push_back(p);
      normals->points.push_back(n);
    }
  }
  vector<float> K = {602.39306640625, 0.0, 314.6370849609375, 0.0, 602.39306640625, 245.04962158203125, 0.0, 0.0, 1.0};
  // pcl::getMinMax3D (tests/Raytracing.cpp:64)
  pcl::PointXYZRGB min_pt = cloud->points[0], max_pt = cloud->points[0];
  for (const auto& p : cloud->points) {
    min_pt.x = min(min_pt.x, p.x); min_pt.y = min(min_pt.y, p.y); min_pt.z = min(min_pt.z, p.z);
    max_pt.x = max(max_pt.x, p.x); max_pt.y = max(max_pt.y, p.y); max_pt.z = max(max_pt.z, p.z);
  }
  // tests/Raytracing.cpp:67-76
  VoxelVolume volume;
  volume.setDimensions(min_pt.x, max_pt.x, min_pt.y, max_pt.y, min_pt.z, max_pt.z);
  double x_resolution = (max_pt.x - min_pt.x) * 125;
  double y_resolution = (max_pt.y - min_pt.y) * 125;
  double z_resolution = (max_pt.z - min_pt.z) * 125;
  volume.setVolumeSize(int(x_resolution), int(y_resolution), int(z_resolution));
  volume.constructVolume();
  volume.integratePointCloud(cloud, normals);
  cout << "dims " << volume.xdim_ << " " << volume.ydim_ << " " << volume.zdim_ << "\n";
  cout << "occupied " << volume.occupied_cells_.size() << "\n";
  auto camera_locations = readCameraLocations(argv[2]);
  Camera cam(K);
  double resolution = volume.voxel_size_;
  int resolution_single_dimension = int(round(cbrt(resolution * 1e9)));
  // tests/Raytracing.cpp:91-92
  RayTracingEngine engine(cam);
  auto res = engine.reverseRayTraceFast(volume, camera_locations[0], true, resolution_single_dimension);
  // what addVolumeWithVoxelsClassified would draw (VisualizationUtilities.hpp:377-429)
  size_t nview = 0, ngood = 0;
  for (auto h : volume.occupied_cells_) {
    int x, y, z;
    tie(x, y, z) = volume.getVoxelCoords(h);
    Voxel* v = volume.voxels_[x][y][z];
    nview += v->view == 1;
    ngood += v->good;
  }
  cout << "found " << res.first << " good " << res.second.size() << " view_flags " << nview << " good_flags " << ngood
       << "\n";
  cout << "goodlist";
  for (auto h : res.second) cout << " " << h;
  cout << "\n";
  // tests/SetCover.cpp:218-240 visibility loop (viz=false, sorted for set_difference)
  vector<vector<unsigned long long int>> regions_covered;
  for (size_t i = 0; i < camera_locations.size(); i++) {
    vector<unsigned long long int> good_points;
    bool found;
    tie(found, good_points) = engine.reverseRayTraceFast(volume, camera_locations[i], false);
    sort(good_points.begin(), good_points.end());
    cout << "Sizes: " << good_points.size() << "\n";
    regions_covered.push_back(good_points);
  }
  // tests/SetCover.cpp:236-239 + include/Algorithms.hpp:38-86
  auto cameras_selected = dmf_compat::setCoverBatched(engine, volume, camera_locations, resolution_single_dimension);
  auto again = Algorithms::greedySetCover(regions_covered);
  cout << "selected";
  for (auto s : cameras_selected) cout << " " << s;
  cout << "\nselected_from_sets";
  for (auto s : again) cout << " " << s;
  cout << "\n";
  // tests/CameraPathGen.cpp:310-331 run_tsp cost map over the camera centres
  auto map = PathPlanning::collisionCostMap(volume, camera_locations);
  cout << "costmap";
  for (auto& row : map)
    for (int m : row) cout << " " << m;
  cout << "\ncollide_from_0";
  for (auto& T : camera_locations) {
    Eigen::Vector3f a, b;
    a << camera_locations[0](0, 3), camera_locations[0](1, 3), camera_locations[0](2, 3);
    b << T(0, 3), T(1, 3), T(2, 3);
    cout << " " << PathPlanning::willCollide(volume, a, b);
  }
  cout << "\n";
  if (argc >= 6) {  // fusion of P depth frames into the same volume's grid
    const int P = stoi(argv[4]);
    vector<uint16_t> depth((size_t)P * 480 * 640);
    ifstream f(argv[3], ios::binary);
    if (!f.read(reinterpret_cast<char*>(depth.data()), (streamsize)(depth.size() * sizeof(uint16_t)))) {
      cerr << "short depth file\n";
      return 3;
    }
    vector<Eigen::Affine3f> fposes(camera_locations.begin(), camera_locations.begin() + P);
    dmf_fuse_params prm;
    dmf_fuse_params_default(&prm);
    prm.dmin_mm = 200;
    prm.dmax_mm = 1000;
    RayTracingEngine::FusionCounts acc;
    engine.fuseDepth(volume, depth, fposes, acc, &prm);
    const vector<int16_t> lo = engine.logOdds(volume, acc, &prm);
    cout << "fusion " << acc.updates << " " << acc.rays << " " << acc.hit_rays << "\n";
    ofstream o(argv[5], ios::binary);
    o.write(reinterpret_cast<const char*>(acc.hits.data()), (streamsize)(acc.hits.size() * sizeof(int32_t)));
    o.write(reinterpret_cast<const char*>(acc.misses.data()), (streamsize)(acc.misses.size() * sizeof(int32_t)));
    o.write(reinterpret_cast<const char*>(lo.data()), (streamsize)(lo.size() * sizeof(int16_t)));
  }
  return 0;
}
