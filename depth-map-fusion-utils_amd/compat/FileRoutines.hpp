// FileRoutines.hpp — drop-in for the reference include/FileRoutines.hpp:33-96: readPointCloud
// (a PCD of PointXYZRGBNormal split into an XYZRGB cloud with black colour and a Normal
// cloud, same console messages) and readCameraLocations (the pose-file format).
#pragma once
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include <pcl/io/pcd_io.h>
#include <pcl/visualization/pcl_visualizer.h>

#include "dmf_types.hpp"

inline void readPointCloud(std::string filename, pcl::PointCloud<pcl::PointXYZRGBNormal>::Ptr cloud_normal,
                           pcl::PointCloud<pcl::PointXYZRGB>::Ptr cloud,
                           pcl::PointCloud<pcl::Normal>::Ptr normals = nullptr) {
  std::cout << "Inside reading function" << std::endl;
  if (pcl::io::loadPCDFile<pcl::PointXYZRGBNormal>(filename, *cloud_normal) == -1) {
    PCL_ERROR("Couldn't read file for base. \n");
    return;
  }
  std::cout << "Parsing the pointcloud" << std::endl;
  for (const pcl::PointXYZRGBNormal& pt : cloud_normal->points) {
    pcl::PointXYZRGB pt_rgb;
    pt_rgb.x = pt.x;
    pt_rgb.y = pt.y;
    pt_rgb.z = pt.z;
    pcl::Normal pt_n;
    for (int a = 0; a < 3; ++a) pt_n.normal[a] = pt.normal[a];
    cloud->points.push_back(pt_rgb);
    if (normals != nullptr) normals->points.push_back(pt_n);
  }
  std::cout << "Pointcloud Parsed" << std::endl;
}

// :69-96: first line = count, then 3 comma-separated rows of 4 per pose
inline std::vector<Eigen::Affine3f> readCameraLocations(std::string filename) {
  std::vector<Eigen::Affine3f> out;
  std::ifstream file(filename);
  std::string line;
  if (!std::getline(file, line)) return out;
  const int length = std::stoi(line);
  for (int i = 0; i < length; i++) {
    Eigen::Affine3f t = Eigen::Affine3f::Identity();
    for (int j = 0; j < 3; j++) {
      std::getline(file, line);
      std::stringstream ss(line);
      std::string tok;
      for (int k = 0; k < 4 && std::getline(ss, tok, ','); k++) t(j, k) = std::stof(tok);
    }
    out.push_back(t);
  }
  return out;
}

// :98-112 writeCameraLocations (the same format)
inline void writeCameraLocations(std::string filename, std::vector<Eigen::Affine3f> transformations) {
  std::ofstream file(filename);
  file << transformations.size() << std::endl;
  for (size_t i = 0; i < transformations.size(); i++)
    for (int j = 0; j < 3; j++) {
      file << transformations[i](j, 0);
      for (int k = 1; k < 4; k++) file << "," << transformations[i](j, k);
      file << std::endl;
    }
}
