// TransformationUtilities.hpp — namespace of the reference include/TransformationUtilities.hpp
// (its Eigen::MatrixXd point-cloud transforms are outside the hot path and not provided;
// the drivers only open the namespace, tests/Raytracing.cpp:50).
#pragma once
#include <vector>

#include "dmf_types.hpp"

namespace TransformationUtilities {
// :147-157 affineMatrixToVector: the 12 entries of rows 0..2
inline std::vector<double> affineMatrixToVector(Eigen::Affine3f t) {
  std::vector<double> out;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) out.push_back(t(i, j));
  return out;
}
}  // namespace TransformationUtilities
