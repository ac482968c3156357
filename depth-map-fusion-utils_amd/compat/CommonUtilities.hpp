// CommonUtilities.hpp — drop-in for the reference include/CommonUtilities.hpp:17-22 (the
// scalar helpers; planeFitting's SVD, :24-40, is outside the hot path and not provided).
#pragma once
#include <cmath>
#include <vector>

#include "dmf_types.hpp"

constexpr int degree(double radian) { return int((radian * 180) / 3.14159); }
constexpr double magnitude(double normal[3]) { return normal[0] * normal[0] + normal[1] * normal[1] + normal[2] * normal[2]; }
inline int angle(double normal[3]) { return degree(std::acos(-normal[2] / magnitude(normal))); }
template <typename T>
constexpr int sgn(T x) { return (T(0) < x) - (x < T(0)); }
