// boost/algorithm/string.hpp for the drop-in build: the reference drivers only open the
// namespace (tests/Raytracing.cpp:47 `using namespace boost::algorithm`).
#pragma once
#include <string>
namespace boost {
namespace algorithm {}
}  // namespace boost
