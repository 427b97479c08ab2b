// Compile-check stand-in for DBoW2's FeatureVector; see tests/compat_stub/opencv2/core/core.hpp.
#pragma once
#include <map>
#include <vector>
#include "BowVector.h"
namespace DBoW2 {
class FeatureVector : public std::map<NodeId, std::vector<unsigned int> > {};
}  // namespace DBoW2
