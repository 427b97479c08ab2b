// Compile-check stand-in for DBoW2's FORB; see tests/compat_stub/opencv2/core/core.hpp.
#pragma once
#include "opencv2/core/core.hpp"
namespace DBoW2 {
class FORB {
 public:
  typedef cv::Mat TDescriptor;
};
}  // namespace DBoW2
