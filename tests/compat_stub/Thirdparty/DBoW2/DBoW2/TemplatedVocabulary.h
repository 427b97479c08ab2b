// Compile-check stand-in for DBoW2's TemplatedVocabulary; see
// tests/compat_stub/opencv2/core/core.hpp.
#pragma once
#include <string>
#include <vector>
#include "BowVector.h"
#include "FeatureVector.h"
namespace DBoW2 {
template <class TDescriptor, class F>
class TemplatedVocabulary {
 public:
  void transform(const std::vector<TDescriptor>& features, BowVector& v, FeatureVector& fv,
                 int levelsup) const;
  bool loadFromTextFile(const std::string& filename);
};
}  // namespace DBoW2
