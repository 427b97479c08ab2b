// Compile-check stand-in for DBoW2's BowVector (declarations the ORB-SLAM2 headers and the
// orbx shims name); see tests/compat_stub/opencv2/core/core.hpp.
#pragma once
#include <map>
namespace DBoW2 {
typedef unsigned int WordId;
typedef double WordValue;
typedef unsigned int NodeId;
enum LNorm { L1, L2 };
enum WeightingType { TF_IDF, TF, IDF, BINARY };
enum ScoringType { L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT };
class BowVector : public std::map<WordId, WordValue> {};
}  // namespace DBoW2
