// Frame_orbx.h — the per-frame work of ORB_SLAM2's Frame / KeyFrame that the library runs on the
// GPU, as functions the reference's own bodies call first (Frame_orbx.cc).  Each returns false
// when it did not produce the result (no device vocabulary loaded, a device error, an extraction
// served by the host fallback), and the reference's body then runs unchanged:
//
//   // System.cc, after mpVocabulary->loadFromTextFile(strVocFile) (System.cc:64-65):
//   ORB_SLAM2::orbx_load_vocabulary(strVocFile);
//
//   void Frame::ComputeBoW() {                                  // Frame.cc:400-407
//     if (mBowVec.empty() && !orbx_compute_bow(mDescriptors, mBowVec, mFeatVec)) {
//       vector<cv::Mat> vCurrentDesc = Converter::toDescriptorVector(mDescriptors);
//       mpORBvocabulary->transform(vCurrentDesc, mBowVec, mFeatVec, 4);
//     }
//   }
//   // KeyFrame::ComputeBoW (KeyFrame.cc) the same way.
//
//   void Frame::ComputeStereoMatches() {                        // Frame.cc:471-643
//     if (orbx_compute_stereo_matches(*this)) return;
//     ... the reference's body ...
//   }
#pragma once
#include <string>

#include "Frame.h"
#include "orbx.h"

namespace ORB_SLAM2 {

// Loads ORBvoc.txt into HBM (orbx_vocabulary_load_text) for the device transform.
bool orbx_load_vocabulary(const std::string& path);
// TemplatedVocabulary::transform(descriptors, BowVector, FeatureVector, levelsup = 4) on the GPU
// (TemplatedVocabulary.h:1127-1259): BowVector and FeatureVector bit-exact.
bool orbx_compute_bow(const cv::Mat& descriptors, DBoW2::BowVector& bow, DBoW2::FeatureVector& fv);
// Frame::ComputeStereoMatches on the left / right extractors' last results (orbx_stereo_matches).
bool orbx_compute_stereo_matches(Frame& F);

// ORBextractor_orbx.cc: the device context of an extractor whose last call ran on the GPU
::orbx_extractor* orbx_context_of(const ORBextractor* self);
// ORBextractor_orbx.cc: mvImagePyramid (ORBextractor.h:88) is exported from HBM lazily — its
// only reader, Frame::ComputeStereoMatches, runs on the device (orbx_compute_stereo_matches).
// This copies the last device extraction's levels into mvImagePyramid; it is a no-op when they
// are already there (or the last call ran on the host, which fills them itself).  Returns false
// on a device error.  Code reading mvImagePyramid elsewhere calls it first.  If the export fails,
// the levels are rebuilt on the host from the extraction's input image, so call it while that
// image is alive and unchanged (Frame's stereo constructor does: ComputeStereoMatches runs right
// after the two extractions, Frame.cc:52-80); the input is released once the levels are out.
bool orbx_materialize_pyramid(ORBextractor* self);

}  // namespace ORB_SLAM2
