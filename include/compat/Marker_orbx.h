// Marker_orbx.h — the AR marker path's cv::ORB and matcher calls on the GPU
// (ORB_SLAM2/src/Marker.cc:76-84, 98-133; AR-1.3/src/ORBMatcher.cpp:44-102).  Marker.cc keeps
// its code and calls these first; each returns false when the caller should run its own OpenCV
// call instead (device error):
//
//   void Marker::setTargetImage(cv::Mat image) {                // Marker.cc:76-84
//     image.copyTo(mImage1);
//     if (!orbx_marker_orb(mImage1, mvKeys1, mDescriptors1)) { ORB orb; orb(mImage1, Mat(), mvKeys1, mDescriptors1); }
//   }
//   bool Marker::Match(cv::Mat image, double meanerr, double ratio) {   // Marker.cc:98-133
//     image.copyTo(mImage2);
//     if (!orbx_marker_orb(mImage2, mvKeys2, mDescriptors2)) { ORB orb; orb(mImage2, Mat(), mvKeys2, mDescriptors2); }
//     if (0 == mDescriptors1.cols || 0 == mDescriptors2.cols) { ...; return false; }
//     vector<DMatch> matches, good_matches;
//     if (!orbx_marker_good_matches(mDescriptors1, mDescriptors2, matches, good_matches)) {
//       ... the reference's BruteForceMatcher<HammingLUT> + filter loop ...
//     }
//     ... the reference's homography / projection-error code from Marker.cc:135 on ...
//   }
#pragma once
#include <vector>

#include "opencv2/opencv.hpp"

// cv::ORB() (OpenCV 2.4 defaults: 500 features, 1.2, 8 levels, edge 31, HARRIS_SCORE, patch 31)
// of a u8 image: keypoints in the order retainBest leaves them, descriptors n x 32.
bool orbx_marker_orb(const cv::Mat& image, std::vector<cv::KeyPoint>& keys, cv::Mat& descriptors);
// BruteForceMatcher<HammingLUT>::match(desc1, desc2, matches) and Marker::Match's filter
// (distance < 0.5 * max_dist, in order).
bool orbx_marker_good_matches(const cv::Mat& desc1, const cv::Mat& desc2,
                              std::vector<cv::DMatch>& matches, std::vector<cv::DMatch>& good);
