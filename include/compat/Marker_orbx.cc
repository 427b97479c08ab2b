// Marker_orbx.cc — see Marker_orbx.h.  One cv::ORB() plan per thread and image size (the
// library rebuilds its plan when the size changes); cv::KeyPoint == orbx_keypoint (28 B),
// cv::DMatch == orbx_dmatch (16 B).
#include "Marker_orbx.h"

#include "orbx.h"

static_assert(sizeof(cv::KeyPoint) == sizeof(orbx_keypoint), "cv::KeyPoint is 28 B");
static_assert(sizeof(cv::DMatch) == sizeof(orbx_dmatch), "cv::DMatch is 16 B");

namespace {
orbx_cvorb* orb_for(int w, int h) {
  static thread_local orbx_cvorb* orb = nullptr;
  if (!orb) {
    const orbx_cvorb_params p{500, 1.2f, 8, 31, 0, 2, ORBX_HARRIS_SCORE, 31};  // cv::ORB()
    if (orbx_cvorb_create(&p, w, h, 1, /*hip_device*/ 0, &orb) != ORBX_OK) orb = nullptr;
  }
  return orb;
}
}  // namespace

bool orbx_marker_orb(const cv::Mat& image, std::vector<cv::KeyPoint>& keys, cv::Mat& descriptors) {
  orbx_cvorb* orb = orb_for(image.cols, image.rows);
  if (!orb) return false;
  int32_t cap = 4096, n = 0;
  std::vector<cv::KeyPoint> buf(cap);
  cv::Mat d(cap, 32, CV_8U);
  int rc = orbx_cvorb_detect(orb, image.data, image.cols, image.rows, (int64_t)image.step,
                             reinterpret_cast<orbx_keypoint*>(buf.data()), d.data, cap, &n);
  if (rc == ORBX_ECAPACITY) {  // grow once and repeat
    cap = n;
    buf.resize(cap);
    d.create(cap, 32, CV_8U);
    rc = orbx_cvorb_detect(orb, image.data, image.cols, image.rows, (int64_t)image.step,
                           reinterpret_cast<orbx_keypoint*>(buf.data()), d.data, cap, &n);
  }
  if (rc != ORBX_OK) return false;
  if (n < 0) return true;  // empty image: orb.cpp returns before touching the outputs
  buf.resize(n);
  keys.swap(buf);
  if (n)
    descriptors = d.rowRange(0, n).clone();
  else
    descriptors.release();
  return true;
}

bool orbx_marker_good_matches(const cv::Mat& desc1, const cv::Mat& desc2,
                              std::vector<cv::DMatch>& matches, std::vector<cv::DMatch>& good) {
  matches.resize(desc1.rows);
  good.resize(desc1.rows);
  int32_t n = 0, ng = 0;
  double min_dist = 0, max_dist = 0;
  if (orbx_bf_match(desc1.data, desc1.rows, desc2.data, desc2.rows,
                    reinterpret_cast<orbx_dmatch*>(matches.data()), &n) != ORBX_OK)
    return false;
  matches.resize(n);
  if (orbx_good_matches(reinterpret_cast<const orbx_dmatch*>(matches.data()), n,
                        reinterpret_cast<orbx_dmatch*>(good.data()), &ng, &min_dist,
                        &max_dist) != ORBX_OK)
    return false;
  good.resize(ng);
  return true;
}
