// ORBextractor_orbx.cc — drop-in replacement of ORB_SLAM2/src/ORBextractor.cc over liborbx.so
// (include/orbx.h).  ORB_SLAM2/include/ORBextractor.h stays byte-identical: its inline getters
// read the data members, so the class layout is ABI-visible; the GPU state lives in
// a side table keyed by `this`.
//
// Build: replace src/ORBextractor.cc by this file and include/compat/ORBextractor_host.cc in the
// library's source list, add -I<repo>/include -I<repo>/include/compat, link -lorbx
// (ar_orbslam2_amd/_lib).
//
// Behaviour per ORBextractor.cc:985-1045: an empty image leaves the outputs untouched; keypoints
// (cv::KeyPoint == orbx_keypoint, 28 B) and descriptors bit-exact with the reference (the
// library's parity tests); mvImagePyramid is exported from HBM on demand
// (orbx_materialize_pyramid, Frame_orbx.h: its only reader, Frame::ComputeStereoMatches, runs on
// the device).  On a device error the call is served by the reference's own code
// (ORBextractorHost), once logged.
#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

#include "ORBextractor.h"
#include "Frame_orbx.h"
#include "ORBextractor_host.h"
#include "orbx.h"

static_assert(sizeof(cv::KeyPoint) == sizeof(orbx_keypoint), "cv::KeyPoint is 28 B");

namespace ORB_SLAM2 {

namespace {

struct ExtractorCtx {
  orbx_extractor* ex = nullptr;
  orbx_params p{};
  ORBextractorHost* host = nullptr;  // built on the first fallback
  bool create_failed = false;        // no device context: every call goes to the host
  bool last_on_device = false;       // the last call's results are resident on the GPU
  bool pyramid_exported = false;     // mvImagePyramid holds the last device call's levels
  // the last device call's input (a header sharing the caller's image): if the pyramid export
  // fails, the host extractor rebuilds mvImagePyramid from it.  Valid only while the caller's
  // pixels are (Frame's constructor, where ComputeStereoMatches runs; Frame_orbx.h), and
  // released once orbx_materialize_pyramid has consumed it
  cv::Mat last_image;
  // the library's raw outputs, kept between calls (one extractor runs on one thread)
  std::vector<orbx_keypoint> kps;
  cv::Mat desc;
};

std::mutex g_mutex;
std::map<const ORBextractor*, ExtractorCtx> g_ctx;

bool same_params(const orbx_params& a, const orbx_params& b) {
  return a.nfeatures == b.nfeatures && a.scale_factor == b.scale_factor &&
         a.nlevels == b.nlevels && a.ini_th_fast == b.ini_th_fast && a.min_th_fast == b.min_th_fast;
}

// The context of `self` for these parameters.  The reference never deletes an extractor (they
// live as long as Tracking, Tracking.cc:455-464) and ORBextractor.h's destructor is inline, so
// there is no hook to free a context; an entry whose parameters differ belongs to an earlier
// object at the same address and is rebuilt.
ExtractorCtx& ctx_of(const ORBextractor* self, const orbx_params& p) {
  std::lock_guard<std::mutex> lock(g_mutex);
  ExtractorCtx& c = g_ctx[self];
  if (c.ex && !same_params(c.p, p)) {
    orbx_extractor_destroy(c.ex);
    delete c.host;
    c = ExtractorCtx{};
  }
  if (c.create_failed && !same_params(c.p, p)) {
    delete c.host;  // built by the constructor's fallback for the earlier parameters
    c = ExtractorCtx{};
  }
  if (!c.ex && !c.create_failed) {  // one attempt per (object, parameters), not one per frame
    c.p = p;
    if (orbx_extractor_create(&p, /*hip_device*/ 0, &c.ex) != ORBX_OK) {
      c.ex = nullptr;
      c.create_failed = true;
    }
  }
  return c;
}

void log_once(const char* what, int rc) {
  static std::once_flag f;
  std::call_once(f, [&] {
    fprintf(stderr, "[orbx] %s failed (%d): falling back to the host ORBextractor\n", what, rc);
  });
}

// mvImagePyramid from the device: level sizes, then one download per level
int export_pyramid(orbx_extractor* ex, int nlevels, std::vector<cv::Mat>& pyr) {
  int rc = ORBX_OK;
  for (int l = 0; l < nlevels && rc == ORBX_OK; ++l) {
    int32_t w = 0, h = 0;
    rc = orbx_extractor_pyramid(ex, l, nullptr, 0, &w, &h);
    if (rc != ORBX_OK) break;
    pyr[l].create(h, w, CV_8U);
    rc = orbx_extractor_pyramid(ex, l, pyr[l].data, (int64_t)pyr[l].step, &w, &h);
  }
  return rc;
}

}  // namespace

// ORBextractor.cc:404-460 — the tables come from the library (same float types as the
// reference's constructor), so the inline getters return identical values.
ORBextractor::ORBextractor(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST,
                           int _minThFAST)
    : nfeatures(_nfeatures), scaleFactor(_scaleFactor), nlevels(_nlevels),
      iniThFAST(_iniThFAST), minThFAST(_minThFAST) {
  mvScaleFactor.resize(nlevels);
  mvInvScaleFactor.resize(nlevels);
  mvLevelSigma2.resize(nlevels);
  mvInvLevelSigma2.resize(nlevels);
  mnFeaturesPerLevel.resize(nlevels);
  mvImagePyramid.resize(nlevels);
  const orbx_params p{nfeatures, _scaleFactor, nlevels, iniThFAST, minThFAST};
  ExtractorCtx& c = ctx_of(this, p);
  int32_t nl = 0;
  if (!c.ex || orbx_extractor_tables(c.ex, &nl, mvScaleFactor.data(), mvInvScaleFactor.data(),
                                     mvLevelSigma2.data(), mvInvLevelSigma2.data(),
                                     mnFeaturesPerLevel.data()) != ORBX_OK) {
    // the reference's constructor computes the same tables on the host
    std::lock_guard<std::mutex> lock(g_mutex);
    c.host = new ORBextractorHost(_nfeatures, _scaleFactor, _nlevels, _iniThFAST, _minThFAST);
    mvScaleFactor = c.host->GetScaleFactors();
    mvInvScaleFactor = c.host->GetInverseScaleFactors();
    mvLevelSigma2 = c.host->GetScaleSigmaSquares();
    mvInvLevelSigma2 = c.host->GetInverseScaleSigmaSquares();
  }
  // umax / pattern are used by the reference's host code only; the library holds its own
}

void ORBextractor::operator()(cv::InputArray _image, cv::InputArray _mask,
                              std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors) {
  if (_image.empty()) return;  // ORBextractor.cc:987-988
  cv::Mat image = _image.getMat();
  const orbx_params p{nfeatures, (float)scaleFactor, nlevels, iniThFAST, minThFAST};
  ExtractorCtx& c = ctx_of(this, p);
  int rc = c.ex ? ORBX_OK : ORBX_EDEVICE;
  int32_t n = 0;
  if (c.ex) {
    int32_t cap = std::max<int32_t>(4 * nfeatures + 64, (int32_t)c.kps.size());
    if ((int32_t)c.kps.size() < cap) c.kps.resize(cap);
    if (c.desc.rows < cap) c.desc.create(cap, 32, CV_8U);
    rc = orbx_extract(c.ex, image.data, image.cols, image.rows, (int64_t)image.step, c.kps.data(),
                      c.desc.data, cap, &n);
    if (rc == ORBX_ECAPACITY) {  // more keypoints than the first guess: grow once, repeat
      cap = n;
      c.kps.resize(cap);
      c.desc.create(cap, 32, CV_8U);
      rc = orbx_extract(c.ex, image.data, image.cols, image.rows, (int64_t)image.step,
                        c.kps.data(), c.desc.data, cap, &n);
    }
    if (rc == ORBX_OK) {
      if (n <= 0) {  // :1005-1006 (no keypoints: descriptors released)
        _keypoints.clear();
        _descriptors.release();
      } else {
        const cv::KeyPoint* k = reinterpret_cast<const cv::KeyPoint*>(c.kps.data());
        _keypoints.assign(k, k + n);
        _descriptors.create(n, 32, CV_8U);  // as ORBextractor.cc:1008-1009
        cv::Mat out = _descriptors.getMat();
        c.desc.rowRange(0, n).copyTo(out);
      }
      // mvImagePyramid (ORBextractor.h:88) is read by Frame::ComputeStereoMatches only, which
      // runs on the device: it is exported on demand (orbx_materialize_pyramid), not per call
      c.last_on_device = true;
      c.pyramid_exported = false;
      c.last_image = image;
      return;
    }
  }
  c.last_on_device = false;
  c.last_image = cv::Mat();
  // device error: the reference's own code on the host, same outputs
  log_once("orbx_extract", rc);
  ORBextractorHost* host;
  {
    std::lock_guard<std::mutex> lock(g_mutex);
    if (!c.host) c.host = new ORBextractorHost(nfeatures, (float)scaleFactor, nlevels, iniThFAST,
                                               minThFAST);
    host = c.host;
  }
  (*host)(_image, _mask, _keypoints, _descriptors);
  mvImagePyramid = host->mvImagePyramid;
}

// The GPU context of an extractor whose last call ran on the device, for the stereo shim
// (orbx_stereo_matches works on the last extraction of the left and right extractors, still
// resident on the GPU); NULL when that call was served by the host fallback.
orbx_extractor* orbx_context_of(const ORBextractor* self) {
  std::lock_guard<std::mutex> lock(g_mutex);
  auto it = g_ctx.find(self);
  return it == g_ctx.end() || !it->second.last_on_device ? nullptr : it->second.ex;
}

bool orbx_materialize_pyramid(ORBextractor* self) {
  if (!self) return false;
  orbx_extractor* ex;
  cv::Mat image;
  {
    std::lock_guard<std::mutex> lock(g_mutex);
    auto it = g_ctx.find(self);
    if (it == g_ctx.end() || !it->second.last_on_device || it->second.pyramid_exported)
      return true;  // host-served call (levels already there) or already exported
    ex = it->second.ex;
    image = it->second.last_image;
  }
  // the extractor is not reentrant (ORBextractor.h), so its owner's thread is the only writer
  int rc = export_pyramid(ex, self->GetLevels(), self->mvImagePyramid);
  if (rc != ORBX_OK) {
    // never leave the previous frame's (or partly exported) levels for the reader: rebuild them
    // with the reference's own ComputePyramid through the host extractor on the same input
    log_once("orbx_extractor_pyramid", rc);
    for (cv::Mat& m : self->mvImagePyramid) m.release();
    if (image.empty()) return false;
    ORBextractorHost* host;
    {
      std::lock_guard<std::mutex> lock(g_mutex);
      ExtractorCtx& c = g_ctx[self];
      if (!c.host) c.host = new ORBextractorHost(c.p.nfeatures, c.p.scale_factor, c.p.nlevels,
                                                 c.p.ini_th_fast, c.p.min_th_fast);
      host = c.host;
    }
    std::vector<cv::KeyPoint> kps;
    cv::Mat desc;
    (*host)(image, cv::Mat(), kps, desc);  // the keypoints equal the device call's (unused)
    self->mvImagePyramid = host->mvImagePyramid;
  }
  std::lock_guard<std::mutex> lock(g_mutex);
  ExtractorCtx& c = g_ctx[self];
  c.pyramid_exported = true;
  c.last_image = cv::Mat();  // consumed: no header on the caller's buffer past this frame
  return true;
}

}  // namespace ORB_SLAM2
