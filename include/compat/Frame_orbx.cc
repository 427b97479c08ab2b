// Frame_orbx.cc — the Frame / KeyFrame work the library runs on the GPU (see Frame_orbx.h):
// Frame::ComputeBoW / KeyFrame::ComputeBoW (TemplatedVocabulary::transform, levelsup 4) and
// Frame::ComputeStereoMatches.  Each returns false instead of failing, and the reference's body
// runs then, so the callers' results are the reference's either way.
#include <memory>
#include <mutex>
#include <vector>

#include "Frame_orbx.h"
#include "ORBextractor.h"

namespace ORB_SLAM2 {

namespace {
// The device vocabulary is shared: a transform running in one thread keeps the vocabulary it
// started with alive while another thread loads a new one (the last holder destroys it).
std::mutex g_voc_mutex;
std::shared_ptr<orbx_vocabulary> g_voc;
}  // namespace

bool orbx_load_vocabulary(const std::string& path) {
  orbx_vocabulary* v = nullptr;
  const bool ok = orbx_vocabulary_load_text(path.c_str(), /*hip_device*/ 0, &v) == ORBX_OK;
  std::shared_ptr<orbx_vocabulary> nv;
  if (ok) nv.reset(v, orbx_vocabulary_destroy);
  std::lock_guard<std::mutex> lock(g_voc_mutex);
  g_voc = nv;
  return ok;
}

bool orbx_compute_bow(const cv::Mat& descriptors, DBoW2::BowVector& bow, DBoW2::FeatureVector& fv) {
  std::shared_ptr<orbx_vocabulary> voc;
  {
    std::lock_guard<std::mutex> lock(g_voc_mutex);
    voc = g_voc;
  }
  if (!voc) return false;
  const int n = descriptors.rows;
  const size_t m = (size_t)std::max(n, 1);
  // the transform's raw outputs, per thread and reused (Tracking and LocalMapping run ComputeBoW)
  struct Scratch {
    std::vector<uint32_t> bw, fi;
    std::vector<double> bv;
    std::vector<int32_t> fo, ff;
  };
  static thread_local Scratch S;
  S.bw.resize(m);
  S.fi.resize(m + 1);
  S.bv.resize(m);
  S.fo.resize(m + 2);
  S.ff.resize(m);
  int32_t nb = 0, nf = 0;
  if (orbx_vocabulary_transform(voc.get(), descriptors.data, n, 4, nullptr, nullptr, S.bw.data(),
                                S.bv.data(), &nb, S.fi.data(), S.fo.data(), S.ff.data(), &nf) != ORBX_OK)
    return false;
  bow.clear();
  fv.clear();
  // ascending ids: every entry placed at the end by hint, no tree search
  for (int i = 0; i < nb; i++) bow.emplace_hint(bow.end(), S.bw[i], S.bv[i]);
  for (int j = 0; j < nf; j++)
    fv.emplace_hint(fv.end(), S.fi[j],
                    std::vector<unsigned int>(S.ff.begin() + S.fo[j], S.ff.begin() + S.fo[j + 1]));
  return true;
}

bool orbx_compute_stereo_matches(Frame& F) {
  orbx_extractor* l = orbx_context_of(F.mpORBextractorLeft);
  orbx_extractor* r = orbx_context_of(F.mpORBextractorRight);
  // the reference's body reads mvImagePyramid: the device extraction (if any) exports it first;
  // should that fail, no stereo match is made rather than one on another frame's levels
  // (mvuRight / mvDepth -1: "no depth", as the reference leaves unmatched keypoints)
  auto host_body_or_no_depth = [&F] {
    const bool okl = orbx_materialize_pyramid(F.mpORBextractorLeft);
    const bool okr = orbx_materialize_pyramid(F.mpORBextractorRight);
    if (okl && okr) return false;  // run the reference's body
    F.mvuRight.assign(F.N, -1.0f);
    F.mvDepth.assign(F.N, -1.0f);
    return true;
  };
  if (!l || !r) return host_body_or_no_depth();  // an extraction served by the host
  std::vector<float> ur(std::max(F.N, 1)), depth(std::max(F.N, 1));
  int32_t n = 0;
  if (orbx_stereo_matches(l, r, F.mb, F.mbf, ur.data(), depth.data(), &n) != ORBX_OK || n != F.N)
    return host_body_or_no_depth();
  F.mvuRight.assign(ur.begin(), ur.begin() + F.N);
  F.mvDepth.assign(depth.begin(), depth.begin() + F.N);
  return true;
}

}  // namespace ORB_SLAM2
