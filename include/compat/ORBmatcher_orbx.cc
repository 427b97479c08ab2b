// ORBmatcher_orbx.cc — drop-in replacement of ORB_SLAM2/src/ORBmatcher.cc over liborbx.so
// (include/orbx.h).  ORB_SLAM2/include/ORBmatcher.h is unchanged.
//
// Build: replace src/ORBmatcher.cc by this file and include/compat/ORBmatcher_host.cc in the
// library's source list (-I<repo>/include -I<repo>/include/compat, -I ORB_SLAM2/src for the
// host file), link -lorbx.
//
// GPU: SearchByBoW (both), SearchForTriangulation, SearchByProjection (all four: local map, last
// frame, relocalisation, loop-closing Sim3), SearchForInitialization, SearchBySim3, Fuse (both:
// the per-point search; the replace / add-observation step stays here, in the reference's
// order).  Only DescriptorDistance on single pairs stays on the host.  Every GPU call falls
// back to the reference's code on a device error (logged once), so callers see the reference's
// results either way.  MapPoint pointers become masks before a call and come back from the
// returned indices after it.  Reentrant: Tracking, LocalMapping and LoopClosing call these at
// once (System.cc:90-95); the library keeps a stream and workspace per thread.
#include <cmath>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "KeyFrame.h"
#include "MapPoint.h"
#include "ORBmatcher.h"
#include "ORBmatcher_host.h"
#include "orbx.h"

namespace ORB_SLAM2 {

const int ORBmatcher::TH_HIGH = 100;
const int ORBmatcher::TH_LOW = 50;
const int ORBmatcher::HISTO_LENGTH = 30;

namespace {

// One message per entry point (the first fallback of each search is logged, not only the
// first of the whole matcher), and a count per entry point for the caller's diagnostics.
void log_fallback(const char* what, int rc) {
  static std::mutex mu;
  static std::map<std::string, long> seen;
  long count;
  {
    std::lock_guard<std::mutex> lk(mu);
    count = ++seen[what];
  }
  if (count == 1)
    fprintf(stderr, "[orbx] %s failed (%d): falling back to the host ORBmatcher\n", what, rc);
}

// DBoW2::FeatureVector (std::map, node ids ascending) as CSR, refilled in place (the vectors
// keep their capacity from call to call)
struct FeatVecCSR {
  std::vector<uint32_t> ids;
  std::vector<int32_t> off, feats;
  orbx_featvec view;
  void assign(const DBoW2::FeatureVector& fv) {
    ids.clear();
    off.clear();
    feats.clear();
    off.push_back(0);
    for (DBoW2::FeatureVector::const_iterator it = fv.begin(); it != fv.end(); ++it) {
      ids.push_back(it->first);
      feats.insert(feats.end(), it->second.begin(), it->second.end());
      off.push_back((int32_t)feats.size());
    }
    view = orbx_featvec{(int32_t)ids.size(), ids.data(), off.data(), feats.data()};
  }
};

// The per-call host buffers of SearchByBoW / SearchForTriangulation, kept per thread (Tracking,
// LocalMapping and LoopClosing call at once) and reused: no allocation per call once warm.
struct CallScratch {
  FeatVecCSR f1, f2;
  std::vector<uint8_t> m1, m2;
  std::vector<float> a1, a2;
  std::vector<int32_t> idx;
};
CallScratch& scratch() {
  static thread_local CallScratch s;
  return s;
}

void angles_of(const std::vector<cv::KeyPoint>& k, std::vector<float>& a) {
  a.resize(k.size());
  for (size_t i = 0; i < k.size(); i++) a[i] = k[i].angle;
}

const orbx_keypoint* keys_of(const std::vector<cv::KeyPoint>& k) {
  return reinterpret_cast<const orbx_keypoint*>(k.data());
}

// A Frame as the tracking searches see it (grid frame: Frame's static members)
orbx_proj_frame frame_view(const Frame& F, const uint8_t* has_mp_obs) {
  orbx_proj_frame f{};
  f.n = F.N;
  f.keys_un = keys_of(F.mvKeysUn);
  f.desc = F.mDescriptors.data;
  f.u_right = F.mvuRight.empty() ? nullptr : F.mvuRight.data();
  f.has_mp_obs = has_mp_obs;
  f.min_x = Frame::mnMinX;
  f.min_y = Frame::mnMinY;
  f.max_x = Frame::mnMaxX;
  f.max_y = Frame::mnMaxY;
  f.grid_w_inv = Frame::mfGridElementWidthInv;
  f.grid_h_inv = Frame::mfGridElementHeightInv;
  f.scale_factors = F.mvScaleFactors.data();
  f.nlevels = (int32_t)F.mvScaleFactors.size();
  return f;
}

// A KeyFrame as KeyFrame::GetFeaturesInArea sees it (its own grid frame, KeyFrame.cc:518-558)
orbx_proj_frame keyframe_view(const KeyFrame* K) {
  orbx_proj_frame f{};
  f.n = K->N;
  f.keys_un = keys_of(K->mvKeysUn);
  f.desc = K->mDescriptors.data;
  f.u_right = K->mvuRight.empty() ? nullptr : K->mvuRight.data();
  f.has_mp_obs = nullptr;
  f.min_x = (float)K->mnMinX;
  f.min_y = (float)K->mnMinY;
  f.max_x = (float)K->mnMaxX;
  f.max_y = (float)K->mnMaxY;
  f.grid_w_inv = K->mfGridElementWidthInv;
  f.grid_h_inv = K->mfGridElementHeightInv;
  f.scale_factors = K->mvScaleFactors.data();
  f.nlevels = (int32_t)K->mvScaleFactors.size();
  return f;
}

}  // namespace

ORBmatcher::ORBmatcher(float nnratio, bool checkOri)
    : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

int ORBmatcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  return ORBmatcherHost::DescriptorDistance(a, b);  // single pairs stay on the host
}

// ------------------------------------------------------------------ SearchByBoW (:159-288)
int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
  CallScratch& S = scratch();
  const std::vector<MapPoint*> vpMP = pKF->GetMapPointMatches();
  S.m1.resize(vpMP.size());
  for (size_t i = 0; i < vpMP.size(); i++) S.m1[i] = vpMP[i] && !vpMP[i]->isBad();
  angles_of(pKF->mvKeysUn, S.a1);
  angles_of(F.mvKeys, S.a2);
  S.f1.assign(pKF->mFeatVec);
  S.f2.assign(F.mFeatVec);
  const orbx_bow_side kf{pKF->N, pKF->mDescriptors.data, S.a1.data(), S.m1.data(), S.f1.view};
  const orbx_bow_side fr{F.N, F.mDescriptors.data, S.a2.data(), nullptr, S.f2.view};
  S.idx.resize(std::max(F.N, 1));
  const std::vector<int32_t>& match = S.idx;
  int32_t n = 0;
  const int rc = orbx_search_by_bow_kf_f(&kf, &fr, mfNNratio, mbCheckOrientation, S.idx.data(), &n);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_by_bow_kf_f", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation).SearchByBoW(pKF, F, vpMapPointMatches);
  }
  vpMapPointMatches.assign(F.N, static_cast<MapPoint*>(NULL));
  for (int i = 0; i < F.N; i++)
    if (match[i] >= 0) vpMapPointMatches[i] = vpMP[match[i]];
  return n;
}

// (:525-658)
int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
  CallScratch& S = scratch();
  const std::vector<MapPoint*> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
  S.m1.resize(vp1.size());
  S.m2.resize(vp2.size());
  for (size_t i = 0; i < vp1.size(); i++) S.m1[i] = vp1[i] && !vp1[i]->isBad();
  for (size_t i = 0; i < vp2.size(); i++) S.m2[i] = vp2[i] && !vp2[i]->isBad();
  angles_of(pKF1->mvKeysUn, S.a1);
  angles_of(pKF2->mvKeysUn, S.a2);
  S.f1.assign(pKF1->mFeatVec);
  S.f2.assign(pKF2->mFeatVec);
  const orbx_bow_side s1{pKF1->N, pKF1->mDescriptors.data, S.a1.data(), S.m1.data(), S.f1.view};
  const orbx_bow_side s2{pKF2->N, pKF2->mDescriptors.data, S.a2.data(), S.m2.data(), S.f2.view};
  S.idx.resize(std::max(pKF1->N, 1));
  const std::vector<int32_t>& match = S.idx;
  int32_t n = 0;
  const int rc = orbx_search_by_bow_kf_kf(&s1, &s2, mfNNratio, mbCheckOrientation, S.idx.data(), &n);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_by_bow_kf_kf", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation).SearchByBoW(pKF1, pKF2, vpMatches12);
  }
  vpMatches12.assign(pKF1->N, static_cast<MapPoint*>(NULL));
  for (int i = 0; i < pKF1->N; i++)
    if (match[i] >= 0) vpMatches12[i] = vp2[match[i]];
  return n;
}

// ------------------------------------------------------------------ SearchForTriangulation
// (:660-826); the epipole with the reference's own cv::Mat arithmetic (:667-673)
int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
                                       std::vector<pair<size_t, size_t> >& vMatchedPairs,
                                       const bool bOnlyStereo) {
  cv::Mat Cw = pKF1->GetCameraCenter();
  cv::Mat R2w = pKF2->GetRotation();
  cv::Mat t2w = pKF2->GetTranslation();
  cv::Mat C2 = R2w * Cw + t2w;
  const float invz = 1.0f / C2.at<float>(2);
  const float ex = pKF2->fx * C2.at<float>(0) * invz + pKF2->cx;
  const float ey = pKF2->fy * C2.at<float>(1) * invz + pKF2->cy;
  CallScratch& S = scratch();
  S.m1.resize(pKF1->N);
  S.m2.resize(pKF2->N);
  // the reference reads GetMapPoint(idx) per candidate (:702, :725), one lock each; one snapshot
  // per keyframe (one lock) reads the same pointers
  {
    const std::vector<MapPoint*> vp1 = pKF1->GetMapPointMatches();
    const std::vector<MapPoint*> vp2 = pKF2->GetMapPointMatches();
    for (int i = 0; i < pKF1->N; i++) S.m1[i] = vp1[i] != NULL;
    for (int i = 0; i < pKF2->N; i++) S.m2[i] = vp2[i] != NULL;
  }
  S.f1.assign(pKF1->mFeatVec);
  S.f2.assign(pKF2->mFeatVec);
  const orbx_tri_side s1{pKF1->N, pKF1->mDescriptors.data, keys_of(pKF1->mvKeysUn),
                         pKF1->mvuRight.data(), S.m1.data(), S.f1.view, pKF1->mvScaleFactors.data(),
                         pKF1->mvLevelSigma2.data(), (int32_t)pKF1->mvScaleFactors.size()};
  const orbx_tri_side s2{pKF2->N, pKF2->mDescriptors.data, keys_of(pKF2->mvKeysUn),
                         pKF2->mvuRight.data(), S.m2.data(), S.f2.view, pKF2->mvScaleFactors.data(),
                         pKF2->mvLevelSigma2.data(), (int32_t)pKF2->mvScaleFactors.size()};
  float F[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) F[3 * r + c] = F12.at<float>(r, c);
  S.idx.resize(2 * std::max(pKF1->N, 1));
  const std::vector<int32_t>& pairs = S.idx;
  int32_t n = 0;
  const int rc = orbx_search_for_triangulation(&s1, &s2, F, ex, ey, bOnlyStereo, mfNNratio,
                                               mbCheckOrientation, S.idx.data(), &n);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_for_triangulation", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation)
        .SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo);
  }
  vMatchedPairs.clear();
  vMatchedPairs.reserve(n);
  for (int i = 0; i < n; i++)  // ascending idx1, as the reference's final loop (:818-823)
    vMatchedPairs.push_back(std::make_pair((size_t)pairs[2 * i], (size_t)pairs[2 * i + 1]));
  return n;
}

// ------------------------------------------------------------------ tracking searches
// SearchByProjection(F, vpMapPoints, th) (:45-137), after Tracking::SearchLocalPoints ran
// isInFrustum on the points
int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints,
                                   const float th) {
  const size_t n = vpMapPoints.size();
  std::vector<uint8_t> track(n), has(std::max(F.N, 1));
  std::vector<float> px(n), py(n), pxr(n), vcos(n);
  std::vector<int32_t> lev(n);
  std::vector<uint8_t> desc(32 * std::max<size_t>(n, 1));
  for (size_t i = 0; i < n; i++) {
    MapPoint* p = vpMapPoints[i];
    track[i] = p->mbTrackInView && !p->isBad();
    px[i] = p->mTrackProjX;
    py[i] = p->mTrackProjY;
    pxr[i] = p->mTrackProjXR;
    lev[i] = p->mnTrackScaleLevel;
    vcos[i] = p->mTrackViewCos;
    if (track[i]) {
      const cv::Mat d = p->GetDescriptor();
      std::copy(d.data, d.data + 32, desc.begin() + 32 * i);
    }
  }
  for (int i = 0; i < F.N; i++)
    has[i] = F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0;
  const orbx_proj_frame fr = frame_view(F, has.data());
  const orbx_proj_points pts{(int32_t)n, track.data(), px.data(), py.data(), pxr.data(),
                             lev.data(), vcos.data(), desc.data()};
  std::vector<int32_t> match(std::max(F.N, 1));
  int32_t nm = 0;
  const int rc = orbx_search_by_projection(&fr, &pts, th, mfNNratio, match.data(), &nm);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_by_projection", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation).SearchByProjection(F, vpMapPoints, th);
  }
  for (int i = 0; i < F.N; i++)
    if (match[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[match[i]];
  return nm;
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) (:1331-1474): the projection of the
// last frame's points with the reference's cv::Mat code (:1341-1382), the search on the GPU
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th,
                                   const bool bMono) {
  const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);
  const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
  const cv::Mat twc = -Rcw.t() * tcw;
  const cv::Mat Rlw = LastFrame.mTcw.rowRange(0, 3).colRange(0, 3);
  const cv::Mat tlw = LastFrame.mTcw.rowRange(0, 3).col(3);
  const cv::Mat tlc = Rlw * twc + tlw;
  const bool bForward = tlc.at<float>(2) > CurrentFrame.mb && !bMono;
  const bool bBackward = -tlc.at<float>(2) > CurrentFrame.mb && !bMono;
  const int nl = LastFrame.N;
  std::vector<uint8_t> valid(std::max(nl, 1)), blocks(std::max(nl, 1)),
      has(std::max(CurrentFrame.N, 1));
  std::vector<float> u(std::max(nl, 1)), v(std::max(nl, 1)), ur(std::max(nl, 1)),
      ang(std::max(nl, 1));
  std::vector<int32_t> oct(std::max(nl, 1));
  std::vector<uint8_t> desc(32 * std::max(nl, 1));
  for (int i = 0; i < nl; i++) {
    MapPoint* pMP = LastFrame.mvpMapPoints[i];
    valid[i] = 0;
    if (!pMP || LastFrame.mvbOutlier[i]) continue;
    cv::Mat x3Dw = pMP->GetWorldPos();
    cv::Mat x3Dc = Rcw * x3Dw + tcw;
    const float xc = x3Dc.at<float>(0);
    const float yc = x3Dc.at<float>(1);
    const float invzc = 1.0 / x3Dc.at<float>(2);
    if (invzc < 0) continue;
    u[i] = CurrentFrame.fx * xc * invzc + CurrentFrame.cx;
    v[i] = CurrentFrame.fy * yc * invzc + CurrentFrame.cy;
    ur[i] = u[i] - CurrentFrame.mbf * invzc;
    oct[i] = LastFrame.mvKeys[i].octave;
    ang[i] = LastFrame.mvKeysUn[i].angle;
    const cv::Mat d = pMP->GetDescriptor();
    std::copy(d.data, d.data + 32, desc.begin() + 32 * i);
    // Tracking::UpdateLastFrame's visual-odometry points have no observations: their feature
    // stays open to later points (:1406-1408)
    blocks[i] = pMP->Observations() > 0;
    valid[i] = 1;
  }
  for (int i = 0; i < CurrentFrame.N; i++)
    has[i] = CurrentFrame.mvpMapPoints[i] && CurrentFrame.mvpMapPoints[i]->Observations() > 0;
  const orbx_proj_frame fr = frame_view(CurrentFrame, has.data());
  const orbx_proj_last last{nl,        valid.data(), u.data(),    v.data(),     ur.data(),
                            oct.data(), ang.data(),   desc.data(), blocks.data()};
  std::vector<int32_t> match(std::max(CurrentFrame.N, 1));
  int32_t nm = 0;
  const int rc = orbx_search_by_projection_last(&fr, &last, th, bForward, bBackward,
                                                mbCheckOrientation, match.data(), &nm);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_by_projection_last", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation)
        .SearchByProjection(CurrentFrame, LastFrame, th, bMono);
  }
  for (int i = 0; i < CurrentFrame.N; i++)
    if (match[i] >= 0) CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[match[i]];
  return nm;
}

// SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:1475-1602,
// Tracking::Relocalization): the projection and gates with the reference's cv::Mat code
// (:1477-1526), the search on the GPU.  Any map point of the current frame blocks its feature.
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF,
                                   const std::set<MapPoint*>& sAlreadyFound, const float th,
                                   const int ORBdist) {
  const cv::Mat Rcw = CurrentFrame.mTcw.rowRange(0, 3).colRange(0, 3);
  const cv::Mat tcw = CurrentFrame.mTcw.rowRange(0, 3).col(3);
  const cv::Mat Ow = -Rcw.t() * tcw;
  const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
  const int nk = (int)vpMPs.size(), m = std::max(nk, 1);
  std::vector<uint8_t> valid(m, 0), has(std::max(CurrentFrame.N, 1)), desc(32 * (size_t)m);
  std::vector<float> u(m), v(m), ang(m);
  std::vector<int32_t> lev(m);
  for (int i = 0; i < nk; i++) {
    MapPoint* pMP = vpMPs[i];
    if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;
    cv::Mat x3Dw = pMP->GetWorldPos();
    cv::Mat x3Dc = Rcw * x3Dw + tcw;
    const float xc = x3Dc.at<float>(0);
    const float yc = x3Dc.at<float>(1);
    const float invzc = 1.0 / x3Dc.at<float>(2);
    u[i] = CurrentFrame.fx * xc * invzc + CurrentFrame.cx;
    v[i] = CurrentFrame.fy * yc * invzc + CurrentFrame.cy;
    // (the image-bounds test runs in the library, as the reference's next lines)
    cv::Mat PO = x3Dw - Ow;
    const float dist3D = cv::norm(PO);
    const float maxDistance = pMP->GetMaxDistanceInvariance();
    const float minDistance = pMP->GetMinDistanceInvariance();
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    lev[i] = pMP->PredictScale(dist3D, CurrentFrame.mfLogScaleFactor);
    ang[i] = pKF->mvKeysUn[i].angle;
    const cv::Mat d = pMP->GetDescriptor();
    std::copy(d.data, d.data + 32, desc.begin() + 32 * i);
    valid[i] = 1;
  }
  for (int i = 0; i < CurrentFrame.N; i++) has[i] = CurrentFrame.mvpMapPoints[i] != NULL;
  orbx_proj_frame fr = frame_view(CurrentFrame, has.data());
  fr.u_right = nullptr;
  const orbx_proj_last pts{nk,         valid.data(), u.data(),    v.data(), nullptr,
                           lev.data(), ang.data(),   desc.data(), nullptr};  // any point blocks
  std::vector<int32_t> match(std::max(CurrentFrame.N, 1));
  int32_t nm = 0;
  const int rc = orbx_search_by_projection_kf(&fr, &pts, th, ORBdist, mbCheckOrientation,
                                              match.data(), &nm);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_by_projection_kf", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation)
        .SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist);
  }
  for (int i = 0; i < CurrentFrame.N; i++)
    if (match[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[match[i]];
  return nm;
}

// SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (:290-403, loop closing): the Sim3
// decomposition, projection and gates with the reference's code (:292-352), the search on the GPU
int ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints,
                                   std::vector<MapPoint*>& vpMatched, int th) {
  const float& fx = pKF->fx;
  const float& fy = pKF->fy;
  const float& cx = pKF->cx;
  const float& cy = pKF->cy;
  cv::Mat sRcw = Scw.rowRange(0, 3).colRange(0, 3);
  const float scw = std::sqrt(sRcw.row(0).dot(sRcw.row(0)));
  cv::Mat Rcw = sRcw / scw;
  cv::Mat tcw = Scw.rowRange(0, 3).col(3) / scw;
  cv::Mat Ow = -Rcw.t() * tcw;
  std::set<MapPoint*> spAlreadyFound(vpMatched.begin(), vpMatched.end());
  spAlreadyFound.erase(static_cast<MapPoint*>(NULL));
  const int np = (int)vpPoints.size(), m = std::max(np, 1);
  std::vector<uint8_t> use(m, 0), desc(32 * (size_t)m), matched(std::max(pKF->N, 1));
  std::vector<float> u(m), v(m);
  std::vector<int32_t> lev(m);
  for (int i = 0; i < np; i++) {
    MapPoint* pMP = vpPoints[i];
    if (pMP->isBad() || spAlreadyFound.count(pMP)) continue;
    cv::Mat p3Dw = pMP->GetWorldPos();
    cv::Mat p3Dc = Rcw * p3Dw + tcw;
    if (p3Dc.at<float>(2) < 0.0) continue;
    const float invz = 1 / p3Dc.at<float>(2);
    const float x = p3Dc.at<float>(0) * invz;
    const float y = p3Dc.at<float>(1) * invz;
    u[i] = fx * x + cx;
    v[i] = fy * y + cy;
    if (!pKF->IsInImage(u[i], v[i])) continue;
    const float maxDistance = pMP->GetMaxDistanceInvariance();
    const float minDistance = pMP->GetMinDistanceInvariance();
    cv::Mat PO = p3Dw - Ow;
    const float dist = cv::norm(PO);
    if (dist < minDistance || dist > maxDistance) continue;
    cv::Mat Pn = pMP->GetNormal();
    if (PO.dot(Pn) < 0.5 * dist) continue;
    lev[i] = pMP->PredictScale(dist, pKF->mfLogScaleFactor);
    const cv::Mat d = pMP->GetDescriptor();
    std::copy(d.data, d.data + 32, desc.begin() + 32 * i);
    use[i] = 1;
  }
  for (int i = 0; i < pKF->N; i++) matched[i] = vpMatched[i] != NULL;
  orbx_proj_frame kf = keyframe_view(pKF);
  kf.has_mp_obs = matched.data();
  const orbx_fuse_points pts{np, use.data(), u.data(), v.data(), nullptr, lev.data(), desc.data()};
  std::vector<int32_t> match(std::max(pKF->N, 1));
  int32_t nm = 0;
  const int rc = orbx_search_by_projection_sim3(&kf, &pts, (float)th, match.data(), &nm);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_by_projection_sim3", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation)
        .SearchByProjection(pKF, Scw, vpPoints, vpMatched, th);
  }
  for (int i = 0; i < pKF->N; i++)
    if (match[i] >= 0) vpMatched[i] = vpPoints[match[i]];
  return nm;
}

// SearchBySim3 (:1105-1329; LoopClosing::ComputeSim3): both directions' projections and gates
// with the reference's code (:1108-1180, :1208-1255), the searches and the agreement on the GPU
int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12,
                             const float& s12, const cv::Mat& R12, const cv::Mat& t12,
                             const float th) {
  const float& fx = pKF1->fx;
  const float& fy = pKF1->fy;
  const float& cx = pKF1->cx;
  const float& cy = pKF1->cy;
  cv::Mat R1w = pKF1->GetRotation();
  cv::Mat t1w = pKF1->GetTranslation();
  cv::Mat R2w = pKF2->GetRotation();
  cv::Mat t2w = pKF2->GetTranslation();
  cv::Mat sR12 = s12 * R12;
  cv::Mat sR21 = (1.0 / s12) * R12.t();
  cv::Mat t21 = -sR21 * t12;
  const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
  const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
  const int N1 = (int)vpMapPoints1.size(), N2 = (int)vpMapPoints2.size();
  std::vector<bool> vbAlreadyMatched1(N1, false), vbAlreadyMatched2(N2, false);
  for (int i = 0; i < N1; i++) {
    MapPoint* pMP = vpMatches12[i];
    if (pMP) {
      vbAlreadyMatched1[i] = true;
      const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
      if (idx2 >= 0 && idx2 < N2) vbAlreadyMatched2[idx2] = true;
    }
  }
  struct Side {
    std::vector<uint8_t> use, desc;
    std::vector<float> u, v;
    std::vector<int32_t> lev;
  } sd[2];
  // direction 0: KF1's points into KF2 (p3Dc2 = sR21 (R1w p + t1w) + t21); 1: KF2's into KF1
  for (int k = 0; k < 2; k++) {
    const std::vector<MapPoint*>& vp = k == 0 ? vpMapPoints1 : vpMapPoints2;
    const std::vector<bool>& already = k == 0 ? vbAlreadyMatched1 : vbAlreadyMatched2;
    KeyFrame* pTo = k == 0 ? pKF2 : pKF1;
    const int n = (int)vp.size(), m = std::max(n, 1);
    Side& S = sd[k];
    S.use.assign(m, 0);
    S.desc.assign(32 * (size_t)m, 0);
    S.u.assign(m, 0.f);
    S.v.assign(m, 0.f);
    S.lev.assign(m, 0);
    for (int i = 0; i < n; i++) {
      MapPoint* pMP = vp[i];
      if (!pMP || already[i] || pMP->isBad()) continue;
      cv::Mat p3Dw = pMP->GetWorldPos();
      cv::Mat p3Dc;
      if (k == 0) {  // the reference's two statements (:1160-1161, :1235-1236)
        cv::Mat p3Dc1 = R1w * p3Dw + t1w;
        p3Dc = sR21 * p3Dc1 + t21;
      } else {
        cv::Mat p3Dc2 = R2w * p3Dw + t2w;
        p3Dc = sR12 * p3Dc2 + t12;
      }
      if (p3Dc.at<float>(2) < 0.0) continue;
      const float invz = 1.0 / p3Dc.at<float>(2);
      const float x = p3Dc.at<float>(0) * invz;
      const float y = p3Dc.at<float>(1) * invz;
      S.u[i] = fx * x + cx;
      S.v[i] = fy * y + cy;
      if (!pTo->IsInImage(S.u[i], S.v[i])) continue;
      const float maxDistance = pMP->GetMaxDistanceInvariance();
      const float minDistance = pMP->GetMinDistanceInvariance();
      const float dist3D = cv::norm(p3Dc);
      if (dist3D < minDistance || dist3D > maxDistance) continue;
      S.lev[i] = pMP->PredictScale(dist3D, pTo->mfLogScaleFactor);
      const cv::Mat d = pMP->GetDescriptor();
      std::copy(d.data, d.data + 32, S.desc.begin() + 32 * i);
      S.use[i] = 1;
    }
  }
  const orbx_proj_frame k1 = keyframe_view(pKF1), k2 = keyframe_view(pKF2);
  const orbx_fuse_points p12{N1, sd[0].use.data(), sd[0].u.data(), sd[0].v.data(), nullptr,
                             sd[0].lev.data(), sd[0].desc.data()};
  const orbx_fuse_points p21{N2, sd[1].use.data(), sd[1].u.data(), sd[1].v.data(), nullptr,
                             sd[1].lev.data(), sd[1].desc.data()};
  std::vector<int32_t> m12(std::max(N1, 1));
  int32_t nFound = 0;
  const int rc = orbx_search_by_sim3(&k1, &k2, &p12, &p21, th, m12.data(), &nFound);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_by_sim3", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation)
        .SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th);
  }
  for (int i1 = 0; i1 < N1; i1++)  // (:1305-1326)
    if (m12[i1] >= 0) vpMatches12[i1] = vpMapPoints2[m12[i1]];
  return nFound;
}

// ------------------------------------------------------------------ SearchForInitialization
// (:405-523; Tracking::MonocularInitialization, Tracking.cc:953)
int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, std::vector<cv::Point2f>& vbPrevMatched,
                                        std::vector<int>& vnMatches12, int windowSize) {
  static_assert(sizeof(cv::Point2f) == 8, "vbPrevMatched is (x, y) float pairs");
  const orbx_proj_frame f1 = frame_view(F1, nullptr), f2 = frame_view(F2, nullptr);
  std::vector<cv::Point2f> prev = vbPrevMatched;
  std::vector<int32_t> m12(std::max(F1.N, 1));
  int32_t nm = 0;
  const int rc = orbx_search_for_initialization(&f1, &f2, reinterpret_cast<float*>(prev.data()),
                                                windowSize, mfNNratio, mbCheckOrientation,
                                                m12.data(), &nm);
  if (rc != ORBX_OK) {
    log_fallback("orbx_search_for_initialization", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation)
        .SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize);
  }
  vbPrevMatched.swap(prev);
  vnMatches12.assign(m12.begin(), m12.begin() + F1.N);
  return nm;
}

// ------------------------------------------------------------------ Fuse
// The gates and projections before the search with the reference's cv::Mat code (:830-893,
// :983-1052); the per-point search on the GPU; then the reference's replace / add-observation
// step in point order.  That step re-checks isBad() / IsInKeyFrame() as the reference's loop
// does at each point.  A point whose descriptor an earlier Replace() rewrote (it absorbed
// observations: ComputeDistinctiveDescriptors) is searched again by the reference's own code.
int ORBmatcher::Fuse(KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, const float th) {
  cv::Mat Rcw = pKF->GetRotation();
  cv::Mat tcw = pKF->GetTranslation();
  const float& fx = pKF->fx;
  const float& fy = pKF->fy;
  const float& cx = pKF->cx;
  const float& cy = pKF->cy;
  const float& bf = pKF->mbf;
  cv::Mat Ow = pKF->GetCameraCenter();
  const int nMPs = (int)vpMapPoints.size();
  const int m = std::max(nMPs, 1);
  std::vector<uint8_t> use(m, 0), desc(32 * (size_t)m);
  std::vector<float> u(m), v(m), ur(m);
  std::vector<int32_t> lev(m);
  for (int i = 0; i < nMPs; i++) {
    MapPoint* pMP = vpMapPoints[i];
    if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
    cv::Mat p3Dw = pMP->GetWorldPos();
    cv::Mat p3Dc = Rcw * p3Dw + tcw;
    if (p3Dc.at<float>(2) < 0.0f) continue;
    const float invz = 1 / p3Dc.at<float>(2);
    const float x = p3Dc.at<float>(0) * invz;
    const float y = p3Dc.at<float>(1) * invz;
    u[i] = fx * x + cx;
    v[i] = fy * y + cy;
    if (!pKF->IsInImage(u[i], v[i])) continue;
    ur[i] = u[i] - bf * invz;
    const float maxDistance = pMP->GetMaxDistanceInvariance();
    const float minDistance = pMP->GetMinDistanceInvariance();
    cv::Mat PO = p3Dw - Ow;
    const float dist3D = cv::norm(PO);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    cv::Mat Pn = pMP->GetNormal();
    if (PO.dot(Pn) < 0.5 * dist3D) continue;
    lev[i] = pMP->PredictScale(dist3D, pKF->mfLogScaleFactor);
    const cv::Mat d = pMP->GetDescriptor();
    std::copy(d.data, d.data + 32, desc.begin() + 32 * i);
    use[i] = 1;
  }
  const orbx_proj_frame kf = keyframe_view(pKF);
  const orbx_fuse_points pts{nMPs, use.data(), u.data(), v.data(), ur.data(), lev.data(),
                             desc.data()};
  std::vector<int32_t> best(m);
  const int rc = orbx_fuse(&kf, pKF->mvInvLevelSigma2.data(), &pts, th, best.data(), nullptr,
                           nullptr);
  if (rc != ORBX_OK) {
    log_fallback("orbx_fuse", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation).Fuse(pKF, vpMapPoints, th);
  }
  int nFused = 0;
  std::set<MapPoint*> rewritten;  // descriptors an earlier Replace() recomputed
  for (int i = 0; i < nMPs; i++) {
    MapPoint* pMP = vpMapPoints[i];
    if (pMP && rewritten.count(pMP)) {  // its gates and search on its new state: the
      nFused += ORBmatcherHost(mfNNratio, mbCheckOrientation)  // reference's own iteration
                    .Fuse(pKF, std::vector<MapPoint*>(1, pMP), th);
      continue;
    }
    if (!use[i] || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
    const int bestIdx = best[i];
    if (bestIdx < 0) continue;  // bestDist > TH_LOW (:955)
    MapPoint* pMPinKF = pKF->GetMapPoint(bestIdx);
    if (pMPinKF) {
      if (!pMPinKF->isBad()) {
        if (pMPinKF->Observations() > pMP->Observations()) {
          pMP->Replace(pMPinKF);
          rewritten.insert(pMPinKF);
        } else {
          pMPinKF->Replace(pMP);
          rewritten.insert(pMP);
        }
      }
    } else {
      pMP->AddObservation(pKF, bestIdx);
      pKF->AddMapPoint(pMP, bestIdx);
    }
    nFused++;
  }
  return nFused;
}

// Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (:980-1103; LoopClosing::SearchAndFuse)
int ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const std::vector<MapPoint*>& vpPoints, float th,
                     std::vector<MapPoint*>& vpReplacePoint) {
  const float& fx = pKF->fx;
  const float& fy = pKF->fy;
  const float& cx = pKF->cx;
  const float& cy = pKF->cy;
  cv::Mat sRcw = Scw.rowRange(0, 3).colRange(0, 3);
  const float scw = std::sqrt(sRcw.row(0).dot(sRcw.row(0)));
  cv::Mat Rcw = sRcw / scw;
  cv::Mat tcw = Scw.rowRange(0, 3).col(3) / scw;
  cv::Mat Ow = -Rcw.t() * tcw;
  const std::set<MapPoint*> spAlreadyFound = pKF->GetMapPoints();
  const int nPoints = (int)vpPoints.size();
  const int m = std::max(nPoints, 1);
  std::vector<uint8_t> use(m, 0), desc(32 * (size_t)m);
  std::vector<float> u(m), v(m);
  std::vector<int32_t> lev(m);
  for (int i = 0; i < nPoints; i++) {
    MapPoint* pMP = vpPoints[i];
    if (pMP->isBad() || spAlreadyFound.count(pMP)) continue;
    cv::Mat p3Dw = pMP->GetWorldPos();
    cv::Mat p3Dc = Rcw * p3Dw + tcw;
    if (p3Dc.at<float>(2) < 0.0f) continue;
    const float invz = 1.0 / p3Dc.at<float>(2);
    const float x = p3Dc.at<float>(0) * invz;
    const float y = p3Dc.at<float>(1) * invz;
    u[i] = fx * x + cx;
    v[i] = fy * y + cy;
    if (!pKF->IsInImage(u[i], v[i])) continue;
    const float maxDistance = pMP->GetMaxDistanceInvariance();
    const float minDistance = pMP->GetMinDistanceInvariance();
    cv::Mat PO = p3Dw - Ow;
    const float dist3D = cv::norm(PO);
    if (dist3D < minDistance || dist3D > maxDistance) continue;
    cv::Mat Pn = pMP->GetNormal();
    if (PO.dot(Pn) < 0.5 * dist3D) continue;
    lev[i] = pMP->PredictScale(dist3D, pKF->mfLogScaleFactor);
    const cv::Mat d = pMP->GetDescriptor();
    std::copy(d.data, d.data + 32, desc.begin() + 32 * i);
    use[i] = 1;
  }
  const orbx_proj_frame kf = keyframe_view(pKF);
  const orbx_fuse_points pts{nPoints, use.data(), u.data(), v.data(), nullptr, lev.data(),
                             desc.data()};
  std::vector<int32_t> best(m);
  const int rc = orbx_fuse_sim3(&kf, &pts, th, best.data(), nullptr, nullptr);
  if (rc != ORBX_OK) {
    log_fallback("orbx_fuse_sim3", rc);
    return ORBmatcherHost(mfNNratio, mbCheckOrientation).Fuse(pKF, Scw, vpPoints, th, vpReplacePoint);
  }
  int nFused = 0;
  for (int i = 0; i < nPoints; i++) {  // (:1084-1099)
    if (!use[i] || best[i] < 0) continue;
    MapPoint* pMP = vpPoints[i];
    MapPoint* pMPinKF = pKF->GetMapPoint(best[i]);
    if (pMPinKF) {
      if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
    } else {
      pMP->AddObservation(pKF, best[i]);
      pKF->AddMapPoint(pMP, best[i]);
    }
    nFused++;
  }
  return nFused;
}

// (CheckDistEpipolarLine, RadiusByViewingCos and ComputeThreeMaxima are called only from the
// reference's own search bodies, which run in ORBmatcherHost; no definition is needed here.)

}  // namespace ORB_SLAM2
