/*
 * orbx.h — C ABI of the MI355X ORB front end (drop-in for ORB-SLAM2's ORBextractor /
 * ORBmatcher hot path).  Plain pointers and sizes only; no torch, HIP or OpenCV types.
 *
 * Reference interfaces each entry point replaces (paths relative to the reference tree):
 *   orbx_extractor_create   ORBextractor::ORBextractor        ORB_SLAM2/include/ORBextractor.h:52-53,
 *                                                             ORB_SLAM2/src/ORBextractor.cc:404-460
 *   orbx_extractor_tables   GetLevels/GetScaleFactor(s)/...    ORB_SLAM2/include/ORBextractor.h:64-86
 *   orbx_extract            ORBextractor::operator()          ORB_SLAM2/include/ORBextractor.h:61-62,
 *                                                             ORB_SLAM2/src/ORBextractor.cc:985-1045
 *   orbx_extractor_pyramid  ORBextractor::mvImagePyramid      ORB_SLAM2/include/ORBextractor.h:88
 *   orbx_descriptor_distance ORBmatcher::DescriptorDistance   ORB_SLAM2/src/ORBmatcher.cc:1650-1666
 *   orbx_search_by_bow_kf_f  ORBmatcher::SearchByBoW(KF*,F&)   ORB_SLAM2/src/ORBmatcher.cc:159-288
 *   orbx_search_by_bow_kf_kf ORBmatcher::SearchByBoW(KF*,KF*)  ORB_SLAM2/src/ORBmatcher.cc:525-658
 *   orbx_search_for_triangulation
 *                           ORBmatcher::SearchForTriangulation ORB_SLAM2/src/ORBmatcher.cc:660-826
 *   orbx_vocabulary_*       DBoW2 TemplatedVocabulary<FORB>: loadFromTextFile and
 *                           transform(features, BowVector&, FeatureVector&, levelsup)
 *                           ORB_SLAM2/Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1259,
 *                           1338-1424 (called by Frame::ComputeBoW, ORB_SLAM2/src/Frame.cc:400-407)
 *
 *   orbx_cvorb_*            cv::ORB (OpenCV 2.4, scoreType HARRIS_SCORE/FAST_SCORE) ::operator()
 *                           as called by the AR marker path: Marker::setTargetImage / Marker::Match
 *                           ORB_SLAM2/src/Marker.cc:76-84, 98-108; AR-1.3/src/ORBMatcher.cpp:121-122
 *   orbx_bf_match           BruteForceMatcher<HammingLUT>::match   ORB_SLAM2/src/Marker.cc:110-113
 *   orbx_good_matches       Marker::Match good-match filter        ORB_SLAM2/src/Marker.cc:115-133
 *   orbx_nn_match           naive_nn_search / naive_nn_search2     AR-1.3/src/ORBMatcher.cpp:44-102,
 *                           Marker::searchMatches                  ORB_SLAM2/src/Marker.cc:314-349
 *   orbx_marker_*           Marker::Match's extract + match + filter for a batch of frames against
 *                           one target (the homography/RANSAC part stays with the caller)
 *
 * Error convention: every function returns 0 on success or a negative ORBX_E* code; nothing
 * throws across the ABI.  The reference has no error returns (asserts are compiled out,
 * ORB_SLAM2/CMakeLists.txt:10-11); callers that must never fail map a negative code to
 * "no features / no matches".
 *
 * Threading: an orbx_extractor is not reentrant (like ORBextractor, which mutates
 * mvImagePyramid); distinct extractors may run concurrently.  Matcher entry points are
 * stateless and reentrant (ORBmatcher is called from the Tracking, LocalMapping and
 * LoopClosing threads at once).
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBX_ABI_VERSION 1

enum {
  ORBX_OK = 0,
  ORBX_EINVAL = -1,     /* bad argument (null pointer, size out of range)          */
  ORBX_ENOMEM = -2,     /* device or host allocation failed                        */
  ORBX_EDEVICE = -3,    /* HIP runtime error                                        */
  ORBX_ECAPACITY = -4,  /* caller buffer too small; *n_out holds the needed count   */
  ORBX_EUNSUPPORTED = -5 /* configuration outside what the path implements          */
};

/* == cv::KeyPoint (OpenCV 2.4): {pt.x, pt.y, size, angle, response, octave, class_id}, 28 B.
 * SURVEY §8a A11. */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orbx_keypoint;

/* ORBextractor constructor arguments (ORB_SLAM2/include/ORBextractor.h:52-53). */
typedef struct {
  int32_t nfeatures;
  float scale_factor;
  int32_t nlevels;
  int32_t ini_th_fast;
  int32_t min_th_fast;
} orbx_params;

/* A DBoW2::FeatureVector in CSR form (std::map<NodeId, vector<unsigned>>,
 * FeatureVector.h:21-52): node_ids ascending; node_offsets[n_nodes+1]; node_feats holds the
 * feature indices of node k at [node_offsets[k], node_offsets[k+1]), ascending. */
typedef struct {
  int32_t n_nodes;
  const uint32_t* node_ids;
  const int32_t* node_offsets;
  const int32_t* node_feats;
} orbx_featvec;

/* One side of SearchByBoW.  `valid[i]` = 1 when feature i has a usable MapPoint
 * (pMP && !pMP->isBad(), ORBmatcher.cc:191-197, 561-583); may be NULL for the Frame side of
 * the KF->Frame variant, which does not look at it. */
typedef struct {
  int32_t n;
  const uint8_t* desc;   /* n x 32 B, row per feature */
  const float* angle;    /* n keypoint angles (degrees) */
  const uint8_t* valid;  /* n or NULL */
  orbx_featvec fv;
} orbx_bow_side;

/* One keyframe of SearchForTriangulation (ORBmatcher.cc:660-826). */
typedef struct {
  int32_t n;
  const uint8_t* desc;          /* n x 32 */
  const orbx_keypoint* keys_un; /* mvKeysUn */
  const float* u_right;         /* mvuRight (<0 = mono); NULL = all mono */
  const uint8_t* has_mp;        /* 1 if GetMapPoint(i) != NULL; NULL = none */
  orbx_featvec fv;
  const float* scale_factors;   /* mvScaleFactors [nlevels] */
  const float* level_sigma2;    /* mvLevelSigma2  [nlevels] */
  int32_t nlevels;
} orbx_tri_side;

/* ------------------------------------------------------------------ extractor */
typedef struct orbx_extractor orbx_extractor;

/* Builds the scale / feature-per-level / umax tables (ORBextractor.cc:404-460) and binds a
 * HIP stream on `hip_device`. */
int orbx_extractor_create(const orbx_params* params, int hip_device, orbx_extractor** out);
int orbx_extractor_destroy(orbx_extractor* ex);

/* Table getters (ORBextractor.h:64-86).  Each array must hold nlevels entries; any may be
 * NULL.  features_per_level = mnFeaturesPerLevel. */
int orbx_extractor_tables(const orbx_extractor* ex, int32_t* nlevels, float* scale_factors,
                          float* inv_scale_factors, float* level_sigma2,
                          float* inv_level_sigma2, int32_t* features_per_level);

/* ORBextractor::operator(): u8 gray image (w x h, row stride `stride` bytes, host memory)
 * -> keypoints (level-major, scaled to level-0 coordinates) and n x 32 descriptors.
 * `cap` is the capacity of kps/desc; on ORBX_ECAPACITY *n_out is the required count.
 * An empty image (w==0 or h==0) returns ORBX_OK with *n_out = -1 and touches nothing,
 * mirroring the early return at ORBextractor.cc:987-988. */
int orbx_extract(orbx_extractor* ex, const uint8_t* img, int32_t w, int32_t h, int64_t stride,
                 orbx_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out);

/* mvImagePyramid export for the last orbx_extract call: level `level` (ROI only, the 19-px
 * border is never read by the hot path) into `out` with row stride `stride`.
 * If out is NULL only *w, *h are written. */
int orbx_extractor_pyramid(orbx_extractor* ex, int32_t level, uint8_t* out, int64_t stride,
                           int32_t* w, int32_t* h);

/* ------------------------------------------------------------------ device batch plan
 * Throughput path: a plan is bound to one extractor configuration, one image size and a
 * maximum batch.  Inputs and outputs live in device memory (HBM); the plan's HIP stream
 * runs everything asynchronously.  Used by bench.py and by multi-stream callers. */
typedef struct orbx_plan orbx_plan;

int orbx_plan_create(const orbx_params* params, int32_t w, int32_t h, int32_t max_batch,
                     int hip_device, orbx_plan** out);
int orbx_plan_destroy(orbx_plan* plan);
/* Per-image output capacity (keypoints) of the plan. */
int orbx_plan_capacity(const orbx_plan* plan, int32_t* kp_cap);
/* d_imgs: device pointer, n_images dense images of w*h bytes (stride = w).  Enqueues the
 * whole extract on the plan's stream; returns without waiting. */
int orbx_plan_extract(orbx_plan* plan, const uint8_t* d_imgs, int32_t n_images);
/* Device pointers of the outputs of the last run: kps [max_batch][kp_cap], desc
 * [max_batch][kp_cap][32], counts [max_batch]. */
int orbx_plan_outputs(orbx_plan* plan, orbx_keypoint** d_kps, uint8_t** d_desc,
                      int32_t** d_counts);
int orbx_plan_sync(orbx_plan* plan);
/* Returns the plan's hipStream_t as an opaque pointer. */
void* orbx_plan_stream(orbx_plan* plan);
/* Stage timing (HIP events around each kernel, on the plan's stream).  enable=1 arms it
 * and clears the accumulators; names/ms/launches are copied for up to `cap` stages. */
int orbx_plan_profile(orbx_plan* plan, int32_t enable);
int orbx_plan_profile_read(orbx_plan* plan, int32_t cap, char (*names)[32], double* total_ms,
                           int64_t* launches, int32_t* n_stages);
/* The kernel instances the profiled runs launched for stage `stage` (profile_read order), under
 * the names rocprofv3 reports ("k_pyramid<true>", "k_fast_cells<44, 42, unsigned int>"),
 * ';'-separated into buf (cap bytes, NUL-terminated).  Lets a benchmark bind a stage's time to
 * the counters of exactly those kernels.  ORBX_ECAPACITY (buf = "") when the list needs more than
 * cap bytes: the list is never returned cut. */
int orbx_plan_profile_kernels(orbx_plan* plan, int32_t stage, char* buf, int32_t cap);

/* ------------------------------------------------------------------ projection searches
 * The current Frame as the tracking searches see it: mvKeysUn, mDescriptors, mvuRight, the
 * feature grid frame (mnMinX.., mfGridElementWidthInv/HeightInv; FRAME_GRID 64 x 48,
 * Frame.h:39-40), mvScaleFactors, and has_mp_obs[i] = mvpMapPoints[i] &&
 * mvpMapPoints[i]->Observations() > 0 (those features are skipped). */
typedef struct {
  int32_t n;
  const orbx_keypoint* keys_un;
  const uint8_t* desc;         /* [n][32] */
  const float* u_right;        /* [n], NULL for monocular */
  const uint8_t* has_mp_obs;   /* [n], NULL = none */
  float min_x, min_y, max_x, max_y;
  float grid_w_inv, grid_h_inv;
  const float* scale_factors;  /* [nlevels] */
  int32_t nlevels;
} orbx_proj_frame;
/* Local-map points for SearchByProjection(Frame&, vector<MapPoint*>, th): per point
 * track = mbTrackInView && !isBad(), and the isInFrustum results mTrackProjX / Y / XR,
 * mnTrackScaleLevel, mTrackViewCos (Frame::isInFrustum, Frame.cc:260-330), descriptor
 * GetDescriptor().  Every point passed has Observations() > 0. */
typedef struct {
  int32_t n;
  const uint8_t* track;
  const float *proj_x, *proj_y, *proj_xr;
  const int32_t* pred_level;
  const float* view_cos;
  const uint8_t* desc;         /* [n][32] */
} orbx_proj_points;
/* Last-frame points for SearchByProjection(CurrentFrame, LastFrame, th, bMono): valid[i] =
 * LastFrame.mvpMapPoints[i] && !mvbOutlier[i] && invzc >= 0; u, v the projection into the
 * current frame and ur = u - mbf*invzc (ORBmatcher.cc:1364-1383, evaluated by the caller with
 * the reference's cv::Mat pose products); octave = LastFrame.mvKeys[i].octave, angle =
 * LastFrame.mvKeysUn[i].angle, desc = pMP->GetDescriptor().
 * blocks[i] = pMP->Observations() > 0 (NULL = every point has observations).  A current-frame
 * feature assigned a point without observations (the visual-odometry points
 * Tracking::UpdateLastFrame adds, Tracking.cc:1181-1221) is not skipped by later points
 * (ORBmatcher.cc:1406-1408): a later point may take it over, and nmatches and the rotation
 * histogram count both assignments, as in the reference.  orbx_search_by_projection_kf ignores
 * blocks (any map point blocks there, :1544). */
typedef struct {
  int32_t n;
  const uint8_t* valid;
  const float *u, *v, *ur;
  const int32_t* octave;
  const float* angle;
  const uint8_t* desc;         /* [n][32] */
  const uint8_t* blocks;       /* [n], nullable */
} orbx_proj_last;
/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)
 * (ORB_SLAM2/src/ORBmatcher.cc:45-137): match[f] = index of the point assigned to frame
 * feature f in this call (F.mvpMapPoints[f] = vpMapPoints[match[f]]), else -1. */
int orbx_search_by_projection(const orbx_proj_frame* frame, const orbx_proj_points* points,
                              float th, float nnratio, int32_t* match, int32_t* nmatches);
/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 * (ORBmatcher.cc:1331-1474): match[f] = last-frame index whose MapPoint is assigned to current
 * feature f, else -1.  forward / backward = bForward / bBackward (:1348-1349). */
int orbx_search_by_projection_last(const orbx_proj_frame* frame, const orbx_proj_last* last,
                                   float th, int32_t forward, int32_t backward,
                                   int32_t check_ori, int32_t* match, int32_t* nmatches);
/* ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
 * vector<int>& vnMatches12, int windowSize) (ORB_SLAM2/src/ORBmatcher.cc:405-523; called by
 * Tracking::MonocularInitialization, Tracking.cc:953) of an ORBmatcher(nnratio, checkOri).
 * f1 = the initial frame (n <= 65534, keys_un, desc; the rest unused), f2 = the current frame
 * (keys_un, desc and its grid frame; u_right / has_mp_obs unused).  prev_matched: [f1->n][2]
 * (x, y) = vbPrevMatched, updated in place as the reference updates it (:517-520);
 * matches12[f1->n] = vnMatches12.  No limit on window size or feature density. */
int orbx_search_for_initialization(const orbx_proj_frame* f1, const orbx_proj_frame* f2,
                                   float* prev_matched, int32_t window_size, float nnratio,
                                   int32_t check_ori, int32_t* matches12, int32_t* nmatches);

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>&
 * sAlreadyFound, const float th, const int ORBdist) (ORB_SLAM2/src/ORBmatcher.cc:1475-1602;
 * Tracking::Relocalization, Tracking.cc:1441-1468) of an ORBmatcher(nnratio, checkOri).
 * frame = CurrentFrame with has_mp_obs[f] = mvpMapPoints[f] != NULL (here any map point blocks a
 * feature, observed or not; u_right unused).  kf_points: one entry per keyframe map point i,
 * valid[i] = pMP && !isBad() && !sAlreadyFound.count(pMP) && minDistance <= dist3D <=
 * maxDistance, u, v its projection into the current frame (the reference's cv::Mat pose
 * products), octave = PredictScale(dist3D, mfLogScaleFactor), angle = pKF->mvKeysUn[i].angle,
 * desc = GetDescriptor(); ur unused.  The window is the predicted level +-1, the first minimum
 * is kept when <= orb_dist, then the rotation filter.  match[f] = the keyframe index whose map
 * point is assigned to current feature f in this call, else -1. */
int orbx_search_by_projection_kf(const orbx_proj_frame* frame, const orbx_proj_last* kf_points,
                                 float th, int32_t orb_dist, int32_t check_ori, int32_t* match,
                                 int32_t* nmatches);
/* ORBmatcher::Fuse, the per-point search of both overloads:
 *   Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, const float th)
 *     (ORB_SLAM2/src/ORBmatcher.cc:828-978; LocalMapping::SearchInNeighbors, LocalMapping.cc:469,
 *     495) -> orbx_fuse;
 *   Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, float th,
 *        vector<MapPoint*>& vpReplacePoint) (:980-1103; LoopClosing::SearchAndFuse) ->
 *     orbx_fuse_sim3.
 * kf = the keyframe: keys_un, desc, u_right (mvuRight; NULL = every entry -1), its grid frame
 * (mnMinX.., mfGridElementWidthInv..) and mvScaleFactors.  Per point the caller evaluates the
 * reference's gates before the search with its own cv::Mat code and passes use[i] = !isBad() &&
 * not already in the keyframe && depth >= 0 && IsInImage(u, v) && minDistance <= dist3D <=
 * maxDistance && PO.dot(Pn) >= 0.5 * dist3D (:849-888, :1008-1046), u, v (and ur = u - bf * invz,
 * orbx_fuse only), pred_level = PredictScale(dist3D, mfLogScaleFactor) and the descriptor.
 * The library runs KeyFrame::GetFeaturesInArea(u, v, th * mvScaleFactors[pred_level]), the
 * level window, orbx_fuse's reprojection gates (inv_level_sigma2 = mvInvLevelSigma2) and the
 * Hamming first minimum: best_idx[i] = bestIdx if bestDist <= TH_LOW else -1, best_dist[i] =
 * bestDist (nullable).  *n_fused = points with best_idx >= 0.  The caller then applies the
 * reference's replace / AddObservation step in point order (:954-974, :1084-1099), re-checking
 * isBad() / IsInKeyFrame(pKF) at that point as the reference's loop does. */
typedef struct {
  int32_t n;
  const uint8_t* use;
  const float *u, *v, *ur;
  const int32_t* pred_level;
  const uint8_t* desc;         /* [n][32] */
} orbx_fuse_points;
int orbx_fuse(const orbx_proj_frame* kf, const float* inv_level_sigma2,
              const orbx_fuse_points* points, float th, int32_t* best_idx, int32_t* best_dist,
              int32_t* n_fused);
int orbx_fuse_sim3(const orbx_proj_frame* kf, const orbx_fuse_points* points, float th,
                   int32_t* best_idx, int32_t* best_dist, int32_t* n_fused);
/* ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints,
 * vector<MapPoint*>& vpMatched, int th) (ORB_SLAM2/src/ORBmatcher.cc:290-403;
 * LoopClosing::ComputeSim3 / CorrectLoop): kf = the keyframe (keys_un, desc, grid frame,
 * mvScaleFactors) with has_mp_obs[f] = vpMatched[f] != NULL on entry.  points: use[i] =
 * !isBad() && not in spAlreadyFound && depth >= 0 && IsInImage(u, v) && minDistance <= dist <=
 * maxDistance && PO.dot(Pn) >= 0.5 * dist (:318-352, evaluated by the caller with Scw), u, v,
 * pred_level = PredictScale(dist, mfLogScaleFactor), desc; ur unused.  match[f] = the point
 * index assigned to keyframe feature f in this call (vpMatched[f] = vpPoints[match[f]]), else
 * -1; *nmatches as the reference returns. */
int orbx_search_by_projection_sim3(const orbx_proj_frame* kf, const orbx_fuse_points* points,
                                   float th, int32_t* match, int32_t* nmatches);
/* ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12,
 * const float& s12, const cv::Mat& R12, const cv::Mat& t12, const float th)
 * (ORB_SLAM2/src/ORBmatcher.cc:1105-1329; LoopClosing::ComputeSim3, LoopClosing.cc:305):
 * kf1 / kf2 the two keyframes (keys_un, desc, grid frame, mvScaleFactors).  points12 = KF1's
 * map points projected into KF2 (n = kf1->n, one per keypoint i1: use[i1] = pMP &&
 * !vbAlreadyMatched1[i1] && !isBad() && depth >= 0 && pKF2->IsInImage(u, v) && minDistance <=
 * dist3D <= maxDistance, u, v, pred_level = PredictScale(dist3D, pKF2->mfLogScaleFactor),
 * desc), points21 = KF2's into KF1 (n = kf2->n, the same gates with vbAlreadyMatched2).
 * matches12[i1] = idx2 where the two directions agree (the caller sets vpMatches12[i1] =
 * vpMapPoints2[idx2]), else -1 (entry left as it was); *n_found as the reference returns. */
int orbx_search_by_sim3(const orbx_proj_frame* kf1, const orbx_proj_frame* kf2,
                        const orbx_fuse_points* points12, const orbx_fuse_points* points21,
                        float th, int32_t* matches12, int32_t* n_found);

/* ------------------------------------------------------------------ stereo
 * Frame::ComputeStereoMatches (ORB_SLAM2/src/Frame.cc:471-643) on the last extraction of a
 * left and a right extractor of the same image size and pyramid: for every left keypoint,
 * mvuRight / mvDepth (-1 when unmatched), host arrays of at least the left keypoint count,
 * which is returned in *n_out.  mb = baseline, mbf = baseline * fx (Frame::mb, Frame::mbf).
 * Where the reference's cv::Mat ranges would leave the pyramid level (it asserts), the
 * keypoint stays unmatched. */
int orbx_stereo_matches(orbx_extractor* left, orbx_extractor* right, float mb, float mbf,
                        float* uright, float* depth, int32_t* n_out);

/* ------------------------------------------------------------------ vocabulary
 * DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary, ORB_SLAM2/include/
 * ORBVocabulary.h), device resident.  Node ids follow DBoW2's file order (root 0, the n
 * nodes given are ids 1..n); word ids number the nodes flagged leaf in that order
 * (TemplatedVocabulary.h:1402-1416). */
typedef struct orbx_vocabulary orbx_vocabulary;
enum { ORBX_WEIGHT_TF_IDF = 0, ORBX_WEIGHT_TF = 1, ORBX_WEIGHT_IDF = 2, ORBX_WEIGHT_BINARY = 3 };
enum {
  ORBX_SCORE_L1 = 0, ORBX_SCORE_L2 = 1, ORBX_SCORE_CHI_SQUARE = 2, ORBX_SCORE_KL = 3,
  ORBX_SCORE_BHATTACHARYYA = 4, ORBX_SCORE_DOT_PRODUCT = 5
};
/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424): header
 * "k L scoring weighting", then one "parent isLeaf d0 .. d31 weight" line per node.  Blank
 * lines are skipped (the reference's trailing-newline phantom node is not created: its
 * descriptor is indeterminate).  ORBX_EINVAL on a header the reference rejects or a parent id
 * that is not an earlier node. */
int orbx_vocabulary_load_text(const char* path, int32_t hip_device, orbx_vocabulary** out);
/* The same tree from arrays (node i of the arrays is node id i+1). */
int orbx_vocabulary_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting,
                           int32_t n_nodes, const int32_t* parent, const uint8_t* is_leaf,
                           const uint8_t* desc, const double* weight, int32_t hip_device,
                           orbx_vocabulary** out);
int orbx_vocabulary_destroy(orbx_vocabulary* voc);
/* n_nodes counts the root. */
int orbx_vocabulary_info(const orbx_vocabulary* voc, int32_t* k, int32_t* L, int32_t* scoring,
                         int32_t* weighting, int32_t* n_nodes, int32_t* n_words);
/* TemplatedVocabulary::transform(features, BowVector& v, FeatureVector& fv, levelsup)
 * (TemplatedVocabulary.h:1127-1198) on n host descriptors.  Outputs (host, capacity n each):
 *   word_of[i], node_of[i]  word id / FeatureVector node id of feature i, 0xFFFFFFFF when the
 *                           word's weight is <= 0 (stopped; nullable outputs)
 *   bow_words/bow_values    BowVector in word-id order (values f64, weighted and normalised as
 *                           the vocabulary's scoring/weighting prescribe), *bow_n entries
 *   fv_node_ids/fv_offsets/fv_feats  FeatureVector in node-id order (CSR; offsets n+1),
 *                           *fv_n nodes.
 * When the descent reaches a leaf above level L - levelsup the FeatureVector node is that
 * leaf (the reference leaves it uninitialised). */
int orbx_vocabulary_transform(const orbx_vocabulary* voc, const uint8_t* desc, int32_t n,
                              int32_t levelsup, uint32_t* word_of, uint32_t* node_of,
                              uint32_t* bow_words, double* bow_values, int32_t* bow_n,
                              uint32_t* fv_node_ids, int32_t* fv_offsets, int32_t* fv_feats,
                              int32_t* fv_n);

/* ------------------------------------------------------------------ device frame pipeline
 * The whole per-frame unit of work of the benchmark on device-resident frames:
 * extract -> Frame::ComputeBoW (vocabulary transform: word ids, BowVector, FeatureVector) ->
 * SearchByBoW(prev-as-KF, cur) -> SearchForTriangulation(prev-as-KF, cur-as-KF).  Frame f of
 * a batch is matched against frame (f-1) mod n.  `voc` must outlive the pipeline and live on
 * the same device. */
typedef struct orbx_frames orbx_frames;
int orbx_frames_create(const orbx_params* params, int32_t w, int32_t h, int32_t max_batch,
                       const orbx_vocabulary* voc, int32_t levelsup, int hip_device,
                       orbx_frames** out);
/* Stereo pipeline (Frame's stereo constructor, ORB_SLAM2/src/Frame.cc:66-123): a frame is an
 * interleaved (left, right) image pair, d_imgs of orbx_frames_run holds 2n images; after the
 * extraction Frame::ComputeStereoMatches fills mvuRight / mvDepth, and ComputeBoW and the
 * matchers run on the left images (SearchForTriangulation with mvuRight). */
int orbx_frames_create_stereo(const orbx_params* params, int32_t w, int32_t h,
                              int32_t max_batch, const orbx_vocabulary* voc, int32_t levelsup,
                              float mb, float mbf, int hip_device, orbx_frames** out);
int orbx_frames_destroy(orbx_frames* fr);
int orbx_frames_capacity(const orbx_frames* fr, int32_t* kp_cap);
/* Host masks [max_batch][kp_cap]: valid = KF-side usable MapPoint for SearchByBoW, has_mp =
 * GetMapPoint(i) != NULL for SearchForTriangulation.  Either may be NULL (left unchanged). */
int orbx_frames_set_masks(orbx_frames* fr, const uint8_t* valid, const uint8_t* has_mp);
int orbx_frames_set_matching(orbx_frames* fr, float bow_ratio, int32_t bow_check_ori,
                             const float F12[9], float ex, float ey, float tri_ratio,
                             int32_t tri_check_ori, int32_t only_stereo);
/* Enqueue one batch (d_imgs: n dense w*h device images); asynchronous. */
int orbx_frames_run(orbx_frames* fr, const uint8_t* d_imgs, int32_t n);
int orbx_frames_sync(orbx_frames* fr);
/* Host copies of the per-frame counts of the last run (synchronises). */
int orbx_frames_results(orbx_frames* fr, int32_t n, int32_t* kp_counts, int32_t* bow_matches,
                        int32_t* tri_matches, int32_t* error);
/* Device pointers: kps/desc [images][kp_cap], counts [images] (images = 2 x frames for
 * stereo, left image of frame f at 2f), FeatureVector node id
 * per feature [max_batch][kp_cap] (0xFFFFFFFF = stopped word), bow match [max_batch][kp_cap]
 * (frame-indexed, value = KF index), triangulation pairs [max_batch][kp_cap][2]. */
int orbx_frames_outputs(orbx_frames* fr, orbx_keypoint** d_kps, uint8_t** d_desc,
                        int32_t** d_counts, uint32_t** d_node_of, int32_t** d_bow_match,
                        int32_t** d_tri_pairs);
/* Device pointers of the BowVectors: word ids / values [max_batch][kp_cap], entries per frame
 * [max_batch]; word id per feature [max_batch][kp_cap] (0xFFFFFFFF = stopped). */
/* Stereo pipelines: mvuRight / mvDepth per left keypoint, [max_batch][kp_cap] device. */
int orbx_frames_stereo(orbx_frames* fr, float** d_uright, float** d_depth);
int orbx_frames_bow(orbx_frames* fr, uint32_t** d_bow_words, double** d_bow_values,
                    int32_t** d_bow_n, uint32_t** d_word_of);
void* orbx_frames_stream(orbx_frames* fr);
int orbx_frames_profile(orbx_frames* fr, int32_t enable);
int orbx_frames_profile_read(orbx_frames* fr, int32_t cap, char (*names)[32], double* total_ms,
                             int64_t* launches, int32_t* n_stages);
int orbx_frames_profile_kernels(orbx_frames* fr, int32_t stage, char* buf, int32_t cap);

/* ------------------------------------------------------------------ matcher */
/* ORBmatcher::DescriptorDistance on n row pairs (host pointers). */
int orbx_descriptor_distance(const uint8_t* a, const uint8_t* b, int32_t n, int32_t* out);

/* SearchByBoW(KeyFrame*, Frame&): match[f] = KF feature index matched to frame feature f,
 * or -1 (vpMapPointMatches[f] = KF MapPoint of that index).  Returns count in *nmatches. */
int orbx_search_by_bow_kf_f(const orbx_bow_side* kf, const orbx_bow_side* f, float nnratio,
                            int32_t check_ori, int32_t* match, int32_t* nmatches);

/* SearchByBoW(KeyFrame*, KeyFrame*): match12[i1] = KF2 index or -1. */
int orbx_search_by_bow_kf_kf(const orbx_bow_side* kf1, const orbx_bow_side* kf2, float nnratio,
                             int32_t check_ori, int32_t* match12, int32_t* nmatches);

/* SearchForTriangulation: pairs (idx1, idx2) ascending in idx1, up to kf1->n pairs.
 * F12 row-major 3x3 f32 (cv::Mat F12.at<float>(r,c) = F12[3r+c]); (ex, ey) the epipole of
 * KF1's centre in KF2 (ORBmatcher.cc:667-673; orbx_epipole computes it). */
int orbx_search_for_triangulation(const orbx_tri_side* kf1, const orbx_tri_side* kf2,
                                  const float F12[9], float ex, float ey, int32_t only_stereo,
                                  float nnratio, int32_t check_ori, int32_t* pairs,
                                  int32_t* nmatches);

/* Epipole exactly as ORBmatcher.cc:667-673 evaluates it (C2 = R2w*Cw + t2w, f32). */
int orbx_epipole(const float R2w[9], const float t2w[3], const float Cw[3], float fx, float fy,
                 float cx, float cy, float* ex, float* ey);

/* ------------------------------------------------------------------ AR marker path (cv::ORB) */
/* cv::ORB constructor arguments (OpenCV 2.4 features2d.hpp): ORB(int nfeatures = 500,
 * float scaleFactor = 1.2f, int nlevels = 8, int edgeThreshold = 31, int firstLevel = 0,
 * int WTA_K = 2, int scoreType = ORB::HARRIS_SCORE, int patchSize = 31).  Marker uses the
 * defaults (Marker.cc:83, 107); AR-1.3's ORBMatcher uses (300, 1.2f, 8, 31, 0, 2, HARRIS, 31)
 * (AR-1.3/src/ORBMatcher.cpp:121-122).  Implemented: firstLevel 0, WTA_K 2, patchSize 31,
 * edgeThreshold >= 18 (the 37 x 37 descriptor window stays inside the level); anything else
 * returns ORBX_EUNSUPPORTED. */
#define ORBX_HARRIS_SCORE 0
#define ORBX_FAST_SCORE 1
typedef struct {
  int32_t nfeatures;
  float scale_factor;
  int32_t nlevels;
  int32_t edge_threshold;
  int32_t first_level;
  int32_t wta_k;
  int32_t score_type;
  int32_t patch_size;
} orbx_cvorb_params;

/* == cv::DMatch (OpenCV 2.4): {queryIdx, trainIdx, imgIdx, distance}, 16 B. */
typedef struct {
  int32_t query_idx, train_idx, img_idx;
  float distance;
} orbx_dmatch;

/* One cv::ORB instance with a batch plan for one image size.  orbx_cvorb_detect is the
 * drop-in for `orb(image, Mat(), keypoints, descriptors)` on a host image (the plan is rebuilt
 * when the size changes); keypoints are level-major in the reference's order (the order
 * KeyPointsFilter::retainBest leaves them in, libstdc++ nth_element/partition), descriptors
 * n x 32.  An empty image returns *n_out = -1 with the outputs untouched (orb.cpp returns
 * early); n == 0 means no keypoints (descriptors released). */
typedef struct orbx_cvorb orbx_cvorb;
int orbx_cvorb_create(const orbx_cvorb_params* params, int32_t w, int32_t h, int32_t max_batch,
                      int hip_device, orbx_cvorb** out);
int orbx_cvorb_destroy(orbx_cvorb* orb);
int orbx_cvorb_capacity(const orbx_cvorb* orb, int32_t* kp_cap);
int orbx_cvorb_detect(orbx_cvorb* orb, const uint8_t* img, int32_t w, int32_t h, int64_t stride,
                      orbx_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out);
/* Throughput path: n dense h*w u8 images already in device memory, asynchronous on the
 * instance's stream.  Outputs [max_batch][kp_cap] keypoints / descriptors, counts [max_batch]
 * (a negative count = that image overflowed the per-level keypoint capacity). */
int orbx_cvorb_run(orbx_cvorb* orb, const uint8_t* d_imgs, int32_t n);
int orbx_cvorb_outputs(orbx_cvorb* orb, orbx_keypoint** d_kps, uint8_t** d_desc,
                       int32_t** d_counts);
int orbx_cvorb_sync(orbx_cvorb* orb);
void* orbx_cvorb_stream(orbx_cvorb* orb);

/* BruteForceMatcher<HammingLUT>::match(query, train, matches): for every query row the first
 * train row of minimum Hamming distance (BFMatcher NORM_HAMMING, k = 1).  out[nq]; *n_out = nq,
 * or 0 when either side is empty (DescriptorMatcher::knnMatch returns early). */
int orbx_bf_match(const uint8_t* query, int32_t nq, const uint8_t* train, int32_t nt,
                  orbx_dmatch* out, int32_t* n_out);
/* Marker::Match's filter: max_dist over the matches (initial 0), keep distance < 0.5*max_dist
 * (double), in order.  Host-side, no device work (n <= a few thousand). */
int orbx_good_matches(const orbx_dmatch* matches, int32_t n, orbx_dmatch* good, int32_t* n_good,
                      double* min_dist, double* max_dist);
/* naive_nn_search2 / Marker::searchMatches: for every query row (keys2) the nearest and second
 * nearest train row (keys1), strict `<` updates; accept when min <= (unsigned)(second * ratio)
 * and min <= max_dist.  ratio <= 0 selects naive_nn_search (no ratio test).  *min_d / *max_d
 * return the extremes over all evaluated pairs (the reference's global minD/maxD; the caller
 * merges them into its running values). */
int orbx_nn_match(const uint8_t* query, int32_t nq, const uint8_t* train, int32_t nt,
                  double ratio, int32_t max_dist, orbx_dmatch* out, int32_t* n_out,
                  int32_t* min_d, int32_t* max_d);

/* Marker::Match for a batch of frames against one target: cv::ORB extraction of every frame,
 * BruteForceMatcher match (query = target descriptors, train = frame descriptors) and the
 * good-match filter, all on the device stream.  Per frame: matches [max_batch][n_target]
 * (train_idx = -1 if the frame has no keypoints), good flags [max_batch][n_target], counts. */
typedef struct orbx_marker orbx_marker;
int orbx_marker_create(const orbx_cvorb_params* params, int32_t w, int32_t h, int32_t max_batch,
                       int hip_device, orbx_marker** out);
int orbx_marker_destroy(orbx_marker* mk);
int orbx_marker_set_target(orbx_marker* mk, const uint8_t* desc, int32_t n);
int orbx_marker_run(orbx_marker* mk, const uint8_t* d_imgs, int32_t n);
int orbx_marker_sync(orbx_marker* mk);
int orbx_marker_results(orbx_marker* mk, int32_t n, int32_t* kp_counts, int32_t* good_counts);
int orbx_marker_outputs(orbx_marker* mk, orbx_dmatch** d_matches, uint8_t** d_good,
                        orbx_keypoint** d_kps, uint8_t** d_desc);
void* orbx_marker_stream(orbx_marker* mk);
int orbx_marker_profile(orbx_marker* mk, int32_t enable);
int orbx_marker_profile_read(orbx_marker* mk, int32_t cap, char (*names)[32], double* total_ms,
                             int64_t* launches, int32_t* n_stages);
int orbx_marker_profile_kernels(orbx_marker* mk, int32_t stage, char* buf, int32_t cap);

/* ------------------------------------------------------------------ test hooks (not product API) */
/* The device computeOrbDescriptor rotation (float)cos/sin((double)(deg * (float)(CV_PI/180.f)))
 * for n host angles; and KeyPointsFilter::retainBest (orb.cpp's nth_element + partition) run by
 * the k_cvselect wave routine on one host array (in LDS when n <= 2560 unless force_global),
 * resp/ids rewritten in the retained order.  Used by tests/test_cvorb_gpu.py. */
int orbx_debug_cvorb_cossin(const float* deg, int64_t n, float* c, float* s);
int orbx_debug_retain_best(float* resp, uint32_t* ids, int32_t n, int32_t n_points,
                           int32_t force_global, int32_t* n_out);
/* The finish step of SearchByBoW (kind 0 KF->Frame: match[n2] with values < n1; kind 1 KF->KF:
 * match[n1], values < n2) or SearchForTriangulation (kind 2: m12[n1], values < n2) over a
 * caller-given match array, orientation check off.  Out-of-range values (a stale match array)
 * are dropped to -1 in out[] and reported as ORBX_EDEVICE; *nmatches counts the kept ones.
 * Used by tests/test_match_gpu.py. */
int orbx_debug_match_finish(int32_t kind, int32_t n1, int32_t n2, const int32_t* match,
                            int32_t* out, int32_t* nmatches);
/* The SearchByBoW node kernel every later call launches, process-wide: 0 chosen per call (the
 * default: calls of at most 4 problems a workgroup per node, batches a wave per node), 1 a
 * workgroup per node, 2 / 3 a wave per node with 4 / 2 register chunks.  Used by
 * tests/test_match_gpu.py to run each form on the same inputs. */
int orbx_debug_bow_kernel(int32_t form);
/* The device glibc sincosf port of computeOrbDescriptor (ORBextractor.cc:103-104, orbx_math.h)
 * for the n floats whose bit patterns are lo, lo+1, ...; s / c host arrays of n.  Used by
 * tests/test_math_gpu.py (every float in [0, 2*pi] against the host libm). */
int orbx_debug_sincosf(uint32_t lo, int64_t n, float* s, float* c);
/* The GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101) image of pyramid level `level` of the last
 * orbx_extract call (ORBextractor.cc:1024-1026, computeDescriptors' working image), w x h of
 * orbx_extractor_pyramid, into out with row stride `stride`.  Used by tests/test_extract_gpu.py. */
int orbx_debug_extractor_blur(orbx_extractor* ex, int32_t level, uint8_t* out, int64_t stride);
/* Level `level` of image `img` of the batch the last orbx_plan_extract call ran: the pyramid level
 * (blurred = 0, ORBextractor.cc:1047-1072) or its GaussianBlur(7x7, 2, 2, BORDER_REFLECT_101) image
 * (blurred = 1, :1024-1026), into out with row stride `stride`.  Used by tests/test_extract_gpu.py
 * (batch plans' row bands: the blur fused into k_pyramid, or k_blur for frames too wide). */
int orbx_debug_plan_level(orbx_plan* plan, int32_t img, int32_t level, int32_t blurred, uint8_t* out,
                          int64_t stride);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_H */
