/*
 * orb_oracle.h — CPU restatement of the reference ORB front end.  TEST INFRASTRUCTURE ONLY:
 * imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * Never linked into, called by, or used as a fallback for the product library.
 *
 * Parity status: the ORB-SLAM2 logic is restated from ORB_SLAM2/src/ORBextractor.cc and
 * ORB_SLAM2/src/ORBmatcher.cc (cited per function in orb_oracle.cc); the OpenCV 2.4
 * primitives it calls (FAST, resize INTER_LINEAR, GaussianBlur, fastAtan2, cvRound) are
 * restated from their published 2.4 algorithm.  The reference needs
 * OpenCV 2.4, which is absent, so it cannot be built here: the oracle is pinned
 * by known-answer tests derived from the reference's own tables (umax, per-level feature
 * counts, pattern checksum, scale tables) and an exhaustive sincosf check against the host
 * glibc; bit parity against real OpenCV 2.4 primitives is UNPINNED.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include "../include/orbx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* tie_mode for DistributeOctTree's final sort:
 *   0 = canonical (size, creation sequence) — the contract shared with the GPU path;
 *   1 = faithful (size, heap address) — the reference's own, non-deterministic order. */
int oracle_extract(const orbx_params* p, const uint8_t* img, int w, int h, int64_t stride,
                   int tie_mode, orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out);

/* Same as oracle_extract but also returns the per-level pyramid (levels packed densely,
 * level l of size lw[l] x lh[l]) when pyr != NULL, and the pre-octree candidate counts. */
int oracle_extract_ex(const orbx_params* p, const uint8_t* img, int w, int h, int64_t stride,
                      int tie_mode, orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out,
                      uint8_t* pyr, int64_t pyr_cap, int* lw, int* lh, int* n_candidates);

int oracle_tables(const orbx_params* p, float* scale, float* inv_scale, float* sigma2,
                  float* inv_sigma2, int* feats_per_level, int* umax16, int* level_w,
                  int* level_h, int w, int h);

/* primitives (known-answer tests) */
void oracle_resize_linear(const uint8_t* src, int sw, int sh, int64_t sstride, uint8_t* dst,
                          int dw, int dh, int64_t dstride);
void oracle_gaussian7(const uint8_t* src, int w, int h, uint8_t* dst);
float oracle_fast_atan2(float y, float x);
int oracle_fast_score(const uint8_t* center, int64_t stride); /* max(q0,-q1)-1 */
/* FAST on one ROI (rows x cols, stride) at threshold t with NMS: xs, ys, scores in raster
 * order; returns the count (<= cap). */
int oracle_fast_roi(const uint8_t* roi, int rows, int cols, int64_t stride, int t, int* xs,
                    int* ys, int* scores, int cap);
float oracle_ic_angle(const uint8_t* img, int64_t stride, int cx, int cy);
void oracle_orb_descriptor(const uint8_t* blurred, int64_t stride, int cx, int cy, float angle,
                           uint8_t* desc32);
void oracle_sincosf(float x, float* s, float* c);
void oracle_sincosf_bits(uint32_t lo, int64_t n, float* s, float* c, int threads);

/* matcher (ORBmatcher.cc) */
int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b);
int oracle_search_by_bow_kf_f(const orbx_bow_side* kf, const orbx_bow_side* f, float nnratio,
                              int check_ori, int32_t* match);
int oracle_search_by_bow_kf_kf(const orbx_bow_side* kf1, const orbx_bow_side* kf2,
                               float nnratio, int check_ori, int32_t* match12);
int oracle_search_for_triangulation(const orbx_tri_side* kf1, const orbx_tri_side* kf2,
                                    const float F12[9], float ex, float ey, int only_stereo,
                                    float nnratio, int check_ori, int32_t* pairs);
void oracle_epipole(const float R2w[9], const float t2w[3], const float Cw[3], float fx,
                    float fy, float cx, float cy, float* ex, float* ey);
/* DBoW2 transform restricted to node ids (TemplatedVocabulary.h:1218-1259), complete
 * k-ary breadth-first layout as in orbx.h. */
void oracle_feature_vector(const uint8_t* voc_desc, int k, int L, int levelsup,
                           const uint8_t* desc, int n, uint32_t* node_of_feature);

/* DBoW2 vocabulary (dbow2_oracle.cc): opaque handle, nodes 1..n_nodes in file order */
void* oracle_voc_create(int k, int L, int scoring, int weighting, int n_nodes,
                        const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc,
                        const double* weight);
void* oracle_voc_load_text(const char* path);
void oracle_voc_destroy(void* h);
void oracle_voc_info(const void* h, int* k, int* L, int* scoring, int* weighting, int* n_nodes,
                     int* n_words);
void oracle_voc_transform(const void* h, const uint8_t* desc, int n, int levelsup,
                          uint32_t* word_of, uint32_t* node_of, uint32_t* bow_words,
                          double* bow_values, int* bow_n, uint32_t* fv_ids, int32_t* fv_off,
                          int32_t* fv_feats, int* fv_n);

/* Frame::ComputeStereoMatches (stereo_oracle.cc): per-level pyramid pointers + strides */
void oracle_stereo_matches(const orbx_keypoint* kl, int nl, const uint8_t* dl,
                           const orbx_keypoint* kr, int nr, const uint8_t* dr,
                           const uint8_t* const* pyrL, const uint8_t* const* pyrR,
                           const int* lw, const int* lh, const int64_t* lstride,
                           const float* scale, const float* inv_scale, float mb, float mbf,
                           float* uright, float* depth, int* sad);

/* tracking searches (projection_oracle.cc) */
int oracle_features_in_area(const orbx_proj_frame* F, float x, float y, float r, int minLevel,
                            int maxLevel, int32_t* out, int cap);
int oracle_search_by_projection(const orbx_proj_frame* F, const orbx_proj_points* M, float th,
                                float nnratio, int32_t* match);
int oracle_search_by_projection_last(const orbx_proj_frame* F, const orbx_proj_last* P, float th,
                                     int forward, int backward, int check_ori, int32_t* match);
int oracle_search_for_initialization(const orbx_proj_frame* F1, const orbx_proj_frame* F2,
                                     float* prev, float nnratio, int check_ori, int window,
                                     int32_t* m12);
int oracle_search_by_projection_kf(const orbx_proj_frame* F, const orbx_proj_last* P, float th,
                                   int ORBdist, int check_ori, int32_t* match);
int oracle_search_by_projection_sim3(const orbx_proj_frame* KF, const orbx_fuse_points* M,
                                     float th, int32_t* match);
int oracle_search_by_sim3(const orbx_proj_frame* KF1, const orbx_proj_frame* KF2,
                          const orbx_fuse_points* M12, const orbx_fuse_points* M21, float th,
                          int32_t* m12);
int oracle_fuse(const orbx_proj_frame* KF, const float* inv_sigma2, const orbx_fuse_points* M,
                float th, int reproj, int32_t* best_idx, int32_t* best_dist);

/* AR marker path (cvorb_oracle.cc): cv::ORB 2.4 + BruteForceMatcher<HammingLUT> + the
 * Marker / AR-1.3 nearest-neighbour matchers */
int oracle_cvorb_levels(const orbx_cvorb_params* p, int w, int h, int* lw, int* lh, float* scale,
                        int* feats);
void oracle_retain_best(float* resp, int32_t* ids, int n, int n_points, int* n_out);
void oracle_cos_sin_f64_range(uint32_t bits0, int64_t n, float* c, float* s, int threads);
float oracle_harris(const uint8_t* img, int64_t stride, int x, int y);
void oracle_cvorb_descriptor(const uint8_t* blurred, int64_t stride, int cx, int cy, float angle,
                             uint8_t* desc32);
void oracle_cos_sin_f64(float deg, float* c, float* s);
int oracle_cvorb_detect(const orbx_cvorb_params* p, const uint8_t* img, int w, int h,
                        int64_t stride, orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out,
                        uint8_t* pyr, int64_t pyr_cap);
int oracle_bf_match(const uint8_t* query, int nq, const uint8_t* train, int nt, orbx_dmatch* out,
                    int* n_out);
int oracle_good_matches(const orbx_dmatch* m, int n, orbx_dmatch* good, int* n_good,
                        double* min_dist, double* max_dist);
int oracle_nn_match(const uint8_t* query, int nq, const uint8_t* train, int nt, double ratio,
                    int max_dist, orbx_dmatch* out, int* n_out, int* min_d, int* max_d);

#ifdef __cplusplus
}
#endif
#endif
