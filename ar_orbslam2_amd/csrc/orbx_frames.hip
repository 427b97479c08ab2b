// orbx_frames.hip — device-resident frame pipeline: the whole "ORB extract + match" unit of
// work of SURVEY §8d for a batch of frames, with no host round trip:
//   extract (plan)  ->  Frame::ComputeBoW: vocabulary descent (k_voc_transform), BowVector
//   (k_bowvec), FeatureVector CSR (k_csr)
//   -> SearchByBoW(prev-as-KF, cur)  ->  SearchForTriangulation(prev-as-KF, cur-as-KF)
// Stereo pipelines take frames as interleaved (left, right) image pairs, run
// Frame::ComputeStereoMatches (orbx_stereo.hip) after the extraction, and feed ComputeBoW and
// the matchers with the left images and their mvuRight (Frame.cc:78-96).
// Frame f of a batch is matched against frame (f-1) mod n of the same batch.  The sequence is
// captured once into a hipGraph per (input pointer, batch size).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "orbx_internal.h"
#include "orbx_match.h"
#include "orbx_vocab.h"
#include "orbx_stereo.h"

using namespace orbx;

struct orbx_frames {
  orbx_plan* plan = nullptr;
  PlanView v{};
  int device = 0;
  // vocabulary
  const orbx_vocabulary* voc = nullptr;
  VocView vv{};
  const VocRanks* ranks = nullptr;
  int scoring = 0, weighting = 0, levelsup = 4, nid_level = 2;
  int nb = 1;
  int max_frames = 0;
  int bow_err_slot() const { return max_frames; }
  // stereo
  int stereo = 0;
  float mb = 0, mbf = 0;
  int st_nrows = 0;
  int64_t st_row_cap = 0;
  int* d_lcounts = nullptr;  // [B] left keypoint counts (stereo)
  float* d_uright = nullptr;  // [B][kp] mvuRight
  float* d_depth = nullptr;   // [B][kp] mvDepth
  int* d_sad = nullptr;       // [B][kp]
  int* d_row_off = nullptr;   // [B][nrows + 1]
  uint2* d_row_idx = nullptr;  // [B][row_cap] row entries
  StereoProblem* d_sprob = nullptr;
  // per frame
  uint32_t* d_node_of = nullptr;  // [B][kp] FeatureVector node id
  uint32_t* d_rank_of = nullptr;  // [B][kp] FeatureVector rank (k_csr bucket)
  uint32_t* d_word_of = nullptr;  // [B][kp]
  double* d_wt_of = nullptr;      // [B][kp]
  uint32_t* d_bow_words = nullptr;  // [B][kp]
  double* d_bow_vals = nullptr;     // [B][kp]
  int* d_bow_n = nullptr;           // [B]
  uint32_t* d_ids = nullptr;      // [B][nb]
  int* d_off = nullptr;           // [B][nb+1]
  int* d_feats = nullptr;         // [B][kp]
  int* d_nn = nullptr;            // [B]
  uint8_t* d_valid = nullptr;     // [B][kp]
  uint8_t* d_hasmp = nullptr;     // [B][kp]
  float *d_sf = nullptr, *d_s2 = nullptr;
  int* d_match = nullptr;      // [B][kp]
  int* d_bow_count = nullptr;  // [B] + error word
  int* d_m12 = nullptr;        // [B][kp]
  int* d_pairs = nullptr;      // [B][kp][2]
  int* d_tri_count = nullptr;  // [B]
  BowProblem* d_bprob = nullptr;
  TriProblem* d_tprob = nullptr;
  int prob_n = -1;
  // matching parameters
  float bow_ratio = 0.7f, tri_ratio = 0.6f;
  int bow_ori = 1, tri_ori = 0, only_stereo = 0;
  float F[9] = {0};
  float ex = 0, ey = 0;
  // graph cache, one executable graph per (input pointer, batch size)
  GraphCache graphs;
  Profiler prof;
  void drop_graphs() { graphs.clear(v.stream); }
};

namespace {

template <class T>
int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) return ORBX_ENOMEM;
  return ORBX_OK;
}

// image index of frame f's (left) image, and the per-frame count array
inline int limg(const orbx_frames* F, int f) { return F->stereo ? 2 * f : f; }
inline int* fcounts(const orbx_frames* F) { return F->stereo ? F->d_lcounts : F->v.d_counts; }

int build_problems(orbx_frames* F, int n) {
  const int kp = F->v.kp_total;
  std::vector<BowProblem> bp(n);
  std::vector<TriProblem> tp(n);
  for (int f = 0; f < n; f++) {
    const int kf = (f - 1 + n) % n;
    auto side = [&](int fr, bool with_valid) {
      DevSide s{};
      s.n = 0;
      s.n_dev = fcounts(F) + fr;
      s.desc = F->v.d_desc + (int64_t)limg(F, fr) * kp * 32;
      s.angle = (const float*)((const char*)(F->v.d_kps + (int64_t)limg(F, fr) * kp) +
                               offsetof(orbx_keypoint, angle));
      s.angle_stride = sizeof(orbx_keypoint) / sizeof(float);
      s.valid = with_valid ? F->d_valid + (int64_t)fr * kp : nullptr;
      s.n_nodes = 0;
      s.n_nodes_dev = F->d_nn + fr;
      s.node_ids = F->d_ids + (int64_t)fr * F->nb;
      s.node_offsets = F->d_off + (int64_t)fr * (F->nb + 1);
      s.node_feats = F->d_feats + (int64_t)fr * kp;
      return s;
    };
    BowProblem& B = bp[f];
    B.s1 = side(kf, true);
    B.s2 = side(f, false);
    B.match = F->d_match + (int64_t)f * kp;
    B.count = F->d_bow_count + f;
    B.error = F->d_bow_count + F->bow_err_slot();
    B.matched2 = nullptr;  // mode 0 reads the match array itself
    B.mode = 0;
    B.nnratio = F->bow_ratio;
    B.check_ori = F->bow_ori;
    auto tside = [&](int fr) {
      DevTriSide s{};
      s.n_dev = fcounts(F) + fr;
      s.desc = F->v.d_desc + (int64_t)limg(F, fr) * kp * 32;
      s.keys_un = F->v.d_kps + (int64_t)limg(F, fr) * kp;
      s.u_right = F->stereo ? F->d_uright + (int64_t)fr * kp : nullptr;
      s.has_mp = F->d_hasmp + (int64_t)fr * kp;
      s.fv.n_nodes_dev = F->d_nn + fr;
      s.fv.node_ids = F->d_ids + (int64_t)fr * F->nb;
      s.fv.node_offsets = F->d_off + (int64_t)fr * (F->nb + 1);
      s.fv.node_feats = F->d_feats + (int64_t)fr * kp;
      s.scale_factors = F->d_sf;
      s.level_sigma2 = F->d_s2;
      return s;
    };
    TriProblem& T = tp[f];
    T.s1 = tside(kf);
    T.s2 = tside(f);
    memcpy(T.F, F->F, sizeof(T.F));
    T.ex = F->ex;
    T.ey = F->ey;
    T.only_stereo = F->only_stereo;
    T.check_ori = F->tri_ori;
    T.m12 = F->d_m12 + (int64_t)f * kp;
    T.pairs = F->d_pairs + (int64_t)f * kp * 2;
    T.count = F->d_tri_count + f;
    T.error = F->d_bow_count + F->bow_err_slot();
  }
  if (F->stereo) {
    std::vector<StereoProblem> sp(n);
    for (int f = 0; f < n; f++) {
      StereoProblem& S = sp[f];
      S.kl = F->v.d_kps + (int64_t)(2 * f) * kp;
      S.dl = F->v.d_desc + (int64_t)(2 * f) * kp * 32;
      S.nl = F->v.d_counts + 2 * f;
      S.kr = F->v.d_kps + (int64_t)(2 * f + 1) * kp;
      S.dr = F->v.d_desc + (int64_t)(2 * f + 1) * kp * 32;
      S.nr = F->v.d_counts + 2 * f + 1;
      S.pyrL = F->v.d_pyr + (int64_t)(2 * f) * F->v.pyr_bytes;
      S.pyrR = F->v.d_pyr + (int64_t)(2 * f + 1) * F->v.pyr_bytes;
      S.uright = F->d_uright + (int64_t)f * kp;
      S.depth = F->d_depth + (int64_t)f * kp;
      S.sad = F->d_sad + (int64_t)f * kp;
      S.row_off = F->d_row_off + (int64_t)f * (F->st_nrows + 1);
      S.row_ent = F->d_row_idx + (int64_t)f * F->st_row_cap;
    }
    ORBX_HIP(hipMemcpy(F->d_sprob, sp.data(), sizeof(StereoProblem) * n, hipMemcpyHostToDevice));
  }
  ORBX_HIP(hipMemcpy(F->d_bprob, bp.data(), sizeof(BowProblem) * n, hipMemcpyHostToDevice));
  ORBX_HIP(hipMemcpy(F->d_tprob, tp.data(), sizeof(TriProblem) * n, hipMemcpyHostToDevice));
  F->prob_n = n;
  return ORBX_OK;
}

int enqueue(orbx_frames* F, const uint8_t* d_in, int n, Profiler* prof) {
  Profiler dummy;
  Profiler& pr = prof ? *prof : dummy;
  const int st_fv = pr.stage("k_voc_transform"), st_bv = pr.stage("k_bowvec"),
            st_csr = pr.stage("k_csr"),
            st_bow = pr.stage("k_bow"), st_tri = pr.stage("k_tri");
  ProfScope scope(pr);
  hipStream_t s = F->v.stream;
  int rc = plan_enqueue(F->plan, d_in, F->stereo ? 2 * n : n, prof);
  if (rc) return rc;
  const int kp = F->v.kp_total;
  const int ist = F->stereo ? 2 : 1;  // image step of the frames' (left) images
  if (F->stereo) {
    const int st_st = pr.stage("k_stereo");
    // left counts of the interleaved (left, right) images, contiguous per frame
    ORBX_HIP(hipMemcpy2DAsync(F->d_lcounts, 4, F->v.d_counts, 8, 4, n, hipMemcpyDeviceToDevice, s));
    rc = launch_stereo(F->d_sprob, n, F->v.d_lv, F->v.g->nlevels, F->st_nrows, F->st_row_cap, kp,
                       F->mb, F->mbf, s);
    if (rc) return rc;
    pr.mark(s, st_st);
  }
  rc = launch_voc_transform(F->vv, F->nid_level, F->ranks->d_rank_of_node, F->v.d_desc,
                            (int64_t)kp * 32 * ist, fcounts(F), 0, kp, F->d_word_of, F->d_rank_of,
                            F->d_node_of, F->d_wt_of, kp, n, s);
  if (rc) return rc;
  pr.mark(s, st_fv);
  // BowVector + FeatureVector in one launch (k_bowfv, stage "k_bowvec"), else the two kernels
  rc = launch_bowfv(F->scoring, F->weighting, F->vv.n_words, F->d_word_of, F->d_rank_of,
                    F->d_wt_of, kp, fcounts(F), 0, kp, F->d_bow_words, F->d_bow_vals, kp,
                    F->d_bow_n, F->nb, F->ranks->d_rank_ids, F->d_ids, F->d_off, F->d_feats, kp,
                    F->d_nn, n, s);
  if (rc == ORBX_EUNSUPPORTED) {
    rc = launch_bowvec(F->scoring, F->weighting, F->d_word_of, F->d_wt_of, kp, fcounts(F), 0, kp,
                       F->d_bow_words, F->d_bow_vals, kp, F->d_bow_n, n, s);
    if (rc) return rc;
    pr.mark(s, st_bv);
    rc = launch_csr(F->d_rank_of, kp, fcounts(F), 0, 0, F->nb, F->ranks->d_rank_ids, F->d_ids,
                    F->d_off, F->d_feats, kp, F->d_nn, n, s);
  } else if (rc == ORBX_OK) {
    pr.mark(s, st_bv);
  }
  if (rc) return rc;
  pr.mark(s, st_csr);
  launch_fill_u32((uint32_t*)F->d_match, (size_t)n * kp, 0xFFFFFFFFu, s);
  rc = launch_bow(F->d_bprob, n, F->nb, s, false, kp / std::max(F->nb, 1));
  if (rc) return rc;
  pr.mark(s, st_bow);
  launch_fill_u32((uint32_t*)F->d_m12, (size_t)n * kp, 0xFFFFFFFFu, s);
  rc = launch_tri(F->d_tprob, n, F->nb, s);
  if (rc) return rc;
  pr.mark(s, st_tri);
  return ORBX_OK;
}

}  // namespace

extern "C" {

static int frames_create(const orbx_params* p, int32_t w, int32_t h, int32_t max_batch,
                         const orbx_vocabulary* voc, int32_t levelsup, int stereo, float mb,
                         float mbf, int hip_device, orbx_frames** out) {
  ORBX_RESOURCE_LOCK;
  if (!p || !out || !voc || levelsup < 0 || max_batch < 1) return ORBX_EINVAL;
  *out = nullptr;
  int voc_dev = 0;
  VocView vv;
  int rc = vocab_view(voc, &vv, &voc_dev);
  if (rc) return rc;
  if (voc_dev != hip_device) return ORBX_EINVAL;
  const VocRanks* R = nullptr;
  rc = vocab_ranks(voc, levelsup, &R);
  if (rc) return rc;
  if (R->nb > 8192) return ORBX_EUNSUPPORTED;  // FeatureVector buckets live in LDS
  orbx_frames* F = new (std::nothrow) orbx_frames();
  if (!F) return ORBX_ENOMEM;
  auto fail = [&](int rc) {
    orbx_frames_destroy(F);
    return rc;
  };
  F->device = hip_device;
  F->prof.on = getenv("ORBX_SYNC_STAGES") != nullptr;  // debugging: eager, stage-synchronous
  F->stereo = stereo;
  F->max_frames = max_batch;
  F->mb = mb;
  F->mbf = mbf;
  rc = orbx_plan_create(p, w, h, stereo ? 2 * max_batch : max_batch, hip_device, &F->plan);
  if (rc) return fail(rc);
  plan_view(F->plan, &F->v);
  if (F->v.kp_total > 8192) return fail(ORBX_EUNSUPPORTED);  // k_bowvec sorts in LDS
  int32_t L = 0;
  orbx_vocabulary_info(voc, nullptr, &L, &F->scoring, &F->weighting, nullptr, nullptr);
  F->voc = voc;
  F->vv = vv;
  F->ranks = R;
  F->levelsup = levelsup;
  F->nid_level = L - levelsup;
  F->nb = std::max(R->nb, 1);
  const size_t B = max_batch, kp = F->v.kp_total;
  if (dalloc(&F->d_node_of, B * kp) || dalloc(&F->d_rank_of, B * kp) ||
      dalloc(&F->d_word_of, B * kp) ||
      dalloc(&F->d_wt_of, B * kp) || dalloc(&F->d_bow_words, B * kp) ||
      dalloc(&F->d_bow_vals, B * kp) || dalloc(&F->d_bow_n, B) ||
      dalloc(&F->d_ids, B * F->nb) || dalloc(&F->d_off, B * (F->nb + 1)) ||
      dalloc(&F->d_feats, B * kp) || dalloc(&F->d_nn, B) || dalloc(&F->d_valid, B * kp) ||
      dalloc(&F->d_hasmp, B * kp) || dalloc(&F->d_sf, p->nlevels) ||
      dalloc(&F->d_s2, p->nlevels) || dalloc(&F->d_match, B * kp) ||
      dalloc(&F->d_bow_count, B + 1) || dalloc(&F->d_m12, B * kp) ||
      dalloc(&F->d_pairs, B * kp * 2) || dalloc(&F->d_tri_count, B) || dalloc(&F->d_bprob, B) ||
      dalloc(&F->d_tprob, B))
    return fail(ORBX_ENOMEM);
  if (stereo) {
    stereo_scratch(*F->v.g, (int)kp, &F->st_nrows, &F->st_row_cap);
    if (dalloc(&F->d_lcounts, B) || dalloc(&F->d_uright, B * kp) ||
        dalloc(&F->d_depth, B * kp) || dalloc(&F->d_sad, B * kp) ||
        dalloc(&F->d_row_off, B * (F->st_nrows + 1)) ||
        dalloc(&F->d_row_idx, B * (size_t)F->st_row_cap) || dalloc(&F->d_sprob, B))
      return fail(ORBX_ENOMEM);
  }
  if (hipMemcpy(F->d_sf, F->v.g->scale, 4 * p->nlevels, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(F->d_s2, F->v.g->sigma2, 4 * p->nlevels, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(F->d_valid, 1, B * kp) != hipSuccess ||
      hipMemset(F->d_hasmp, 0, B * kp) != hipSuccess ||
      hipMemset(F->d_bow_count, 0, 4 * (B + 1)) != hipSuccess ||
      hipMemset(F->d_tri_count, 0, 4 * B) != hipSuccess)
    return fail(ORBX_EDEVICE);
  *out = F;
  return ORBX_OK;
}

int orbx_frames_create(const orbx_params* p, int32_t w, int32_t h, int32_t max_batch,
                       const orbx_vocabulary* voc, int32_t levelsup, int hip_device,
                       orbx_frames** out) {
  return frames_create(p, w, h, max_batch, voc, levelsup, 0, 0.f, 0.f, hip_device, out);
}

int orbx_frames_create_stereo(const orbx_params* p, int32_t w, int32_t h, int32_t max_batch,
                              const orbx_vocabulary* voc, int32_t levelsup, float mb, float mbf,
                              int hip_device, orbx_frames** out) {
  return frames_create(p, w, h, max_batch, voc, levelsup, 1, mb, mbf, hip_device, out);
}

int orbx_frames_destroy(orbx_frames* F) {
  ORBX_RESOURCE_LOCK;
  if (!F) return ORBX_OK;
  F->drop_graphs();
  void* ptrs[] = {F->d_lcounts, F->d_uright, F->d_depth, F->d_sad, F->d_row_off, F->d_row_idx,
                  F->d_sprob, F->d_rank_of, F->d_word_of, F->d_wt_of, F->d_bow_words, F->d_bow_vals, F->d_bow_n,
                  F->d_node_of, F->d_ids,   F->d_off,       F->d_feats,
                  F->d_nn,    F->d_valid,   F->d_hasmp, F->d_sf,        F->d_s2,
                  F->d_match, F->d_bow_count, F->d_m12, F->d_pairs,     F->d_tri_count,
                  F->d_bprob, F->d_tprob};
  for (void* p : ptrs)
    if (p) hipFree(p);
  if (F->plan) orbx_plan_destroy(F->plan);
  delete F;
  return ORBX_OK;
}

int orbx_frames_capacity(const orbx_frames* F, int32_t* kp_cap) {
  if (!F || !kp_cap) return ORBX_EINVAL;
  *kp_cap = F->v.kp_total;
  return ORBX_OK;
}

int orbx_frames_set_masks(orbx_frames* F, const uint8_t* valid, const uint8_t* has_mp) {
  if (!F) return ORBX_EINVAL;
  const size_t bytes = (size_t)F->max_frames * F->v.kp_total;
  if (valid) ORBX_HIP(hipMemcpy(F->d_valid, valid, bytes, hipMemcpyHostToDevice));
  if (has_mp) ORBX_HIP(hipMemcpy(F->d_hasmp, has_mp, bytes, hipMemcpyHostToDevice));
  return ORBX_OK;
}

int orbx_frames_set_matching(orbx_frames* F, float bow_ratio, int32_t bow_check_ori,
                             const float F12[9], float ex, float ey, float tri_ratio,
                             int32_t tri_check_ori, int32_t only_stereo) {
  if (!F || !F12) return ORBX_EINVAL;
  F->bow_ratio = bow_ratio;
  F->bow_ori = bow_check_ori;
  memcpy(F->F, F12, sizeof(F->F));
  F->ex = ex;
  F->ey = ey;
  F->tri_ratio = tri_ratio;
  F->tri_ori = tri_check_ori;
  F->only_stereo = only_stereo;
  F->prob_n = -1;  // rebuild problem descriptors
  F->drop_graphs();
  return ORBX_OK;
}

int orbx_frames_run(orbx_frames* F, const uint8_t* d_imgs, int32_t n) {
  if (!F || !d_imgs || n < 1 || n > F->max_frames) return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(F->device));
  if (F->prob_n != n) {
    int rc = build_problems(F, n);
    if (rc) return rc;
    F->drop_graphs();
  }
  if (F->prof.on) return enqueue(F, d_imgs, n, &F->prof);
  return run_graph(F->graphs, F->v.stream, d_imgs, n,
                   [&] { return enqueue(F, d_imgs, n, nullptr); });
}

int orbx_frames_sync(orbx_frames* F) {
  if (!F) return ORBX_EINVAL;
  ORBX_HIP(hipStreamSynchronize(F->v.stream));
  return ORBX_OK;
}

int orbx_frames_results(orbx_frames* F, int32_t n, int32_t* kp_counts, int32_t* bow_matches,
                        int32_t* tri_matches, int32_t* error) {
  if (!F || n < 1 || n > F->max_frames) return ORBX_EINVAL;
  hipStream_t s = F->v.stream;
  if (kp_counts) ORBX_HIP(hipMemcpyAsync(kp_counts, fcounts(F), 4 * n, hipMemcpyDeviceToHost, s));
  if (bow_matches)
    ORBX_HIP(hipMemcpyAsync(bow_matches, F->d_bow_count, 4 * n, hipMemcpyDeviceToHost, s));
  if (tri_matches)
    ORBX_HIP(hipMemcpyAsync(tri_matches, F->d_tri_count, 4 * n, hipMemcpyDeviceToHost, s));
  if (error)
    ORBX_HIP(hipMemcpyAsync(error, F->d_bow_count + F->bow_err_slot(), 4, hipMemcpyDeviceToHost, s));
  ORBX_HIP(hipStreamSynchronize(s));
  return ORBX_OK;
}

int orbx_frames_outputs(orbx_frames* F, orbx_keypoint** d_kps, uint8_t** d_desc,
                        int32_t** d_counts, uint32_t** d_node_of, int32_t** d_bow_match,
                        int32_t** d_tri_pairs) {
  if (!F) return ORBX_EINVAL;
  if (d_kps) *d_kps = F->v.d_kps;
  if (d_desc) *d_desc = F->v.d_desc;
  if (d_counts) *d_counts = F->v.d_counts;
  if (d_node_of) *d_node_of = F->d_node_of;
  if (d_bow_match) *d_bow_match = F->d_match;
  if (d_tri_pairs) *d_tri_pairs = F->d_pairs;
  return ORBX_OK;
}

int orbx_frames_stereo(orbx_frames* F, float** d_uright, float** d_depth) {
  if (!F || !F->stereo) return ORBX_EINVAL;
  if (d_uright) *d_uright = F->d_uright;
  if (d_depth) *d_depth = F->d_depth;
  return ORBX_OK;
}

int orbx_frames_bow(orbx_frames* F, uint32_t** d_bow_words, double** d_bow_values,
                    int32_t** d_bow_n, uint32_t** d_word_of) {
  if (!F) return ORBX_EINVAL;
  if (d_bow_words) *d_bow_words = F->d_bow_words;
  if (d_bow_values) *d_bow_values = F->d_bow_vals;
  if (d_bow_n) *d_bow_n = F->d_bow_n;
  if (d_word_of) *d_word_of = F->d_word_of;
  return ORBX_OK;
}

void* orbx_frames_stream(orbx_frames* F) { return F ? (void*)F->v.stream : nullptr; }

int orbx_frames_profile(orbx_frames* F, int32_t enable) {
  if (!F) return ORBX_EINVAL;
  F->prof.on = enable != 0;
  F->prof.reset();
  return ORBX_OK;
}

int orbx_frames_profile_read(orbx_frames* F, int32_t cap, char (*names)[32], double* total_ms,
                             int64_t* launches, int32_t* n_stages) {
  if (!F) return ORBX_EINVAL;
  if (F->prof.collect() != 0) return ORBX_EDEVICE;
  const int n = (int)F->prof.names.size();
  if (n_stages) *n_stages = n;
  for (int i = 0; i < n && i < cap; i++) {
    if (names) {
      strncpy(names[i], F->prof.names[i].c_str(), 31);
      names[i][31] = 0;
    }
    if (total_ms) total_ms[i] = F->prof.ms[i];
    if (launches) launches[i] = F->prof.launches[i];
  }
  return ORBX_OK;
}

int orbx_frames_profile_kernels(orbx_frames* F, int32_t stage, char* buf, int32_t cap) {
  if (!F) return ORBX_EINVAL;
  const int r = F->prof.kernels_of(stage, buf, cap);
  return r == 0 ? ORBX_OK : r > 0 ? ORBX_ECAPACITY : ORBX_EINVAL;
}

}  // extern "C"
