// orbx_api.hip — the drop-in C ABI around a plan: ORBextractor semantics for one host image
// (ORB_SLAM2/src/ORBextractor.cc:404-460, 985-1045; ORB_SLAM2/include/ORBextractor.h:52-88).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "orbx_internal.h"
#include "orbx_match.h"
#include "orbx_stereo.h"

using namespace orbx;

extern "C" int orbx_plan_level_dims(const orbx_plan* P, int level, int* w, int* h);
extern "C" int orbx_plan_level_download(orbx_plan* P, int img, int level, uint8_t* out,
                                        int64_t stride);
extern "C" int orbx_plan_level_download_buf(orbx_plan* P, int img, int level, uint8_t* out,
                                            int64_t stride, int blurred);

// One ORBextractor: a batch-1 plan for the current image size plus pinned host staging.  A
// call is one graph launch — pinned image -> HBM copy, the whole extraction, and one copy of
// the plan's output block (count, keypoints, descriptors) back to pinned memory — and one
// stream synchronisation; the caller's pageable image / output buffers are touched only by
// host memcpy.
struct orbx_extractor {
  orbx_params params{};
  Geometry tables;  // scale / sigma / features-per-level (no image size)
  int device = 0;
  orbx_plan* plan = nullptr;
  int pw = 0, ph = 0;
  uint8_t* d_img = nullptr;
  uint8_t* h_img = nullptr;  // pinned [h][w]
  char* h_out = nullptr;     // pinned copy of the plan's output block
  size_t kps_off = 0, desc_off = 0, out_bytes = 0;
  GraphCache graphs;
  bool has_run = false;
  void release() {
    ORBX_RESOURCE_LOCK;
    if (plan) graphs.clear((hipStream_t)orbx_plan_stream(plan));
    if (plan) orbx_plan_destroy(plan);
    if (d_img) (void)hipFree(d_img);
    if (h_img) (void)hipHostFree(h_img);
    if (h_out) (void)hipHostFree(h_out);
    plan = nullptr;
    d_img = h_img = nullptr;
    h_out = nullptr;
    pw = ph = 0;
  }
};

extern "C" {

int orbx_extractor_create(const orbx_params* params, int hip_device, orbx_extractor** out) {
  if (!params || !out || params->nlevels < 1 || params->nlevels > kMaxLevels ||
      params->nfeatures < 0 || !(params->scale_factor > 0))
    return ORBX_EINVAL;
  orbx_extractor* ex = new (std::nothrow) orbx_extractor();
  if (!ex) return ORBX_ENOMEM;
  ex->params = *params;
  ex->device = hip_device;
  build_tables(*params, &ex->tables);
  *out = ex;
  return ORBX_OK;
}

int orbx_extractor_destroy(orbx_extractor* ex) {
  ORBX_RESOURCE_LOCK;
  if (!ex) return ORBX_OK;
  ex->release();
  delete ex;
  return ORBX_OK;
}

int orbx_extractor_tables(const orbx_extractor* ex, int32_t* nlevels, float* scale_factors,
                          float* inv_scale_factors, float* level_sigma2, float* inv_level_sigma2,
                          int32_t* features_per_level) {
  if (!ex) return ORBX_EINVAL;
  const Geometry& g = ex->tables;
  if (nlevels) *nlevels = g.nlevels;
  for (int l = 0; l < g.nlevels; l++) {
    if (scale_factors) scale_factors[l] = g.scale[l];
    if (inv_scale_factors) inv_scale_factors[l] = g.inv_scale[l];
    if (level_sigma2) level_sigma2[l] = g.sigma2[l];
    if (inv_level_sigma2) inv_level_sigma2[l] = g.inv_sigma2[l];
    if (features_per_level) features_per_level[l] = g.feats[l];
  }
  return ORBX_OK;
}

int orbx_extract(orbx_extractor* ex, const uint8_t* img, int32_t w, int32_t h, int64_t stride,
                 orbx_keypoint* kps, uint8_t* desc, int32_t cap, int32_t* n_out) {
  if (!ex || !n_out) return ORBX_EINVAL;
  if (w <= 0 || h <= 0) {  // operator() returns early on an empty image (:987-988)
    *n_out = -1;
    return ORBX_OK;
  }
  if (!img || stride < w || cap < 0 || (cap > 0 && (!kps || !desc))) return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(ex->device));
  if (!ex->plan || ex->pw != w || ex->ph != h) {
    ORBX_RESOURCE_LOCK;
    ex->release();
    int rc = orbx_plan_create(&ex->params, w, h, 1, ex->device, &ex->plan);
    if (rc != ORBX_OK) return rc;
    plan_output_block(ex->plan, &ex->kps_off, &ex->desc_off, &ex->out_bytes);
    if (hipMalloc(&ex->d_img, (size_t)w * h) != hipSuccess ||
        hipHostMalloc(&ex->h_img, (size_t)w * h, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&ex->h_out, ex->out_bytes, hipHostMallocDefault) != hipSuccess) {
      ex->release();
      return ORBX_ENOMEM;
    }
    ex->pw = w;
    ex->ph = h;
  }
  hipStream_t s = (hipStream_t)orbx_plan_stream(ex->plan);
  orbx_keypoint* d_kps;
  uint8_t* d_desc;
  int32_t* d_counts;
  orbx_plan_outputs(ex->plan, &d_kps, &d_desc, &d_counts);
  // the caller's image (a pageable cv::Mat) into pinned staging
  if (stride == w) {
    memcpy(ex->h_img, img, (size_t)w * h);
  } else {
    for (int y = 0; y < h; y++) memcpy(ex->h_img + (size_t)y * w, img + (size_t)y * stride, w);
  }
  auto enqueue = [&]() -> int {
    ORBX_HIP(hipMemcpyAsync(ex->d_img, ex->h_img, (size_t)w * h, hipMemcpyHostToDevice, s));
    const int r = plan_enqueue(ex->plan, ex->d_img, 1, nullptr);
    if (r != ORBX_OK) return r;
    ORBX_HIP(hipMemcpyAsync(ex->h_out, d_counts, ex->out_bytes, hipMemcpyDeviceToHost, s));
    return ORBX_OK;
  };
  // one captured graph per input (direct launches measured slower: 0.131 vs 0.120 ms per call)
  int rc = run_graph(ex->graphs, s, ex->h_img, 1, enqueue);
  if (rc != ORBX_OK) return rc;
  ORBX_HIP(orbx::wait_stream(s));
  ex->has_run = true;
  const int32_t n = *(const int32_t*)ex->h_out;
  *n_out = n;
  if (n > cap) return ORBX_ECAPACITY;
  if (n > 0) {
    memcpy(kps, ex->h_out + ex->kps_off, sizeof(orbx_keypoint) * n);
    memcpy(desc, ex->h_out + ex->desc_off, (size_t)32 * n);
  }
  return ORBX_OK;
}

int orbx_extractor_pyramid(orbx_extractor* ex, int32_t level, uint8_t* out, int64_t stride,
                           int32_t* w, int32_t* h) {
  if (!ex || !ex->plan || !ex->has_run) return ORBX_EINVAL;
  int lw = 0, lh = 0;
  int rc = orbx_plan_level_dims(ex->plan, level, &lw, &lh);
  if (rc != ORBX_OK) return rc;
  if (w) *w = lw;
  if (h) *h = lh;
  if (!out) return ORBX_OK;
  if (stride < lw) return ORBX_EINVAL;
  return orbx_plan_level_download(ex->plan, 0, level, out, stride);
}

// Test hook (orbx.h): the GaussianBlur'd level of the last extraction (ORBextractor.cc:1024-1026).
int orbx_debug_extractor_blur(orbx_extractor* ex, int32_t level, uint8_t* out, int64_t stride) {
  if (!ex || !ex->plan || !ex->has_run || !out) return ORBX_EINVAL;
  int lw = 0, lh = 0;
  int rc = orbx_plan_level_dims(ex->plan, level, &lw, &lh);
  if (rc != ORBX_OK) return rc;
  if (stride < lw) return ORBX_EINVAL;
  return orbx_plan_level_download_buf(ex->plan, 0, level, out, stride, 1);
}

// Frame::ComputeStereoMatches (ORB_SLAM2/src/Frame.cc:471-643) on the last extraction of a
// left and a right extractor (their keypoints, descriptors and mvImagePyramid are still
// resident on the device).  uright / depth: host arrays of the left keypoint count.
int orbx_stereo_matches(orbx_extractor* left, orbx_extractor* right, float mb, float mbf,
                        float* uright, float* depth, int32_t* n_out) {
  if (!left || !right || !uright || !depth || !left->has_run || !right->has_run)
    return ORBX_EINVAL;
  if (left->pw != right->pw || left->ph != right->ph || left->device != right->device ||
      left->params.nlevels != right->params.nlevels ||
      left->params.scale_factor != right->params.scale_factor)
    return ORBX_EINVAL;
  ORBX_HIP(hipSetDevice(left->device));
  PlanView vl, vr;
  plan_view(left->plan, &vl);
  plan_view(right->plan, &vr);
  int nrows;
  int64_t row_cap;
  stereo_scratch(*vl.g, vr.kp_total, &nrows, &row_cap);
  const int kp = vl.kp_total;
  Stager st;
  const size_t oprob = st.add(nullptr, sizeof(StereoProblem));
  const size_t ouse = st.add(nullptr, (size_t)kp * 4), odep = st.add(nullptr, (size_t)kp * 4),
               osad = st.add(nullptr, (size_t)kp * 4), ocnt = st.add(nullptr, 4),
               ooff = st.add(nullptr, ((size_t)nrows + 1) * 4),
               oidx = st.add(nullptr, (size_t)row_cap * 8);
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  StereoProblem P{};
  P.kl = vl.d_kps;
  P.dl = vl.d_desc;
  P.nl = vl.d_counts;
  P.kr = vr.d_kps;
  P.dr = vr.d_desc;
  P.nr = vr.d_counts;
  P.pyrL = vl.d_pyr;
  P.pyrR = vr.d_pyr;
  P.uright = dptr<float>(base, ouse);
  P.depth = dptr<float>(base, odep);
  P.sad = dptr<int>(base, osad);
  P.row_off = dptr<int>(base, ooff);
  P.row_ent = dptr<uint2>(base, oidx);
  ORBX_HIP(hipMemcpyAsync(base + oprob, &P, sizeof(P), hipMemcpyHostToDevice, s));
  rc = launch_stereo(dptr<StereoProblem>(base, oprob), 1, vl.d_lv, vl.g->nlevels, nrows, row_cap,
                     kp, mb, mbf, s);
  if (rc) return rc;
  int32_t n = 0;
  ORBX_HIP(hipMemcpyAsync(&n, vl.d_counts, 4, hipMemcpyDeviceToHost, s));
  ORBX_HIP(orbx::wait_stream(s));
  (void)ocnt;
  if (n > 0) {
    ORBX_HIP(hipMemcpyAsync(uright, base + ouse, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(depth, base + odep, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    ORBX_HIP(orbx::wait_stream(s));
  }
  if (n_out) *n_out = n;
  return ORBX_OK;
}

}  // extern "C"
