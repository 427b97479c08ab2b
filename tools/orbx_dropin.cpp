// orbx_dropin — measures the drop-in per-frame path the way ORB-SLAM2 calls it (bench.py
// --dropin).  K host threads, each one camera with its own extractor (the reference keeps one
// ORBextractor per camera and runs the stereo pair's two on two threads, Frame.cc:83-86), push
// pageable host images (cv::Mat) one frame per call through the C ABI:
//   orbx_extract                    ORBextractor::operator()    Frame.cc:252-258, ORBextractor.cc:985-1045
//   orbx_vocabulary_transform       Frame::ComputeBoW           Frame.cc:400-407
//   orbx_search_by_bow_kf_f         SearchByBoW(KF*, F&)        Tracking.cc:1132-1136 (TrackReferenceKeyFrame)
//   orbx_search_for_triangulation   SearchForTriangulation      LocalMapping.cc:238-241
// with the previous frame of the same camera as the keyframe.  Prints one JSON line: aggregate
// frames/s and per-frame latency (median / mean, as mono_tum.cc:113-121 reports tracking time),
// per call.
//
// MODE "capi" (default) calls the C ABI directly with buffers reused across frames.  MODE
// "shim" replays what the reference-side shims (include/compat/*.cc) do around each call, so the
// number is what Frame.cc:252-258 / Tracking.cc:1132-1136 / LocalMapping.cc:238-241 would see
// with the shims linked in — everything but OpenCV itself, which is not in this image:
//   ORBextractor_orbx.cc   the library writes into the extractor's kept keypoint / descriptor
//                          blocks, then the keypoint vector of n and descriptors.create(n, 32) +
//                          the row copy; no pyramid export (mvImagePyramid is materialised on demand, mono never does)
//   Frame_orbx.cc          per-call output vectors, then BowVector / FeatureVector as the
//                          reference's std::maps (map<WordId, double>, map<NodeId,
//                          vector<unsigned>>)
//   ORBmatcher_orbx.cc     GetMapPointMatches() copies, the validity masks (isBad per point),
//                          angles, the std::map FeatureVectors -> CSR for both sides, the match
//                          vector back to MapPoint pointers; SearchForTriangulation's
//                          one GetMapPointMatches() snapshot per keyframe and the
//                          vector<pair<size_t, size_t>> result
// The shims' scratch (CSR, masks, angles, the transform's and matchers' raw outputs) is kept per
// thread and reused from call to call, as the shims keep it (CallScratch).
// In shim mode thread 0 also writes its first and last timed frames to DIR/dump_first.bin and
// DIR/dump_last.bin (what the shims hand back to Frame / ORBmatcher's callers: keypoints,
// descriptors, the std::map BowVector and FeatureVector, SearchByBoW's MapPoint pointers as
// point indices, SearchForTriangulation's pairs, with the masks and the geometry the calls used)
// for tests/test_dropin_gpu.py to check against the CPU oracle.
//
// usage: orbx_dropin DIR W H NFEATURES N_IMG THREADS WARMUP FRAMES DEVICE [MODE]
//   DIR/frames.u8       THREADS x N_IMG x H x W u8 images
//   DIR/voc_parent.i32, voc_leaf.u8, voc_desc.u8, voc_weight.f64   k=10, L=6 vocabulary nodes
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "orbx.h"

namespace {

using Clock = std::chrono::steady_clock;

std::vector<char> slurp(const std::string& path) {
  std::vector<char> v;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path.c_str());
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  v.resize((size_t)n);
  if (n && fread(v.data(), 1, (size_t)n, f) != (size_t)n) {
    fprintf(stderr, "short read %s\n", path.c_str());
    exit(2);
  }
  fclose(f);
  return v;
}

#define CK(x)                                                        \
  do {                                                               \
    int rc_ = (x);                                                   \
    if (rc_ != ORBX_OK) {                                            \
      fprintf(stderr, "%s failed: %d (line %d)\n", #x, rc_, __LINE__); \
      exit(3);                                                       \
    }                                                                \
  } while (0)

// One frame as the matchers see it (Frame / KeyFrame members the calls read).
struct FrameData {
  int n = 0;
  std::vector<orbx_keypoint> kps;
  std::vector<uint8_t> desc;
  std::vector<float> angle;
  std::vector<uint8_t> valid, has_mp;
  std::vector<uint32_t> fv_ids, bow_words;
  std::vector<int32_t> fv_off, fv_feats;
  std::vector<double> bow_values;
  std::vector<uint32_t> word_of, node_of;
  int fv_n = 0, bow_n = 0;
  void reserve(int cap) {
    kps.resize(cap);
    desc.resize((size_t)cap * 32);
    angle.resize(cap);
    valid.resize(cap);
    has_mp.resize(cap);
    fv_ids.resize(cap);
    fv_off.resize(cap + 1);
    fv_feats.resize(cap);
    bow_words.resize(cap);
    bow_values.resize(cap);
    word_of.resize(cap);
    node_of.resize(cap);
  }
  orbx_featvec fv() const { return {fv_n, fv_ids.data(), fv_off.data(), fv_feats.data()}; }
};

// ----------------------------------------------------------------- the shims' host side
// Stand-ins for the reference's objects with the members the shims touch.
struct MapPointStub {
  bool bad = false;
  bool isBad() const { return bad; }  // MapPoint::isBad locks mMutexFeatures in the reference
};
typedef std::map<uint32_t, double> BowVectorMap;                   // DBoW2::BowVector
typedef std::map<uint32_t, std::vector<unsigned int> > FeatVecMap;  // DBoW2::FeatureVector

struct ShimFrame {  // a Frame / KeyFrame: mvKeysUn, mDescriptors, BoW, map points
  int N = 0;
  std::vector<orbx_keypoint> keys;
  std::vector<uint8_t> desc;  // the n x 32 cv::Mat
  BowVectorMap bow;
  FeatVecMap fv;
  // mvpMapPoints.  The bench's unit of work draws SearchByBoW's "valid" (60 %) and
  // triangulation's "has a point" (40 %) independently, so the stand-in keeps one array per call
  // to do the same work as the capi mode; the reference reads both from one array.
  std::vector<MapPointStub*> mps, mps_tri;
  mutable std::mutex mutex_features;
  std::vector<MapPointStub*> GetMapPointMatches() const {
    std::lock_guard<std::mutex> lk(mutex_features);
    return mps;
  }
  std::vector<MapPointStub*> GetMapPointMatchesTri() const {  // triangulation's draw
    std::lock_guard<std::mutex> lk(mutex_features);
    return mps_tri;
  }
};

struct FeatVecCSR {  // ORBmatcher_orbx.cc's std::map -> CSR (capacity kept between calls)
  std::vector<uint32_t> ids;
  std::vector<int32_t> off, feats;
  orbx_featvec view;
  void assign(const FeatVecMap& fv) {
    ids.clear();
    off.clear();
    feats.clear();
    off.push_back(0);
    for (FeatVecMap::const_iterator it = fv.begin(); it != fv.end(); ++it) {
      ids.push_back(it->first);
      feats.insert(feats.end(), it->second.begin(), it->second.end());
      off.push_back((int32_t)feats.size());
    }
    view = orbx_featvec{(int32_t)ids.size(), ids.data(), off.data(), feats.data()};
  }
};

// the shims' per-thread scratch (ORBmatcher_orbx.cc, Frame_orbx.cc: CallScratch)
struct CallScratch {
  FeatVecCSR f1, f2;
  std::vector<uint8_t> m1, m2;
  std::vector<float> a1, a2;
  std::vector<int32_t> idx, fo, ff;
  std::vector<uint32_t> bw, fi;
  std::vector<double> bv;
  std::vector<orbx_keypoint> kps;  // ORBextractor_orbx.cc's ExtractorCtx::kps / desc
  std::vector<uint8_t> desc;
};
CallScratch& scratch() {
  static thread_local CallScratch s;
  return s;
}

void angles_of(const std::vector<orbx_keypoint>& k, std::vector<float>& a) {
  a.resize(k.size());
  for (size_t i = 0; i < k.size(); i++) a[i] = k[i].angle;
}

// ORBextractor::operator() as ORBextractor_orbx.cc runs it
int shim_extract(orbx_extractor* ex, const uint8_t* img, int W, int H, int nfeatures,
                 ShimFrame& F) {
  CallScratch& S = scratch();
  int32_t cap = std::max<int32_t>(4 * nfeatures + 64, (int32_t)S.kps.size()), n = 0;
  if ((int32_t)S.kps.size() < cap) S.kps.resize(cap);
  if (S.desc.size() < (size_t)cap * 32) S.desc.resize((size_t)cap * 32);
  int rc = orbx_extract(ex, img, W, H, W, S.kps.data(), S.desc.data(), cap, &n);
  if (rc == ORBX_ECAPACITY) {
    cap = n;
    S.kps.resize(cap);
    S.desc.resize((size_t)cap * 32);
    rc = orbx_extract(ex, img, W, H, W, S.kps.data(), S.desc.data(), cap, &n);
  }
  if (rc != ORBX_OK) return rc;
  n = std::max(n, 0);
  F.keys.assign(S.kps.begin(), S.kps.begin() + n);
  F.desc.assign(S.desc.begin(), S.desc.begin() + (size_t)n * 32);  // create(n, 32) + copyTo
  F.N = n;
  return ORBX_OK;
}

// Frame::ComputeBoW as Frame_orbx.cc runs it: ascending ids, so every map entry is placed at
// the end by hint (no tree search)
int shim_compute_bow(orbx_vocabulary* voc, ShimFrame& F) {
  CallScratch& S = scratch();
  const int n = F.N;
  const size_t m = (size_t)std::max(n, 1);
  S.bw.resize(m);
  S.fi.resize(m + 1);
  S.bv.resize(m);
  S.fo.resize(m + 2);
  S.ff.resize(m);
  int32_t nb = 0, nf = 0;
  const int rc = orbx_vocabulary_transform(voc, F.desc.data(), n, 4, nullptr, nullptr, S.bw.data(),
                                           S.bv.data(), &nb, S.fi.data(), S.fo.data(), S.ff.data(), &nf);
  if (rc != ORBX_OK) return rc;
  F.bow.clear();
  F.fv.clear();
  for (int i = 0; i < nb; i++) F.bow.emplace_hint(F.bow.end(), S.bw[i], S.bv[i]);
  for (int j = 0; j < nf; j++)
    F.fv.emplace_hint(F.fv.end(), S.fi[j],
                      std::vector<unsigned int>(S.ff.begin() + S.fo[j], S.ff.begin() + S.fo[j + 1]));
  return ORBX_OK;
}

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) as ORBmatcher_orbx.cc runs it
int shim_search_by_bow(const ShimFrame& KF, const ShimFrame& F, std::vector<MapPointStub*>& out,
                       int32_t* nmatches) {
  CallScratch& S = scratch();
  const std::vector<MapPointStub*> vpMP = KF.GetMapPointMatches();
  S.m1.resize(vpMP.size());
  for (size_t i = 0; i < vpMP.size(); i++) S.m1[i] = vpMP[i] && !vpMP[i]->isBad();
  angles_of(KF.keys, S.a1);
  angles_of(F.keys, S.a2);
  S.f1.assign(KF.fv);
  S.f2.assign(F.fv);
  const orbx_bow_side kf{KF.N, KF.desc.data(), S.a1.data(), S.m1.data(), S.f1.view};
  const orbx_bow_side fr{F.N, F.desc.data(), S.a2.data(), nullptr, S.f2.view};
  S.idx.resize(std::max(F.N, 1));
  const int rc = orbx_search_by_bow_kf_f(&kf, &fr, 0.7f, 1, S.idx.data(), nmatches);
  if (rc != ORBX_OK) return rc;
  out.assign(F.N, nullptr);
  for (int i = 0; i < F.N; i++)
    if (S.idx[i] >= 0) out[i] = vpMP[S.idx[i]];
  return ORBX_OK;
}

// ORBmatcher::SearchForTriangulation as ORBmatcher_orbx.cc runs it (the epipole's three cv::Mat
// products are left out)
int shim_search_for_triangulation(const ShimFrame& K1, const ShimFrame& K2, const float* F12,
                                  float ex, float ey, const float* scale, const float* sigma2,
                                  int nl, std::vector<std::pair<size_t, size_t> >& pairs_out,
                                  int32_t* nmatches) {
  CallScratch& S = scratch();
  S.m1.resize(K1.N);
  S.m2.resize(K2.N);
  {
    const std::vector<MapPointStub*> vp1 = K1.GetMapPointMatchesTri(), vp2 = K2.GetMapPointMatchesTri();
    for (int i = 0; i < K1.N; i++) S.m1[i] = vp1[i] != nullptr;
    for (int i = 0; i < K2.N; i++) S.m2[i] = vp2[i] != nullptr;
  }
  S.f1.assign(K1.fv);
  S.f2.assign(K2.fv);
  const orbx_tri_side s1{K1.N, K1.desc.data(), K1.keys.data(), nullptr, S.m1.data(), S.f1.view,
                         scale, sigma2, nl};
  const orbx_tri_side s2{K2.N, K2.desc.data(), K2.keys.data(), nullptr, S.m2.data(), S.f2.view,
                         scale, sigma2, nl};
  S.idx.resize(2 * std::max(K1.N, 1));
  const int rc = orbx_search_for_triangulation(&s1, &s2, F12, ex, ey, 0, 0.6f, 0, S.idx.data(),
                                               nmatches);
  if (rc != ORBX_OK) return rc;
  pairs_out.clear();
  pairs_out.reserve(*nmatches);
  for (int i = 0; i < *nmatches; i++)
    pairs_out.push_back(std::make_pair((size_t)S.idx[2 * i], (size_t)S.idx[2 * i + 1]));
  return ORBX_OK;
}

// One frame's shim outputs for the oracle check (tests/test_dropin_gpu.py reads this layout)
struct Dump {
  FILE* f;
  explicit Dump(const std::string& path) : f(fopen(path.c_str(), "wb")) {}
  ~Dump() {
    if (f) fclose(f);
  }
  void raw(const void* p, size_t n) {
    if (f && n) fwrite(p, 1, n, f);
  }
  void i32(int32_t v) { raw(&v, 4); }
  void u8(bool v) {
    const uint8_t b = v ? 1 : 0;
    raw(&b, 1);
  }
  void frame(const ShimFrame& F) {
    i32(F.N);
    raw(F.keys.data(), sizeof(orbx_keypoint) * F.N);
    raw(F.desc.data(), (size_t)32 * F.N);
    i32((int32_t)F.bow.size());
    for (const auto& e : F.bow) i32((int32_t)e.first);
    for (const auto& e : F.bow) raw(&e.second, 8);
    i32((int32_t)F.fv.size());
    for (const auto& e : F.fv) i32((int32_t)e.first);
    int32_t o = 0;
    i32(o);
    for (const auto& e : F.fv) i32(o += (int32_t)e.second.size());
    for (const auto& e : F.fv)
      for (unsigned v : e.second) i32((int32_t)v);
  }
};

struct Stats {
  std::vector<double> total, extract, bow, search_bow, search_tri;
  long long matches_bow = 0, matches_tri = 0, keypoints = 0;
};

double median(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  const size_t m = v.size() / 2;
  return v.size() % 2 ? v[m] : 0.5 * (v[m - 1] + v[m]);
}
double mean(const std::vector<double>& v) {
  double s = 0;
  for (double x : v) s += x;
  return v.empty() ? 0 : s / v.size();
}
double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 10) {
    fprintf(stderr, "usage: %s DIR W H NFEATURES N_IMG THREADS WARMUP FRAMES DEVICE [capi|shim]\n",
            argv[0]);
    return 1;
  }
  const std::string mode = argc > 10 ? argv[10] : "capi";
  if (mode != "capi" && mode != "shim") {
    fprintf(stderr, "MODE must be capi or shim\n");
    return 1;
  }
  const bool shim = mode == "shim";
  const std::string dir = argv[1];
  const int W = atoi(argv[2]), H = atoi(argv[3]), NF = atoi(argv[4]), NIMG = atoi(argv[5]);
  const int T = atoi(argv[6]), WARM = atoi(argv[7]), FR = atoi(argv[8]), DEV = atoi(argv[9]);
  const std::vector<char> frames = slurp(dir + "/frames.u8");
  if (frames.size() != (size_t)T * NIMG * W * H) {
    fprintf(stderr, "frames.u8 has %zu bytes, expected %zu\n", frames.size(),
            (size_t)T * NIMG * W * H);
    return 2;
  }
  const std::vector<char> parent = slurp(dir + "/voc_parent.i32"), leaf = slurp(dir + "/voc_leaf.u8"),
                          vdesc = slurp(dir + "/voc_desc.u8"), weight = slurp(dir + "/voc_weight.f64");
  const int n_nodes = (int)(parent.size() / 4);
  orbx_vocabulary* voc = nullptr;
  CK(orbx_vocabulary_create(10, 6, ORBX_SCORE_L1, ORBX_WEIGHT_TF_IDF, n_nodes,
                            (const int32_t*)parent.data(), (const uint8_t*)leaf.data(),
                            (const uint8_t*)vdesc.data(), (const double*)weight.data(), DEV, &voc));

  // SearchForTriangulation geometry: R = I, t = (0.10, 0.02, 0.05), TUM1 K
  const float fx = 517.306408f, fy = 516.469215f, cx = 318.643040f, cy = 255.313989f;
  const float tx = 0.10f, ty = 0.02f, tz = 0.05f;
  const float Kinv[9] = {1 / fx, 0, -cx / fx, 0, 1 / fy, -cy / fy, 0, 0, 1};
  const float Tx[9] = {0, -tz, ty, tz, 0, -tx, -ty, tx, 0};
  float A[9], F12[9];
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      float s = 0;
      for (int k = 0; k < 3; k++) s += Tx[3 * r + k] * Kinv[3 * k + c];
      A[3 * r + c] = s;
    }
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      float s = 0;
      for (int k = 0; k < 3; k++) s += Kinv[3 * k + r] * A[3 * k + c];  // Kinv^T * A
      F12[3 * r + c] = s;
    }
  const float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, tv[3] = {tx, ty, tz}, Cw[3] = {0, 0, 0};
  float ex = 0, ey = 0;
  CK(orbx_epipole(R, tv, Cw, fx, fy, cx, cy, &ex, &ey));

  std::vector<Stats> stats(T);
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<double> thread_wall(T, 0.0);
  auto worker = [&](int t) {
    orbx_params prm{NF, 1.2f, 8, 20, 7};
    orbx_extractor* exr = nullptr;
    CK(orbx_extractor_create(&prm, DEV, &exr));
    float scale[8], sigma2[8];
    int32_t nl = 0;
    CK(orbx_extractor_tables(exr, &nl, scale, nullptr, sigma2, nullptr, nullptr));
    const int cap = NF * 2 + 64;
    FrameData fd[2];
    fd[0].reserve(cap);
    fd[1].reserve(cap);
    std::vector<int32_t> match(cap), pairs((size_t)cap * 2);
    Stats& st = stats[t];
    uint32_t lcg = 0x9E3779B9u * (t + 1);
    auto rnd = [&]() {
      lcg = lcg * 1664525u + 1013904223u;
      return (lcg >> 8) * (1.0f / 16777216.0f);
    };
    ready++;
    while (!go.load()) std::this_thread::yield();
    // shim mode: frames with their map points (the masks' 60 % / 40 % as stub MapPoints)
    ShimFrame sf[2];
    std::vector<MapPointStub> mp_pool((size_t)4 * cap);
    std::vector<MapPointStub*> bow_out;
    std::vector<std::pair<size_t, size_t> > tri_out;
    Clock::time_point t_start;
    for (int f = 0; f < WARM + FR && shim; f++) {
      if (f == WARM) t_start = Clock::now();
      ShimFrame& cur = sf[f & 1];
      ShimFrame& prev = sf[(f + 1) & 1];
      const uint8_t* img = (const uint8_t*)frames.data() + ((size_t)t * NIMG + f % NIMG) * W * H;
      const auto a = Clock::now();
      CK(shim_extract(exr, img, W, H, NF, cur));
      const auto b = Clock::now();
      CK(shim_compute_bow(voc, cur));
      // map points: SearchByBoW's "valid" (60 %), triangulation's "has a point" (40 %)
      cur.mps.assign(cur.N, nullptr);
      cur.mps_tri.assign(cur.N, nullptr);
      for (int i = 0; i < cur.N; i++) {
        MapPointStub* m = &mp_pool[(size_t)(f & 1) * 2 * cap + i];
        m->bad = false;
        cur.mps[i] = rnd() < 0.6f ? m : nullptr;
        cur.mps_tri[i] = rnd() < 0.4f ? m : nullptr;
      }
      const auto c = Clock::now();
      auto d = c, e = c;
      int32_t nb = 0, nt = 0;
      if (f > 0) {
        CK(shim_search_by_bow(prev, cur, bow_out, &nb));
        d = Clock::now();
        CK(shim_search_for_triangulation(prev, cur, F12, ex, ey, scale, sigma2, nl, tri_out, &nt));
        e = Clock::now();
      }
      if (f >= WARM) {
        auto ms = [](Clock::time_point x, Clock::time_point y) {
          return std::chrono::duration<double, std::milli>(y - x).count();
        };
        st.total.push_back(ms(a, e));
        st.extract.push_back(ms(a, b));
        st.bow.push_back(ms(b, c));
        st.search_bow.push_back(ms(c, d));
        st.search_tri.push_back(ms(d, e));
        st.matches_bow += nb;
        st.matches_tri += nt;
        st.keypoints += cur.N;
      }
      if (t == 0 && f > 0 && (f == std::max(WARM, 1) || f == WARM + FR - 1)) {
        // after the timing of this frame: the first and last timed frames of thread 0
        Dump D(dir + (f == WARM + FR - 1 ? "/dump_last.bin" : "/dump_first.bin"));
        D.raw("ORBXDMP1", 8);
        D.i32(f);
        D.i32(f % NIMG);
        D.i32((f - 1) % NIMG);
        D.raw(F12, 36);
        D.raw(&ex, 4);
        D.raw(&ey, 4);
        D.i32(nl);
        D.raw(scale, 4 * nl);
        D.raw(sigma2, 4 * nl);
        D.frame(prev);
        D.frame(cur);
        const MapPointStub* pbase = &mp_pool[(size_t)((f + 1) & 1) * 2 * cap];
        for (int i = 0; i < prev.N; i++) D.u8(prev.mps[i] && !prev.mps[i]->isBad());
        for (int i = 0; i < prev.N; i++) D.u8(prev.mps_tri[i] != nullptr);
        for (int i = 0; i < cur.N; i++) D.u8(cur.mps_tri[i] != nullptr);
        D.i32(nb);
        for (int i = 0; i < cur.N; i++) D.i32(bow_out[i] ? (int32_t)(bow_out[i] - pbase) : -1);
        D.i32(nt);
        for (const auto& pr : tri_out) {
          D.i32((int32_t)pr.first);
          D.i32((int32_t)pr.second);
        }
      }
    }
    for (int f = 0; f < WARM + FR && !shim; f++) {
      if (f == WARM) t_start = Clock::now();
      FrameData& cur = fd[f & 1];
      FrameData& prev = fd[(f + 1) & 1];
      const uint8_t* img = (const uint8_t*)frames.data() + ((size_t)t * NIMG + f % NIMG) * W * H;
      const auto a = Clock::now();
      int32_t n = 0;
      CK(orbx_extract(exr, img, W, H, W, cur.kps.data(), cur.desc.data(), cap, &n));
      cur.n = n;
      const auto b = Clock::now();
      CK(orbx_vocabulary_transform(voc, cur.desc.data(), n, 4, cur.word_of.data(),
                                   cur.node_of.data(), cur.bow_words.data(), cur.bow_values.data(),
                                   &cur.bow_n, cur.fv_ids.data(), cur.fv_off.data(),
                                   cur.fv_feats.data(), &cur.fv_n));
      for (int i = 0; i < n; i++) {
        cur.angle[i] = cur.kps[i].angle;
        cur.valid[i] = rnd() < 0.6f;
        cur.has_mp[i] = rnd() < 0.4f;
      }
      const auto c = Clock::now();
      auto d = c, e = c;
      int32_t nb = 0, nt = 0;
      if (f > 0) {
        orbx_bow_side kf{prev.n, prev.desc.data(), prev.angle.data(), prev.valid.data(), prev.fv()};
        orbx_bow_side fr{cur.n, cur.desc.data(), cur.angle.data(), nullptr, cur.fv()};
        CK(orbx_search_by_bow_kf_f(&kf, &fr, 0.7f, 1, match.data(), &nb));
        d = Clock::now();
        orbx_tri_side k1{prev.n, prev.desc.data(), prev.kps.data(), nullptr, prev.has_mp.data(),
                         prev.fv(), scale, sigma2, nl};
        orbx_tri_side k2{cur.n, cur.desc.data(), cur.kps.data(), nullptr, cur.has_mp.data(),
                         cur.fv(), scale, sigma2, nl};
        CK(orbx_search_for_triangulation(&k1, &k2, F12, ex, ey, 0, 0.6f, 0, pairs.data(), &nt));
        e = Clock::now();
      }
      if (f >= WARM) {
        auto ms = [](Clock::time_point x, Clock::time_point y) {
          return std::chrono::duration<double, std::milli>(y - x).count();
        };
        st.total.push_back(ms(a, e));
        st.extract.push_back(ms(a, b));
        st.bow.push_back(ms(b, c));
        st.search_bow.push_back(ms(c, d));
        st.search_tri.push_back(ms(d, e));
        st.matches_bow += nb;
        st.matches_tri += nt;
        st.keypoints += n;
      }
    }
    thread_wall[t] = std::chrono::duration<double>(Clock::now() - t_start).count();
    orbx_extractor_destroy(exr);
  };
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++) th.emplace_back(worker, t);
  while (ready.load() < T) std::this_thread::yield();
  go = true;
  for (auto& x : th) x.join();

  Stats all;
  for (auto& s : stats) {
    all.total.insert(all.total.end(), s.total.begin(), s.total.end());
    all.extract.insert(all.extract.end(), s.extract.begin(), s.extract.end());
    all.bow.insert(all.bow.end(), s.bow.begin(), s.bow.end());
    all.search_bow.insert(all.search_bow.end(), s.search_bow.begin(), s.search_bow.end());
    all.search_tri.insert(all.search_tri.end(), s.search_tri.begin(), s.search_tri.end());
    all.matches_bow += s.matches_bow;
    all.matches_tri += s.matches_tri;
    all.keypoints += s.keypoints;
  }
  const double wall = *std::max_element(thread_wall.begin(), thread_wall.end());
  const double nfr = (double)all.total.size();
  printf("{\"mode\": \"%s\", \"fps\": %.2f, \"frames\": %d, \"threads\": %d, \"wall_s\": %.4f, "
         "\"median_ms\": %.4f, \"mean_ms\": %.4f, \"p90_ms\": %.4f, "
         "\"per_call_median_ms\": {\"orbx_extract\": %.4f, \"orbx_vocabulary_transform\": %.4f, "
         "\"orbx_search_by_bow_kf_f\": %.4f, \"orbx_search_for_triangulation\": %.4f}, "
         "\"per_call_mean_ms\": {\"orbx_extract\": %.4f, \"orbx_vocabulary_transform\": %.4f, "
         "\"orbx_search_by_bow_kf_f\": %.4f, \"orbx_search_for_triangulation\": %.4f}, "
         "\"keypoints_per_frame\": %.1f, \"bow_matches_per_frame\": %.1f, "
         "\"triangulation_matches_per_frame\": %.1f}\n",
         mode.c_str(), nfr / wall, (int)nfr, T, wall, median(all.total), mean(all.total), pct(all.total, 0.9),
         median(all.extract), median(all.bow), median(all.search_bow), median(all.search_tri),
         mean(all.extract), mean(all.bow), mean(all.search_bow), mean(all.search_tri),
         all.keypoints / nfr, all.matches_bow / nfr, all.matches_tri / nfr);
  orbx_vocabulary_destroy(voc);
  return 0;
}
