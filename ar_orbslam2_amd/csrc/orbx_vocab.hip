// orbx_vocab.hip — DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> on the device:
// text loader, greedy Hamming descent, BowVector and FeatureVector
// (ORB_SLAM2/Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h, BowVector.cpp, FeatureVector.cpp).
//
//   k_voc_transform  one 16- (k <= 16) or 32-lane group per feature: lane c scores child c of
//                    the current node, the group's (distance, child) minimum picks the next
//                    node; child records are contiguous per parent so a level is one
//                    coalesced round trip (transform, TemplatedVocabulary.h:1218-1259)
//   k_bowvec         one workgroup per image: stable LSD radix sort of the features by word
//                    in LDS, per-word weight sums in feature order (BowVector::addWeight /
//                    addIfNotExist, BowVector.cpp:38-62), then the scoring's L1/L2
//                    normalisation as one ordered pass (BowVector::normalize, :66-98)
//   k_bowfv          one workgroup per image of up to 2048 features (4096 in calls of at most 4
//                    images): the BowVector above and
//                    the FeatureVector CSR together, from two in-register bitonic sorts merged
//                    by rank (one launch instead of k_bowvec + k_csr)
// Otherwise the FeatureVector CSR reuses k_csr (orbx_match.hip) over the node ranks built here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "orbx_internal.h"
#include "orbx_match.h"
#include "orbx_vocab.h"

#pragma clang fp contract(off)

struct orbx_vocabulary {
  int device = 0;
  int k = 0, L = 0, scoring = 0, weighting = 0;
  int n_nodes = 1, n_words = 0;  // n_nodes counts the root
  int max_children = 0;          // the widest node (VocView::k), found once at build
  // host tree (node ids in file order)
  std::vector<int> parent, depth, child_begin, nchild;
  std::vector<uint32_t> child_ids;  // per-parent contiguous child records
  std::vector<int> word_of_node;    // 0 unless flagged leaf (Node(): word_id(0))
  // device
  uint8_t* d_cdesc = nullptr;
  int4* d_cmeta = nullptr;
  double* d_weight = nullptr;
  double* d_word_weight = nullptr;
  std::mutex m;
  std::vector<orbx::VocRanks*> ranks;
  ~orbx_vocabulary() {
    for (void* p : {(void*)d_cdesc, (void*)d_cmeta, (void*)d_weight, (void*)d_word_weight})
      if (p) (void)hipFree(p);
    for (auto* r : ranks) {
      if (r->d_rank_of_node) (void)hipFree(r->d_rank_of_node);
      if (r->d_rank_ids) (void)hipFree(r->d_rank_ids);
      delete r;
    }
  }
};

namespace orbx {

// ------------------------------------------------------------------ k_voc_transform
template <int G>
__global__ __launch_bounds__(256) void k_voc_transform(VocView V, int nid_level,
                                                       const uint32_t* __restrict__ rank_of_node,
                                                       const uint8_t* __restrict__ desc,
                                                       int64_t desc_stride,
                                                       const int* __restrict__ counts,
                                                       int n_fixed, uint32_t* __restrict__ word_out,
                                                       uint32_t* __restrict__ rank_out,
                                                       uint32_t* __restrict__ node_out,
                                                       double* __restrict__ weight_out,
                                                       int64_t out_stride, VocHostOut ho) {
  const int img = blockIdx.y, tid = threadIdx.x;
  const int c = tid & (G - 1);
  const int f = blockIdx.x * (256 / G) + tid / G;
  const int n = counts ? counts[img] : n_fixed;
  const bool active = f < n;  // uniform within a group
  uint64_t d[4] = {0, 0, 0, 0};
  if (active) {
    const uint4* q = (const uint4*)(desc + img * desc_stride + (int64_t)f * 32);
    const uint4 a = q[0], b = q[1];
    d[0] = a.x | ((uint64_t)a.y << 32);
    d[1] = a.z | ((uint64_t)a.w << 32);
    d[2] = b.x | ((uint64_t)b.y << 32);
    d[3] = b.z | ((uint64_t)b.w << 32);
  }
  int cb = V.root_cb, nc = (active && V.n_words > 0) ? V.root_nc : 0;
  int node = 0, level = 0, word = 0;
  uint32_t nid = nid_level <= 0 ? 0u : 0xFFFFFFFFu;
  const int lane = tid & 63, gbase = lane & ~(G - 1);
  while (__any(nc > 0)) {
    const bool go = nc > 0;
    int key = 0x7FFFFFFF;
    int4 meta = make_int4(0, 0, 0, 0);
    if (go && c < nc) {
      const uint4* cd = (const uint4*)(V.cdesc + (int64_t)(cb + c) * 32);
      const uint4 a = cd[0], b = cd[1];
      const int dist = __popcll(d[0] ^ (a.x | ((uint64_t)a.y << 32))) +
                       __popcll(d[1] ^ (a.z | ((uint64_t)a.w << 32))) +
                       __popcll(d[2] ^ (b.x | ((uint64_t)b.y << 32))) +
                       __popcll(d[3] ^ (b.z | ((uint64_t)b.w << 32)));
      meta = V.cmeta[cb + c];
      key = dist * 64 + c;  // strict `d < best_d` over children in order: lowest c on ties
    }
    if constexpr (G == 16) {
      key = (int)row16_min((uint32_t)key);  // keys are >= 0
    } else {
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) key = min(key, __shfl_xor(key, o));
    }
    const int src = gbase + (key & 63);
    const int mx = __shfl(meta.x, src), my = __shfl(meta.y, src), mz = __shfl(meta.z, src),
              mw = __shfl(meta.w, src);
    if (go) {
      ++level;
      node = mx;
      cb = my;
      nc = mz;
      word = mw;
      if (level == nid_level) nid = (uint32_t)node;
    }
  }
  if (!active || c != 0) return;
  if (ho.desc_copy) {  // one-image calls: the descriptors into the frame cache's entry
    uint4* q = (uint4*)(ho.desc_copy + (int64_t)f * 32);
    q[0] = make_uint4((uint32_t)d[0], (uint32_t)(d[0] >> 32), (uint32_t)d[1], (uint32_t)(d[1] >> 32));
    q[1] = make_uint4((uint32_t)d[2], (uint32_t)(d[2] >> 32), (uint32_t)d[3], (uint32_t)(d[3] >> 32));
  }
  const int64_t o = img * out_stride + f;
  if (V.n_words == 0) {  // transform: if(empty()) return;
    word_out[o] = 0xFFFFFFFFu;
    rank_out[o] = 0xFFFFFFFFu;
    if (node_out) node_out[o] = 0xFFFFFFFFu;
    weight_out[o] = 0;
    if (ho.word_of) ho.word_of[f] = 0xFFFFFFFFu;
    if (ho.node_of) ho.node_of[f] = 0xFFFFFFFFu;
    return;
  }
  if (nid == 0xFFFFFFFFu) nid = (uint32_t)node;  // leaf above L - levelsup (header)
  const double w = V.weight[node];
  weight_out[o] = w;
  const bool keep = w > 0;  // `if(w > 0) // not stopped`
  word_out[o] = keep ? (uint32_t)word : 0xFFFFFFFFu;
  rank_out[o] = keep ? rank_of_node[nid] : 0xFFFFFFFFu;
  if (node_out) node_out[o] = keep ? nid : 0xFFFFFFFFu;
  if (ho.word_of) ho.word_of[f] = keep ? (uint32_t)word : 0xFFFFFFFFu;
  if (ho.node_of) ho.node_of[f] = keep ? nid : 0xFFFFFFFFu;
}

// ------------------------------------------------------------------ k_bowvec
__device__ __forceinline__ int block_excl_scan(int v, int* s_tmp, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int incl = wave_scan_incl(v);
  if (lane == 63) s_tmp[wid] = incl;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < 4; w++) {
    if (w < wid) base += s_tmp[w];
    tot += s_tmp[w];
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

// Stable LSD radix sort of the non-stopped features by word id (10-bit digits, as many passes
// as the largest word id needs), so each word's features stay in index order: the order
// BowVector::addWeight accumulates them in.  Keys are (word << 32 | feature) pairs; every
// wave scatters its own contiguous quarter of the current order, behind per-(digit, wave)
// offsets (digit-major, wave-minor: stable).
constexpr int kRadixBits = 10, kRadixB = 1 << kRadixBits;

__global__ __launch_bounds__(256) void k_bowvec(int must, int l1, int tf,
                                                const uint32_t* __restrict__ word_of,
                                                const double* __restrict__ weight_of,
                                                int64_t in_stride, const int* __restrict__ counts,
                                                int n_fixed, int cap,
                                                uint32_t* __restrict__ out_words,
                                                double* __restrict__ out_vals, int64_t out_stride,
                                                int* __restrict__ out_n) {
  extern __shared__ __align__(16) int sm[];
  uint64_t* s_a = (uint64_t*)sm;            // [cap] keys (ping)
  uint64_t* s_b = s_a + cap;                // [cap] keys (pong)
  int* s_cnt = (int*)(s_b + cap);           // [kRadixB][4] per (digit, wave)
  __shared__ int s_tmp[4];
  __shared__ unsigned s_max;
  __shared__ double s_norm;
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = counts ? counts[img] : n_fixed;
  const uint32_t* wo = word_of + img * in_stride;
  const double* wt = weight_of + img * in_stride;
  if (tid == 0) s_max = 0;
  const int per = cap / 256;  // thread t owns indices [t*per, (t+1)*per)
  uint32_t* s_w = (uint32_t*)s_b;  // words staged in the pong buffer
  for (int i = tid; i < cap; i += 256) s_w[i] = i < n ? wo[i] : 0xFFFFFFFFu;  // coalesced
  __syncthreads();
  int cnt = 0;
  unsigned mx = 0;
  for (int i = tid * per; i < (tid + 1) * per; i++) {
    const uint32_t w = s_w[i];
    if (w != 0xFFFFFFFFu) {
      cnt++;
      mx = max(mx, w);
    }
  }
  atomicMax(&s_max, mx);
  int m;
  int pos = block_excl_scan(cnt, s_tmp, &m);  // stable compaction of the kept features
  for (int i = tid * per; i < (tid + 1) * per; i++) {
    const uint32_t w = s_w[i];
    if (w != 0xFFFFFFFFu) s_a[pos++] = ((uint64_t)w << 32) | (uint32_t)i;
  }
  __syncthreads();
  const unsigned wmax = s_max;
  const int q0 = (int)(((int64_t)m * wid) / 4), q1 = (int)(((int64_t)m * (wid + 1)) / 4);
  for (int shift = 0; m > 0 && shift < 32 && (shift == 0 || (wmax >> shift) != 0);
       shift += kRadixBits) {
    for (int b = tid; b < 4 * kRadixB; b += 256) s_cnt[b] = 0;
    __syncthreads();
    for (int j = q0 + lane; j < q1; j += 64)
      atomicAdd(&s_cnt[4 * ((int)(s_a[j] >> (32 + shift)) & (kRadixB - 1)) + wid], 1);
    __syncthreads();
    {  // exclusive scan over (digit, wave): 32 entries per thread
      constexpr int E = 4 * kRadixB / 256;
      int c[E], sum = 0;
#pragma unroll
      for (int q = 0; q < E; q++) {
        c[q] = s_cnt[tid * E + q];
        sum += c[q];
      }
      int tot;
      int base = block_excl_scan(sum, s_tmp, &tot);
#pragma unroll
      for (int q = 0; q < E; q++) {
        s_cnt[tid * E + q] = base;
        base += c[q];
      }
    }
    __syncthreads();
    {  // stable scatter of this wave's quarter, 64 keys at a time
      const uint64_t lt = (1ull << lane) - 1, gt = ~((2ull << lane) - 1);
      for (int c0 = q0; c0 < q1; c0 += 64) {
        const int j = c0 + lane;
        const bool valid = j < q1;
        const uint64_t key = valid ? s_a[j] : 0;
        const int dg = (int)(key >> (32 + shift)) & (kRadixB - 1);
        uint64_t eq = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < kRadixBits; bit++) {
          const uint64_t mb = __ballot(valid && ((dg >> bit) & 1));
          eq &= ((dg >> bit) & 1) ? mb : ~mb;
        }
        if (valid) {
          int* slot = &s_cnt[4 * dg + wid];
          const int base = *slot;
          s_b[base + __popcll(eq & lt)] = key;
          if ((eq & gt) == 0) *slot = base + __popcll(eq);  // last lane of the digit
        }
      }
    }
    __syncthreads();
    uint64_t* t = s_a;
    s_a = s_b;
    s_b = t;
  }
  // run starts of equal words (contiguous chunks per thread, stable block scan), kept in
  // the free pong buffer
  int* s_pos = (int*)s_b;
  cnt = 0;
  for (int j = tid * per; j < (tid + 1) * per; j++)
    cnt += j < m && (j == 0 || (s_a[j] >> 32) != (s_a[j - 1] >> 32));
  int nu;
  pos = block_excl_scan(cnt, s_tmp, &nu);
  for (int j = tid * per; j < (tid + 1) * per; j++)
    if (j < m && (j == 0 || (s_a[j] >> 32) != (s_a[j - 1] >> 32))) s_pos[pos++] = j;
  if (tid == 0) s_pos[nu] = m;
  __syncthreads();
  uint32_t* ow = out_words + img * out_stride;
  double* ov = out_vals + img * out_stride;
  for (int o = tid; o < nu; o += 256) {
    const int a = s_pos[o], b = s_pos[o + 1];
    double v = wt[(uint32_t)s_a[a]];  // insert(value_type(id, w)) of the first occurrence
    if (tf)
      for (int j = a + 1; j < b; j++) v += wt[(uint32_t)s_a[j]];  // addWeight, feature order
    if (tf && !must) v /= (double)nu;  // TemplatedVocabulary.h:1165-1172
    ow[o] = (uint32_t)(s_a[a] >> 32);
    ov[o] = v;
  }
  if (tid == 0) out_n[img] = nu;
  if (!must) return;
  __syncthreads();
  // the values back into LDS (over the pong keys) for the ordered normalisation pass
  double* s_val = (double*)s_b;
  for (int o = tid; o < nu; o += 256) s_val[o] = ov[o];
  __syncthreads();
  if (tid == 0) {  // BowVector::normalize: one ordered pass over the words
    // (the adds stay in word order; LDS reads are batched 8 at a time)
    double norm = 0.0;
    int o = 0;
    if (l1) {
      for (; o + 8 <= nu; o += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = s_val[o + j];
#pragma unroll
        for (int j = 0; j < 8; j++) norm += fabs(v[j]);
      }
      for (; o < nu; o++) norm += fabs(s_val[o]);
    } else {
      // built -O3 -march=native (Thirdparty/DBoW2/CMakeLists.txt): `norm += v * v` contracts
      for (; o + 8 <= nu; o += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = s_val[o + j];
#pragma unroll
        for (int j = 0; j < 8; j++) norm = fma(v[j], v[j], norm);
      }
      for (; o < nu; o++) norm = fma(s_val[o], s_val[o], norm);
      norm = sqrt(norm);
    }
    s_norm = norm;
  }
  __syncthreads();
  const double norm = s_norm;
  if (norm > 0.0)
    for (int o = tid; o < nu; o += 256) ov[o] = s_val[o] / norm;
}

int launch_voc_transform(const VocView& V, int nid_level, const uint32_t* d_rank_of_node,
                         const uint8_t* d_desc, int64_t desc_stride_img, const int* d_counts,
                         int n_fixed, int max_n, uint32_t* d_word_of, uint32_t* d_rank_of,
                         uint32_t* d_node_of, double* d_weight_of, int64_t out_stride_img,
                         int nimg, hipStream_t s, const VocHostOut& ho) {
  if (max_n <= 0 || nimg <= 0) return ORBX_OK;
  if (V.k <= 16) {
    note_kernel("k_voc_transform<16>");
    hipLaunchKernelGGL(k_voc_transform<16>, dim3((max_n + 15) / 16, nimg), dim3(256), 0, s, V,
                       nid_level, d_rank_of_node, d_desc, desc_stride_img, d_counts, n_fixed,
                       d_word_of, d_rank_of, d_node_of, d_weight_of, out_stride_img, ho);
  } else if (V.k <= 32) {
    note_kernel("k_voc_transform<32>");
    hipLaunchKernelGGL(k_voc_transform<32>, dim3((max_n + 7) / 8, nimg), dim3(256), 0, s, V,
                       nid_level, d_rank_of_node, d_desc, desc_stride_img, d_counts, n_fixed,
                       d_word_of, d_rank_of, d_node_of, d_weight_of, out_stride_img, ho);
  } else {
    return ORBX_EUNSUPPORTED;
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_voc_transform");
}

int bowvec_cap(int max_n) {
  int cap = 256;
  while (cap < max_n) cap <<= 1;
  return cap;
}

int launch_bowvec(int scoring, int weighting, const uint32_t* d_word_of,
                  const double* d_weight_of, int64_t in_stride, const int* d_counts, int n_fixed,
                  int max_n, uint32_t* d_words, double* d_values, int64_t out_stride,
                  int* d_nwords, int nimg, hipStream_t s) {
  if (nimg <= 0) return ORBX_OK;
  const int cap = bowvec_cap(std::max(max_n, 1));
  const size_t smem = 16 * (size_t)cap + 16 * kRadixB;
  if (cap > 8192) return ORBX_EUNSUPPORTED;
  const int must = scoring != ORBX_SCORE_DOT_PRODUCT;
  const int l1 = scoring != ORBX_SCORE_L2;
  const int tf = weighting == ORBX_WEIGHT_TF_IDF || weighting == ORBX_WEIGHT_TF;
  if (smem > 64 * 1024) {  // more than the default dynamic LDS limit (8192 features: 104 KB)
    static std::once_flag once;
    static hipError_t attr = hipSuccess;
    std::call_once(once, [] {
      attr = hipFuncSetAttribute((const void*)k_bowvec, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 16 * 8192 + 16 * kRadixB);
    });
    if (attr != hipSuccess) return report_hip(attr, "hipFuncSetAttribute(k_bowvec)");
  }
  note_kernel("k_bowvec");
  hipLaunchKernelGGL(k_bowvec, dim3(nimg), dim3(256), smem, s, must, l1, tf, d_word_of,
                     d_weight_of, in_stride, d_counts, n_fixed, cap, d_words, d_values,
                     out_stride, d_nwords);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_bowvec");
}

// ------------------------------------------------------------------ k_bowfv
// BowVector and FeatureVector of an image in one workgroup, for images of at most 256 * NPL
// features whose word ids and FeatureVector ranks fit beside a feature index in 32 bits.  Both
// orders are stable sorts of (key << IB | feature) words — word for the BowVector
// (BowVector::addWeight / addIfNotExist in feature order, BowVector.cpp:38-62), FeatureVector
// rank for the node lists (FeatureVector::addFeature, FeatureVector.cpp:31-45) — so both are
// sorts of distinct 32-bit keys:
//  (1) every wave sorts its 64 * NPL keys of each order in registers (bitonic network: NPL keys
//      per lane, partners inside a lane or across lanes by DPP / swizzle / bpermute);
//  (2) the four sorted runs merge by rank: a key's place = its place in its run + the keys
//      below it in the three other runs (branch-free binary searches in LDS);
//  (3) waves 0 / 1 find the word / node runs in LDS; the workgroup sums each word's weights in
//      feature order (weights staged in LDS with the keys) and writes the FeatureVector CSR
//      (node ids, offsets, features); one lane runs the scoring's ordered normalisation
//      (BowVector::normalize, :66-98).
// It replaces k_bowvec + k_csr (a radix sort with ~15 workgroup barriers, and a wave-serial
// bucket placement) where it applies: one launch and three barriers per image.
template <int M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v) {
  if constexpr (M == 1) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad [1,0,3,2]
  } else if constexpr (M == 2) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad [2,3,0,1]
  } else if constexpr (M < 32) {
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (M << 10));  // xor within 32
  } else {
    return (uint32_t)__shfl_xor((int)v, M);
  }
}

// Bitonic sort of a wave's 64 * NPL keys of two independent arrays (ascending; element
// e = lane * NPL + r).  Stage (k, j): e meets e ^ j, ascending where e & k == 0.
template <int NPL, int K, int J>
__device__ __forceinline__ void bitonic_stage(uint32_t (&a)[NPL], uint32_t (&b)[NPL], int lane) {
  if constexpr (J < NPL) {
#pragma unroll
    for (int r = 0; r < NPL; r++) {
      if (r & J) continue;
      const bool asc = K < NPL ? (r & K) == 0 : ((lane * NPL) & K) == 0;
      const uint32_t la = min(a[r], a[r | J]), ha = max(a[r], a[r | J]);
      const uint32_t lb = min(b[r], b[r | J]), hb = max(b[r], b[r | J]);
      a[r] = asc ? la : ha;
      a[r | J] = asc ? ha : la;
      b[r] = asc ? lb : hb;
      b[r | J] = asc ? hb : lb;
    }
  } else {
    constexpr int LJ = J / NPL;
    const bool takemin = (((lane * NPL) & K) == 0) == ((lane & LJ) == 0);
    uint32_t ya[NPL], yb[NPL];
#pragma unroll
    for (int r = 0; r < NPL; r++) {
      ya[r] = lane_xor<LJ>(a[r]);
      yb[r] = lane_xor<LJ>(b[r]);
    }
#pragma unroll
    for (int r = 0; r < NPL; r++) {
      a[r] = takemin ? min(a[r], ya[r]) : max(a[r], ya[r]);
      b[r] = takemin ? min(b[r], yb[r]) : max(b[r], yb[r]);
    }
  }
}

template <int NPL, int K, int J>
__device__ __forceinline__ void bitonic_js(uint32_t (&a)[NPL], uint32_t (&b)[NPL], int lane) {
  bitonic_stage<NPL, K, J>(a, b, lane);
  if constexpr (J > 1) bitonic_js<NPL, K, J / 2>(a, b, lane);
}

template <int NPL, int K>
__device__ __forceinline__ void bitonic_ks(uint32_t (&a)[NPL], uint32_t (&b)[NPL], int lane) {
  bitonic_js<NPL, K, K / 2>(a, b, lane);
  if constexpr (K < 64 * NPL) bitonic_ks<NPL, 2 * K>(a, b, lane);
}

constexpr uint32_t kBowSent = 0xFFFFFFFFu;  // no key (padding, stopped word): sorts last

template <int NPL>
__global__ __launch_bounds__(256) void k_bowfv(int must, int l1, int tf,
                                               const uint32_t* __restrict__ word_of,
                                               const uint32_t* __restrict__ rank_of,
                                               const double* __restrict__ weight_of,
                                               int64_t in_stride, const int* __restrict__ counts,
                                               int n_fixed, uint32_t* __restrict__ out_words,
                                               double* __restrict__ out_vals, int64_t out_stride,
                                               int* __restrict__ out_n, int nb,
                                               const uint32_t* __restrict__ rank_ids,
                                               uint32_t* __restrict__ node_ids,
                                               int* __restrict__ offsets, int* __restrict__ feats,
                                               int64_t feats_stride, int* __restrict__ n_nodes,
                                               VocHostOut ho) {
  constexpr int R = 64 * NPL, CAP = 4 * R;
  constexpr int IB = __builtin_ctz(CAP);
  constexpr uint32_t IMASK = (1u << IB) - 1u;
  extern __shared__ __align__(16) uint32_t smb[];
  uint32_t* runA = smb;                      // [CAP] the four sorted runs (word keys)
  uint32_t* runB = smb + CAP;                // [CAP] (rank keys)
  uint32_t* mA = smb + 2 * CAP;              // [CAP] merged
  uint32_t* mB = smb + 3 * CAP;              // [CAP]
  double* s_wt = (double*)(smb + 4 * CAP);   // [CAP] feature weights
  int* s_start = (int*)(smb + 6 * CAP);      // [CAP + 1] word run starts
  int* s_nstart = (int*)(smb + 7 * CAP + 4); // [CAP + 1] node run starts
  double* s_val = (double*)smb;              // [CAP] over the runs, after the merge
  __shared__ int s_cnt[2][4];
  __shared__ int s_nu, s_nn;
  __shared__ double s_norm;
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = counts ? counts[img] : n_fixed;
  const uint32_t* wo = word_of + img * in_stride;
  const uint32_t* ro = rank_of + img * in_stride;
  const double* wt = weight_of + img * in_stride;
  for (int i = tid; i < n; i += 256) s_wt[i] = wt[i];  // coalesced; read after the merge barrier
  uint32_t a[NPL], b[NPL];
  int ca = 0, cb = 0;
#pragma unroll
  for (int r = 0; r < NPL; r++) {
    const int i = wid * R + lane * NPL + r;
    const uint32_t w = i < n ? wo[i] : kBowSent, k = i < n ? ro[i] : kBowSent;
    a[r] = w != kBowSent ? (w << IB) | (uint32_t)i : kBowSent;
    b[r] = k != kBowSent ? (k << IB) | (uint32_t)i : kBowSent;
    ca += a[r] != kBowSent;
    cb += b[r] != kBowSent;
  }
  ca = wave_scan_incl(ca);
  cb = wave_scan_incl(cb);
  if (lane == 63) {
    s_cnt[0][wid] = ca;
    s_cnt[1][wid] = cb;
  }
  bitonic_ks<NPL, 2>(a, b, lane);
#pragma unroll
  for (int r = 0; r < NPL; r++) {
    runA[wid * R + lane * NPL + r] = a[r];
    runB[wid * R + lane * NPL + r] = b[r];
  }
  __syncthreads();
  const int m_a = s_cnt[0][0] + s_cnt[0][1] + s_cnt[0][2] + s_cnt[0][3];
  const int m_b = s_cnt[1][0] + s_cnt[1][1] + s_cnt[1][2] + s_cnt[1][3];
  {  // merge by rank: keys are distinct, so a key's place is unique
    int pa[NPL], pb[NPL];
#pragma unroll
    for (int r = 0; r < NPL; r++) pa[r] = pb[r] = lane * NPL + r;
#pragma unroll
    for (int o = 1; o < 4; o++) {
      const int w2 = (wid + o) & 3;
      const uint32_t* qa = runA + w2 * R;
      const uint32_t* qb = runB + w2 * R;
      int la[NPL], lb[NPL];
#pragma unroll
      for (int r = 0; r < NPL; r++) la[r] = lb[r] = 0;
#pragma unroll
      for (int st = R / 2; st > 0; st >>= 1) {  // la = min(keys below, R - 1)
#pragma unroll
        for (int r = 0; r < NPL; r++) {
          la[r] += qa[la[r] + st - 1] < a[r] ? st : 0;
          lb[r] += qb[lb[r] + st - 1] < b[r] ? st : 0;
        }
      }
#pragma unroll
      for (int r = 0; r < NPL; r++) {
        pa[r] += la[r] + (qa[la[r]] < a[r]);
        pb[r] += lb[r] + (qb[lb[r]] < b[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < NPL; r++) {
      if (a[r] != kBowSent) mA[pa[r]] = a[r];
      if (b[r] != kBowSent) mB[pb[r]] = b[r];
    }
  }
  __syncthreads();
  // run starts from LDS alone: wave 0 the words (BowVector entries), wave 1 the FeatureVector
  // nodes
  const uint64_t lt = (1ull << lane) - 1;
  if (wid < 2) {
    const uint32_t* mk = wid == 0 ? mA : mB;
    const int mm = wid == 0 ? m_a : m_b;
    int* starts = wid == 0 ? s_start : s_nstart;
    int cnt = 0;
    for (int c0 = 0; c0 < mm; c0 += 64) {
      const int j = c0 + lane;
      const bool valid = j < mm;
      const uint32_t x = valid ? mk[j] : 0u, px = valid && j > 0 ? mk[j - 1] : 0u;
      const bool st = valid && (j == 0 || (x >> IB) != (px >> IB));
      const uint64_t ball = __ballot(st);
      if (st) starts[cnt + __popcll(ball & lt)] = j;
      cnt += __popcll(ball);
    }
    if (lane == 0) {
      starts[cnt] = mm;
      if (wid == 0) s_nu = cnt;
      else s_nn = cnt;
    }
  }
  __syncthreads();
  const int nu = s_nu, nn = s_nn;
  // the whole workgroup: word weights summed in feature order (LDS), the CSR written out
  uint32_t* ow = out_words + img * out_stride;
  double* ov = out_vals + img * out_stride;
  for (int o = tid; o < nu; o += 256) {
    const int s0 = s_start[o], s1 = s_start[o + 1];
    const uint32_t x = mA[s0];
    double v = s_wt[x & IMASK];  // insert(value_type(id, w)) of the first occurrence
    if (tf)
      for (int j = s0 + 1; j < s1; j++) v += s_wt[mA[j] & IMASK];  // addWeight, feature order
    if (tf && !must) v /= (double)nu;  // TemplatedVocabulary.h:1165-1172
    ow[o] = x >> IB;
    if (ho.words) ho.words[o] = x >> IB;
    if (must) {
      s_val[o] = v;
    } else {
      ov[o] = v;
      if (ho.values) ho.values[o] = v;
    }
  }
  {
    uint32_t* oid = node_ids + (int64_t)img * nb;
    int* ooff = offsets + (int64_t)img * (nb + 1);
    int* of = feats + img * feats_stride;
    for (int q = tid; q < nn; q += 256) {
      const int j = s_nstart[q];
      const uint32_t id = rank_ids[mB[j] >> IB];
      oid[q] = id;
      ooff[q] = j;
      if (ho.ids) {
        ho.ids[q] = id;
        ho.off[q] = j;
      }
    }
    for (int j = tid; j < m_b; j += 256) {
      of[j] = (int)(mB[j] & IMASK);
      if (ho.feats) ho.feats[j] = (int)(mB[j] & IMASK);
    }
    if (tid == 0) {
      ooff[nn] = m_b;
      n_nodes[img] = nn;
      out_n[img] = nu;
      if (ho.off) ho.off[nn] = m_b;
      if (ho.nn) *ho.nn = nn;
      if (ho.nwords) *ho.nwords = nu;
    }
  }
  if (!must) return;
  __syncthreads();
  if (tid == 0) {  // BowVector::normalize: one ordered pass over the words (LDS reads 8 ahead)
    double norm = 0.0;
    int o = 0;
    if (l1) {
      for (; o + 8 <= nu; o += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = s_val[o + j];
#pragma unroll
        for (int j = 0; j < 8; j++) norm += fabs(v[j]);
      }
      for (; o < nu; o++) norm += fabs(s_val[o]);
    } else {
      // built -O3 -march=native (Thirdparty/DBoW2/CMakeLists.txt): `norm += v * v` contracts
      for (; o + 8 <= nu; o += 8) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = s_val[o + j];
#pragma unroll
        for (int j = 0; j < 8; j++) norm = fma(v[j], v[j], norm);
      }
      for (; o < nu; o++) norm = fma(s_val[o], s_val[o], norm);
      norm = sqrt(norm);
    }
    s_norm = norm;
  }
  __syncthreads();
  const double norm = s_norm;
  for (int o = tid; o < nu; o += 256) {
    const double v = norm > 0.0 ? s_val[o] / norm : s_val[o];
    ov[o] = v;
    if (ho.values) ho.values[o] = v;
  }
}

template <int NPL>
static int launch_bowfv_t(int must, int l1, int tf, const uint32_t* d_word_of,
                          const uint32_t* d_rank_of, const double* d_weight_of, int64_t in_stride,
                          const int* d_counts, int n_fixed, uint32_t* d_words, double* d_values,
                          int64_t out_stride, int* d_nwords, int nb, const uint32_t* d_rank_ids,
                          uint32_t* d_ids, int* d_off, int* d_feats, int64_t feats_stride,
                          int* d_nn, int nimg, hipStream_t s, const VocHostOut& ho) {
  constexpr int CAP = 256 * NPL;
  constexpr size_t smem = (size_t)CAP * 32 + 32;  // runs, merged orders, weights, run starts
  if constexpr (smem > 64 * 1024) {
    static std::once_flag once;
    static hipError_t attr = hipSuccess;
    std::call_once(once, [] {
      attr = hipFuncSetAttribute((const void*)k_bowfv<NPL>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    });
    if (attr != hipSuccess) return report_hip(attr, "hipFuncSetAttribute(k_bowfv)");
  }
  note_kernel(("k_bowfv<" + std::to_string(NPL) + ">").c_str());
  hipLaunchKernelGGL(k_bowfv<NPL>, dim3(nimg), dim3(256), smem, s, must, l1, tf, d_word_of,
                     d_rank_of, d_weight_of, in_stride, d_counts, n_fixed, d_words, d_values,
                     out_stride, d_nwords, nb, d_rank_ids, d_ids, d_off, d_feats, feats_stride,
                     d_nn, ho);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_bowfv");
}

int launch_bowfv(int scoring, int weighting, int n_words, const uint32_t* d_word_of,
                 const uint32_t* d_rank_of, const double* d_weight_of, int64_t in_stride,
                 const int* d_counts, int n_fixed, int max_n, uint32_t* d_words, double* d_values,
                 int64_t out_stride, int* d_nwords, int nb, const uint32_t* d_rank_ids,
                 uint32_t* d_ids, int* d_off, int* d_feats, int64_t feats_stride, int* d_nn,
                 int nimg, hipStream_t s, const VocHostOut& ho) {
  if (!d_rank_ids || nb < 1) return ORBX_EUNSUPPORTED;
  if (nimg <= 0) return ORBX_OK;
  const int must = scoring != ORBX_SCORE_DOT_PRODUCT;
  const int l1 = scoring != ORBX_SCORE_L2;
  const int tf = weighting == ORBX_WEIGHT_TF_IDF || weighting == ORBX_WEIGHT_TF;
  // keys (id << IB | feature) stay below the sentinel: id < 2^(32 - IB) - 1
  auto fits = [&](int cap, int ib) {
    const int64_t lim = ((int64_t)1 << (32 - ib)) - 1;
    return max_n <= cap && n_words < lim && nb < lim;
  };
#define ORBX_BOWFV_ARGS                                                                        \
  must, l1, tf, d_word_of, d_rank_of, d_weight_of, in_stride, d_counts, n_fixed, d_words,     \
      d_values, out_stride, d_nwords, nb, d_rank_ids, d_ids, d_off, d_feats, feats_stride, d_nn, \
      nimg, s, ho
  if (fits(1024, 10)) return launch_bowfv_t<4>(ORBX_BOWFV_ARGS);
  if (fits(2048, 11)) return launch_bowfv_t<8>(ORBX_BOWFV_ARGS);
  // 16 keys per lane take every VGPR (512, and a few spilled): one wave per SIMD.  A call of a
  // few images keeps it (a single frame's latency); batches of such frames take k_bowvec +
  // k_csr instead (C5's line 46.7-46.8 k -> 47.4 k frames/s)
  if (fits(4096, 12) && nimg <= 4) return launch_bowfv_t<16>(ORBX_BOWFV_ARGS);
#undef ORBX_BOWFV_ARGS
  return ORBX_EUNSUPPORTED;
}

// ------------------------------------------------------------------ host side
namespace {

template <class T>
int dalloc(T** p, size_t count) {
  if (count == 0) count = 1;
  if (hipMalloc((void**)p, count * sizeof(T)) != hipSuccess) return ORBX_ENOMEM;
  return ORBX_OK;
}

// Build the tree and upload it (node i of the arrays is node id i + 1).
int build_vocabulary(orbx_vocabulary* V, int n, const int32_t* parent, const uint8_t* is_leaf,
                     const uint8_t* desc, const double* weight) {
  const int N = n + 1;
  V->n_nodes = N;
  V->parent.assign(N, 0);
  V->depth.assign(N, 0);
  V->word_of_node.assign(N, 0);
  std::vector<std::vector<uint32_t>> children(N);
  std::vector<double> w(N, 0.0);  // root: Node(): weight(0)
  std::vector<int> words;
  for (int i = 0; i < n; i++) {
    const int nid = i + 1, pid = parent[i];
    if (pid < 0 || pid >= nid) return ORBX_EINVAL;  // m_nodes[pid] must already exist
    V->parent[nid] = pid;
    V->depth[nid] = V->depth[pid] + 1;
    children[pid].push_back((uint32_t)nid);
    w[nid] = weight[i];
    if (is_leaf[i]) {
      V->word_of_node[nid] = (int)words.size();
      words.push_back(nid);
    }
  }
  V->n_words = (int)words.size();
  // per-parent contiguous child records
  V->child_begin.assign(N, 0);
  V->nchild.assign(N, 0);
  V->child_ids.clear();
  V->child_ids.reserve(n);
  for (int p = 0; p < N; p++) {
    V->child_begin[p] = (int)V->child_ids.size();
    V->nchild[p] = (int)children[p].size();
    if (V->nchild[p] > 32) return ORBX_EUNSUPPORTED;  // more children than a lane group
    V->max_children = std::max(V->max_children, V->nchild[p]);
    V->child_ids.insert(V->child_ids.end(), children[p].begin(), children[p].end());
  }
  std::vector<uint8_t> cdesc((size_t)std::max(n, 1) * 32);
  std::vector<int4> cmeta(std::max(n, 1));
  for (size_t j = 0; j < V->child_ids.size(); j++) {
    const uint32_t c = V->child_ids[j];
    memcpy(&cdesc[j * 32], desc + (size_t)(c - 1) * 32, 32);
    cmeta[j] = make_int4((int)c, V->child_begin[c], V->nchild[c], V->word_of_node[c]);
  }
  std::vector<double> ww(std::max(V->n_words, 1), 0.0);
  for (int k = 0; k < V->n_words; k++) ww[k] = w[words[k]];
  if (hipSetDevice(V->device) != hipSuccess) return ORBX_EDEVICE;
  if (dalloc(&V->d_cdesc, cdesc.size()) || dalloc(&V->d_cmeta, cmeta.size()) ||
      dalloc(&V->d_weight, (size_t)N) || dalloc(&V->d_word_weight, ww.size()))
    return ORBX_ENOMEM;
  if (hipMemcpy(V->d_cdesc, cdesc.data(), cdesc.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(V->d_cmeta, cmeta.data(), cmeta.size() * sizeof(int4), hipMemcpyHostToDevice) !=
          hipSuccess ||
      hipMemcpy(V->d_weight, w.data(), (size_t)N * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(V->d_word_weight, ww.data(), ww.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
    return ORBX_EDEVICE;
  return ORBX_OK;
}

// strtol-based "int int 32*int double" line parser (std::stringstream >> semantics for
// well-formed lines; FORB::fromString keeps a byte whose token fails to parse as 0 here,
// the cv::Mat byte it leaves untouched is indeterminate in the reference)
bool parse_node_line(const char* s, int* pid, int* leaf, uint8_t* d, double* w) {
  char* e;
  errno = 0;
  long v = strtol(s, &e, 10);
  if (e == s) return false;
  *pid = (int)v;
  s = e;
  v = strtol(s, &e, 10);
  *leaf = e == s ? 0 : (int)v;
  s = e;
  for (int i = 0; i < 32; i++) {
    v = strtol(s, &e, 10);
    d[i] = e == s ? 0 : (uint8_t)v;
    s = e;
  }
  const double x = strtod(s, &e);
  *w = e == s ? 0.0 : x;
  return true;
}

}  // namespace

int vocab_view(const orbx_vocabulary* V, VocView* v, int* device) {
  if (!V || !v) return ORBX_EINVAL;
  v->cdesc = V->d_cdesc;
  v->cmeta = V->d_cmeta;
  v->weight = V->d_weight;
  v->word_weight = V->d_word_weight;
  v->root_cb = V->child_begin.empty() ? 0 : V->child_begin[0];
  v->root_nc = V->nchild.empty() ? 0 : V->nchild[0];
  v->n_words = V->n_words;
  v->k = V->max_children;  // (a scan of every node here cost ~0.2 ms per drop-in call)
  if (device) *device = V->device;
  return ORBX_OK;
}

// FeatureVector keys for a levelsup: the nodes at depth L - levelsup, plus the leaves above
// it (where the descent stops early), ranked by ascending id.
int vocab_ranks(const orbx_vocabulary* Vc, int levelsup, const VocRanks** out) {
  orbx_vocabulary* V = const_cast<orbx_vocabulary*>(Vc);
  {  // the usual case, a table built before: V->m alone (never held while waiting for the
     // resource lock, so the lock order below stays deadlock-free), no process-wide lock
    std::lock_guard<std::mutex> lk(V->m);
    for (auto* r : V->ranks)
      if (r->levelsup == levelsup) {
        *out = r;
        return ORBX_OK;
      }
  }
  ORBX_RESOURCE_LOCK;  // before V->m: frames_create holds it when it gets here
  std::lock_guard<std::mutex> lk(V->m);
  for (auto* r : V->ranks)
    if (r->levelsup == levelsup) {
      *out = r;
      return ORBX_OK;
    }
  const int nid_level = V->L - levelsup;
  std::vector<uint32_t> ids;
  std::vector<uint32_t> rank(V->n_nodes, 0xFFFFFFFFu);
  if (nid_level <= 0) {
    ids.push_back(0);
  } else {
    for (int i = 1; i < V->n_nodes; i++)
      if (V->depth[i] == nid_level || (V->depth[i] < nid_level && V->nchild[i] == 0))
        ids.push_back((uint32_t)i);
  }
  for (size_t b = 0; b < ids.size(); b++) rank[ids[b]] = (uint32_t)b;
  VocRanks* r = new (std::nothrow) VocRanks();
  if (!r) return ORBX_ENOMEM;
  r->levelsup = levelsup;
  r->nb = (int)ids.size();
  if (hipSetDevice(V->device) != hipSuccess) {
    delete r;
    return ORBX_EDEVICE;
  }
  if (dalloc(&r->d_rank_of_node, rank.size()) || dalloc(&r->d_rank_ids, ids.size()) ||
      hipMemcpy(r->d_rank_of_node, rank.data(), rank.size() * 4, hipMemcpyHostToDevice) !=
          hipSuccess ||
      (ids.size() &&
       hipMemcpy(r->d_rank_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice) !=
           hipSuccess)) {
    if (r->d_rank_of_node) (void)hipFree(r->d_rank_of_node);
    if (r->d_rank_ids) (void)hipFree(r->d_rank_ids);
    delete r;
    return ORBX_ENOMEM;
  }
  V->ranks.push_back(r);
  *out = r;
  return ORBX_OK;
}

}  // namespace orbx

using namespace orbx;

extern "C" {

int orbx_vocabulary_create(int32_t k, int32_t L, int32_t scoring, int32_t weighting,
                           int32_t n_nodes, const int32_t* parent, const uint8_t* is_leaf,
                           const uint8_t* desc, const double* weight, int32_t hip_device,
                           orbx_vocabulary** out) {
  ORBX_RESOURCE_LOCK;
  if (!out) return ORBX_EINVAL;
  *out = nullptr;
  // the loader's header check (TemplatedVocabulary.h:1360-1364)
  if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 ||
      weighting > 3 || n_nodes < 0)
    return ORBX_EINVAL;
  if (n_nodes > 0 && (!parent || !is_leaf || !desc || !weight)) return ORBX_EINVAL;
  orbx_vocabulary* V = new (std::nothrow) orbx_vocabulary();
  if (!V) return ORBX_ENOMEM;
  V->device = hip_device;
  V->k = k;
  V->L = L;
  V->scoring = scoring;
  V->weighting = weighting;
  const int rc = build_vocabulary(V, n_nodes, parent, is_leaf, desc, weight);
  if (rc) {
    delete V;
    return rc;
  }
  *out = V;
  return ORBX_OK;
}

int orbx_vocabulary_load_text(const char* path, int32_t hip_device, orbx_vocabulary** out) {
  ORBX_RESOURCE_LOCK;
  if (!path || !out) return ORBX_EINVAL;
  *out = nullptr;
  FILE* f = fopen(path, "r");
  if (!f) return ORBX_EINVAL;
  std::string line;
  char buf[4096];
  auto getline = [&](std::string& s) -> bool {
    s.clear();
    while (fgets(buf, sizeof(buf), f)) {
      s += buf;
      if (!s.empty() && s.back() == '\n') return true;
    }
    return !s.empty();
  };
  int k = -1, L = -1, n1 = -1, n2 = -1;
  if (!getline(line) || sscanf(line.c_str(), "%d %d %d %d", &k, &L, &n1, &n2) != 4) {
    fclose(f);
    return ORBX_EINVAL;
  }
  if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3) {
    fclose(f);
    return ORBX_EINVAL;
  }
  std::vector<int32_t> parent;
  std::vector<uint8_t> leaf, desc;
  std::vector<double> weight;
  while (getline(line)) {
    if (line.find_first_not_of(" \t\r\n") == std::string::npos) continue;
    int pid, lf;
    uint8_t d[32];
    double w;
    if (!parse_node_line(line.c_str(), &pid, &lf, d, &w)) {
      fclose(f);
      return ORBX_EINVAL;
    }
    parent.push_back(pid);
    leaf.push_back(lf > 0);
    desc.insert(desc.end(), d, d + 32);
    weight.push_back(w);
  }
  fclose(f);
  return orbx_vocabulary_create(k, L, n1, n2, (int32_t)parent.size(), parent.data(),
                                leaf.data(), desc.data(), weight.data(), hip_device, out);
}

int orbx_vocabulary_destroy(orbx_vocabulary* voc) {
  ORBX_RESOURCE_LOCK;
  delete voc;
  return ORBX_OK;
}

int orbx_vocabulary_info(const orbx_vocabulary* V, int32_t* k, int32_t* L, int32_t* scoring,
                         int32_t* weighting, int32_t* n_nodes, int32_t* n_words) {
  if (!V) return ORBX_EINVAL;
  if (k) *k = V->k;
  if (L) *L = V->L;
  if (scoring) *scoring = V->scoring;
  if (weighting) *weighting = V->weighting;
  if (n_nodes) *n_nodes = V->n_nodes;
  if (n_words) *n_words = V->n_words;
  return ORBX_OK;
}

}  // extern "C"

namespace {

// Frame::ComputeBoW of the per-frame chain on the frame cache (orbx_match.h): the descriptors are
// read by k_voc_transform from the thread's pinned stager and copied into the frame's entry as
// they are read (a frame seen before reads them from HBM), the FeatureVector is written into the
// entry for the matchers that follow, and every output the caller wants is written by the kernels
// into the pinned stager as well: no copy kernel.  ORBX_EUNSUPPORTED: the staged path applies.
int transform_resident(const orbx_vocabulary* V, const VocView& view, const VocRanks* R,
                       const uint8_t* desc, int n, int levelsup, uint32_t* word_of,
                       uint32_t* node_of, uint32_t* bow_words, double* bow_values, int32_t* bow_n,
                       uint32_t* fv_node_ids, int32_t* fv_offsets, int32_t* fv_feats,
                       int32_t* fv_n) {
  if (n <= 0 || n > 4096 || !res_enabled()) return ORBX_EUNSUPPORTED;
  bool hit = false;
  ResEntry* e = res_acquire(n, desc, &hit);
  if (!e) return ORBX_EUNSUPPORTED;
  struct Guard {
    ResEntry* e;
    bool ok = false, fill = false;
    ~Guard() {
      if (fill && !ok) res_invalidate(e);
      res_release(e);
    }
  } g{e};
  g.fill = !hit;
  // the FeatureVector goes into the entry when no other call can be reading it there
  const bool own_fv = !hit || res_exclusive_without_fv(e);
  const int nn = std::max(n, 1);
  Stager st;
  const size_t od = hit ? (size_t)-1 : st.add(desc, (size_t)n * 32);
  const size_t ohw = word_of ? st.add(nullptr, (size_t)nn * 4) : (size_t)-1;
  const size_t ohn = node_of ? st.add(nullptr, (size_t)nn * 4) : (size_t)-1;
  const size_t obw = st.add(nullptr, (size_t)nn * 4), obv = st.add(nullptr, (size_t)nn * 8),
               obn = st.add(nullptr, 4), ofi = st.add(nullptr, (size_t)nn * 4),
               ofo = st.add(nullptr, ((size_t)nn + 1) * 4), off = st.add(nullptr, (size_t)nn * 4),
               ofn = st.add(nullptr, 4);
  if (!st.host.pinned) return ORBX_EUNSUPPORTED;
  char* hb = st.host.data();
  // device scratch: word, rank, weight per feature, the BowVector and, when the entry's is
  // not ours to write, the FeatureVector
  const size_t dw = 0, dr = dw + (size_t)nn * 4, dwt = (dr + (size_t)nn * 4 + 15) & ~size_t(15),
               dbw = dwt + (size_t)nn * 8, dbv = (dbw + (size_t)nn * 4 + 15) & ~size_t(15),
               dbn = dbv + (size_t)nn * 8, dfi = dbn + 16, dfo = dfi + (size_t)nn * 4,
               dff = dfo + ((size_t)nn + 1) * 4 + 12, dfn = dff + (size_t)nn * 4, dend = dfn + 16;
  int rc = tls_ws.reserve(dend);
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  VocHostOut ho{};
  ho.desc_copy = hit ? nullptr : e->d_desc();
  ho.word_of = ohw == (size_t)-1 ? nullptr : (uint32_t*)(hb + ohw);
  ho.node_of = ohn == (size_t)-1 ? nullptr : (uint32_t*)(hb + ohn);
  rc = launch_voc_transform(view, V->L - levelsup, R->d_rank_of_node,
                            hit ? e->d_desc() : (const uint8_t*)(hb + od), 0, nullptr, n, n,
                            dptr<uint32_t>(base, dw), dptr<uint32_t>(base, dr), nullptr,
                            dptr<double>(base, dwt), 0, 1, s, ho);
  if (rc) return rc;
  VocHostOut hb2{};
  hb2.words = (uint32_t*)(hb + obw);
  hb2.values = (double*)(hb + obv);
  hb2.nwords = (int*)(hb + obn);
  hb2.ids = (uint32_t*)(hb + ofi);
  hb2.off = (int*)(hb + ofo);
  hb2.feats = (int*)(hb + off);
  hb2.nn = (int*)(hb + ofn);
  rc = launch_bowfv(V->scoring, V->weighting, V->n_words, dptr<uint32_t>(base, dw),
                    dptr<uint32_t>(base, dr), dptr<double>(base, dwt), 0, nullptr, n, n,
                    dptr<uint32_t>(base, dbw), dptr<double>(base, dbv), 0, dptr<int>(base, dbn),
                    R->nb, R->d_rank_ids, own_fv ? e->d_ids() : dptr<uint32_t>(base, dfi),
                    own_fv ? e->d_off() : dptr<int>(base, dfo),
                    own_fv ? e->d_feats() : dptr<int>(base, dff), 0, dptr<int>(base, dfn), 1, s,
                    hb2);
  if (rc == ORBX_EUNSUPPORTED) {  // the descriptor copy may be in flight: let it land
    ORBX_HIP(orbx::wait_stream(s));
    return ORBX_EUNSUPPORTED;
  }
  if (rc) return rc;
  ORBX_HIP(orbx::wait_stream(s));
  const int nb = *(const int*)(hb + obn), nf = *(const int*)(hb + ofn);
  memcpy(bow_words, hb + obw, (size_t)nb * 4);
  memcpy(bow_values, hb + obv, (size_t)nb * 8);
  *bow_n = nb;
  memcpy(fv_node_ids, hb + ofi, (size_t)nf * 4);
  memcpy(fv_offsets, hb + ofo, ((size_t)nf + 1) * 4);
  const int nfeat = ((const int*)(hb + ofo))[nf];
  memcpy(fv_feats, hb + off, (size_t)nfeat * 4);
  *fv_n = nf;
  if (word_of) memcpy(word_of, hb + ohw, (size_t)n * 4);
  if (node_of) memcpy(node_of, hb + ohn, (size_t)n * 4);
  orbx_featvec fv{nf, fv_node_ids, fv_offsets, fv_feats};
  res_mark_filled(e, !hit, own_fv ? &fv : nullptr, nullptr);
  g.ok = true;
  return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_vocabulary_transform(const orbx_vocabulary* V, const uint8_t* desc, int32_t n,
                              int32_t levelsup, uint32_t* word_of, uint32_t* node_of,
                              uint32_t* bow_words, double* bow_values, int32_t* bow_n,
                              uint32_t* fv_node_ids, int32_t* fv_offsets, int32_t* fv_feats,
                              int32_t* fv_n) {
  if (!V || n < 0 || (n && !desc) || !bow_words || !bow_values || !bow_n || !fv_node_ids ||
      !fv_offsets || !fv_feats || !fv_n)
    return ORBX_EINVAL;
  if (n > 8192) return ORBX_EUNSUPPORTED;
  const VocRanks* R = nullptr;
  int rc = vocab_ranks(V, levelsup, &R);
  if (rc) return rc;
  if (R->nb > 8192) return ORBX_EUNSUPPORTED;  // k_csr buckets live in LDS
  VocView view;
  vocab_view(V, &view, nullptr);
  {
    const int rr = transform_resident(V, view, R, desc, n, levelsup, word_of, node_of, bow_words,
                                      bow_values, bow_n, fv_node_ids, fv_offsets, fv_feats, fv_n);
    if (rr != ORBX_EUNSUPPORTED) return rr;
  }
  const int nn = std::max(n, 1);
  Stager st;
  const size_t od = st.add(desc, (size_t)n * 32);
  const size_t upload = st.host.size();
  const size_t ow = st.add(nullptr, (size_t)nn * 4), orank = st.add(nullptr, (size_t)nn * 4),
               onode = st.add(nullptr, (size_t)nn * 4),
               owt = st.add(nullptr, (size_t)nn * 8), obw = st.add(nullptr, (size_t)nn * 4),
               obv = st.add(nullptr, (size_t)nn * 8), obn = st.add(nullptr, 4),
               ofi = st.add(nullptr, (size_t)R->nb * 4),
               ofo = st.add(nullptr, ((size_t)R->nb + 1) * 4), off = st.add(nullptr, (size_t)nn * 4),
               ofn = st.add(nullptr, 4);
  rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  if (upload) ORBX_HIP(tls_ws.upload(st.host, upload));
  if (n > 0) {
    rc = launch_voc_transform(view, V->L - levelsup, R->d_rank_of_node, dptr<uint8_t>(base, od),
                              0, nullptr, n, n, dptr<uint32_t>(base, ow),
                              dptr<uint32_t>(base, orank), dptr<uint32_t>(base, onode),
                              dptr<double>(base, owt), 0, 1, s);
    if (rc) return rc;
  }
  rc = launch_bowfv(V->scoring, V->weighting, V->n_words, dptr<uint32_t>(base, ow),
                    dptr<uint32_t>(base, orank), dptr<double>(base, owt), 0, nullptr, n, n,
                    dptr<uint32_t>(base, obw), dptr<double>(base, obv), 0, dptr<int>(base, obn),
                    R->nb, R->d_rank_ids, dptr<uint32_t>(base, ofi), dptr<int>(base, ofo),
                    dptr<int>(base, off), 0, dptr<int>(base, ofn), 1, s);
  if (rc == ORBX_EUNSUPPORTED) {
    rc = launch_bowvec(V->scoring, V->weighting, dptr<uint32_t>(base, ow),
                       dptr<double>(base, owt), 0, nullptr, n, n, dptr<uint32_t>(base, obw),
                       dptr<double>(base, obv), 0, dptr<int>(base, obn), 1, s);
    if (rc) return rc;
    rc = launch_csr(dptr<uint32_t>(base, orank), 0, nullptr, n, 0, std::max(R->nb, 1),
                    R->d_rank_ids, dptr<uint32_t>(base, ofi), dptr<int>(base, ofo),
                    dptr<int>(base, off), 0, dptr<int>(base, ofn), 1, s);
  }
  if (rc) return rc;
  ORBX_HIP(tls_ws.download(ow, st.host.size() - ow));
  ORBX_HIP(orbx::wait_stream(s));
  auto at = [&](size_t o) { return (const char*)tls_ws.h + o; };
  const int nb = *(const int*)at(obn), nf = *(const int*)at(ofn);
  memcpy(bow_words, at(obw), (size_t)nb * 4);
  memcpy(bow_values, at(obv), (size_t)nb * 8);
  *bow_n = nb;
  memcpy(fv_node_ids, at(ofi), (size_t)nf * 4);
  memcpy(fv_offsets, at(ofo), ((size_t)nf + 1) * 4);
  const int nfeat = ((const int*)at(ofo))[nf];
  memcpy(fv_feats, at(off), (size_t)nfeat * 4);
  *fv_n = nf;
  if (word_of && n) memcpy(word_of, at(ow), (size_t)n * 4);
  if (node_of && n) memcpy(node_of, at(onode), (size_t)n * 4);
  return ORBX_OK;
}

}  // extern "C"
