// orbx_match.hip — gfx950 kernels for ORBmatcher::SearchByBoW (both overloads),
// SearchForTriangulation, DescriptorDistance and the DBoW2 node-id transform feeding them.
//
//   k_bow_nodes   one wave per keyframe vocabulary node; KF features in node order, the node's
//                 candidate features across lanes (popcount over 4 x u64), wave min/second-min
//                 reduction (ORBmatcher.cc:187-250 / 557-622)
//   k_bow_finish  one workgroup per problem: rotation histogram, ComputeThreeMaxima, filter
//                 (ORBmatcher.cc:267-285 / 637-655, 1604-1645)
//   k_tri_nodes   one wave per KF1 node, one lane per KF1 feature (ORBmatcher.cc:694-792)
//   k_tri_finish  rotation filter + ordered (idx1 ascending) pair compaction (:794-823)
//   k_csr         FeatureVector build: stable bucket sort of feature indices by node id
//                 (FeatureVector.cpp:31-45)
#include <atomic>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "orbx_internal.h"
#include "orbx_match.h"

#pragma clang fp contract(off)

namespace orbx {

constexpr int kTH_LOW = 50;
constexpr int kHISTO = 30;

__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
  const uint64_t* pa = (const uint64_t*)a;
  const uint64_t* pb = (const uint64_t*)b;
  return __popcll(pa[0] ^ pb[0]) + __popcll(pa[1] ^ pb[1]) + __popcll(pa[2] ^ pb[2]) +
         __popcll(pa[3] ^ pb[3]);
}

__device__ __forceinline__ int hamming_regs(const uint64_t d[4], const uint8_t* b) {
  const uint64_t* pb = (const uint64_t*)b;
  return __popcll(d[0] ^ pb[0]) + __popcll(d[1] ^ pb[1]) + __popcll(d[2] ^ pb[2]) +
         __popcll(d[3] ^ pb[3]);
}

// std::lower_bound over a sorted array by the whole wave (wave-uniform arguments): each round
// probes up to 64 evenly spaced positions at once, so a node lookup costs 2-3 dependent loads
// instead of log2(n)
__device__ __forceinline__ int wave_lower_bound(const uint32_t* a, int n, uint32_t v, int lane) {
  int lo = 0, len = n;
  while (len > 64) {
    const int step = (len + 63) >> 6;
    const int K = (len + step - 1) / step;  // probes lo, lo + step, ... (K <= 64)
    const int c = __popcll(__ballot(lane < K && a[lo + lane * step] < v));
    if (c == 0) return lo;
    const int pc1 = lo + (c - 1) * step;  // a[pc1] < v
    const int hi = c < K ? lo + c * step : lo + len;  // a[hi] >= v, or the end
    lo = pc1 + 1;
    len = hi - lo;
  }
  return lo + __popcll(__ballot(lane < len && a[lo + lane] < v));
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {
  const float factor = 1.0f / kHISTO;
  float rot = a1 - a2;
  if (rot < 0.0) rot += 360.0f;
  int bin = (int)roundf(rot * factor);
  if (bin == kHISTO) bin = 0;
  return bin;
}

__device__ __forceinline__ void bow_finish(const BowProblem* __restrict__ probs, const int pi);
__device__ __forceinline__ void tri_finish(const TriProblem* __restrict__ probs, const int pi);
__device__ __forceinline__ bool last_workgroup(int* done);

// ------------------------------------------------------------------ SearchByBoW
// One wave per KF node a of problem pi (every lane of the wave active; the problem read through
// the kernel's __restrict__ pointer, so its fields stay in scalar registers across the stores)
template <int CH>
__device__ __forceinline__ void bow_node_wave(const BowProblem* __restrict__ probs, const int pi,
                                              const int a, const int lane) {
  const BowProblem& P = probs[pi];
  if (a >= side_nodes(P.s1)) return;
  const uint32_t id = P.s1.node_ids[a];
  // the KF node's first 64 features (index, validity, descriptor: one round of loads) are in
  // flight during the frame node lookup
  const int a0 = P.s1.node_offsets[a], a1 = P.s1.node_offsets[a + 1];
  int i1_l = -1;
  bool ok_l = false;
  uint64_t dl0 = 0, dl1 = 0, dl2 = 0, dl3 = 0;
  auto load_kf = [&](int c0) {
    const int my = c0 + lane;
    i1_l = -1;
    ok_l = false;
    dl0 = dl1 = dl2 = dl3 = 0;
    if (my < a1) {
      i1_l = P.s1.node_feats[my];
      ok_l = !P.s1.valid || P.s1.valid[i1_l];
      const uint64_t* q = (const uint64_t*)(P.s1.desc + (int64_t)i1_l * 32);
      dl0 = q[0]; dl1 = q[1]; dl2 = q[2]; dl3 = q[3];
    }
  };
  load_kf(a0);
  const int nn2 = side_nodes(P.s2);
  const int b = wave_lower_bound(P.s2.node_ids, nn2, id, lane);
  if (b >= nn2 || P.s2.node_ids[b] != id) return;
  const int f0 = P.s2.node_offsets[b], m = P.s2.node_offsets[b + 1] - f0;
  const bool kfkf = P.mode == 1;
  // vbMatched2 / vpMapPointMatches[realIdxF] (ORBmatcher.cc:215-216, 598-599): a feature
  // belongs to one node, so only this wave reads or sets the flags of the node's candidates.
  // Up to kBowRegCands candidates they live in a register bitmap (bit c of lane l: candidate
  // l + 64c); larger nodes (no limit in the reference) keep them in memory: mode 0 reads the
  // output itself (match[i2] >= 0), mode 1 the zeroed matched2 flags.
  const bool big = m > kBowRegCands;
  // the candidates of chunks 0 .. CH-1 (positions lane + 64 c) stay in registers
  // for the whole node: descriptor, index and validity (bit c of okr); later chunks of a larger
  // node are read from memory per KF feature
  uint64_t reg[CH][4];
  int i2r[CH];
  uint32_t okr = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) {
    const int jj = lane + 64 * c;
    reg[c][0] = reg[c][1] = reg[c][2] = reg[c][3] = 0;
    i2r[c] = -1;
    if (jj < m) {
      const int i2 = P.s2.node_feats[f0 + jj];
      const uint64_t* p = (const uint64_t*)(P.s2.desc + (int64_t)i2 * 32);
      reg[c][0] = p[0]; reg[c][1] = p[1]; reg[c][2] = p[2]; reg[c][3] = p[3];
      i2r[c] = i2;
      if (!kfkf || !P.s2.valid || P.s2.valid[i2]) okr |= 1u << c;
    }
  }
  uint64_t matched = 0;  // bit c: candidate lane + 64c already matched in this call
  // Without `big`, the matches of register candidates are stored after the loops (a global
  // store inside the serial per-feature loop made the next feature wait for its completion):
  // mode 0 keeps the KF feature matched to candidate lane + 64 c in mval[c] of the candidate's
  // lane, mode 1 the candidate index matched to a prefetched KF feature in res_l of its lane
  int mval[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) mval[c] = -1;
  for (int c0 = a0; c0 < a1; c0 += 64) {
    // up to 64 KF features of the node (index, validity, descriptor) in registers, so the
    // serial per-feature loop below only shuffles registers
    if (c0 != a0) load_kf(c0);
    int res_l = -1;
    uint64_t okm = __ballot(ok_l);
    while (okm) {
      const int j = __builtin_ctzll(okm);
      okm &= okm - 1;
      const int i1 = __shfl(i1_l, j);
      const uint64_t d1[4] = {(uint64_t)__shfl((long long)dl0, j), (uint64_t)__shfl((long long)dl1, j),
                              (uint64_t)__shfl((long long)dl2, j), (uint64_t)__shfl((long long)dl3, j)};
      int b1 = 256, bp = 0x7FFFFFFF, b2 = 256;
      // candidates in position order (lane + 64 c ascending per lane): strict < keeps the first
      auto offer = [&](int dist, int jj) {
        if (dist < b1) {
          b2 = b1;
          b1 = dist;
          bp = jj;
        } else if (dist < b2) {
          b2 = dist;
        }
      };
#pragma unroll
      for (int c = 0; c < CH; c++) {
        if (c * 64 >= m) break;  // wave-uniform
        const int jj = lane + 64 * c;
        if (!((okr >> c) & 1)) continue;
        if (!big && ((matched >> c) & 1)) continue;
        if (big && (kfkf ? __hip_atomic_load(P.matched2 + i2r[c], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) != 0
                         : __hip_atomic_load(P.match + i2r[c], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) >= 0))
          continue;
        offer(__popcll(d1[0] ^ reg[c][0]) + __popcll(d1[1] ^ reg[c][1]) +
                  __popcll(d1[2] ^ reg[c][2]) + __popcll(d1[3] ^ reg[c][3]), jj);
      }
      for (int c = CH; c * 64 < m; c++) {
        const int jj = lane + 64 * c;
        if (jj >= m) continue;
        if (!big && ((matched >> c) & 1)) continue;
        const int i2 = P.s2.node_feats[f0 + jj];
        if (big && (kfkf ? __hip_atomic_load(P.matched2 + i2, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) != 0
                         : __hip_atomic_load(P.match + i2, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) >= 0))
          continue;
        if (kfkf && P.s2.valid && !P.s2.valid[i2]) continue;
        offer(hamming_regs(d1, P.s2.desc + (int64_t)i2 * 32), jj);
      }
      // wave merge of (best1, position, best2), what the sequential loop yields: the minimum
      // of the key (best1 << 23 | position) is best1 at its first position; best2 is then the
      // minimum over the lanes of best1, except the winning lane, which offers its own best2.
      // best1 <= 256 takes 9 bits, a position < kBowMaxSide2 the other 23 (the host entry
      // points reject larger sides; a lane without a candidate offers position 0x7FFFFF)
      {
        const uint32_t key = ((uint32_t)b1 << 23) | (uint32_t)min(bp, kBowPosMask);
        const uint32_t K = wave_min_u32(key);
        const int B2 = (int)wave_min_u32(key == K ? (uint32_t)b2 : (uint32_t)b1);
        b1 = (int)(K >> 23);
        bp = (int)(K & (uint32_t)kBowPosMask);
        b2 = B2;
      }
      const bool pass = kfkf ? b1 < kTH_LOW : b1 <= kTH_LOW;
      if (pass && static_cast<float>(b1) < P.nnratio * static_cast<float>(b2)) {
        const int cb = bp >> 6, lb = bp & 63;  // wave-uniform
        if (lb == lane) matched |= 1ull << cb;
        if (big) {
          if (lane == 0) {
            const int i2 = P.s2.node_feats[f0 + bp];
            if (kfkf) {
              P.match[i1] = i2;
              __hip_atomic_store(P.matched2 + i2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              __hip_atomic_store(P.match + i2, i1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
          // the flag store completes before the next feature's scan reads it
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        } else if (cb < CH) {
          if (kfkf) {
            int i2c = i2r[0];
#pragma unroll
            for (int c = 1; c < CH; c++) i2c = cb == c ? i2r[c] : i2c;
            const int i2 = __builtin_amdgcn_readlane(i2c, lb);
            if (lane == j) res_l = i2;
          } else if (lane == lb) {
#pragma unroll
            for (int c = 0; c < CH; c++) mval[c] = cb == c ? i1 : mval[c];
          }
        } else if (lane == lb) {  // a candidate past the register chunks: stored now
          const int i2 = P.s2.node_feats[f0 + bp];
          if (kfkf) P.match[i1] = i2;
          else P.match[i2] = i1;
        }
      }
    }
    if (res_l >= 0) P.match[i1_l] = res_l;
  }
#pragma unroll
  for (int c = 0; c < CH; c++)
    if (mval[c] >= 0) P.match[i2r[c]] = mval[c];
}

// CH candidate chunks of 64 in registers: kBowDescChunks (2), or 4 for frames whose vocabulary
// nodes hold many features (C5's 4,000 per frame: 0.62 -> 0.52 ms per 256 frames; at C2's 1,000
// the extra registers cost occupancy: 0.113 -> 0.138 ms)
template <int CH>
__global__ __launch_bounds__(256) void k_bow_nodes(const BowProblem* __restrict__ probs) {
  bow_node_wave<CH>(probs, blockIdx.y, blockIdx.x * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
}

// Latency form of k_bow_nodes for calls with few problems (the per-frame drop-in call), where
// one wave per node leaves the GPU idle behind the node with the longest serial loop: one
// workgroup per KF node of at most kBwgCands candidates, and no serial loop.  The greedy scan
// (each KF feature in node order takes its best candidate not matched by an earlier one,
// ORBmatcher.cc:187-250 / 557-622) is solved as a triangular fixed point:
//  (1) every KF feature's kBwgK smallest (distance << 8 | position) keys over all candidates,
//      the candidates split over the four waves (partial lists merged by wave 0), distances
//      kept in LDS;
//  (2) wave 0 (lane = KF feature) repeats "take the first two keys of my list whose candidate
//      no lower lane claims" until no lane's claim changes.  Feature k's outcome depends only on
//      the claims of features < k, so iteration t settles features < t and the fixed point is
//      the sequential result; a feature whose list runs out of unclaimed keys while more valid
//      candidates exist rescans its distance row.
constexpr int kBwgCands = 128;  // claim masks: two u64
constexpr int kBwgK = 8;
constexpr uint32_t kBwgSent = 0xFFFFFFFFu;

__device__ __forceinline__ void topk_insert(uint32_t (&L)[kBwgK], uint32_t key) {
#pragma unroll
  for (int q = 0; q < kBwgK; q++) {
    const uint32_t lo = min(L[q], key);
    key = max(L[q], key);
    L[q] = lo;
  }
}

__device__ __forceinline__ uint32_t wave_or_excl(uint32_t u) {  // OR over the lanes below
  u |= dpp0<0x111, 0xF, true>(u);   // row_shr:1
  u |= dpp0<0x112, 0xF, true>(u);   // row_shr:2
  u |= dpp0<0x114, 0xF, true>(u);   // row_shr:4
  u |= dpp0<0x118, 0xF, true>(u);   // row_shr:8
  u |= dpp0<0x142, 0xA, false>(u);  // row_bcast:15
  u |= dpp0<0x143, 0xC, false>(u);  // row_bcast:31
  const int lane = threadIdx.x & 63;
  const uint32_t below = (uint32_t)__shfl((int)u, lane > 0 ? lane - 1 : 0);
  return lane > 0 ? below : 0u;
}

__device__ __forceinline__ uint64_t wave_or_all64(uint64_t v) {  // OR over the wave
  const uint32_t lo = wave_or_excl((uint32_t)v) | (uint32_t)v;
  const uint32_t hi = wave_or_excl((uint32_t)(v >> 32)) | (uint32_t)(v >> 32);
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, 63) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32);
}

__device__ __forceinline__ bool claimed(uint64_t m0, uint64_t m1, int pos) {
  return ((pos < 64 ? m0 >> pos : m1 >> (pos - 64)) & 1) != 0;
}

__device__ __forceinline__ void bow_nodes_wg(const BowProblem* __restrict__ probs, const int pi) {
  const BowProblem& P = probs[pi];
  const int a = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (a >= side_nodes(P.s1)) return;
  __shared__ uint64_t s_cd[kBwgCands][4];
  __shared__ int s_ci2[kBwgCands];
  __shared__ uint16_t s_dist[64][kBwgCands + 2];  // odd dword row stride
  __shared__ uint32_t s_list[4][kBwgK][64];
  __shared__ int s_b, s_nv;
  const uint32_t id = P.s1.node_ids[a];
  if (tid < 64) {
    const int nn2 = side_nodes(P.s2);
    const int b = wave_lower_bound(P.s2.node_ids, nn2, id, lane);
    if (lane == 0) s_b = b < nn2 && P.s2.node_ids[b] == id ? b : -1;
  }
  __syncthreads();
  const int b = s_b;
  if (b < 0) return;  // workgroup-uniform
  const int f0 = P.s2.node_offsets[b], m = P.s2.node_offsets[b + 1] - f0;
  if (m > kBwgCands) {  // the wave form (no candidate limit)
    if (wid == 0) bow_node_wave<kBowDescChunks>(probs, pi, a, lane);
    return;
  }
  const bool kfkf = P.mode == 1;
  if (tid < 64) {  // candidates: descriptor, index, validity (mode 1: pMP2 of KF2)
    int nv = 0;
    for (int j0 = 0; j0 < m; j0 += 64) {
      const int j = j0 + lane;
      int i2 = -1;
      if (j < m) {
        i2 = P.s2.node_feats[f0 + j];
        const uint64_t* q = (const uint64_t*)(P.s2.desc + (int64_t)i2 * 32);
        s_cd[j][0] = q[0];
        s_cd[j][1] = q[1];
        s_cd[j][2] = q[2];
        s_cd[j][3] = q[3];
        if (kfkf && P.s2.valid && !P.s2.valid[i2]) i2 = -1;
        s_ci2[j] = i2;
      }
      nv += __popcll(__ballot(i2 >= 0));
    }
    if (lane == 0) s_nv = nv;
  }
  __syncthreads();
  const int nv = s_nv;
  const int mq = (m + 3) >> 2, jb = wid * mq, je = min(m, jb + mq);
  uint64_t M0 = 0, M1 = 0;  // candidates claimed by earlier chunks (wave 0)
  const int a0 = P.s1.node_offsets[a], a1 = P.s1.node_offsets[a + 1];
  for (int c0 = a0; c0 < a1; c0 += 64) {
    const int k = c0 + lane;
    int i1 = -1;
    bool ok1 = false;
    uint64_t d1[4] = {0, 0, 0, 0};
    if (k < a1) {
      i1 = P.s1.node_feats[k];
      ok1 = !P.s1.valid || P.s1.valid[i1];
      if (ok1) {
        const uint64_t* q = (const uint64_t*)(P.s1.desc + (int64_t)i1 * 32);
        d1[0] = q[0]; d1[1] = q[1]; d1[2] = q[2]; d1[3] = q[3];
      }
    }
    uint32_t L[kBwgK];
#pragma unroll
    for (int q = 0; q < kBwgK; q++) L[q] = kBwgSent;
    for (int j = jb; j < je; j++) {  // this wave's quarter, in position order
      if (s_ci2[j] < 0) continue;    // uniform
      const int d = __popcll(d1[0] ^ s_cd[j][0]) + __popcll(d1[1] ^ s_cd[j][1]) +
                    __popcll(d1[2] ^ s_cd[j][2]) + __popcll(d1[3] ^ s_cd[j][3]);
      s_dist[lane][j] = (uint16_t)d;
      topk_insert(L, ((uint32_t)d << 8) | (uint32_t)j);
    }
#pragma unroll
    for (int q = 0; q < kBwgK; q++) s_list[wid][q][lane] = L[q];
    __syncthreads();
    if (wid == 0) {
      for (int w = 1; w < 4; w++) {  // merge the other waves' lists (sorted: stop at the first miss)
        for (int q = 0; q < kBwgK; q++) {
          const uint32_t e = s_list[w][q][lane];
          if (e >= L[kBwgK - 1]) break;
          topk_insert(L, e);
        }
      }
      const bool more = nv > kBwgK;  // the lists may not hold every valid candidate
      int out = -1;
      for (;;) {
        const uint64_t mine0 = out >= 0 && out < 64 ? 1ull << out : 0ull;
        const uint64_t mine1 = out >= 64 ? 1ull << (out - 64) : 0ull;
        const uint64_t E0 = M0 | wave_or_excl((uint32_t)mine0) |
                            ((uint64_t)wave_or_excl((uint32_t)(mine0 >> 32)) << 32);
        const uint64_t E1 = M1 | wave_or_excl((uint32_t)mine1) |
                            ((uint64_t)wave_or_excl((uint32_t)(mine1 >> 32)) << 32);
        int nout = -1;
        if (ok1) {
          int b1 = 256, bp = -1, b2 = 256, found = 0;
#pragma unroll
          for (int q = 0; q < kBwgK; q++) {
            const uint32_t e = L[q];
            if (found == 2 || e == kBwgSent) continue;
            const int pos = (int)(e & 0xFF);
            if (claimed(E0, E1, pos)) continue;
            if (found == 0) {
              b1 = (int)(e >> 8);
              bp = pos;
            } else {
              b2 = (int)(e >> 8);
            }
            found++;
          }
          if (found < 2 && more) {  // the next unclaimed key lies past the list: the whole row
            b1 = 256, bp = -1, b2 = 256;
            for (int j = 0; j < m; j++) {
              if (s_ci2[j] < 0 || claimed(E0, E1, j)) continue;
              const int d = s_dist[lane][j];
              if (d < b1) {
                b2 = b1;
                b1 = d;
                bp = j;
              } else if (d < b2) {
                b2 = d;
              }
            }
          }
          const bool pass = kfkf ? b1 < kTH_LOW : b1 <= kTH_LOW;
          if (bp >= 0 && pass && static_cast<float>(b1) < P.nnratio * static_cast<float>(b2))
            nout = bp;
        }
        const bool changed = __ballot(nout != out) != 0;
        out = nout;
        if (!changed) break;
      }
      if (out >= 0) {
        const int i2 = s_ci2[out];
        if (kfkf) P.match[i1] = i2;
        else P.match[i2] = i1;
      }
      M0 |= wave_or_all64(out >= 0 && out < 64 ? 1ull << out : 0ull);
      M1 |= wave_or_all64(out >= 64 ? 1ull << (out - 64) : 0ull);
    }
    __syncthreads();  // s_list / s_dist are rewritten by the next chunk
  }
}

// The workgroup's problem into LDS: the kernels read its fields throughout, and a resident
// call's problem lives in pinned host memory (one PCIe read per workgroup, not one per use).
template <class T>
__device__ __forceinline__ void stage_problem(T* dst, const T* __restrict__ src) {
  static_assert(sizeof(T) % 4 == 0, "problem in dwords");
  for (int i = threadIdx.x; i < (int)(sizeof(T) / 4); i += blockDim.x)
    ((int*)dst)[i] = ((const int*)src)[i];
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_bow_nodes_wg(const BowProblem* __restrict__ probs) {
  __shared__ BowProblem s_p;
  stage_problem(&s_p, probs + blockIdx.y);
  bow_nodes_wg(&s_p, 0);
  if (s_p.done && last_workgroup(s_p.done)) bow_finish(&s_p, 0);
}

// ComputeThreeMaxima (ORBmatcher.cc:1604-1645)
__device__ void three_maxima(const int* h, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  ind1 = ind2 = ind3 = -1;
  for (int i = 0; i < kHISTO; i++) {
    const int s = h[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      ind3 = ind2; ind2 = ind1; ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      ind3 = ind2; ind2 = i;
    } else if (s > max3) {
      max3 = s;
      ind3 = i;
    }
  }
  if (max2 < 0.1f * (float)max1) {
    ind2 = -1;
    ind3 = -1;
  } else if (max3 < 0.1f * (float)max1) {
    ind3 = -1;
  }
}

// Rotation consistency filter + count.  Entries: mode 0 indexed by F feature (value = KF idx),
// mode 1 / triangulation indexed by side-1 feature (value = side-2 idx).
constexpr int kFinishRegs = 8;  // entries per thread per gather round (n <= 2048: one round)

__device__ __forceinline__ void bow_finish(const BowProblem* __restrict__ probs, const int pi) {
  const BowProblem& P = probs[pi];
  __shared__ int hist[kHISTO];
  __shared__ int s_ind[3];
  __shared__ int s_cnt;
  const int tid = threadIdx.x;
  if (tid < kHISTO) hist[tid] = 0;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  const bool kfkf = P.mode == 1;
  const int n = kfkf ? side_n(P.s1) : side_n(P.s2);
  const int n_other = kfkf ? side_n(P.s2) : side_n(P.s1);  // range of a match value
  const bool ori = P.check_ori;
  // entries i0 + tid + 256 r (r < kFinishRegs): the matches, then the angle pairs, each with
  // every load of the round in flight (the stores of dropped entries come after the loads:
  // between them they kept the compiler from batching the angle loads)
  int m[kFinishRegs], bin[kFinishRegs];
  auto gather = [&](int i0) {
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) {
      const int i = i0 + tid + 256 * r;
      m[r] = i < n ? P.match[i] : -1;
    }
    uint32_t bad = 0;
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) {
      if (m[r] >= n_other) {  // stale or corrupt index: report, drop, never dereference
        bad |= 1u << r;
        m[r] = -1;
      }
    }
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) {
      const int i = i0 + tid + 256 * r;
      bin[r] = -1;
      if (ori && m[r] >= 0)
        bin[r] = kfkf ? rot_bin(side_angle(P.s1, i), side_angle(P.s2, m[r]))
                      : rot_bin(side_angle(P.s1, m[r]), side_angle(P.s2, i));
    }
    if (bad) {
      atomicOr(P.error, ORBX_DEVERR_INDEX);
#pragma unroll
      for (int r = 0; r < kFinishRegs; r++)
        if ((bad >> r) & 1) P.match[i0 + tid + 256 * r] = -1;
    }
  };
  auto filter = [&](int i0) {  // after ComputeThreeMaxima: drop the other bins, count the rest
    int c = 0;
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) {
      if (m[r] < 0) continue;
      if (ori && bin[r] != s_ind[0] && bin[r] != s_ind[1] && bin[r] != s_ind[2]) {
        P.match[i0 + tid + 256 * r] = -1;
        continue;
      }
      c++;
    }
    return c;
  };
  const bool one_round = n <= 256 * kFinishRegs;
  for (int i0 = 0; i0 < n || i0 == 0; i0 += 256 * kFinishRegs) {
    gather(i0);
    if (ori) {
#pragma unroll
      for (int r = 0; r < kFinishRegs; r++)
        if (bin[r] >= 0) atomicAdd(&hist[bin[r]], 1);
    }
    if (one_round) break;
  }
  if (ori) {
    __syncthreads();
    if (tid == 0) three_maxima(hist, s_ind[0], s_ind[1], s_ind[2]);
    __syncthreads();
  }
  int local = 0;
  if (one_round) {
    local = filter(0);
  } else {
    for (int i0 = 0; i0 < n; i0 += 256 * kFinishRegs) {
      gather(i0);
      local += filter(i0);
    }
  }
  atomicAdd(&s_cnt, local);
  __syncthreads();
  if (tid == 0) *P.count = s_cnt;
  if (P.match_host) {  // a resident call: results to pinned host memory, scratch back to clean
    for (int i = tid; i < n; i += 256) {
      P.match_host[i] = P.match[i];
      P.match[i] = -1;
    }
    if (kfkf && P.matched2)
      for (int i = tid; i < n_other; i += 256) P.matched2[i] = 0;
    if (tid == 0) {
      P.ctrl_host[0] = s_cnt;
      P.ctrl_host[1] = atomicExch(P.error, 0);
      if (P.done) atomicExch(P.done, 0);
    }
  }
}

__global__ __launch_bounds__(256) void k_bow_finish(const BowProblem* __restrict__ probs) {
  __shared__ BowProblem s_p;
  stage_problem(&s_p, probs + blockIdx.x);
  bow_finish(&s_p, 0);
}

// The last workgroup of a node kernel to finish (counted in *done, zeroed by the host) runs the
// problem's finish: one launch fewer on the latency path.  Stores of every workgroup are made
// visible device-wide before its count (release), and read after the last count (acquire).
__device__ __forceinline__ bool last_workgroup(int* done) {
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    s_last = atomicAdd(done, 1) == (int)(gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return false;
  __threadfence();
  return true;
}

// ------------------------------------------------------------------ SearchForTriangulation
// CheckDistEpipolarLine (ORBmatcher.cc:140-157) with the reference binary's FMA pattern
// (SURVEY A.7).
__device__ __forceinline__ bool epipolar_ok(float x1, float y1, float x2, float y2,
                                            const float* F, float sigma2) {
  const float a = __builtin_fmaf(x1, F[0], y1 * F[3]) + F[6];
  const float b = __builtin_fmaf(x1, F[1], y1 * F[4]) + F[7];
  const float c = __builtin_fmaf(y1, F[5], x1 * F[2]) + F[8];
  const float num = __builtin_fmaf(b, y2, x2 * a) + c;
  const float den = __builtin_fmaf(a, a, b * b);
  if (den == 0) return false;
  const float dsqr = num * num / den;
  return (double)dsqr < 3.84 * (double)sigma2;
}

// One wave per KF1 node.  The reference scans the KF2 node's features in order for each KF1
// feature, keeping the last one at the running minimum distance that passes the checks
// (ORBmatcher.cc:716-769): that is the candidate of largest node position among those at the
// minimum passing distance, since a later equal distance replaces and a larger one never does.
// So the scan of one KF1 feature splits over several lanes: with n1 KF1 features in the chunk,
// G = 64 / n1 lanes per feature each scan every G-th staged KF2 feature, keeping the minimum of
// (dist << 32 | ~position), and the G partial minima meet in an LDS atomic minimum.
__global__ __launch_bounds__(256) void k_tri_nodes(const TriProblem* __restrict__ probs) {
  const TriProblem& P = probs[blockIdx.y];
  const int a = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (a >= tri_nodes(P.s1)) return;
  const int wv = threadIdx.x >> 6;
  // KF2 features are staged 64 at a time in this wave's LDS (descriptor, keypoint,
  // stereo/map-point flags); the KF1 features' best keys meet in LDS
  __shared__ uint64_t s_d[4][64][4];
  __shared__ float s_x[4][64], s_y[4][64];
  __shared__ int s_i2[4][64], s_oct[4][64];
  __shared__ unsigned long long s_key[4][64];
  const int a0 = P.s1.fv.node_offsets[a], a1 = P.s1.fv.node_offsets[a + 1];
  // a KF1 chunk: this lane's feature u (every G-th candidate from g), its flags, keypoint and
  // descriptor in one round of loads (all depend on the feature index only)
  int n1, G, u, g, i1;
  bool live, st1;
  orbx_keypoint kp1;
  uint64_t d1[4];
  auto load_kf1 = [&](int pa0) {
    n1 = min(64, a1 - pa0);
    G = 64 / n1;  // lanes per KF1 feature (wave-uniform)
    u = lane % n1;
    g = lane / n1;
    i1 = P.s1.fv.node_feats[pa0 + u];
    const bool hm = P.s1.has_mp && P.s1.has_mp[i1];
    st1 = P.s1.u_right ? P.s1.u_right[i1] >= 0 : false;
    kp1 = P.s1.keys_un[i1];
    const uint64_t* q = (const uint64_t*)(P.s1.desc + (int64_t)i1 * 32);
    d1[0] = q[0]; d1[1] = q[1]; d1[2] = q[2]; d1[3] = q[3];
    live = g < G && !hm && !(P.only_stereo && !st1);
  };
  if (a0 < a1) load_kf1(a0);  // in flight during the KF2 node lookup
  const uint32_t id = P.s1.fv.node_ids[a];
  const int nn2 = tri_nodes(P.s2);
  const int b = wave_lower_bound(P.s2.fv.node_ids, nn2, id, lane);
  if (b >= nn2 || P.s2.fv.node_ids[b] != id) return;
  const int f0 = P.s2.fv.node_offsets[b], f1 = P.s2.fv.node_offsets[b + 1];
  for (int pa0 = a0; pa0 < a1; pa0 += 64) {
    if (pa0 != a0) load_kf1(pa0);
    s_key[wv][lane] = ~0ull;
    unsigned long long best = ~0ull;
    for (int pb0 = f0; pb0 < f1; pb0 += 64) {
      const int nb = min(64, f1 - pb0);
      {  // stage chunk: entry skipped (i2 = -1) when it has a map point or fails only_stereo;
         // the flags, descriptor and keypoint load together
        int i2 = -1;
        if (lane < nb) {
          i2 = P.s2.fv.node_feats[pb0 + lane];
          const bool st2 = P.s2.u_right ? P.s2.u_right[i2] >= 0 : false;
          const bool hm2 = P.s2.has_mp && P.s2.has_mp[i2];
          const uint64_t* q = (const uint64_t*)(P.s2.desc + (int64_t)i2 * 32);
          const uint64_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
          const orbx_keypoint kp2 = P.s2.keys_un[i2];
          // `vbMatched2[idx2] || pMP2` (:728): vbMatched2 is never set in this function
          if (hm2 || (P.only_stereo && !st2)) {
            i2 = -1;
          } else {
            s_d[wv][lane][0] = q0;
            s_d[wv][lane][1] = q1;
            s_d[wv][lane][2] = q2;
            s_d[wv][lane][3] = q3;
            s_x[wv][lane] = kp2.x;
            s_y[wv][lane] = kp2.y;
            s_oct[wv][lane] = kp2.octave | (st2 ? 0x10000 : 0);
          }
        }
        s_i2[wv][lane] = i2;
      }
      __builtin_amdgcn_wave_barrier();  // the chunk's LDS writes precede every lane's reads
      if (live) {
        for (int j = g; j < nb; j += G) {
          if (s_i2[wv][j] < 0) continue;
          const uint64_t* dd = s_d[wv][j];
          const int dist = __popcll(d1[0] ^ dd[0]) + __popcll(d1[1] ^ dd[1]) +
                           __popcll(d1[2] ^ dd[2]) + __popcll(d1[3] ^ dd[3]);
          if (dist > kTH_LOW) continue;
          const unsigned long long key =
              ((unsigned long long)dist << 32) | (uint32_t)~(pb0 - f0 + j);
          if (key > best) continue;  // (dist > bestDist in the reference; equal: later wins)
          const int oc2 = s_oct[wv][j];
          const bool st2 = oc2 >> 16;
          const int oct2 = oc2 & 0xFFFF;
          const float x2 = s_x[wv][j], y2 = s_y[wv][j];
          if (!st1 && !st2) {
            const float dex = P.ex - x2, dey = P.ey - y2;
            if (__builtin_fmaf(dex, dex, dey * dey) < 100 * P.s2.scale_factors[oct2]) continue;
          }
          if (epipolar_ok(kp1.x, kp1.y, x2, y2, P.F, P.s2.level_sigma2[oct2])) best = key;
        }
      }
      __builtin_amdgcn_wave_barrier();  // every lane's reads precede the next chunk's writes
    }
    if (live) atomicMin(&s_key[wv][u], best);
    __builtin_amdgcn_wave_barrier();
    if (lane < n1 && live) {
      const unsigned long long key = s_key[wv][lane];
      P.m12[i1] = key == ~0ull ? -1 : P.s2.fv.node_feats[f0 + (int)~(uint32_t)key];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Latency form of k_tri_nodes for calls with few problems (the per-keyframe-pair drop-in call),
// where one wave per node leaves the GPU idle behind the largest node: one workgroup per KF1
// node, the KF2 node staged 256 features at a time for the whole workgroup and G = 256 / n1
// lanes per KF1 feature, so a node's scan is spread over four times as many lanes.  Same keys,
// same LDS minimum, same result.
__device__ __forceinline__ void tri_nodes_wg(const TriProblem* __restrict__ probs, const int pi) {
  const TriProblem& P = probs[pi];
  const int a = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  if (a >= tri_nodes(P.s1)) return;
  __shared__ uint64_t s_d[256][4];
  __shared__ float s_x[256], s_y[256];
  __shared__ int s_i2[256], s_oct[256];
  __shared__ unsigned long long s_key[64];
  __shared__ int s_b;
  const uint32_t id = P.s1.fv.node_ids[a];
  if (tid < 64) {
    const int nn2 = tri_nodes(P.s2);
    const int b = wave_lower_bound(P.s2.fv.node_ids, nn2, id, lane);
    if (lane == 0) s_b = b < nn2 && P.s2.fv.node_ids[b] == id ? b : -1;
  }
  __syncthreads();
  const int b = s_b;
  if (b < 0) return;  // workgroup-uniform
  const int f0 = P.s2.fv.node_offsets[b], f1 = P.s2.fv.node_offsets[b + 1];
  const int a1 = P.s1.fv.node_offsets[a + 1];
  for (int pa0 = P.s1.fv.node_offsets[a]; pa0 < a1; pa0 += 64) {
    const int n1 = min(64, a1 - pa0);
    const int G = 256 / n1;                    // lanes per KF1 feature
    const int u = tid % n1, g = tid / n1;
    bool live = g < G;
    const int i1 = P.s1.fv.node_feats[pa0 + u];
    bool st1 = false;
    if (live) {
      if (P.s1.has_mp && P.s1.has_mp[i1]) live = false;
      st1 = P.s1.u_right ? P.s1.u_right[i1] >= 0 : false;
      if (P.only_stereo && !st1) live = false;
    }
    orbx_keypoint kp1{};
    uint64_t d1[4] = {0, 0, 0, 0};
    if (live) {
      kp1 = P.s1.keys_un[i1];
      const uint64_t* q = (const uint64_t*)(P.s1.desc + (int64_t)i1 * 32);
      d1[0] = q[0]; d1[1] = q[1]; d1[2] = q[2]; d1[3] = q[3];
    }
    if (tid < 64) s_key[tid] = ~0ull;
    unsigned long long best = ~0ull;
    for (int pb0 = f0; pb0 < f1; pb0 += 256) {
      const int nb = min(256, f1 - pb0);
      __syncthreads();  // the previous chunk's reads (and the key reset) are done
      {
        int i2 = -1;
        if (tid < nb) {
          i2 = P.s2.fv.node_feats[pb0 + tid];
          const bool st2 = P.s2.u_right ? P.s2.u_right[i2] >= 0 : false;
          if ((P.s2.has_mp && P.s2.has_mp[i2]) || (P.only_stereo && !st2)) {  // (:728)
            i2 = -1;
          } else {
            const uint64_t* q = (const uint64_t*)(P.s2.desc + (int64_t)i2 * 32);
            s_d[tid][0] = q[0];
            s_d[tid][1] = q[1];
            s_d[tid][2] = q[2];
            s_d[tid][3] = q[3];
            const orbx_keypoint kp2 = P.s2.keys_un[i2];
            s_x[tid] = kp2.x;
            s_y[tid] = kp2.y;
            s_oct[tid] = kp2.octave | (st2 ? 0x10000 : 0);
          }
        }
        s_i2[tid] = i2;
      }
      __syncthreads();
      if (live) {
        for (int j = g; j < nb; j += G) {
          if (s_i2[j] < 0) continue;
          const uint64_t* dd = s_d[j];
          const int dist = __popcll(d1[0] ^ dd[0]) + __popcll(d1[1] ^ dd[1]) +
                           __popcll(d1[2] ^ dd[2]) + __popcll(d1[3] ^ dd[3]);
          if (dist > kTH_LOW) continue;
          const unsigned long long key =
              ((unsigned long long)dist << 32) | (uint32_t)~(pb0 - f0 + j);
          if (key > best) continue;
          const int oc2 = s_oct[j];
          const bool st2 = oc2 >> 16;
          const int oct2 = oc2 & 0xFFFF;
          const float x2 = s_x[j], y2 = s_y[j];
          if (!st1 && !st2) {
            const float dex = P.ex - x2, dey = P.ey - y2;
            if (__builtin_fmaf(dex, dex, dey * dey) < 100 * P.s2.scale_factors[oct2]) continue;
          }
          if (epipolar_ok(kp1.x, kp1.y, x2, y2, P.F, P.s2.level_sigma2[oct2])) best = key;
        }
      }
    }
    if (live && best != ~0ull) atomicMin(&s_key[u], best);
    __syncthreads();
    if (tid < n1 && live) {  // g == 0: the feature's own liveness
      const unsigned long long key = s_key[tid];
      P.m12[i1] = key == ~0ull ? -1 : P.s2.fv.node_feats[f0 + (int)~(uint32_t)key];
    }
    __syncthreads();  // s_key is reset for the next KF1 chunk
  }
}

// a resident call's level tables travel inside the problem: point the sides at the LDS copy
__device__ __forceinline__ void tri_inline_tables(TriProblem& p) {
  if (!p.tab_inline) return;
  if (threadIdx.x == 0) {
    p.s1.scale_factors = p.tab[0];
    p.s1.level_sigma2 = p.tab[1];
    p.s2.scale_factors = p.tab[2];
    p.s2.level_sigma2 = p.tab[3];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_tri_nodes_wg(const TriProblem* __restrict__ probs) {
  __shared__ TriProblem s_p;
  stage_problem(&s_p, probs + blockIdx.y);
  tri_inline_tables(s_p);
  tri_nodes_wg(&s_p, 0);
  if (s_p.done && last_workgroup(s_p.done)) tri_finish(&s_p, 0);
}

__device__ __forceinline__ void tri_finish(const TriProblem* __restrict__ probs, const int pi) {
  const TriProblem& P = probs[pi];
  __shared__ int hist[kHISTO];
  __shared__ int s_ind[3];
  __shared__ int s_scan[4];
  const int tid = threadIdx.x;
  const int n = tri_n(P.s1), n2 = tri_n(P.s2);
  if (tid < kHISTO) hist[tid] = 0;
  __syncthreads();
  // rounds of kFinishRegs entries per thread, every load of a round in flight before its
  // atomics and stores
  if (P.check_ori) {
    for (int i0 = tid; i0 < n; i0 += 256 * kFinishRegs) {
      int m[kFinishRegs];
      float a1[kFinishRegs], a2[kFinishRegs];
#pragma unroll
      for (int r = 0; r < kFinishRegs; r++) {
        const int i = i0 + 256 * r;
        m[r] = i < n ? P.m12[i] : -1;
      }
#pragma unroll
      for (int r = 0; r < kFinishRegs; r++) {
        const bool ok = m[r] >= 0 && m[r] < n2;
        a1[r] = ok ? P.s1.keys_un[i0 + 256 * r].angle : 0.f;
        a2[r] = ok ? P.s2.keys_un[m[r]].angle : 0.f;
      }
#pragma unroll
      for (int r = 0; r < kFinishRegs; r++)
        if (m[r] >= 0 && m[r] < n2) atomicAdd(&hist[rot_bin(a1[r], a2[r])], 1);
    }
    __syncthreads();
    if (tid == 0) three_maxima(hist, s_ind[0], s_ind[1], s_ind[2]);
    __syncthreads();
  }
  // ordered compaction over idx1 (chunked per thread for stability)
  const int per = (n + 255) / 256;
  const int beg = min(tid * per, n), end = min(beg + per, n);
  int mine = 0;
  for (int b0 = beg; b0 < end; b0 += kFinishRegs) {
    int m[kFinishRegs], bin[kFinishRegs];
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) m[r] = b0 + r < end ? P.m12[b0 + r] : -1;
    uint32_t bad = 0;
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++)
      if (m[r] >= n2) {  // stale or corrupt index: report, drop, never dereference
        bad |= 1u << r;
        m[r] = -1;
      }
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++)
      bin[r] = (m[r] >= 0 && P.check_ori)
                   ? rot_bin(P.s1.keys_un[b0 + r].angle, P.s2.keys_un[m[r]].angle)
                   : -1;
    if (bad && P.error) atomicOr(P.error, ORBX_DEVERR_INDEX);
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) {
      if (m[r] >= 0 && P.check_ori && bin[r] != s_ind[0] && bin[r] != s_ind[1] &&
          bin[r] != s_ind[2]) {
        bad |= 1u << r;
        m[r] = -1;
      }
      if ((bad >> r) & 1) P.m12[b0 + r] = -1;
      mine += m[r] >= 0;
    }
  }
  // exclusive scan of the per-thread counts (DPP wave scans + the 4 wave totals)
  const int lane = tid & 63, wid = tid >> 6;
  const int incl = wave_scan_incl(mine);
  if (lane == 63) s_scan[wid] = incl;
  __syncthreads();
  int pos = incl - mine, total = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    pos += w < wid ? s_scan[w] : 0;
    total += s_scan[w];
  }
  int* const pairs = P.pairs_host ? P.pairs_host : P.pairs;  // resident calls: pinned host
  for (int b0 = beg; b0 < end; b0 += kFinishRegs) {
    int m[kFinishRegs];
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) m[r] = b0 + r < end ? P.m12[b0 + r] : -1;
#pragma unroll
    for (int r = 0; r < kFinishRegs; r++) {
      if (m[r] >= 0) {
        pairs[2 * pos] = b0 + r;
        pairs[2 * pos + 1] = m[r];
        pos++;
      }
    }
  }
  if (tid == 0) *P.count = total;
  if (P.pairs_host) {  // scratch back to clean for the next resident call
    __syncthreads();   // every m12 read above is done
    for (int i = tid; i < n; i += 256) P.m12[i] = -1;
    if (tid == 0) {
      P.ctrl_host[0] = total;
      P.ctrl_host[1] = P.error ? atomicExch(P.error, 0) : 0;
      if (P.done) atomicExch(P.done, 0);
    }
  }
}

__global__ __launch_bounds__(256) void k_tri_finish(const TriProblem* __restrict__ probs) {
  __shared__ TriProblem s_p;
  stage_problem(&s_p, probs + blockIdx.x);
  tri_inline_tables(s_p);
  tri_finish(&s_p, 0);
}

// ------------------------------------------------------------------ vocabulary + FeatureVector
// Stable bucket sort of feature indices by node bucket (one workgroup per image): bucket of
// feature i = node_of[i] - id_lo in [0, nb), or 0xFFFFFFFF for a feature the FeatureVector
// skips (stopped word).  Bucket b is node id rank_ids[b] (or id_lo + b when rank_ids is null);
// buckets ascend with node id.  Output: node_ids ascending, offsets, feats ascending within
// each node (FeatureVector::addFeature in index order, FeatureVector.cpp:31-45).
__global__ __launch_bounds__(256) void k_csr(const uint32_t* __restrict__ node_of,
                                             int64_t node_stride, const int* __restrict__ counts,
                                             int n_fixed, uint32_t id_lo, int nb,
                                             const uint32_t* __restrict__ rank_ids,
                                             uint32_t* __restrict__ node_ids,
                                             int* __restrict__ offsets, int* __restrict__ feats,
                                             int64_t feats_stride, int* __restrict__ n_nodes,
                                             int stage_cap) {
  extern __shared__ int sm[];
  int* cnt = sm;       // nb
  int* cur = sm + nb;  // nb
  const int img = blockIdx.x, tid = threadIdx.x;
  const int n = counts ? counts[img] : n_fixed;
  const uint32_t* nodes = node_of + img * node_stride;
  if (n <= stage_cap) {  // the image's node ids into LDS in one coalesced round
    uint32_t* s_nodes = (uint32_t*)(sm + 2 * nb);
    for (int i = tid; i < n; i += 256) s_nodes[i] = nodes[i];
    nodes = s_nodes;
  }
  uint32_t* oid = node_ids + (int64_t)img * nb;        // [img][nb]
  int* ooff = offsets + (int64_t)img * (nb + 1);       // [img][nb + 1]
  int* of = feats + img * feats_stride;                // [img][feats_stride]
  for (int i = tid; i < nb; i += 256) cnt[i] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += 256)
    if (nodes[i] != 0xFFFFFFFFu) atomicAdd(&cnt[nodes[i] - id_lo], 1);
  __syncthreads();
  // bucket starts: wave-0 exclusive scan over the nb buckets, 64 at a time
  if (tid < 64) {
    int run = 0, nn = 0;
    for (int b0 = 0; b0 < nb; b0 += 64) {
      const int b = b0 + tid;
      const int c = b < nb ? cnt[b] : 0;
      const int incl = wave_scan_incl(c);
      const uint64_t ne = __ballot(c > 0);
      const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(ne >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)ne, 0));
      if (b < nb) {
        cur[b] = run + incl - c;
        if (c > 0) {
          oid[nn + rank] = rank_ids ? rank_ids[b] : id_lo + b;
          ooff[nn + rank] = run + incl - c;
        }
      }
      run += __shfl(incl, 63);
      nn += __popcll(ne);
    }
    if (tid == 0) {
      ooff[nn] = run;
      n_nodes[img] = nn;
    }
  }
  __syncthreads();
  // stable placement by wave 0: chunks of 64 features in index order; a lane's rank inside its
  // bucket = lanes below it with the same bucket, from one ballot per bucket-id bit
  if (tid < 64) {
    int nbits = 1;
    while ((1 << nbits) < nb) nbits++;
    const uint64_t lt = (1ull << tid) - 1, gt = ~((2ull << tid) - 1);
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int i = c0 + tid;
      const uint32_t nd = i < n ? nodes[i] : 0xFFFFFFFFu;
      const bool valid = nd != 0xFFFFFFFFu;
      const int bk = valid ? (int)(nd - id_lo) : 0;
      uint64_t eq = __ballot(valid);
      for (int bit = 0; bit < nbits; bit++) {
        const uint64_t m = __ballot(valid && ((bk >> bit) & 1));
        eq &= ((bk >> bit) & 1) ? m : ~m;
      }
      if (valid) {
        const int base = cur[bk];
        of[base + __popcll(eq & lt)] = i;
        if ((eq & gt) == 0) cur[bk] = base + __popcll(eq);  // last lane of the bucket
      }
    }
  }
}

__global__ void k_distance(const uint8_t* a, const uint8_t* b, int n, int* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = hamming32(a + (int64_t)i * 32, b + (int64_t)i * 32);
}

// ------------------------------------------------------------------ launchers
// calls with at most kBowWgProbs problems use the workgroup-per-node SearchByBoW
// (ORBX_BOW_WG_PROBS overrides the limit for experiments)
constexpr int kBowWgProbs = 4;

namespace {
std::atomic<int> g_bow_form{0};  // orbx_debug_bow_kernel: 0 = chosen per call
}

int launch_bow(const BowProblem* d_probs, int nprob, int max_nodes1, hipStream_t s,
               bool fused_finish, int feats_per_node) {
  if (nprob <= 0) return ORBX_OK;
  // 1 the workgroup form (calls of few problems: the drop-in), else a wave per node with 4
  // register chunks (2) for frames with many features per vocabulary node, or with 2 (3).
  // (A 16- or 32-lane group per node, several nodes per wave, measured slower: 0.16-0.17 vs 0.115
  // ms per 512 C2 frames — the group's per-feature broadcasts need ds_bpermute where the wave
  // form's are readlanes.)
  int form = g_bow_form.load(std::memory_order_relaxed);
  if (form < 1 || form > 3) form = nprob <= kBowWgProbs ? 1 : feats_per_node >= kBowWideNode ? 2 : 3;
  const bool wg = max_nodes1 > 0 && form == 1;
  if (max_nodes1 > 0) {
    if (form == 1)
      hipLaunchKernelGGL(k_bow_nodes_wg, dim3(max_nodes1, nprob), dim3(256), 0, s, d_probs);
    else if (form == 2)
      hipLaunchKernelGGL(k_bow_nodes<4>, dim3((max_nodes1 + 3) / 4, nprob), dim3(256), 0, s, d_probs);
    else
      hipLaunchKernelGGL(k_bow_nodes<kBowDescChunks>, dim3((max_nodes1 + 3) / 4, nprob), dim3(256),
                         0, s, d_probs);
  }
  if (!(wg && fused_finish))  // else the node kernel's last workgroup ran it
    hipLaunchKernelGGL(k_bow_finish, dim3(nprob), dim3(256), 0, s, d_probs);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_bow");
}

// calls with at most kTriWgProbs keyframe pairs use the workgroup-per-node form
// (ORBX_TRI_WG_PROBS overrides the limit for experiments)
constexpr int kTriWgProbs = 4;

int launch_tri(const TriProblem* d_probs, int nprob, int max_nodes1, hipStream_t s,
               bool fused_finish) {
  if (nprob <= 0) return ORBX_OK;
  const bool wg = max_nodes1 > 0 && nprob <= kTriWgProbs;
  if (wg)
    hipLaunchKernelGGL(k_tri_nodes_wg, dim3(max_nodes1, nprob), dim3(256), 0, s, d_probs);
  else if (max_nodes1 > 0)
    hipLaunchKernelGGL(k_tri_nodes, dim3((max_nodes1 + 3) / 4, nprob), dim3(256), 0, s, d_probs);
  if (!(wg && fused_finish))  // else the node kernel's last workgroup ran it
    hipLaunchKernelGGL(k_tri_finish, dim3(nprob), dim3(256), 0, s, d_probs);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_tri");
}

int launch_csr(const uint32_t* d_node_of, int64_t node_stride, const int* d_counts, int n_fixed,
               uint32_t id_lo, int nb, const uint32_t* d_rank_ids, uint32_t* d_ids, int* d_off,
               int* d_feats, int64_t feats_stride, int* d_nn, int nimg, hipStream_t s) {
  if (nimg <= 0) return ORBX_OK;
  size_t smem = (size_t)(2 * nb) * 4;
  if (smem > 64 * 1024) return ORBX_EUNSUPPORTED;
  // the node ids staged in LDS too when the per-image capacity fits beside the buckets
  const int64_t per_img = std::max<int64_t>(feats_stride, n_fixed);  // features per image, at most
  const int stage_cap = smem + (size_t)per_img * 4 <= 32 * 1024 ? (int)per_img : 0;
  smem += (size_t)stage_cap * 4;
  note_kernel("k_csr");
  hipLaunchKernelGGL(k_csr, dim3(nimg), dim3(256), smem, s, d_node_of, node_stride, d_counts,
                     n_fixed, id_lo, nb, d_rank_ids, d_ids, d_off, d_feats, feats_stride, d_nn,
                     stage_cap);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_csr");
}

// Copies on the compute queue (one of the ends pinned host memory, read or written over PCIe by
// the kernel itself): an asynchronous copy outside a graph goes to a DMA engine, and a
// DMA -> kernel -> DMA chain waits ~10 us at each engine switch, which for the per-frame calls'
// few-KB payloads is longer than the copies
__global__ __launch_bounds__(256) void k_copy(uint8_t* __restrict__ dst,
                                              const uint8_t* __restrict__ src, size_t n) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const size_t n16 = n >> 4;
    for (size_t i = t; i < n16; i += stride) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    for (size_t i = (n16 << 4) + t; i < n; i += stride) dst[i] = src[i];
  } else {
    for (size_t i = t; i < n; i += stride) dst[i] = src[i];
  }
}

hipError_t queue_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((bytes + 4095) / 4096, 256);
  hipLaunchKernelGGL(k_copy, dim3((unsigned)blocks), dim3(256), 0, s, (uint8_t*)dst,
                     (const uint8_t*)src, bytes);
  return hipGetLastError();
}

// ------------------------------------------------------------------ host-pointer ABI
thread_local Workspace tls_ws;
thread_local PinnedBuf tls_stage;

// ------------------------------------------------------------------ resident frames
namespace {
std::mutex g_res_mutex;
ResEntry g_res[kResEntries];
uint64_t g_res_clock = 0;
}  // namespace

bool res_enabled() {  // ORBX_NO_RESIDENT=1: every call takes the staged path (A/B runs)
  static const bool on = getenv("ORBX_NO_RESIDENT") == nullptr;
  return on;
}

ResEntry* res_acquire(int n, const uint8_t* desc, bool* hit) {
  if (n <= 0 || n > kResMaxFeatures || !desc || !hit) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(g_res_mutex);
  const size_t bytes = (size_t)n * 32;
  ResEntry* victim = nullptr;
  for (ResEntry& e : g_res) {
    if (e.ready && e.device == dev && e.n == n && memcmp(e.h_desc.data(), desc, bytes) == 0) {
      e.refs++;
      e.stamp = ++g_res_clock;
      *hit = true;
      return &e;
    }
    if (e.refs == 0 && (!victim || e.stamp < victim->stamp)) victim = &e;  // free ones: stamp 0
  }
  if (!victim) return nullptr;  // every entry in use by a call in flight
  if (victim->device != dev || victim->cap < n) {
    ORBX_RESOURCE_LOCK;
    if (victim->d) (void)hipFree(victim->d);
    victim->d = nullptr;
    victim->cap = 0;
    const int cap = std::max(1024, (n + 255) & ~255);
    if (hipMalloc(&victim->d, ResEntry::bytes(cap)) != hipSuccess) {
      victim->d = nullptr;
      victim->device = -1;
      victim->n = -1;
      return nullptr;
    }
    victim->cap = cap;
    victim->device = dev;
  }
  victim->n = n;
  victim->ready = false;
  victim->fv_n = -1;
  victim->has_keys = false;
  victim->h_desc.assign(desc, desc + bytes);
  victim->refs = 1;
  victim->stamp = ++g_res_clock;
  *hit = false;
  return victim;
}

void res_release(ResEntry* e) {
  if (!e) return;
  std::lock_guard<std::mutex> lock(g_res_mutex);
  e->refs--;
}

bool res_fv_matches(const ResEntry* e, const orbx_featvec& fv) {
  std::lock_guard<std::mutex> lock(g_res_mutex);
  if (e->fv_n != fv.n_nodes) return false;
  const int nn = fv.n_nodes;
  if (nn == 0) return true;
  const int m = fv.node_offsets[nn];
  return memcmp(e->h_ids.data(), fv.node_ids, (size_t)nn * 4) == 0 &&
         memcmp(e->h_off.data(), fv.node_offsets, ((size_t)nn + 1) * 4) == 0 &&
         (int)e->h_feats.size() == m && memcmp(e->h_feats.data(), fv.node_feats, (size_t)m * 4) == 0;
}

bool res_keys_match(const ResEntry* e, const orbx_keypoint* keys) {
  std::lock_guard<std::mutex> lock(g_res_mutex);
  return e->has_keys && memcmp(e->h_keys.data(), keys, sizeof(orbx_keypoint) * e->n) == 0;
}

void res_mark_filled(ResEntry* e, bool desc, const orbx_featvec* fv, const orbx_keypoint* keys) {
  std::lock_guard<std::mutex> lock(g_res_mutex);
  if (desc) e->ready = true;
  if (fv) {
    const int nn = fv->n_nodes, m = nn ? fv->node_offsets[nn] : 0;
    e->h_ids.assign(fv->node_ids, fv->node_ids + nn);
    e->h_off.assign(fv->node_offsets, fv->node_offsets + nn + 1);
    if (nn == 0) e->h_off.assign(1, 0);
    e->h_feats.assign(fv->node_feats, fv->node_feats + m);
    e->fv_n = nn;
  }
  if (keys) {
    e->h_keys.assign(keys, keys + e->n);
    e->has_keys = true;
  }
}

bool res_exclusive_without_fv(const ResEntry* e) {
  std::lock_guard<std::mutex> lock(g_res_mutex);
  return e->refs == 1 && e->fv_n < 0;
}

void res_invalidate(ResEntry* e) {
  std::lock_guard<std::mutex> lock(g_res_mutex);
  e->ready = false;
  e->n = -1;
  e->fv_n = -1;
  e->has_keys = false;
  e->stamp = 0;
}

namespace {
struct ResScratchHolder {
  ResScratch r;
  ~ResScratchHolder() {
    ORBX_RESOURCE_LOCK;
    if (r.d) (void)hipFree(r.d);
  }
};
thread_local ResScratchHolder tls_res;
}  // namespace

ResScratch* res_scratch(int cap) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  if (tls_ws.reserve(256) != ORBX_OK) return nullptr;  // the thread's stream
  ResScratch& r = tls_res.r;
  if (r.device != dev || r.cap < cap) {
    ORBX_RESOURCE_LOCK;
    if (r.d) (void)hipFree(r.d);
    r.d = nullptr;
    r.cap = 0;
    const int c = std::max(4096, (cap + 1023) & ~1023);
    if (hipMalloc(&r.d, ((size_t)3 * c + 16) * 4) != hipSuccess) {
      r.d = nullptr;
      r.device = -1;
      return nullptr;
    }
    r.cap = c;
    r.device = dev;
    r.dirty = true;
  }
  if (r.dirty) {
    hipStream_t s = tls_ws.stream;
    if (hipMemsetAsync(r.match(), 0xFF, (size_t)r.cap * 4, s) != hipSuccess ||
        hipMemsetAsync(r.matched2(), 0, (size_t)r.cap * 4, s) != hipSuccess ||
        hipMemsetAsync(r.m12(), 0xFF, (size_t)r.cap * 4, s) != hipSuccess ||
        hipMemsetAsync(r.ctrl(), 0, 16 * 4, s) != hipSuccess || wait_stream(s) != hipSuccess)
      return nullptr;
    r.dirty = false;
  }
  return &r;
}

}  // namespace orbx

using namespace orbx;

namespace {

struct SideOffs {
  size_t desc, angle, valid, ids, offs, feats;
};

bool side_ok(const orbx_bow_side* s) {
  return s && s->n >= 0 && (s->n == 0 || (s->desc && s->angle)) && s->fv.n_nodes >= 0 &&
         (s->fv.n_nodes == 0 || (s->fv.node_ids && s->fv.node_offsets && s->fv.node_feats));
}

// Every feature index must be inside [0, n) so no kernel reads out of bounds.
bool fv_ok(const orbx_featvec& fv, int n) {
  if (fv.n_nodes == 0) return true;
  if (fv.node_offsets[0] != 0) return false;
  for (int k = 0; k < fv.n_nodes; k++) {
    if (fv.node_offsets[k + 1] < fv.node_offsets[k]) return false;
    if (k && fv.node_ids[k] <= fv.node_ids[k - 1]) return false;
  }
  for (int i = 0; i < fv.node_offsets[fv.n_nodes]; i++)
    if (fv.node_feats[i] < 0 || fv.node_feats[i] >= n) return false;
  return true;
}

SideOffs stage_side(Stager& st, const orbx_bow_side* s) {
  SideOffs o;
  o.desc = st.add(s->desc, (size_t)s->n * 32);
  o.angle = st.add(s->angle, (size_t)s->n * 4);
  o.valid = s->valid ? st.add(s->valid, (size_t)s->n) : (size_t)-1;
  o.ids = st.add(s->fv.node_ids, (size_t)s->fv.n_nodes * 4);
  o.offs = st.add(s->fv.node_offsets, (size_t)(s->fv.n_nodes + 1) * 4);
  o.feats = st.add(s->fv.node_feats,
                   (size_t)(s->fv.n_nodes ? s->fv.node_offsets[s->fv.n_nodes] : 0) * 4);
  return o;
}

DevSide dev_side(char* base, const SideOffs& o, const orbx_bow_side* s) {
  DevSide d{};
  d.n = s->n;
  d.desc = dptr<const uint8_t>(base, o.desc);
  d.angle = dptr<const float>(base, o.angle);
  d.angle_stride = 1;
  d.valid = o.valid == (size_t)-1 ? nullptr : dptr<const uint8_t>(base, o.valid);
  d.n_nodes = s->fv.n_nodes;
  d.node_ids = dptr<const uint32_t>(base, o.ids);
  d.node_offsets = dptr<const int>(base, o.offs);
  d.node_feats = dptr<const int>(base, o.feats);
  return d;
}

// A frame-cache entry held for the duration of a call, with what the call must still upload
// into it (a whole block image staged at `up`: descriptors, FeatureVector and, for
// SearchForTriangulation, keypoints).
struct Held {
  ResEntry* e = nullptr;
  bool need_desc = false, need_fv = false, need_keys = false, committed = false;
  size_t up = (size_t)-1, up_bytes = 0;
  char* up_dst = nullptr;
  Held() = default;
  Held(const Held&) = delete;
  ~Held() {
    if (e && need() && !committed) res_invalidate(e);  // an upload that may not have landed
    res_release(e);
  }
  bool need() const { return need_desc || need_fv || need_keys; }
};



// Finds (or claims) the entry of a side's descriptors and decides what to upload.  false: the
// resident path does not apply (no entry free, or the FeatureVector / keypoints differ from an
// entry another call is using).
bool res_side(Held& h, int n, const uint8_t* desc, const orbx_featvec& fv, const orbx_keypoint* keys) {
  bool hit = false;
  h.e = res_acquire(n, desc, &hit);
  if (!h.e) return false;
  h.need_desc = !hit;
  h.need_fv = !hit || !res_fv_matches(h.e, fv);
  h.need_keys = keys && (!hit || !res_keys_match(h.e, keys));
  if (hit && (h.need_fv || h.need_keys)) {  // rewriting a part another call may be reading
    bool shared;
    {
      std::lock_guard<std::mutex> lock(g_res_mutex);
      shared = h.e->refs > 1;
    }
    if (shared) return false;
  }
  return true;
}

// The block image of a side for an entry upload (desc | fv ids | offsets | feats | keypoints,
// at the entry's capacity offsets).
void stage_block(Stager& st, Held& h, int n, const uint8_t* desc, const orbx_featvec& fv,
                 const orbx_keypoint* keys) {
  if (!h.need()) return;
  const int cap = h.e->cap;
  if (!h.need_desc && !h.need_fv) {  // the keypoints alone (the current frame's first triangulation)
    h.up_bytes = sizeof(orbx_keypoint) * n;
    h.up = st.add(keys, h.up_bytes);
    h.up_dst = (char*)h.e->d_keys();
    return;
  }
  h.up_bytes = keys ? ResEntry::bytes(cap) : (size_t)cap * 32 + ResEntry::fv_bytes(cap);
  h.up = st.add(nullptr, h.up_bytes);
  h.up_dst = h.e->d;
  char* b = st.host.data() + h.up;
  memcpy(b, desc, (size_t)n * 32);
  const int nn = fv.n_nodes, m = nn ? fv.node_offsets[nn] : 0;
  if (nn) memcpy(b + (size_t)cap * 32, fv.node_ids, (size_t)nn * 4);
  if (nn) memcpy(b + (size_t)cap * 36, fv.node_offsets, ((size_t)nn + 1) * 4);
  if (m) memcpy(b + (size_t)cap * 40 + 4, fv.node_feats, (size_t)m * 4);
  if (keys) memcpy(b + (size_t)cap * 44 + 16, keys, sizeof(orbx_keypoint) * n);
}

// after a successful call: the uploaded parts are now resident
void commit_block(Held& h, const orbx_featvec& fv, const orbx_keypoint* keys) {
  if (h.need()) res_mark_filled(h.e, h.need_desc, &fv, keys);
  h.committed = true;
}

// SearchByBoW with both sides' descriptors and FeatureVectors resident in the frame cache (a side
// seen for the first time is uploaded into its entry, one copy), the per-call arrays (angles,
// validity, the problem) read by the kernels from the thread's pinned stager and the results
// written by the finish into it: in the per-frame chain no copy kernel runs at all.
// ORBX_EUNSUPPORTED: not applicable, the caller takes the staged path.
int run_bow_resident(const orbx_bow_side* s1, const orbx_bow_side* s2, float nnratio, int check_ori,
                     int mode, int32_t* match_out, int32_t* nmatches) {
  if (s1->n <= 0 || s2->n <= 0 || s1->n > kResMaxFeatures || s2->n > kResMaxFeatures)
    return ORBX_EUNSUPPORTED;
  const int nout = mode == 1 ? s1->n : s2->n;
  Held h1, h2;
  if (!res_side(h1, s1->n, s1->desc, s1->fv, nullptr) || !res_side(h2, s2->n, s2->desc, s2->fv, nullptr))
    return ORBX_EUNSUPPORTED;
  if (h1.e == h2.e) return ORBX_EUNSUPPORTED;  // the same frame on both sides
  ResScratch* rs = res_scratch(std::max(s1->n, s2->n));
  if (!rs) return ORBX_EUNSUPPORTED;
  Stager st;
  stage_block(st, h1, s1->n, s1->desc, s1->fv, nullptr);
  stage_block(st, h2, s2->n, s2->desc, s2->fv, nullptr);
  // the per-call arrays and the problem: one upload into the workspace (read by every
  // workgroup: over PCIe from the stager they put a round trip on each one's critical path)
  const size_t osmall = (st.host.size() + 15) & ~size_t(15);
  const size_t oa1 = st.add(s1->angle, (size_t)s1->n * 4), oa2 = st.add(s2->angle, (size_t)s2->n * 4);
  const size_t ov1 = s1->valid ? st.add(s1->valid, (size_t)s1->n) : (size_t)-1;
  const size_t ov2 = s2->valid ? st.add(s2->valid, (size_t)s2->n) : (size_t)-1;
  const size_t oprob = st.add(nullptr, sizeof(BowProblem));
  const size_t osmall_end = st.host.size();
  const size_t omatch = st.add(nullptr, (size_t)nout * 4), octrl = st.add(nullptr, 16);
  char* hb = st.host.data();  // final: every add is done
  if (!st.host.pinned) return ORBX_EUNSUPPORTED;
  if (tls_ws.reserve(osmall_end - osmall) != ORBX_OK) return ORBX_EUNSUPPORTED;
  char* db = tls_ws.d - osmall;  // device address of stager offset o: db + o
  auto side = [&](const orbx_bow_side* sd, const Held& h, size_t oa, size_t ov) {
    DevSide d{};
    d.n = sd->n;
    d.desc = h.e->d_desc();
    d.angle = (const float*)(db + oa);
    d.angle_stride = 1;
    d.valid = ov == (size_t)-1 ? nullptr : (const uint8_t*)(db + ov);
    d.n_nodes = sd->fv.n_nodes;
    d.node_ids = h.e->d_ids();
    d.node_offsets = h.e->d_off();
    d.node_feats = h.e->d_feats();
    return d;
  };
  BowProblem P{};
  P.s1 = side(s1, h1, oa1, ov1);
  P.s2 = side(s2, h2, oa2, ov2);
  P.match = rs->match();
  P.matched2 = rs->matched2();
  P.done = rs->ctrl() + 0;
  P.error = rs->ctrl() + 1;
  P.count = rs->ctrl() + 4;
  P.mode = mode;
  P.nnratio = nnratio;
  P.check_ori = check_ori;
  P.match_host = (int*)(hb + omatch);
  P.ctrl_host = (int*)(hb + octrl);
  memcpy(hb + oprob, &P, sizeof(P));
  hipStream_t s = tls_ws.stream;
  rs->dirty = true;  // until the finish has restored it
  for (Held* h : {&h1, &h2})
    if (h->need()) ORBX_HIP(queue_copy(h->up_dst, hb + h->up, h->up_bytes, s));
  ORBX_HIP(queue_copy(db + osmall, hb + osmall, osmall_end - osmall, s));
  int rc = launch_bow((const BowProblem*)(db + oprob), 1, s1->fv.n_nodes, s, true);
  if (rc) return rc;
  ORBX_HIP(orbx::wait_stream(s));
  rs->dirty = false;
  commit_block(h1, s1->fv, nullptr);
  commit_block(h2, s2->fv, nullptr);
  const int* res = (const int*)(hb + octrl);
  if (res[1]) return report(ORBX_EDEVICE, "SearchByBoW: a match index outside the keyframe");
  memcpy(match_out, hb + omatch, (size_t)nout * 4);
  *nmatches = res[0];
  return ORBX_OK;
}

int run_bow(const orbx_bow_side* s1, const orbx_bow_side* s2, float nnratio, int check_ori,
            int mode, int32_t* match_out, int32_t* nmatches) {
  if (!side_ok(s1) || !side_ok(s2) || !match_out || !nmatches) return ORBX_EINVAL;
  if (!fv_ok(s1->fv, s1->n) || !fv_ok(s2->fv, s2->n)) return ORBX_EINVAL;
  if (s2->n >= kBowMaxSide2) return report(ORBX_EUNSUPPORTED, "SearchByBoW: side 2 above 2^23 features");
  if (res_enabled()) {
    const int rr = run_bow_resident(s1, s2, nnratio, check_ori, mode, match_out, nmatches);
    if (rr != ORBX_EUNSUPPORTED) return rr;
  }
  const int nout = mode == 1 ? s1->n : s2->n;
  Stager st;
  SideOffs o1 = stage_side(st, s1), o2 = stage_side(st, s2);
  const size_t omatch = st.add(nullptr, (size_t)std::max(nout, 1) * 4);
  const size_t ocount = st.add(nullptr, 16);
  const size_t oprob = st.add(nullptr, sizeof(BowProblem));
  const size_t omatched2 = st.add(nullptr, (size_t)std::max(s2->n, 1) * 4);  // mode 1, big nodes
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  BowProblem P{};
  P.s1 = dev_side(base, o1, s1);
  P.s2 = dev_side(base, o2, s2);
  P.match = dptr<int>(base, omatch);
  P.count = dptr<int>(base, ocount);
  P.error = dptr<int>(base, ocount + 4);
  P.matched2 = dptr<int>(base, omatched2);
  P.done = dptr<int>(base, ocount + 8);
  P.mode = mode;
  P.nnratio = nnratio;
  P.check_ori = check_ori;
  memcpy(st.host.data() + oprob, &P, sizeof(P));
  memset(st.host.data() + omatch, 0xFF, (size_t)std::max(nout, 1) * 4);
  memset(st.host.data() + ocount, 0, 16);
  memset(st.host.data() + omatched2, 0, (size_t)std::max(s2->n, 1) * 4);
  hipStream_t s = tls_ws.stream;
  ORBX_HIP(tls_ws.upload(st.host, st.host.size()));
  rc = launch_bow(dptr<BowProblem>(base, oprob), 1, s1->fv.n_nodes, s, true);
  if (rc) return rc;
  ORBX_HIP(tls_ws.download(omatch, ocount + 8 - omatch));  // match array and count / error
  ORBX_HIP(orbx::wait_stream(s));
  const int* res = (const int*)(tls_ws.h + ocount);
  if (res[1]) return report(ORBX_EDEVICE, "SearchByBoW: a match index outside the keyframe");
  if (nout > 0) memcpy(match_out, tls_ws.h + omatch, (size_t)nout * 4);
  *nmatches = res[0];
  return ORBX_OK;
}

// SearchForTriangulation with both keyframes' descriptors, FeatureVectors and keypoints
// resident in the frame cache (run_bow_resident's scheme; the level tables travel inside the
// problem, mvuRight and the map-point flags are read from the pinned stager).
int tri_resident(const orbx_tri_side* k1, const orbx_tri_side* k2, const float F12[9], float ex,
                 float ey, int only_stereo, int check_ori, int32_t* pairs, int32_t* nmatches) {
  if (k1->n <= 0 || k2->n <= 0 || k1->n > kResMaxFeatures || k2->n > kResMaxFeatures ||
      k1->nlevels > 16 || k2->nlevels > 16)
    return ORBX_EUNSUPPORTED;
  Held h1, h2;
  if (!res_side(h1, k1->n, k1->desc, k1->fv, nullptr) || !res_side(h2, k2->n, k2->desc, k2->fv, nullptr))
    return ORBX_EUNSUPPORTED;
  if (h1.e == h2.e) return ORBX_EUNSUPPORTED;
  ResScratch* rs = res_scratch(std::max(k1->n, k2->n));
  if (!rs) return ORBX_EUNSUPPORTED;
  Stager st;
  stage_block(st, h1, k1->n, k1->desc, k1->fv, nullptr);
  stage_block(st, h2, k2->n, k2->desc, k2->fv, nullptr);
  const orbx_tri_side* ks[2] = {k1, k2};
  // the per-call arrays (keypoints, mvuRight, map-point flags) and the problem: one upload
  const size_t osmall = (st.host.size() + 15) & ~size_t(15);
  size_t okeys[2], our[2], omp[2];
  for (int i = 0; i < 2; i++) {
    okeys[i] = st.add(ks[i]->keys_un, sizeof(orbx_keypoint) * ks[i]->n);
    our[i] = ks[i]->u_right ? st.add(ks[i]->u_right, (size_t)ks[i]->n * 4) : (size_t)-1;
    omp[i] = ks[i]->has_mp ? st.add(ks[i]->has_mp, (size_t)ks[i]->n) : (size_t)-1;
  }
  const size_t oprob = st.add(nullptr, sizeof(TriProblem));
  const size_t osmall_end = st.host.size();
  const size_t opairs = st.add(nullptr, (size_t)k1->n * 8), octrl = st.add(nullptr, 16);
  if (!st.host.pinned) return ORBX_EUNSUPPORTED;
  if (tls_ws.reserve(osmall_end - osmall) != ORBX_OK) return ORBX_EUNSUPPORTED;
  char* hb = st.host.data();
  char* db = tls_ws.d - osmall;
  TriProblem P{};
  DevTriSide* ds[2] = {&P.s1, &P.s2};
  const Held* hs[2] = {&h1, &h2};
  for (int i = 0; i < 2; i++) {
    const orbx_tri_side* k = ks[i];
    const ResEntry* e = hs[i]->e;
    DevTriSide& d = *ds[i];
    d.n = k->n;
    d.desc = e->d_desc();
    d.keys_un = (const orbx_keypoint*)(db + okeys[i]);
    d.u_right = our[i] == (size_t)-1 ? nullptr : (const float*)(db + our[i]);
    d.has_mp = omp[i] == (size_t)-1 ? nullptr : (const uint8_t*)(db + omp[i]);
    d.fv.n_nodes = k->fv.n_nodes;
    d.fv.node_ids = e->d_ids();
    d.fv.node_offsets = e->d_off();
    d.fv.node_feats = e->d_feats();
    for (int l = 0; l < k->nlevels; l++) {
      P.tab[2 * i][l] = k->scale_factors[l];
      P.tab[2 * i + 1][l] = k->level_sigma2[l];
    }
  }
  P.tab_inline = 1;
  memcpy(P.F, F12, 36);
  P.ex = ex;
  P.ey = ey;
  P.only_stereo = only_stereo;
  P.check_ori = check_ori;
  P.m12 = rs->m12();
  P.done = rs->ctrl() + 2;
  P.error = rs->ctrl() + 3;
  P.count = rs->ctrl() + 5;
  P.pairs_host = (int*)(hb + opairs);
  P.ctrl_host = (int*)(hb + octrl);
  memcpy(hb + oprob, &P, sizeof(P));
  hipStream_t s = tls_ws.stream;
  rs->dirty = true;
  for (Held* h : {&h1, &h2})
    if (h->need()) ORBX_HIP(queue_copy(h->up_dst, hb + h->up, h->up_bytes, s));
  ORBX_HIP(queue_copy(db + osmall, hb + osmall, osmall_end - osmall, s));
  int rc = launch_tri((const TriProblem*)(db + oprob), 1, k1->fv.n_nodes, s, true);
  if (rc) return rc;
  ORBX_HIP(orbx::wait_stream(s));
  rs->dirty = false;
  commit_block(h1, k1->fv, nullptr);
  commit_block(h2, k2->fv, nullptr);
  const int* res = (const int*)(hb + octrl);
  if (res[1]) return report(ORBX_EDEVICE, "SearchForTriangulation: a match index outside KF2");
  if (res[0] > 0) memcpy(pairs, hb + opairs, (size_t)res[0] * 8);
  *nmatches = res[0];
  return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_search_by_bow_kf_f(const orbx_bow_side* kf, const orbx_bow_side* f, float nnratio,
                            int32_t check_ori, int32_t* match, int32_t* nmatches) {
  return run_bow(kf, f, nnratio, check_ori, 0, match, nmatches);
}

int orbx_search_by_bow_kf_kf(const orbx_bow_side* kf1, const orbx_bow_side* kf2, float nnratio,
                             int32_t check_ori, int32_t* match12, int32_t* nmatches) {
  return run_bow(kf1, kf2, nnratio, check_ori, 1, match12, nmatches);
}

int orbx_search_for_triangulation(const orbx_tri_side* k1, const orbx_tri_side* k2,
                                  const float F12[9], float ex, float ey, int32_t only_stereo,
                                  float /*nnratio: not used by the reference here*/,
                                  int32_t check_ori, int32_t* pairs, int32_t* nmatches) {
  const orbx_tri_side* ks[2] = {k1, k2};
  for (const orbx_tri_side* k : ks) {
    if (!k || k->n < 0 || (k->n && (!k->desc || !k->keys_un)) || !k->scale_factors ||
        !k->level_sigma2 || k->nlevels < 1 || k->fv.n_nodes < 0 ||
        (k->fv.n_nodes && (!k->fv.node_ids || !k->fv.node_offsets || !k->fv.node_feats)))
      return ORBX_EINVAL;
    if (!fv_ok(k->fv, k->n)) return ORBX_EINVAL;
    for (int i = 0; i < k->n; i++)
      if (k->keys_un[i].octave < 0 || k->keys_un[i].octave >= k->nlevels) return ORBX_EINVAL;
  }
  if (!F12 || !pairs || !nmatches) return ORBX_EINVAL;
  if (res_enabled()) {
    const int rr = tri_resident(k1, k2, F12, ex, ey, only_stereo, check_ori, pairs, nmatches);
    if (rr != ORBX_EUNSUPPORTED) return rr;
  }
  Stager st;
  size_t o[2][9];
  for (int s = 0; s < 2; s++) {
    const orbx_tri_side* k = ks[s];
    o[s][0] = st.add(k->desc, (size_t)k->n * 32);
    o[s][1] = st.add(k->keys_un, (size_t)k->n * sizeof(orbx_keypoint));
    o[s][2] = k->u_right ? st.add(k->u_right, (size_t)k->n * 4) : (size_t)-1;
    o[s][3] = k->has_mp ? st.add(k->has_mp, (size_t)k->n) : (size_t)-1;
    o[s][4] = st.add(k->fv.node_ids, (size_t)k->fv.n_nodes * 4);
    o[s][5] = st.add(k->fv.node_offsets, (size_t)(k->fv.n_nodes + 1) * 4);
    o[s][6] = st.add(k->fv.node_feats,
                     (size_t)(k->fv.n_nodes ? k->fv.node_offsets[k->fv.n_nodes] : 0) * 4);
    o[s][7] = st.add(k->scale_factors, (size_t)k->nlevels * 4);
    o[s][8] = st.add(k->level_sigma2, (size_t)k->nlevels * 4);
  }
  const int n1 = std::max(k1->n, 1);
  const size_t om12 = st.add(nullptr, (size_t)n1 * 4);
  const size_t opairs = st.add(nullptr, (size_t)n1 * 8);
  const size_t ocount = st.add(nullptr, 16);
  const size_t oprob = st.add(nullptr, sizeof(TriProblem));
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  TriProblem P{};
  DevTriSide* ds[2] = {&P.s1, &P.s2};
  for (int s = 0; s < 2; s++) {
    const orbx_tri_side* k = ks[s];
    DevTriSide& d = *ds[s];
    d.n = k->n;
    d.desc = dptr<const uint8_t>(base, o[s][0]);
    d.keys_un = dptr<const orbx_keypoint>(base, o[s][1]);
    d.u_right = o[s][2] == (size_t)-1 ? nullptr : dptr<const float>(base, o[s][2]);
    d.has_mp = o[s][3] == (size_t)-1 ? nullptr : dptr<const uint8_t>(base, o[s][3]);
    d.fv.n_nodes = k->fv.n_nodes;
    d.fv.node_ids = dptr<const uint32_t>(base, o[s][4]);
    d.fv.node_offsets = dptr<const int>(base, o[s][5]);
    d.fv.node_feats = dptr<const int>(base, o[s][6]);
    d.scale_factors = dptr<const float>(base, o[s][7]);
    d.level_sigma2 = dptr<const float>(base, o[s][8]);
  }
  memcpy(P.F, F12, 36);
  P.ex = ex;
  P.ey = ey;
  P.only_stereo = only_stereo;
  P.check_ori = check_ori;
  P.m12 = dptr<int>(base, om12);
  P.pairs = dptr<int>(base, opairs);
  P.count = dptr<int>(base, ocount);
  P.error = dptr<int>(base, ocount + 4);
  P.done = dptr<int>(base, ocount + 8);
  memcpy(st.host.data() + oprob, &P, sizeof(P));
  memset(st.host.data() + om12, 0xFF, (size_t)n1 * 4);
  memset(st.host.data() + ocount, 0, 16);
  hipStream_t s = tls_ws.stream;
  ORBX_HIP(tls_ws.upload(st.host, st.host.size()));
  rc = launch_tri(dptr<TriProblem>(base, oprob), 1, k1->fv.n_nodes, s, true);
  if (rc) return rc;
  ORBX_HIP(tls_ws.download(opairs, ocount + 8 - opairs));  // pairs and count / error
  ORBX_HIP(orbx::wait_stream(s));
  const int* res = (const int*)(tls_ws.h + ocount);
  if (res[1]) return report(ORBX_EDEVICE, "SearchForTriangulation: a match index outside KF2");
  const int cnt = res[0];
  if (cnt > 0) memcpy(pairs, tls_ws.h + opairs, (size_t)cnt * 8);
  *nmatches = cnt;
  return ORBX_OK;
}

int orbx_epipole(const float R[9], const float t[3], const float Cw[3], float fx, float fy,
                 float cx, float cy, float* ex, float* ey) {
  // Caller-side helper (LocalMapping computes it before SearchForTriangulation,
  // ORBmatcher.cc:667-673).  cv::Mat C2 = R2w*Cw + t2w in f32; ex = fmaf(invz, fx*C2x, cx).
  if (!R || !t || !Cw || !ex || !ey) return ORBX_EINVAL;
  float C2[3];
  for (int r = 0; r < 3; r++) {
    double s = 0;
    for (int c = 0; c < 3; c++) s += (double)R[3 * r + c] * (double)Cw[c];
    C2[r] = (float)s + t[r];
  }
  const float invz = 1.0f / C2[2];
  *ex = fmaf(invz, fx * C2[0], cx);
  *ey = fmaf(invz, fy * C2[1], cy);
  return ORBX_OK;
}

int orbx_descriptor_distance(const uint8_t* a, const uint8_t* b, int32_t n, int32_t* out) {
  if (n < 0 || (n > 0 && (!a || !b || !out))) return ORBX_EINVAL;
  if (n == 0) return ORBX_OK;
  Stager st;
  const size_t oa = st.add(a, (size_t)n * 32), ob = st.add(b, (size_t)n * 32);
  const size_t oo = st.add(nullptr, (size_t)n * 4);
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  ORBX_HIP(host_copy(base, st.host.data(), oo, st.host.pinned, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_distance, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)(base + oa), (const uint8_t*)(base + ob), n,
                     dptr<int>(base, oo));
  ORBX_HIP(hipGetLastError());
  ORBX_HIP(hipMemcpyAsync(out, base + oo, (size_t)n * 4, hipMemcpyDeviceToHost, s));
  ORBX_HIP(orbx::wait_stream(s));
  return ORBX_OK;
}

// Test hook: the finish step of SearchByBoW (kind 0: KF->Frame, match indexed by frame feature
// with KF values < n1; kind 1: KF->KF, indexed by KF1 feature with values < n2) or of
// SearchForTriangulation (kind 2: indexed by KF1 feature, values < n2) over a caller-given match
// array, without the orientation check.  Out-of-range values are what a stale match array
// would hold: the kernels must drop them (out[i] = -1) and report ORBX_EDEVICE, never read
// through them.
int orbx_debug_bow_kernel(int32_t form) {
  if (form < 0 || form > 3) return ORBX_EINVAL;
  g_bow_form.store(form, std::memory_order_relaxed);
  return ORBX_OK;
}

int orbx_debug_match_finish(int32_t kind, int32_t n1, int32_t n2, const int32_t* match,
                            int32_t* out, int32_t* nmatches) {
  if (kind < 0 || kind > 2 || n1 < 0 || n2 < 0 || !match || !out || !nmatches) return ORBX_EINVAL;
  const int n = kind == 0 ? n2 : n1;
  Stager st;
  const size_t om = st.add(match, (size_t)std::max(n, 1) * 4);
  const size_t ocount = st.add(nullptr, 16);
  const size_t oprob = st.add(nullptr, std::max(sizeof(BowProblem), sizeof(TriProblem)));
  const size_t opairs = st.add(nullptr, (size_t)std::max(n, 1) * 8);
  memset(st.host.data() + ocount, 0, 16);
  int rc = tls_ws.reserve(st.host.size());
  if (rc) return rc;
  char* base = tls_ws.d;
  hipStream_t s = tls_ws.stream;
  if (kind < 2) {
    BowProblem P{};
    P.s1.n = n1;
    P.s2.n = n2;
    P.match = dptr<int>(base, om);
    P.count = dptr<int>(base, ocount);
    P.error = dptr<int>(base, ocount + 4);
    P.mode = kind;
    memcpy(st.host.data() + oprob, &P, sizeof(P));
  } else {
    TriProblem P{};
    P.s1.n = n1;
    P.s2.n = n2;
    P.m12 = dptr<int>(base, om);
    P.pairs = dptr<int>(base, opairs);
    P.count = dptr<int>(base, ocount);
    P.error = dptr<int>(base, ocount + 4);
    memcpy(st.host.data() + oprob, &P, sizeof(P));
  }
  ORBX_HIP(host_copy(base, st.host.data(), st.host.size(), st.host.pinned, hipMemcpyHostToDevice, s));
  if (kind < 2)
    hipLaunchKernelGGL(k_bow_finish, dim3(1), dim3(256), 0, s, dptr<const BowProblem>(base, oprob));
  else
    hipLaunchKernelGGL(k_tri_finish, dim3(1), dim3(256), 0, s, dptr<const TriProblem>(base, oprob));
  ORBX_HIP(hipGetLastError());
  int res[2] = {0, 0};
  ORBX_HIP(hipMemcpyAsync(res, base + ocount, 8, hipMemcpyDeviceToHost, s));
  if (n > 0) ORBX_HIP(hipMemcpyAsync(out, base + om, (size_t)n * 4, hipMemcpyDeviceToHost, s));
  ORBX_HIP(orbx::wait_stream(s));
  *nmatches = res[0];
  return res[1] ? ORBX_EDEVICE : ORBX_OK;
}

}  // extern "C"

