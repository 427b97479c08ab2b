// orbx_match.h — device-side problem descriptors for the matcher kernels (orbx_match.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/orbx.h"

namespace orbx {

// One side of SearchByBoW, all pointers in device memory.
struct DevSide {
  int n;
  const int* n_dev;        // nullable: when set, the feature count lives in device memory
  const uint8_t* desc;
  const float* angle;      // angle of feature i at angle[i * angle_stride]
  int angle_stride;
  const uint8_t* valid;    // nullable: all valid
  int n_nodes;
  const int* n_nodes_dev;  // nullable: device-side node count
  const uint32_t* node_ids;
  const int* node_offsets;
  const int* node_feats;
};

__device__ __forceinline__ int side_n(const DevSide& s) { return s.n_dev ? *s.n_dev : s.n; }
__device__ __forceinline__ int side_nodes(const DevSide& s) {
  return s.n_nodes_dev ? *s.n_nodes_dev : s.n_nodes;
}
__device__ __forceinline__ float side_angle(const DevSide& s, int i) {
  return s.angle[(int64_t)i * s.angle_stride];
}

// mode 0 = SearchByBoW(KF, Frame): s1 = KF, s2 = Frame, match[F idx] = KF idx, accept <= 50.
// mode 1 = SearchByBoW(KF1, KF2): match[KF1 idx] = KF2 idx, accept < 50, valid on both sides.
struct BowProblem {
  DevSide s1, s2;
  int* match;  // pre-filled with -1
  int* count;
  int* error;  // bit 1 (ORBX_DEVERR_INDEX): a match index outside the other side
  int* matched2;  // mode 1, nodes above kBowRegCands candidates: vbMatched2 flags [s2.n], zeroed
  int* done;      // nullable, zeroed: k_bow_nodes_wg's finished-workgroup counter (the last one
                  // runs the finish); null: k_bow_finish is launched after it
  int mode;
  float nnratio;
  int check_ori;
  // nullable (the resident per-frame calls): the finish writes the match array to match_host
  // and (count, error) to ctrl_host in pinned host memory, then returns match / matched2 /
  // error / done to their clean state (-1, 0, 0, 0) for the next call: no copy launches
  int* match_host;
  int* ctrl_host;
};

struct DevFeatVec {
  int n_nodes;
  const int* n_nodes_dev;  // nullable
  const uint32_t* node_ids;
  const int* node_offsets;
  const int* node_feats;
};

struct DevTriSide {
  int n;
  const int* n_dev;  // nullable
  const uint8_t* desc;
  const orbx_keypoint* keys_un;
  const float* u_right;   // nullable: mono
  const uint8_t* has_mp;  // nullable: none
  DevFeatVec fv;
  const float* scale_factors;
  const float* level_sigma2;
};

__device__ __forceinline__ int tri_n(const DevTriSide& s) { return s.n_dev ? *s.n_dev : s.n; }
__device__ __forceinline__ int tri_nodes(const DevTriSide& s) {
  return s.fv.n_nodes_dev ? *s.fv.n_nodes_dev : s.fv.n_nodes;
}

struct TriProblem {
  DevTriSide s1, s2;
  float F[9];
  float ex, ey;
  int only_stereo;
  int check_ori;
  int* m12;    // [s1.n], pre-filled with -1
  int* pairs;  // [s1.n][2]
  int* count;
  int* error;  // bit 1 (ORBX_DEVERR_INDEX): a match index outside KF2
  int* done;   // nullable, zeroed: k_tri_nodes_wg's finished-workgroup counter (as BowProblem)
  // nullable (resident calls, as BowProblem): pairs go to pairs_host, (count, error) to
  // ctrl_host, and m12 / error / done return to their clean state
  int* pairs_host;
  int* ctrl_host;
  // tab_inline: the sides' scale_factors / level_sigma2 are tab[0..1] / tab[2..3] (the kernels
  // point them at their LDS copy of the problem), not device arrays
  int tab_inline;
  float tab[4][16];
};

// device error bits of the matcher problems: a finish kernel read a match index outside the
// other side's features (stale or corrupt match array); the entry is dropped, never dereferenced
constexpr int ORBX_DEVERR_INDEX = 2;
// candidates per vocabulary node whose vbMatched2 flags k_bow_nodes keeps in a per-lane register
// bitmap (64 chunks of 64); larger nodes keep them in global memory
constexpr int kBowRegCands = 64 * 64;
// k_bow_nodes: candidate chunks of 64 kept in registers for a whole node (8 VGPRs each; 1 or 4
// measured no faster at C2, and the wide-node instance keeps 4)
constexpr int kBowDescChunks = 2;
// SearchByBoW's wave merge packs (best distance, node position) into 32 bits: side 2 of a
// problem holds fewer than 2^23 features (the entry points reject more)
constexpr int kBowMaxSide2 = 1 << 23;
constexpr int kBowPosMask = kBowMaxSide2 - 1;

// fused_finish: every problem's `done` counter is set and zeroed, and a call taking the
// workgroup-per-node kernel runs the finish in its last workgroup instead of a second launch
// feats_per_node: features per frame over vocabulary nodes (a hint: at kBowWideNode and above
// the batched kernel keeps 4 candidate chunks in registers)
constexpr int kBowWideNode = 32;
int launch_bow(const BowProblem* d_probs, int nprob, int max_nodes1, hipStream_t s,
               bool fused_finish = false, int feats_per_node = 0);
int launch_tri(const TriProblem* d_probs, int nprob, int max_nodes1, hipStream_t s,
               bool fused_finish = false);
int launch_csr(const uint32_t* d_node_of, int64_t node_stride, const int* d_counts, int n_fixed,
               uint32_t id_lo, int nb, const uint32_t* d_rank_ids, uint32_t* d_ids, int* d_off,
               int* d_feats, int64_t feats_stride, int* d_nn, int nimg, hipStream_t s);
// d_ids is [nimg][nb], d_off is [nimg][nb + 1], d_feats is [nimg][feats_stride].

// ------------------------------------------------------------------ host-pointer ABI helpers
// bytes between device memory and pinned host memory by a kernel on stream s (orbx_match.hip)
hipError_t queue_copy(void* dst, const void* src, size_t bytes, hipStream_t s);
// the same when the host side is pinned, else an asynchronous hipMemcpy
inline hipError_t host_copy(void* dst, const void* src, size_t bytes, bool pinned,
                            hipMemcpyKind kind, hipStream_t s) {
  return pinned ? queue_copy(dst, src, bytes, s) : hipMemcpyAsync(dst, src, bytes, kind, s);
}

// Growable pinned host buffer (pageable fallback if pinning fails); new bytes read as zero.
struct PinnedBuf {
  char* p = nullptr;
  size_t n = 0, cap = 0;
  bool pinned = false;
  char* data() { return p; }
  const char* data() const { return p; }
  size_t size() const { return n; }
  void resize(size_t m) {
    if (m > cap) grow(std::max(m, 2 * cap + 4096));
    if (m > n) memset(p + n, 0, m - n);
    n = m;
  }
  void grow(size_t want) {
    ORBX_RESOURCE_LOCK;
    char* q = nullptr;
    const bool pin = hipHostMalloc(&q, want, hipHostMallocDefault) == hipSuccess;
    if (!pin) q = (char*)malloc(want);
    if (!q) abort();  // host memory exhausted
    if (n) memcpy(q, p, n);
    release();
    p = q;
    cap = want;
    pinned = pin;
  }
  void release() {
    if (p) {
      if (pinned) (void)hipHostFree(p);
      else free(p);
    }
    p = nullptr;
    cap = 0;
  }
  ~PinnedBuf() {
    ORBX_RESOURCE_LOCK;
    release();
  }
};
extern thread_local PinnedBuf tls_stage;

// Per-thread device workspace (ORBmatcher / the vocabulary are called from the Tracking,
// LocalMapping and LoopClosing threads at once; each thread gets its own stream and buffers).
struct Workspace {
  hipStream_t stream = nullptr;
  char* d = nullptr;  // device buffer, cap bytes
  char* h = nullptr;  // pinned host mirror, cap bytes: uploads and downloads go through it
  size_t cap = 0;
  int device = -1;
  void free_all() {
    if (d) (void)hipFree(d);
    if (h) (void)hipHostFree(h);
    d = nullptr;
    h = nullptr;
    cap = 0;
  }
  ~Workspace() {
    ORBX_RESOURCE_LOCK;
    free_all();
    if (stream) (void)hipStreamDestroy(stream);
  }
  int reserve(size_t bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (device == dev && stream && bytes <= cap) return ORBX_OK;
    ORBX_RESOURCE_LOCK;
    if (device != dev) {
      free_all();
      if (stream) (void)hipStreamDestroy(stream);
      stream = nullptr;
      device = dev;
    }
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess)
      return ORBX_EDEVICE;
    if (bytes <= cap) return ORBX_OK;
    const size_t want = std::max(bytes, cap * 2);
    free_all();
    if (hipMalloc(&d, want) != hipSuccess ||
        hipHostMalloc(&h, want, hipHostMallocDefault) != hipSuccess) {
      free_all();
      return ORBX_ENOMEM;
    }
    cap = want;
    return ORBX_OK;
  }
  // uploads the packed host arrays (a Stager's pinned buffer: one copy kernel reading it, no
  // host copy; a DMA when pinning failed)
  hipError_t upload(const PinnedBuf& host, size_t bytes) {
    return host_copy(d, host.data(), bytes, host.pinned, hipMemcpyHostToDevice, stream);
  }
  // device range [off, off + bytes) into the same range of the pinned mirror
  hipError_t download(size_t off, size_t bytes) {
    return queue_copy(h + off, d + off, bytes, stream);
  }
};
extern thread_local Workspace tls_ws;

// ------------------------------------------------------------------ resident frames
// The per-frame drop-in chain (Frame::ComputeBoW, SearchByBoW(KF, F), SearchForTriangulation)
// hands the library the same frame's arrays call after call, and a keyframe's for many frames
// (the reference keyframe of TrackReferenceKeyFrame, Tracking.cc:1127-1136; KeyFrame copies the
// Frame's descriptors, KeyFrame.cc:31).  A frame's descriptors and FeatureVector stay in HBM in
// an entry of this cache, found by content (feature count, then the descriptor bytes compared
// with the entry's host copy: an address or an id could name another frame after a free or a
// Tracking::Reset).  Entries are claimed least-recently-used; one in use by a call in flight is
// never reclaimed.
constexpr int kResEntries = 16;
// false when ORBX_NO_RESIDENT is set: every call takes the staged per-call copies (A/B runs)
bool res_enabled();
constexpr int kResMaxFeatures = 8192;
struct ResEntry {
  int device = -1;
  int cap = 0;          // features the device block holds
  int n = -1;           // descriptors held (-1: free)
  bool ready = false;   // the device descriptors are filled (a claiming call set them)
  int fv_n = -1;        // FeatureVector nodes held (-1: none)
  bool has_keys = false;  // keypoints (mvKeysUn) held
  uint64_t stamp = 0;
  int refs = 0;
  // device block: desc [cap][32] | fv ids [cap] | fv offsets [cap + 1] | fv feats [cap] |
  // keypoints [cap] (28 B)
  char* d = nullptr;
  std::vector<uint8_t> h_desc;
  std::vector<uint32_t> h_ids;
  std::vector<int> h_off, h_feats;
  std::vector<orbx_keypoint> h_keys;
  uint8_t* d_desc() const { return (uint8_t*)d; }
  uint32_t* d_ids() const { return (uint32_t*)(d + (size_t)cap * 32); }
  int* d_off() const { return (int*)(d + (size_t)cap * 36); }
  int* d_feats() const { return (int*)(d + (size_t)cap * 40 + 4); }
  orbx_keypoint* d_keys() const { return (orbx_keypoint*)(d + (size_t)cap * 44 + 16); }  // 16-B aligned
  static size_t fv_bytes(int cap) { return (size_t)cap * 12 + 4; }  // ids | offsets | feats
  static size_t bytes(int cap) { return (size_t)cap * 72 + 16; }
};
// The entry holding these n descriptors on the current device (*hit), or a reclaimed one now
// assigned to them whose device copy the caller must fill (!*hit).  nullptr: n out of range or
// no entry free (every one in use).  Every non-null return is released by res_release.
ResEntry* res_acquire(int n, const uint8_t* desc, bool* hit);
void res_release(ResEntry* e);
// whether the entry's device FeatureVector / keypoints equal these host arrays
bool res_fv_matches(const ResEntry* e, const orbx_featvec& fv);
bool res_keys_match(const ResEntry* e, const orbx_keypoint* keys);
// after the call that filled them has completed: the entry's device descriptors, FeatureVector
// and keypoints equal these host arrays (nullptr: that part unchanged)
void res_mark_filled(ResEntry* e, bool desc, const orbx_featvec* fv, const orbx_keypoint* keys);
// drops the entry's contents (a failed fill)
void res_invalidate(ResEntry* e);
// the caller is the entry's only user and it holds no FeatureVector yet
bool res_exclusive_without_fv(const ResEntry* e);

// Per-thread device scratch of the resident calls, kept in its clean state between calls (the
// finish kernels restore it): bow match [cap] = -1, matched2 [cap] = 0, tri m12 [cap] = -1,
// control words (bow done / error, tri done / error) = 0.
struct ResScratch {
  int device = -1;
  int cap = 0;
  bool dirty = true;  // a call failed between launch and finish: re-initialise first
  char* d = nullptr;
  int* match() const { return (int*)d; }
  int* matched2() const { return (int*)d + cap; }
  int* m12() const { return (int*)d + 2 * (size_t)cap; }
  int* ctrl() const { return (int*)d + 3 * (size_t)cap; }  // [0] bow done [1] bow error [2] tri done [3] tri error [4..7] device counts
};
// the calling thread's scratch for at least cap features (re-initialised when grown or dirty,
// synchronously on the thread's stream); nullptr on an allocation failure
ResScratch* res_scratch(int cap);

// Packs host arrays into one staging buffer, uploaded with one copy.  The buffer is the
// calling thread's pinned arena (one Stager per thread at a time: every entry point stages,
// uploads and waits for its stream before returning), so the upload is a DMA from it.
struct Stager {
  PinnedBuf& host;
  Stager() : host(tls_stage) { host.n = 0; }
  Stager(const Stager&) = delete;
  size_t add(const void* p, size_t bytes) {
    const size_t off = (host.size() + 15) & ~size_t(15);
    host.resize(off + bytes);
    if (p && bytes) memcpy(host.data() + off, p, bytes);
    return off;
  }
};

template <class T>
static inline T* dptr(char* base, size_t off) {
  return (T*)(base + off);
}
}  // namespace orbx
