// orbx_stereo.hip — Frame::ComputeStereoMatches (ORB_SLAM2/src/Frame.cc:471-643) on the GPU,
// on the left/right extractions and raw pyramids already resident in HBM.
//
//   k_stereo_rows    one workgroup per stereo frame: the row table vRowIndices (Frame.cc:478-
//                    497) as CSR — every right keypoint registered in rows
//                    floor(y - 2s) .. ceil(y + 2s); order inside a row is irrelevant because
//                    the best candidate is the (distance, right index) minimum, which is the
//                    reference's first-minimum over ascending right indices
//   k_stereo_match   one wave per left keypoint: candidates of its row across lanes (octave
//                    +-1, u window), Hamming minimum, then the 11 x 11 SAD slide over
//                    incR = -5..5 (121 pixels across lanes, one DPP wave reduction per shift;
//                    the centred float windows of the reference have integer entries, so the
//                    integer SAD equals cv::norm(IL, IR, NORM_L1) exactly), parabola fit in f32.
//                    Row entries carry the right keypoint's x and octave (no keypoint reload);
//                    both windows are staged in LDS by aligned dword loads (two rounds, not 24
//                    byte loads per lane: the vector memory pipeline bounded this kernel)
//   k_stereo_filter  one workgroup per frame: median of the retained SADs by a two-level
//                    histogram select, thDist = 1.5f*1.4f*median, invalidate SAD >= thDist
//                    (Frame.cc:626-642)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>

#include "orbx_internal.h"
#include "orbx_stereo.h"

#pragma clang fp contract(off)

namespace orbx {

constexpr int kTH_HIGH = 100;  // ORBmatcher::TH_HIGH (ORBmatcher.cc:37)
constexpr int kW = 5, kL = 5;  // window half size, slide half range (Frame.cc:565, 572)

int stereo_row_span(const Geometry& g) {
  // ceil(y + r) - floor(y - r) + 1 <= 2r + 3 with r = 2 * scale
  return (int)std::ceil(4.0f * g.scale[g.nlevels - 1]) + 3;
}

void stereo_scratch(const Geometry& g, int kp_cap, int* nrows, int64_t* row_cap) {
  *nrows = g.lv[0].h;
  *row_cap = (int64_t)kp_cap * stereo_row_span(g);
}

__global__ __launch_bounds__(256) void k_stereo_rows(const StereoProblem* __restrict__ probs,
                                                     const LevelGeom* __restrict__ lv,
                                                     int nrows, int64_t row_cap) {
  extern __shared__ int s_cnt[];  // [nrows]
  __shared__ int s_tmp[4];
  const StereoProblem& P = probs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nr = *P.nr;
  for (int r = tid; r < nrows; r += 256) s_cnt[r] = 0;
  __syncthreads();
  for (int i = tid; i < nr; i += 256) {
    const orbx_keypoint k = P.kr[i];
    const float r = 2.0f * lv[k.octave].scale;
    const int maxr = min((int)ceilf(k.y + r), nrows - 1);
    const int minr = max((int)floorf(k.y - r), 0);
    for (int y = minr; y <= maxr; y++) atomicAdd(&s_cnt[y], 1);
  }
  __syncthreads();
  // exclusive scan of the row counts: contiguous chunk per thread
  const int per = (nrows + 255) / 256;
  int sum = 0;
  for (int r = tid * per; r < min((tid + 1) * per, nrows); r++) sum += s_cnt[r];
  const int incl = wave_scan_incl(sum);
  if (lane == 63) s_tmp[wid] = incl;
  __syncthreads();
  int base = incl - sum;
  for (int w = 0; w < wid; w++) base += s_tmp[w];
  __syncthreads();
  for (int r = tid * per; r < min((tid + 1) * per, nrows); r++) {
    const int c = s_cnt[r];
    P.row_off[r] = base;
    s_cnt[r] = base;  // fill cursor
    base += c;
  }
  if (tid == 255) P.row_off[nrows] = base;  // the last chunk ends at the total
  __syncthreads();
  for (int i = tid; i < nr; i += 256) {
    const orbx_keypoint k = P.kr[i];
    const float r = 2.0f * lv[k.octave].scale;
    const int maxr = min((int)ceilf(k.y + r), nrows - 1);
    const int minr = max((int)floorf(k.y - r), 0);
    for (int y = minr; y <= maxr; y++) {
      const int slot = atomicAdd(&s_cnt[y], 1);
      if (slot < row_cap) P.row_ent[slot] = make_uint2((uint32_t)i | ((uint32_t)k.octave << 16),
                                                       __float_as_uint(k.x));
    }
  }
}

// kStG lanes per left keypoint, kStKP per workgroup (Frame::ComputeStereoMatches,
// Frame.cc:471-643): the keypoint's chain of dependent loads (row band, candidates, the
// windows) is latency, so several keypoints share a wave's issue slots; the candidate scan, the
// 121 window pixels (eight per lane) and the SAD sums run on the keypoint's 16 lanes (DPP row
// sums and minima).
// lanes per left keypoint: 16 (C3 / C4 stereo 0.41 / 0.72 ms per 512 frames; a half-wave 0.52 /
// 0.90, a wave 0.72 / 1.21), and keypoints per workgroup
constexpr int kStG = 16;
constexpr int kStKP = 256 / kStG;

template <int G>
__device__ __forceinline__ int grp_sum(int v) {
  v = row16_sum(v);
  if constexpr (G == 32) v += __builtin_amdgcn_ds_swizzle(v, 0x401F);
  return v;
}
template <int G>
__device__ __forceinline__ uint32_t grp_min_u32(uint32_t v) {
  v = row16_min(v);
  if constexpr (G == 32) v = min(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F));
  return v;
}

__global__ __launch_bounds__(256) void k_stereo_match(const StereoProblem* __restrict__ probs,
                                                      const LevelGeom* __restrict__ lv,
                                                      int nrows, float mb, float mbf) {
  constexpr int NG = kStG;
  constexpr int KP = ((2 * kW + 1) * (2 * kW + 1) + NG - 1) / NG;  // window pixels per lane
  const StereoProblem& P = probs[blockIdx.y];
  const int lane = threadIdx.x & 63, hl = lane & (NG - 1);
  const int hw = threadIdx.x / NG;  // the workgroup's keypoint group
  const int iL0 = blockIdx.x * kStKP + (threadIdx.x >> 6) * (64 / NG);  // the wave's first keypoint
  const int nl = *P.nl;
  if (iL0 >= nl) return;  // wave-uniform
  const int iL = iL0 + (lane / NG);
  const bool live = iL < nl;  // uniform in the keypoint's lanes
  const orbx_keypoint kpL = P.kl[live ? iL : iL0];
  float uright = -1.0f, depth = -1.0f;
  int sad_out = -1;
  const float minZ = mb, minD = -3.0f;
  const float maxD = mbf / minZ;
  const float vL = kpL.y, uL = kpL.x;
  const int levelL = kpL.octave;
  const int row = (int)vL;  // vRowIndices[vL]: float -> index truncation
  bool ok = live && row >= 0 && row < nrows;
  int bestDist = kTH_HIGH;
  float uR0 = 0.0f;
  const float minU = uL - maxD, maxU = uL - minD;
  if (ok && maxU < 0) ok = false;
  // the left window (IL) depends only on the left keypoint: its loads are issued here, ahead of
  // the candidate search, so their latency overlaps it (values used only when the reference
  // would take the window)
  const LevelGeom& G = lv[levelL];
  const float scaleFactor = G.inv_scale;
  const float scaleduL = roundf(kpL.x * scaleFactor);
  const float scaledvL = roundf(kpL.y * scaleFactor);
  const int y0 = (int)scaledvL - kW, xl0 = (int)scaleduL - kW;
  const bool left_in = y0 >= 0 && y0 + 2 * kW < G.h && xl0 >= 0 && xl0 + 2 * kW < G.w;
  const int64_t pitch = G.pitch;
  const uint8_t* PL = P.pyrL + G.pyr_off;
  const uint8_t* PR = P.pyrR + G.pyr_off;
  int yy[KP], xx[KP];
  bool has[KP];
#pragma unroll
  for (int k = 0; k < KP; k++) {
    const int p = hl + NG * k;
    has[k] = p < (2 * kW + 1) * (2 * kW + 1);
    yy[k] = has[k] ? p / (2 * kW + 1) : 0;
    xx[k] = has[k] ? p - yy[k] * (2 * kW + 1) : 0;
  }
  // its 11 rows x 11 columns as 4 aligned dwords per row (44: two per lane), kept in registers
  // until the window is staged in LDS for the SAD; a dword starting at or past w is not read
  const int al = xl0 & ~3, lo = xl0 - al;
  constexpr int KLW = ((2 * kW + 1) * 4 + NG - 1) / NG;
  uint32_t lw[KLW];
#pragma unroll
  for (int r = 0; r < KLW; r++) lw[r] = 0u;
#pragma unroll
  for (int r = 0; r < KLW; r++) {
    const int i = hl + NG * r;
    if (ok && left_in && i < (2 * kW + 1) * 4 && al + 4 * (i & 3) < G.w)
      lw[r] = *(const uint32_t*)(PL + (int64_t)(y0 + (i >> 2)) * pitch + al + 4 * (i & 3));
  }
  if (ok) {
    const int c0 = P.row_off[row], c1 = P.row_off[row + 1];
    const uint64_t* q = (const uint64_t*)(P.dl + (int64_t)iL * 32);
    const uint64_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
    int key = INT_MAX;  // (distance << 16) | right index: first minimum in right-index order
    float ukey = 0.0f;  // the u of this lane's best key (no reload of the winner's keypoint)
    for (int j = c0 + hl; j < c1; j += NG) {
      const uint2 e = P.row_ent[j];  // (index | octave << 16, x): no keypoint reload
      const int iR = (int)(e.x & 0xFFFFu), octR = (int)(e.x >> 16);
      if (octR < levelL - 1 || octR > levelL + 1) continue;
      const float uR = __uint_as_float(e.y);
      if (uR >= minU && uR <= maxU) {
        const uint64_t* r = (const uint64_t*)(P.dr + (int64_t)iR * 32);
        const int dist = __popcll(d0 ^ r[0]) + __popcll(d1 ^ r[1]) + __popcll(d2 ^ r[2]) +
                         __popcll(d3 ^ r[3]);
        const int k2 = (dist << 16) | iR;
        if (k2 < key) {
          key = k2;
          ukey = uR;
        }
      }
    }
    const int kmin = (int)grp_min_u32<NG>((uint32_t)key);  // key >= 0: the same minimum
    if (kmin != INT_MAX && (kmin >> 16) < bestDist) {
      bestDist = kmin >> 16;
      const int gb = lane & ~(NG - 1);
      const uint32_t who = (uint32_t)(__ballot(key == kmin) >> gb);  // unique keys
      uR0 = __shfl(ukey, gb + (int)__builtin_ctz(who));
    }
    ok = bestDist < kTH_HIGH;
  }
  if (ok) {  // subpixel match by correlation (Frame.cc:555-618)
    const float scaleduR0 = roundf(uR0 * scaleFactor);
    const float iniu = scaleduR0 + kL - kW;
    const float endu = scaleduR0 + kL + kW + 1;
    const int xr = (int)scaleduR0;
    ok = !(iniu < 0 || endu >= G.w);
    // windows the reference would take with cv::Mat ranges (they assert inside the level)
    if (ok && (!left_in || xr - kL - kW < 0)) ok = false;
    if (ok) {
      // the right window's 11 rows x 21 columns (xr - 10 .. xr + 10, every shift) staged in
      // this keypoint's LDS by aligned dword loads (6 per row, 66 in all); dwords starting at
      // or past w stay unread (the window ends at xr + 10 <= w - 2; the pitch is >= w + 4)
      __shared__ uint32_t s_rw[kStKP][2 * kW + 1][6];
      __shared__ uint32_t s_lw[kStKP][2 * kW + 1][4];
#pragma unroll
      for (int r = 0; r < KLW; r++) {
        const int i = hl + NG * r;
        if (i < (2 * kW + 1) * 4) s_lw[hw][i >> 2][i & 3] = lw[r];
      }
      const int ar = (xr - 2 * kL) & ~3, ro = (xr - 2 * kL) - ar;  // ar >= 0: xr >= 10
      for (int i = hl; i < (2 * kW + 1) * 6; i += NG) {  // 66 dwords
        const int rr = i / 6, dw = i - rr * 6;
        s_rw[hw][rr][dw] = ar + 4 * dw < G.w
                               ? *(const uint32_t*)(PR + (int64_t)(y0 + rr) * pitch + ar + 4 * dw)
                               : 0u;
      }
      __builtin_amdgcn_wave_barrier();
      const uint8_t* rw = (const uint8_t*)s_rw[hw];  // byte (row, c) at rw[row * 24 + c]
      const uint8_t* lwb = (const uint8_t*)s_lw[hw];  // byte (row, c) at lwb[row * 16 + c]
      const int cL = lwb[kW * 16 + lo + kW];
      int a[KP];
#pragma unroll
      for (int k = 0; k < KP; k++) a[k] = has[k] ? (int)lwb[yy[k] * 16 + lo + xx[k]] - cL : 0;
      int vd[2 * kL + 1];
      int bestSad = INT_MAX, bestinc = 0;
#pragma unroll
      for (int inc = -kL; inc <= kL; inc++) {
        // window column of (xx, inc): xr + inc - kW + xx - (xr - 10) = inc + kL + xx
        const int cR = rw[kW * 24 + ro + inc + 2 * kL];  // the shifted window's centre
        int acc = 0;
#pragma unroll
        for (int k = 0; k < KP; k++) {
          if (has[k]) {
            const int b = (int)rw[yy[k] * 24 + ro + inc + kL + xx[k]] - cR;
            acc += abs(a[k] - b);
          }
        }
        const int dist = grp_sum<NG>(acc);
        vd[inc + kL] = dist;
        if (dist < bestSad) {  // `(float)dist < bestDist(int)`: exact integers
          bestSad = dist;
          bestinc = inc;
        }
      }
      ok = !(bestinc == -kL || bestinc == kL);
      if (ok) {
        const float dist1 = (float)vd[kL + bestinc - 1];
        const float dist2 = (float)vd[kL + bestinc];
        const float dist3 = (float)vd[kL + bestinc + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        ok = !(deltaR < -1 || deltaR > 1);  // NaN passes, as in the reference
        if (ok) {
          float bestuR = G.scale * ((float)scaleduR0 + (float)bestinc + deltaR);
          float disparity = (uL - bestuR);
          if (disparity >= 0 && disparity < maxD) {
            if (disparity <= 0) {
              disparity = 0.01f;
              bestuR = (float)((double)uL - 0.01);  // `uL-0.01` is a double expression
            }
            depth = mbf / disparity;
            uright = bestuR;
            sad_out = bestSad;
          }
        }
      }
    }
  }
  if (live && hl == 0) {
    P.uright[iL] = uright;
    P.depth[iL] = depth;
    P.sad[iL] = sad_out;
  }
}

__global__ __launch_bounds__(256) void k_stereo_filter(const StereoProblem* __restrict__ probs) {
  __shared__ int s_h[256];
  __shared__ int s_sel[2];
  const StereoProblem& P = probs[blockIdx.x];
  const int tid = threadIdx.x;
  const int nl = *P.nl;
  // the (m/2)-th smallest retained SAD: high byte, then low byte (SAD < 121 * 510 < 2^16)
  s_h[tid] = 0;
  __syncthreads();
  for (int i = tid; i < nl; i += 256) {
    const int v = P.sad[i];
    if (v >= 0) atomicAdd(&s_h[(v >> 8) & 255], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int m = 0;
    for (int b = 0; b < 256; b++) m += s_h[b];
    int k = m / 2, b = 0;
    while (b < 256 && k >= s_h[b]) k -= s_h[b++];
    s_sel[0] = m > 0 ? b : -1;
    s_sel[1] = k;
  }
  __syncthreads();
  const int hb = s_sel[0];
  if (hb < 0) return;  // nothing retained (the reference indexes an empty vector)
  const int krem = s_sel[1];
  __syncthreads();
  s_h[tid] = 0;
  __syncthreads();
  for (int i = tid; i < nl; i += 256) {
    const int v = P.sad[i];
    if (v >= 0 && (v >> 8) == hb) atomicAdd(&s_h[v & 255], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int k = krem, b = 0;
    while (k >= s_h[b]) k -= s_h[b++];
    s_sel[0] = (hb << 8) | b;
  }
  __syncthreads();
  const float median = (float)s_sel[0];
  const float c = 1.5f * 1.4f;
  const float thDist = c * median;
  for (int i = tid; i < nl; i += 256) {
    const int v = P.sad[i];
    if (v >= 0 && !((float)v < thDist)) {
      P.uright[i] = -1.0f;
      P.depth[i] = -1.0f;
      P.sad[i] = -1;
    }
  }
}

int launch_stereo(const StereoProblem* d_probs, int nprob, const LevelGeom* d_lv, int nlevels,
                  int nrows, int64_t row_cap, int kp_cap, float mb, float mbf, hipStream_t s) {
  (void)nlevels;
  if (nprob <= 0) return ORBX_OK;
  if (nrows < 1 || (size_t)nrows * 4 > 64 * 1024 || kp_cap > 65535) return ORBX_EUNSUPPORTED;
  hipLaunchKernelGGL(k_stereo_rows, dim3(nprob), dim3(256), (size_t)nrows * 4, s, d_probs, d_lv,
                     nrows, row_cap);
  hipLaunchKernelGGL(k_stereo_match, dim3((kp_cap + kStKP - 1) / kStKP, nprob), dim3(256), 0, s, d_probs,
                     d_lv, nrows, mb, mbf);
  hipLaunchKernelGGL(k_stereo_filter, dim3(nprob), dim3(256), 0, s, d_probs);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_stereo");
}

}  // namespace orbx
