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
//                    incR = -5..5 (121 pixels across lanes, one wave reduction per shift; the
//                    centred float windows of the reference have integer entries, so the
//                    integer SAD equals cv::norm(IL, IR, NORM_L1) exactly), parabola fit in f32
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
      if (slot < row_cap) P.row_idx[slot] = i;
    }
  }
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(256) void k_stereo_match(const StereoProblem* __restrict__ probs,
                                                      const LevelGeom* __restrict__ lv,
                                                      int nrows, float mb, float mbf) {
  const StereoProblem& P = probs[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int iL = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nl = *P.nl;
  if (iL >= nl) return;
  const orbx_keypoint kpL = P.kl[iL];
  float uright = -1.0f, depth = -1.0f;
  int sad_out = -1;
  const float minZ = mb, minD = -3.0f;
  const float maxD = mbf / minZ;
  const float vL = kpL.y, uL = kpL.x;
  const int levelL = kpL.octave;
  const int row = (int)vL;  // vRowIndices[vL]: float -> index truncation
  bool ok = row >= 0 && row < nrows;
  int bestDist = kTH_HIGH, bestIdxR = 0;
  const float minU = uL - maxD, maxU = uL - minD;
  if (ok && maxU < 0) ok = false;
  if (ok) {
    const int c0 = P.row_off[row], c1 = P.row_off[row + 1];
    const uint64_t* q = (const uint64_t*)(P.dl + (int64_t)iL * 32);
    const uint64_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
    int key = INT_MAX;  // (distance << 16) | right index: first minimum in right-index order
    for (int j = c0 + lane; j < c1; j += 64) {
      const int iR = P.row_idx[j];
      const orbx_keypoint kpR = P.kr[iR];
      if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
      const float uR = kpR.x;
      if (uR >= minU && uR <= maxU) {
        const uint64_t* r = (const uint64_t*)(P.dr + (int64_t)iR * 32);
        const int dist = __popcll(d0 ^ r[0]) + __popcll(d1 ^ r[1]) + __popcll(d2 ^ r[2]) +
                         __popcll(d3 ^ r[3]);
        key = min(key, (dist << 16) | iR);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) key = min(key, __shfl_xor(key, o));
    if (key != INT_MAX && (key >> 16) < bestDist) {
      bestDist = key >> 16;
      bestIdxR = key & 0xFFFF;
    }
    ok = bestDist < kTH_HIGH;
  }
  if (ok) {  // subpixel match by correlation (Frame.cc:555-618)
    const LevelGeom& G = lv[levelL];
    const float uR0 = P.kr[bestIdxR].x;
    const float scaleFactor = G.inv_scale;
    const float scaleduL = roundf(kpL.x * scaleFactor);
    const float scaledvL = roundf(kpL.y * scaleFactor);
    const float scaleduR0 = roundf(uR0 * scaleFactor);
    const float iniu = scaleduR0 + kL - kW;
    const float endu = scaleduR0 + kL + kW + 1;
    const int y0 = (int)scaledvL - kW, xl0 = (int)scaleduL - kW, xr = (int)scaleduR0;
    ok = !(iniu < 0 || endu >= G.w);
    // windows the reference would take with cv::Mat ranges (they assert inside the level)
    if (ok && (y0 < 0 || y0 + 2 * kW >= G.h || xl0 < 0 || xl0 + 2 * kW >= G.w ||
               xr - kL - kW < 0))
      ok = false;
    if (ok) {
      const uint8_t* PL = P.pyrL + G.pyr_off;
      const uint8_t* PR = P.pyrR + G.pyr_off;
      const int64_t pitch = G.pitch;
      const int cL = PL[(int64_t)(y0 + kW) * pitch + xl0 + kW];
      // centres of the 11 shifted right windows, one per lane, broadcast below
      const int cRl = lane < 2 * kL + 1 ? PR[(int64_t)(y0 + kW) * pitch + xr + lane - kL] : 0;
      int a[2], yy[2], xx[2];
      bool has[2];
#pragma unroll
      for (int k = 0; k < 2; k++) {
        const int p = lane + 64 * k;
        has[k] = p < (2 * kW + 1) * (2 * kW + 1);
        yy[k] = has[k] ? p / (2 * kW + 1) : 0;
        xx[k] = has[k] ? p - yy[k] * (2 * kW + 1) : 0;
        a[k] = has[k] ? (int)PL[(int64_t)(y0 + yy[k]) * pitch + xl0 + xx[k]] - cL : 0;
      }
      int vd[2 * kL + 1];
      int bestSad = INT_MAX, bestinc = 0;
#pragma unroll
      for (int inc = -kL; inc <= kL; inc++) {
        const int cR = __shfl(cRl, inc + kL);
        int acc = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
          if (has[k]) {
            const int b = (int)PR[(int64_t)(y0 + yy[k]) * pitch + xr + inc - kW + xx[k]] - cR;
            acc += abs(a[k] - b);
          }
        }
        const int dist = wave_sum(acc);
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
  if (lane == 0) {
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
  hipLaunchKernelGGL(k_stereo_match, dim3((kp_cap + 3) / 4, nprob), dim3(256), 0, s, d_probs,
                     d_lv, nrows, mb, mbf);
  hipLaunchKernelGGL(k_stereo_filter, dim3(nprob), dim3(256), 0, s, d_probs);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? ORBX_OK : report_hip(e, "launch_stereo");
}

}  // namespace orbx
