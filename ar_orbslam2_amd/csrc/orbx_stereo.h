// orbx_stereo.h — Frame::ComputeStereoMatches on device-resident extractor outputs
// (orbx_stereo.hip), used by the drop-in orbx_stereo_matches and the stereo frame pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orbx_internal.h"

namespace orbx {

// One stereo frame: left / right keypoints, descriptors and counts of one extraction each,
// and the image blocks of their pitched raw pyramids (mvImagePyramid).
struct StereoProblem {
  const orbx_keypoint* kl;
  const uint8_t* dl;
  const int* nl;
  const orbx_keypoint* kr;
  const uint8_t* dr;
  const int* nr;
  const uint8_t* pyrL;
  const uint8_t* pyrR;
  float* uright;  // [kp_cap] mvuRight
  float* depth;   // [kp_cap] mvDepth
  int* sad;       // [kp_cap] SAD of the retained match, -1 otherwise
  int* row_off;   // scratch [nrows + 1]
  uint2* row_ent;  // scratch [row_cap]: right keypoint (index | octave << 16, x bits)
};

// Rows a right keypoint is registered in (Frame.cc:486-497) are at most this many.
int stereo_row_span(const Geometry& g);
// Scratch sizes for one problem.
void stereo_scratch(const Geometry& g, int kp_cap, int* nrows, int64_t* row_cap);
int launch_stereo(const StereoProblem* d_probs, int nprob, const LevelGeom* d_lv, int nlevels,
                  int nrows, int64_t row_cap, int kp_cap, float mb, float mbf, hipStream_t s);

}  // namespace orbx
