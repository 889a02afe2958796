// Window features shared by the FFN and decision-tree kernels.
#pragma once

#include "vad_common.h"

namespace vad {

// Feature triple of coefficient c over a 5-frame window a0..a4 (frames
// centre-2 .. centre+2): (Mn, M+1 - M-1, (M+2 - Mn) - (Mn - M-2)) with Mn the
// centre normalised by the window mean / std (ddof 0) in analyser mode
// (sklearn_analyser.py:52-69,103-107) or the raw centre in offline mode
// (file_processing.py:51-66).  fp32 arithmetic; the reference's fp64 std is 0
// exactly when all five values are equal (0/0 = NaN there), so that case is
// tested explicitly instead of relying on fp32 rounding of the mean.
struct Feat3 {
  float mn, d1, d2;
};

__device__ __forceinline__ Feat3 feature_triple(float a0, float a1, float a2, float a3, float a4,
                                                int mode) {
  float mn = a2;
  if (mode == VAD_FEAT_ANALYSER) {
    const float mean = ((((a0 + a1) + a2) + a3) + a4) * 0.2f;
    const float e0 = a0 - mean, e1 = a1 - mean, e2 = a2 - mean, e3 = a3 - mean, e4 = a4 - mean;
    const float var = fmaf(e4, e4, fmaf(e3, e3, fmaf(e2, e2, fmaf(e1, e1, e0 * e0)))) * 0.2f;
    const bool flat = (a0 == a1) & (a1 == a2) & (a2 == a3) & (a3 == a4);
    // branch-free: the NaN is added in rather than selected around the rsqrt
    mn = e2 * rsqrtf(var) + (flat ? __builtin_nanf("") : 0.f);
  }
  return {mn, a3 - a1, (a4 - mn) - (mn - a0)};
}

// Feature f (0 .. 3*mfcc_n-1) of the window whose 5 MFCC rows are r0..r4.
__device__ __forceinline__ float window_feature(const float* __restrict__ r0,
                                               const float* __restrict__ r1,
                                               const float* __restrict__ r2,
                                               const float* __restrict__ r3,
                                               const float* __restrict__ r4, int f, int mfcc_n,
                                               int mode) {
  const int t = f / mfcc_n;
  const int c = f - t * mfcc_n;
  const Feat3 ft = feature_triple(r0[c], r1[c], r2[c], r3[c], r4[c], mode);
  return t == 0 ? ft.mn : t == 1 ? ft.d1 : ft.d2;
}

}  // namespace vad
