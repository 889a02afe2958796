// Window features shared by the FFN and decision-tree kernels.
#pragma once

#include "vad_common.h"

namespace vad {

// Feature triple of coefficient c over a 5-frame window a0..a4 (frames
// centre-2 .. centre+2): (Mn, M+1 - M-1, (M+2 - Mn) - (Mn - M-2)) with Mn the
// centre normalised by the window mean / std (ddof 0) in analyser mode
// (sklearn_analyser.py:52-69,103-107) or the raw centre in offline mode
// (file_processing.py:51-66).  fp32 arithmetic, except where a coefficient
// is flat (all five values equal): there the reference's own fp64 formula on
// these fp32 values -- mean = ((((x+x)+x)+x)+x)/5 is exact (every partial sum
// of five floats fits a double), so x - mean = 0 and Mn = 0/0 = NaN, exactly
// as numpy gives on these MFCCs; fp32 rounding of the mean could instead
// leave a tiny non-zero std and a finite Mn, so flatness is tested
// explicitly.  The reference run agrees: in tests/golden/analyser.npz every
// digital-silence window has all 13 Mn (and D2) NaN in the row the reference
// passed to predict, the positions the kernels give (DESIGN.md section 2;
// only the oracle's explicit fp64 DCT matrix rounds a silent coefficient
// differently from frame to frame).
struct Feat3 {
  float mn, d1, d2;
};

__device__ __forceinline__ Feat3 feature_triple(float a0, float a1, float a2, float a3, float a4,
                                                int mode) {
  float mn = a2;
  if (mode == VAD_FEAT_ANALYSER) {
    // e_i = a_i - sum / 5 as one fma each, written out: the rounding every
    // kernel has used (clang contracted a_i - sum * 0.2f), now independent of
    // how a kernel's code is vectorised or scheduled
    const float sum = (((a0 + a1) + a2) + a3) + a4;
    const float e0 = fmaf(sum, -0.2f, a0), e1 = fmaf(sum, -0.2f, a1), e2 = fmaf(sum, -0.2f, a2),
                e3 = fmaf(sum, -0.2f, a3), e4 = fmaf(sum, -0.2f, a4);
    // var * 2^24: v_rsq_f32 on a normal input for every var >= 2^-150,
    // without the denormal-input fix-up rsqrtf wraps around it (five VALU
    // operations per item); the 2^12 goes back into e2 exactly.  For every
    // normal var the result is rsqrtf's bit for bit (v_rsq_f32(x 2^24) 2^12
    // == v_rsq_f32(x) over all 1.93e9 normal x below 2^104 on gfx950,
    // tools/checks/rsq_scale_check.hip).  Range edges (documented at
    // vad_features_f32, locked by test_feature_range_edges): a var whose
    // scaled value overflows (std past ~2^52) gives Mn = 0, squares that
    // underflow (std below ~2^-75) give Mn = +-inf
    const float var_s = fmaf(e4, e4, fmaf(e3, e3, fmaf(e2, e2, fmaf(e1, e1, e0 * e0)))) * (0.2f * 0x1p24f);
    const bool flat = (a0 == a1) & (a1 == a2) & (a2 == a3) & (a3 == a4);
    // branch-free: the NaN is added in rather than selected around the rsqrt
    mn = fmaf(e2 * 0x1p12f, __builtin_amdgcn_rsqf(var_s), flat ? __builtin_nanf("") : 0.f);
  }
  return {mn, a3 - a1, (a4 - mn) - (mn - a0)};
}

// The same triple for kernels that flag NaN windows themselves (the wave
// tile: a flagged window's features go to the MLP as 0 and its logits are
// NaN): Mn without the NaN added in, and `bad` = flat coefficient or a NaN
// Mn (an overflowed var times a zero / infinite e2) -- exactly the windows
// whose feature_triple Mn is NaN, one select cheaper per item.
__device__ __forceinline__ Feat3 feature_triple_flagged(float a0, float a1, float a2, float a3, float a4,
                                                        int mode, bool& bad) {
  if (mode != VAD_FEAT_ANALYSER) {
    bad = false;
    return {a2, a3 - a1, (a4 - a2) - (a2 - a0)};
  }
  const float sum = (((a0 + a1) + a2) + a3) + a4;
  const float e0 = fmaf(sum, -0.2f, a0), e1 = fmaf(sum, -0.2f, a1), e2 = fmaf(sum, -0.2f, a2),
              e3 = fmaf(sum, -0.2f, a3), e4 = fmaf(sum, -0.2f, a4);
  const float var_s = fmaf(e4, e4, fmaf(e3, e3, fmaf(e2, e2, fmaf(e1, e1, e0 * e0)))) * (0.2f * 0x1p24f);
  const bool flat = (a0 == a1) & (a1 == a2) & (a2 == a3) & (a3 == a4);
  const float mn = fmaf(e2 * 0x1p12f, __builtin_amdgcn_rsqf(var_s), 0.f);
  bad = flat | (mn != mn);
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
