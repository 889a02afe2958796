// Fused MFCC kernel for gfx950: framing -> 512-point real FFT -> |X/512|^2 ->
// sparse mel matvec -> (==0 -> eps) -> log10 -> lifter x DCT-II ortho.
//
// Reference semantics: mfcc.py:59-78 (get_spec_mag, get_mfcc_from_spec,
// lifter), file_processing.py:80-103 (framing).
//
// Work decomposition (one 512-thread workgroup = 8 waves per 64-frame tile):
//   phase 1  16 lanes per frame, 32 frames per pass, 2 passes.
//            The real 512-point FFT is a 256-point complex FFT of
//            z[n] = x[2n] + i x[2n+1] (x[t] = 0 for t >= 400, so z[n >= 200]
//            = 0), split 16 x 16:
//              stage A  lane n2 owns z[16 n1 + n2] (n1 < 13 non-zero), DFT16
//                       in registers, twiddle W256^(n2 k1), store to LDS;
//              stage B  lane j owns the even half of column cE and the odd
//                       half of column cO = 16 - cE (two DFT8s in registers),
//                       so the real-FFT partner Z[256-k] of every Z[k] it
//                       holds is in its own registers (column 0 is the one
//                       exception, handled by a per-lane select);
//              post     X[k] = (S - i W512^k D) / 2, P[k] = |X[k] / 512|^2,
//                       written to an LDS power tile P[64][257].
//   phase 2  one frame per lane, each wave owns a band of filters (balanced
//            by tap count at plan time): wave-uniform tap loop with scalar
//            weights, log10, partial lifter x DCT sums.
//   phase 3  partials of the 8 waves summed through LDS, coalesced store.
#include "vad_common.h"

namespace vad {

constexpr int kTile = 64;        // frames per workgroup tile
constexpr int kThreads = 512;    // 8 waves
constexpr int kWaves = kThreads / 64;
constexpr int kGroups = kThreads / 16;  // frames per phase-1 pass
constexpr int kColStride = 17;   // float2 per LDS column (16 + 1 pad)
constexpr int kGroupScratch = 16 * kColStride;  // float2 per frame group
constexpr int kPStride = kBins + 1;             // floats per P row (bank pad)

enum Mode { kAudioToMfcc = 0, kAudioToSpec = 1, kSpecToMfcc = 2 };

// Load z[16 n1 + n2] = (x[32 n1 + 2 n2], x[32 n1 + 2 n2 + 1]), n1 < NZ.
template <int NZ, bool VEC2>
__device__ __forceinline__ void load_stage_a(const float* __restrict__ fr, int len, int n2,
                                             float2 (&u)[16]) {
#pragma unroll
  for (int n1 = 0; n1 < NZ; ++n1) {
    const int t = 32 * n1 + 2 * n2;
    if constexpr (VEC2) {
      if (t + 1 < len) {
        u[n1] = *reinterpret_cast<const float2*>(fr + t);
      } else {
        u[n1] = make_float2(t < len ? fr[t] : 0.f, 0.f);
      }
    } else {
      u[n1] = make_float2(t < len ? fr[t] : 0.f, t + 1 < len ? fr[t + 1] : 0.f);
    }
  }
}

// Phase 1 for one frame group: power spectrum of frame `fr` into P (LDS row
// or global row, stride 1).  j = lane within the 16-lane group.
template <int NZ, bool VEC2>
__device__ __forceinline__ void frame_power(const MfccDev* __restrict__ plan,
                                            const float* __restrict__ fr, int len, bool valid,
                                            int j, float2* __restrict__ scr,
                                            float* __restrict__ prow) {
  // ---- stage A: DFT16 over n1 for n2 = j -------------------------------
  float2 u[16];
  if (valid) {
    load_stage_a<NZ, VEC2>(fr, len, j, u);
  } else {
#pragma unroll
    for (int n = 0; n < NZ; ++n) u[n] = make_float2(0.f, 0.f);
  }
  dft16<NZ>(u);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) u[k1] = cmul(u[k1], plan->tw_a[j * 16 + k1]);
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) scr[k1 * kColStride + j] = u[k1];
  __builtin_amdgcn_wave_barrier();

  // ---- stage B: even half of column cE, odd half of column cO ----------
  int cE, cO;
  if (j < 14) {
    const int p = (j >> 1) + 1;
    cE = (j & 1) ? 16 - p : p;
    cO = 16 - cE;
  } else {
    cE = cO = (j == 14) ? 0 : 8;
  }
  float2 E[8], O[8];
  {
    float2 col[16];
#pragma unroll
    for (int n = 0; n < 16; ++n) col[n] = scr[cE * kColStride + n];
    dft16_even(col, E);  // E[m] = Z[cE + 32 m]
#pragma unroll
    for (int n = 0; n < 16; ++n) col[n] = scr[cO * kColStride + n];
    dft16_odd(col, O);   // O[m] = Z[cO + 32 m + 16]
  }
  __builtin_amdgcn_wave_barrier();

  // ---- real-FFT split: X[k] = (S - i W^k D)/2, S = a + conj(b), D = a - conj(b)
  const bool col0 = (j == 14);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    {  // slot E[m], bin k = cE + 32 m, partner Z[256 - k]
      const int k = cE + 32 * m;
      const float2 a = E[m];
      const float2 b0 = O[7 - m], b1 = E[(8 - m) & 7];
      const float2 b = make_float2(col0 ? b1.x : b0.x, col0 ? b1.y : b0.y);
      const float2 S = make_float2(a.x + b.x, a.y - b.y);
      const float2 D = make_float2(a.x - b.x, a.y + b.y);
      const float2 T = cmul(D, plan->tw_b[k]);
      const float xr = S.x + T.y, xi = S.y - T.x;
      prow[k] = fmaf(xr, xr, xi * xi) * 0x1p-20f;
    }
    {  // slot O[m], bin k = cO + 32 m + 16
      const int k = cO + 32 * m + 16;
      const float2 a = O[m];
      const float2 b0 = E[7 - m], b1 = O[7 - m];
      const float2 b = make_float2(col0 ? b1.x : b0.x, col0 ? b1.y : b0.y);
      const float2 S = make_float2(a.x + b.x, a.y - b.y);
      const float2 D = make_float2(a.x - b.x, a.y + b.y);
      const float2 T = cmul(D, plan->tw_b[k]);
      const float xr = S.x + T.y, xi = S.y - T.x;
      prow[k] = fmaf(xr, xr, xi * xi) * 0x1p-20f;
    }
  }
}

// Phase 2: frame `lane` of the tile, filters [fb, fe): returns partial
// lifter x DCT sums in acc[].
__device__ __forceinline__ void mel_log_dct(const MfccDev* __restrict__ plan,
                                            const float* __restrict__ prow, int fb, int fe,
                                            float (&acc)[kMaxCoefs]) {
  const float eps = 0x1p-52f;  // np.finfo(float).eps, mfcc.py:74
#pragma unroll
  for (int c = 0; c < kMaxCoefs; ++c) acc[c] = 0.f;
  for (int m = fb; m < fe; ++m) {
    const int lo = plan->f_lo[m], n = plan->f_len[m];
    const float* w = plan->taps + plan->f_off[m];
    float e0 = 0.f, e1 = 0.f;
    int t = 0;
    for (; t + 1 < n; t += 2) {
      e0 = fmaf(w[t], prow[lo + t], e0);
      e1 = fmaf(w[t + 1], prow[lo + t + 1], e1);
    }
    if (t < n) e0 = fmaf(w[t], prow[lo + t], e0);
    float e = e0 + e1;
    e = (e == 0.f) ? eps : e;
    const float lg = __log10f(e);
#pragma unroll
    for (int c = 0; c < kMaxCoefs; ++c) acc[c] = fmaf(plan->dct[c * kMaxFilters + m], lg, acc[c]);
  }
}

template <int MODE, int NZ, bool VEC2>
__global__ __launch_bounds__(kThreads, 1) void mfcc_kernel(
    const MfccDev* __restrict__ plan, const float* __restrict__ src, int64_t frame_stride,
    int frame_len, int64_t n_frames, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* P = reinterpret_cast<float*>(smem);                                   // [64][257]
  float2* scr = reinterpret_cast<float2*>(smem + kTile * kPStride * sizeof(float));
  float* part = reinterpret_cast<float*>(scr);                                 // phase 3 reuse

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int grp = tid >> 4;  // frame group 0..31
  const int j = tid & 15;
  const int len = frame_len < kFftN ? frame_len : kFftN;
  const int mfcc_n = plan->mfcc_n;
  const int64_t n_tiles = (n_frames + kTile - 1) / kTile;

  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    const int64_t f0 = tile * kTile;
    if constexpr (MODE == kSpecToMfcc) {
      // stage the tile's spectra into P (coalesced rows)
      for (int i = tid; i < kTile * kBins; i += kThreads) {
        const int lf = i / kBins, k = i - lf * kBins;
        const int64_t f = f0 + lf;
        P[lf * kPStride + k] = (f < n_frames) ? src[f * kBins + k] : 0.f;
      }
    } else {
#pragma unroll 1
      for (int pass = 0; pass < kTile / kGroups; ++pass) {
        const int lf = pass * kGroups + grp;
        const int64_t f = f0 + lf;
        const bool valid = f < n_frames;
        const float* fr = src + (valid ? f : 0) * frame_stride;
        if constexpr (MODE == kAudioToSpec) {
          float* prow = out + (valid ? f : 0) * kBins;
          if (valid) frame_power<NZ, VEC2>(plan, fr, len, valid, j, scr + grp * kGroupScratch, prow);
        } else {
          frame_power<NZ, VEC2>(plan, fr, len, valid, j, scr + grp * kGroupScratch,
                                P + lf * kPStride);
        }
      }
    }
    if constexpr (MODE != kAudioToSpec) {
      __syncthreads();
      float acc[kMaxCoefs];
      mel_log_dct(plan, P + lane * kPStride, plan->wave_fbeg[wave], plan->wave_fend[wave], acc);
      // part[wave][c][lane]
      for (int c = 0; c < mfcc_n; ++c) part[(wave * kMaxCoefs + c) * 64 + lane] = acc[c];
      __syncthreads();
      const int64_t nf = (n_frames - f0) < kTile ? (n_frames - f0) : kTile;
      for (int i = tid; i < nf * mfcc_n; i += kThreads) {
        const int lf = i / mfcc_n, c = i - lf * mfcc_n;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += part[(w * kMaxCoefs + c) * 64 + lf];
        out[f0 * mfcc_n + i] = s;
      }
      __syncthreads();
    }
  }
}

size_t mfcc_smem_bytes() {
  const size_t p = kTile * kPStride * sizeof(float);  // 65792 B, 16-B multiple
  const size_t s = kGroups * kGroupScratch * sizeof(float2);
  const size_t part = kWaves * kMaxCoefs * 64 * sizeof(float);
  return p + (s > part ? s : part);
}

template <int MODE, int NZ, bool VEC2>
static hipError_t launch_t(const MfccDev* plan, const float* src, int64_t stride, int len,
                           int64_t n, float* out, hipStream_t st) {
  const int64_t n_tiles = (n + kTile - 1) / kTile;
  const int grid = (int)(n_tiles < 4096 ? n_tiles : 4096);
  const size_t smem = mfcc_smem_bytes();
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mfcc_kernel<MODE, NZ, VEC2>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((mfcc_kernel<MODE, NZ, VEC2>), dim3(grid), dim3(kThreads), smem, st, plan,
                     src, stride, len, n, out);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_m(const MfccDev* plan, const float* src, int64_t stride, int len,
                           int64_t n, float* out, hipStream_t st) {
  const int used = len < kFftN ? len : kFftN;
  const bool vec2 = ((reinterpret_cast<uintptr_t>(src) & 7) == 0) && ((stride & 1) == 0);
  if (used <= 32 * 13) {
    return vec2 ? launch_t<MODE, 13, true>(plan, src, stride, len, n, out, st)
                : launch_t<MODE, 13, false>(plan, src, stride, len, n, out, st);
  }
  return vec2 ? launch_t<MODE, 16, true>(plan, src, stride, len, n, out, st)
              : launch_t<MODE, 16, false>(plan, src, stride, len, n, out, st);
}

hipError_t launch_mfcc(int mode, const MfccDev* plan, const float* src, int64_t stride, int len,
                       int64_t n, float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  switch (mode) {
    case kAudioToMfcc: return launch_m<kAudioToMfcc>(plan, src, stride, len, n, out, st);
    case kAudioToSpec: return launch_m<kAudioToSpec>(plan, src, stride, len, n, out, st);
    default: return launch_t<kSpecToMfcc, 13, false>(plan, src, 0, 0, n, out, st);
  }
}

}  // namespace vad
