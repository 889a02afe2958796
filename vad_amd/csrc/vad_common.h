// Shared device-side definitions for the MI355X (gfx950) VAD hot path.
//
// Everything here is CDNA4-native: 64-lane waves, LDS-staged exchanges,
// f32 MFMA for the FFN.  No CUDA shims, no dual paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vad_amd.h"

namespace vad {

constexpr int kFftN = 512;          // mfcc.py:61 np.fft.fft(frame, 512)
constexpr int kBins = kFftN / 2;    // bins 0..255 kept (Nyquist dropped)
constexpr int kMaxFilters = VAD_MAX_FILTERS;
constexpr int kMaxCoefs = VAD_MAX_MFCC;
constexpr int kMaxTaps = VAD_MAX_TAPS;

// Device-resident MFCC plan.  Read by every wave through scalar loads
// (the indices are wave-uniform), so it lives in plain global memory.
struct MfccDev {
  int n_filters;
  int mfcc_n;
  int wave_fbeg[16];                 // phase-2 filter range per wave
  int wave_fend[16];
  int f_lo[kMaxFilters];             // first tap bin of filter m
  int f_len[kMaxFilters];            // number of taps (contiguous bins)
  int f_off[kMaxFilters];            // offset of filter m's taps in `taps`
  float taps[kMaxTaps];              // filterbank weights (fp32 of the fp64 bank)
  float dct[kMaxCoefs * kMaxFilters];  // lifter(L) x DCT-II ortho, [c][m]
  float2 tw_a[256];                  // W256^(n2*k1), [n2][k1]
  float2 tw_b[256];                  // W512^k
};


typedef float f32x4 __attribute__((ext_vector_type(4)));

// Device view of an FFN plan (passed by value as a kernel argument).
struct FfnDev {
  int n_layers;
  int dims[VAD_MAX_FFN_LAYERS + 1];
  int n_classes;
  int ks0;                        // K-steps of layer 0 = ceil(in_dim / 4) (16 = generic)
  int tiles[VAD_MAX_FFN_LAYERS];  // 16-row output tiles per layer
  const float* frag;              // [slot][64] per-lane fragments: A operands, then biases
};

// Launchers (defined in the .hip translation units).
size_t mfcc_smem_bytes();
hipError_t launch_mfcc(int mode, const MfccDev* plan, int spec, const float* src, int64_t stride,
                       int len, int64_t n, float* out, hipStream_t st);
hipError_t launch_ffn(const FfnDev& net, int src, const float* in, int64_t n_rows, int mfcc_n,
                      int mode, uint8_t* labels, hipStream_t st);
hipError_t launch_stream_ffn(const FfnDev& net, const float* newrow, float* ring, int* count,
                             int64_t n_streams, int mfcc_n, uint8_t* labels, hipStream_t st);
hipError_t launch_features(const float* mfcc, int64_t n_rows, int mfcc_n, int mode, float* out,
                           hipStream_t st);

// ---------------------------------------------------------------------------
// complex helpers (float2 = re, im)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}
// multiply by -i
__device__ __forceinline__ float2 cmul_mi(float2 a) { return make_float2(a.y, -a.x); }
// multiply by +i
__device__ __forceinline__ float2 cmul_pi(float2 a) { return make_float2(-a.y, a.x); }

constexpr float kC8 = 0.70710678118654752440f;   // cos(pi/4)
constexpr float kC16 = 0.92387953251128675613f;  // cos(pi/8)
constexpr float kS16 = 0.38268343236508977173f;  // sin(pi/8)

// forward DFT4 in place (W4 = -i)
__device__ __forceinline__ void dft4(float2& x0, float2& x1, float2& x2, float2& x3) {
  const float2 t0 = cadd(x0, x2), t1 = csub(x0, x2);
  const float2 t2 = cadd(x1, x3), t3 = csub(x1, x3);
  x0 = cadd(t0, t2);
  x2 = csub(t0, t2);
  x1 = cadd(t1, cmul_mi(t3));
  x3 = csub(t1, cmul_mi(t3));
}

// W8^1 * o and W8^3 * o
__device__ __forceinline__ float2 mul_w8_1(float2 o) { return make_float2(kC8 * (o.x + o.y), kC8 * (o.y - o.x)); }
__device__ __forceinline__ float2 mul_w8_3(float2 o) { return make_float2(kC8 * (o.y - o.x), -kC8 * (o.x + o.y)); }

// forward DFT8: x[0..7] -> X[0..7] (natural order), radix-2 over two DFT4s
__device__ __forceinline__ void dft8(float2 (&x)[8]) {
  float2 e0 = x[0], e1 = x[2], e2 = x[4], e3 = x[6];
  float2 o0 = x[1], o1 = x[3], o2 = x[5], o3 = x[7];
  dft4(e0, e1, e2, e3);
  dft4(o0, o1, o2, o3);
  o1 = mul_w8_1(o1);
  o2 = cmul_mi(o2);
  o3 = mul_w8_3(o3);
  x[0] = cadd(e0, o0); x[4] = csub(e0, o0);
  x[1] = cadd(e1, o1); x[5] = csub(e1, o1);
  x[2] = cadd(e2, o2); x[6] = csub(e2, o2);
  x[3] = cadd(e3, o3); x[7] = csub(e3, o3);
}

// W16^e for e in [0,16) as compile-time constants
template <int E>
__device__ __forceinline__ float2 mul_w16(float2 a) {
  constexpr int e = E & 15;
  if constexpr (e == 0) return a;
  else if constexpr (e == 4) return cmul_mi(a);
  else if constexpr (e == 8) return make_float2(-a.x, -a.y);
  else if constexpr (e == 12) return cmul_pi(a);
  else if constexpr (e == 2) return mul_w8_1(a);
  else if constexpr (e == 6) return mul_w8_3(a);
  else if constexpr (e == 10) return make_float2(-kC8 * (a.x + a.y), kC8 * (a.x - a.y));  // W8^5
  else if constexpr (e == 14) return make_float2(kC8 * (a.x - a.y), kC8 * (a.x + a.y));   // W8^7
  else {
    // e odd: cos(2 pi e / 16), -sin(2 pi e / 16)
    constexpr float c = (e == 1 || e == 15) ? kC16 : (e == 3 || e == 13) ? kS16
                      : (e == 5 || e == 11) ? -kS16 : -kC16;
    constexpr float s = (e == 1 || e == 7) ? kS16 : (e == 3 || e == 5) ? kC16
                      : (e == 9 || e == 15) ? -kS16 : -kC16;
    return make_float2(fmaf(a.x, c, a.y * s), fmaf(a.y, c, -a.x * s));
  }
}

// forward DFT16 in place: x[n] -> X[k] (natural order).  4x4 Cooley-Tukey:
// n = 4a + b, k = c + 4d.  Inputs x[n] for n >= NZ are known zeros.
template <int NZ>
__device__ __forceinline__ void dft16(float2 (&x)[16]) {
#pragma unroll
  for (int n = NZ; n < 16; ++n) x[n] = make_float2(0.f, 0.f);
  float2 v[4][4];  // v[b][c]
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    float2 a0 = x[b], a1 = x[4 + b], a2 = x[8 + b], a3 = x[12 + b];
    dft4(a0, a1, a2, a3);
    v[b][0] = a0; v[b][1] = a1; v[b][2] = a2; v[b][3] = a3;
  }
  v[1][1] = mul_w16<1>(v[1][1]); v[1][2] = mul_w16<2>(v[1][2]); v[1][3] = mul_w16<3>(v[1][3]);
  v[2][1] = mul_w16<2>(v[2][1]); v[2][2] = mul_w16<4>(v[2][2]); v[2][3] = mul_w16<6>(v[2][3]);
  v[3][1] = mul_w16<3>(v[3][1]); v[3][2] = mul_w16<6>(v[3][2]); v[3][3] = mul_w16<9>(v[3][3]);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float2 b0 = v[0][c], b1 = v[1][c], b2 = v[2][c], b3 = v[3][c];
    dft4(b0, b1, b2, b3);
    x[c] = b0; x[c + 4] = b1; x[c + 8] = b2; x[c + 12] = b3;
  }
}

// Even half of a DFT16 (outputs k = 2m): DFT8(u[n] + u[n+8]).
__device__ __forceinline__ void dft16_even(const float2 (&u)[16], float2 (&o)[8]) {
#pragma unroll
  for (int n = 0; n < 8; ++n) o[n] = cadd(u[n], u[n + 8]);
  dft8(o);
}

// Odd half of a DFT16 (outputs k = 2m+1): DFT8((u[n] - u[n+8]) W16^n).
__device__ __forceinline__ void dft16_odd(const float2 (&u)[16], float2 (&o)[8]) {
  o[0] = csub(u[0], u[8]);
  o[1] = mul_w16<1>(csub(u[1], u[9]));
  o[2] = mul_w16<2>(csub(u[2], u[10]));
  o[3] = mul_w16<3>(csub(u[3], u[11]));
  o[4] = mul_w16<4>(csub(u[4], u[12]));
  o[5] = mul_w16<5>(csub(u[5], u[13]));
  o[6] = mul_w16<6>(csub(u[6], u[14]));
  o[7] = mul_w16<7>(csub(u[7], u[15]));
  dft8(o);
}

// NaN-keeping ReLU (numpy / Keras keep NaN; fmaxf would drop it).
__device__ __forceinline__ float relu_nan(float x) { return x < 0.f ? 0.f : x; }

}  // namespace vad
