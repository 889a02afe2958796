// Per-frame features of the energy / ZCR / spectral analyser
// (realtime_analysis/simple_analyzer.py: SimpleAnalyser), in fp64 like the
// reference (np.fft.fft of a float64 frame):
//
//   out[0]      stEnergy(frame)               sum x^2 / n            (:162-169, :284-299)
//   out[1]      stZCR(frame) * frame_size     (sum |diff(sign x)| / 2) / (n-1) * n   (:210-215)
//   out[2]      np.std(|fft|)                 over all L bins        (:203-208, :263-273)
//   out[3 + b]  stEnergy(|fft|[b*W:(b+1)*W])  band energies         (:171-197, :319-360)
//
// with |fft| = sqrt(re^2 + im^2) of the L-point DFT of
// [zeros(pad), frame, zeros(pad)] (L = n + 2 pad; pad = 0 -> frame[:fftn])
// (:386-400), stEnergy / stZCR restated from pyAudioAnalysis
// (audioFeatureExtraction.stEnergy / stZCR; the package is absent here).
//
// One 256-thread workgroup per frame: samples and the complex spectrum in
// LDS; a radix-2 FFT when L is a power of two (the reference's 400-sample
// frames: L = 512), a direct DFT otherwise (e.g. 401 samples: L = 513).
#include "vad_common.h"

namespace vad {

constexpr int kSimpleThreads = 256;
constexpr int kSimpleMaxL = 1024;

__device__ double block_sum(double v, double* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int s = kSimpleThreads / 2; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kSimpleThreads) void simple_features_kernel(
    const float* __restrict__ frames, int64_t n_frames, int frame_len, int64_t frame_stride,
    int L, int pad, int band_bins, int n_bands, double* __restrict__ out) {
  __shared__ double re[kSimpleMaxL], im[kSimpleMaxL];
  __shared__ double red[kSimpleThreads];
  const int t = threadIdx.x;
  const bool pow2 = (L & (L - 1)) == 0;
  int log2L = 0;
  while ((1 << log2L) < L) ++log2L;
  const int n_out = 3 + n_bands;
  for (int64_t f = blockIdx.x; f < n_frames; f += gridDim.x) {
    const float* x = frames + f * frame_stride;
    // ---- time-domain features ------------------------------------------
    double e = 0.0, z = 0.0;
    for (int i = t; i < frame_len; i += kSimpleThreads) {
      const double v = (double)x[i];
      e += v * v;
      if (i + 1 < frame_len) {
        const double w = (double)x[i + 1];
        const double sv = (double)((v > 0.0) - (v < 0.0)), sw = (double)((w > 0.0) - (w < 0.0));
        z += fabs(sw - sv);
      }
    }
    e = block_sum(e, red);
    z = block_sum(z, red);
    // ---- spectrum ---------------------------------------------------------
    for (int i = t; i < L; i += kSimpleThreads) {
      const int s = i - pad;  // sample index (pad = 0: the first L samples)
      const double v = (s >= 0 && s < frame_len) ? (double)x[s] : 0.0;
      if (pow2) {
        int r = 0;  // bit-reversed position
        for (int b = 0; b < log2L; ++b) r |= ((i >> b) & 1) << (log2L - 1 - b);
        re[r] = v;
        im[r] = 0.0;
      } else {
        re[i] = v;
      }
    }
    __syncthreads();
    double mag_sum = 0.0;
    if (pow2) {
      for (int len = 2; len <= L; len <<= 1) {  // iterative radix-2 DIT
        const int half = len >> 1;
        for (int b = t; b < (L >> 1); b += kSimpleThreads) {
          const int grp = b / half, k = b - grp * half;
          const int i0 = grp * len + k, i1 = i0 + half;
          double s, c;
          sincospi(-2.0 * (double)k / (double)len, &s, &c);
          const double xr = re[i1] * c - im[i1] * s, xi = re[i1] * s + im[i1] * c;
          const double ar = re[i0], ai = im[i0];
          re[i0] = ar + xr;
          im[i0] = ai + xi;
          re[i1] = ar - xr;
          im[i1] = ai - xi;
        }
        __syncthreads();
      }
      for (int k = t; k < L; k += kSimpleThreads) {
        const double m = sqrt(re[k] * re[k] + im[k] * im[k]);
        mag_sum += m;
        re[k] = m;  // magnitudes replace the real parts
      }
    } else {
      // direct DFT: X[k] = sum_n x[n] exp(-2 pi i (k n mod L) / L)
      double mk[kSimpleMaxL / kSimpleThreads + 1];
      int q = 0;
      for (int k = t; k < L; k += kSimpleThreads, ++q) {
        double ar = 0.0, ai = 0.0;
        int kn = 0;
        for (int n = 0; n < L; ++n) {
          double s, c;
          sincospi(-2.0 * (double)kn / (double)L, &s, &c);
          ar += re[n] * c;
          ai += re[n] * s;
          kn += k;
          if (kn >= L) kn -= L;
        }
        mk[q] = sqrt(ar * ar + ai * ai);
      }
      __syncthreads();
      q = 0;
      for (int k = t; k < L; k += kSimpleThreads, ++q) {
        re[k] = mk[q];
        mag_sum += mk[q];
      }
    }
    __syncthreads();
    const double mean = block_sum(mag_sum, red) / (double)L;
    double ssd = 0.0;
    for (int k = t; k < L; k += kSimpleThreads) {
      const double d = re[k] - mean;
      ssd += d * d;
    }
    ssd = block_sum(ssd, red);
    double* o = out + f * n_out;
    for (int b = 0; b < n_bands; ++b) {
      double be = 0.0;
      for (int k = b * band_bins + t; k < (b + 1) * band_bins; k += kSimpleThreads) be += re[k] * re[k];
      be = block_sum(be, red);
      if (t == 0) o[3 + b] = be / (double)band_bins;
    }
    if (t == 0) {
      o[0] = e / (double)frame_len;
      o[1] = (z * 0.5) / ((double)frame_len - 1.0) * (double)frame_len;
      o[2] = sqrt(ssd / (double)L);
    }
    __syncthreads();
  }
}

hipError_t launch_simple_features(const float* frames, int64_t n_frames, int frame_len,
                                  int64_t frame_stride, int L, int pad, int band_bins, int n_bands,
                                  double* out, hipStream_t st) {
  if (n_frames <= 0) return hipSuccess;
  int64_t blocks = n_frames < 4096 ? n_frames : 4096;
  hipLaunchKernelGGL(simple_features_kernel, dim3((int)blocks), dim3(kSimpleThreads), 0, st, frames,
                     n_frames, frame_len, frame_stride, L, pad, band_bins, n_bands, out);
  return hipGetLastError();
}

}  // namespace vad
