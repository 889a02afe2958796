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
// Power-of-two L (the reference's 400-sample frames: L = 512): one wave per
// frame (simple_features_wave_kernel, below); otherwise (e.g. 401 samples:
// L = 513) one 256-thread workgroup per frame with a direct DFT.  Frames of
// up to 8192 samples: L <= 8192, or 8193 when the pad is odd.
#include "vad_common.h"

namespace vad {

constexpr int kSimpleThreads = 256;
constexpr int kSimpleMaxL = 8193;
constexpr int kSimpleLds = 160 * 1024;

// Workgroup sum: a butterfly within each wave (DPP / permute shuffles),
// then the four wave partials in a fixed order (deterministic).
__device__ double block_sum(double v, double* red) {
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const double r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// Non-power-of-two L (e.g. 401 samples: L = 513): one workgroup per frame,
// direct DFT (the power-of-two lengths go to simple_features_wave_kernel).
// Dynamic LDS: the padded frame re[L], then the magnitudes mag[L].
__global__ __launch_bounds__(kSimpleThreads) void simple_features_kernel(
    const float* __restrict__ frames, int64_t n_frames, int frame_len, int64_t frame_stride,
    int L, int pad, int band_bins, int n_bands, double* __restrict__ out) {
  extern __shared__ double dsm[];
  double* re = dsm;
  double* mag = dsm + L;
  __shared__ double red[kSimpleThreads / 64];
  const int t = threadIdx.x;
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
    // ---- spectrum: X[k] = sum_n x[n] exp(-2 pi i (k n mod L) / L) -------------
    for (int i = t; i < L; i += kSimpleThreads) {
      const int s = i - pad;  // sample index (pad = 0: the first L samples)
      re[i] = (s >= 0 && s < frame_len) ? (double)x[s] : 0.0;
    }
    __syncthreads();
    double mag_sum = 0.0;
    for (int k = t; k < L; k += kSimpleThreads) {
      double ar = 0.0, ai = 0.0;
      int kn = 0;
      // twiddle exp(-2 pi i kn / L): exact (sincospi) every 16th term, a
      // rotation by exp(-2 pi i k / L) in between -- 16x fewer sincospi than
      // one per term (an 8193-point frame made 67M calls), each twiddle
      // within ~16 roundings of the exact one
      double sk, ck;
      sincospi(-2.0 * (double)k / (double)L, &sk, &ck);
      double s = 0.0, c = 1.0;
      for (int n = 0; n < L; ++n) {
        if ((n & 15) == 0) sincospi(-2.0 * (double)kn / (double)L, &s, &c);
        ar += re[n] * c;
        ai += re[n] * s;
        const double c2 = c * ck - s * sk;
        s = fma(s, ck, c * sk);
        c = c2;
        kn += k;
        if (kn >= L) kn -= L;
      }
      const double m = sqrt(ar * ar + ai * ai);
      mag[k] = m;
      mag_sum += m;
    }
    __syncthreads();
    const double mean = block_sum(mag_sum, red) / (double)L;
    double ssd = 0.0;
    for (int k = t; k < L; k += kSimpleThreads) {
      const double d = mag[k] - mean;
      ssd += d * d;
    }
    ssd = block_sum(ssd, red);
    double* o = out + f * n_out;
    for (int b = 0; b < n_bands; ++b) {
      double be = 0.0;
      for (int k = b * band_bins + t; k < (b + 1) * band_bins; k += kSimpleThreads) be += mag[k] * mag[k];
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

// Power-of-two L (the reference's 400-sample frames: L = 512): one wave per
// frame, no workgroup barriers -- the wave's own LDS slice holds its
// spectrum (LDS operations are in order within a wave), reductions are wave
// butterflies, and the twiddle table is shared by the workgroup.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m);
  return v;
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// tw_lds: the W_L^j table in LDS (L <= 4096); above, each butterfly computes
// its twiddle (the 8192-point frame's two 64 KB arrays fill the LDS).
__global__ __launch_bounds__(kSimpleThreads) void simple_features_wave_kernel(
    const float* __restrict__ frames, int64_t n_frames, int frame_len, int64_t frame_stride,
    int L, int pad, int band_bins, int n_bands, int tw_lds, double* __restrict__ out) {
  extern __shared__ double sm[];  // [L/2] cos, [L/2] sin (tw_lds), then per wave [L] re, [L] im
  double* twc = sm;
  double* tws = sm + (L >> 1);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int waves = blockDim.x >> 6;
  double* re = sm + (tw_lds ? L : 0) + wave * 2 * L;
  double* im = re + L;
  int log2L = 0;
  while ((1 << log2L) < L) ++log2L;
  if (tw_lds) {
    for (int j = threadIdx.x; j < (L >> 1); j += blockDim.x)
      sincospi(-2.0 * (double)j / (double)L, &tws[j], &twc[j]);
  }
  __syncthreads();
  const int n_out = 3 + n_bands;
  const int64_t nw = (int64_t)gridDim.x * waves;
  for (int64_t f = (int64_t)blockIdx.x * waves + wave; f < n_frames; f += nw) {
    const float* x = frames + f * frame_stride;
    double e = 0.0, z = 0.0;
    for (int i = lane; i < frame_len; i += 64) {
      const double v = (double)x[i];
      e += v * v;
      if (i + 1 < frame_len) {
        const double w = (double)x[i + 1];
        const double sv = (double)((v > 0.0) - (v < 0.0)), sw = (double)((w > 0.0) - (w < 0.0));
        z += fabs(sw - sv);
      }
    }
    e = wave_sum(e);
    z = wave_sum(z);
    for (int i = lane; i < L; i += 64) {
      const int sidx = i - pad;
      const double v = (sidx >= 0 && sidx < frame_len) ? (double)x[sidx] : 0.0;
      const int r = (int)(__builtin_bitreverse32((unsigned)i) >> (32 - log2L));
      re[r] = v;
      im[r] = 0.0;
    }
    wave_lds_sync();
    for (int len = 2; len <= L; len <<= 1) {  // iterative radix-2 DIT, as the block kernel
      const int half = len >> 1;
      for (int b = lane; b < (L >> 1); b += 64) {
        const int grp = b / half, k = b - grp * half;
        const int i0 = grp * len + k, i1 = i0 + half;
        const int tw = k * (L / len);
        double c, s;
        if (tw_lds) {
          c = twc[tw];
          s = tws[tw];
        } else {
          sincospi(-2.0 * (double)tw / (double)L, &s, &c);
        }
        const double xr = re[i1] * c - im[i1] * s, xi = re[i1] * s + im[i1] * c;
        const double ar = re[i0], ai = im[i0];
        re[i0] = ar + xr;
        im[i0] = ai + xi;
        re[i1] = ar - xr;
        im[i1] = ai - xi;
      }
      wave_lds_sync();
    }
    double mag_sum = 0.0;
    for (int k = lane; k < L; k += 64) {
      const double m = sqrt(re[k] * re[k] + im[k] * im[k]);
      mag_sum += m;
      re[k] = m;
    }
    const double mean = wave_sum(mag_sum) / (double)L;
    double ssd = 0.0;
    for (int k = lane; k < L; k += 64) {
      const double d = re[k] - mean;
      ssd += d * d;
    }
    ssd = wave_sum(ssd);
    double* o = out + f * n_out;
    for (int b = 0; b < n_bands; ++b) {
      double be = 0.0;
      for (int k = b * band_bins + lane; k < (b + 1) * band_bins; k += 64) be += re[k] * re[k];
      be = wave_sum(be);
      if (lane == 0) o[3 + b] = be / (double)band_bins;
    }
    if (lane == 0) {
      o[0] = e / (double)frame_len;
      o[1] = (z * 0.5) / ((double)frame_len - 1.0) * (double)frame_len;
      o[2] = sqrt(ssd / (double)L);
    }
    wave_lds_sync();  // the next frame overwrites re / im
  }
}

hipError_t launch_simple_features(const float* frames, int64_t n_frames, int frame_len,
                                  int64_t frame_stride, int L, int pad, int band_bins, int n_bands,
                                  double* out, hipStream_t st) {
  if (n_frames <= 0) return hipSuccess;
  if (L > kSimpleMaxL) return hipErrorInvalidValue;
  if ((L & (L - 1)) == 0) {
    // waves per block: as many (up to 4) as the LDS holds beside the twiddle
    // table (L = 512: 36 KB; 2048: 144 KB; 4096: 32 KB of twiddles + two
    // waves x 64 KB = 160 KB, the whole budget -- the kernel declares no
    // static LDS, checked below; 8192: one wave, 128 KB, twiddles computed
    // per butterfly)
    const int tw_lds = L <= 4096;
    const size_t tw_bytes = tw_lds ? (size_t)L * sizeof(double) : 0;
    const size_t wave_bytes = (size_t)2 * L * sizeof(double);
    int waves = 4;
    while (waves > 1 && tw_bytes + waves * wave_bytes > (size_t)kSimpleLds) --waves;
    const size_t smem = tw_bytes + waves * wave_bytes;
    static size_t static_lds = ~(size_t)0;  // the kernel's own __shared__ bytes (0 today)
    if (static_lds == ~(size_t)0) {
      hipFuncAttributes fa{};
      if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&simple_features_wave_kernel)) != hipSuccess)
        return hipErrorInvalidValue;
      static_lds = fa.sharedSizeBytes;
    }
    if (smem + static_lds > (size_t)kSimpleLds) return hipErrorInvalidValue;
    static std::atomic<unsigned long long> attr_done{0};
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&simple_features_wave_kernel), kSimpleLds, attr_done);
    if (e != hipSuccess) return e;
    int64_t blocks = (n_frames + waves - 1) / waves;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(simple_features_wave_kernel, dim3((int)blocks), dim3(64 * waves), smem, st,
                       frames, n_frames, frame_len, frame_stride, L, pad, band_bins, n_bands, tw_lds, out);
    return hipGetLastError();
  }
  static std::atomic<unsigned long long> attr_done_d{0};
  const size_t smem = (size_t)2 * L * sizeof(double);  // L = 8193: 128 KB
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&simple_features_kernel), kSimpleLds - 1024, attr_done_d);
  if (e != hipSuccess) return e;
  int64_t blocks = n_frames < 4096 ? n_frames : 4096;
  hipLaunchKernelGGL(simple_features_kernel, dim3((int)blocks), dim3(kSimpleThreads), smem, st, frames,
                     n_frames, frame_len, frame_stride, L, pad, band_bins, n_bands, out);
  return hipGetLastError();
}

}  // namespace vad
