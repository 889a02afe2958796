// Spectra and MFCCs for any FFT length (mfcc.py:59-78 with fft_n other than
// 512).  get_spec_mag takes np.fft.fft(frame, fft_n)[0:fft_n/2] / fft_n and
// squares its magnitude; every reference call site passes 512 (config.py:27,
// sklearn_analyser.py:21), which runs the radix-16 x 16 kernels
// (mfcc_kernel.hip).  This path serves the other lengths the API accepts:
// a direct DFT per frame, fp64 accumulation against a per-plan fp64 twiddle
// table, then the plan's sparse mel taps, (== 0 -> eps), log10 and
// lifter x DCT.  One 256-thread block per frame (grid-stride over frames).
#include "vad_common.h"

namespace vad {

enum GenericMode { kGenMfcc = 0, kGenSpec = 1, kGenSpecToMfcc = 2 };

template <typename TIN, int MODE>
__global__ __launch_bounds__(256) void generic_mfcc_kernel(const MfccDev* __restrict__ plan,
                                                           const TIN* __restrict__ src, int64_t stride,
                                                           int len, int64_t n, int fft_n, int bins,
                                                           const double2* __restrict__ tw,
                                                           float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
  const int L = len < fft_n ? len : fft_n;  // zero-padded, or truncated to fft_n samples
  double* x = reinterpret_cast<double*>(gsm);                                // [L]
  float* P = reinterpret_cast<float*>(gsm + sizeof(double) * (size_t)fft_n);  // [bins]
  float* lm = P + bins;                                                       // [n_filters]
  const int nf = plan->n_filters, mfcc_n = plan->mfcc_n;
  for (int64_t f = blockIdx.x; f < n; f += gridDim.x) {
    if constexpr (MODE == kGenSpecToMfcc) {
      for (int k = threadIdx.x; k < bins; k += blockDim.x) P[k] = (float)src[f * stride + k];
    } else {
      for (int t = threadIdx.x; t < L; t += blockDim.x) x[t] = (double)(float)src[f * stride + t];
      __syncthreads();
      // X[k] = sum_t x[t] W^(k t), W = exp(-2 pi i / fft_n); the table index
      // k t mod fft_n advances by k per sample
      for (int k = threadIdx.x; k < bins; k += blockDim.x) {
        double re = 0.0, im = 0.0;
        int idx = 0;
        for (int t = 0; t < L; ++t) {
          const double2 w = tw[idx];
          re = fma(x[t], w.x, re);
          im = fma(x[t], w.y, im);
          idx += k;
          if (idx >= fft_n) idx -= fft_n;
        }
        const double inv = 1.0 / (double)fft_n;
        re *= inv;
        im *= inv;
        const float p = (float)fma(re, re, im * im);
        if constexpr (MODE == kGenSpec) out[f * bins + k] = p;
        else P[k] = p;
      }
    }
    if constexpr (MODE != kGenSpec) {
      __syncthreads();
      // mel energies (the plan's taps over contiguous bin ranges), mfcc.py:73-75
      for (int m = threadIdx.x; m < nf; m += blockDim.x) {
        const int lo = plan->f_lo[m], nt = plan->f_len[m];
        const float* w = plan->taps + plan->f_off[m];
        float e = 0.f;
        for (int t = 0; t < nt; ++t) e = fmaf(w[t], P[lo + t], e);
        e = (e == 0.f) ? 0x1p-52f : e;  // np.finfo(float).eps
        lm[m] = log10f(e);
      }
      __syncthreads();
      // lifter x DCT-II ortho, mfcc.py:76-78
      for (int c = threadIdx.x; c < mfcc_n; c += blockDim.x) {
        const float* d = plan->dct + c * kMaxFilters;
        float acc = 0.f;
        for (int m = 0; m < nf; ++m) acc = fmaf(d[m], lm[m], acc);
        out[f * mfcc_n + c] = acc;
      }
    }
    __syncthreads();  // x, P and lm are reused by the next frame
  }
}

size_t generic_smem_bytes(int fft_n, int bins) {
  return sizeof(double) * (size_t)fft_n + sizeof(float) * ((size_t)bins + kMaxFilters);
}

template <typename TIN, int MODE>
static hipError_t launch_generic_t(const MfccDev* plan, const TIN* src, int64_t stride, int len, int64_t n,
                                   int fft_n, const double2* tw, float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int bins = fft_n / 2;
  const size_t smem = generic_smem_bytes(fft_n, bins);
  static std::atomic<unsigned long long> attr_done{0};
  const hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&generic_mfcc_kernel<TIN, MODE>),
                                      (int)generic_smem_bytes(kMaxGenericFft, kMaxGenericFft / 2), attr_done);
  if (e != hipSuccess) return e;
  const int64_t grid = n < 4096 ? n : 4096;
  hipLaunchKernelGGL((generic_mfcc_kernel<TIN, MODE>), dim3((unsigned)grid), dim3(256), smem, st, plan, src, stride,
                     len, n, fft_n, bins, tw, out);
  return hipGetLastError();
}

// mode: 0 frames -> MFCC, 1 frames -> spectra, 2 spectra (stride = bins) -> MFCC
hipError_t launch_generic(int mode, const MfccDev* plan, const float* src, int64_t stride, int len, int64_t n,
                          int fft_n, const double2* tw, float* out, hipStream_t st) {
  switch (mode) {
    case kGenMfcc: return launch_generic_t<float, kGenMfcc>(plan, src, stride, len, n, fft_n, tw, out, st);
    case kGenSpec: return launch_generic_t<float, kGenSpec>(plan, src, stride, len, n, fft_n, tw, out, st);
    default: return launch_generic_t<float, kGenSpecToMfcc>(plan, src, stride, len, n, fft_n, tw, out, st);
  }
}

hipError_t launch_generic_i16(int mode, const MfccDev* plan, const int16_t* src, int64_t stride, int len,
                              int64_t n, int fft_n, const double2* tw, float* out, hipStream_t st) {
  if (mode == kGenSpec) return launch_generic_t<int16_t, kGenSpec>(plan, src, stride, len, n, fft_n, tw, out, st);
  return launch_generic_t<int16_t, kGenMfcc>(plan, src, stride, len, n, fft_n, tw, out, st);
}

}  // namespace vad
