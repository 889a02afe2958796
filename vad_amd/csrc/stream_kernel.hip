// Streaming frame assembly: every stream's frame buffer advances by one hop
// (the oldest `hop` samples drop out, the new ones are appended), i.e. the
// frame that SKLearnAnalyzer.feed_frame (sklearn_analyser.py:46-82) receives
// when vad.py:37-49 cuts the live signal into 25 ms frames every 10 ms.
//
// One wave per stream, in place: the wave loads its whole row into
// registers, then stores it shifted.  Store i (sample t = lane + 64 i) waits
// for its own load, hence for every older load of the wave (vmcnt is in
// order), and a younger load i2 > i reads samples >= 64 i2 + hop > 64 i + 63,
// beyond anything store i writes -- so no sample is overwritten before it is
// read.
#include "vad_common.h"

namespace vad {

template <int NR>  // registers per lane: frame_len <= 64 NR
__global__ __launch_bounds__(256) void stream_push_kernel(float* __restrict__ frames, int64_t fstride,
                                                          int len, const float* __restrict__ hop,
                                                          int64_t hstride, int hlen, int64_t n_streams) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= n_streams) return;
  float* row = frames + s * fstride;
  const float* h = hop + s * hstride;
  const int keep = len - hlen;
  float v[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = lane + 64 * i;
    v[i] = t < keep ? row[t + hlen] : (t < len ? h[t - keep] : 0.f);
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = lane + 64 * i;
    if (t < len) row[t] = v[i];
  }
}

hipError_t launch_stream_push(float* frames, int64_t fstride, int len, const float* hop, int64_t hstride,
                              int hlen, int64_t n_streams, hipStream_t st) {
  if (n_streams <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n_streams + 3) / 4));
  if (len <= 64 * 7)
    hipLaunchKernelGGL(stream_push_kernel<7>, grid, dim3(256), 0, st, frames, fstride, len, hop, hstride,
                       hlen, n_streams);
  else
    hipLaunchKernelGGL(stream_push_kernel<16>, grid, dim3(256), 0, st, frames, fstride, len, hop, hstride,
                       hlen, n_streams);
  return hipGetLastError();
}

// Optional pre-emphasis (not in the reference pipeline, mfcc.py:59-61; the
// python_speech_features convention): y[0] = x[0], y[t] = x[t] - a x[t-1]
// along each row (a whole clip is one row).  Elementwise, 16-B vector loads
// of four samples plus the one before them; out of place.
__global__ __launch_bounds__(256) void preemphasis_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                          int64_t n_rows, int64_t row_len, int64_t stride,
                                                          float a) {
#pragma clang fp contract(off)  // a rounded product, then the difference: numpy's two roundings
  const int64_t quads = (row_len + 3) / 4;
  const int64_t total = n_rows * quads;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / quads, q = i - r * quads;
    const float* xr = x + r * stride;
    float* yr = y + r * stride;
    const int64_t t0 = 4 * q;
    float prev = t0 > 0 ? xr[t0 - 1] : 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t t = t0 + k;
      if (t < row_len) {
        const float v = xr[t];
        yr[t] = t == 0 ? v : v - a * prev;
        prev = v;
      }
    }
  }
}

hipError_t launch_preemphasis(const float* x, float* y, int64_t n_rows, int64_t row_len, int64_t stride, float a,
                              hipStream_t st) {
  if (n_rows <= 0 || row_len <= 0) return hipSuccess;
  int64_t blocks = (n_rows * ((row_len + 3) / 4) + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(preemphasis_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, y, n_rows, row_len, stride,
                     a);
  return hipGetLastError();
}

}  // namespace vad
