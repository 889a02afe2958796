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

}  // namespace vad
