// Offline dataset export: scale_features (reference dataset/utils.py:5-34)
// on device.  Feature rows are [mfcc(C) | delta1(C) | delta2(C)]
// (file_processing.py:51-66 layout, as vad_features_f32 mode OFFLINE emits
// them); one global mean and one population std (np.std, ddof 0) per group
// over every value of the chunk, then x = (x - mean) / std in place.
//
// Statistics in fp64 (the reference's arrays are float64) with a fixed
// reduction order: kScaleBlocks block partials, summed in block order by one
// thread per group -- deterministic run to run.  Two passes (mean, then the
// sum of squared deviations), as np.std computes it.
#include "vad_common.h"

namespace vad {

constexpr int kScaleBlocks = 1024;
constexpr int kScaleThreads = 256;

// pass 0: sums; pass 1: squared deviations from stats[0..2]
template <int PASS>
__global__ __launch_bounds__(kScaleThreads) void scale_partials_kernel(
    const float* __restrict__ x, int64_t n_rows, int mfcc_n, const double* __restrict__ stats,
    double* __restrict__ partials) {
  __shared__ double red[3][kScaleThreads];
  const int row_len = 3 * mfcc_n;
  const int64_t total = n_rows * row_len;
  double acc[3] = {0.0, 0.0, 0.0};
  double mean[3] = {0.0, 0.0, 0.0};
  if (PASS == 1) {
    mean[0] = stats[0];
    mean[1] = stats[1];
    mean[2] = stats[2];
  }
  for (int64_t i = (int64_t)blockIdx.x * kScaleThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kScaleThreads) {
    const int64_t r = i / row_len;
    const int g = (int)((i - r * row_len) / mfcc_n);
    const double v = (double)x[i];
    const double d = PASS == 0 ? v : v - mean[g];
    const double term = PASS == 0 ? d : d * d;
    acc[0] += g == 0 ? term : 0.0;
    acc[1] += g == 1 ? term : 0.0;
    acc[2] += g == 2 ? term : 0.0;
  }
  for (int g = 0; g < 3; ++g) red[g][threadIdx.x] = acc[g];
  __syncthreads();
  for (int s = kScaleThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int g = 0; g < 3; ++g) red[g][threadIdx.x] += red[g][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < 3) partials[blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x][0];
}

// stats[0..2] = mean (PASS 0) or stats[3..5] = std (PASS 1)
template <int PASS>
__global__ void scale_finalize_kernel(const double* __restrict__ partials, int n_blocks,
                                      int64_t per_group, double* __restrict__ stats) {
  const int g = threadIdx.x;
  if (g >= 3) return;
  double s = 0.0;
  for (int b = 0; b < n_blocks; ++b) s += partials[b * 3 + g];
  const double m = s / (double)per_group;
  if (PASS == 0) stats[g] = m;
  else stats[3 + g] = sqrt(m);
}

__global__ __launch_bounds__(kScaleThreads) void scale_apply_kernel(float* __restrict__ x,
                                                                    int64_t n_rows, int mfcc_n,
                                                                    const double* __restrict__ stats) {
  const int row_len = 3 * mfcc_n;
  const int64_t total = n_rows * row_len;
  const double m[3] = {stats[0], stats[1], stats[2]};
  const double sd[3] = {stats[3], stats[4], stats[5]};
  for (int64_t i = (int64_t)blockIdx.x * kScaleThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kScaleThreads) {
    const int64_t r = i / row_len;
    const int g = (int)((i - r * row_len) / mfcc_n);
    x[i] = (float)(((double)x[i] - m[g]) / sd[g]);  // std 0 -> inf / nan, like numpy
  }
}

size_t scale_workspace_bytes() { return (size_t)(kScaleBlocks * 3 + 6) * sizeof(double); }

hipError_t launch_scale_features(float* x, int64_t n_rows, int mfcc_n, double* ws, hipStream_t st) {
  if (n_rows <= 0) return hipSuccess;
  double* partials = ws;
  double* stats = ws + kScaleBlocks * 3;
  const int64_t per_group = n_rows * mfcc_n;
  hipLaunchKernelGGL(scale_partials_kernel<0>, dim3(kScaleBlocks), dim3(kScaleThreads), 0, st, x,
                     n_rows, mfcc_n, stats, partials);
  hipLaunchKernelGGL(scale_finalize_kernel<0>, dim3(1), dim3(64), 0, st, partials, kScaleBlocks,
                     per_group, stats);
  hipLaunchKernelGGL(scale_partials_kernel<1>, dim3(kScaleBlocks), dim3(kScaleThreads), 0, st, x,
                     n_rows, mfcc_n, stats, partials);
  hipLaunchKernelGGL(scale_finalize_kernel<1>, dim3(1), dim3(64), 0, st, partials, kScaleBlocks,
                     per_group, stats);
  int64_t blocks = (n_rows * 3 * mfcc_n + kScaleThreads - 1) / kScaleThreads;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(scale_apply_kernel, dim3((int)blocks), dim3(kScaleThreads), 0, st, x, n_rows,
                     mfcc_n, stats);
  return hipGetLastError();
}

}  // namespace vad
