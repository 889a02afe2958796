// Co-residency probe: can FFN-shaped work (MFMA + VALU, few VGPRs, no LDS)
// run on the CUs the MFCC kernel occupies (8 waves x 211 VGPRs, 157.7 KB LDS)
// and fill its idle issue slots?  filler_kernel: one wave per 64 threads,
// <= 80 VGPRs (waves_per_eu 6), per "tile" 32 v_mfma_f32_16x16x32_f16 and
// ~256 fp32 VALU operations (the 13-64-64-2 FFN's per-16-window budget).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/micro/coresident.hip -o bin_tmp/libcoresident.so
#include <hip/hip_runtime.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void filler_kernel(float* out, int tiles,
                                                                                              float seed) {
  const int lane = threadIdx.x;
  h8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (_Float16)(seed * (lane + i));
    b[i] = (_Float16)(seed * (lane - i));
  }
  f4 acc[4] = {};
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = seed + lane * 0.25f + i;
  for (int t = 0; t < tiles; ++t) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[m], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaf(v[i], 0.999f, acc[r][i & 3] * 1e-9f);
    }
  }
  float s = 0.f;
  for (int m = 0; m < 4; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 64 + lane] = s;
}

extern "C" int filler_launch(float* out, int blocks, int tiles, void* stream) {
  hipLaunchKernelGGL(filler_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, out, tiles, 1.0f);
  return (int)hipGetLastError();
}
