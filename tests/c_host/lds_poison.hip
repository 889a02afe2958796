// Test helper (not part of the product library): fills the whole LDS of
// every CU with one float value, so that a test can check that a kernel run
// right after it does not depend on stale LDS contents
// (tests/test_gpu_fused.py::test_fused_independent_of_stale_lds).
// Built by vad_amd.build.build_c_host() into tests/c_host/liblds_poison.so.
#include <hip/hip_runtime.h>

constexpr int kLdsBytes = 160 * 1024;

__global__ __launch_bounds__(1024) void lds_fill_kernel(float v, float* sink) {
  extern __shared__ float s[];
  volatile float* vs = s;
  for (int i = threadIdx.x; i < kLdsBytes / 4; i += blockDim.x) vs[i] = v;
  __syncthreads();
  // one read back (bit pattern: v may be a NaN), so the stores cannot be
  // treated as dead
  if (threadIdx.x == 0 && __float_as_uint(vs[blockIdx.x % (kLdsBytes / 4)]) != __float_as_uint(v)) sink[0] = 1.f;
}

extern "C" int lds_poison(float v, float* sink, int n_blocks, void* stream) {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&lds_fill_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(lds_fill_kernel, dim3(n_blocks), dim3(1024), kLdsBytes, (hipStream_t)stream, v, sink);
  return (int)hipGetLastError();
}
