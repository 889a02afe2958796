// Semantics check of gfx950 v_permlane{16,32}_swap as xor-16 / xor-32 lane sums.
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ __forceinline__ float xsum16(float p) {
  float q = p;
  asm volatile("" : "+v"(q));  // distinct registers for vdst / vsrc
  auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, p), __builtin_bit_cast(unsigned, q), false, false);
  return __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
}
__device__ __forceinline__ float xsum32(float p) {
  float q = p;
  asm volatile("" : "+v"(q));
  auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, p), __builtin_bit_cast(unsigned, q), false, false);
  return __builtin_bit_cast(float, r[0]) + __builtin_bit_cast(float, r[1]);
}
// inline-asm form: both operands are read and written
__device__ __forceinline__ float xsum16_asm(float p) {
  float a = p, b = p;
  asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return a + b;
}
__device__ __forceinline__ float xsum32_asm(float p) {
  float a = p, b = p;
  asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return a + b;
}
__global__ void k(float* o, const float* a) {
  const float p = a[threadIdx.x];
  o[threadIdx.x] = xsum16(p);
  o[64 + threadIdx.x] = p + __shfl_xor(p, 16);
  o[128 + threadIdx.x] = xsum32(p);
  o[192 + threadIdx.x] = p + __shfl_xor(p, 32);
  o[256 + threadIdx.x] = xsum16_asm(p);
  o[320 + threadIdx.x] = xsum32_asm(p);
}
int main() {
  float h[64], r[384];
  for (int i = 0; i < 64; ++i) h[i] = 1.0f + i * 0.37f + (i * i % 7) * 1e-3f;
  float *da, *dout;
  (void)hipMalloc(&da, 256); (void)hipMalloc(&dout, 1536);
  (void)hipMemcpy(da, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dout, da);
  (void)hipMemcpy(r, dout, 1536, hipMemcpyDeviceToHost);
  int bad16 = 0, bad32 = 0, abad16 = 0, abad32 = 0;
  for (int i = 0; i < 64; ++i) {
    bad16 += r[i] != r[64 + i];
    bad32 += r[128 + i] != r[192 + i];
    abad16 += r[256 + i] != r[64 + i];
    abad32 += r[320 + i] != r[192 + i];
  }
  printf("asm forms: permlane16 mismatches %d, permlane32 mismatches %d\n", abad16, abad32);
  printf("permlane16_swap sum mismatches %d, permlane32_swap sum mismatches %d (lane 0: %g %g / %g %g)\n",
         bad16, bad32, r[0], r[64], r[128], r[192]);
  return (abad16 || abad32) ? 1 : 0;
}
