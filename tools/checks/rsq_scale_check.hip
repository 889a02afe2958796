// Exhaustive check behind features.h's analyser normalisation: for every
// positive normal float x with x * 2^24 finite, v_rsq_f32(x) equals
// v_rsq_f32(x * 2^24) * 2^12 bit for bit (the 2^24 pre-scale that lets the
// features skip rsqrtf's denormal fix-up leaves every normal input's result
// unchanged).  Prints the mismatch count (0 expected) and the first few.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void check(unsigned long long* bad, unsigned* first, unsigned lo, unsigned n) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned bits = lo + i;
  const float x = __builtin_bit_cast(float, bits);
  const float a = __builtin_amdgcn_rsqf(x);
  const float b = __builtin_amdgcn_rsqf(x * 0x1p24f) * 0x1p12f;
  if (__builtin_bit_cast(unsigned, a) != __builtin_bit_cast(unsigned, b)) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k < 8) first[k] = bits;
  }
}

int main() {
  unsigned long long* bad;
  unsigned* first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 32);
  hipMemset(bad, 0, 8);
  hipMemset(first, 0, 32);
  const unsigned lo = 0x00800000u;          // smallest positive normal
  const unsigned hi = (127u + 104u) << 23;  // 2^104: x * 2^24 stays finite below
  const unsigned n = hi - lo;
  hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, bad, first, lo, n);
  unsigned long long h = 0;
  unsigned f[8];
  hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
  printf("checked %u normal floats in [2^-126, 2^104): %llu mismatches\n", n, h);
  for (unsigned k = 0; k < (h < 8 ? h : 8); ++k) printf("  x bits 0x%08x\n", f[k]);
  return h != 0;
}
