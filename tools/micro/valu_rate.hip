// Microbenchmark: SIMD cycles per wave-instruction of packed vs scalar fp32
// VALU, with 1 or 2 waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ void bench(float* out, unsigned long long* cyc, int iters) {
  v2f a[16];
  float s[32];
  for (int i = 0; i < 16; ++i) a[i] = (v2f){(float)threadIdx.x * i, 1.f + i};
  for (int i = 0; i < 32; ++i) s[i] = (float)threadIdx.x + i;
  const v2f m = (v2f){1.0001f, 0.9999f};
  const v2f c = (v2f){0.5f, 0.25f};
  const float sg = __builtin_amdgcn_readfirstlane((int)threadIdx.x) * 0.5f;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (KIND == 0) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(m), "v"(c));
      if constexpr (KIND == 1) {
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[2 * i]) : "v"(m.x), "v"(c.x));
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[2 * i + 1]) : "v"(m.y), "v"(c.y));
      }
      if constexpr (KIND == 2) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
      if constexpr (KIND == 3) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[i]) : "v"(c.x));
      if constexpr (KIND == 4) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(s[i]) : "v"(m.x), "v"(c.x));
      if constexpr (KIND == 5) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(m));
      if constexpr (KIND == 6) asm volatile("v_fmac_f32_e32 %0, 0x3f812345, %1" : "+v"(s[i]) : "v"(c.x));
      if constexpr (KIND == 7) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(s[i]) : "s"(sg), "v"(c.x));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int i = 0; i < 16; ++i) r += a[i].x + a[i].y;
  for (int i = 0; i < 32; ++i) r += s[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

template <int KIND>
void run(const char* name, int threads) {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 256 * 1024 * 4);
  (void)hipMalloc(&cyc, 256 * 16 * 8);
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    bench<KIND><<<256, threads>>>(out, cyc, iters);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  const int per_iter = (KIND == 1) ? 32 : 16;
  const double instr = (double)iters * per_iter;       // per wave
  const int wps = threads / 256;                        // waves per SIMD
  unsigned long long hc[256 * 16];
  (void)hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost);
  // s_memtime ticks of wave 0 of block 0 over its loop: SIMD cycles per
  // wave-instruction (all waves of the SIMD issuing) and the implied clock
  const double cyc_per = (double)hc[0] / (instr * wps);
  printf("%-14s waves/SIMD=%d  wall ns per wave-instr per SIMD=%.3f  cycles=%.2f  clock=%.2f GHz\n",
         name, wps, best * 1e6 / (instr * wps), cyc_per, cyc_per / (best * 1e6 / (instr * wps)));
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  for (int t : {256, 512, 1024}) {
    run<0>("v_pk_fma_f32", t);
    run<1>("v_fma_f32", t);
    run<2>("v_pk_add_f32", t);
    run<3>("v_add_f32", t);
    run<4>("v_fmac_f32", t);
    run<5>("v_pk_mul_f32", t);
    run<6>("v_fmac literal", t);
    run<7>("v_fmac sgpr", t);
  }
  return 0;
}
