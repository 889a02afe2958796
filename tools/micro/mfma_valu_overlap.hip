// Microbenchmark: does f32 MFMA (v_mfma_f32_16x16x4_f32) on one wave overlap
// with packed-fp32 VALU on the other wave of the same SIMD?
// 512 threads per block = 2 waves per SIMD.  Modes: 0 = both waves VALU,
// 1 = both waves MFMA, 2 = waves 0-3 MFMA + waves 4-7 VALU, 3 = only waves 0-3
// MFMA (others exit), 4 = only waves 4-7 VALU.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ void valu_work(float* out, int iters) {
  v2f a[16];
  for (int i = 0; i < 16; ++i) a[i] = (v2f){(float)threadIdx.x * i, 1.f + i};
  const v2f m = (v2f){1.0001f, 0.9999f}, c = (v2f){0.5f, 0.25f};
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(m), "v"(c));
  float r = 0.f;
  for (int i = 0; i < 16; ++i) r += a[i].x + a[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__device__ void mfma_work(float* out, int iters) {
  v4f acc[4] = {};
  float a = threadIdx.x * 0.001f, b = 1.0f;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // 4 independent accumulators, 4 MFMAs per 16 VALU slots
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
  float r = 0.f;
  for (int i = 0; i < 4; ++i) r += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
// the FFN's MFMA: v_mfma_f32_16x16x32_f16, 4 independent accumulators
__device__ void mfma16_work(float* out, int iters) {
  v4f acc[4] = {};
  h8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(threadIdx.x * 0.001f); b[i] = (_Float16)1.f; }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
  float r = 0.f;
  for (int i = 0; i < 4; ++i) r += acc[i].x + acc[i].y + acc[i].z + acc[i].w;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
// scalar fp32 VALU (the FFN's epilogues are mostly scalar)
__device__ void svalu_work(float* out, int iters) {
  float a[16];
  const float m1 = 1.0001f;
  for (int i = 0; i < 16; ++i) a[i] = (float)threadIdx.x * i;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(a[i]) : "v"(m1));
  float r = 0.f;
  for (int i = 0; i < 16; ++i) r += a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k(float* out, int mode, int iters_v, int iters_m) {
  const int w = threadIdx.x >> 6;
  const bool older = w < 4;
  if (mode == 0) valu_work(out, iters_v);
  else if (mode == 1) mfma_work(out, iters_m);
  else if (mode == 2) { if (older) mfma_work(out, iters_m); else valu_work(out, iters_v); }
  else if (mode == 3) { if (older) mfma_work(out, iters_m); }
  else if (mode == 4) { if (!older) valu_work(out, iters_v); }
  else if (mode == 5) { if (older) valu_work(out, iters_v); else mfma_work(out, iters_m); }
  else if (mode == 6) { if (older) mfma16_work(out, iters_m); }
  else if (mode == 7) { if (!older) svalu_work(out, iters_v); }
  else if (mode == 8) { if (older) mfma16_work(out, iters_m); else svalu_work(out, iters_v); }
  else if (mode == 9) { if (older) svalu_work(out, iters_v); else svalu_work(out, iters_v); }
  else if (mode == 10) { if (older) mfma16_work(out, iters_m); else valu_work(out, iters_v); }
  else if (mode == 11) { if (older) mfma_work(out, iters_m); else svalu_work(out, iters_v); }
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 1024 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iv = 40000;  // 64k pk_fma per wave
  const int im = 20000;  // 8k MFMA per wave (x32 cyc = 256k cyc)
  const char* names[] = {"both VALU", "both MFMA", "old MFMA + young VALU", "old MFMA only",
                         "young VALU only", "old VALU + young MFMA", "old f16 MFMA only",
                         "young scalar VALU only", "old f16 MFMA + young scalar", "both scalar VALU",
                         "old f16 MFMA + young pk", "old f32 MFMA + young scalar"};
  for (int mm = 0; mm < 24; ++mm) {
    const int mode = mm % 12;
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      (void)hipEventRecord(e0);
      k<<<256, 512>>>(out, mode, iv, im);
      (void)hipEventRecord(e1);
      (void)hipDeviceSynchronize();
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    printf("%-24s %.3f ms\n", names[mode], best);
  }
  // waves per SIMD 1 / 2 / 3 / 4 (blocks of 256 / 512 / 768 / 1024 threads,
  // every wave busy): scalar (mode 9) and packed (mode 0) throughput per SIMD
  for (int wps = 1; wps <= 4; ++wps) {
    for (int mode : {9, 0}) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        (void)hipEventRecord(e0);
        k<<<256, 256 * wps>>>(out, mode, iv, im);
        (void)hipEventRecord(e1);
        (void)hipDeviceSynchronize();
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
      }
      // instructions per SIMD: wps waves x iv x 16
      printf("%d waves/SIMD %-7s %.3f ms  %.3f ns per wave-instruction per SIMD\n", wps,
             mode == 9 ? "scalar" : "packed", best, best * 1e6 / (wps * (double)iv * 16));
    }
  }
  return 0;
}
