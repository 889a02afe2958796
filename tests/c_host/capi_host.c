/*
 * A host that is not Python: plain C against include/vad_amd.h and
 * libvad_amd.so (plus the HIP runtime for device buffers), the way a
 * cgo / JNI / N-API binding of the reference's path would drive it.
 *
 *   capi_host <dir>    reads <dir>/fb.f64 (26 x 256 filterbank, the host
 *                      get_mel_filterbanks), <dir>/audio.f32 (a clip),
 *                      <dir>/mfcc_ref.f32 (the oracle's MFCCs, F x 13),
 *                      <dir>/ffn.f32 + <dir>/labels_ref.u8 (13-64-64-2
 *                      weights, oracle labels where decisive, 255 elsewhere)
 * and checks vad_mfcc_f32, vad_mfcc_ffn (workspace and fused forms), the
 * clip as one stream through vad_stream_hops, and a world-size-1 vad_rccl
 * gather.  Exit status 0 = all checks passed.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vad_amd.h"

#define CHECK(x)                                                         \
  do {                                                                   \
    int rc_ = (int)(x);                                                  \
    if (rc_ != 0) {                                                      \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, rc_); \
      return 1;                                                          \
    }                                                                    \
  } while (0)

static void* slurp(const char* dir, const char* name, size_t* n) {
  char path[1024];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *n = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  void* p = malloc(*n);
  if (fread(p, 1, *n, f) != *n) { free(p); p = NULL; }
  fclose(f);
  return p;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  size_t nfb, na, nm, nw, nl;
  double* fb = (double*)slurp(argv[1], "fb.f64", &nfb);
  float* audio = (float*)slurp(argv[1], "audio.f32", &na);
  float* mref = (float*)slurp(argv[1], "mfcc_ref.f32", &nm);
  float* w = (float*)slurp(argv[1], "ffn.f32", &nw);
  uint8_t* lref = (uint8_t*)slurp(argv[1], "labels_ref.u8", &nl);
  if (!fb || !audio || !mref || !w || !lref) return 3;
  const int64_t n_samples = (int64_t)(na / 4);
  const int64_t F = vad_n_frames(n_samples, 400, 160);
  if ((size_t)F * 13 * 4 != nm || (size_t)(F - 5) != nl) return 4;
  printf("%s: %lld samples, %lld frames\n", vad_version(), (long long)n_samples, (long long)F);

  vad_mfcc_plan* plan = NULL;
  CHECK(vad_mfcc_plan_create(fb, 26, 512, 13, 22, &plan));
  printf("plan variant %d (1 = compiled 26-filter bank)\n", vad_mfcc_plan_variant(plan));
  float *d_audio, *d_mfcc;
  uint8_t *d_lab, *d_lab2;
  void* d_ws;
  CHECK(hipMalloc((void**)&d_audio, na));
  CHECK(hipMalloc((void**)&d_mfcc, nm));
  CHECK(hipMalloc((void**)&d_lab, nl));
  CHECK(hipMalloc((void**)&d_lab2, nl));
  CHECK(hipMemcpy(d_audio, audio, na, hipMemcpyHostToDevice));

  /* get_mfcc of every frame (mfcc.py:67-78) vs the oracle, per-frame norms */
  CHECK(vad_mfcc_f32(plan, d_audio, 160, 400, F, d_mfcc, NULL));
  float* m = (float*)malloc(nm);
  CHECK(hipMemcpy(m, d_mfcc, nm, hipMemcpyDeviceToHost));
  double worst = 0;
  for (int64_t f = 0; f < F; ++f) {
    double num = 0, den = 0;
    for (int c = 0; c < 13; ++c) {
      const double d = (double)m[f * 13 + c] - mref[f * 13 + c];
      num += d * d;
      den += (double)mref[f * 13 + c] * mref[f * 13 + c];
    }
    const double rel = sqrt(num / den);
    if (rel > worst) worst = rel;
  }
  printf("MFCC worst per-frame relative error %.3e\n", worst);
  if (!(worst <= 1e-4)) return 5;

  /* the FFN (Keras layout W (in, out), then b) and the clip labels */
  const int32_t dims[4] = {13, 64, 64, 2};
  const float* W[3] = {w, w + 13 * 64 + 64, w + 13 * 64 + 64 + 64 * 64 + 64};
  const float* B[3] = {w + 13 * 64, w + 13 * 64 + 64 + 64 * 64, w + 13 * 64 + 64 + 64 * 64 + 64 + 64 * 2};
  vad_ffn_plan* ffn = NULL;
  CHECK(vad_ffn_plan_create(3, dims, W, B, &ffn));
  const size_t ws = vad_mfcc_ffn_workspace_bytes(plan, ffn, n_samples, 400, 160);
  CHECK(hipMalloc(&d_ws, ws));
  CHECK(vad_mfcc_ffn(plan, ffn, d_audio, n_samples, 400, 160, VAD_FEAT_ANALYSER, d_lab, d_ws, ws, NULL));
  if (!vad_mfcc_ffn_fusable(plan, ffn, 400, 160)) return 6;
  CHECK(vad_mfcc_ffn(plan, ffn, d_audio, n_samples, 400, 160, VAD_FEAT_ANALYSER, d_lab2, NULL, 0, NULL));
  uint8_t* lab = (uint8_t*)malloc(nl);
  uint8_t* lab2 = (uint8_t*)malloc(nl);
  CHECK(hipMemcpy(lab, d_lab, nl, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(lab2, d_lab2, nl, hipMemcpyDeviceToHost));
  size_t checked = 0;
  for (size_t i = 0; i < nl; ++i) {
    if (lab[i] != lab2[i]) { fprintf(stderr, "fused != two-kernel at %zu\n", i); return 7; }
    if (lref[i] != 255) {
      ++checked;
      if (lab[i] != lref[i]) { fprintf(stderr, "label %zu: %d vs oracle %d\n", i, lab[i], lref[i]); return 8; }
    }
  }
  printf("labels: %zu windows, %zu decisive ones equal the oracle, fused == two-kernel\n", nl, checked);

  /* the streaming form (vad.py:32-59's loop, sklearn_analyser.py:46-82 per
   * hop): the clip as one live stream, 8 hops of 160 new samples per
   * vad_stream_hops call, read in place from the clip; hop t's label is the
   * class of clip window t - 5 (255 for the first five hops) */
  {
    const int K = 8;
    const int64_t T = (F / K) * K;
    float *d_frames, *d_ring;
    int32_t* d_count;
    uint8_t* d_hl;
    CHECK(hipMalloc((void**)&d_frames, 400 * 4));
    CHECK(hipMalloc((void**)&d_ring, 5 * 13 * 4));
    CHECK(hipMalloc((void**)&d_count, 4));
    CHECK(hipMalloc((void**)&d_hl, (size_t)T));
    CHECK(hipMemset(d_frames, 0, 400 * 4));
    CHECK(hipMemcpy(d_frames + 160, d_audio, 240 * 4, hipMemcpyDeviceToDevice));  /* the carry */
    CHECK(hipMemset(d_ring, 0, 5 * 13 * 4));
    CHECK(hipMemset(d_count, 0, 4));
    for (int64_t b = 0; b < T / K; ++b)
      CHECK(vad_stream_hops(plan, ffn, d_frames, 400, 400, d_audio + 240 + 160 * K * b, 160, 160, 1, K, 160,
                            d_ring, d_count, d_hl + K * b, 1, NULL));
    uint8_t* hl = (uint8_t*)malloc((size_t)T);
    CHECK(hipMemcpy(hl, d_hl, (size_t)T, hipMemcpyDeviceToHost));
    size_t hchecked = 0;
    for (int64_t t = 0; t < T; ++t) {
      if (t < 5) {
        if (hl[t] != 255) { fprintf(stderr, "hop %lld: %d before the window fills\n", (long long)t, hl[t]); return 10; }
      } else if (lref[t - 5] != 255) {
        ++hchecked;
        if (hl[t] != lref[t - 5]) {
          fprintf(stderr, "hop %lld: %d vs oracle %d\n", (long long)t, hl[t], lref[t - 5]);
          return 11;
        }
      }
    }
    printf("stream: %lld hops in blocks of %d, %zu decisive labels equal the oracle\n", (long long)T, K, hchecked);
    free(hl);
    CHECK(hipFree(d_frames));
    CHECK(hipFree(d_ring));
    CHECK(hipFree(d_count));
    CHECK(hipFree(d_hl));
  }

  /* the multi-GPU label gather, a group of one */
  if (vad_rccl_available()) {
    char id[VAD_RCCL_ID_BYTES];
    vad_rccl_comm* comm = NULL;
    CHECK(vad_rccl_unique_id(id));
    CHECK(vad_rccl_init(&comm, 1, id, 0));
    CHECK(hipMemset(d_lab2, 0, nl));
    CHECK(vad_rccl_gather_u8(comm, d_lab, d_lab2, nl, 0, NULL));
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(lab2, d_lab2, nl, hipMemcpyDeviceToHost));
    if (memcmp(lab, lab2, nl) != 0) return 9;
    CHECK(vad_rccl_destroy(comm));
    printf("RCCL gather (world 1): ok\n");
  } else {
    printf("RCCL not loadable: gather check skipped\n");
  }
  CHECK(vad_ffn_plan_destroy(ffn));
  CHECK(vad_mfcc_plan_destroy(plan));
  printf("C host: all checks passed\n");
  return 0;
}
