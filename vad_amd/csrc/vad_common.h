// Shared device-side definitions for the MI355X (gfx950) VAD hot path.
//
// Everything here is CDNA4-native: 64-lane waves, LDS-staged exchanges,
// f32 MFMA for the FFN.  No CUDA shims, no dual paths.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "../../include/vad_amd.h"

namespace vad {

constexpr int kFftN = 512;          // mfcc.py:61 np.fft.fft(frame, 512)
constexpr int kBins = kFftN / 2;    // bins 0..255 kept (Nyquist dropped)
constexpr int kMaxFilters = VAD_MAX_FILTERS;
constexpr int kMaxCoefs = VAD_MAX_MFCC;
constexpr int kMaxTaps = VAD_MAX_TAPS;
constexpr int kMaxGenericFft = VAD_MAX_FFT_N;  // other FFT lengths: spec_generic.hip

// Device-resident MFCC plan.  Read by every wave through scalar loads
// (the indices are wave-uniform), so it lives in plain global memory.
struct MfccDev {
  int n_filters;
  int mfcc_n;
  int wave_fbeg[16];                 // phase-2 filter range per wave
  int wave_fend[16];
  int f_lo[kMaxFilters];             // first tap bin of filter m
  int f_len[kMaxFilters];            // number of taps (contiguous bins)
  int f_off[kMaxFilters];            // offset of filter m's taps in `taps`
  float taps[kMaxTaps];              // filterbank weights (fp32 of the fp64 bank)
  float dct[kMaxCoefs * kMaxFilters];  // lifter(L) x DCT-II ortho, [c][m]
  float2 tw_a[256];                  // W256^(n2*k1), [n2][k1]
  float2 tw_b[256];                  // W512^k
  float window[kFftN];               // optional analysis window (kSpecWindow plans), 0 past the frame
};

// plan variant of a plan with an analysis window (vad_mfcc_plan_set_window)
constexpr int kSpecWindow = 3;
// the launch-time form of a windowed plan whose filterbank is also the
// compiled 26 / 40-filter bank (capi.hip launch_spec): the reference framing
// then runs the paired-frame kernel with those tables and the window
constexpr int kSpecWindow26 = 5;
constexpr int kSpecWindow40 = 6;


typedef float f32x4 __attribute__((ext_vector_type(4)));

// Device view of an FFN plan (passed by value as a kernel argument).
struct FfnDev {
  int n_layers;
  int dims[VAD_MAX_FFN_LAYERS + 1];
  int n_classes;
  int ks0;                        // K-steps of layer 0 = ceil(in_dim / 4) (16 = generic)
  int tiles[VAD_MAX_FFN_LAYERS];  // 16-row output tiles per layer
  const float* frag;              // [slot][64] per-lane fragments: A operands, then biases
  // split-f16 MFMA weights (ref39 / bl13; null = exact f32 MFMA only):
  // [slot][64 lanes][4 words] of packed f16, slot = ((layer, mt, s), hi | lo)
  const uint32_t* fragh;
  // optional (tests): the fp32 logits of every classified row,
  // logits[row * n_classes + c] (null: labels only)
  float* logits;
  // the Keras weights for the one-wave-per-stream VALU forward of the
  // streaming hop kernel: per layer W_l transposed, row o (output unit o)
  // at woff + o * wstride holding W_l[k][o] for k < din rounded up to 4
  // (wstride = that, or 4 more, so that wstride / 4 is odd: lanes reading
  // their rows as 16-B vectors hit every LDS bank once per 16 lanes), then
  // b_l at boff
  const float* wraw;
  int wraw_n;  // floats in wraw
  int woff[VAD_MAX_FFN_LAYERS];
  int boff[VAD_MAX_FFN_LAYERS];
  int wstride[VAD_MAX_FFN_LAYERS];
  // 1: with analyser inputs (|Mn| <= sqrt(5), or a NaN / inf the kernels
  // handle as they come) every finite layer-1 input is below 32768 in
  // magnitude, so that layer needs no f16-range check (capi.hip, from the
  // layer-0 weights: max_j |b_j| + sqrt(5) sum_k |W[k][j]|)
  int h1_bounded;
};

// Decision-tree node (tree_kernel.hip): internal if feature >= 0 (go left
// iff x[feature] <= threshold, or x[feature] is NaN and nan_left), else a
// leaf of class index `leaf`.
struct TreeNode {
  int feature;
  int left;
  int right;
  short leaf;
  short nan_left;  // a NaN feature goes left (sklearn missing_go_to_left)
  double threshold;
};

// Compact node for the LDS-resident walk: 16 B.  feature >= 0: internal,
// bit 30 = missing_go_to_left, bits 0..15 = feature; feature < 0: leaf of
// class -1 - feature.  thr = the largest float <= threshold, so for a float
// x, x <= thr exactly when (double)x <= threshold (sklearn's comparison).
struct TreeNodeC {
  float thr;
  int feature;
  int left;
  int right;
};

// XCD-balanced tile runs of the persistent MFCC kernel (paired-frame path).
// The 8 XCDs of an MI355X run at their own shader clocks under load (one
// box: 2.04-2.26 GHz), while every workgroup of an equal split does the
// same number of cycles, so the slowest XCD sets the launch time.  `word`
// holds 8 weights (8 bits each, >= 1; 0 = equal split): workgroup b's
// share of the tiles is proportional to the weight of b mod 8 (the XCD
// the dispatcher deals it to; a different placement costs balance, never
// correctness: the runs always partition the tiles exactly).  `stats`
// (host-mapped, may be null): per workgroup (tiles << 40) | s_memrealtime
// ticks, from which the host derives the next launch's weights.
struct MfccBalance {
  unsigned long long word = 0;
  unsigned long long* stats = nullptr;
};
// first tile of workgroup b's run (b = G: n_tiles)
__host__ __device__ inline int64_t balanced_tile(unsigned long long word, int64_t n_tiles, int b, int G) {
  if (word == 0) return (int64_t)b * n_tiles / G;
  int64_t w8 = 0, part = 0;
  for (int x = 0; x < 8; ++x) {
    const int64_t w = (int64_t)((word >> (8 * x)) & 255u);
    w8 += w;
    part += x < (b & 7) ? w : 0;
  }
  int64_t tot = (int64_t)(G >> 3) * w8;
  for (int x = 0; x < (G & 7); ++x) tot += (int64_t)((word >> (8 * x)) & 255u);
  return n_tiles * ((int64_t)(b >> 3) * w8 + part) / tot;
}

// Launchers (defined in the .hip translation units).
size_t mfcc_smem_bytes();
hipError_t launch_mfcc(int mode, const MfccDev* plan, int spec, const float* src, int64_t stride,
                       int len, int64_t n, float* out, hipStream_t st, const MfccBalance& bal = MfccBalance());
hipError_t launch_mfcc_i16(int mode, const MfccDev* plan, int spec, const int16_t* src,
                           int64_t stride, int len, int64_t n, float* out, hipStream_t st,
                           const MfccBalance& bal = MfccBalance());
bool mfcc_ffn_fusable(int spec, const FfnDev& net, int frame_size, int hop, const void* audio, int tin_bytes);
hipError_t launch_mfcc_ffn(const MfccDev* plan, const FfnDev& net, const void* audio, int tin_bytes,
                           int64_t n_frames, int mode, uint8_t* labels, hipStream_t st);
hipError_t launch_ffn(const FfnDev& net, int src, const float* in, int64_t n_rows, int mfcc_n,
                      int mode, uint8_t* labels, hipStream_t st);
hipError_t launch_stream_ffn(const FfnDev& net, const float* newrow, float* ring, int* count,
                             int64_t n_streams, int mfcc_n, uint8_t* labels, hipStream_t st);
hipError_t launch_stream_hop(const MfccDev* plan, const float* blob, int blob_n, int nf, int n_taps,
                             const FfnDev& net, float* frames, int64_t fstride, int len,
                             const float* hop, int64_t hstride, int hlen, int64_t n_streams, int mfcc_n,
                             float* ring, int* count, uint8_t* labels, int n_hops, int64_t hop_kstride,
                             int64_t lab_kstride, hipStream_t st);
hipError_t launch_stream_push(float* frames, int64_t fstride, int len, const float* hop, int64_t hstride,
                              int hlen, int64_t n_streams, hipStream_t st);
hipError_t launch_preemphasis(const float* x, float* y, int64_t n_rows, int64_t row_len, int64_t stride, float a,
                              hipStream_t st);
// any fft_n other than 512 (spec_generic.hip): mode 0 frames -> MFCC,
// 1 frames -> spectra, 2 spectra -> MFCC; tw = exp(-2 pi i m / fft_n), fp64
hipError_t launch_generic(int mode, const MfccDev* plan, const float* src, int64_t stride, int len, int64_t n,
                          int fft_n, const double2* tw, float* out, hipStream_t st);
hipError_t launch_generic_i16(int mode, const MfccDev* plan, const int16_t* src, int64_t stride, int len,
                              int64_t n, int fft_n, const double2* tw, float* out, hipStream_t st);
hipError_t launch_features(const float* mfcc, int64_t n_rows, int mfcc_n, int mode, float* out,
                           hipStream_t st);
hipError_t launch_simple_features(const float* frames, int64_t n_frames, int frame_len,
                                  int64_t frame_stride, int L, int pad, int band_bins, int n_bands,
                                  double* out, hipStream_t st);
size_t scale_workspace_bytes();
hipError_t launch_scale_features(float* x, int64_t n_rows, int mfcc_n, double* ws, hipStream_t st);
int64_t format_csv_rows(const float* rows, int64_t n_rows, int n_cols, double label, char* buf,
                        int64_t buf_size);
hipError_t launch_tree_rows(const TreeNode* nodes, int n_nodes, const float* x, int64_t n, int dim,
                            uint8_t* labels, hipStream_t st);
hipError_t launch_tree_windows(const TreeNode* nodes, const TreeNodeC* cnodes, int n_nodes,
                               const float* mfcc, int64_t n_rows,
                               int mfcc_n, int mode, uint8_t* labels, hipStream_t st);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per kernel and device
// (`done`: one bit per device ordinal, a static of the launch site).
inline hipError_t ensure_dyn_lds(const void* fn, int bytes, std::atomic<unsigned long long>& done) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const unsigned long long bit = 1ull << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
  return e;
}

// log10 of a positive energy: native v_log_f32 (with a pre-scale for tiny
// inputs) times log10(2) -- ~1e-7 relative, far inside the 1e-4 budget.
__device__ __forceinline__ float log10_pos(float e) {
  const bool tiny = e < 0x1p-100f;
  const float x = tiny ? e * 0x1p64f : e;
  const float l2 = __builtin_amdgcn_logf(x);  // log2
  return fmaf(l2, 0.30102999566398120f, tiny ? -19.26591972249479649f : 0.f);
}

// NaN-keeping ReLU (numpy / Keras keep NaN; fmaxf would drop it).
__device__ __forceinline__ float relu_nan(float x) { return x < 0.f ? 0.f : x; }

// Floats per row of a table whose rows lanes read as 16-B vectors: n rounded
// up to 4, plus 4 when that is a multiple of 8 (a stride of 4 x odd floats
// puts 16 consecutive lanes' vectors on distinct LDS banks)
__host__ __device__ constexpr int vec_row_stride(int n) {
  return ((n + 3) & ~3) % 8 == 0 ? ((n + 3) & ~3) + 4 : ((n + 3) & ~3);
}

}  // namespace vad
