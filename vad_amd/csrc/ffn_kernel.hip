// Features (5-frame window, normalisation, deltas) + FFN forward on f32 MFMA.
//
// Reference semantics:
//   features  realtime_analysis/sklearn_analyser.py:52-69,103-107 (analyser,
//             normalised centre) and dataset/file_processing.py:40-70
//             (offline, unnormalised);
//   FFN       learning/ffn_trainer.py:106-116: Dense -> relu (-> relu) ->
//             Dense -> relu -> ... -> Dense -> softmax; predict = argmax.
//
// Layout: one wave classifies a tile of 16 windows with
// v_mfma_f32_16x16x4_f32 (exact f32: a k-ordered fma chain).  The network
// runs transposed, H^T = W^T X^T, so a layer's accumulator tile (rows =
// hidden units 4g + r on lane group g = lane>>4, register r; column = window
// lane&15) IS the next layer's B operand for K-step (tile, r) -- no lane
// shuffles between layers.  The W^T A-operand fragments and the bias
// fragments are laid out per lane on the host ("frag" slots) and held in
// VGPRs for the whole persistent loop.
#include "vad_common.h"
#include "features.h"
#include "ffn_dev.h"

namespace vad {

// Source of the layer-0 operands.
enum Src { kFromMfcc = 0, kFromRows = 1 };

// One wave per 16-window tile, persistent over tiles.
template <int KS0, int T1, int T2, int T3, int T4, int NC, int SRC>
__global__ __launch_bounds__(256) void ffn_kernel(FfnDev net, const float* __restrict__ in,
                                                  int64_t n_rows, int mfcc_n, int mode,
                                                  uint8_t* __restrict__ labels) {
  using TP = Topo<KS0, T1, T2, T3, T4, NC>;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int jw = lane & 15;
  const int in_dim = net.dims[0];

  float fa[TP::NA];
  float fb[TP::NB];
  float fv[TP::NV + TP::NVB + 1];
  load_frags<TP>(net.frag, lane, fa, fb, fv);

  const int64_t n_tiles = (n_rows + 15) / 16;
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t tile = wave_id; tile < n_tiles; tile += n_waves) {
    const int64_t w = tile * 16 + jw;
    const bool valid = w < n_rows;
    float x[KS0];
#pragma unroll
    for (int s = 0; s < KS0; ++s) {
      const int f = 4 * s + g;
      float v = 0.f;
      if (f < in_dim && valid) {
        if constexpr (SRC == kFromMfcc) {
          const float* r0 = in + w * mfcc_n;
          v = window_feature(r0, r0 + mfcc_n, r0 + 2 * mfcc_n, r0 + 3 * mfcc_n, r0 + 4 * mfcc_n,
                             f, mfcc_n, mode);
        } else {
          v = in[w * in_dim + f];
        }
      }
      x[s] = v;
    }
    const f32x4 z = mlp_forward<KS0, T1, T2, T3, T4, NC>(fa, fb, fv, x);
    if (g == 0 && valid) {
      labels[w] = (uint8_t)argmax_classes(z, net.n_classes);
      store_logits(net.logits, w, z, net.n_classes);
    }
  }
}

// Windows of an MFCC sequence, 64 per block iteration (4 waves x 16):
//   A  the 68 MFCC rows the chunk needs are staged in LDS (coalesced; loaded
//      into registers two chunks ahead);
//   B  every (window, coefficient) feature triple is computed once, by one
//      thread, from LDS into an LDS feature tile;
//   C  each wave runs the MFMA chain on 16 windows with its layer-0 B
//      operands read from the tile, then the argmax.
// rows / X are double-buffered, so two barriers per chunk order the phases.
#ifndef VAD_FFN_WIN_PRIO
#define VAD_FFN_WIN_PRIO 1  // issue priority of phase C, the MFMA chain (0: none)
#endif
constexpr int kChunk = 64;
constexpr int kXStride = 68;  // floats per feature row: 16-B aligned, conflict-free b128 reads

template <int KS0, int T1, int T2, int T3, int T4, int NC, int MN, bool H3, int MODE = -1>
__device__ __forceinline__ void ffn_window_body(const FfnDev& net, const float* __restrict__ mfcc,
                                                int64_t n_rows, int mfcc_n_rt, int mode_rt,
                                                uint8_t* __restrict__ labels) {
  const int mode = MODE >= 0 ? MODE : mode_rt;  // compile-time feature form: no branches
  using TP = Topo<KS0, T1, T2, T3, T4, NC>;
  using HP = HTopo<TP, KS0, T1, T2, T3, T4>;
  static_assert(!H3 || (MN > 0 && MN * (kChunk / 4) <= 256), "split-f16 needs the sliding feature phase");
  __shared__ float rows[2][(kChunk + 4) * kMaxCoefs];
  __shared__ __attribute__((aligned(16))) float X[2][kChunk * kXStride];
  // H3: windows with a NaN feature (a flat coefficient) -- their features go
  // to the MLP as 0 and their logits are set to NaN (class 0), as the
  // reference's NaN-propagating forward would give
  __shared__ int wnan[2][kChunk];
  const int mfcc_n = MN > 0 ? MN : mfcc_n_rt;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int g = lane >> 4;
  const int jw = lane & 15;
  const int in_dim = net.dims[0];
  const int nfeat = 3 * mfcc_n;

  // split-f16 (H3): the f16 weight fragments stay in VGPRs in place of the
  // f32 ones
  constexpr int kNA = H3 ? 1 : TP::NA;
  constexpr int kNH = H3 ? HP::NS : 1;
  float fa[kNA];
  float fb[TP::NB];
  float fv[TP::NV + TP::NVB + 1];
  u4 fh[kNH][2];
  if constexpr (H3) {
    load_frags<TP, true>(net.frag, lane, fa, fb, fv);
    load_fragh<HP>(net.fragh, lane, fh);
    // feature columns the layer-0 reads past the features stay 0
    for (int i = tid; i < 2 * kChunk * kXStride; i += 256) (&X[0][0])[i] = 0.f;
  } else {
    load_frags<TP>(net.frag, lane, fa, fb, fv);
  }

  const int64_t n_frames = n_rows + 5;
  const int64_t n_chunks = (n_rows + kChunk - 1) / kChunk;
  // rows of a chunk: (kChunk + 4) x mfcc_n floats, <= 5 per thread, loaded
  // two chunks ahead
  constexpr int kRowRegs = ((kChunk + 4) * kMaxCoefs + 255) / 256;
  float pre[2][kRowRegs];
  // MN > 0: rows packed at stride MN, so a chunk's rows are one contiguous
  // run of (kChunk + 4) * MN floats copied element for element (branch-free:
  // out-of-range lanes load element 0 and keep 0)
  constexpr int kPackRegs = MN > 0 ? ((kChunk + 4) * MN + 255) / 256 : 1;
  static_assert(MN == 0 || 256 * kPackRegs <= (kChunk + 4) * kMaxCoefs, "packed rows overflow");
  auto load_rows = [&](int64_t ch, float (&dst)[kRowRegs]) {
    const int64_t base = ch * kChunk;
    const int64_t avail = ch < n_chunks ? n_frames - base : 0;
    const int nr = (int)(avail < kChunk + 4 ? avail : kChunk + 4);
    if constexpr (MN > 0) {
#pragma unroll
      for (int q = 0; q < kPackRegs; ++q) {
        const int i = tid + 256 * q;
        const bool ok = i < nr * MN;
        const float v = mfcc[ok ? base * MN + i : 0];
        dst[q] = ok ? v : 0.f;
      }
    } else {
#pragma unroll
      for (int q = 0; q < kRowRegs; ++q) {
        const int i = tid + 256 * q;
        dst[q] = i < nr * mfcc_n ? mfcc[base * mfcc_n + i] : 0.f;
      }
    }
  };
  load_rows(blockIdx.x, pre[0]);
  load_rows(blockIdx.x + gridDim.x, pre[1]);
  int buf = 0;
  for (int64_t ch = blockIdx.x; ch < n_chunks; ch += gridDim.x, buf ^= 1) {
    const int64_t base = ch * kChunk;
    float* rw_ = rows[buf];
    float* Xb = X[buf];
    // ---- A: rows base .. base+67 (prefetched) ------------------------------
    if constexpr (MN > 0) {
#pragma unroll
      for (int q = 0; q < kPackRegs; ++q) {
        rw_[tid + 256 * q] = pre[0][q];  // rows at stride MN (slots past the chunk unused)
        pre[0][q] = pre[1][q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < kRowRegs; ++q) {
        const int i = tid + 256 * q;
        if (i < (kChunk + 4) * mfcc_n) {
          const int r = i / mfcc_n, c = i - r * mfcc_n;
          rw_[r * kMaxCoefs + c] = pre[0][q];
        }
        pre[0][q] = pre[1][q];
      }
    }
    if (H3 && tid < kChunk) wnan[buf][tid] = 0;
    __syncthreads();
    load_rows(ch + 2 * (int64_t)gridDim.x, pre[1]);
    // ---- B: features (sklearn_analyser.py:52-69 / file_processing.py:51-66)
    const int64_t nwin64 = n_rows - base;
    const int nwin = (int)(nwin64 < kChunk ? nwin64 : kChunk);
    if constexpr (MN > 0 && MN * (kChunk / 4) <= 256) {
      // thread (c, q): coefficient c of windows 4q .. 4q+3, sliding over the
      // eight rows 4q .. 4q+7 they span (all loads issued at once); windows
      // past nwin read rows past the clip (zero-filled): written, not used
      const int c = tid % MN, q = tid / MN;
      if (q < kChunk / 4) {
        float a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = rw_[(4 * q + k) * MN + c];
        const bool m0 = !H3 || c < in_dim, m1 = !H3 || MN + c < in_dim, m2 = !H3 || 2 * MN + c < in_dim;
        // feature groups no input of this topology can reach (in_dim <= 4 KS0)
        constexpr bool kD1 = !H3 || MN < 4 * KS0, kD2 = !H3 || 2 * MN < 4 * KS0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const Feat3 ft = feature_triple(a[k], a[k + 1], a[k + 2], a[k + 3], a[k + 4], mode);
          float* xw = Xb + (4 * q + k) * kXStride;
          if constexpr (H3) {
            // mn is NaN exactly when the coefficient is flat (d2 with it);
            // the flag is or-ed in by every coefficient thread, branch-free
            const bool nan = (m0 || (kD2 && m2)) && ft.mn != ft.mn;
            __hip_atomic_fetch_or(&wnan[buf][4 * q + k], (int)nan, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            xw[c] = m0 && !nan ? ft.mn : 0.f;
            if constexpr (kD1) xw[MN + c] = m1 ? ft.d1 : 0.f;
            if constexpr (kD2) xw[2 * MN + c] = m2 && !nan ? ft.d2 : 0.f;
          } else {
            xw[c] = ft.mn;
            xw[MN + c] = ft.d1;
            xw[2 * MN + c] = ft.d2;
          }
        }
      }
    } else
    for (int i = tid; i < nwin * mfcc_n; i += 256) {
      const int w = i / mfcc_n, c = i - w * mfcc_n;
      constexpr int kRS = MN > 0 ? MN : kMaxCoefs;  // row stride of the staged rows
      const float* r = rw_ + w * kRS + c;
      const Feat3 ft = feature_triple(r[0], r[kRS], r[2 * kRS], r[3 * kRS], r[4 * kRS], mode);
      float* xw = Xb + w * kXStride;
      if constexpr (H3) {  // the split-f16 layer 0 reads every column: unused ones are 0
        xw[c] = c < in_dim ? ft.mn : 0.f;
        xw[mfcc_n + c] = mfcc_n + c < in_dim ? ft.d1 : 0.f;
        xw[2 * mfcc_n + c] = 2 * mfcc_n + c < in_dim ? ft.d2 : 0.f;
      } else {
        xw[c] = ft.mn;
        xw[mfcc_n + c] = ft.d1;
        xw[2 * mfcc_n + c] = ft.d2;
      }
    }
    __syncthreads();
    // ---- C: MFMA chain, 16 windows per wave --------------------------------
    const int wl = wv * 16 + jw;
    const int64_t w = base + wl;
#if VAD_FFN_WIN_PRIO
    // the MFMA chain at raised issue priority, as in ffn_wave_kernel (A/B,
    // exact f32: 116.6 -> 114.4 us per 1M windows, profiles/r05/ab/ffn_win_prio_ab.json)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(VAD_FFN_WIN_PRIO);
    __builtin_amdgcn_sched_barrier(0);
#endif
    f32x4 z;
    if constexpr (H3) {
      // windows past nwin read stale (finite) features: computed, not stored
      float x0[HP::K0][8];
      // kMerge0 (<= 16 inputs): lane group g takes inputs 8 (g & 1) + q
      constexpr bool M0 = kMerge0<KS0>;
      const v4f* xr = reinterpret_cast<const v4f*>(Xb + wl * kXStride + 8 * (M0 ? (g & 1) : g));
#pragma unroll
      for (int s = 0; s < HP::K0; ++s) {
        const v4f lo4 = xr[8 * s], hi4 = xr[8 * s + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x0[s][q] = lo4[q];
          x0[s][q + 4] = hi4[q];
        }
      }
      if constexpr (M0) {  // the 13 analyser inputs; columns 13..15 zeroed in registers
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (8 + q >= 13) x0[0][q] = 8 * (g & 1) + q < 13 ? x0[0][q] : 0.f;
      }
      z = mlp_forward_h3<KS0, T1, T2, T3, T4, NC>(FragRegs{fh}, (const float*)fb, (const float*)fv, x0);
      if (wnan[buf][wl]) z = (f32x4){__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    } else {
      float x[KS0];
#pragma unroll
      for (int s = 0; s < KS0; ++s) {
        const int f = 4 * s + g;
        x[s] = (f < in_dim && f < nfeat && wl < nwin) ? Xb[wl * kXStride + f] : 0.f;
      }
      z = mlp_forward<KS0, T1, T2, T3, T4, NC>(fa, fb, fv, x);
    }
#if VAD_FFN_WIN_PRIO
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
#endif
    if (g == 0 && wl < nwin) {
      labels[w] = (uint8_t)argmax_classes(z, net.n_classes);
      store_logits(net.logits, w, z, net.n_classes);
    }
  }
}

template <int KS0, int T1, int T2, int T3, int T4, int NC, int MN>
__global__ __launch_bounds__(256) void ffn_window_kernel(FfnDev net, const float* __restrict__ mfcc,
                                                         int64_t n_rows, int mfcc_n_rt, int mode,
                                                         uint8_t* __restrict__ labels) {
  ffn_window_body<KS0, T1, T2, T3, T4, NC, MN, false>(net, mfcc, n_rows, mfcc_n_rt, mode, labels);
}

// split-f16 variant: two 4-wave blocks per CU (<= 256 registers per lane),
// one instance per feature form
template <int KS0, int T1, int T2, int T3, int T4, int NC, int MN, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void ffn_window_h3_kernel(
    FfnDev net, const float* __restrict__ mfcc, int64_t n_rows, int mfcc_n_rt, int mode,
    uint8_t* __restrict__ labels) {
  ffn_window_body<KS0, T1, T2, T3, T4, NC, MN, true, MODE>(net, mfcc, n_rows, mfcc_n_rt, mode, labels);
}

// ---------------------------------------------------------------------------
// Wave-autonomous window kernel (split-f16 topologies, 13 coefficients).
// Each wave owns whole 16-window tiles end to end: the tile's 20 MFCC rows
// (16 windows + 4 halo rows, one contiguous run of 260 floats) are loaded
// into registers one tile ahead, staged in a wave-private LDS slice, turned
// into the tile's 16 x 13 feature triples (3.25 per lane; item i reads
// R[i + 13 d], conflict-free) in a second wave-private slice, read back as
// the layer-0 B operands and classified.  No workgroup barriers: the waves of
// a SIMD drift freely, so one wave's LDS / MFMA latency hides behind the
// other's VALU work (the 64-window block kernel above pays two barriers and
// a block-wide load -> features -> MLP chain per chunk).
//   NaN windows (a flat coefficient, the analyser's 0/0): the feature item
// writes 0 and flags its window; the window's logits become NaN -> class 0,
// as in ffn_window_body.
// ---------------------------------------------------------------------------
#ifndef VAD_FFN_WAVE
#define VAD_FFN_WAVE 1  // 0: the 64-window block kernel for the split-f16 topologies
#endif
#ifndef VAD_FFN_PF
#define VAD_FFN_PF 2  // wave kernel: row prefetch depth in tiles (3, 4: no faster)
#endif
#ifndef VAD_FFN_WAVE_MFMA_OUT
#define VAD_FFN_WAVE_MFMA_OUT 0
#endif
// Residency of the wave kernel per topology (measured per 1M windows):
// 39-64-32-16-3 keeps its split-f16 weight fragments in a workgroup-shared
// LDS copy and runs 3 waves per SIMD at 168 VGPRs (75 vs 81 us with the
// fragments in VGPRs at 2 waves); 13-64-64-2 is as fast either way (67 us)
// and keeps them in VGPRs at 2 waves (LDS at 2 waves: 72.5 us; at 4 waves
// the 128-VGPR budget spills: 140 us).  With more than two classes its
// output layer no longer fits beside the VGPR fragments (scratch spills:
// 101 us for 13-64-64-3), so those read the fragments from LDS too (78 us).
#ifndef VAD_FFN_LDS_SLOTS
#define VAD_FFN_LDS_SLOTS 1
#endif
// kLdsSlots (13-64-64-2): the bias and VALU output-layer slots (one value
// per lane group) move to a workgroup-shared LDS table read per tile, which
// frees their ~70 VGPRs for a third wave per SIMD while the split-f16
// fragments stay in VGPRs (a lone wave issues scalar VALU work at about a
// third of the rate two waves reach together: tools/micro/mfma_valu_overlap)
#ifndef VAD_FFN_ALL_LDS
#define VAD_FFN_ALL_LDS 1  // 13-64-64-2: fragments and slots in LDS, 4 waves per SIMD (0: 3 waves)
#endif
template <int KS0, int NC>
struct WaveResidency {
  static constexpr bool kAll = VAD_FFN_ALL_LDS != 0 && KS0 == 4 && NC <= 2;
  static constexpr bool kLdsFrags = KS0 == 10 || NC > 2 || kAll;
  static constexpr bool kLdsSlots = (VAD_FFN_LDS_SLOTS != 0 && !kLdsFrags) || kAll;
#ifndef VAD_FFN_ALL_WPS
#define VAD_FFN_ALL_WPS 4
#endif
  static constexpr int kWavesPerSimd = kAll ? VAD_FFN_ALL_WPS : KS0 == 10 ? 3 : kLdsSlots ? 3 : 2;
};
// Fragments with the hi halves (and layer 0's lo halves) in VGPRs and the lo
// halves of slots >= LO_FROM read from a workgroup-shared LDS copy
// ([slot - LO_FROM][lane], one ds_read_b128 per MFMA that uses one): the
// register file keeps the operands of two of the three products per layer.
template <int LO_FROM>
struct FragSplitRes {
  const u4 (*p)[2];
  const u4* lo;  // fhlo_s + lane
  int base;      // slot offset of this accessor (compile-time after inlining)
  __device__ u4 get(int sl, int h) const {
    return (h == 1 && base + sl >= LO_FROM) ? lo[(base + sl - LO_FROM) * 64] : p[sl][h];
  }
  __device__ FragSplitRes at(int off) const { return {p + off, lo, base + off}; }
};
// a lane group's row of the slot table: slot s at p[s] (16-B aligned rows,
// so a layer's four consecutive bias slots are one ds_read_b128)
struct LdsRow {
  const float* p;
  __device__ float operator[](int s) const { return p[s]; }
  __device__ LdsRow operator+(int off) const { return {p + off}; }
};
constexpr int kWRows = (kWTile + 4) * 13;        // staged MFCC floats per tile (260)
constexpr int kWRowRegs = (kWRows + 63) / 64;    // 5 per lane

#ifndef VAD_FFN_WPB
#define VAD_FFN_WPB 4  // waves per block (sharing one LDS fragment copy)
#endif
constexpr int kWpb = VAD_FFN_WPB;
// LG: the launch also writes the logits (net.logits, tests); without it a
// two-class network with a VALU output layer (13-64-64-2) takes its labels
// from the logit difference (valu_label2: one dot product instead of two)
template <int KS0, int T1, int T2, int T3, int T4, int NC, int MODE, bool LG>
__global__ __launch_bounds__(64 * kWpb) __attribute__((amdgpu_waves_per_eu(WaveResidency<KS0, NC>::kWavesPerSimd))) void ffn_wave_kernel(
    FfnDev net, const float* __restrict__ mfcc, int64_t n_rows, uint8_t* __restrict__ labels) {
  // VAD_FFN_WAVE_MFMA_OUT: the output layer on the MFMA too (the plan's
  // fragh holds its slots after the hidden layers'); default: bl13's on the
  // VALU (its 6-MFMA single-tile chain measured 3 us slower per 1M windows)
  using TP = Topo<KS0, T1, T2, T3, T4, NC, VAD_FFN_WAVE_MFMA_OUT != 0>;
  using HP = HTopo<TP, KS0, T1, T2, T3, T4>;
  constexpr int MN = 13;
  static_assert(KS0 == 4 || KS0 == 10, "specialised topologies: 13 or 39 inputs");
  constexpr int IN = KS0 == 4 ? MN : 3 * MN;  // network inputs (features 0 .. IN-1)
  constexpr int XS = 32 * HP::K0 + 4;         // floats per feature row: 16-B aligned
  __shared__ float rows_s[kWpb][kWRows];
  __shared__ __attribute__((aligned(16))) float x_s[kWpb][kWTile * XS];
  __shared__ int flat_s[kWpb][kWTile];  // per window: some coefficient is flat (NaN features)
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int g = lane >> 4;
  const int jw = lane & 15;
  float* R = rows_s[wv];
  float* X = x_s[wv];
  int* FL = flat_s[wv];

  constexpr bool kLdsFrags = WaveResidency<KS0, NC>::kLdsFrags;
  constexpr bool kLdsSlots = WaveResidency<KS0, NC>::kLdsSlots;
  constexpr int NSL = TP::NB + TP::NV + TP::NVB;  // bias + output-layer slots
  // the logit-difference slots (valu_label2): TIL*4 weights, then the bias.
  // Launches that also write the logits (LG) take their labels from the same
  // difference (a label must not depend on whether the logits
  // were requested)
  constexpr bool kDiff = NC == 2 && TP::VL && TP::NL == 3 && kLdsSlots;
  constexpr int NSD = kDiff ? TP::TIL * 4 + 1 : 0;
  constexpr int NSLP = (NSL + NSD + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float slot_s[kLdsSlots ? 4 * NSLP : 1];
// issue priority of a tile's MFMA / split / label chain (VAD_FFN_PRIO) and of
// its features (VAD_FFN_PRIO_FEAT; when set, held to the next tile's
// features).  A/B (profiles/r05/ab/ffn_prio_ab_*.json): the chain at 3 takes
// 13-64-64-2 from 50.2 to 48.5 us per 1M windows; features at 3 gain half
// that, both raised no more
#ifndef VAD_FFN_PRIO
#define VAD_FFN_PRIO 3
#endif
#ifndef VAD_FFN_PRIO_FEAT
#define VAD_FFN_PRIO_FEAT 0
#endif
#ifndef VAD_FFN_LO_ALL
#define VAD_FFN_LO_ALL 1  // 1: every lo half in LDS; 0: those after layer 0 only
#endif
  constexpr int kLoFrom = VAD_FFN_LO_ALL ? 0 : HP::S0;
  constexpr int kLoSlots = kLdsSlots && !kLdsFrags ? HP::NS - kLoFrom : 0;
  __shared__ u4 fhlo_s[kLoSlots > 0 ? kLoSlots * 64 : 1];
  float fa[1];
  float fb[kLdsSlots ? 1 : TP::NB];
  float fv[kLdsSlots ? 1 : TP::NV + TP::NVB + 1];
  if constexpr (kLdsSlots) {
    // slot sl of lane group gg (the host's fragment order: biases, then the
    // VALU layer's class slots, then its biases after 4 classes' worth)
    auto slot_val = [&](int sl, int gg) {
      const int src_sl = sl < TP::NB ? TP::NA_ALL + sl
                                     : TP::NA_ALL + TP::NB + (sl - TP::NB < TP::NV ? sl - TP::NB
                                                                                  : 4 * TP::TIL * 4 + sl - TP::NB - TP::NV);
      return net.frag[src_sl * 64 + 16 * gg];
    };
    for (int i = threadIdx.x; i < 4 * NSLP; i += 64 * kWpb) {
      const int gg = i / NSLP, sl = i - gg * NSLP;
      float v = 0.f;
      if (sl < NSL) {
        v = slot_val(sl, gg);
      } else if (sl < NSL + NSD) {  // class 1 minus class 0 (weights, then the bias)
        const int q = sl - NSL;
        v = q < TP::TIL * 4 ? slot_val(TP::NB + TP::TIL * 4 + q, gg) - slot_val(TP::NB + q, gg)
                            : slot_val(TP::NB + TP::NV + 1, gg) - slot_val(TP::NB + TP::NV, gg);
      }
      slot_s[i] = v;
    }
    // the lo halves of the layers after the first: [slot - S0][lane]
    for (int i = threadIdx.x; i < kLoSlots * 64; i += 64 * kWpb)
      fhlo_s[i] = reinterpret_cast<const u4*>(net.fragh)[(2 * (kLoFrom + i / 64) + 1) * 64 + (i & 63)];
    __syncthreads();
  } else {
    load_frags<TP, true>(net.frag, lane, fa, fb, fv);
  }
  const auto fbs = [&] {
    if constexpr (kLdsSlots) return LdsRow{slot_s + g * NSLP};
    else return (const float*)fb;
  }();
  const auto fvs = [&] {
    if constexpr (kLdsSlots) return LdsRow{slot_s + g * NSLP + TP::NB};
    else return (const float*)fv;
  }();
  __shared__ u4 fh_s[kLdsFrags ? HP::NS * 2 * 64 : 1];
  u4 fh_r[kLdsFrags ? 1 : HP::NS][2];
  if constexpr (kLdsFrags) {
    for (int i = threadIdx.x; i < HP::NS * 2 * 64; i += 64 * kWpb) fh_s[i] = reinterpret_cast<const u4*>(net.fragh)[i];
    __syncthreads();
  } else {
    load_fragh<HP>(net.fragh, lane, *reinterpret_cast<u4(*)[HP::NS][2]>(fh_r));
  }
  const auto fh = [&] {
    if constexpr (kLdsFrags) return FragLds{fh_s, lane};
    else if constexpr (kLdsSlots) return FragSplitRes<kLoFrom>{fh_r, fhlo_s + lane, 0};
    else return FragRegs{fh_r};
  }();
  // feature columns IN .. 32 K0 - 1 are read by layer 0 and stay 0
  for (int i = lane; i < kWTile * XS; i += 64) X[i] = 0.f;

  const int64_t n_tiles = (n_rows + kWTile - 1) / kWTile;
  const int64_t total = (n_rows + 4) * MN;  // MFCC floats the windows can read
  const int64_t wave_id = (int64_t)blockIdx.x * kWpb + wv;
  const int64_t n_waves = (int64_t)gridDim.x * kWpb;
  // branch-free and select-free (a select on the loaded value would make the
  // prefetch wait at the loop's back edge): offsets past the rows clamp to
  // the last float, so the last tile's unused windows see finite rows.  The
  // tile base is wave-uniform (a scalar address), the lane offsets 32-bit.
  auto load = [&](int64_t t, float (&dst)[kWRowRegs]) {
    const int64_t base = t * (kWTile * MN);
    const float* tb = mfcc + base;
    const int64_t rem = total - 1 - base;  // >= 0 for t < n_tiles
    const unsigned limb = 4u * (unsigned)(rem < kWRows ? rem : kWRows);  // byte offset clamp
#pragma unroll
    for (int q = 0; q < kWRowRegs; ++q) {
      const unsigned ob = 4u * (unsigned)(lane + 64 * q);
      dst[q] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(tb) + (ob < limb ? ob : limb));
    }
  };
  // every fragment load done before the loop: the waitcnt pass would
  // otherwise leave counter waits for them in the loop body, where they
  // also wait on the row prefetches
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt 0
  // one tile: rows (prefetched two tiles ahead in `pre`) -> R; pre reloaded
  // with tile tn's rows; features -> X; MLP; label
  auto tile_body = [&](int64_t t, int64_t tn, float (&pre)[kWRowRegs]) {
    wave_lds_handoff();  // the previous tile's reads of R / X / FL come first
#pragma unroll
    for (int q = 0; q < kWRowRegs; ++q)
      if (lane + 64 * q < kWRows) R[lane + 64 * q] = pre[q];
    load(tn < n_tiles ? tn : t, pre);
#if VAD_FFN_PRIO_FEAT
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(VAD_FFN_PRIO_FEAT);
    __builtin_amdgcn_sched_barrier(0);
#endif
    wave_tile_features<IN, XS, MODE>(R, X, FL, lane);
#if VAD_FFN_PRIO || VAD_FFN_PRIO_FEAT
    // the MFMA / split chain at raised issue priority: the SIMD's arbiter
    // favours the wave deepest in its chain over the others' features
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(VAD_FFN_PRIO);
    __builtin_amdgcn_sched_barrier(0);
#endif
    f32x4 z;
    int lab;
    if constexpr (kDiff) {
      lab = wave_tile_label2<KS0, T1, T2, IN, XS, false, wave_tile_in_bounded<MODE, IN>>(
          X, FL, lane, fh, fbs, fvs, LdsRow{slot_s + g * NSLP + NSL}, net.h1_bounded, LG ? &z : nullptr);
    } else {
      lab = wave_tile_classify<KS0, T1, T2, T3, T4, NC, VAD_FFN_WAVE_MFMA_OUT != 0, IN, XS, false,
                               wave_tile_in_bounded<MODE, IN>>(X, FL, lane, fh, fbs, fvs, net.n_classes, z);
    }
#if VAD_FFN_PRIO && !VAD_FFN_PRIO_FEAT
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
#endif
    const int64_t w = t * kWTile + jw;
    if (g == 0 && w < n_rows) {
      labels[w] = (uint8_t)lab;
      if constexpr (LG) store_logits(net.logits, w, z, net.n_classes);
    }
  };
  // kPF tiles per trip (VAD_FFN_PF; 1 in the all-LDS residency, whose
  // 128-VGPR budget a second prefetch set would spill), each with its own
  // prefetch registers (no copies at the back edge): a tile's rows are
  // loaded kPF tiles ahead
#ifndef VAD_FFN_PF_ALL
#define VAD_FFN_PF_ALL 1
#endif
  constexpr int kPF = WaveResidency<KS0, NC>::kAll ? VAD_FFN_PF_ALL : VAD_FFN_PF;
  float pre[kPF][kWRowRegs];
#pragma unroll
  for (int k = 0; k < kPF; ++k) {
    const int64_t tk = wave_id + k * n_waves;
    load(tk < n_tiles ? tk : 0, pre[k]);
  }
  for (int64_t t = wave_id; t < n_tiles; t += kPF * n_waves) {
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int64_t tk = t + k * n_waves;
      if (k > 0 && tk >= n_tiles) break;
      tile_body(tk, tk + kPF * n_waves, pre[k]);
    }
  }
}

// ---------------------------------------------------------------------------
// Tile groups (13-64-64-2, labels only): the wave kernel above with each
// wave taking NT 16-window tiles per iteration (tiles t, t + n_waves, ...):
// the NT tiles' rows, their features over one item range (NT x 208 items:
// 7 rounds for a pair where two single tiles take 8), their operands, then
// the hidden layers of all NT through mlp_hidden2_h3_multi (every LDS
// fragment read feeds NT MFMAs, the NT chains interleave) and the logit-
// difference label of each.  Labels bit-identical to ffn_wave_kernel.
// Feature rows at stride 20 (16 columns read, conflict-free ds_read_b128):
// per wave NT x (1,040 + 1,280) B of LDS.  VAD_FFN_GROUP = NT (0: off) for
// the labels-only analyser launches of 13-64-64-2.
// ---------------------------------------------------------------------------
#ifndef VAD_FFN_GROUP
#define VAD_FFN_GROUP 2
#endif
// waves per SIMD each group size fits: a pair 120 VGPRs (layer 1 one output
// tile at a time, VAD_FFN_L1_MTMAJOR) and 64.1 KB of LDS per 8-wave block
// (two blocks per CU): 4; larger groups 2
#ifndef VAD_FFN_GROUP_WPS
#define VAD_FFN_GROUP_WPS 0  // 0: by group size
#endif
template <int NT>
constexpr int kGroupWps = VAD_FFN_GROUP_WPS ? VAD_FFN_GROUP_WPS : NT <= 2 ? 4 : 2;
#ifndef VAD_FFN_GROUP_WPB
#define VAD_FFN_GROUP_WPB 8  // waves per block (sharing the block's LDS fragments)
#endif
constexpr int kGWpb = VAD_FFN_GROUP_WPB;
template <int MODE, int NT>
__global__ __launch_bounds__(64 * kGWpb) __attribute__((amdgpu_waves_per_eu(kGroupWps<NT>))) void ffn_wave_group_kernel(
    FfnDev net, const float* __restrict__ mfcc, int64_t n_rows, uint8_t* __restrict__ labels) {
  constexpr int KS0 = 4, T1 = 4, T2 = 4, NC = 2, MN = 13, IN = 13, XS = 20;
  using TP = Topo<KS0, T1, T2, 1, 0, NC, false>;
  using HP = HTopo<TP, KS0, T1, T2, 1, 0>;
  static_assert(TP::VL && TP::NL == 3, "VALU output layer");
  __shared__ float rows_s[kGWpb][NT][kWRows];
  __shared__ __attribute__((aligned(16))) float x_s[kGWpb][NT][kWTile * XS];
  __shared__ int flat_s[kGWpb][NT][kWTile];
  constexpr int NSL = TP::NB + TP::NV + TP::NVB;
  constexpr int NSD = TP::TIL * 4 + 1;
  constexpr int NSLP = (NSL + NSD + 3) & ~3;
  __shared__ __attribute__((aligned(16))) float slot_s[4 * NSLP];
  __shared__ u4 fh_s[HP::NS * 2 * 64];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int jw = lane & 15;
  const int64_t n_tiles = (n_rows + kWTile - 1) / kWTile;
  const int64_t total = (n_rows + 4) * MN;
  const int64_t wave_id = (int64_t)blockIdx.x * kGWpb + wv;
  const int64_t n_waves = (int64_t)gridDim.x * kGWpb;
  auto load = [&](int64_t t, float (&dst)[kWRowRegs]) {
    const int64_t base = t * (kWTile * MN);
    const float* tb = mfcc + base;
    const int64_t rem = total - 1 - base;
    const unsigned limb = 4u * (unsigned)(rem < kWRows ? rem : kWRows);
#pragma unroll
    for (int q = 0; q < kWRowRegs; ++q) {
      const unsigned ob = 4u * (unsigned)(lane + 64 * q);
      dst[q] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(tb) + (ob < limb ? ob : limb));
    }
  };
  // tile k of the group at t: t + k n_waves (clamped to t past the end:
  // computed, not stored)
  auto member = [&](int64_t t, int k) { return t + k * n_waves < n_tiles ? t + k * n_waves : t; };
  // the first group's rows are requested before the block stages its tables,
  // so the two latencies overlap
  float pre[NT][kWRowRegs];
  if (wave_id < n_tiles) {
#pragma unroll
    for (int k = 0; k < NT; ++k) load(member(wave_id, k), pre[k]);
  }
  // the slot table (biases, output-layer weights, the class-1 minus class-0
  // difference) and the split-f16 fragments, as in ffn_wave_kernel's kAll
  {
    auto slot_val = [&](int sl, int gg) {
      const int src_sl = sl < TP::NB ? TP::NA_ALL + sl
                                     : TP::NA_ALL + TP::NB + (sl - TP::NB < TP::NV ? sl - TP::NB
                                                                                  : 4 * TP::TIL * 4 + sl - TP::NB - TP::NV);
      return net.frag[src_sl * 64 + 16 * gg];
    };
    for (int i = threadIdx.x; i < 4 * NSLP; i += 64 * kGWpb) {
      const int gg = i / NSLP, sl = i - gg * NSLP;
      float v = 0.f;
      if (sl < NSL) {
        v = slot_val(sl, gg);
      } else if (sl < NSL + NSD) {
        const int q = sl - NSL;
        v = q < TP::TIL * 4 ? slot_val(TP::NB + TP::TIL * 4 + q, gg) - slot_val(TP::NB + q, gg)
                            : slot_val(TP::NB + TP::NV + 1, gg) - slot_val(TP::NB + TP::NV, gg);
      }
      slot_s[i] = v;
    }
    for (int i = threadIdx.x; i < HP::NS * 2 * 64; i += 64 * kGWpb) fh_s[i] = reinterpret_cast<const u4*>(net.fragh)[i];
    __syncthreads();
  }
  const LdsRow fbs{slot_s + g * NSLP};
  const LdsRow fvs{slot_s + g * NSLP + TP::NB};
  const LdsRow fds{slot_s + g * NSLP + NSL};
  const FragLds fh{fh_s, lane};
  for (int k = 0; k < NT; ++k)
    for (int i = lane; i < kWTile * XS; i += 64) x_s[wv][k][i] = 0.f;  // columns 13.. stay 0

  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt 0: no staging-load waits left for the loop body
  for (int64_t t = wave_id; t < n_tiles; t += NT * n_waves) {
    const int64_t tn = t + NT * n_waves < n_tiles ? t + NT * n_waves : t;
    wave_lds_handoff();
#pragma unroll
    for (int k = 0; k < NT; ++k)
#pragma unroll
      for (int q = 0; q < kWRowRegs; ++q)
        if (lane + 64 * q < kWRows) rows_s[wv][k][lane + 64 * q] = pre[k][q];
#pragma unroll
    for (int k = 0; k < NT; ++k) load(member(tn, k), pre[k]);
    wave_tile_features<IN, XS, MODE, NT, kWRows - kWTile * MN>(rows_s[wv][0], x_s[wv][0], flat_s[wv][0], lane);
#if VAD_FFN_PRIO
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(VAD_FFN_PRIO);
    __builtin_amdgcn_sched_barrier(0);
#endif
    float x[NT][1][8];
    int fl[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) fl[k] = wave_tile_operands<1, IN, XS, false>(x_s[wv][k], flat_s[wv][k], lane, x[k]);
    f32x4 h[NT][T2];
    mlp_hidden2_h3_multi<KS0, T1, T2, NT>(fh, fbs, x, h);
    int lab[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) lab[k] = valu_label2<TP, T2>(fds, fvs, h[k], fl[k]);
#if VAD_FFN_PRIO
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int k = 0; k < NT; ++k) {
      const int64_t tk = member(t, k);
      const int64_t w = tk * kWTile + jw;
      if (g == 0 && (k == 0 || tk != t) && w < n_rows) labels[w] = (uint8_t)lab[k];
    }
  }
}

// Streaming step for S analyser streams (sklearn_analyser.py:46-82): the
// window of each stream is its 5-slot MFCC ring in arrival order
// (slot (count + d) % 5, oldest first); classify it if count >= 5, then push
// the new frame's MFCC into the oldest slot (:74 after :71).
template <int KS0, int T1, int T2, int T3, int T4, int NC>
__global__ __launch_bounds__(256) void stream_ffn_kernel(FfnDev net, const float* __restrict__ newrow,
                                                         float* __restrict__ ring,
                                                         int* __restrict__ count, int64_t n_streams,
                                                         int mfcc_n, uint8_t* __restrict__ labels) {
  using TP = Topo<KS0, T1, T2, T3, T4, NC>;
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  const int jw = lane & 15;
  const int in_dim = net.dims[0];
  float fa[TP::NA];
  float fb[TP::NB];
  float fv[TP::NV + TP::NVB + 1];
  load_frags<TP>(net.frag, lane, fa, fb, fv);

  const int64_t n_tiles = (n_streams + 15) / 16;
  const int64_t wave_id = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t n_waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t tile = wave_id; tile < n_tiles; tile += n_waves) {
    const int64_t s = tile * 16 + jw;
    const bool valid = s < n_streams;
    const int c = valid ? count[s] : 0;
    const bool have = valid && c >= 5;
    float* rs = ring + s * 5 * mfcc_n;
    float x[KS0];
#pragma unroll
    for (int k = 0; k < KS0; ++k) {
      const int f = 4 * k + g;
      float v = 0.f;
      if (have && f < in_dim) {
        v = window_feature(rs + ((c + 0) % 5) * mfcc_n, rs + ((c + 1) % 5) * mfcc_n,
                           rs + ((c + 2) % 5) * mfcc_n, rs + ((c + 3) % 5) * mfcc_n,
                           rs + ((c + 4) % 5) * mfcc_n, f, mfcc_n, VAD_FEAT_ANALYSER);
      }
      x[k] = v;
    }
    const f32x4 z = mlp_forward<KS0, T1, T2, T3, T4, NC>(fa, fb, fv, x);
    if (valid) {
      if (g == 0) labels[s] = have ? (uint8_t)argmax_classes(z, net.n_classes) : (uint8_t)255;
      float* dst = rs + (c % 5) * mfcc_n;
      for (int cc = g; cc < mfcc_n; cc += 4) dst[cc] = newrow[s * mfcc_n + cc];
      if (g == 0) count[s] = (c + 1 >= 10) ? c + 1 - 5 : c + 1;
    }
  }
}

// Feature rows only (offline export / tests): one thread per (window, feature).
__global__ __launch_bounds__(256) void features_kernel(const float* __restrict__ mfcc,
                                                       int64_t n_rows, int mfcc_n, int mode,
                                                       float* __restrict__ out) {
  const int nf = 3 * mfcc_n;
  const int64_t total = n_rows * nf;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = i / nf;
    const int f = (int)(i - w * nf);
    const float* r0 = mfcc + w * mfcc_n;
    out[i] = window_feature(r0, r0 + mfcc_n, r0 + 2 * mfcc_n, r0 + 3 * mfcc_n, r0 + 4 * mfcc_n, f,
                            mfcc_n, mode);
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int KS0, int T1, int T2, int T3, int T4, int NC = 4>
static hipError_t launch_stream_topo(const FfnDev& net, const float* newrow, float* ring, int* count,
                                     int64_t n_streams, int mfcc_n, uint8_t* labels, hipStream_t st) {
  const int64_t n_tiles = (n_streams + 15) / 16;
  int64_t blocks = (n_tiles + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL((stream_ffn_kernel<KS0, T1, T2, T3, T4, NC>), dim3((int)blocks), dim3(256), 0, st,
                     net, newrow, ring, count, n_streams, mfcc_n, labels);
  return hipGetLastError();
}

static int ffn_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <int KS0, int T1, int T2, int T3, int T4, int NC = 4>
static hipError_t launch_topo(const FfnDev& net, int src, const float* in, int64_t n_rows,
                              int mfcc_n, int mode, uint8_t* labels, hipStream_t st) {
  const int64_t n_tiles = (n_rows + 15) / 16;
  int64_t blocks = (n_tiles + 3) / 4;
  if (blocks > 2048) blocks = 2048;
  if (src == kFromMfcc) {
    int64_t chunks = (n_rows + kChunk - 1) / kChunk;
    // persistent: one resident wave of blocks (2 per CU at ~200 registers),
    // so each block loads its weight fragments once and streams its chunks
    const int64_t cap = 2 * ffn_num_cus();
    if (chunks > cap) chunks = cap;
    // split-f16 MFMA: the two specialised topologies, when the plan has fragh
    constexpr bool kH3 = (KS0 == 10 && T1 == 4 && T2 == 2 && T3 == 1 && T4 == 1) ||
                         (KS0 == 4 && T1 == 4 && T2 == 4 && T3 == 1 && T4 == 0);
    if constexpr (kH3) {
      if constexpr (KS0 == 4 && NC <= 2) {
        // tile groups: labels-only analyser launches whose layer-1 inputs the
        // host proved f16-bounded (the single-tile kernel keeps the rescale)
        if (VAD_FFN_GROUP >= 2 && mfcc_n == 13 && net.fragh && !net.logits && net.h1_bounded &&
            mode == VAD_FEAT_ANALYSER && net.n_classes == 2) {
          constexpr int NT = VAD_FFN_GROUP >= 2 ? VAD_FFN_GROUP : 2;
          const int64_t n_tiles = (n_rows + kWTile - 1) / kWTile;
          int64_t gblocks = ((n_tiles + NT - 1) / NT + kGWpb - 1) / kGWpb;
          const int64_t gcap = kGroupWps<NT> * 4 / kGWpb * ffn_num_cus();
          if (gblocks > gcap) gblocks = gcap;
          hipLaunchKernelGGL((ffn_wave_group_kernel<VAD_FEAT_ANALYSER, NT>), dim3((int)gblocks), dim3(64 * kGWpb), 0, st,
                             net, in, n_rows, labels);
          return hipGetLastError();
        }
      }
      if (mfcc_n == 13 && net.fragh && VAD_FFN_WAVE) {
        // one resident wave per SIMD pair slot: 2 blocks of 4 waves per CU
        int64_t wblocks = (n_rows + kWpb * kWTile - 1) / (kWpb * kWTile);
        const int64_t wcap = WaveResidency<KS0, NC>::kWavesPerSimd * 4 / kWpb * ffn_num_cus();
        if (wblocks > wcap) wblocks = wcap;
        const dim3 grid((int)wblocks), blk(64 * kWpb);
        if (mode == VAD_FEAT_OFFLINE) {
          if (net.logits)
            hipLaunchKernelGGL((ffn_wave_kernel<KS0, T1, T2, T3, T4, NC, VAD_FEAT_OFFLINE, true>), grid, blk, 0, st,
                               net, in, n_rows, labels);
          else
            hipLaunchKernelGGL((ffn_wave_kernel<KS0, T1, T2, T3, T4, NC, VAD_FEAT_OFFLINE, false>), grid, blk, 0, st,
                               net, in, n_rows, labels);
        } else {
          if (net.logits)
            hipLaunchKernelGGL((ffn_wave_kernel<KS0, T1, T2, T3, T4, NC, VAD_FEAT_ANALYSER, true>), grid, blk, 0, st,
                               net, in, n_rows, labels);
          else
            hipLaunchKernelGGL((ffn_wave_kernel<KS0, T1, T2, T3, T4, NC, VAD_FEAT_ANALYSER, false>), grid, blk, 0, st,
                               net, in, n_rows, labels);
        }
        return hipGetLastError();
      }
      if (mfcc_n == 13 && net.fragh) {
        if (mode == VAD_FEAT_OFFLINE)
          hipLaunchKernelGGL((ffn_window_h3_kernel<KS0, T1, T2, T3, T4, NC, 13, VAD_FEAT_OFFLINE>),
                             dim3((int)chunks), dim3(256), 0, st, net, in, n_rows, mfcc_n, mode, labels);
        else
          hipLaunchKernelGGL((ffn_window_h3_kernel<KS0, T1, T2, T3, T4, NC, 13, VAD_FEAT_ANALYSER>),
                             dim3((int)chunks), dim3(256), 0, st, net, in, n_rows, mfcc_n, mode, labels);
        return hipGetLastError();
      }
    }
    if (mfcc_n == 13)
      hipLaunchKernelGGL((ffn_window_kernel<KS0, T1, T2, T3, T4, NC, 13>), dim3((int)chunks), dim3(256), 0,
                         st, net, in, n_rows, mfcc_n, mode, labels);
    else
      hipLaunchKernelGGL((ffn_window_kernel<KS0, T1, T2, T3, T4, NC, 0>), dim3((int)chunks), dim3(256), 0,
                         st, net, in, n_rows, mfcc_n, mode, labels);
  } else
    hipLaunchKernelGGL((ffn_kernel<KS0, T1, T2, T3, T4, NC, kFromRows>), dim3((int)blocks), dim3(256), 0,
                       st, net, in, n_rows, mfcc_n, mode, labels);
  return hipGetLastError();
}

// Topologies compiled: the reference Keras FFN 39-64-32-16-3
// (ffn_trainer.py:106-116), BASELINE config 3's 13-64-64-2, and a padded
// generic shape for anything else within the limits.
hipError_t launch_ffn(const FfnDev& net, int src, const float* in, int64_t n_rows, int mfcc_n,
                      int mode, uint8_t* labels, hipStream_t st) {
  if (n_rows <= 0) return hipSuccess;
  const int* t = net.tiles;
  if (net.n_layers == 4 && net.ks0 == 10 && t[0] == 4 && t[1] == 2 && t[2] == 1 && t[3] == 1)
    return launch_topo<10, 4, 2, 1, 1>(net, src, in, n_rows, mfcc_n, mode, labels, st);
  if (net.n_layers == 3 && net.ks0 == 4 && t[0] == 4 && t[1] == 4 && t[2] == 1) {
    if (net.n_classes <= 2)
      return launch_topo<4, 4, 4, 1, 0, 2>(net, src, in, n_rows, mfcc_n, mode, labels, st);
    return launch_topo<4, 4, 4, 1, 0>(net, src, in, n_rows, mfcc_n, mode, labels, st);
  }
  switch (net.n_layers) {
    case 1: return launch_topo<16, 1, 0, 0, 0>(net, src, in, n_rows, mfcc_n, mode, labels, st);
    case 2: return launch_topo<16, 4, 1, 0, 0>(net, src, in, n_rows, mfcc_n, mode, labels, st);
    case 3: return launch_topo<16, 4, 4, 1, 0>(net, src, in, n_rows, mfcc_n, mode, labels, st);
    default: return launch_topo<16, 4, 4, 4, 1>(net, src, in, n_rows, mfcc_n, mode, labels, st);
  }
}

hipError_t launch_stream_ffn(const FfnDev& net, const float* newrow, float* ring, int* count,
                             int64_t n_streams, int mfcc_n, uint8_t* labels, hipStream_t st) {
  if (n_streams <= 0) return hipSuccess;
  const int* t = net.tiles;
  if (net.n_layers == 4 && net.ks0 == 10 && t[0] == 4 && t[1] == 2 && t[2] == 1 && t[3] == 1)
    return launch_stream_topo<10, 4, 2, 1, 1>(net, newrow, ring, count, n_streams, mfcc_n, labels, st);
  if (net.n_layers == 3 && net.ks0 == 4 && t[0] == 4 && t[1] == 4 && t[2] == 1) {
    if (net.n_classes <= 2)
      return launch_stream_topo<4, 4, 4, 1, 0, 2>(net, newrow, ring, count, n_streams, mfcc_n, labels, st);
    return launch_stream_topo<4, 4, 4, 1, 0>(net, newrow, ring, count, n_streams, mfcc_n, labels, st);
  }
  switch (net.n_layers) {
    case 1: return launch_stream_topo<16, 1, 0, 0, 0>(net, newrow, ring, count, n_streams, mfcc_n, labels, st);
    case 2: return launch_stream_topo<16, 4, 1, 0, 0>(net, newrow, ring, count, n_streams, mfcc_n, labels, st);
    case 3: return launch_stream_topo<16, 4, 4, 1, 0>(net, newrow, ring, count, n_streams, mfcc_n, labels, st);
    default: return launch_stream_topo<16, 4, 4, 4, 1>(net, newrow, ring, count, n_streams, mfcc_n, labels, st);
  }
}

hipError_t launch_features(const float* mfcc, int64_t n_rows, int mfcc_n, int mode, float* out,
                           hipStream_t st) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows * 3 * mfcc_n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(features_kernel, dim3((int)blocks), dim3(256), 0, st, mfcc, n_rows, mfcc_n,
                     mode, out);
  return hipGetLastError();
}

}  // namespace vad
