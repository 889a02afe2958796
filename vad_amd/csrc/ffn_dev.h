// Device building blocks of the FFN forward (ffn_trainer.py:106-116), shared by
// the window / wave kernels (ffn_kernel.hip) and the fused MFCC + FFN kernel
// (mfcc_kernel.hip): argmax, exact-f32 MFMA layers, the split-f16 MFMA
// layers, the VALU output layer and the per-lane fragment accessors.
#pragma once

#include "vad_common.h"
#include "features.h"

#ifndef VAD_FEAT_FLAGGED
#define VAD_FEAT_FLAGGED 1  // wave tile: flag NaN windows without adding the NaN in (one select less per item)
#endif
#ifndef VAD_FFN_MERGE0_SCALED
#define VAD_FFN_MERGE0_SCALED 1  // merged layer 0: each lane forms only its own half (no select)
#endif
#ifndef VAD_FFN_L1_MTMAJOR
#define VAD_FFN_L1_MTMAJOR 1  // tile groups' layer 1 one output tile at a time (its fragments only live)
#endif


namespace vad {

// argmax of softmax(z) with np.argmax semantics on the fp32 logits: any NaN
// (or an all-NaN softmax from +inf / all -inf) -> class 0; else first max.
__device__ __forceinline__ int argmax_classes(const f32x4 z, int n_classes) {
  // two classes (n_classes is wave-uniform): the same rules in two compares --
  // z1 > z0 is false when either is NaN, z0 = +inf or both are -inf, and
  // z1 < +inf rejects z1 = +inf (and NaN); ties go to class 0 (first max)
  if (n_classes == 2) return (z[1] > z[0]) & (z[1] < INFINITY);
  bool bad = false;
  float best = z[0];
  int arg = 0;
  bool any_pinf = false, all_ninf = true;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r < n_classes) {
      const float v = z[r];
      bad |= (v != v);
      any_pinf |= (v == INFINITY);
      all_ninf &= (v == -INFINITY);
      if (r > 0 && v > best) { best = v; arg = r; }
    }
  }
  if (bad || any_pinf || all_ninf) return 0;
  return arg;
}

// One MFMA layer: out[mt] = bias + sum over (t, r) of A[mt][t*4+r] x in[t][r].
// The K loop is outermost so the TO independent accumulator chains interleave
// (v_mfma_f32_16x16x4_f32: 32-cycle issue, 40-cycle dependent latency).
template <int TO, int TI>
__device__ __forceinline__ void dense_layer(const float* __restrict__ a, const float* __restrict__ b,
                                            const f32x4 (&in)[TI], f32x4 (&out)[TO], bool relu) {
  // TO == 1: two chains (even / odd K-steps) so consecutive MFMAs never wait
  // on each other; summed at the end (fixed order: deterministic).
  constexpr int NCH = TO == 1 ? 2 : 1;
  f32x4 acc[TO][NCH];
#pragma unroll
  for (int mt = 0; mt < TO; ++mt) {
    acc[mt][0] = (f32x4){b[mt * 4 + 0], b[mt * 4 + 1], b[mt * 4 + 2], b[mt * 4 + 3]};
    if constexpr (NCH == 2) acc[mt][NCH - 1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int t = 0; t < TI; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int mt = 0; mt < TO; ++mt) {
        f32x4& ac = acc[mt][(t * 4 + r) % NCH];
        ac = __builtin_amdgcn_mfma_f32_16x16x4f32(a[(mt * TI + t) * 4 + r], in[t][r], ac, 0, 0, 0);
      }
    }
  }
  // keep the whole layer's MFMAs back to back; the epilogue (bias already in,
  // ReLU) then waits once for the last accumulator instead of interleaving
  // accumulator reads into the next layer's MFMA stream
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int mt = 0; mt < TO; ++mt) {
    f32x4 v = acc[mt][0];
    if constexpr (NCH == 2) v = v + acc[mt][1];
    if (relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = relu_nan(v[r]);
    }
    out[mt] = v;
  }
  __builtin_amdgcn_sched_barrier(0);
}

// Network shape: KS0 layer-0 K-steps (4 features each), Tl = 16-row output
// tiles of layer l (0 = absent); the last present layer has one tile.  NC =
// classes the argmax reads (<= 4).  VL: the output layer runs on the VALU
// when its input spans >= 2 tiles -- a 16-row MFMA tile would waste 16-NC of
// its rows (13-64-64-2: 16 MFMAs per 16 windows become 32 FMAs per lane and a
// cross-lane sum).  NOVL keeps the output layer on the MFMA regardless (the
// wave kernel's split-f16 form, where it is the cheaper of the two).
template <int KS0, int T1, int T2, int T3, int T4, int NC = 4, bool NOVL = false>
struct Topo {
  static constexpr int NL = (T1 > 0) + (T2 > 0) + (T3 > 0) + (T4 > 0);
  static constexpr int TIL = NL == 2 ? T1 : NL == 3 ? T2 : NL == 4 ? T3 : 0;  // last layer's input tiles
  static constexpr bool VL = !NOVL && NL >= 2 && TIL >= 2;
  static constexpr int A0 = T1 * KS0;
  static constexpr int A1 = T2 * T1 * 4;
  static constexpr int A2 = T3 * T2 * 4;
  static constexpr int A3 = T4 * T3 * 4;
  static constexpr int NA_ALL = A0 + A1 + A2 + A3;
  static constexpr int A_LAST = NL == 1 ? A0 : NL == 2 ? A1 : NL == 3 ? A2 : A3;
  static constexpr int NB = 4 * (T1 + T2 + T3 + T4);
  // slots the kernel keeps in VGPRs: the output layer's MFMA A operands are
  // skipped when it runs on the VALU (they stay in the fragment array)
  static constexpr int NA = VL ? NA_ALL - A_LAST : NA_ALL;
  // VALU output layer: after the A and bias slots, slot (c*TIL + t)*4 + r ->
  // W_last[16t + 4g + r][c] (4 classes), then 4 slots of b_last[c]
  static constexpr int NV = VL ? NC * TIL * 4 : 0;
  static constexpr int NVB = VL ? NC : 0;
};

// Load the per-lane weight fragments a network keeps in VGPRs.
template <class TP, bool NO_A = false>
__device__ __forceinline__ void load_frags(const float* __restrict__ frag, int lane,
                                           float (&fa)[NO_A ? 1 : TP::NA], float (&fb)[TP::NB],
                                           float (&fv)[TP::NV + TP::NVB + 1]) {
  if constexpr (NO_A) {
    fa[0] = 0.f;
  } else {
#pragma unroll
    for (int s = 0; s < TP::NA; ++s) fa[s] = frag[s * 64 + lane];
  }
#pragma unroll
  for (int s = 0; s < TP::NB; ++s) fb[s] = frag[(TP::NA_ALL + s) * 64 + lane];
  constexpr int v0 = TP::NA_ALL + TP::NB;
  constexpr int ncl = TP::VL ? TP::NV / (TP::TIL * 4) : 0;
#pragma unroll
  for (int c = 0; c < ncl; ++c)
#pragma unroll
    for (int q = 0; q < TP::TIL * 4; ++q) fv[c * TP::TIL * 4 + q] = frag[(v0 + c * TP::TIL * 4 + q) * 64 + lane];
#pragma unroll
  for (int c = 0; c < TP::NVB; ++c) fv[TP::NV + c] = frag[(v0 + 4 * TP::TIL * 4 + c) * 64 + lane];
  fv[TP::NV + TP::NVB] = 0.f;
}

// Cross-row sums on the gfx950 row-swap permutes (VALU, no LDS round trip
// like ds_bpermute): v_permlane16_swap exchanges rows 1 / 3 of its first
// operand with rows 0 / 2 of its second, so with both holding p the two
// results add to p + p[lane ^ 16]; v_permlane32_swap likewise gives
// p + p[lane ^ 32].  Each lane's sum takes its operands in the same order as
// p + __shfl_xor(p, 16) then + __shfl_xor(., 32) (fp add commutes: results
// identical).  Inline asm: the clang builtin returns the first operand twice
// (checked on the device, tools/micro/permlane_check.hip); the s_nops cover
// the VALU-write -> permlane-read and permlane-write -> VALU-read distances
// the compiler cannot see through asm.
__device__ __forceinline__ float lane_sum_xor48(float p) {
  float a = p, b = p;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  float s = a + b;
  float c = s, d = s;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(c), "+v"(d));
  return c + d;
}
__device__ __forceinline__ int lane_or_xor48(int v) {
  int a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  int o = a | b;
  int c = o, d = o;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(c), "+v"(d));
  return c | d;
}

// VALU output layer: lane (g, window jw) holds hidden units 16t + 4g + r of
// its window; each class is a 16-term partial sum per lane, completed across
// the four lane groups (xor 16, xor 32: a fixed association, deterministic).
template <class TP, int TI, class FV = const float*>
__device__ __forceinline__ f32x4 valu_out_layer(FV fv, const f32x4 (&h)[TI], float bias_scale = 1.f) {
  constexpr int NC = TP::NVB;
  f32x4 z = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    float p0 = 0.f, p1 = 0.f;
#pragma unroll
    for (int t = 0; t < TI; ++t) {
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        p0 = fmaf(fv[(c * TI + t) * 4 + r], h[t][r], p0);
        p1 = fmaf(fv[(c * TI + t) * 4 + r + 1], h[t][r + 1], p1);
      }
    }
    const float p = lane_sum_xor48(p0 + p1);
    z[c] = p + fv[TP::NV + c] * bias_scale;
  }
  return z;
}

// Two-class label from the logit difference (labels-only launches of a
// network whose output layer runs on the VALU, 13-64-64-2): z1 - z0 =
// (W1 - W0) h + (b1 - b0) as ONE dot product per lane -- fd holds the TI*4
// difference weights of the lane group, then the bias difference (staged by
// the kernel, f32 differences of the plan's slots) -- instead of one per
// class, so label = d > 0 wherever the logits are finite: np.argmax's
// choice whenever the two logits differ by more than their rounding (a
// near-tie may fall either way, as between any two f32 summation orders; the
// labels' parity is the fp64 oracle's margin rule).  A
// non-finite d in a window that is not flagged (an overflowed layer) reruns
// the wave's output layer in the two-logit form, whose argmax rules (NaN,
// +-inf) decide then; a flagged window (wnan: its logits are NaN) is class 0.
template <class TP, int TI, class FD, class FV>
__device__ __forceinline__ int valu_label2(FD fd, FV fv, const f32x4 (&h)[TI], int wnan) {
  float p0 = 0.f, p1 = 0.f;
#pragma unroll
  for (int t = 0; t < TI; ++t) {
#pragma unroll
    for (int r = 0; r < 4; r += 2) {
      p0 = fmaf(fd[t * 4 + r], h[t][r], p0);
      p1 = fmaf(fd[t * 4 + r + 1], h[t][r + 1], p1);
    }
  }
  const float d = lane_sum_xor48(p0 + p1) + fd[TI * 4];
  const bool bad = !wnan && !(__builtin_fabsf(d) < INFINITY);
  if (__builtin_amdgcn_ballot_w64(bad)) {  // wave-uniform and rare: the two-logit rules
    f32x4 z = valu_out_layer<TP, TI, FV>(fv, h);
    if (wnan) z = (f32x4){__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    return argmax_classes(z, 2);
  }
  return wnan ? 0 : (d > 0.f);
}

template <int KS0, int T1, int T2, int T3, int T4, int NC>
__device__ __forceinline__ f32x4 mlp_forward(const float* __restrict__ fa, const float* __restrict__ fb,
                                             const float* __restrict__ fv, const float (&x)[KS0]) {
  using TP = Topo<KS0, T1, T2, T3, T4, NC>;
  f32x4 h1[T1];
#pragma unroll
  for (int mt = 0; mt < T1; ++mt) h1[mt] = (f32x4){fb[mt * 4 + 0], fb[mt * 4 + 1], fb[mt * 4 + 2], fb[mt * 4 + 3]};
#pragma unroll
  for (int s = 0; s < KS0; ++s) {
#pragma unroll
    for (int mt = 0; mt < T1; ++mt)
      h1[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[mt * KS0 + s], x[s], h1[mt], 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  if (TP::NL > 1) {
#pragma unroll
    for (int mt = 0; mt < T1; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) h1[mt][r] = relu_nan(h1[mt][r]);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (TP::NL == 1) return h1[0];
  else if constexpr (TP::NL == 2 && TP::VL) return valu_out_layer<TP, T1>(fv, h1);
  else {
    f32x4 h2[T2];
    dense_layer<T2, T1>(fa + TP::A0, fb + 4 * T1, h1, h2, TP::NL > 2);
    if constexpr (TP::NL == 2) return h2[0];
    else if constexpr (TP::NL == 3 && TP::VL) return valu_out_layer<TP, T2>(fv, h2);
    else {
      f32x4 h3[T3];
      dense_layer<T3, T2>(fa + TP::A0 + TP::A1, fb + 4 * (T1 + T2), h2, h3, TP::NL > 3);
      if constexpr (TP::NL == 3) return h3[0];
      else if constexpr (TP::VL) return valu_out_layer<TP, T3>(fv, h3);
      else {
        f32x4 h4[T4];
        dense_layer<T4, T3>(fa + TP::A0 + TP::A1 + TP::A2, fb + 4 * (T1 + T2 + T3), h3, h4, false);
        return h4[0];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Split-f16 MFMA forward (the specialised topologies): every GEMM operand is
// split as v = hi + lo with hi = f16(v), lo = f16(v - hi) (RNE), and a layer
// accumulates lo*hi + hi*lo + hi*hi on v_mfma_f32_16x16x32_f16 (f32
// accumulate; the dropped lo*lo term is ~2^-22 of a product).  16x16x32
// f16 takes 16 cycles against 32 for 16x16x4 f32 at 8x the K: the three
// products cost 3/16 of the exact-f32 MFMA time.  f16 holds |v| < 65504
// (NaN passes through as NaN): a tile with a larger layer input reruns on
// the exact f32 path.
// Operand layout (16x16x32): A lane (g, i) holds A[i][8g + q], B lane (g, j)
// holds B[8g + q][j], q = 0..7; D lane (g, j) holds D[4g + r][j].  The K
// order inside a K-step is the host's (capi.hip fragh): layer 0 k = input
// 32 s + 8g + q; later layers take the previous accumulator tiles 2s and
// 2s + 1 as the lane holds them, so no lane exchange between layers.
// ---------------------------------------------------------------------------
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr float kH3Max = 65504.f;  // largest finite f16

// v - f32(half SEL of the packed f16 pair hp), exact (v - f16(v) is a float):
// one v_fma_mix_f32 (-hi * 1 + v, the f16 operand widened inside the fma)
// instead of a conversion and a subtraction.  Inline asm is safe here: its
// result goes to the v_cvt_pk_f16_f32 that forms the lo halves (a VALU read,
// interlocked), never straight to an MFMA operand, whose read hazard after an
// asm VALU write the compiler could not pad.
template <int SEL>
__device__ __forceinline__ float sub_f16_half(float v, unsigned hp) {
  float d;
  if constexpr (SEL == 0)
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(hp), "v"(v));
  else
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(hp), "v"(v));
  return d;
}

__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
  u4 hw, lw;
#pragma unroll
  for (int q = 0; q < 8; q += 2) {
    const f2 p = {v[q], v[q + 1]};
    const h2 h = __builtin_convertvector(p, h2);
    const unsigned hb = __builtin_bit_cast(unsigned, h);
    const f2 d = {sub_f16_half<0>(v[q], hb), sub_f16_half<1>(v[q + 1], hb)};
    const h2 r = __builtin_convertvector(d, h2);
    hw[q / 2] = hb;
    lw[q / 2] = __builtin_bit_cast(unsigned, r);
  }
  hi = __builtin_bit_cast(h8, hw);
  lo = __builtin_bit_cast(h8, lw);
}

// v - s f32(half SEL of hp), s = 0 or 1 (a VGPR): the merged first layer's
// per-lane half (dense_h3 MERGE0)
template <int SEL>
__device__ __forceinline__ float sub_f16_half_scaled(float v, unsigned hp, float s) {
  float d;
  if constexpr (SEL == 0)
    asm("v_fma_mix_f32 %0, -%1, %3, %2 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(hp), "v"(v), "v"(s));
  else
    asm("v_fma_mix_f32 %0, -%1, %3, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d) : "v"(hp), "v"(v), "v"(s));
  return d;
}

__device__ __forceinline__ void split8_merged(const float (&v)[8], h8& out, float s) {
  u4 w;
#pragma unroll
  for (int q = 0; q < 8; q += 2) {
    const f2 p = {v[q], v[q + 1]};
    const h2 h = __builtin_convertvector(p, h2);
    const unsigned hb = __builtin_bit_cast(unsigned, h);
    const f2 d = {sub_f16_half_scaled<0>(v[q], hb, s), sub_f16_half_scaled<1>(v[q + 1], hb, s)};
    w[q / 2] = __builtin_bit_cast(unsigned, __builtin_convertvector(d, h2));
  }
  out = __builtin_bit_cast(h8, w);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = __builtin_fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Scale of one layer's inputs (wave-uniform): 1 while every |input| fits
// f16 (NaN passes through f16 as NaN and does not count), else the power of
// two that brings the wave's largest into [2^14, 2^15) -- the inputs are
// scaled in place and the layer unscales its result exactly.
template <int K, bool NONNEG = false>
__device__ __forceinline__ float layer_scale(float (&v)[K][8]) {
  // inputs are NaN-free (ffn_window_body masks NaN windows) and VALU
  // results or LDS reads (never MFMA results, whose read hazard inline asm
  // would hide): one v_max3 per pair, no canonicalising maxNum sequence.
  // NONNEG (the ReLU'd inputs of layers >= 1): an unsigned-integer max3 on
  // the bits, which orders non-negative floats like their values (no asm,
  // so no hazard padding around it)
  float m = 0.f;
  if constexpr (NONNEG) {
    unsigned mb = 0u;
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float e = v[s][q];
        const unsigned b = __builtin_bit_cast(unsigned, e);
        mb = mb > b ? mb : b;
      }
    m = __builtin_bit_cast(float, mb);
  } else {
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
      for (int q = 0; q < 8; q += 2)
        asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(m) : "v"(m), "v"(v[s][q]), "v"(v[s][q + 1]));
  }
  if (__builtin_amdgcn_ballot_w64(m >= kH3Max) == 0) return 1.f;
  // wave-uniform from here (readfirstlane): the callers' sc == 1 tests
  // become scalar branches, not exec-masked regions
  m = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, wave_max(m))));
  if (!(m < INFINITY)) return 1.f;  // inf stays inf (-> NaN logits, class 0)
  // m >= 65504 is a normal float: 2^(14 - exponent(m)), built from its bits
  const int e = (int)((__builtin_bit_cast(unsigned, m) >> 23) & 0xff) - 127;
  const float sc = __builtin_bit_cast(float, (unsigned)(127 + 14 - e) << 23);
#pragma unroll
  for (int s = 0; s < K; ++s)
#pragma unroll
    for (int q = 0; q < 8; ++q) v[s][q] *= sc;
  return sc;
}

// Layer inputs after a layer with TI accumulator tiles: K-step s takes tiles
// 2s and 2s + 1 as the lane holds them.
template <int TI>
__device__ __forceinline__ void acts_of(const f32x4 (&h)[TI], float (&v)[(TI + 1) / 2][8]) {
#pragma unroll
  for (int s = 0; s < (TI + 1) / 2; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[s][q] = h[2 * s][q];
      v[s][q + 4] = 2 * s + 1 < TI ? h[2 * s + 1][q] : 0.f;
    }
}

// out[mt] = bias + sum_s lo*hi + hi*lo + hi*hi (small terms first) on inputs
// v (scaled by sc, see layer_scale); the TO accumulator chains interleave.
// BOUNDED: the caller guarantees every input is finite and < 65504 in
// magnitude, or an infinity (layer_scale's answer is 1 then too): no check.
// bounded_rt: the same guarantee known at run time (wave-uniform).
template <int TO, int KS, class FB, bool NONNEG = false, bool MERGE0 = false, bool BOUNDED = false, class FH>
__device__ __forceinline__ void dense_h3(FH A, FB b, float (&v)[KS][8], f32x4 (&out)[TO], bool relu,
                                         bool bounded_rt = false) {
  const float sc = (BOUNDED || bounded_rt) ? 1.f : layer_scale<KS, NONNEG>(v);
  h8 bh[KS], bl[KS];
  if constexpr (MERGE0 && VAD_FFN_MERGE0_SCALED) {
    // lane groups g < 2 feed hi halves, g >= 2 lo halves: one split with the
    // residual scaled by 0 / 1 per lane, f16(v - s f32(f16 v)), gives each
    // lane its own half (s = 0: f16(v) bit for bit) without computing both
    // and selecting
    split8_merged(v[0], bh[0], (__builtin_amdgcn_workitem_id_x() & 63) >= 32 ? 1.f : 0.f);
    bl[0] = bh[0];
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) split8(v[s], bh[s], bl[s]);
  }
  // MERGE0 (a first layer of <= 16 inputs, one K-step): lane group g < 2
  // feeds the hi halves of inputs 8 (g & 1) + q as k = 0..15, g >= 2 their lo
  // halves as k = 16..31, against A = [W_lo | 0] then [W_hi | W_hi] (the
  // host's fragments): lo*hi, then hi*hi + hi*lo in one product -- two MFMAs
  // per tile instead of three
  const bool lo_half = (__builtin_amdgcn_workitem_id_x() & 63) >= 32;
  auto chain = [&](const f32x4 (&init)[TO], f32x4 (&acc)[TO]) {
    if constexpr (MERGE0) {
      static_assert(KS == 1, "merged first layer: one K-step");
      const h8 bm = lo_half ? bl[0] : bh[0];
#pragma unroll
      for (int mt = 0; mt < TO; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, A.get(mt, 1)), bm, init[mt], 0, 0, 0);
#pragma unroll
      for (int mt = 0; mt < TO; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, A.get(mt, 0)), bm, acc[mt], 0, 0, 0);
      return;
    }
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mt = 0; mt < TO; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, A.get(mt * KS + s, 1)), bh[s],
                                                         s == 0 ? init[mt] : acc[mt], 0, 0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mt = 0; mt < TO; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, A.get(mt * KS + s, 0)), bl[s],
                                                         acc[mt], 0, 0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int mt = 0; mt < TO; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, A.get(mt * KS + s, 0)), bh[s],
                                                         acc[mt], 0, 0, 0);
  };
  f32x4 bias[TO], acc[TO];
#pragma unroll
  for (int mt = 0; mt < TO; ++mt) bias[mt] = (f32x4){b[mt * 4 + 0], b[mt * 4 + 1], b[mt * 4 + 2], b[mt * 4 + 3]};
  if (sc == 1.f) {
    chain(bias, acc);  // the bias registers are the first MFMA's C operand
  } else {             // rare: scaled inputs, scaled bias, exact unscale
    f32x4 sb[TO];
#pragma unroll
    for (int mt = 0; mt < TO; ++mt) sb[mt] = bias[mt] * sc;
    chain(sb, acc);
    const float inv = 1.f / sc;  // exact: a power of two
#pragma unroll
    for (int mt = 0; mt < TO; ++mt) acc[mt] *= inv;
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int mt = 0; mt < TO; ++mt) {
    f32x4 o = acc[mt];
    // NaN-free here, so the ReLU is a signed-integer max with 0 on the bits
    // (negative floats, -0 included, are negative integers): one v_max_i32
    // per value -- a float max / med3 on an MFMA result compiles to a
    // canonicalising v_max_f32 first, two instructions per value
    if (relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // (the element goes through a scalar first: clang's bit_cast of an
        // ext_vector element expression reads element 0 whatever the index)
        const float e = o[r];
        const int bits = __builtin_bit_cast(int, e);
        o[r] = __builtin_bit_cast(float, bits > 0 ? bits : 0);
      }
    }
    out[mt] = o;
  }
  __builtin_amdgcn_sched_barrier(0);
}

// A first layer of <= 16 inputs (13-64-64-2) carries both halves of its
// split-f16 inputs in one K-step of 32 (dense_h3 MERGE0; capi.hip builds its
// fragments to match).
template <int KS0>
constexpr bool kMerge0 = 4 * KS0 <= 16;

// Split-f16 shape of a Topo: K-steps per layer and fragment slots.
template <class TP, int KS0, int T1, int T2, int T3, int T4>
struct HTopo {
  static constexpr int HL = TP::VL ? TP::NL - 1 : TP::NL;  // layers on split-f16 MFMA
  static constexpr int K0 = (4 * KS0 + 31) / 32;
  static constexpr int K1 = (T1 + 1) / 2, K2 = (T2 + 1) / 2, K3 = (T3 + 1) / 2;
  static constexpr int S0 = T1 * K0;
  static constexpr int S1 = HL > 1 ? T2 * K1 : 0;
  static constexpr int S2 = HL > 2 ? T3 * K2 : 0;
  static constexpr int S3 = HL > 3 ? T4 * K3 : 0;
  static constexpr int NS = S0 + S1 + S2 + S3;
};

template <class HP>
__device__ __forceinline__ void load_fragh(const uint32_t* __restrict__ fragh, int lane, u4 (&fh)[HP::NS][2]) {
  const u4* f = reinterpret_cast<const u4*>(fragh);
#pragma unroll
  for (int sl = 0; sl < HP::NS; ++sl) {
    fh[sl][0] = f[(2 * sl) * 64 + lane];
    fh[sl][1] = f[(2 * sl + 1) * 64 + lane];
  }
}

// Split-f16 weight fragments: slot sl, half h (0 = hi, 1 = lo) of this
// lane, from registers (FragRegs) or from a workgroup-shared LDS copy
// (FragLds, the plan's [slot][half][lane] layout).
struct FragRegs {
  const u4 (*p)[2];
  __device__ u4 get(int sl, int h) const { return p[sl][h]; }
  __device__ FragRegs at(int off) const { return {p + off}; }
};
struct FragLds {
  const u4* p;
  int lane;
  __device__ u4 get(int sl, int h) const { return p[(2 * sl + h) * 64 + lane]; }
  __device__ FragLds at(int off) const { return {p + 2 * off * 64, lane}; }
};

// Forward of one 16-window tile: x0 holds the layer-0 inputs of K-step s,
// k = 8g + q (g = lane >> 4).
template <int KS0, int T1, int T2, int T3, int T4, int NC, class FB, class FV, bool NOVL = false,
          bool IN_BOUNDED = false, class FH>
__device__ __forceinline__ f32x4 mlp_forward_h3(FH fh, FB fb, FV fv, float (&x0)[(4 * KS0 + 31) / 32][8]) {
  using TP = Topo<KS0, T1, T2, T3, T4, NC, NOVL>;
  using HP = HTopo<TP, KS0, T1, T2, T3, T4>;
  f32x4 h1[T1];
  dense_h3<T1, HP::K0, FB, false, kMerge0<KS0>, IN_BOUNDED>(fh, fb, x0, h1, TP::NL > 1);
  if constexpr (TP::NL == 1) return h1[0];
  else if constexpr (TP::NL == 2 && TP::VL) return valu_out_layer<TP, T1, FV>(fv, h1);
  else {
    float v1[HP::K1][8];
    acts_of<T1>(h1, v1);
    f32x4 h2[T2];
    dense_h3<T2, HP::K1, FB, true>(fh.at(HP::S0), fb + 4 * T1, v1, h2, TP::NL > 2);
    if constexpr (TP::NL == 2) return h2[0];
    else if constexpr (TP::NL == 3 && TP::VL) return valu_out_layer<TP, T2, FV>(fv, h2);
    else {
      float v2[HP::K2][8];
      acts_of<T2>(h2, v2);
      f32x4 h3[T3];
      dense_h3<T3, HP::K2, FB, true>(fh.at(HP::S0 + HP::S1), fb + 4 * (T1 + T2), v2, h3,
                               TP::NL > 3);
      if constexpr (TP::NL == 3) return h3[0];
      else if constexpr (TP::VL) return valu_out_layer<TP, T3, FV>(fv, h3);
      else {
        float v3[HP::K3][8];
        acts_of<T3>(h3, v3);
        f32x4 h4[T4];
        dense_h3<T4, HP::K3, FB, true>(fh.at(HP::S0 + HP::S1 + HP::S2), fb + 4 * (T1 + T2 + T3),
                                 v3, h4, false);
        return h4[0];
      }
    }
  }
}


// The hidden layers of a three-layer split-f16 network whose output layer
// runs on the VALU (13-64-64-2): the last hidden layer's accumulator tiles,
// for valu_label2.
// h1_bounded (FfnDev::h1_bounded, meaningful with IN_BOUNDED inputs): layer
// 1 skips its f16-range check too.
template <int KS0, int T1, int T2, class FB, bool IN_BOUNDED, class FH>
__device__ __forceinline__ void mlp_hidden2_h3(FH fh, FB fb, float (&x0)[(4 * KS0 + 31) / 32][8], f32x4 (&h2)[T2],
                                               bool h1_bounded) {
  using TP = Topo<KS0, T1, T2, 1, 0, 2, false>;
  using HP = HTopo<TP, KS0, T1, T2, 1, 0>;
  static_assert(TP::NL == 3 && TP::VL, "three layers, the output layer on the VALU");
  f32x4 h1[T1];
  dense_h3<T1, HP::K0, FB, false, kMerge0<KS0>, IN_BOUNDED>(fh, fb, x0, h1, true);
  float v1[HP::K1][8];
  acts_of<T1>(h1, v1);
  dense_h3<T2, HP::K1, FB, true>(fh.at(HP::S0), fb + 4 * T1, v1, h2, true, IN_BOUNDED && h1_bounded);
}

// The hidden layers of a 13-64-64-2-shaped network (merged first layer,
// bounded inputs, layer 1 under the host's bound) for NT 16-window tiles at
// once (the tile-group kernel): every weight fragment read (from LDS) feeds
// the NT tiles' MFMAs, and their accumulator chains interleave.  Per tile
// the arithmetic is dense_h3's, operation for operation: results
// bit-identical to NT mlp_hidden2_h3 calls.
template <int KS0, int T1, int T2, int NT, class FB, class FH>
__device__ __forceinline__ void mlp_hidden2_h3_multi(FH fh, FB fb, float (&x)[NT][1][8], f32x4 (&h)[NT][T2]) {
  using TP = Topo<KS0, T1, T2, 1, 0, 2, false>;
  using HP = HTopo<TP, KS0, T1, T2, 1, 0>;
  static_assert(kMerge0<KS0> && HP::K0 == 1, "merged first layer");
  constexpr int K1 = HP::K1;
  const float s = (__builtin_amdgcn_workitem_id_x() & 63) >= 32 ? 1.f : 0.f;
  auto relu4 = [](f32x4 o) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float e = o[r];
      const int bits = __builtin_bit_cast(int, e);
      o[r] = __builtin_bit_cast(float, bits > 0 ? bits : 0);
    }
    return o;
  };
  // layer 0: lo*hi, then hi*hi + hi*lo, each fragment on every tile
  h8 b0[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) split8_merged(x[t][0], b0[t], s);
  f32x4 h1[NT][T1];
  {
    f32x4 bias[T1];
#pragma unroll
    for (int mt = 0; mt < T1; ++mt) bias[mt] = (f32x4){fb[mt * 4 + 0], fb[mt * 4 + 1], fb[mt * 4 + 2], fb[mt * 4 + 3]};
#pragma unroll
    for (int mt = 0; mt < T1; ++mt) {
      const h8 a1 = __builtin_bit_cast(h8, fh.get(mt, 1));
#pragma unroll
      for (int t = 0; t < NT; ++t) h1[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0[t], bias[mt], 0, 0, 0);
    }
#pragma unroll
    for (int mt = 0; mt < T1; ++mt) {
      const h8 a0 = __builtin_bit_cast(h8, fh.get(mt, 0));
#pragma unroll
      for (int t = 0; t < NT; ++t) h1[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0[t], h1[t][mt], 0, 0, 0);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < T1; ++mt) h1[t][mt] = relu4(h1[t][mt]);
  __builtin_amdgcn_sched_barrier(0);
  // layer 1: lo*hi + hi*lo + hi*hi, small terms first, fragments shared
  h8 bh[NT][K1], bl[NT][K1];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float v[K1][8];
    acts_of<T1>(h1[t], v);
#pragma unroll
    for (int k = 0; k < K1; ++k) split8(v[k], bh[t][k], bl[t][k]);
  }
  const FH A = fh.at(HP::S0);
  const FB b1 = fb + 4 * T1;
  f32x4 bias[T2];
#pragma unroll
  for (int mt = 0; mt < T2; ++mt) bias[mt] = (f32x4){b1[mt * 4 + 0], b1[mt * 4 + 1], b1[mt * 4 + 2], b1[mt * 4 + 3]};
#if VAD_FFN_L1_MTMAJOR
  // one output tile mt at a time (its K1 lo and K1 hi fragments live, not
  // the layer's 2 T2 K1): each accumulator's products in the same order as
  // below, so the results are identical
#pragma unroll
  for (int mt = 0; mt < T2; ++mt) {
    h8 lo[K1], hi[K1];
#pragma unroll
    for (int k = 0; k < K1; ++k) {
      lo[k] = __builtin_bit_cast(h8, A.get(mt * K1 + k, 1));
      hi[k] = __builtin_bit_cast(h8, A.get(mt * K1 + k, 0));
    }
#pragma unroll
    for (int k = 0; k < K1; ++k)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        h[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo[k], bh[t][k], k == 0 ? bias[mt] : h[t][mt], 0, 0, 0);
#pragma unroll
    for (int k = 0; k < K1; ++k)
#pragma unroll
      for (int t = 0; t < NT; ++t) h[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi[k], bl[t][k], h[t][mt], 0, 0, 0);
#pragma unroll
    for (int k = 0; k < K1; ++k)
#pragma unroll
      for (int t = 0; t < NT; ++t) h[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi[k], bh[t][k], h[t][mt], 0, 0, 0);
  }
#else
#pragma unroll
  for (int k = 0; k < K1; ++k)
#pragma unroll
    for (int mt = 0; mt < T2; ++mt) {
      const h8 lo = __builtin_bit_cast(h8, A.get(mt * K1 + k, 1));
#pragma unroll
      for (int t = 0; t < NT; ++t)
        h[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo, bh[t][k], k == 0 ? bias[mt] : h[t][mt], 0, 0, 0);
    }
#pragma unroll
  for (int k = 0; k < K1; ++k)
#pragma unroll
    for (int mt = 0; mt < T2; ++mt) {
      const h8 hi = __builtin_bit_cast(h8, A.get(mt * K1 + k, 0));
#pragma unroll
      for (int t = 0; t < NT; ++t) h[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, bl[t][k], h[t][mt], 0, 0, 0);
    }
#pragma unroll
  for (int k = 0; k < K1; ++k)
#pragma unroll
    for (int mt = 0; mt < T2; ++mt) {
      const h8 hi = __builtin_bit_cast(h8, A.get(mt * K1 + k, 0));
#pragma unroll
      for (int t = 0; t < NT; ++t) h[t][mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi, bh[t][k], h[t][mt], 0, 0, 0);
    }
#endif
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int mt = 0; mt < T2; ++mt) h[t][mt] = relu4(h[t][mt]);
  __builtin_amdgcn_sched_barrier(0);
}

// Per-lane fragment slots read straight from global memory (L1 / L2
// resident: the plan's tables are a few tens of KB), for kernels whose VGPRs
// and LDS are taken by other work (the fused MFCC + FFN kernel).
//   FragGlobal: split-f16 slot sl, half h of this lane (plan fragh layout)
//   LaneSlots:  f32 slot s of this lane (plan frag layout, base slot b0)
//   VluSlots:   the VALU output layer's slots (classes < NC, then biases;
//               the host lays out 4 classes, so the biases sit at 4 TIL4)
struct FragGlobal {
  const u4* p;
  int lane;
  __device__ u4 get(int sl, int h) const { return p[(2 * sl + h) * 64 + lane]; }
  __device__ FragGlobal at(int off) const { return {p + 2 * off * 64, lane}; }
};
struct LaneSlots {
  const float* p;  // frag + b0 * 64 + lane
  __device__ float operator[](int s) const { return p[s * 64]; }
  __device__ LaneSlots operator+(int off) const { return {p + off * 64}; }
};
template <int NV, int TIL4>
struct VluSlots {
  const float* p;
  __device__ float operator[](int i) const { return p[(i < NV ? i : 4 * TIL4 + i - NV) * 64]; }
};
// The same slots from a compact LDS table tbl[slot * 4 + g] (a bias / output
// weight slot holds one value per lane group g = lane >> 4, so the 64-lane
// slot shrinks to 4 floats); p = tbl + 4 b0 + g.  The VALU output layer's
// table is compact too (its NC class slots, then its NC biases).
struct LdsSlots {
  const float* p;
  __device__ float operator[](int s) const { return p[4 * s]; }
  __device__ LdsSlots operator+(int off) const { return {p + 4 * off}; }
};


// ---------------------------------------------------------------------------
// One 16-window tile of a wave (the wave kernel's and the fused kernel's
// common tail).  R holds the tile's 20 MFCC rows at stride 13 (row w + d is
// frame d of window w); X (16 x XS floats) and FL (16 ints) are wave-private
// LDS scratch.
// ---------------------------------------------------------------------------
constexpr int kWTile = 16;  // windows per wave tile


// Lanes of one wave hand data to each other through LDS (rows -> features ->
// operands).  A wave's LDS operations execute in order, so no wait is needed,
// but in the language model each lane's accesses are independent and the
// compiler may move one lane's store past a load of another address once no
// branch separates them: this compiler barrier (no instruction) keeps the
// hand-off order.
__device__ __forceinline__ void wave_lds_handoff() { asm volatile("" ::: "memory"); }

// Features (sklearn_analyser.py:52-69 / file_processing.py:51-66): item
// i = 13 w + c is coefficient c of window w; its rows are R[i + 13 d].  A
// flat coefficient (the analyser's 0/0: mn and d2 NaN) writes its features
// as 0 and stores 1 into its window's flag (after the wave's own zeroing
// stores, in LDS order; a ds_or_b32 from all 13 coefficient lanes instead
// serialises on the one address: +2.5 us per 1M windows).
// NT tiles at once (the pair kernel: NT = 2): their items run on one range
// (NT * 208 items, ceil(NT * 208 / 64) rounds instead of NT * 4), tile k's
// rows at R + k (208 + RGAP), its feature rows and flags right after tile
// k - 1's (X + 16 k XS, FL + 16 k).
template <int IN, int XS, int MODE, int NT = 1, int RGAP = 0>
__device__ __forceinline__ void wave_tile_features(const float* __restrict__ R, float* __restrict__ X,
                                                   int* __restrict__ FL, int lane) {
  constexpr int MN = 13;
  constexpr int NI = NT * kWTile * MN;  // items
  wave_lds_handoff();  // the rows R were stored by other lanes of this wave
  if (lane < NT * kWTile) FL[lane] = 0;
#pragma unroll
  for (int r = 0; r < (NI + 63) / 64; ++r) {
    const int it = lane + 64 * r;
    if (r < NI / 64 || it < NI) {
      const int w = it / MN, c = it - MN * w;
      // the row offset of tile it / 208 (compile-time outside the one round
      // that straddles two tiles)
      int ri = it;
#pragma unroll
      for (int k = 1; k < NT; ++k) {
        constexpr int kTileItems = kWTile * MN;
        if (64 * r >= k * kTileItems) ri += RGAP;
        else if (64 * r + 63 >= k * kTileItems) ri += it >= k * kTileItems ? RGAP : 0;
      }
#if VAD_FEAT_FLAGGED
      bool flat;
      const Feat3 ft = feature_triple_flagged(R[ri], R[ri + MN], R[ri + 2 * MN], R[ri + 3 * MN],
                                              R[ri + 4 * MN], MODE, flat);
#else
      const Feat3 ft = feature_triple(R[ri], R[ri + MN], R[ri + 2 * MN], R[ri + 3 * MN],
                                      R[ri + 4 * MN], MODE);
      const bool flat = ft.mn != ft.mn;
#endif
      if (flat) FL[w] = 1;
      float* xw = X + w * XS;
      xw[c] = flat ? 0.f : ft.mn;
      if constexpr (IN > MN) {
        xw[MN + c] = ft.d1;
        xw[2 * MN + c] = flat ? 0.f : ft.d2;
      }
    }
  }
  wave_lds_handoff();  // other lanes read X / FL next (wave_tile_operands)
}

// Layer-0 B operands of window lane & 15 from X (lane (g, jw) holds
// features 32 s + 8 g + q of window jw) and the window's NaN flag.  MASK:
// X's columns IN .. 32 K0 - 1 hold stale data (not kept zero) and are zeroed
// in registers; without it the caller keeps them zero.
template <int K0, int IN, int XS, bool MASK>
__device__ __forceinline__ int wave_tile_operands(const float* __restrict__ X, const int* __restrict__ FL,
                                                  int lane, float (&x0)[K0][8]) {
  const int g = lane >> 4, jw = lane & 15;
  if constexpr (IN <= 16) {  // kMerge0: lane group g takes inputs 8 (g & 1) + q
    static_assert(K0 == 1, "one K-step");
    const v4f* xm = reinterpret_cast<const v4f*>(X + jw * XS + 8 * (g & 1));
    const v4f lo4 = xm[0], hi4 = xm[1];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      x0[0][q] = lo4[q];
      x0[0][q + 4] = hi4[q];
    }
    if constexpr (MASK) {  // else X's columns IN .. 15 are kept zero by the caller
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (8 + q >= IN) x0[0][q] = 8 * (g & 1) + q < IN ? x0[0][q] : 0.f;
    }
    return FL[jw];
  }
  const v4f* xr = reinterpret_cast<const v4f*>(X + jw * XS + 8 * g);
#pragma unroll
  for (int s = 0; s < K0; ++s) {
    const v4f lo4 = xr[8 * s], hi4 = xr[8 * s + 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      x0[s][q] = lo4[q];
      x0[s][q + 4] = hi4[q];
    }
  }
  if constexpr (MASK) {
#pragma unroll
    for (int s = 0; s < K0; ++s)
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (32 * s + q + 24 >= IN) x0[s][q] = 32 * s + 8 * g + q < IN ? x0[s][q] : 0.f;
  }
  return FL[jw];
}

// Analyser-mode inputs of a 13-input network are Mn = e2 / std alone: |Mn| <=
// sqrt(5) whenever finite (e2^2 <= sum of the five e_i^2 = 5 var), a NaN
// (flat or overflowed window: zeroed and flagged by the features) or +-inf
// (var = 0 from underflowed squares) -- never a finite value past f16's
// range, so layer 0 skips its range check (identical results).
template <int MODE, int IN>
constexpr bool wave_tile_in_bounded = MODE == VAD_FEAT_ANALYSER && IN == 13;

// Label of window lane & 15 (valid on every lane) from its layer-0 operands:
// the split-f16 forward, the NaN flag, argmax; z = its logits.
template <int KS0, int T1, int T2, int T3, int T4, int NC, bool NOVL, bool IN_BOUNDED, class FH, class FB,
          class FV>
__device__ __forceinline__ int wave_tile_mlp(float (&x0)[(4 * KS0 + 31) / 32][8], int wnan, FH fh, FB fb, FV fv,
                                             int n_classes, f32x4& z) {
  z = mlp_forward_h3<KS0, T1, T2, T3, T4, NC, FB, FV, NOVL, IN_BOUNDED>(fh, fb, fv, x0);
  if (wnan) z = (f32x4){__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
  return argmax_classes(z, n_classes);
}

// IN_BOUNDED (wave_tile_in_bounded): layer 0's inputs need no f16-range check
template <int KS0, int T1, int T2, int T3, int T4, int NC, bool NOVL, int IN, int XS, bool MASK, bool IN_BOUNDED,
          class FH, class FB, class FV>
__device__ __forceinline__ int wave_tile_classify(const float* __restrict__ X, const int* __restrict__ FL,
                                                  int lane, FH fh, FB fb, FV fv, int n_classes, f32x4& z) {
  constexpr int K0 = (4 * KS0 + 31) / 32;
  float x0[K0][8];
  const int wnan = wave_tile_operands<K0, IN, XS, MASK>(X, FL, lane, x0);
  return wave_tile_mlp<KS0, T1, T2, T3, T4, NC, NOVL, IN_BOUNDED>(x0, wnan, fh, fb, fv, n_classes, z);
}

// Label of window lane & 15 by the logit difference (valu_label2): every
// launch of a 13-64-64-2-shaped network; fd = the lane group's difference
// slots (TI*4 weights, then the bias).  z (when given: launches that also
// write the logits) receives the two logits from the same hidden layer, so a
// window's label never depends on whether its logits were requested.
template <int KS0, int T1, int T2, int IN, int XS, bool MASK, bool IN_BOUNDED, class FH, class FB, class FV, class FD>
__device__ __forceinline__ int wave_tile_label2(const float* __restrict__ X, const int* __restrict__ FL, int lane,
                                                FH fh, FB fb, FV fv, FD fd, int h1_bounded,
                                                f32x4* z = nullptr) {
  constexpr int K0 = (4 * KS0 + 31) / 32;
  using TP = Topo<KS0, T1, T2, 1, 0, 2, false>;
  float x0[K0][8];
  const int wnan = wave_tile_operands<K0, IN, XS, MASK>(X, FL, lane, x0);
  f32x4 h2[T2];
  mlp_hidden2_h3<KS0, T1, T2, FB, IN_BOUNDED>(fh, fb, x0, h2, h1_bounded != 0);
  if (z) {
    f32x4 zz = valu_out_layer<TP, T2, FV>(fv, h2);
    if (wnan) zz = (f32x4){__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    *z = zz;
  }
  return valu_label2<TP, T2>(fd, fv, h2, wnan);
}

// optional logits output (FfnDev::logits, tests): row w's fp32 logits
__device__ __forceinline__ void store_logits(float* logits, int64_t w, const f32x4& z, int n_classes) {
  if (!logits) return;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < n_classes) logits[w * n_classes + c] = z[c];
}

}  // namespace vad
