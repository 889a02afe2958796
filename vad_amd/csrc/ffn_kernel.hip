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

namespace vad {

// argmax of softmax(z) with np.argmax semantics on the fp32 logits: any NaN
// (or an all-NaN softmax from +inf / all -inf) -> class 0; else first max.
__device__ __forceinline__ int argmax_classes(const f32x4 z, int n_classes) {
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

__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
  // plain conversions, not v_fma_mix* inline asm (one instruction less per
  // value, but the compiler cannot see an asm VALU write that a following
  // MFMA reads as an operand, so it could not pad that hazard)
  u4 hw, lw;
#pragma unroll
  for (int q = 0; q < 8; q += 2) {
    const f2 p = {v[q], v[q + 1]};
    const h2 h = __builtin_convertvector(p, h2);
    const h2 r = __builtin_convertvector(p - __builtin_convertvector(h, f2), h2);
    hw[q / 2] = __builtin_bit_cast(unsigned, h);
    lw[q / 2] = __builtin_bit_cast(unsigned, r);
  }
  hi = __builtin_bit_cast(h8, hw);
  lo = __builtin_bit_cast(h8, lw);
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
template <int K>
__device__ __forceinline__ float layer_scale(float (&v)[K][8]) {
  // inputs are NaN-free (ffn_window_body masks NaN windows) and VALU
  // results or LDS reads (never MFMA results, whose read hazard inline asm
  // would hide): one v_max3 per pair, no canonicalising maxNum sequence
  float m = 0.f;
#pragma unroll
  for (int s = 0; s < K; ++s)
#pragma unroll
    for (int q = 0; q < 8; q += 2)
      asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(m) : "v"(m), "v"(v[s][q]), "v"(v[s][q + 1]));
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
template <int TO, int KS, class FB, class FH>
__device__ __forceinline__ void dense_h3(FH A, FB b, float (&v)[KS][8], f32x4 (&out)[TO], bool relu) {
  const float sc = layer_scale<KS>(v);
  h8 bh[KS], bl[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) split8(v[s], bh[s], bl[s]);
  auto chain = [&](const f32x4 (&init)[TO], f32x4 (&acc)[TO]) {
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
    // NaN-free here: clamp to [0, inf) is the ReLU (a builtin, not asm: the
    // operand is an MFMA result, whose read hazard the compiler must see)
    if (relu) {
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = __builtin_amdgcn_fmed3f(o[r], 0.f, __builtin_inff());
    }
    out[mt] = o;
  }
  __builtin_amdgcn_sched_barrier(0);
}

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
          class FH>
__device__ __forceinline__ f32x4 mlp_forward_h3(FH fh, FB fb, FV fv, float (&x0)[(4 * KS0 + 31) / 32][8]) {
  using TP = Topo<KS0, T1, T2, T3, T4, NC, NOVL>;
  using HP = HTopo<TP, KS0, T1, T2, T3, T4>;
  f32x4 h1[T1];
  dense_h3<T1, HP::K0, FB>(fh, fb, x0, h1, TP::NL > 1);
  if constexpr (TP::NL == 1) return h1[0];
  else if constexpr (TP::NL == 2 && TP::VL) return valu_out_layer<TP, T1, FV>(fv, h1);
  else {
    float v1[HP::K1][8];
    acts_of<T1>(h1, v1);
    f32x4 h2[T2];
    dense_h3<T2, HP::K1, FB>(fh.at(HP::S0), fb + 4 * T1, v1, h2, TP::NL > 2);
    if constexpr (TP::NL == 2) return h2[0];
    else if constexpr (TP::NL == 3 && TP::VL) return valu_out_layer<TP, T2, FV>(fv, h2);
    else {
      float v2[HP::K2][8];
      acts_of<T2>(h2, v2);
      f32x4 h3[T3];
      dense_h3<T3, HP::K2, FB>(fh.at(HP::S0 + HP::S1), fb + 4 * (T1 + T2), v2, h3,
                               TP::NL > 3);
      if constexpr (TP::NL == 3) return h3[0];
      else if constexpr (TP::VL) return valu_out_layer<TP, T3, FV>(fv, h3);
      else {
        float v3[HP::K3][8];
        acts_of<T3>(h3, v3);
        f32x4 h4[T4];
        dense_h3<T4, HP::K3, FB>(fh.at(HP::S0 + HP::S1 + HP::S2), fb + 4 * (T1 + T2 + T3),
                                 v3, h4, false);
        return h4[0];
      }
    }
  }
}

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
    if (g == 0 && valid) labels[w] = (uint8_t)argmax_classes(z, net.n_classes);
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
#ifndef VAD_FFN_DIAG
#define VAD_FFN_DIAG 0  // diagnostic builds only: 1 skips the features, 2 the MLP
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
      if (q < kChunk / 4 && VAD_FFN_DIAG != 1) {
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
    for (int i = tid; i < (VAD_FFN_DIAG == 1 ? 0 : nwin * mfcc_n); i += 256) {
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
    f32x4 z;
    if constexpr (H3) {
      // windows past nwin read stale (finite) features: computed, not stored
      float x0[HP::K0][8];
      const v4f* xr = reinterpret_cast<const v4f*>(Xb + wl * kXStride + 8 * g);
#pragma unroll
      for (int s = 0; s < HP::K0; ++s) {
        const v4f lo4 = xr[8 * s], hi4 = xr[8 * s + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x0[s][q] = lo4[q];
          x0[s][q + 4] = hi4[q];
        }
      }
      if (VAD_FFN_DIAG == 2) z = (f32x4){x0[0][0], x0[0][1], 0.f, 0.f};
      else z = mlp_forward_h3<KS0, T1, T2, T3, T4, NC>(FragRegs{fh}, (const float*)fb, (const float*)fv, x0);
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
    if (g == 0 && wl < nwin) labels[w] = (uint8_t)argmax_classes(z, net.n_classes);
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
template <int KS0, int NC>
struct WaveResidency {
  static constexpr bool kLdsFrags = KS0 == 10 || NC > 2;
  static constexpr int kWavesPerSimd = KS0 == 10 ? 3 : 2;
};
constexpr int kWTile = 16;                       // windows per wave tile
constexpr int kWRows = (kWTile + 4) * 13;        // staged MFCC floats per tile (260)
constexpr int kWRowRegs = (kWRows + 63) / 64;    // 5 per lane

template <int KS0, int T1, int T2, int T3, int T4, int NC, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WaveResidency<KS0, NC>::kWavesPerSimd))) void ffn_wave_kernel(
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
  __shared__ float rows_s[4][kWRows];
  __shared__ __attribute__((aligned(16))) float x_s[4][kWTile * XS];
  __shared__ int flat_s[4][kWTile];  // per window: some coefficient is flat (NaN features)
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
  const int g = lane >> 4;
  const int jw = lane & 15;
  float* R = rows_s[wv];
  float* X = x_s[wv];
  int* FL = flat_s[wv];

  float fa[1];
  float fb[TP::NB];
  float fv[TP::NV + TP::NVB + 1];
  load_frags<TP, true>(net.frag, lane, fa, fb, fv);
  constexpr bool kLdsFrags = WaveResidency<KS0, NC>::kLdsFrags;
  __shared__ u4 fh_s[kLdsFrags ? HP::NS * 2 * 64 : 1];
  u4 fh_r[kLdsFrags ? 1 : HP::NS][2];
  if constexpr (kLdsFrags) {
    for (int i = threadIdx.x; i < HP::NS * 2 * 64; i += 256) fh_s[i] = reinterpret_cast<const u4*>(net.fragh)[i];
    __syncthreads();
  } else {
    load_fragh<HP>(net.fragh, lane, *reinterpret_cast<u4(*)[HP::NS][2]>(fh_r));
  }
  const auto fh = [&] {
    if constexpr (kLdsFrags) return FragLds{fh_s, lane};
    else return FragRegs{fh_r};
  }();
  // feature columns IN .. 32 K0 - 1 are read by layer 0 and stay 0
  for (int i = lane; i < kWTile * XS; i += 64) X[i] = 0.f;

  const int64_t n_tiles = (n_rows + kWTile - 1) / kWTile;
  const int64_t total = (n_rows + 4) * MN;  // MFCC floats the windows can read
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + wv;
  const int64_t n_waves = (int64_t)gridDim.x * 4;
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
#pragma unroll
    for (int q = 0; q < kWRowRegs; ++q)
      if (lane + 64 * q < kWRows) R[lane + 64 * q] = pre[q];
    load(tn < n_tiles ? tn : t, pre);
    // features (sklearn_analyser.py:52-69 / file_processing.py:51-66): item
    // i = 13 w + c is coefficient c of window w; its rows are R[i + 13 d].
    // A flat coefficient (the analyser's 0/0: mn and d2 NaN) writes its
    // features as 0 and stores 1 into its window's flag (after the wave's own
    // zeroing stores, in LDS order; a ds_or_b32 from all 13 coefficient lanes
    // instead serialises on the one address: +2.5 us per 1M windows)
    if (lane < kWTile) FL[lane] = 0;
#pragma unroll
    for (int r = 0; r < (kWTile * MN + 63) / 64; ++r) {
      const int it = lane + 64 * r;
      if ((r < kWTile * MN / 64 || it < kWTile * MN) && VAD_FFN_DIAG != 1) {
        const int w = it / MN, c = it - MN * w;
        const Feat3 ft = feature_triple(R[it], R[it + MN], R[it + 2 * MN], R[it + 3 * MN],
                                        R[it + 4 * MN], MODE);
        const bool flat = ft.mn != ft.mn;
        if (flat) FL[w] = 1;
        float* xw = X + w * XS;
        xw[c] = flat ? 0.f : ft.mn;
        if constexpr (IN > MN) {
          xw[MN + c] = ft.d1;
          xw[2 * MN + c] = flat ? 0.f : ft.d2;
        }
      }
    }
    // layer-0 B operands: lane (g, jw) holds features 32 s + 8 g + q of window jw
    float x0[HP::K0][8];
    const v4f* xr = reinterpret_cast<const v4f*>(X + jw * XS + 8 * g);
#pragma unroll
    for (int s = 0; s < HP::K0; ++s) {
      const v4f lo4 = xr[8 * s], hi4 = xr[8 * s + 1];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        x0[s][q] = lo4[q];
        x0[s][q + 4] = hi4[q];
      }
    }
    const int wnan = FL[jw];
    f32x4 z;
    if (VAD_FFN_DIAG == 2) z = (f32x4){x0[0][0], x0[0][1], 0.f, 0.f};
    else z = mlp_forward_h3<KS0, T1, T2, T3, T4, NC, const float*, const float*, VAD_FFN_WAVE_MFMA_OUT != 0>(
        fh, (const float*)fb, (const float*)fv, x0);
    if (wnan) z = (f32x4){__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
    const int64_t w = t * kWTile + jw;
    if (g == 0 && w < n_rows) labels[w] = (uint8_t)argmax_classes(z, net.n_classes);
  };
  // VAD_FFN_PF tiles per trip, each with its own prefetch registers (no
  // copies at the back edge): a tile's rows are loaded PF tiles ahead
  float pre[VAD_FFN_PF][kWRowRegs];
#pragma unroll
  for (int k = 0; k < VAD_FFN_PF; ++k) {
    const int64_t tk = wave_id + k * n_waves;
    load(tk < n_tiles ? tk : 0, pre[k]);
  }
  for (int64_t t = wave_id; t < n_tiles; t += VAD_FFN_PF * n_waves) {
#pragma unroll
    for (int k = 0; k < VAD_FFN_PF; ++k) {
      const int64_t tk = t + k * n_waves;
      if (k > 0 && tk >= n_tiles) break;
      tile_body(tk, tk + VAD_FFN_PF * n_waves, pre[k]);
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
      if (mfcc_n == 13 && net.fragh && VAD_FFN_WAVE) {
        // one resident wave per SIMD pair slot: 2 blocks of 4 waves per CU
        int64_t wblocks = (n_rows + 4 * kWTile - 1) / (4 * kWTile);
        const int64_t wcap = WaveResidency<KS0, NC>::kWavesPerSimd * ffn_num_cus();
        if (wblocks > wcap) wblocks = wcap;
        if (mode == VAD_FEAT_OFFLINE)
          hipLaunchKernelGGL((ffn_wave_kernel<KS0, T1, T2, T3, T4, NC, VAD_FEAT_OFFLINE>),
                             dim3((int)wblocks), dim3(256), 0, st, net, in, n_rows, labels);
        else
          hipLaunchKernelGGL((ffn_wave_kernel<KS0, T1, T2, T3, T4, NC, VAD_FEAT_ANALYSER>),
                             dim3((int)wblocks), dim3(256), 0, st, net, in, n_rows, labels);
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
