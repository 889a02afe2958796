// Fused MFCC kernel for gfx950: framing -> 512-point real FFT -> |X/512|^2 ->
// sparse mel matvec -> (==0 -> eps) -> log10 -> lifter x DCT-II ortho.
//
// Reference semantics: mfcc.py:59-78 (get_spec_mag, get_mfcc_from_spec,
// lifter), file_processing.py:80-103 (framing).
//
// Work decomposition (one 512-thread workgroup = 8 waves per 64-frame tile):
//   phase 1  16 lanes per frame, 32 frames per pass, 2 passes.
//            The real 512-point FFT is a 256-point complex FFT of
//            z[n] = x[2n] + i x[2n+1] (x[t] = 0 for t >= 400, so z[n >= 200]
//            = 0), split 16 x 16:
//              stage A  lane n2 owns z[16 n1 + n2] (n1 < 13 non-zero), DFT16
//                       in registers, twiddle W256^(n2 k1), store to LDS;
//              stage B  lane j owns the even half of column cE and the odd
//                       half of column cO = 16 - cE (two DFT8s in registers),
//                       so the real-FFT partner Z[256-k] of every Z[k] it
//                       holds is in its own registers (column 0 is the one
//                       exception, handled by a per-lane select);
//              post     X[k] = (S - i W512^k D) / 2, P[k] = |X[k] / 512|^2,
//                       written to an LDS power tile P[64][260].
//   phase 2a one frame per lane, each wave owns a band of filters (balanced
//            by tap count): mel energies, (==0 -> eps), log10 -> LDS log-mel
//            rows.
//   phase 2b one frame per lane, waves 0..3 own coefficients c = w + 4 i:
//            lifter x DCT of the log-mel rows, stored to the MFCC rows.  It
//            runs deferred, in the next tile after phase 1, on the waves that
//            finish their FFT first -- two barriers per tile.
#include <type_traits>

#include "vad_common.h"
#include "fft_pk.h"
#include "mel_tables.h"
#include "ffn_dev.h"

namespace vad {

constexpr int kTile = 64;        // frames per workgroup tile
constexpr int kThreads = 512;    // 8 waves, one workgroup per CU
constexpr int kGroups = kThreads / 16;  // frames per phase-1 pass
constexpr int kColStride = 18;   // complex per LDS column: 16-B aligned columns whose
                                 // ds_read_b128 lane groups hit disjoint banks
constexpr int kGroupScratch = 16 * kColStride;  // float2 per frame group
constexpr int kPStride = kBins + 4;  // floats per P row: 16-B aligned rows, conflict-free
                                     // ds_read_b128 (260 = 4 mod 64 dwords)

enum Mode { kAudioToMfcc = 0, kAudioToSpec = 1, kSpecToMfcc = 2 };

// Sample loads by input type: fp32, or int16 PCM (the reference reads int16
// audio and converts with astype(float32), vad.py:37 / file_processing.py:26-35;
// the conversion is exact, so both inputs give identical spectra).
template <typename TIN>
struct Samples;
template <>
struct Samples<float> {
  static constexpr int kPairAlign = 8;  // bytes for one aligned 2-sample load
  __device__ static v2f pair(const float* p) {
    return *reinterpret_cast<const v2f*>(p);
  }
  __device__ static float one(const float* p) { return *p; }
  __device__ static v2f raw_pair(const float* p) { return pair(p); }
  __device__ static v2f raw_two(const float* p0, const float* p1) { return (v2f){*p0, *p1}; }
  __device__ static v2f cvt(v2f r) { return r; }
};
template <>
struct Samples<int16_t> {
  static constexpr int kPairAlign = 4;
  __device__ static v2f pair(const int16_t* p) {
    const int v = *reinterpret_cast<const int*>(p);
    return (v2f){(float)(int16_t)(v & 0xffff), (float)(v >> 16)};
  }
  __device__ static float one(const int16_t* p) { return (float)*p; }
  // prefetched pairs stay raw (the two int16 in one dword, in .x) until
  // their stage A: converting at the load would wait for it right there
  // (the loads sit in sched_barrier-fenced regions), which serialised the
  // one-tile-ahead prefetch of the int16 kernel
  __device__ static v2f raw_pair(const int16_t* p) {
    const int v = *reinterpret_cast<const int*>(p);
    return (v2f){__builtin_bit_cast(float, v), 0.f};
  }
  __device__ static v2f raw_two(const int16_t* p0, const int16_t* p1) {
    const int v = (int)(unsigned short)*p0 | ((int)*p1 << 16);
    return (v2f){__builtin_bit_cast(float, v), 0.f};
  }
  __device__ static v2f cvt(v2f r) {
    const int v = __builtin_bit_cast(int, r.x);
    return (v2f){(float)(int16_t)(v & 0xffff), (float)(v >> 16)};
  }
};

// Load z[16 n1 + n2] = (x[32 n1 + 2 n2], x[32 n1 + 2 n2 + 1]), n1 < NZ.
// Branch-free and wait-free: every load is issued unconditionally from an
// address clamped into the frame, so all NZ loads of a pass are in flight
// at once; the zero padding (x[t] = 0 for t >= len) is applied later by
// pad_stage_a, at first use.  LEN > 0 fixes the frame length at compile time
// (400 for clips); VEC2 (pair-aligned frames of even length) loads a sample
// pair per load.

template <typename TIN, int NZ, bool VEC2, int LEN, int B = 0, int E = NZ>
__device__ __forceinline__ void load_stage_a(const TIN* __restrict__ fr, int len_rt, int n2,
                                             v2f (&u)[NZ]) {
  const int len = LEN > 0 ? LEN : len_rt;
#pragma unroll
  for (int n1 = B; n1 < (E < NZ ? E : NZ); ++n1) {
    const int t = 32 * n1 + 2 * n2;
    if constexpr (VEC2) {
      const int tc = t < len - 2 ? t : len - 2;
      u[n1] = Samples<TIN>::raw_pair(fr + tc);
    } else {
      const int t0 = t < len - 1 ? t : len - 1;
      const int t1 = t + 1 < len - 1 ? t + 1 : len - 1;
      u[n1] = Samples<TIN>::raw_two(fr + t0, fr + t1);
    }
  }
}

template <int NZ, int LEN, int NU = NZ>
__device__ __forceinline__ void pad_stage_a(int len_rt, int n2, v2f (&u)[NU]) {
  const int len = LEN > 0 ? LEN : len_rt;
#pragma unroll
  for (int n1 = 0; n1 < NZ; ++n1) {
    if (LEN > 0 && 32 * n1 + 31 < LEN) continue;  // every lane in range (compile time)
    const int t = 32 * n1 + 2 * n2;
    u[n1].x = t < len ? u[n1].x : 0.f;
    u[n1].y = t + 1 < len ? u[n1].y : 0.f;
  }
}

// Per-lane constants of a 16-lane FFT group, loaded once per workgroup.
//   stage B: lane j owns the even half of column cE and the odd half of
//   column cO = 16 - cE (lanes 0..13 cover columns 1..7 / 9..15, lane 14
//   column 0, lane 15 column 8); the pair m = (a_m, b_m) of the real-FFT
//   split is (E[m], O[7-m]) = (Z[k], Z[256-k]) with k = cE + 32 m.
//   Column 0 pairs k2 with -k2 (mod 16) instead, i.e. E with E and O with
//   O; lane 14 keeps whichever half of the regular pair already matches:
//   m = 1..3 (E[m], E[8-m]), m = 4..7 (O[m], O[7-m]), so it needs one
//   select per pair, not two; its m = 0 pair (E[0], E[4]) holds the two
//   self-partnered bins 0 and 128, fixed up explicitly.
struct LaneConsts {
  v2f twa[16];     // W256^(j k1)
  v2f twb[8];      // W512^kE(m)
  int cE, cO;
  int e0;          // kE(m) = e0 + 32 m (+ off4 for m >= 4)
  int off4;        // 16 on the column-0 lane (its m >= 4 pairs are odd bins), else 0
  int kO0;         // kO(0); kO(m >= 1) = 256 - kE(m)
  bool col0;
};

__device__ __forceinline__ void lane_consts(const MfccDev* __restrict__ plan, int j, LaneConsts& L) {
  if (j < 14) {
    const int p = (j >> 1) + 1;
    L.cE = (j & 1) ? 16 - p : p;
    L.cO = 16 - L.cE;
  } else {
    L.cE = L.cO = (j == 14) ? 0 : 8;
  }
  L.col0 = (j == 14);
  L.e0 = L.cE;
  L.off4 = L.col0 ? 16 : 0;
  L.kO0 = L.col0 ? 128 : 256 - L.cE;
  const v2f* ta = reinterpret_cast<const v2f*>(plan->tw_a);
  const v2f* tb = reinterpret_cast<const v2f*>(plan->tw_b);
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) L.twa[k1] = ta[j * 16 + k1];
#pragma unroll
  for (int m = 0; m < 8; ++m) L.twb[m] = tb[L.e0 + 32 * m + (m >= 4 ? L.off4 : 0)];
}

// Per-lane twiddles staged in LDS (the fused kernel: its VGPRs go to the FFN
// between tiles): row j of twa holds W256^(j k1), k1 = 0..15, at a stride of
// 18 complex, row j of twb lane j's eight W512^kE(m) at a stride of 10 --
// 16-B aligned rows whose ds_read_b128 lane groups hit disjoint banks (the
// four 16-lane groups of a wave read the same rows: broadcasts).
constexpr int kTwaStride = 18, kTwbStride = 10;
constexpr size_t kTwLdsBytes = (size_t)16 * (kTwaStride + kTwbStride) * sizeof(v2f);

__device__ __forceinline__ void lane_ints(int j, LaneConsts& L) {
  if (j < 14) {
    const int p = (j >> 1) + 1;
    L.cE = (j & 1) ? 16 - p : p;
    L.cO = 16 - L.cE;
  } else {
    L.cE = L.cO = (j == 14) ? 0 : 8;
  }
  L.col0 = (j == 14);
  L.e0 = L.cE;
  L.off4 = L.col0 ? 16 : 0;
  L.kO0 = L.col0 ? 128 : 256 - L.cE;
}

__device__ __forceinline__ void stage_twiddles(const MfccDev* __restrict__ plan, v2f* __restrict__ tw, int tid,
                                               int nthreads) {
  for (int i = tid; i < 16 * 16; i += nthreads) {
    const int j = i >> 4, k = i & 15;
    tw[j * kTwaStride + k] = reinterpret_cast<const v2f*>(plan->tw_a)[i];
    if (k < 8) {
      LaneConsts L;
      lane_ints(j, L);
      tw[16 * kTwaStride + j * kTwbStride + k] =
          reinterpret_cast<const v2f*>(plan->tw_b)[L.e0 + 32 * k + (k >= 4 ? L.off4 : 0)];
    }
  }
}

__device__ __forceinline__ void lane_consts_lds(const v2f* __restrict__ tw, int j, LaneConsts& L) {
  lane_ints(j, L);
  const v4f* a = reinterpret_cast<const v4f*>(__builtin_assume_aligned(tw + j * kTwaStride, 16));
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const v4f t = a[q];
    L.twa[2 * q] = t.xy;
    L.twa[2 * q + 1] = t.zw;
  }
  const v4f* b = reinterpret_cast<const v4f*>(__builtin_assume_aligned(tw + 16 * kTwaStride + j * kTwbStride, 16));
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const v4f t = b[q];
    L.twb[2 * q] = t.xy;
    L.twb[2 * q + 1] = t.zw;
  }
}

// Phase 1 for one frame of a 16-lane group, in three steps so that a wave
// can overlap one pass's LDS transpose with the next pass's stage A:
//   stage_a   DFT16 over n1 for n2 = j, twiddle W256^(j k1) (registers)
//   store_a   the 16 results to the group's LDS transpose block
//   read_b    column cE and column cO back (16 ds_read_b128, left in flight)
//   finish_b  even half of column cE, odd half of column cO, real-FFT split,
//             power into prow (LDS row, or a global row in spectrum mode).
// SCALE multiplies |2X|^2 into P = |X/512|^2 (2^-20); the MFCC modes fold
// that factor into the mel taps.  Every complex operation is packed fp32
// (fft_pk.h).
template <typename TIN, int NZ, int LEN, bool WIN = false>
__device__ __forceinline__ void stage_a(const v2f (&u_in)[NZ], int len, const LaneConsts& L, int j,
                                        v2f (&u)[16], const float* wv = nullptr) {
#pragma unroll
  for (int n = 0; n < NZ; ++n) {
    u[n] = Samples<TIN>::cvt(u_in[n]);
    if constexpr (WIN) u[n] = u[n] * (v2f){wv[2 * n], wv[2 * n + 1]};
  }
  pad_stage_a<NZ, LEN, 16>(len, j, u);
  pk::dft16<NZ>(u);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) u[k1] = pk::cmul(u[k1], L.twa[k1]);
}

// Paired frames (hop = 32 HOPC samples): chunk c of frame F + 1 is chunk
// c + HOPC of frame F, so one buffer of NZ + HOPC chunks, buf[c] =
// (x[32 c + 2 n2], x[32 c + 2 n2 + 1]) from frame F's start, feeds both
// frames.  Chunks that can reach past frame F's LEN samples clamp their
// offset to lim (frame F + 1's last pair, or frame F's when F + 1 does not
// exist), so no load leaves the signal; pad_stage_a zeroes what each frame
// does not own.
template <typename TIN, int B, int E, int LEN, int NB>
__device__ __forceinline__ void load_chunks(const TIN* __restrict__ base, int lim, int n2,
                                            v2f (&buf)[NB]) {
#pragma unroll
  for (int c = B; c < E; ++c) {
    int o = 32 * c + 2 * n2;
    if (32 * c + 30 > LEN - 2) o = o < lim ? o : lim;
    buf[c % NB] = Samples<TIN>::raw_pair(base + o);  // chunk c in slot c mod NB
  }
}

// stage A of the frame whose chunk n1 is buf[OFF + n1]
template <typename TIN, int NZ, int LEN, int OFF, int NB, bool WIN = false>
__device__ __forceinline__ void stage_a_at(const v2f (&buf)[NB], const LaneConsts& L, int j,
                                           v2f (&u)[16], const float* wv = nullptr) {
#pragma unroll
  for (int n = 0; n < NZ; ++n) {
    u[n] = Samples<TIN>::cvt(buf[OFF + n]);
    // optional analysis window (not in the reference, mfcc.py:59-61): the
    // frame-relative samples 32 n + 2 j, + 1 of this lane
    if constexpr (WIN) u[n] = u[n] * (v2f){wv[2 * n], wv[2 * n + 1]};
  }
  pad_stage_a<NZ, LEN, 16>(LEN, j, u);
  pk::dft16<NZ>(u);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) u[k1] = pk::cmul(u[k1], L.twa[k1]);
}

__device__ __forceinline__ void store_a(const v2f (&u)[16], v2f* __restrict__ scr, int j) {
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) scr[k1 * kColStride + j] = u[k1];
}

__device__ __forceinline__ void read_b(const LaneConsts& L, const v2f* __restrict__ scr,
                                       v2f (&col)[32]) {
  const v4f* ce = reinterpret_cast<const v4f*>(__builtin_assume_aligned(scr + L.cE * kColStride, 16));
  const v4f* co = reinterpret_cast<const v4f*>(__builtin_assume_aligned(scr + L.cO * kColStride, 16));
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const v4f t = ce[q];
    col[2 * q] = t.xy;
    col[2 * q + 1] = t.zw;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const v4f t = co[q];
    col[16 + 2 * q] = t.xy;
    col[16 + 2 * q + 1] = t.zw;
  }
}

template <bool SCALE>
__device__ __forceinline__ void finish_b(const LaneConsts& L, v2f (&col)[32],
                                         float* __restrict__ prow) {
  v2f E[8], O[8];
  float pkv[8], pnv[8];
  pk::dft16_even(*reinterpret_cast<v2f(*)[16]>(&col[0]), E);   // E[m] = Z[cE + 32 m]
  pk::dft16_odd(*reinterpret_cast<v2f(*)[16]>(&col[16]), O);   // O[m] = Z[cO + 32 m + 16]

  // ---- real-FFT split on pairs (a, b) = (Z[k], Z[256-k]):
  //   2 X[k] = S - i W^k D,  2 X[256-k] = conj(S) - i conj(W^k D),
  //   S = a + conj(b), D = a - conj(b),  W = W512
  //   U = (Re 2X[k], Re 2X[256-k]), V = (Im 2X[k], Im 2X[256-k])
  // column-0 lane: (E[0], E[4]) = (Z0, Z128); (E[m], E[8-m]) = (Z[32 m],
  // Z[256 - 32 m]) for m = 1..3; (O[m], O[7-m]) = (Z[32 m + 16],
  // Z[240 - 32 m]) for m = 4..7
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const v2f a = (m >= 4 && L.col0) ? O[m] : E[m];
    const v2f b = (m < 4 && L.col0) ? E[m == 0 ? 4 : (8 - m) & 7] : O[7 - m];
    const v2f S = pk::add_conj(a, b);
    const v2f T = pk::cmul(pk::sub_conj(a, b), L.twb[m]);
    const v2f U = pk::split_u(S, T);
    const v2f V = pk::split_v(S, T);
    v2f p2 = U * U + V * V;  // (|2X[k]|^2, |2X[256-k]|^2)
    if constexpr (SCALE) p2 = p2 * 0x1p-20f;
    float pk = p2.x, pn = p2.y;
    if (m == 0) {  // lane 14: bins 0 and 128 are their own partners
      const float s0 = a.x + a.y;                                 // X[0] = Re Z0 + Im Z0
      const float p0 = 4.f * s0 * s0 * (SCALE ? 0x1p-20f : 1.f);
      const float p128 = 4.f * fmaf(b.x, b.x, b.y * b.y) * (SCALE ? 0x1p-20f : 1.f);
      pk = L.col0 ? p0 : pk;
      pn = L.col0 ? p128 : pn;
    }
    pkv[m] = pk;
    pnv[m] = pn;
  }
  // stores grouped by base: kE = e0 + 32 m (m < 4) or e0 + off4 + 32 m
  // (m >= 4), kO = 256 - kE (m >= 1): constant offsets from three bases, so
  // the load/store optimiser pairs them into ds_write2_b32 (16 stores ->
  // 7 pairs + 2; one ds_write_b32 per store measured 2-6 us slower per 1M
  // frames)
  float* pe0 = prow + L.e0;
  float* pe4 = prow + L.e0 + L.off4;
#pragma unroll
  for (int m = 0; m < 4; ++m) pe0[32 * m] = pkv[m];
#pragma unroll
  for (int m = 4; m < 8; ++m) pe4[32 * m] = pkv[m];
  prow[L.kO0] = pnv[0];
  float* po0 = prow + 256 - L.e0;
#pragma unroll
  for (int m = 1; m < 4; ++m) po0[-32 * m] = pnv[m];
  float* po4 = prow + 256 - L.e0 - L.off4;
#pragma unroll
  for (int m = 4; m < 8; ++m) po4[-32 * m] = pnv[m];
}

// Log-mel rows of a tile, [64][LMS] fp32: LMS is 4 x odd, so the
// frame-per-lane ds_read_b128 of phase 2b hits disjoint banks.
template <int SPEC>
constexpr int lm_stride() { return SPEC == 1 ? 28 : SPEC == 2 ? 44 : kMaxFilters + 4; }
constexpr int kLmFloats = kTile * (kMaxFilters + 4);
constexpr int kDctGroups = 4;  // phase 2b: waves 0..3, coefficients c = w, w+4, w+8, w+12

// Phase 2a (runtime plan): frame `lane`, filters [fb, fe) -> log-mel row.
__device__ __forceinline__ void mel_log(const MfccDev* __restrict__ plan,
                                        const float* __restrict__ prow, int fb, int fe,
                                        float* __restrict__ lrow) {
  const float eps = 0x1p-52f;  // np.finfo(float).eps, mfcc.py:74
  for (int m = fb; m < fe; ++m) {
    const int lo = plan->f_lo[m], n = plan->f_len[m];
    const float* w = plan->taps + plan->f_off[m];
    const float* pr = prow + lo;
    float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;
    int t = 0;
    for (; t + 3 < n; t += 4) {
      e0 = fmaf(w[t], pr[t], e0);
      e1 = fmaf(w[t + 1], pr[t + 1], e1);
      e2 = fmaf(w[t + 2], pr[t + 2], e2);
      e3 = fmaf(w[t + 3], pr[t + 3], e3);
    }
    for (; t < n; ++t) e0 = fmaf(w[t], pr[t], e0);
    float e = (e0 + e1) + (e2 + e3);
    e = (e == 0.f) ? eps : e;
    lrow[m] = log10_pos(e);
  }
}

// Phase 2b (runtime plan): lifter x DCT of one log-mel row for the
// coefficients c = g + 4 i of group g.
__device__ __forceinline__ void dct_rt(const MfccDev* __restrict__ plan,
                                       const float* __restrict__ lrow, int g, int mfcc_n,
                                       float (&acc)[4]) {
  const int nf = plan->n_filters;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = g + kDctGroups * i;
    float s0 = 0.f, s1 = 0.f;
    if (c < mfcc_n) {
      const float* d = plan->dct + c * kMaxFilters;
      int m = 0;
      for (; m + 1 < nf; m += 2) {
        s0 = fmaf(d[m], lrow[m], s0);
        s1 = fmaf(d[m + 1], lrow[m + 1], s1);
      }
      if (m < nf) s0 = fmaf(d[m], lrow[m], s0);
    }
    acc[i] = s0 + s1;
  }
}

// Straight-line phase-2 code for a compile-time filterbank T (mel_tables.h),
// generated into mel_code.h: mel_band_code<T, W> reads every bin of wave W's
// filter band once from the frame's LDS power row as a 16-B vector, feeds it
// to its (at most two) filters with literal weights and writes log10 of the
// band's energies; dct_code<T, G> is the lifter x DCT of a log-mel row for
// coefficient group G.
template <class T, int W>
__device__ __forceinline__ void mel_band_code(const float* __restrict__ prow,
                                              float* __restrict__ lm);
template <class T, int G>
__device__ __forceinline__ void dct_code(const float* __restrict__ lm, float (&acc)[4]);

#include "mel_code.h"

template <class T>
__device__ __forceinline__ void mel_dispatch(int wave, const float* prow, float* lrow) {
  prow = static_cast<const float*>(__builtin_assume_aligned(prow, 16));
  switch (wave) {
    case 0: mel_band_code<T, 0>(prow, lrow); break;
    case 1: mel_band_code<T, 1>(prow, lrow); break;
    case 2: mel_band_code<T, 2>(prow, lrow); break;
    case 3: mel_band_code<T, 3>(prow, lrow); break;
    case 4: mel_band_code<T, 4>(prow, lrow); break;
    case 5: mel_band_code<T, 5>(prow, lrow); break;
    case 6: mel_band_code<T, 6>(prow, lrow); break;
    default: mel_band_code<T, 7>(prow, lrow); break;
  }
}

template <class T>
__device__ __forceinline__ void dct_dispatch(int g, const float* lrow, float (&acc)[4]) {
  lrow = static_cast<const float*>(__builtin_assume_aligned(lrow, 16));
  switch (g) {
    case 0: dct_code<T, 0>(lrow, acc); break;
    case 1: dct_code<T, 1>(lrow, acc); break;
    case 2: dct_code<T, 2>(lrow, acc); break;
    default: dct_code<T, 3>(lrow, acc); break;
  }
}

// Phase 2a: one frame per lane, wave `wave` owns a band of filters: mel
// energies, (==0 -> eps), log10 into the tile's log-mel rows.
template <int SPEC>
__device__ __forceinline__ void phase2a(const MfccDev* __restrict__ plan, const float* P,
                                        float* lm, int wave, int lane) {
  const float* prow = P + lane * kPStride;
  float* lrow = lm + lane * lm_stride<SPEC>();
  if constexpr (SPEC == 1) mel_dispatch<Mel26>(wave, prow, lrow);
  else if constexpr (SPEC == 2) mel_dispatch<Mel40>(wave, prow, lrow);
  else mel_log(plan, prow, plan->wave_fbeg[wave], plan->wave_fend[wave], lrow);
}

// Phase 2b (waves 0..3): lifter x DCT of the tile's log-mel rows, one frame
// per lane, coefficients c = wave + 4 i, stored straight to the MFCC rows.
template <int SPEC, bool STORE = true>
__device__ __forceinline__ void phase2b(const MfccDev* __restrict__ plan, const float* lm,
                                        int wave, int lane, int64_t f0, int64_t n_frames,
                                        int mfcc_n_rt, float* __restrict__ out) {
  constexpr int NC = SPEC == 1 ? Mel26::NC : SPEC == 2 ? Mel40::NC : 0;
  const int mfcc_n = NC > 0 ? NC : mfcc_n_rt;
  const float* lrow = lm + lane * lm_stride<SPEC>();
  float acc[4];
  if constexpr (SPEC == 1) dct_dispatch<Mel26>(wave, lrow, acc);
  else if constexpr (SPEC == 2) dct_dispatch<Mel40>(wave, lrow, acc);
  else dct_rt(plan, lrow, wave, mfcc_n, acc);
  const int64_t f = f0 + lane;
  if constexpr (STORE) {
    if (f < n_frames) {
      float* o = out + f * mfcc_n;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (wave + kDctGroups * i < mfcc_n) o[wave + kDctGroups * i] = acc[i];
    }
  } else {
    if (acc[0] == 12345.f) out[0] = acc[1] + acc[2] + acc[3];  // keep the work live
  }
}

// lifter x DCT on the f32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32,
// a k-ordered fma chain, bit for bit the VALU dct_code chains), one 16-frame
// block of log-mel rows per call: A = rows r0 .. r0 + 15 (lane l: row l & 15,
// filter 4 s + l / 16), B = the [filter][16 coefficients] table dtb (zero past
// the filters / coefficients; the rows' pad columns are zero), D[frame][coef]
// (lane l: coefficient l & 15, frames 4 (l / 16) + r).  Row r0 + i is frame
// f0 + r0 + i.
template <int SPEC>
constexpr int dct_k_steps() { return SPEC == 1 ? 7 : 10; }

template <int SPEC>
__device__ __forceinline__ void dct_mfma16(const float* __restrict__ lm, const float* __restrict__ dtb, int r0,
                                           int lane, int64_t f0, int64_t f_end, float* __restrict__ out) {
  constexpr int KS = dct_k_steps<SPEC>(), LMS = lm_stride<SPEC>(), MN = 13;
  asm volatile("" : "+v"(lane));  // addresses per call (hoisted, they would stay live through the FFT)
  const float* arow = lm + (r0 + (lane & 15)) * LMS + (lane >> 4);
  const float* brow = dtb + (lane >> 4) * 16 + (lane & 15);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(arow[4 * s], brow[64 * s], acc, 0, 0, 0);
  const int c = lane & 15;
  const int64_t fb = f0 + r0 + 4 * (lane >> 4);
  if (c < MN) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (fb + r < f_end) out[(fb + r) * MN + c] = acc[r];
  }
}

// the DCT table dtb and the zero pad columns of `rows` log-mel rows
template <int SPEC>
__device__ __forceinline__ void dct_mfma_setup(const MfccDev* __restrict__ plan, float* __restrict__ dtb,
                                               float* __restrict__ lm, int rows, int tid, int nthreads) {
  constexpr int KS = dct_k_steps<SPEC>(), LMS = lm_stride<SPEC>(), NF = SPEC == 1 ? 26 : 40, MN = 13;
  static_assert(4 * KS >= NF && 4 * KS <= LMS, "DCT K steps");
  for (int i = tid; i < 4 * KS * 16; i += nthreads) {
    const int m = i >> 4, c = i & 15;
    dtb[i] = (c < MN && m < NF) ? plan->dct[c * kMaxFilters + m] : 0.f;
  }
  for (int i = tid; i < rows * (LMS - NF); i += nthreads) lm[(i / (LMS - NF)) * LMS + NF + i % (LMS - NF)] = 0.f;
}

#ifndef VAD_DCT_MFMA
#define VAD_DCT_MFMA 1  // 0: lifter x DCT on the VALU (dct_code) in mfcc_kernel too
#endif
// phase 2b of mfcc_kernel (waves 0..3 of a 64-frame tile): the MFMA form for
// the compiled banks, else the VALU form
template <int SPEC, bool STORE>
__device__ __forceinline__ void phase2b_any(const MfccDev* __restrict__ plan, const float* lm, const float* dtb,
                                            int wave, int lane, int64_t f0, int64_t n_frames, int mfcc_n,
                                            float* __restrict__ out) {
  if constexpr (SPEC >= 1 && STORE && VAD_DCT_MFMA) dct_mfma16<SPEC>(lm, dtb, 16 * wave, lane, f0, n_frames, out);
  else phase2b<SPEC, STORE>(plan, lm, wave, lane, f0, n_frames, mfcc_n, out);
}

// Milestone priorities (paired-frame loop, fp32 input): a wave lowers its
// issue priority (s_setprio 3 -> 0) each time it passes a phase-1 milestone
// (tile start, pass-0 transpose issued, pass-1 stage A, pass-0 power row),
// so the younger wave of a SIMD, which loses every tie on age, gets the VALU
// until it reaches the same milestone and the two reach the first barrier
// closer together: -7 us per 1M frames on fp32 input; on int16 input -4 us
// since its samples are converted at first use (before that, with the
// prefetch serialised by the conversion, +3.5 us).
template <typename TIN>
constexpr bool kMilestonePrio = true;

// (Placements measured: 3/2/1/0 at these four; 3/2/-/1 + 0 after the pass-1
// power row +4 us; 3/-/2/1 + 0 there the same.  Spreading the DCT over all
// 8 waves, or running it at the top of the next tile, is slower with them,
// and so is giving the younger waves priority 1 in phase 2a or in the last
// phase-1 segment.)
#define VAD_MILESTONE(k)                                 \
  do {                                                   \
    if constexpr (kMilestonePrio<TIN>) {                 \
      __builtin_amdgcn_sched_barrier(0);                 \
      __builtin_amdgcn_s_setprio(k);                     \
      __builtin_amdgcn_sched_barrier(0);                 \
    }                                                    \
  } while (0)

constexpr size_t kPBytes = (size_t)kTile * kPStride * sizeof(float);          // 66,560
constexpr size_t kScrBytes = (size_t)kGroups * kGroupScratch * sizeof(v2f);  // 73,728
constexpr size_t kLmBytes = (size_t)kLmFloats * sizeof(float);               // 17,408

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations (lgkmcnt) but not for its vector-memory ones (__syncthreads'
// release fence would drain vmcnt, i.e. wait for the next tile's sample
// loads at every barrier and cut the prefetch distance to a fraction of a
// tile); the empty asm statements keep the compiler from moving memory
// accesses across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // vmcnt 63, expcnt 7, lgkmcnt 0
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// HOPC > 0 (LEN > 0, VEC2, hop = 32 HOPC samples): paired-frame phase 1.
// (The diagnostic instrumentation of earlier rounds -- in-kernel stamps,
// phase-1-only and L2-resident-source builds -- lives in git history before
// round 4; DESIGN.md section 4 cites its measurements.)
template <typename TIN, int MODE, int NZ, bool VEC2, int LEN, int SPEC, int HOPC = 0, bool WIN = false>
__global__ __launch_bounds__(kThreads, 1) void mfcc_kernel(
    const MfccDev* __restrict__ plan, const TIN* __restrict__ src, int64_t frame_stride,
    int frame_len, int64_t n_frames, float* __restrict__ out, MfccBalance bal) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* P = reinterpret_cast<float*>(smem);                      // [64][260] power rows
  v2f* scr = reinterpret_cast<v2f*>(smem + kPBytes);              // FFT transposes
  float* lm = reinterpret_cast<float*>(smem + kPBytes + kScrBytes);  // [64][LMS] log-mel
  float* dtb = lm + kTile * lm_stride<SPEC>();  // the MFMA DCT's operand table (SPEC 1 / 2), inside the log-mel region

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  // wave-uniform (SGPR): the plan reads in phase 2 become scalar loads that
  // do not queue behind the prefetched samples on vmcnt
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = tid >> 4;  // frame group 0..31
  const int j = tid & 15;
  const int len = frame_len < kFftN ? frame_len : kFftN;
  const int mfcc_n = plan->mfcc_n;
  const int64_t n_tiles = (n_frames + kTile - 1) / kTile;
  if constexpr (MODE == kAudioToMfcc && SPEC >= 1 && VAD_DCT_MFMA) {
    static_assert(kTile * lm_stride<SPEC>() + 4 * dct_k_steps<SPEC>() * 16 <= kLmFloats, "DCT table in the log-mel region");
    dct_mfma_setup<SPEC>(plan, dtb, lm, kTile, tid, kThreads);  // read after the first tile's barriers
  }

  if constexpr (MODE == kSpecToMfcc) {
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
      const int64_t f0 = tile * kTile;
      for (int i = tid; i < kTile * kBins; i += kThreads) {
        const int lf = i / kBins, k = i - lf * kBins;
        const int64_t f = f0 + lf;
        // the taps carry the FFT path's 2^-20: undo it on true spectra (exact)
        P[lf * kPStride + k] = (f < n_frames) ? (float)src[f * kBins + k] * 0x1p20f : 0.f;
      }
      __syncthreads();  // P complete; the previous tile's phase 2b is done
      phase2a<SPEC>(plan, P, lm, wave, lane);
      __syncthreads();  // log-mel rows complete; P free
      if (wave < kDctGroups) phase2b<SPEC>(plan, lm, wave, lane, f0, n_frames, mfcc_n, out);
    }
  } else if constexpr (HOPC > 0) {
    // Lane group grp runs frames F = f0 + 2 grp (pass 0) and F + 1 (pass 1)
    // from one NZ + HOPC chunk buffer: 18 sample-pair loads per group and
    // tile instead of 26 (the texture path, not HBM, limits the loads: the
    // frames overlap 2.5x).  The next tile's chunks are issued in three
    // batches as the buffer frees up: 0..HOPC-1 after pass 0's stage A,
    // the rest after pass 1's, split around pass 0's finish.
    static_assert(LEN > 0 && VEC2, "paired frames need the fixed frame length");
    constexpr int NB = NZ + HOPC;
    v2f* gscr = scr + grp * kGroupScratch;
    LaneConsts L;
    lane_consts(plan, j, L);
    float wv[WIN ? 2 * NZ : 1];  // the optional window's samples of this lane (both frames)
    if constexpr (WIN) {
#pragma unroll
      for (int n1 = 0; n1 < NZ; ++n1) {
        wv[2 * n1] = plan->window[32 * n1 + 2 * j];
        wv[2 * n1 + 1] = plan->window[32 * n1 + 2 * j + 1];
      }
    }
    const int64_t flast = n_frames - 1;
    // Runs of 32-frame units: workgroup b owns frames [32 u_b, 32 u_(b+1)),
    // u_b = b U / G over the clip's U = ceil(F / 32) units, in 64-frame
    // tiles from its start; a run of an odd number of units ends in a HALF
    // tile of <= 32 frames, which every wave runs as pass 0 only (lane group
    // grp: frame f0 + grp), so its phase 1 costs about half a tile on all
    // eight waves instead of a full tile's (C2, 100k frames: 12.2 units of
    // work per workgroup, a makespan of 6.5 tiles instead of 7; C3: 61.5
    // instead of 62).  (Frame-granular runs with one wave running the last
    // few frames measured C2 -1.6 %, C3 +0.7 % in round 5: a lone wave on its
    // SIMD issues at a third of a pair's rate.)  XCD-balanced runs
    // (MfccBalance word != 0) stay tile-granular.
    // tile runs balanced over the XCDs' clocks (MfccBalance; word 0: equal)
    const unsigned long long rt0 = bal.stats ? __builtin_amdgcn_s_memrealtime() : 0;
    int64_t f_beg, f_end0;
    if (bal.word == 0) {
      const int64_t n_units = (n_frames + 31) / 32;
      f_beg = (int64_t)blockIdx.x * n_units / gridDim.x * 32;
      f_end0 = ((int64_t)blockIdx.x + 1) * n_units / gridDim.x * 32;
    } else {
      f_beg = balanced_tile(bal.word, n_tiles, blockIdx.x, gridDim.x) * kTile;
      f_end0 = balanced_tile(bal.word, n_tiles, blockIdx.x + 1, gridDim.x) * kTile;
    }
    const int64_t f_end = f_end0 < n_frames ? f_end0 : n_frames;
    int64_t tile = 0;  // local tile index
    const int64_t t_end = (f_end - f_beg + kTile - 1) / kTile;
    // the last tile is a half tile when it holds <= 32 frames
    const int64_t t_half = (t_end > 0 && f_end - f_beg - (t_end - 1) * kTile <= kTile / 2) ? t_end - 1 : -1;
    // lane group grp's first frame in tile t: 2 grp (paired passes) or grp
    // (the half tile's single pass)
    auto pair_base = [&](int64_t t, int& lim) {
      const int64_t F = f_beg + t * kTile + (t == t_half ? grp : 2 * grp);
      lim = F < flast ? 32 * HOPC + LEN - 2 : LEN - 2;
      return src + (F < flast ? F : flast) * frame_stride;
    };
    v2f buf[NB];
    {
      int lim;
      const TIN* b0 = pair_base(tile, lim);
      load_chunks<TIN, 0, NB, LEN>(b0, lim, j, buf);
    }
    __builtin_amdgcn_sched_barrier(0);
    int64_t prev_f0 = -1;
    // one tile; its buffer is refilled with the next tile's chunks as it frees up
    auto tile_body = [&](auto half_tag, v2f (&buf)[NB]) {
      constexpr bool HALF = decltype(half_tag)::value;
      const int64_t f0 = f_beg + tile * kTile;
      const int64_t fa = f0 + (HALF ? grp : 2 * grp), fb = fa + 1;
      // wave-uniform: some frame of the wave is in the run
      const bool active = f0 + (HALF ? 4 : 8) * wave < f_end;
      float* prow_a;
      float* prow_b;
      if constexpr (MODE == kAudioToSpec) {
        prow_a = out + (fa < f_end ? fa : flast) * kBins;
        prow_b = out + (fb < f_end ? fb : flast) * kBins;
      } else {
        prow_a = P + (HALF ? grp : 2 * grp) * kPStride;
        prow_b = P + (2 * grp + 1) * kPStride;
      }
      int lim;
      const TIN* nb = pair_base(tile + 1, lim);
      if (active && HALF) {  // phase 1, pass 0 only (the run's last tile: no prefetch)
        v2f u[16], col[32];
        stage_a_at<TIN, NZ, LEN, 0, NB, WIN>(buf, L, j, u, wv);
        __builtin_amdgcn_sched_barrier(0);
        store_a(u, gscr, j);
        read_b(L, gscr, col);
        if (MODE != kAudioToSpec || fa < f_end) finish_b<MODE == kAudioToSpec>(L, col, prow_a);
      } else if (active) {  // phase 1
        v2f u[16], col[32];
        VAD_MILESTONE(3);
        stage_a_at<TIN, NZ, LEN, 0, NB, WIN>(buf, L, j, u, wv);
        __builtin_amdgcn_sched_barrier(0);
        load_chunks<TIN, 0, HOPC, LEN>(nb, lim, j, buf);
        __builtin_amdgcn_sched_barrier(0);
        store_a(u, gscr, j);
        read_b(L, gscr, col);
        __builtin_amdgcn_sched_barrier(0);
        VAD_MILESTONE(2);
        // pass 1's stage A covers the latency of pass 0's transpose reads
        stage_a_at<TIN, NZ, LEN, HOPC, NB, WIN>(buf, L, j, u, wv);
        __builtin_amdgcn_sched_barrier(0);
        load_chunks<TIN, HOPC, NZ, LEN>(nb, lim, j, buf);
        __builtin_amdgcn_sched_barrier(0);
        VAD_MILESTONE(1);
        if (MODE != kAudioToSpec || fa < f_end) finish_b<MODE == kAudioToSpec>(L, col, prow_a);
        __builtin_amdgcn_sched_barrier(0);
        load_chunks<TIN, NZ, NB, LEN>(nb, lim, j, buf);
        __builtin_amdgcn_sched_barrier(0);
        VAD_MILESTONE(0);
        store_a(u, gscr, j);  // after pass 0's reads in program order (LDS is in order per wave)
        read_b(L, gscr, col);
        if (MODE != kAudioToSpec || fb < f_end) finish_b<MODE == kAudioToSpec>(L, col, prow_b);
      }
      if constexpr (MODE == kAudioToMfcc) {
        __builtin_amdgcn_sched_barrier(0);
        if (prev_f0 >= 0 && wave < kDctGroups)
          phase2b_any<SPEC, true>(plan, lm, dtb, wave, lane, prev_f0, f_end, mfcc_n, out);
        lds_barrier();  // P complete; log-mel rows consumed
        // (a half tile's rows 32..63 hold the previous tile's power: their
        // log-mel rows are computed and never stored, phase 2b stops at f_end)
        phase2a<SPEC>(plan, P, lm, wave, lane);
        lds_barrier();  // log-mel rows complete; P and the FFT scratch free
        prev_f0 = f0;
      }
    };
    for (; tile < (t_half >= 0 ? t_half : t_end); ++tile) tile_body(std::false_type{}, buf);
    if (t_half >= 0) {
      tile_body(std::true_type{}, buf);
      ++tile;
    }

    if constexpr (MODE == kAudioToMfcc) {
      if (prev_f0 >= 0 && wave < kDctGroups)
        phase2b_any<SPEC, true>(plan, lm, dtb, wave, lane, prev_f0, f_end, mfcc_n, out);
    }
    // this run's speed for the host's next balance (runs of >= 8 tiles only:
    // shorter ones are mostly launch ramp)
    if (bal.stats && tid == 0 && t_end >= 8)
      bal.stats[blockIdx.x] = ((unsigned long long)t_end << 40) | (__builtin_amdgcn_s_memrealtime() - rt0);
  } else {
    v2f* gscr = scr + grp * kGroupScratch;
    LaneConsts L;
    lane_consts(plan, j, L);
    // optional analysis window (plan->window, default off: not in the
    // reference, mfcc.py:59-61): lane j's samples 32 n1 + 2 j, + 1
    float wv[WIN ? 2 * NZ : 1];
    if constexpr (WIN) {
#pragma unroll
      for (int n1 = 0; n1 < NZ; ++n1) {
        wv[2 * n1] = plan->window[32 * n1 + 2 * j];
        wv[2 * n1 + 1] = plan->window[32 * n1 + 2 * j + 1];
      }
    }
    // software pipeline: the samples of the next pass are in flight while
    // the current pass computes
    v2f bufA[NZ], bufB[NZ];
    const int64_t flast = n_frames - 1;  // out-of-range frames load the last frame (unused)
    auto pass_src = [&](int64_t t, int pass) {
      int64_t f = t * kTile + pass * kGroups + grp;
      f = f < flast ? f : flast;
      return src + f * frame_stride;
    };
    auto load_pass = [&](int64_t t, int pass, v2f (&buf)[NZ]) {
      load_stage_a<TIN, NZ, VEC2, LEN>(pass_src(t, pass), len, j, buf);
    };
    // each workgroup owns a contiguous run of tiles: consecutive tiles are
    // adjacent in memory (shared halo in this XCD's L2, page-local loads)
    // contiguous, balanced runs: workgroup b owns tiles [b T / G, (b + 1) T / G)
    int64_t tile = (int64_t)blockIdx.x * n_tiles / gridDim.x;
    const int64_t t_end = ((int64_t)blockIdx.x + 1) * n_tiles / gridDim.x;
    // issue order = the steady state's (pass 0 then pass 1): the waitcnt
    // pass merges the prologue into the loop header, and an interleaved
    // prologue would make the first stage A wait for every load in flight
    load_pass(tile, 0, bufA);
    __builtin_amdgcn_sched_barrier(0);
    load_pass(tile, 1, bufB);
    __builtin_amdgcn_sched_barrier(0);
    int64_t prev_f0 = -1;  // tile whose log-mel rows await phase 2b
    // Per tile and wave: two passes of 4 frames.  Each pass's samples are
    // loaded one tile ahead, right after its stage A consumed the previous
    // ones; pass 1's stage A runs while pass 0's transpose reads are in
    // flight.  sched_barriers pin that order (the scheduler would otherwise
    // hoist the loads or sink the reads).
    for (; tile < t_end; ++tile) {
      const int64_t f0 = tile * kTile;
      const int64_t fa = f0 + grp, fb = f0 + kGroups + grp;
      float* prow_a;
      float* prow_b;
      if constexpr (MODE == kAudioToSpec) {
        prow_a = out + (fa < n_frames ? fa : flast) * kBins;
        prow_b = out + (fb < n_frames ? fb : flast) * kBins;
      } else {
        prow_a = P + grp * kPStride;
        prow_b = P + (kGroups + grp) * kPStride;
      }
      v2f u[16], col[32];
      if (LEN > 0) {
        // the next tile's sample loads go out in chunks spread over the
        // tile: a wave's 13 back-to-back pair loads (x 8 waves) would fill
        // the texture address queue and hold every wave at its load burst
        const TIN* sa = pass_src(tile + 1, 0);
        const TIN* sb = pass_src(tile + 1, 1);
        stage_a<TIN, NZ, LEN>(bufA, len, L, j, u);
        __builtin_amdgcn_sched_barrier(0);
        load_stage_a<TIN, NZ, VEC2, LEN, 0, 5>(sa, len, j, bufA);
        __builtin_amdgcn_sched_barrier(0);
        store_a(u, gscr, j);
        read_b(L, gscr, col);
        __builtin_amdgcn_sched_barrier(0);
        load_stage_a<TIN, NZ, VEC2, LEN, 5, 9>(sa, len, j, bufA);
        __builtin_amdgcn_sched_barrier(0);
        stage_a<TIN, NZ, LEN>(bufB, len, L, j, u);
        __builtin_amdgcn_sched_barrier(0);
        load_stage_a<TIN, NZ, VEC2, LEN, 9, NZ>(sa, len, j, bufA);
        load_stage_a<TIN, NZ, VEC2, LEN, 0, 4>(sb, len, j, bufB);
        __builtin_amdgcn_sched_barrier(0);
        if (MODE != kAudioToSpec || fa < n_frames) finish_b<MODE == kAudioToSpec>(L, col, prow_a);
        __builtin_amdgcn_sched_barrier(0);
        load_stage_a<TIN, NZ, VEC2, LEN, 4, 8>(sb, len, j, bufB);
        __builtin_amdgcn_sched_barrier(0);
        store_a(u, gscr, j);
        read_b(L, gscr, col);
        if (MODE != kAudioToSpec || fb < n_frames) finish_b<MODE == kAudioToSpec>(L, col, prow_b);
        __builtin_amdgcn_sched_barrier(0);
        load_stage_a<TIN, NZ, VEC2, LEN, 8, NZ>(sb, len, j, bufB);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        stage_a<TIN, NZ, LEN, WIN>(bufA, len, L, j, u, wv);
        __builtin_amdgcn_sched_barrier(0);
        load_pass(tile + 1, 0, bufA);
        __builtin_amdgcn_sched_barrier(0);
        store_a(u, gscr, j);
        read_b(L, gscr, col);
        if constexpr (LEN > 0) {
          // overlap: pass 1's stage A covers the latency of pass 0's reads
          __builtin_amdgcn_sched_barrier(0);
          stage_a<TIN, NZ, LEN, WIN>(bufB, len, L, j, u, wv);
          __builtin_amdgcn_sched_barrier(0);
          load_pass(tile + 1, 1, bufB);
          __builtin_amdgcn_sched_barrier(0);
          if (MODE != kAudioToSpec || fa < n_frames) finish_b<MODE == kAudioToSpec>(L, col, prow_a);
        } else {
          // runtime frame length: the sequential order keeps the generic
          // variants within 256 VGPRs
          if (MODE != kAudioToSpec || fa < n_frames) finish_b<MODE == kAudioToSpec>(L, col, prow_a);
          __builtin_amdgcn_sched_barrier(0);
          stage_a<TIN, NZ, LEN, WIN>(bufB, len, L, j, u, wv);
          __builtin_amdgcn_sched_barrier(0);
          load_pass(tile + 1, 1, bufB);
          __builtin_amdgcn_sched_barrier(0);
        }
        store_a(u, gscr, j);  // after pass 0's reads in program order (LDS is in order per wave)
        read_b(L, gscr, col);
        if (MODE != kAudioToSpec || fb < n_frames) finish_b<MODE == kAudioToSpec>(L, col, prow_b);
      }
      if constexpr (MODE == kAudioToMfcc) {
        __builtin_amdgcn_sched_barrier(0);
        // the previous tile's DCT runs on the waves that finish phase 1
        // first (waves 0..3 are older and win VALU arbitration on their
        // SIMD) while their SIMD partners are still in their FFT
        if (prev_f0 >= 0 && wave < kDctGroups)
          phase2b_any<SPEC, true>(plan, lm, dtb, wave, lane, prev_f0, n_frames, mfcc_n, out);
        lds_barrier();  // P complete; log-mel rows consumed
        phase2a<SPEC>(plan, P, lm, wave, lane);
        lds_barrier();  // log-mel rows complete; P and the FFT scratch free
        prev_f0 = f0;
      }
    }
    if constexpr (MODE == kAudioToMfcc) {
      if (prev_f0 >= 0 && wave < kDctGroups)
        phase2b_any<SPEC, true>(plan, lm, dtb, wave, lane, prev_f0, n_frames, mfcc_n, out);
    }
  }
}

// ---------------------------------------------------------------------------
// Fused clip path: framing -> MFCC -> 5-frame window features -> FFN ->
// labels (mfcc.py:59-78, sklearn_analyser.py:52-71 / file_processing.py:51-66,
// ffn_trainer.py:106-116); the MFCC rows never leave the CU.
//   Workgroup b owns windows [wb, we) (window i = frames i .. i+4) and runs
//   frames [wb, we + 4) in 64-frame tiles of its own: the 4-frame halo is
//   recomputed by the neighbour (4 frames per workgroup, 0.1 % at 1M frames).
//   Per tile t (two barriers, as in mfcc_kernel's paired-frame loop):
//     phase 1     all waves: FFT of tile t -> power rows P;
//     waves 0..3  lifter x DCT of tile t-1's log-mel rows -> MFCC ring buffer
//                 (t-1) & 1, rows 4..67 (rows 0..3: tile t-2's last four,
//                 copied); then the FFN of tile t-2's 64 windows from buffer
//                 t & 1, wave w taking windows 16 w .. 16 w + 15: features
//                 into its own (now idle) FFT scratch slice, split-f16 MFMA
//                 forward with the weight fragments read from L1 / L2 (the
//                 VGPRs and LDS are the FFT's), label store;
//     barrier;  phase 2a (mel + log10 of tile t);  barrier.
//   Buffer (t-2) & 1 was completed before tile t-1's first barrier and is
//   next written in tile t+1, after tile t's second barrier.
// ---------------------------------------------------------------------------
// The compiler may not treat loads through a laundered pointer as loop
// invariant: the FFN's weight fragments and the FFT's per-lane twiddles are
// re-read where they are used instead of being hoisted out of the tile loop
// (where ~170 VGPRs of them would stay live through the FFT and spill).
template <class Ptr>
__device__ __forceinline__ Ptr launder(Ptr p) {
  asm volatile("" : "+s"(p));
  return p;
}

constexpr int kRingRows = kTile + 4;
constexpr int kRingFloats = kRingRows * 13;

// compact per-lane-group tables of the FFN's bias and VALU output-layer
// slots (LdsSlots): 4 floats per slot, at most 36 bias + 68 output slots (bl13, 4 classes)
constexpr int kSlotTableFloats = 4 * 112;

template <int SPEC>
constexpr size_t fused_smem_bytes() {
  return kPBytes + kScrBytes + (size_t)kTile * lm_stride<SPEC>() * sizeof(float) +
         2 * (size_t)kRingFloats * sizeof(float) + kSlotTableFloats * sizeof(float) + kTwLdsBytes;
}

template <typename TIN, int SPEC, int MODE, int KS0, int T1, int T2, int T3, int T4, int NC>
__global__ __launch_bounds__(kThreads, 1) void mfcc_ffn_kernel(const MfccDev* __restrict__ plan, FfnDev net,
                                                               const TIN* __restrict__ src, int64_t n_frames,
                                                               uint8_t* __restrict__ labels) {
  using T = std::conditional_t<SPEC == 1, Mel26, Mel40>;
  static_assert(T::NC == 13, "the wave tile reads 13 coefficients per row");
  constexpr int LEN = 400, HOPC = 5, NZ = 13, NB = NZ + HOPC, MN = 13;
  using TP = Topo<KS0, T1, T2, T3, T4, NC>;
  using HP = HTopo<TP, KS0, T1, T2, T3, T4>;
  constexpr int IN = KS0 == 4 ? MN : 3 * MN;  // network inputs (features 0 .. IN-1)
  constexpr int XS = 32 * HP::K0 + 4;         // floats per feature row: 16-B aligned
  static_assert((kWTile * XS + kWTile) * 4 <= 4 * kGroupScratch * (int)sizeof(v2f),
                "a wave's features fit its FFT scratch slice");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* P = reinterpret_cast<float*>(smem);                      // [64][260] power rows
  v2f* scr = reinterpret_cast<v2f*>(smem + kPBytes);              // FFT transposes
  float* lm = reinterpret_cast<float*>(smem + kPBytes + kScrBytes);  // [64][LMS] log-mel
  float* ring = lm + kTile * lm_stride<SPEC>();                   // 2 x [68][13] MFCC rows
  float* stbl = ring + 2 * kRingFloats;                           // FFN bias / output slots
  v2f* tw = reinterpret_cast<v2f*>(stbl + kSlotTableFloats);      // per-lane FFT twiddles

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = tid >> 4;
  const int j = tid & 15;
  const int64_t n_win = n_frames - 5;
  const int64_t wb = n_win * blockIdx.x / gridDim.x;
  const int64_t we = n_win * (blockIdx.x + 1) / gridDim.x;
  if (wb >= we) return;  // workgroup-uniform
  const int64_t fs = wb;  // first frame of tile 0
  const int n_t = (int)((we + 4 - fs + kTile - 1) / kTile);

  v2f* gscr = scr + grp * kGroupScratch;
  LaneConsts L;
  stage_twiddles(plan, tw, tid, kThreads);
  const int64_t flast = n_frames - 1;
  auto pair_base = [&](int t, int& lim) __attribute__((always_inline)) {
    const int64_t F = fs + (int64_t)t * kTile + 2 * grp;
    lim = F < flast ? 32 * HOPC + LEN - 2 : LEN - 2;
    return src + (F < flast ? F : flast) * (32 * HOPC);
  };
  // bias and VALU output-layer slots: one value per lane group -> LDS table
  // (a two-class network with a VALU output layer also gets the logit-
  // difference slots of valu_label2 after them, as the window kernel does,
  // so both clip forms classify with the same arithmetic)
  constexpr bool kDiff = NC == 2 && TP::VL && TP::NL == 3;
  constexpr int NS = TP::NB + TP::NV + TP::NVB;
  constexpr int NSD = kDiff ? TP::TIL * 4 + 1 : 0;
  {
    static_assert(4 * (NS + NSD) <= kSlotTableFloats, "slot table");
    auto slot_val = [&](int sl, int gg) {
      // slots after the biases: the VALU layer's (host order: 4 classes, then biases)
      const int src_sl = sl < TP::NB ? TP::NA_ALL + sl
                                     : TP::NA_ALL + TP::NB + (sl - TP::NB < TP::NV ? sl - TP::NB
                                                                                  : 4 * TP::TIL * 4 + sl - TP::NB - TP::NV);
      return net.frag[src_sl * 64 + 16 * gg];
    };
    for (int i = tid; i < 4 * (NS + NSD); i += kThreads) {
      const int sl = i >> 2, gg = i & 3;
      float v;
      if (sl < NS) {
        v = slot_val(sl, gg);
      } else {  // class 1 minus class 0 (weights, then the bias)
        const int q = sl - NS;
        v = q < TP::TIL * 4 ? slot_val(TP::NB + TP::TIL * 4 + q, gg) - slot_val(TP::NB + q, gg)
                            : slot_val(TP::NB + TP::NV + 1, gg) - slot_val(TP::NB + TP::NV, gg);
      }
      stbl[i] = v;
    }
  }
  float* X = reinterpret_cast<float*>(scr + 4 * wave * kGroupScratch);  // waves 0..3: own slice
  int* FL = reinterpret_cast<int*>(X + kWTile * XS);
  const int g4 = lane >> 4;

  // lifter x DCT of tile tt's log-mel rows (one frame per lane, coefficients
  // wave + 4 i) into ring buffer tt & 1, plus the carried rows
  auto dct_to_ring = [&](int tt) __attribute__((always_inline)) {
    float acc[4];
    dct_dispatch<T>(wave, lm + lane * lm_stride<SPEC>(), acc);
    float* M = ring + (tt & 1) * kRingFloats;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (wave + kDctGroups * i < MN) M[(4 + lane) * MN + wave + kDctGroups * i] = acc[i];
    // rows 0..3: the previous tile's last four.  Tile 0 has none: its rows
    // 0..3 feed only windows before wb (never stored), but they share wave
    // 0's 16-window tile with stored windows, so they must hold finite,
    // in-range values -- uninitialised LDS could force the tile's f16 rescale
    // (layer_scale) and perturb its real windows (found by
    // tests/test_gpu_fuzz.py: a fused label differing from the two-kernel one)
    if (wave == 0 && lane < 4 * MN)
      M[lane] = tt > 0 ? ring[((tt + 1) & 1) * kRingFloats + kTile * MN + lane] : 0.f;
  };
  // windows 16 wave .. 16 wave + 15 of ring buffer tt & 1 (row r = frame
  // fs + 64 tt - 4 + r; window 16 wave + jw starts at that row)
  // FFN of a 16-window tile of ring buffer tt & 1 (waves 0..3, windows
  // 16 wave .. 16 wave + 15): features into the wave's FFT scratch slice,
  // layer-0 operands, split-f16 forward, label.  The weight fragments are
  // requested by the caller before the next tile's last sample batch, so the
  // vmcnt wait for them does not also wait for those samples.
  auto fetch_frags = [&](u4 (&frh)[HP::NS][2]) __attribute__((always_inline)) {
    load_fragh<HP>(reinterpret_cast<const uint32_t*>(launder(net.fragh)), lane, frh);
  };
  auto ffn_tile = [&](int tt, u4 (&frh)[HP::NS][2]) __attribute__((always_inline)) {
    const float* R = ring + (tt & 1) * kRingFloats + 16 * wave * MN;
    wave_tile_features<IN, XS, MODE>(R, X, FL, lane);
    const LdsSlots fb{stbl + g4};
    const LdsSlots fv{stbl + 4 * TP::NB + g4};
    int lab;
    if constexpr (kDiff) {
      lab = wave_tile_label2<KS0, T1, T2, IN, XS, true, wave_tile_in_bounded<MODE, IN>>(
          X, FL, lane, FragRegs{frh}, fb, fv, LdsSlots{stbl + 4 * NS + g4}, net.h1_bounded);
    } else {
      f32x4 z;
      lab = wave_tile_classify<KS0, T1, T2, T3, T4, NC, false, IN, XS, true, wave_tile_in_bounded<MODE, IN>>(
          X, FL, lane, FragRegs{frh}, fb, fv, net.n_classes, z);
    }
    const int64_t i = fs + (int64_t)tt * kTile - 4 + 16 * wave + (lane & 15);
    if (lane < 16 && i >= wb && i < we) labels[i] = (uint8_t)lab;
  };

  __syncthreads();  // twiddles and slot tables staged
  v2f buf[NB];
  {
    int lim;
    const TIN* b0 = pair_base(0, lim);
    load_chunks<TIN, 0, NB, LEN>(b0, lim, j, buf);
  }
  __builtin_amdgcn_sched_barrier(0);
  for (int t = 0; t < n_t; ++t) {
    // twiddles from LDS each tile: dead (and their VGPRs free for the FFN)
    // between phase 1 and the next tile
    lane_consts_lds(tw, j, L);
    float* prow_a = P + (2 * grp) * kPStride;
    float* prow_b = P + (2 * grp + 1) * kPStride;
    int lim;
    const TIN* nb = pair_base(t + 1, lim);
    v2f u[16], col[32];
    VAD_MILESTONE(3);
    stage_a_at<TIN, NZ, LEN, 0>(buf, L, j, u);
    __builtin_amdgcn_sched_barrier(0);
    load_chunks<TIN, 0, HOPC, LEN>(nb, lim, j, buf);
    __builtin_amdgcn_sched_barrier(0);
    store_a(u, gscr, j);
    read_b(L, gscr, col);
    __builtin_amdgcn_sched_barrier(0);
    VAD_MILESTONE(2);
    stage_a_at<TIN, NZ, LEN, HOPC>(buf, L, j, u);
    __builtin_amdgcn_sched_barrier(0);
    load_chunks<TIN, HOPC, NZ, LEN>(nb, lim, j, buf);
    __builtin_amdgcn_sched_barrier(0);
    VAD_MILESTONE(1);
    finish_b<false>(L, col, prow_a);
    __builtin_amdgcn_sched_barrier(0);
    if (wave >= kDctGroups) load_chunks<TIN, NZ, NB, LEN>(nb, lim, j, buf);  // waves 0..3: below
    __builtin_amdgcn_sched_barrier(0);
    VAD_MILESTONE(0);
    store_a(u, gscr, j);
    read_b(L, gscr, col);
    finish_b<false>(L, col, prow_b);
    __builtin_amdgcn_sched_barrier(0);
    if (wave < kDctGroups) {
      if (t >= 2) {
        u4 frh[HP::NS][2];
        fetch_frags(frh);
        __builtin_amdgcn_sched_barrier(0);
        load_chunks<TIN, NZ, NB, LEN>(nb, lim, j, buf);
        __builtin_amdgcn_sched_barrier(0);
        dct_to_ring(t - 1);
        ffn_tile(t - 2, frh);
      } else {
        load_chunks<TIN, NZ, NB, LEN>(nb, lim, j, buf);
        if (t >= 1) dct_to_ring(t - 1);
      }
    }
    lds_barrier();  // P complete; log-mel rows consumed; ring buffer (t-1) & 1 complete
    phase2a<SPEC>(plan, P, lm, wave, lane);
    lds_barrier();  // log-mel rows complete; P and the FFT scratch free
  }
  if (wave < kDctGroups) {
    u4 frh[HP::NS][2];
    fetch_frags(frh);
    dct_to_ring(n_t - 1);
    if (n_t >= 2) ffn_tile(n_t - 2, frh);
  }
  lds_barrier();
  if (wave < kDctGroups) {
    u4 frh[HP::NS][2];
    fetch_frags(frh);
    ffn_tile(n_t - 1, frh);
  }
}

static int num_cus();


size_t mfcc_smem_bytes() { return kPBytes + kScrBytes + kLmBytes; }  // 157,696 B

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

template <typename TIN, int MODE, int NZ, bool VEC2, int LEN = 0, int SPEC = 0, int HOPC = 0, bool WIN = false>
static hipError_t launch_t(const MfccDev* plan, const TIN* src, int64_t stride, int len,
                           int64_t n, float* out, hipStream_t st, const MfccBalance& bal = MfccBalance()) {
  const int64_t n_tiles = (n + kTile - 1) / kTile;
  const int cap = num_cus();  // persistent, LDS-bound: one workgroup per CU
  const int grid = (int)(n_tiles < cap ? n_tiles : cap);
  const size_t smem = mfcc_smem_bytes();
  static std::atomic<unsigned long long> attr_done{0};
  const hipError_t e = ensure_dyn_lds(
      reinterpret_cast<const void*>(&mfcc_kernel<TIN, MODE, NZ, VEC2, LEN, SPEC, HOPC, WIN>), (int)smem,
      attr_done);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((mfcc_kernel<TIN, MODE, NZ, VEC2, LEN, SPEC, HOPC, WIN>), dim3(grid), dim3(kThreads),
                     smem, st, plan, src, stride, len, n, out, bal);
  return hipGetLastError();
}

template <typename TIN, int MODE>
static hipError_t launch_m(const MfccDev* plan, int spec, const TIN* src, int64_t stride, int len,
                           int64_t n, float* out, hipStream_t st, const MfccBalance& bal = MfccBalance()) {
  const int used = len < kFftN ? len : kFftN;
  const bool vec2 = ((reinterpret_cast<uintptr_t>(src) % Samples<TIN>::kPairAlign) == 0) &&
                    ((stride & 1) == 0) && ((used & 1) == 0);
  if ((spec == kSpecWindow || spec == kSpecWindow26 || spec == kSpecWindow40) && used == 400 && vec2 &&
      stride == 160) {
    // optional analysis window at the reference framing: the paired-frame
    // kernel with the window applied in its stage A (and the generated mel
    // code when the bank is a compiled one)
    if (spec == kSpecWindow26) return launch_t<TIN, MODE, 13, true, 400, 1, 5, true>(plan, src, stride, len, n, out, st, bal);
    if (spec == kSpecWindow40) return launch_t<TIN, MODE, 13, true, 400, 2, 5, true>(plan, src, stride, len, n, out, st, bal);
    return launch_t<TIN, MODE, 13, true, 400, 0, 5, true>(plan, src, stride, len, n, out, st, bal);
  }
  if (spec == kSpecWindow26 || spec == kSpecWindow40) spec = kSpecWindow;
  if (spec == kSpecWindow) {  // optional analysis window: the runtime-table kernel with WIN
    if (used <= 32 * 13)
      return vec2 ? launch_t<TIN, MODE, 13, true, 0, 0, 0, true>(plan, src, stride, len, n, out, st)
                  : launch_t<TIN, MODE, 13, false, 0, 0, 0, true>(plan, src, stride, len, n, out, st);
    return vec2 ? launch_t<TIN, MODE, 16, true, 0, 0, 0, true>(plan, src, stride, len, n, out, st)
                : launch_t<TIN, MODE, 16, false, 0, 0, 0, true>(plan, src, stride, len, n, out, st);
  }
  if (used == 400 && vec2) {  // the reference framing (config.py:21): fully specialised
    if (MODE == kAudioToMfcc && spec == 1) {
      if (stride == 160)
        return launch_t<TIN, MODE, 13, true, 400, 1, 5>(plan, src, stride, len, n, out, st, bal);
      return launch_t<TIN, MODE, 13, true, 400, 1>(plan, src, stride, len, n, out, st);
    }
    if (MODE == kAudioToMfcc && spec == 2) {
      if (stride == 160)
        return launch_t<TIN, MODE, 13, true, 400, 2, 5>(plan, src, stride, len, n, out, st, bal);
      return launch_t<TIN, MODE, 13, true, 400, 2>(plan, src, stride, len, n, out, st);
    }
    if (stride == 160)
      return launch_t<TIN, MODE, 13, true, 400, 0, 5>(plan, src, stride, len, n, out, st, bal);
    return launch_t<TIN, MODE, 13, true, 400>(plan, src, stride, len, n, out, st);
  }
  if (used <= 32 * 13) {
    return vec2 ? launch_t<TIN, MODE, 13, true>(plan, src, stride, len, n, out, st)
                : launch_t<TIN, MODE, 13, false>(plan, src, stride, len, n, out, st);
  }
  return vec2 ? launch_t<TIN, MODE, 16, true>(plan, src, stride, len, n, out, st)
              : launch_t<TIN, MODE, 16, false>(plan, src, stride, len, n, out, st);
}

hipError_t launch_mfcc(int mode, const MfccDev* plan, int spec, const float* src, int64_t stride,
                       int len, int64_t n, float* out, hipStream_t st, const MfccBalance& bal) {
  if (n <= 0) return hipSuccess;
  switch (mode) {
    case kAudioToMfcc: return launch_m<float, kAudioToMfcc>(plan, spec, src, stride, len, n, out, st, bal);
    case kAudioToSpec:
      return launch_m<float, kAudioToSpec>(plan, spec == kSpecWindow || spec == kSpecWindow26 || spec == kSpecWindow40
                                                     ? kSpecWindow : 0, src, stride, len, n, out, st);
    default:
      // spectra in: the window was applied before the FFT
      if (spec == kSpecWindow26) spec = 1;
      if (spec == kSpecWindow40) spec = 2;
      if (spec == 1) return launch_t<float, kSpecToMfcc, 13, false, 0, 1>(plan, src, 0, 0, n, out, st);
      if (spec == kSpecWindow) spec = 0;
      if (spec == 2) return launch_t<float, kSpecToMfcc, 13, false, 0, 2>(plan, src, 0, 0, n, out, st);
      return launch_t<float, kSpecToMfcc, 13, false, 0>(plan, src, 0, 0, n, out, st);
  }
}

hipError_t launch_mfcc_i16(int mode, const MfccDev* plan, int spec, const int16_t* src,
                           int64_t stride, int len, int64_t n, float* out, hipStream_t st, const MfccBalance& bal) {
  if (n <= 0) return hipSuccess;
  if (mode == kAudioToSpec)
    return launch_m<int16_t, kAudioToSpec>(plan, spec == kSpecWindow || spec == kSpecWindow26 || spec == kSpecWindow40
                                                       ? kSpecWindow : 0, src, stride, len, n, out, st);
  return launch_m<int16_t, kAudioToMfcc>(plan, spec, src, stride, len, n, out, st, bal);
}

// Fused clip entry (vad_mfcc_ffn): the reference framing (400 / 160), the
// compiled 26-filter bank and a split-f16 topology; false -> the caller runs
// the two-kernel path through a workspace.
bool mfcc_ffn_fusable(int spec, const FfnDev& net, int frame_size, int hop, const void* audio, int tin_bytes) {
  if (spec != 1 || frame_size != 400 || hop != 160 || !net.fragh) return false;
  if (reinterpret_cast<uintptr_t>(audio) % (2 * tin_bytes) != 0) return false;  // sample-pair loads
  const int* t = net.tiles;
  const bool ref39 = net.n_layers == 4 && net.ks0 == 10 && t[0] == 4 && t[1] == 2 && t[2] == 1 && t[3] == 1;
  const bool bl13 = net.n_layers == 3 && net.ks0 == 4 && t[0] == 4 && t[1] == 4 && t[2] == 1;
  return ref39 || bl13;
}

template <typename TIN, int MODE, int KS0, int T1, int T2, int T3, int T4, int NC>
static hipError_t launch_fused_t(const MfccDev* plan, const FfnDev& net, const TIN* src, int64_t n_frames,
                                 uint8_t* labels, hipStream_t st) {
  const int64_t n_win = n_frames - 5;
  const int64_t want = (n_win + kTile - 1) / kTile;
  const int cap = num_cus();  // persistent, LDS-bound: one workgroup per CU
  const int grid = (int)(want < cap ? want : cap);
  constexpr size_t smem = fused_smem_bytes<1>();
  static std::atomic<unsigned long long> attr_done{0};
  const hipError_t e = ensure_dyn_lds(
      reinterpret_cast<const void*>(&mfcc_ffn_kernel<TIN, 1, MODE, KS0, T1, T2, T3, T4, NC>), (int)smem, attr_done);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((mfcc_ffn_kernel<TIN, 1, MODE, KS0, T1, T2, T3, T4, NC>), dim3(grid), dim3(kThreads), smem, st,
                     plan, net, src, n_frames, labels);
  return hipGetLastError();
}

template <typename TIN, int MODE>
static hipError_t launch_fused_m(const MfccDev* plan, const FfnDev& net, const TIN* src, int64_t n_frames,
                                 uint8_t* labels, hipStream_t st) {
  if (net.ks0 == 10) return launch_fused_t<TIN, MODE, 10, 4, 2, 1, 1, 4>(plan, net, src, n_frames, labels, st);
  if (net.n_classes <= 2) return launch_fused_t<TIN, MODE, 4, 4, 4, 1, 0, 2>(plan, net, src, n_frames, labels, st);
  return launch_fused_t<TIN, MODE, 4, 4, 4, 1, 0, 4>(plan, net, src, n_frames, labels, st);
}

hipError_t launch_mfcc_ffn(const MfccDev* plan, const FfnDev& net, const void* audio, int tin_bytes,
                           int64_t n_frames, int mode, uint8_t* labels, hipStream_t st) {
  if (n_frames <= 5) return hipSuccess;
  if (tin_bytes == 2) {
    const int16_t* a = static_cast<const int16_t*>(audio);
    return mode == VAD_FEAT_OFFLINE ? launch_fused_m<int16_t, VAD_FEAT_OFFLINE>(plan, net, a, n_frames, labels, st)
                                    : launch_fused_m<int16_t, VAD_FEAT_ANALYSER>(plan, net, a, n_frames, labels, st);
  }
  const float* a = static_cast<const float*>(audio);
  return mode == VAD_FEAT_OFFLINE ? launch_fused_m<float, VAD_FEAT_OFFLINE>(plan, net, a, n_frames, labels, st)
                                  : launch_fused_m<float, VAD_FEAT_ANALYSER>(plan, net, a, n_frames, labels, st);
}

}  // namespace vad
