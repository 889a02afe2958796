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
//                       written to an LDS power tile P[64][257].
//   phase 2  one frame per lane, each wave owns a band of filters (balanced
//            by tap count at plan time): wave-uniform tap loop with scalar
//            weights, log10, partial lifter x DCT sums.
//   phase 3  partials of the 8 waves summed through LDS, coalesced store.
#include <stdlib.h>

#include "vad_common.h"
#include "fft_pk.h"
#include "mel_tables.h"

namespace vad {

constexpr int kTile = 64;        // frames per workgroup tile
constexpr int kThreads = 512;    // 8 waves
constexpr int kWaves = kThreads / 64;
constexpr int kGroups = kThreads / 16;  // frames per phase-1 pass
constexpr int kColStride = 17;   // float2 per LDS column (16 + 1 pad)
constexpr int kGroupScratch = 16 * kColStride;  // float2 per frame group
constexpr int kPStride = kBins + 4;  // floats per P row: 16-B aligned rows, conflict-free
                                     // ds_read_b128 (260 = 4 mod 64 dwords)

enum Mode { kAudioToMfcc = 0, kAudioToSpec = 1, kSpecToMfcc = 2 };

// Load z[16 n1 + n2] = (x[32 n1 + 2 n2], x[32 n1 + 2 n2 + 1]), n1 < NZ.
// Branch-free and wait-free: every load is issued unconditionally from an
// address clamped into the frame, so all NZ loads of a pass are in flight
// at once; the zero padding (x[t] = 0 for t >= len) is applied later by
// pad_stage_a, at first use.  LEN > 0 fixes the frame length at compile time
// (400 for clips); VEC2 (8-byte aligned frames of even length) loads 8 B.
template <int NZ, bool VEC2, int LEN>
__device__ __forceinline__ void load_stage_a(const float* __restrict__ fr, int len_rt, int n2,
                                             v2f (&u)[NZ]) {
  const int len = LEN > 0 ? LEN : len_rt;
#pragma unroll
  for (int n1 = 0; n1 < NZ; ++n1) {
    const int t = 32 * n1 + 2 * n2;
    if constexpr (VEC2) {
      const int tc = t < len - 2 ? t : len - 2;
      u[n1] = *reinterpret_cast<const v2f*>(fr + tc);
    } else {
      const int t0 = t < len - 1 ? t : len - 1;
      const int t1 = t + 1 < len - 1 ? t + 1 : len - 1;
      u[n1] = (v2f){fr[t0], fr[t1]};
    }
  }
}

template <int NZ, int LEN>
__device__ __forceinline__ void pad_stage_a(int len_rt, int n2, v2f (&u)[NZ]) {
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
//   Column 0 pairs k2 with -k2 (mod 16) instead, so lane 14 permutes its
//   registers into (Z[16 m], Z[256 - 16 m]) pairs; its m = 0 pair holds the
//   two self-partnered bins 0 and 128, fixed up explicitly.
struct LaneConsts {
  v2f twa[16];     // W256^(j k1)
  v2f twb[8];      // W512^kE(m)
  int cE, cO;
  int e0, es;      // kE(m) = e0 + es*m
  int o0;          // kO(m) = o0 - es*m (m >= 1)
  int kO0;         // kO(0)
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
  L.es = L.col0 ? 16 : 32;
  L.o0 = 256 - L.cE;
  L.kO0 = L.col0 ? 128 : 256 - L.cE;
  const v2f* ta = reinterpret_cast<const v2f*>(plan->tw_a);
  const v2f* tb = reinterpret_cast<const v2f*>(plan->tw_b);
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) L.twa[k1] = ta[j * 16 + k1];
#pragma unroll
  for (int m = 0; m < 8; ++m) L.twb[m] = tb[L.e0 + L.es * m];
}

// Phase 1 for one frame of a 16-lane group: power spectrum into prow
// (LDS row, or a global row in spectrum mode).  SCALE multiplies |2X|^2 into
// P = |X/512|^2 (2^-20); the MFCC modes fold that factor into the mel taps.
// Every complex operation is packed fp32 (fft_pk.h).
template <int NZ, int LEN, bool SCALE>
__device__ __forceinline__ void frame_power(v2f (&u_in)[NZ], int len, const LaneConsts& L, int j,
                                            v2f* __restrict__ scr, float* __restrict__ prow) {
  // ---- stage A: DFT16 over n1 for n2 = j, twiddle W256^(j k1), to LDS ----
  pad_stage_a<NZ, LEN>(len, j, u_in);
  v2f u[16];
#pragma unroll
  for (int n = 0; n < NZ; ++n) u[n] = u_in[n];
  pk::dft16<NZ>(u);
#pragma unroll
  for (int k1 = 1; k1 < 16; ++k1) u[k1] = pk::cmul(u[k1], L.twa[k1]);
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) scr[k1 * kColStride + j] = u[k1];
  __builtin_amdgcn_wave_barrier();

  // ---- stage B: even half of column cE, odd half of column cO ----------
  v2f E[8], O[8];
  {
    v2f col[16];
#pragma unroll
    for (int n = 0; n < 16; ++n) col[n] = scr[L.cE * kColStride + n];
    pk::dft16_even(col, E);  // E[m] = Z[cE + 32 m]
#pragma unroll
    for (int n = 0; n < 16; ++n) col[n] = scr[L.cO * kColStride + n];
    pk::dft16_odd(col, O);   // O[m] = Z[cO + 32 m + 16]
  }
  __builtin_amdgcn_wave_barrier();

  // ---- real-FFT split on pairs (a, b) = (Z[k], Z[256-k]):
  //   2 X[k] = S - i W^k D,  2 X[256-k] = conj(S) - i conj(W^k D),
  //   S = a + conj(b), D = a - conj(b),  W = W512
  //   U = (Re 2X[k], Re 2X[256-k]), V = (Im 2X[k], Im 2X[256-k])
  // column-0 lane: E' = (Z0, Z16, ..., Z112), O'[7-m] = Z[256 - 16 m]
  const v2f Ep[8] = {E[0], O[0], E[1], O[1], E[2], O[2], E[3], O[3]};
  const v2f Op[8] = {O[4], E[5], O[5], E[6], O[6], E[7], O[7], E[4]};
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const v2f a = L.col0 ? Ep[m] : E[m];
    const v2f b = L.col0 ? Op[7 - m] : O[7 - m];
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
    const int kE = L.e0 + L.es * m;
    const int kO = m == 0 ? L.kO0 : L.o0 - L.es * m;
    prow[kE] = pk;
    prow[kO] = pn;
  }
}

// Phase 2: frame `lane` of the tile, filters [fb, fe): partial lifter x DCT
// sums in acc[].
__device__ __forceinline__ void mel_log_dct(const MfccDev* __restrict__ plan,
                                            const float* __restrict__ prow, int fb, int fe,
                                            float (&acc)[kMaxCoefs]) {
  const float eps = 0x1p-52f;  // np.finfo(float).eps, mfcc.py:74
#pragma unroll
  for (int c = 0; c < kMaxCoefs; ++c) acc[c] = 0.f;
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
    const float lg = __log10f(e);
#pragma unroll
    for (int c = 0; c < kMaxCoefs; ++c) acc[c] = fmaf(plan->dct[c * kMaxFilters + m], lg, acc[c]);
  }
}

// log10 of a positive energy: native v_log_f32 (with a pre-scale for tiny
// inputs) times log10(2) -- ~1e-7 relative, far inside the 1e-4 budget.
__device__ __forceinline__ float log10_pos(float e) {
  const bool tiny = e < 0x1p-100f;
  const float x = tiny ? e * 0x1p64f : e;
  const float l2 = __builtin_amdgcn_logf(x);  // log2
  return fmaf(l2, 0.30102999566398120f, tiny ? -19.26591972249479649f : 0.f);
}

// Phase 2 specialised for a compile-time filterbank T (mel_tables.h): wave W
// owns filters [band[W], band[W+1]); every bin of the band is read once from
// the frame's LDS row as a 16-B vector and fed to its (at most two) filters
// with literal weights; log10; partial lifter x DCT sums.
// Phase 2 specialised for a compile-time filterbank T (mel_tables.h): wave W
// owns filters [band[W], band[W+1]); every bin of its band is read once from
// the frame's LDS row as a 16-B vector and fed to its (at most two) filters,
// then log10 and the partial lifter x DCT sums.  The bodies are generated
// (mel_code.h) as straight-line v_fmac_f32 with 32-bit literal weights.
template <class T, int W>
__device__ __forceinline__ void mel_band_code(const float* __restrict__ prow,
                                              float (&acc)[kMaxCoefs]);

#include "mel_code.h"

template <class T, int W>
__device__ __forceinline__ void mel_band(const float* __restrict__ prow, int z,
                                         float (&acc)[kMaxCoefs]) {
  (void)z;
  mel_band_code<T, W>(static_cast<const float*>(__builtin_assume_aligned(prow, 16)), acc);
}

template <class T>
__device__ __forceinline__ void mel_dispatch(int wave, const float* prow, int z,
                                             float (&acc)[kMaxCoefs]) {
  switch (wave) {
    case 0: mel_band<T, 0>(prow, z, acc); break;
    case 1: mel_band<T, 1>(prow, z, acc); break;
    case 2: mel_band<T, 2>(prow, z, acc); break;
    case 3: mel_band<T, 3>(prow, z, acc); break;
    case 4: mel_band<T, 4>(prow, z, acc); break;
    case 5: mel_band<T, 5>(prow, z, acc); break;
    case 6: mel_band<T, 6>(prow, z, acc); break;
    default: mel_band<T, 7>(prow, z, acc); break;
  }
}

constexpr int kPartStride = kMaxCoefs + 1;  // floats per (wave, frame) partial row

// Phases 2 + 3 for one tile: mel / log / DCT partials per wave, summed
// through LDS, coalesced store of the tile's MFCC rows.  SPEC 0 = runtime
// plan, 1 = Mel26, 2 = Mel40 (compile-time tables).
template <int SPEC>
__device__ __forceinline__ void tile_mfcc(const MfccDev* __restrict__ plan, const float* P,
                                          float* part, int tid, int wave, int lane, int64_t f0,
                                          int64_t n_frames, int mfcc_n_rt, float* __restrict__ out) {
  constexpr int NC = SPEC == 1 ? Mel26::NC : SPEC == 2 ? Mel40::NC : 0;
  const int mfcc_n = NC > 0 ? NC : mfcc_n_rt;
  __syncthreads();
  float acc[kMaxCoefs];
  const int z = __builtin_amdgcn_readfirstlane((int)(f0 >> 48));  // 0, opaque per tile
  if constexpr (SPEC == 1) mel_dispatch<Mel26>(wave, P + lane * kPStride, z, acc);
  else if constexpr (SPEC == 2) mel_dispatch<Mel40>(wave, P + lane * kPStride, z, acc);
  else mel_log_dct(plan, P + lane * kPStride, plan->wave_fbeg[wave], plan->wave_fend[wave], acc);
#pragma unroll
  for (int c = 0; c < (NC > 0 ? NC : kMaxCoefs); ++c) part[(wave * 64 + lane) * kPartStride + c] = acc[c];
  __syncthreads();
  const int64_t nf = (n_frames - f0) < kTile ? (n_frames - f0) : kTile;
  for (int i = tid; i < nf * mfcc_n; i += kThreads) {
    const int lf = i / mfcc_n, c = i - lf * mfcc_n;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += part[(w * 64 + lf) * kPartStride + c];
    out[f0 * mfcc_n + i] = s;
  }
  __syncthreads();
}

// DIAG (diagnostic builds only, VAD_DIAG env): 1 = skip the FFT (phase 1
// keeps its loads and P stores), 2 = skip phases 2-3, 3 = both (loads only),
// 4 = FFT on register data without loads, no phases 2-3.  Outputs are wrong.
template <int MODE, int NZ, bool VEC2, int LEN, int SPEC, int DIAG = 0>
__global__ __launch_bounds__(kThreads, 1) void mfcc_kernel(
    const MfccDev* __restrict__ plan, const float* __restrict__ src, int64_t frame_stride,
    int frame_len, int64_t n_frames, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* P = reinterpret_cast<float*>(smem);                                   // [64][257]
  v2f* scr = reinterpret_cast<v2f*>(smem + kTile * kPStride * sizeof(float));
  float* part = reinterpret_cast<float*>(scr);            // phase 3 reuse: [wave][64][17]

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

  if constexpr (MODE == kSpecToMfcc) {
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
      const int64_t f0 = tile * kTile;
      for (int i = tid; i < kTile * kBins; i += kThreads) {
        const int lf = i / kBins, k = i - lf * kBins;
        const int64_t f = f0 + lf;
        // the taps carry the FFT path's 2^-20: undo it on true spectra (exact)
        P[lf * kPStride + k] = (f < n_frames) ? src[f * kBins + k] * 0x1p20f : 0.f;
      }
      tile_mfcc<SPEC>(plan, P, part, tid, wave, lane, f0, n_frames, mfcc_n, out);
    }
  } else {
    v2f* gscr = scr + grp * kGroupScratch;
    LaneConsts L;
    lane_consts(plan, j, L);
    // software pipeline: the samples of the next pass are in flight while
    // the current pass computes
    v2f bufA[NZ], bufB[NZ];
    const int64_t flast = n_frames - 1;  // out-of-range frames load the last frame (unused)
    int64_t tile = blockIdx.x;
    {
      int64_t f = tile * kTile + grp;
      f = f < flast ? f : flast;
      load_stage_a<NZ, VEC2, LEN>(src + f * frame_stride, len, j, bufA);
    }
    for (; tile < n_tiles; tile += gridDim.x) {
      const int64_t f0 = tile * kTile;
      {  // prefetch pass 1 of this tile
        int64_t f = f0 + kGroups + grp;
        f = f < flast ? f : flast;
        if constexpr (DIAG == 4) {
#pragma unroll
          for (int n = 0; n < NZ; ++n) bufB[n] = (v2f){(float)(f + n), (float)(j - n)};
        } else {
          load_stage_a<NZ, VEC2, LEN>(src + f * frame_stride, len, j, bufB);
        }
      }
      // keep the scheduler from hoisting the next pass's FFT above this
      // pass (that would wait on the loads just issued and defeat the
      // prefetch distance)
      __builtin_amdgcn_sched_barrier(0);
      {  // pass 0
        const int64_t f = f0 + grp;
        if constexpr (MODE == kAudioToSpec) {
          if (f < n_frames) frame_power<NZ, LEN, true>(bufA, len, L, j, gscr, out + f * kBins);
        } else {
          if constexpr (DIAG == 1 || DIAG == 3) {
            P[grp * kPStride + j] = bufA[j % NZ].x + bufA[(j + 5) % NZ].y;
          } else {
            frame_power<NZ, LEN, false>(bufA, len, L, j, gscr, P + grp * kPStride);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      {  // prefetch pass 0 of the next tile
        int64_t f = (tile + gridDim.x) * kTile + grp;
        f = f < flast ? f : flast;
        if constexpr (DIAG == 4) {
#pragma unroll
          for (int n = 0; n < NZ; ++n) bufA[n] = (v2f){(float)(f - n), (float)(j + n)};
        } else {
          load_stage_a<NZ, VEC2, LEN>(src + f * frame_stride, len, j, bufA);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      {  // pass 1
        const int64_t f = f0 + kGroups + grp;
        if constexpr (MODE == kAudioToSpec) {
          if (f < n_frames) frame_power<NZ, LEN, true>(bufB, len, L, j, gscr, out + f * kBins);
        } else {
          if constexpr (DIAG == 1 || DIAG == 3) {
            P[(kGroups + grp) * kPStride + j] = bufB[j % NZ].x + bufB[(j + 5) % NZ].y;
          } else {
            frame_power<NZ, LEN, false>(bufB, len, L, j, gscr, P + (kGroups + grp) * kPStride);
          }
        }
      }
      if constexpr (MODE == kAudioToMfcc && DIAG <= 1)
        tile_mfcc<SPEC>(plan, P, part, tid, wave, lane, f0, n_frames, mfcc_n, out);
      if constexpr (DIAG >= 2) {
        __syncthreads();
        if (tid < 64) out[f0 * 13 + tid] = P[tid * kPStride + (tid & 15)];
        __syncthreads();
      }
    }
  }
}

size_t mfcc_smem_bytes() {
  const size_t p = kTile * kPStride * sizeof(float);  // 65792 B, 16-B multiple
  const size_t s = kGroups * kGroupScratch * sizeof(v2f);
  const size_t part = kWaves * 64 * kPartStride * sizeof(float);
  return p + (s > part ? s : part);
}

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

template <int MODE, int NZ, bool VEC2, int LEN = 0, int SPEC = 0, int DIAG = 0>
static hipError_t launch_t(const MfccDev* plan, const float* src, int64_t stride, int len,
                           int64_t n, float* out, hipStream_t st) {
  const int64_t n_tiles = (n + kTile - 1) / kTile;
  const int cap = num_cus();  // persistent: one 512-thread workgroup per CU (LDS-bound)
  const int grid = (int)(n_tiles < cap ? n_tiles : cap);
  const size_t smem = mfcc_smem_bytes();
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&mfcc_kernel<MODE, NZ, VEC2, LEN, SPEC, DIAG>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((mfcc_kernel<MODE, NZ, VEC2, LEN, SPEC, DIAG>), dim3(grid), dim3(kThreads), smem, st, plan,
                     src, stride, len, n, out);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_m(const MfccDev* plan, int spec, const float* src, int64_t stride, int len,
                           int64_t n, float* out, hipStream_t st) {
  const int used = len < kFftN ? len : kFftN;
  const bool vec2 = ((reinterpret_cast<uintptr_t>(src) & 7) == 0) && ((stride & 1) == 0) &&
                    ((used & 1) == 0);
  if (used == 400 && vec2) {  // the reference framing (config.py:21): fully specialised
    if (MODE == kAudioToMfcc && spec == 1) {
      static const int diag = getenv("VAD_DIAG") ? atoi(getenv("VAD_DIAG")) : 0;
      if (diag == 1) return launch_t<MODE, 13, true, 400, 1, 1>(plan, src, stride, len, n, out, st);
      if (diag == 2) return launch_t<MODE, 13, true, 400, 1, 2>(plan, src, stride, len, n, out, st);
      if (diag == 3) return launch_t<MODE, 13, true, 400, 1, 3>(plan, src, stride, len, n, out, st);
      if (diag == 4) return launch_t<MODE, 13, true, 400, 1, 4>(plan, src, stride, len, n, out, st);
      return launch_t<MODE, 13, true, 400, 1>(plan, src, stride, len, n, out, st);
    }
    if (MODE == kAudioToMfcc && spec == 2)
      return launch_t<MODE, 13, true, 400, 2>(plan, src, stride, len, n, out, st);
    return launch_t<MODE, 13, true, 400>(plan, src, stride, len, n, out, st);
  }
  if (used <= 32 * 13) {
    return vec2 ? launch_t<MODE, 13, true>(plan, src, stride, len, n, out, st)
                : launch_t<MODE, 13, false>(plan, src, stride, len, n, out, st);
  }
  return vec2 ? launch_t<MODE, 16, true>(plan, src, stride, len, n, out, st)
              : launch_t<MODE, 16, false>(plan, src, stride, len, n, out, st);
}

hipError_t launch_mfcc(int mode, const MfccDev* plan, int spec, const float* src, int64_t stride,
                       int len, int64_t n, float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  switch (mode) {
    case kAudioToMfcc: return launch_m<kAudioToMfcc>(plan, spec, src, stride, len, n, out, st);
    case kAudioToSpec: return launch_m<kAudioToSpec>(plan, 0, src, stride, len, n, out, st);
    default:
      if (spec == 1) return launch_t<kSpecToMfcc, 13, false, 0, 1>(plan, src, 0, 0, n, out, st);
      if (spec == 2) return launch_t<kSpecToMfcc, 13, false, 0, 2>(plan, src, 0, 0, n, out, st);
      return launch_t<kSpecToMfcc, 13, false, 0>(plan, src, 0, 0, n, out, st);
  }
}

}  // namespace vad
