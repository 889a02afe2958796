// Matrix-core MFCC kernel for the reference framing (400-sample frames,
// 160-sample hop, 512-point real DFT; mfcc.py:59-78, file_processing.py:80-103).
// Included by mfcc_kernel.hip after its phase-2 helpers (phase2a, dct_mfma16).
//
// Phase 1 is the 512-point DFT of each zero-padded 400-sample frame as two
// dense GEMM stages on v_mfma_f32_16x16x32_f16, every operand split into
// f16 halves v = hi + lo (three products hi*lo, lo*hi, hi*hi accumulated in
// f32: ~22 significant bits per operand; the dropped lo*lo is ~2^-22 of a
// product).  With n = 16 n1 + n2 (n1 < 25 non-zero) and k = kp + 32 k2:
//   stage A  per n2: A[n2][kp] = sum_n1 x[16 n1 + n2] W32^(n1 kp) for the
//            real input's 17 distinct kp as 32 real rows (p = 2 kp + re|im,
//            p = 1 holds Re A[16]; Im A[0] = Im A[16] = 0);
//   stage B  per kp: X[kp + 32 k2] = sum_n2 W512^(n2 (kp + 32 k2)) A[n2][kp]
//            (twiddles folded into the matrix), k2 < 8; the mirror bins
//            X[32 - kp + 32 k2] = conj of the same matrix applied to A with
//            the odd n2 negated, row 7 - k2.
// A wave owns 16 frames (the MFMA columns) and half of stage A's rows (ty:
// kp 0..7 or 8..15), i.e. exactly the kp its stage B needs: the only
// exchange between the stages is a 4 x 4 block transpose across the wave's
// lane groups (v_permlane32_swap / v_permlane16_swap), no LDS.
//
// Samples reach the matrix cores through a per-tile staging image in LDS:
// row r (= sample mod 16), column q (= sample / 16 from the tile start),
// hi and lo f16 images, q pairs per dword.  A tile's 10,480 samples are
// loaded once (16-B loads, one tile ahead), scaled by a power of two 2^sc so
// the tile's largest finite |x| lands in [2^9, 2^10) (|A| < 25 * 2^10 stays
// in f16 range; tiles whose largest |x| is in [32, 32768) -- int16-range
// audio -- all take sc = -5, so integer samples are exact and give the same
// bits in every tile), split with v_fma_mix{lo,hi}_f16 and stored.  The
// power rows |y|^2 = |X|^2 2^(2 sc) go to the [64][260] power tile that the
// shared phase 2 (mel + log10, then the lifter x DCT on the f32 MFMA)
// reads; phase 2a multiplies each mel energy by 2^(2 - 2 sc) (exact), which
// restores the |2X|^2 scale the compiled taps expect.
//
// Non-finite samples: the tile's max runs over the raw bits (signed and
// unsigned max), which also flags NaN / inf; a flagged tile takes its scale
// from the finite samples only and masks the B-operand slots past n1 = 24
// (samples that belong to later frames), so a NaN / inf turns exactly the
// frames that contain it into NaN rows, as the reference's float path does.
//
// Per tile (two barriers):
//   stage A + B (all 8 waves) -> power rows; max of the next tile's samples
//   barrier
//   split + store the next tile's staging image; request the tile after it;
//   phase 2a (mel, log10) -> log-mel rows
//   barrier
//   lifter x DCT (waves 0..3, f32 MFMA) -> MFCC rows
#pragma once
// (inside namespace vad)

namespace mx {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kHop = 160, kLen = 400;
constexpr int kTileSamples = kTile * kHop + (kLen - kHop);  // 10,480
constexpr int kQDw = 328;      // q-pair dwords per staging row (q < 656)
constexpr int kRow = 332;      // staging row stride in dwords (== 12 mod 64: conflict-free task stores)
constexpr int kTasks = 4 * kQDw;  // staging tasks per tile: (4-sample chunk c, q pair d)
constexpr int kTaskRounds = (kTasks + kThreads - 1) / kThreads;  // 3
constexpr size_t kImgBytes = (size_t)16 * kRow * 4;              // 21,248 per image
constexpr size_t kStageOff = kPBytes;
constexpr size_t kLmOff = kStageOff + 2 * kImgBytes;
constexpr size_t kWbOff = kLmOff + kLmBytes;                     // stage-B operand images
constexpr size_t kWbBytes = (size_t)17 * 2 * 64 * 16;            // 34,816
constexpr size_t kRedOff = kWbOff + kWbBytes;
constexpr size_t kSmemBytes = kRedOff + 16 * 4;                  // 161,344

__device__ __forceinline__ f4 mfma(u4 a, u4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}
// W x (hi + lo) with W = wh + wl: the two small products first
__device__ __forceinline__ f4 mfma3(u4 wh, u4 wl, u4 bh, u4 bl) {
  f4 c = mfma(wl, bh, (f4){0.f, 0.f, 0.f, 0.f});
  c = mfma(wh, bl, c);
  return mfma(wh, bh, c);
}

// (a, b) -> packed f16 hi = (f16(a s), f16(b s)) and lo = (f16(a s - hi.x),
// f16(b s - hi.y)); s a power of two, a s exact, a s - hi exact in f32
__device__ __forceinline__ void split_scaled(float a, float b, float s, unsigned& hi, unsigned& lo) {
  asm volatile("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=v"(hi) : "v"(a), "v"(s));
  asm volatile("v_fma_mixhi_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "+v"(hi) : "v"(b), "v"(s));
  asm volatile("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel:[0,0,0] op_sel_hi:[0,0,1]" : "=v"(lo) : "v"(a), "v"(s), "v"(hi));
  asm volatile("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo) : "v"(b), "v"(s), "v"(hi));
}
// the same without a scale (stage A results, |v| < 2^15)
__device__ __forceinline__ void split2(float a, float b, unsigned& hi, unsigned& lo) {
  asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(hi) : "v"(a), "v"(b));
  asm volatile("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel:[0,0,0] op_sel_hi:[0,0,1]" : "=v"(lo) : "v"(a), "v"(hi));
  asm volatile("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lo) : "v"(b), "v"(hi));
}

__device__ __forceinline__ void swap32(unsigned& a, unsigned& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void swap16(unsigned& a, unsigned& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}

// Sample loads of one staging task (4 consecutive samples at offset o and
// at o + 16 from the tile's base) as floats; V4: one 16-B (fp32) / 8-B
// (int16) load each, else per-sample loads with the offset clamped to lim
// (the tail tile, misaligned sources).  base is wave-uniform and o a 32-bit
// lane offset, so each load is one SGPR base + VGPR offset.
template <typename TIN, bool V4>
__device__ __forceinline__ void load_task(const TIN* __restrict__ base, int o, int lim, float (&v)[8]) {
  if constexpr (V4) {
    if constexpr (std::is_same_v<TIN, float>) {
      const f4 a = *reinterpret_cast<const f4*>(base + o);
      const f4 b = *reinterpret_cast<const f4*>(base + o + 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = a[j];
        v[4 + j] = b[j];
      }
    } else {
      typedef int i2 __attribute__((ext_vector_type(2)));
      const i2 a = *reinterpret_cast<const i2*>(base + o);
      const i2 b = *reinterpret_cast<const i2*>(base + o + 16);
      v[0] = (float)(int16_t)(a.x & 0xffff);
      v[1] = (float)(a.x >> 16);
      v[2] = (float)(int16_t)(a.y & 0xffff);
      v[3] = (float)(a.y >> 16);
      v[4] = (float)(int16_t)(b.x & 0xffff);
      v[5] = (float)(b.x >> 16);
      v[6] = (float)(int16_t)(b.y & 0xffff);
      v[7] = (float)(b.y >> 16);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int t = o + (j & 3) + (j >> 2) * 16;
      t = t < lim ? t : lim;
      v[j] = (float)base[t];
    }
  }
}

// Stage A for one wave: 16 n2 x (three MFMAs + split of the four results).
// R[b][(n2 & 3) * 4 + {Ha, Hb, La, Lb}] for b = n2 >> 2: the two kp of this
// lane group (a = 2 g, b = 2 g + 1 within the wave's half), hi / lo halves.
// four consecutive staging dwords from p: PAR -1 any alignment (two
// ds_read2_b32), 0 p 8-B aligned (two ds_read_b64), 1 p + 1 8-B aligned
// (ds_read_b32, ds_read_b64, ds_read_b32)
template <int PAR>
__device__ __forceinline__ u4 read4(const unsigned* p) {
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  if constexpr (PAR == 0) {
    const u2* q = reinterpret_cast<const u2*>(__builtin_assume_aligned(p, 8));
    const u2 a = q[0], b = q[1];
    return (u4){a.x, a.y, b.x, b.y};
  } else if constexpr (PAR == 1) {
    const u2 m = *reinterpret_cast<const u2*>(__builtin_assume_aligned(p + 1, 8));
    return (u4){p[0], m.x, m.y, p[3]};
  } else {
    return (u4){p[0], p[1], p[2], p[3]};
  }
}

template <bool MASK, int PAR>
__device__ __forceinline__ void stage_a(const unsigned* __restrict__ SH, const unsigned* __restrict__ SL, int qd,
                                        unsigned m0, unsigned m1, u4 wah, u4 wal, unsigned (&R)[4][16]) {
#pragma unroll
  for (int n2 = 0; n2 < 16; ++n2) {
    u4 bh = read4<PAR>(SH + n2 * kRow + qd);
    u4 bl = read4<PAR>(SL + n2 * kRow + qd);
    if constexpr (MASK) {  // lane group 3: only n1 = 24 belongs to this frame
      bh = (u4){bh.x & m0, bh.y & m1, bh.z & m1, bh.w & m1};
      bl = (u4){bl.x & m0, bl.y & m1, bl.z & m1, bl.w & m1};
    }
    const f4 acc = mfma3(wah, wal, bh, bl);
    unsigned ha, la, hb, lb;
    split2(acc[0], acc[1], ha, la);
    split2(acc[2], acc[3], hb, lb);
    R[n2 >> 2][(n2 & 3) * 4 + 0] = ha;
    R[n2 >> 2][(n2 & 3) * 4 + 1] = hb;
    R[n2 >> 2][(n2 & 3) * 4 + 2] = la;
    R[n2 >> 2][(n2 & 3) * 4 + 3] = lb;
  }
}

// One tile of phase 1 for wave (bt, ty): stage A, the lane-group transpose,
// stage B and the power rows of frames 16 bt + i.
//   Lane group g holds, for every kp = 8 ty + kk of its wave, the direct bins
//   kp + 32 k2 (k2 = 2 g, 2 g + 1) and the mirror bins 32 (7 - 2 g) + 32 - kp,
//   32 (6 - 2 g) + 32 - kp (for kp = 0: the bins 16 + 32 k2 of the same two
//   blocks, from matrix 16, whose rows are ordered k2 = 7 - slot for that).
//   PERM (compiled banks): the power row's upper half-blocks are rotated by
//   one (gen_tables.mx_col), so each lane's 32 values are four aligned runs
//   of eight: 8 ds_write_b128 (conflict-free) instead of 32 ds_write_b32.
//   PAR -1: column i is frame 16 bt + i; 0 / 1 (batches of one frame
//   parity, so every staging read is 8-B aligned or off by one dword): frame
//   2 i + PAR + 32 (bt >> 1).  The power row of column i is row 16 bt + i
//   either way (phase 2a is row-agnostic; the DCT maps rows back to frames).
template <bool MASK, bool PERM, int PAR>
__device__ __forceinline__ void phase1(const unsigned* __restrict__ SH, const unsigned* __restrict__ SL,
                                       float* __restrict__ P, const u4* __restrict__ WB, int lane, int bt, int ty,
                                       u4 wah, u4 wal) {
  asm volatile("" : "+v"(lane));  // per-tile addresses (hoisted out of the tile loop they would stay live)
  const int g = lane >> 4, i = lane & 15;
  const int f = PAR < 0 ? 16 * bt + i : 2 * i + PAR + 32 * (bt >> 1);
  const int qd = 5 * f + 4 * g;  // dword of q = 10 f + 8 g in row n2
  const unsigned m0 = g == 3 ? 0x0000ffffu : 0xffffffffu, m1 = g == 3 ? 0u : 0xffffffffu;
  unsigned R[4][16];
  stage_a<MASK, PAR>(SH, SL, qd, m0, m1, wah, wal, R);
  // 4 x 4 block transpose across the lane groups: slot s <- source group s
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    swap32(R[0][k], R[2][k]);
    swap32(R[1][k], R[3][k]);
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    swap16(R[0][k], R[1][k]);
    swap16(R[2][k], R[3][k]);
  }
  float* prow = P + (16 * bt + i) * kPStride;
  const int ka = 2 * g, kb = 2 * g + 1;  // k2 of output rows 4 g, 4 g + 2
  f4 pd[2][2], pm[2][2];  // PERM: direct / mirror runs [k2 pair][half], element kk & 3 / (7 - kk) & 3
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kk = 2 * s + h, kp = 8 * ty + kk;
      const u4 dh = {R[s][0 + h], R[s][4 + h], R[s][8 + h], R[s][12 + h]};
      const u4 dl = {R[s][2 + h], R[s][6 + h], R[s][10 + h], R[s][14 + h]};
      const u4 wbh = WB[(kp * 2 + 0) * 64 + lane], wbl = WB[(kp * 2 + 1) * 64 + lane];
      const f4 y = mfma3(wbh, wbl, dh, dl);
      const float y0 = fmaf(y[1], y[1], y[0] * y[0]), y1 = fmaf(y[3], y[3], y[2] * y[2]);
      f4 z;
      if (kk == 0 && ty == 0) {  // kp = 0: bins 16 + 32 (7 - 2 g), 16 + 32 (6 - 2 g)
        z = mfma3(WB[(16 * 2 + 0) * 64 + lane], WB[(16 * 2 + 1) * 64 + lane], dh, dl);
      } else {  // the mirror bins 32 - kp + 32 (7 - k2): odd n2 negated
        const u4 fh = {dh[0], dh[1] ^ 0x80008000u, dh[2], dh[3] ^ 0x80008000u};
        const u4 fl = {dl[0], dl[1] ^ 0x80008000u, dl[2], dl[3] ^ 0x80008000u};
        z = mfma3(wbh, wbl, fh, fl);
      }
      const float z0 = fmaf(z[1], z[1], z[0] * z[0]), z1 = fmaf(z[3], z[3], z[2] * z[2]);
      if constexpr (PERM) {
        pd[0][kk >> 2][kk & 3] = y0;
        pd[1][kk >> 2][kk & 3] = y1;
        pm[0][(7 - kk) >> 2][(7 - kk) & 3] = z0;
        pm[1][(7 - kk) >> 2][(7 - kk) & 3] = z1;
      } else {
        prow[kp + 32 * ka] = y0;
        prow[kp + 32 * kb] = y1;
        if (kk == 0 && ty == 0) {
          prow[16 + 32 * (7 - ka)] = z0;
          prow[16 + 32 * (7 - kb)] = z1;
        } else {
          prow[256 - kp - 32 * ka] = z0;
          prow[224 - kp - 32 * ka] = z1;
        }
      }
    }
  }
  if constexpr (PERM) {
    // direct runs at columns 32 k2 + 8 ty, mirror runs (position 7 - kk) at
    // 32 (7 - k2) + 24 - 8 ty
    f4* d0 = reinterpret_cast<f4*>(__builtin_assume_aligned(prow + 32 * ka + 8 * ty, 16));
    f4* d1 = reinterpret_cast<f4*>(__builtin_assume_aligned(prow + 32 * kb + 8 * ty, 16));
    f4* m0p = reinterpret_cast<f4*>(__builtin_assume_aligned(prow + 32 * (7 - ka) + 24 - 8 * ty, 16));
    f4* m1p = reinterpret_cast<f4*>(__builtin_assume_aligned(prow + 32 * (7 - kb) + 24 - 8 * ty, 16));
    d0[0] = pd[0][0];
    d0[1] = pd[0][1];
    d1[0] = pd[1][0];
    d1[1] = pd[1][1];
    m0p[0] = pm[0][0];
    m0p[1] = pm[0][1];
    m1p[0] = pm[1][0];
    m1p[1] = pm[1][1];
  }
}

// the wave's max of its task values over the raw bits: unsigned (largest
// negative magnitude, or the largest positive value if none is negative)
// and signed (largest positive value)
__device__ __forceinline__ void bits_max(const float (&v)[kTaskRounds][8], int nr, unsigned& um, int& sm) {
  um = 0u;
  sm = 0;
#pragma unroll
  for (int r = 0; r < kTaskRounds; ++r) {
    if (r < nr) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned b = __builtin_bit_cast(unsigned, v[r][j]);
        um = um > b ? um : b;
        sm = sm > (int)b ? sm : (int)b;
      }
    }
  }
}
// max finite |x| bits (non-finite values excluded)
__device__ __forceinline__ unsigned finite_max(const float (&v)[kTaskRounds][8], int nr) {
  unsigned m = 0u;
#pragma unroll
  for (int r = 0; r < kTaskRounds; ++r) {
    if (r < nr) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned b = __builtin_bit_cast(unsigned, v[r][j]) & 0x7fffffffu;
        const unsigned f = b < 0x7f800000u ? b : 0u;
        m = m > f ? m : f;
      }
    }
  }
  return m;
}
__device__ __forceinline__ unsigned wave_umax(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned w = (unsigned)__shfl_xor((int)v, o);
    v = v > w ? v : w;
  }
  return v;
}
__device__ __forceinline__ int wave_smax(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int w = __shfl_xor(v, o);
    v = v > w ? v : w;
  }
  return v;
}

// the tile scale from the largest finite |x| (bits): 2^sc
__device__ __forceinline__ int tile_sc(unsigned tm_bits) {
  if (tm_bits == 0u) return 0;
  const float tm = __builtin_bit_cast(float, tm_bits);
  if (tm >= 32.f && tm < 32768.f) return -5;
  const int e = __builtin_amdgcn_frexp_expf(tm);  // tm = m 2^e, m in [0.5, 1)
  const int sc = 10 - e;
  return sc > 127 ? 127 : sc;
}

#ifndef VAD_MX_PAR
#define VAD_MX_PAR 1  // 0 (A/B builds): frames 16 bt + i per batch, staging reads by ds_read2_b32
#endif

// lifter x DCT of 16 log-mel rows r0 .. r0 + 15 (dct_mfma16) whose row
// r0 + j is frame fb + fs j
template <int SPEC>
__device__ __forceinline__ void dct_rows(const float* __restrict__ lm, const float* __restrict__ dtb, int r0, int lane,
                                         int64_t fb, int fs, int64_t f_end, float* __restrict__ out) {
  constexpr int KS = dct_k_steps<SPEC>(), LMS = lm_stride<SPEC>(), MN = 13;
  asm volatile("" : "+v"(lane));
  const float* arow = lm + (r0 + (lane & 15)) * LMS + (lane >> 4);
  const float* brow = dtb + (lane >> 4) * 16 + (lane & 15);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(arow[4 * s], brow[64 * s], acc, 0, 0, 0);
  const int c = lane & 15;
  const int64_t f = fb + fs * 4 * (lane >> 4);
  if (c < MN) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (f + fs * r < f_end) out[(f + fs * r) * MN + c] = acc[r];
  }
}

#ifndef VAD_MX_PERM
#define VAD_MX_PERM 1  // 0 (A/B builds): plain power rows, 32 ds_write_b32 per lane and tile
#endif
template <int SPEC>
constexpr bool kMxPerm = SPEC >= 1 && VAD_MX_PERM;
// (the runtime-tap path keeps frame-ordered rows: its VALU DCT stores row l as frame f0 + l)
template <int SPEC>
constexpr bool kMxPar = SPEC >= 1 && VAD_MX_PAR;

}  // namespace mx

// TIN float / int16_t; SPEC 1 / 2 the compiled 26 / 40-filter banks, 0 the
// plan's runtime taps; V4: 16-B aligned source (8-B for int16).
template <typename TIN, int SPEC, bool V4>
__global__ __launch_bounds__(kThreads, 1) void mfcc_mx_kernel(const MfccDev* __restrict__ plan,
                                                             const TIN* __restrict__ src, int64_t n_frames,
                                                             float* __restrict__ out, MfccBalance bal) {
  using namespace mx;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* P = reinterpret_cast<float*>(smem);
  unsigned* SH = reinterpret_cast<unsigned*>(smem + kStageOff);
  unsigned* SL = SH + 16 * kRow;
  float* lm = reinterpret_cast<float*>(smem + kLmOff);
  float* dtb = lm + kTile * lm_stride<SPEC>();
  u4* WB = reinterpret_cast<u4*>(smem + kWbOff);
  unsigned* red = reinterpret_cast<unsigned*>(smem + kRedOff);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bt = wave & 3, ty = wave >> 2;
  const int mfcc_n = plan->mfcc_n;
  const int64_t n_samples = (int64_t)kHop * (n_frames - 1) + kLen;
  const int64_t n_tiles = (n_frames + kTile - 1) / kTile;
  if constexpr (SPEC >= 1) dct_mfma_setup<SPEC>(plan, dtb, lm, kTile, tid, kThreads);

  // operand images of the DFT matrices (plan->mx_a / mx_b: [m][hi|lo][lane][4])
  const u4* ta = reinterpret_cast<const u4*>(plan->mx_a);
  const u4* tb = reinterpret_cast<const u4*>(plan->mx_b);
  const u4 wah = ta[(ty * 2 + 0) * 64 + lane], wal = ta[(ty * 2 + 1) * 64 + lane];
  for (int k = tid; k < 17 * 2 * 64; k += kThreads) WB[k] = tb[k];
  // the staging rows' pad dwords (read by lane group 3 of frame 63 with a
  // zero weight: must be finite)
  if (tid < 2 * 16 * (kRow - kQDw)) SH[(tid >> 2) * kRow + kQDw + (tid & 3)] = 0u;

  // tile runs (balanced over the XCDs' clocks when bal.word != 0)
  const unsigned long long rt0 = bal.stats ? __builtin_amdgcn_s_memrealtime() : 0;
  const int64_t f_beg = balanced_tile(bal.word, n_tiles, blockIdx.x, gridDim.x) * kTile;
  const int64_t f_end0 = balanced_tile(bal.word, n_tiles, blockIdx.x + 1, gridDim.x) * kTile;
  const int64_t f_end = f_end0 < n_frames ? f_end0 : n_frames;
  const int64_t t_end = (f_end - f_beg + kTile - 1) / kTile;
  if (t_end <= 0) return;  // uniform over the workgroup

  // staging tasks of this thread: k = tid + 512 r, chunk c = k & 3, pair d = k >> 2
  const int nr = tid + kThreads * (kTaskRounds - 1) < kTasks ? kTaskRounds : kTaskRounds - 1;
  float v[kTaskRounds][8];
  auto load_tile = [&](int64_t t) {
    const int64_t s0 = (f_beg + t * kTile) * kHop;
    const TIN* base = src + s0;
    const int64_t rem = n_samples - 1 - s0;
    const int lim = (int)(rem < 32 * kQDw ? rem : 32 * kQDw);
    const bool full = rem >= 32 * kQDw;  // uniform: no clamping needed
#pragma unroll
    for (int r = 0; r < kTaskRounds; ++r) {
      if (r < nr) {
        const int k = tid + kThreads * r;
        const int o = 32 * (k >> 2) + 4 * (k & 3);
        if (V4 && full) load_task<TIN, V4>(base, o, lim, v[r]);
        else load_task<TIN, false>(base, o, lim, v[r]);
      }
    }
  };
  // the tile's scale: max over the waves' partial maxima (after a barrier)
  auto publish_max = [&]() {
    unsigned um;
    int sm;
    bits_max(v, nr, um, sm);
    um = wave_umax(um);
    sm = wave_smax(sm);
    if (lane == 0) {
      red[wave] = um;
      red[8 + wave] = (unsigned)sm;
    }
  };
  // -> (sc, non-finite flag); a flagged tile's scale needs a second round
  auto read_scale = [&](bool& bad) {
    unsigned um = 0u;
    int sm = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const unsigned a = red[w];
      const int b = (int)red[8 + w];
      um = um > a ? um : a;
      sm = sm > b ? sm : b;
    }
    const unsigned mu = um & 0x7fffffffu, ms = (unsigned)(sm > 0 ? sm : 0);
    const unsigned tm = mu > ms ? mu : ms;
    bad = tm >= 0x7f800000u;
    return tm;
  };
  auto stage_store = [&](int sc) {
    const float s = __builtin_ldexpf(1.f, sc);
    int tk = tid;
    asm volatile("" : "+v"(tk));  // addresses per tile, not hoisted
#pragma unroll
    for (int r = 0; r < kTaskRounds; ++r) {
      if (r < nr) {
        const int k = tk + kThreads * r;
        const int c = k & 3, d = k >> 2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned hi, lo;
          split_scaled(v[r][j], v[r][4 + j], s, hi, lo);
          SH[(4 * c + j) * kRow + d] = hi;
          SL[(4 * c + j) * kRow + d] = lo;
        }
      }
    }
  };
  // scale of the tile in v: reads red after a barrier; a tile with NaN / inf
  // takes a second, finite-only round (two more barriers, rare)
  auto tile_scale = [&](bool& bad) {
    unsigned tm = read_scale(bad);
    if (bad) {
      lds_barrier();  // every wave has read red
      const unsigned m = wave_umax(finite_max(v, nr));
      if (lane == 0) red[wave] = m;
      lds_barrier();
      tm = 0u;
#pragma unroll
      for (int w = 0; w < 8; ++w) tm = tm > red[w] ? tm : red[w];
    }
    return tile_sc(tm);
  };

  // prologue: tile 0 staged, tile 1 requested
  load_tile(0);
  publish_max();
  lds_barrier();
  bool bad;
  int sc = tile_scale(bad);
  stage_store(sc);
  if (t_end > 1) load_tile(1);
  lds_barrier();

  for (int64_t t = 0; t < t_end; ++t) {
    const int64_t f0 = f_beg + t * kTile;
    // ---- phase 1: stage A + B -> power rows of tile t
    if (!kMxPar<SPEC>) {
      if (bad) phase1<true, kMxPerm<SPEC>, -1>(SH, SL, P, WB, lane, bt, ty, wah, wal);
      else phase1<false, kMxPerm<SPEC>, -1>(SH, SL, P, WB, lane, bt, ty, wah, wal);
    } else if (bt & 1) {
      if (bad) phase1<true, kMxPerm<SPEC>, 1>(SH, SL, P, WB, lane, bt, ty, wah, wal);
      else phase1<false, kMxPerm<SPEC>, 1>(SH, SL, P, WB, lane, bt, ty, wah, wal);
    } else {
      if (bad) phase1<true, kMxPerm<SPEC>, 0>(SH, SL, P, WB, lane, bt, ty, wah, wal);
      else phase1<false, kMxPerm<SPEC>, 0>(SH, SL, P, WB, lane, bt, ty, wah, wal);
    }
    const bool more = t + 1 < t_end;
    if (more) publish_max();
    lds_barrier();  // power rows complete; staging image consumed; maxima published
    const int ek = 2 - 2 * sc;  // |2X|^2 = |y|^2 2^(2 - 2 sc)
    if (more) {
      sc = tile_scale(bad);
      stage_store(sc);
      if (t + 2 < t_end) load_tile(t + 2);
    }
    if constexpr (kMxPerm<SPEC>) phase2a_mx<SPEC>(plan, P, lm, wave, lane, ek);
    else phase2a<SPEC>(plan, P, lm, wave, lane, ek);
    lds_barrier();  // log-mel rows complete; next staging image written; power rows free
    if (wave < kDctGroups) {  // rows 16 w .. 16 w + 15 = batch w
      if constexpr (kMxPar<SPEC>)
        dct_rows<SPEC>(lm, dtb, 16 * wave, lane, f0 + (wave & 1) + 32 * (wave >> 1), 2, f_end, out);
      else if constexpr (SPEC >= 1)
        dct_rows<SPEC>(lm, dtb, 16 * wave, lane, f0 + 16 * wave, 1, f_end, out);
      else
        phase2b<SPEC>(plan, lm, wave, lane, f0, f_end, mfcc_n, out);
    }
  }
  if (bal.stats && tid == 0 && t_end >= 8)
    bal.stats[blockIdx.x] = ((unsigned long long)t_end << 40) | (__builtin_amdgcn_s_memrealtime() - rt0);
}
