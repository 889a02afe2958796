// Streaming frame assembly: every stream's frame buffer advances by one hop
// (the oldest `hop` samples drop out, the new ones are appended), i.e. the
// frame that SKLearnAnalyzer.feed_frame (sklearn_analyser.py:46-82) receives
// when vad.py:37-49 cuts the live signal into 25 ms frames every 10 ms.
//
// One wave per stream, in place: the wave loads its whole row into
// registers, then stores it shifted.  Store i (sample t = lane + 64 i) waits
// for its own load, hence for every older load of the wave (vmcnt is in
// order), and a younger load i2 > i reads samples >= 64 i2 + hop > 64 i + 63,
// beyond anything store i writes -- so no sample is overwritten before it is
// read.
#include "vad_common.h"
#include "features.h"
#include "ffn_dev.h"

namespace vad {

template <int NR>  // registers per lane: frame_len <= 64 NR
__global__ __launch_bounds__(256) void stream_push_kernel(float* __restrict__ frames, int64_t fstride,
                                                          int len, const float* __restrict__ hop,
                                                          int64_t hstride, int hlen, int64_t n_streams) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= n_streams) return;
  float* row = frames + s * fstride;
  const float* h = hop + s * hstride;
  const int keep = len - hlen;
  float v[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = lane + 64 * i;
    v[i] = t < keep ? row[t + hlen] : (t < len ? h[t - keep] : 0.f);
  }
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = lane + 64 * i;
    if (t < len) row[t] = v[i];
  }
}

hipError_t launch_stream_push(float* frames, int64_t fstride, int len, const float* hop, int64_t hstride,
                              int hlen, int64_t n_streams, hipStream_t st) {
  if (n_streams <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n_streams + 3) / 4));
  if (len <= 64 * 7)
    hipLaunchKernelGGL(stream_push_kernel<7>, grid, dim3(256), 0, st, frames, fstride, len, hop, hstride,
                       hlen, n_streams);
  else
    hipLaunchKernelGGL(stream_push_kernel<16>, grid, dim3(256), 0, st, frames, fstride, len, hop, hstride,
                       hlen, n_streams);
  return hipGetLastError();
}

// Optional pre-emphasis (not in the reference pipeline, mfcc.py:59-61; the
// python_speech_features convention): y[0] = x[0], y[t] = x[t] - a x[t-1]
// along each row (a whole clip is one row).  Elementwise, 16-B vector loads
// of four samples plus the one before them; out of place.
// y[0] = x[0], y[t] = x[t] - a x[t-1] per row (python_speech_features
// sigproc.preemphasis; an optional stage, not in the reference).  Rows go
// over blockIdx.y (no 64-bit division per element); 16-B aligned rows move
// as float4 (four outputs per lane, the one earlier sample as a scalar load
// that the neighbour lane's vector load has already brought into L1).
template <bool VEC4>
__global__ __launch_bounds__(256) void preemphasis_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                          int64_t n_rows, int64_t row_len, int64_t stride,
                                                          float a) {
#pragma clang fp contract(off)  // a rounded product, then the difference: numpy's two roundings
  const int64_t quads = (row_len + 3) / 4;
  for (int64_t r = blockIdx.y; r < n_rows; r += gridDim.y) {
    const float* xr = x + r * stride;
    float* yr = y + r * stride;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads;
         q += (int64_t)gridDim.x * blockDim.x) {
      const int64_t t0 = 4 * q;
      const float prev = t0 > 0 ? xr[t0 - 1] : 0.f;
      if (VEC4 && t0 + 3 < row_len) {
        const float4 v = *reinterpret_cast<const float4*>(xr + t0);
        float4 o;
        o.x = t0 == 0 ? v.x : v.x - a * prev;
        o.y = v.y - a * v.x;
        o.z = v.z - a * v.y;
        o.w = v.w - a * v.z;
        *reinterpret_cast<float4*>(yr + t0) = o;
      } else {
        float p = prev;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t t = t0 + k;
          if (t < row_len) {
            const float v = xr[t];
            yr[t] = t == 0 ? v : v - a * p;
            p = v;
          }
        }
      }
    }
  }
}

hipError_t launch_preemphasis(const float* x, float* y, int64_t n_rows, int64_t row_len, int64_t stride, float a,
                              hipStream_t st) {
  if (n_rows <= 0 || row_len <= 0) return hipSuccess;
  const int64_t quads = (row_len + 3) / 4;
  int64_t bx = (quads + 255) / 256;
  if (bx > 8192) bx = 8192;
  int64_t by = n_rows < 65535 ? n_rows : 65535;
  while (bx * by > 65536 && bx > 1) bx = (bx + 1) / 2;  // about 16M threads in all
  const bool vec4 = (reinterpret_cast<uintptr_t>(x) % 16 == 0) && (reinterpret_cast<uintptr_t>(y) % 16 == 0) &&
                    (n_rows == 1 || stride % 4 == 0);
  if (vec4)
    hipLaunchKernelGGL(preemphasis_kernel<true>, dim3((unsigned)bx, (unsigned)by), dim3(256), 0, st, x, y, n_rows,
                       row_len, stride, a);
  else
    hipLaunchKernelGGL(preemphasis_kernel<false>, dim3((unsigned)bx, (unsigned)by), dim3(256), 0, st, x, y, n_rows,
                       row_len, stride, a);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// One analyser hop of every stream in ONE kernel, one wave per stream
// (BASELINE config 5: many small batches, latency first).  The clip kernels
// spread a 64-frame tile over a workgroup; a hop brings one frame per
// stream, so here each wave owns its stream end to end:
//   frame    advance the 400-sample buffer by the hop (as stream_push_kernel)
//   FFT      z[n] = x[2n] + i x[2n+1] (zero past min(len, 512)), 256-point
//            Stockham radix-4 (4 stages through wave-private LDS, lane j
//            one butterfly per stage), then the real-FFT split into
//            |2X[k]|^2, k = 0..255 (the 2^-20 of |X/512|^2 sits in the taps)
//   mel      lane m: filter m's taps, (==0 -> eps), log10 (mfcc.py:72-75)
//   DCT      lane c: lifter x DCT-II ortho row c (mfcc.py:76-78)
//   window   the ring's five rows in arrival order -> analyser features
//            (sklearn_analyser.py:52-69), classified if the stream has seen
//            five frames, then the new row pushed (:71-74)
//   FFN      exact f32 on the VALU, lane o = output unit o, weights as given
//            (ffn_trainer.py:106-116), NaN-keeping ReLU, np.argmax rules.
// Lanes within the wave exchange through LDS only (in order per wave): no
// workgroup barrier anywhere.
// ---------------------------------------------------------------------------
// Per-wave LDS scratch (floats): the FFT's ping-pong buffers (the power
// row reuses the first once the transform is done), the log-mel row, two
// activation rows.
#ifndef VAD_HOP_Q
#define VAD_HOP_Q 4
#endif
constexpr int kHopZ = 2 * (256 + 32);              // one 256-point complex buffer, padded
// complex element i of a buffer sits at i + i / 8: the Stockham stores of the
// first stages (stride 4 and 16 complex across lanes) spread over the banks
#ifndef VAD_HOP_PAD
#define VAD_HOP_PAD 1
#endif
__device__ __forceinline__ int zp(int i) { return VAD_HOP_PAD ? i + (i >> 3) : i; }
constexpr int kHopWaveFloats = 2 * kHopZ + kMaxFilters + 64 + 64;

// Block-shared LDS, staged once per block from the plans (the per-stream
// chain would otherwise wait on one L2 round trip per tap, DCT term and
// weight): twiddles, filter ranges and taps, the DCT rows, the FFN weights.
struct HopTables {
  const float2* tw;  // W512^k, k < 256
  const int* f_lo;
  const int* f_len;
  const int* f_off;
  const float* taps;
  const float* dct;  // [c][m], stride vec_row_stride(nf), 16-B aligned
  const float* w;    // the FFN weights (FfnDev::wraw: transposed rows)
};

__device__ __forceinline__ float2 cmulf(float2 a, float2 w) {
  return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}

// W256^m, 0 <= m < 256, from the W512^k table
__device__ __forceinline__ float2 w256(const float2* __restrict__ tw, int m) {
  const float2 t = tw[2 * (m & 127)];
  return m < 128 ? t : make_float2(-t.x, -t.y);
}

// NR: 64-sample chunks of the frame a lane holds (7: frames up to 448
// samples, the reference's 400; 16: up to 1024) -- the frame and the next
// hop's samples stay in registers across hops, so the bound matters
template <int NR>
__global__ __launch_bounds__(1024) void stream_hop_kernel(const float* __restrict__ blob, int blob_n, int nf,
                                                          int n_taps, FfnDev net,
                                                          float* __restrict__ frames, int64_t fstride, int len,
                                                          const float* __restrict__ hop, int64_t hstride,
                                                          int hlen, int64_t n_streams, int mfcc_n,
                                                          float* __restrict__ ring, int* __restrict__ count,
                                                          uint8_t* __restrict__ labels, int n_hops,
                                                          int64_t hop_kstride, int64_t lab_kstride) {
  extern __shared__ __attribute__((aligned(16))) float hsm[];
  const int waves = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  // -- stage the plans' tables (the MFCC plan's hop blob, then the FFN
  // weights) by LDS-DMA (global_load_lds_dwordx4: 1 KB per wave-instruction,
  // no registers, all in flight at once), then request the stream's state
  // and the FFT's twiddles (registers), then the block's only barrier.
  // (A/B, 512 streams, profiles/r05/ab/hop_staging_ab.json: 10.26 us per
  // one-hop launch against 10.56 for register staging with LDS twiddles;
  // the barrier moved after the first hop's FFT, so that the staging would
  // overlap it, measured 10.84: the mid-hop barrier costs more than it hides)
  float* base = hsm + waves * kHopWaveFloats;
  {
    const float4* m4 = reinterpret_cast<const float4*>(blob);
    const float4* w4 = reinterpret_cast<const float4*>(net.wraw);
    const int nm4 = blob_n >> 2, n4 = nm4 + (net.wraw_n >> 2);
    for (int c0 = wv * 64; c0 < n4; c0 += (int)blockDim.x) {  // wave-uniform chunk base
      const int c = c0 + lane;
      if (c < n4)
        __builtin_amdgcn_global_load_lds(c < nm4 ? (const void*)(m4 + c) : (const void*)(w4 + (c - nm4)),
                                         (__attribute__((address_space(3))) void*)(base + 4 * c0), 16, 0, 0);
    }
  }
  HopTables T;
  T.tw = reinterpret_cast<const float2*>(base);
  const int* ilo = reinterpret_cast<const int*>(base + 2 * 256);
  T.f_lo = ilo;
  T.f_len = ilo + nf;
  T.f_off = ilo + 2 * nf;
  T.taps = base + ((2 * 256 + 3 * nf + 3) & ~3);  // 16-B aligned rows of n_taps (a multiple of 4) in all
  T.dct = T.taps + n_taps;
  T.w = base + blob_n;

  const int64_t s = (int64_t)blockIdx.x * waves + wv;
  const int64_t sc = s < n_streams ? s : 0;
  // -- the stream's state, requested before the barrier so its latency
  // overlaps the staging: the frame as it stands (registers, sample t =
  // lane + 64 i), the first hop's new samples at the positions they take in
  // the advanced frame, the frame count and the MFCC ring
  float* row = frames + sc * fstride;
  const int keep = len - hlen;
  float v[NR], hn[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = lane + 64 * i;
    v[i] = t < len ? row[t] : 0.f;
    hn[i] = (t >= keep && t < len) ? hop[sc * hstride + (t - keep)] : 0.f;
  }
  int c = count[sc];
  float* rs = ring + sc * 5 * mfcc_n;
  float rv[5];
#pragma unroll
  for (int d = 0; d < 5; ++d) rv[d] = lane < mfcc_n ? rs[d * mfcc_n + lane] : 0.f;
  // this lane's FFT twiddles (W512^k table = the blob's first 256 complex):
  // stage st's radix-4 butterfly multiplies by W256^(j m), m = (lane mod
  // 4^st) 64 / 4^st, j = 1..3; the real-FFT split by W512^(lane + 64 q)
  // (the 16-chunk build, whose frame registers leave no room for them, reads
  // them from the staged table where it uses them)
  const float2* tw_g = reinterpret_cast<const float2*>(blob);
  constexpr bool kTwReg = NR <= 7;
  float2 twr[3][3], tws[4];
  if constexpr (kTwReg) {
#pragma unroll
    for (int st = 1; st < 4; ++st) {
      const int ns = 1 << (2 * st);
      const int m = (lane & (ns - 1)) * (64 >> (2 * st));
#pragma unroll
      for (int jj = 1; jj < 4; ++jj) twr[st - 1][jj - 1] = w256(tw_g, jj * m);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) tws[q] = tw_g[lane + 64 * q];
  }
  // the staged tables are complete: LDS-DMA writes count on vmcnt, not
  // lgkmcnt, and a workgroup-scope release fence need not drain vmcnt, so the
  // wait is explicit (vmcnt 0, before the barrier; the state and twiddle
  // loads above are needed right after it anyway).  Locked by
  // test_hop_kernel_waits_for_lds_dma_before_barrier (the built ISA).
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt 0, expcnt 7, lgkmcnt 15
  __syncthreads();
  if (s >= n_streams) return;  // wave-uniform; no barrier below
  float* scr = hsm + wv * kHopWaveFloats;
  float2* z0 = reinterpret_cast<float2*>(scr);
  float2* z1 = reinterpret_cast<float2*>(scr + kHopZ);
  float* lmr = scr + 2 * kHopZ;
  float* act_a = lmr + kMaxFilters;
  float* act_b = act_a + 64;
  float* fb = scr;  // the frame shift goes through the FFT buffers (2 kHopZ >= 1024 floats)
  const int used = len < kFftN ? len : kFftN;

  // K hops of this stream back to back: the same computation per hop as K
  // launches of one hop (state carried in registers), the tables staged once
  for (int k = 0; k < n_hops; ++k) {
    // the lane index, opaque per hop: otherwise the compiler hoists every
    // lane-dependent LDS address of the hop out of the loop and runs out of
    // registers holding them
    int ln = lane;
    asm volatile("" : "+v"(ln));
    // -- frame: shift by the hop (through LDS: sample t + hlen belongs to
    // another ln), append the new samples (stream_push_kernel)
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int t = ln + 64 * i;
      if (t < len) fb[t] = v[i];
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int t = ln + 64 * i;
      v[i] = t < keep ? fb[t + hlen] : hn[i];
    }
    asm volatile("" ::: "memory");
    if (k + 1 < n_hops) {  // the next hop's samples, in flight during this one
      const float* hs = hop + (int64_t)(k + 1) * hop_kstride + s * hstride;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        const int t = ln + 64 * i;
        hn[i] = (t >= keep && t < len) ? hs[t - keep] : 0.f;
      }
    }
    uint8_t* lab_k = labels + (int64_t)k * lab_kstride;
    // samples of the FFT (np.fft.fft(x, 512): zero-pad / truncate, mfcc.py:61)
    float* xs = reinterpret_cast<float*>(z1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // all 512 inputs: the zero padding past the frame too
      const int t = ln + 64 * i;  // sample t = component t & 1 of complex t / 2
      xs[2 * zp(t >> 1) + (t & 1)] = (i < NR && t < used) ? v[i < NR ? i : 0] : 0.f;
    }
    // LDS is in order within a wave; these keep the compiler from moving
    // accesses of one phase (other lanes' data, other element types) across
    // the next
    asm volatile("" ::: "memory");

    // -- 256-point complex FFT, Stockham radix-4
    float2* src = z1;
    float2* dst = z0;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int ns = 1 << (2 * st);  // 1, 4, 16, 64
      const int kk = ln & (ns - 1);
      float2 a0 = src[zp(ln)], a1 = src[zp(ln + 64)], a2 = src[zp(ln + 128)], a3 = src[zp(ln + 192)];
      if (st > 0) {  // W_{4 ns}^(j k) = W256^(64 j k / ns)
        const int m = kk * (64 >> (2 * st));
        a1 = cmulf(a1, kTwReg ? twr[st - 1][0] : w256(T.tw, m));
        a2 = cmulf(a2, kTwReg ? twr[st - 1][1] : w256(T.tw, 2 * m));
        a3 = cmulf(a3, kTwReg ? twr[st - 1][2] : w256(T.tw, 3 * m));
      }
      const float2 b0 = make_float2(a0.x + a2.x, a0.y + a2.y), b1 = make_float2(a0.x - a2.x, a0.y - a2.y);
      const float2 b2 = make_float2(a1.x + a3.x, a1.y + a3.y), b3 = make_float2(a1.x - a3.x, a1.y - a3.y);
      const int o = (ln >> (2 * st)) * (4 * ns) + kk;
      dst[zp(o)] = make_float2(b0.x + b2.x, b0.y + b2.y);
      dst[zp(o + ns)] = make_float2(b1.x + b3.y, b1.y - b3.x);      // b1 - i b3
      dst[zp(o + 2 * ns)] = make_float2(b0.x - b2.x, b0.y - b2.y);
      dst[zp(o + 3 * ns)] = make_float2(b1.x - b3.y, b1.y + b3.x);  // b1 + i b3
      float2* t = src;
      src = dst;
      dst = t;
      asm volatile("" ::: "memory");
    }
    // -- real-FFT split: 2X[k] = S - i W512^k D, S = Z[k] + conj(Z[-k]),
    // D = Z[k] - conj(Z[-k]); |2X|^2 into the free buffer
    float* pw = reinterpret_cast<float*>(dst);
    float pk[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kb = ln + 64 * q;
      const float2 zk = src[zp(kb)], zn = src[zp((256 - kb) & 255)];
      const float2 S = make_float2(zk.x + zn.x, zk.y - zn.y);
      const float2 D = make_float2(zk.x - zn.x, zk.y + zn.y);
      const float2 Tw = cmulf(D, kTwReg ? tws[q] : T.tw[kb]);
      const float u = S.x + Tw.y, vv = S.y - Tw.x;
      pk[q] = fmaf(u, u, vv * vv);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) pw[ln + 64 * q] = pk[q];
    asm volatile("" ::: "memory");
    // -- mel + log10 (ln m), lifter x DCT (ln c)
    if (ln < nf) {
      // the filter's 16-B aligned tap row against the power bins from its
      // first bin rounded down to 4: four taps per pair of 16-B reads, one
      // fma chain in bin order (the zero taps around the filter add +0)
      const int lo4 = T.f_lo[ln], n4 = T.f_len[ln];
      const float4* wt4 = reinterpret_cast<const float4*>(T.taps + T.f_off[ln]);
      const float4* pw4 = reinterpret_cast<const float4*>(pw + lo4);
      float e = 0.f;
#pragma unroll 2
      for (int t = 0; t < n4; t += 4) {
        const float4 w = wt4[t >> 2], q = pw4[t >> 2];
        e = fmaf(w.x, q.x, e);
        e = fmaf(w.y, q.y, e);
        e = fmaf(w.z, q.z, e);
        e = fmaf(w.w, q.w, e);
      }
      lmr[ln] = log10_pos(e == 0.f ? 0x1p-52f : e);  // mfcc.py:74-75
    }
    asm volatile("" ::: "memory");
    float mf = 0.f;
    if (ln < mfcc_n) {
      // one fma chain in m order; four terms per pair of 16-B reads (the
      // lane's row, the log-mel row broadcast)
      const float4* d4 = reinterpret_cast<const float4*>(T.dct + ln * vec_row_stride(nf));
      const float4* l4 = reinterpret_cast<const float4*>(lmr);
      int m = 0;
#pragma unroll 4
      for (; m + 4 <= nf; m += 4) {
        const float4 d = d4[m >> 2], l = l4[m >> 2];
        mf = fmaf(d.x, l.x, mf);
        mf = fmaf(d.y, l.y, mf);
        mf = fmaf(d.z, l.z, mf);
        mf = fmaf(d.w, l.w, mf);
      }
      const float* d = T.dct + ln * vec_row_stride(nf);
      for (; m < nf; ++m) mf = fmaf(d[m], lmr[m], mf);
    }
    // -- window of the five previous frames, then push the new row
    const bool have = c >= 5;
    act_a[ln] = 0.f;  // feature columns past 3 mfcc_n: zero (the FFN reads them in fours)
    asm volatile("" ::: "memory");
    if (ln < mfcc_n) {
      if (have) {
        // slot (c + d) % 5, d = 0..4: the ring in arrival order, oldest first
        float r[5];
#pragma unroll
        for (int d = 0; d < 5; ++d) {
          const int q = (c + d) % 5;
          r[d] = q == 0 ? rv[0] : q == 1 ? rv[1] : q == 2 ? rv[2] : q == 3 ? rv[3] : rv[4];
        }
        const Feat3 ft = feature_triple(r[0], r[1], r[2], r[3], r[4], VAD_FEAT_ANALYSER);
        act_a[ln] = ft.mn;
        act_a[mfcc_n + ln] = ft.d1;
        act_a[2 * mfcc_n + ln] = ft.d2;
      }
      const int q = c % 5;  // the push (ring slot of the oldest row)
#pragma unroll
      for (int d = 0; d < 5; ++d) rv[d] = q == d ? mf : rv[d];
    }
    asm volatile("" ::: "memory");
    {
      // layer 0 reads its inputs in fours: a network narrower than the feature
      // triple (13-64-64-N takes the 13 normalised coefficients) must see zeros,
      // not the delta columns, in the rest of its last block (stored after the
      // features: LDS is in order per wave)
      const int din0 = net.dims[0];
      if (ln >= din0 && ln < ((din0 + 3) & ~3)) act_a[ln] = 0.f;
    }
    asm volatile("" ::: "memory");
    uint8_t label = 255;
    if (have) {
      // -- FFN: exact f32, ln o of each layer
      float* hin = act_a;
      float* hout = act_b;
      const int nl = net.n_layers;
      for (int l = 0; l < nl; ++l) {
        const int din = net.dims[l], dout = net.dims[l + 1];
        // four inputs per step (one ds_read_b128 broadcast), four partial
        // sums; inputs past din are zero and the weight rows past W_l read
        // the next finite values of the block (zero-padded at its end)
        // the lane's transposed row: four weights per 16-B read
        const float4* w4 = reinterpret_cast<const float4*>(T.w + net.woff[l] + ln * net.wstride[l]);
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        if (ln < dout) {
          const float4* h4 = reinterpret_cast<const float4*>(hin);
#pragma unroll 4
          for (int kq = 0; kq < din; kq += 4) {
            const float4 h = h4[kq >> 2], w = w4[kq >> 2];
            a0 = fmaf(w.x, h.x, a0);
            a1 = fmaf(w.y, h.y, a1);
            a2 = fmaf(w.z, h.z, a2);
            a3 = fmaf(w.w, h.w, a3);
          }
        }
        const float acc = T.w[net.boff[l] + (ln < dout ? ln : 0)] + ((a0 + a1) + (a2 + a3));
        hout[ln] = ln < dout ? (l + 1 < nl ? relu_nan(acc) : acc) : 0.f;
        float* t = hin;
        hin = hout;
        hout = t;
        asm volatile("" ::: "memory");
      }
      const f32x4 zl = {hin[0], hin[1 < net.n_classes ? 1 : 0], hin[2 < net.n_classes ? 2 : 0],
                        hin[3 < net.n_classes ? 3 : 0]};
      label = (uint8_t)argmax_classes(zl, net.n_classes);
    }
    if (ln == 0) lab_k[s] = label;
    c = (c + 1 >= 10) ? c + 1 - 5 : c + 1;
    asm volatile("" ::: "memory");
  }
  // -- the stream's state back: frame, ring, count
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = lane + 64 * i;
    if (t < len) row[t] = v[i];
  }
  if (lane < mfcc_n) {
#pragma unroll
    for (int d = 0; d < 5; ++d) rs[d * mfcc_n + lane] = rv[d];
  }
  if (lane == 0) count[s] = c;
}

hipError_t launch_stream_hop(const MfccDev* plan, const float* blob, int blob_n, int nf, int n_taps,
                             const FfnDev& net, float* frames, int64_t fstride, int len, const float* hop,
                             int64_t hstride, int hlen, int64_t n_streams, int mfcc_n, float* ring, int* count,
                             uint8_t* labels, int n_hops, int64_t hop_kstride, int64_t lab_kstride,
                             hipStream_t st) {
  (void)plan;
  if (n_streams <= 0 || n_hops <= 0) return hipSuccess;
  const size_t tables = (size_t)(blob_n + net.wraw_n) * sizeof(float);
  // streams per block: at least VAD_HOP_MIN_WAVES (one wave per SIMD), then
  // spread over every CU (each block stages the ~26 KB of tables from L2
  // once; the per-stream chain is LDS-bound, so fewer waves per CU run it
  // faster), up to 16 waves when there are more streams than CUs, and as
  // many as the LDS holds.  512 streams, A/B on one box: 2 waves per block
  // on 256 CUs 11.0-11.3 us per hop, 4 on 128 CUs 10.4, 8 on 64 CUs 10.8
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
  }
#ifndef VAD_HOP_MIN_WAVES
#define VAD_HOP_MIN_WAVES 4
#endif
#ifndef VAD_HOP_MIN_WAVES_K
#define VAD_HOP_MIN_WAVES_K 1  // launches of several hops: the staging amortises over the hops, so
                               // one stream per block spreads over more CUs (K = 8: 8.2 vs 8.4 us
                               // per hop, K = 32: 7.4 vs 7.6 with 4 per block)
#endif
  int waves = n_hops > 1 ? VAD_HOP_MIN_WAVES_K : VAD_HOP_MIN_WAVES;
  while (waves < 16 && (int64_t)waves * n_cu < n_streams) waves <<= 1;
  while (waves > 1 && tables + (size_t)waves * kHopWaveFloats * sizeof(float) > 160 * 1024) waves >>= 1;
  const size_t smem = tables + (size_t)waves * kHopWaveFloats * sizeof(float);
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  static std::atomic<unsigned long long> attr_done{0};
  static std::atomic<unsigned long long> attr_done16{0};
  const bool small = len <= 7 * 64;
  const void* fn = small ? reinterpret_cast<const void*>(&stream_hop_kernel<7>)
                         : reinterpret_cast<const void*>(&stream_hop_kernel<16>);
  const hipError_t e = ensure_dyn_lds(fn, 160 * 1024, small ? attr_done : attr_done16);
  if (e != hipSuccess) return e;
  const dim3 grid((unsigned)((n_streams + waves - 1) / waves));
  if (small)
    hipLaunchKernelGGL(stream_hop_kernel<7>, grid, dim3(64 * waves), smem, st, blob, blob_n, nf, n_taps, net, frames,
                       fstride, len, hop, hstride, hlen, n_streams, mfcc_n, ring, count, labels, n_hops, hop_kstride,
                       lab_kstride);
  else
    hipLaunchKernelGGL(stream_hop_kernel<16>, grid, dim3(64 * waves), smem, st, blob, blob_n, nf, n_taps, net, frames,
                       fstride, len, hop, hstride, hlen, n_streams, mfcc_n, ring, count, labels, n_hops, hop_kstride,
                       lab_kstride);
  return hipGetLastError();
}

}  // namespace vad
