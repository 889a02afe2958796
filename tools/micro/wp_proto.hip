// Prototype (round 5): a barrier-free, wave-private MFCC pipeline for the
// reference framing (400 / 160, 512-point FFT, the compiled 26-filter bank).
//
// Each wave owns a contiguous run of frames end to end; nothing is shared
// between waves after the one-off table staging, so there is no workgroup
// barrier in the frame loop and the waves of a SIMD drift apart freely.
//   * 4 waves per workgroup (one per SIMD), 3 workgroups per CU = 3 waves per
//     SIMD (the shipped mfcc_kernel runs 2, bound by its 157.7 KB tile).
//   * Per wave and pair-tile (8 frames): each 16-lane group runs frames F and
//     F + 1 from one 18-chunk sample buffer, as the shipped paired-frame
//     phase 1 does (the same stage_a_at / store_a / read_b / finish_b code,
//     so the power spectra are bit for bit the shipped kernel's), but one
//     frame per "tile": the group's power row goes into its own transpose
//     block (2.3 KB, reused), and the group's 16 lanes run that frame's mel
//     bank right away, lane j taking filter filt[r][j] in round r over an
//     aligned window of b128 power quads with zero-padded weights (two
//     accumulators, even / odd bins: each filter's sum is the generated
//     code's two interleaved chains, bit for bit), then (==0 -> eps), log10
//     into a wave-private 16-row log-mel ring.
//   * Every 16 frames the wave's f32-MFMA lifter x DCT (dct_mfma16, the
//     shipped one) turns the ring into MFCC rows.
// Tables (per-lane twiddles, the DCT operand table, the mel lane weights)
// are staged into LDS once per workgroup; the twiddles are re-read from LDS
// right where each stage needs them, so they hold no VGPRs across the loop.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared
//        -fvisibility=hidden -mllvm -amdgpu-sched-strategy=max-ilp
//        tools/micro/wp_proto.hip -o tools/bin/libwp_proto.so
#include "../../vad_amd/csrc/mfcc_kernel.hip"

#include <stddef.h>

#ifndef WP_VARIANT
#define WP_VARIANT 0  // diagnostics: 1 no mel, 2 no mel + no DCT, 3 twiddles in VGPRs
#endif

namespace vad {
namespace wp {

constexpr int kWaves = 4;
constexpr int kThr = 64 * kWaves;
constexpr int kLMS = 28;  // ring row stride: 26 filters + 2 zero columns (the MFMA's K pad)
constexpr int kRingRows = 16;
constexpr size_t kWaveScrBytes = (size_t)4 * kGroupScratch * sizeof(v2f);  // 9,216
constexpr size_t kWaveBytes = kWaveScrBytes + (size_t)kRingRows * kLMS * sizeof(float);  // 11,008

// mel lanes of the 26-filter bank: filters sorted by width (widest first),
// round r takes sorted filters 16 r .. 16 r + 15, lane j the j-th of them;
// lane j's window starts at the filter's first tap rounded down to a
// multiple of 4 and spans nq[r] quads (the round's widest window)
struct LanePlan {
  int nr;
  int nq[3];
  int filt[3][16];  // -1: idle lane
  int base[3][16];
};

template <class T>
constexpr LanePlan make_plan() {
  LanePlan p{};
  int order[T::NF] = {};
  for (int i = 0; i < T::NF; ++i) order[i] = i;
  for (int i = 0; i < T::NF; ++i)  // stable selection sort, widest first
    for (int k = i + 1; k < T::NF; ++k)
      if (T::len[order[k]] > T::len[order[i]]) {
        const int t = order[i];
        order[i] = order[k];
        order[k] = t;
      }
  p.nr = (T::NF + 15) / 16;
  for (int r = 0; r < 3; ++r) {
    p.nq[r] = 0;
    for (int j = 0; j < 16; ++j) {
      const int s = 16 * r + j;
      p.filt[r][j] = (r < p.nr && s < T::NF) ? order[s] : -1;
      const int m = p.filt[r][j];
      p.base[r][j] = m >= 0 ? (T::lo[m] & ~3) : 0;
      if (m >= 0) {
        const int q = ((T::lo[m] & 3) + T::len[m] + 3) / 4;
        p.nq[r] = q > p.nq[r] ? q : p.nq[r];
      }
    }
  }
  return p;
}

constexpr LanePlan kPlan26 = make_plan<Mel26>();
__constant__ LanePlan kPlanDev = make_plan<Mel26>();  // runtime-indexed copy (table staging)
constexpr int kWQuads = kPlan26.nq[0] + kPlan26.nq[1] + kPlan26.nq[2];

constexpr size_t kTwOff = 0;
constexpr size_t kDtbOff = kTwOff + kTwLdsBytes;                          // 3,584
constexpr size_t kWtOff = kDtbOff + (size_t)4 * 7 * 16 * sizeof(float);   // + 1,792
constexpr size_t kItOff = kWtOff + (size_t)kWQuads * 16 * sizeof(v4f);
constexpr size_t kWaveOff = kItOff + (size_t)3 * 16 * 2 * sizeof(int);
constexpr size_t kSmem = kWaveOff + kWaves * kWaveBytes;

__device__ __forceinline__ void load_twa(const v2f* __restrict__ tw, int j, LaneConsts& L) {
  const v4f* a = reinterpret_cast<const v4f*>(__builtin_assume_aligned(launder(tw) + j * kTwaStride, 16));
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const v4f t = a[q];
    L.twa[2 * q] = t.xy;
    L.twa[2 * q + 1] = t.zw;
  }
}

__device__ __forceinline__ void load_twb(const v2f* __restrict__ tw, int j, LaneConsts& L) {
  const v4f* b = reinterpret_cast<const v4f*>(
      __builtin_assume_aligned(launder(tw) + 16 * kTwaStride + j * kTwbStride, 16));
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const v4f t = b[q];
    L.twb[2 * q] = t.xy;
    L.twb[2 * q + 1] = t.zw;
  }
}

// one frame's mel energies + log10 into ring row `lrow`: lane j of the frame's
// 16-lane group runs filter filt[R][j] of round R
template <int R, int WOFF>
__device__ __forceinline__ void mel_round(const float* __restrict__ prow, const v4f* __restrict__ wt,
                                          const int* __restrict__ it, int j, float* __restrict__ lrow) {
  constexpr int NQ = kPlan26.nq[R];
  const int base = it[(2 * R) * 16 + j];
  const int m = it[(2 * R + 1) * 16 + j];
  const v4f* pq = reinterpret_cast<const v4f*>(__builtin_assume_aligned(prow + base, 16));
  const v4f* wq = wt + WOFF * 16 + j;
  float e0 = 0.f, e1 = 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const v4f p = pq[q];
    const v4f w = wq[16 * q];
    e0 = fmaf(w.x, p.x, e0);
    e1 = fmaf(w.y, p.y, e1);
    e0 = fmaf(w.z, p.z, e0);
    e1 = fmaf(w.w, p.w, e1);
  }
  float e = e0 + e1;
  e = (e == 0.f) ? 0x1p-52f : e;
  if (m >= 0) lrow[m] = log10_pos(e);
}

__device__ __forceinline__ void mel_lanes(const float* __restrict__ prow, const v4f* __restrict__ wt,
                                          const int* __restrict__ it, int j, float* __restrict__ lrow) {
  static_assert(kPlan26.nr == 2, "two rounds of 16 mel lanes");
  mel_round<0, 0>(prow, wt, it, j, lrow);
  mel_round<1, kPlan26.nq[0]>(prow, wt, it, j, lrow);
}

__global__ __launch_bounds__(kThr, WP_VARIANT == 3 ? 2 : 3) void wp_mfcc_kernel(const MfccDev* __restrict__ plan,
                                                           const float* __restrict__ src, int64_t n_frames,
                                                           float* __restrict__ out) {
  constexpr int LEN = 400, HOPC = 5, NZ = 13, NB = NZ + HOPC;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  v2f* tw = reinterpret_cast<v2f*>(smem + kTwOff);
  float* dtb = reinterpret_cast<float*>(smem + kDtbOff);
  v4f* wt = reinterpret_cast<v4f*>(smem + kWtOff);
  int* it = reinterpret_cast<int*>(smem + kItOff);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int j = lane & 15;
  unsigned char* wbase = smem + kWaveOff + wave * kWaveBytes;
  v2f* gscr = reinterpret_cast<v2f*>(wbase) + g * kGroupScratch;
  float* prow = reinterpret_cast<float*>(gscr);  // the group's power row, in its transpose block
  float* ring = reinterpret_cast<float*>(wbase + kWaveScrBytes);

  // ---- one-off staging (the only barrier)
  stage_twiddles(plan, tw, tid, kThr);
  for (int i = tid; i < 4 * 7 * 16; i += kThr) {
    const int m = i >> 4, c = i & 15;
    dtb[i] = (c < 13 && m < 26) ? plan->dct[c * kMaxFilters + m] : 0.f;
  }
  for (int i = tid; i < kWQuads * 16 * 4; i += kThr) {
    const int comp = i & 3, jj = (i >> 2) & 15, qq = i >> 6;
    int r = 0, q = qq;
    while (r < 2 && q >= kPlanDev.nq[r]) q -= kPlanDev.nq[r++];
    const int m = kPlanDev.filt[r][jj];
    const int k = kPlanDev.base[r][jj] + 4 * q + comp;
    float w = 0.f;
    if (m >= 0 && k >= plan->f_lo[m] && k < plan->f_lo[m] + plan->f_len[m]) w = plan->taps[plan->f_off[m] + k - plan->f_lo[m]];
    reinterpret_cast<float*>(wt)[i] = w;
  }
  if (tid < 3 * 16) {
    const int r = tid >> 4, jj = tid & 15;
    it[(2 * r) * 16 + jj] = kPlanDev.base[r][jj];
    it[(2 * r + 1) * 16 + jj] = kPlanDev.filt[r][jj];
  }
  for (int i = lane; i < kRingRows * 2; i += 64) ring[(i >> 1) * kLMS + 26 + (i & 1)] = 0.f;
  __syncthreads();

  // ---- this wave's run of pair-tiles (8 frames each)
  const int64_t n_pt = (n_frames + 7) / 8;
  const int64_t nw = (int64_t)gridDim.x * kWaves;
  const int64_t wg = (int64_t)blockIdx.x * kWaves + wave;
  const int64_t pt_beg = wg * n_pt / nw, pt_end = (wg + 1) * n_pt / nw;
  if (pt_beg >= pt_end) return;  // wave-uniform; no barrier follows
  const int64_t f_beg = pt_beg * 8;
  const int64_t f_end = pt_end * 8 < n_frames ? pt_end * 8 : n_frames;
  const int n_loc = (int)(pt_end - pt_beg);
  const int64_t flast = n_frames - 1;
  LaneConsts L;
  lane_ints(j, L);
  if (WP_VARIANT == 3) lane_consts(plan, j, L);
  auto pair_base = [&](int i, int& lim) __attribute__((always_inline)) {
    const int64_t F = f_beg + 8 * (int64_t)i + 2 * g;
    lim = F < flast ? 32 * HOPC + LEN - 2 : LEN - 2;
    return src + (F < flast ? F : flast) * (32 * HOPC);
  };
  v2f buf[NB];
  {
    int lim;
    const float* b0 = pair_base(0, lim);
    load_chunks<float, 0, NB, LEN>(b0, lim, j, buf);
  }
  __builtin_amdgcn_sched_barrier(0);
  for (int i = 0; i < n_loc; ++i) {
    int lim;
    const float* nb = pair_base(i + 1, lim);
    const int rb = 8 * (i & 1) + 2 * g;  // ring rows of frames F, F + 1
    v2f u[16], col[32];
    // frame F
    if (WP_VARIANT != 3) load_twa(tw, j, L);
    stage_a_at<float, NZ, LEN, 0, NB>(buf, L, j, u);
    __builtin_amdgcn_sched_barrier(0);
    load_chunks<float, 0, HOPC, LEN>(nb, lim, j, buf);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");  // the previous frame's mel reads of this block come first
    store_a(u, gscr, j);
    read_b(L, gscr, col);
    if (WP_VARIANT != 3) load_twb(tw, j, L);
    finish_b<false>(L, col, prow);
    asm volatile("" ::: "memory");
    if (WP_VARIANT == 0 || WP_VARIANT == 3) mel_lanes(prow, wt, it, j, ring + rb * kLMS);
    __builtin_amdgcn_sched_barrier(0);
    // frame F + 1
    if (WP_VARIANT != 3) load_twa(tw, j, L);
    stage_a_at<float, NZ, LEN, HOPC, NB>(buf, L, j, u);
    __builtin_amdgcn_sched_barrier(0);
    load_chunks<float, HOPC, NB, LEN>(nb, lim, j, buf);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    store_a(u, gscr, j);
    read_b(L, gscr, col);
    if (WP_VARIANT != 3) load_twb(tw, j, L);
    finish_b<false>(L, col, prow);
    asm volatile("" ::: "memory");
    if (WP_VARIANT == 0 || WP_VARIANT == 3) mel_lanes(prow, wt, it, j, ring + (rb + 1) * kLMS);
    __builtin_amdgcn_sched_barrier(0);
    if (WP_VARIANT != 2 && ((i & 1) || i == n_loc - 1)) {  // 16 ring rows (or the run's last 8): lifter x DCT on the MFMA
      asm volatile("" ::: "memory");
      dct_mfma16<1>(ring, dtb, 0, lane, f_beg + 16 * (int64_t)(i >> 1), f_end, out);
      asm volatile("" ::: "memory");
    }
  }
}

struct PlanHead {  // the leading fields of capi.hip's vad_mfcc_plan
  MfccDev host;
  MfccDev* dev;
};

}  // namespace wp
}  // namespace vad

extern "C" __attribute__((visibility("default"))) int wp_mfcc(const void* plan_handle, const float* src,
                                                             long long n_frames, float* out, int wg_per_cu,
                                                             void* stream) {
  using namespace vad;
  using namespace vad::wp;
  const MfccDev* dev = reinterpret_cast<const PlanHead*>(plan_handle)->dev;
  if (n_frames <= 0) return 0;
  int cus = 256;
  int d = 0;
  (void)hipGetDevice(&d);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d);
  const int64_t want = (n_frames + 8 * kWaves - 1) / (8 * kWaves);
  const int64_t cap = (int64_t)cus * (wg_per_cu > 0 ? wg_per_cu : 3);
  const int grid = (int)(want < cap ? want : cap);
  static std::atomic<unsigned long long> attr{0};
  hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(&wp_mfcc_kernel), (int)kSmem, attr);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(wp_mfcc_kernel, dim3(grid), dim3(kThr), kSmem, (hipStream_t)stream, dev, src,
                     (int64_t)n_frames, out);
  return (int)hipGetLastError();
}

extern "C" __attribute__((visibility("default"))) long long wp_smem_bytes() { return (long long)vad::wp::kSmem; }
