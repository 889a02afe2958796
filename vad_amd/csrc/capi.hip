// extern "C" boundary of libvad_amd.so (include/vad_amd.h): plans, argument
// checking and kernel dispatch.  Host-side work here is one-off plan setup
// (filterbank -> sparse taps, lifter x DCT matrix, twiddles, FFN fragments);
// every hot entry point only validates and launches.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "vad_common.h"
#include "mel_tables.h"

using namespace vad;

// Host side of the MFCC kernel's XCD balance (vad_common.h MfccBalance):
// the kernel's paired-frame runs write (tiles, ticks) per workgroup into
// host-mapped memory; each launch folds the latest ones into per-XCD speed
// weights (workgroup b on XCD b mod 8) and passes them as a kernel argument,
// so every workgroup of a launch splits the tiles from the same 8 bytes.
// Opt-in (VAD_MFCC_BALANCE=1): on the boxes measured it moved the MFCC
// launch by -1 % but the whole C3 step by +0.6 %.
#ifndef VAD_BALANCE_DEFAULT
#define VAD_BALANCE_DEFAULT 0
#endif

namespace {
constexpr int kBalSlots = 1024;  // workgroups of a launch (<= CUs)
struct BalanceHost {
  unsigned long long* stats_host = nullptr;  // pinned, mapped
  unsigned long long* stats_dev = nullptr;
  float w[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  unsigned long long word = 0;    // the weights in use
  unsigned long long calls = 0;
  unsigned long long forced = 0;  // VAD_MFCC_BALANCE_WORD (tests): fixed weights
  std::mutex mu;
};

BalanceHost* balance_create() {
  const char* env = getenv("VAD_MFCC_BALANCE");
  if (env ? atoi(env) == 0 : VAD_BALANCE_DEFAULT == 0) return nullptr;
  BalanceHost* b = new BalanceHost();
  void* h = nullptr;
  if (hipHostMalloc(&h, kBalSlots * sizeof(unsigned long long), hipHostMallocMapped) != hipSuccess) {
    delete b;
    return nullptr;
  }
  memset(h, 0, kBalSlots * sizeof(unsigned long long));
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    delete b;
    return nullptr;
  }
  b->stats_host = (unsigned long long*)h;
  b->stats_dev = (unsigned long long*)d;
  if (const char* fw = getenv("VAD_MFCC_BALANCE_WORD")) {
    b->forced = strtoull(fw, nullptr, 0);
    for (int x = 0; x < 8; ++x)  // every weight >= 1, or no forcing
      if (((b->forced >> (8 * x)) & 255u) == 0) b->forced = 0;
  }
  return b;
}

void balance_destroy(BalanceHost* b) {
  if (!b) return;
  (void)hipDeviceSynchronize();  // no launch of this plan may still write its stats
  (void)hipHostFree(b->stats_host);
  delete b;
}

// this launch's weights from the stats the earlier launches left (a launch
// still running leaves some of its blocks' entries old: any mix is a valid,
// if less even, split)
MfccBalance balance_for_launch(BalanceHost* b) {
  MfccBalance r;
  if (!b) return r;
  if (b->forced) {
    r.word = b->forced;
    r.stats = b->stats_dev;
    return r;
  }
  // one launch in kStatsEvery writes stats (their PCIe stores delay the
  // launch's end by ~1 us); the weights are refolded halfway to the next
  std::lock_guard<std::mutex> lk(b->mu);
  constexpr unsigned long long kStatsEvery = 16;
  const unsigned long long c = b->calls++;
  if (c % kStatsEvery == kStatsEvery / 2 || b->word == 0) {
    double tiles[8] = {}, ticks[8] = {};
    const volatile unsigned long long* st = b->stats_host;
    for (int i = 0; i < kBalSlots; ++i) {
      const unsigned long long v = st[i];
      if (!v) continue;
      tiles[i & 7] += (double)(v >> 40);
      ticks[i & 7] += (double)(v & ((1ull << 40) - 1));
    }
    bool all = true;
    double sp[8], mx = 0.;
    for (int x = 0; x < 8; ++x) {
      all = all && tiles[x] > 0. && ticks[x] > 0.;
      sp[x] = ticks[x] > 0. ? tiles[x] / ticks[x] : 0.;
      mx = sp[x] > mx ? sp[x] : mx;
    }
    if (all && mx > 0.) {
      // a block's speed is its tiles per tick whatever its share, so the new
      // weights are the speeds (smoothed: the clocks drift with load and
      // temperature)
      for (int x = 0; x < 8; ++x) b->w[x] = 0.5f * b->w[x] + 0.5f * (float)(sp[x] / mx);
    }
    float wm = 0.f;
    for (int x = 0; x < 8; ++x) wm = b->w[x] > wm ? b->w[x] : wm;
    unsigned long long word = 0;
    for (int x = 0; x < 8; ++x) {
      int q = (int)lrintf(255.f * b->w[x] / wm);
      q = q < 128 ? 128 : (q > 255 ? 255 : q);  // at most a 2x spread
      word |= (unsigned long long)q << (8 * x);
    }
    b->word = word;
    static const int dbg = getenv("VAD_MFCC_BALANCE_DEBUG") ? atoi(getenv("VAD_MFCC_BALANCE_DEBUG")) : 0;
    if (dbg) {
      fprintf(stderr, "balance: word %016llx speeds", word);
      for (int x = 0; x < 8; ++x) fprintf(stderr, " %.4f", sp[x]);
      fprintf(stderr, "\n");
    }
  }
  r.word = b->word;
  r.stats = c % kStatsEvery == 0 ? b->stats_dev : nullptr;
  return r;
}
}  // namespace

struct vad_mfcc_plan {
  MfccDev host;      // host copy (for introspection)
  MfccDev* dev;      // device copy read by the kernels
  int spec;          // 1/2: equals the compile-time Mel26/Mel40 tables bit for bit;
                     // kSpecWindow: an analysis window is set
  int table_spec;    // the compile-time table match without a window
  float* hop_blob;   // stream_hop_kernel's tables, one contiguous block (LDS-staged per launch)
  int hop_blob_n;    // floats (a multiple of 4)
  int n_taps;
  int fft_n;         // 512, or another length run by spec_generic.hip
  int bins;          // fft_n / 2 spectrum bins kept (mfcc.py:61)
  double2* tw_gen;   // exp(-2 pi i m / fft_n), m < fft_n (other lengths only)
  BalanceHost* bal;  // the MFCC kernel's XCD balance (null: equal runs)
  bool generic() const { return fft_n != kFftN; }
};

// n_hops > 1 blocks of n_streams hop rows: disjoint in either ordering
// (hop-major: each block past the previous block's last row; stream-major:
// each row's K hops before the next row), never repeating (block stride > 0)
static bool vad_hop_layout_disjoint(int64_t n_streams, int32_t n_hops, int64_t block_stride, int64_t hop_stride,
                                    int32_t hop_len) {
  if (block_stride <= 0) return false;
  if (block_stride >= (n_streams - 1) * hop_stride + hop_len) return true;
  // stream-major: a stream's K hops apart from each other, then the next stream
  return block_stride >= hop_len && hop_stride >= (int64_t)(n_hops - 1) * block_stride + hop_len;
}

// The spec a launch passes: a windowed plan whose bank is a compiled one
// says which (kSpecWindow26 / 40), so the reference framing keeps the
// generated mel code; vad_mfcc_plan_variant still reports kSpecWindow.
static int launch_spec(const vad_mfcc_plan* p) {
  if (p->spec != kSpecWindow) return p->spec;
  return p->table_spec == 1 ? kSpecWindow26 : p->table_spec == 2 ? kSpecWindow40 : kSpecWindow;
}

// Does the runtime plan equal compile-time table T (taps, ranges, DCT rows)?
template <class T>
static bool matches_table(const MfccDev& h) {
  if (h.n_filters != T::NF || h.mfcc_n != T::NC) return false;
  for (int m = 0; m < T::NF; ++m) {
    if (h.f_lo[m] != T::lo[m] || h.f_len[m] != T::len[m]) return false;
    for (int k = 0; k < kBins; ++k) {
      const bool in = k >= T::lo[m] && k < T::lo[m] + T::len[m];
      const float v = in ? h.taps[h.f_off[m] + k - T::lo[m]] : 0.f;
      if (memcmp(&v, &T::w[m][k], sizeof(float)) != 0) return false;
    }
  }
  for (int c = 0; c < T::NC; ++c)
    for (int m = 0; m < T::NF; ++m)
      if (memcmp(&h.dct[c * kMaxFilters + m], &T::dct[c][m], sizeof(float)) != 0) return false;
  return true;
}

struct vad_ffn_plan {
  FfnDev net;        // by-value kernel argument, frag -> device buffer
  float* frag_dev;
  uint32_t* fragh_dev;  // split-f16 weights (null when the topology has none)
  float* wraw_dev;      // the weights as given (streaming hop kernel)
};

#define VAD_TRY(x)                          \
  do {                                      \
    hipError_t e_ = (x);                    \
    if (e_ != hipSuccess) return (int)e_;   \
  } while (0)

extern "C" {

const char* vad_version(void) { return "vad_amd 0.1 (gfx950)"; }

int64_t vad_n_frames(int64_t n_samples, int32_t frame_size, int32_t hop) {
  if (frame_size <= 0 || hop <= 0 || n_samples <= frame_size) return 0;
  return (n_samples - frame_size - 1) / hop + 1;  // while len - offset > frame_size
}

int vad_mfcc_plan_create(const double* fb, int32_t n_filters, int32_t fft_n, int32_t mfcc_n,
                         int32_t lifter_L, vad_mfcc_plan** out) {
  if (!fb || !out || n_filters <= 0 || mfcc_n <= 0) return VAD_EINVAL;
  if (fft_n < 2 || fft_n > VAD_MAX_FFT_N) return VAD_EUNSUPPORTED;
  if (n_filters > VAD_MAX_FILTERS || mfcc_n > VAD_MAX_MFCC || mfcc_n > n_filters)
    return VAD_EUNSUPPORTED;
  vad_mfcc_plan* p = (vad_mfcc_plan*)calloc(1, sizeof(vad_mfcc_plan));
  if (!p) return VAD_ENOMEM;
  MfccDev& h = p->host;
  h.n_filters = n_filters;
  h.mfcc_n = mfcc_n;
  p->fft_n = fft_n;
  p->bins = fft_n / 2;
  const int bins = p->bins;
  // filterbank rows -> contiguous tap ranges [first non-zero, last non-zero]
  // (NaN counts as non-zero: a degenerate reference filter stays NaN).
  int off = 0;
  std::vector<int> cost(n_filters);
  for (int m = 0; m < n_filters; ++m) {
    const double* row = fb + (size_t)m * bins;
    int lo = -1, hi = -1;
    for (int k = 0; k < bins; ++k)
      if (row[k] != 0.0) { if (lo < 0) lo = k; hi = k; }
    const int n = lo < 0 ? 0 : hi - lo + 1;
    if (off + n > VAD_MAX_TAPS) { free(p); return VAD_EUNSUPPORTED; }
    h.f_lo[m] = lo < 0 ? 0 : lo;
    h.f_len[m] = n;
    h.f_off[m] = off;
    // x 2^-20: the FFT path produces |2X|^2 and P = |X/512|^2 = |2X|^2 2^-20
    // (exact); the direct DFT of other lengths produces P itself
    const float tsc = p->generic() ? 1.f : 0x1p-20f;
    for (int t = 0; t < n; ++t) h.taps[off + t] = (float)row[lo + t] * tsc;
    off += n;
    cost[m] = n + 8;  // taps + (==0 -> eps) + log10, in VALU-op units
  }
  // balance contiguous filter bands over the 8 waves of phase 2
  {
    const int waves = 8;
    long total = 0;
    for (int m = 0; m < n_filters; ++m) total += cost[m];
    int m = 0;
    long acc = 0;
    for (int w = 0; w < 16; ++w) { h.wave_fbeg[w] = n_filters; h.wave_fend[w] = n_filters; }
    for (int w = 0; w < waves; ++w) {
      h.wave_fbeg[w] = m;
      const long target = total * (w + 1) / waves;
      while (m < n_filters && (acc + cost[m] / 2 <= target || w == waves - 1)) acc += cost[m++];
      h.wave_fend[w] = m;
    }
  }
  // lifter (mfcc.py:85-90) x DCT-II ortho (scipy.fftpack, mfcc.py:76), [c][m]
  for (int c = 0; c < kMaxCoefs; ++c) {
    const double lift = lifter_L > 0 ? 1.0 + (lifter_L / 2.0) * sin(M_PI * c / lifter_L) : 1.0;
    const double sc = c == 0 ? sqrt(1.0 / (4.0 * n_filters)) : sqrt(1.0 / (2.0 * n_filters));
    for (int m = 0; m < kMaxFilters; ++m) {
      double v = 0.0;
      if (c < mfcc_n && m < n_filters)
        v = lift * sc * 2.0 * cos(M_PI * c * (2.0 * m + 1.0) / (2.0 * n_filters));
      h.dct[c * kMaxFilters + m] = (float)v;
    }
  }
  for (int n2 = 0; n2 < 16; ++n2)
    for (int k1 = 0; k1 < 16; ++k1) {
      const double a = -2.0 * M_PI * n2 * k1 / 256.0;
      h.tw_a[n2 * 16 + k1] = make_float2((float)cos(a), (float)sin(a));
    }
  for (int k = 0; k < 256; ++k) {
    const double a = -2.0 * M_PI * k / 512.0;
    h.tw_b[k] = make_float2((float)cos(a), (float)sin(a));
  }
  p->spec = p->table_spec = p->generic() ? 0 : matches_table<Mel26>(h) ? 1 : matches_table<Mel40>(h) ? 2 : 0;
  if (p->generic()) {
    std::vector<double2> tw(fft_n);
    for (int m = 0; m < fft_n; ++m) {
      const double a = -2.0 * M_PI * (double)m / (double)fft_n;
      tw[m] = make_double2(cos(a), sin(a));
    }
    hipError_t e = hipMalloc((void**)&p->tw_gen, tw.size() * sizeof(double2));
    if (e == hipSuccess) e = hipMemcpy(p->tw_gen, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(p->tw_gen); free(p); return (int)e; }
  }
  // the streaming hop kernel's tables as one block: W512^k (256 complex);
  // per filter its first bin rounded down to 4, its tap count from there
  // rounded up to 4 and its row offset (as int bits); the 16-B aligned tap
  // rows (the filter's taps at their bins, zero around them: a lane reads
  // four taps and four power bins per pair of 16-B reads, and the zero taps
  // add +0 to a sum of non-negative terms); the DCT rows
  std::vector<float> rows;
  std::vector<int> lo4(n_filters), n4(n_filters), off4(n_filters);
  for (int m = 0; m < n_filters; ++m) {
    const int lo = h.f_lo[m], n = h.f_len[m];
    lo4[m] = lo & ~3;
    n4[m] = n > 0 ? ((lo + n + 3) & ~3) - lo4[m] : 0;
    off4[m] = (int)rows.size();
    for (int t = 0; t < n4[m]; ++t) {
      const int bin = lo4[m] + t;
      rows.push_back(bin >= lo && bin < lo + n ? h.taps[h.f_off[m] + bin - lo] : 0.f);
    }
  }
  p->n_taps = (int)rows.size();  // a multiple of 4
  std::vector<float> blob;
  for (int k = 0; k < 256; ++k) { blob.push_back(h.tw_b[k].x); blob.push_back(h.tw_b[k].y); }
  for (const std::vector<int>* arr : {&lo4, &n4, &off4})
    for (int m = 0; m < n_filters; ++m) { float f; memcpy(&f, &(*arr)[m], 4); blob.push_back(f); }
  while (blob.size() % 4) blob.push_back(0.f);
  blob.insert(blob.end(), rows.begin(), rows.end());
  // the DCT rows (16-B aligned: every tap row is a multiple of 4 floats) at
  // stride vec_row_stride(nf), zero padded
  for (int c = 0; c < mfcc_n; ++c)
    for (int m = 0; m < vec_row_stride(n_filters); ++m)
      blob.push_back(m < n_filters ? h.dct[c * kMaxFilters + m] : 0.f);
  while (blob.size() % 4) blob.push_back(0.f);
  p->hop_blob_n = (int)blob.size();
  hipError_t e = hipMalloc((void**)&p->hop_blob, blob.size() * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(p->hop_blob, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) { (void)hipFree(p->hop_blob); (void)hipFree(p->tw_gen); free(p); return (int)e; }
  e = hipMalloc((void**)&p->dev, sizeof(MfccDev));
  if (e != hipSuccess) { (void)hipFree(p->hop_blob); (void)hipFree(p->tw_gen); free(p); return (int)e; }
  e = hipMemcpy(p->dev, &h, sizeof(MfccDev), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p->dev); (void)hipFree(p->hop_blob); (void)hipFree(p->tw_gen); free(p); return (int)e;
  }
  p->bal = balance_create();
  *out = p;
  return VAD_OK;
}

int vad_mfcc_plan_destroy(vad_mfcc_plan* p) {
  if (!p) return VAD_OK;
  balance_destroy(p->bal);
  (void)hipFree(p->dev);
  (void)hipFree(p->hop_blob);
  (void)hipFree(p->tw_gen);
  free(p);
  return VAD_OK;
}

int32_t vad_mfcc_plan_variant(const vad_mfcc_plan* p) { return p ? p->spec : -1; }

int vad_mfcc_plan_set_window(vad_mfcc_plan* p, const float* window_host, int32_t len) {
  if (!p) return VAD_EINVAL;
  if (p->generic()) return VAD_EUNSUPPORTED;  // the window multiplies the radix-16 kernels' frames
  if (window_host && (len <= 0 || len > kFftN)) return VAD_EINVAL;
  for (int t = 0; t < kFftN; ++t) p->host.window[t] = window_host && t < len ? window_host[t] : 0.f;
  const hipError_t e = hipMemcpy(p->dev->window, p->host.window, sizeof(p->host.window), hipMemcpyHostToDevice);
  if (e != hipSuccess) return (int)e;
  p->spec = window_host ? kSpecWindow : p->table_spec;
  return VAD_OK;
}

int vad_preemphasis_f32(const float* x, float* y, int64_t n_rows, int64_t row_len, int64_t row_stride,
                        float coeff, void* stream) {
  if (n_rows < 0 || row_len < 0 || row_stride < row_len) return VAD_EINVAL;
  if (n_rows == 0 || row_len == 0) return VAD_OK;
  if (!x || !y || x == y) return VAD_EINVAL;
  return (int)launch_preemphasis(x, y, n_rows, row_len, row_stride, coeff, (hipStream_t)stream);
}

int vad_mfcc_plan_set_variant(vad_mfcc_plan* p, int32_t variant) {
  if (!p) return VAD_EINVAL;
  if (p->spec == kSpecWindow) return VAD_EINVAL;  // windowed plans run the runtime-table kernel
  if (variant == 0) { p->spec = 0; return VAD_OK; }
  if (p->generic()) return VAD_EINVAL;
  if (variant == 1 && matches_table<Mel26>(p->host)) { p->spec = 1; return VAD_OK; }
  if (variant == 2 && matches_table<Mel40>(p->host)) { p->spec = 2; return VAD_OK; }
  return VAD_EINVAL;
}

static int check_frames(const vad_mfcc_plan* p, const void* src, int64_t stride, int32_t len,
                        int64_t n, const void* dst) {
  if (!p || n < 0) return VAD_EINVAL;
  if (n == 0) return VAD_OK;
  if (!src || !dst || stride < 0 || len <= 0) return VAD_EINVAL;
  return VAD_OK;
}

int vad_spec_f32(const vad_mfcc_plan* p, const float* src, int64_t stride, int32_t len, int64_t n,
                 float* spec, void* stream) {
  int r = check_frames(p, src, stride, len, n, spec);
  if (r || n == 0) return r;
  if (p->generic()) return (int)launch_generic(1, p->dev, src, stride, len, n, p->fft_n, p->tw_gen, spec,
                                               (hipStream_t)stream);
  return (int)launch_mfcc(1, p->dev, launch_spec(p), src, stride, len, n, spec, (hipStream_t)stream);
}

int vad_mfcc_f32(const vad_mfcc_plan* p, const float* src, int64_t stride, int32_t len, int64_t n,
                 float* mfcc, void* stream) {
  int r = check_frames(p, src, stride, len, n, mfcc);
  if (r || n == 0) return r;
  if (p->generic()) return (int)launch_generic(0, p->dev, src, stride, len, n, p->fft_n, p->tw_gen, mfcc,
                                               (hipStream_t)stream);
  return (int)launch_mfcc(0, p->dev, launch_spec(p), src, stride, len, n, mfcc, (hipStream_t)stream,
                         balance_for_launch(p->bal));
}

int vad_spec_i16(const vad_mfcc_plan* p, const int16_t* src, int64_t stride, int32_t len, int64_t n,
                 float* spec, void* stream) {
  int r = check_frames(p, src, stride, len, n, spec);
  if (r || n == 0) return r;
  if (p->generic()) return (int)launch_generic_i16(1, p->dev, src, stride, len, n, p->fft_n, p->tw_gen, spec,
                                                   (hipStream_t)stream);
  return (int)launch_mfcc_i16(1, p->dev, launch_spec(p), src, stride, len, n, spec, (hipStream_t)stream);
}

int vad_mfcc_i16(const vad_mfcc_plan* p, const int16_t* src, int64_t stride, int32_t len, int64_t n,
                 float* mfcc, void* stream) {
  int r = check_frames(p, src, stride, len, n, mfcc);
  if (r || n == 0) return r;
  if (p->generic()) return (int)launch_generic_i16(0, p->dev, src, stride, len, n, p->fft_n, p->tw_gen, mfcc,
                                                   (hipStream_t)stream);
  return (int)launch_mfcc_i16(0, p->dev, launch_spec(p), src, stride, len, n, mfcc, (hipStream_t)stream,
                             balance_for_launch(p->bal));
}

int vad_mfcc_from_spec_f32(const vad_mfcc_plan* p, const float* spec, int64_t n, float* mfcc,
                           void* stream) {
  if (!p) return VAD_EINVAL;
  int r = check_frames(p, spec, p->bins, p->bins, n, mfcc);
  if (r || n == 0) return r;
  if (p->generic()) return (int)launch_generic(2, p->dev, spec, p->bins, p->bins, n, p->fft_n, p->tw_gen, mfcc,
                                               (hipStream_t)stream);
  return (int)launch_mfcc(2, p->dev, launch_spec(p), spec, kBins, kBins, n, mfcc, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------
// FFN plan
// ---------------------------------------------------------------------------
int vad_ffn_plan_create(int32_t n_layers, const int32_t* dims, const float* const* W,
                        const float* const* b, vad_ffn_plan** out) {
  if (!dims || !W || !b || !out || n_layers < 1) return VAD_EINVAL;
  if (n_layers > VAD_MAX_FFN_LAYERS) return VAD_EUNSUPPORTED;
  for (int l = 0; l <= n_layers; ++l)
    if (dims[l] <= 0) return VAD_EINVAL;
  if (dims[0] > 64 || dims[n_layers] > 4) return VAD_EUNSUPPORTED;
  for (int l = 1; l < n_layers; ++l)
    if (dims[l] > 64) return VAD_EUNSUPPORTED;
  for (int l = 0; l < n_layers; ++l)
    if (!W[l] || !b[l]) return VAD_EINVAL;

  FfnDev net;
  memset(&net, 0, sizeof(net));
  net.n_layers = n_layers;
  for (int l = 0; l <= n_layers; ++l) net.dims[l] = dims[l];
  net.n_classes = dims[n_layers];
  // natural shape; the kernels specialise two topologies, everything else
  // runs on a padded generic shape (ks0 16, 4 tiles per hidden layer)
  int ks0 = (dims[0] + 3) / 4;
  int tiles[VAD_MAX_FFN_LAYERS] = {0, 0, 0, 0};
  for (int l = 0; l < n_layers; ++l) tiles[l] = l + 1 < n_layers ? (dims[l + 1] + 15) / 16 : 1;
  const bool ref39 = n_layers == 4 && ks0 == 10 && tiles[0] == 4 && tiles[1] == 2 &&
                     tiles[2] == 1 && tiles[3] == 1;
  const bool bl13 = n_layers == 3 && ks0 == 4 && tiles[0] == 4 && tiles[1] == 4 && tiles[2] == 1;
  if (!ref39 && !bl13) {
    ks0 = 16;
    for (int l = 0; l < n_layers; ++l) tiles[l] = l + 1 < n_layers ? 4 : 1;
  }
  net.ks0 = ks0;
  for (int l = 0; l < VAD_MAX_FFN_LAYERS; ++l) net.tiles[l] = tiles[l];

  // fragments, in the kernels' slot order
  auto w_at = [&](int l, int k, int o) -> float {  // W_l[k][o] (Keras (in, out))
    if (k >= dims[l] || o >= dims[l + 1]) return 0.f;
    return W[l][(size_t)k * dims[l + 1] + o];
  };
  auto b_at = [&](int l, int o) -> float { return o < dims[l + 1] ? b[l][o] : 0.f; };
  std::vector<float> frag;
  auto push_slot = [&](auto fn) {
    for (int lane = 0; lane < 64; ++lane) frag.push_back(fn(lane >> 4, lane & 15));
  };
  // layer 0 A: slot mt*ks0 + s -> W0[4s + g][16mt + i]
  for (int mt = 0; mt < tiles[0]; ++mt)
    for (int s = 0; s < ks0; ++s)
      push_slot([&](int g, int i) { return w_at(0, 4 * s + g, 16 * mt + i); });
  // layer l >= 1 A: slot (mt*TI + t)*4 + r -> W_l[16t + 4g + r][16mt + i]
  for (int l = 1; l < n_layers; ++l)
    for (int mt = 0; mt < tiles[l]; ++mt)
      for (int t = 0; t < tiles[l - 1]; ++t)
        for (int r = 0; r < 4; ++r)
          push_slot([&](int g, int i) { return w_at(l, 16 * t + 4 * g + r, 16 * mt + i); });
  // biases: layer l, slot mt*4 + r -> b_l[16mt + 4g + r]
  for (int l = 0; l < n_layers; ++l)
    for (int mt = 0; mt < tiles[l]; ++mt)
      for (int r = 0; r < 4; ++r) push_slot([&](int g, int) { return b_at(l, 16 * mt + 4 * g + r); });
  // output layer on the VALU (kernels' Topo::VL: >= 2 input tiles): slot
  // (c*TIL + t)*4 + r -> W_last[16t + 4g + r][c] for 4 classes, then b_last[c]
  if (n_layers >= 2 && tiles[n_layers - 2] >= 2) {
    const int l = n_layers - 1, til = tiles[n_layers - 2];
    for (int c = 0; c < 4; ++c)
      for (int t = 0; t < til; ++t)
        for (int r = 0; r < 4; ++r)
          push_slot([&](int g, int) { return w_at(l, 16 * t + 4 * g + r, c); });
    for (int c = 0; c < 4; ++c) push_slot([&](int, int) { return b_at(l, c); });
  }

  // split-f16 weights for the specialised topologies (ffn_kernel.hip
  // dense_h3): W = hi + lo, both f16 (RNE), per (layer l, tile mt, K-step s)
  // a hi slot and a lo slot of 8 halves per lane.  A[i][k] with row i = lane
  // & 15 -> output unit 16 mt + i and k = 8 (lane >> 4) + q -> input unit
  // 32 s + k at layer 0, else 16 (2 s + (q >> 2)) + 4 (lane >> 4) + (q & 3):
  // the previous layer's accumulator rows as the lane holds them.
  std::vector<uint32_t> fragh;
  const bool use_h3 = ref39 || bl13;
  const bool merge0 = dims[0] <= 16;  // == kMerge0<KS0> of the kernels (bl13)
  if (use_h3) {
    // every layer, output included: the block kernel runs bl13's output
    // layer on the VALU and reads only the hidden layers' slots (the first
    // ones); the wave kernel runs all of them on the MFMA
    for (int l = 0; l < n_layers; ++l) {
      const int ks = l == 0 ? (dims[0] + 31) / 32 : (tiles[l - 1] + 1) / 2;
      for (int mt = 0; mt < tiles[l]; ++mt)
        for (int s = 0; s < ks; ++s)
          for (int part = 0; part < 2; ++part)
            for (int lane = 0; lane < 64; ++lane) {
              const int i = lane & 15, g = lane >> 4;
              _Float16 h[8];
              for (int q = 0; q < 8; ++q) {
                if (l == 0 && merge0) {
                  // <= 16 inputs: one K-step holds both halves of the input,
                  // k = 0..15 its hi halves, 16..31 its lo halves (ffn_dev.h
                  // dense_h3 MERGE0); part 0 = [W_hi | W_hi], part 1 = [W_lo | 0]
                  const int k = 8 * g + q;
                  const float w = w_at(0, k & 15, 16 * mt + i);
                  const _Float16 hi = (_Float16)w;
                  h[q] = part == 0 ? hi : (k < 16 ? (_Float16)(w - (float)hi) : (_Float16)0.f);
                  continue;
                }
                const int k = l == 0 ? 32 * s + 8 * g + q
                                     : 16 * (2 * s + (q >> 2)) + 4 * g + (q & 3);
                const bool in_range = l == 0 || 2 * s + (q >> 2) < tiles[l - 1];
                const float w = in_range ? w_at(l, k, 16 * mt + i) : 0.f;
                const _Float16 hi = (_Float16)w;
                h[q] = part == 0 ? hi : (_Float16)(w - (float)hi);
              }
              uint32_t word[4];
              memcpy(word, h, sizeof(word));
              for (int q = 0; q < 4; ++q) fragh.push_back(word[q]);
            }
    }
  }

  // the streaming forward's weights (FfnDev::wraw): first the weights as
  // given, W_l (in, out) row-major then b_l, with zero rows past the last
  // layer; then each W_l transposed from that flat array, row o holding
  // flat[W_l + k dout + o] for k < din rounded up to 4 -- past din these are
  // the same values (the next rows of the flat array) a four-at-a-time read
  // of the (in, out) layout met, against zero inputs, so the forward's
  // arithmetic is unchanged -- and the biases
  std::vector<float> flat;
  int flat_w[VAD_MAX_FFN_LAYERS], flat_b[VAD_MAX_FFN_LAYERS];
  for (int l = 0; l < n_layers; ++l) {
    flat_w[l] = (int)flat.size();
    flat.insert(flat.end(), W[l], W[l] + (size_t)dims[l] * dims[l + 1]);
    flat_b[l] = (int)flat.size();
    flat.insert(flat.end(), b[l], b[l] + dims[l + 1]);
  }
  flat.insert(flat.end(), 3 * 64 + 4, 0.f);
  std::vector<float> wraw;
  for (int l = 0; l < n_layers; ++l) {
    const int din = dims[l], dout = dims[l + 1], S = vec_row_stride(din);
    net.wstride[l] = S;
    net.woff[l] = (int)wraw.size();
    for (int o = 0; o < dout; ++o)
      for (int k = 0; k < S; ++k)
        wraw.push_back(k < ((din + 3) & ~3) ? flat[flat_w[l] + (size_t)k * dout + o] : 0.f);
    net.boff[l] = (int)wraw.size();
    wraw.insert(wraw.end(), b[l], b[l] + dout);
    while (wraw.size() % 4) wraw.push_back(0.f);
  }
  net.wraw_n = (int)wraw.size();
  // layer-1 inputs of a 13-input network on analyser features (|Mn| <=
  // sqrt(5), ffn_dev.h wave_tile_in_bounded): bounded by max_j |b0_j| +
  // sqrt(5) sum_k |W0[k][j]|; a bound under 32768 leaves 2x headroom to the
  // f16 range for the split-f16 rounding of layer 0 (the check it skips only
  // ever answers "scale 1" then)
  net.h1_bounded = 0;
  if (n_layers >= 2 && dims[0] == 13) {
    double worst = 0.0;
    for (int j = 0; j < dims[1]; ++j) {
      double acc = fabs((double)b[0][j]);
      for (int k = 0; k < dims[0]; ++k) acc += sqrt(5.0) * fabs((double)W[0][(size_t)k * dims[1] + j]);
      worst = acc > worst ? acc : worst;
    }
    net.h1_bounded = worst < 32768.0 ? 1 : 0;
  }

  vad_ffn_plan* p = (vad_ffn_plan*)calloc(1, sizeof(vad_ffn_plan));
  if (!p) return VAD_ENOMEM;
  hipError_t e = hipMalloc((void**)&p->wraw_dev, wraw.size() * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(p->wraw_dev, wraw.data(), wraw.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) { (void)hipFree(p->wraw_dev); free(p); return (int)e; }
  net.wraw = p->wraw_dev;
  e = hipMalloc((void**)&p->frag_dev, frag.size() * sizeof(float));
  if (e != hipSuccess) { free(p); return (int)e; }
  e = hipMemcpy(p->frag_dev, frag.data(), frag.size() * sizeof(float), hipMemcpyHostToDevice);
  if (e != hipSuccess) { (void)hipFree(p->frag_dev); (void)hipFree(p->wraw_dev); free(p); return (int)e; }
  net.frag = p->frag_dev;
  net.fragh = nullptr;
  if (!fragh.empty()) {
    e = hipMalloc((void**)&p->fragh_dev, fragh.size() * sizeof(uint32_t));
    if (e == hipSuccess)
      e = hipMemcpy(p->fragh_dev, fragh.data(), fragh.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(p->fragh_dev);
      (void)hipFree(p->frag_dev);
      (void)hipFree(p->wraw_dev);
      free(p);
      return (int)e;
    }
    net.fragh = p->fragh_dev;
  }
  p->net = net;
  *out = p;
  return VAD_OK;
}

int32_t vad_ffn_plan_arith(const vad_ffn_plan* p) {
  if (!p) return -1;
  return p->net.fragh ? VAD_FFN_SPLIT_F16 : VAD_FFN_EXACT_F32;
}

int vad_ffn_plan_set_arith(vad_ffn_plan* p, int32_t arith) {
  if (!p) return VAD_EINVAL;
  if (arith == VAD_FFN_EXACT_F32) { p->net.fragh = nullptr; return VAD_OK; }
  if (arith == VAD_FFN_SPLIT_F16 && p->fragh_dev) { p->net.fragh = p->fragh_dev; return VAD_OK; }
  return VAD_EINVAL;
}

int vad_ffn_plan_destroy(vad_ffn_plan* p) {
  if (!p) return VAD_OK;
  (void)hipFree(p->frag_dev);
  if (p->fragh_dev) (void)hipFree(p->fragh_dev);
  (void)hipFree(p->wraw_dev);
  free(p);
  return VAD_OK;
}

struct vad_tree_plan {
  TreeNode* nodes_dev;
  TreeNodeC* cnodes_dev;  // compact copy for the LDS-resident window walk
  int n_nodes;
  int n_features;
};

int vad_tree_plan_create(int32_t n_nodes, const int32_t* feature, const double* threshold,
                         const int32_t* left, const int32_t* right, const int32_t* leaf_class,
                         const uint8_t* nan_left, int32_t n_features, vad_tree_plan** out) {
  if (!feature || !threshold || !left || !right || !leaf_class || !out || n_nodes <= 0 ||
      n_features <= 0)
    return VAD_EINVAL;
  if (n_nodes > (1 << 24) || n_features > 3 * VAD_MAX_MFCC + 16) return VAD_EUNSUPPORTED;
  std::vector<TreeNode> h((size_t)n_nodes);
  for (int i = 0; i < n_nodes; ++i) {
    TreeNode& nd = h[i];
    nd.feature = feature[i] >= 0 ? feature[i] : -1;
    nd.threshold = threshold[i];
    nd.left = left[i];
    nd.right = right[i];
    nd.leaf = (short)(leaf_class[i] < 0 || leaf_class[i] > 255 ? -1 : leaf_class[i]);
    nd.nan_left = (short)(nan_left ? (nan_left[i] != 0) : 0);
    if (nd.feature >= 0) {  // internal: children in range, feature in the row
      if (nd.feature >= n_features || nd.left <= 0 || nd.left >= n_nodes || nd.right <= 0 ||
          nd.right >= n_nodes)
        return VAD_EINVAL;
    } else if (nd.leaf < 0) {
      return VAD_EINVAL;
    }
  }
  std::vector<TreeNodeC> c((size_t)n_nodes);
  for (int i = 0; i < n_nodes; ++i) {
    const TreeNode& nd = h[i];
    TreeNodeC& cn = c[i];
    float f = (float)nd.threshold;  // round down to a float: x <= f  <=>  (double)x <= threshold
    if ((double)f > nd.threshold) f = nextafterf(f, -INFINITY);
    cn.thr = f;
    cn.feature = nd.feature >= 0 ? (nd.feature | (nd.nan_left ? 1 << 30 : 0)) : -1 - nd.leaf;
    cn.left = nd.left;
    cn.right = nd.right;
  }
  vad_tree_plan* p = (vad_tree_plan*)calloc(1, sizeof(vad_tree_plan));
  if (!p) return VAD_ENOMEM;
  hipError_t e = hipMalloc((void**)&p->nodes_dev, h.size() * sizeof(TreeNode));
  if (e != hipSuccess) { free(p); return (int)e; }
  e = hipMalloc((void**)&p->cnodes_dev, c.size() * sizeof(TreeNodeC));
  if (e != hipSuccess) { (void)hipFree(p->nodes_dev); free(p); return (int)e; }
  e = hipMemcpy(p->nodes_dev, h.data(), h.size() * sizeof(TreeNode), hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(p->cnodes_dev, c.data(), c.size() * sizeof(TreeNodeC), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p->nodes_dev);
    (void)hipFree(p->cnodes_dev);
    free(p);
    return (int)e;
  }
  p->n_nodes = n_nodes;
  p->n_features = n_features;
  *out = p;
  return VAD_OK;
}

int vad_tree_plan_destroy(vad_tree_plan* p) {
  if (!p) return VAD_OK;
  (void)hipFree(p->nodes_dev);
  (void)hipFree(p->cnodes_dev);
  free(p);
  return VAD_OK;
}

int vad_tree_predict(const vad_tree_plan* t, const float* x, int64_t n, uint8_t* labels,
                     void* stream) {
  if (!t || n < 0) return VAD_EINVAL;
  if (n == 0) return VAD_OK;
  if (!x || !labels) return VAD_EINVAL;
  return (int)launch_tree_rows(t->nodes_dev, t->n_nodes, x, n, t->n_features, labels,
                               (hipStream_t)stream);
}

int vad_features_tree(const vad_tree_plan* t, const float* mfcc, int64_t n_frames, int32_t mfcc_n,
                      int32_t mode, uint8_t* labels, void* stream) {
  if (!t || n_frames < 0 || mfcc_n <= 0 || mfcc_n > VAD_MAX_MFCC || (mode != 0 && mode != 1))
    return VAD_EINVAL;
  if (t->n_features > 3 * mfcc_n) return VAD_EINVAL;
  const int64_t rows = n_frames > 5 ? n_frames - 5 : 0;
  if (rows == 0) return VAD_OK;
  if (!mfcc || !labels) return VAD_EINVAL;
  return (int)launch_tree_windows(t->nodes_dev, t->cnodes_dev, t->n_nodes, mfcc, rows, mfcc_n, mode, labels,
                                  (hipStream_t)stream);
}

int vad_simple_features(const float* frames, int64_t n_frames, int32_t frame_len,
                        int64_t frame_stride, int32_t fft_len, int32_t pad, int32_t band_bins,
                        int32_t n_bands, double* out, void* stream) {
  if (n_frames < 0 || frame_len < 2 || pad < 0 || frame_stride < 0 || band_bins < 1 || n_bands < 0)
    return VAD_EINVAL;
  if (fft_len != frame_len + 2 * pad || frame_len > 8192 || fft_len > 8193 || n_bands * band_bins > fft_len)
    return VAD_EUNSUPPORTED;
  if (n_frames == 0) return VAD_OK;
  if (!frames || !out) return VAD_EINVAL;
  return (int)launch_simple_features(frames, n_frames, frame_len, frame_stride, fft_len, pad,
                                     band_bins, n_bands, out, (hipStream_t)stream);
}

size_t vad_scale_workspace_bytes(void) { return scale_workspace_bytes(); }

int vad_scale_features(float* rows, int64_t n_rows, int32_t mfcc_n, void* workspace,
                       size_t workspace_bytes, void* stream) {
  if (n_rows < 0 || mfcc_n <= 0 || mfcc_n > VAD_MAX_MFCC) return VAD_EINVAL;
  if (n_rows == 0) return VAD_OK;
  if (!rows || !workspace || workspace_bytes < scale_workspace_bytes()) return VAD_EINVAL;
  return (int)launch_scale_features(rows, n_rows, mfcc_n, (double*)workspace, (hipStream_t)stream);
}

int64_t vad_format_csv_rows(const float* rows, int64_t n_rows, int32_t n_cols, double label,
                            char* buf, int64_t buf_size) {
  if (n_rows < 0 || n_cols <= 0 || (n_rows > 0 && !rows)) return VAD_EINVAL;
  if (n_rows == 0) return 0;
  return format_csv_rows(rows, n_rows, n_cols, label, buf, buf_size);
}

int vad_features_f32(const float* mfcc, int64_t n_frames, int32_t mfcc_n, int32_t mode,
                     float* features, void* stream) {
  if (n_frames < 0 || mfcc_n <= 0 || mfcc_n > VAD_MAX_MFCC || (mode != 0 && mode != 1))
    return VAD_EINVAL;
  const int64_t rows = n_frames > 5 ? n_frames - 5 : 0;
  if (rows == 0) return VAD_OK;
  if (!mfcc || !features) return VAD_EINVAL;
  return (int)launch_features(mfcc, rows, mfcc_n, mode, features, (hipStream_t)stream);
}

int vad_features_ffn(const vad_ffn_plan* ffn, const float* mfcc, int64_t n_frames, int32_t mfcc_n,
                     int32_t mode, uint8_t* labels, void* stream) {
  if (!ffn || n_frames < 0 || mfcc_n <= 0 || mfcc_n > VAD_MAX_MFCC || (mode != 0 && mode != 1))
    return VAD_EINVAL;
  if (ffn->net.dims[0] > 3 * mfcc_n) return VAD_EINVAL;
  const int64_t rows = n_frames > 5 ? n_frames - 5 : 0;
  if (rows == 0) return VAD_OK;
  if (!mfcc || !labels) return VAD_EINVAL;
  return (int)launch_ffn(ffn->net, 0, mfcc, rows, mfcc_n, mode, labels, (hipStream_t)stream);
}

int vad_features_ffn_logits(const vad_ffn_plan* ffn, const float* mfcc, int64_t n_frames, int32_t mfcc_n,
                            int32_t mode, uint8_t* labels, float* logits, void* stream) {
  if (!ffn || n_frames < 0 || mfcc_n <= 0 || mfcc_n > VAD_MAX_MFCC || (mode != 0 && mode != 1))
    return VAD_EINVAL;
  if (ffn->net.dims[0] > 3 * mfcc_n) return VAD_EINVAL;
  const int64_t rows = n_frames > 5 ? n_frames - 5 : 0;
  if (rows == 0) return VAD_OK;
  if (!mfcc || !labels || !logits) return VAD_EINVAL;
  FfnDev net = ffn->net;
  net.logits = logits;
  return (int)launch_ffn(net, 0, mfcc, rows, mfcc_n, mode, labels, (hipStream_t)stream);
}

int vad_ffn_predict(const vad_ffn_plan* ffn, const float* x, int64_t n, uint8_t* labels,
                    void* stream) {
  if (!ffn || n < 0) return VAD_EINVAL;
  if (n == 0) return VAD_OK;
  if (!x || !labels) return VAD_EINVAL;
  return (int)launch_ffn(ffn->net, 1, x, n, 0, 0, labels, (hipStream_t)stream);
}

size_t vad_mfcc_ffn_workspace_bytes(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, int64_t n_samples,
                                    int32_t frame_size, int32_t hop) {
  if (!plan || !ffn) return 0;
  const int64_t f = vad_n_frames(n_samples, frame_size, hop);
  return (size_t)f * plan->host.mfcc_n * sizeof(float);
}

int32_t vad_mfcc_ffn_fusable(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, int32_t frame_size, int32_t hop) {
  if (!plan || !ffn) return 0;
  return mfcc_ffn_fusable(plan->spec, ffn->net, frame_size, hop, nullptr, 4) ? 1 : 0;
}

// Shared body of vad_mfcc_ffn / vad_mfcc_ffn_i16: with a workspace, the MFCC
// kernel writes the rows there and the window kernel classifies them (the
// faster form on gfx950); without one, the fused kernel keeps
// them on chip.
static int mfcc_ffn_entry(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, const void* audio, int tin_bytes,
                          int64_t n_samples, int32_t frame_size, int32_t hop, int32_t mode, uint8_t* labels,
                          void* workspace, size_t workspace_bytes, void* stream) {
  if (!plan || !ffn || n_samples < 0 || frame_size <= 0 || hop <= 0 || (mode != 0 && mode != 1))
    return VAD_EINVAL;
  const int64_t f = vad_n_frames(n_samples, frame_size, hop);
  if (f <= 5) return VAD_OK;
  if (!audio || !labels) return VAD_EINVAL;
  if (ffn->net.dims[0] > 3 * plan->host.mfcc_n) return VAD_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (!workspace) {
    if (plan->generic()) return VAD_EUNSUPPORTED;  // the fused kernel is the fft_n = 512 pipeline
    if (!mfcc_ffn_fusable(plan->spec, ffn->net, frame_size, hop, audio, tin_bytes)) return VAD_EINVAL;
    return (int)launch_mfcc_ffn(plan->dev, ffn->net, audio, tin_bytes, f, mode, labels, st);
  }
  const size_t need = (size_t)f * plan->host.mfcc_n * sizeof(float);
  if (workspace_bytes < need) return VAD_EINVAL;
  float* mf = (float*)workspace;
  if (plan->generic() && tin_bytes == 2)
    VAD_TRY(launch_generic_i16(0, plan->dev, (const int16_t*)audio, hop, frame_size, f, plan->fft_n, plan->tw_gen,
                               mf, st));
  else if (plan->generic())
    VAD_TRY(launch_generic(0, plan->dev, (const float*)audio, hop, frame_size, f, plan->fft_n, plan->tw_gen, mf,
                           st));
  else if (tin_bytes == 2)
    VAD_TRY(launch_mfcc_i16(0, plan->dev, launch_spec(plan), (const int16_t*)audio, hop, frame_size, f, mf, st,
                            balance_for_launch(plan->bal)));
  else
    VAD_TRY(launch_mfcc(0, plan->dev, launch_spec(plan), (const float*)audio, hop, frame_size, f, mf, st,
                        balance_for_launch(plan->bal)));
  return (int)launch_ffn(ffn->net, 0, mf, f - 5, plan->host.mfcc_n, mode, labels, st);
}

int vad_mfcc_ffn(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, const float* audio,
                 int64_t n_samples, int32_t frame_size, int32_t hop, int32_t mode,
                 uint8_t* labels, void* workspace, size_t workspace_bytes, void* stream) {
  return mfcc_ffn_entry(plan, ffn, audio, 4, n_samples, frame_size, hop, mode, labels, workspace,
                        workspace_bytes, stream);
}

int vad_mfcc_ffn_i16(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, const int16_t* audio,
                     int64_t n_samples, int32_t frame_size, int32_t hop, int32_t mode,
                     uint8_t* labels, void* workspace, size_t workspace_bytes, void* stream) {
  return mfcc_ffn_entry(plan, ffn, audio, 2, n_samples, frame_size, hop, mode, labels, workspace,
                        workspace_bytes, stream);
}

int64_t vad_stream_ring_floats(int64_t n_streams, int32_t mfcc_n) {
  return n_streams * 5 * (int64_t)mfcc_n;
}

int vad_stream_push_hop(float* frames, int64_t frame_stride, int32_t frame_len, const float* hop,
                        int64_t hop_stride, int32_t hop_len, int64_t n_streams, void* stream) {
  if (n_streams < 0 || frame_len <= 0 || frame_len > 1024 || hop_len <= 0 || hop_len > frame_len ||
      frame_stride < frame_len || hop_stride < hop_len)
    return VAD_EINVAL;
  if (n_streams == 0) return VAD_OK;
  if (!frames || !hop) return VAD_EINVAL;
  return (int)launch_stream_push(frames, frame_stride, frame_len, hop, hop_stride, hop_len, n_streams,
                                 (hipStream_t)stream);
}

int vad_stream_hops(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, float* frames, int64_t frame_stride,
                    int32_t frame_len, const float* hop, int64_t hop_stride, int32_t hop_len, int64_t n_streams,
                    int32_t n_hops, int64_t hop_block_stride, float* ring, int32_t* count, uint8_t* labels,
                    int64_t label_block_stride, void* stream) {
  if (!plan || !ffn || n_streams < 0 || n_hops < 0 || frame_len <= 0 || frame_len > 1024 || hop_len <= 0 ||
      hop_len > frame_len || frame_stride < frame_len || hop_stride < hop_len)
    return VAD_EINVAL;
  if (n_hops > 1 && label_block_stride < n_streams) return VAD_EINVAL;  // label rows of two hops would overlap
  // hop k's block must not be hop k-1's (a zero or negative stride would
  // replay, or walk backwards over, the new samples), and no two (hop,
  // stream) rows may overlap: either ordering of a disjoint layout is fine,
  // hop-major (blocks of S rows) or stream-major ((S, K*hop) viewed as
  // (K, S, hop): block stride hop, row stride K*hop)
  if (n_hops > 1 && !vad_hop_layout_disjoint(n_streams, n_hops, hop_block_stride, hop_stride, hop_len))
    return VAD_EINVAL;
  if (n_streams == 0 || n_hops == 0) return VAD_OK;
  if (!frames || !hop || !ring || !count || !labels) return VAD_EINVAL;
  if (ffn->net.dims[0] > 3 * plan->host.mfcc_n) return VAD_EINVAL;
  if (plan->generic()) return VAD_EUNSUPPORTED;  // its FFT is the 256-point Stockham of fft_n = 512
  if (plan->spec == kSpecWindow) return VAD_EUNSUPPORTED;  // its table blob carries no analysis window
  return (int)launch_stream_hop(plan->dev, plan->hop_blob, plan->hop_blob_n, plan->host.n_filters, plan->n_taps,
                                ffn->net, frames, frame_stride, frame_len, hop, hop_stride, hop_len,
                                n_streams, plan->host.mfcc_n, ring, count, labels, n_hops, hop_block_stride,
                                label_block_stride, (hipStream_t)stream);
}

int vad_stream_hop(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, float* frames, int64_t frame_stride,
                   int32_t frame_len, const float* hop, int64_t hop_stride, int32_t hop_len, int64_t n_streams,
                   float* ring, int32_t* count, uint8_t* labels, void* stream) {
  return vad_stream_hops(plan, ffn, frames, frame_stride, frame_len, hop, hop_stride, hop_len, n_streams, 1, 0,
                         ring, count, labels, 0, stream);
}

int vad_stream_step(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, const float* frames,
                    int64_t frame_stride, int32_t frame_len, int64_t n_streams, float* ring,
                    int32_t* count, uint8_t* labels, float* mfcc_scratch, void* stream) {
  if (!plan || !ffn || n_streams < 0 || frame_len <= 0 || frame_stride < 0) return VAD_EINVAL;
  if (n_streams == 0) return VAD_OK;
  if (!frames || !ring || !count || !labels || !mfcc_scratch) return VAD_EINVAL;
  if (ffn->net.dims[0] > 3 * plan->host.mfcc_n) return VAD_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  if (plan->generic())
    VAD_TRY(launch_generic(0, plan->dev, frames, frame_stride, frame_len, n_streams, plan->fft_n, plan->tw_gen,
                           mfcc_scratch, st));
  else
    VAD_TRY(launch_mfcc(0, plan->dev, launch_spec(plan), frames, frame_stride, frame_len, n_streams, mfcc_scratch, st));
  return (int)launch_stream_ffn(ffn->net, mfcc_scratch, ring, count, n_streams, plan->host.mfcc_n,
                                labels, st);
}

// Replay of a captured graph (a hop block with its host copies,
// vad_amd.stream.StreamBatch.capture): hipGraphLaunch on the caller's stream.
int vad_graph_launch(void* graph_exec, void* stream) {
  if (!graph_exec) return VAD_EINVAL;
  return (int)hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream);
}

// A captured step prepared for replay.  A graph of exactly one kernel node
// (the one-hop step of StreamBatch, kernel="hop") is dispatched as that
// node: its captured function, grid, block, dynamic LDS and argument values
// (kernelParams point into the graph's own copy, so the graph must outlive
// the plan) go to hipLaunchKernel -- on ROCm 7.2 a hipGraphLaunch of one
// kernel node costs ~5 us more host time per call than the launch it wraps
// (profiles/r06/c5_graph/), so back-to-back one-hop replays were host-bound
// at ~15 us against ~10 us launched directly.  Any other graph replays
// through hipGraphLaunch.
struct vad_graph_plan {
  hipGraphExec_t exec;
  int32_t n_nodes;
  bool direct;
  hipKernelNodeParams kp;
};

int vad_graph_plan_create(void* graph, void* graph_exec, vad_graph_plan** out) {
  if (!graph || !graph_exec || !out) return VAD_EINVAL;
  *out = nullptr;
  size_t n = 0;
  hipError_t e = hipGraphGetNodes((hipGraph_t)graph, nullptr, &n);
  if (e != hipSuccess) return (int)e;
  vad_graph_plan* p = (vad_graph_plan*)calloc(1, sizeof(vad_graph_plan));
  if (!p) return VAD_ENOMEM;
  p->exec = (hipGraphExec_t)graph_exec;
  p->n_nodes = (int32_t)n;
  p->direct = false;
  if (n == 1) {
    hipGraphNode_t node;
    size_t one = 1;
    hipGraphNodeType ty;
    if (hipGraphGetNodes((hipGraph_t)graph, &node, &one) == hipSuccess && one == 1 &&
        hipGraphNodeGetType(node, &ty) == hipSuccess && ty == hipGraphNodeTypeKernel &&
        hipGraphKernelNodeGetParams(node, &p->kp) == hipSuccess && p->kp.func && p->kp.kernelParams &&
        !p->kp.extra)
      p->direct = true;
  }
  *out = p;
  return VAD_OK;
}

int vad_graph_plan_launch(const vad_graph_plan* p, void* stream) {
  if (!p) return VAD_EINVAL;
  if (p->direct)
    return (int)hipLaunchKernel(p->kp.func, p->kp.gridDim, p->kp.blockDim, p->kp.kernelParams,
                                p->kp.sharedMemBytes, (hipStream_t)stream);
  return (int)hipGraphLaunch(p->exec, (hipStream_t)stream);
}

int32_t vad_graph_plan_direct(const vad_graph_plan* p) { return p && p->direct ? 1 : 0; }

int vad_graph_plan_destroy(vad_graph_plan* p) {
  free(p);
  return VAD_OK;
}

}  // extern "C"
