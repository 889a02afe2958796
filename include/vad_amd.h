/*
 * vad_amd.h -- C ABI of libvad_amd.so, the MI355X-native MFCC + FFN VAD path.
 *
 * The reference (nameofuser1/vad) is pure Python with no FFI, so there is no
 * existing binding to match byte for byte; each entry point below names the
 * reference function whose semantics it implements (file:line in the
 * reference tree) and the Python host layer (vad_amd/, ctypes) that mirrors
 * the reference API on top of it.
 *
 * Conventions
 *   - All data pointers are DEVICE pointers owned by the caller (torch tensors
 *     on the host side).  Plans own small device buffers of their own.
 *   - `stream` is a hipStream_t passed as void* (0 = the null stream).
 *   - No allocation, no host synchronisation on any hot call: every hot call
 *     is capturable into a hipGraph.
 *   - Return value: 0 on success, a negative VAD_E* code for argument
 *     errors, or a positive hipError_t from the HIP runtime.
 */
#ifndef VAD_AMD_H
#define VAD_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VAD_MAX_FILTERS 64
#define VAD_MAX_MFCC 16
#define VAD_MAX_TAPS 16384
#define VAD_FFT_N 512
#define VAD_MAX_FFT_N 8192  /* other fft_n (2..8192) run a direct-DFT path */
#define VAD_MAX_FFN_LAYERS 4

#define VAD_OK 0
#define VAD_EINVAL (-1)        /* bad argument (null, negative size, ...) */
#define VAD_EUNSUPPORTED (-2)  /* valid for the reference, not built here (see each entry) */
#define VAD_ENOMEM (-3)
#define VAD_ERCCL (-4)         /* RCCL returned an error: vad_rccl_error_string() */

typedef struct vad_mfcc_plan vad_mfcc_plan;
typedef struct vad_ffn_plan vad_ffn_plan;

/* Library version string. */
const char* vad_version(void);

/* Number of frames split_into_frames() yields: frames are taken while
 * len - offset > frame_size (reference dataset/file_processing.py:99). */
int64_t vad_n_frames(int64_t n_samples, int32_t frame_size, int32_t hop);

/* ---------------------------------------------------------------------------
 * MFCC plan.  Replaces the per-call arguments of mfcc.get_mfcc /
 * get_mfcc_from_spec (reference mfcc.py:67-78): the (n_filters, 256)
 * filterbank from get_mel_filterbanks (mfcc.py:39-56, built on the host in
 * fp64 exactly as the reference does), the MFCC count (mfcc.py:76 [:mfcc_n])
 * and the lifter length (mfcc.py:85, L=22 in every reference call).
 * fft_n: any length 2..VAD_MAX_FFT_N, as np.fft.fft(frame, fft_n) takes
 * (mfcc.py:61; the filterbank is then (n_filters, fft_n / 2)).  512, the
 * reference's only value (config.py:27, sklearn_analyser.py:21), runs the
 * radix-16 x 16 kernels; other lengths a direct DFT with fp64 accumulation
 * (vad_mfcc_f32 / _i16, vad_spec_*, vad_mfcc_from_spec_f32, the workspace
 * form of vad_mfcc_ffn and vad_stream_step; the fused clip kernel, the
 * analysis window and vad_stream_hop return VAD_EUNSUPPORTED for them).
 * ------------------------------------------------------------------------- */
int vad_mfcc_plan_create(const double* filterbank_host, int32_t n_filters, int32_t fft_n,
                         int32_t mfcc_n, int32_t lifter_L, vad_mfcc_plan** out);
/* destroy: frees the plan's device tables with hipFree, which waits for the
 * device, so launches still queued with the plan complete first (a plan
 * captured in a hipGraph must outlive the graph's replays). */
int vad_mfcc_plan_destroy(vad_mfcc_plan* plan);

/* Kernel variant a plan dispatches to: 0 = runtime filterbank tables,
 * 1 / 2 = the compile-time tables of the reference's 26 / 40-filter banks
 * (selected only when the plan equals them bit for bit).  set_variant(0)
 * forces the runtime path (tests compare the two). */
int32_t vad_mfcc_plan_variant(const vad_mfcc_plan* plan);
int vad_mfcc_plan_set_variant(vad_mfcc_plan* plan, int32_t variant);

/* Optional stages NOT in the reference (mfcc.py:59-61 feeds the raw frame to
 * the FFT: rectangular window, no pre-emphasis; BASELINE's north_star names
 * both).  Default off; with both off every output is bit-identical to a plan
 * that never had them.  Parity for them is pinned to the oracle's
 * restatement only (python_speech_features conventions).
 *   set_window: multiply sample t of every frame by window_host[t] (t < len
 *     <= 512, e.g. numpy.hamming(400)) before the FFT; NULL removes it.
 *     Windowed plans run the runtime-table kernel (variant kSpecWindow = 3).
 *   vad_preemphasis_f32: y[r][0] = x[r][0], y[r][t] = x[r][t] - coeff
 *     x[r][t-1] for each of n_rows rows of row_len samples (a clip: one row),
 *     out of place -- run before framing. */
int vad_mfcc_plan_set_window(vad_mfcc_plan* plan, const float* window_host, int32_t len);
int vad_preemphasis_f32(const float* x, float* y, int64_t n_rows, int64_t row_len, int64_t row_stride,
                        float coeff, void* stream);

/* Frames f = 0..n_frames-1 start at src + f*frame_stride and hold frame_len
 * samples (fp32); only the first min(frame_len, 512) feed the 512-point FFT
 * (np.fft.fft(x, 512) zero-pads / truncates, mfcc.py:61).
 * A clip framed at hop H is frame_stride = H, frame_len = 400
 * (file_processing.py:80-103); a frame matrix is frame_stride = row length. */

/* get_spec_mag (mfcc.py:59-61) of every frame -> spec[f*256 + k], fp32. */
int vad_spec_f32(const vad_mfcc_plan* plan, const float* src, int64_t frame_stride,
                 int32_t frame_len, int64_t n_frames, float* spec, void* stream);

/* get_mfcc (mfcc.py:67-69) of every frame -> mfcc[f*mfcc_n + c], fp32. */
int vad_mfcc_f32(const vad_mfcc_plan* plan, const float* src, int64_t frame_stride,
                 int32_t frame_len, int64_t n_frames, float* mfcc, void* stream);

/* int16 PCM input: the same as vad_spec_f32 / vad_mfcc_f32 on the samples
 * converted to fp32 (exact), i.e. the reference's int16 wav data followed by
 * astype(float32) (vad.py:37, dataset/file_processing.py:26-35), at half the
 * input bytes.  Frames are src + f*frame_stride (in samples). */
int vad_spec_i16(const vad_mfcc_plan* plan, const int16_t* src, int64_t frame_stride,
                 int32_t frame_len, int64_t n_frames, float* spec, void* stream);
int vad_mfcc_i16(const vad_mfcc_plan* plan, const int16_t* src, int64_t frame_stride,
                 int32_t frame_len, int64_t n_frames, float* mfcc, void* stream);

/* get_mfcc_from_spec (mfcc.py:72-78) of n spectra spec[f*256 + k]. */
int vad_mfcc_from_spec_f32(const vad_mfcc_plan* plan, const float* spec, int64_t n,
                           float* mfcc, void* stream);

/* ---------------------------------------------------------------------------
 * FFN plan: a Keras Sequential of Dense layers with ReLU between them and a
 * softmax at the end, predicted class = argmax (reference
 * learning/ffn_trainer.py:106-116; config.py:45-47 labels).  Weights are
 * Keras-layout W (in, out) row-major fp32 and b (out).  Constraints of this
 * build: 1..4 layers, in_dim <= 64, hidden <= 64, classes <= 4.
 * ------------------------------------------------------------------------- */
int vad_ffn_plan_create(int32_t n_layers, const int32_t* dims /* n_layers+1 */,
                        const float* const* W_host, const float* const* b_host,
                        vad_ffn_plan** out);
int vad_ffn_plan_destroy(vad_ffn_plan* plan);

/* Arithmetic of the forward.  VAD_FFN_SPLIT_F16 (the default of the two
 * specialised topologies 39-64-32-16-3 and 13-64-64-N): every GEMM operand
 * split v = hi + lo into two f16 halves, lo*hi + hi*lo + hi*hi accumulated in
 * f32 on v_mfma_f32_16x16x32_f16 (~22-bit operands, logits within a few f32
 * ulps of an exact-f32 forward; tests/test_gpu_fullsize.py bounds it).
 * VAD_FFN_EXACT_F32: v_mfma_f32_16x16x4_f32 (exact f32 products; every other
 * topology always runs this).  set_arith returns VAD_EINVAL for split-f16 on
 * a topology without it. */
#define VAD_FFN_EXACT_F32 0
#define VAD_FFN_SPLIT_F16 1
int32_t vad_ffn_plan_arith(const vad_ffn_plan* plan);
int vad_ffn_plan_set_arith(vad_ffn_plan* plan, int32_t arith);

/* Feature rows (reference feature layout, 39 = 3 x 13):
 *   mode VAD_FEAT_ANALYSER: [Mn, M+1 - M-1, (M+2 - Mn) - (Mn - M-2)] with the
 *     centre MFCC normalised by the 5-frame mean / std (ddof 0)
 *     (realtime_analysis/sklearn_analyser.py:52-69,103-107);
 *   mode VAD_FEAT_OFFLINE: [Mc, M+1 - M-1, (M+2 - Mc) - (Mc - M-2)], no
 *     normalisation (dataset/file_processing.py:40-70).
 * Row i is centred on MFCC frame i+2, i = 0..n_frames-6 (F-5 rows; the last
 * full window is never emitted, exactly as both reference loops do).
 * Supported range (analyser mode): the normalisation is fp32, v_rsq_f32 on
 * 0.2 * var * 2^24.  For caller-supplied rows whose 5-frame std lies in
 * [2^-60, 2^50] Mn is the fp32 formula's (log-MFCCs of any audio are far
 * inside); past ~2^52 the scaled variance overflows and Mn = 0, below ~2^-75
 * the squares underflow and Mn = +-inf, where the reference's fp64 gives a
 * finite value (tests/test_gpu_parity.py::test_feature_range_edges). */
#define VAD_FEAT_ANALYSER 0
#define VAD_FEAT_OFFLINE 1

/* features[i*3*mfcc_n + j] (fp32), i < n_frames-5. */
int vad_features_f32(const float* mfcc, int64_t n_frames, int32_t mfcc_n, int32_t mode,
                     float* features, void* stream);

/* Labels of every analyser window: classifier.predict of the features above
 * (sklearn_analyser.py:71) -> labels[i] (uint8), i < n_frames-5. */
int vad_features_ffn(const vad_ffn_plan* ffn, const float* mfcc, int64_t n_frames,
                     int32_t mfcc_n, int32_t mode, uint8_t* labels, void* stream);

/* The same labels plus every window's fp32 logits, logits[i*n_classes + c]
 * (before the softmax; parity tests of the FFN arithmetic). */
int vad_features_ffn_logits(const vad_ffn_plan* ffn, const float* mfcc, int64_t n_frames,
                            int32_t mfcc_n, int32_t mode, uint8_t* labels, float* logits, void* stream);

/* FFN forward over caller-built feature rows x[i*in_dim + j] (predict on a
 * batch, ffn_trainer.py:106-116) -> labels[i]. */
int vad_ffn_predict(const vad_ffn_plan* ffn, const float* x, int64_t n, uint8_t* labels,
                    void* stream);

/* Clip path: framing + MFCC + features + FFN (dataset_creator/process_file
 * framing, file_processing.py:38-70, with the analyser's classifier call,
 * sklearn_analyser.py:71).  labels[i] for windows i < n_frames-5 of the clip.
 * Two forms, identical labels:
 *   workspace != NULL (>= vad_mfcc_ffn_workspace_bytes(): the clip's MFCC
 *     rows): the MFCC kernel, then the window kernel -- the faster form on
 *     gfx950;
 *   workspace == NULL: one fused kernel, the MFCC rows never leave the CU --
 *     for the reference framing (frame 400, hop 160), the compiled 26-filter
 *     bank, a split-f16 FFN topology (39-64-32-16-3 or 13-64-64-N) and
 *     pair-aligned audio (8 B fp32 / 4 B int16: every torch allocation is);
 *     VAD_EINVAL otherwise.  vad_mfcc_ffn_fusable() tells whether the plans
 *     and framing qualify. */
size_t vad_mfcc_ffn_workspace_bytes(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, int64_t n_samples,
                                    int32_t frame_size, int32_t hop);
int32_t vad_mfcc_ffn_fusable(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, int32_t frame_size,
                             int32_t hop);
int vad_mfcc_ffn(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, const float* audio,
                 int64_t n_samples, int32_t frame_size, int32_t hop, int32_t mode,
                 uint8_t* labels, void* workspace, size_t workspace_bytes, void* stream);
/* The same from int16 PCM (the wav samples vad.py:37 converts with
 * astype(float32); the conversion is exact, so the labels are identical). */
int vad_mfcc_ffn_i16(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, const int16_t* audio,
                     int64_t n_samples, int32_t frame_size, int32_t hop, int32_t mode,
                     uint8_t* labels, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Decision-tree plan: the classifier vad.py deploys
 * (learning/decision_classifier_trainer.py:26-35: sklearn
 * DecisionTreeClassifier, predict through sklearn_analyser.py:71) as a flat
 * node table, e.g. from an sklearn tree_: feature[i] (< 0 for a leaf),
 * threshold[i] (float64), left[i] / right[i] (children_left / _right),
 * leaf_class[i] = argmax of the leaf's value row (class index), and nan_left[i]
 * (missing_go_to_left, sklearn >= 1.3; NULL: NaN goes right).  Traversal is
 * sklearn's: left iff float32(x[feature]) <= threshold (compared in double).
 * Returned labels are class indices (uint8); the caller maps them through
 * classes_.  Constraints: 1 <= n_nodes <= 2^24, feature < n_features <= 64.
 * ------------------------------------------------------------------------- */
typedef struct vad_tree_plan vad_tree_plan;

int vad_tree_plan_create(int32_t n_nodes, const int32_t* feature, const double* threshold,
                         const int32_t* left, const int32_t* right, const int32_t* leaf_class,
                         const uint8_t* nan_left, int32_t n_features, vad_tree_plan** out);
int vad_tree_plan_destroy(vad_tree_plan* plan);

/* labels[i] of caller-built feature rows x[i*n_features + f] (fp32). */
int vad_tree_predict(const vad_tree_plan* tree, const float* x, int64_t n, uint8_t* labels,
                     void* stream);

/* Labels of every window of an MFCC sequence (features as vad_features_f32,
 * mode VAD_FEAT_ANALYSER or VAD_FEAT_OFFLINE), labels[i], i < n_frames-5. */
int vad_features_tree(const vad_tree_plan* tree, const float* mfcc, int64_t n_frames,
                      int32_t mfcc_n, int32_t mode, uint8_t* labels, void* stream);

/* ---------------------------------------------------------------------------
 * Offline dataset export (dataset_creator.py:58-66 -> file_processing.py,
 * dataset/utils.py).
 * ------------------------------------------------------------------------- */

/* scale_features (dataset/utils.py:5-34) of feature rows
 * rows[i*3*mfcc_n + t*mfcc_n + c] (t: mfcc / delta1 / delta2, the OFFLINE
 * layout), in place on the device: one global mean and population std per
 * group t over all rows, x = (x - mean_t) / std_t; statistics in fp64.
 * `workspace` (device, >= vad_scale_workspace_bytes()) ends with the six
 * doubles mean[3], std[3]. */
size_t vad_scale_workspace_bytes(void);
int vad_scale_features(float* rows, int64_t n_rows, int32_t mfcc_n, void* workspace,
                       size_t workspace_bytes, void* stream);

/* CSV text of host feature rows as write_features writes them
 * (file_processing.py:126-146: features, then the label; values printed like
 * numpy float32, rows ending in "\r\n").  Returns the bytes written, or
 * -(bytes needed) when buf is NULL or too small. */
int64_t vad_format_csv_rows(const float* rows, int64_t n_rows, int32_t n_cols, double label,
                            char* buf, int64_t buf_size);

/* ---------------------------------------------------------------------------
 * Energy / ZCR / spectral analyser (realtime_analysis/simple_analyzer.py,
 * SimpleAnalyser): per-frame features in fp64, out[f*(3+n_bands) + i]:
 *   0  stEnergy(frame)                    = sum x^2 / frame_len
 *   1  stZCR(frame) * frame_len           (:210-215)
 *   2  np.std(|fft|) over all fft_len bins (:203-208)
 *   3+b stEnergy(|fft|[b*band_bins : (b+1)*band_bins])   (:171-197)
 * |fft| = |DFT_fft_len([zeros(pad), frame, zeros(pad)])| with
 * fft_len = frame_len + 2*pad (:386-400; pad 0: the frame itself): frames of
 * up to 8192 samples, fft_len up to 8193 (a power of two runs a radix-2 FFT,
 * any other length -- the reference's odd pads -- a direct DFT).
 * stEnergy / stZCR are pyAudioAnalysis's (restated; the package is absent).
 * Frames are frames + f*frame_stride (fp32 samples, exact for int16 audio).
 * ------------------------------------------------------------------------- */
int vad_simple_features(const float* frames, int64_t n_frames, int32_t frame_len,
                        int64_t frame_stride, int32_t fft_len, int32_t pad, int32_t band_bins,
                        int32_t n_bands, double* out, void* stream);

/* ---------------------------------------------------------------------------
 * Streaming: S independent analyser streams advanced by one frame each
 * (SKLearnAnalyzer.feed_frame, sklearn_analyser.py:46-82, for S streams at
 * once).  State lives in device buffers the caller allocates with the sizes
 * below; every stream's state is independent.
 *   frames[s*frame_stride + t], t < frame_len: the new frame of stream s.
 *   ring: (S, 5, mfcc_n) fp32 MFCC ring; count: (S,) int32 frames seen.
 * After the call, labels[s] = class of the window centred 3 calls ago, or
 * 255 while the stream has seen fewer than 5 frames before this one
 * (feed_frame returns None for its first 5 calls, :48-50).
 * ------------------------------------------------------------------------- */
int64_t vad_stream_ring_floats(int64_t n_streams, int32_t mfcc_n);
/* Advance every stream's frame buffer by one hop, in place:
 *   frames[s, 0 : L-H] <- frames[s, H : L];  frames[s, L-H : L] <- hop[s, 0 : H]
 * (L = frame_len <= 1024, H = hop_len, 0 < H <= L), i.e. the next frame the
 * live loop of vad.py:37-49 hands to feed_frame.  One kernel; capturable. */
int vad_stream_push_hop(float* frames, int64_t frame_stride, int32_t frame_len, const float* hop,
                        int64_t hop_stride, int32_t hop_len, int64_t n_streams, void* stream);
/* One hop of every stream in ONE kernel (one wave per stream): advance the
 * frame buffer by the hop (as vad_stream_push_hop), 512-point FFT of the new
 * frame, mel / log10 / lifter x DCT, classify the ring's window, push the
 * new MFCC row (as vad_stream_step) -- the FFN forward in exact f32 on the
 * VALU, one output unit per lane.  The hipGraph-free, latency-first form of
 * push_hop + step for many small batches (BASELINE config 5). */
int vad_stream_hop(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, float* frames, int64_t frame_stride,
                   int32_t frame_len, const float* hop, int64_t hop_stride, int32_t hop_len, int64_t n_streams,
                   float* ring, int32_t* count, uint8_t* labels, void* stream);
/* n_hops consecutive hops of every stream in ONE kernel: exactly n_hops calls
 * of vad_stream_hop, hop k's new samples at hop + k * hop_block_stride (row s
 * at + s * hop_stride), its labels at labels + k * label_block_stride.  The
 * plan tables are staged into LDS once per launch instead of once per hop;
 * the form a hipGraph captures for many hops per replay (n_hops = 1 is
 * vad_stream_hop).  Same refusals as vad_stream_hop, plus VAD_EINVAL for
 * n_hops < 0, or n_hops > 1 with label_block_stride < n_streams, or with
 * hop rows that repeat or overlap: hop_block_stride must be > 0 and the rows
 * disjoint in one of the two orderings, hop-major (hop_block_stride >=
 * (n_streams - 1) * hop_stride + hop_len) or stream-major (hop_block_stride
 * >= hop_len and hop_stride >= (n_hops - 1) * hop_block_stride + hop_len,
 * e.g. an (S, K * hop) buffer viewed as (K, S, hop)). */
int vad_stream_hops(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, float* frames, int64_t frame_stride,
                    int32_t frame_len, const float* hop, int64_t hop_stride, int32_t hop_len, int64_t n_streams,
                    int32_t n_hops, int64_t hop_block_stride, float* ring, int32_t* count, uint8_t* labels,
                    int64_t label_block_stride, void* stream);
int vad_stream_step(const vad_mfcc_plan* plan, const vad_ffn_plan* ffn, const float* frames,
                    int64_t frame_stride, int32_t frame_len, int64_t n_streams, float* ring,
                    int32_t* count, uint8_t* labels, float* mfcc_scratch, void* stream);
/* Replay a captured hipGraph (hipGraphExec_t) on `stream`: the per-hop step
 * of a StreamBatch captured with its host I/O (the H2D copy of every
 * stream's new samples from pinned memory, the hop kernel, the D2H copy of
 * the labels -- vad.py:32-59's loop body for S streams).  The capture itself
 * is the host's (hipStreamBeginCapture / torch.cuda.graph); this entry only
 * launches, so a host replays without a runtime wrapper in between. */
int vad_graph_launch(void* graph_exec, void* stream);
/* The same replay, prepared once from the captured hipGraph_t and its
 * hipGraphExec_t (StreamBatch.capture keeps both; the graph must outlive the
 * plan): a graph of exactly one kernel node -- the one-hop step -- is
 * dispatched as that node (its captured function, grid, block, dynamic LDS
 * and argument values), whose host cost is a kernel launch's rather than
 * hipGraphLaunch's (~5 us more per call on ROCm 7.2); any other graph goes
 * through hipGraphLaunch.  vad_graph_plan_direct says which (1: the node). */
typedef struct vad_graph_plan vad_graph_plan;
int vad_graph_plan_create(void* graph, void* graph_exec, vad_graph_plan** out);
int vad_graph_plan_launch(const vad_graph_plan* plan, void* stream);
int32_t vad_graph_plan_direct(const vad_graph_plan* plan);
int vad_graph_plan_destroy(vad_graph_plan* plan);

/* ---------------------------------------------------------------------------
 * Multi-GPU clip sharding: one process per GPU, each
 * classifying its shard (vad_amd/dist.py split_clip: windows [w_lo, w_hi)
 * from samples [160 w_lo, 160 (w_hi + 4) + 401)), then ONE collective: the
 * gather of the per-window uint8 decisions to the root over RCCL / xGMI.
 * The reference's only parallelism is dataset_creator.py:84's process pool;
 * these entries replace nothing there -- they are the host-agnostic form of
 * vad_amd.dist.LabelGather (torch.distributed "nccl").  RCCL is resolved at
 * run time (the process's loaded copy, else librccl.so.1).
 * ------------------------------------------------------------------------- */
#define VAD_RCCL_ID_BYTES 128
typedef struct vad_rccl_comm vad_rccl_comm;
int vad_rccl_available(void);
const char* vad_rccl_error_string(void);
/* ncclGetUniqueId on the root; the caller ships the 128 bytes to every rank. */
int vad_rccl_unique_id(void* id_out /* VAD_RCCL_ID_BYTES */);
/* ncclCommInitRank on the current HIP device. */
int vad_rccl_init(vad_rccl_comm** out, int32_t nranks, const void* id, int32_t rank);
/* ncclGather of `count` uint8 per rank: recv (root only) = nranks * count,
 * rank r's block at recv + r * count.  Enqueued on `stream`. */
int vad_rccl_gather_u8(vad_rccl_comm* comm, const uint8_t* send, uint8_t* recv, size_t count, int32_t root,
                       void* stream);
int vad_rccl_destroy(vad_rccl_comm* comm);

#ifdef __cplusplus
}
#endif
#endif /* VAD_AMD_H */
