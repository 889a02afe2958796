// Decision-tree classifier (the classifier vad.py deploys:
// learning/decision_classifier_trainer.py:26-35, sklearn
// DecisionTreeClassifier(min_samples_split=22, max_depth=25,
// min_samples_leaf=20), called through the predict protocol of
// realtime_analysis/sklearn_analyser.py:71) as a flat node table.
//
// Traversal semantics are sklearn's (sklearn/tree/_tree.pyx, apply_dense):
// X is converted to float32, and at an internal node the row goes left iff
// X[i, feature] <= threshold, the comparison in double (float32 feature
// promoted, float64 threshold) -- so a float32 feature row gives exactly
// sklearn's leaf.  A NaN feature (the analyser's constant-window Mn) follows
// the node's missing_go_to_left (sklearn >= 1.3; older releases rejected NaN
// input with a ValueError).  The leaf's class is argmax of its value row (first max),
// resolved on the host when the table is built.
//
// Window path: 256 windows per block; their MFCC rows are staged in LDS, the
// 39 features of each window computed once into an LDS row, and each thread
// walks the tree for its window reading features from LDS.  Tables of up to
// kLdsNodes nodes are copied once per block into LDS in the compact 16-B
// form (float threshold rounded down, flags packed into the feature word), so
// every level of the walk is two dependent LDS reads instead of an L1/L2 load
// of a 24-B node; larger tables are walked from global memory.
#include "vad_common.h"
#include "features.h"

namespace vad {

constexpr int kTreeWin = 256;                   // windows per block
constexpr int kTreeXStride = 3 * kMaxCoefs + 1;  // floats per LDS feature row (49: odd)

__device__ __forceinline__ int tree_walk(const TreeNode* __restrict__ nodes, int n_nodes,
                                         const float* __restrict__ x, int x_step) {
  int node = 0;
  // every root-to-leaf path has < n_nodes edges; the bound only guards a
  // malformed table against looping forever
  for (int it = 0; it < n_nodes; ++it) {
    const TreeNode nd = nodes[node];
    if (nd.feature < 0) return nd.leaf;
    const float xv = x[nd.feature * x_step];
    const bool left = xv != xv ? nd.nan_left != 0 : (double)xv <= nd.threshold;
    node = left ? nd.left : nd.right;
  }
  return 0;
}

// Feature rows x[i*dim + f] (vad_tree_predict).
__global__ __launch_bounds__(256) void tree_rows_kernel(const TreeNode* __restrict__ nodes,
                                                        int n_nodes, const float* __restrict__ x,
                                                        int64_t n, int dim,
                                                        uint8_t* __restrict__ labels) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    labels[i] = (uint8_t)tree_walk(nodes, n_nodes, x + i * dim, 1);
}

// Windows of an MFCC sequence (vad_features_tree), 256 per block iteration.
constexpr int kLdsNodes = 3072;  // 48 KB of compact nodes

__device__ __forceinline__ int tree_walk_c(const TreeNodeC* nodes, int n_nodes, const float* x) {
  int node = 0;
  for (int it = 0; it < n_nodes; ++it) {
    const TreeNodeC nd = nodes[node];
    if (nd.feature < 0) return -1 - nd.feature;
    const float xv = x[nd.feature & 0xffff];
    const bool left = xv != xv ? (nd.feature >> 30) != 0 : xv <= nd.thr;
    node = left ? nd.left : nd.right;
  }
  return 0;
}

template <int MN, bool LDSN>
__global__ __launch_bounds__(256) void tree_window_kernel(const TreeNode* __restrict__ nodes,
                                                          const TreeNodeC* __restrict__ cnodes,
                                                          int n_nodes,
                                                          const float* __restrict__ mfcc,
                                                          int64_t n_rows, int mfcc_n_rt, int mode,
                                                          uint8_t* __restrict__ labels) {
  // feature rows: 3 MN floats (odd for MN = 13, so the walk's per-thread
  // reads spread over the banks)
  constexpr int XS = MN > 0 ? 3 * MN : kTreeXStride;
  constexpr int RS = MN > 0 ? MN : kMaxCoefs;
  __shared__ float rows[(kTreeWin + 4) * RS];
  __shared__ float X[kTreeWin * XS];
  extern __shared__ TreeNodeC cn_s[];
  const int mfcc_n = MN > 0 ? MN : mfcc_n_rt;
  const int tid = threadIdx.x;
  if constexpr (LDSN) {
    for (int i = tid; i < n_nodes; i += 256) cn_s[i] = cnodes[i];
    // (visible after the first chunk's barrier)
  }
  const int64_t n_frames = n_rows + 5;
  const int64_t n_chunks = (n_rows + kTreeWin - 1) / kTreeWin;
  for (int64_t ch = blockIdx.x; ch < n_chunks; ch += gridDim.x) {
    const int64_t base = ch * kTreeWin;
    const int64_t avail = n_frames - base;
    const int nr = (int)(avail < kTreeWin + 4 ? avail : kTreeWin + 4);
    for (int i = tid; i < nr * mfcc_n; i += 256) {
      const int r = i / mfcc_n, c = i - r * mfcc_n;
      rows[r * RS + c] = mfcc[base * mfcc_n + i];
    }
    __syncthreads();
    const int64_t nwin64 = n_rows - base;
    const int nwin = (int)(nwin64 < kTreeWin ? nwin64 : kTreeWin);
    for (int i = tid; i < nwin * mfcc_n; i += 256) {
      const int w = i / mfcc_n, c = i - w * mfcc_n;
      const float* rw = rows + w * RS + c;
      const Feat3 ft = feature_triple(rw[0], rw[RS], rw[2 * RS], rw[3 * RS], rw[4 * RS], mode);
      float* xw = X + w * XS;
      xw[c] = ft.mn;
      xw[mfcc_n + c] = ft.d1;
      xw[2 * mfcc_n + c] = ft.d2;
    }
    __syncthreads();
    if (tid < nwin) {
      if constexpr (LDSN) labels[base + tid] = (uint8_t)tree_walk_c(cn_s, n_nodes, X + tid * XS);
      else labels[base + tid] = (uint8_t)tree_walk(nodes, n_nodes, X + tid * XS, 1);
    }
    __syncthreads();
  }
}

static int tree_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

hipError_t launch_tree_rows(const TreeNode* nodes, int n_nodes, const float* x, int64_t n, int dim,
                            uint8_t* labels, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  const int64_t cap = 8 * tree_num_cus();
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(tree_rows_kernel, dim3((int)blocks), dim3(256), 0, st, nodes, n_nodes, x, n, dim,
                     labels);
  return hipGetLastError();
}

hipError_t launch_tree_windows(const TreeNode* nodes, const TreeNodeC* cnodes, int n_nodes,
                               const float* mfcc, int64_t n_rows, int mfcc_n, int mode,
                               uint8_t* labels, hipStream_t st) {
  if (n_rows <= 0) return hipSuccess;
  int64_t blocks = (n_rows + kTreeWin - 1) / kTreeWin;
  const int64_t cap = 4 * tree_num_cus();
  if (blocks > cap) blocks = cap;
  // 1M windows, 977-node fixture tree: 71 us from LDS, 109 us from global
  const bool lds = cnodes && n_nodes <= kLdsNodes;
  const size_t smem = lds ? (size_t)n_nodes * sizeof(TreeNodeC) : 0;
  if (mfcc_n == 13 && lds)
    hipLaunchKernelGGL((tree_window_kernel<13, true>), dim3((int)blocks), dim3(256), smem, st, nodes,
                       cnodes, n_nodes, mfcc, n_rows, mfcc_n, mode, labels);
  else if (mfcc_n == 13)
    hipLaunchKernelGGL((tree_window_kernel<13, false>), dim3((int)blocks), dim3(256), 0, st, nodes,
                       cnodes, n_nodes, mfcc, n_rows, mfcc_n, mode, labels);
  else if (lds)
    hipLaunchKernelGGL((tree_window_kernel<0, true>), dim3((int)blocks), dim3(256), smem, st, nodes,
                       cnodes, n_nodes, mfcc, n_rows, mfcc_n, mode, labels);
  else
    hipLaunchKernelGGL((tree_window_kernel<0, false>), dim3((int)blocks), dim3(256), 0, st, nodes,
                       cnodes, n_nodes, mfcc, n_rows, mfcc_n, mode, labels);
  return hipGetLastError();
}

}  // namespace vad
