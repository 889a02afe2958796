"""Decision-tree classifier on the GPU (the classifier vad.py deploys:
learning/decision_classifier_trainer.py:26-35, an sklearn
``DecisionTreeClassifier(min_samples_split=22, max_depth=25,
min_samples_leaf=20)`` used through the ``predict`` protocol of
realtime_analysis/sklearn_analyser.py:71).

The tree is a flat node table (feature, threshold, left, right, leaf class)
walked by ``tree_kernel.hip`` with sklearn's rule: left iff
``float32(x[feature]) <= threshold``, a NaN feature following the node's
``missing_go_to_left`` (sklearn >= 1.3).  ``predict`` returns class *values*
(``classes_[index]``), like sklearn.  Tables are stored as ``.npz`` (arrays
only) -- a pickled sklearn estimator can be converted with ``from_sklearn``.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr
from .plan import _out

_KEYS = ("feature", "threshold", "left", "right", "leaf", "nan_left", "classes")


class TreePlan:
    """Device node table (include/vad_amd.h vad_tree_plan)."""

    def __init__(self, feature, threshold, left, right, leaf, nan_left, n_features):
        f = np.ascontiguousarray(feature, np.int32)
        t = np.ascontiguousarray(threshold, np.float64)
        lt = np.ascontiguousarray(left, np.int32)
        rt = np.ascontiguousarray(right, np.int32)
        lf = np.ascontiguousarray(leaf, np.int32)
        nl = np.ascontiguousarray(nan_left, np.uint8)
        n = f.shape[0]
        if not (t.shape == lt.shape == rt.shape == lf.shape == nl.shape == (n,)):
            raise ValueError("node arrays must have one entry per node")
        h = ctypes.c_void_p()
        check(lib().vad_tree_plan_create(n, f.ctypes.data, t.ctypes.data, lt.ctypes.data,
                                         rt.ctypes.data, lf.ctypes.data, nl.ctypes.data,
                                         int(n_features), ctypes.byref(h)), "vad_tree_plan_create")
        self._h = h
        self._destroy = lib().vad_tree_plan_destroy
        self.n_features = int(n_features)

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        destroy = getattr(self, "_destroy", None)  # bound at creation: module globals
        if h is not None and h.value and destroy is not None:  # may be gone at exit
            destroy(h)
            self._h = None


class TreeClassifier:
    """GPU decision tree with the sklearn ``predict`` protocol."""

    def __init__(self, feature, threshold, left, right, leaf, nan_left, classes, n_features):
        self.nan_left = np.asarray(nan_left, np.uint8)
        self.feature = np.asarray(feature, np.int32)
        self.threshold = np.asarray(threshold, np.float64)
        self.left = np.asarray(left, np.int32)
        self.right = np.asarray(right, np.int32)
        self.leaf = np.asarray(leaf, np.int32)
        self.classes_ = np.asarray(classes)
        self.n_features = int(n_features)
        self._plan = None

    # -- construction ----------------------------------------------------
    @classmethod
    def from_sklearn(cls, clf):
        """From a fitted sklearn DecisionTreeClassifier (single output)."""
        t = clf.tree_
        value = np.asarray(t.value)
        if value.ndim == 3:
            if value.shape[1] != 1:
                raise ValueError("multi-output trees are not supported")
            value = value[:, 0, :]
        leaf = np.argmax(value, axis=1)  # sklearn predict: classes_[argmax(proba)], first max
        feature = np.where(np.asarray(t.children_left) < 0, -1, np.asarray(t.feature))
        nan_left = np.asarray(getattr(t, "missing_go_to_left", np.zeros(t.node_count, np.uint8)))
        return cls(feature, t.threshold, t.children_left, t.children_right, leaf, nan_left,
                   clf.classes_, t.n_features)

    @staticmethod
    def looks_like_sklearn_tree(obj):
        t = getattr(obj, "tree_", None)
        return (t is not None and hasattr(obj, "classes_") and hasattr(t, "children_left")
                and hasattr(t, "threshold") and hasattr(t, "feature") and hasattr(t, "value"))

    @classmethod
    def load(cls, path):
        with np.load(path, allow_pickle=False) as z:
            return cls(*(z[k] for k in _KEYS), int(z["n_features"]))

    def save(self, path):
        np.savez(path, feature=self.feature, threshold=self.threshold, left=self.left,
                 right=self.right, leaf=self.leaf, nan_left=self.nan_left, classes=self.classes_,
                 n_features=np.int64(self.n_features))

    @property
    def plan(self) -> TreePlan:
        if self._plan is None:
            self._plan = TreePlan(self.feature, self.threshold, self.left, self.right, self.leaf,
                                  self.nan_left, self.n_features)
        return self._plan

    @property
    def in_dim(self):
        return self.n_features

    # -- inference --------------------------------------------------------
    def predict_device(self, x, out=None, stream=None):
        """Class indices (uint8, device) of device feature rows x (n, n_features) fp32."""
        if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype == torch.float32):
            raise TypeError("x must be a CUDA float32 tensor")
        x = x.contiguous().reshape(-1, self.n_features)  # kept alive until the launch is queued
        n = x.shape[0]
        out = _out(out, (n,), torch.uint8, x.device)
        check(lib().vad_tree_predict(self.plan.handle, ptr(x), n, ptr(out), stream_ptr(stream)),
              "vad_tree_predict")
        _keep_for_stream(x, stream)
        return out

    def predict(self, X):
        """sklearn's predict: class values of feature rows X (n, n_features) or (n_features,)."""
        x = np.asarray(X, dtype=np.float32).reshape(-1, self.n_features)
        idx = self.predict_device(torch.from_numpy(np.ascontiguousarray(x)).cuda())
        return self.classes_[idx.cpu().numpy().astype(np.int64)]

    def window_labels(self, mfcc, mode=_lib.FEAT_ANALYSER, out=None, stream=None):
        """Class indices (uint8, device) of every 5-frame window of an MFCC sequence."""
        if not (isinstance(mfcc, torch.Tensor) and mfcc.is_cuda and mfcc.dtype == torch.float32):
            raise TypeError("mfcc must be a CUDA float32 tensor")
        f, c = mfcc.shape
        rows = max(f - 5, 0)
        out = _out(out, (rows,), torch.uint8, mfcc.device)
        m = mfcc.contiguous()  # a temporary copy must outlive the asynchronous kernel
        check(lib().vad_features_tree(self.plan.handle, ptr(m), f, c, int(mode),
                                      ptr(out), stream_ptr(stream)), "vad_features_tree")
        _keep_for_stream(m, stream)
        return out


def _keep_for_stream(t, stream):
    """A tensor read by a kernel queued on `stream` (not the current stream)
    must not be recycled by the caching allocator for current-stream work
    before that kernel ran."""
    if stream is not None and stream != torch.cuda.current_stream(t.device):
        t.record_stream(stream)
