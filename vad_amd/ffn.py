"""The FFN classifier (reference learning/ffn_trainer.py:106-116) behind the
duck-typed ``predict`` protocol the analyser uses
(realtime_analysis/sklearn_analyser.py:71): ``predict(X) -> class ids``.

Weights are Keras-layout ``W (in, out)``, ``b (out,)`` float32, stored as an
``.npz`` with keys ``W0, b0, W1, b1, ...`` (the reference never committed
trained weights).

Arithmetic: the two specialised topologies (39-64-32-16-3, 13-64-64-N) run
"split-f16" by default -- every GEMM operand split v = hi + lo into f16
halves, lo*hi + hi*lo + hi*hi accumulated in f32 on v_mfma_f32_16x16x32_f16
(~22-bit operands: logits within a few f32 ulps of an exact-f32 forward);
arith="f32" (and every other topology) runs exact f32 products on
v_mfma_f32_16x16x4_f32.
"""
from __future__ import annotations

import numpy as np
import torch

from .plan import FfnPlan

# The reference topology (ffn_trainer.py:106-116) and BASELINE config 3's.
TOPOLOGY_REF39 = (39, 64, 32, 16, 3)
TOPOLOGY_BL13 = (13, 64, 64, 2)


def load_layers(path, prefix=""):
    """Layers [(W, b), ...] from an .npz (keys {prefix}W{i}, {prefix}b{i})."""
    with np.load(path, allow_pickle=False) as z:
        layers, i = [], 0
        while f"{prefix}W{i}" in z:
            layers.append((z[f"{prefix}W{i}"].astype(np.float32), z[f"{prefix}b{i}"].astype(np.float32)))
            i += 1
    if not layers:
        raise ValueError(f"no FFN layers '{prefix}W0..' in {path}")
    return layers


def save_layers(path, layers, prefix=""):
    np.savez(path, **{f"{prefix}{k}{i}": v for i, (w, b) in enumerate(layers)
                      for k, v in (("W", w), ("b", b))})


def random_layers(dims=TOPOLOGY_REF39, seed=0):
    """Seeded He-uniform Keras-shaped layers (synthetic weights for benches)."""
    rng = np.random.default_rng(seed)
    out = []
    for a, b in zip(dims[:-1], dims[1:]):
        lim = np.sqrt(6.0 / a)
        out.append((rng.uniform(-lim, lim, (a, b)).astype(np.float32),
                    (0.05 * rng.standard_normal(b)).astype(np.float32)))
    return out


class FFNClassifier:
    """GPU FFN with the sklearn/Keras ``predict`` protocol."""

    def __init__(self, layers, arith="split_f16"):
        self.layers = [(np.asarray(w, np.float32), np.asarray(b, np.float32)) for w, b in layers]
        if arith not in ("split_f16", "f32"):
            raise ValueError("arith must be 'split_f16' or 'f32'")
        self.arith_request = arith
        self._plan = None

    @classmethod
    def load(cls, path, prefix=""):
        return cls(load_layers(path, prefix))

    def save(self, path):
        save_layers(path, self.layers)

    @property
    def plan(self) -> FfnPlan:
        if self._plan is None:
            self._plan = FfnPlan(self.layers)
            if self.arith_request == "f32":
                self._plan.set_arith("f32")
        return self._plan

    @property
    def arith(self):
        """The arithmetic the plan runs: "split_f16" or "f32"."""
        return self.plan.arith

    @property
    def in_dim(self):
        return self.layers[0][0].shape[0]

    def predict(self, X):
        """Class ids (int64 ndarray) of feature rows X (n, in_dim) or (in_dim,)."""
        x = np.asarray(X, dtype=np.float32).reshape(-1, self.in_dim)
        t = torch.from_numpy(np.ascontiguousarray(x)).cuda()
        return self.plan.predict(t).cpu().numpy().astype(np.int64)

    def predict_device(self, x, out=None):
        """Labels (uint8, device) of device feature rows x (n, in_dim) fp32."""
        return self.plan.predict(x, out=out)

    # pickle support: weights travel, the device plan is rebuilt lazily
    def __getstate__(self):
        return {"layers": self.layers, "arith": self.arith_request}

    def __setstate__(self, st):
        self.layers = st["layers"]
        self.arith_request = st.get("arith", "split_f16")
        self._plan = None
