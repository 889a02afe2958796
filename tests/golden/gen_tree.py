"""Decision-tree fixture (tests/golden/tree.npz).

Trains scikit-learn's DecisionTreeClassifier with the reference's parameters
(learning/decision_classifier_trainer.py:26-29: min_samples_split=22,
max_depth=25, min_samples_leaf=20) on analyser features of synthetic clips
(the oracle's restatement of sklearn_analyser.py:52-69), with labels from a
log-energy rule plus 10% flipped labels so the tree grows deep, and records
sklearn's own predictions on held-out rows (some with NaN features, the
analyser's constant-window case).  The reference's trained blob is missing
(.MISSING_LARGE_BLOBS), so the tree is synthetic; the fixture pins the
traversal, not a model.  Only arrays are stored (no pickle).

    python tests/golden/gen_tree.py
"""
import os
import sys

import numpy as np
import sklearn
from sklearn.tree import DecisionTreeClassifier

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import vad_oracle as O  # noqa: E402


def features_and_labels(seed, frames, fb, rng):
    clip = O.synth_clip(O.samples_for_frames(frames), seed)
    m = O.mfcc_batch(clip, fb)
    x = O.analyser_features_fast(m)
    c0 = m[2:-3, 0]  # raw log-energy cepstrum of each window's centre frame
    y = (c0 > np.median(c0)).astype(np.int64)
    flip = rng.random(len(y)) < 0.10
    y[flip] = 1 - y[flip]
    ok = ~np.isnan(x).any(axis=1)
    return x, y, ok


def main():
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    rng = np.random.default_rng(7)
    xs, ys = [], []
    for seed in range(20, 26):
        x, y, ok = features_and_labels(seed, 3000, fb, rng)
        xs.append(x[ok])
        ys.append(y[ok])
    X, y = np.concatenate(xs).astype(np.float32), np.concatenate(ys)
    clf = DecisionTreeClassifier(min_samples_split=22, max_depth=25, min_samples_leaf=20,
                                 random_state=0).fit(X, y)
    xt, _, _ = features_and_labels(40, 2000, fb, rng)
    xt = xt.astype(np.float32)
    xt[::97, 0] = np.nan  # NaN rows: missing_go_to_left
    pred = clf.predict(xt)
    t = O.tree_arrays(clf)
    np.savez_compressed(os.path.join(HERE, "tree.npz"), x_test=xt, y_test=pred,
                        sklearn_version=np.array(sklearn.__version__),
                        **{k: np.asarray(v) for k, v in t.items()})
    print("tree nodes", len(t["feature"]), "depth", clf.get_depth(), "test rows", len(xt),
          "class-1 share", float(pred.mean()))


if __name__ == "__main__":
    main()
