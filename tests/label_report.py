"""Label agreement of a device run with the fp64 oracle (SURVEY.md 8(c):
"report any frame below the margin separately").

`label_agreement` counts the windows whose device label differs from the
oracle's, lists each with its fp64 top-2 logit margin, and bins the margins of
all windows and of the disagreeing ones into a decade histogram.  When
`name` is given the report is also written to gpurun_out/<name>.json (the GPU
box merges gpurun_out/ back; profiles/ keeps the committed copies).
"""
import json
import os

import numpy as np

EDGES = [0.0, 1e-7, 1e-6, 1e-5, 1e-4, 1e-3, 1e-2, 5e-2, 1e-1, 1.0, np.inf]


def label_agreement(got, ref, margin, name=None, extra=None):
    got = np.asarray(got)
    ref = np.asarray(ref)
    margin = np.asarray(margin, np.float64)
    bad = np.flatnonzero(got != ref)
    h_all, _ = np.histogram(margin, bins=EDGES)
    h_bad, _ = np.histogram(margin[bad], bins=EDGES)
    rep = {
        "windows": int(got.size),
        "disagree": int(bad.size),
        "disagree_windows": [{"window": int(i), "device": int(got[i]), "oracle": int(ref[i]),
                              "margin": float(margin[i])} for i in bad[:200]],
        "max_margin_of_disagreement": float(margin[bad].max()) if bad.size else None,
        "margin_hist_edges": [float(e) for e in EDGES],
        "margin_hist_all": [int(c) for c in h_all],
        "margin_hist_disagree": [int(c) for c in h_bad],
        "min_margin": float(margin.min()) if margin.size else None,
    }
    if extra:
        rep.update(extra)
    print(f"label agreement{f' ({name})' if name else ''}: {rep['disagree']} of {rep['windows']} windows "
          f"differ from the fp64 oracle; margins of those: "
          f"{[round(d['margin'], 9) for d in rep['disagree_windows'][:20]]}", flush=True)
    if name:
        root = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        d = os.path.join(root, "gpurun_out")
        try:
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, name + ".json"), "w") as f:
                json.dump(rep, f, indent=1)
        except OSError:
            pass
    return rep


def record_vs_baseline(name, values):
    """Write `values` beside the previous round's committed numbers
    (profiles/regression_baseline.json) to gpurun_out/<name>.json, with an
    `increased` flag per key: a kernel time past `flag_time_ratio` x its
    baseline, a disagreement count above it.  A record, not a bound: the
    tests' own gates stay as they are, the flags make drifts visible."""
    root = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = {}
    bp = os.path.join(root, "profiles", "regression_baseline.json")
    if os.path.exists(bp):
        with open(bp) as f:
            base = json.load(f)
    ratio = float(base.get("flag_time_ratio", 1.1))
    rec = {"source": base.get("source"), "values": {}}
    for k, v in values.items():
        b = base.get(k)
        inc = None
        if b is not None:
            inc = bool(v > b * ratio) if k.endswith("_ms") else bool(v > b)
        rec["values"][k] = {"now": v, "baseline": b, "increased": inc}
        if inc:
            print(f"REGRESSION FLAG {name}: {k} = {v} vs baseline {b}", flush=True)
    d = os.path.join(root, "gpurun_out")
    try:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".json"), "w") as f:
            json.dump(rec, f, indent=1)
    except OSError:
        pass
    return rec
