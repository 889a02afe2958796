"""Golden fixtures for the offline dataset export (tests/golden/dataset.npz),
made by running the UNMODIFIED reference dataset modules in the build
container:

  dataset/sph.py             read                 (SPHERE decode)
  dataset/stm_parser.py      parse / get_samples_indices
  dataset/file_processing.py split_into_frames (with a transcript),
                             process_file, create_table_header, write_features
  dataset/utils.py           scale_features

The modules are Python 2; they run under these shims, applied to the module
namespaces only (no source is changed or copied):
  * ``open`` in sph / stm_parser returns a file whose readline / read give
    ``str`` (latin-1) like Python 2's binary files;
  * ``range`` in sph floors its float argument (Py2 ``len(chunk) / width``);
  * ``np`` in sph is numpy except that ``zeros`` returns an int16 array whose
    item assignment wraps (numpy 1 behaviour; numpy 2 raises OverflowError
    for values >= 32768, i.e. every negative big-endian sample);
  * ``fft_n`` is an int whose ``/`` floors (mfcc.py:45-46,61), and h5py /
    cPickle are stubbed as in gen_golden.py.
Inputs (the wav / sph / stm file bytes) and outputs are stored as arrays, so
the tests recreate the files anywhere.

    python tests/golden/gen_dataset.py
"""
from __future__ import annotations

import builtins
import copy
import csv
import io
import os
import queue
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from gen_golden import REF, FloorInt, import_reference  # noqa: E402
from oracle import vad_oracle as O  # noqa: E402


class _Py2File:
    """Binary file whose reads return str (latin-1), as Python 2's do."""

    def __init__(self, fname, mode="rb"):
        with builtins.open(fname, "rb") as f:
            self._b = f.read()
        self._p = 0

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def readline(self, limit=-1):
        end = self._b.find(b"\n", self._p)
        end = len(self._b) if end < 0 else end + 1
        if limit is not None and limit >= 0:
            end = min(end, self._p + limit)
        s = self._b[self._p:end]
        self._p = end
        return s.decode("latin-1")

    def read(self, n=-1):
        end = len(self._b) if n is None or n < 0 else min(len(self._b), self._p + n)
        s = self._b[self._p:end]
        self._p = end
        return s.decode("latin-1")


class _WrapInt16(np.ndarray):
    def __setitem__(self, k, v):
        super().__setitem__(k, np.array(int(v) & 0xFFFF, np.uint16).view(np.int16))


class _NpShim(types.ModuleType):
    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def zeros(shape, dtype=float):
        return np.zeros(shape, dtype).view(_WrapInt16) if np.dtype(dtype) == np.int16 \
            else np.zeros(shape, dtype)


def sph_bytes(samples, width, count=None, rate=16000, truncate=None):
    n = len(samples) if count is None else count
    head = (f"NIST_1A\n   1024\nsample_count -i {n}\nsample_n_bytes -i {width}\n"
            f"channel_count -i 1\nsample_byte_format -s2 10\nsample_rate -i {rate}\n"
            "sample_coding -s3 pcm\nend_head\n").encode()
    v = np.asarray(samples, np.int64) & ((1 << (8 * width)) - 1)
    body = b"".join(int(x).to_bytes(width, "big") for x in v)
    if truncate is not None:
        body = body[:truncate]
    return head + body


STM = (b"talk1 1 spk1 0.0 0.5 <o,f0,male> hello there\n"
       b"talk1 1 spk1 0.75 1.3125 <o,f0,male> more words here\n"
       b"talk1 1 spk1 1.5 1.6 <o,f0,male> ignore_time_segment_in_scoring\n"
       b"talk1 1 spk1 1.7 1.8\n"
       b"talk1 1 spk1 2.0 2.2539 <o,f0,male> tail\n")


def main():
    mfcc_mod, _, fp = import_reference()
    sys.path.insert(0, os.path.join(REF, "dataset"))
    import importlib.util
    import sph
    import stm_parser
    spec = importlib.util.spec_from_file_location("dataset_utils", os.path.join(REF, "dataset",
                                                                                "utils.py"))
    ds_utils = importlib.util.module_from_spec(spec)  # dataset/utils.py (root utils.py shadows it)
    spec.loader.exec_module(ds_utils)
    for m in (sph, stm_parser):
        m.open = _Py2File
    sph.range = lambda x: builtins.range(int(x))
    sph.np = _NpShim("numpy_shim")

    rng = np.random.default_rng(5)
    out = {}
    tmp = tempfile.mkdtemp()
    # ---- SPHERE: 16-bit with negatives, 8-bit, truncated body -----------
    cases = {
        "sph16": (np.clip(O.synth_clip(8000, 51), -32768, 32767).astype(np.int64), 2, None, None),
        "sph8": (rng.integers(0, 256, 1000), 1, None, None),
        "sph16trunc": (rng.integers(-32768, 32768, 3000), 2, 3000, 2 * 2500 + 1),
    }
    for name, (s, w, cnt, trunc) in cases.items():
        b = sph_bytes(s, w, cnt, truncate=trunc)
        p = os.path.join(tmp, name + ".sph")
        with open(p, "wb") as f:
            f.write(b)
        r = sph.read(p)
        out[f"{name}_bytes"] = np.frombuffer(b, np.uint8)
        out[f"{name}_data"] = np.asarray(r.data, np.int16)
        out[f"{name}_meta"] = np.array([r.channels, r.framerate, r.sample_width])
    # ---- STM ------------------------------------------------------------
    ps = os.path.join(tmp, "talk1.stm")
    with open(ps, "wb") as f:
        f.write(STM)
    out["stm_bytes"] = np.frombuffer(STM, np.uint8)
    st, en = stm_parser.parse(ps)
    out["stm_starts"], out["stm_ends"] = np.asarray(st, np.float32), np.asarray(en, np.float32)
    si, ei = stm_parser.get_samples_indices(ps, 16000)
    out["stm_sidx"], out["stm_eidx"] = np.asarray(si), np.asarray(ei)
    # ---- framing with a transcript --------------------------------------
    data = out["sph16_data"]
    frames = fp.split_into_frames(data, 400, 160, ps, 16000)
    out["tr_frames"] = np.asarray(frames, np.int16)
    # ---- process_file on wav + sph files, scale_features, csv -----------
    from scipy.io import wavfile
    fb = mfcc_mod.get_mel_filterbanks(300, 8000, FloorInt(512), 26, 16000)
    files = []
    for i, seed in enumerate((61, 62)):
        x = np.clip(O.synth_clip(160 * 120 + 241, seed), -32768, 32767).astype(np.int16)
        p = os.path.join(tmp, f"clip{i}.wav")
        wavfile.write(p, 16000, x)
        with open(p, "rb") as f:
            out[f"wav{i}_bytes"] = np.frombuffer(f.read(), np.uint8)
        files.append(p)
    files.append(os.path.join(tmp, "sph16.sph"))
    q = queue.Queue(1)
    q.put(0)
    feats = [fp.process_file([p, 400, 160, FloorInt(512), fb, 13, q, None]) for p in files]
    for i, ff in enumerate(feats):
        out[f"feat{i}"] = np.asarray([np.concatenate(fr) for fr in ff])
    tr_feats = fp.process_file([files[2], 400, 160, FloorInt(512), fb, 13, q, ps])
    out["feat_tr"] = np.asarray([np.concatenate(fr) for fr in tr_feats])
    scaled = ds_utils.scale_features(copy.deepcopy(feats))
    out["scaled"] = np.asarray([np.concatenate(fr) for ff in scaled for fr in ff])
    out["header"] = np.array(fp.create_table_header(13))
    s = io.StringIO()
    fp.write_features(csv.writer(s), scaled, 1)
    out["csv_text"] = np.frombuffer(s.getvalue().encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "dataset.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
