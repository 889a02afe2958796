"""Offline dataset export on the GPU: process_file (wav / sph, with and
without a transcript), scale_features and the CSV rows against the
reference's own outputs (tests/golden/dataset.npz).

Tolerances: MFCC deltas per row ||d||/||ref|| <= 1e-3 (the fp32 MFCCs are
within 1e-4 of the reference's fp64 ones, see test_gpu_parity.py; deltas
are differences of them); scaled features max |d| <= 1e-4 * max |ref| per
row (fp32 storage of values normalised in fp64)."""
import csv
import io

import numpy as np
import pytest

from vad_amd import dataset as D

pytestmark = pytest.mark.gpu


def _write(tmp_path, name, arr):
    p = tmp_path / name
    p.write_bytes(np.asarray(arr, np.uint8).tobytes())
    return str(p)


def _files(tmp_path, g):
    return [_write(tmp_path, "clip0.wav", g["wav0_bytes"]),
            _write(tmp_path, "clip1.wav", g["wav1_bytes"]),
            _write(tmp_path, "sph16.sph", g["sph16_bytes"])]


def _row_rel(a, b):
    return np.linalg.norm(a - b, axis=1) / np.maximum(np.linalg.norm(b, axis=1), 1e-30)


def test_process_file_matches_reference(tmp_path, golden):
    from oracle import vad_oracle as O
    g = golden("dataset")
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    files = _files(tmp_path, g)
    for i, p in enumerate(files):
        feats = D.process_file([p, 400, 160, 512, fb, 13, None, None])
        got = np.asarray([np.concatenate(fr) for fr in feats])
        assert got.shape == g[f"feat{i}"].shape
        assert _row_rel(got, g[f"feat{i}"]).max() <= 1e-3
    stm = _write(tmp_path, "talk1.stm", g["stm_bytes"])
    feats = D.process_file([files[2], 400, 160, 512, fb, 13, None, stm])
    got = np.asarray([np.concatenate(fr) for fr in feats])
    assert got.shape == g["feat_tr"].shape
    assert _row_rel(got, g["feat_tr"]).max() <= 1e-3


def test_scale_features_matches_reference(golden):
    g = golden("dataset")
    c = 13
    ref = g["scaled"]
    # reference structure, scaled in place
    feats = [[(r[:c].copy(), r[c:2 * c].copy(), r[2 * c:].copy()) for r in g[f"feat{i}"]]
             for i in range(3)]
    out = D.scale_features(feats)
    assert out is feats
    got = np.asarray([np.concatenate(fr) for ff in out for fr in ff])
    mx = np.abs(got - ref).max(axis=1) / np.abs(ref).max(axis=1)
    assert mx.max() <= 1e-4
    # array form
    arr = np.concatenate([g[f"feat{i}"] for i in range(3)]).astype(np.float32)
    got2 = D.scale_features(arr)
    assert np.abs(got2 - ref).max() <= 1e-4 * np.abs(ref).max()
    # statistics: numpy's on the same fp32 rows
    import torch
    t = torch.from_numpy(arr).cuda()
    mean, std = D.scale_rows_device(t)
    a64 = arr.astype(np.float64).reshape(len(arr), 3, c)
    assert np.allclose(mean, a64.mean(axis=(0, 2)), rtol=1e-12, atol=1e-12)
    assert np.allclose(std, a64.std(axis=(0, 2)), rtol=1e-12)


def test_export_end_to_end_csv(tmp_path, golden):
    """process_file -> scale_features -> CSV rows (native formatter) parses
    back to the reference CSV's numbers (load_csv reads float32)."""
    from oracle import vad_oracle as O
    g = golden("dataset")
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    rows = np.concatenate([D.file_features(p) for p in _files(tmp_path, g)])
    scaled = D.scale_features(rows)
    text = D.format_csv_rows(scaled, 1)
    ours = np.array([list(map(float, r)) for r in csv.reader(io.StringIO(text))])
    ref = np.array([list(map(float, r)) for r in csv.reader(io.StringIO(g["csv_text"].tobytes().decode()))])
    assert ours.shape == ref.shape == (273, 40)
    assert np.array_equal(ours[:, -1], ref[:, -1])
    mx = np.abs(ours[:, :-1] - ref[:, :-1]).max(axis=1) / np.abs(ref[:, :-1]).max(axis=1)
    assert mx.max() <= 1e-4
