"""Offline dataset export, host side (no GPU): SPHERE / STM / framing /
header / CSV text against the reference's own outputs
(tests/golden/dataset.npz, made by tests/golden/gen_dataset.py running the
unmodified reference modules), and the native CSV formatter against numpy's
float32 printing."""
import csv
import io

import numpy as np
import pytest

from vad_amd import dataset as D


def _write(tmp_path, name, arr):
    p = tmp_path / name
    p.write_bytes(np.asarray(arr, np.uint8).tobytes())
    return str(p)


@pytest.mark.parametrize("name", ["sph16", "sph8", "sph16trunc"])
def test_sph_read_matches_reference(tmp_path, golden, name):
    g = golden("dataset")
    s = D.sph_read(_write(tmp_path, name + ".sph", g[name + "_bytes"]))
    assert np.array_equal(s.data, g[name + "_data"]) and s.data.dtype == np.int16
    assert [s.channels, s.framerate, s.sample_width] == list(g[name + "_meta"])


def test_stm_matches_reference(tmp_path, golden):
    g = golden("dataset")
    p = _write(tmp_path, "talk1.stm", g["stm_bytes"])
    st, en = D.stm_parse(p)
    assert np.array_equal(st, g["stm_starts"]) and np.array_equal(en, g["stm_ends"])
    si, ei = D.get_samples_indices(p, 16000)
    assert np.array_equal(si, g["stm_sidx"]) and np.array_equal(ei, g["stm_eidx"])


def test_split_with_transcript_matches_reference(tmp_path, golden):
    g = golden("dataset")
    p = _write(tmp_path, "talk1.stm", g["stm_bytes"])
    fr = D.split_into_frames(g["sph16_data"], 400, 160, p, 16000)
    assert np.array_equal(np.asarray(fr, np.int16), g["tr_frames"])
    with pytest.raises(Exception):
        D.split_into_frames(g["sph16_data"], 400, 160, p, None)


def test_header_and_writer_text_match_reference(golden):
    g = golden("dataset")
    assert D.create_table_header(13) == list(g["header"])
    # write_features on the reference's own (scaled, float64) features
    c = 13
    rows = g["scaled"]
    sizes = [len(g["feat0"]), len(g["feat1"]), len(g["feat2"])]
    feats, i = [], 0
    for n in sizes:
        feats.append([(r[:c], r[c:2 * c], r[2 * c:]) for r in rows[i:i + n]])
        i += n
    s = io.StringIO()
    D.write_features(csv.writer(s), feats, 1)
    assert s.getvalue().encode() == g["csv_text"].tobytes()


def test_native_csv_formatter_matches_numpy_float32():
    rng = np.random.default_rng(9)
    v = (rng.standard_normal(39 * 3000) * 10.0 ** rng.integers(-9, 21, 39 * 3000)).astype(np.float32)
    v[:16] = [0.0, -0.0, 1.0, 3.0, 1e-4, 9.999e-5, 1e16, 9.99e15, 1e-5, np.nan, np.inf, -np.inf,
              0.1, 123456789.0, 1e-45, -3.4e38]
    rows = v.reshape(-1, 39)
    for label in (0, 1, 2):
        s = io.StringIO()
        csv.writer(s).writerows([list(r) + [np.float64(label)] for r in rows])
        assert D.format_csv_rows(rows, label) == s.getvalue()
    assert D.format_csv_rows(np.zeros((0, 39), np.float32), 1) == ""
