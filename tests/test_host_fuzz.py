"""Property-based (hypothesis) tests of the host logic, CPU only.

  split_clip     the shards of a clip partition its F - 5 windows in rank
                 order, each segment (with its 240-sample + 4-frame halo,
                 SURVEY 8(e)) frames to exactly its own windows, and the
                 oracle's labels of the segments concatenate to the oracle's
                 labels of the whole clip (the halo rule, end to end)
  hop layouts    hop_rows_disjoint (stream.py; capi.hip's
                 vad_hop_layout_disjoint is the same rule) only accepts
                 layouts whose K x S hop rows are pairwise disjoint (checked
                 by brute force, for row strides >= the hop length, which
                 the C ABI requires first), and accepts both contiguous
                 orderings
"""
import os

import numpy as np
import pytest

from oracle import vad_oracle as O

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_SCALE = int(os.environ.get("VAD_FUZZ_SCALE", "1"))  # deep runs: see tests/test_gpu_fuzz.py
_SEED = os.environ.get("VAD_FUZZ_SEED")
FUZZ = settings(max_examples=200 * _SCALE, deadline=None, derandomize=_SEED is None, database=None)


def fuzz(n):
    s = settings(FUZZ, max_examples=n * _SCALE)
    return s if _SEED is None else (lambda f: hyp.seed(int(_SEED))(s(f)))


@fuzz(200)
@given(n=st.integers(0, 2_000_000), world=st.integers(1, 8))
def test_split_clip_partitions_windows(n, world):
    from vad_amd.dist import n_frames, split_clip
    n_win = max(n_frames(n) - 5, 0)
    assert n_frames(n) == O.n_frames(n)
    nxt = 0
    for r in range(world):
        sh = split_clip(n, r, world)
        assert sh.win_lo == nxt and sh.win_hi >= sh.win_lo
        nxt = sh.win_hi
        if sh.n_windows:
            assert 0 <= sh.sample_lo < sh.sample_hi <= n
            assert sh.sample_lo == 160 * sh.win_lo  # window w starts at frame w
            assert max(n_frames(sh.sample_hi - sh.sample_lo) - 5, 0) == sh.n_windows
    assert nxt == n_win


@fuzz(25)
@given(frames=st.integers(0, 60), extra=st.integers(0, 159), world=st.integers(1, 5),
       seed=st.integers(0, 2 ** 31))
def test_split_clip_labels_concatenate(frames, extra, world, seed):
    from vad_amd.dist import split_clip
    from vad_amd.ffn import TOPOLOGY_BL13, random_layers
    n = 160 * frames + 241 + extra if frames else extra
    clip = O.synth_clip(n, seed=seed, segment=400)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    lay = random_layers(TOPOLOGY_BL13, seed=1)

    def labels(x):
        if O.n_frames(len(x)) <= 5:
            return np.zeros((0,), np.int64)
        f = O.analyser_features_fast(O.mfcc_batch(x, fb))[:, :13]
        return O.ffn_labels(f, lay)

    whole = labels(clip)
    parts = []
    for r in range(world):
        sh = split_clip(n, r, world)
        if sh.n_windows:
            part = labels(clip[sh.sample_lo:sh.sample_hi])
            assert len(part) == sh.n_windows
            parts.append(part)
    got = np.concatenate(parts) if parts else np.zeros((0,), np.int64)
    np.testing.assert_array_equal(got, whole)


def _rows_disjoint_brute(S, K, block, hs, hl):
    starts = sorted(k * block + s * hs for k in range(K) for s in range(S))
    return all(b - a >= hl for a, b in zip(starts, starts[1:]))


@fuzz(200)
@given(S=st.integers(1, 12), K=st.integers(1, 9), hl=st.integers(1, 200),
       block=st.integers(-3000, 3000), gap=st.integers(0, 3000))
def test_hop_rows_disjoint_is_sound(S, K, block, gap, hl):
    """Rows of one hop never overlap: vad_stream_hops rejects hop_stride <
    hop_len before this rule applies, so the row stride is hl + gap."""
    from vad_amd.stream import hop_rows_disjoint
    hs = hl + gap
    if hop_rows_disjoint(S, K, block, hs, hl):
        assert _rows_disjoint_brute(S, K, block, hs, hl)


@fuzz(200)
@given(S=st.integers(1, 64), K=st.integers(1, 16), hl=st.integers(1, 400), pad=st.integers(0, 64))
def test_hop_rows_disjoint_accepts_contiguous_orderings(S, K, hl, pad):
    from vad_amd.stream import hop_rows_disjoint
    row = hl + pad
    assert hop_rows_disjoint(S, K, S * row, row, hl)   # (K, S, row): hop-major
    assert hop_rows_disjoint(S, K, row, K * row, hl)   # (S, K * row): stream-major


@fuzz(300)
@given(words=st.lists(st.integers(0, 2 ** 32 - 1), min_size=1, max_size=3 * 39),
       label=st.sampled_from([0, 1, 2]), n_cols=st.sampled_from([1, 3, 39]))
def test_csv_formatter_any_float32(words, label, n_cols):
    """vad_format_csv_rows (the native write_features formatter) against
    csv.writer over numpy's float32 str, on arbitrary float32 bit patterns:
    every exponent, subnormals, signed zeros, infinities and NaN payloads."""
    import csv
    import io
    from vad_amd import dataset as D
    k = len(words) // n_cols * n_cols
    if k == 0:
        return
    rows = np.asarray(words[:k], np.uint32).view(np.float32).reshape(-1, n_cols)
    s = io.StringIO()
    csv.writer(s).writerows([list(r) + [np.float64(label)] for r in rows])
    assert D.format_csv_rows(rows, label) == s.getvalue()


@fuzz(300)
@given(low=st.floats(0.0, 4000.0), span=st.floats(0.05, 1.0), fft_n=st.integers(2, 8192),
       n_filters=st.integers(1, 64), sr=st.sampled_from([8000, 16000, 22050, 44100, 48000]))
def test_mel_filterbanks_any_parameters(low, span, fft_n, n_filters, sr):
    """vad_amd.mfcc.get_mel_filterbanks (the host side of a plan, mfcc.py:5-56)
    equals the oracle's restatement bit for bit -- NaN where the reference
    divides 0 by 0 -- for any band, FFT length, filter count and rate."""
    import warnings
    from vad_amd import mfcc as M
    high = low + span * (sr / 2 - low)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        got = M.get_mel_filterbanks(low, high, fft_n, n_filters, sr)
        ref = O.get_mel_filterbanks(low, high, fft_n, n_filters, sr)
    assert got.shape == ref.shape == (n_filters, fft_n // 2)
    np.testing.assert_array_equal(got, ref)


@fuzz(150)
@given(count=st.integers(0, 3000), width=st.integers(1, 4), channels=st.integers(1, 2),
       rate=st.sampled_from([8000, 16000, 44100]), keep=st.floats(0.0, 1.0), seed=st.integers(0, 2 ** 32 - 1))
def test_sph_read_round_trip(tmp_path_factory, count, width, channels, rate, keep, seed):
    """dataset.sph_read (sph.py:33-64) on SPHERE files written here: nine
    header lines, then big-endian samples of any width; each sample is the
    low 16 bits of its big-endian value (the reference's int16 store), a
    truncated file leaves the missing samples 0."""
    from vad_amd import dataset as D
    rng = np.random.default_rng(seed)
    vals = [int(v) for v in rng.integers(0, 256 ** width, count, dtype=np.uint64)]
    header = [b"NIST_1A", b"   1024", b"sample_count -i %d" % count, b"sample_n_bytes -i %d" % width,
              b"channel_count -i %d" % channels, b"sample_byte_format -s2 10",
              b"sample_rate -i %d" % rate, b"sample_coding -s3 pcm", b"end_head"]
    body = b"".join(v.to_bytes(width, "big") for v in vals)
    cut = int(keep * len(body))
    p = tmp_path_factory.mktemp("sph") / "a.sph"
    p.write_bytes(b"\n".join(header) + b"\n" + body[:cut])
    s = D.sph_read(str(p))
    n_full = cut // width
    want = np.zeros(count, np.int16)
    want[:n_full] = np.array([v & 0xFFFF for v in vals[:n_full]], np.uint16).view(np.int16)
    assert (s.channels, s.framerate, s.sample_width) == (channels, rate, width)
    np.testing.assert_array_equal(s.data, want)
