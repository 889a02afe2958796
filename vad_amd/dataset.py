"""Offline dataset export, GPU edition of the reference's dataset pipeline
(dataset_creator.py:58-66 -> Pool.map(process_file) -> scale_features ->
write_features).

Same functions and argument conventions as the reference modules:

  dataset/sph.py             ``sph_read`` (class ``Sph``)
  dataset/stm_parser.py      ``stm_parse``, ``get_samples_indices``
  dataset/file_processing.py ``split_into_frames`` (with STM segments),
                             ``process_file``, ``create_table_header``,
                             ``write_features``
  dataset/utils.py           ``scale_features``

The MFCC / delta features run on the GPU (one clip per call, the offline
feature rows of ``vad_features_f32``), ``scale_features`` is a device
reduction (``vad_scale_features``), and the CSV text is produced by a native
multithreaded formatter (``vad_format_csv_rows``) that prints values exactly
as numpy prints float32.  ``write_features`` keeps the reference's
``csv.writer`` interface.
"""
from __future__ import annotations

import csv
import ctypes

import numpy as np
import torch

from . import _lib
from .config import MfccConfig
from .pipeline import VadPipeline

# ----------------------------------------------------------------------------
# dataset/sph.py
# ----------------------------------------------------------------------------


class Sph:
    """sph.py:9-30."""

    def __init__(self, channels, framerate, sample_width, data):
        self._channels = channels
        self._framerate = framerate
        self._sample_width = sample_width
        self._data = data

    @property
    def channels(self):
        return self._channels

    @property
    def framerate(self):
        return self._framerate

    @property
    def sample_width(self):
        return self._sample_width

    @property
    def data(self):
        return self._data


def sph_read(fname):
    """sph.py:33-64: nine header lines (sample_count, sample_n_bytes,
    channel_count, sample_rate taken from lines 3, 4, 5, 7, third field),
    then big-endian samples right after them, stored into int16 (wrapping, as
    the reference's numpy-1 assignment did).  At most sample_count samples;
    a truncated file yields fewer (the rest stay 0)."""
    with open(fname, "rb") as f:
        header = [f.readline(1024) for _ in range(9)]
        samples_num = int(header[2].split(b" ")[2])
        sample_width = int(header[3].split(b" ")[2])
        channels = int(header[4].split(b" ")[2])
        framerate = int(header[6].split(b" ")[2])
        raw = f.read(samples_num * sample_width)
    n = len(raw) // sample_width
    b = np.frombuffer(raw[:n * sample_width], np.uint8).reshape(n, sample_width).astype(np.uint64)
    v = np.zeros(n, np.uint64)
    for j in range(sample_width):  # big-endian: byte j carries bits 8*(w-1-j)
        v |= b[:, j] << np.uint64(8 * (sample_width - 1 - j))
    samples = np.zeros((samples_num,), dtype=np.int16)
    samples[:n] = (v & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16)
    return Sph(channels, framerate, sample_width, samples)


# ----------------------------------------------------------------------------
# dataset/stm_parser.py
# ----------------------------------------------------------------------------
def stm_parse(fname):
    """stm_parser.py:5-19: [starts, ends] float32 of every STM line with >= 7
    space-separated fields whose 7th is not ignore_time_segment_in_scoring."""
    starts, ends = [], []
    with open(fname, "rb") as f:
        for line in iter(lambda: f.readline(1024), b""):
            items = line.split(b" ")
            if len(items) < 7 or items[6].strip() == b"ignore_time_segment_in_scoring":
                continue
            starts.append(np.float32(items[3]))
            ends.append(np.float32(items[4]))
    return [np.array(starts, np.float32), np.array(ends, np.float32)]


def get_samples_indices(fname, samplerate=16384):
    """stm_parser.py:22-26: float32 seconds x rate -> int32 (truncation)."""
    starts, ends = stm_parse(fname)
    return ((starts * samplerate).astype(np.int32, copy=False),
            (ends * samplerate).astype(np.int32, copy=False))


# ----------------------------------------------------------------------------
# dataset/file_processing.py
# ----------------------------------------------------------------------------
def read_audio(fname):
    """file_processing.py:26-35: (sample_rate, samples) of a .wav or .sph."""
    if fname.endswith(".wav"):
        from scipy.io import wavfile
        return wavfile.read(fname)
    if fname.endswith(".sph"):
        s = sph_read(fname)
        return s.framerate, s.data
    raise ValueError("Wrong file format: " + str(fname))


def gather_segments(data, transcription_path, frame_rate):
    """file_processing.py:87-94: concatenation of data[start:end] over the
    transcript's segments (int16, as the reference's new_data)."""
    starts, ends = get_samples_indices(transcription_path, frame_rate)
    parts = [np.asarray(data[s:e]) for s, e in zip(starts, ends)]
    return np.concatenate([np.array([], np.int16)] + parts) if parts else np.array([], np.int16)


def split_into_frames(data, frame_size, step, transcription_path=None, frame_rate=None):
    """file_processing.py:80-103: frames data[o:o+size] while len - o > size,
    after gathering the transcript's segments when a transcript is given."""
    if transcription_path and frame_rate:
        data = gather_segments(data, transcription_path, frame_rate)
    elif transcription_path and frame_rate is None:
        raise Exception('You must specify frame_rate')
    frames, offset = [], 0
    while len(data) - offset > frame_size:
        frames.append(data[offset:offset + frame_size])
        offset += step
    return frames


_PIPES = {}


def _pipeline(frame_size, frame_step, fft_n, n_filters, mfcc_num):
    key = (frame_size, frame_step, fft_n, n_filters, mfcc_num)
    if key not in _PIPES:
        cfg = MfccConfig(frame_size=frame_size, hop=frame_step, fft_n=fft_n,
                         n_filters=n_filters, n_mfcc=mfcc_num)
        _PIPES[key] = VadPipeline(cfg=cfg, mode="offline")
    return _PIPES[key]


def file_features(fname, frame_size=400, frame_step=160, fft_n=512, n_filters=26, mfcc_num=13,
                  transcription_path=None, device_out=False):
    """Feature rows of one file as a (F-5, 3*mfcc_num) float32 array (or a
    device tensor): process_file's features without the per-row tuples."""
    rate, raw = read_audio(fname)
    if transcription_path:
        raw = gather_segments(raw, transcription_path, rate)
    pipe = _pipeline(frame_size, frame_step, fft_n, n_filters, mfcc_num)
    a = torch.from_numpy(np.ascontiguousarray(np.asarray(raw))).cuda()
    if a.dtype != torch.int16:
        a = a.float()
    feats = _lib_window_features(pipe.mfcc(a), _lib.FEAT_OFFLINE)
    return feats if device_out else feats.cpu().numpy()


def _lib_window_features(mfcc, mode):
    from .plan import window_features
    return window_features(mfcc, mode)


def process_file(args):
    """file_processing.py:14-77 with the same argument list
    [fname, frame_size, frame_step, fft_n, mel_filterbank, mfcc_num,
    counter_queue, transcription_path]: the list of (mfcc, delta1, delta2)
    float64 tuples of the file.  mel_filterbank must be the reference
    filterbank of the (low, high, n_filters) configuration (its row count
    selects n_filters); counter_queue may be None."""
    fname, frame_size, frame_step, fft_n, fbank, mfcc_num = args[:6]
    counter_queue = args[6] if len(args) > 6 else None
    transcription_path = args[7] if len(args) > 7 else None
    f = file_features(fname, frame_size, frame_step, fft_n, int(np.asarray(fbank).shape[0]),
                      mfcc_num, transcription_path).astype(np.float64)
    c = mfcc_num
    features = [(r[:c], r[c:2 * c], r[2 * c:]) for r in f]
    if counter_queue is not None:
        processed = counter_queue.get() + 1
        if processed % 5 == 0:
            print("Processed " + str(processed) + ' files')
        counter_queue.put(processed)
    return features


def create_table_header(mfcc_len):
    """file_processing.py:106-123."""
    return ([f'MFCC Coef{i + 1}' for i in range(mfcc_len)]
            + [f'First delta{i + 1}' for i in range(mfcc_len)]
            + [f'Second delta{i + 1}' for i in range(mfcc_len)] + ['voiced'])


def write_features(writer, features, label):
    """file_processing.py:126-146: one csv row per window (features, label)."""
    for file_features_ in features:
        rows = [np.concatenate((fr[0], fr[1], fr[2], [label])) for fr in file_features_]
        writer.writerows(rows)


def format_csv_rows(rows, label):
    """CSV text (str) of float32 feature rows (n, 3*C) and one label, exactly
    as write_features + csv.writer print them for float32 values; native,
    multithreaded."""
    x = np.ascontiguousarray(np.asarray(rows, np.float32))
    if x.ndim != 2:
        raise ValueError("rows must be (n, n_cols)")
    n, k = x.shape
    if n == 0:
        return ""
    cap = n * (k * 24 + 48)
    buf = ctypes.create_string_buffer(cap)
    w = _lib.lib().vad_format_csv_rows(x.ctypes.data, n, k, float(label), buf, cap)
    if w < 0:
        raise _lib.VadError("vad_format_csv_rows: buffer too small")
    return buf.raw[:w].decode("ascii")


def write_feature_rows(fobj, rows, label):
    """Fast write_features for one (n, 3*C) array: appends its CSV text."""
    fobj.write(format_csv_rows(rows, label))


# ----------------------------------------------------------------------------
# dataset/utils.py
# ----------------------------------------------------------------------------
_SCALE_WS = {}


def scale_rows_device(rows):
    """scale_features on a device (n, 3*C) fp32 tensor, in place; returns
    (mean[3], std[3]) as float64 numpy arrays."""
    if not (isinstance(rows, torch.Tensor) and rows.is_cuda and rows.dtype == torch.float32
            and rows.is_contiguous() and rows.dim() == 2 and rows.shape[1] % 3 == 0):
        raise TypeError("rows must be a contiguous (n, 3*C) float32 CUDA tensor")
    lib = _lib.lib()
    nb = int(lib.vad_scale_workspace_bytes())
    dev = rows.device
    ws = _SCALE_WS.get(dev)
    if ws is None:
        ws = _SCALE_WS[dev] = torch.zeros((nb // 8,), dtype=torch.float64, device=dev)
    _lib.check(lib.vad_scale_features(_lib.ptr(rows), rows.shape[0], rows.shape[1] // 3,
                                      _lib.ptr(ws), nb, _lib.stream_ptr()), "vad_scale_features")
    st = ws[-6:].cpu().numpy()
    return st[:3].copy(), st[3:].copy()


def scale_features(features):
    """utils.py:5-34: global mean / std per group (mfcc, delta1, delta2) over
    every value of the chunk, then (x - mean) / std.  Accepts the reference
    structure (list of files of lists of (mfcc, d1, d2) tuples, modified in
    place and returned, like the reference) or an (n, 3*C) / (n, 3, C) array
    (a scaled float32 copy is returned).  The statistics run on the GPU."""
    if isinstance(features, np.ndarray) or isinstance(features, torch.Tensor):
        x = torch.as_tensor(np.asarray(features, np.float32) if isinstance(features, np.ndarray)
                            else features).float()
        shape = x.shape
        t = x.reshape(shape[0], -1).contiguous().cuda()
        scale_rows_device(t)
        return t.cpu().numpy().reshape(shape)
    rows = [np.concatenate(fr) for ff in features for fr in ff]
    if not rows:
        return features
    c = len(features[0][0][0]) if features and features[0] else len(rows[0]) // 3
    t = torch.from_numpy(np.asarray(rows, np.float32)).cuda()
    scale_rows_device(t)
    scaled = t.cpu().numpy().astype(np.float64)
    i = 0
    for ff in features:
        for fr in ff:
            for g in range(3):
                fr[g][:] = scaled[i, g * c:(g + 1) * c]
            i += 1
    return features
