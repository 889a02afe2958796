"""Host objects owning the device plans of libvad_amd (include/vad_amd.h).

``MfccPlan`` holds the filterbank/DCT/twiddle plan of one MFCC configuration
and runs the HIP MFCC kernel on device tensors; ``FfnPlan`` holds an FFN's
MFMA fragments.  Both are thin: all arithmetic happens in the HIP kernels.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr, stream_ptr
from .config import MfccConfig


def _device(dev=None):
    if dev is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return torch.device(dev)


def _require_cuda_tensor(t, name, dtype=torch.float32):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) torch tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def check_out(out, shape, dtype, device, name="out"):
    """A caller-supplied output must be exactly what the kernel writes: a
    contiguous tensor of this shape and dtype on the input's device (anything
    else would be an out-of-bounds or foreign-device write)."""
    if not isinstance(out, torch.Tensor) or not out.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) torch tensor")
    if out.device != torch.device(device):
        raise ValueError(f"{name} is on {out.device}, the input on {device}")
    if out.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {out.dtype}")
    if tuple(out.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(out.shape)}")
    if not out.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return out


def _out(out, shape, dtype, device, name="out"):
    if out is None:
        return torch.empty(shape, dtype=dtype, device=device)
    return check_out(out, shape, dtype, device, name)


def n_frames(n_samples, frame_size=400, hop=160):
    """Frames split_into_frames yields (file_processing.py:99: len - offset > size)."""
    return int(lib().vad_n_frames(int(n_samples), int(frame_size), int(hop)))


class MfccPlan:
    """MFCC plan for a (n_filters, 256) filterbank (mfcc.py:39-56) + mfcc_n + lifter."""

    def __init__(self, filterbank, mfcc_n=13, fft_n=512, lifter_L=22):
        fb = np.ascontiguousarray(np.asarray(filterbank, dtype=np.float64))
        if fb.ndim != 2 or fb.shape[1] != fft_n // 2:
            raise ValueError(f"filterbank must be (n_filters, {fft_n // 2}), got {fb.shape}")
        self.filterbank = fb
        self.n_filters = fb.shape[0]
        self.mfcc_n = int(mfcc_n)
        self.fft_n = int(fft_n)
        h = ctypes.c_void_p()
        check(lib().vad_mfcc_plan_create(fb.ctypes.data_as(ctypes.c_void_p), self.n_filters,
                                          self.fft_n, self.mfcc_n, int(lifter_L), ctypes.byref(h)),
              "vad_mfcc_plan_create")
        self._h = h
        self._destroy = lib().vad_mfcc_plan_destroy

    @classmethod
    def from_config(cls, cfg: MfccConfig = MfccConfig()):
        from .mfcc import get_mel_filterbanks
        fb = get_mel_filterbanks(cfg.low_hz, cfg.high_hz, cfg.fft_n, cfg.n_filters, cfg.sample_rate)
        plan = cls(fb, cfg.n_mfcc, cfg.fft_n, cfg.lifter)
        if cfg.window is not None:
            if cfg.window != "hamming":
                raise ValueError(f"unknown window {cfg.window!r} (None or 'hamming')")
            plan.set_window(np.hamming(cfg.frame_size))
        return plan

    def set_window(self, window):
        """Multiply every frame by `window` (<= 512 samples) before the FFT --
        an optional stage the reference does not have; None removes it."""
        if window is None:
            check(lib().vad_mfcc_plan_set_window(self._h, None, 0), "vad_mfcc_plan_set_window")
            return
        w = np.ascontiguousarray(np.asarray(window, np.float32).reshape(-1))
        check(lib().vad_mfcc_plan_set_window(self._h, w.ctypes.data_as(ctypes.c_void_p), w.size),
              "vad_mfcc_plan_set_window")

    @property
    def handle(self):
        return self._h

    @property
    def variant(self):
        """0 = runtime tables, 1/2 = compile-time Mel26/Mel40 kernel."""
        return int(lib().vad_mfcc_plan_variant(self._h))

    def set_variant(self, v):
        check(lib().vad_mfcc_plan_set_variant(self._h, int(v)), "vad_mfcc_plan_set_variant")

    def __del__(self):
        h = getattr(self, "_h", None)
        destroy = getattr(self, "_destroy", None)  # bound at creation: module globals
        if h is not None and h.value and destroy is not None:  # may be gone at exit
            destroy(h)
            self._h = None

    # -- frame sources ------------------------------------------------------
    @staticmethod
    def _frames_args(src, frame_len, frame_stride, n):
        if isinstance(src, torch.Tensor) and src.dtype == torch.int16:
            _require_cuda_tensor(src, "src", torch.int16)
        else:
            _require_cuda_tensor(src, "src")
        if src.dim() == 2 and frame_len is None:
            n, frame_len = src.shape
            frame_stride = frame_len
        if frame_len is None or frame_stride is None or n is None:
            raise ValueError("give a (n, frame_len) frame matrix or frame_len/frame_stride/n")
        if n > 0 and (n - 1) * frame_stride + min(frame_len, 512) > src.numel():
            raise ValueError("frames run past the end of src")
        return int(frame_len), int(frame_stride), int(n)

    def spec(self, src, frame_len=None, frame_stride=None, n=None, out=None, stream=None):
        """get_spec_mag (mfcc.py:59-61) of every frame -> (n, 256) fp32 (src fp32 or int16)."""
        frame_len, frame_stride, n = self._frames_args(src, frame_len, frame_stride, n)
        out = _out(out, (n, self.fft_n // 2), torch.float32, src.device)
        fn = "vad_spec_i16" if src.dtype == torch.int16 else "vad_spec_f32"
        check(getattr(lib(), fn)(self._h, ptr(src), frame_stride, frame_len, n, ptr(out),
                                 stream_ptr(stream)), fn)
        return out

    def mfcc(self, src, frame_len=None, frame_stride=None, n=None, out=None, stream=None):
        """get_mfcc (mfcc.py:67-69) of every frame -> (n, mfcc_n) fp32 (src fp32 or int16)."""
        frame_len, frame_stride, n = self._frames_args(src, frame_len, frame_stride, n)
        out = _out(out, (n, self.mfcc_n), torch.float32, src.device)
        fn = "vad_mfcc_i16" if src.dtype == torch.int16 else "vad_mfcc_f32"
        check(getattr(lib(), fn)(self._h, ptr(src), frame_stride, frame_len, n, ptr(out),
                                 stream_ptr(stream)), fn)
        return out

    def clip_mfcc(self, audio, frame_size=400, hop=160, out=None, stream=None):
        """MFCC of every frame split_into_frames takes from a clip (file_processing.py:80-103).

        `audio` is fp32, or int16 PCM (converted exactly on load, like the
        reference's astype(float32) of its int16 wav data, vad.py:37)."""
        _require_cuda_tensor(audio, "audio", audio.dtype if audio.dtype == torch.int16 else torch.float32)
        f = n_frames(audio.numel(), frame_size, hop)
        return self.mfcc(audio, frame_len=frame_size, frame_stride=hop, n=f, out=out, stream=stream)

    def from_spec(self, spec, out=None, stream=None):
        """get_mfcc_from_spec (mfcc.py:72-78) of (n, 256) spectra -> (n, mfcc_n)."""
        _require_cuda_tensor(spec, "spec")
        if spec.dim() != 2 or spec.shape[1] != self.fft_n // 2:
            raise ValueError("spec must be (n, 256)")
        n = spec.shape[0]
        out = _out(out, (n, self.mfcc_n), torch.float32, spec.device)
        check(lib().vad_mfcc_from_spec_f32(self._h, ptr(spec), n, ptr(out), stream_ptr(stream)),
              "vad_mfcc_from_spec_f32")
        return out


class FfnPlan:
    """Device fragments of a Keras-style MLP (ffn_trainer.py:106-116)."""

    def __init__(self, layers):
        self.layers = [(np.ascontiguousarray(np.asarray(w, np.float32)),
                        np.ascontiguousarray(np.asarray(b, np.float32)).reshape(-1))
                       for w, b in layers]
        dims = [self.layers[0][0].shape[0]] + [w.shape[1] for w, _ in self.layers]
        for (w, b), i, o in zip(self.layers, dims[:-1], dims[1:]):
            if w.shape != (i, o) or b.shape != (o,):
                raise ValueError(f"layer shapes do not chain: W {w.shape}, b {b.shape}")
        self.dims = dims
        n = len(self.layers)
        d = (ctypes.c_int32 * (n + 1))(*dims)
        wp = (ctypes.c_void_p * n)(*[w.ctypes.data for w, _ in self.layers])
        bp = (ctypes.c_void_p * n)(*[b.ctypes.data for _, b in self.layers])
        h = ctypes.c_void_p()
        check(lib().vad_ffn_plan_create(n, d, wp, bp, ctypes.byref(h)), "vad_ffn_plan_create")
        self._h = h
        self._destroy = lib().vad_ffn_plan_destroy

    @property
    def handle(self):
        return self._h

    @property
    def in_dim(self):
        return self.dims[0]

    @property
    def n_classes(self):
        return self.dims[-1]

    @property
    def arith(self):
        """"split_f16" (v_mfma_f32_16x16x32_f16 on hi/lo f16 halves of every
        operand, the specialised topologies' default) or "f32" (exact f32 MFMA)."""
        return "split_f16" if lib().vad_ffn_plan_arith(self._h) == _lib.FFN_SPLIT_F16 else "f32"

    def set_arith(self, arith):
        code = {"split_f16": _lib.FFN_SPLIT_F16, "f32": _lib.FFN_EXACT_F32}[arith]
        check(lib().vad_ffn_plan_set_arith(self._h, code), "vad_ffn_plan_set_arith")

    def __del__(self):
        h = getattr(self, "_h", None)
        destroy = getattr(self, "_destroy", None)  # bound at creation: module globals
        if h is not None and h.value and destroy is not None:  # may be gone at exit
            destroy(h)
            self._h = None

    def predict(self, x, out=None, stream=None):
        """Labels (uint8) of feature rows x (n, in_dim) fp32 on the device."""
        _require_cuda_tensor(x, "x")
        if x.dim() != 2 or x.shape[1] != self.in_dim:
            raise ValueError(f"x must be (n, {self.in_dim})")
        n = x.shape[0]
        out = _out(out, (n,), torch.uint8, x.device)
        check(lib().vad_ffn_predict(self._h, ptr(x), n, ptr(out), stream_ptr(stream)),
              "vad_ffn_predict")
        return out

    def window_labels(self, mfcc, mode=_lib.FEAT_ANALYSER, out=None, stream=None):
        """Labels of every 5-frame window of an MFCC sequence (F-5 rows)."""
        _require_cuda_tensor(mfcc, "mfcc")
        f, c = mfcc.shape
        rows = max(f - 5, 0)
        out = _out(out, (rows,), torch.uint8, mfcc.device)
        check(lib().vad_features_ffn(self._h, ptr(mfcc), f, c, int(mode), ptr(out),
                                     stream_ptr(stream)), "vad_features_ffn")
        return out


def preemphasis(x, coeff, out=None, stream=None):
    """y[0] = x[0], y[t] = x[t] - coeff x[t-1] of a device fp32 clip (1-D) or
    of every row of a frame matrix (2-D): an optional stage, not in the
    reference."""
    _require_cuda_tensor(x, "x")
    rows, n = (1, x.numel()) if x.dim() == 1 else tuple(x.shape)
    if out is None and stream is not None:
        # allocated on the stream that writes (and, in VadPipeline, reads) it:
        # the caching allocator may not hand it to other streams' work early
        with torch.cuda.stream(stream):
            out = torch.empty(tuple(x.shape), dtype=torch.float32, device=x.device)
    out = _out(out, tuple(x.shape), torch.float32, x.device)
    check(lib().vad_preemphasis_f32(ptr(x), ptr(out), rows, n, n, ctypes.c_float(coeff), stream_ptr(stream)),
          "vad_preemphasis_f32")
    return out


def window_logits(ffn_plan, mfcc, mode=_lib.FEAT_ANALYSER, stream=None):
    """(labels uint8 (F-5,), logits fp32 (F-5, n_classes)) of every window of
    an MFCC sequence, from the same kernel as FfnPlan.window_labels."""
    _require_cuda_tensor(mfcc, "mfcc")
    f, c = mfcc.shape
    rows = max(f - 5, 0)
    labels = torch.empty((rows,), dtype=torch.uint8, device=mfcc.device)
    logits = torch.empty((rows, ffn_plan.n_classes), dtype=torch.float32, device=mfcc.device)
    check(lib().vad_features_ffn_logits(ffn_plan.handle, ptr(mfcc), f, c, int(mode), ptr(labels), ptr(logits),
                                        stream_ptr(stream)), "vad_features_ffn_logits")
    return labels, logits


def window_features(mfcc, mode=_lib.FEAT_ANALYSER, out=None, stream=None):
    """(F-5, 3*n) feature rows of an (F, n) MFCC sequence (analyser or offline form)."""
    _require_cuda_tensor(mfcc, "mfcc")
    f, c = mfcc.shape
    rows = max(f - 5, 0)
    out = _out(out, (rows, 3 * c), torch.float32, mfcc.device)
    check(lib().vad_features_f32(ptr(mfcc), f, c, int(mode), ptr(out), stream_ptr(stream)),
          "vad_features_f32")
    return out
