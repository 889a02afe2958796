"""ctypes binding of libvad_amd.so (include/vad_amd.h).

torch is imported first so that libamdhip64.so.7 resolves to the copy torch
already loaded: the library and PyTorch then share one HIP runtime, one
device context and the same streams.  There is no fallback: if the library
is missing or a call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VAD_AMD_LIB", os.path.join(_HERE, "lib", "libvad_amd.so"))

VAD_OK = 0
VAD_EINVAL = -1
VAD_EUNSUPPORTED = -2
VAD_ENOMEM = -3
VAD_ERCCL = -4
FEAT_ANALYSER = 0
FEAT_OFFLINE = 1
FFN_EXACT_F32 = 0
FFN_SPLIT_F16 = 1

c_i32, c_i64, c_vp, c_sz = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t
c_int = ctypes.c_int

# name -> (restype, argtypes); every symbol include/vad_amd.h declares
SIGNATURES = {
    "vad_version": (ctypes.c_char_p, []),
    "vad_n_frames": (c_i64, [c_i64, c_i32, c_i32]),
    "vad_mfcc_plan_create": (c_int, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp]),
    "vad_mfcc_plan_destroy": (c_int, [c_vp]),
    "vad_mfcc_plan_variant": (c_i32, [c_vp]),
    "vad_mfcc_plan_set_variant": (c_int, [c_vp, c_i32]),
    "vad_mfcc_plan_set_window": (c_int, [c_vp, c_vp, c_i32]),
    "vad_preemphasis_f32": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, ctypes.c_float, c_vp]),
    "vad_spec_f32": (c_int, [c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp]),
    "vad_mfcc_f32": (c_int, [c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp]),
    "vad_spec_i16": (c_int, [c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp]),
    "vad_mfcc_i16": (c_int, [c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp]),
    "vad_mfcc_from_spec_f32": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "vad_ffn_plan_create": (c_int, [c_i32, c_vp, c_vp, c_vp, c_vp]),
    "vad_ffn_plan_destroy": (c_int, [c_vp]),
    "vad_ffn_plan_arith": (c_i32, [c_vp]),
    "vad_ffn_plan_set_arith": (c_int, [c_vp, c_i32]),
    "vad_features_f32": (c_int, [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "vad_features_ffn": (c_int, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "vad_features_ffn_logits": (c_int, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp]),
    "vad_ffn_predict": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "vad_tree_plan_create": (c_int, [c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "vad_tree_plan_destroy": (c_int, [c_vp]),
    "vad_tree_predict": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp]),
    "vad_features_tree": (c_int, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp]),
    "vad_simple_features": (c_int, [c_vp, c_i64, c_i32, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp,
                                    c_vp]),
    "vad_scale_workspace_bytes": (c_sz, []),
    "vad_scale_features": (c_int, [c_vp, c_i64, c_i32, c_vp, c_sz, c_vp]),
    "vad_format_csv_rows": (c_i64, [c_vp, c_i64, c_i32, ctypes.c_double, c_vp, c_i64]),
    "vad_mfcc_ffn_workspace_bytes": (c_sz, [c_vp, c_vp, c_i64, c_i32, c_i32]),
    "vad_mfcc_ffn": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_sz,
                             c_vp]),
    "vad_mfcc_ffn_i16": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_vp, c_vp, c_sz,
                                 c_vp]),
    "vad_mfcc_ffn_fusable": (c_i32, [c_vp, c_vp, c_i32, c_i32]),
    "vad_stream_ring_floats": (c_i64, [c_i64, c_i32]),
    "vad_stream_push_hop": (c_int, [c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_i64, c_vp]),
    "vad_stream_hop": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp,
                               c_vp]),
    "vad_stream_hops": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_i64, c_i32, c_i64, c_vp,
                                c_vp, c_vp, c_i64, c_vp]),
    "vad_stream_step": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp,
                                c_vp]),
    "vad_graph_launch": (c_int, [c_vp, c_vp]),
    "vad_graph_plan_create": (c_int, [c_vp, c_vp, c_vp]),
    "vad_graph_plan_launch": (c_int, [c_vp, c_vp]),
    "vad_graph_plan_direct": (c_i32, [c_vp]),
    "vad_graph_plan_destroy": (c_int, [c_vp]),
    "vad_rccl_available": (c_int, []),
    "vad_rccl_error_string": (ctypes.c_char_p, []),
    "vad_rccl_unique_id": (c_int, [c_vp]),
    "vad_rccl_init": (c_int, [c_vp, c_i32, c_vp, c_i32]),
    "vad_rccl_gather_u8": (c_int, [c_vp, c_vp, c_vp, c_sz, c_i32, c_vp]),
    "vad_rccl_destroy": (c_int, [c_vp]),
}


class VadError(RuntimeError):
    """A libvad_amd call failed (negative VAD_E* code or a hipError_t)."""


_lib = None


def lib():
    """The loaded library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libvad_amd.so not found at {LIB_PATH}: build it with "
                "`python -m vad_amd.build` (there is no CPU fallback)")
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(code, what):
    if code != VAD_OK:
        names = {VAD_EINVAL: "invalid argument", VAD_EUNSUPPORTED: "unsupported configuration",
                 VAD_ENOMEM: "out of memory"}
        if code == VAD_ERCCL:
            raise VadError(f"{what} failed: RCCL: {lib().vad_rccl_error_string().decode()}")
        raise VadError(f"{what} failed: {names.get(code, f'hipError_t {code}')}")


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(stream=None):
    """hipStream_t of a torch stream (default: the current stream of the
    current device, read without building a Stream object: this sits on
    every per-hop launch path)."""
    if stream is None and _raw_stream is not None:
        return ctypes.c_void_p(_raw_stream(torch.cuda.current_device()))
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
