"""A non-Python host on the C ABI: tests/c_host/capi_host (plain C against
include/vad_amd.h, built on the CPU by ``vad_amd.build.build_c_host``) reads
oracle-made inputs from files and checks vad_mfcc_f32, vad_mfcc_ffn (both
clip forms), the clip as one stream through vad_stream_hops (8 hops per call)
and a world-size-1 vad_rccl gather, the way a cgo / JNI binding of
the reference's path (mfcc.py:67-78, sklearn_analyser.py:46-82) would call
them.  It runs as a child process, so it owns its own HIP context."""
import os
import subprocess

import numpy as np
import pytest

from oracle import vad_oracle as O

pytestmark = pytest.mark.gpu

HOST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_host", "capi_host")


def test_c_host_against_oracle(tmp_path):
    assert os.path.exists(HOST), "tests/c_host/capi_host not built (vad_amd.build.build_c_host)"
    from vad_amd.ffn import TOPOLOGY_BL13, random_layers
    F = 30_000  # several 64-frame tiles per workgroup of the persistent loop
    clip = O.synth_clip(O.samples_for_frames(F), seed=71)
    fb = O.get_mel_filterbanks(300, 8000, 512, 26, 16000)
    ref = O.mfcc_batch(clip, fb)
    layers = random_layers(TOPOLOGY_BL13, seed=5)
    x = O.analyser_features_fast(ref)[:, :13]
    lab = O.ffn_labels(x, layers).astype(np.uint8)
    lab[~(O.ffn_margin(x, layers) > 0.05)] = 255  # 255 = not decisive, unchecked
    np.ascontiguousarray(fb, np.float64).tofile(tmp_path / "fb.f64")
    np.ascontiguousarray(clip, np.float32).tofile(tmp_path / "audio.f32")
    np.ascontiguousarray(ref, np.float32).tofile(tmp_path / "mfcc_ref.f32")
    np.concatenate([np.concatenate([np.asarray(W, np.float32).ravel(), np.asarray(b, np.float32).ravel()])
                    for W, b in layers]).tofile(tmp_path / "ffn.f32")
    lab.tofile(tmp_path / "labels_ref.u8")
    r = subprocess.run([HOST, str(tmp_path)], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "all checks passed" in r.stdout
