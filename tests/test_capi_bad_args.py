"""Every C-ABI entry refuses bad arguments without touching them: null
handles and pointers with otherwise valid sizes, and negative sizes, return a
negative VAD_E* code (or the documented neutral value), never crash.  Runs on
the CPU: every refusal must happen before any HIP call.  The calls run in a
child process, so a crash fails this test instead of the test run."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes, json, sys
sys.path.insert(0, sys.argv[1])
from vad_amd import _lib
L = _lib.lib()
N = None  # NULL
res = {}
def call(name, *args):
    res[name + repr(args)] = int(getattr(L, name)(*args))
# plans: NULL handle, everything else valid-looking
call("vad_mfcc_plan_create", N, 26, 512, 13, 22, N)
call("vad_mfcc_plan_set_variant", N, 1)
call("vad_mfcc_plan_set_window", N, N, 400)
call("vad_preemphasis_f32", N, N, 1, 100, 100, 0.97, N)
call("vad_preemphasis_f32", N, N, -1, 100, 100, 0.97, N)
for fn in ("vad_spec_f32", "vad_mfcc_f32", "vad_spec_i16", "vad_mfcc_i16"):
    call(fn, N, N, 160, 400, 10, N, N)
    call(fn, N, N, 160, 400, -1, N, N)
call("vad_mfcc_from_spec_f32", N, N, 10, N, N)
call("vad_ffn_plan_create", 3, N, N, N, N)
call("vad_ffn_plan_create", -1, N, N, N, N)
call("vad_ffn_plan_set_arith", N, 1)
call("vad_features_f32", N, 10, 13, 0, N, N)
call("vad_features_f32", N, -1, 13, 0, N, N)
call("vad_features_ffn", N, N, 10, 13, 0, N, N)
call("vad_features_ffn_logits", N, N, 10, 13, 0, N, N, N)
call("vad_ffn_predict", N, N, 10, N, N)
call("vad_tree_plan_create", 3, N, N, N, N, N, N, 39, N)
call("vad_tree_plan_create", -1, N, N, N, N, N, N, 39, N)
call("vad_tree_predict", N, N, 10, N, N)
call("vad_features_tree", N, N, 10, 13, 0, N, N)
call("vad_simple_features", N, 10, 400, 400, 512, 56, 32, 4, N, N)
call("vad_simple_features", N, 10, 400, 400, 9000, 56, 32, 4, N, N)
call("vad_scale_features", N, 10, 13, N, 1 << 20, N)
call("vad_scale_features", N, -1, 13, N, 1 << 20, N)
call("vad_mfcc_ffn", N, N, N, 100000, 400, 160, 0, N, N, 0, N)
call("vad_mfcc_ffn_i16", N, N, N, 100000, 400, 160, 0, N, N, 0, N)
call("vad_stream_push_hop", N, 400, 400, N, 160, 160, 10, N)
call("vad_stream_push_hop", N, 400, 400, N, 160, 500, 10, N)
call("vad_stream_hop", N, N, N, 400, 400, N, 160, 160, 10, N, N, N, N)
call("vad_stream_hops", N, N, N, 400, 400, N, 160, 160, 10, 8, 1600, N, N, N, 10, N)
call("vad_stream_step", N, N, N, 400, 400, 10, N, N, N, N, N)
call("vad_graph_launch", N, N)
call("vad_graph_plan_create", N, N, N)
call("vad_graph_plan_launch", N, N)
call("vad_rccl_init", N, 1, N, 0)
call("vad_rccl_gather_u8", N, N, N, 10, 0, N)
# neutral values
neutral = {
    "vad_mfcc_plan_destroy": int(L.vad_mfcc_plan_destroy(N)),
    "vad_ffn_plan_destroy": int(L.vad_ffn_plan_destroy(N)),
    "vad_tree_plan_destroy": int(L.vad_tree_plan_destroy(N)),
    "vad_rccl_destroy": int(L.vad_rccl_destroy(N)),
    "vad_mfcc_plan_variant": int(L.vad_mfcc_plan_variant(N)),
    "vad_mfcc_ffn_fusable": int(L.vad_mfcc_ffn_fusable(N, N, 400, 160)),
    "vad_mfcc_ffn_workspace_bytes": int(L.vad_mfcc_ffn_workspace_bytes(N, N, 100000, 400, 160)),
    "vad_n_frames_neg": int(L.vad_n_frames(-5, 400, 160)),
    "vad_stream_ring_floats_neg": int(L.vad_stream_ring_floats(-1, 13)),
    "vad_format_csv_rows_null": int(L.vad_format_csv_rows(N, 3, 39, 1.0, N, 100)),
}
print(json.dumps({"calls": res, "neutral": neutral}))
'''


def test_every_entry_refuses_bad_arguments():
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], capture_output=True, text=True, timeout=300,
                       cwd=REPO)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    bad = {k: v for k, v in out["calls"].items() if v >= 0}
    assert not bad, bad  # every refusal is a negative VAD_E* code
    n = out["neutral"]
    for k in ("vad_mfcc_plan_destroy", "vad_ffn_plan_destroy", "vad_tree_plan_destroy", "vad_rccl_destroy"):
        assert n[k] == 0, k  # destroy(NULL) is a no-op
    assert n["vad_mfcc_plan_variant"] < 0
    assert n["vad_mfcc_ffn_fusable"] == 0
    assert n["vad_mfcc_ffn_workspace_bytes"] == 0
    assert n["vad_n_frames_neg"] == 0
    assert n["vad_stream_ring_floats_neg"] <= 0
    assert n["vad_format_csv_rows_null"] < 0
