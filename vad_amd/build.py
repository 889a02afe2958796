"""Build libvad_amd.so (gfx950) in-tree with hipcc.

    python -m vad_amd.build            # or __graft_entry__.build()

The library is one hipcc link of the .hip translation units under csrc/;
it lands in vad_amd/lib/ (git-ignored, but shipped to the GPU box by gpurun).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libvad_amd.so")
ARCH = os.environ.get("VAD_OFFLOAD_ARCH", "gfx950")
SOURCES = ["capi.hip", "mfcc_kernel.hip", "ffn_kernel.hip", "tree_kernel.hip",
           "dataset_kernel.hip", "csv_format.hip", "simple_kernel.hip", "stream_kernel.hip", "rccl.hip",
           "spec_generic.hip"]
# per-translation-unit code-generation flags: the FFT's packed-fp32 chains
# run ~5% faster under the ILP-oriented machine scheduler (fewer dependent
# pairs back to back, i.e. fewer hazard s_nops and stalls)
UNIT_FLAGS = {
    "mfcc_kernel.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "ffn_kernel.hip": [],
    "tree_kernel.hip": [],
    "dataset_kernel.hip": [],
    "csv_format.hip": [],
    "simple_kernel.hip": [],
    "stream_kernel.hip": [],
    "capi.hip": [],
    "rccl.hip": [],
    "spec_generic.hip": [],
}


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "vad_amd.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, defines=(), out=None):
    """Build the library; ``defines`` / ``out`` make an experiment variant
    (e.g. ``-DVAD_SPLIT_LOADS=0`` into lib/libvad_amd_<name>.so)."""
    lib = out or LIB
    if out is None and not force and not needs_build():
        return LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    base = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function"]
    # experiment variants: VAD_UNIT_FLAGS="unit.hip:-flag,-flag;unit2.hip:..." adds per-unit flags
    extra = {}
    for item in filter(None, os.environ.get("VAD_UNIT_FLAGS", "").split(";")):
        unit, _, flags = item.partition(":")
        extra[unit] = flags.split(",")
    procs, objs = [], []
    for name in SOURCES:  # one object per unit, compiled in parallel
        obj = os.path.join(LIB_DIR, os.path.basename(lib) + "." + name.replace(".hip", ".o"))
        cmd = base + list(defines) + UNIT_FLAGS.get(name, []) + extra.get(name, []) + \
            ["-c", os.path.join(CSRC, name), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc -c")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp"] + objs + ["-ldl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    for obj in objs:
        os.remove(obj)
    return lib


C_HOST_DIR = os.path.join(os.path.dirname(HERE), "tests", "c_host")


def build_c_host(verbose=True):
    """The plain-C test host (tests/c_host): gcc against include/vad_amd.h and
    the in-tree library, built here so GPU runs only execute it; and the
    test-only LDS-poisoning helper (liblds_poison.so)."""
    cmd = ["make", "-C", C_HOST_DIR, "-s", "capi_host", "liblds_poison.so"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return os.path.join(C_HOST_DIR, "capi_host")


if __name__ == "__main__":
    args = sys.argv[1:]
    if "--variant" in args:  # python -m vad_amd.build --variant NAME -DX=1 ...
        name = args[args.index("--variant") + 1]
        build(defines=[a for a in args if a.startswith("-D")],
              out=os.path.join(LIB_DIR, f"libvad_amd_{name}.so"))
    else:
        build(force="--force" in args)
