"""Build libewk.so (HIP kernels + C ABI) for gfx950, in-tree.

    python -m easywakeword_amd.build        # or __graft_entry__.build()

hipcc cross-compiles for gfx950 without a GPU.  The .so lands next to this
file so it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["ewk_mfcc.hip", "ewk_gate.hip", "ewk_level3.hip", "ewk_gather.hip", "ewk_engine.cpp", "ewk_tables.cpp"]
HEADERS = ["ewk_internal.h", "ewk_gate.h", "ewk_rescore.h", "ewk_db64.h", os.path.join("..", "..", "include", "ewk.h")]
LIB = os.path.join(HERE, "libewk.so")
ARCH = os.environ.get("EWK_OFFLOAD_ARCH", "gfx950")
# Per-source flags.  The scorer is VALU-issue bound: SLP-packed f32 ops (v_pk_add_f32)
# cost more issue slots than the two scalar ops they replace on gfx950 and force
# register-pair moves (-3.3 % k_score_f32 time without them).
EXTRA = {"ewk_mfcc.hip": ["-fno-slp-vectorize"]}


def _hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.isabs(c) and os.path.exists(c):
            return c
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, out: str = None, defines=()) -> str:
    """Compile every source for gfx950 and link libewk.so (or `out`)."""
    lib = out or LIB
    if out is None and not force and not needs_build():
        return LIB
    objs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.rsplit(".", 1)[0] + ".o")
        obj = obj + "".join(f".{d}" for d in defines).replace("=", "_")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-function"] + EXTRA.get(src, []) + [f"-D{d}" for d in defines] + \
            ["-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        objs.append(obj)
    tmp = lib + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


ROOT = os.path.dirname(HERE)
C_HOST_SRC = os.path.join(ROOT, "examples", "c_positives_rccl.cpp")
C_HOST_BIN = os.path.join(ROOT, "examples", "c_positives_rccl")


def build_c_host(verbose: bool = False) -> str:
    """The C-host example (examples/c_positives_rccl.cpp): libewk.so + RCCL, no Python."""
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
           C_HOST_SRC, "-L", HERE, "-lewk", "-lrccl", "-Wl,-rpath,$ORIGIN/../easywakeword_amd", "-o", C_HOST_BIN]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return C_HOST_BIN


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
