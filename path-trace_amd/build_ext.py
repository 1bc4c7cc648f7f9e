"""Builds libpt.so (the C-ABI runtime) in-tree with hipcc for gfx950 hosts.

    python path-trace_amd/build_ext.py

The per-scene megakernels are generated at run time and compiled for gfx950
by hiprtc (csrc/jit.cpp); `precompile()` fills the code-object cache for the
benchmark scenes so a GPU box only loads them.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libpt.so")
SOURCES = ["runtime.cpp", "codegen.cpp", "jit.cpp", "imageio.cpp", "devsrc.cpp"]
HEADERS = ["internal.h", "device/pt_device.h", "../../include/pt/pt.h", "../../include/pt/pt_engine.h"]


def _embed_device_header() -> None:
    for name, inc in (("pt_device.h", "pt_device_src.inc"), ("pt_user_object.h", "pt_user_object_src.inc")):
        with open(os.path.join(CSRC, "device", name)) as f:
            text = f.read()
        if ")PTDEV\"" in text:
            raise RuntimeError("device header contains the raw-string delimiter")
        out = 'R"PTDEV(' + text + ')PTDEV"\n'
        path = os.path.join(CSRC, inc)
        old = open(path).read() if os.path.exists(path) else None
        if old != out:
            with open(path, "w") as f:
                f.write(out)


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = SOURCES + HEADERS + ["pt_device_src.inc", "pt_user_object_src.inc"]
    return any(os.path.getmtime(os.path.join(CSRC, d)) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    _embed_device_header()
    if not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    cmd = ["hipcc", "--offload-arch=gfx950", "-std=c++17", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
           "-Wall", "-Wno-unused-result", "-o", LIB + ".tmp"]
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    cmd += ["-ldl", "-lz"]  # hiprtc is dlopen'ed by path (csrc/jit.cpp); zlib for PNG
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
