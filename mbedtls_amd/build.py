"""Build libtlsrec.so in-tree (hipcc for gfx950 + gcc for the host C).

    python -m mbedtls_amd.build          # incremental
    python -m mbedtls_amd.build --force  # rebuild everything

The shared library lands next to this file (mbedtls_amd/libtlsrec.so) so
that it travels with a gpurun snapshot; objects go to build/.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
OBJ = os.path.join(ROOT, "build")
LIB = os.path.join(PKG, "libtlsrec.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# parallel compiles: the box exports MAX_JOBS=16; here 8 CPUs (and ~2 GB per hipcc)
JOBS = max(1, min(int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 1, 8))
ARCH = "gfx950"
HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result",
             "-Wno-unused-value", "-I" + INC, "-I" + CSRC]
C_FLAGS = ["-O2", "-fPIC", "-std=c11", "-Wall", "-Wextra", "-I" + INC, "-I" + CSRC]

HEADERS = ["tlsrec_device.h", "tlsrec_frame.h", "tlsrec_internal.h", "tlsrec_recdev.h", "tlsrec_gcm.h"]
UNITS = [("gcm_dec.hip", "hip"), ("gcm_enc.hip", "hip"), ("gcm_alt_dec.hip", "hip"), ("gcm_alt_enc.hip", "hip"),
         ("kernels.hip", "hip"), ("engine.hip", "hip"), ("keysched.hip", "hip"), ("stream.hip", "hip"), ("ccm.hip", "hip"), ("ticket.hip", "hip"),
         ("server.hip", "hip"), ("tlsrec_host.c", "c")]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _deps():
    return [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INC, "tlsrec.h")]


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    dep_time = max(_mtime(p) for p in _deps())
    objs, cmds = [], []
    for src, kind in UNITS:
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src.rsplit(".", 1)[0] + ".o")
        objs.append(o)
        if not force and _mtime(o) > max(_mtime(s), dep_time):
            continue
        if kind == "hip":
            cmds.append([HIPCC] + HIP_FLAGS + ["-c", s, "-o", o])
        else:
            cmds.append(["gcc"] + C_FLAGS + ["-c", s, "-o", o])
    # translation units compile in parallel (kernels.hip dominates)
    from concurrent.futures import ThreadPoolExecutor
    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    with ThreadPoolExecutor(max_workers=min(JOBS, max(1, len(cmds)))) as ex:
        list(ex.map(run, cmds))
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", LIB] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
