"""Build libtlsrec.so in-tree (hipcc for gfx950 + gcc for the host C).

    python -m mbedtls_amd.build          # incremental
    python -m mbedtls_amd.build --force  # rebuild everything

The shared library lands next to this file (mbedtls_amd/libtlsrec.so) so
that it travels with a gpurun snapshot; objects go to build/.

Beside it, libtlsrec_test.so: the same library compiled with
-DTLSREC_TEST_HOOKS (the reference's MBEDTLS_TEST_HOOKS, ssl_misc.h:2685) --
the tlsrec__test_* entry points and the kernels' unreached-record compare
exist only there.  Only tests/ load it (tests/test_fail_closed_gpu.py through
mbedtls_amd._abi.use_library); units that hold no hook share their objects.
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
TEST_LIB = os.path.join(PKG, "libtlsrec_test.so")
TEST_OBJ = os.path.join(OBJ, "test_hooks")

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
# units whose code changes under TLSREC_TEST_HOOKS (TLSREC_HOOK_SKIP, the hook entry points)
HOOK_UNITS = {"gcm_dec.hip", "gcm_enc.hip", "gcm_alt_dec.hip", "gcm_alt_enc.hip", "kernels.hip", "engine.hip",
              "ccm.hip", "server.hip"}


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _deps():
    return [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INC, "tlsrec.h")]


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(TEST_OBJ, exist_ok=True)
    dep_time = max(_mtime(p) for p in _deps())
    objs, test_objs, cmds = [], [], []
    for src, kind in UNITS:
        s = os.path.join(CSRC, src)
        stem = src.rsplit(".", 1)[0] + ".o"
        variants = [(os.path.join(OBJ, stem), [])]
        if src in HOOK_UNITS:
            variants.append((os.path.join(TEST_OBJ, stem), ["-DTLSREC_TEST_HOOKS"]))
        objs.append(variants[0][0])
        test_objs.append(variants[-1][0])
        for o, extra in variants:
            if not force and _mtime(o) > max(_mtime(s), dep_time):
                continue
            if kind == "hip":
                cmds.append([HIPCC] + HIP_FLAGS + extra + ["-c", s, "-o", o])
            else:
                cmds.append(["gcc"] + C_FLAGS + extra + ["-c", s, "-o", o])
    # translation units compile in parallel, the slowest first (the GCM units dominate)
    cmds.sort(key=lambda c: 0 if any("gcm_" in x for x in c) else (1 if any("kernels" in x for x in c) else 2))
    from concurrent.futures import ThreadPoolExecutor
    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    with ThreadPoolExecutor(max_workers=min(JOBS, max(1, len(cmds)))) as ex:
        list(ex.map(run, cmds))
    for lib, lib_objs in ((LIB, objs), (TEST_LIB, test_objs)):
        if force or _mtime(lib) < max(_mtime(o) for o in lib_objs):
            cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", lib] + lib_objs
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
