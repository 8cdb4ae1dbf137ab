"""Build libmorpheus_mx.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

    python -m project_morpheus_amd.build        # or __graft_entry__.build()
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmorpheus_mx.so")
SOURCES = ["capi.hip", "llm_kernels.hip", "llm_batched.hip", "llm_batched_v4.hip", "llm_mega.hip",
           "llm_batched_v7.hip", "snac_kernels.hip"]
HEADERS = ["mx_common.h", "mx_llm_kernels.h", "mx_snac_kernels.h"]
ARCH = os.environ.get("MORPHEUS_MX_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "morpheus_mx.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return LIB
    objs, procs = [], []
    for s in SOURCES:  # translation units compile in parallel
        src = os.path.join(CSRC, s)
        obj = os.path.join(CSRC, s.replace(".hip", ".o"))
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
               "-munsafe-fp-atomics", "-Wno-unused-result", "-x", "hip", "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    tmp = LIB + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
