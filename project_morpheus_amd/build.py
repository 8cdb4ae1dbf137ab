"""Build libmorpheus_mx.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

    python -m project_morpheus_amd.build        # or __graft_entry__.build()
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# Diagnostic variants, each its own library and object directory (load one with
# MORPHEUS_MX_LIB): MORPHEUS_MX_ROWS_TRACE=1 -> libmorpheus_mx_trace.so (multi-row GEMM phase
# stamps, mx_llm_bench_gemv_trace; the product library never carries them: 1-4 % per step);
# MORPHEUS_MX_VARIANT=<name> with MORPHEUS_MX_DEFS="-D..." -> libmorpheus_mx_<name>.so
# (build-time experiment knobs such as MX_ROWS_NP, MX_ROWS_WLOAD_PLAIN)
TRACE = os.environ.get("MORPHEUS_MX_ROWS_TRACE", "0") == "1"
VARIANT = "trace" if TRACE else os.environ.get("MORPHEUS_MX_VARIANT", "")
LIB = os.path.join(HERE, f"libmorpheus_mx_{VARIANT}.so" if VARIANT else "libmorpheus_mx.so")
OBJ_DIR = os.path.join(CSRC, f"build_{VARIANT}" if VARIANT else "build")  # objects (git-ignored)
DEFS = (["-DMX_ROWS_TRACE=1"] if TRACE else []) + \
    (os.environ.get("MORPHEUS_MX_DEFS", "").split() if VARIANT and not TRACE else [])
SOURCES = ["capi.hip", "llm_kernels.hip", "rows_v4_dispatch.hip", "rows_v4_qkv.hip",
           "rows_v4_resid.hip", "rows_v4_silu.hip", "rows_v4_head.hip", "head_b1.hip",
           "sample_kernels.hip", "snac_kernels.hip", "engine_b1.hip"]
HEADERS = ["mx_common.h", "mx_llm_kernels.h", "mx_snac_kernels.h", "mx_rows_common.h",
           "mx_rows_v4.inc", "mx_engine.h"]
ARCH = os.environ.get("MORPHEUS_MX_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _obj(s: str) -> str:
    return os.path.join(OBJ_DIR, s.replace(".hip", ".o"))


def _includes(path: str, seen=None) -> set:
    """Local headers a source includes, transitively (#include "...")."""
    seen = set() if seen is None else seen
    try:
        text = open(path).read()
    except OSError:
        return seen
    for m in re.finditer(r'#include\s+"([^"]+)"', text):
        h = os.path.normpath(os.path.join(os.path.dirname(path), m.group(1)))
        if h not in seen:
            seen.add(h)
            _includes(h, seen)
    return seen


def _stale(s: str, hdr=None) -> bool:
    o = _obj(s)
    if not os.path.exists(o):
        return True
    src = os.path.join(CSRC, s)
    deps = [src] + [h for h in _includes(src) if os.path.exists(h)]
    return os.path.getmtime(o) < max(os.path.getmtime(d) for d in deps)


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(_stale(s) or os.path.getmtime(_obj(s)) > t for s in SOURCES)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the translation units that changed (all of them with ``force``), in parallel,
    into csrc/build/, then link the shared library."""
    if not force and not needs_build():
        return LIB
    os.makedirs(OBJ_DIR, exist_ok=True)
    procs = []
    for s in SOURCES:
        if not force and not _stale(s):
            continue
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
               "-munsafe-fp-atomics", "-Wno-unused-result"] + DEFS + ["-x", "hip", "-c",
               os.path.join(CSRC, s), "-o", _obj(s) + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd, s))
    for p, cmd, s in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
        os.replace(_obj(s) + ".tmp", _obj(s))
    tmp = LIB + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + \
        [_obj(s) for s in SOURCES]
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
