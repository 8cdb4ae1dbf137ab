"""The C-ABI library builds for gfx950, loads, and exports every symbol in include/*.h.

No compute calls here (no GPU in the CPU tier); -m gpu tests drive the kernels.
"""
import ctypes
import glob
import os
import re

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(mx_[a-z0-9_]+)\s*\(", src))
    return names


@pytest.fixture(scope="module")
def lib_path():
    from project_morpheus_amd import build
    return build.build()


def test_library_exports_header_symbols(lib_path):
    import torch  # noqa: F401  (the library binds torch's HIP runtime)
    lib = ctypes.CDLL(lib_path)
    declared = _declared()
    assert len(declared) >= 20
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    lib.mx_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.mx_version()


def test_ctypes_binding_covers_header(lib_path):
    from project_morpheus_amd import _lib
    assert set(_lib.EXPORTS) == _declared()
    lib = _lib.load(lib_path)
    for n in _lib.EXPORTS:
        assert getattr(lib, n).argtypes is not None or n == "mx_version"


def test_code_object_targets_gfx950(lib_path):
    # the .hip_fatbin section embeds an offload bundle whose entry names the target
    data = open(lib_path, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_engine_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from project_morpheus_amd import _lib
    with pytest.raises(_lib.MxUnavailable):
        _lib.require_gpu()


def test_header_option_list_matches_set_option():
    """include/morpheus_mx.h documents exactly the keys capi.hip mx_llm_set_option accepts."""
    src = open(os.path.join(ROOT, "project_morpheus_amd", "csrc", "capi.hip")).read()
    body = src[src.index('extern "C" int mx_llm_set_option'):]
    body = body[:body.index("unknown option")]
    accepted = set(re.findall(r'k == "([a-z0-9_]+)"', body))
    hdr = open(os.path.join(ROOT, "include", "morpheus_mx.h")).read()
    doc = hdr[hdr.index("Tuning knobs"):hdr.index("int mx_llm_set_option")]
    documented = set(re.findall(r'"([a-z0-9_]+)"', doc))
    assert accepted == documented, (accepted - documented, documented - accepted)
