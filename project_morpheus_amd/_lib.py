"""ctypes binding of libmorpheus_mx.so (include/morpheus_mx.h).

The product path has no CPU fallback: if the library is missing or fails to load, every
engine constructor raises ``MxUnavailable``.  ``torch`` is imported first so that the
library binds to the HIP runtime torch already loaded (same SONAME, one runtime per
process), which lets torch tensors' device pointers be handed across the ABI.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (loads the process' HIP runtime before our library)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MORPHEUS_MX_LIB", os.path.join(HERE, "libmorpheus_mx.so"))

MX_DTYPE_F32 = 0
MX_DTYPE_BF16 = 1
MX_DTYPE_FP8 = 2      # OCP e4m3 bytes

MX_WEIGHTS = {"bf16": 0, "fp8": 1}


class MxUnavailable(RuntimeError):
    pass


MX_ERR_ARG, MX_ERR_HIP, MX_ERR_STATE, MX_ERR_OOM = -1, -2, -3, -4


class MxError(RuntimeError):
    """A non-zero return of the C ABI; ``rc`` is the MX_ERR_* code."""

    def __init__(self, msg: str, rc: int = 0):
        super().__init__(msg)
        self.rc = rc


class LlmConfig(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "hidden", "layers", "heads", "kv_heads", "head_dim", "ffn", "vocab",
        "max_slots", "max_pos", "max_batch", "max_prefill")] + [
        ("eps", C.c_float), ("tied", C.c_int32), ("wdtype", C.c_int32)]


class Sampling(C.Structure):
    """mx_sampling: temperature <= 0 is greedy (the parity mode)."""
    _fields_ = [("temperature", C.c_float), ("top_p", C.c_float),
                ("repetition_penalty", C.c_float), ("seed", C.c_uint64)]


_P = C.c_void_p
_SIGS = {
    "mx_version": (C.c_char_p, []),
    "mx_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(_P), C.POINTER(_P)]),
    "mx_host_free": (C.c_int, [_P]),
    "mx_llm_create": (C.c_int, [C.c_int, C.POINTER(LlmConfig), C.POINTER(_P)]),
    "mx_llm_set_weight": (C.c_int, [_P, C.c_char_p, _P, C.c_int64, C.c_int]),
    "mx_llm_set_rope": (C.c_int, [_P, _P, _P, C.c_int]),
    "mx_llm_finalize": (C.c_int, [_P]),
    "mx_llm_prefill": (C.c_int, [_P, C.c_int, C.c_int, _P, C.c_int, C.POINTER(Sampling), _P]),
    "mx_llm_decode": (C.c_int, [_P, C.c_int, _P]),
    "mx_llm_check": (C.c_int, [_P, _P]),
    "mx_llm_decode_profiled": (C.c_int, [_P, C.c_int, _P, C.POINTER(C.c_double), C.c_int]),
    "mx_llm_set_option": (C.c_int, [_P, C.c_char_p, C.c_int]),
    "mx_llm_engine_trace": (C.c_int, [_P, C.POINTER(C.c_uint64), C.c_int, C.POINTER(C.c_int)]),
    "mx_llm_bench_gemv_streams": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.POINTER(C.c_float)]),
    "mx_llm_bench_gemv_trace": (C.c_int, [_P, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.c_int,
                                          C.POINTER(C.c_int)]),
    "mx_llm_bench_gemv": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float),
                                    C.POINTER(C.c_double)]),
    "mx_llm_bench_attention": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_float)]),
    "mx_llm_release_row": (C.c_int, [_P, C.c_int, _P]),
    "mx_llm_move_row": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "mx_llm_row_state": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mx_llm_history": (C.POINTER(C.c_int32), [_P]),
    "mx_llm_debug_logits": (C.c_int, [_P, C.c_int]),
    "mx_llm_read_logits": (C.c_int, [_P, C.c_int, _P, _P]),
    "mx_llm_last_error": (C.c_char_p, [_P]),
    "mx_llm_destroy": (None, [_P]),
    "mx_snac_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "mx_snac_set_weight": (C.c_int, [_P, C.c_char_p, _P, C.c_int64, C.c_int]),
    "mx_snac_finalize": (C.c_int, [_P]),
    "mx_snac_decode": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_uint64, _P, _P, _P,
                                 C.c_int, C.c_int, _P]),
    "mx_snac_last_error": (C.c_char_p, [_P]),
    "mx_snac_destroy": (None, [_P]),
}
EXPORTS = tuple(_SIGS)

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load (once) and type the library; raises MxUnavailable if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise MxUnavailable(
                f"{path} not built: run `python -m project_morpheus_amd.build` "
                "(the MI355X path has no CPU fallback)")
        try:
            lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
        except OSError as e:
            raise MxUnavailable(f"cannot load {path}: {e}") from e
        # an older library named by MORPHEUS_MX_LIB (same-box A/B runs) may lack entry points
        # added since; the in-tree product library must export every one
        older = os.path.abspath(path) != os.path.join(HERE, "libmorpheus_mx.so")
        for name, (res, args) in _SIGS.items():
            if older and not hasattr(lib, name):
                continue
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
        return lib


def check(rc: int, err_fn, handle) -> None:
    if rc != 0:
        msg = err_fn(handle)
        raise MxError(f"morpheus_mx error {rc}: {msg.decode() if msg else ''}", rc)


def require_gpu() -> None:
    if not torch.cuda.is_available():
        raise MxUnavailable("no HIP device visible: the MI355X path has no CPU fallback")


class HostBuffer:
    """Pinned, device-mapped host memory (mx_host_alloc) with a numpy view."""

    def __init__(self, nbytes: int):
        import numpy as np
        lib = load()
        h, d = C.c_void_p(), C.c_void_p()
        if lib.mx_host_alloc(nbytes, C.byref(h), C.byref(d)) != 0:
            raise MxError("mx_host_alloc failed")
        self.host, self.dev, self.nbytes = h.value, d.value, nbytes
        self._np = np

    def view(self, dtype, count=None, offset=0):
        np = self._np
        n = count if count is not None else (self.nbytes - offset) // np.dtype(dtype).itemsize
        buf = (C.c_char * self.nbytes).from_address(self.host)
        return np.frombuffer(buf, dtype=dtype, count=n, offset=offset)

    def dev_ptr(self, offset=0) -> int:
        return self.dev + offset

    def free(self):
        if self.host:
            load().mx_host_free(self.host)
            self.host = self.dev = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
