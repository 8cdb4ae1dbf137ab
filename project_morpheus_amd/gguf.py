"""GGUF checkpoints (the reference CPU path's ``Orpheus-3b-FT-Q8_0.gguf``) -> engine weights.

The reference's CPU engine is llama.cpp loading a Q8_0 GGUF (.env.example:10,
Morpheus_Client/tts_engine/llama_local.py:42-52).  This module reads that file format
natively -- no llama.cpp -- so the MI355X engine can run the same checkpoint:

* GGUF v2/v3 container: magic ``GGUF``, version, tensor count, metadata key/values (typed),
  tensor infos (name, dims with ne[0] the contiguous one, ggml type, offset), data aligned
  to ``general.alignment`` (default 32);
* tensor types F32, F16, BF16 and Q8_0 (blocks of 32 along ne[0]: fp16 scale d + 32 int8,
  value = d * q; llama.cpp ggml-quants ``dequantize_row_q8_0``);
* llama.cpp tensor names (``token_embd``, ``blk.N.attn_q`` ...) -> the engine's names, and the
  rotary layout: llama.cpp's converter permutes q/k rows of every head to the interleaved
  (GPT-J) order (convert_hf_to_gguf.py ``LlamaModel.permute``); the engine uses the HF
  rotate-half order, so those rows are permuted back;
* ``config_from_gguf``: the Llama hyper-parameters from ``llama.*`` metadata.

``write_gguf`` writes the same format (used by the tests to round-trip synthetic weights).
Q8_0 weights dequantise to bf16 for the bf16 engine exactly when d*q is representable
(|q| <= 127 with an fp16 scale: d*q has <= 8+11 significant bits, so not always) -- the loader
keeps fp32 and the engine rounds to bf16 (RNE) when it packs them.
"""
from __future__ import annotations

import struct
from typing import Any, BinaryIO, Dict, List, Optional, Tuple

import numpy as np

from .config import OrpheusConfig

GGUF_MAGIC = b"GGUF"
# metadata value types
_U8, _I8, _U16, _I16, _U32, _I32, _F32, _BOOL, _STR, _ARR, _U64, _I64, _F64 = range(13)
_SCALAR = {_U8: "<B", _I8: "<b", _U16: "<H", _I16: "<h", _U32: "<I", _I32: "<i", _F32: "<f",
           _BOOL: "<?", _U64: "<Q", _I64: "<q", _F64: "<d"}
# ggml tensor types
GGML_F32, GGML_F16, GGML_Q8_0, GGML_BF16 = 0, 1, 8, 30
Q8_BLOCK = 32


def _read_str(f: BinaryIO) -> str:
    (n,) = struct.unpack("<Q", f.read(8))
    return f.read(n).decode("utf-8")


def _read_value(f: BinaryIO, t: int):
    if t in _SCALAR:
        fmt = _SCALAR[t]
        return struct.unpack(fmt, f.read(struct.calcsize(fmt)))[0]
    if t == _STR:
        return _read_str(f)
    if t == _ARR:
        (et,) = struct.unpack("<I", f.read(4))
        (n,) = struct.unpack("<Q", f.read(8))
        if et in _SCALAR:
            dt = np.dtype(_SCALAR[et])
            return np.frombuffer(f.read(n * dt.itemsize), dtype=dt).tolist()
        return [_read_value(f, et) for _ in range(n)]
    raise ValueError(f"GGUF: unknown metadata type {t}")


class GGUFFile:
    """Parsed header of a GGUF file; tensors are read on demand (memory-mapped)."""

    def __init__(self, path: str):
        self.path = path
        with open(path, "rb") as f:
            if f.read(4) != GGUF_MAGIC:
                raise ValueError(f"{path}: not a GGUF file")
            (self.version,) = struct.unpack("<I", f.read(4))
            if self.version not in (2, 3):
                raise ValueError(f"{path}: GGUF version {self.version} unsupported")
            n_tensors, n_kv = struct.unpack("<QQ", f.read(16))
            self.meta: Dict[str, Any] = {}
            for _ in range(n_kv):
                k = _read_str(f)
                (t,) = struct.unpack("<I", f.read(4))
                self.meta[k] = _read_value(f, t)
            self.tensors: Dict[str, Tuple[Tuple[int, ...], int, int]] = {}
            for _ in range(n_tensors):
                name = _read_str(f)
                (nd,) = struct.unpack("<I", f.read(4))
                dims = struct.unpack(f"<{nd}Q", f.read(8 * nd))
                ttype, off = struct.unpack("<IQ", f.read(12))
                self.tensors[name] = (tuple(dims), ttype, off)
            align = int(self.meta.get("general.alignment", 32))
            pos = f.tell()
            self.data_start = (pos + align - 1) // align * align
        self._mm = np.memmap(path, dtype=np.uint8, mode="r")

    def tensor(self, name: str) -> np.ndarray:
        """fp32 array shaped [ne[n-1], ..., ne[0]] (row-major, ne[0] contiguous)."""
        dims, ttype, off = self.tensors[name]
        shape = tuple(reversed(dims))
        n = int(np.prod(dims))
        base = self.data_start + off
        if ttype == GGML_F32:
            return np.frombuffer(self._mm[base:base + 4 * n], dtype="<f4").reshape(shape).copy()
        if ttype == GGML_F16:
            return np.frombuffer(self._mm[base:base + 2 * n], dtype="<f2").astype(np.float32).reshape(shape)
        if ttype == GGML_BF16:
            u = np.frombuffer(self._mm[base:base + 2 * n], dtype="<u2").astype(np.uint32) << 16
            return u.view(np.float32).reshape(shape)
        if ttype == GGML_Q8_0:
            if dims[0] % Q8_BLOCK:
                raise ValueError(f"{name}: Q8_0 row of {dims[0]} not a multiple of 32")
            nb = n // Q8_BLOCK
            raw = np.frombuffer(self._mm[base:base + 34 * nb], dtype=np.uint8).reshape(nb, 34)
            d = raw[:, :2].copy().view("<f2").astype(np.float32)          # [nb, 1]
            q = raw[:, 2:].view(np.int8).astype(np.float32)                # [nb, 32]
            return (d * q).reshape(shape)
        raise ValueError(f"{name}: ggml type {ttype} not supported (F32/F16/BF16/Q8_0)")


def config_from_gguf(g: GGUFFile) -> OrpheusConfig:
    m = g.meta
    arch = m.get("general.architecture", "llama")
    p = arch + "."
    heads = int(m[p + "attention.head_count"])
    hidden = int(m[p + "embedding_length"])
    vocab = len(m["tokenizer.ggml.tokens"]) if "tokenizer.ggml.tokens" in m else \
        int(m.get(p + "vocab_size", g.tensors["token_embd.weight"][0][1]))
    return OrpheusConfig(
        hidden=hidden, layers=int(m[p + "block_count"]), heads=heads,
        kv_heads=int(m.get(p + "attention.head_count_kv", heads)),
        head_dim=int(m.get(p + "attention.key_length", hidden // heads)),
        ffn=int(m[p + "feed_forward_length"]), vocab=vocab,
        eps=float(m.get(p + "attention.layer_norm_rms_epsilon", 1e-5)),
        rope_theta=float(m.get(p + "rope.freq_base", 10000.0)),
        tied="output.weight" not in g.tensors)


def _unpermute_rope(w: np.ndarray, n_head: int) -> np.ndarray:
    """Inverse of convert_hf_to_gguf ``permute``: interleaved (GPT-J) rows -> rotate-half."""
    r, c = w.shape
    return w.reshape(n_head, r // n_head // 2, 2, c).swapaxes(1, 2).reshape(r, c)


def _permute_rope(w: np.ndarray, n_head: int) -> np.ndarray:
    r, c = w.shape
    return w.reshape(n_head, 2, r // n_head // 2, c).swapaxes(1, 2).reshape(r, c)


_NAMES = {"attn_norm": "attn_norm", "attn_q": "wq", "attn_k": "wk", "attn_v": "wv",
          "attn_output": "wo", "ffn_norm": "mlp_norm", "ffn_gate": "wg", "ffn_up": "wu",
          "ffn_down": "wd"}


def load_gguf_llm(path: str, dtype="bfloat16"):
    """-> (OrpheusConfig, {engine weight name: torch tensor}) from a llama.cpp GGUF."""
    import torch
    g = GGUFFile(path)
    cfg = config_from_gguf(g)
    td = getattr(torch, dtype)
    out = {"embed": torch.from_numpy(g.tensor("token_embd.weight")).to(td),
           "norm": torch.from_numpy(g.tensor("output_norm.weight")).to(td)}
    if "output.weight" in g.tensors:
        out["lm_head"] = torch.from_numpy(g.tensor("output.weight")).to(td)
    for i in range(cfg.layers):
        for src, dst in _NAMES.items():
            w = g.tensor(f"blk.{i}.{src}.weight")
            if src == "attn_q":
                w = _unpermute_rope(w, cfg.heads)
            elif src == "attn_k":
                w = _unpermute_rope(w, cfg.kv_heads)
            out[f"l{i}.{dst}"] = torch.from_numpy(np.ascontiguousarray(w)).to(td)
    return cfg, out


# ------------------------------------------------------------------------------ writer
def quantize_q8_0(w: np.ndarray) -> bytes:
    """ggml ``quantize_row_q8_0_ref``: per 32-block d = amax / 127 (fp16), q = round(x / d)."""
    x = np.asarray(w, dtype=np.float32).reshape(-1, Q8_BLOCK)
    amax = np.abs(x).max(axis=1)
    d = (amax / 127.0).astype(np.float32)
    inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1.0), 0.0).astype(np.float32)
    q = np.round(x * inv[:, None]).astype(np.int8)
    blk = np.empty((x.shape[0], 34), dtype=np.uint8)
    blk[:, :2] = d.astype("<f2").view(np.uint8).reshape(-1, 2)
    blk[:, 2:] = q.view(np.uint8)
    return blk.tobytes()


def _w_str(f, s: str):
    b = s.encode()
    f.write(struct.pack("<Q", len(b)) + b)


def _w_value(f, v):
    if isinstance(v, bool):
        f.write(struct.pack("<I?", _BOOL, v))
    elif isinstance(v, int):
        f.write(struct.pack("<Iq" if v < 0 else "<IQ", _I64 if v < 0 else _U64, v))
    elif isinstance(v, float):
        f.write(struct.pack("<If", _F32, v))
    elif isinstance(v, str):
        f.write(struct.pack("<I", _STR))
        _w_str(f, v)
    elif isinstance(v, (list, tuple)):
        f.write(struct.pack("<II", _ARR, _STR if v and isinstance(v[0], str) else _I32))
        f.write(struct.pack("<Q", len(v)))
        for x in v:
            if isinstance(x, str):
                _w_str(f, x)
            else:
                f.write(struct.pack("<i", x))
    else:
        raise TypeError(type(v))


def write_gguf(path: str, meta: Dict[str, Any], tensors: Dict[str, Tuple[np.ndarray, int]],
               alignment: int = 32) -> None:
    """tensors: name -> (array [rows, cols] or [n], ggml type F32 / F16 / Q8_0)."""
    blobs: List[Tuple[str, Tuple[int, ...], int, bytes]] = []
    for name, (a, t) in tensors.items():
        a = np.ascontiguousarray(a, dtype=np.float32)
        dims = tuple(reversed(a.shape))
        if t == GGML_F32:
            b = a.astype("<f4").tobytes()
        elif t == GGML_F16:
            b = a.astype("<f2").tobytes()
        elif t == GGML_Q8_0:
            b = quantize_q8_0(a)
        else:
            raise ValueError(t)
        blobs.append((name, dims, t, b))
    with open(path, "wb") as f:
        f.write(GGUF_MAGIC + struct.pack("<IQQ", 3, len(blobs), len(meta) + 1))
        _w_str(f, "general.alignment")
        f.write(struct.pack("<II", _U32, alignment))
        for k, v in meta.items():
            _w_str(f, k)
            _w_value(f, v)
        off = 0
        offs = []
        for name, dims, t, b in blobs:
            _w_str(f, name)
            f.write(struct.pack("<I", len(dims)) + struct.pack(f"<{len(dims)}Q", *dims))
            f.write(struct.pack("<IQ", t, off))
            offs.append(off)
            off = (off + len(b) + alignment - 1) // alignment * alignment
        pad = (-f.tell()) % alignment
        f.write(b"\0" * pad)
        for (name, dims, t, b), o in zip(blobs, offs):
            f.write(b)
            f.write(b"\0" * ((-len(b)) % alignment))


def export_gguf(path: str, cfg: OrpheusConfig, weights: Dict[str, "object"],
                qtype: int = GGML_Q8_0, tokens: Optional[List[str]] = None) -> None:
    """Engine-named weights -> a llama.cpp-layout GGUF (q/k rows permuted as the converter
    does, norms F32, matrices ``qtype``)."""
    def np32(t):
        return t.float().cpu().numpy() if hasattr(t, "float") else np.asarray(t, np.float32)

    meta = {"general.architecture": "llama", "llama.block_count": cfg.layers,
            "llama.embedding_length": cfg.hidden, "llama.feed_forward_length": cfg.ffn,
            "llama.attention.head_count": cfg.heads,
            "llama.attention.head_count_kv": cfg.kv_heads,
            "llama.attention.layer_norm_rms_epsilon": float(cfg.eps),
            "llama.rope.freq_base": float(cfg.rope_theta), "llama.vocab_size": cfg.vocab}
    if tokens is not None:
        meta["tokenizer.ggml.tokens"] = tokens
    t = {"token_embd.weight": (np32(weights["embed"]), qtype),
         "output_norm.weight": (np32(weights["norm"]), GGML_F32)}
    if "lm_head" in weights:
        t["output.weight"] = (np32(weights["lm_head"]), qtype)
    inv = {v: k for k, v in _NAMES.items()}
    for i in range(cfg.layers):
        for dst, src in inv.items():
            w = np32(weights[f"l{i}.{dst}"])
            if src == "attn_q":
                w = _permute_rope(w, cfg.heads)
            elif src == "attn_k":
                w = _permute_rope(w, cfg.kv_heads)
            t[f"blk.{i}.{src}.weight"] = (w, GGML_F32 if w.ndim == 1 else qtype)
    write_gguf(path, meta, t)
