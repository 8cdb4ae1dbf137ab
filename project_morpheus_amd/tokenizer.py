"""Text -> token ids for the Orpheus prompt.

Three sources, in order:

* ``MORPHEUS_MX_TOKENIZER`` = a directory or file holding the Orpheus ``tokenizer.json``: the
  Llama-3 tokenizer via the ``tokenizers`` package, BOS 128000 first, as the HF tokenizer call
  in engine_class.py:86 does;
* ``MORPHEUS_MX_TOKENIZER`` or ``LLAMA_MODEL_PATH`` = a ``.gguf`` file (the reference CPU
  path's single artefact, llama_local.py:42-52, .env.example:10): the byte-level BPE
  vocabulary stored in the GGUF metadata (``tokenizer.ggml.tokens / merges / token_type /
  bos_token_id``), rebuilt here as the same ``tokenizers`` pipeline llama.cpp runs for a
  Llama-3 (``llama-bpe``) vocabulary: the Llama-3 split regex, byte-level mapping, BPE with
  ``ignore_merges`` (a word that is itself a token is not merged further), control and
  user-defined tokens matched whole;
* otherwise (this environment has no tokenizer files and no network) a deterministic
  SYNTHETIC tokenizer mapping words/punctuation to ids in [1000, 128000) so prompts have
  realistic lengths; for synthetic-weight runs only.
"""
from __future__ import annotations

import hashlib
import os
import re
from typing import Any, Dict, List, Optional

from .config import BOS, MX_TOKENIZER

# The Llama-3 pre-tokenizer split (tokenizer.json "pre_tokenizer" of Llama-3 / llama.cpp
# LLAMA_VOCAB_PRE_TYPE_LLAMA3)
LLAMA3_SPLIT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
                r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
# llama.cpp token types (llama_token_type): 3 = control, 4 = user defined
_CONTROL, _USER_DEFINED = 3, 4


def hf_tokenizer_from_gguf_meta(meta: Dict[str, Any]):
    """GGUF ``tokenizer.ggml.*`` metadata -> a ``tokenizers.Tokenizer`` (byte-level BPE)."""
    from tokenizers import AddedToken, Regex, decoders, models, pre_tokenizers
    from tokenizers import Tokenizer as HFTok
    kind = meta.get("tokenizer.ggml.model", "gpt2")
    if kind != "gpt2":
        raise ValueError(f"GGUF tokenizer model {kind!r} unsupported: Orpheus / Llama-3 "
                         "ship a byte-level BPE ('gpt2') vocabulary")
    tokens: List[str] = list(meta["tokenizer.ggml.tokens"])
    merges = [tuple(m.split(" ", 1)) for m in meta.get("tokenizer.ggml.merges", [])]
    types = list(meta.get("tokenizer.ggml.token_type", [1] * len(tokens)))
    vocab: Dict[str, int] = {}
    for i, t in enumerate(tokens):
        vocab.setdefault(t, i)
    tk = HFTok(models.BPE(vocab=vocab, merges=merges, ignore_merges=True))
    tk.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, trim_offsets=True, use_regex=False)])
    tk.decoder = decoders.ByteLevel()
    special = [AddedToken(t, special=True, normalized=False)
               for t, ty in zip(tokens, types) if ty in (_CONTROL, _USER_DEFINED)]
    if special:
        tk.add_special_tokens(special)
    return tk


class Tokenizer:
    def __init__(self, path: Optional[str] = MX_TOKENIZER):
        self.synthetic = True
        self._tok = None
        self.bos: Optional[int] = BOS
        if path is None:
            lm = os.environ.get("LLAMA_MODEL_PATH")
            if lm and lm.endswith(".gguf") and os.path.exists(lm):
                path = lm
        if path:
            if path.endswith(".gguf"):
                from .gguf import GGUFFile
                meta = GGUFFile(path).meta
                self._tok = hf_tokenizer_from_gguf_meta(meta)
                add_bos = bool(meta.get("tokenizer.ggml.add_bos_token", True))
                self.bos = int(meta.get("tokenizer.ggml.bos_token_id", BOS)) if add_bos else None
            else:
                from tokenizers import Tokenizer as HFTok
                f = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
                self._tok = HFTok.from_file(f)
            self.synthetic = False

    def encode(self, text: str) -> List[int]:
        if self._tok is not None:
            ids = self._tok.encode(text, add_special_tokens=False).ids
            return ([self.bos] if self.bos is not None else []) + list(ids)
        pieces = re.findall(r"\w+|[^\w\s]", text, flags=re.UNICODE)
        out = [BOS]
        for p in pieces:
            h = int.from_bytes(hashlib.blake2s(p.encode(), digest_size=4).digest(), "little")
            out.append(1000 + h % 127000)
        return out

    def decode(self, ids: List[int]) -> str:
        if self._tok is None:
            return ""
        return self._tok.decode(list(ids), skip_special_tokens=False)


_default: Optional[Tokenizer] = None


def default_tokenizer() -> Tokenizer:
    global _default
    if _default is None:
        _default = Tokenizer()
    return _default
