"""Text -> token ids for the Orpheus prompt.

With ``MORPHEUS_MX_TOKENIZER`` (a directory holding the Orpheus ``tokenizer.json``) the
real Llama-3 tokenizer runs via the ``tokenizers`` package, BOS 128000 first, as the HF
tokenizer call in engine_class.py:86 does.  Without it (this environment has no tokenizer
files and no network) a deterministic SYNTHETIC tokenizer maps words/punctuation to ids
in [1000, 128000) so prompts have realistic lengths; it is for synthetic-weight runs only.
"""
from __future__ import annotations

import hashlib
import os
import re
from typing import List, Optional

from .config import BOS, MX_TOKENIZER


class Tokenizer:
    def __init__(self, path: Optional[str] = MX_TOKENIZER):
        self.synthetic = True
        self._tok = None
        if path:
            from tokenizers import Tokenizer as HFTok
            f = os.path.join(path, "tokenizer.json") if os.path.isdir(path) else path
            self._tok = HFTok.from_file(f)
            self.synthetic = False

    def encode(self, text: str) -> List[int]:
        if self._tok is not None:
            ids = self._tok.encode(text, add_special_tokens=False).ids
            return [BOS] + list(ids)
        pieces = re.findall(r"\w+|[^\w\s]", text, flags=re.UNICODE)
        out = [BOS]
        for p in pieces:
            h = int.from_bytes(hashlib.blake2s(p.encode(), digest_size=4).digest(), "little")
            out.append(1000 + h % 127000)
        return out


_default: Optional[Tokenizer] = None


def default_tokenizer() -> Tokenizer:
    global _default
    if _default is None:
        _default = Tokenizer()
    return _default
