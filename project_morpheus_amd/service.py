"""Per-process synthesis service: weights -> LlmEngine + SnacDecoder + Synthesizer.

The reference keeps one cached model per process behind an asyncio.Lock + lru_cache
(llama_local.py:35-59); this is the MI355X equivalent: one engine per GPU process, created
on first use, utterances serialized through a lock (one process per GPU).
"""
from __future__ import annotations

import threading
import warnings
from typing import Iterator, Optional

import torch

from . import config as C
from . import inference as I
from .engine import LlmEngine, SnacDecoder, Synthesizer, UtteranceStats
from .tokenizer import Tokenizer, default_tokenizer
from .weights import (load_hf_llm, load_snac_state_dict, synthetic_llm_weights,
                      synthetic_snac_weights)


class Service:
    def __init__(self, device: int = C.MX_DEVICE, cfg: Optional[C.OrpheusConfig] = None,
                 llm_weights=None, snac_weights=None, max_pos: int = 2048,
                 tokenizer: Optional[Tokenizer] = None, max_prefill: int = 512):
        torch.cuda.set_device(device)
        if cfg is None:
            cfg = C.OrpheusConfig.from_hf(C.MX_WEIGHTS) if C.MX_WEIGHTS else C.OrpheusConfig()
        if llm_weights is None:
            if C.MX_WEIGHTS:
                llm_weights = load_hf_llm(C.MX_WEIGHTS, device=f"cuda:{device}")
            else:
                warnings.warn("MORPHEUS_MX_WEIGHTS unset: seeded SYNTHETIC Orpheus weights")
                llm_weights = synthetic_llm_weights(cfg, seed=0, device=f"cuda:{device}")
        if snac_weights is None:
            snac_weights = load_snac_state_dict(C.MX_SNAC) if C.MX_SNAC else \
                synthetic_snac_weights()
        self.cfg = cfg
        self.llm = LlmEngine(cfg, llm_weights, device=device, max_slots=1, max_pos=max_pos,
                             max_batch=1, max_prefill=max_prefill)
        del llm_weights
        self.snac = SnacDecoder(snac_weights, device=device)
        self.synth = Synthesizer(self.llm, self.snac)
        self.tok = tokenizer or default_tokenizer()
        self.lock = threading.Lock()

    def prompt_ids(self, text: str, voice: str):
        return I.prompt_ids(self.tok.encode(f"{I.resolve_voice(voice)}: {text}"))

    def stream(self, text: str, voice: str = I.DEFAULT_VOICE, max_tokens: Optional[int] = None,
               penalty: float = I.REPETITION_PENALTY, stats: Optional[UtteranceStats] = None,
               cancel: Optional[threading.Event] = None) -> Iterator[bytes]:
        ids = self.prompt_ids(text, voice)
        max_tokens = max_tokens or I.MAX_TOKENS
        with self.lock:
            for pcm in self.synth.run(ids, max_tokens, penalty, stats=stats):
                if cancel is not None and cancel.is_set():
                    break
                yield pcm


_service: Optional[Service] = None
_service_lock = threading.Lock()


def get_service() -> Service:
    global _service
    with _service_lock:
        if _service is None:
            _service = Service(max_pos=min(C.MX_MAX_POS, 8192))
        return _service
