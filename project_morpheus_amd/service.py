"""Per-GPU synthesis service: weights -> LlmEngine + SnacDecoder + a continuous-batching loop.

The reference keeps one cached model per process behind an asyncio.Lock + lru_cache
(llama_local.py:35-59) and, on its GPU path, hands every request to vLLM's continuous batcher
from its own thread (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:114-134).  Here
one ``Service`` per GPU process owns the engine and a ``BatchSynthesizer`` running online:
concurrent adapters ``submit`` streams that join the batch as they arrive (no lock, no
one-slot serialisation); ``cancel`` (barge-in) frees the stream's KV row.  Several GPUs are
served by ``dispatch.GpuPool`` (one worker process per GPU, least-loaded assignment).

Generation parameters follow the reference's module globals at call time
(``inference.TEMPERATURE / TOP_P / MAX_TOKENS``, updated by ``update_generation_params``,
inference.py:75-105) with the fixed repetition penalty 1.1.
"""
from __future__ import annotations

import queue
import threading
import warnings
from typing import Iterator, Optional

import numpy as np
import torch

from . import config as C
from . import inference as I
from .batching import BatchSynthesizer, StreamHandle, StreamRequest
from .engine import LlmEngine, SnacDecoder
from .tokenizer import Tokenizer, default_tokenizer
from .weights import (load_hf_llm, load_snac_state_dict, synthetic_llm_weights,
                      synthetic_snac_weights)


class Service:
    def __init__(self, device: int = C.MX_DEVICE, cfg: Optional[C.OrpheusConfig] = None,
                 llm_weights=None, snac_weights=None, max_pos: int = 2048,
                 tokenizer: Optional[Tokenizer] = None, max_prefill: int = 512,
                 max_batch: int = C.MX_MAX_SLOTS, synthetic_audio: Optional[bool] = None):
        """``synthetic_audio``: feed the SNAC schedule a seeded audio-code stream per request
        (default: whenever the LLM weights are synthetic, which never speak)."""
        torch.cuda.set_device(device)
        synthetic = False
        if cfg is None:
            cfg = C.OrpheusConfig.from_hf(C.MX_WEIGHTS) if C.MX_WEIGHTS else C.OrpheusConfig()
        if llm_weights is None:
            if C.MX_WEIGHTS:
                llm_weights = load_hf_llm(C.MX_WEIGHTS, device=f"cuda:{device}")
            else:
                warnings.warn("MORPHEUS_MX_WEIGHTS unset: seeded SYNTHETIC Orpheus weights")
                llm_weights = synthetic_llm_weights(cfg, seed=0, device=f"cuda:{device}")
                synthetic = True
        if snac_weights is None:
            snac_weights = load_snac_state_dict(C.MX_SNAC) if C.MX_SNAC else \
                synthetic_snac_weights()
        self.cfg, self.device = cfg, device
        self.synthetic_audio = synthetic if synthetic_audio is None else synthetic_audio
        self.llm = LlmEngine(cfg, llm_weights, device=device, max_slots=max_batch,
                             max_pos=max_pos, max_batch=max_batch, max_prefill=max_prefill)
        del llm_weights
        self.snac = SnacDecoder(snac_weights, device=device, max_batch=max_batch)
        self.batch = BatchSynthesizer(self.llm, self.snac).start()
        self.tok = tokenizer or default_tokenizer()

    @classmethod
    def from_engines(cls, llm: LlmEngine, snac: SnacDecoder, cfg: C.OrpheusConfig,
                     synthetic_audio: bool, tokenizer: Optional[Tokenizer] = None) -> "Service":
        """A service over engines that already exist (bench: the configs[1] line through the
        shipped adapter -> Service -> BatchSynthesizer path, on the bench's own weights)."""
        self = cls.__new__(cls)
        self.cfg, self.device = cfg, llm.device
        self.synthetic_audio = synthetic_audio
        self.llm, self.snac = llm, snac
        self.batch = BatchSynthesizer(llm, snac).start()
        self.tok = tokenizer or default_tokenizer()
        return self

    @property
    def outstanding_tokens(self) -> int:
        return self.batch.outstanding_tokens

    def prompt_ids(self, text: str, voice: str):
        return I.prompt_ids(self.tok.encode(f"{I.resolve_voice(voice)}: {text}"))

    def submit(self, text: str, voice: str = I.DEFAULT_VOICE, max_tokens: Optional[int] = None,
               penalty: float = I.REPETITION_PENALTY, temperature: Optional[float] = None,
               top_p: Optional[float] = None, seed: Optional[int] = None,
               prompt_ids=None) -> StreamHandle:
        """Queue one utterance on this GPU's batch loop (non-blocking)."""
        ids = list(prompt_ids) if prompt_ids is not None else self.prompt_ids(text, voice)
        max_tokens = max_tokens or I.MAX_TOKENS
        # one utterance's random streams (sampling, SNAC noise, synthetic codes) come from ONE
        # per-request seed, so its audio never depends on arrival order or batch company;
        # without a seed it is fresh per request (config.request_seed / CONTENT_SEED)
        key = C.request_seed(ids, seed)
        req = StreamRequest(
            prompt_ids=ids, max_tokens=max_tokens, penalty=penalty,
            temperature=I.TEMPERATURE if temperature is None else temperature,
            top_p=I.TOP_P if top_p is None else top_p, seed=key, noise_seed=key,
            inject_ids=C.synthetic_audio_ids(max_tokens, seed=key)
            if self.synthetic_audio else None)
        if self.synthetic_audio:
            req.stop_ids = ()  # synthetic weights decode the full budget (bench contract)
        return self.batch.submit(req)

    def submit_tokens(self, prompt_ids, max_tokens: Optional[int] = None,
                      temperature: Optional[float] = None, top_p: Optional[float] = None,
                      penalty: float = I.REPETITION_PENALTY, seed: Optional[int] = None):
        """Token-only stream (completions surface): a TokenHandle of generated ids."""
        ids = list(prompt_ids)
        key = C.request_seed(ids, seed)
        req = StreamRequest(prompt_ids=ids, max_tokens=max_tokens or I.MAX_TOKENS,
                            penalty=penalty,
                            temperature=I.TEMPERATURE if temperature is None else temperature,
                            top_p=I.TOP_P if top_p is None else top_p, seed=key, audio=False)
        return self.batch.submit(req)

    def stream(self, text: str, voice: str = I.DEFAULT_VOICE, max_tokens: Optional[int] = None,
               penalty: float = I.REPETITION_PENALTY, stats=None,
               cancel: Optional[threading.Event] = None, **kw) -> Iterator[bytes]:
        """PCM16 chunks of one utterance in order; ``cancel`` (or closing the generator)
        cancels the stream on the GPU and frees its row."""
        h = self.submit(text, voice, max_tokens, penalty, **kw)
        try:
            while True:
                if cancel is not None and cancel.is_set():
                    return
                try:
                    c = h.get(timeout=0.05)
                except queue.Empty:
                    continue
                if c is None:
                    return
                yield c
        finally:
            h.cancel()
            if stats is not None:
                stats.tokens = len(h.req.tokens)
                stats.samples = h.req.samples

    def close(self) -> None:
        self.batch.stop()


_service: Optional[Service] = None
_service_lock = threading.Lock()


def get_service():
    """The process' synthesis backend: one ``Service`` on this GPU, or a ``GpuPool`` of
    worker processes when MORPHEUS_MX_GPUS > 1 (both expose ``stream`` / ``submit``)."""
    global _service
    with _service_lock:
        if _service is None:
            if C.MX_GPUS > 1:
                from .dispatch import GpuPool
                _service = GpuPool(C.MX_GPUS)
            else:
                _service = Service(max_pos=min(C.MX_MAX_POS, 8192))
        return _service
