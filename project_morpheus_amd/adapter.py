"""MxTTSAdapter: the drop-in ``tts_engine`` adapter backed by the MI355X engine.

Contract (Morpheus_Client/tts_engine/llama_local.py:90-157; pinned by the reference's
tests/test_tts_adapter_chunking.py:25-44):
  * ``MxTTSAdapter(prompt, voice=DEFAULT_VOICE, *, use_batching=False, max_batch_chars=1000)``;
  * ``await pull(chunk_size)`` returns at most ``chunk_size`` PCM **bytes**;
    ``duration_ms = len(pcm) / 2 / SAMPLE_RATE * 1000``; ``eos`` once the stream is
    exhausted and the buffer empty; a final ``AudioChunk(b"", 0.0, eos=True)`` after that;
  * ``await reset()`` after barge-in drops buffered audio and cancels the utterance.
Registered into Morpheus's registry as ``"mi355x"`` via ``register(registry)`` with
``mx_describe`` (keys of adapter_registry.py:51-60) and ``mx_voice_mapper``
(adapter_registry.py:39-45 semantics).

Synthesis runs in a producer thread (the source is a blocking iterator; the engine loop
must keep the GPU queue full while the orchestrator makes its small pulls).  ``pull`` first
takes whatever the producer has already queued without leaving the event loop, and awaits
the next chunk through ``asyncio.to_thread`` (like llama_local.py:79) only when the buffer
cannot cover the request.  The producer never blocks indefinitely: it puts with a timeout
and gives up once cancelled, and ``reset`` drains the old queue, so a barge-in or a client
that stops pulling cannot wedge the service (the GPU stream is cancelled and its KV row
freed through the source generator's ``finally``).
"""
from __future__ import annotations

import asyncio
import queue
import threading
from typing import Any, Callable, Dict, Iterator, Optional

from . import inference as I
from .audio import AudioChunk

_END = object()


def _default_source(prompt: str, voice: str, use_batching: bool, max_batch_chars: int,
                    cancel: threading.Event) -> Iterator[bytes]:
    """Every long-form part is submitted at once (they decode as concurrent rows of the
    GPU's batch) and their PCM is yielded in part order."""
    from .service import get_service
    svc = get_service()
    handles = [svc.submit(part, voice) for part in
               I.batch_sentences(prompt, max_batch_chars, use_batching)]
    try:
        for h in handles:
            while True:
                if cancel.is_set():
                    return
                try:
                    c = h.get(timeout=0.05)
                except queue.Empty:
                    continue
                if c is None:
                    break
                yield c
    finally:
        for h in handles:
            h.cancel()


class MxTTSAdapter:
    # injectable for tests: (prompt, voice, use_batching, max_batch_chars, cancel) -> bytes iter
    source: Callable[..., Iterator[bytes]] = staticmethod(_default_source)

    def __init__(self, prompt: str, voice: str = I.DEFAULT_VOICE, *, use_batching: bool = False,
                 max_batch_chars: int = 1000, pull_unit: Optional[str] = None) -> None:
        """``pull_unit``: "bytes" (the reference contract, default) or "ms" (the unit the
        descriptor declares: ``pull(n)`` returns n ms of PCM); default from
        ``config.PULL_UNIT`` (MORPHEUS_MX_PULL_UNIT)."""
        from .config import PULL_UNIT
        self.prompt = prompt
        self.voice = voice
        self.use_batching = use_batching
        self.max_batch_chars = max_batch_chars
        unit = pull_unit or PULL_UNIT
        if unit not in ("bytes", "ms"):
            raise ValueError(f"pull_unit must be 'bytes' or 'ms', got {unit!r}")
        # bytes per pull unit: 1, or 24 kHz x 2 bytes / 1000 = 48 per millisecond
        self._unit_bytes = 1 if unit == "bytes" else 2 * I.SAMPLE_RATE // 1000
        self._buffer = bytearray()
        self._exhausted = False
        self._q: Optional[queue.Queue] = None
        self._cancel: Optional[threading.Event] = None
        self._thread: Optional[threading.Thread] = None

    def _start(self) -> None:
        if self._q is not None or self._exhausted:
            return
        q: queue.Queue = queue.Queue(maxsize=64)
        cancel = threading.Event()
        src = self.source(self.prompt, self.voice, self.use_batching, self.max_batch_chars,
                          cancel)

        def put(item) -> bool:
            while not cancel.is_set():
                try:
                    q.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    continue
            return False

        def produce():
            try:
                for pcm in src:
                    if cancel.is_set() or not put(bytes(pcm)):
                        break
            except BaseException as e:  # surfaced to the caller of pull()
                put(e)
            finally:
                close = getattr(src, "close", None)
                if close is not None:
                    close()  # runs the source's finally: GPU stream cancelled, row freed
                put(_END)

        self._q, self._cancel = q, cancel
        self._thread = threading.Thread(target=produce, name="mx-tts", daemon=True)
        self._thread.start()

    def _take(self, item) -> None:
        if item is _END:
            self._exhausted = True
        elif isinstance(item, BaseException):
            self._exhausted = True
            raise item
        else:
            self._buffer.extend(item)

    async def pull(self, chunk_size: int) -> AudioChunk:
        chunk_size *= self._unit_bytes
        self._start()
        q = self._q
        while len(self._buffer) < chunk_size and not self._exhausted:
            try:
                item = q.get_nowait()  # already produced: no thread hop
            except queue.Empty:
                item = await asyncio.to_thread(q.get)
            self._take(item)
        if self._exhausted and not self._buffer:
            return AudioChunk(pcm=b"", duration_ms=0.0, eos=True)
        pcm = bytes(self._buffer[:chunk_size])
        del self._buffer[:chunk_size]
        return AudioChunk(pcm=pcm, duration_ms=len(pcm) / 2 / I.SAMPLE_RATE * 1000.0,
                          eos=self._exhausted and not self._buffer)

    async def reset(self) -> None:
        """Barge-in (llama_local.py:152-157): cancel the utterance, drop buffered audio."""
        if self._cancel is not None:
            self._cancel.set()
        q = self._q
        if q is not None:  # unblock a producer waiting on a full queue
            try:
                while True:
                    q.get_nowait()
            except queue.Empty:
                pass
        self._q = None
        self._cancel = None
        self._thread = None
        self._buffer.clear()
        self._exhausted = False


# The reference's import path for the adapter class name
TTSAdapter = MxTTSAdapter


def mx_describe() -> Dict[str, Any]:
    return {
        "name": "mi355x",
        "streaming": True,
        "unit": "ms",
        "granularity": [8, 12, 16, 24, 32, 48, 64],
        "voices": list(I.AVAILABLE_VOICES),
        "supports_barge_in": True,
        "supports_seed": False,
        "stateful_context": "minimal",
    }


def mx_voice_mapper(schema) -> Dict[str, Any]:
    voice = getattr(schema, "voice", None) or getattr(schema, "timbre", None) or I.DEFAULT_VOICE
    return {"voice": voice if voice in I.AVAILABLE_VOICES else I.DEFAULT_VOICE}


def register(registry, name: str = "mi355x", constructor=None) -> None:
    """``registry.register(name, constructor, describe, voice_mapper)`` (adapter_registry.py:76-83)."""
    registry.register(name, constructor or MxTTSAdapter, mx_describe, mx_voice_mapper)


class AdapterRegistry:
    """The registry contract the reference server creates adapters through
    (tts_engine/adapter_registry.py:70-98): ``register``, ``available`` (name -> descriptor)
    and ``create(name, *, prompt, voice, **kw)`` = ``constructor(prompt=prompt,
    **voice_mapper(voice), **kw)``.  This build's server keeps one with ``mi355x``; the
    reference's own registry takes the same adapter through ``register``."""

    def __init__(self) -> None:
        self._specs: Dict[str, tuple] = {}

    def register(self, name: str, constructor, describe, voice_mapper) -> None:
        self._specs[name] = (constructor, describe, voice_mapper)

    def available(self) -> Dict[str, Dict[str, Any]]:
        return {name: spec[1]() for name, spec in self._specs.items()}

    def create(self, name: str, *, prompt: str, voice, **kw):
        constructor, _, mapper = self._specs[name]
        params = mapper(voice)
        params.update(kw)
        return constructor(prompt=prompt, **params)
