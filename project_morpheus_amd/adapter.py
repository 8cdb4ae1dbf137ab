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

Synthesis runs in a producer thread (the engine loop must keep the GPU queue full while
the orchestrator makes its small pulls); ``pull`` awaits the next chunk through
``asyncio.to_thread`` like llama_local.py:79.
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
    from .service import get_service
    svc = get_service()
    for part in I.batch_sentences(prompt, max_batch_chars, use_batching):
        for pcm in svc.stream(part, voice, cancel=cancel):
            yield pcm
        if cancel.is_set():
            return


class MxTTSAdapter:
    # injectable for tests: (prompt, voice, use_batching, max_batch_chars, cancel) -> bytes iter
    source: Callable[..., Iterator[bytes]] = staticmethod(_default_source)

    def __init__(self, prompt: str, voice: str = I.DEFAULT_VOICE, *, use_batching: bool = False,
                 max_batch_chars: int = 1000) -> None:
        self.prompt = prompt
        self.voice = voice
        self.use_batching = use_batching
        self.max_batch_chars = max_batch_chars
        self._buffer = bytearray()
        self._exhausted = False
        self._q: Optional[queue.Queue] = None
        self._cancel: Optional[threading.Event] = None
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None

    def _start(self) -> None:
        if self._q is not None or self._exhausted:
            return
        q: queue.Queue = queue.Queue(maxsize=64)
        cancel = threading.Event()

        def produce():
            try:
                for pcm in self.source(self.prompt, self.voice, self.use_batching,
                                       self.max_batch_chars, cancel):
                    if cancel.is_set():
                        break
                    q.put(bytes(pcm))
            except BaseException as e:  # surfaced to the caller of pull()
                q.put(e)
            finally:
                q.put(_END)

        self._q, self._cancel = q, cancel
        self._thread = threading.Thread(target=produce, name="mx-tts", daemon=True)
        self._thread.start()

    async def pull(self, chunk_size: int) -> AudioChunk:
        self._start()
        while len(self._buffer) < chunk_size and not self._exhausted:
            item = await asyncio.to_thread(self._q.get)
            if item is _END:
                self._exhausted = True
                break
            if isinstance(item, BaseException):
                self._exhausted = True
                raise item
            self._buffer.extend(item)
        if self._exhausted and not self._buffer:
            return AudioChunk(pcm=b"", duration_ms=0.0, eos=True)
        pcm = bytes(self._buffer[:chunk_size])
        del self._buffer[:chunk_size]
        return AudioChunk(pcm=pcm, duration_ms=len(pcm) / 2 / I.SAMPLE_RATE * 1000.0,
                          eos=self._exhausted and not self._buffer)

    async def reset(self) -> None:
        if self._cancel is not None:
            self._cancel.set()
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


def register(registry, name: str = "mi355x") -> None:
    """``registry.register(name, constructor, describe, voice_mapper)`` (adapter_registry.py:76-83)."""
    registry.register(name, MxTTSAdapter, mx_describe, mx_voice_mapper)
