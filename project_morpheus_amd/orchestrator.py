"""The reference's orchestrated serving contract, restated for the MI355X adapter.

The reference server never drains an adapter directly: ``/v1/audio/speech`` runs
``orchestrated_pcm_stream`` (Morpheus_Client/server.py:127-158), i.e. an ``Orchestrator``
(orchestrator/core.py:74-125) that pulls ``ladder.current`` units per call from the adapter
(a ``ChunkLadder`` of 8..64, chunk_ladder.py:7, starting at 8 and stepped by the playback
buffer depth against a 50-250 ms comfort band), builds a JSON log entry with the base64 PCM
of every pull (core.py:97-104), feeds ``stitch_chunks`` (overlap 0) and the WAV streamer
(server.py:72-77).  The adapter contract counts ``pull(n)`` in BYTES (llama_local.py:131),
so in steady state the ladder sits at 8-byte pulls: thousands of pulls per audio second,
which capped the reference's HTTP-level RTF at 12-19x on its CPU.

This module restates that control flow so the same serving path can be measured against
the MI355X engine (bench.py ``http_level_orchestrator``) and served (``server.build_app(
orchestrated=True)``).  The adapter side is what the build controls: ``MxTTSAdapter.pull``
answers tiny pulls from its buffer without leaving the event loop (adapter.py).
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import time
from dataclasses import dataclass, field
from typing import AsyncGenerator, Callable, List, Optional, Tuple

from . import inference as I
from .audio import AudioChunk
from .stitcher import stitch_chunks

logger = logging.getLogger(__name__)

DEFAULT_LADDER: List[int] = [8, 12, 16, 24, 32, 48, 64]


@dataclass
class ChunkLadder:
    """chunk_ladder.py:10-60: step up while the buffer is shallow, down while it is deep."""
    ladder: List[int] = field(default_factory=lambda: DEFAULT_LADDER.copy())
    index: int = 0

    @property
    def current(self) -> int:
        return self.ladder[self.index]

    def step_up(self) -> None:
        if self.index < len(self.ladder) - 1:
            self.index += 1

    def step_down(self) -> None:
        if self.index > 0:
            self.index -= 1

    def reset(self) -> None:
        self.index = 0

    def adapt(self, depth_ms: float, band: Tuple[float, float]) -> None:
        low, high = band
        if depth_ms < low:
            self.step_up()
        elif depth_ms > high:
            self.step_down()


@dataclass
class PlaybackBuffer:
    """orchestrator/buffer.py:14-43 (nothing consumes it on the server path)."""
    capacity_ms: float
    depth_ms: float = 0.0

    def add(self, duration_ms: float) -> None:
        self.depth_ms += duration_ms

    def consume(self, duration_ms: float) -> None:
        self.depth_ms = max(0.0, self.depth_ms - duration_ms)

    def reset(self) -> None:
        self.depth_ms = 0.0


class Orchestrator:
    """core.py:27-125: adaptive pulls, per-pull structured log, barge-in reset."""

    def __init__(self, adapter, buffer: PlaybackBuffer, ladder: Optional[ChunkLadder] = None,
                 comfort_band: Tuple[float, float] = (50.0, 250.0)):
        self.adapter = adapter
        self.buffer = buffer
        self.ladder = ladder or ChunkLadder()
        self.comfort_band = comfort_band
        self._barge_in = asyncio.Event()
        self.timeline: list = []
        self.pulls = 0

    def signal_barge_in(self) -> None:
        self._barge_in.set()

    def _record(self, stage: str, start: float, result: str) -> None:
        self.timeline.append({"stage": stage,
                              "duration_ms": (time.perf_counter() - start) * 1000.0,
                              "result": result})

    async def stream(self, on_event: Optional[Callable[[dict], None]] = None
                     ) -> AsyncGenerator[AudioChunk, None]:
        chunk_id = 0
        while not self._barge_in.is_set():
            adapter_name = getattr(self.adapter, "name", self.adapter.__class__.__name__)
            window = self.ladder.current
            start = time.perf_counter()
            chunk = await self.adapter.pull(window)
            render_ms = (time.perf_counter() - start) * 1000.0
            self.pulls += 1
            self._record("adapter_pull", start, "eos" if chunk.eos else "ok")
            log_entry = {"chunk_id": chunk_id, "adapter": adapter_name, "token_window": window,
                         "render_ms": render_ms,
                         "pcm": base64.b64encode(chunk.pcm).decode("ascii")}
            logger.info(json.dumps(log_entry))
            if on_event is not None:
                on_event(log_entry)
            self.buffer.add(chunk.duration_ms)
            yield chunk
            if chunk.eos:
                break
            self.ladder.adapt(self.buffer.depth_ms, self.comfort_band)
            chunk_id += 1
        if self._barge_in.is_set():
            start = time.perf_counter()
            await self.adapter.reset()
            self.buffer.reset()
            self._barge_in.clear()
            self._record("barge_in_reset", start, "ok")


async def orchestrated_pcm_stream(adapter, orchestrators: Optional[list] = None):
    """server.py:127-158 after adapter creation: Orchestrator -> stitch_chunks -> PCM bytes."""
    orch = Orchestrator(adapter, PlaybackBuffer(capacity_ms=1000), ChunkLadder())
    if orchestrators is not None:
        orchestrators.append(orch)
    async for chunk in stitch_chunks(orch.stream(), sample_rate=I.SAMPLE_RATE):
        yield chunk.pcm
