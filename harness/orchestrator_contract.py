"""The pull pattern the reference server applies to an adapter, as a bench / test driver.

Behaviour followed (reference files under /root/reference/Morpheus_Client/):
* ``server.py:127-158`` -- both speech routes stream ``orchestrated_pcm_stream``: an
  orchestrator over the adapter, ``stitch_chunks`` with overlap 0, then the WAV frames;
* ``orchestrator/core.py:74-125`` -- each call pulls ``window`` units, logs one JSON record per
  pull (chunk id, adapter name, window, render time, base64 PCM) at INFO, adds the chunk's
  duration to the playback depth, stops at eos, then adapts the window; a barge-in ends the
  loop and resets adapter and depth;
* ``orchestrator/chunk_ladder.py:7-60`` -- windows 8, 12, 16, 24, 32, 48, 64, starting at
  8; one rung up while the depth is below 50 ms, one down above 250 ms;
* ``orchestrator/buffer.py:14-43`` -- the depth only grows on the server path.

The adapter contract counts pulls in bytes (llama_local.py:131), so this driver makes
thousands of tiny pulls per audio second: it is how the HTTP-level bench lines and the
server golden test exercise ``MxTTSAdapter``.  Not imported by ``project_morpheus_amd``.
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import time
from typing import AsyncIterator, Callable, List, Optional

from project_morpheus_amd import inference as I
from project_morpheus_amd.stitcher import stitch_chunks

log = logging.getLogger(__name__)

WINDOWS = (8, 12, 16, 24, 32, 48, 64)
COMFORT_MS = (50.0, 250.0)


def next_rung(rung: int, depth_ms: float) -> int:
    """chunk_ladder.py:51-60 for the default ladder: the rung after one adaptation."""
    if depth_ms < COMFORT_MS[0]:
        return min(rung + 1, len(WINDOWS) - 1)
    if depth_ms > COMFORT_MS[1]:
        return max(rung - 1, 0)
    return rung


class PullDriver:
    """One request's pull loop; ``pulls`` and ``timeline`` are read by the bench."""

    def __init__(self, adapter):
        self.adapter = adapter
        self.rung = 0
        self.depth_ms = 0.0
        self.pulls = 0
        self.timeline: list = []
        self._stop = asyncio.Event()

    @property
    def window(self) -> int:
        return WINDOWS[self.rung]

    def signal_barge_in(self) -> None:
        self._stop.set()

    async def stream(self, on_event: Optional[Callable[[dict], None]] = None) -> AsyncIterator:
        name = getattr(self.adapter, "name", type(self.adapter).__name__)
        n = 0
        while not self._stop.is_set():
            w = self.window
            t0 = time.perf_counter()
            chunk = await self.adapter.pull(w)
            dt = time.perf_counter() - t0
            self.pulls += 1
            self.timeline.append({"stage": "adapter_pull", "duration_ms": dt * 1e3,
                                  "result": "eos" if chunk.eos else "ok"})
            rec = {"chunk_id": n, "adapter": name, "token_window": w, "render_ms": dt * 1e3,
                   "pcm": base64.b64encode(chunk.pcm).decode("ascii")}
            log.info(json.dumps(rec))
            if on_event is not None:
                on_event(rec)
            self.depth_ms += chunk.duration_ms
            yield chunk
            if chunk.eos:
                break
            self.rung = next_rung(self.rung, self.depth_ms)
            n += 1
        if self._stop.is_set():
            t0 = time.perf_counter()
            await self.adapter.reset()
            self.depth_ms = 0.0
            self._stop.clear()
            self.timeline.append({"stage": "barge_in_reset",
                                  "duration_ms": (time.perf_counter() - t0) * 1e3,
                                  "result": "ok"})


def orchestrated_pcm_stream(adapter, drivers: Optional[List[PullDriver]] = None):
    """``server.build_app(orchestrated_stream=...)`` hook: the reference server's stream body
    for one adapter (PCM bytes, stitched with overlap 0)."""
    drv = PullDriver(adapter)
    if drivers is not None:
        drivers.append(drv)

    async def body():
        async for chunk in stitch_chunks(drv.stream(), sample_rate=I.SAMPLE_RATE):
            yield chunk.pcm
    return body()
