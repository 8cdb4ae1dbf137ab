"""Overlap-add stitcher over AudioChunk streams.

Same contract as Morpheus_Client/orchestrator/stitcher.py:10-79 (``stitch_chunks``): a tail
of ``overlap_ms`` is held back from each chunk and linearly cross-faded (fade-out of the
tail, fade-in of the next head, ``endpoint=False`` ramps) into the next chunk; the
overlap is clamped to what both sides hold; ``eos`` flushes; markers pass only with
``emit_markers``.  With ``overlap_ms=0`` (the server's setting, server.py:154-156) chunks
pass through unchanged.
"""
from __future__ import annotations

from typing import AsyncGenerator, AsyncIterator

import numpy as np

from .audio import AudioChunk


def _chunk(pcm: np.ndarray, sr: int, markers, eos: bool) -> AudioChunk:
    return AudioChunk(pcm=pcm.astype("<i2").tobytes(), duration_ms=len(pcm) / sr * 1000.0,
                      markers=markers, eos=eos)


async def stitch_chunks(chunks: AsyncIterator[AudioChunk], *, sample_rate: int,
                        overlap_ms: float = 0.0,
                        emit_markers: bool = False) -> AsyncGenerator[AudioChunk, None]:
    ov_n = int(overlap_ms * sample_rate / 1000.0)
    held = np.zeros(0, dtype=np.int16)
    async for c in chunks:
        cur = np.frombuffer(c.pcm, dtype=np.int16)
        if held.size:
            k = min(ov_n, held.size, cur.size) if ov_n > 0 else 0
            if k:
                mixed = held[-k:] * np.linspace(1.0, 0.0, k, endpoint=False) + \
                    cur[:k] * np.linspace(0.0, 1.0, k, endpoint=False)
                cur = np.concatenate([held[:-k], mixed, cur[k:]])
            else:
                cur = np.concatenate([held, cur])
        mk = c.markers if emit_markers else None
        if c.eos:
            yield _chunk(cur, sample_rate, mk, True)
            held = np.zeros(0, dtype=np.int16)
            break
        if ov_n > 0:
            if cur.size <= ov_n:
                held = cur
                continue
            held = cur[-ov_n:]
            cur = cur[:-ov_n]
        else:
            held = np.zeros(0, dtype=np.int16)
        yield _chunk(cur, sample_rate, mk, False)
    if held.size:
        yield _chunk(held, sample_rate, None, True)
