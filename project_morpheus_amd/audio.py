"""AudioChunk: the unit the orchestrator pulls (Morpheus_Client/orchestrator/adapter.py:13-34).

Field-for-field the reference dataclass, so Morpheus's Orchestrator / stitcher / server
consume chunks from this package unchanged (they read ``.pcm``, ``.duration_ms``,
``.markers``, ``.eos`` only).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional


@dataclass
class AudioChunk:
    pcm: bytes                      # PCM16 little-endian mono
    duration_ms: float
    markers: Optional[object] = None
    eos: bool = False
