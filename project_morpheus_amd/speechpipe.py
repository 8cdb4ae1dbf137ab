"""Drop-in for Morpheus_Client/tts_engine/speechpipe.py, backed by the MI355X SNAC kernels.

Same names and semantics (speechpipe.py:64,146,191,295):
  ``turn_token_into_id(token_string, index) -> int | None``
  ``convert_to_audio(multiframe, count) -> bytes | None``
  ``async tokens_decoder(token_gen) -> async bytes``      (window schedule incl. EOS flush)
  ``async tokens_decoder_sync(token_gen) -> async bytes``  (drops empty chunks, keeps order)
and the module globals ``model`` (here a ``SnacDecoder``, created on first use instead of at
import so importing never touches the GPU) and ``snac_device``.

Differences by design: no per-element device writes or host syncs per window (the
de-interleave runs inside the SNAC embed kernel); a code of 4096 passes the range check as
in the reference and then raises ``IndexError`` (what the reference's CPU embedding lookup
does) instead of reading past the codebook.  The id-level engine path
(``engine.Synthesizer``) shares the schedule in ``schedule.py`` and skips strings entirely.
"""
from __future__ import annotations

import asyncio
import os
from typing import AsyncIterator, List, Optional

import numpy as np

from .schedule import WindowScheduler, frames_for_slice, parse_token_text, window_valid

snac_device = "cuda"
CUSTOM_TOKEN_PREFIX = "<custom_token_"
_model = None
_seed = [0]


def _get_model():
    global _model
    if _model is None:
        from .engine import SnacDecoder
        from .config import MX_SNAC
        from .weights import load_snac_state_dict, synthetic_snac_weights
        w = load_snac_state_dict(MX_SNAC) if MX_SNAC else synthetic_snac_weights()
        _model = SnacDecoder(w, device=int(os.environ.get("MORPHEUS_MX_DEVICE", "0")))
    return _model


def __getattr__(name):  # PEP 562: ``speechpipe.model`` loads lazily
    if name == "model":
        return _get_model()
    raise AttributeError(name)


def turn_token_into_id(token_string: str, index: int) -> Optional[int]:
    return parse_token_text(token_string, index)


def convert_to_audio(multiframe: List[int], count: int) -> Optional[bytes]:
    if len(multiframe) < 7:
        return None
    nf = len(multiframe) // 7
    win = [int(v) for v in multiframe[: 7 * nf]]
    if not window_valid(win):
        return None
    if max(win) >= 4096:
        raise IndexError("index out of range in self (SNAC codebook has 4096 entries)")
    import torch
    m = _get_model()
    # only the frames the kept samples [2048, 4096) depend on (schedule.frames_for_slice)
    win = win[: 7 * frames_for_slice(nf, min(4096, 2048 * nf))]
    codes = torch.tensor(win, dtype=torch.int32, device=f"cuda:{m.device}").reshape(1, -1)
    _seed[0] += 1
    pcm, _ = m.decode(codes, seed=_seed[0])
    return pcm.cpu().numpy().tobytes()


async def tokens_decoder(token_gen: AsyncIterator[str]):
    sched = WindowScheduler()
    async for text in token_gen:
        for win in sched.push(turn_token_into_id(text, sched.count)):
            yield convert_to_audio(win, sched.count)
    for win in sched.flush():
        yield convert_to_audio(win, sched.count)


async def tokens_decoder_sync(syn_token_gen):
    """Producer task + bounded queue (speechpipe.py:295-337); empty chunks dropped."""
    q: asyncio.Queue = asyncio.Queue(maxsize=32)

    async def produce():
        try:
            async for chunk in tokens_decoder(syn_token_gen):
                if chunk:
                    await q.put(chunk)
        except Exception as e:  # the reference prints and ends the stream
            print(f"Error in audio producer: {e}")
        finally:
            await q.put(None)

    task = asyncio.create_task(produce())
    while True:
        item = await q.get()
        if item is None:
            break
        yield item
    await task
