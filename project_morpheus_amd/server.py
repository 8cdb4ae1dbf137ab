"""The ``/v1/audio/speech`` and ``/ws/tts`` streaming surface over ``MxTTSAdapter``.

Restates the reference routes (Morpheus_Client/server.py:50-87 RIFF header + raw PCM16 frames,
:161-190 ``SpeechRequest`` / ``create_speech_api``, :209-222 ``tts_ws``) for the MI355X
adapter, so the HTTP-level path can be served and measured without the reference's control
plane (orchestrator ladder / playback buffer / text sources are out of scope).
With the server's stitcher at ``overlap_ms=0`` (server.py:154-156) the reference body is the
adapter's PCM concatenated, which is what is streamed here.

    uvicorn project_morpheus_amd.server:app          # or build_app(adapter_cls=...)
"""
from __future__ import annotations

import struct
from typing import Optional

from pydantic import BaseModel, ValidationError
from starlette.applications import Starlette
from starlette.exceptions import HTTPException
from starlette.requests import Request
from starlette.responses import JSONResponse, StreamingResponse
from starlette.routing import Route, WebSocketRoute
from starlette.websockets import WebSocket, WebSocketDisconnect

from . import inference as I
from .adapter import MxTTSAdapter

PULL_BYTES = 4096  # one reference SNAC window per pull (speechpipe.py:120-135)


def riff_header(sample_rate: int = I.SAMPLE_RATE) -> bytes:
    """PCM16 mono WAV header with unknown (0xFFFFFFFF) RIFF and data sizes (server.py:50-69)."""
    return struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 0xFFFFFFFF, b"WAVE", b"fmt ", 16, 1, 1,
                       sample_rate, sample_rate * 2, 2, 16, b"data", 0xFFFFFFFF)


class SpeechRequest(BaseModel):
    input: str
    model: str = "mi355x"
    voice: str = I.DEFAULT_VOICE
    response_format: str = "wav"
    speed: float = 1.0


async def adapter_pcm(adapter) -> "AsyncIterator[bytes]":
    """Drain an adapter with fixed-size pulls until eos; empty chunks are not emitted."""
    while True:
        chunk = await adapter.pull(PULL_BYTES)
        if chunk.pcm:
            yield chunk.pcm
        if chunk.eos:
            return


def _service_tokens(prompt_ids, **params):
    from .service import get_service
    return get_service().submit_tokens(prompt_ids, **params)


def build_app(adapter_cls=MxTTSAdapter, token_source=_service_tokens, encode=None,
              decode=None, orchestrated: bool = False, orchestrators=None) -> Starlette:
    """``token_source(prompt_ids, **params)`` backs /v1/completions (default: this GPU's
    service); ``encode`` / ``decode`` default to the process tokenizer.  ``orchestrated``:
    /v1/audio/speech runs the reference's Orchestrator contract (ladder pulls of 8-64 bytes,
    per-pull JSON/base64 log, stitcher; orchestrator.py) instead of 4096-byte pulls."""
    from .completions import build_route
    from .tokenizer import default_tokenizer
    if encode is None:
        encode = lambda s: default_tokenizer().encode(s)  # noqa: E731
    async def speech(request: Request) -> StreamingResponse:
        try:
            payload = SpeechRequest(**await request.json())
        except ValidationError as exc:
            raise HTTPException(status_code=400, detail=str(exc)) from exc
        if not payload.input:
            raise HTTPException(status_code=400, detail="Missing input text")
        adapter = adapter_cls(payload.input, I.resolve_voice(payload.voice),
                              use_batching=len(payload.input) > 1000, max_batch_chars=1000)

        async def body():
            done = False
            try:
                yield riff_header()
                if orchestrated:
                    from .orchestrator import orchestrated_pcm_stream
                    pcm_iter = orchestrated_pcm_stream(adapter, orchestrators)
                else:
                    pcm_iter = adapter_pcm(adapter)
                async for pcm in pcm_iter:
                    yield pcm
                done = True
            finally:
                if not done:  # client went away: cancel the GPU stream, free its row
                    await adapter.reset()

        return StreamingResponse(body(), media_type="audio/wav")

    async def voices(request: Request) -> JSONResponse:
        return JSONResponse({"status": "ok", "voices": list(I.AVAILABLE_VOICES),
                             "languages": list(I.AVAILABLE_LANGUAGES),
                             "default": I.DEFAULT_VOICE})

    async def tts_ws(websocket: WebSocket) -> None:
        await websocket.accept()
        try:
            prompt = websocket.query_params.get("prompt") or ""
            if not prompt:
                await websocket.close(code=1008)
                return
            voice = I.resolve_voice(websocket.query_params.get("voice") or I.DEFAULT_VOICE)
            adapter = adapter_cls(prompt, voice)
            try:
                await websocket.send_bytes(riff_header())
                async for pcm in adapter_pcm(adapter):
                    await websocket.send_bytes(pcm)
                await websocket.close()
            finally:
                await adapter.reset()  # no-op after a complete stream; cancels otherwise
        except WebSocketDisconnect:
            pass

    return Starlette(routes=[Route("/v1/audio/speech", speech, methods=["POST"]),
                             Route("/v1/completions", build_route(token_source, encode, decode),
                                   methods=["POST"]),
                             Route("/v1/audio/voices", voices, methods=["GET"]),
                             WebSocketRoute("/ws/tts", tts_ws)])


app: Optional[Starlette] = build_app()
