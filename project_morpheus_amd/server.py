"""The ``/v1/audio/speech`` and ``/ws/tts`` streaming surface over ``MxTTSAdapter``.

Restates the reference routes (Morpheus_Client/server.py:50-87 RIFF header + raw PCM16 frames,
:127-158 ``orchestrated_pcm_stream``, :161-190 ``SpeechRequest`` / ``create_speech_api``,
:209-222 ``tts_ws``, :236-239 ``/adapters``, :243-289 adapter / voice selection by
``POST /config``) for the MI355X adapter.  The reference runs BOTH speech routes through its
control plane's Orchestrator (server.py:127-158), which this package does not restate
(reused as-is above the adapter).  ``orchestrated_stream`` is that hook: a
callable ``adapter -> async iterator of PCM bytes`` (the reference's orchestrated stream in a
deployment, ``harness.orchestrator_contract.orchestrated_pcm_stream`` in the bench and the
tests); without it the routes drain the adapter with 4096-byte pulls (one SNAC window each).
With the harness driver the routes are pinned to the reference server's own bytes by
tests/test_server_golden.py (golden made by importing ``Morpheus_Client.server`` with this
adapter registered, tests/golden/make_server_golden.py).

Out of scope (control plane): text sources, ``/stats``, barge-in routes, the
admin UI and ``.env`` persistence of ``/config``.

    uvicorn project_morpheus_amd.server:app          # or build_app(adapter_cls=...)

The module-level ``app`` differs from the reference server in one observable way unless a
deployment configures the control plane's stream: without ``orchestrated_stream`` it serves
plain 4096-byte pulls, so the reference's ladder pull pattern and its per-pull INFO log record
are absent (the PCM bytes are the same).  ``MORPHEUS_MX_ORCHESTRATED_STREAM=module:callable``
(e.g. ``harness.orchestrator_contract:orchestrated_pcm_stream``, or the deployment's own
Orchestrator stream) selects the stream the module-level ``app`` uses.
"""
from __future__ import annotations

import importlib
import os
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
from .adapter import AdapterRegistry, MxTTSAdapter, register

PULL_BYTES = 4096  # one reference SNAC window per pull (speechpipe.py:120-135), unorchestrated


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


class VoiceSchema(BaseModel):
    """adapter_registry.py:22-36 (only ``voice`` / ``timbre`` are read by the mapper)."""
    voice: Optional[str] = None
    timbre: Optional[str] = None
    prosody: Optional[str] = None
    accent: Optional[str] = None
    emotion_priors: Optional[str] = None
    pace: Optional[str] = None


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


def build_app(adapter_cls=None, token_source=_service_tokens, encode=None,
              decode=None, orchestrated_stream=None,
              registry: Optional[AdapterRegistry] = None) -> Starlette:
    """``adapter_cls`` (tests / bench): the class registered as ``mi355x`` (default
    ``MxTTSAdapter``).  ``token_source(prompt_ids, **params)`` backs /v1/completions (default:
    this GPU's service); ``encode`` / ``decode`` default to the process tokenizer.
    ``orchestrated_stream(adapter)``: the control plane's PCM stream over an adapter (module
    docstring); None = plain 4096-byte pulls."""
    from .completions import build_route
    from .tokenizer import default_tokenizer
    if encode is None:
        encode = lambda s: default_tokenizer().encode(s)  # noqa: E731
    if registry is None:
        registry = AdapterRegistry()
        register(registry, constructor=adapter_cls or MxTTSAdapter)
    state = {"adapter": "mi355x", "voice": VoiceSchema(voice=I.DEFAULT_VOICE)}

    def make_adapter(prompt: str, voice, **kw):
        schema = state["voice"] if voice is None else VoiceSchema(voice=voice)
        return registry.create(state["adapter"], prompt=prompt, voice=schema, **kw)

    def pcm_stream(adapter):
        if orchestrated_stream is not None:
            return orchestrated_stream(adapter)
        return adapter_pcm(adapter)

    async def speech(request: Request) -> StreamingResponse:
        try:
            payload = SpeechRequest(**await request.json())
        except ValidationError as exc:
            raise HTTPException(status_code=400, detail=str(exc)) from exc
        if not payload.input:
            raise HTTPException(status_code=400, detail="Missing input text")
        adapter = make_adapter(payload.input, payload.voice,
                               use_batching=len(payload.input) > 1000, max_batch_chars=1000)

        async def body():
            done = False
            try:
                yield riff_header()
                async for pcm in pcm_stream(adapter):
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
            adapter = make_adapter(prompt, websocket.query_params.get("voice"))
            try:
                await websocket.send_bytes(riff_header())
                async for pcm in pcm_stream(adapter):
                    await websocket.send_bytes(pcm)
                await websocket.close()
            finally:
                await adapter.reset()  # no-op after a complete stream; cancels otherwise
        except WebSocketDisconnect:
            pass

    async def adapters(request: Request) -> JSONResponse:
        return JSONResponse(registry.available())

    async def get_config(request: Request) -> JSONResponse:
        return JSONResponse({"adapter": state["adapter"], "voice": state["voice"].voice})

    async def update_config(request: Request) -> JSONResponse:
        """server.py:243-289, the adapter / voice part (no .env persistence)."""
        try:
            data = await request.json()
        except Exception as exc:
            raise HTTPException(status_code=400, detail=str(exc)) from exc
        name = data.get("adapter")
        if name:
            if name not in registry.available():
                raise HTTPException(status_code=404, detail="Unknown adapter")
            state["adapter"] = name
        voice = data.get("voice")
        if voice:
            state["voice"] = VoiceSchema(**voice) if isinstance(voice, dict) \
                else VoiceSchema(voice=voice)
        return JSONResponse({"message": "ok", "adapter": state["adapter"],
                             "voice": state["voice"].model_dump()})

    return Starlette(routes=[Route("/v1/audio/speech", speech, methods=["POST"]),
                             Route("/v1/completions", build_route(token_source, encode, decode),
                                   methods=["POST"]),
                             Route("/v1/audio/voices", voices, methods=["GET"]),
                             WebSocketRoute("/ws/tts", tts_ws),
                             Route("/adapters", adapters, methods=["GET"]),
                             Route("/config", get_config, methods=["GET"]),
                             Route("/config", update_config, methods=["POST"])])


def configured_stream():
    """The orchestrated stream named by ``MORPHEUS_MX_ORCHESTRATED_STREAM`` ("module:callable"),
    or None (plain 4096-byte pulls)."""
    spec = os.environ.get("MORPHEUS_MX_ORCHESTRATED_STREAM", "").strip()
    if not spec:
        return None
    mod, sep, name = spec.partition(":")
    if not sep or not name:
        raise ValueError(f"MORPHEUS_MX_ORCHESTRATED_STREAM must be module:callable, got {spec!r}")
    return getattr(importlib.import_module(mod), name)


app: Optional[Starlette] = build_app(orchestrated_stream=configured_stream())
