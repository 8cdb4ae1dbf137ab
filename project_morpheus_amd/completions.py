"""OpenAI-style ``/v1/completions`` token stream over the MI355X engine.

Other Morpheus instances use a remote completions server as their LLM
(Morpheus_Client/tts_engine/remote_backend.py:64-117): they POST ``prompt`` (the string
framing ``<|audio|>{voice}: {text}<|eot_id|>``, inference.py:209-223), ``max_tokens``,
``temperature``, ``top_p``, ``repeat_penalty``, ``stream`` and ``model``, and read SSE
``data:`` events whose ``choices[0].text`` carries ``<custom_token_N>`` pieces until
``data: [DONE]``.  This module serves that contract from the per-GPU batch loop: the
request joins the continuous batch as a token-only stream (no SNAC work), and every token
the loop reads back is sent as one event.
"""
from __future__ import annotations

import asyncio
import json
import queue
import time
from typing import Any, Callable, Dict, List, Optional

from . import inference as I
from .config import CUSTOM_TOKEN_BASE

AUDIO_OPEN, AUDIO_CLOSE = "<|audio|>", "<|eot_id|>"


def prompt_ids_from_text(prompt: str, encode: Callable[[str], List[int]]) -> List[int]:
    """The string framing -> the id framing the engine decodes (P1): ``<|audio|>`` is the
    start-of-human marker, ``<|eot_id|>`` the end tokens; other prompts are taken as text."""
    if prompt.startswith(AUDIO_OPEN):
        inner = prompt[len(AUDIO_OPEN):]
        if inner.endswith(AUDIO_CLOSE):
            inner = inner[:-len(AUDIO_CLOSE)]
        return I.prompt_ids(encode(inner))
    return list(encode(prompt))


def token_text(tok: int, decode: Optional[Callable[[List[int]], str]] = None) -> str:
    if tok >= CUSTOM_TOKEN_BASE:
        return f"<custom_token_{tok - CUSTOM_TOKEN_BASE}>"
    return decode([tok]) if decode is not None else ""


def sse_event(cid: str, created: int, model: str, text: str, finish: Optional[str]) -> str:
    return "data: " + json.dumps({
        "id": cid, "object": "text_completion", "created": created, "model": model,
        "choices": [{"text": text, "index": 0, "logprobs": None, "finish_reason": finish}]},
        separators=(",", ":")) + "\n\n"


def params_from_payload(p: Dict[str, Any]) -> Dict[str, Any]:
    """Generation parameters of a request; ValueError (HTTP 400) for values the engine
    cannot run (non-numbers, temperature < 0, top_p outside (0, 1], penalty <= 0)."""
    from .batching import check_params
    try:
        out = {"max_tokens": int(p.get("max_tokens") or I.MAX_TOKENS),
               "temperature": float(p.get("temperature", I.TEMPERATURE)),
               "top_p": float(p.get("top_p", I.TOP_P)),
               "penalty": float(p.get("repeat_penalty", p.get("repetition_penalty",
                                                              I.REPETITION_PENALTY)))}
    except (TypeError, ValueError) as e:
        raise ValueError(f"bad generation parameter: {e}") from e
    check_params(out["penalty"], out["temperature"], out["top_p"], out["max_tokens"])
    return out


async def next_token(handle, poll_s: float = 0.002):
    """Await the next token of a handle without parking a thread per request."""
    while True:
        try:
            return handle.get(timeout=0)
        except queue.Empty:
            await asyncio.sleep(poll_s)


def build_route(token_source: Callable[..., Any], encode: Callable[[str], List[int]],
                decode: Optional[Callable[[List[int]], str]] = None):
    """Starlette endpoint.  ``token_source(prompt_ids, **params)`` returns a handle with
    ``get(timeout)`` -> token id | None (end) and ``cancel()``."""
    from starlette.requests import Request
    from starlette.responses import JSONResponse, StreamingResponse

    async def completions(request: Request):
        try:
            payload = await request.json()
        except Exception:
            return JSONResponse({"error": "invalid JSON"}, status_code=400)
        prompt = payload.get("prompt")
        if not isinstance(prompt, str) or not prompt:
            return JSONResponse({"error": "missing prompt"}, status_code=400)
        try:
            params = params_from_payload(payload)
            ids = prompt_ids_from_text(prompt, encode)
            handle = token_source(ids, **params)
        except ValueError as e:  # rejected before it reaches the GPU loop
            return JSONResponse({"error": str(e)}, status_code=400)
        model = str(payload.get("model", "orpheus-mi355x"))
        cid, created = f"cmpl-{id(handle):x}", int(time.time())

        async def events():
            n, finished = 0, False
            try:
                while True:
                    tok = await next_token(handle)
                    if tok is None:
                        break
                    n += 1
                    yield sse_event(cid, created, model, token_text(tok, decode), None)
                finished = True
                reason = "length" if n >= params["max_tokens"] else "stop"
                yield sse_event(cid, created, model, "", reason)
                yield "data: [DONE]\n\n"
            finally:
                if not finished:
                    handle.cancel()

        if payload.get("stream", False):
            return StreamingResponse(events(), media_type="text/event-stream")
        texts = []
        while True:
            tok = await next_token(handle)
            if tok is None:
                break
            texts.append(token_text(tok, decode))
        return JSONResponse({
            "id": cid, "object": "text_completion", "created": created, "model": model,
            "choices": [{"text": "".join(texts), "index": 0, "logprobs": None,
                         "finish_reason": "length" if len(texts) >= params["max_tokens"]
                         else "stop"}],
            "usage": {"prompt_tokens": len(ids), "completion_tokens": len(texts),
                      "total_tokens": len(ids) + len(texts)}})

    return completions
