"""Oracle: restatement of the reference client's completions-stream parsing (TEST INFRASTRUCTURE).

``generate_tokens_from_api`` (Morpheus_Client/tts_engine/remote_backend.py:103-117) reads an
OpenAI-style SSE body line by line: ``data: [DONE]`` ends the stream; every other ``data:``
line is JSON whose ``choices[0].text`` is split on ``>`` and each piece re-suffixed with
``>`` (so an event ending in ``>`` also yields a bare ``">"``, and an empty text yields
``">"``); undecodable JSON lines are skipped.  Pinned by tests/golden/sse_golden.json,
generated from the reference module itself (tests/golden/make_sse_golden.py).
"""
from __future__ import annotations

import json
from typing import Iterable, List


def parse_sse_tokens(lines: Iterable[str]) -> List[str]:
    out: List[str] = []
    for line in lines:
        if not line or not line.startswith("data: "):
            continue
        data_str = line[6:]
        if data_str.strip() == "[DONE]":
            break
        try:
            data = json.loads(data_str)
        except json.JSONDecodeError:
            continue
        if "choices" in data and data["choices"]:
            for piece in data["choices"][0].get("text", "").split(">"):
                out.append(f"{piece}>")
    return out
