"""Golden vectors for the OpenAI-style completions token stream, from the REFERENCE client.

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_sse_golden.py

Imports ``Morpheus_Client.tts_engine.remote_backend`` from /root/reference (stubs only for
the absent ``dotenv`` / ``snac`` packages, as make_host_golden.py) and drives its
``generate_tokens_from_api`` (remote_backend.py:64-117) against an in-process
``httpx.MockTransport`` serving fixed SSE bodies -- no network.  Records, per body, the
token texts the reference yields, and the request payload it sends (prompt framing and the
``prompt, max_tokens, temperature, top_p, repeat_penalty, stream, model`` keys).

Output: ``tests/golden/sse_golden.json`` (inputs + expected outputs only).
"""
from __future__ import annotations

import asyncio
import json
import os
import sys
import types

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sse_golden.json")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def chunk(text):
    return "data: " + json.dumps({"id": "cmpl-x", "object": "text_completion",
                                  "choices": [{"text": text, "index": 0,
                                               "finish_reason": None}]}) + "\n\n"


BODIES = {
    "one_token_per_event": "".join(chunk(f"<custom_token_{n}>") for n in (10, 4106, 8200, 20))
    + "data: [DONE]\n\n",
    "several_tokens_per_event": chunk("<custom_token_11><custom_token_4107>")
    + chunk("<custom_token_8203><custom_token_12290><custom_token_16400>")
    + "data: [DONE]\n\n",
    "text_and_empty_and_malformed": chunk("Hello") + chunk("") + "data: {not json}\n\n"
    + ": keep-alive\n\n" + chunk("<custom_token_4096>") + "data: [DONE]\n\n"
    + chunk("<custom_token_5>"),
    "no_done_marker": chunk("<custom_token_100>") + chunk("<custom_token_200>"),
}


def main():
    from make_host_golden import load_reference
    import httpx
    _, remote, _, _, _ = load_reference()
    sent = []

    def handler(request: httpx.Request) -> httpx.Response:
        sent.append(json.loads(request.content))
        return httpx.Response(200, text=BODIES[handler.body],
                              headers={"content-type": "text/event-stream"})

    real = httpx.AsyncClient
    remote.httpx = types.SimpleNamespace(
        AsyncClient=lambda *a, **k: real(transport=httpx.MockTransport(handler)))
    remote.API_URL = "http://mock/v1/completions"

    async def tokens(prompt):
        return [t async for t in remote.generate_tokens_from_api(prompt, voice="leo",
                                                                 max_tokens=77)]

    golden = {"source": "/root/reference/Morpheus_Client/tts_engine/remote_backend.py:64-117",
              "cases": []}
    for name, body in BODIES.items():
        handler.body = name
        golden["cases"].append({"name": name, "sse": body,
                                "tokens": asyncio.run(tokens("Hello world"))})
    golden["payload"] = sent[0]
    with open(OUT, "w") as f:
        json.dump(golden, f, indent=1)
    print(f"wrote {OUT}: {len(golden['cases'])} cases")


if __name__ == "__main__":
    main()
