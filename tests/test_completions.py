"""/v1/completions token stream (project_morpheus_amd/completions.py) against the reference
client's contract (remote_backend.py:64-117), on CPU with a fake token source.

* The restated client parser (oracle/remote_ref.py) reproduces the reference's own token
  texts on every golden SSE body (tests/golden/sse_golden.json, made by the reference).
* The reference's request payload (same golden file) is accepted as sent; its parameters
  reach the engine; the SSE the server emits, parsed by the client's rules and fed through
  ``turn_token_into_id`` (schedule.parse_token_text), recovers the engine's token ids.
"""
import json
import os
import queue

from starlette.testclient import TestClient

from oracle import remote_ref as R
from project_morpheus_amd import inference as I
from project_morpheus_amd.completions import prompt_ids_from_text
from project_morpheus_amd.config import CUSTOM_TOKEN_BASE
from project_morpheus_amd.schedule import parse_token_text
from project_morpheus_amd.server import build_app
from project_morpheus_amd.tokenizer import Tokenizer

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "sse_golden.json")))


def test_parser_matches_reference_on_golden_bodies():
    for case in GOLDEN["cases"]:
        assert R.parse_sse_tokens(case["sse"].split("\n")) == case["tokens"], case["name"]


class _Handle:
    def __init__(self, toks):
        self.q = queue.Queue()
        for t in toks:
            self.q.put(t)
        self.q.put(None)
        self.cancelled = False

    def get(self, timeout=None):
        return self.q.get(timeout=timeout) if timeout else self.q.get_nowait()

    def cancel(self):
        self.cancelled = True


def _app(toks, seen):
    tok = Tokenizer(None)

    def source(ids, **params):
        seen.append((ids, params))
        return _Handle(toks)
    return build_app(token_source=source, encode=tok.encode), tok


def test_reference_payload_round_trip():
    # a 7-phase audio stream: custom token n = code + 10 + 4096 * (k % 7)
    codes = [5, 4000, 17, 1, 4095, 2048, 300, 12, 9]
    toks = [CUSTOM_TOKEN_BASE + 10 + 4096 * (k % 7) + c for k, c in enumerate(codes)]
    seen = []
    app, tok = _app(toks, seen)
    r = TestClient(app).post("/v1/completions", json=GOLDEN["payload"])
    assert r.status_code == 200 and r.headers["content-type"].startswith("text/event-stream")
    texts = R.parse_sse_tokens(r.text.split("\n"))
    # what the reference client does with them (speechpipe.turn_token_into_id per token)
    got, count = [], 0
    for t in texts:
        c = parse_token_text(t, count)
        if c is not None and c > 0:
            got.append(c)
            count += 1
    assert got == codes
    ids, params = seen[0]
    p = GOLDEN["payload"]
    assert ids == I.prompt_ids(tok.encode("leo: Hello world"))
    assert ids == prompt_ids_from_text(p["prompt"], tok.encode)
    assert params == {"max_tokens": p["max_tokens"], "temperature": p["temperature"],
                      "top_p": p["top_p"], "penalty": p["repeat_penalty"]}


def test_non_streaming_and_errors():
    seen = []
    app, _ = _app([CUSTOM_TOKEN_BASE + 11, CUSTOM_TOKEN_BASE + 4107], seen)
    c = TestClient(app)
    j = c.post("/v1/completions", json={"prompt": "<|audio|>tara: hi<|eot_id|>",
                                        "max_tokens": 2}).json()
    assert j["choices"][0]["text"] == "<custom_token_11><custom_token_4107>"
    assert j["choices"][0]["finish_reason"] == "length"
    assert j["usage"]["completion_tokens"] == 2
    assert c.post("/v1/completions", json={"max_tokens": 2}).status_code == 400


def test_bad_generation_parameters_are_rejected_before_the_engine():
    """A request the device cannot run is a 400 for that request, not a loop failure."""
    seen = []
    app, _ = _app([CUSTOM_TOKEN_BASE + 11], seen)
    c = TestClient(app)
    base = {"prompt": "<|audio|>tara: hi<|eot_id|>", "max_tokens": 2}
    for bad in ({"top_p": 0.0}, {"top_p": -1}, {"top_p": 1.5}, {"repeat_penalty": 0},
                {"repeat_penalty": -2.0}, {"temperature": -0.1}, {"temperature": "hot"},
                {"max_tokens": -3}):
        r = c.post("/v1/completions", json=dict(base, **bad))
        assert r.status_code == 400, bad
    assert seen == []
    assert c.post("/v1/completions", json=base).status_code == 200
    import pytest
    from project_morpheus_amd.batching import check_params
    with pytest.raises(ValueError):
        check_params(1.1, float("nan"), 0.9, 10)


def test_request_seed_is_fresh_unless_content_seeded(monkeypatch):
    from project_morpheus_amd import config as C
    ids = [1, 2, 3]
    assert C.request_seed(ids, 7) == 7
    monkeypatch.setattr(C, "CONTENT_SEED", 0)
    assert len({C.request_seed(ids) for _ in range(8)}) == 8
    monkeypatch.setattr(C, "CONTENT_SEED", 1)
    assert C.request_seed(ids) == C.request_seed(list(ids)) != C.request_seed([1, 2, 4])
