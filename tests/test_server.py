"""``/v1/audio/speech`` + ``/ws/tts`` surface (reference Morpheus_Client/server.py:50-222) on CPU.

The adapter's synthesis source is replaced by a deterministic PCM generator, so these tests
check the HTTP / WebSocket framing, request validation and long-form switch; the GPU engine
behind the adapter is covered by tests/test_gpu_engine.py and bench.py's http_level line.
"""
import struct

import pytest

import numpy as np
from starlette.testclient import TestClient

from project_morpheus_amd import inference as I
from project_morpheus_amd.adapter import MxTTSAdapter
from project_morpheus_amd.server import build_app, riff_header

CALLS = []


def _pcm_for(prompt):
    rng = np.random.default_rng(len(prompt))
    return [rng.integers(-3000, 3000, size=n).astype(np.int16).tobytes()
            for n in (0, 2048, 2048, 1000, 2048)]


class FakeAdapter(MxTTSAdapter):
    @staticmethod
    def source(prompt, voice, use_batching, max_batch_chars, cancel):
        CALLS.append((prompt, voice, use_batching, max_batch_chars))
        yield from _pcm_for(prompt)


def _client():
    return TestClient(build_app(adapter_cls=FakeAdapter))


def test_riff_header_layout():
    h = riff_header()
    assert len(h) == 44
    f = struct.unpack("<4sI4s4sIHHIIHH4sI", h)
    assert f[0] == b"RIFF" and f[1] == 0xFFFFFFFF and f[2] == b"WAVE" and f[3] == b"fmt "
    assert f[4:11] == (16, 1, 1, I.SAMPLE_RATE, 2 * I.SAMPLE_RATE, 2, 16)
    assert f[11] == b"data" and f[12] == 0xFFFFFFFF


def test_speech_streams_header_then_pcm():
    CALLS.clear()
    r = _client().post("/v1/audio/speech", json={"input": "Hello world", "voice": "leo"})
    assert r.status_code == 200
    assert r.headers["content-type"].startswith("audio/wav")
    assert r.content == riff_header() + b"".join(_pcm_for("Hello world"))
    assert CALLS == [("Hello world", "leo", False, 1000)]


def test_speech_unknown_voice_falls_back_and_long_input_batches():
    CALLS.clear()
    text = "A sentence here. " * 80
    r = _client().post("/v1/audio/speech", json={"input": text, "voice": "nobody"})
    assert r.status_code == 200
    assert CALLS == [(text, I.DEFAULT_VOICE, True, 1000)]


def test_speech_rejects_empty_and_invalid():
    c = _client()
    assert c.post("/v1/audio/speech", json={"input": ""}).status_code == 400
    assert c.post("/v1/audio/speech", json={"voice": "tara"}).status_code == 400


def test_voices():
    j = _client().get("/v1/audio/voices").json()
    assert j["default"] == I.DEFAULT_VOICE and I.DEFAULT_VOICE in j["voices"]


def test_ws_tts_frames():
    with _client().websocket_connect("/ws/tts?prompt=Hi%20there&voice=tara") as ws:
        frames = [ws.receive_bytes()]
        try:
            while True:
                frames.append(ws.receive_bytes())
        except Exception:
            pass
    assert frames[0] == riff_header()
    assert b"".join(frames[1:]) == b"".join(_pcm_for("Hi there"))


def test_module_app_stream_is_configurable(monkeypatch):
    """MORPHEUS_MX_ORCHESTRATED_STREAM selects the module-level app's orchestrated stream
    (the default app serves plain pulls, not the reference's ladder + log)."""
    from project_morpheus_amd import server
    monkeypatch.delenv("MORPHEUS_MX_ORCHESTRATED_STREAM", raising=False)
    assert server.configured_stream() is None
    monkeypatch.setenv("MORPHEUS_MX_ORCHESTRATED_STREAM",
                       "harness.orchestrator_contract:orchestrated_pcm_stream")
    from harness.orchestrator_contract import orchestrated_pcm_stream
    assert server.configured_stream() is orchestrated_pcm_stream
    monkeypatch.setenv("MORPHEUS_MX_ORCHESTRATED_STREAM", "no_colon")
    with pytest.raises(ValueError):
        server.configured_stream()
