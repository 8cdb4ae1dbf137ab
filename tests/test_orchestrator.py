"""The reference server's pull pattern (harness/orchestrator_contract.py, the bench / test
driver) on CPU: the ladder starts at 8 and steps by buffer depth (chunk_ladder.py:10-60),
every pull is logged with its base64 PCM (core.py:97-104), PCM arrives intact through
stitch_chunks and the WAV streamer, and barge-in resets the adapter."""
import asyncio
import base64
import functools

from starlette.testclient import TestClient

from harness.orchestrator_contract import PullDriver, next_rung, orchestrated_pcm_stream
from project_morpheus_amd.adapter import MxTTSAdapter
from project_morpheus_amd.server import build_app, riff_header

PCM = [bytes(range(256)) * 8, b"", bytes(range(100)), bytes(range(200)) * 3]


class Fake(MxTTSAdapter):
    @staticmethod
    def source(prompt, voice, use_batching, max_batch_chars, cancel):
        yield from PCM


def test_ladder_adapt():
    d = PullDriver(None)
    assert d.window == 8
    d.rung = next_rung(d.rung, 10.0)
    assert d.window == 12
    d.rung = next_rung(d.rung, 300.0)
    assert d.window == 8
    d.rung = next_rung(d.rung, 300.0)
    assert d.window == 8
    for _ in range(10):
        d.rung = next_rung(d.rung, 0.0)
    assert d.window == 64
    d.rung = next_rung(d.rung, 100.0)   # inside the comfort band: stays
    assert d.window == 64


def test_orchestrator_pulls_log_and_pcm():
    events = []

    async def go():
        o = PullDriver(Fake("x"))
        out = [c async for c in o.stream(on_event=events.append)]
        return o, out

    o, out = asyncio.run(go())
    pcm = b"".join(c.pcm for c in out)
    assert pcm == b"".join(PCM)
    assert out[-1].eos and o.pulls == len(events)
    assert b"".join(base64.b64decode(e["pcm"]) for e in events) == pcm
    windows = [e["token_window"] for e in events]
    assert windows[0] == 8 and max(windows) <= 64 and min(windows) >= 8


def test_barge_in_resets_adapter():
    class Counting(Fake):
        resets = 0

        async def reset(self):
            Counting.resets += 1
            await super().reset()

    async def go():
        o = PullDriver(Counting("x"))
        n = 0
        async for _ in o.stream():
            n += 1
            if n == 3:
                o.signal_barge_in()
        return o

    o = asyncio.run(go())
    assert Counting.resets == 1 and o.timeline[-1]["stage"] == "barge_in_reset"


def test_orchestrated_speech_route():
    orchs = []
    app = build_app(adapter_cls=Fake, orchestrated_stream=functools.partial(
        orchestrated_pcm_stream, drivers=orchs))
    r = TestClient(app).post("/v1/audio/speech", json={"input": "Hello", "voice": "tara"})
    assert r.status_code == 200
    assert r.content == riff_header() + b"".join(PCM)
    assert orchs and orchs[0].pulls >= len(b"".join(PCM)) // 64


def test_ms_pull_unit_option():
    """MORPHEUS_MX_PULL_UNIT=ms / pull_unit="ms": pull(n) returns n ms of PCM (48 n bytes),
    what the adapter descriptor declares (adapter_registry.py:54); default stays bytes."""
    async def go(unit):
        a = Fake("x", pull_unit=unit)
        o = PullDriver(a)
        out = [c async for c in o.stream()]
        return o.pulls, b"".join(c.pcm for c in out), [len(c.pcm) for c in out]

    n_b, pcm_b, _ = asyncio.run(go("bytes"))
    n_ms, pcm_ms, sizes = asyncio.run(go("ms"))
    assert pcm_b == pcm_ms == b"".join(PCM)
    assert sizes[0] == 8 * 48 and n_ms < n_b / 10
    import pytest
    with pytest.raises(ValueError):
        Fake("x", pull_unit="frames")
