"""Host-side rows of the hot path against golden vectors recorded from the REFERENCE
(tests/golden/make_host_golden.py): sentence split, long-form batching, WAV crossfade
stitch, AudioChunk overlap-add stitcher and the adapter's pull() byte slicing."""
import asyncio
import base64
import json
import os
import wave

import numpy as np
import pytest

from project_morpheus_amd import inference as I
from project_morpheus_amd.adapter import MxTTSAdapter
from project_morpheus_amd.audio import AudioChunk
from project_morpheus_amd.stitcher import stitch_chunks

GOLD = os.path.join(os.path.dirname(__file__), "golden", "host_golden.json")


@pytest.fixture(scope="module")
def host_golden():
    with open(GOLD) as fh:
        return json.load(fh)


def test_split_text_into_sentences(host_golden):
    for case in host_golden["split"]:
        assert I.split_text_into_sentences(case["text"]) == case["out"], case["text"][:60]


def test_long_form_batches(host_golden):
    for case in host_golden["batches"]:
        got = I.batch_sentences(case["text"], case["max_batch_chars"], case["use_batching"])
        assert got == case["out"]


def test_stitch_wav_files_crossfade(host_golden, tmp_path):
    for k, case in enumerate(host_golden["stitch_wav"]):
        files = []
        for i, b64 in enumerate(case["segments"]):
            f = tmp_path / f"c{k}_{i}.wav"
            with wave.open(str(f), "wb") as w:
                w.setnchannels(1)
                w.setsampwidth(2)
                w.setframerate(24000)
                w.writeframes(base64.b64decode(b64))
            files.append(str(f))
        out = tmp_path / f"c{k}_out.wav"
        I.stitch_wav_files(files, str(out), crossfade_ms=50)
        with wave.open(str(out), "rb") as w:
            assert w.readframes(w.getnframes()) == base64.b64decode(case["out"])


def test_stitch_chunks_overlap_add(host_golden):
    async def run(chunks, ov, em):
        async def src():
            for c in chunks:
                yield c
        return [c async for c in stitch_chunks(src(), sample_rate=1000, overlap_ms=ov,
                                                emit_markers=em)]

    for case in host_golden["stitch_chunks"]:
        vals = case["chunks"]
        chunks = [AudioChunk(pcm=np.asarray(v, dtype=np.int16).tobytes(), duration_ms=len(v),
                             markers={"i": i}, eos=False) for i, v in enumerate(vals)]
        if not case.get("no_eos"):
            chunks[-1] = AudioChunk(pcm=chunks[-1].pcm, duration_ms=len(vals[-1]),
                                    markers={"i": len(vals) - 1}, eos=True)
        else:
            chunks = [AudioChunk(pcm=c.pcm, duration_ms=c.duration_ms) for c in chunks]
        got = asyncio.run(run(chunks, case["overlap_ms"], case["emit_markers"]))
        want = case["out"]
        assert len(got) == len(want)
        for g, w in zip(got, want):
            assert np.frombuffer(g.pcm, dtype=np.int16).tolist() == w["pcm"]
            assert g.duration_ms == pytest.approx(w["duration_ms"])
            assert g.markers == w["markers"] and g.eos == w["eos"]


def test_adapter_pull_slicing(host_golden):
    for case in host_golden["adapter_pull"]:
        parts = [base64.b64decode(p) for p in case["parts"]]

        class A(MxTTSAdapter):
            @staticmethod
            def source(prompt, voice, use_batching, max_batch_chars, cancel):
                yield from parts

        ad = A("hi", "tara")

        async def pulls():
            return [await ad.pull(s) for s in case["sizes"]]
        got = asyncio.run(pulls())
        for g, w in zip(got, case["out"]):
            assert g.pcm == base64.b64decode(w["pcm"])
            assert g.duration_ms == pytest.approx(w["duration_ms"])
            assert g.eos == w["eos"]


def test_registry_contract():
    """register(registry) follows adapter_registry.py:76-98: create(name, *, prompt, voice,
    **kw) -> constructor(prompt=prompt, **voice_mapper(voice), **kw)."""
    from types import SimpleNamespace

    from project_morpheus_amd.adapter import mx_describe, mx_voice_mapper, register

    class Registry:  # the reference's AdapterRegistry call pattern
        def __init__(self):
            self._a = {}

        def register(self, name, constructor, describe, voice_mapper):
            self._a[name] = (constructor, describe, voice_mapper)

        def create(self, name, *, prompt, voice, **kw):
            ctor, _d, vm = self._a[name]
            return ctor(prompt=prompt, **vm(voice), **kw)

    reg = Registry()
    register(reg)
    ad = reg.create("mi355x", prompt="Hello", voice=SimpleNamespace(voice="leo", timbre=None),
                    use_batching=True, max_batch_chars=500)
    assert isinstance(ad, MxTTSAdapter) and ad.voice == "leo" and ad.max_batch_chars == 500
    assert mx_voice_mapper(SimpleNamespace(voice="nobody", timbre=None)) == {"voice": I.DEFAULT_VOICE}
    d = mx_describe()
    assert set(d) >= {"name", "streaming", "unit", "granularity", "voices", "supports_barge_in",
                      "supports_seed", "stateful_context"}


def test_adapter_reset_restarts_and_clears():
    calls = []

    class A(MxTTSAdapter):
        @staticmethod
        def source(prompt, voice, use_batching, max_batch_chars, cancel):
            calls.append(prompt)
            yield b"\x01\x00" * 8
            yield b"\x02\x00" * 8

    ad = A("p", "tara")

    async def go():
        a = await ad.pull(4)
        await ad.reset()
        b = await ad.pull(100)
        c = await ad.pull(100)
        return a, b, c
    a, b, c = asyncio.run(go())
    assert a.pcm == b"\x01\x00" * 2 and not a.eos
    assert b.pcm == b"\x01\x00" * 8 + b"\x02\x00" * 8 and b.eos
    assert c.pcm == b"" and c.eos
    assert calls == ["p", "p"]


def test_adapter_reset_does_not_wedge_the_producer():
    """a producer far ahead of the puller (> queue size) must not block
    forever after reset(); a second adapter still completes."""
    import asyncio
    import threading

    from project_morpheus_amd.adapter import MxTTSAdapter

    closed = threading.Event()

    class Busy(MxTTSAdapter):
        @staticmethod
        def source(prompt, voice, use_batching, max_batch_chars, cancel):
            try:
                for i in range(500):
                    yield bytes([i % 256]) * 100
            finally:
                closed.set()

    async def go():
        a = Busy("x")
        c = await a.pull(100)
        assert len(c.pcm) == 100
        await asyncio.sleep(0.3)  # producer fills the 64-entry queue and waits
        t = a._thread
        await a.reset()
        t.join(timeout=5)
        assert not t.is_alive() and closed.is_set()
        b = Busy("y")
        total = 0
        while True:
            ch = await b.pull(4096)
            total += len(ch.pcm)
            if ch.eos:
                break
        return total

    assert asyncio.run(go()) == 500 * 100
