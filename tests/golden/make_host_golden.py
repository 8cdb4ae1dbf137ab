"""Generate golden vectors for the host-side rows of the hot path from the REFERENCE modules.

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_host_golden.py

Imports ``Morpheus_Client`` from /root/reference with stub modules for the packages the
image lacks (``dotenv``: no-op ``load_dotenv``; ``snac``: never called here) and records,
for fixed inputs (seeded text generator, seed 5 as SURVEY.md §8d's long_read workload):

* ``split_text_into_sentences`` (tts_engine/inference.py:249-292);
* the long-form sentence batches of ``generate_speech_from_api``
  (tts_engine/remote_backend.py:221-241), captured by replacing its module-level
  ``generate_tokens_from_api`` / ``tokens_decoder`` with recorders (no network);
* ``stitch_wav_files`` 50 ms crossfade output (inference.py:294-365) on small WAVs;
* ``stitch_chunks`` overlap-add (orchestrator/stitcher.py:10-79) on AudioChunk sequences;
* ``llama_local.TTSAdapter.pull`` slicing (llama_local.py:120-150) over a fake model stream.

Output: ``tests/golden/host_golden.json`` (inputs + expected outputs only).
"""
from __future__ import annotations

import asyncio
import base64
import json
import os
import sys
import tempfile
import types
import wave

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host_golden.json")

WORDS = ("the of and to a in is you that it he was for on are as with his they I at be "
         "this have from or one had by word but not what all were we when your can said "
         "there use an each which she do how their if will up other about out many then "
         "them these so some her would make like him into time has look two more write go "
         "see number no way could people my than first water been call who oil its now find "
         "Dr. Mr. St. U.S. e.g. etc.").split()


def synth_text(rng, n_chars):
    """Seeded prose with sentence punctuation, abbreviations and short sentences."""
    out, cur = [], []
    while sum(len(w) + 1 for w in out) < n_chars:
        w = WORDS[int(rng.integers(0, len(WORDS)))]
        cur.append(w)
        if len(cur) >= int(rng.integers(1, 14)):
            end = "!?."[int(rng.integers(0, 3))] if rng.random() < 0.9 else ""
            out.extend(cur[:-1] + [cur[-1] + end])
            cur = []
            if rng.random() < 0.1:
                out[-1] += "\n"
    return " ".join(out).replace("\n ", "\n")[:n_chars]


def load_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("dotenv", types.SimpleNamespace(load_dotenv=lambda *a, **k: None))
    class _NoSNAC:  # speechpipe loads a model at import; it is never called here
        @classmethod
        def from_pretrained(cls, *_a, **_k):
            return cls()

        def eval(self):
            return self

        def to(self, *_a, **_k):
            return self

    sys.modules.setdefault("snac", types.SimpleNamespace(SNAC=_NoSNAC))
    sys.path.insert(0, REF)
    import Morpheus_Client.orchestrator.stitcher as stitcher  # noqa: E402
    import Morpheus_Client.tts_engine.inference as inference  # noqa: E402
    import Morpheus_Client.tts_engine.llama_local as llama_local  # noqa: E402
    import Morpheus_Client.tts_engine.remote_backend as remote  # noqa: E402
    from Morpheus_Client.orchestrator.adapter import AudioChunk  # noqa: E402
    return inference, remote, stitcher, llama_local, AudioChunk


def main():
    inference, remote, stitcher, llama_local, AudioChunk = load_reference()
    rng = np.random.default_rng(5)
    golden = {"source": REF, "split": [], "batches": [], "stitch_wav": [], "stitch_chunks": [],
              "adapter_pull": []}

    # (1) sentence splitting
    texts = ["", "Hello world.", "Hi. Ok. Yes! No? Fine.", "Dr. Smith went to Washington. He left.",
             "A.B. test. Ends with no punctuation", "Line one.\nLine two!\tTab three? end",
             "Short. " * 12, "x" * 50 + ". " + "y" * 10 + "! z"]
    texts += [synth_text(rng, n) for n in (120, 400, 999, 1000, 1001, 3000, 3000, 4500)]
    for t in texts:
        golden["split"].append({"text": t, "out": inference.split_text_into_sentences(t)})

    # (2) long-form batching inside generate_speech_from_api (no network: recorders)
    recorded = []

    def fake_tokens(prompt, **_kw):
        recorded.append(prompt)
        return None

    async def fake_decoder(_gen):
        if False:
            yield b""

    remote.generate_tokens_from_api = fake_tokens
    remote.tokens_decoder = fake_decoder

    async def batches_of(text, use_batching, max_chars):
        recorded.clear()
        agen = await remote.generate_speech_from_api(text, use_batching=use_batching,
                                                     max_batch_chars=max_chars)
        async for _ in agen:
            pass
        return list(recorded)

    for t, ub, mc in [(texts[-1], True, 1000), (texts[-2], True, 1000), (texts[-3], True, 1000),
                      (texts[-5], True, 1000), (texts[-6], True, 1000), (texts[-4], False, 1000),
                      (texts[-1], True, 400), (texts[3], True, 10)]:
        golden["batches"].append({"text": t, "use_batching": ub, "max_batch_chars": mc,
                                  "out": asyncio.run(batches_of(t, ub, mc))})

    # (3) stitch_wav_files crossfade on small WAVs
    with tempfile.TemporaryDirectory() as d:
        for lens in ([3000, 2500, 4000], [800, 3000], [3000, 900, 3000], [5000], [1200, 1200]):
            files, segs = [], []
            for i, n in enumerate(lens):
                seg = rng.integers(-20000, 20000, size=n).astype(np.int16)
                f = os.path.join(d, f"in{i}.wav")
                with wave.open(f, "wb") as w:
                    w.setnchannels(1)
                    w.setsampwidth(2)
                    w.setframerate(24000)
                    w.writeframes(seg.tobytes())
                files.append(f)
                segs.append(base64.b64encode(seg.tobytes()).decode())
            outf = os.path.join(d, "out.wav")
            inference.stitch_wav_files(files, outf, crossfade_ms=50)
            with wave.open(outf, "rb") as w:
                out = w.readframes(w.getnframes())
            golden["stitch_wav"].append({"segments": segs,
                                         "out": base64.b64encode(out).decode()})

    # (4) stitch_chunks overlap-add on AudioChunk sequences
    async def run_stitch(chunks, overlap_ms, emit_markers):
        async def src():
            for c in chunks:
                yield c
        res = []
        async for c in stitcher.stitch_chunks(src(), sample_rate=1000, overlap_ms=overlap_ms,
                                              emit_markers=emit_markers):
            res.append({"pcm": np.frombuffer(c.pcm, dtype=np.int16).tolist(),
                        "duration_ms": c.duration_ms, "markers": c.markers, "eos": c.eos})
        return res

    def mk(vals, eos=False, markers=None):
        a = np.asarray(vals, dtype=np.int16)
        return AudioChunk(pcm=a.tobytes(), duration_ms=len(a), markers=markers, eos=eos)

    seqs = [
        ([[0, 1, 2, 3, 4], [4, 3, 2, 1, 0]], 0, False),
        ([[0, 1, 2, 3, 4], [4, 3, 2, 1, 0]], 2, False),
        ([[10] * 7, [20] * 7, [30] * 7], 3, False),
        ([[1, 2], [3, 4, 5, 6], [7]], 3, False),
        ([[5] * 10, [6] * 10], 4, True),
    ]
    for vals, ov, em in seqs:
        chunks = [mk(v, markers={"i": i}) for i, v in enumerate(vals)]
        chunks[-1] = mk(vals[-1], eos=True, markers={"i": len(vals) - 1})
        golden["stitch_chunks"].append({"chunks": vals, "overlap_ms": ov, "emit_markers": em,
                                        "out": asyncio.run(run_stitch(chunks, ov, em))})
    # no eos chunk: the held tail is flushed at the end
    chunks = [mk([1, 2, 3, 4, 5, 6]), mk([7, 8, 9, 10, 11, 12])]
    golden["stitch_chunks"].append({"chunks": [[1, 2, 3, 4, 5, 6], [7, 8, 9, 10, 11, 12]],
                                    "overlap_ms": 2, "emit_markers": False, "no_eos": True,
                                    "out": asyncio.run(run_stitch(chunks, 2, False))})

    # (5) llama_local.TTSAdapter.pull slicing over a fake model stream
    async def fake_load():
        return None

    def make_stream(parts):
        async def _stream(_model, *_a):
            for p in parts:
                yield bytes(p)
        return _stream

    llama_local._load_model = fake_load
    for parts, sizes in [([b"\x01\x02" * 5, b"\x03\x04" * 3], [4, 4, 4, 4, 4, 4]),
                         ([b"a" * 7, b"b" * 2, b"c" * 9], [8, 8, 8, 8, 8]),
                         ([b"z" * 3], [64, 64]),
                         ([], [8, 8]),
                         ([b"q" * 100], [16, 48, 64, 64])]:
        llama_local._stream_from_model = make_stream(parts)
        ad = llama_local.TTSAdapter("hi", "tara")

        async def pulls():
            out = []
            for s in sizes:
                c = await ad.pull(s)
                out.append({"pcm": base64.b64encode(c.pcm).decode(),
                            "duration_ms": c.duration_ms, "eos": c.eos})
            return out
        golden["adapter_pull"].append({"parts": [base64.b64encode(p).decode() for p in parts],
                                       "sizes": sizes, "out": asyncio.run(pulls())})

    with open(OUT, "w") as fh:
        json.dump(golden, fh, indent=0, sort_keys=True)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
