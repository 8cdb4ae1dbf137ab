"""Generate golden vectors for the speechpipe host logic from the REFERENCE module.

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_speechpipe_golden.py

It loads ``/root/reference/Morpheus_Client/tts_engine/speechpipe.py`` as a stand-alone
module (no package ``__init__``), with a *recording fake* ``snac`` module installed in
``sys.modules``: the third-party SNAC codec is not installed here and its weights are a
remote fetch.  The fake's ``decode`` returns a deterministic float32
waveform computed from the codes (``fake_decode`` below, restated verbatim in
``tests/test_speechpipe_golden.py``), so the reference's window schedule
(``speechpipe.py:191-293``), de-interleave (``:84-98``), range check (``:108-111``),
slice and PCM16 epilogue (``:120-135``) are all exercised for real.

Output: ``tests/golden/speechpipe_golden.json`` (inputs + expected outputs only).
"""
from __future__ import annotations

import asyncio
import hashlib
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/Morpheus_Client/tts_engine/speechpipe.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "speechpipe_golden.json")

CALLS: list = []


def fake_decode(c0, c1, c2):
    """Deterministic stand-in for SNAC.decode: 2048 samples per frame, float32."""
    n = len(c0)
    j = np.arange(2048 * n, dtype=np.int64)
    f = j // 2048
    c0 = np.asarray(c0, dtype=np.int64)
    c1 = np.asarray(c1, dtype=np.int64)
    c2 = np.asarray(c2, dtype=np.int64)
    v = (c0[f] + 3 * c1[2 * f] + 5 * c2[4 * f + 3] + (j % 2048)) % 4001
    return (v.astype(np.float32) / np.float32(4000.0)) - np.float32(0.5)


class _RecordingSNAC:
    @classmethod
    def from_pretrained(cls, *_a, **_k):
        return cls()

    def eval(self):
        return self

    def to(self, *_a, **_k):
        return self

    def decode(self, codes):
        c0, c1, c2 = (c.reshape(-1).tolist() for c in codes)
        CALLS.append([c0, c1, c2])
        audio = fake_decode(c0, c1, c2)
        return torch.from_numpy(audio).reshape(1, 1, -1)


def load_reference():
    sys.dont_write_bytecode = True
    sys.modules["snac"] = types.SimpleNamespace(SNAC=_RecordingSNAC)
    spec = importlib.util.spec_from_file_location("ref_speechpipe", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.snac_device == "cpu"
    return mod


def tok(n: int) -> str:
    return f"<custom_token_{n}>"


def audio_tok(code: int, phase: int) -> str:
    # speechpipe.py:181 inverted: n = code + 10 + 4096 * phase
    return tok(code + 10 + 4096 * phase)


def stream_from_codes(codes):
    return [audio_tok(c, i % 7) for i, c in enumerate(codes)]


async def _agen(items):
    for it in items:
        yield it


def run_decoder(mod, strings):
    CALLS.clear()

    async def go():
        return [b async for b in mod.tokens_decoder(_agen(strings))]

    outs = asyncio.run(go())
    windows = [list(c) for c in CALLS]
    CALLS.clear()

    async def go_sync():
        return [b async for b in mod.tokens_decoder_sync(_agen(strings))]

    outs_sync = asyncio.run(go_sync())
    CALLS.clear()
    return {
        "windows": windows,
        "out_lens": [len(b) for b in outs],
        "out_sha256": [hashlib.sha256(b).hexdigest() for b in outs],
        "sync_lens": [len(b) for b in outs_sync],
        "sync_sha256": [hashlib.sha256(b).hexdigest() for b in outs_sync],
    }


def main():
    mod = load_reference()
    rng = np.random.default_rng(20250824)
    golden = {"source": REF, "turn_token_into_id": [], "streams": [], "convert_to_audio": []}

    # (1) turn_token_into_id cases (speechpipe.py:146-189)
    cases = [
        (tok(10), 0), (tok(4105), 0), (tok(4106), 1), (tok(10 + 4096 * 6 + 17), 6),
        (tok(10 + 4096 * 6 + 17), 13), (tok(9), 0), (tok(10), 3), (tok(4106), 0),
        ("hello", 0), ("", 2), ("<custom_token_abc>", 0), ("<custom_token_12", 0),
        ("  <custom_token_200>  ", 4), ("prefix<custom_token_5><custom_token_300>", 0),
        ("<custom_token_300>tail", 0), ("<custom_token_-5>", 0), ("<custom_token_ 42>", 0),
        ("<custom_token_1_000>", 0), (tok(128), 7), (tok(4096 + 10), 0),
    ]
    for s, i in cases:
        golden["turn_token_into_id"].append({"s": s, "i": i, "out": mod.turn_token_into_id(s, i)})

    # (2) streams through tokens_decoder / tokens_decoder_sync (speechpipe.py:191-337)
    def rand_codes(n):
        return rng.integers(1, 4096, size=n).tolist()

    specs = []
    for n in (0, 6, 7, 8, 13, 14, 27, 28, 30, 35, 42, 48, 49, 50, 56, 63, 70, 77, 100, 141):
        specs.append((f"plain_{n}", stream_from_codes(rand_codes(n))))
    # code 0 is dropped (token > 0, :215) and shifts the 7-phase
    c = rand_codes(40)
    s = stream_from_codes(c)
    s.insert(9, audio_tok(0, 9 % 7))
    s.insert(20, audio_tok(0, 5))
    specs.append(("zero_drop", s))
    # non-custom strings interleaved (turn_token_into_id -> None)
    s = stream_from_codes(rand_codes(60))
    for k in (0, 5, 33, 50):
        s.insert(k, "hello")
    specs.append(("noncustom", s))
    # out-of-range code in the first window: first window retries on buffer[-7:] (:233-241)
    c = rand_codes(40)
    s = stream_from_codes(c)
    s[3] = tok(-100 + 10 + 4096 * 3)  # negative code -> dropped? no: -100 <= 0 is dropped
    specs.append(("neg_drop", s))
    c = rand_codes(45)
    s = stream_from_codes(c)
    s[2] = audio_tok(4097, 2)  # > 4096 -> window rejected by the range check (:108-111)
    specs.append(("oob_first", s))
    c = rand_codes(70)
    s = stream_from_codes(c)
    s[40] = audio_tok(5000, 40 % 7)
    specs.append(("oob_mid", s))
    # cumulative text (vLLM outputs[0].text is cumulative; :169-174 uses rfind)
    strs = stream_from_codes(rand_codes(35))
    cum, acc = [], ""
    for t in strs:
        acc += t
        cum.append(acc)
    specs.append(("cumulative", cum))
    # phase-shifted: a code whose phase is wrong gives a code outside [1,4095]
    s = stream_from_codes(rand_codes(30))
    s[11] = audio_tok(100, 2)  # wrong phase offset -> large negative/positive code
    specs.append(("wrong_phase", s))

    for name, strings in specs:
        rec = run_decoder(mod, strings)
        rec["name"] = name
        rec["tokens"] = strings
        golden["streams"].append(rec)

    # (5) PCM16 epilogue: convert_to_audio on fixed windows (speechpipe.py:64-137)
    for n_frames in (1, 2, 4, 7):
        codes = rand_codes(7 * n_frames + 3)  # trailing partial frame is ignored (:72-73)
        CALLS.clear()
        out = mod.convert_to_audio(codes, 7 * n_frames)
        golden["convert_to_audio"].append({
            "multiframe": codes, "windows": [list(x) for x in CALLS],
            "out_hex": out.hex() if out is not None else None,
        })
    for bad in ([4097] * 7, [-1] + [5] * 6, [1] * 6):
        CALLS.clear()
        out = mod.convert_to_audio(bad, 7)
        golden["convert_to_audio"].append({"multiframe": bad, "windows": [list(x) for x in CALLS],
                                           "out_hex": out.hex() if out is not None else None})

    with open(OUT, "w") as fh:
        json.dump(golden, fh, indent=0, sort_keys=True)
    print("wrote", OUT, os.path.getsize(OUT), "bytes;", len(golden["streams"]), "streams")


if __name__ == "__main__":
    main()
