"""speechpipe host logic vs golden vectors generated from the REFERENCE module.

Golden file: tests/golden/speechpipe_golden.json, made by
tests/golden/make_speechpipe_golden.py (reference speechpipe.py + recording fake SNAC).
Checks (1) the oracle restatement, (2) the product schedule (string and id level) and
(3) the product drop-in ``speechpipe.turn_token_into_id`` against the same vectors.
"""
import asyncio
import hashlib

import numpy as np
import pytest

from oracle import speechpipe_ref as ref
from project_morpheus_amd import schedule


def fake_decode(c0, c1, c2):
    """Restated verbatim from tests/golden/make_speechpipe_golden.py."""
    n = len(c0)
    j = np.arange(2048 * n, dtype=np.int64)
    f = j // 2048
    c0 = np.asarray(c0, dtype=np.int64)
    c1 = np.asarray(c1, dtype=np.int64)
    c2 = np.asarray(c2, dtype=np.int64)
    v = (c0[f] + 3 * c1[2 * f] + 5 * c2[4 * f + 3] + (j % 2048)) % 4001
    return (v.astype(np.float32) / np.float32(4000.0)) - np.float32(0.5)


def _sha(bs):
    return [hashlib.sha256(b).hexdigest() for b in bs]


def test_turn_token_into_id_oracle(golden):
    for case in golden["turn_token_into_id"]:
        assert ref.parse_custom_token(case["s"], case["i"]) == case["out"], case


def test_turn_token_into_id_product(golden):
    from project_morpheus_amd import speechpipe
    for case in golden["turn_token_into_id"]:
        assert schedule.parse_token_text(case["s"], case["i"]) == case["out"], case
        assert speechpipe.turn_token_into_id(case["s"], case["i"]) == case["out"], case


@pytest.mark.parametrize("idx", range(27))
def test_decode_stream_oracle(golden, idx):
    rec = golden["streams"][idx]
    wins = []
    outs = ref.decode_stream(rec["tokens"], fake_decode, windows_out=wins)
    decoded = [list(ref.deinterleave(w)) for w in wins if ref.codes_valid(*ref.deinterleave(w))]
    assert decoded == rec["windows"], rec["name"]
    assert [len(o) for o in outs] == rec["out_lens"], rec["name"]
    assert _sha(outs) == rec["out_sha256"], rec["name"]
    sync = ref.drop_empty(outs)
    assert _sha(sync) == rec["sync_sha256"], rec["name"]


def _product_windows(tokens, id_level=False):
    s = schedule.WindowScheduler()
    wins = []
    for t in tokens:
        if id_level:
            # id-level path: strings -> ids -> code_of_id (what the engine sees on device)
            code = None
            if t.startswith("<custom_token_") and t.endswith(">") and "><" not in t:
                try:
                    n = int(t[len("<custom_token_"):-1])
                    code = schedule.code_of_id(128256 + n, s.count) if n >= 0 else None
                except ValueError:
                    code = None
            else:
                code = schedule.parse_token_text(t, s.count)
        else:
            code = schedule.parse_token_text(t, s.count)
        wins.extend(s.push(code))
    wins.extend(s.flush())
    return wins


@pytest.mark.parametrize("idx", range(27))
def test_product_schedule(golden, idx):
    rec = golden["streams"][idx]
    wins = _product_windows(rec["tokens"])
    assert [list(schedule.deinterleave(w)) for w in wins] == rec["windows"], rec["name"]
    outs = [ref.pcm16_epilogue(fake_decode(*schedule.deinterleave(w))) for w in wins]
    assert _sha(outs) == rec["out_sha256"], rec["name"]


@pytest.mark.parametrize("idx", range(20))
def test_product_schedule_id_level(golden, idx):
    rec = golden["streams"][idx]  # the plain_* streams: pure custom-token ids
    wins = _product_windows(rec["tokens"], id_level=True)
    assert [list(schedule.deinterleave(w)) for w in wins] == rec["windows"], rec["name"]


def test_convert_to_audio_epilogue(golden):
    for case in golden["convert_to_audio"]:
        wins = []
        out = ref.convert_window(case["multiframe"], lambda *c: (wins.append([list(x) for x in c]),
                                                                   fake_decode(*c))[1])
        assert wins == case["windows"]
        assert (out.hex() if out is not None else None) == case["out_hex"]


def test_product_tokens_decoder_with_fake_model(golden, monkeypatch):
    """The product's async tokens_decoder / tokens_decoder_sync over a fake SNAC."""
    from project_morpheus_amd import speechpipe

    def fake_convert(multiframe, count):
        nf = len(multiframe) // 7
        win = multiframe[: 7 * nf]
        if not schedule.window_valid(win):
            return None
        return ref.pcm16_epilogue(fake_decode(*schedule.deinterleave(win)))

    monkeypatch.setattr(speechpipe, "convert_to_audio", fake_convert)

    async def agen(items):
        for it in items:
            yield it

    for rec in golden["streams"]:
        async def run():
            a = [b async for b in speechpipe.tokens_decoder(agen(rec["tokens"]))]
            b = [x async for x in speechpipe.tokens_decoder_sync(agen(rec["tokens"]))]
            return a, b
        a, b = asyncio.run(run())
        assert _sha(a) == rec["out_sha256"], rec["name"]
        assert _sha(b) == rec["sync_sha256"], rec["name"]
