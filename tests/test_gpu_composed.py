"""The composed hot path under GPU parity, with NO injected ids (BASELINE north_star's claim):
model-emitted token ids -> ``code_of_id`` -> reference window schedule -> (batched) SNAC ->
PCM16, against llama_ref greedy -> the same ids as ``<custom_token_N>`` strings ->
speechpipe_ref (speechpipe.py:146-293) -> snac_ref with the device's NoiseBlock noise.

The LLM weights speak (tests/_speaking.py): their greedy decode walks a designed script with
text ids, a code-0 id, a special id, an out-of-range code (invalid windows, first-window
retry) and end-of-speech.  Checked at B = 1 (``engine.Synthesizer``), at B = 4
(``batching.BatchSynthesizer``, four different scripts in one batch) and through the GPU-backed
drop-in ``speechpipe.tokens_decoder_sync`` / ``convert_to_audio`` on the same token text.
Token ids must be identical (the scripts' argmax margins are > 5, tests/test_speaking_oracle.py);
PCM within 1 LSB.
"""
import asyncio

import numpy as np
import pytest

from _speaking import STARTS, four_scripts, speaking_config, speaking_weights
from oracle import llama_ref as L
from oracle import snac_ref
from oracle import speechpipe_ref as SP
from project_morpheus_amd import config as C
from project_morpheus_amd import inference as I
from project_morpheus_amd.batching import window_seed
from project_morpheus_amd.weights import synthetic_snac_weights

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def world():
    cfg = speaking_config()
    scripts = four_scripts()
    w = speaking_weights(cfg, dict(zip(STARTS, scripts)))
    sw = synthetic_snac_weights(seed=8)  # NoiseBlocks ON: compared with the device noise
    ref = L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                 kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab,
                                 tied=False), w, max_pos=512)
    return cfg, w, sw, scripts, ref


def _strings(toks):
    return [f"<custom_token_{t - C.CUSTOM_TOKEN_BASE}>" if t >= C.CUSTOM_TOKEN_BASE
            else f" text{t}" for t in toks]


def _oracle(ref, sw, prompt, n_max, noise_seed_of_window):
    toks = L.greedy_generate(ref, prompt, n_max, 1.1, stop_ids=C.STOP_IDS)
    j = [0]
    wins = []

    def dec(c0, c1, c2):
        noise = snac_ref.window_noise(noise_seed_of_window(j[0]), len(c0))
        j[0] += 1
        return snac_ref.decode(sw, c0, c1, c2, noise=noise).reshape(-1).numpy()

    pcm = SP.drop_empty(SP.decode_stream(_strings(toks), dec, windows_out=wins))
    return toks, pcm, wins


def _same_pcm(got, want, what):
    assert len(got) == len(want), f"{what}: {len(got)} vs {len(want)} chunks"
    for i, (a, b) in enumerate(zip(got, want)):
        x = np.frombuffer(a, dtype=np.int16).astype(np.int32)
        y = np.frombuffer(b, dtype=np.int16).astype(np.int32)
        assert x.shape == y.shape, f"{what} chunk {i}"
        assert np.abs(x - y).max() <= 1, f"{what} chunk {i}"


def test_single_stream_model_tokens_to_pcm(world):
    from project_morpheus_amd.engine import (LlmEngine, SnacDecoder, Synthesizer,
                                             UtteranceStats)
    cfg, w, sw, scripts, ref = world
    llm = LlmEngine(cfg, w, max_slots=1, max_pos=512, max_batch=1, max_prefill=64)
    syn = Synthesizer(llm, SnacDecoder(sw, max_frames=7), depth=3)
    prompt = I.prompt_ids([1001, 1002, 1003])
    n_max = len(scripts[0]) + 8
    st = UtteranceStats()
    got = list(syn.run(prompt, n_max, 1.1, stats=st, noise_seed=4242))
    toks, want, wins = _oracle(ref, sw, prompt, n_max, lambda j: window_seed(4242, j))
    assert toks == scripts[0]                      # the oracle speaks the script ...
    assert st.token_ids == toks                    # ... and so does the GPU, id for id
    valid = [x for x in wins if SP.codes_valid(*SP.deinterleave(x))]
    assert st.windows == len(valid) and len(valid) < len(wins)  # invalid windows skipped
    _same_pcm(got, want, "B=1")
    llm.close()


def test_batch_of_four_scripts(world):
    from project_morpheus_amd.batching import BatchSynthesizer, StreamRequest
    from project_morpheus_amd.engine import LlmEngine, SnacDecoder
    cfg, w, sw, scripts, ref = world
    llm = LlmEngine(cfg, w, max_slots=4, max_pos=512, max_batch=4, max_prefill=64)
    syn = BatchSynthesizer(llm, SnacDecoder(sw, max_frames=7, max_batch=8), depth=2)
    reqs = []
    for b in range(4):
        prompt = [1001 + b, 1002, 1003 + 5 * b, STARTS[b]][: 2 + b % 3] + [STARTS[b]]
        reqs.append(StreamRequest(prompt_ids=prompt, max_tokens=len(scripts[b]) + 8,
                                  arrival=0.003 * b, noise_seed=777 + b))
    chunks = {id(r): [] for r in reqs}
    syn.run(reqs, on_chunk=lambda r, c: chunks[id(r)].append(c))
    for b, r in enumerate(reqs):
        toks, want, _ = _oracle(ref, sw, list(r.prompt_ids), r.max_tokens,
                                lambda j, s=r.noise_seed: window_seed(s, j))
        assert toks == scripts[b], f"oracle stream {b}"
        assert r.tokens == toks, f"GPU stream {b}"
        _same_pcm(chunks[id(r)], want, f"B=4 stream {b}")
    llm.close()


def test_speechpipe_drop_in_on_model_tokens(world):
    """The GPU-backed drop-in module (speechpipe.py:64,146,191,295 names) on the token TEXT
    the model emitted: window k of the module draws its noise from seed k (module counter)."""
    from project_morpheus_amd import speechpipe
    from project_morpheus_amd.engine import SnacDecoder
    cfg, w, sw, scripts, ref = world
    prompt = I.prompt_ids([1001, 1002, 1003])
    saved = (speechpipe._model, speechpipe._seed[0])
    speechpipe._model = SnacDecoder(sw, max_frames=7)
    speechpipe._seed[0] = 0
    try:
        toks, want, wins = _oracle(ref, sw, prompt, len(scripts[0]) + 8, lambda j: j + 1)
        texts = _strings(toks)

        async def gen():
            for t in texts:
                yield t

        async def collect():
            return [c async for c in speechpipe.tokens_decoder_sync(gen())]

        got = asyncio.run(collect())
        _same_pcm(got, want, "tokens_decoder_sync")
        # convert_to_audio on one valid 28-token window and on the invalid ones
        good = [x for x in wins if len(x) == 28 and SP.codes_valid(*SP.deinterleave(x))][0]
        bad = [x for x in wins if not SP.codes_valid(*SP.deinterleave(x))][0]
        assert speechpipe.convert_to_audio(bad, 0) is None
        k = speechpipe._seed[0] + 1
        a = speechpipe.convert_to_audio(good, 28)
        c0, c1, c2 = SP.deinterleave(good)
        b = SP.pcm16_epilogue(snac_ref.decode(sw, c0, c1, c2, noise=snac_ref.window_noise(
            k, len(c0))).reshape(-1).numpy())
        _same_pcm([a], [b], "convert_to_audio")
        assert speechpipe.turn_token_into_id(texts[1], 0) == SP.parse_custom_token(texts[1], 0)
    finally:
        speechpipe._model, speechpipe._seed[0] = saved
