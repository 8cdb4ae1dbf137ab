"""The drop-in boundary on the GPU: adapters over the per-GPU continuous-batching service.

* Two concurrent ``mi355x`` adapters (created through the reference registry contract,
  adapter_registry.py:90-98) each yield the PCM that the same request yields alone: streams
  join one batch, and every stream's random inputs (synthetic audio codes, SNAC noise) are
  its own, so batching changes nothing but kernel summation order (PCM within 1 LSB).
* Each stream's audio equals the oracle pipeline: the reference window schedule
  (oracle/speechpipe_ref.py) through the SNAC oracle with the device's noise restated
  (oracle/snac_ref.window_noise).
* ``reset()`` mid-stream (barge-in, llama_local.py:152-157) cancels the GPU stream and frees
  its decode row; a following request still decodes the oracle's greedy tokens.
"""
import asyncio
import time

import numpy as np
import pytest
import torch

from oracle import llama_ref as L
from oracle import snac_ref
from oracle import speechpipe_ref as SP
from project_morpheus_amd import config as C
from project_morpheus_amd import inference as I
from project_morpheus_amd.batching import window_seed
from project_morpheus_amd.weights import synthetic_llm_weights, synthetic_snac_weights

pytestmark = pytest.mark.gpu

CFG = C.OrpheusConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024)


class _Registry:
    """The reference registry's create() contract: constructor(prompt=, **voice_map, **kw)."""

    def __init__(self):
        self.entries = {}

    def register(self, name, ctor, describe, mapper):
        self.entries[name] = (ctor, describe, mapper)

    def create(self, name, *, prompt, voice, **kw):
        ctor, _, mapper = self.entries[name]
        return ctor(prompt=prompt, **mapper(voice), **kw)


class _Voice:
    def __init__(self, voice):
        self.voice = voice


@pytest.fixture(scope="module")
def svc():
    from project_morpheus_amd import service
    w = synthetic_llm_weights(CFG, seed=71, std=0.05, norm_jitter=0.5)
    sw = synthetic_snac_weights(seed=72)
    s = service.Service(device=0, cfg=CFG, llm_weights=w, snac_weights=sw, max_pos=512,
                        max_prefill=128, max_batch=4, synthetic_audio=True)
    s.test_weights = (w, sw)
    old = service._service
    service._service = s
    saved = (I.TEMPERATURE, I.MAX_TOKENS, C.CONTENT_SEED)
    I.update_generation_params(temperature=0.0, max_tokens=84)   # greedy: the parity mode
    C.CONTENT_SEED = 1  # solo and concurrent runs of one text draw the same random streams
    yield s
    I.update_generation_params(temperature=saved[0], max_tokens=saved[1])
    C.CONTENT_SEED = saved[2]
    service._service = old
    s.close()


def _drain(adapter, pull=4096):
    async def go():
        out = bytearray()
        while True:
            ch = await adapter.pull(pull)
            out += ch.pcm
            if ch.eos:
                return bytes(out)
    return asyncio.run(go())


def _adapters(texts):
    from project_morpheus_amd.adapter import register
    reg = _Registry()
    register(reg)
    return [reg.create("mi355x", prompt=t, voice=_Voice("leo")) for t in texts]


def _oracle_pcm(svc, text, voice="leo"):
    """Reference schedule + SNAC oracle + device noise for one request of the service."""
    _, sw = svc.test_weights
    ids = svc.prompt_ids(text, voice)
    h = svc.submit(text, voice)  # only to learn the request's seeds and inject stream
    req = h.req
    list(h.chunks())
    strings = [f"<custom_token_{t - C.CUSTOM_TOKEN_BASE}>" for t in req.inject_ids]
    j = [0]

    def dec(c0, c1, c2):
        noise = snac_ref.window_noise(window_seed(req.noise_seed, j[0]), len(c0))
        j[0] += 1
        return snac_ref.decode(sw, c0, c1, c2, noise=noise).reshape(-1).numpy()

    return b"".join(SP.drop_empty(SP.decode_stream(strings, dec))), req, ids


def _close(a, b, what):
    x = np.frombuffer(a, dtype=np.int16).astype(np.int32)
    y = np.frombuffer(b, dtype=np.int16).astype(np.int32)
    assert x.shape == y.shape, what
    assert np.abs(x - y).max() <= 1, what


def test_concurrent_adapters_match_solo_and_oracle(svc):
    texts = ["Hello world, this is stream one.", "A second, different stream of text!"]
    solo = [_drain(a) for a in _adapters(texts)]
    assert all(len(p) > 0 for p in solo)
    import threading
    got = [None, None]
    ads = _adapters(texts)

    def run(i):
        got[i] = _drain(ads[i], pull=8)  # the orchestrator's smallest ladder pull
    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    for i in range(2):
        _close(got[i], solo[i], f"stream {i} concurrent vs solo")
        want, _, _ = _oracle_pcm(svc, texts[i])
        _close(got[i], want, f"stream {i} vs oracle")


def test_reset_frees_row_and_next_request_is_exact(svc):
    (a,) = _adapters(["A stream that will be interrupted by a barge-in."])

    async def barge():
        ch = await a.pull(4096)
        assert ch.pcm
        await a.reset()
    asyncio.run(barge())
    deadline = time.time() + 30
    while (svc.batch._live or svc.batch.outstanding_tokens) and time.time() < deadline:
        time.sleep(0.01)
    assert not svc.batch._live and svc.batch.outstanding_tokens == 0
    # every decode row is parked on the scratch slot again
    llm = svc.llm
    assert all(not llm.row_state(r)[0] for r in range(llm.max_batch))
    # the next request still follows the oracle's greedy decode
    text = "After the barge-in, a new request."
    h = svc.submit(text, "tara")
    list(h.chunks())
    toks = h.req.tokens
    w, _ = svc.test_weights
    ref = L.LlamaRef(L.RefConfig(hidden=CFG.hidden, layers=CFG.layers, heads=CFG.heads,
                                 kv_heads=CFG.kv_heads, ffn=CFG.ffn, vocab=CFG.vocab), w,
                     max_pos=512)
    r_toks, r_logits = L.greedy_generate(ref, h.req.prompt_ids, len(toks), 1.1,
                                         return_logits=True)
    for k, (g, o) in enumerate(zip(toks, r_toks)):
        if g != o:
            top2 = np.sort(r_logits[k].numpy())[-2:]
            assert top2[1] - top2[0] < 1e-2, f"step {k}"
            break
    assert llm is svc.llm


def test_bad_request_fails_alone_and_the_loop_serves_on(svc):
    """a request the device rejects (MX_ERR_ARG at prefill) errors by itself;
    the batch loop keeps serving the next request."""
    from project_morpheus_amd.batching import StreamRequest, TokenHandle
    with pytest.raises(ValueError):
        svc.submit_tokens([1, 2, 3], top_p=0.0)
    # bypass submit()'s check: the loop itself must isolate the failure
    req = StreamRequest(prompt_ids=[5, 6, 7], max_tokens=4, top_p=-1.0, audio=False)
    h = TokenHandle(req)
    req.on_chunk, req.on_done, req.on_token = h._chunk, h._done, h._token
    with svc.batch._cv:
        svc.batch._inbox.append(req)
        svc.batch._cv.notify()
    with pytest.raises(ValueError):
        while h.get(timeout=60) is not None:
            pass
    g = svc.submit_tokens([5, 6, 7], max_tokens=6, temperature=0.0)
    toks = []
    while True:
        t = g.get(timeout=60)
        if t is None:
            break
        toks.append(t)
    assert len(toks) == 6
