"""End-to-end GPU utterance (prefill -> hipGraph decode loop -> schedule -> SNAC -> PCM)
against the CPU oracle pipeline (llama_ref greedy + speechpipe_ref schedule + snac_ref).

NoiseBlock weights are zeroed here so the stochastic noise drops out and PCM is
comparable chunk by chunk (noise parity itself is covered in test_gpu_snac.py).
"""
import numpy as np
import pytest
import torch

from oracle import llama_ref as L
from oracle import snac_ref
from oracle import speechpipe_ref as SP
from _parity import check_tokens
from project_morpheus_amd import config as C
from project_morpheus_amd.weights import synthetic_llm_weights, synthetic_snac_weights

pytestmark = pytest.mark.gpu


def _synthetic_audio_ids(n, seed=2):
    rng = np.random.default_rng(seed)
    codes = rng.integers(1, 4096, size=n)
    return [int(C.AUDIO_CODE_BASE + 4096 * (i % 7) + c) for i, c in enumerate(codes)]


@pytest.fixture(scope="module")
def setup():
    from project_morpheus_amd.engine import LlmEngine, SnacDecoder, Synthesizer
    cfg = C.OrpheusConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024, vocab=1000)
    w = synthetic_llm_weights(cfg, seed=21, std=0.05, norm_jitter=0.5)
    sw = synthetic_snac_weights(seed=4)
    for b in range(4):
        sw[f"b{b}.noise.w"].zero_()
    eng = LlmEngine(cfg, w, max_slots=2, max_pos=512, max_batch=1, max_prefill=64)
    dec = SnacDecoder(sw, max_frames=7)
    return cfg, w, sw, Synthesizer(eng, dec, depth=3)


def test_utterance_matches_oracle(setup):
    from project_morpheus_amd.engine import UtteranceStats
    cfg, w, sw, syn = setup
    prompt = [int(x) for x in np.random.default_rng(5).integers(0, cfg.vocab, 15)]
    n_tok = 120
    inject = _synthetic_audio_ids(n_tok)
    st = UtteranceStats()
    chunks = list(syn.run(prompt, n_tok, 1.1, stop_ids=(), inject_ids=inject, stats=st))
    # LLM tokens: tie-aware greedy identity with the oracle
    ref = L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                 kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab), w,
                     max_pos=512)
    # teacher-forced on the GPU's tokens: every step compared (tie-aware, tests/_parity.py)
    assert len(st.token_ids) == n_tok
    _, r_logits = L.greedy_generate(ref, prompt, n_tok, 1.1, return_logits=True,
                                    forced=st.token_ids)
    assert check_tokens(st.token_ids, r_logits, what="utterance") >= 0.8 * n_tok
    # audio: same schedule + same windows through the CPU SNAC oracle
    strings = [f"<custom_token_{t - C.CUSTOM_TOKEN_BASE}>" for t in inject]

    def dec(c0, c1, c2):
        return snac_ref.decode(sw, c0, c1, c2).reshape(-1).numpy()

    want = SP.drop_empty(SP.decode_stream(strings, dec))
    assert len(chunks) == len(want) == st.windows - 1   # first 1-frame window is empty
    for a, b in zip(chunks, want):
        x = np.frombuffer(a, dtype=np.int16).astype(np.int32)
        y = np.frombuffer(b, dtype=np.int16).astype(np.int32)
        assert x.shape == y.shape == (2048,)
        assert np.abs(x - y).max() <= 1
    assert st.samples == 2048 * len(want)
    assert st.first_audio_ms is not None


def test_stop_token_ends_utterance(setup):
    """A stop id ends generation at that step (vLLM stop_token_ids semantics)."""
    cfg, w, sw, syn = setup
    prompt = [3, 1, 4, 1, 5]
    from project_morpheus_amd.engine import UtteranceStats
    st = UtteranceStats()
    list(syn.run(prompt, 30, 1.1, stop_ids=(), stats=st))
    stop_tok = st.token_ids[9]
    st2 = UtteranceStats()
    list(syn.run(prompt, 30, 1.1, stop_ids=(stop_tok,), stats=st2))
    assert st2.token_ids == st.token_ids[: st.token_ids.index(stop_tok) + 1]
