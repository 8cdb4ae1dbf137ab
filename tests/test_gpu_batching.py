"""Continuous batching (BatchSynthesizer) on the GPU vs the CPU oracle pipeline.

6 streams with staggered arrivals and ragged lengths share 4 decode rows (rows are reused
after a stream ends).  Per stream: the LLM tokens follow the oracle's greedy decode
(tie-aware, as in test_gpu_engine.py) and the PCM equals the oracle's window schedule run
through the SNAC oracle (NoiseBlock weights zeroed so the stochastic noise drops out).
"""
import numpy as np
import pytest

from oracle import llama_ref as L
from oracle import snac_ref
from oracle import speechpipe_ref as SP
from _parity import check_tokens
from project_morpheus_amd import config as C
from project_morpheus_amd.weights import synthetic_llm_weights, synthetic_snac_weights

pytestmark = pytest.mark.gpu


def _audio_ids(n, seed):
    rng = np.random.default_rng(seed)
    codes = rng.integers(1, 4096, size=n)
    return [int(C.AUDIO_CODE_BASE + 4096 * (i % 7) + c) for i, c in enumerate(codes)]


def test_batch_synthesizer_matches_oracle():
    from project_morpheus_amd.batching import BatchSynthesizer, StreamRequest
    from project_morpheus_amd.engine import LlmEngine, SnacDecoder
    cfg = C.OrpheusConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024, vocab=1000)
    w = synthetic_llm_weights(cfg, seed=41, std=0.05, norm_jitter=0.5)
    sw = synthetic_snac_weights(seed=5)
    for b in range(4):
        sw[f"b{b}.noise.w"].zero_()
    llm = LlmEngine(cfg, w, max_slots=4, max_pos=512, max_batch=4, max_prefill=64)
    dec = SnacDecoder(sw, max_frames=7, max_batch=8)
    syn = BatchSynthesizer(llm, dec, depth=2)
    rng = np.random.default_rng(11)
    reqs = []
    for i, n_tok in enumerate((60, 75, 35, 90, 50, 64)):
        prompt = [int(x) for x in rng.integers(0, cfg.vocab, 6 + 3 * i)]
        reqs.append(StreamRequest(prompt_ids=prompt, max_tokens=n_tok, arrival=0.004 * i,
                                  inject_ids=_audio_ids(n_tok, 100 + i), stop_ids=()))
    chunks = {id(r): [] for r in reqs}
    syn.run(reqs, on_chunk=lambda r, b: chunks[id(r)].append(b))

    ref = L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                 kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab), w,
                     max_pos=512)

    def dec_ref(c0, c1, c2):
        return snac_ref.decode(sw, c0, c1, c2).reshape(-1).numpy()

    for r in reqs:
        assert len(r.tokens) == r.max_tokens
        _, r_logits = L.greedy_generate(ref, r.prompt_ids, r.max_tokens, 1.1,
                                        return_logits=True, forced=r.tokens)
        assert check_tokens(r.tokens, r_logits, what=f"stream {reqs.index(r)}") \
            >= 0.8 * r.max_tokens
        strings = [f"<custom_token_{t - C.CUSTOM_TOKEN_BASE}>" for t in r.inject_ids]
        want = SP.drop_empty(SP.decode_stream(strings, dec_ref))
        got = chunks[id(r)]
        assert len(got) == len(want)
        for a, b in zip(got, want):
            x = np.frombuffer(a, dtype=np.int16).astype(np.int32)
            y = np.frombuffer(b, dtype=np.int16).astype(np.int32)
            assert x.shape == y.shape
            assert np.abs(x - y).max() <= 1
        assert r.first_audio_ms is not None and r.t_done is not None


def test_compaction_moves_live_streams_and_keeps_them_exact():
    """Row compaction on the GPU (mx_llm_move_row): four streams admitted together with
    max_tokens 20 / 90 / 35 / 70, so rows 0 and 2 free up while rows 1 and 3 still decode
    with steps queued (depth 2); the stream in row 3 moves into row 0 mid-decode.  Every
    stream's tokens follow the oracle teacher-forced (tie-aware), every PCM window matches
    the SNAC oracle, the moves happened, and the later steps ran the 2-row class."""
    from project_morpheus_amd.batching import BatchSynthesizer, StreamRequest
    from project_morpheus_amd.engine import LlmEngine, SnacDecoder
    cfg = C.OrpheusConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024, vocab=1000)
    w = synthetic_llm_weights(cfg, seed=43, std=0.05, norm_jitter=0.5)
    sw = synthetic_snac_weights(seed=6)
    for b in range(4):
        sw[f"b{b}.noise.w"].zero_()
    llm = LlmEngine(cfg, w, max_slots=4, max_pos=512, max_batch=4, max_prefill=64)
    moves = []
    real_move = llm.move_row

    def counting_move(dst, src, stream):
        moves.append((dst, src))
        return real_move(dst, src, stream)
    llm.move_row = counting_move
    dec = SnacDecoder(sw, max_frames=7, max_batch=8)
    syn = BatchSynthesizer(llm, dec, depth=2)
    rng = np.random.default_rng(12)
    reqs = []
    for i, n_tok in enumerate((20, 90, 35, 70)):
        prompt = [int(x) for x in rng.integers(0, cfg.vocab, 5 + 4 * i)]
        reqs.append(StreamRequest(prompt_ids=prompt, max_tokens=n_tok, arrival=0.0,
                                  inject_ids=_audio_ids(n_tok, 200 + i), stop_ids=()))
    chunks = {id(r): [] for r in reqs}
    syn.run(reqs, on_chunk=lambda r, b: chunks[id(r)].append(b))
    assert (0, 3) in moves, moves
    assert syn.row_steps[2] > 0 and syn.row_steps[4] > 0, dict(syn.row_steps)

    ref = L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                 kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab), w,
                     max_pos=512)

    def dec_ref(c0, c1, c2):
        return snac_ref.decode(sw, c0, c1, c2).reshape(-1).numpy()

    for i, r in enumerate(reqs):
        assert len(r.tokens) == r.max_tokens
        _, r_logits = L.greedy_generate(ref, r.prompt_ids, r.max_tokens, 1.1,
                                        return_logits=True, forced=r.tokens)
        assert check_tokens(r.tokens, r_logits, what=f"stream {i}") >= 0.8 * r.max_tokens
        strings = [f"<custom_token_{t - C.CUSTOM_TOKEN_BASE}>" for t in r.inject_ids]
        want = SP.drop_empty(SP.decode_stream(strings, dec_ref))
        got = chunks[id(r)]
        assert len(got) == len(want), i
        for a, b in zip(got, want):
            x = np.frombuffer(a, dtype=np.int16).astype(np.int32)
            y = np.frombuffer(b, dtype=np.int16).astype(np.int32)
            assert np.abs(x - y).max() <= 1
