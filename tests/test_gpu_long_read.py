"""configs[3] on one GPU: the long_read path end to end on the HIP engine.

Documents -> the reference's <=1000-char long-form batches (sharding.plan_jobs, pinned by
tests/golden/host_golden.json) -> jobs served by BatchSynthesizer through
sharding.run_sharded(world=1) -> per-document assembly with the 50 ms crossfade
(stitch_wav_files).  Checked against the oracle pipeline: each job's tokens follow the LLM
oracle's greedy decode (tie-aware), each job's audio is the reference window schedule
through the SNAC oracle with the device noise restated, and the assembled documents equal
the oracle jobs assembled the same way (PCM within 1 LSB, crossfade rounding within 2).
"""
import numpy as np
import pytest

from oracle import llama_ref as L
from oracle import snac_ref
from oracle import speechpipe_ref as SP
from _parity import check_tokens
from project_morpheus_amd import config as C
from project_morpheus_amd import sharding as S
from project_morpheus_amd.weights import synthetic_llm_weights, synthetic_snac_weights

pytestmark = pytest.mark.gpu


def test_long_read_one_gpu_matches_oracle():
    from project_morpheus_amd.batching import BatchSynthesizer, StreamRequest, window_seed
    from project_morpheus_amd.engine import LlmEngine, SnacDecoder
    from project_morpheus_amd.tokenizer import Tokenizer
    cfg = C.OrpheusConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024)
    w = synthetic_llm_weights(cfg, seed=81, std=0.05, norm_jitter=0.5)
    sw = synthetic_snac_weights(seed=82)
    docs = S.long_read_documents(2, 1500, seed=5)
    max_tokens = 63
    jobs = S.plan_jobs(docs, Tokenizer(None).encode, "tara", max_tokens)
    assert len(jobs) >= 4
    llm = LlmEngine(cfg, w, max_slots=4, max_pos=1024, max_batch=4, max_prefill=512)
    dec = SnacDecoder(sw, max_frames=7, max_batch=8)
    syn = BatchSynthesizer(llm, dec, depth=2)
    reqs = {}

    def synthesize(mine):
        rs = [StreamRequest(prompt_ids=j.prompt_ids, max_tokens=j.max_tokens, stop_ids=(),
                            inject_ids=C.synthetic_audio_ids(j.max_tokens, 100 + i),
                            noise_seed=500 + i) for i, j in enumerate(mine)]
        syn.run(rs, on_chunk=lambda r, b: r.pcm.append(b))
        for i, r in enumerate(rs):
            reqs[i] = r
        return [b"".join(r.pcm) for r in rs]

    out = S.run_sharded(jobs, 0, 1, synthesize, crossfade_ms=50.0)
    assert sorted(out) == list(range(len(docs)))

    ref = L.LlamaRef(L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                                 kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab), w,
                     max_pos=1024)
    want_pcm = {}
    for i, j in enumerate(jobs):
        r = reqs[i]
        assert len(r.tokens) == max_tokens
        _, r_logits = L.greedy_generate(ref, j.prompt_ids, max_tokens, 1.1,
                                        return_logits=True, forced=r.tokens)
        assert check_tokens(r.tokens, r_logits, what=f"job {i}") >= 0.8 * max_tokens
        strings = [f"<custom_token_{t - C.CUSTOM_TOKEN_BASE}>" for t in r.inject_ids]
        wi = [0]

        def dec_ref(c0, c1, c2, i=i, wi=wi):
            nz = snac_ref.window_noise(window_seed(500 + i, wi[0]), len(c0))
            wi[0] += 1
            return snac_ref.decode(sw, c0, c1, c2, noise=nz).reshape(-1).numpy()

        want = b"".join(SP.drop_empty(SP.decode_stream(strings, dec_ref)))
        got = b"".join(r.pcm)
        x = np.frombuffer(got, dtype=np.int16).astype(np.int32)
        y = np.frombuffer(want, dtype=np.int16).astype(np.int32)
        assert x.shape == y.shape and np.abs(x - y).max() <= 1, f"job {i}"
        want_pcm[i] = want
    want_docs = S.assemble(jobs, want_pcm, crossfade_ms=50.0)
    for d in out:
        x, y = out[d].astype(np.int32), want_docs[d].astype(np.int32)
        assert x.shape == y.shape and np.abs(x - y).max() <= 2, f"doc {d}"
