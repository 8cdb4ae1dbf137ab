"""GPU parity of the persistent one-row decode engine (option b1_engine, csrc/engine_b1.hip)
against the fp32 CPU oracle, teacher-forced and tie-aware (tests/_parity.py), at the
tolerances of tests/test_gpu_llm.py (logits 5e-3; 1.5e-2 at 28 layers).

The engine runs every layer of a one-row step in one launch: LDS-DMA weight ring, granule
hand-offs between CUs, attention split over (kv head, 128 positions) items with the new
position taken from the hand-off granules and the splits merged by the last arriving item.
The cases cover one split (no ticket), the ticket merge with the new position in the last
split, bf16 and e4m3 weights, GQA 4 (small widths) and 3 (Orpheus widths), and the full
28-layer Orpheus-3B shape configs[1] runs.
"""
import numpy as np
import pytest
import torch

from oracle import llama_ref as L
from project_morpheus_amd import config as C
from project_morpheus_amd.weights import dequantize_fp8, quantize_fp8, synthetic_llm_weights

from _parity import rows_teacher_forced

pytestmark = pytest.mark.gpu

ENGINE = {"b1_engine": 1}


def _small():
    # the smallest shape the engine takes: hidden = heads x 128, multiples of 1024
    return C.OrpheusConfig(hidden=1024, layers=2, heads=8, kv_heads=2, ffn=2048, vocab=1000)


@pytest.mark.parametrize("prompt_len,steps", [(13, 40), (250, 30)])
def test_engine_small_bf16(prompt_len, steps):
    """L 14..53: one attention split per kv head (no ticket); L 251..280: 2 -> 3 splits,
    the ticket merge, the new position alone in its split at L 257."""
    cfg = _small()
    w = synthetic_llm_weights(cfg, seed=101, std=0.05, norm_jitter=0.5)
    prompt = [int(x) for x in np.random.default_rng(prompt_len).integers(0, cfg.vocab, prompt_len)]
    assert rows_teacher_forced(cfg, w, [prompt], steps, max_pos=512, max_prefill=256,
                               options=ENGINE) >= 0.75 * steps


def test_engine_small_fp8():
    cfg = _small()
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=102, std=0.05, norm_jitter=0.5), cfg)
    prompt = [int(x) for x in np.random.default_rng(7).integers(0, cfg.vocab, 140)]
    assert rows_teacher_forced(cfg, qw, [prompt], 30, max_pos=512, max_prefill=256,
                               options=ENGINE, wdtype="fp8",
                               ref_w=dequantize_fp8(qw)) >= 0.75 * 30


@pytest.mark.parametrize("wdtype", ["bf16", "fp8"])
def test_engine_orpheus_width(wdtype):
    """Orpheus widths (2 layers, 16,384-entry vocabulary): 600-id prompt, L 601..640 over 5
    attention splits merged by the ticket."""
    cfg = C.OrpheusConfig(layers=2, vocab=16384)
    w = synthetic_llm_weights(cfg, seed=103)
    ref_w = None
    if wdtype == "fp8":
        w = quantize_fp8(w, cfg)
        ref_w = dequantize_fp8(w)
    prompt = [int(x) for x in np.random.default_rng(8).integers(0, cfg.vocab, 600)]
    steps = 40
    assert rows_teacher_forced(cfg, w, [prompt], steps, max_pos=1024, max_prefill=640,
                               options=ENGINE, wdtype=wdtype, ref_w=ref_w) >= 0.75 * steps


def test_engine_full_depth_orpheus_3b():
    """configs[1]'s exact model through the engine: 28 layers, the 156,940-entry tied lm_head
    (tolerance as test_gpu_llm.test_full_depth_orpheus_3b_single_stream)."""
    from project_morpheus_amd.engine import LlmEngine

    from _coverage import check_declared
    cfg = C.OrpheusConfig()
    w = synthetic_llm_weights(cfg, seed=0, device="cuda")
    prompt = [128259, 128000] + [int(x) for x in np.random.default_rng(31).integers(1000, 128000, 24)] \
        + [128009, 128260, 128261, 128257]
    steps = 10
    check_declared(cfg, [len(prompt)], steps, False, ENGINE)
    eng = LlmEngine(cfg, w, device=0, max_slots=1, max_pos=256, max_batch=1, max_prefill=64)
    eng.set_option("b1_engine", 1)
    eng.enable_logits()
    st = torch.cuda.Stream()
    toks, logits = [], []
    eng.prefill(0, 0, prompt, 1.1, st)
    for k in range(steps):
        if k:
            eng.decode(1, st)
        logits.append(eng.read_logits(0, st))
        toks.append(int(eng.hist[0, len(prompt) + k]))
    eng.close()
    wc = {k: v.cpu() for k, v in w.items()}
    del w
    torch.cuda.empty_cache()
    rc = L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                     kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab)
    ref = L.LlamaRef(rc, wc, max_pos=256)
    del wc
    _, r_logits = L.greedy_generate(ref, prompt, steps, 1.1, return_logits=True, forced=toks)
    agree = 0
    for k in range(steps):
        rl = r_logits[k].numpy()
        d = np.abs(logits[k] - rl)
        np.testing.assert_allclose(logits[k], rl, atol=1.5e-2, rtol=1.5e-2, err_msg=f"step {k}")
        assert float(d.mean()) <= 3e-3, f"step {k}: mean |d| {d.mean():.2e}"
        if toks[k] == int(np.argmax(rl)):
            agree += 1
        else:
            top2 = np.sort(rl)[-2:]
            assert top2[1] - top2[0] < 3e-2, f"step {k}"
    assert agree >= 8


def test_engine_status_word_stays_clear_over_many_steps():
    """200 graph-replayed engine steps (L 20..220, splits 1 -> 2): no launch gives up (the
    host checks the status word at every decode call and raises if one did)."""
    from project_morpheus_amd.engine import LlmEngine
    cfg = _small()
    w = synthetic_llm_weights(cfg, seed=104, std=0.05, norm_jitter=0.5)
    eng = LlmEngine(cfg, w, device=0, max_slots=1, max_pos=512, max_batch=1, max_prefill=64)
    eng.set_option("b1_engine", 1)
    st = torch.cuda.Stream()
    eng.prefill(0, 0, list(range(20)), 1.1, st)
    for _ in range(200):
        eng.decode(1, st)
    st.synchronize()
    eng.decode(1, st)   # raises if any earlier launch timed out
    st.synchronize()
    eng.close()


def test_engine_give_up_commits_nothing_and_recovers():
    """A forced give-up (option engine_timeout = 1 tick) mid-stream: the failed steps commit
    nothing (history -1, the row does not advance, h is the step's input again), the host check
    raises and clears the attention tickets, and with the default bound restored the stream
    continues exactly as the oracle's (L 251..280: 2 -> 3 splits, the ticket merge)."""
    from oracle import llama_ref as L
    from project_morpheus_amd._lib import MxError
    from project_morpheus_amd.engine import LlmEngine

    from _parity import check_tokens
    cfg = _small()
    w = synthetic_llm_weights(cfg, seed=105, std=0.05, norm_jitter=0.5)
    prompt = [int(x) for x in np.random.default_rng(9).integers(0, cfg.vocab, 250)]
    eng = LlmEngine(cfg, w, device=0, max_slots=1, max_pos=512, max_batch=1, max_prefill=256)
    eng.set_option("b1_engine", 1)
    eng.enable_logits()
    st = torch.cuda.Stream()
    toks, logits = [], []

    def record(k):
        st.synchronize()
        eng.check(st)
        logits.append(eng.read_logits(0, st))
        toks.append(int(eng.hist[0, len(prompt) + k]))

    eng.prefill(0, 0, prompt, 1.1, st)
    record(0)
    for k in range(1, 10):
        eng.decode(1, st)
        record(k)
    eng.set_option("engine_timeout", 1)
    eng.decode(1, st)
    st.synchronize()
    with pytest.raises(MxError, match="gave up"):
        eng.check(st)
    assert int(eng.hist[0, len(prompt) + 10]) == -1
    eng.check(st)  # cleared
    eng.set_option("engine_timeout", 0)
    for k in range(10, 30):
        eng.decode(1, st)
        record(k)
    eng.close()
    rc = L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                     kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab)
    ref = L.LlamaRef(rc, w, max_pos=512)
    _, r_logits = L.greedy_generate(ref, prompt, len(toks), 1.1, return_logits=True, forced=toks)
    for k in range(len(toks)):
        np.testing.assert_allclose(logits[k], r_logits[k].numpy(), atol=5e-3, rtol=5e-3,
                                   err_msg=f"step {k}")
    assert check_tokens(toks, r_logits, 1e-2) >= 0.75 * len(toks)
