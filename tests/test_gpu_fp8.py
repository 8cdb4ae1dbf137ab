"""fp8 (OCP e4m3, per-row scales) decode vs the CPU oracle run on the dequantised weights.

BASELINE configs[4].  The oracle (oracle/llama_ref.py) runs exactly the model the GPU runs:
W = scale[row] * e4m3 (weights.dequantize_fp8).  Single-row steps use the fp8 GEMV
(v_cvt_pk_f32_fp8), the lm_head and multi-row steps the fp8 -> bf16 MFMA kernel.
Tolerances as tests/test_gpu_llm.py.
"""
import numpy as np
import pytest
import torch

from oracle import llama_ref as L
from project_morpheus_amd import config as C
from project_morpheus_amd.weights import (dequantize_fp8, quantize_fp8,
                                          synthetic_llm_weights)

from _coverage import check_declared
from _parity import (LONG_SHAPES, STRADDLE, b1_attention_shapes, check_tokens,
                     rows_teacher_forced)

pytestmark = pytest.mark.gpu

LOGIT_TOL = 5e-3
TIE_MARGIN = 1e-2


def _cfg():
    return C.OrpheusConfig(hidden=1024, layers=2, heads=8, kv_heads=2, ffn=2048, vocab=1000)


def _run(cfg, qw, prompts, steps, info=None, options=None, max_pos=512, max_prefill=128):
    from project_morpheus_amd.engine import LlmEngine
    B = len(prompts)
    check_declared(cfg, [len(p) for p in prompts], steps, True, options)
    eng = LlmEngine(cfg, qw, device=0, max_slots=B, max_pos=max_pos, max_batch=B,
                    max_prefill=max_prefill, wdtype="fp8")
    for k, v in (options or {}).items():
        eng.set_option(k, v)
    eng.enable_logits()
    st = torch.cuda.Stream()
    toks = [[] for _ in range(B)]
    logits = [[] for _ in range(B)]
    for r, p in enumerate(prompts):
        eng.prefill(r, r, p, 1.1, st)
    for k in range(steps):
        if k > 0:
            eng.decode(B, st)
        st.synchronize()
        for r, p in enumerate(prompts):
            logits[r].append(eng.read_logits(r, st))
            toks[r].append(int(eng.hist[r, len(p) + k]))
    eng.close()
    return toks, logits


def _check(cfg, qw, prompts, steps, info=None, options=None, max_pos=512, max_prefill=128):
    toks, logits = _run(cfg, qw, prompts, steps, info=info, options=options, max_pos=max_pos,
                        max_prefill=max_prefill)
    rc = L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                     kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab)
    ref = L.LlamaRef(rc, dequantize_fp8(qw), max_pos=max_pos)
    agree = 0
    for r, p in enumerate(prompts):
        _, rl = L.greedy_generate(ref, p, steps, 1.1, return_logits=True, forced=toks[r])
        for k in range(steps):
            o = rl[k].numpy()
            np.testing.assert_allclose(logits[r][k], o, atol=LOGIT_TOL, rtol=LOGIT_TOL,
                                       err_msg=f"row {r} step {k}")
            assert toks[r][k] == int(np.argmax(logits[r][k]))
        agree += check_tokens(toks[r], rl, TIE_MARGIN, what=f"row {r}")
    return agree


def test_fp8_single_stream():
    cfg = _cfg()
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=51, std=0.05, norm_jitter=0.5), cfg)
    rng = np.random.default_rng(12)
    prompt = [int(x) for x in rng.integers(0, cfg.vocab, 17)]
    assert _check(cfg, qw, [prompt], 30) >= 24


def test_fp8_batched_6_rows():
    cfg = _cfg()
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=52, std=0.05, norm_jitter=0.5), cfg)
    rng = np.random.default_rng(13)
    prompts = [[int(x) for x in rng.integers(0, cfg.vocab, 4 + 3 * i)] for i in range(6)]
    assert _check(cfg, qw, prompts, 10) >= 0.8 * 60


def test_fp8_single_stream_orpheus_width():
    """configs[4]'s one-row kernels at Orpheus widths (2 layers): the fp8 GEMV (16 e4m3 per
    16-byte load, v_cvt_pk_f32_fp8, per-row scales) and the fp8 lm_head; a 120-id prompt so
    the context crosses one attention split."""
    cfg = C.OrpheusConfig(layers=2)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=53), cfg)
    rng = np.random.default_rng(14)
    prompt = [int(x) for x in rng.integers(1000, 128000, 120)]
    assert _check(cfg, qw, [prompt], 16) >= 12


def test_fp8_single_stream_orpheus_width_no_gemv_balance():
    """Option gemv_balance = 0 with e4m3 weights: the one-row qkv GEMV on 4-wave blocks and the
    merging o-proj on 8-wave blocks at 5 attention splits (NSM 8)."""
    cfg = C.OrpheusConfig(layers=2, vocab=16384)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=92), cfg)
    rng = np.random.default_rng(93)
    prompt = [int(x) for x in rng.integers(0, cfg.vocab, 600)]
    assert _check(cfg, qw, [prompt], 16, options={"gemv_balance": 0}, max_pos=1024,
                  max_prefill=600) >= 12


def test_fp8_batched_orpheus_width_8_rows():
    """configs[4] per GPU: 8 fp8 streams at Orpheus widths through the default multi-row GEMM
    with e4m3 weight tiles (converted in registers to bf16 MFMA fragments, per-row scales in
    the epilogue), ragged prompts."""
    cfg = C.OrpheusConfig(layers=2)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=54), cfg)
    rng = np.random.default_rng(15)
    prompts = [[int(x) for x in rng.integers(1000, 128000, 5 + 4 * i)] for i in range(8)]
    assert _check(cfg, qw, prompts, 6) >= 0.8 * 8 * 6


def test_fp8_batched_orpheus_width_8_rows_split_k_seam():
    """Options rows_atomic = 0 and rows_qkv_parts = 0 with e4m3 weights: the qkv and residual
    projections' K ranges merged by the split-K seam (row scales applied by the last arriver)."""
    cfg = C.OrpheusConfig(layers=2)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=55), cfg)
    rng = np.random.default_rng(16)
    prompts = [[int(x) for x in rng.integers(1000, 128000, 5 + 4 * i)] for i in range(8)]
    assert _check(cfg, qw, prompts, 6, options={"rows_atomic": 0, "rows_qkv_parts": 0}) >= 0.8 * 8 * 6


def test_fp8_lm_head_grid_stride_orpheus_width():
    """Option head_b1 = 0 with e4m3 weights: the grid-stride one-row fp8 lm_head (8 rows per
    wave) instead of the default persistent head_b1.hip kernel, full vocabulary."""
    cfg = C.OrpheusConfig(layers=2)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=58), cfg)
    prompt = [int(x) for x in np.random.default_rng(19).integers(1000, 128000, 40)]
    assert _check(cfg, qw, [prompt], 12, options={"head_b1": 0}) >= 9


def test_fp8_batched_orpheus_width_8_rows_split_attention_merged_in_oproj():
    """configs[4] per GPU at a context where the 8-row attention splits (prompts of 300-335
    ids, 2 splits of 256): option rows_merge merges the splits in the e4m3 o-projection."""
    cfg = C.OrpheusConfig(layers=2, vocab=16384)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=59), cfg)
    rng = np.random.default_rng(20)
    prompts = [[int(x) for x in rng.integers(0, cfg.vocab, 300 + 5 * i)] for i in range(8)]
    assert _check(cfg, qw, prompts, 4, options={"rows_merge": 1}, max_pos=512,
                  max_prefill=384) >= 0.8 * 8 * 4


def test_fp8_single_stream_long_context():
    """The default fp8 one-row path over configs[1]'s context range (L 200 -> 1,260): the fp8
    merging o-proj at NSM 2 / 4 / 8 and the 256-position attention past 1,024."""
    cfg = _cfg()
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=55, std=0.05, norm_jitter=0.5), cfg)
    prompt = [int(x) for x in np.random.default_rng(16).integers(0, cfg.vocab, 200)]
    steps = 1060
    assert LONG_SHAPES <= b1_attention_shapes(201, 200 + steps)
    assert _check(cfg, qw, [prompt], steps, max_pos=1280, max_prefill=256) >= 0.6 * steps


def test_fp8_single_stream_orpheus_width_long_context():
    """configs[4]'s one-row instantiations at Orpheus widths (the KCH = 3 fp8 merging o-proj
    gemv1<3,2,1,false,8,true,NSM>) at L 600 -> 1,120, teacher-forced (2 layers, 16,384-entry
    vocabulary: see test_gpu_llm.test_long_context_orpheus_width_default_path)."""
    cfg = C.OrpheusConfig(layers=2, vocab=16384)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=56), cfg)
    prompt = [int(x) for x in np.random.default_rng(17).integers(0, cfg.vocab, 600)]
    steps = 520
    assert LONG_SHAPES <= b1_attention_shapes(601, 600 + steps)
    assert _check(cfg, qw, [prompt], steps, max_pos=1152, max_prefill=640) >= 0.7 * steps


def test_fp8_one_row_orpheus_width_split_classes():
    """The e4m3 one-row merging o-proj at NSM 2 and 4 (gemv1<3,2,1,false,6,true,2|4>): a
    185-id prompt, L 186..200 crosses 2 -> 3 attention splits of 96 positions."""
    cfg = C.OrpheusConfig(layers=2, vocab=16384)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=79), cfg)
    prompt = [int(x) for x in np.random.default_rng(80).integers(0, cfg.vocab, 185)]
    assert b1_attention_shapes(186, 200) == {(3, 1, 2), (3, 1, 3)}
    assert _check(cfg, qw, [prompt], 16, max_pos=512, max_prefill=256) >= 12


@pytest.mark.parametrize("case", ["nsm2", "nsm4"])
def test_fp8_rows_merge_straddling_splits_orpheus_width(case):
    """configs[4]'s e4m3 merging o-projection (gemm_rows_kernel<1,1,1,false,3,true,2,NSM>)
    where the 8 rows of one launch have different split counts (1..2 under NSM 2, 1..4 under
    NSM 4; the cases of test_gpu_llm.test_rows_merge_straddling_splits_orpheus_width, on the
    256-position splits of 8-wave blocks: option att_nw6 = 0)."""
    lens, steps = STRADDLE[case]
    cfg = C.OrpheusConfig(layers=2, vocab=16384)
    qw = quantize_fp8(synthetic_llm_weights(cfg, seed=81 if case == "nsm2" else 82), cfg)
    rng = np.random.default_rng(83)
    prefix = [int(x) for x in rng.integers(0, cfg.vocab, 190)]
    prompts = [prefix + [int(x) for x in rng.integers(0, cfg.vocab, n - 190)] for n in lens]
    assert rows_teacher_forced(cfg, qw, prompts, steps, shared_prefix=190, max_pos=1024,
                               max_prefill=768, wdtype="fp8", ref_w=dequantize_fp8(qw),
                               options={"att_nw6": 0}) >= 0.8 * 8 * steps
