"""Shared token checks of the GPU parity tests (teacher-forced, tie-aware).

The oracle is run teacher-forced on the GPU's own tokens (``llama_ref.greedy_generate(...,
forced=...)`` / ``teacher_forced_rows``), so every step of a stream is compared, not only
the steps before a first near-tie divergence.  At each step the GPU's token must be the
oracle's argmax, or -- where bf16 KV rounding makes two candidates a near-tie -- a token
whose oracle logit is within ``margin`` of the oracle's maximum.
"""
import numpy as np


def check_tokens(got, ref_logits, margin=1e-2, what=""):
    """Returns the number of steps whose token equals the oracle's argmax; asserts every
    other step is a near-tie that the GPU resolved to a near-top candidate."""
    assert len(ref_logits) >= len(got), (len(ref_logits), len(got))
    agree = 0
    for k, g in enumerate(got):
        rl = ref_logits[k]
        rl = rl.numpy() if hasattr(rl, "numpy") else np.asarray(rl)
        top = int(np.argmax(rl))
        if int(g) == top:
            agree += 1
            continue
        gap = float(rl[top] - rl[int(g)])
        assert gap < margin, f"{what} step {k}: token {g} is {gap:.3e} below the oracle's {top}"
    return agree


def b1_attention_shapes(l_lo, l_hi):
    """(waves, chunks per wave, splits) the default one-row path launches for contexts
    l_lo..l_hi -- a restatement of capi.hip att_b1_shape, so the long-context tests can
    assert which kernel variants they reached."""
    out = set()
    for L_ in range(l_lo, l_hi + 1):  # (options att_b1_short = 1, att_b1_nw6 = 1, the defaults)
        for nw, cpw in ((3, 1), (4, 1), (6, 1), (4, 2), (4, 4), (8, 4), (8, 8)):
            S = 32 * nw * cpw
            if (L_ + S - 1) // S <= 8:
                out.add((nw, cpw, (L_ + S - 1) // S))
                break
    return out


# the default one-row shapes configs[1] reaches past L 600: 7..8 splits of 96 positions to
# L 768, 7..8 of 128 to 1,024 (the o-proj's NSM = 8 split merge), then 6 splits of 192
LONG_SHAPES = {(3, 1, 7), (3, 1, 8), (4, 1, 7), (4, 1, 8), (6, 1, 6)}


# 8 rows whose own split counts differ inside one launch: the o-projection merging
# at most 2 splits (rows of 1 and 2 splits of 256 positions) and at most 4 (rows of 1..4
# splits; the launch crosses 768 -> 4 splits at step 9).  A shared 190-id prefix + tails.
STRADDLE = {"nsm2": ([200, 215, 230, 250, 262, 280, 400, 497], 12),
            "nsm4": ([200, 260, 330, 480, 520, 600, 700, 760], 12)}


def rows_teacher_forced(cfg, w, prompts, steps, shared_prefix=0, max_pos=1024, max_prefill=256,
                        options=None, wdtype="bf16", ref_w=None, logit_tol=5e-3,
                        tie_margin=1e-2):
    """Several streams on their own slots and decode rows, stepped together (the B >= 2
    path), every row teacher-forced against the oracle (``llama_ref.teacher_forced_rows``;
    ``shared_prefix`` ids common to every prompt are run once).  ``ref_w``: the oracle's
    weights when they differ from the engine's (fp8: the dequantised matrices).  Asserts the
    logits of every (row, step) and the tie-aware tokens; returns the argmax agreements."""
    import torch

    from oracle import llama_ref as L
    from project_morpheus_amd.engine import LlmEngine

    from _coverage import check_declared
    B = len(prompts)
    check_declared(cfg, [len(p) for p in prompts], steps, wdtype == "fp8", options)
    eng = LlmEngine(cfg, w, device=0, max_slots=B, max_pos=max_pos, max_batch=B,
                    max_prefill=max_prefill, wdtype=wdtype)
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
    rc = L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                     kv_heads=cfg.kv_heads, head_dim=cfg.head_dim, ffn=cfg.ffn,
                     vocab=cfg.vocab, eps=cfg.eps, rope_theta=cfg.rope_theta,
                     rope_scaling=cfg.rope_scaling)
    ref = L.LlamaRef(rc, ref_w if ref_w is not None else w, max_pos=max_pos)
    r_logits = L.teacher_forced_rows(ref, prompts, toks, 1.1, shared_prefix=shared_prefix)
    agree = 0
    for r in range(B):
        for k in range(steps):
            np.testing.assert_allclose(logits[r][k], r_logits[r][k].numpy(), atol=logit_tol,
                                       rtol=logit_tol, err_msg=f"row {r} step {k}")
            assert toks[r][k] == int(np.argmax(logits[r][k]))
        agree += check_tokens(toks[r], r_logits[r], tie_margin, what=f"row {r}")
    return agree
