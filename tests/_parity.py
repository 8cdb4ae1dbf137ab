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
    for L_ in range(l_lo, l_hi + 1):
        for nw, cpw in ((4, 1), (4, 2), (4, 4), (8, 4), (8, 8)):
            S = 32 * nw * cpw
            if (L_ + S - 1) // S <= 8:
                out.add((nw, cpw, (L_ + S - 1) // S))
                break
    return out


# the default one-row shapes configs[1] reaches past L 512: 5..8 splits of 128 positions
# (the o-proj's NSM = 8 split merge), then 5 splits of 256 past L 1,024
LONG_SHAPES = {(4, 1, n) for n in range(5, 9)} | {(4, 2, 5)}
