"""Oracle: numpy restatement of the temperature + top-p sampler (TEST INFRASTRUCTURE).

The reference samples inside third-party engines: vLLM ``SamplingParams(temperature, top_p,
repetition_penalty)`` (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:106-112) and
llama.cpp with the same knobs (Morpheus_Client/tts_engine/inference.py:75-105,
llama_local.py:77).  Their random streams cannot be reproduced, so the build defines its own
seeded stream and this module states the SAME definition independently of the GPU's radix
select (csrc/sample_kernels.hip), by sorting:

  e_i = exp((l_i - max l) / T) (float32), f_i = floor(e_i * 2^40) (uint64),
  Z = sum f_i, thr = max(1, floor(float64(Z) * top_p)) (Z when top_p >= 1),
  keep i iff sum_{j: e_j > e_i} f_j < thr,
  u_i = ((philox4x32_10(key=seed, ctr=(i, pos, 0, 0)).x0 >> 9) + 0.5) * 2^-23  (exact in
        float32, so 0 < u_i < 1: a 24-bit draw rounded to 1.0 would lose the race),
  token = argmax over kept i of e_i / -log(u_i)   (smallest index on ties).

Greedy (temperature <= 0) is argmax of the penalised logits.  Parity unpinned against vLLM /
llama.cpp (different random streams by construction); pinned against the GPU sampler on
identical logits in tests/test_gpu_sampling.py, and against a brute-force frequency check in
tests/test_sampling_ref.py.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox_x0(c0: np.ndarray, c1: int, seed: int) -> np.ndarray:
    """Word 0 of Philox4x32-10 for counters (c0[i], c1, 0, 0), key (seed lo, seed hi)."""
    x0 = np.asarray(c0, dtype=np.uint64) & MASK
    x1 = np.full_like(x0, np.uint64(c1) & MASK)
    x2 = np.zeros_like(x0)
    x3 = np.zeros_like(x0)
    k0 = np.uint64(seed & 0xFFFFFFFF)
    k1 = np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * x0
        p1 = M1 * x2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        x0, x1, x2, x3 = (hi1 ^ x1 ^ k0) & MASK, lo1, (hi0 ^ x3 ^ k1) & MASK, lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return x0.astype(np.uint32)


def nucleus(logits: np.ndarray, temperature: float, top_p: float):
    """-> (e float32 [V], kept bool [V], f uint64 [V], thr)."""
    lg = np.asarray(logits, dtype=np.float32)
    m = lg.max()
    e = np.exp((lg - m) / np.float32(temperature)).astype(np.float32)
    f = np.floor(e.astype(np.float64) * 2.0 ** 40).astype(np.uint64)
    Z = int(f.sum(dtype=np.uint64))
    thr = Z if top_p >= 1.0 else max(1, int(np.float64(Z) * np.float64(np.float32(top_p))))
    order = np.argsort(-e, kind="stable")
    es, fs = e[order], f[order]
    # mass strictly above each distinct value: cumulative mass of the previous groups
    cum = np.cumsum(fs, dtype=np.uint64)
    first = np.ones(len(es), dtype=bool)
    first[1:] = es[1:] != es[:-1]
    grp_start = np.maximum.accumulate(np.where(first, np.arange(len(es)), 0))
    above = np.where(grp_start > 0, cum[np.maximum(grp_start - 1, 0)], np.uint64(0))
    keep_sorted = (above < np.uint64(thr)) & (fs > 0)
    kept = np.zeros(len(e), dtype=bool)
    kept[order] = keep_sorted
    return e, kept, f, thr


def sample(logits: np.ndarray, temperature: float, top_p: float, seed: int, pos: int,
           return_margin: bool = False):
    """One token from penalised ``logits`` at RNG counter ``pos`` (the row's input position)."""
    lg = np.asarray(logits, dtype=np.float32)
    if temperature <= 0:
        tok = int(np.argmax(lg))
        return (tok, np.inf) if return_margin else tok
    e, kept, _, _ = nucleus(lg, temperature, top_p)
    idx = np.nonzero(kept)[0]
    x = philox_x0(idx, pos, seed)
    u = ((x >> 9).astype(np.float32) + np.float32(0.5)) * np.float32(2.0 ** -23)
    s = e[idx] / -np.log(u)
    best = int(np.argmax(s))          # first index among equal maxima = smallest token id
    tok = int(idx[best])
    if not return_margin:
        return tok
    srt = np.sort(s)
    margin = float((srt[-1] - srt[-2]) / srt[-1]) if len(srt) > 1 else np.inf
    return tok, margin
