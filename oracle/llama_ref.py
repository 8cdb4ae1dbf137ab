"""Oracle: torch-fp32 CPU restatement of the Orpheus (Llama-3.2-3B) decoder (TEST INFRASTRUCTURE).

The reference runs this model inside third-party engines that are not vendored: vLLM
``AsyncLLMEngine.generate`` (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:117,
bf16) or llama.cpp (Morpheus_Client/tts_engine/llama_local.py:48-52,77).  This module
restates the Llama-3 decoder under the build's PRECISION CONTRACT:

  * weights stored bf16, every product computed in fp32 (bf16 -> fp32 is exact);
  * residual stream, norms, q/k/v, softmax, SwiGLU and logits in fp32;
  * K and V are rounded to bf16 (RNE) when written to the cache, as vLLM's bf16 cache does;
  * RMSNorm eps 1e-5, RoPE rotate-half with llama3 frequency scaling, GQA;
  * repetition penalty on the seen set (prompt + generated): l>0 -> l/p, else l*p
    (HF/vLLM form, engine_class.py:106-112, inference.py:105), then greedy argmax
    (first index among equal maxima, as torch.argmax).

Pinned against ``transformers.LlamaForCausalLM`` (installed 5.x) on small seeded configs
in tests/test_oracle_llama.py (bf16 KV rounding disabled for that comparison).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch


@dataclass
class RefConfig:
    hidden: int = 3072
    layers: int = 28
    heads: int = 24
    kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 8192
    vocab: int = 156940
    eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = field(default_factory=lambda: {
        "rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
        "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    tied: bool = True


def inv_freq(cfg: RefConfig) -> torch.Tensor:
    """Llama-3 RoPE frequencies in float64 (HF ``_compute_llama3_parameters`` formula)."""
    d = cfg.head_dim
    base = 1.0 / (cfg.rope_theta ** (torch.arange(0, d, 2, dtype=torch.float64) / d))
    rs = cfg.rope_scaling
    if not rs or rs.get("rope_type", rs.get("type")) != "llama3":
        return base
    factor, lo, hi = rs["factor"], rs["low_freq_factor"], rs["high_freq_factor"]
    old = rs["original_max_position_embeddings"]
    lo_wl, hi_wl = old / lo, old / hi
    wl = 2 * math.pi / base
    out = torch.where(wl > lo_wl, base / factor, base)
    smooth = (old / wl - lo) / (hi - lo)
    smoothed = (1 - smooth) * out / factor + smooth * out
    medium = (wl >= hi_wl) & (wl <= lo_wl)
    return torch.where(medium, smoothed, out)


def rope_cos_sin(cfg: RefConfig, positions: torch.Tensor):
    ang = positions.to(torch.float64)[:, None] * inv_freq(cfg)[None, :]
    return torch.cos(ang).float(), torch.sin(ang).float()         # [n, d/2] each


def _rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    # x [n, h, d]; rotate-half: (x1, x2) -> (x1 c - x2 s, x2 c + x1 s)
    h = x.shape[-1] // 2
    x1, x2 = x[..., :h], x[..., h:]
    c, s = cos[:, None, :], sin[:, None, :]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def _rms(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


class LlamaRef:
    """Batched (rows = (slot, position, token)) fp32 decoder with a per-slot bf16 KV cache."""

    def __init__(self, cfg: RefConfig, w: Dict[str, torch.Tensor], max_pos: int = 2048,
                 round_kv: bool = True):
        self.cfg = cfg
        self.max_pos = max_pos
        self.round_kv = round_kv
        self.w = {k: v.float() for k, v in w.items()}
        if "lm_head" not in self.w:
            self.w["lm_head"] = self.w["embed"]
        self.cache: Dict[int, torch.Tensor] = {}

    def _slot(self, s: int) -> torch.Tensor:
        if s not in self.cache:
            c = self.cfg
            self.cache[s] = torch.zeros(c.layers, 2, c.kv_heads, self.max_pos, c.head_dim)
        return self.cache[s]

    def free(self, s: int) -> None:
        self.cache.pop(s, None)

    @torch.no_grad()
    def forward(self, tokens: Sequence[int], slots: Sequence[int],
                positions: Sequence[int], last_only: bool = False) -> torch.Tensor:
        """Rows (token, slot, position) through every layer; logits [n, V] (``last_only``:
        the last row's only, [1, V] -- a prefill needs no more, and at Orpheus width the
        full [n, 156,940] product dominates a long prompt)."""
        c, w = self.cfg, self.w
        n = len(tokens)
        pos = torch.as_tensor(positions, dtype=torch.int64)
        cos, sin = rope_cos_sin(c, pos)
        h = w["embed"][torch.as_tensor(tokens, dtype=torch.int64)].clone()      # [n,H]
        scale = 1.0 / math.sqrt(c.head_dim)
        group = c.heads // c.kv_heads
        # rows grouped by slot: each group attends causally over its slot's cache in one
        # masked product (row i sees positions [0, positions[i]])
        groups: Dict[int, List[int]] = {}
        for i, s in enumerate(slots):
            groups.setdefault(int(s), []).append(i)
        for l in range(c.layers):
            p = f"l{l}."
            xn = _rms(h, w[p + "attn_norm"], c.eps)
            q = (xn @ w[p + "wq"].T).view(n, c.heads, c.head_dim)
            k = (xn @ w[p + "wk"].T).view(n, c.kv_heads, c.head_dim)
            v = (xn @ w[p + "wv"].T).view(n, c.kv_heads, c.head_dim)
            q, k = _rope(q, cos, sin), _rope(k, cos, sin)
            if self.round_kv:
                k, v = k.bfloat16().float(), v.bfloat16().float()
            for i in range(n):                      # write every row's K/V first ...
                kv = self._slot(slots[i])
                kv[l, 0, :, positions[i]] = k[i]
                kv[l, 1, :, positions[i]] = v[i]
            att = torch.empty(n, c.heads, c.head_dim)
            for s, rows in groups.items():          # ... then attend causally over [0, pos]
                kv = self._slot(s)
                ri = torch.as_tensor(rows, dtype=torch.int64)
                rp = pos[ri]
                L = int(rp.max()) + 1
                K = kv[l, 0, :, :L].repeat_interleave(group, dim=0)        # [heads, L, d]
                V = kv[l, 1, :, :L].repeat_interleave(group, dim=0)
                sc = torch.einsum("rhd,hld->rhl", q[ri], K) * scale
                mask = torch.arange(L)[None, :] > rp[:, None]              # [r, L]
                sc = sc.masked_fill(mask[:, None, :], float("-inf"))
                att[ri] = torch.einsum("rhl,hld->rhd", torch.softmax(sc, dim=-1), V)
            h = h + att.view(n, -1) @ w[p + "wo"].T
            xn = _rms(h, w[p + "mlp_norm"], c.eps)
            g = xn @ w[p + "wg"].T
            u = xn @ w[p + "wu"].T
            h = h + (torch.nn.functional.silu(g) * u) @ w[p + "wd"].T
        if last_only:
            h = h[-1:]
        return _rms(h, w["norm"], c.eps) @ w["lm_head"].T                      # [n,V]


def apply_penalty(logits: torch.Tensor, seen: Sequence[int], penalty: float) -> torch.Tensor:
    out = logits.clone()
    if penalty != 1.0 and len(seen):
        idx = torch.as_tensor(sorted(set(int(t) for t in seen)), dtype=torch.int64)
        v = out[idx]
        out[idx] = torch.where(v > 0, v / penalty, v * penalty)
    return out


def greedy_generate(model: LlamaRef, prompt: Sequence[int], n_steps: int,
                    penalty: float = 1.1, slot: int = 0, stop_ids=(),
                    return_logits: bool = False, forced: Optional[Sequence[int]] = None):
    """Prefill ``prompt`` then ``n_steps`` greedy steps; returns generated ids.

    ``forced`` (teacher forcing, parity harness only): feed ``forced[k]`` as the k-th
    generated token instead of the oracle's own argmax, so the logits of every later step
    can still be compared after a near-tie flipped one argmax."""
    model.free(slot)
    seen = list(prompt)
    logits = model.forward(list(prompt), [slot] * len(prompt), list(range(len(prompt))),
                           last_only=True)[-1]
    out: List[int] = []
    trace = []
    pos = len(prompt)
    for _ in range(n_steps):
        pl = apply_penalty(logits, seen, penalty)
        nxt = int(torch.argmax(pl))
        if forced is not None and len(out) < len(forced):
            nxt = int(forced[len(out)])
        if return_logits:
            trace.append(pl)
        out.append(nxt)
        seen.append(nxt)
        if nxt in stop_ids:
            break
        logits = model.forward([nxt], [slot], [pos])[0]
        pos += 1
    return (out, trace) if return_logits else out


def teacher_forced_rows(model: LlamaRef, prompts: Sequence[Sequence[int]],
                        forced: Sequence[Sequence[int]], penalty: float = 1.1,
                        shared_prefix: int = 0) -> List[List[torch.Tensor]]:
    """Penalised logits of every step of several streams, each on its own slot and
    teacher-forced with ``forced[r]`` (the GPU's tokens): the same numbers as
    ``greedy_generate(..., forced=forced[r], return_logits=True)`` per row, but one
    ``forward`` per step for all rows (one pass over the lm_head instead of one per row).

    ``shared_prefix`` > 0: every prompt starts with the same ``shared_prefix`` ids; their
    K/V are computed once on slot 0 and copied to the other slots (the rows' caches are then
    exactly what separate prefills would write)."""
    R = len(prompts)
    for r in range(R):
        model.free(r)
    if shared_prefix:
        pre = list(prompts[0][:shared_prefix])
        assert all(list(p[:shared_prefix]) == pre for p in prompts)
        model.forward(pre, [0] * len(pre), list(range(len(pre))), last_only=True)
        for r in range(1, R):
            model.cache[r] = model.cache[0].clone()
    last = []
    for r, p in enumerate(prompts):
        tail = list(p[shared_prefix:])
        assert tail, "each prompt needs at least one id past the shared prefix"
        last.append(model.forward(tail, [r] * len(tail),
                                  list(range(shared_prefix, len(p))), last_only=True)[-1])
    seen = [list(p) for p in prompts]
    steps = len(forced[0])
    assert all(len(f) == steps for f in forced)
    trace: List[List[torch.Tensor]] = [[] for _ in range(R)]
    logits = torch.stack(last)
    for k in range(steps):
        for r in range(R):
            trace[r].append(apply_penalty(logits[r], seen[r], penalty))
            seen[r].append(int(forced[r][k]))
        if k + 1 < steps:
            logits = model.forward([int(forced[r][k]) for r in range(R)], list(range(R)),
                                   [len(prompts[r]) + k for r in range(R)])
    return trace
