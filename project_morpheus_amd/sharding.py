"""Batch-sharding of independent utterance jobs over the GPUs of one node.

The reference synthesises long text by splitting it into sentence batches of at most
``max_batch_chars`` (tts_engine/inference.py:249-292, remote_backend.py:221-241) and
generating them one after another as independent prompts (remote_backend.py:182-193); the
segments are then joined by plain concatenation on the streaming path (orchestrator/
stitcher.py with ``overlap_ms=0``, server.py:154-156) or with a 50 ms crossfade for files
(``stitch_wav_files``, inference.py:294-365).  Those batches share nothing, so the MI355X
path spreads them over one process per GPU:

* ``plan_jobs``    — documents -> ordered (doc, part) jobs with their prompt ids;
* ``assign``       — longest-first greedy balance of jobs over ranks (deterministic);
* ``gather_pcm``   — the only collective: each rank's PCM (bytes) to rank 0 through
                     ``torch.distributed`` point-to-point sends (RCCL over xGMI with the
                     ``nccl`` backend, CPU tensors with ``gloo``), metadata by
                     ``all_gather_object``;
* ``assemble``     — rank 0 rebuilds every document in part order (concat or crossfade).

No tensor parallelism and no per-step collective: every GPU holds a full weight replica
(6.6 GB bf16 of 288 GB) and decodes its own streams.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from . import inference as I


@dataclass
class Job:
    doc: int
    part: int
    text: str
    prompt_ids: List[int] = field(default_factory=list)
    max_tokens: int = 0

    @property
    def cost(self) -> int:
        return self.max_tokens or len(self.text)


def plan_jobs(docs: Sequence[str], encode: Callable[[str], List[int]], voice: str,
              max_tokens: int, max_batch_chars: int = 1000) -> List[Job]:
    """Every document -> its long-form batches (same split as the reference), in order."""
    jobs = []
    for d, text in enumerate(docs):
        for p, part in enumerate(I.batch_sentences(text, max_batch_chars, True)):
            ids = I.prompt_ids(encode(f"{I.resolve_voice(voice)}: {part}"))
            jobs.append(Job(d, p, part, ids, max_tokens))
    return jobs


def assign(jobs: Sequence[Job], world: int) -> List[List[int]]:
    """Job indices per rank: longest-processing-time first onto the least-loaded rank
    (ties: lowest rank, then job order), so every rank derives the same plan."""
    load = [0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    order = sorted(range(len(jobs)), key=lambda i: (-jobs[i].cost, i))
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += jobs[i].cost
    return [sorted(x) for x in out]


def gather_pcm(mine: Dict[int, bytes], rank: int, world: int, device=None,
               group=None) -> Optional[Dict[int, bytes]]:
    """All ranks' {job index: PCM16 bytes} -> rank 0 (None elsewhere)."""
    if world == 1:
        return dict(mine)
    import torch
    import torch.distributed as dist
    meta = [(k, len(v)) for k, v in sorted(mine.items())]
    metas: List = [None] * world
    dist.all_gather_object(metas, meta, group=group)
    if device is None:
        device = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    if rank != 0:
        buf = b"".join(mine[k] for k, _ in meta)
        if buf:
            t = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(device)
            dist.send(t, dst=0, group=group)
        return None
    out = dict(mine)
    for r in range(1, world):
        total = sum(n for _, n in metas[r])
        if not total:
            continue
        t = torch.empty(total, dtype=torch.uint8, device=device)
        dist.recv(t, src=r, group=group)
        data = t.cpu().numpy().tobytes()
        off = 0
        for k, n in metas[r]:
            out[k] = data[off:off + n]
            off += n
    return out


def assemble(jobs: Sequence[Job], pcm: Dict[int, bytes],
             crossfade_ms: float = 0.0) -> Dict[int, np.ndarray]:
    """Rank 0: document -> int16 samples, parts in order; ``crossfade_ms=0`` is the
    streaming path's plain concatenation, 50 is ``stitch_wav_files``'s crossfade."""
    by_doc: Dict[int, List] = {}
    for i, j in enumerate(jobs):
        by_doc.setdefault(j.doc, []).append((j.part, np.frombuffer(pcm[i], dtype=np.int16)))
    out = {}
    for d, parts in by_doc.items():
        segs = [s for _, s in sorted(parts, key=lambda x: x[0])]
        if crossfade_ms > 0:
            out[d] = I.crossfade_join(segs, crossfade_ms)
        else:
            out[d] = np.concatenate(segs) if segs else np.zeros(0, dtype=np.int16)
    return out


def run_sharded(jobs: Sequence[Job], rank: int, world: int,
                synthesize: Callable[[List[Job]], List[bytes]], device=None,
                group=None, crossfade_ms: float = 0.0) -> Optional[Dict[int, np.ndarray]]:
    """This rank's share of ``jobs`` through ``synthesize`` (-> PCM bytes per job, in the
    given order), gathered and assembled on rank 0."""
    mine_idx = assign(jobs, world)[rank]
    pcm = synthesize([jobs[i] for i in mine_idx]) if mine_idx else []
    mine = {i: bytes(p) for i, p in zip(mine_idx, pcm)}
    allpcm = gather_pcm(mine, rank, world, device=device, group=group)
    if allpcm is None:
        return None
    return assemble(jobs, allpcm, crossfade_ms)


_WORDS = ("the of and to a in is you that it he was for on are as with his they I at be this "
          "have from or one had by word but not what all were we when your can said there use "
          "an each which she do how their if will up other about out many then them these so "
          "some her would make like him into time has look two more write go see number no "
          "way could people my than first water been call who oil its now find long down day "
          "did get come made may part").split()


def long_read_documents(n_docs: int = 16, n_chars: int = 3000, seed: int = 5) -> List[str]:
    """Synthetic ``long_read`` workload (BASELINE configs[3]): seeded prose
    with sentence punctuation, ~``n_chars`` per document."""
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(n_docs):
        words, total = [], 0
        while total < n_chars:
            k = int(rng.integers(4, 18))
            sent = [_WORDS[int(rng.integers(0, len(_WORDS)))] for _ in range(k)]
            s = " ".join(sent).capitalize() + ".!?"[int(rng.integers(0, 3))]
            words.append(s)
            total += len(s) + 1
        docs.append(" ".join(words))
    return docs


def roofline_wall(jobs: Sequence[Job], weight_bytes: int, kv_bytes_per_pos: int,
                  max_rows: int = 32, hbm_bps: float = 8e12) -> float:
    """HBM-roofline time for ONE GPU to serve ``jobs`` through the continuous-batching loop:
    jobs are admitted in order, at most ``max_rows`` at a time; every prefill streams the
    weights once, and every decode step streams them once plus the KV cache of each live row
    (``kv_bytes_per_pos`` per position).  A lower bound of the wall (it ignores compute,
    launch gaps and the SNAC work), used to bound strong scaling (``scaling_bound``)."""
    live: List[List[int]] = []          # [position, tokens left]
    pending = [(len(j.prompt_ids), j.max_tokens) for j in jobs]
    total = 0.0
    while pending or live:
        while pending and len(live) < max_rows:
            p, t = pending.pop(0)
            total += weight_bytes
            live.append([p, t - 1])     # the prefill picks the first token
        live = [r for r in live if r[1] > 0]
        if not live:
            continue
        total += weight_bytes + kv_bytes_per_pos * sum(r[0] + 1 for r in live)
        for r in live:
            r[0] += 1
            r[1] -= 1
    return total / hbm_bps


def scaling_bound(jobs: Sequence[Job], world: int, weight_bytes: int, kv_bytes_per_pos: int,
                  max_rows: int = 32) -> dict:
    """Strong-scaling bound of a FIXED job list spread over ``world`` GPUs by ``assign``,
    every GPU at its HBM roofline: efficiency = T(1 GPU) / (world x T(most loaded rank)).
    One GPU batches up to ``max_rows`` streams per weight read; ``world`` GPUs each batch
    only their share, so the weight bytes per token grow with ``world`` and the bound falls
    below 1 even with perfect kernels."""
    t1 = roofline_wall(jobs, weight_bytes, kv_bytes_per_pos, max_rows)
    plan = assign(jobs, world)
    tn = max(roofline_wall([jobs[i] for i in mine], weight_bytes, kv_bytes_per_pos, max_rows)
             for mine in plan)
    return {"world": world, "t1_roofline_s": round(t1, 4), "tn_roofline_s": round(tn, 4),
            "efficiency_bound": round(t1 / (world * tn), 4)}
