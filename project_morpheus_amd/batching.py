"""Continuous batching of concurrent utterance streams on one GPU (BASELINE configs 3 and 5).

The reference serves concurrent requests by handing them to vLLM's continuous-batching
engine, one request per thread (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:
114-134), and decodes each stream's SNAC windows independently (speechpipe.py:191-293).
``BatchSynthesizer`` is that loop for the MI355X engine:

* every stream owns one KV slot and one decode row; a step decodes all rows at once
  (``mx_llm_decode(n_rows)``, hipGraph per row count), rows without a stream are parked;
* a new stream is admitted as soon as it has arrived and a row is free: its prefill is
  enqueued between steps (ordered on the same HIP stream, nothing drains);
* ``depth`` steps stay queued on the GPU; tokens are read from the host-mapped history
  when a step's event completes, never by a per-token copy;
* each stream keeps the reference window schedule (``schedule.WindowScheduler``); the
  windows that become due in one host iteration are grouped by frame count and decoded by
  ONE batched SNAC call per group on a second HIP stream, PCM read from host-mapped memory.
"""
from __future__ import annotations

import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .config import STOP_IDS
from .engine import SAMPLES_PER_FRAME, SLICE_HI, SLICE_LO, LlmEngine, SnacDecoder
from .schedule import WindowScheduler, code_of_id


@dataclass
class StreamRequest:
    prompt_ids: Sequence[int]
    max_tokens: int
    arrival: float = 0.0                    # seconds after run start
    inject_ids: Optional[Sequence[int]] = None  # synthetic audio ids (bench, random weights)
    stop_ids: Sequence[int] = STOP_IDS
    penalty: float = 1.1
    # filled in by the synthesizer
    tokens: List[int] = field(default_factory=list)
    pcm: List[bytes] = field(default_factory=list)
    samples: int = 0
    windows: int = 0
    t_admit: Optional[float] = None
    t_first_audio: Optional[float] = None
    t_done: Optional[float] = None

    @property
    def audio_seconds(self) -> float:
        return self.samples / 24000.0

    @property
    def first_audio_ms(self) -> Optional[float]:
        if self.t_first_audio is None:
            return None
        return 1e3 * (self.t_first_audio - self.arrival)


class _Row:
    def __init__(self, idx: int):
        self.idx = idx
        self.req: Optional[StreamRequest] = None
        self.sched: Optional[WindowScheduler] = None
        self.n0 = 0          # prompt length (position of generated token 0)
        self.issued = 0      # generated tokens whose step has been enqueued
        self.stopped = False


class _BatchRing:
    """Host-mapped staging for batched SNAC calls: codes in, PCM16 out, zero-copy."""

    def __init__(self, n: int, max_batch: int, max_frames: int):
        self.n, self.max_batch = n, max_batch
        self.cbytes = max_batch * 7 * max_frames * 4
        self.pbytes = max_batch * (SLICE_HI - SLICE_LO) * 2
        self.buf = _lib.HostBuffer(n * (self.cbytes + self.pbytes))
        self.codes = [self.buf.view(np.int32, max_batch * 7 * max_frames, i * self.cbytes)
                      for i in range(n)]
        base = n * self.cbytes
        self.pcm = [self.buf.view(np.int16, max_batch * (SLICE_HI - SLICE_LO),
                                  base + i * self.pbytes) for i in range(n)]
        self.codes_dev = [self.buf.dev_ptr(i * self.cbytes) for i in range(n)]
        self.pcm_dev = [self.buf.dev_ptr(base + i * self.pbytes) for i in range(n)]


class BatchSynthesizer:
    def __init__(self, llm: LlmEngine, snac: SnacDecoder, depth: int = 2, seed: int = 0):
        if llm.max_slots < llm.max_batch:
            raise ValueError("BatchSynthesizer needs one KV slot per decode row")
        self.llm, self.snac, self.depth, self.seed = llm, snac, depth, seed
        self.stream = torch.cuda.Stream(llm.device)
        self.snac_stream = torch.cuda.Stream(llm.device)
        self.ring = _BatchRing(16, snac.max_batch, snac.max_frames)
        self._calls = 0

    # ---------------------------------------------------------------------------------
    def run(self, requests: List[StreamRequest], on_chunk=None) -> float:
        """Serve ``requests`` (admitted in arrival order) to completion; returns wall seconds.
        ``on_chunk(request, pcm_bytes)`` is called for every non-empty PCM chunk in order."""
        llm, B = self.llm, self.llm.max_batch
        rows = [_Row(i) for i in range(B)]
        waiting: Deque[StreamRequest] = deque(sorted(requests, key=lambda r: r.arrival))
        inflight: Deque = deque()   # (event, [(row, req, k)])
        pending: Deque = deque()    # (event, ring index, [(req, nbytes)])
        t0 = time.perf_counter()
        done = 0

        def now():
            return time.perf_counter() - t0

        def active_rows():
            return [r for r in rows if r.req is not None and not r.stopped]

        def admit():
            for r in rows:
                if not waiting or waiting[0].arrival > now():
                    return
                if r.req is None:
                    req = waiting.popleft()
                    r.req, r.sched, r.n0 = req, WindowScheduler(), len(req.prompt_ids)
                    r.issued, r.stopped = 1, False
                    req.t_admit = now()
                    llm.prefill(r.idx, r.idx, req.prompt_ids, req.penalty, self.stream)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                    inflight.append((ev, [(r, req, 0)]))

        def launch_windows(due: List):
            """due: [(req, window codes)] -> one SNAC call per frame-count group."""
            groups: Dict[int, List] = {}
            for req, win in due:
                groups.setdefault(len(win) // 7, []).append((req, win))
            for nf, items in groups.items():
                for s in range(0, len(items), self.ring.max_batch):
                    chunk = items[s:s + self.ring.max_batch]
                    i = self._calls % self.ring.n
                    while len(pending) >= self.ring.n:
                        drain(block=True, upto=1)
                    codes = self.ring.codes[i]
                    for j, (_, win) in enumerate(chunk):
                        codes[j * 7 * nf:(j + 1) * 7 * nf] = win[:7 * nf]
                    lo, hi = SLICE_LO, min(SLICE_HI, SAMPLES_PER_FRAME * nf)
                    hi = max(lo, hi)
                    self.snac.decode_ptr(self.ring.codes_dev[i], nf, len(chunk), 0,
                                         (self.seed * 1000003 + self._calls) & 0xFFFFFFFFFFFF,
                                         self.ring.pcm_dev[i] if hi > lo else 0, 0, lo, hi,
                                         self.snac_stream)
                    e = torch.cuda.Event()
                    e.record(self.snac_stream)
                    pending.append((e, i, [(req, (hi - lo) * 2) for req, _ in chunk]))
                    for req, _ in chunk:
                        req.windows += 1
                    self._calls += 1

        def drain(block: bool, upto: Optional[int] = None):
            k = 0
            while pending and (upto is None or k < upto):
                e, i, items = pending[0]
                if not block and not e.query():
                    return
                e.synchronize()
                pending.popleft()
                k += 1
                pcm = self.ring.pcm[i]
                for j, (req, nbytes) in enumerate(items):
                    if not nbytes:
                        continue
                    n = nbytes // 2
                    data = pcm[j * n:(j + 1) * n].tobytes()
                    req.samples += n
                    if req.t_first_audio is None:
                        req.t_first_audio = now()
                    if on_chunk is not None:
                        on_chunk(req, data)

        def finish(r: _Row, due: List):
            for win in r.sched.flush():
                due.append((r.req, win))
            r.req.t_done = now()
            llm.release_row(r.idx, self.stream)
            r.req, r.sched, r.stopped = None, None, False

        while done < len(requests):
            admit()
            act = active_rows()
            # keep `depth` steps queued for the rows that still need tokens
            while act and len(inflight) < self.depth:
                n_rows = max(r.idx for r in act) + 1
                need = [r for r in act if r.issued < r.req.max_tokens]
                if not need:
                    break
                llm.decode(n_rows, need[0].req.penalty, self.stream)
                ev = torch.cuda.Event()
                ev.record(self.stream)
                entries = []
                for r in act:
                    if r.issued < r.req.max_tokens:
                        entries.append((r, r.req, r.issued))
                        r.issued += 1
                inflight.append((ev, entries))
            if not inflight:
                if waiting:  # idle until the next arrival
                    time.sleep(max(0.0, min(0.001, waiting[0].arrival - now())))
                    continue
                break
            ev, entries = inflight.popleft()
            ev.synchronize()
            due: List = []
            for r, req, k in entries:
                if r.req is not req or r.stopped:
                    continue  # speculative step of a stream that already ended
                tok = int(llm.hist[r.idx, r.n0 + k])
                req.tokens.append(tok)
                feed = int(req.inject_ids[k]) if req.inject_ids is not None else tok
                for win in r.sched.push(code_of_id(feed, r.sched.count)):
                    due.append((req, win))
                if tok in req.stop_ids or len(req.tokens) >= req.max_tokens:
                    r.stopped = True
            for r in rows:
                if r.req is not None and r.stopped:
                    finish(r, due)
                    done += 1
            if due:
                launch_windows(due)
            drain(block=False)
        for e, _ in inflight:
            e.synchronize()
        drain(block=True)
        return time.perf_counter() - t0
