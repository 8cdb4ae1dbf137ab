"""Continuous batching of concurrent utterance streams on one GPU (BASELINE configs 3-5, and
the serving path behind every adapter).

The reference serves concurrent requests by handing them to vLLM's continuous-batching
engine, one request per thread (Orpheus-TTS/orpheus_tts_pypi/orpheus_tts/engine_class.py:
114-134), and decodes each stream's SNAC windows independently (speechpipe.py:191-293).
``BatchSynthesizer`` is that loop for the MI355X engine:

* every stream owns one KV slot and one decode row; a step decodes rows [0, n_rows) at once
  (``mx_llm_decode(n_rows)``: one hipGraph per row count, the one-launch step for one row),
  rows without a stream are parked on the scratch slot; each row decodes under its own
  generation parameters (penalty, temperature, top-p, seed: per-slot state set at prefill);
* rows are compacted: when a stream ends, the highest live row moves into the lowest free
  one (``mx_llm_move_row``: same KV slot, stream-ordered between steps), so a step runs the
  row class of the live stream count, not of the highest row index ever used;
* a stream is admitted as soon as it has arrived and a row is free: its prefill is enqueued
  between steps (ordered on the same HIP stream, nothing drains);
* ``depth`` steps stay queued on the GPU; tokens are read from the host-mapped history when
  a step's event completes, never by a per-token copy;
* a stream that has issued all its tokens is parked at once (its position never runs past
  ``max_pos``); a cancelled stream (``StreamRequest.cancel``, the adapter's ``reset``) frees
  its row at the next iteration and its undelivered audio is dropped;
* each stream keeps the reference window schedule (``schedule.WindowScheduler``); the
  windows that become due in one host iteration are grouped by frame count and decoded by
  ONE batched SNAC call per group on a second HIP stream, PCM read from host-mapped memory.
  NoiseBlock noise of window j of a stream is drawn from (stream noise seed, j) only, so a
  stream's audio does not depend on what it was batched with.

Two drivers share the loop: ``run(requests)`` (offline: arrival times, bench / long-form
jobs) and ``start()`` + ``submit(request) -> StreamHandle`` (online: the per-GPU service the
adapters use; a background thread owns the GPU).
"""
from __future__ import annotations

import collections

import queue
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .config import BATCH_DEPTH, SNAC_MAX_HOLD, SNAC_MIN_BATCH, STOP_IDS
from .engine import SAMPLES_PER_FRAME, SLICE_HI, SLICE_LO, LlmEngine, SnacDecoder
from .schedule import WindowScheduler, code_of_id, frames_for_slice

_MASK48 = 0xFFFFFFFFFFFF


def window_seed(noise_seed: int, j: int) -> int:
    """Noise seed of a stream's j-th SNAC window (batching-invariant)."""
    return (noise_seed * 1000003 + j) & _MASK48


@dataclass(eq=False)
class StreamRequest:
    prompt_ids: Sequence[int]
    max_tokens: int
    arrival: float = 0.0                    # seconds after run start (offline driver)
    inject_ids: Optional[Sequence[int]] = None  # synthetic audio ids (bench, random weights)
    stop_ids: Sequence[int] = STOP_IDS
    penalty: float = 1.1
    temperature: float = 0.0                # <= 0: greedy (the parity mode)
    top_p: float = 1.0
    seed: int = 0                           # sampling stream (Philox key)
    noise_seed: Optional[int] = None        # SNAC noise stream (None: assigned at admission)
    on_chunk: Optional[Callable[["StreamRequest", bytes], None]] = None
    on_done: Optional[Callable[["StreamRequest"], None]] = None
    on_token: Optional[Callable[["StreamRequest", int], None]] = None
    audio: bool = True                      # False: token stream only (no SNAC windows)
    # filled in by the synthesizer
    tokens: List[int] = field(default_factory=list)
    pcm: List[bytes] = field(default_factory=list)  # for callers that collect chunks here
    samples: int = 0
    windows: int = 0
    cancelled: bool = False
    error: Optional[BaseException] = None
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

    def cancel(self) -> None:
        """Barge-in: the loop frees the row at its next iteration, nothing more is emitted."""
        self.cancelled = True


def check_params(penalty: float, temperature: float, top_p: float, max_tokens: int) -> None:
    """Reject generation parameters the device cannot run (mx_llm_prefill returns MX_ERR_ARG
    for them): a bad request must fail alone, at submit time, never inside the GPU loop."""
    import math
    for name, v in (("repetition_penalty", penalty), ("temperature", temperature),
                    ("top_p", top_p)):
        if not isinstance(v, (int, float)) or not math.isfinite(v):
            raise ValueError(f"{name} must be a finite number, got {v!r}")
    if penalty <= 0:
        raise ValueError(f"repetition_penalty must be > 0, got {penalty}")
    if temperature < 0:
        raise ValueError(f"temperature must be >= 0, got {temperature}")
    if not 0 < top_p <= 1:
        raise ValueError(f"top_p must be in (0, 1], got {top_p}")
    if not isinstance(max_tokens, int) or max_tokens < 1:
        raise ValueError(f"max_tokens must be a positive integer, got {max_tokens!r}")


class _Row:
    """One stream's decode state; ``idx`` is the device row it decodes in (rows are compacted,
    so it can change), ``slot`` its KV slot (fixed for the stream's life)."""

    def __init__(self, idx: int):
        self.idx = idx
        self.slot = -1
        self.req: Optional[StreamRequest] = None
        self.sched: Optional[WindowScheduler] = None
        self.n0 = 0          # prompt length (position of generated token 0)
        self.issued = 0      # generated tokens whose step has been enqueued
        self.limit = 0       # tokens this row may issue (max_tokens clipped to max_pos)
        self.parked = False  # released on the device (all tokens issued / stopped)
        self.stopped = False


def plan_compaction(rows: List[_Row]) -> List[Tuple[int, int]]:
    """Row compaction plan, applied to ``rows`` in place: while a free row (no stream) sits
    below the highest row still decoding, that row's stream moves into the lowest free row.
    Returns the device moves (dst, src) in order (``mx_llm_move_row``).  ``rows[i].idx == i``
    holds before and after; a stream keeps its KV slot, so host reads by slot are unaffected,
    and the steps already queued for the old row index run before the move on the stream.
    Rows that are parked (all tokens issued) or stopped stay where they are: they decode no
    more steps, so they never set the row class."""
    moves = []
    while True:
        free = [r for r in rows if r.req is None]
        live = [r for r in rows if r.req is not None and not r.stopped and not r.parked]
        if not free or not live:
            return moves
        lo, hi = free[0], live[-1]
        if lo.idx > hi.idx:
            return moves
        i, j = lo.idx, hi.idx
        moves.append((i, j))
        rows[i], rows[j] = hi, lo
        hi.idx, lo.idx = i, j


class _BatchRing:
    """Host-mapped staging for batched SNAC calls: codes and noise seeds in, PCM16 out."""

    def __init__(self, n: int, max_batch: int, max_frames: int):
        self.n, self.max_batch = n, max_batch
        self.cbytes = max_batch * 7 * max_frames * 4
        self.sbytes = max_batch * 8
        self.pbytes = max_batch * (SLICE_HI - SLICE_LO) * 2
        per = (self.cbytes + self.sbytes + self.pbytes + 255) // 256 * 256
        self.buf = _lib.HostBuffer(n * per)
        self.codes = [self.buf.view(np.int32, max_batch * 7 * max_frames, i * per)
                      for i in range(n)]
        self.seeds = [self.buf.view(np.uint64, max_batch, i * per + self.cbytes)
                      for i in range(n)]
        self.pcm = [self.buf.view(np.int16, max_batch * (SLICE_HI - SLICE_LO),
                                  i * per + self.cbytes + self.sbytes) for i in range(n)]
        self.codes_dev = [self.buf.dev_ptr(i * per) for i in range(n)]
        self.seeds_dev = [self.buf.dev_ptr(i * per + self.cbytes) for i in range(n)]
        self.pcm_dev = [self.buf.dev_ptr(i * per + self.cbytes + self.sbytes) for i in range(n)]


class StreamHandle:
    """Online stream: PCM chunks arrive through a queue filled by the loop thread (never
    blocks the loop: the queue is unbounded, one utterance is at most ~1 MB of PCM)."""

    _END = object()

    def __init__(self, req: StreamRequest):
        self.req = req
        self._q: "queue.Queue" = queue.Queue()

    def _chunk(self, req, data: bytes) -> None:
        self._q.put(data)

    def _done(self, req) -> None:
        self._q.put(self._END)

    def get(self, timeout: Optional[float] = None):
        """Next PCM chunk, or None at the end of the stream; re-raises a loop failure."""
        item = self._q.get(timeout=timeout)
        if item is self._END:
            self._q.put(self._END)  # the end stays visible to later calls
            if self.req.error is not None:
                raise self.req.error
            return None
        return item

    def chunks(self) -> Iterator[bytes]:
        while True:
            c = self.get()
            if c is None:
                return
            yield c

    def cancel(self) -> None:
        self.req.cancel()


class TokenHandle(StreamHandle):
    """Online token-only stream (the /v1/completions surface): ``get`` -> token id | None."""

    def _token(self, req, tok: int) -> None:
        self._q.put(tok)


class BatchSynthesizer:
    def __init__(self, llm: LlmEngine, snac: SnacDecoder, depth: Optional[int] = None, seed: int = 0,
                 snac_min_batch: Optional[int] = None, snac_max_hold: Optional[int] = None,
                 compact: bool = True):
        if llm.max_slots < llm.max_batch:
            raise ValueError("BatchSynthesizer needs one KV slot per decode row")
        self.llm, self.snac, self.seed = llm, snac, seed
        self.compact = compact  # row compaction (mx_llm_move_row) when streams end
        self.row_steps = collections.Counter()  # decode steps issued per row count (stats)
        self.depth = max(1, BATCH_DEPTH if depth is None else depth)
        # SNAC window coalescing: due windows are held until `snac_min_batch` of them are
        # ready or the oldest has waited `snac_max_hold` decode steps (a stream's first window
        # and closing streams' windows go at once).  Staggered streams make ~streams / 7
        # windows due per step; a bigger SNAC batch costs less per window.
        self.snac_min_batch = max(1, SNAC_MIN_BATCH if snac_min_batch is None else snac_min_batch)
        self.snac_max_hold = max(0, SNAC_MAX_HOLD if snac_max_hold is None else snac_max_hold)
        self.stream = torch.cuda.Stream(llm.device)
        self.snac_stream = torch.cuda.Stream(llm.device)
        self.ring = _BatchRing(16, snac.max_batch, snac.max_frames)
        self._calls = 0
        self._admitted = 0
        self._live: List[StreamRequest] = []
        # online driver
        self._inbox: Deque[StreamRequest] = deque()
        self._cv = threading.Condition()
        self._thread: Optional[threading.Thread] = None
        self._stop = False
        self._t0 = time.perf_counter()
        self.outstanding_tokens = 0  # tokens still owed to submitted streams (dispatch load)

    # ---------------------------------------------------------------------------------
    def run(self, requests: List[StreamRequest], on_chunk=None) -> float:
        """Serve ``requests`` (admitted in arrival order) to completion; returns wall seconds.
        ``on_chunk(request, pcm_bytes)`` is called for every non-empty PCM chunk in order."""
        waiting: Deque[StreamRequest] = deque(sorted(requests, key=lambda r: r.arrival))
        if on_chunk is not None:
            for r in waiting:
                r.on_chunk = r.on_chunk or on_chunk
        n = len(waiting)
        finished = [0]

        def done_cb(_req):
            finished[0] += 1

        t0 = time.perf_counter()

        def poll(now):
            out = []
            while waiting and waiting[0].arrival <= now:
                out.append(waiting.popleft())
            return out

        def idle(now):
            if waiting:
                time.sleep(max(0.0, min(0.001, waiting[0].arrival - now)))

        self._loop(t0, poll, idle, lambda: finished[0] >= n and not waiting, done_cb)
        return time.perf_counter() - t0

    # ---------------------------------------------------------------------------------
    def start(self) -> "BatchSynthesizer":
        """Online mode: a daemon thread owns the GPU and serves ``submit``-ted streams."""
        if self._thread is None:
            self._t0 = time.perf_counter()
            self._stop = False
            self._thread = threading.Thread(target=self._serve, name="mx-batch", daemon=True)
            self._thread.start()
        return self

    def submit(self, req: StreamRequest) -> StreamHandle:
        check_params(req.penalty, req.temperature, req.top_p, req.max_tokens)
        if self._thread is None:
            self.start()
        h = StreamHandle(req) if req.audio else TokenHandle(req)
        req.on_chunk, req.on_done = h._chunk, h._done
        if not req.audio:
            req.on_token = h._token
        req.arrival = time.perf_counter() - self._t0
        with self._cv:
            if self._stop:
                raise RuntimeError("BatchSynthesizer stopped")
            self._inbox.append(req)
            self.outstanding_tokens += req.max_tokens
            self._cv.notify()
        return h

    def stop(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def _serve(self) -> None:
        def poll(now):
            with self._cv:
                out = list(self._inbox)
                self._inbox.clear()
            return out

        def idle(now):
            with self._cv:
                if not self._inbox and not self._stop:
                    self._cv.wait(timeout=0.05)

        def done_cb(req):
            with self._cv:
                self.outstanding_tokens -= req.max_tokens

        try:
            self._loop(self._t0, poll, idle, lambda: self._stop, done_cb)
        except BaseException as e:  # fail every stream loudly, never hang a consumer
            with self._cv:
                self._stop = True
                orphans = list(self._inbox) + list(self._live)
                self._inbox.clear()
            for req in orphans:
                req.error = e
                if req.on_done is not None:
                    req.on_done(req)
            raise

    # ---------------------------------------------------------------------------------
    def _loop(self, t0: float, poll, idle, finished, done_cb) -> None:
        llm, B = self.llm, self.llm.max_batch
        rows = [_Row(i) for i in range(B)]
        free_slots = set(range(llm.max_slots))
        waiting: Deque[StreamRequest] = deque()
        inflight: Deque = deque()   # (event, [(row, req, k)])
        pending: Deque = deque()    # (event, ring index, [(req, nbytes)])
        closing: Deque = deque()    # streams whose end waits for their last SNAC call
        held: List = []             # due SNAC windows not launched yet (coalescing)
        held_age = [0]              # decode steps the oldest held window has waited
        live = self._live

        def now():
            return time.perf_counter() - t0

        def complete(req: StreamRequest) -> None:
            req.t_done = now()
            if any(q is req for q in live):
                live.remove(req)
            done_cb(req)
            if req.on_done is not None:
                req.on_done(req)

        def park(r: _Row):
            if not r.parked:
                llm.release_row(r.idx, self.stream)
                r.parked = True

        def admit():
            for r in rows:
                if not waiting:
                    return
                if r.req is not None:
                    continue
                req = waiting.popleft()
                if req.cancelled:
                    complete(req)
                    continue
                n0 = len(req.prompt_ids)
                if n0 < 1 or n0 > llm.max_prefill or n0 >= llm.max_pos:
                    req.error = ValueError(f"prompt of {n0} ids does not fit (max_prefill "
                                           f"{llm.max_prefill}, max_pos {llm.max_pos})")
                    complete(req)
                    continue
                if req.noise_seed is None:
                    req.noise_seed = (self.seed * 1000003 + self._admitted) & _MASK48
                self._admitted += 1
                slot = min(free_slots)
                try:  # a request the device rejects fails alone; the loop serves on
                    check_params(req.penalty, req.temperature, req.top_p, req.max_tokens)
                    llm.prefill(slot, r.idx, req.prompt_ids, req.penalty, self.stream,
                                temperature=req.temperature, top_p=req.top_p, seed=req.seed)
                except (ValueError, _lib.MxError) as e:
                    if isinstance(e, _lib.MxError) and e.rc != _lib.MX_ERR_ARG:
                        raise  # a device failure is not this request's fault
                    req.error = e
                    complete(req)
                    continue
                free_slots.discard(slot)
                r.slot = slot
                r.req, r.sched, r.n0 = req, WindowScheduler(), n0
                r.limit = max(1, min(req.max_tokens, llm.max_pos - n0))
                r.issued, r.stopped, r.parked = 1, False, False
                req.t_admit = now()
                live.append(req)
                ev = torch.cuda.Event()
                ev.record(self.stream)
                inflight.append((ev, [(r, req, 0)]))
                if r.issued >= r.limit:
                    park(r)

        def launch_windows(due: List):
            """due: [(req, window index, codes)] -> one SNAC call per frame-count group."""
            groups: Dict[int, List] = {}
            for item in due:  # grouped by the frames the kept slice depends on (7 -> 5)
                n = len(item[2]) // 7
                groups.setdefault(frames_for_slice(n, min(SLICE_HI, SAMPLES_PER_FRAME * n)),
                                  []).append(item)
            for nf, items in groups.items():
                for s in range(0, len(items), self.ring.max_batch):
                    chunk = items[s:s + self.ring.max_batch]
                    i = self._calls % self.ring.n
                    while len(pending) >= self.ring.n:
                        drain(block=True, upto=1)
                    codes, seeds = self.ring.codes[i], self.ring.seeds[i]
                    for j, (req, widx, win) in enumerate(chunk):
                        codes[j * 7 * nf:(j + 1) * 7 * nf] = win[:7 * nf]
                        seeds[j] = window_seed(req.noise_seed, widx)
                    lo, hi = SLICE_LO, min(SLICE_HI, SAMPLES_PER_FRAME * nf)
                    hi = max(lo, hi)
                    self.snac.decode_ptr(self.ring.codes_dev[i], nf, len(chunk), 0, 0,
                                         self.ring.pcm_dev[i] if hi > lo else 0, 0, lo, hi,
                                         self.snac_stream, seeds_ptr=self.ring.seeds_dev[i])
                    e = torch.cuda.Event()
                    e.record(self.snac_stream)
                    pending.append((e, i, [(req, (hi - lo) * 2) for req, _, _ in chunk]))
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
                    if not nbytes or req.cancelled:
                        continue
                    n = nbytes // 2
                    data = pcm[j * n:(j + 1) * n].tobytes()
                    req.samples += n
                    if req.t_first_audio is None:
                        req.t_first_audio = now()
                    if req.on_chunk is not None:
                        req.on_chunk(req, data)

        def finish(r: _Row, due: List):
            req = r.req
            if not req.cancelled and req.audio:
                for win in r.sched.flush():
                    due.append((req, req.windows, win))
                    req.windows += 1
            park(r)
            closing.append(req)
            free_slots.add(r.slot)
            r.req, r.sched, r.stopped, r.parked, r.slot = None, None, False, False, -1

        def compact():
            """Live rows to a prefix (plan_compaction), so a step runs the row class of the
            live stream count: a lone stream in row 31 no longer costs a 32-row step."""
            if not self.compact:
                return
            for dst, src in plan_compaction(rows):
                llm.move_row(dst, src, self.stream)

        def announce():
            # a closing stream's windows were all launched when it closed: once no pending
            # SNAC call holds one of them, its end is announced (in close order)
            while closing:
                req = closing[0]
                if any(q is req for _, _, items in pending for q, _ in items):
                    return
                closing.popleft()
                complete(req)

        while True:
            waiting.extend(poll(now()))
            for r in rows:  # barge-in: free cancelled rows now
                if r.req is not None and r.req.cancelled:
                    finish(r, [])
            admit()
            compact()
            act = [r for r in rows if r.req is not None and not r.stopped and not r.parked]
            # keep `depth` steps queued for the rows that still need tokens
            while act and len(inflight) < self.depth:
                n_rows = max(r.idx for r in act) + 1
                llm.decode(n_rows, self.stream)
                self.row_steps[n_rows] += 1
                ev = torch.cuda.Event()
                ev.record(self.stream)
                entries = []
                for r in act:
                    entries.append((r, r.req, r.issued))
                    r.issued += 1
                    if r.issued >= r.limit:
                        park(r)
                inflight.append((ev, entries))
                act = [r for r in act if not r.parked]
            if not inflight:
                drain(block=bool(pending) and not waiting)
                announce()
                if finished() and not pending and not closing and not waiting and \
                        all(r.req is None for r in rows):
                    break
                if not pending and not closing:
                    idle(now())
                continue
            ev, entries = inflight.popleft()
            ev.synchronize()
            llm.check(self.stream)
            due: List = []
            for r, req, k in entries:
                if r.req is not req or r.stopped or req.cancelled:
                    continue  # speculative step of a stream that already ended
                tok = int(llm.hist[r.slot, r.n0 + k])
                req.tokens.append(tok)
                if req.on_token is not None:
                    req.on_token(req, tok)
                if req.audio:
                    feed = int(req.inject_ids[k]) if req.inject_ids is not None else tok
                    for win in r.sched.push(code_of_id(feed, r.sched.count)):
                        due.append((req, req.windows, win))
                        req.windows += 1
                if tok in req.stop_ids or len(req.tokens) >= r.limit:
                    r.stopped = True
            for r in rows:
                if r.req is not None and r.stopped:
                    finish(r, due)
            if held:
                held_age[0] += 1
            held.extend(due)
            if held and (len(held) >= self.snac_min_batch or held_age[0] >= self.snac_max_hold or
                         closing or any(w == 0 for _, w, _ in held) or not inflight):
                launch_windows(held)
                held.clear()
                held_age[0] = 0
            drain(block=False)
            announce()
        for e, _ in inflight:
            e.synchronize()
