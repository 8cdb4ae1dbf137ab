"""Serving over the GPUs of one node: one worker process per GPU, least-loaded dispatch.

SURVEY.md §8(e): utterance streams are independent, so each GPU holds a full weight replica
in its own process (no GIL shared between GPUs, no per-step collective) and rank 0 -- the
process that runs the HTTP surface -- assigns every new stream to the worker with the fewest
outstanding tokens.  The reference has one engine per process and no multi-GPU serving
(its vLLM engine is created with default parallelism, engine_class.py:48-60); this is the
MI355X replacement for running one server per GPU behind a balancer.

Requests and PCM cross process boundaries through ``multiprocessing`` queues (a stream is
~1 MB of PCM at most, 2 KB - 4 KB per chunk); nothing on the data path needs RCCL.
``GpuPool`` exposes the same ``submit`` / ``stream`` surface as ``service.Service``.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import queue
import threading
import time
from typing import Callable, Dict, Iterator, List, Optional

from . import inference as I


def _service_factory(device: int):
    from .service import Service
    from . import config as C
    return Service(device=device, max_pos=min(C.MX_MAX_POS, 8192))


def _worker(device: int, inbox, outbox, factory: Callable, content_seed: int = 0) -> None:
    """Worker process: one Service on `device`; forwards each stream's chunks to rank 0.
    ``content_seed``: the parent's ``config.CONTENT_SEED`` (a spawn child re-imports config
    from the environment, so a value the parent set in-process would otherwise be lost)."""
    from . import config
    config.CONTENT_SEED = content_seed
    try:
        svc = factory(device)
    except BaseException as e:  # report and exit: the pool marks this worker dead
        outbox.put(("dead", -1, (device, repr(e))))
        return
    outbox.put(("ready", -1, (device, None)))
    handles: Dict[int, object] = {}
    lock = threading.Lock()

    def pump(rid, h):
        err = None
        try:
            while True:
                c = h.get()
                if c is None:
                    break
                outbox.put(("chunk", rid, c))
        except BaseException as e:
            err = repr(e)
        with lock:
            handles.pop(rid, None)
        outbox.put(("end", rid, err))

    while True:
        msg = inbox.get()
        kind = msg[0]
        if kind == "stop":
            break
        if kind in ("submit", "submit_tokens"):
            try:
                if kind == "submit":
                    _, rid, text, voice, kw = msg
                    h = svc.submit(text, voice, **kw)
                else:  # token-only stream (/v1/completions): chunks are token ids
                    _, rid, ids, kw = msg
                    h = svc.submit_tokens(ids, **kw)
            except BaseException as e:
                outbox.put(("end", rid, repr(e)))
                continue
            with lock:
                handles[rid] = h
            threading.Thread(target=pump, args=(rid, h), daemon=True).start()
        elif kind == "cancel":
            with lock:
                h = handles.get(msg[1])
            if h is not None:
                h.cancel()
    close = getattr(svc, "close", None)
    if close is not None:
        close()


class PoolHandle:
    """Rank-0 view of one remote stream (same surface as batching.StreamHandle)."""

    def __init__(self, pool: "GpuPool", rid: int, worker: int, cost: int):
        self.pool, self.rid, self.worker, self.cost = pool, rid, worker, cost
        self._q: "queue.Queue" = queue.Queue()
        self.error: Optional[str] = None
        self._ended = False

    def get(self, timeout: Optional[float] = None):
        if self._ended:
            return None
        item = self._q.get(timeout=timeout)
        if item is None:
            self._ended = True
            if self.error is not None:
                raise RuntimeError(f"worker {self.worker}: {self.error}")
        return item

    def chunks(self) -> Iterator[bytes]:
        while True:
            c = self.get()
            if c is None:
                return
            yield c

    def cancel(self) -> None:
        self.pool._cancel(self)


def _content_seed() -> int:
    from . import config
    return int(config.CONTENT_SEED)


class GpuPool:
    def __init__(self, n_workers: int, factory: Callable = _service_factory,
                 devices: Optional[List[int]] = None, start_timeout: float = 600.0,
                 poll_s: float = 0.5, respawn: bool = True):
        ctx = mp.get_context("spawn")
        self.factory, self.poll_s, self.respawn = factory, poll_s, respawn
        self._respawned: Dict[int, bool] = {}
        self.devices = devices if devices is not None else list(range(n_workers))
        self.inboxes = [ctx.Queue() for _ in self.devices]
        self.outbox = ctx.Queue()
        self.procs = [ctx.Process(target=_worker, args=(d, ib, self.outbox, factory,
                                                          _content_seed()),
                                  daemon=True) for d, ib in zip(self.devices, self.inboxes)]
        for p in self.procs:
            p.start()
        self.load = [0] * len(self.devices)   # outstanding tokens per worker
        self.alive = [False] * len(self.devices)
        self._handles: Dict[int, PoolHandle] = {}
        self._lock = threading.Lock()
        self._ids = itertools.count()
        ready = 0
        while ready < len(self.devices):
            kind, _, info = self.outbox.get(timeout=start_timeout)
            if kind == "dead":
                self.close()
                raise RuntimeError(f"GPU worker failed to start: {info[1]}")
            ready += 1
        self.alive = [True] * len(self.devices)
        self._reader = threading.Thread(target=self._read, name="mx-pool", daemon=True)
        self._reader.start()

    def _read(self) -> None:
        # liveness is checked on a clock, not only when the outbox goes quiet: while other
        # workers stream chunks the outbox never empties, and a dead worker's clients would
        # otherwise wait forever
        next_reap = time.monotonic() + self.poll_s
        while True:
            now = time.monotonic()
            if now >= next_reap:
                self._reap()
                next_reap = now + self.poll_s
            try:
                kind, rid, payload = self.outbox.get(timeout=max(0.0, next_reap - now))
            except queue.Empty:
                continue
            except (EOFError, OSError):
                return
            if kind == "closed":
                return
            if kind in ("ready", "dead"):  # a replacement worker came up (or failed to)
                w = self.devices.index(payload[0])
                with self._lock:
                    self.alive[w] = kind == "ready"
                continue
            with self._lock:
                h = self._handles.get(rid)
                if kind == "end" and h is not None:
                    self._handles.pop(rid, None)
                    self.load[h.worker] -= h.cost
            if h is None:
                continue
            if kind == "chunk":
                h._q.put(payload)
            elif kind == "end":
                h.error = payload
                h._q.put(None)

    def _reap(self) -> None:
        """A worker that died after startup (GPU fault, OOM, signal) ends every stream it
        held with an error and takes no new ones; a fresh process replaces it (never a
        re-exec of a process that touched the GPU)."""
        for w, p in enumerate(self.procs):
            if not self.alive[w] or p.is_alive():
                continue
            with self._lock:
                self.alive[w] = False
                lost = [h for h in self._handles.values() if h.worker == w]
                for h in lost:
                    self._handles.pop(h.rid, None)
                self.load[w] = 0
            for h in lost:
                h.error = f"GPU worker {w} died (exit code {p.exitcode})"
                h._q.put(None)
            if self.respawn and not self._respawned.get(w):  # once per slot: no crash loop
                self._spawn(w)

    def _spawn(self, w: int) -> None:
        """Start a replacement worker for slot ``w``; it takes requests once ready."""
        ctx = mp.get_context("spawn")
        self.inboxes[w] = ctx.Queue()
        self.procs[w] = ctx.Process(target=_worker, args=(self.devices[w], self.inboxes[w],
                                                          self.outbox, self.factory,
                                                          _content_seed()), daemon=True)
        self.procs[w].start()
        self._respawned[w] = True

    def pick(self) -> int:
        """Least outstanding tokens over live workers; ties to the lowest index."""
        live = [i for i in range(len(self.load)) if self.alive[i]]
        if not live:
            raise RuntimeError("no GPU worker is alive")
        return min(live, key=lambda i: (self.load[i], i))

    def _enqueue(self, cost: int, make_msg) -> PoolHandle:
        with self._lock:
            w = self.pick()
            rid = next(self._ids)
            h = PoolHandle(self, rid, w, cost)
            self._handles[rid] = h
            self.load[w] += cost
        self.inboxes[w].put(make_msg(rid))
        return h

    def submit(self, text: str, voice: str = I.DEFAULT_VOICE, max_tokens: Optional[int] = None,
               **kw) -> PoolHandle:
        kw = dict(kw, max_tokens=max_tokens)
        return self._enqueue(max_tokens or I.MAX_TOKENS,
                             lambda rid: ("submit", rid, text, voice, kw))

    def submit_tokens(self, prompt_ids, max_tokens: Optional[int] = None, **kw) -> PoolHandle:
        """Token-only stream on the least-loaded GPU (/v1/completions): ``get`` -> id | None."""
        kw = dict(kw, max_tokens=max_tokens)
        ids = [int(t) for t in prompt_ids]
        return self._enqueue(max_tokens or I.MAX_TOKENS,
                             lambda rid: ("submit_tokens", rid, ids, kw))

    def stream(self, text: str, voice: str = I.DEFAULT_VOICE, max_tokens: Optional[int] = None,
               cancel: Optional[threading.Event] = None, **kw) -> Iterator[bytes]:
        h = self.submit(text, voice, max_tokens, **kw)
        try:
            while True:
                if cancel is not None and cancel.is_set():
                    return
                try:
                    c = h.get(timeout=0.05)
                except queue.Empty:
                    continue
                if c is None:
                    return
                yield c
        finally:
            h.cancel()

    def _cancel(self, h: PoolHandle) -> None:
        with self._lock:
            live = h.rid in self._handles
        if live:
            self.inboxes[h.worker].put(("cancel", h.rid))

    def close(self) -> None:
        for ib in self.inboxes:
            ib.put(("stop",))
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self.outbox.put(("closed", -1, None))
