"""GpuPool (project_morpheus_amd/dispatch.py) on CPU with fake per-GPU services: worker
processes, least-loaded assignment by outstanding tokens, in-order chunks, cancel, errors."""
import queue
import time

import pytest

from _fakes import fake_factory, fake_pcm
from project_morpheus_amd.dispatch import GpuPool


@pytest.fixture(scope="module")
def pool():
    p = GpuPool(3, factory=fake_factory, start_timeout=120)
    yield p
    p.close()


def test_streams_arrive_in_order(pool):
    h = pool.submit("hello", "tara", max_tokens=70)
    assert list(h.chunks()) == fake_pcm("hello", h.worker, 10)


def test_least_loaded_assignment(pool):
    a = pool.submit("slow a", "tara", max_tokens=700)   # worker 0 (all idle)
    b = pool.submit("slow b", "tara", max_tokens=140)   # worker 1
    c = pool.submit("slow c", "tara", max_tokens=70)    # worker 2
    d = pool.submit("slow d", "tara", max_tokens=70)    # least loaded now: worker 2 (70)
    assert (a.worker, b.worker, c.worker, d.worker) == (0, 1, 2, 2)
    for h in (a, b, c, d):
        list(h.chunks())
    deadline = time.time() + 10
    while any(pool.load) and time.time() < deadline:
        time.sleep(0.01)
    assert pool.load == [0, 0, 0]


def test_cancel_stops_stream(pool):
    h = pool.submit("slow long", "tara", max_tokens=7000)
    first = h.get(timeout=30)
    assert first is not None
    h.cancel()
    n = 0
    while h.get(timeout=30) is not None:
        n += 1
    assert n < 999


def test_worker_error_surfaces(pool):
    h = pool.submit("fail now", "tara", max_tokens=14)
    with pytest.raises(RuntimeError, match="boom"):
        list(h.chunks())


def test_stream_generator(pool):
    got = b"".join(pool.stream("xyz", "tara", max_tokens=21))
    assert len(got) == 3 * (128 + 3)


def test_submit_tokens_routes_to_a_worker(pool):
    """/v1/completions on a multi-GPU pool: token streams go through the same dispatch."""
    h = pool.submit_tokens([5, 6, 7], max_tokens=5)
    toks = []
    while True:
        t = h.get(timeout=30)
        if t is None:
            break
        toks.append(t)
    assert toks == [5 + h.worker, 6 + h.worker, 7 + h.worker, 5 + h.worker, 6 + h.worker]


def test_dead_worker_fails_its_streams_and_is_replaced():
    p = GpuPool(2, factory=fake_factory, start_timeout=120, poll_s=0.1)
    try:
        h = p.submit("die soon", "tara", max_tokens=7000)
        assert h.worker == 0
        with pytest.raises(RuntimeError, match="died"):
            while h.get(timeout=60) is not None:
                pass
        assert p.load[0] == 0
        # the other worker still serves; the replacement for worker 0 comes up
        assert b"".join(p.stream("abc", "tara", max_tokens=14))
        deadline = time.time() + 120
        while not p.alive[0] and time.time() < deadline:
            time.sleep(0.1)
        assert p.alive[0]
        g = p.submit("after", "tara", max_tokens=7)
        assert list(g.chunks()) == fake_pcm("after", g.worker, 1)
    finally:
        p.close()


def test_dead_worker_is_reaped_while_another_streams():
    """The outbox never goes quiet while a live worker streams chunks every 20 ms; the dead
    worker's client must still get its error (liveness is checked on a clock)."""
    p = GpuPool(2, factory=fake_factory, start_timeout=120, poll_s=0.5, respawn=False)
    try:
        h = p.submit("die soon", "tara", max_tokens=7000)
        busy = p.submit("slow busy", "tara", max_tokens=70000)   # 10,000 chunks, 20 ms apart
        assert (h.worker, busy.worker) == (0, 1)
        t0 = time.time()
        with pytest.raises(RuntimeError, match="died"):
            while h.get(timeout=60) is not None:
                pass
        assert time.time() - t0 < 15
        assert busy.get(timeout=30) is not None   # the other stream is still live
        busy.cancel()
        while busy.get(timeout=30) is not None:
            pass
    finally:
        p.close()


def test_workers_inherit_the_parents_content_seed(monkeypatch):
    """MORPHEUS_MX_CONTENT_SEED set in-process (as the parity tests do) reaches spawned
    workers, which re-import config from the environment."""
    from project_morpheus_amd import config as C
    monkeypatch.setattr(C, "CONTENT_SEED", 1)
    p = GpuPool(1, factory=fake_factory, start_timeout=120)
    try:
        h = p.submit_tokens([-1], max_tokens=1)
        assert h.get(timeout=30) == 1
    finally:
        p.close()
