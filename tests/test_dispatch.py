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
