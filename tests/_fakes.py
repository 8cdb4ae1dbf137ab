"""Fake per-GPU services for CPU tests of dispatch / adapters (no HIP device needed)."""
import os
import queue
import threading
import time


class FakeHandle:
    def __init__(self, chunks, delay=0.0, fail=None):
        self._q = queue.Queue()
        self.cancelled = threading.Event()

        def run():
            for c in chunks:
                if self.cancelled.is_set():
                    break
                if delay:
                    time.sleep(delay)
                self._q.put(c)
            if fail and not self.cancelled.is_set():
                self._q.put(RuntimeError(fail))
            self._q.put(None)

        threading.Thread(target=run, daemon=True).start()

    def get(self, timeout=None):
        item = self._q.get(timeout=timeout)
        if isinstance(item, BaseException):
            raise item
        return item

    def cancel(self):
        self.cancelled.set()


def fake_pcm(text, device, n):
    return [bytes([device, i % 256]) * 64 + text.encode() for i in range(n)]


class FakeService:
    def __init__(self, device):
        self.device = device

    def submit(self, text, voice, max_tokens=None, **kw):
        if text.startswith("die"):  # the worker process dies mid-stream (GPU fault, OOM)
            threading.Timer(0.3, lambda: os._exit(3)).start()
            return FakeHandle([b"x"] * 1000, delay=0.01)
        n = max(1, (max_tokens or 70) // 7)
        delay = 0.02 if text.startswith("slow") else 0.0
        fail = "boom" if text.startswith("fail") else None
        return FakeHandle(fake_pcm(text, self.device, n), delay=delay, fail=fail)


    def submit_tokens(self, prompt_ids, max_tokens=None, **kw):
        """Token ids: the prompt ids echoed with the device added, max_tokens of them
        (prompt [-1]: the worker's config.CONTENT_SEED, for the seed-propagation test)."""
        if list(prompt_ids) == [-1]:
            from project_morpheus_amd import config
            return FakeHandle([int(config.CONTENT_SEED)])
        n = max_tokens or 8
        toks = [(int(prompt_ids[i % len(prompt_ids)]) + self.device) for i in range(n)]
        return FakeHandle(toks)


def fake_factory(device):
    return FakeService(device)
