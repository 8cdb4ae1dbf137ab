"""Deterministic PCM source for the server golden (tests/golden/make_server_golden.py) and its
test (tests/test_server_golden.py): ``MxTTSAdapter`` unchanged, its synthesis source replaced
by seeded PCM chunks whose sizes mimic the engine's SNAC windows (a first 0-byte window,
4096-byte windows, a short flush window)."""
import numpy as np

from project_morpheus_amd.adapter import MxTTSAdapter

CALLS = []


def pcm_for(prompt: str):
    rng = np.random.default_rng(len(prompt))
    return [rng.integers(-3000, 3000, size=n).astype(np.int16).tobytes()
            for n in (0, 2048, 2048, 1000, 2048, 37)]


class GoldenAdapter(MxTTSAdapter):
    @staticmethod
    def source(prompt, voice, use_batching, max_batch_chars, cancel):
        CALLS.append((prompt, voice, use_batching, max_batch_chars))
        yield from pcm_for(prompt)
