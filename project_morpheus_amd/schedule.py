"""Host logic of speechpipe: token -> SNAC code, and the sliding-window schedule.

Reproduces Morpheus_Client/tts_engine/speechpipe.py byte for byte (pinned by
tests/golden/speechpipe_golden.json, generated from the reference module):

* ``parse_token_text`` = ``turn_token_into_id`` (speechpipe.py:146-189), string form;
* ``code_of_id``       = the same at the token-id level (no string round trip);
* ``WindowScheduler``  = ``tokens_decoder``'s window choice (speechpipe.py:191-293):
  first window ``buffer[-7:]`` retried every accepted token until one passes the range
  check; then at every 7th accepted token ``buffer[-49:]`` (len >= 49) or ``buffer[-28:]``
  (len >= 28); at end of stream the last 49 / last 28 / last-token padding to 28.
  Codes <= 0 are not accepted (``token > 0``, :215) and so shift the 7-phase.
* ``window_valid``     = the range check of ``convert_to_audio`` (:108-111): codes in
  [0, 4096] (4096 passes the check although the codebook has 4096 rows).
* ``frames_for_slice`` = how many of a window's frames the kept PCM slice depends on.
"""
from __future__ import annotations

from typing import List, Optional

from .config import CUSTOM_TOKEN_BASE

_PREFIX = "<custom_token_"
_PLEN = len(_PREFIX)


def parse_token_text(text: str, index: int) -> Optional[int]:
    if _PREFIX not in text:
        return None
    text = text.strip()
    start = text.rfind(_PREFIX)
    if start < 0:
        return None
    tail = text[start:]
    if not tail.endswith(">"):
        return None
    try:
        n = int(tail[_PLEN:-1])
    except (ValueError, IndexError):
        return None
    return n - 10 - 4096 * (index % 7)


def code_of_id(token_id: int, index: int) -> Optional[int]:
    """Token id -> SNAC code for accepted-token index ``index`` (None: not a custom token)."""
    if token_id < CUSTOM_TOKEN_BASE:
        return None
    return token_id - CUSTOM_TOKEN_BASE - 10 - 4096 * (index % 7)


def window_valid(win: List[int]) -> bool:
    n = (len(win) // 7) * 7
    if n == 0:
        return False
    for v in win[:n]:
        if v < 0 or v > 4096:
            return False
    return True


# SNAC's receptive field reaches fewer than RIGHT_CONTEXT_FRAMES frames (3 x 2,048 samples)
# past the end of an output span: in the 24 kHz decoder the input depthwise conv (k7 over 4
# latent steps per frame), the four polyphase ConvTransposes and their dilated (1, 3, 9) k7
# residual units add up to less than that.  Measured on the oracle (tests/test_oracle_snac.py):
# perturbing frames 5 and 6 of a 7-frame window leaves samples [2048, 4096) bit-identical, and
# decoding frames 0-4 alone (NoiseBlock noise keyed by position, so shared) gives them within
# 5e-6 (fp32 summation order of the shorter convolutions).
SAMPLES_PER_FRAME = 2048
RIGHT_CONTEXT_FRAMES = 3


def frames_for_slice(n_frames: int, hi: int) -> int:
    """Frames of an ``n_frames`` window that samples [.., hi) depend on: the 49-code window
    speechpipe keeps [2048, 4096) of is decoded as its first 5 frames (2/7 less SNAC work)."""
    return min(n_frames, -(-hi // SAMPLES_PER_FRAME) + RIGHT_CONTEXT_FRAMES)


def deinterleave(win: List[int]):
    """speechpipe.py:84-98: per frame t0 -> c0; t1,t4 -> c1; t2,t3,t5,t6 -> c2."""
    nf = len(win) // 7
    c0 = [win[7 * f] for f in range(nf)]
    c1 = [win[7 * f + j] for f in range(nf) for j in (1, 4)]
    c2 = [win[7 * f + j] for f in range(nf) for j in (2, 3, 5, 6)]
    return c0, c1, c2


class WindowScheduler:
    FIRST = 7
    MIN = 28
    IDEAL = 49
    EVERY = 7

    def __init__(self):
        self.buffer: List[int] = []
        self.count = 0
        self.first_done = False

    def push(self, code: Optional[int]) -> List[List[int]]:
        """Accept one parsed code; return the (valid) windows to decode now."""
        if code is None or code <= 0:
            return []
        self.buffer.append(code)
        self.count += 1
        if not self.first_done:
            if self.count >= self.FIRST:
                win = self.buffer[-self.FIRST:]
                if window_valid(win):
                    self.first_done = True
                    return [win]
            return []
        if self.count % self.EVERY:
            return []
        if len(self.buffer) >= self.IDEAL:
            win = self.buffer[-self.IDEAL:]
        elif len(self.buffer) >= self.MIN:
            win = self.buffer[-self.MIN:]
        else:
            return []
        return [win] if window_valid(win) else []

    def flush(self) -> List[List[int]]:
        b = self.buffer
        if len(b) >= self.IDEAL:
            win = b[-self.IDEAL:]
        elif len(b) >= self.MIN:
            win = b[-self.MIN:]
        elif len(b) >= self.EVERY:
            win = b + [b[-1]] * (self.MIN - len(b))
        else:
            return []
        return [win] if window_valid(win) else []
