"""Generation parameters, voices, prompt framing and long-form helpers.

Mirrors Morpheus_Client/tts_engine/inference.py (same names and semantics):
  * ``MAX_TOKENS/TEMPERATURE/TOP_P`` from ``ORPHEUS_*`` env (:75-90),
    ``update_generation_params`` (:93-102), ``REPETITION_PENALTY = 1.1`` (:105),
    ``SAMPLE_RATE`` (:108);
  * voice lists and ``DEFAULT_VOICE`` (:125-159);
  * ``START_TOKEN_ID`` / ``END_TOKEN_IDS`` (:166-167), ``format_prompt`` string form (:209-223);
  * id form of the prompt, ``OrpheusModel._format_prompt`` (engine_class.py:77-98);
  * ``split_text_into_sentences`` (:249-292), sentence batching
    (remote_backend.py:221-241) and the crossfade of ``stitch_wav_files`` (:294-365).
The hardware banner and audio playback are not on the hot path and are not mirrored.
"""
from __future__ import annotations

import os
import wave
from typing import Iterable, List, Sequence

import numpy as np


def _env(name, default, cast):
    try:
        return cast(os.environ.get(name, default))
    except (TypeError, ValueError):
        return cast(default)


MAX_TOKENS = _env("ORPHEUS_MAX_TOKENS", "8192", int)
TEMPERATURE = _env("ORPHEUS_TEMPERATURE", "0.6", float)
TOP_P = _env("ORPHEUS_TOP_P", "0.9", float)
REPETITION_PENALTY = 1.1
SAMPLE_RATE = _env("ORPHEUS_SAMPLE_RATE", "24000", int)


def update_generation_params(*, temperature=None, top_p=None, max_tokens=None) -> None:
    global TEMPERATURE, TOP_P, MAX_TOKENS
    if temperature is not None:
        TEMPERATURE = float(temperature)
    if top_p is not None:
        TOP_P = float(top_p)
    if max_tokens is not None:
        MAX_TOKENS = int(max_tokens)


VOICES_BY_LANGUAGE = {
    "english": ["tara", "leah", "jess", "leo", "dan", "mia", "zac", "zoe"],
    "french": ["pierre", "amelie", "marie"],
    "german": ["jana", "thomas", "max"],
    "korean": ["유나", "준서"],
    "hindi": ["ऋतिका"],
    "mandarin": ["长乐", "白芷"],
    "spanish": ["javi", "sergio", "maria"],
    "italian": ["pietro", "giulia", "carlo"],
}
AVAILABLE_VOICES = [v for vs in VOICES_BY_LANGUAGE.values() for v in vs]
DEFAULT_VOICE = "tara"
VOICE_TO_LANGUAGE = {v: lang for lang, vs in VOICES_BY_LANGUAGE.items() for v in vs}
AVAILABLE_LANGUAGES = list(VOICES_BY_LANGUAGE)

START_TOKEN_ID = 128259
END_TOKEN_IDS = [128009, 128260, 128261, 128257]


def resolve_voice(voice: str) -> str:
    return voice if voice in AVAILABLE_VOICES else DEFAULT_VOICE


def format_prompt(prompt: str, voice: str = DEFAULT_VOICE) -> str:
    """String framing sent to remote completions servers (inference.py:209-223)."""
    return f"<|audio|>{resolve_voice(voice)}: {prompt}<|eot_id|>"


def prompt_ids(text_ids: Sequence[int]) -> List[int]:
    """Id framing: [start_of_human] + tokenizer('{voice}: {text}') + end tokens."""
    return [START_TOKEN_ID] + list(text_ids) + list(END_TOKEN_IDS)


def split_text_into_sentences(text: str) -> List[str]:
    """Sentence split: a whitespace char after . ! ? ends a sentence unless the char two
    back is '.' or ' ' (abbreviation heuristic); pieces < 20 chars merge forward."""
    pieces: List[str] = []
    cur: List[str] = []
    for ch in text:
        cur.append(ch)
        n = len(cur)
        if ch in " \n\t" and n > 1 and cur[-2] in ".!?" and n > 3 and cur[-3] not in ". ":
            pieces.append("".join(cur).strip())
            cur = []
    tail = "".join(cur)
    if tail.strip():
        pieces.append(tail.strip())
    merged: List[str] = []
    i = 0
    while i < len(pieces):
        s = pieces[i]
        while i < len(pieces) - 1 and len(s) < 20:
            i += 1
            s = s + " " + pieces[i]
        merged.append(s)
        i += 1
    return merged


def batch_sentences(text: str, max_batch_chars: int = 1000, use_batching: bool = True) -> List[str]:
    """Independent prompts for long-form synthesis (remote_backend.py:221-241)."""
    if not (use_batching and len(text) >= max_batch_chars):
        return [text]
    out: List[str] = []
    cur = ""
    for s in split_text_into_sentences(text):
        if cur and len(cur) + len(s) > max_batch_chars:
            out.append(cur)
            cur = s
        else:
            cur = f"{cur} {s}" if cur else s
    if cur:
        out.append(cur)
    return out


def crossfade_join(segments: Iterable[np.ndarray], crossfade_ms: float = 50) -> np.ndarray:
    """int16 segments joined with a linear crossfade (stitch_wav_files' arithmetic)."""
    n = int(SAMPLE_RATE * crossfade_ms / 1000)
    out = None
    for seg in segments:
        seg = np.asarray(seg, dtype=np.int16)
        if out is None:
            out = seg
        elif len(out) >= n and len(seg) >= n:
            mix = (out[-n:] * np.linspace(1.0, 0.0, n) + seg[:n] * np.linspace(0.0, 1.0, n))
            out = np.concatenate([out[:-n], mix.astype(np.int16), seg[n:]])
        else:
            out = np.concatenate([out, seg])
    return out if out is not None else np.zeros(0, dtype=np.int16)


def stitch_wav_files(input_files: Sequence[str], output_file: str, crossfade_ms: float = 50):
    if not input_files:
        return
    params, segs = None, []
    for f in input_files:
        with wave.open(f, "rb") as w:
            params = params or w.getparams()
            segs.append(np.frombuffer(w.readframes(w.getnframes()), dtype=np.int16))
    with wave.open(output_file, "wb") as w:
        w.setparams(params)
        w.writeframes(crossfade_join(segs, crossfade_ms).tobytes())


def list_available_voices() -> List[str]:
    return list(AVAILABLE_VOICES)
