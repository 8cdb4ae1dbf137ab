"""Model shapes, RoPE tables and environment knobs for the MI355X Orpheus path.

Orpheus-3B is Llama-3.2-3B (Orpheus-TTS/pretrain/config.yaml:2) with 28,683 added
``<custom_token_i>`` ids (Orpheus-TTS/pretrain/train.py:173-176): vocab 156,940.  A real
checkpoint's ``config.json`` overrides these defaults (``OrpheusConfig.from_hf``).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field
from typing import Optional

import numpy as np

# Token-id map: <custom_token_n> = 128256 + n; audio code for phase k is
# id - 128266 - 4096 k (speechpipe.py:181).  Specials: inference.py:166-167,
# realtime_streaming_example/main.py:43.
CUSTOM_TOKEN_BASE = 128256
AUDIO_CODE_BASE = CUSTOM_TOKEN_BASE + 10
START_OF_HUMAN = 128259
END_OF_TEXT = 128009
END_OF_HUMAN = 128260
START_OF_AI = 128261
START_OF_SPEECH = 128257
END_OF_SPEECH = 128258
BOS = 128000
STOP_IDS = (END_OF_SPEECH,)


@dataclass
class OrpheusConfig:
    hidden: int = 3072
    layers: int = 28
    heads: int = 24
    kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 8192
    vocab: int = 156940
    eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = field(default_factory=lambda: {
        "rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
        "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    tied: bool = True

    @classmethod
    def from_hf(cls, path: str) -> "OrpheusConfig":
        with open(os.path.join(path, "config.json") if os.path.isdir(path) else path) as fh:
            j = json.load(fh)
        heads = j["num_attention_heads"]
        return cls(hidden=j["hidden_size"], layers=j["num_hidden_layers"], heads=heads,
                   kv_heads=j.get("num_key_value_heads", heads),
                   head_dim=j.get("head_dim") or j["hidden_size"] // heads,
                   ffn=j["intermediate_size"], vocab=j["vocab_size"],
                   eps=j.get("rms_norm_eps", 1e-5), rope_theta=j.get("rope_theta", 10000.0),
                   rope_scaling=j.get("rope_scaling"),
                   tied=bool(j.get("tie_word_embeddings", False)))

    def params(self) -> int:
        per = (self.heads + 2 * self.kv_heads) * self.head_dim * self.hidden \
            + self.hidden * self.heads * self.head_dim + 3 * self.hidden * self.ffn
        return self.layers * per + self.vocab * self.hidden * (1 if self.tied else 2)

    def step_weight_bytes(self) -> int:
        """Bytes of bf16 weights streamed by one decode step (tied lm_head counted once)."""
        per = (self.heads + 2 * self.kv_heads) * self.head_dim * self.hidden \
            + self.hidden * self.heads * self.head_dim + 3 * self.hidden * self.ffn
        return 2 * (self.layers * per + self.vocab * self.hidden)

    def kv_bytes_per_position(self) -> int:
        return self.layers * 2 * self.kv_heads * self.head_dim * 2

    def to_dict(self):
        return asdict(self)


def rope_inv_freq(cfg: OrpheusConfig) -> np.ndarray:
    """llama3-scaled RoPE frequencies (float64)."""
    d = cfg.head_dim
    inv = 1.0 / cfg.rope_theta ** (np.arange(0, d, 2, dtype=np.float64) / d)
    rs = cfg.rope_scaling or {}
    if rs.get("rope_type", rs.get("type")) != "llama3":
        return inv
    f, lo, hi = rs["factor"], rs["low_freq_factor"], rs["high_freq_factor"]
    ctx = rs["original_max_position_embeddings"]
    wavelen = 2.0 * math.pi / inv
    out = np.where(wavelen > ctx / lo, inv / f, inv)
    t = (ctx / wavelen - lo) / (hi - lo)
    mid = (wavelen >= ctx / hi) & (wavelen <= ctx / lo)
    return np.where(mid, (1.0 - t) * out / f + t * out, out)


def rope_tables(cfg: OrpheusConfig, n_pos: int):
    """cos/sin [n_pos][head_dim/2] fp32; angles formed in float64."""
    ang = np.arange(n_pos, dtype=np.float64)[:, None] * rope_inv_freq(cfg)[None, :]
    return (np.ascontiguousarray(np.cos(ang).astype(np.float32)),
            np.ascontiguousarray(np.sin(ang).astype(np.float32)))


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except (TypeError, ValueError):
        return default


# Environment knobs, same style as the reference's ORPHEUS_* / LLAMA_* (SURVEY.md §5).
MX_WEIGHTS = os.environ.get("MORPHEUS_MX_WEIGHTS")      # HF dir (config.json + safetensors)
MX_SNAC = os.environ.get("MORPHEUS_MX_SNAC", os.environ.get("ORPHEUS_SNAC_PATH"))
MX_TOKENIZER = os.environ.get("MORPHEUS_MX_TOKENIZER")  # dir with tokenizer.json
MX_DEVICE = env_int("MORPHEUS_MX_DEVICE", 0)
MX_MAX_POS = env_int("MORPHEUS_MX_MAX_POS", env_int("LLAMA_N_CTX", 8192))
MX_MAX_SLOTS = env_int("MORPHEUS_MX_MAX_SLOTS", 8)
MX_GPUS = env_int("MORPHEUS_MX_GPUS", 1)                # worker processes (one per GPU)
# batched SNAC window coalescing (batching.BatchSynthesizer): launch when this many windows
# are due, or when the oldest has waited SNAC_MAX_HOLD decode steps (12 / 2 measured in round 2:
# configs[2] 96.8 -> 99.2x, p50 first audio +1.4 ms; profiles/r02_bench_snac_coalescing.log;
# 16 / 3 since round 6's receptive-field cut: the configs[2] loop 3.253 -> 3.241 s,
# profiles/r06_snac_coalescing_sweep.log)
# decode steps the batcher keeps queued ahead of the host (batching.BatchSynthesizer)
BATCH_DEPTH = env_int("MORPHEUS_MX_BATCH_DEPTH", 2)
SNAC_MIN_BATCH = env_int("MORPHEUS_MX_SNAC_MIN_BATCH", 16)
SNAC_MAX_HOLD = env_int("MORPHEUS_MX_SNAC_MAX_HOLD", 3)
# Random streams of a request given no seed (sampling + SNAC noise): 0 (default) draws a fresh
# 64-bit seed per request, as vLLM SamplingParams(seed=None) and llama.cpp's default do, so
# "regenerate" gives new audio; 1 derives it from the prompt ids (reproducible bench / parity
# runs: the same text gives the same audio whatever the batch company or arrival order).
CONTENT_SEED = env_int("MORPHEUS_MX_CONTENT_SEED", 0)
# mx_llm_set_option knobs applied to every LlmEngine at creation: MORPHEUS_MX_OPT_<key>=<int>
# (A/B runs and parity sweeps of a non-default kernel choice, e.g. MORPHEUS_MX_OPT_head_b1=0).
ENGINE_OPTIONS = {k[len("MORPHEUS_MX_OPT_"):]: int(v) for k, v in os.environ.items()
                  if k.startswith("MORPHEUS_MX_OPT_")}
# Unit of MxTTSAdapter.pull(n): "bytes" (default; the reference adapters slice bytes,
# llama_local.py:131-150, pinned by tests/test_tts_adapter_chunking.py) or "ms" (what the
# adapter descriptor declares, adapter_registry.py:54: n milliseconds of PCM = 48 n bytes).
PULL_UNIT = os.environ.get("MORPHEUS_MX_PULL_UNIT", "bytes")


def request_seed(prompt_ids, seed=None) -> int:
    """The seed of one request: ``seed`` if given, else content-derived (CONTENT_SEED=1) or a
    fresh random 64-bit value."""
    if seed is not None:
        return int(seed)
    if CONTENT_SEED:
        import zlib
        return zlib.crc32(np.asarray(prompt_ids, dtype=np.int32).tobytes())
    import secrets
    return secrets.randbits(64)


def synthetic_audio_ids(n: int, seed: int):
    """Seeded audio-token stream for synthetic weights: random weights never
    speak, so the SNAC schedule consumes uniform codes in [1, 4095] per phase instead."""
    rng = np.random.default_rng(seed)
    codes = rng.integers(1, 4096, size=n)
    return [int(AUDIO_CODE_BASE + 4096 * (i % 7) + c) for i, c in enumerate(codes)]
