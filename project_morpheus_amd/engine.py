"""Host side of the MI355X path: LLM and SNAC contexts, and the utterance runner.

* ``LlmEngine``   wraps mx_llm_* (replaces vLLM ``AsyncLLMEngine.generate``,
                  engine_class.py:117, and llama.cpp ``Llama``, llama_local.py:42-52).
* ``SnacDecoder`` wraps mx_snac_* (replaces ``SNAC.decode`` + slice + PCM16,
                  speechpipe.py:76-129).
* ``Synthesizer`` is the Orpheus decoder loop (engine_class.py:103-134 +
                  speechpipe.py:191-337) at the token-id level: prefill, hipGraph decode
                  steps kept ``depth`` deep in the GPU queue, the reference's window schedule
                  on the host, SNAC windows on a second HIP stream, PCM read from
                  host-mapped memory.  No per-token string formatting, no per-token sync.
"""
from __future__ import annotations

import ctypes as C
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterator, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .config import ENGINE_OPTIONS, STOP_IDS, OrpheusConfig, rope_tables
from .schedule import WindowScheduler, code_of_id, frames_for_slice

SAMPLES_PER_FRAME = 2048
SLICE_LO, SLICE_HI = 2048, 4096


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return _lib.MX_DTYPE_BF16
    if t.dtype == torch.float32:
        return _lib.MX_DTYPE_F32
    if t.dtype == torch.float8_e4m3fn:
        return _lib.MX_DTYPE_FP8
    raise TypeError(f"unsupported weight dtype {t.dtype}")


class LlmEngine:
    """One mx_llm context on one GPU (weights replicated per GPU)."""

    def __init__(self, cfg: OrpheusConfig, weights: Dict[str, torch.Tensor], device: int = 0,
                 max_slots: int = 4, max_pos: int = 2048, max_batch: int = 1,
                 max_prefill: int = 256, wdtype: str = "bf16"):
        """``wdtype="fp8"``: matrices as e4m3 + per-row ``.scale`` (weights.quantize_fp8)."""
        _lib.require_gpu()
        self.lib = _lib.load()
        self.cfg, self.device = cfg, device
        self.max_slots, self.max_pos, self.max_batch = max_slots, max_pos, max_batch
        self.max_prefill = max_prefill
        c = _lib.LlmConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                           kv_heads=cfg.kv_heads, head_dim=cfg.head_dim, ffn=cfg.ffn,
                           vocab=cfg.vocab, max_slots=max_slots, max_pos=max_pos,
                           max_batch=max_batch, max_prefill=max_prefill, eps=cfg.eps,
                           tied=int(cfg.tied), wdtype=_lib.MX_WEIGHTS[wdtype])
        self.wdtype = wdtype
        h = C.c_void_p()
        torch.cuda.set_device(device)
        rc = self.lib.mx_llm_create(device, C.byref(c), C.byref(h))
        _lib.check(rc, self.lib.mx_llm_last_error, None)
        self.h = h
        dev = torch.device("cuda", device)
        for name, t in weights.items():
            td = t.to(dev).contiguous()
            rc = self.lib.mx_llm_set_weight(h, name.encode(), C.c_void_p(td.data_ptr()),
                                            td.numel(), _dtype_code(td))
            self._check(rc)
            del td
        cos, sin = rope_tables(cfg, max_pos)
        self._check(self.lib.mx_llm_set_rope(h, cos.ctypes.data, sin.ctypes.data, max_pos))
        self._check(self.lib.mx_llm_finalize(h))
        for key, val in ENGINE_OPTIONS.items():   # MORPHEUS_MX_OPT_<key>=<int> overrides
            self.set_option(key, val)
        hp = self.lib.mx_llm_history(h)
        n = (max_slots + 1) * max_pos
        self.hist = np.ctypeslib.as_array(hp, shape=(n,)).reshape(max_slots + 1, max_pos)
        torch.cuda.synchronize(device)

    def _check(self, rc):
        _lib.check(rc, self.lib.mx_llm_last_error, self.h)

    def prefill(self, slot: int, row: int, ids: Sequence[int], penalty: float, stream, *,
                temperature: float = 0.0, top_p: float = 1.0, seed: int = 0) -> None:
        """Prefill ``ids`` into KV ``slot`` bound to decode ``row``; the slot decodes under
        (penalty, temperature, top_p, seed) until the next prefill (temperature 0 = greedy)."""
        arr = np.ascontiguousarray(np.asarray(ids, dtype=np.int32))
        sp = _lib.Sampling(temperature=float(temperature), top_p=float(top_p),
                           repetition_penalty=float(penalty), seed=int(seed) & (2**64 - 1))
        self._check(self.lib.mx_llm_prefill(self.h, slot, row, arr.ctypes.data, len(arr),
                                            C.byref(sp), C.c_void_p(stream.cuda_stream)))

    def decode(self, n_rows: int, stream) -> None:
        """One step for rows [0, n_rows), each under its slot's generation parameters."""
        self._check(self.lib.mx_llm_decode(self.h, n_rows, C.c_void_p(stream.cuda_stream)))

    def check(self, stream) -> None:
        """After waiting for a step: raises if a persistent-engine launch gave up on a
        bounded wait (that step committed nothing; the next decode recomputes it)."""
        self._check(self.lib.mx_llm_check(self.h, C.c_void_p(stream.cuda_stream)))

    PROFILE_CLASSES = ("qkv", "attention", "o_proj", "gate_up", "down", "lm_head", "commit",
                       "engine")

    def decode_profiled(self, n_rows: int, stream) -> Dict[str, float]:
        """One eager step with HIP events around every launch: ms per launch class
        (summed over layers) on the engine's own stream."""
        n = len(self.PROFILE_CLASSES)
        ms = (C.c_double * n)()
        self._check(self.lib.mx_llm_decode_profiled(self.h, n_rows,
                                                    C.c_void_p(stream.cuda_stream), ms, n))
        return {k: ms[i] for i, k in enumerate(self.PROFILE_CLASSES)}

    GEMV_KINDS = {"qkv": 0, "o_proj": 1, "gate_up": 2, "down": 3, "o_proj_merge": 4,
                  "lm_head": 5}

    def bench_gemv(self, which: str, reps: int = 4, n_rows: int = 1):
        """(mean µs per launch, weight bytes per launch) of the ``n_rows``-row decode
        GEMV/GEMM, timed in a hipGraph sweeping all layers (roofline probe; idle context)."""
        us, nb = C.c_float(0.0), C.c_double(0.0)
        self._check(self.lib.mx_llm_bench_gemv(self.h, self.GEMV_KINDS[which], n_rows, reps,
                                               C.byref(us), C.byref(nb)))
        return us.value, nb.value

    def bench_gemv_streams(self, which: str, n_rows: int, nstreams: int, reps: int = 2) -> float:
        """µs per launch of one stream's all-layer sweep with ``nstreams`` concurrent copies
        (include/morpheus_mx.h mx_llm_bench_gemv_streams)."""
        us = C.c_float(0.0)
        self._check(self.lib.mx_llm_bench_gemv_streams(self.h, self.GEMV_KINDS[which], n_rows,
                                                       reps, nstreams, C.byref(us)))
        return us.value

    def bench_gemv_trace(self, which: str, n_rows: int, cap_blocks: int = 2048) -> np.ndarray:
        """Per-block phase stamps [blocks][8] (100 MHz clock) of one multi-row launch of
        ``which`` (include/morpheus_mx.h mx_llm_bench_gemv_trace)."""
        buf = (C.c_uint64 * (cap_blocks * 8))()
        nb = C.c_int(0)
        self._check(self.lib.mx_llm_bench_gemv_trace(self.h, self.GEMV_KINDS[which], n_rows, buf,
                                                     cap_blocks, C.byref(nb)))
        arr = np.frombuffer(buf, dtype=np.uint64, count=nb.value * 8)
        return arr.reshape(nb.value, 8).copy()

    def bench_attention(self, L: int, n_rows: int = 1, cpw: int = 1, debug: int = 0,
                        reps: int = 200) -> float:
        us = C.c_float(0.0)
        self._check(self.lib.mx_llm_bench_attention(self.h, L, n_rows, cpw, debug, reps,
                                                    C.byref(us)))
        return us.value

    def engine_trace(self) -> np.ndarray:
        """Timeline of the last persistent-engine launch (option engine_trace): clock stamps
        (100 MHz) [grid][layers][12], see include/morpheus_mx.h mx_llm_engine_trace."""
        n = 1024 * self.cfg.layers * 12
        buf = (C.c_uint64 * n)()
        grid = C.c_int(0)
        self._check(self.lib.mx_llm_engine_trace(self.h, buf, n, C.byref(grid)))
        arr = np.frombuffer(buf, dtype=np.uint64, count=grid.value * self.cfg.layers * 12)
        return arr.reshape(grid.value, self.cfg.layers, 12).copy()

    def set_option(self, key: str, value: int) -> None:
        self._check(self.lib.mx_llm_set_option(self.h, key.encode(), int(value)))

    def enable_logits(self) -> None:
        """Parity/debug mode: keep the penalised logits of each row (before first decode)."""
        self._check(self.lib.mx_llm_debug_logits(self.h, 1))

    def read_logits(self, row: int, stream) -> np.ndarray:
        out = np.empty(self.cfg.vocab, dtype=np.float32)
        self._check(self.lib.mx_llm_read_logits(self.h, row, out.ctypes.data,
                                                C.c_void_p(stream.cuda_stream)))
        return out

    def row_state(self, row: int):
        """(active, next position) of decode row ``row`` (host view)."""
        a, p = C.c_int(0), C.c_int(0)
        self._check(self.lib.mx_llm_row_state(self.h, row, C.byref(a), C.byref(p)))
        return bool(a.value), p.value

    def release_row(self, row: int, stream) -> None:
        self._check(self.lib.mx_llm_release_row(self.h, row, C.c_void_p(stream.cuda_stream)))

    def move_row(self, dst: int, src: int, stream) -> None:
        """Compaction: row ``src``'s stream continues in parked row ``dst`` (same KV slot)."""
        self._check(self.lib.mx_llm_move_row(self.h, dst, src, C.c_void_p(stream.cuda_stream)))

    def close(self):
        if getattr(self, "h", None):
            self.lib.mx_llm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SnacDecoder:
    """One mx_snac context (fp32 SNAC 24 kHz decoder)."""

    NOISE_PER_FRAME = 3360  # 32 + 256 + 1024 + 2048 samples of NoiseBlock noise per frame

    def __init__(self, weights: Dict[str, torch.Tensor], device: int = 0, max_frames: int = 7,
                 max_batch: int = 1):
        _lib.require_gpu()
        self.lib = _lib.load()
        self.device, self.max_frames, self.max_batch = device, max_frames, max_batch
        h = C.c_void_p()
        torch.cuda.set_device(device)
        _lib.check(self.lib.mx_snac_create(device, max_frames, max_batch, C.byref(h)),
                   self.lib.mx_snac_last_error, None)
        self.h = h
        dev = torch.device("cuda", device)
        for name, t in weights.items():
            td = t.to(dev).contiguous()
            self._check(self.lib.mx_snac_set_weight(h, name.encode(), C.c_void_p(td.data_ptr()),
                                                    td.numel(), _dtype_code(td)))
        self._check(self.lib.mx_snac_finalize(h))
        torch.cuda.synchronize(device)

    def _check(self, rc):
        _lib.check(rc, self.lib.mx_snac_last_error, self.h)

    def decode_ptr(self, frames_ptr: int, n_frames: int, batch: int, noise_ptr: int, seed: int,
                   pcm_ptr: int, audio_ptr: int, lo: int, hi: int, stream,
                   seeds_ptr: int = 0) -> None:
        """seeds_ptr: device-accessible uint64 [batch] noise seed per window (0: ``seed``)."""
        self._check(self.lib.mx_snac_decode(self.h, C.c_void_p(frames_ptr), n_frames, batch,
                                            C.c_void_p(noise_ptr), seed, C.c_void_p(seeds_ptr),
                                            C.c_void_p(pcm_ptr), C.c_void_p(audio_ptr), lo, hi,
                                            C.c_void_p(stream.cuda_stream)))

    def decode(self, codes: torch.Tensor, noise: Optional[torch.Tensor] = None, seed: int = 0,
               lo: int = SLICE_LO, hi: int = SLICE_HI, want_audio: bool = False, stream=None):
        """codes [B, 7N] int32 (device) -> (pcm int16 [B, hi'-lo'], audio fp32 [B, 2048N]|None)."""
        stream = stream or torch.cuda.current_stream(self.device)
        codes = codes.to(torch.int32).contiguous()
        B, n7 = codes.shape
        n = n7 // 7
        hi_c = min(hi, SAMPLES_PER_FRAME * n)
        lo_c = min(lo, hi_c)
        pcm = torch.empty(B, hi_c - lo_c, dtype=torch.int16, device=codes.device)
        audio = torch.empty(B, SAMPLES_PER_FRAME * n, dtype=torch.float32,
                            device=codes.device) if want_audio else None
        if noise is not None:
            noise = noise.to(torch.float32).contiguous()
            assert noise.shape == (B, self.NOISE_PER_FRAME * n)
        self.decode_ptr(codes.data_ptr(), n, B, noise.data_ptr() if noise is not None else 0,
                        seed, pcm.data_ptr() if pcm.numel() else 0,
                        audio.data_ptr() if audio is not None else 0, lo_c, hi_c, stream)
        return pcm, audio

    def close(self):
        if getattr(self, "h", None):
            self.lib.mx_snac_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class UtteranceStats:
    tokens: int = 0
    windows: int = 0
    samples: int = 0
    t_start: float = 0.0
    t_first_audio: Optional[float] = None
    t_end: float = 0.0
    token_ids: List[int] = field(default_factory=list)

    @property
    def audio_seconds(self) -> float:
        return self.samples / 24000.0

    @property
    def first_audio_ms(self) -> Optional[float]:
        return None if self.t_first_audio is None else 1e3 * (self.t_first_audio - self.t_start)


class _WindowRing:
    """Host-mapped staging for SNAC windows: codes in, PCM16 out, zero-copy."""

    def __init__(self, n: int = 32, max_frames: int = 7):
        self.n = n
        self.codes_bytes = 7 * max_frames * 4
        self.buf = _lib.HostBuffer(n * (self.codes_bytes + 4096))
        self.codes = [self.buf.view(np.int32, 7 * max_frames, i * self.codes_bytes)
                      for i in range(n)]
        base = n * self.codes_bytes
        self.pcm = [self.buf.view(np.int16, 2048, base + i * 4096) for i in range(n)]
        self.codes_dev = [self.buf.dev_ptr(i * self.codes_bytes) for i in range(n)]
        self.pcm_dev = [self.buf.dev_ptr(base + i * 4096) for i in range(n)]


class Synthesizer:
    """The per-GPU decoder loop.  ``run`` yields PCM16 bytes chunks in order."""

    def __init__(self, llm: LlmEngine, snac: SnacDecoder, depth: int = 3, seed: int = 0):
        self.llm, self.snac = llm, snac
        self.depth = depth
        self.stream = torch.cuda.Stream(llm.device)
        self.snac_stream = torch.cuda.Stream(llm.device)
        self.ring = _WindowRing(32, snac.max_frames)
        self.seed = seed
        self._windows = 0

    def run(self, prompt_ids: Sequence[int], max_tokens: int, penalty: float = 1.1,
            stop_ids: Sequence[int] = STOP_IDS, inject_ids: Optional[Sequence[int]] = None,
            stats: Optional[UtteranceStats] = None, slot: int = 0, row: int = 0,
            temperature: float = 0.0, top_p: float = 1.0, seed: int = 0,
            noise_seed: Optional[int] = None) -> Iterator[bytes]:
        """Prefill, then decode up to ``max_tokens`` tokens (engine_class.py:103-134), greedy
        unless ``temperature`` > 0.  Window j's SNAC noise is drawn from (noise_seed, j).

        ``inject_ids`` (bench / synthetic weights): token ids fed to the SNAC
        schedule in place of the model's own tokens; the LLM still decodes every step.
        """
        st = stats if stats is not None else UtteranceStats()
        st.t_start = time.perf_counter()
        llm, n0 = self.llm, len(prompt_ids)
        max_tokens = min(max_tokens, llm.max_pos - n0)
        sched = WindowScheduler()
        pending: deque = deque()   # (ring index, event, n_frames, nbytes)
        inflight: deque = deque()  # (token index, event)
        stop = set(int(s) for s in stop_ids)

        llm.prefill(slot, row, prompt_ids, penalty, self.stream, temperature=temperature,
                    top_p=top_p, seed=seed)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        inflight.append((0, ev))
        launched, done, stopped = 1, 0, False
        nseed = self.seed if noise_seed is None else noise_seed
        widx = [0]  # windows of this utterance (noise stream index)

        def launch_window(win: List[int]):
            i = self._windows % self.ring.n
            if len(pending) >= self.ring.n:
                yield from drain(block=True, upto=1)
            lo, hi = SLICE_LO, min(SLICE_HI, SAMPLES_PER_FRAME * (len(win) // 7))
            nf = frames_for_slice(len(win) // 7, hi)  # the frames the kept slice depends on
            self.ring.codes[i][: 7 * nf] = win[: 7 * nf]
            self.snac.decode_ptr(self.ring.codes_dev[i], nf, 1, 0,
                                 (nseed * 1000003 + widx[0]) & 0xFFFFFFFFFFFF,
                                 self.ring.pcm_dev[i], 0, lo, max(lo, hi), self.snac_stream)
            e = torch.cuda.Event()
            e.record(self.snac_stream)
            pending.append((i, e, max(0, hi - lo) * 2))
            self._windows += 1
            widx[0] += 1
            st.windows += 1

        def drain(block: bool, upto: Optional[int] = None):
            k = 0
            while pending and (upto is None or k < upto):
                i, e, nbytes = pending[0]
                if not block and not e.query():
                    return
                e.synchronize()
                pending.popleft()
                k += 1
                if nbytes:
                    data = self.ring.pcm[i][: nbytes // 2].tobytes()
                    st.samples += nbytes // 2
                    if st.t_first_audio is None:
                        st.t_first_audio = time.perf_counter()
                    yield data

        try:
            while done < max_tokens:
                while (not stopped and launched < max_tokens and launched - done < self.depth):
                    llm.decode(1, self.stream)
                    e = torch.cuda.Event()
                    e.record(self.stream)
                    inflight.append((launched, e))
                    launched += 1
                k, e = inflight.popleft()
                e.synchronize()
                llm.check(self.stream)
                tok = int(llm.hist[slot, n0 + k])
                done += 1
                st.tokens += 1
                st.token_ids.append(tok)
                feed = int(inject_ids[k]) if inject_ids is not None else tok
                for win in sched.push(code_of_id(feed, sched.count)):
                    yield from launch_window(win)
                yield from drain(block=False)
                if tok in stop:
                    stopped = True
                    break
            for win in sched.flush():
                yield from launch_window(win)
            yield from drain(block=True)
        finally:
            # normal end, error or the consumer closing the generator (barge-in): wait for
            # the speculative steps and the SNAC calls still queued (their results are
            # dropped), then give the row back -- the slot is free for the next utterance
            for _, e in inflight:
                e.synchronize()
            for _, e, _ in pending:
                e.synchronize()
            pending.clear()
            llm.release_row(row, self.stream)
            self.stream.synchronize()
            st.t_end = time.perf_counter()
