"""Headline benchmark: Orpheus-3B bf16 TTS, audio-sec / wall-sec (RTF) + p50 first audio.

Workload (BASELINE.json configs[1]): one utterance per step per GPU — a "Hello world"-sized
prompt (voice-framed, synthetic tokenizer), prefill, 1200 greedy decode steps
(engine_class.py:103 max_tokens) with repetition penalty 1.1 on hipGraph-captured steps,
the reference window schedule, and SNAC 24 kHz windows on a second HIP stream.  Weights are
seeded synthetic Orpheus-3B shapes (no checkpoints offline); since random weights never
speak, the SNAC schedule consumes a seeded synthetic audio-token stream injected at the id
level while the LLM still decodes every step.  Multi-GPU: one process per
GPU, independent utterances per rank (batch-sharded streams, no data-path collective),
max-over-ranks time, ``scaling: weak``.

    python bench.py [--gpus N --steps K --warmup W]

``--gpus N`` without a launcher (no ``WORLD_SIZE`` in the environment) starts the N rank
processes itself, one per GPU, before anything touches a GPU (``launch_ranks``); under
``torch.distributed.run`` each rank checks that the world it joined has N ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "audio-sec/wall-sec (RTF) + p50 first-chunk latency, Orpheus-3B bf16"
PEAK_HBM_GBS = 8000.0
MAX_TOKENS = 1200


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--max-tokens", type=int, default=MAX_TOKENS)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-steps", type=int, default=24)
    p.add_argument("--batch", type=int, default=32,
                   help="configs[2]: concurrent streams per GPU (0 skips it)")
    p.add_argument("--fp8-batch", type=int, default=8,
                   help="configs[4]: fp8 streams per GPU (0 skips the fp8 section)")
    p.add_argument("--no-http", action="store_true", help="skip the HTTP-level line")
    p.add_argument("--compaction-ab", action="store_true",
                   help="also run configs[2] without decode-row compaction (A/B record)")
    p.add_argument("--long-read-docs", type=int, default=16,
                   help="configs[3]: long_read documents (0 skips it)")
    p.add_argument("--step-pos", type=int, default=600,
                   help="position at which the bare decode-step time is measured")
    p.add_argument("--share-of", type=str, default="2,4,8",
                   help="N = 1: also time configs[3]'s largest per-rank share of an N-GPU "
                        "run on this GPU, for each N of the comma list ('0' skips it)")
    p.add_argument("--dry-run", action="store_true",
                   help="rank plumbing only: gloo process group, barrier, rank count; no GPU")
    return p.parse_args()


def launch_ranks(n: int) -> int:
    """``--gpus N`` with no launcher: start N copies of this script as rank processes (RANK /
    LOCAL_RANK = GPU index, WORLD_SIZE = N, rendezvous on 127.0.0.1), wait for all of them and
    return the worst exit code.  The parent never initialises a GPU (it starts children, it
    does not exec), and only rank 0 prints the result line."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [None] * n
    try:
        while any(rc is None for rc in rcs):
            for i, pr in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = pr.poll()
            if any(rc not in (None, 0) for rc in rcs):  # one rank failed: stop the others
                for i, pr in enumerate(procs):
                    if rcs[i] is None:
                        pr.send_signal(signal.SIGTERM)
                for i, pr in enumerate(procs):
                    if rcs[i] is None:
                        try:
                            rcs[i] = pr.wait(timeout=30)
                        except subprocess.TimeoutExpired:
                            pr.kill()
                            rcs[i] = pr.wait()
                break
            time.sleep(0.2)
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    bad = [rc for rc in rcs if rc]
    return max(bad, key=abs) if bad else 0


def dry_run(args, rank: int, world: int) -> None:
    """The rank plumbing of a multi-GPU run without the GPU: join a gloo group, barrier, sum
    one per rank; rank 0 prints the count beside ``n_gpus``."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
    else:
        seen = 1
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": seen,
                          "gpus_flag": args.gpus}), flush=True)
    if world > 1:
        dist.destroy_process_group()


PMC_RECORD = next((f for f in ("r06_pmc_gemv.json", "r04_pmc_gemv.json", "r03_pmc_gemv.json",
                               "r02_pmc_gemv.json")
                   if os.path.exists(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                  "profiles", f))), "r02_pmc_gemv.json")


def pmc_traffic(kind, record=PMC_RECORD):
    """HBM bytes per launch of kernel ``kind`` measured by PMC counters in separate rocprofv3
    passes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; scripts/pmc_gemv.py and
    scripts/gpu_pmc_b1.sh, summarised under profiles/); None when that record is absent."""
    path = os.path.join(ROOT, "profiles", record)
    try:
        with open(path) as fh:
            return json.load(fh)["kernels"][kind]["traffic_bytes"]
    except (OSError, KeyError, ValueError):
        return None


# the dominant kernel as rocprofv3 names it (so the line joins the committed kernel-trace
# summaries under profiles/ mechanically)
ROOFLINE_KERNEL = "gemv1_kernel<6, 2, 2, true, 4, false, 0>"


def rocprof_fields(nbytes):
    """The same kernel's frac from the committed rocprofv3 average (kernel time only)."""
    us, path = rocprof_avg_us()
    if us is None:
        return {}
    return {"rocprof_avg_us": round(us, 3), "rocprof_frac": round(nbytes / (us * 1e3) / PEAK_HBM_GBS, 4),
            "rocprof_source": path}


def rocprof_avg_us(kernel=ROOFLINE_KERNEL):
    """(average launch duration in us, file) of ``kernel`` in the newest committed rocprofv3
    --kernel-trace --stats summary of a whole bench run (profiles/r*_bench_kernel_stats*.csv)."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_bench_kernel_stats*.csv")),
                   key=lambda f: (os.path.basename(f)[:3], "final" in os.path.basename(f),
                                  os.path.basename(f)))
    for path in reversed(files):
        try:
            with open(path) as fh:
                for r in csv.DictReader(fh):
                    if f"mx::{kernel}(" in r.get("Name", ""):
                        return float(r["AverageNs"]) / 1e3, os.path.relpath(path, ROOT)
        except (OSError, KeyError, ValueError):
            continue
    return None, None


from project_morpheus_amd.config import synthetic_audio_ids  # noqa: E402


def cpu_baseline(cfg, prompt, positions=(120, 360, 600, 840, 1080), per_pos=4):
    """Oracle (torch fp32, one thread per physical host core) on a bounded sample of the same
    workload (~15-30 s of CPU work): prefill of the same prompt, ``per_pos`` decode steps of
    the full 28-layer model at each of ``positions`` (spread over the utterance's 10..1210
    context range, so the attention cost is averaged the way the utterance sees it), and four
    7-frame SNAC windows; extrapolated to RTF for the 1200-token utterance."""
    import psutil
    import torch

    physical = psutil.cpu_count(logical=False) or os.cpu_count() or 1
    # the GPU box grants this job a CPU share (OMP_NUM_THREADS), not the whole host
    cores = min(physical, int(os.environ.get("OMP_NUM_THREADS") or physical))
    torch.set_num_threads(cores)

    from oracle import llama_ref as L
    from oracle import snac_ref
    from project_morpheus_amd.weights import llm_shapes, synthetic_snac_weights

    rc = L.RefConfig(hidden=cfg.hidden, layers=cfg.layers, heads=cfg.heads,
                     kv_heads=cfg.kv_heads, ffn=cfg.ffn, vocab=cfg.vocab)
    # values do not change fp32 CPU matmul speed: fill fast instead of sampling 3.3 G normals
    w = {k: torch.full(s, 0.01, dtype=torch.float32) for k, s in llm_shapes(cfg).items()}
    ref = L.LlamaRef(rc, w, max_pos=max(positions) + per_pos + 8)
    t0 = time.perf_counter()
    ref.forward(prompt, [0] * len(prompt), list(range(len(prompt))), last_only=True)
    t_prefill = time.perf_counter() - t0
    n_decode = len(positions) * per_pos
    t0 = time.perf_counter()
    for p in positions:
        for i in range(per_pos):
            ref.forward([5], [0], [p + i])
    t_tok = (time.perf_counter() - t0) / n_decode
    sw = synthetic_snac_weights()
    codes = [[1] * 7, [2] * 14, [3] * 28]
    t0 = time.perf_counter()
    for _ in range(4):
        snac_ref.decode(sw, *codes)
    t_win = (time.perf_counter() - t0) / 4
    from project_morpheus_amd.schedule import WindowScheduler
    n = MAX_TOKENS
    ws = WindowScheduler()
    windows = sum(len(ws.push(1 + i % 4000)) for i in range(n)) + len(ws.flush())
    wall = t_prefill + n * t_tok + windows * t_win
    audio = (windows - 1) * 2048 / 24000.0  # the first 1-frame window emits nothing
    return {"value": round(audio / wall, 5), "unit": "audio-sec/wall-sec",
            "cores": torch.get_num_threads(), "kind": "port",
            "sample": (f"oracle/llama_ref fp32 Orpheus-3B on {cores} threads (host: {physical} "
                       f"physical / {os.cpu_count()} logical cores): prefill {len(prompt)} ids "
                       f"({t_prefill:.2f}s) + {n_decode} decode steps ({per_pos} at each of "
                       f"positions {list(positions)}; {t_tok*1e3:.0f} ms/step) "
                       f"+ 4 SNAC 7-frame windows ({t_win*1e3:.0f} ms each), extrapolated to "
                       f"{n} tokens / {windows} windows"),
            "tok_per_s": round(1.0 / t_tok, 3)}


def run_batched(args, llm, snac, prompt, rank, world, dist, n_streams=None, label=None,
                compact=True):
    """configs[2]: ``n_streams`` (default ``args.batch``) utterances per GPU arriving with
    exponential gaps (mean 10 ms, seed 4), synthetic prompts of 16-64 ids, ``max_tokens``
    each, served by the continuous-batching loop; aggregate RTF = all audio / wall time
    (max over ranks)."""
    n_streams = n_streams or args.batch
    import numpy as np
    import torch

    from project_morpheus_amd import inference as I
    from project_morpheus_amd.batching import BatchSynthesizer, StreamRequest
    syn = BatchSynthesizer(llm, snac, seed=rank, compact=compact)
    rng = np.random.default_rng(4 + 1000 * rank)

    def requests():
        t, out = 0.0, []
        for i in range(n_streams):
            n = int(rng.integers(16, 65))
            ids = I.prompt_ids([int(x) for x in rng.integers(1000, 120000, n - 5)])
            out.append(StreamRequest(prompt_ids=ids, max_tokens=args.max_tokens, arrival=t,
                                     inject_ids=synthetic_audio_ids(args.max_tokens,
                                                                    seed=10 + i + 1000 * rank),
                                     stop_ids=()))
            t += float(rng.exponential(0.010))
        return out

    syn.run(requests())  # warmup (captures the per-row-count graphs)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    reqs = requests()
    syn.row_steps.clear()
    wall = syn.run(reqs)
    steps = sum(syn.row_steps.values())
    row_steps = sum(k * v for k, v in syn.row_steps.items())
    torch.cuda.synchronize()
    audio = sum(r.audio_seconds for r in reqs)
    firsts = [r.first_audio_ms for r in reqs]
    if world > 1:
        t = torch.tensor([wall], device="cuda")
        a = torch.tensor([audio], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
        wall, audio = float(t.item()), float(a.item())
        fl = [None] * world
        dist.all_gather_object(fl, firsts)
        firsts = [x for r in fl for x in r]
    return {"workload": label or (f"configs[2]: {n_streams} concurrent utterances per GPU, "
                                  "continuous batching, batched SNAC, exp arrivals mean 10 ms "
                                  "(seed 4)"),
            "streams": n_streams * world, "value": round(audio / wall, 3),
            "unit": "audio-sec/wall-sec", "wall_s": round(wall, 3),
            "audio_seconds": round(audio, 2),
            "p50_first_audio_ms": round(statistics.median(firsts), 2),
            "tok_per_s": round(n_streams * world * args.max_tokens / wall, 1),
            "decode_steps": steps, "mean_rows_per_step": round(row_steps / max(1, steps), 2)}


async def _asgi_speech(app, text: str):
    """One ``POST /v1/audio/speech`` through an ASGI app (no sockets): (t0, [(t, nbytes)])."""
    import asyncio
    import json as _json
    body = _json.dumps({"input": text, "voice": "tara"}).encode()
    sent = {"done": False}
    marks = []

    async def receive():
        if not sent["done"]:
            sent["done"] = True
            return {"type": "http.request", "body": body, "more_body": False}
        await asyncio.sleep(3600)
        return {"type": "http.disconnect"}

    async def send(msg):
        if msg["type"] == "http.response.body":
            marks.append((time.perf_counter(), len(msg.get("body", b""))))

    scope = {"type": "http", "asgi": {"version": "3.0"}, "http_version": "1.1",
             "method": "POST", "scheme": "http", "path": "/v1/audio/speech",
             "raw_path": b"/v1/audio/speech", "query_string": b"", "root_path": "",
             "headers": [(b"content-type", b"application/json")],
             "client": ("127.0.0.1", 1), "server": ("127.0.0.1", 80)}
    t0 = time.perf_counter()
    await app(scope, receive, send)
    return t0, marks


def _orchestrated(drivers):
    """The reference server's pull pattern over the adapter (harness/orchestrator_contract.py),
    collecting each request's driver for its pull count."""
    import functools

    from harness.orchestrator_contract import orchestrated_pcm_stream
    return functools.partial(orchestrated_pcm_stream, drivers=drivers)


def _http_result(workload, t0, marks, orchs=None):
    pcm = sum(n for _, n in marks) - 44
    wall = marks[-1][0] - t0
    first_pcm = next((t for t, n in marks[1:] if n > 0), t0)
    out = {"workload": workload, "value": round(pcm / 2 / 24000.0 / wall, 3),
           "unit": "audio-sec/wall-sec", "first_audio_ms": round(1e3 * (first_pcm - t0), 2),
           "bytes": pcm}
    if orchs:
        out["pulls"] = orchs[-1].pulls
        out["mean_pull_bytes"] = round(pcm / max(1, orchs[-1].pulls), 2)
        out["pulls_per_s"] = round(orchs[-1].pulls / wall, 1)
    return out


def run_http(args, syn, prompt_text, inject, local, orchestrated=False):
    """configs[1] at the HTTP level: one ``POST /v1/audio/speech`` through the ASGI app of
    ``project_morpheus_amd.server`` (no sockets), the adapter's source bound to this
    process's ``Synthesizer``.  RTF = audio / wall from request start to the last body chunk;
    first audio = first non-empty PCM chunk after the header."""
    import asyncio

    import torch

    from project_morpheus_amd import inference as I
    from project_morpheus_amd.adapter import MxTTSAdapter
    from project_morpheus_amd.server import build_app
    from project_morpheus_amd.tokenizer import Tokenizer
    tok = Tokenizer(None)

    class BenchAdapter(MxTTSAdapter):
        @staticmethod
        def source(prompt, voice, use_batching, max_batch_chars, cancel):
            torch.cuda.set_device(local)
            ids = I.prompt_ids(tok.encode(f"{voice}: {prompt}"))
            for pcm in syn.run(ids, args.max_tokens, 1.1, stop_ids=(), inject_ids=inject):
                if cancel.is_set():
                    return
                yield pcm

    orchs = []
    app = build_app(adapter_cls=BenchAdapter,
                    orchestrated_stream=_orchestrated(orchs) if orchestrated else None)
    asyncio.run(_asgi_speech(app, prompt_text))  # warm
    t0, marks = asyncio.run(_asgi_speech(app, prompt_text))
    return _http_result("configs[1] via POST /v1/audio/speech (ASGI app, RIFF + PCM16 stream), "
                        "engine.Synthesizer source"
                        + (", reference Orchestrator contract: ChunkLadder byte pulls (8-64), "
                           "per-pull JSON/base64 log, stitch_chunks, WAV streamer"
                           if orchestrated else ", 4096-byte pulls"), t0, marks, orchs)


def run_http_service(args, llm, snac, cfg, prompt_text):
    """configs[1] through the SHIPPED serving path: ``POST /v1/audio/speech`` -> default
    ``MxTTSAdapter`` source -> ``service.Service`` -> ``BatchSynthesizer`` (continuous batching
    loop, one live stream) on this process's engines, orchestrated byte pulls as the
    reference server (server.py:127-158)."""
    import asyncio

    from project_morpheus_amd import inference as I
    from project_morpheus_amd import service as S
    from project_morpheus_amd.server import build_app
    from project_morpheus_amd.tokenizer import Tokenizer
    saved = (I.TEMPERATURE, I.MAX_TOKENS)
    I.update_generation_params(temperature=0.0, max_tokens=args.max_tokens)  # greedy
    svc = S.Service.from_engines(llm, snac, cfg, synthetic_audio=True, tokenizer=Tokenizer(None))
    old, S._service = S._service, svc
    try:
        orchs = []
        app = build_app(orchestrated_stream=_orchestrated(orchs))
        asyncio.run(_asgi_speech(app, prompt_text))  # warm (graphs)
        t0, marks = asyncio.run(_asgi_speech(app, prompt_text))
    finally:
        S._service = old
        svc.close()
        I.update_generation_params(temperature=saved[0], max_tokens=saved[1])
    return _http_result("configs[1] via POST /v1/audio/speech -> default MxTTSAdapter -> "
                        "Service -> BatchSynthesizer (shipped path), reference Orchestrator "
                        "byte pulls", t0, marks, orchs)


def run_orchestrator_ceiling(audio_seconds: float, unit: str):
    """Host ceiling of the orchestrated HTTP path alone: the adapter's source yields an
    already-synthesised utterance (PCM in memory, 4096-byte windows) at once, so the RTF is
    what the Orchestrator's ladder pulls + base64 JSON log + stitcher + WAV streamer sustain
    (reference orchestrator/core.py:89-117) with ``pull_unit`` = bytes (the reference
    contract) or ms (the descriptor's unit, config.PULL_UNIT)."""
    import asyncio

    from project_morpheus_amd.adapter import MxTTSAdapter
    from project_morpheus_amd.server import build_app
    n = int(audio_seconds * 24000) * 2
    pcm = (bytes(range(256)) * (n // 256 + 1))[:n]

    class Prefilled(MxTTSAdapter):
        def __init__(self, *a, **k):
            super().__init__(*a, pull_unit=unit, **k)

        @staticmethod
        def source(prompt, voice, use_batching, max_batch_chars, cancel):
            for i in range(0, len(pcm), 4096):
                yield pcm[i:i + 4096]

    orchs = []
    app = build_app(adapter_cls=Prefilled, orchestrated_stream=_orchestrated(orchs))
    asyncio.run(_asgi_speech(app, "Hello world"))
    t0, marks = asyncio.run(_asgi_speech(app, "Hello world"))
    return _http_result(f"orchestrated HTTP path with a pre-filled source ({audio_seconds:.1f} s "
                        f"of PCM in memory), pull unit {unit}: the host ceiling, no GPU",
                        t0, marks, orchs)


def run_long_read(args, llm, snac, rank, world, dist):
    """configs[3]: ``long_read`` — 16 synthetic documents x ~3,000 chars (seed 5) split into
    the reference's <=1000-char long-form batches, every batch an independent utterance of
    ``max_tokens``; the jobs are sharded over the ranks (longest first, least loaded), each
    rank serves its share through the continuous-batching loop, PCM is gathered to rank 0
    over RCCL and stitched per document (50 ms crossfade, stitch_wav_files).  Total work is
    fixed, so this is ``strong`` scaling; value = all documents' audio / max-over-ranks wall."""
    import numpy as np
    import torch

    from project_morpheus_amd import sharding as S
    from project_morpheus_amd.batching import BatchSynthesizer, StreamRequest
    from project_morpheus_amd.tokenizer import Tokenizer
    docs = S.long_read_documents(args.long_read_docs, 3000, seed=5)
    jobs = S.plan_jobs(docs, Tokenizer(None).encode, "tara", args.max_tokens)
    syn = BatchSynthesizer(llm, snac, seed=rank)
    job_index = {id(j): i for i, j in enumerate(jobs)}

    def synthesize(mine):
        reqs = [StreamRequest(prompt_ids=j.prompt_ids, max_tokens=j.max_tokens,
                              inject_ids=synthetic_audio_ids(j.max_tokens,
                                                             seed=100 + job_index[id(j)]),
                              stop_ids=()) for j in mine]
        syn.run(reqs, on_chunk=lambda req, data: req.pcm.append(data))
        return [b"".join(r.pcm) for r in reqs]

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = S.run_sharded(jobs, rank, world, synthesize, device="cuda" if world > 1 else None,
                        crossfade_ms=50.0)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    if rank != 0:
        return None
    audio = sum(len(v) for v in out.values()) / 24000.0
    mine = S.assign(jobs, world)
    share = None
    shares = [int(x) for x in str(args.share_of).split(",") if x.strip() and int(x) > 1]
    if world == 1 and shares:
        # strong-scaling forecast measured on hardware: the most loaded rank of an N-GPU run
        # (assign() is deterministic, so this is exactly its job list) served alone on this
        # GPU, for every N asked; beside it the HBM-roofline bound of the same split
        # (sharding.scaling_bound: one GPU batches up to 32 streams per weight read, N GPUs
        # only 64 / N each, so even perfect kernels cannot scale this fixed workload linearly)
        cfg = llm.cfg
        share = {}
        for n_share in shares:
            plan = S.assign(jobs, n_share)
            r_max = max(range(n_share), key=lambda r: (sum(jobs[i].cost for i in plan[r]), -r))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pcm = synthesize([jobs[i] for i in plan[r_max]])
            torch.cuda.synchronize()
            t_share = time.perf_counter() - t0
            bound = S.scaling_bound(jobs, n_share, cfg.step_weight_bytes(),
                                    cfg.kv_bytes_per_position(), max_rows=llm.max_batch)
            share[str(n_share)] = {
                "share_of": n_share, "rank": r_max, "jobs": len(plan[r_max]),
                "wall_s": round(t_share, 3),
                "audio_seconds": round(sum(len(p) for p in pcm) / 2 / 24000.0, 2),
                "predicted_value": round(audio / t_share, 3),
                "predicted_strong_scaling_eff": round(wall / n_share / t_share, 4),
                "roofline_eff_bound": bound["efficiency_bound"]}
        share["note"] = ("per N: the most loaded rank's jobs of an N-GPU run timed alone on one "
                         "GPU; predicted value = all documents' audio / that wall (the rank-0 "
                         "gather and stitch excluded); roofline_eff_bound = the strong-scaling "
                         "efficiency this fixed 64-job split allows with every GPU at its HBM "
                         "roofline (sharding.scaling_bound: 32 rows per weight read on 1 GPU, "
                         "64 / N on N GPUs)")
    return {"workload": (f"configs[3]: long_read, {len(docs)} documents x ~3000 chars (seed 5) "
                         f"-> {len(jobs)} <=1000-char batches x {args.max_tokens} tokens, "
                         f"sharded over {world} GPU(s), continuous batching per GPU, ordered "
                         "gather to rank 0 + 50 ms crossfade stitch"),
            "scaling": "strong", "documents": len(docs), "jobs": len(jobs),
            "jobs_per_rank": [len(m) for m in mine],
            "value": round(audio / wall, 3), "unit": "audio-sec/wall-sec",
            "wall_s": round(wall, 3), "audio_seconds": round(audio, 2),
            "doc_samples_min": int(min(len(v) for v in out.values())),
            **({"rank_share": share} if share else {})}


def run_fp8(args, cfg, local, snac, prompt, inject, rank, world, dist):
    """configs[4] on this GPU: Orpheus-3B with fp8 e4m3 weights (per-row scales), fp8
    GEMV / fp8->bf16 MFMA kernels; ``args.fp8_batch`` streams per GPU batched, plus one
    single-stream utterance (the north_star's >= 30x single-stream target)."""
    import torch

    from project_morpheus_amd.engine import LlmEngine, Synthesizer, UtteranceStats
    from project_morpheus_amd.weights import quantize_fp8, synthetic_llm_weights
    w = quantize_fp8(synthetic_llm_weights(cfg, seed=0, device=f"cuda:{local}"), cfg)
    llm8 = LlmEngine(cfg, w, device=local, max_slots=args.fp8_batch, max_pos=2048,
                     max_batch=args.fp8_batch, max_prefill=256, wdtype="fp8")
    del w
    torch.cuda.empty_cache()
    out = {"weights": "fp8 e4m3 + fp32 per-row scale (3.30 GB streamed per step)"}
    out["batched"] = run_batched(args, llm8, snac, prompt, rank, world, dist,
                                 n_streams=args.fp8_batch,
                                 label=f"configs[4]: fp8, {args.fp8_batch} streams per GPU "
                                       f"({args.fp8_batch * 8} over 8 GPUs), continuous "
                                       "batching, batched SNAC")
    syn = Synthesizer(llm8, snac, depth=3, seed=rank)

    def utt():
        st = UtteranceStats()
        for _ in syn.run(prompt, args.max_tokens, 1.1, stop_ids=(), inject_ids=inject, stats=st):
            pass
        return st
    utt()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = utt()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out["single_stream"] = {"value": round(st.audio_seconds / wall, 3),
                            "unit": "audio-sec/wall-sec",
                            "first_audio_ms": round(st.first_audio_ms, 2),
                            "ms_per_token": round(1e3 * wall / st.tokens, 4)}
    llm8.close()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    if args.dry_run:
        dry_run(args, rank, world)
        return
    import numpy as np
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    from project_morpheus_amd import config as C
    from project_morpheus_amd import inference as I
    from project_morpheus_amd.engine import (LlmEngine, SnacDecoder, Synthesizer,
                                             UtteranceStats)
    from project_morpheus_amd.tokenizer import Tokenizer
    from project_morpheus_amd.weights import synthetic_llm_weights, synthetic_snac_weights

    cfg = C.OrpheusConfig()
    free0 = torch.cuda.mem_get_info(local)[0]
    w = synthetic_llm_weights(cfg, seed=0, device=f"cuda:{local}")
    B3 = args.batch
    llm = LlmEngine(cfg, w, device=local, max_slots=max(1, B3), max_pos=2048,
                    max_batch=max(1, B3), max_prefill=512)
    del w
    torch.cuda.empty_cache()
    # device memory the engine holds (driver view): bf16 weights row-major for the one-row
    # GEMVs + the fragment-major copies the multi-row GEMMs read, KV cache and workspaces
    engine_hbm_gb = round((free0 - torch.cuda.mem_get_info(local)[0]) / 1e9, 2)
    snac = SnacDecoder(synthetic_snac_weights(), device=local, max_frames=7,
                       max_batch=max(1, B3))
    syn = Synthesizer(llm, snac, depth=3, seed=rank)
    tok = Tokenizer(None)
    prompt = I.prompt_ids(tok.encode("tara: Hello world"))
    inject = synthetic_audio_ids(args.max_tokens, seed=2 + rank)

    def utterance():
        st = UtteranceStats()
        for _ in syn.run(prompt, args.max_tokens, 1.1, stop_ids=(), inject_ids=inject, stats=st):
            pass
        return st

    for _ in range(args.warmup):
        utterance()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = [utterance() for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    audio = sum(s.audio_seconds for s in stats)
    firsts = [s.first_audio_ms for s in stats]
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        a = torch.tensor([audio], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
        elapsed, audio = float(t.item()), float(a.item())
        fl = [None] * world
        dist.all_gather_object(fl, firsts)
        firsts = [x for r in fl for x in r]

    # ---- configs[1] at the HTTP level (rank 0 only: one request through the ASGI app) ----
    http_level = http_orch = http_service = ceiling = None
    if rank == 0 and not args.no_http:
        http_level = run_http(args, syn, "Hello world", inject, local)
        http_orch = run_http(args, syn, "Hello world", inject, local, orchestrated=True)
        http_service = run_http_service(args, llm, snac, cfg, "Hello world")
        utt_s = audio / max(1, args.steps) / max(1, world)
        ceiling = {u: run_orchestrator_ceiling(utt_s, u) for u in ("bytes", "ms")}

    # ---- configs[2]: B concurrent streams per GPU, continuous batching + batched SNAC ----
    batched = batched_nc = None
    if B3 > 0:
        batched = run_batched(args, llm, snac, prompt, rank, world, dist)
        if args.compaction_ab:
            batched_nc = run_batched(args, llm, snac, prompt, rank, world, dist,
                                     label="configs[2] without decode-row compaction",
                                     compact=False)

    # ---- configs[3]: long_read documents sharded over the ranks, gathered + stitched ----
    long_read = None
    if args.long_read_docs > 0:
        long_read = run_long_read(args, llm, snac, rank, world, dist)

    # ---- configs[4] per GPU: fp8 weights, args.fp8_batch streams per GPU (64 over 8 GPUs) ----
    fp8 = None
    if args.fp8_batch > 0:
        fp8 = run_fp8(args, cfg, local, snac, prompt, inject, rank, world, dist)

    # ---- roofline of the dominant kernel (gate/up GEMV, 2*ffn*hidden bf16 per launch) ----
    # HIP events around one hipGraph of back-to-back launches of that kernel sweeping all 28
    # layers' weights (as a decode step streams them), on the engine's capture stream
    st = syn.stream
    st.synchronize()
    gemv_us = {}
    for kind in ("gate_up", "qkv", "o_proj", "down"):
        us, nbytes = llm.bench_gemv(kind, reps=4)
        gemv_us[kind] = (us, nbytes)
    gu_us, gu_bytes = gemv_us["gate_up"]
    gu_gbs = gu_bytes / (gu_us * 1e-6) / 1e9
    llm.prefill(0, 0, prompt, 1.1, st)
    for _ in range(3):
        llm.decode(1, st)
    prof = {}
    for _ in range(args.profile_steps):
        for k, v in llm.decode_profiled(1, st).items():
            prof[k] = prof.get(k, 0.0) + v
    per_step_us = {k: round(1e3 * v / args.profile_steps, 2) for k, v in prof.items()}
    llm.release_row(0, st)
    st.synchronize()
    # pure decode step (graph replay, no SNAC) against the whole-step byte roofline
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n_rep = 50
    llm.prefill(0, 0, prompt, 1.1, st)
    for _ in range(args.step_pos - len(prompt)):   # measure the step at a mid-utterance length
        llm.decode(1, st)
    ev0.record(st)
    for _ in range(n_rep):
        llm.decode(1, st)
    ev1.record(st)
    ev1.synchronize()
    step_ms = ev0.elapsed_time(ev1) / n_rep
    pos = args.step_pos + n_rep // 2
    step_bytes = cfg.step_weight_bytes() + pos * cfg.kv_bytes_per_position()
    llm.release_row(0, st)
    st.synchronize()

    if rank == 0:
        steps_audio = audio
        value = steps_audio / elapsed
        res = {
            "metric": METRIC, "value": round(value, 4), "unit": "audio-sec/wall-sec",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic",
            "config": {"workload": "configs[1]: Orpheus-3B bf16 single stream per GPU, "
                                   "SNAC 24 kHz, greedy + rep-penalty 1.1, hipGraph decode step",
                       "model": "orpheus-3b (synthetic weights)", "global_batch": world,
                       "seq_len": len(prompt) + args.max_tokens, "prompt_ids": len(prompt),
                       "max_tokens": args.max_tokens, "parallelism": f"streams{world}"},
            "p50_first_audio_ms": round(statistics.median(firsts), 2),
            "audio_seconds": round(audio, 3),
            "http_level": http_level,
            "http_level_orchestrator": http_orch,
            "http_level_service": http_service,
            "orchestrator_ceiling": ceiling,
            "configs_2_batched": batched,
            **({"configs_2_no_compaction": batched_nc} if batched_nc else {}),
            "configs_3_long_read": long_read,
            "configs_4_fp8": fp8,
            "engine_hbm_gb": engine_hbm_gb,
            "decode_step_ms": round(step_ms, 4),
            "decode_tok_per_s": round(1e3 / step_ms, 1),
            "step_roofline": {"bytes": step_bytes, "achieved_gbs": round(step_bytes / step_ms / 1e6, 1),
                              "frac": round(step_bytes / step_ms / 1e6 / PEAK_HBM_GBS, 4)},
            "roofline": {"kernel": ROOFLINE_KERNEL,
                         "what": "one-row RMSNorm + gate/up [16384 x 3072] + SiLU*up (EPI_SILU, NORM)",
                         "bound": "hbm", "achieved": round(gu_gbs, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(gu_gbs / PEAK_HBM_GBS, 4),
                         "avg_launch_us": round(gu_us, 3), "bytes_per_launch": gu_bytes,
                         "avg_launch_us_source": "HIP events around one hipGraph of 4 x 28 "
                                                 "back-to-back launches (launch gaps included)",
                         **rocprof_fields(gu_bytes),
                         "traffic": pmc_traffic("gate_up"),
                         "traffic_source": f"profiles/{PMC_RECORD} (rocprofv3 --pmc "
                                           "FETCH_SIZE / WRITE_SIZE, separate passes)"},
            "eager_step_us_by_kernel": per_step_us,
            "gemv_graph_us": {k: {"us": round(v[0], 2), "GB/s": round(v[1] / v[0] / 1e3, 1)}
                              for k, v in gemv_us.items()},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(cfg, prompt)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
