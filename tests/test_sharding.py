"""Batch-sharding of long-read jobs over ranks on CPU with ``gloo``.

The synthesis function is a deterministic stand-in (PCM derived from the job text), so the
test checks the plan, the balance, the rank-0 gather and the per-document reassembly —
everything the multi-GPU path adds on top of the single-GPU engine.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from project_morpheus_amd import inference as I
from project_morpheus_amd import sharding as S
from project_morpheus_amd.tokenizer import Tokenizer


def _fake_pcm(job: S.Job) -> bytes:
    """Ragged, text-dependent PCM (length 0..3999 samples) for one job."""
    h = hashlib.blake2s(job.text.encode()).digest()
    n = int.from_bytes(h[:2], "little") % 4000
    rng = np.random.default_rng(int.from_bytes(h[2:10], "little"))
    return rng.integers(-30000, 30000, size=n).astype(np.int16).tobytes()


def _synth(jobs):
    return [_fake_pcm(j) for j in jobs]


def _jobs(n_docs=6, n_chars=2500):
    tok = Tokenizer(None)
    docs = S.long_read_documents(n_docs, n_chars, seed=5)
    docs.append("Short one.")  # a document that stays one batch
    docs.append("")            # an empty document: one empty job
    return docs, S.plan_jobs(docs, tok.encode, "tara", max_tokens=0)


def _expected(docs, jobs, crossfade_ms):
    out = {}
    for d in range(len(docs)):
        segs = [np.frombuffer(_fake_pcm(j), dtype=np.int16) for j in jobs if j.doc == d]
        out[d] = (I.crossfade_join(segs, crossfade_ms) if crossfade_ms
                  else np.concatenate(segs))
    return out


def test_plan_follows_reference_batching():
    docs, jobs = _jobs()
    for d, text in enumerate(docs):
        parts = [j for j in jobs if j.doc == d]
        assert [j.part for j in parts] == list(range(len(parts)))
        assert [j.text for j in parts] == I.batch_sentences(text, 1000, True)
        for j in parts:
            assert j.prompt_ids[0] == I.START_TOKEN_ID
            assert j.prompt_ids[-4:] == I.END_TOKEN_IDS
    assert max(len(j.text) for j in jobs) <= 1000 + 200  # one long sentence may overflow


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_assign_is_a_balanced_partition(world):
    _, jobs = _jobs(12, 3000)
    plan = S.assign(jobs, world)
    flat = sorted(i for r in plan for i in r)
    assert flat == list(range(len(jobs)))
    loads = [sum(jobs[i].cost for i in r) for r in plan]
    # LPT bound: max load <= mean + largest job
    assert max(loads) <= sum(loads) / world + max(j.cost for j in jobs)
    assert plan == S.assign(jobs, world)  # deterministic


def test_assign_more_ranks_than_jobs():
    _, jobs = _jobs(1, 300)
    plan = S.assign(jobs, 8)
    assert sorted(i for r in plan for i in r) == list(range(len(jobs)))
    assert sum(1 for r in plan if not r) == 8 - len(jobs)


@pytest.mark.parametrize("crossfade_ms", [0.0, 50.0])
def test_single_rank_assembly(crossfade_ms):
    docs, jobs = _jobs()
    out = S.run_sharded(jobs, 0, 1, _synth, crossfade_ms=crossfade_ms)
    exp = _expected(docs, jobs, crossfade_ms)
    assert sorted(out) == sorted(exp)
    for d in exp:
        np.testing.assert_array_equal(out[d], exp[d])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, crossfade_ms, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        docs, jobs = _jobs()
        seen = []

        def synth(js):
            seen.extend((j.doc, j.part) for j in js)
            return _synth(js)

        out = S.run_sharded(jobs, rank, world, synth, crossfade_ms=crossfade_ms)
        mine = {(jobs[i].doc, jobs[i].part) for i in S.assign(jobs, world)[rank]}
        assert set(seen) == mine
        if rank == 0:
            np.savez(result_path, **{f"d{d}": v for d, v in out.items()})
        else:
            assert out is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("crossfade_ms", [0.0, 50.0])
def test_gloo_world2_gather_matches_single_rank(tmp_path, crossfade_ms):
    path = str(tmp_path / "out.npz")
    mp.spawn(_worker, args=(2, _free_port(), crossfade_ms, path), nprocs=2, join=True)
    docs, jobs = _jobs()
    exp = _expected(docs, jobs, crossfade_ms)
    with np.load(path) as z:
        got = {int(k[1:]): z[k] for k in z.files}
    assert sorted(got) == sorted(exp)
    for d in exp:
        np.testing.assert_array_equal(got[d], exp[d])


def test_scaling_bound_of_the_long_read_split():
    """configs[3]'s fixed 64-job workload: with every GPU at its HBM roofline, 1 GPU batches
    32 streams per weight read and N GPUs 64 / N, so strong scaling is bounded below linear
    (bench.py reports this bound beside the measured per-N rank-share forecast)."""
    from project_morpheus_amd import config as C
    from project_morpheus_amd.tokenizer import Tokenizer
    cfg = C.OrpheusConfig()
    jobs = S.plan_jobs(S.long_read_documents(16, 3000, seed=5), Tokenizer(None).encode,
                       "tara", 1200)
    assert len(jobs) == 64
    b = {n: S.scaling_bound(jobs, n, cfg.step_weight_bytes(), cfg.kv_bytes_per_position())
         for n in (1, 2, 4, 8)}
    assert b[1]["efficiency_bound"] == 1.0
    assert 1.0 >= b[2]["efficiency_bound"] > b[4]["efficiency_bound"] > b[8]["efficiency_bound"]
    assert 0.25 < b[8]["efficiency_bound"] < 0.45
    # the roofline wall of one GPU: 2 waves of 32 rows x 1,200 steps of >= 6.6 GB each
    assert b[1]["t1_roofline_s"] > 2 * 1200 * cfg.step_weight_bytes() / 8e12


def test_roofline_wall_counts_prefills_and_kv():
    j = [S.Job(0, i, "x", prompt_ids=[1] * 10, max_tokens=3) for i in range(3)]
    W, kv = 100, 1
    # 3 prefills (3 W) + 2 decode steps over 3 rows at positions 10 -> 11, 11 -> 12
    want = 3 * W + (W + 3 * 11) + (W + 3 * 12)
    assert abs(S.roofline_wall(j, W, kv, max_rows=32, hbm_bps=1.0) - want) < 1e-9
    # max_rows 2: rows 0, 1 first (2 prefills, 2 steps), then row 2 (1 prefill, 2 steps)
    want2 = 2 * W + (W + 2 * 11) + (W + 2 * 12) + W + (W + 11) + (W + 12)
    assert abs(S.roofline_wall(j, W, kv, max_rows=2, hbm_bps=1.0) - want2) < 1e-9
