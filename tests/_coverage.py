"""Registry of the GPU parity tests' engine runs at Orpheus widths, and the bench's envelope.

Every `-m gpu` test that builds an LlmEngine at Orpheus widths (hidden 3,072) declares its
runs here; the test helpers check at run time that the run they perform is the declared one
(``check_declared``), so this table cannot drift from the tests.  From the declared runs,
``tests/_dispatch.py`` (a restatement of the library's dispatch) derives the kernel
instantiations each test compares with the oracle, and ``tests/test_kernel_coverage.py``
asserts on the CPU that:

* every instantiation the bench can reach (``bench_envelope``) is compared by some test;
* every instantiation in the committed rocprofv3 summary of the bench run
  (``profiles/*bench_kernel_stats*.csv``) is in the envelope (the restatement is checked
  against what the hardware actually ran).

A run is ``(dims, f8, lens, steps, opts)``: prompts of ``lens`` ids prefilled on their own
rows, then ``steps`` tokens per row (``_dispatch.run_keys``).
"""
from __future__ import annotations

import os

from _dispatch import ORPHEUS, ORPHEUS_16K, Dims, decode_keys, prefill_keys, run_keys


def _r(dims, lens, steps, f8=False, **opts):
    return (dims, f8, tuple(lens), steps, tuple(sorted(opts.items())))


def _rows(n, base, step=1, extra=6):
    """tests/test_gpu_llm._orpheus_prompts lengths: base + step i text ids + 6 framing ids"""
    return [base + step * i + extra for i in range(n)]


# test node (file::name[param]) -> its engine runs at Orpheus widths
GPU_RUNS = {
    # ---- bf16, one row --------------------------------------------------------------
    "test_gpu_llm.py::test_decode_parity_orpheus_width_2_layers":
        [_r(ORPHEUS, [18], 24)],
    "test_gpu_llm.py::test_decode_parity_orpheus_width_no_o_merge":
        [_r(ORPHEUS, [18], 12, o_merge=0)],
    **{f"test_gpu_llm.py::test_decode_parity_orpheus_width_no_gemv_balance[{p}]":
       [_r(ORPHEUS_16K, [p], 16, gemv_balance=0)] for p in (200, 300, 600)},
    **{f"test_gpu_llm.py::test_decode_parity_orpheus_width_short_splits[{p}]":
       [_r(ORPHEUS_16K, [p], 16, att_b1_short=2)] for p in (200, 600)},
    "test_gpu_llm.py::test_lm_head_grid_stride_orpheus_width":
        [_r(ORPHEUS, [24], 16, head_b1=0)],
    "test_gpu_llm.py::test_full_depth_orpheus_3b_single_stream":
        [_r(ORPHEUS, [30], 10)],
    "test_gpu_llm.py::test_long_context_orpheus_width_default_path":
        [_r(ORPHEUS_16K, [600], 520)],
    "test_gpu_llm.py::test_one_row_orpheus_width_split_classes":
        [_r(ORPHEUS_16K, [185], 16)],
    "test_gpu_llm.py::test_long_context_orpheus_width_past_2048_4096[2048]":
        [_r(ORPHEUS_16K, [2040], 16)],
    "test_gpu_llm.py::test_long_context_orpheus_width_past_2048_4096[4096]":
        [_r(ORPHEUS_16K, [4090], 12)],
    # ---- bf16, several rows ---------------------------------------------------------
    "test_gpu_llm.py::test_batched_decode_orpheus_width_4_rows":
        [_r(ORPHEUS, [14, 17, 20, 23], 10)],
    "test_gpu_llm.py::test_batched_decode_orpheus_width_6_rows":
        [_r(ORPHEUS, _rows(6, 6), 6)],
    "test_gpu_llm.py::test_batched_decode_orpheus_width_6_rows_split_k_seam":
        [_r(ORPHEUS, _rows(6, 6), 6, rows_atomic=0, rows_qkv_parts=0)],
    "test_gpu_llm.py::test_batched_decode_orpheus_width_32_rows":
        [_r(ORPHEUS, _rows(32, 4), 5)],
    "test_gpu_llm.py::test_batched_decode_orpheus_width_64_rows":
        [_r(ORPHEUS, _rows(64, 3), 3)],
    "test_gpu_llm.py::test_batched_lm_head_k_split_orpheus_width[2048]":
        [_r(ORPHEUS, _rows(12, 4), 4, rows_head_target=2048)],
    "test_gpu_llm.py::test_batched_lm_head_k_split_orpheus_width[4096]":
        [_r(ORPHEUS, _rows(12, 4), 4, rows_head_target=4096)],
    "test_gpu_llm.py::test_batched_decode_orpheus_width_32_rows_long_context":
        [_r(ORPHEUS_16K, [1400 + 5 + r for r in range(32)], 12)],
    **{f"test_gpu_llm.py::test_batched_decode_orpheus_width_32_rows_attention_chunks[{p}]":
       [_r(ORPHEUS_16K, [p + 5 + r for r in range(32)], 6)] for p in (280, 560, 850)},
    "test_gpu_llm.py::test_prefill_batch_tile_classes_orpheus_width":
        [_r(ORPHEUS_16K, [100, 150], 6)],
    "test_gpu_llm.py::test_rows_merge_straddling_splits_orpheus_width[nsm2]":
        [_r(ORPHEUS_16K, [200, 215, 230, 250, 262, 280, 400, 497], 12, att_nw6=0)],
    "test_gpu_llm.py::test_rows_merge_straddling_splits_orpheus_width[nsm4]":
        [_r(ORPHEUS_16K, [200, 260, 330, 480, 520, 600, 700, 760], 12, att_nw6=0)],
    "test_gpu_llm.py::test_batched_decode_orpheus_width_8_rows_split_attention[0]":
        [_r(ORPHEUS_16K, [520 + 3 + 5 * r for r in range(8)], 8, rows_merge=0)],
    "test_gpu_llm.py::test_batched_decode_orpheus_width_8_rows_split_attention[1]":
        [_r(ORPHEUS_16K, [520 + 3 + 5 * r for r in range(8)], 8, rows_merge=1)],
    **{f"test_gpu_llm.py::test_batched_decode_orpheus_width_8_rows_six_wave_attention[{p}]":
       [_r(ORPHEUS_16K, [p + 3 + 9 * r for r in range(8)], 6)] for p in (520, 1100)},
    "test_gpu_llm.py::test_batched_decode_orpheus_width_8_rows_eight_wave_attention":
        [_r(ORPHEUS_16K, [520 + 3 + 9 * r for r in range(8)], 6, att_nw6=0)],
    # ---- fp8 (e4m3 weights) -----------------------------------------------------------
    "test_gpu_fp8.py::test_fp8_single_stream_orpheus_width":
        [_r(ORPHEUS, [120], 16, f8=True)],
    "test_gpu_fp8.py::test_fp8_batched_orpheus_width_8_rows":
        [_r(ORPHEUS, [5 + 4 * i for i in range(8)], 6, f8=True)],
    "test_gpu_fp8.py::test_fp8_batched_orpheus_width_8_rows_split_k_seam":
        [_r(ORPHEUS, [5 + 4 * i for i in range(8)], 6, f8=True, rows_atomic=0, rows_qkv_parts=0)],
    "test_gpu_fp8.py::test_fp8_single_stream_orpheus_width_no_gemv_balance":
        [_r(ORPHEUS_16K, [600], 16, f8=True, gemv_balance=0)],
    "test_gpu_fp8.py::test_fp8_lm_head_grid_stride_orpheus_width":
        [_r(ORPHEUS, [40], 12, f8=True, head_b1=0)],
    "test_gpu_fp8.py::test_fp8_batched_orpheus_width_8_rows_split_attention_merged_in_oproj":
        [_r(ORPHEUS_16K, [300 + 5 * i for i in range(8)], 4, f8=True, rows_merge=1)],
    "test_gpu_fp8.py::test_fp8_single_stream_orpheus_width_long_context":
        [_r(ORPHEUS_16K, [600], 520, f8=True)],
    "test_gpu_fp8.py::test_fp8_one_row_orpheus_width_split_classes":
        [_r(ORPHEUS_16K, [185], 16, f8=True)],
    "test_gpu_fp8.py::test_fp8_rows_merge_straddling_splits_orpheus_width[nsm2]":
        [_r(ORPHEUS_16K, [200, 215, 230, 250, 262, 280, 400, 497], 12, f8=True, att_nw6=0)],
    "test_gpu_fp8.py::test_fp8_rows_merge_straddling_splits_orpheus_width[nsm4]":
        [_r(ORPHEUS_16K, [200, 260, 330, 480, 520, 600, 700, 760], 12, f8=True, att_nw6=0)],
    # ---- the persistent one-row engine (option b1_engine) ----------------------------
    "test_gpu_engine_b1.py::test_engine_orpheus_width[bf16]":
        [_r(ORPHEUS_16K, [600], 40, b1_engine=1)],
    "test_gpu_engine_b1.py::test_engine_orpheus_width[fp8]":
        [_r(ORPHEUS_16K, [600], 40, f8=True, b1_engine=1)],
    "test_gpu_engine_b1.py::test_engine_full_depth_orpheus_3b":
        [_r(ORPHEUS, [30], 10, b1_engine=1)],
    # ---- sampling -------------------------------------------------------------------
    "test_gpu_sampling.py::test_sampling_one_row_hidden_3072_product_mode":
        [_r(ORPHEUS_16K, [9], 12)] * 3,
}


# SNAC: test node -> the (frames, windows) of each mx_snac_decode call it compares with the
# oracle (tests/_snac_dispatch.py derives the kernel keys; tests/test_snac_coverage.py checks
# them against the serving envelope and the bench trace)
SNAC_RUNS = {
    **{f"test_gpu_snac.py::test_snac_window_parity[{n}-{b}]": [(n, b)]
       for n, b in ((1, 1), (4, 1), (7, 1), (7, 3), (2, 2), (1, 5), (4, 9), (7, 12), (5, 1),
                    (5, 12))},
    "test_gpu_snac.py::test_snac_batched_32_windows_matches_oracle": [(7, 32)],
    # PCM-only calls: blocks 1-3 on the kept slice's receptive field (capi.hip snac_cut)
    **{f"test_gpu_snac.py::test_snac_cut_pcm_parity[{n}-{b}]": [(n, b, True)]
       for n, b in ((5, 1), (4, 5), (5, 12), (5, 32))},
}


def check_declared_snac(n_frames, batch, cut=False):
    """cut: a PCM-only call with the serving slice (blocks 1-3 cut to its receptive field)."""
    node = current_test()
    runs = SNAC_RUNS.get(node)
    assert runs is not None, f"{node}: SNAC GPU run not declared in tests/_coverage.py"
    run = (n_frames, batch, True) if cut else (n_frames, batch)
    assert run in runs, f"{node}: {run} is not declared ({runs})"


def current_test():
    """'file.py::name[param]' of the running pytest test ('' outside pytest)."""
    node = os.environ.get("PYTEST_CURRENT_TEST", "").rsplit(" ", 1)[0]
    return node.split("/")[-1]


def dims_of(cfg) -> Dims:
    return Dims(cfg.hidden, cfg.heads, cfg.kv_heads, cfg.ffn, cfg.vocab)


def check_declared(cfg, lens, steps, f8=False, opts=None):
    """Called by the GPU test helpers before a run: at Orpheus widths the run must be one the
    registry declares for the running test (so the coverage check sees what the tests run)."""
    if cfg.hidden != 3072:
        return
    node = current_test()
    runs = GPU_RUNS.get(node)
    assert runs is not None, f"{node}: Orpheus-width GPU run not declared in tests/_coverage.py"
    run = _r(dims_of(cfg), lens, steps, f8, **(opts or {}))
    assert run in runs, f"{node}: run {run} is not the declared one ({runs})"


def keys_of(node):
    keys = set()
    for dims, f8, lens, steps, opts in GPU_RUNS[node]:
        keys |= run_keys(dims, f8, list(lens), steps, dict(opts))
    return keys


def covered_keys():
    out = set()
    for node in GPU_RUNS:
        out |= keys_of(node)
    return out


def probe_keys():
    """bench.py's roofline section: mx_llm_bench_gemv sweeps of the qkv / o-proj / gate-up /
    down GEMVs over every layer, one row (capi.hip: the o-proj probe runs without the split
    merge, rows per wave from the rpw_o option, i.e. 1)."""
    from _dispatch import DEFAULTS, EPI_QKV, EPI_RESID, EPI_SILU, gemv_launch
    d, o = ORPHEUS, DEFAULTS
    H, QD = d.hidden, d.heads * 128
    return {gemv_launch(QD + 2 * d.kv_heads * 128, H, 1, EPI_QKV, True, False, o),
            gemv_launch(H, QD, 1, EPI_RESID, False, False, o, rpw=o["rpw_o"]),
            gemv_launch(2 * d.ffn, H, 1, EPI_SILU, True, False, o, rpw=o["rpw_gu"]),
            gemv_launch(H, d.ffn, 1, EPI_RESID, False, False, o, rpw=o["rpw_down"])}


def bench_envelope(prompt_len=10, stream_prompts=(16, 64), job_prompts=(22, 259),
                   max_tokens=1200, batch=32, fp8_batch=8, opts=None):
    """Every (rows, longest span) a default bench.py run can step, at Orpheus widths:
    configs[1] and the HTTP lines (one bf16 row), configs[2] (<= 32 rows, prompts of 16..64
    ids), configs[3] long_read and its 8-GPU rank share (<= 32 rows, the jobs' 22..259-id
    prompts), configs[4] (<= 8 e4m3 rows and one e4m3 row).  Rows x spans are taken as a
    product (a superset of what one run steps).  ``opts``: library options that differ from
    today's defaults (a trace recorded under an earlier default)."""
    keys = set()
    d = ORPHEUS
    s_lo, s_hi = stream_prompts
    j_lo, j_hi = job_prompts
    for f8 in (False, True):
        for L in range(2, max(prompt_len, s_hi) + max_tokens + 1):
            keys |= decode_keys(d, 1, L, f8, opts)
        for n in [prompt_len] + list(range(s_lo, s_hi + 1)):
            keys |= prefill_keys(d, n, f8, opts)
    for R in range(2, batch + 1):
        for L in range(s_lo + 1, max(s_hi, j_hi) + max_tokens + 1):
            keys |= decode_keys(d, R, L, False, opts)
    for n in range(s_lo, j_hi + 1):
        keys |= prefill_keys(d, n, False, opts)
    for n in range(j_lo, s_lo):
        keys |= prefill_keys(d, n, False, opts)
    for R in range(2, fp8_batch + 1):
        for L in range(s_lo + 1, s_hi + max_tokens + 1):
            keys |= decode_keys(d, R, L, True, opts)
    return keys
