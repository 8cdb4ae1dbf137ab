"""CPU check: every SNAC kernel instantiation the serving path can run is compared with the
oracle by a `-m gpu` test (tests/_snac_dispatch.py, tests/_coverage.py SNAC_RUNS), the SNAC
twin of tests/test_kernel_coverage.py.

1. the restatement of the SNAC dispatch (capi.hip snac_enqueue / pick_tiles, snac_kernels.hip
   launch_conv_gemm / launch_dwconv) predicts what the hardware ran: every SNAC kernel in the
   committed rocprofv3 summaries of full bench runs is named by the serving envelope (1-, 4-
   and 7-frame windows, 1..32 per call);
2. every key of the envelope (instantiation + edge class) is reached by a declared GPU run;
3. the declared runs are the ones the GPU tests perform (``check_declared_snac`` inside them).
"""
import csv
import os
import re

import _snac_dispatch as S
from _coverage import SNAC_RUNS

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH_TRACES = ["profiles/r05_bench_kernel_stats_final.csv"]
_SNAC = re.compile(r"(?:void )?mx::((?:conv_gemm\w*|dwconv|snac_\w+|set_io)_kernel(?:<[^>]*>)?)\(")
PLUMBING = {"set_io_kernel"}  # stores the call's pointers for the captured graph (no arithmetic)


def _traced(path):
    with open(os.path.join(ROOT, path)) as fh:
        return {m.group(1) for r in csv.DictReader(fh) if (m := _SNAC.match(r["Name"]))}


def _covered():
    keys = set()
    for runs in SNAC_RUNS.values():
        for run in runs:
            n, b = run[:2]
            keys |= S.window_keys(n, b, *S.serving_slice(n)) if len(run) > 2 else S.window_keys(n, b)
    return keys


# bench traces recorded before PCM-only calls were cut to the kept slice's receptive field
UNCUT = {"profiles/r06_bench_kernel_stats_v1.csv", "profiles/r06_bench_kernel_stats_final.csv"}


def test_restatement_predicts_the_bench_trace():
    for path in BENCH_TRACES + sorted(
            p for p in (f"profiles/{f}" for f in os.listdir(os.path.join(ROOT, "profiles")))
            if re.match(r"profiles/r0[6-9]_bench_kernel_stats.*\.csv$", p)):
        cut = path not in UNCUT and path not in BENCH_TRACES
        names = {S.name_of(k) for k in S.envelope(cut=cut)}
        traced = _traced(path) - PLUMBING
        assert traced, path
        assert traced <= names, (path, sorted(traced - names))


def test_every_serving_snac_key_is_compared_on_the_gpu():
    missing = S.envelope() - _covered()
    assert not missing, sorted(missing)


def test_declared_snac_runs_exist():
    src = open(os.path.join(ROOT, "tests", "test_gpu_snac.py")).read()
    for node in SNAC_RUNS:
        name = node.split("::")[1].split("[")[0]
        assert f"def {name}(" in src, node
        if "[" in node:
            n, b = node.split("[")[1].rstrip("]").split("-")
            assert f"({n}, {b})" in src, node


def test_pick_tiles_restatement_spot_values():
    """A few launches whose instantiation the r05 trace shows: a single 7-frame window's input
    1x1 conv (32 M-tiles x 1 column tile, K 768: WK 4) and first ConvTranspose (16 M-tiles x 8
    phases, K 2 x 1,024: WK 8)."""
    assert S.conv_gemm_key(1024, 768, 28, 1, 1, 1) == "conv_gemm_kernel<4, 2> [ragged]"
    assert S.conv_gemm_key(512, 1024, 28, 1, 2, 8) == "conv_gemm_kernel<8, 2> [ragged]"
    assert S.conv_gemm_key(1024, 768, 28, 8, 1, 1).startswith("conv_gemm_tiled_kernel<1>")
    assert not S.conv_gemm_key(1024, 768, 28, 7, 1, 1).startswith("conv_gemm_tiled_kernel<1>")
    assert S.dwconv_key(32, 1792) == "dwconv_kernel<64>"
    assert S.dwconv_key(1, 1792) == "dwconv_kernel<16>"
