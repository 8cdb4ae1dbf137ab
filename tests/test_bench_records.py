"""The measurement records bench.py reads on the GPU box (CPU only: files under profiles/).

``roofline.traffic`` in the bench line comes from the newest PMC record
(``profiles/r0N_pmc_gemv.json``, rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
``scripts/gpu_pmc_b1.sh``); it must exist, cover the dominant kernel, and price every one-row
kernel of the step close to its algorithmic bytes."""
import importlib.util
import json
import os

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_records_probe", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_reads_the_newest_pmc_record():
    b = _bench()
    records = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles"))
                     if f.endswith("_pmc_gemv.json"))
    assert records and b.PMC_RECORD == records[-1]
    gate_up = b.pmc_traffic("gate_up")
    assert gate_up is not None and gate_up >= 100663296  # 16384 x 3072 bf16 per launch


def test_pmc_record_prices_the_one_row_kernels():
    b = _bench()
    rec = json.load(open(os.path.join(ROOT, "profiles", b.PMC_RECORD)))
    kernels = rec["kernels"]
    for kind in ("qkv", "gate_up", "down"):
        assert kind in kernels
    for kind, e in kernels.items():
        assert e["traffic_bytes"] == e["hbm_read_bytes"] + e["hbm_write_bytes"], kind
        assert 0.99 <= e["traffic_over_algorithmic"] <= 1.10, (kind, e["traffic_over_algorithmic"])
