"""Run the single-row decode GEMVs (all 28 layers' weights, graph sweeps) for PMC collection.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o pmc -- python3 scripts/pmc_gemv.py
    python3 scripts/pmc_summary.py OUT/.../pmc_counter_collection.csv

Each sweep streams 28 different layers' weights (2.8 GB for gate/up), so nothing is served from
the 256 MiB Infinity Cache and FETCH_SIZE prices the HBM side of one launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import synthetic_llm_weights
    cfg = C.OrpheusConfig()
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    llm = LlmEngine(cfg, w, device=0, max_slots=1, max_pos=2048, max_batch=1, max_prefill=64)
    del w
    torch.cuda.empty_cache()
    for kind in ("qkv", "o_proj", "gate_up", "down"):
        us, nb = llm.bench_gemv(kind, reps=1)
        print(f"{kind}: {us:.2f} us/launch, {nb:.0f} weight bytes/launch", flush=True)


if __name__ == "__main__":
    main()
