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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--kinds", default="qkv,o_proj,gate_up,down")
    ap.add_argument("--options", default="", help="k=v,k=v set_option knobs")
    ap.add_argument("--fp8", action="store_true", help="e4m3 weights + per-row scales")
    args = ap.parse_args()
    import torch
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import synthetic_llm_weights
    cfg = C.OrpheusConfig()
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    if args.fp8:
        from project_morpheus_amd.weights import quantize_fp8
        w = quantize_fp8(w, cfg)
    R = args.rows
    llm = LlmEngine(cfg, w, device=0, max_slots=R, max_pos=2048, max_batch=R, max_prefill=64,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    for kv in filter(None, args.options.split(",")):
        k, v = kv.split("=")
        llm.set_option(k, int(v))
    for kind in args.kinds.split(","):
        us, nb = llm.bench_gemv(kind, reps=1, n_rows=R)
        print(f"{kind}: {us:.2f} us/launch, {nb:.0f} weight bytes/launch", flush=True)


if __name__ == "__main__":
    main()
