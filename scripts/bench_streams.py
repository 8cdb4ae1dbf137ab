"""Do concurrent multi-row row groups overlap?  One GEMV kind's all-layer sweep at R rows on
1 stream, against the same sweep at R/2 rows on 2 concurrent streams (each its own split-K
workspace; full Orpheus-3B shapes, synthetic weights).

    python scripts/bench_streams.py [--rows 32] [--kinds qkv,o_proj,gate_up,down] [--fp8]

Prints µs per launch: 1 x R, 1 x R/2, and 2 x R/2 concurrent (wall per launch of one stream;
below 2 x (1 x R/2) means the two groups overlap each other's fixed costs)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--kinds", default="qkv,o_proj,gate_up,down")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
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
    llm = LlmEngine(cfg, w, device=0, max_slots=R, max_pos=1024, max_batch=R, max_prefill=64,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    for kind in args.kinds.split(","):
        for _ in range(2):
            full = llm.bench_gemv_streams(kind, R, 1, args.reps)
            half = llm.bench_gemv_streams(kind, R // 2, 1, args.reps)
            two = llm.bench_gemv_streams(kind, R // 2, 2, args.reps)
            print(json.dumps({"kind": kind, "rows": R, "one_stream_R_us": round(full, 2),
                              "one_stream_half_us": round(half, 2),
                              "two_streams_half_us": round(two, 2),
                              "overlap": round(2 * half / two, 3) if two else None}), flush=True)
    llm.close()


if __name__ == "__main__":
    main()
