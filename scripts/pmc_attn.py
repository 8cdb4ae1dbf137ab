"""Batched attention under PMC / timing sweep (diagnostic): R rows, context L, one layer."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--lens", default="600")
    ap.add_argument("--cpw", type=int, default=4)
    ap.add_argument("--nw", type=int, default=8)
    args = ap.parse_args()
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import synthetic_llm_weights
    cfg = C.OrpheusConfig(layers=1, vocab=1024)
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    llm = LlmEngine(cfg, w, device=0, max_slots=32, max_pos=4096, max_batch=32, max_prefill=64)
    llm.set_option("att_nw_batch" if args.rows > 1 else "att_nw", args.nw)
    for L in [int(s) for s in args.lens.split(",")]:
        us = llm.bench_attention(L, args.rows, args.cpw, 0)
        kv = args.rows * L * cfg.kv_heads * 128 * 2 * 2
        print(json.dumps({"rows": args.rows, "L": L, "cpw": args.cpw, "nw": args.nw,
                          "us": round(us, 2), "kv_MB": round(kv / 1e6, 2),
                          "GB/s": round(kv / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
