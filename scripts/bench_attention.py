"""Attention kernel micro-benchmark vs context length (diagnostic)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import synthetic_llm_weights
    cfg = C.OrpheusConfig(layers=1, vocab=1024)
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    llm = LlmEngine(cfg, w, device=0, max_slots=32, max_pos=2048, max_batch=32, max_prefill=64)
    out = {}
    for rows in (1, 8, 32):
        for nw in (4, 8):
            llm.set_option("att_nw" if rows == 1 else "att_nw_batch", nw)
            for cpw in (1, 2, 4):
                key = f"rows{rows}_nw{nw}_cpw{cpw}"
                out[key] = {L: round(llm.bench_attention(L, rows, cpw, 0), 2)
                            for L in (64, 256, 512, 640, 1024, 1280, 2048)}
                print(key, json.dumps(out[key]), flush=True)


if __name__ == "__main__":
    main()
