"""Prefill timing of the full Orpheus-3B shape (synthetic weights): one prompt of n ids through
all 28 layers + lm_head (the multi-row GEMM at R = n rows), bf16 and fp8 weights (diagnostic).

    python scripts/prefill_time.py [--lens 16,64,256,512] [--fp8]

Prints ms per prefill and the GEMM rate: 2 * 3.30 G params * n FLOP / time."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="16,64,128,256,512")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--opt", action="append", default=[], help="engine option key=value")
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
    lens = [int(s) for s in args.lens.split(",")]
    llm = LlmEngine(cfg, w, device=0, max_slots=1, max_pos=2048, max_batch=1,
                    max_prefill=max(lens), wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    for kv in args.opt:
        k, v = kv.split("=")
        llm.set_option(k, int(v))
    st = torch.cuda.Stream()
    params = 3_300_864_000
    for n in lens:
        ids = [1000 + (i * 7919) % 120000 for i in range(n)]
        llm.prefill(0, 0, ids, 1.1, st)
        st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.reps):
            llm.prefill(0, 0, ids, 1.1, st)
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(json.dumps({"n": n, "opts": args.opt, "wdtype": "fp8" if args.fp8 else "bf16", "ms": round(ms, 3),
                          "TFLOP/s": round(2 * params * n / (ms * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
