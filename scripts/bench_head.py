"""lm_head launch time by row count and head option (full Orpheus-3B shapes, synthetic weights).

    python scripts/bench_head.py [--rows 2,4,8,16,32] [--fp8] [--variants base,mt1,t2048]

mx_llm_bench_gemv kind "lm_head": penalty + argmax epilogue over the 156,940-entry vocabulary,
timed in a hipGraph; prints µs per launch and the weight-stream rate per (rows, variant)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "base": {},
    "mt1": {"rows_head_mt": 1},
    "mt2": {"rows_head_mt": 2},
    "t1024": {"rows_head_target": 1024},
    "t2048": {"rows_head_target": 2048},
    "t4096": {"rows_head_target": 4096},
    "mt1_t2048": {"rows_head_mt": 1, "rows_head_target": 2048},
}
DEFAULTS = {"rows_head_mt": 1, "rows_head_target": 0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="2,4,8,16,32")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    import torch
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import synthetic_llm_weights
    rows = [int(r) for r in args.rows.split(",")]
    cfg = C.OrpheusConfig()
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    if args.fp8:
        from project_morpheus_amd.weights import quantize_fp8
        w = quantize_fp8(w, cfg)
    R = max(rows)
    llm = LlmEngine(cfg, w, device=0, max_slots=R, max_pos=1024, max_batch=R, max_prefill=64,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    for name in args.variants.split(","):
        for k, v in dict(DEFAULTS, **VARIANTS[name]).items():
            llm.set_option(k, v)
        line = {"variant": name, "fp8": args.fp8}
        for r in rows:
            us, nb = llm.bench_gemv("lm_head", reps=args.reps, n_rows=r)
            line[r] = {"us": round(us, 2), "GB/s": round(nb / us / 1e3, 1)}
        print(json.dumps(line), flush=True)
    llm.close()


if __name__ == "__main__":
    main()
