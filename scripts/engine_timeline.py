"""Phase timeline of the persistent one-row engine (option b1_engine) on the full Orpheus-3B
shape: one traced step at --pos, per layer the median over CUs of each phase's span (µs), and
the loader's streaming span.

    python scripts/engine_timeline.py [--pos 600] [--fp8] [--slots 7] [--depth 2]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["in_wait", "qkv", "attn", "o_wait", "o", "gu_wait", "gu", "down_wait", "down"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pos", type=int, default=600)
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--slots", type=int, default=7)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--loaders", type=int, default=2)
    ap.add_argument("--dbg", type=int, default=0, help="1: no hand-off waits, 2: no weight stream")
    args = ap.parse_args()
    import torch
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import quantize_fp8, synthetic_llm_weights
    cfg = C.OrpheusConfig()
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    if args.fp8:
        w = quantize_fp8(w, cfg)
    llm = LlmEngine(cfg, w, device=0, max_slots=1, max_pos=2048, max_batch=1, max_prefill=64,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    llm.set_option("engine_slots", args.slots)
    llm.set_option("engine_depth", args.depth)
    llm.set_option("engine_loaders", args.loaders)
    llm.set_option("b1_engine", 1)
    llm.set_option("engine_trace", 1)
    llm.set_option("engine_dbg", args.dbg)
    st = torch.cuda.Stream()
    prompt = list(range(1000, 1020))
    llm.prefill(0, 0, prompt, 1.1, st)
    for _ in range(args.pos - len(prompt)):
        llm.decode(1, st)
    st.synchronize()
    tr = llm.engine_trace().astype(np.int64)   # [G][layers][12]
    G, Lyr, _ = tr.shape
    t0 = tr[:, 0, 10].min()
    us = (tr - t0) / 100.0                       # 100 MHz -> µs
    out = {"pos": args.pos, "fp8": args.fp8, "slots": args.slots, "depth": args.depth,
           "dbg": args.dbg, "grid": G,
           "step_us": float(us[:, -1, 9].max()), "layers": []}
    for l in range(Lyr):
        row = {"layer": l, "start_med": round(float(np.median(us[:, l, 0])), 2)}
        for i, name in enumerate(PHASES):
            row[name] = round(float(np.median(us[:, l, i + 1] - us[:, l, i])), 2)
        row["layer_med"] = round(float(np.median(us[:, l, 9] - us[:, l, 0])), 2)
        row["loader_stream"] = round(float(np.median(us[:, l, 11] - us[:, l, 10])), 2)
        row["loader_lead"] = round(float(np.median(us[:, l, 0] - us[:, l, 10])), 2)
        out["layers"].append(row)
    mids = out["layers"][2:-2] or out["layers"]
    out["mid_layer_median"] = {k: round(float(np.median([r[k] for r in mids])), 2)
                               for k in PHASES + ["layer_med", "loader_stream"]}
    print(json.dumps(out["mid_layer_median"]))
    print(json.dumps({k: out[k] for k in ("pos", "fp8", "slots", "depth", "dbg", "grid", "step_us")}))
    for r in out["layers"][:3] + out["layers"][-2:]:
        print(json.dumps(r))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"engine_timeline_{'fp8' if args.fp8 else 'bf16'}"
                           f"_p{args.pos}_s{args.slots}_d{args.depth}_l{args.loaders}_x{args.dbg}.json"), "w") as fh:
        json.dump(out, fh)
    llm.close()


if __name__ == "__main__":
    main()
