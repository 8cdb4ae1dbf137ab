"""Decode steps of the full Orpheus-3B shape (synthetic weights) for a rocprofv3 kernel trace:
prefill, decode to --pos, then --steps traced steps (B = --rows).  Pair with step_gaps.py.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 scripts/trace_step.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pos", type=int, default=600)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--fp8", action="store_true")
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
    R = args.rows
    llm = LlmEngine(cfg, w, device=0, max_slots=R, max_pos=2048, max_batch=R, max_prefill=256,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    for kv in args.opt:
        k, v = kv.split("=")
        llm.set_option(k, int(v))
    st = torch.cuda.Stream()
    prompt = list(range(1000, 1020))
    for r in range(R):
        llm.prefill(r, r, prompt, 1.1, st)
    for _ in range(args.pos - len(prompt)):
        llm.decode(R, st)
    st.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.steps):
        llm.decode(R, st)
    e1.record(st)
    e1.synchronize()
    print(f"rows {R} pos {args.pos} {' '.join(args.opt)}: {e0.elapsed_time(e1) / args.steps:.4f} ms/step",
          flush=True)


if __name__ == "__main__":
    main()
