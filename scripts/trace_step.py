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
    ap.add_argument("--timeline", action="store_true", help="per-stage timeline of one step")
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
    if args.timeline and R == 1:
        llm.set_option("step_trace", 1)
        for _ in range(3):
            llm.decode(1, st)
        tr = llm.step_trace(st)
        timeline_report(tr, cfg.layers)


def timeline_report(tr, layers):
    """Per-stage timeline of one one-launch step (us from the first block's entry)."""
    import numpy as np
    names = ["qkv", "att", "o", "gu", "down", "head", "finish"]
    t0 = tr[:, 0].min()
    us = lambda v: (v.astype(np.float64) - float(t0)) / 100.0  # noqa: E731  (100 MHz clock)
    role = (tr[:, 3] >> np.uint64(32)).astype(int)
    layer = (tr[:, 3] & np.uint64(0xFFFFFFFF)).astype(int)
    print(f"step span {(tr[:, 2].max() - t0) / 100.0:.1f} us, blocks {len(tr)}", flush=True)
    rows = []
    for l in list(range(layers)) + [-1]:
        for r, nm in enumerate(names):
            m = (role == r) & ((layer == l) if l >= 0 else (role >= 5))
            if l >= 0 and r >= 5 or l < 0 and r < 5 or not m.any():
                continue
            e, w, d = us(tr[m, 0]), us(tr[m, 1]), us(tr[m, 2])
            rows.append((l, nm, int(m.sum()), e.min(), e.max(), w.min(), w.max(), d.min(), d.max(),
                         float(np.median(w - e)), float(np.median(d - w))))
    print("layer stage  blocks  entry[min,max]   waitdone[min,max]   end[min,max]   "
          "med(wait-entry) med(end-wait)")
    for r in rows:
        if r[0] in (0, 1, 13, 27, -1):
            print(f"{r[0]:5d} {r[1]:6s} {r[2]:6d}  {r[3]:8.1f} {r[4]:8.1f}  {r[5]:8.1f} {r[6]:8.1f}  "
                  f"{r[7]:8.1f} {r[8]:8.1f}  {r[9]:7.2f} {r[10]:7.2f}")
    # per-layer span: first qkv entry -> last down end
    spans = [max(x[8] for x in rows if x[0] == l) - min(x[3] for x in rows if x[0] == l)
             for l in range(layers)]
    print("per-layer span us (first entry -> last end):", [round(v, 1) for v in spans[:6]], "...")
    ends = {(x[0], x[1]): x[8] for x in rows}
    gaps = [ends[(l, "down")] - ends[(l - 1, "down")] for l in range(1, layers)]
    print(f"layer period (down end to down end) median {sorted(gaps)[len(gaps) // 2]:.1f} us")


if __name__ == "__main__":
    main()
