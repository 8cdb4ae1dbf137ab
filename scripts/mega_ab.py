"""Single-stream decode step: persistent launch (option mega=1) vs per-kernel launches (mega=0).

    python scripts/mega_ab.py [--fp8] [--pos 600] [--ring 32]

Full Orpheus-3B shapes, synthetic weights; graph-replayed steps timed with HIP events on the
engine's stream, alternating variants so drift hits both.  Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--pos", type=int, default=600)
    ap.add_argument("--ring", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=50)
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
    llm = LlmEngine(cfg, w, device=0, max_slots=2, max_pos=2048, max_batch=1, max_prefill=64,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    llm.set_option("mega_ring", args.ring)
    st = torch.cuda.Stream()
    llm.prefill(0, 0, list(range(1000, 1020)), 1.1, st)
    for _ in range(args.pos - 20):
        llm.decode(1, 1.1, st)
    st.synchronize()
    res = {"mega": [], "kernels": []}
    for _ in range(args.rounds):
        for name, on in (("mega", 1), ("kernels", 0)):
            llm.set_option("mega", on)
            for _ in range(3):
                llm.decode(1, 1.1, st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.steps):
                llm.decode(1, 1.1, st)
            e1.record(st)
            e1.synchronize()
            res[name].append(round(e0.elapsed_time(e1) / args.steps, 4))
    llm.set_option("mega", 1)
    info = llm.mega_info(st)
    out = {"fp8": args.fp8, "pos": args.pos, "ring": args.ring, "mega_info": info,
           "step_ms": {k: sorted(v)[len(v) // 2] for k, v in res.items()}, "all": res}
    wbytes = cfg.params() * (1 if args.fp8 else 2)
    for k in ("mega", "kernels"):
        out[k + "_TBps"] = round(wbytes / (out["step_ms"][k] * 1e-3) / 1e12, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
