"""Where the persistent single-stream step spends its time: control-wave event clocks.

    python scripts/mega_trace.py [--fp8] [--pos 600]

Runs full Orpheus-3B shapes (synthetic weights) to position --pos, enables option mega_trace,
replays one step and prints, per segment of a layer, the median over blocks and middle layers
and the max over blocks (microseconds).  Events (llm_mega.hip control wave):
 0 A_Q  1 Q signalled  2 Q counter seen (attention blocks)  3 attention done  4 all heads done
 5 B_Q (att staged)  6 A_O  7 O counter seen  8 B_O (h staged)  9 next K/V staged  10 A_G
 11 G counter seen  12 B_G (act staged)  13 A_D  14 D counter seen  15 B_D (h staged)"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEGMENTS = [  # name, from event (None = previous layer's 15), to event
    ("qkv_compute", ("prev", 15), 0), ("q_finalize", 0, 1), ("q_wait", 1, 2),
    ("attention", 2, 3), ("heads_wait", 1, 4), ("stage_att", 4, 5), ("o_compute", 5, 6),
    ("o_fin_wait", 6, 7), ("stage_h", 7, 8), ("kv_stage", 8, 9), ("gu_compute", 8, 10),
    ("g_fin_wait", 10, 11), ("stage_act", 11, 12), ("down_compute", 12, 13),
    ("d_fin_wait", 13, 14), ("stage_hq", 14, 15), ("layer", ("prev", 15), 15)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--pos", type=int, default=600)
    ap.add_argument("--ring", type=int, default=32)
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
    llm.set_option("mega", 1)
    llm.set_option("mega_ring", args.ring)
    st = torch.cuda.Stream()
    llm.prefill(0, 0, list(range(1000, 1020)), 1.1, st)
    for _ in range(args.pos - 20):
        llm.decode(1, 1.1, st)
    llm.set_option("mega_trace", 1)
    for _ in range(3):
        llm.decode(1, 1.1, st)
    st.synchronize()
    t = llm.mega_trace().astype(np.float64) / 100.0  # -> microseconds
    nl = cfg.layers
    att_blocks = np.where(t[:, 1, 3] > 0)[0]
    out = {"fp8": args.fp8, "pos": args.pos, "ring": args.ring, "att_blocks": int(len(att_blocks)),
           "step_us": round(float(t[:, nl - 1, 15].max() - t[:, 0, 0].min()), 1)}
    seg = {}
    for name, a, b in SEGMENTS:
        vals = []
        for l in range(1, nl - 1):
            ta = t[:, l - 1, 15] if a == ("prev", 15) else t[:, l, a]
            tb = t[:, l, b]
            blocks = att_blocks if name in ("q_wait", "attention") else np.arange(256)
            vals.append((tb - ta)[blocks])
        v = np.stack(vals)
        seg[name] = {"med": round(float(np.median(v)), 2), "max": round(float(v.max(axis=1).mean()), 2)}
    out["segments_us"] = seg
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
