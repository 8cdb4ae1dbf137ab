"""Per-block phase timeline of the multi-row (generation 4) decode GEMMs, full Orpheus-3B shapes.

    python scripts/rows_block_trace.py [--rows 8,32] [--fp8] [--kinds qkv,o_proj,gate_up,down,lm_head]

Each kind's last-layer launch inside an all-layer hipGraph sweep records s_memrealtime stamps
(100 MHz) per block (include/morpheus_mx.h mx_llm_bench_gemv_trace).  Prints, per (rows, kind),
times in µs from the earliest block entry: the launch span, block entry spread, first weight
sub-chunk consumed, main loop end, split-K publish + ticket, last-arriver merge, epilogue end
(medians and maxima over blocks).  Needs the diagnostic library:

    MORPHEUS_MX_ROWS_TRACE=1 python -m project_morpheus_amd.build
    MORPHEUS_MX_LIB=project_morpheus_amd/libmorpheus_mx_trace.so python scripts/rows_block_trace.py"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarize(st):
    t = st.astype(np.float64) / 100.0  # µs
    ok = st[:, 0] > 0
    t, st = t[ok], st[ok]
    t0 = t[:, 0].min()
    rel = np.where(st > 0, t - t0, np.nan)
    out = {"blocks": int(len(t)), "span_us": round(float(np.nanmax(rel[:, 6])), 2)}
    names = ["entry", "x_staged", "first_w", "loop_end", "published", "merged", "end"]
    for k, n in enumerate(names):
        col = rel[:, k]
        col = col[~np.isnan(col)]
        if len(col):
            out[n] = {"p50": round(float(np.median(col)), 2), "max": round(float(col.max()), 2),
                      "n": int(len(col))}
    d = rel[:, 3] - rel[:, 0]
    out["loop_us_p50"] = round(float(np.nanmedian(d)), 2)
    seam = rel[:, 4] - rel[:, 3]
    if np.any(~np.isnan(seam)):
        out["publish_us_p50"] = round(float(np.nanmedian(seam)), 2)
        m = rel[:, 5] - rel[:, 4]
        out["merge_us_p50"] = round(float(np.nanmedian(m)), 2)
    e = rel[:, 6] - np.where(np.isnan(rel[:, 5]), rel[:, 3], rel[:, 5])
    out["epilogue_us_p50"] = round(float(np.nanmedian(e)), 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="8,32")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--kinds", default="qkv,o_proj,gate_up,down,lm_head")
    ap.add_argument("--options", default="", help="k=v,k=v set_option knobs")
    ap.add_argument("--raw", default="", help="write the raw stamps (npz) here")
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
    for kv in filter(None, args.options.split(",")):
        k, v = kv.split("=")
        llm.set_option(k, int(v))
    raw = {}
    for r in rows:
        for kind in args.kinds.split(","):
            us, nb = llm.bench_gemv(kind, reps=2, n_rows=r)
            st = llm.bench_gemv_trace(kind, r)
            raw[f"{kind}_r{r}"] = st
            s = summarize(st)
            print(json.dumps({"rows": r, "kind": kind, "graph_us": round(us, 2),
                              "weight_MB": round(nb / 1e6, 2), **s}), flush=True)
    if args.raw:
        np.savez_compressed(args.raw, **raw)
    llm.close()


if __name__ == "__main__":
    main()
