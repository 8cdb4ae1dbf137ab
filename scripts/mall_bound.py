"""On-die bound of the decode GEMVs: each kind's all-layer graph sweep (the roofline probe,
weights streamed from HBM) against the same sweep over layer 0 only (option bench_one_layer:
its weights stay resident in the 256 MiB Infinity Cache).  The difference is what a prefetch of
the next launch's weights into the Infinity Cache could buy at most.

    python scripts/mall_bound.py [--rows 1,8] [--fp8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1,8")
    ap.add_argument("--fp8", action="store_true")
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
    rows = [int(r) for r in args.rows.split(",")]
    R = max(rows)
    llm = LlmEngine(cfg, w, device=0, max_slots=R, max_pos=2048, max_batch=R, max_prefill=64,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    for r in rows:
        kinds = ["qkv", "o_proj_merge" if r == 1 else "o_proj", "gate_up", "down"]
        for kind in kinds:
            res = {}
            for one in (0, 1):
                llm.set_option("bench_one_layer", one)
                us, nb = llm.bench_gemv(kind, reps=4, n_rows=r)
                res["resident" if one else "streamed"] = round(us, 2)
            llm.set_option("bench_one_layer", 0)
            res.update(rows=r, kind=kind, wdtype="fp8" if args.fp8 else "bf16", weight_bytes=nb,
                       streamed_tbs=round(nb / res["streamed"] / 1e6, 2),
                       resident_tbs=round(nb / res["resident"] / 1e6, 2))
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
