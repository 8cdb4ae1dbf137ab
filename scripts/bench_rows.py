"""Decode GEMV/GEMM efficiency by row count (full Orpheus-3B shapes, synthetic weights).

    python scripts/bench_rows.py [--rows 1,2,4,8,16,32,64] [--fp8] [--profile-rows 32]

For every row count: µs per launch of qkv / o_proj / gate_up / down (hipGraph sweep over the
28 layers) and the weight-stream rate; then one eager per-class profile of a full decode
step at --profile-rows rows (position ~600)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1,2,4,8,16,32,64")
    ap.add_argument("--fp8", action="store_true")
    ap.add_argument("--profile-rows", type=int, default=32)
    ap.add_argument("--pos", type=int, default=600)
    ap.add_argument("--options", default="", help="k=v,k=v set_option knobs")
    args = ap.parse_args()
    import torch
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import synthetic_llm_weights
    rows = [int(r) for r in args.rows.split(",")]
    R = max(rows + [max(1, args.profile_rows)])
    cfg = C.OrpheusConfig()
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    if args.fp8:
        from project_morpheus_amd.weights import quantize_fp8
        w = quantize_fp8(w, cfg)
    llm = LlmEngine(cfg, w, device=0, max_slots=R, max_pos=2048, max_batch=R, max_prefill=256,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    for kv in filter(None, args.options.split(",")):
        k, v = kv.split("=")
        llm.set_option(k, int(v))
    out = {}
    for r in rows:
        line = {}
        for kind in ("qkv", "o_proj", "gate_up", "down"):
            us, nb = llm.bench_gemv(kind, reps=4, n_rows=r)
            line[kind] = {"us": round(us, 2), "GB/s": round(nb / us / 1e3, 1)}
        tot = sum(v["us"] for v in line.values())
        line["sum_us"] = round(tot, 2)
        out[r] = line
        print(f"rows {r}: " + json.dumps(line), flush=True)
    st = torch.cuda.Stream()
    P = args.profile_rows
    if P <= 0:
        return
    prompt = list(range(1000, 1020))
    for i in range(P):
        llm.prefill(i, i, prompt, 1.1, st)
    for _ in range(args.pos - len(prompt)):
        llm.decode(P, st)
    prof = {}
    n = 8
    for _ in range(n):
        for k, v in llm.decode_profiled(P, st).items():
            prof[k] = prof.get(k, 0.0) + v / n
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(20):
        llm.decode(P, st)
    e1.record(st)
    e1.synchronize()
    print(json.dumps({"profile_rows": P, "pos": args.pos,
                      "eager_us_by_class": {k: round(1e3 * v, 1) for k, v in prof.items()},
                      "graph_step_ms": round(e0.elapsed_time(e1) / 20, 4)}), flush=True)


if __name__ == "__main__":
    main()
