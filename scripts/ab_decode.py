"""A/B decode-step variants on the full Orpheus-3B shape (synthetic weights), one process,
interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

    python scripts/ab_decode.py [--pos 1200] [--reps 50] [--rounds 3]

Each variant is a dict of mx_llm_set_option knobs; prints the hipGraph replay time of one
B=1 step at position --pos for every round, and the median."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULTS = {"legacy_gemv": 0, "att_cpw": 0, "att_cpw_batch": 0, "att_nw": 4, "att_nw_batch": 8,
            "gemv_wpb": 4, "rpw_o": 0, "rpw_gu": 0, "rpw_down": 0, "rows_lds_pad": 0,
            "o_merge": 1, "rows_frag": 1, "rows_target": 0, "rows_pw": 2, "rows_pw_f8": 2,
            "rows_head_mt": 1, "rows_head_target": 0, "rows_nt_max": 0, "rows_nt1": 2, "head_b1": 1, "rows_merge": 1, "engine_slots": 7, "engine_depth": 2, "engine_loaders": 2, "b1_engine": 0, "rows_atomic": 1, "rows_qkv_parts": 1,
            "rows_target_qkv": 0, "rows_target_o": 0, "rows_target_gu": 0, "rows_target_down": 0,
            "att_nw6": 1, "gemv_balance": 1, "att_b1_short": 1, "att_b1_nw6": 1}
VARIANTS = {
    "base": {},
    "no_nw6": {"att_nw6": 0},
    "short0": {"att_b1_short": 0},
    "short2": {"att_b1_short": 2},
    "no_balance": {"gemv_balance": 0},
    "no_b1_nw6": {"att_b1_nw6": 0},
    "b1_61": {"att_cpw": 1, "att_nw": 6},
    "b1_32": {"att_cpw": 2, "att_nw": 3},
    "b1_81": {"att_cpw": 1, "att_nw": 8},
    "ticket": {"o_merge": 0, "att_cpw": 1},
    "rpw_o2": {"rpw_o": 2},
    "cpw2": {"att_cpw": 2},
    "cpw2_rpw_o2": {"att_cpw": 2, "rpw_o": 2},
    "rpw_gu4": {"rpw_gu": 4},
    "rpw_gu2": {"rpw_gu": 2},
    "wpb8_down2": {"gemv_wpb": 8, "rpw_down": 2},
    "rpw_down2": {"rpw_down": 2},
    "wpb8": {"gemv_wpb": 8},
    "gu4_down2": {"rpw_gu": 4, "rpw_down": 2},
    "rowmajor": {"rows_frag": 0},
    "t128": {"rows_target": 128},
    "t256": {"rows_target": 256},
    "t384": {"rows_target": 384},
    "t512": {"rows_target": 512},
    "pw1": {"rows_pw": 1},
    "f8pw1": {"rows_pw_f8": 1},
    "t96": {"rows_target": 96},
    "nw8": {"att_cpw": 1, "att_nw": 8},
    "hmt1": {"rows_head_mt": 1},
    "hmt2": {"rows_head_mt": 2},
    "nt1_none": {"rows_nt1": 0},
    "nt1_q": {"rows_nt1": 1},
    "nt1_d": {"rows_nt1": 8},
    "nt1_qd": {"rows_nt1": 9},
    "nt1_o": {"rows_nt1": 2},
    "nt1_oq": {"rows_nt1": 3},
    "nt1_od": {"rows_nt1": 10},
    "nt1_oqd": {"rows_nt1": 11},
    "nt1_ogu": {"rows_nt1": 6},
    "nt1_oh": {"rows_nt1": 18},
    "nt1_all": {"rows_nt1": 15},
    "nohead1": {"head_b1": 0},
    "tmerge": {"rows_merge": 0},
    "nwb4": {"att_nw_batch": 4},
    "cpwb2": {"att_cpw_batch": 2},
    "cpwb4": {"att_cpw_batch": 4},
    "cpwb6": {"att_cpw_batch": 6},
    "ht1024": {"rows_head_target": 1024},
    "ht2048": {"rows_head_target": 2048},
    "ht4096": {"rows_head_target": 4096},
    "hmt1_ht2048": {"rows_head_mt": 1, "rows_head_target": 2048},
    "seam": {"rows_atomic": 0, "rows_qkv_parts": 0},
    "qkvseam": {"rows_qkv_parts": 0},
    "tq192": {"rows_target_qkv": 192},
    "tq256": {"rows_target_qkv": 256},
    "tq384": {"rows_target_qkv": 384},
    "td96": {"rows_target_down": 96},
    "td256": {"rows_target_down": 256},
    "td384": {"rows_target_down": 384},
    "tgu384": {"rows_target_gu": 384},
    "to384": {"rows_target_o": 384},
    "atomic": {"rows_atomic": 1},
    "atomic_t384": {"rows_atomic": 1, "rows_target": 384},
    "atomic_t128": {"rows_atomic": 1, "rows_target": 128},
    "atomic_nt1q": {"rows_atomic": 1, "rows_nt1": 1},
    "engine": {"b1_engine": 1},
    "engine_s6": {"b1_engine": 1, "engine_slots": 6},
    "engine_s5": {"b1_engine": 1, "engine_slots": 5},
    "engine_d3": {"b1_engine": 1, "engine_depth": 3},
    "engine_l1": {"b1_engine": 1, "engine_loaders": 1},
    "engine_l1d3": {"b1_engine": 1, "engine_loaders": 1, "engine_depth": 3},
    "engine_d3s6": {"b1_engine": 1, "engine_depth": 3, "engine_slots": 6},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pos", default="300,600,1100")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--rows", type=int, default=1)
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
    R = args.rows
    llm = LlmEngine(cfg, w, device=0, max_slots=R, max_pos=2048, max_batch=R, max_prefill=256,
                    wdtype="fp8" if args.fp8 else "bf16")
    del w
    torch.cuda.empty_cache()
    st = torch.cuda.Stream()
    prompt = list(range(1000, 1020))
    names = args.variants.split(",")
    positions = [int(p) for p in str(args.pos).split(",")]
    res = {(n, p): [] for n in names for p in positions}
    for rnd in range(args.rounds):
        for name in names:
            opts = dict(DEFAULTS, **VARIANTS[name])
            for k, v in opts.items():
                try:
                    llm.set_option(k, v)
                except Exception:  # an older library (MORPHEUS_MX_LIB) without this knob
                    if v != DEFAULTS.get(k) or k in VARIANTS[name]:
                        raise
            for pos in positions:
                for r in range(R):
                    llm.prefill(r, r, prompt, 1.1, st)
                for _ in range(pos - len(prompt)):
                    llm.decode(R, st)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.reps):
                    llm.decode(R, st)
                e1.record(st)
                e1.synchronize()
                res[(name, pos)].append(round(e0.elapsed_time(e1) / args.reps, 4))
                for r in range(R):
                    llm.release_row(r, st)
                st.synchronize()
        print(f"round {rnd}: " + json.dumps({f"{n}@{p}": res[(n, p)][-1]
                                            for n in names for p in positions}), flush=True)
    for n in names:
        print(n, {p: statistics.median(res[(n, p)]) for p in positions}, flush=True)


if __name__ == "__main__":
    main()
