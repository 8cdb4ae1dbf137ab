"""SNAC window decode timing (diagnostic): ms per window for N frames x B windows."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="1x1,4x1,7x1,7x4,7x16,7x32", help="frames x batch list")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from project_morpheus_amd.engine import SnacDecoder
    from project_morpheus_amd.weights import synthetic_snac_weights
    dec = SnacDecoder(synthetic_snac_weights(), device=0, max_frames=7, max_batch=32)
    st = torch.cuda.Stream()
    out = {}
    for n, B in (tuple(int(v) for v in c.split("x")) for c in args.cases.split(",")):
        codes = torch.randint(0, 4096, (B, 7 * n), dtype=torch.int32, device="cuda")
        for _ in range(3):
            dec.decode(codes, seed=1, stream=st)
        st.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = args.reps
        e0.record(st)
        for i in range(reps):
            dec.decode(codes, seed=i, stream=st)
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out[f"N{n}_B{B}"] = {"ms_per_call": round(ms, 4), "ms_per_window": round(ms / B, 4)}
        print(f"N{n}_B{B}", json.dumps(out[f"N{n}_B{B}"]), flush=True)


if __name__ == "__main__":
    main()
