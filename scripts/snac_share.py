"""What the batched SNAC costs the configs[2] loop: the same 32-stream continuous-batching run
(bench.run_batched's arrivals and prompts, synthetic weights) with SNAC windows on (the bench)
and off (token streams only), wall seconds and decode steps of each.

    python scripts/snac_share.py [--streams 32] [--max-tokens 1200]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=32)
    ap.add_argument("--max-tokens", type=int, default=1200)
    args = ap.parse_args()
    import numpy as np
    import torch

    from project_morpheus_amd import config as C
    from project_morpheus_amd.config import synthetic_audio_ids
    from project_morpheus_amd import inference as I
    from project_morpheus_amd.batching import BatchSynthesizer, StreamRequest
    from project_morpheus_amd.engine import LlmEngine, SnacDecoder
    from project_morpheus_amd.weights import synthetic_llm_weights, synthetic_snac_weights
    cfg = C.OrpheusConfig()
    B = args.streams
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    llm = LlmEngine(cfg, w, device=0, max_slots=B, max_pos=2048, max_batch=B, max_prefill=512)
    del w
    torch.cuda.empty_cache()
    snac = SnacDecoder(synthetic_snac_weights(), device=0, max_frames=7, max_batch=B)
    syn = BatchSynthesizer(llm, snac, seed=0, compact=True)

    def requests(audio):
        rng = np.random.default_rng(4)
        t, out = 0.0, []
        for i in range(B):
            n = int(rng.integers(16, 65))
            ids = I.prompt_ids([int(x) for x in rng.integers(1000, 120000, n - 5)])
            out.append(StreamRequest(prompt_ids=ids, max_tokens=args.max_tokens, arrival=t,
                                     inject_ids=synthetic_audio_ids(args.max_tokens, seed=10 + i),
                                     stop_ids=(), audio=audio))
            t += float(rng.exponential(0.010))
        return out

    syn.run(requests(True))  # warmup: graphs for every row count
    for rnd in range(2):
        for audio in (True, False):
            reqs = requests(audio)
            syn.row_steps.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            wall = syn.run(reqs)
            torch.cuda.synchronize()
            steps = sum(syn.row_steps.values())
            print(json.dumps({"round": rnd, "snac": audio, "wall_s": round(wall, 3),
                              "host_s": round(time.perf_counter() - t0, 3), "decode_steps": steps,
                              "audio_s": round(sum(r.audio_seconds for r in reqs), 2)}), flush=True)
    llm.close()
    snac.close()


if __name__ == "__main__":
    main()
