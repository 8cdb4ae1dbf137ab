"""Diagnostic: max |GPU - oracle| logits over a batched run, MFMA rows path vs legacy."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import llama_ref as L  # noqa: E402
from project_morpheus_amd import config as C  # noqa: E402
from project_morpheus_amd.engine import LlmEngine  # noqa: E402
from project_morpheus_amd.weights import synthetic_llm_weights  # noqa: E402


def run(cfg, w, prompts, steps, legacy):
    B = len(prompts)
    eng = LlmEngine(cfg, w, device=0, max_slots=B, max_pos=512, max_batch=B, max_prefill=256)
    eng.set_option("legacy_gemv", legacy)
    eng.enable_logits()
    st = torch.cuda.Stream()
    toks = [[] for _ in range(B)]
    logits = [[] for _ in range(B)]
    for r, p in enumerate(prompts):
        eng.prefill(r, r, p, 1.1, st)
    for k in range(steps):
        if k > 0:
            eng.decode(B, st)
        st.synchronize()
        for r, p in enumerate(prompts):
            logits[r].append(eng.read_logits(r, st))
            toks[r].append(int(eng.hist[r, len(p) + k]))
    eng.close()
    return toks, logits


def main():
    cfg = C.OrpheusConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024, vocab=1000)
    w = synthetic_llm_weights(cfg, seed=31, std=0.05, norm_jitter=0.5)
    rng = np.random.default_rng(7)
    prompts = [[int(x) for x in rng.integers(0, cfg.vocab, 5 + 2 * i)] for i in range(20)]
    ref = L.LlamaRef(L.RefConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024,
                                 vocab=1000), w, max_pos=512)
    for legacy in (0, 1):
        toks, logits = run(cfg, w, prompts, 12, legacy)
        d0, dall = [], []
        for r, p in enumerate(prompts):
            _, rl = L.greedy_generate(ref, p, 12, 1.1, return_logits=True, forced=toks[r])
            for k in range(12):
                dd = np.abs(logits[r][k] - rl[k].numpy())
                dall.append(dd.max())
                if k == 0:
                    d0.append(dd.max())
        print(f"legacy={legacy}: step0 max {max(d0):.2e} median {np.median(d0):.2e}; "
              f"all max {max(dall):.2e} median {np.median(dall):.2e}", flush=True)
    # no-rounding oracle (fp32 KV) against the same GPU run: how much is bf16-KV flips?
    ref32 = L.LlamaRef(L.RefConfig(hidden=512, layers=2, heads=4, kv_heads=2, ffn=1024,
                                   vocab=1000), w, max_pos=512, round_kv=False)
    toks, logits = run(cfg, w, prompts, 12, 0)
    d = []
    for r, p in enumerate(prompts):
        _, rl = L.greedy_generate(ref32, p, 12, 1.1, return_logits=True, forced=toks[r])
        d += [np.abs(logits[r][k] - rl[k].numpy()).max() for k in range(12)]
    print(f"vs fp32-KV oracle: max {max(d):.2e} median {np.median(d):.2e}")


if __name__ == "__main__":
    main()
