"""Per-wave timestamps (s_memrealtime, 100 MHz) of one multi-row GEMM launch (rows_dbg=7)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "o_proj"
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    import torch
    from project_morpheus_amd import config as C
    from project_morpheus_amd.engine import LlmEngine
    from project_morpheus_amd.weights import synthetic_llm_weights
    cfg = C.OrpheusConfig()
    cfg.layers = 2
    w = synthetic_llm_weights(cfg, seed=0, device="cuda:0")
    llm = LlmEngine(cfg, w, device=0, max_slots=rows, max_pos=2048, max_batch=rows,
                    max_prefill=256)
    llm.bench_gemv(kind, reps=1, n_rows=rows)
    torch.cuda.synchronize()
    llm.set_option("rows_dbg", 1)
    sys.stdout.flush()
    llm.bench_gemv(kind, reps=1, n_rows=rows)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
