"""profiles/r03_pmc_step.json from gpu_pmc_r03.sh's summaries: HBM bytes per launch of the
one-launch step kernel against its algorithmic bytes (weights + KV at the traced position)."""
import json
import os
import sys

out, args = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
rows = {}
for name in ("fetch", "write", "sq"):
    with open(os.path.join(out, name + ".summary.jsonl")) as fh:
        for line in fh:
            r = json.loads(line)
            rows.setdefault(r["counter"], r)
pos = 600
for tok in args.split("--"):
    if tok.strip().startswith("pos"):
        pos = int(tok.split()[1])
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from project_morpheus_amd.config import OrpheusConfig  # noqa: E402
cfg = OrpheusConfig()
alg = cfg.step_weight_bytes() + (pos + 3) * cfg.kv_bytes_per_position()
rd = rows["FETCH_SIZE"]["hbm_read_bytes"]
wr = rows["WRITE_SIZE"]["hbm_write_bytes"]
sq = {k: rows[k]["median"] for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                     "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES") if k in rows}
rec = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ (separate passes, "
                 f"scripts/gpu_pmc_r03.sh) over scripts/trace_step.py {args}: medians over the "
                 "traced step launches; hbm_read_bytes = FETCH_SIZE x 1024 x 2 (gfx950 "
                 "correction, MI355X_MICROARCH.md HBM)",
       "kernels": {"step": {"kernel": rows["FETCH_SIZE"]["kernel"], "algorithmic_bytes": alg,
                            "hbm_read_bytes": rd, "hbm_write_bytes": wr,
                            "traffic_bytes": rd + wr,
                            "traffic_over_algorithmic": round((rd + wr) / alg, 4),
                            "sq": sq,
                            "sq_wait_any_frac": round(sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"], 4)
                            if "SQ_WAIT_ANY" in sq and sq.get("SQ_WAVE_CYCLES") else None}}}
print(json.dumps(rec, indent=1))
