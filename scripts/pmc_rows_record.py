"""Build profiles/rNN_pmc_rows{8,8fp8,32}.json from scripts/gpu_pmc_rows_kinds.sh summaries:
per projection kind of the multi-row GEMM (generation 4), HBM read / write bytes per launch
(FETCH_SIZE x 1024 x 2, gfx950 correction; WRITE_SIZE x 1024) against the weight bytes, and the
SQ pass (wait / issue / MFMA fractions of wave cycles).

    python scripts/pmc_rows_record.py OUT_DIR [ROUND_PREFIX, default r06]"""
import json
import os
import re
import sys

H, QKV, F = 3072, 5120, 8192


def kind_of(name):
    m = re.search(r"gemm_rows_kernel<(\d+), (\d+), (\d+), (\w+), (\d+), (\w+), (\d+), (\d+)>", name)
    if not m:
        return None
    epi, sub = int(m.group(3)), int(m.group(5))
    if epi == 3:
        return "qkv"
    if epi == 2:
        return "gate_up"
    if epi == 1:  # K = 3,072 (o-proj) has 24 sub-chunks, K = 8,192 (down) 64
        return "o_proj" if sub % 3 == 0 else "down"
    return None


def main():
    out_dir = sys.argv[1]
    prefix = sys.argv[2] if len(sys.argv) > 2 else "r06"
    for tag, esz in (("rows8", 2), ("rows8fp8", 1), ("rows32", 2)):
        weights = {"qkv": QKV * H * esz, "o_proj": H * H * esz, "gate_up": 2 * F * H * esz,
                   "down": H * F * esz}
        rec = {"source": (f"scripts/gpu_pmc_rows_kinds.sh: rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE and an "
                          f"8-counter SQ pass (separate runs) over scripts/pmc_gemv.py ({tag}): one "
                          "hipGraph sweep of all 28 layers per kind; hbm_read_bytes = FETCH_SIZE x 1024 x 2 "
                          "(MI355X_MICROARCH.md gfx950 correction), medians per launch"),
               "kernels": {}}
        for pass_ in ("FETCH_SIZE", "WRITE_SIZE", "SQ"):
            path = os.path.join(out_dir, f"{tag}.{pass_}.summary.jsonl")
            if not os.path.exists(path):
                continue
            for line in open(path):
                d = json.loads(line)
                k = kind_of(d["kernel"])
                if not k:
                    continue
                e = rec["kernels"].setdefault(k, {"kernel": d["kernel"], "weight_bytes": weights[k]})
                if d["counter"] == "FETCH_SIZE":
                    e["hbm_read_bytes"] = d["hbm_read_bytes"]
                elif d["counter"] == "WRITE_SIZE":
                    e["hbm_write_bytes"] = d["hbm_write_bytes"]
                else:
                    e[d["counter"]] = d["median"]
        for e in rec["kernels"].values():
            if "hbm_read_bytes" in e:
                e["read_over_weight_bytes"] = round(e["hbm_read_bytes"] / e["weight_bytes"], 4)
            wc = e.get("SQ_WAVE_CYCLES")
            if wc:
                for c, f in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                             ("SQ_ACTIVE_INST_ANY", "active_inst_frac")):
                    if c in e:
                        e[f] = round(e[c] / wc, 4)
        path = os.path.join(out_dir, f"{prefix}_pmc_{tag}.json")
        json.dump(rec, open(path, "w"), indent=1)
        print(path, json.dumps({k: {x: v.get(x) for x in ("read_over_weight_bytes", "wait_any_frac",
                                                          "active_inst_frac")}
                                for k, v in rec["kernels"].items()}))


if __name__ == "__main__":
    main()
