"""Build profiles/<name>.json (the bench's PMC traffic record) from the FETCH_SIZE / WRITE_SIZE
summaries of scripts/pmc_summary.py over scripts/pmc_gemv.py --rows 1.

    python scripts/pmc_gemv_record.py FETCH.summary.json WRITE.summary.json OUT.json SOURCE"""
import json
import sys

KINDS = {"gemv1_kernel<6, 2, 3,": ("qkv", 31457280), "gemv1_kernel<6, 1, 1, false, 4": ("o_proj", 18874368),
         "gemv1_kernel<6, 2, 2,": ("gate_up", 100663296), "gemv1_kernel<16, 1, 1,": ("down", 50331648),
         # the product's one-row o-proj: merges 8 attention splits in its prologue (weights only
         # counted as algorithmic; the split partials it re-reads are the difference)
         "gemv1_kernel<6, 2, 1, false, 8, false, 8>": ("o_proj_merge", 18874368),
         "head_b1_kernel<6, 2, false>": ("lm_head", 156940 * 3072 * 2)}


def main():
    fetch, write, out, source = sys.argv[1:5]
    rec = {"source": source, "kernels": {}}
    for path, key in ((fetch, "hbm_read_bytes"), (write, "hbm_write_bytes")):
        for line in open(path):
            d = json.loads(line)
            for pat, (kind, nbytes) in KINDS.items():
                if pat in d["kernel"]:
                    e = rec["kernels"].setdefault(kind, {"kernel": d["kernel"], "algorithmic_bytes": nbytes})
                    e[key] = d[key]
    for e in rec["kernels"].values():
        e["traffic_bytes"] = e.get("hbm_read_bytes", 0.0) + e.get("hbm_write_bytes", 0.0)
        e["traffic_over_algorithmic"] = round(e["traffic_bytes"] / e["algorithmic_bytes"], 4)
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
