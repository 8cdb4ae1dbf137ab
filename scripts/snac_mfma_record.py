"""MFMA-utilisation and traffic record of SNAC's block-tiled conv-GEMM (conv_gemm_tiled_kernel<1>)
in the 7-frame x 32-window decode (configs[2]'s batched vocoder shape).

    python scripts/snac_mfma_record.py KERNEL_TRACE.csv SQ.csv FETCH.csv WRITE.csv

Every mx_snac_decode call launches the tiled kernel 21 times in a fixed order (capi.hip
snac_enqueue: the input 1x1 conv, then per DecoderBlock the ConvTranspose, the NoiseBlock and
three ResidualUnit 1x1 convs); dispatches are attributed to shapes by their position in that
order (tests/_snac_dispatch.py restates the same sequence).  Per shape:

* useful FLOPs = 2 M K N (fp32 operands: the GEMM the oracle computes), N = windows x Tin x
  phases; executed MFMA = 6 v_mfma_f32_16x16x32_bf16 per 16 x 16 x 32 step (the split-bf16
  operands) over the padded 128-column tiles;
* MFMA utilisation = executed MFMA x 16 cycles (one 16x16x32 bf16 per 16 cycles per SIMD,
  MI355X_MICROARCH.md cycle table) / (kernel duration x 2.4 GHz x 1,024 SIMDs), and the
  counter's own view SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1,024) next to it;
* HBM bytes = FETCH_SIZE x 1024 x 2 (gfx950 correction) + WRITE_SIZE x 1024.
"""
import csv
import json
import statistics
import sys

K_RATES = (8, 8, 4, 2)
B, NF = 32, 7
PEAK_BF16_TFLOPS = 2500.0   # dense bf16 MFMA, MI355X_MICROARCH.md
CLOCK_HZ = 2.4e9
SIMDS = 1024


def shapes():
    T = 4 * NF
    out = [("in.pw", 1024, 768, T, 1)]
    for b in range(4):
        cin = 1024 >> b
        cout = cin // 2
        out.append((f"b{b}.up", cout, 2 * cin, T, K_RATES[b]))
        T *= K_RATES[b]
        out.append((f"b{b}.noise", cout, cout, T, 1))
        out += [(f"b{b}.r{r}.pw", cout, cout, T, 1) for r in range(3)]
    return out


def rows(path, name="conv_gemm_tiled"):
    with open(path) as fh:
        rs = [r for r in csv.DictReader(fh) if name in (r.get("Kernel_Name") or "")]
    return sorted(rs, key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))


def by_dispatch(path, counter):
    d = {}
    for r in rows(path):
        if r.get("Counter_Name") == counter:
            d.setdefault(int(r["Dispatch_Id"]), 0.0)
            d[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def main():
    kt, sq, fetch, write = sys.argv[1:5]
    S = shapes()
    n = len(S)
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in rows(kt)]
    ctr = {c: by_dispatch(sq, c) for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
                                           "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY")}
    ctr["FETCH_SIZE"] = by_dispatch(fetch, "FETCH_SIZE")
    ctr["WRITE_SIZE"] = by_dispatch(write, "WRITE_SIZE")
    rec = {"source": "scripts/gpu_r06_c.sh: rocprofv3 --kernel-trace and three --pmc passes over "
                     "scripts/bench_snac.py --cases 7x32 --reps 3; medians per shape over the calls",
           "peak_bf16_tflops": PEAK_BF16_TFLOPS, "shapes": []}
    tot = {"dur": 0.0, "useful": 0.0, "exec": 0.0}
    for i, (name, M, K, Tin, nph) in enumerate(S):
        d = dur[i::n]
        N = B * Tin * nph
        useful = 2.0 * M * K * N
        cols = -(-(B * Tin) // 128) * 128
        n_mfma = (M // 16) * (cols // 16) * (K // 32) * nph * 6
        t = statistics.median(d) if d else float("nan")
        e = {"shape": name, "M": M, "K": K, "N": N, "launches": len(d), "us": round(t * 1e6, 2),
             "useful_tflops": round(useful / t / 1e12, 1),
             "executed_bf16_tflops": round(2.0 * 16 * 16 * 32 * n_mfma / t / 1e12, 1),
             "mfma_util": round(n_mfma * 16 / (t * CLOCK_HZ * SIMDS), 3)}
        c = {k: statistics.median(v[i::n]) for k, v in ctr.items() if v[i::n]}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            e["ctr_mfma_busy_over_active"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                                   (c["GRBM_GUI_ACTIVE"] / 8 * SIMDS), 3)
            e["ctr_mfma_busy_over_predicted"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (n_mfma * 16), 3)
        if c.get("SQ_WAVE_CYCLES"):
            e["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
            e["active_inst_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
        if "FETCH_SIZE" in c:
            e["hbm_read_mb"] = round(c["FETCH_SIZE"] * 2048 / 1e6, 2)
        if "WRITE_SIZE" in c:
            e["hbm_write_mb"] = round(c["WRITE_SIZE"] * 1024 / 1e6, 2)
        rec["shapes"].append(e)
        tot["dur"] += t
        tot["useful"] += useful
        tot["exec"] += 2.0 * 16 * 16 * 32 * n_mfma
    rec["all_tiled_launches"] = {
        "us_per_call": round(tot["dur"] * 1e6, 1),
        "useful_tflops": round(tot["useful"] / tot["dur"] / 1e12, 1),
        "executed_bf16_tflops": round(tot["exec"] / tot["dur"] / 1e12, 1),
        "executed_over_peak": round(tot["exec"] / tot["dur"] / 1e12 / PEAK_BF16_TFLOPS, 3)}
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
