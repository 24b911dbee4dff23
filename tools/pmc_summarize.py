"""Summarize rocprofv3 PMC passes (tools/pmc_round.sh output) per window pair:
per-launch averages of each counter over the k_verify dispatches, plus derived
HBM bytes (FETCH_SIZE corrected per MI355X_MICROARCH.md §HBM) and rates.

    python3 tools/pmc_summarize.py gpurun_out/pmc > profiles/<name>.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                # the fast-path kernel only (not k_verify_slow's launches)
                if not row["Kernel_Name"].startswith("void k_verify<"):
                    continue
                key = (os.path.basename(os.path.dirname(f)), row["Dispatch_Id"])
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    avg = defaultdict(list)
    for (_, _), cs in per.items():
        for k, v in cs.items():
            avg[k].append(v)
    return {k: sum(v) / len(v) for k, v in avg.items()}


def main(root):
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "w*_*"))):
        c = load(d)
        g, q = os.path.basename(d)[1:].split("_")
        # items per dispatch from the SQ pass (64 per wave), so that a workload
        # whose launches are not all 1M items (e.g. a split batch) still gives
        # per-verify figures; the per-launch numbers are scaled to 1M items
        items = c["SQ_WAVES"] * 64 if c.get("SQ_WAVES") else float(1 << 20)
        scale = (1 << 20) / items
        r = {"windows": {"G": int(g), "Q": int(q)}, "items_per_launch": 1 << 20,
             "items_per_profiled_dispatch": items, "counters": c}
        if "FETCH_SIZE" in c:
            r["hbm_bytes_per_launch"] = (c["FETCH_SIZE"] * 1024 * 2 + c.get("WRITE_SIZE", 0) * 1024) * scale
        if "SQ_INSTS_VALU" in c:
            # per 64 verifies (one wave)
            r["valu_wave_instr_per_verify"] = c["SQ_INSTS_VALU"] * 64 / items
        if "GRBM_GUI_ACTIVE" in c and "SQ_BUSY_CYCLES" in c:
            r["valu_instr_per_simd_cycle"] = c["SQ_INSTS_VALU"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
            r["wait_inst_any_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
            r["active_valu_frac_of_wave_cycles"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        if "TCP_UTCL1_TRANSLATION_MISS_sum" in c:
            m, h = c["TCP_UTCL1_TRANSLATION_MISS_sum"], c.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0)
            r["utcl1_miss_rate"] = m / max(m + h, 1)
        if "TCP_TCC_READ_REQ_LATENCY_sum" in c:
            r["tcp_tcc_read_latency_cycles"] = (c["TCP_TCC_READ_REQ_LATENCY_sum"]
                                                / max(c.get("TCP_TCC_READ_REQ_sum", 1), 1))
        out[os.path.basename(d)] = r
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
