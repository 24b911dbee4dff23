"""Summarize a rocprofv3 --kernel-trace --hip-runtime-trace run of
tools/single_call_probe.py: per lone call, hipLaunchKernel's API time, the
launch's return to the kernel's start, and the kernel itself.

    python tools/single_trace_summary.py gpurun_out/prof_sc_TAG OUT.json "note"
"""
import csv
import json
import sys
from collections import Counter

import numpy as np


def main() -> None:
    d, out, note = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""
    kt = list(csv.DictReader(open(d + "/sc_kernel_trace.csv")))
    api = list(csv.DictReader(open(d + "/sc_hip_api_trace.csv")))
    launch = {r["Correlation_Id"]: r for r in api if r["Function"] == "hipLaunchKernel"}
    res = {"source": note, "kernels": dict(Counter(k["Kernel_Name"].split("(")[0] for k in kt))}
    for name in sorted({k["Kernel_Name"].split("(")[0] for k in kt}):
        if not name.replace("void ", "").startswith("k_verify"):
            continue
        rows = []
        for k in kt:
            if k["Kernel_Name"].split("(")[0] != name or k["Correlation_Id"] not in launch:
                continue
            L = launch[k["Correlation_Id"]]
            rows.append(((int(L["End_Timestamp"]) - int(L["Start_Timestamp"])) / 1e3,
                         (int(k["Start_Timestamp"]) - int(L["End_Timestamp"])) / 1e3,
                         (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3))
        a = np.array(rows)
        res[name] = {nm: {"p10": float(np.percentile(a[:, i], 10)), "p50": float(np.median(a[:, i])),
                          "p90": float(np.percentile(a[:, i], 90))}
                     for i, nm in enumerate(["hipLaunchKernel_api_us", "launch_return_to_kernel_start_us",
                                             "kernel_us"])}
        res[name]["launches"] = len(a)
    res["hip_api_calls"] = dict(Counter(r["Function"] for r in api).most_common(10))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
