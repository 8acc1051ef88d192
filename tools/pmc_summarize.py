#!/usr/bin/env python3
"""Summarise the rocprofv3 output of tools/pmc_passes.sh into one JSON file of
per-kernel averages (duration from the kernel trace, counters from the PMC
passes), with the gfx950 FETCH_SIZE correction applied (MI355X_MICROARCH.md,
HBM section: FETCH_SIZE tallies 128-B requests at 64 B -> x2).

    python tools/pmc_summarize.py gpurun_out/pmc profiles/r01/pmc_summary.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    """kernel family name: strip namespaces, template args and the signature"""
    n = name.replace("(anonymous namespace)::", "")
    n = (n[5:] if n.startswith("void ") else n).split("(")[0]
    m = re.match(r"([A-Za-z_0-9:]+)(<.*>)?", n.strip())
    return (m.group(1) + (m.group(2) or "")) if m else n


def read_counters(root):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            per = defaultdict(lambda: defaultdict(float))  # (dispatch) -> counter -> sum
            names = {}
            for row in csv.DictReader(fh):
                d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                names[d] = short(row["Kernel_Name"])
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
            for d, cs in per.items():
                for c, v in cs.items():
                    vals[names[d]][c].append(v)
    return vals


def read_stats(root):
    out = {}
    for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                out[short(row["Name"])] = {"calls": int(row["Calls"]),
                                           "avg_us": float(row["AverageNs"]) / 1000.0,
                                           "min_us": float(row["MinNs"]) / 1000.0,
                                           "max_us": float(row["MaxNs"]) / 1000.0,
                                           "pct": float(row["Percentage"])}
    return out


def main(src, dst):
    summary = {"source": "tools/pmc_passes.sh (rocprofv3, ROCm 7.2, gfx950)",
               "fetch_size_correction": 2.0,
               "kernel_trace_bench": read_stats(os.path.join(src, "kt")),
               "kernel_trace_eager": read_stats(os.path.join(src, "kt_eager")),
               "counters": {}}
    for sub in ("fetch", "write", "l2", "sq"):
        for k, cs in read_counters(os.path.join(src, sub)).items():
            ent = summary["counters"].setdefault(k, {})
            for c, v in cs.items():
                ent[c] = sum(v) / len(v)
                ent[c + "_dispatches"] = len(v)
    # the EMD training call's own pass (tools/profile_kernels.py emdtrain)
    emdt = {}
    for k, cs in read_counters(os.path.join(src, "sq_emdtrain")).items():
        ent = emdt.setdefault(k, {})
        for c, v in cs.items():
            ent[c] = sum(v) / len(v)
            ent[c + "_dispatches"] = len(v)
    if emdt:
        summary["counters_emd_training_call"] = emdt
        summary["kernel_trace_emd_training_call"] = read_stats(os.path.join(src, "kt_emdtrain"))
    for k, ent in summary["counters"].items():
        if "FETCH_SIZE" in ent:  # KB per dispatch -> bytes, corrected
            ent["hbm_read_bytes"] = ent["FETCH_SIZE"] * 1024.0 * 2.0
        if "WRITE_SIZE" in ent:
            ent["hbm_write_bytes"] = ent["WRITE_SIZE"] * 1024.0
        if "hbm_read_bytes" in ent and "hbm_write_bytes" in ent:
            ent["hbm_bytes"] = ent["hbm_read_bytes"] + ent["hbm_write_bytes"]
        if "TCC_HIT_sum" in ent and "TCC_MISS_sum" in ent:
            tot = ent["TCC_HIT_sum"] + ent["TCC_MISS_sum"]
            ent["l2_hit_rate"] = ent["TCC_HIT_sum"] / tot if tot else None
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    for k, ent in sorted(summary["counters"].items()):
        print(k, {c: round(v, 3) if isinstance(v, float) else v for c, v in ent.items()
                  if not c.endswith("_dispatches")})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
