#!/usr/bin/env python3
"""Per-variant HBM-side bytes per launch of the one-launch Chamfer step from
the `pmcf` passes of tools/gpu_run.sh (rocprofv3 FETCH_SIZE and WRITE_SIZE of
`tools/profile_kernels.py fused V,...`): median over a variant's 20 launches,
FETCH_SIZE x2 (the MI355X guide's gfx950 correction) + WRITE_SIZE, with the
kernel trace's average duration.  usage: pmcf_summary.py gpurun_out/TAG"""
import collections
import csv
import re
import glob
import os
import statistics
import sys


def short(name):
    m = re.search(r"chamfer_loss_grad_kernel<[^>]*>", name)
    return m.group(0) if m else name


def per_dispatch(path):
    agg = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if "chamfer_loss_grad_kernel" not in r["Kernel_Name"]:
            continue
        agg[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
    out = collections.defaultdict(list)
    for d, v in agg.items():
        out[names[d]].append(v)
    return out


def main():
    base = sys.argv[1]
    fetch = per_dispatch(glob.glob(os.path.join(base, "pmcf_fetch", "*counter_collection.csv"))[0])
    write = per_dispatch(glob.glob(os.path.join(base, "pmcf_write", "*counter_collection.csv"))[0])
    dur = collections.defaultdict(list)
    for p in glob.glob(os.path.join(base, "pmcf_kt", "*kernel_trace.csv")):
        for r in csv.DictReader(open(p)):
            if "chamfer_loss_grad_kernel" in r["Kernel_Name"]:
                dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in fetch:
        f = statistics.median(fetch[k]) * 1024
        w = statistics.median(write.get(k, [0.0])) * 1024
        d = dur.get(k)
        print(f"{k}\n  fetch {f / 1e6:.3f} MB x2 + write {w / 1e6:.3f} MB = {(2 * f + w) / 1e6:.3f} MB per launch"
              + (f"; trace median {statistics.median(d):.2f} us over {len(d)} launches" if d else ""))


if __name__ == "__main__":
    main()
