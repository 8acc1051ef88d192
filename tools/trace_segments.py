#!/usr/bin/env python3
"""Per-segment durations of one kernel in a rocprofv3 kernel trace: launches
separated by more than GAP_US of idle form one segment (the bench's warmup,
timed region, 200-launch graphs and the ~45 ms sustained run come out as
separate segments), each with its launch count, mean and median.

    python tools/trace_segments.py TRACE.csv 'KERNEL NAME PREFIX' [GAP_US]
"""
import csv
import statistics
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    gap_us = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(name)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if not rows:
        raise SystemExit("no launches of " + name)
    segs = [[]]
    for i, r in enumerate(rows):
        if i and (int(r["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1000.0 > gap_us:
            segs.append([])
        segs[-1].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    allv = [v for s in segs for v in s]
    print(f"{name}: {len(allv)} launches, mean {statistics.mean(allv):.2f} us; segments (gap > {gap_us:g} us) "
          f"of >= 10 launches:")
    singles = [s[0] for s in segs if len(s) == 1]
    for k, s in enumerate(segs):
        if len(s) >= 10:
            print(f"  segment {k:3d}: {len(s):5d} launches, mean {statistics.mean(s):6.2f}, median "
                  f"{statistics.median(s):6.2f} us")
    if singles:
        print(f"  single launches (eager side legs): {len(singles)}, mean {statistics.mean(singles):.2f} us")


if __name__ == "__main__":
    main()
