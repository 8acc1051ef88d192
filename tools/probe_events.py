#!/usr/bin/env python3
"""Does recording the timing events inside the bench's timed region cost wall
time?  The one-launch Chamfer step (the bench's clouds, --steps 20 --warmup 5
shape), interleaved trials of three region forms per launch form:

    wall      sync; t0; K launches; sync; t1                 (no events)
    ev_in     sync; t0; e0; K launches; e1; sync; t1         (bench.py round-5 form)
    ev_out    sync; e0; t0; K launches; e1; sync; t1         (start event before the clock)

    python tools/probe_events.py
"""
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def region(fn, K, dev, s, form):
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if form == "ev_out":
        e0.record(s)
    t0 = time.perf_counter()
    if form == "ev_in":
        e0.record(s)
    fn(K)
    if form != "wall":
        e1.record(s)
    torch.cuda.synchronize(dev)
    t = (time.perf_counter() - t0) * 1e6 / K
    ev = e0.elapsed_time(e1) * 1000.0 / K if form != "wall" else float("nan")
    return t, ev


def main():
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    K, W = 20, 5
    step = bench.ChamferStep(dev, 1, seed=bench.BENCH_SEED, slots=K)
    for _ in range(3):
        step(0)
    torch.cuda.synchronize(dev)
    go = step.launcher()
    g = bench.capture_steps(step, K, dev, 1, False)
    g.replay()
    torch.cuda.synchronize(dev)
    launch = {"c_loop": (lambda k: go(k)), "graph20": (lambda k: g.replay())}
    forms = ("wall", "ev_in", "ev_out")
    res = {(l, f): [] for l in launch for f in forms}
    for trial in range(10):
        for l, fn in launch.items():
            for f in forms:
                go(W) if l == "c_loop" else g.replay()
                res[(l, f)].append(region(fn, K, dev, s, f))
    for (l, f), rows in res.items():
        w = statistics.median(r[0] for r in rows)
        e = statistics.median(r[1] for r in rows)
        print(f"{l:8s} {f:7s} wall median {w:6.2f} us/step  events median {e:6.2f} us/step  wall-events {w - e:6.2f}"
              f"   [{' '.join(f'{r[0]:.2f}' for r in rows)}]", flush=True)
    print(f"kernel_avg_us (200-launch graph): {bench.kernel_avg_us(lambda: step(0), 200, dev):.2f}", flush=True)


if __name__ == "__main__":
    main()
