#!/usr/bin/env python3
"""The bench's timed region as the driver runs it (--steps 20 --warmup 5),
repeated: per trial W warm launches, an idle gap, then K timed launches (wall
clock with synchronize on both sides, and HIP events at the region's edges),
for the direct C-loop form and the 20-step graph form -- to see what the
first timed launches cost after the GPU idles.

    python tools/probe_timed.py
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    K, W = 20, 5
    step = bench.ChamferStep(dev, 1, seed=bench.BENCH_SEED, slots=K)
    for _ in range(3):
        step(0)
    torch.cuda.synchronize(dev)
    go = step.launcher()
    g = bench.capture_steps(step, K, dev, 1, False)
    g.replay()
    torch.cuda.synchronize(dev)
    forms = {"c_loop": (lambda k: go(k)), "graph20": (lambda k: g.replay())}
    for gap_ms in (0.0, 1.0, 20.0):
        for name, fn in forms.items():
            rows = []
            for trial in range(6):
                if name == "c_loop":
                    go(W)
                else:
                    g.replay()
                torch.cuda.synchronize(dev)
                if gap_ms:
                    time.sleep(gap_ms * 1e-3)
                gpu = []
                t = bench.time_region(lambda: fn(K), 1, dev, 1, gpu=gpu)
                rows.append((t * 1e6 / K, gpu[0] * 1e6 / K))
            print(f"gap {gap_ms:4.1f} ms {name:8s}: " + "  ".join(f"{w:5.2f}/{e:5.2f}" for w, e in rows) +
                  "   (wall/events us per step)", flush=True)
    # the timed region with a spin on the end event before the closing
    # synchronize (the blocking wait's wake-up is not in the region)
    s = torch.cuda.current_stream(dev)
    for name, fn in forms.items():
        rows = []
        for trial in range(6):
            fn(W) if name == "c_loop" else g.replay()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(s)
            fn(K)
            e1.record(s)
            while not e1.query():
                pass
            torch.cuda.synchronize(dev)
            t = time.perf_counter() - t0
            rows.append((t * 1e6 / K, e0.elapsed_time(e1) * 1000.0 / K))
        print(f"spin-end  {name:8s}: " + "  ".join(f"{w:5.2f}/{e:5.2f}" for w, e in rows), flush=True)
    print(f"kernel_avg_us (200-launch graph): {bench.kernel_avg_us(lambda: step(0), 200, dev):.2f}", flush=True)


if __name__ == "__main__":
    main()
