#!/usr/bin/env python3
"""The one-launch step's time against how long the GPU has been busy.

tools/ab_bench_gap.py (profiles/r06/ab_bench_gap_r06j.txt) found the same
kernel, buffers and clouds at 13.6-13.7 us per launch after tens of ms of
back-to-back work and at 14.4-14.6 us after any idle >= 50 ms.  This probe
times consecutive 200-launch graphs of the bench's step after 1 s idle and,
after each graph, a one-wave clock probe on the same stream
(pcm_tune_clock_rate: s_memtime over s_memrealtime ticks = the shader clock
it ran at).

    python tools/clock_state.py [REPLAYS]
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import bench  # noqa: E402
import pcm_hip  # noqa: E402
from tune_chamfer import graph_of  # noqa: E402


def main():
    replays = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    reps = 200
    step = bench.ChamferStep(dev, 1, seed=bench.BENCH_SEED, slots=1)
    for _ in range(5):
        step(0)
    g = graph_of(lambda: step(0), reps)
    out = torch.zeros(3, dtype=torch.int64, device=dev)

    def ghz():
        pcm_hip.tune_clock_rate(out)
        r, c, _ = out.tolist()
        return 0.1 * c / max(r, 1)

    torch.cuda.synchronize()
    for rnd in range(2):
        time.sleep(1.0)
        print(f"round {rnd}: after 1 s idle, probe clock {ghz():.2f} GHz", flush=True)
        busy = 0.0
        for i in range(replays):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            f = ghz()  # queued behind the graph: runs right after it
            us = e0.elapsed_time(e1) * 1000.0
            busy += us
            print(f"  graph {i:2d}: {us / reps:6.2f} us per launch, busy so far {busy / 1000.0:6.1f} ms, "
                  f"probe clock after it {f:.2f} GHz", flush=True)


if __name__ == "__main__":
    main()
