#!/usr/bin/env python3
"""Matched A/B of the two launch forms of bench.py's N=1 timed region
(VERDICT round 5, item 4), in one process on one box, alternating order:

  c_loop  K direct launches of pcm_chamfer_loss_grad from one host call
          (pcm_chamfer_loss_grad_steps, arguments bound once);
  graph   replays of the warmed GRAPH_STEPS-step hipGraph of the same step
          (the form bench.py uses at N > 1, where each step's all-reduce is
          captured beside it).

Each sample is the bench's region exactly: synchronize, perf_counter, the K
steps, synchronize (time_region), with HIP events at its edges for the GPU
side.  K = 20 (the driver's --steps) and K = 200.

    python tools/ab_launch_form.py [rounds]
"""
import json
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    step = bench.ChamferStep(dev, 1, seed=bench.BENCH_SEED, slots=bench.GRAPH_STEPS)
    for i in range(3):
        step(i)
    torch.cuda.synchronize(dev)
    per = bench.GRAPH_STEPS
    g_many = bench.capture_steps(step, per, dev, 1, False)
    go = step.launcher()
    g_many.replay()
    go(5)
    torch.cuda.synchronize(dev)

    forms = {
        "c_loop": lambda k: go(k),
        "graph": lambda k: [g_many.replay() for _ in range(k // per)],
    }
    res = {}
    for k in (20, 200):
        samples = {f: [] for f in forms}
        gpu = {f: [] for f in forms}
        for r in range(rounds):
            order = list(forms) if r % 2 == 0 else list(forms)[::-1]
            for f in order:
                forms[f](k)  # the region's own warmup, last before it
                torch.cuda.synchronize(dev)
                gt = []
                t = bench.time_region(lambda: forms[f](k), 1, dev, 1, gpu=gt)
                samples[f].append(t * 1e6 / k)
                gpu[f].append(gt[0] * 1e6 / k)
        res[f"K={k}"] = {f: {"wall_us_per_step_median": statistics.median(samples[f]),
                             "wall_us_per_step_min": min(samples[f]),
                             "gpu_us_per_step_median": statistics.median(gpu[f]),
                             "wall_samples": [round(x, 3) for x in samples[f]]} for f in forms}
        for f in forms:
            print(f"K={k:4d} {f:7s} wall {statistics.median(samples[f]):7.3f} us/step (min "
                  f"{min(samples[f]):7.3f})  gpu {statistics.median(gpu[f]):7.3f}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
