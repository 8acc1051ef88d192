#!/usr/bin/env python3
"""Does the GPU's busy state move the EMD forward?
BASELINE config 3 (B=16, N=1024, eps 0.005, 50 iterations; bench.py's clouds,
seed 3): per-forward time of 10 eager forwards (bench.py emd_leg's form) right
after the GPU sat idle for 0.3 s, against the same 10 after ~`warm_ms` of
back-to-back forwards.  Alternating, `rounds` times each."""
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    warm_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(3)
    x1 = torch.rand(16, 1024, 3, generator=g).to(dev)
    x2 = torch.rand(16, 1024, 3, generator=g).to(dev)
    d = torch.empty(16, 1024, device=dev)
    a = torch.empty(16, 1024, dtype=torch.int32, device=dev)
    ws = pcm_hip.emd_workspace(dev, 16, 1024)
    s = torch.cuda.current_stream(dev)

    def fwd():
        pcm_hip.emd_forward(x1, x2, 0.005, 50, d, a, None, ws)

    def timed(reps=10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fwd()
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1000.0 / reps

    for _ in range(5):
        fwd()
    torch.cuda.synchronize()
    ref = (d.clone(), a.clone())
    res = {"idle": [], "warm": []}
    for _ in range(rounds):
        time.sleep(0.3)
        res["idle"].append(timed())
        t_end = time.perf_counter() + warm_ms / 1e3
        while time.perf_counter() < t_end:
            fwd()
            torch.cuda.synchronize()
        res["warm"].append(timed())
    same = torch.equal(d, ref[0]) and torch.equal(a, ref[1])
    for k, v in res.items():
        print(f"{k}: median {statistics.median(v):.1f} us per forward, all {[round(x, 1) for x in v]}")
    print(f"outputs unchanged: {same}")


if __name__ == "__main__":
    main()
