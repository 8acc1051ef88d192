#!/usr/bin/env python3
"""How much does the one-launch Chamfer step's time depend on the cloud draw?
Times pcm_chamfer_loss_grad at BASELINE config 2 (B=32, N=M=1024) for several
seeded uniform clouds (torch.rand on the CPU, as bench.py draws them) and two
graph lengths, with HIP events around a graph replay (median of 5)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402

B, N, M = 32, 1024, 1024


def timed(x1, x2, reps, dev):
    d1, d2 = torch.empty(B, N, device=dev), torch.empty(B, M, device=dev)
    i1 = torch.empty(B, N, dtype=torch.int32, device=dev)
    i2 = torch.empty(B, M, dtype=torch.int32, device=dev)
    g1, g2 = torch.empty(B, N, 3, device=dev), torch.empty(B, M, 3, device=dev)
    mo = torch.empty(3, device=dev)
    ws = pcm_hip.chamfer_workspace(dev, B, N, M)
    w1, w2 = 1.0 / (B * N), 1.0 / (B * M)

    def launch():
        pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo, g1, g2, ws)

    for _ in range(5):
        launch()
    s = torch.cuda.current_stream(dev)
    cs = torch.cuda.Stream(dev)
    cs.wait_stream(s)
    with torch.cuda.stream(cs):
        launch()
    s.wait_stream(cs)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            launch()
    g.replay()
    out = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1000.0 / reps)
    return sorted(out)[2]


def main():
    dev = torch.device("cuda:0")
    for seed in (0, 1, 2, 3, 42, 1234, 1235):
        g = torch.Generator(device="cpu").manual_seed(seed)
        a = torch.rand(B, N, 3, generator=g)
        c = torch.rand(B, M, 3, generator=g)
        x1, x2 = a.to(dev), c.to(dev)
        t50 = timed(x1, x2, 50, dev)
        t200 = timed(x1, x2, 200, dev)
        print(f"seed {seed:5d}: {t50:6.2f} us (50 per graph)  {t200:6.2f} us (200 per graph)", flush=True)


if __name__ == "__main__":
    main()
