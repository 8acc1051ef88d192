#!/usr/bin/env python3
"""Probe: do timing events recorded inside a captured hipGraph (external=True)
give per-kernel durations after one replay?  Compares with eager events."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, N = 32, 1024
    g = torch.Generator().manual_seed(0)
    x1 = torch.rand(B, N, 3, generator=g).to(dev)
    x2 = torch.rand(B, N, 3, generator=g).to(dev)
    d1, d2 = torch.empty(B, N, device=dev), torch.empty(B, N, device=dev)
    i1 = torch.empty(B, N, dtype=torch.int32, device=dev)
    i2 = torch.empty(B, N, dtype=torch.int32, device=dev)
    mo = torch.empty(2, device=dev)
    ws = pcm_hip.chamfer_workspace(dev, B, N, N)
    K = 50
    ev = [torch.cuda.Event(enable_timing=True, external=True) for _ in range(2 * K)]
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        for _ in range(3):
            pcm_hip.chamfer_forward_loss(x1, x2, d1, d2, i1, i2, mo, ws)
    torch.cuda.current_stream(dev).wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for k in range(K):
            ev[2 * k].record()
            pcm_hip.chamfer_forward_loss(x1, x2, d1, d2, i1, i2, mo, ws)
            ev[2 * k + 1].record()
    for rep in range(3):
        gr.replay()
        torch.cuda.synchronize()
        ts = [ev[2 * k].elapsed_time(ev[2 * k + 1]) * 1000 for k in range(K)]
        print(f"replay {rep}: per-kernel us mean {sum(ts) / K:.2f} min {min(ts):.2f} max {max(ts):.2f}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    e1.synchronize()
    print(f"whole replay / K: {e0.elapsed_time(e1) * 1000 / K:.2f} us")


if __name__ == "__main__":
    main()
