#!/usr/bin/env python3
"""EMD diagnostics on BASELINE config 3 (B=16, N=1024, eps=0.005, 50 iters):
per-iteration unassigned / full-scan counts and graph-replay device time."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def main(b=16, n=1024, eps=0.005, iters=50):
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(3)
    x1 = torch.rand(b, n, 3, generator=g).to(dev)
    x2 = torch.rand(b, n, 3, generator=g).to(dev)
    d = torch.empty(b, n, device=dev)
    a = torch.empty(b, n, dtype=torch.int32, device=dev)
    st = torch.zeros(3 * iters + 16 + b, dtype=torch.int32, device=dev)
    pcm_hip.tune_emd_forward_stats(x1, x2, eps, iters, d, a, st)
    torch.cuda.synchronize()
    st = st.cpu()
    ph = st[2 * iters:2 * iters + 6].tolist()
    b1t = st[2 * iters + 16:3 * iters + 16].tolist()
    wall = st[3 * iters + 16:3 * iters + 16 + b].tolist()
    fb, nw0, tf, te = st[2 * iters + 6:2 * iters + 10].tolist()
    print(f"fast-scan fallbacks (all batches): {fb}; batch-0 wave-0 scans: {nw0}, "
          f"fast {tf / 100.0 / max(nw0, 1):.2f} us/scan, exact-fallback {te / 100.0 / max(nw0, 1):.2f} us/scan")
    st = st[:2 * iters].view(iters, 2)
    names = ["compact", "bid-from-cache", "full-scans", "claim", "assign", "reset"]
    print("batch-0 phase wall time over all iterations (us):",
          ", ".join(f"{nm}={v / 100.0:.1f}" for nm, v in zip(names, ph)))
    print("iter: unassigned(sum over batch) full-scans")
    print(" ".join(f"{i}:{int(st[i,0])}/{int(st[i,1])}" for i in range(iters)))
    print("batch-0 cache-bid time per iteration (us):", " ".join(f"{v / 100.0:.2f}" for v in b1t))
    print("auction wall time per batch element (us):", " ".join(f"{v / 100.0:.1f}" for v in wall))
    print("total unassigned", int(st[:, 0].sum()), "total full scans", int(st[:, 1].sum()))
    pcm_hip.emd_forward(x1, x2, eps, iters, d, a)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        pcm_hip.emd_forward(x1, x2, eps, iters, d, a)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(5):
            pcm_hip.emd_forward(x1, x2, eps, iters, d, a)
    gr.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(4):
        gr.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 20
    print(f"EMD forward B={b} N={n} iters={iters}: {us:.1f} us/call (graph)  {iters / (us * 1e-6):.0f} iters/s")


if __name__ == "__main__":
    main()
