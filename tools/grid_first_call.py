#!/usr/bin/env python3
"""Per-call device time of the config-5 grid search kernel in a FRESH process
(one grid_nn_kernel<float> call of 148 us among
43-46 us calls in profiles/r05/pmc_summary.json kernel_trace_eager).

    python tools/grid_first_call.py ORDER

ORDER is a comma list of forwards run in this order, each one launch timed by
HIP events on its stream: f32 / f16 (the public grid forward, B=8,
N=M=16384), tiny (the same search kernel forced at B=1, N=M=64 through the
tuning entry: a small dispatch of the same code), dense (a dense forward of
config 2, no scratch).  The search kernel spills 4 VGPRs to scratch
(.private_segment_fixed_size 20); the runtime backs a queue's scratch on the
first dispatch that needs it, and that dispatch's traced duration includes it.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def main():
    order = sys.argv[1].split(",")
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    b, n = 8, 16384
    x = torch.rand(b, n, 3, generator=g).to(dev)
    y = torch.rand(b, n, 3, generator=g).to(dev)
    xs = {"f32": (x, y), "f16": (x.half(), y.half())}
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, n, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, n, dtype=torch.int32, device=dev)
    t1, t2 = torch.rand(1, 64, 3, device=dev), torch.rand(1, 64, 3, device=dev)
    e1, e2 = torch.empty(1, 64, device=dev), torch.empty(1, 64, device=dev)
    k1 = torch.empty(1, 64, dtype=torch.int32, device=dev)
    k2 = torch.empty(1, 64, dtype=torch.int32, device=dev)
    c1, c2 = torch.rand(32, 1024, 3, device=dev), torch.rand(32, 1024, 3, device=dev)
    f1, f2 = torch.empty(32, 1024, device=dev), torch.empty(32, 1024, device=dev)
    j1 = torch.empty(32, 1024, dtype=torch.int32, device=dev)
    j2 = torch.empty(32, 1024, dtype=torch.int32, device=dev)
    ws = pcm_hip.forward_workspace(dev, b, n, n)
    torch.cuda.synchronize()
    out = []
    for what in order:
        e0, e9 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if what in xs:
            a, c = xs[what]
            e0.record()
            pcm_hip.chamfer_forward(a, c, d1, d2, i1, i2)
            e9.record()
        elif what == "tiny":
            e0.record()
            pcm_hip.tune_chamfer_forward_grid(t1, t2, e1, e2, k1, k2, workspace=ws)
            e9.record()
        elif what == "dense":
            e0.record()
            pcm_hip.chamfer_forward(c1, c2, f1, f2, j1, j2)
            e9.record()
        else:
            raise SystemExit(f"unknown {what}")
        e9.synchronize()
        out.append((what, round(e0.elapsed_time(e9) * 1000.0, 1)))
        print(f"{what:6s} {out[-1][1]:9.1f} us (build + search)", flush=True)
    print(json.dumps({"order": order, "us": out}))


if __name__ == "__main__":
    main()
