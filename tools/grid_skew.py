#!/usr/bin/env python3
"""Config-5 grid forward: the search kernel's per-XCD start skew behind the
build (tools/grid_diag.py, r06v: XCD 0's waves start 9.7 us after XCD 3's when
the search follows the build, <= 1.5 us when it runs alone).  Each form runs
build and search on one stream, with something between them:

  direct     nothing (the product's order)
  sync       a host synchronize
  stamp1     a one-wave kernel (pcm_tune_clock_stamp)
  occupy256  256 one-wave workgroups that return at once (pcm_tune_occupy)

and prints the search waves' start median/max per XCD (us after the first
wave's start), the search span, and the form's graph-timed duration."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pcm_hip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, n = 8, 16384
    g = torch.Generator().manual_seed(5)
    x1 = torch.rand(b, n, 3, generator=g).half().to(dev)
    x2 = torch.rand(b, n, 3, generator=g).half().to(dev)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, n, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, n, dtype=torch.int32, device=dev)
    ws = pcm_hip.forward_workspace(dev, b, n, n, force_grid=True)
    waves = b * 2 * (n // 64)
    clk = torch.zeros(1, dtype=torch.int64, device=dev)

    def between(form):
        if form == "sync":
            torch.cuda.synchronize()
        elif form == "stamp1":
            pcm_hip.tune_clock_stamp(clk)
        elif form == "occupy256":
            pcm_hip.tune_occupy(dev, 256, 64, 0, 0)

    def run(form, stats=None):
        pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="build", workspace=ws)
        between(form)
        pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="search", workspace=ws, stats=stats)

    forms = ["direct", "sync", "stamp1", "occupy256"]
    for form in forms:
        run(form)
    torch.cuda.synchronize()
    for rnd in range(2):
        for form in forms:
            st = torch.zeros(waves * 12, dtype=torch.int32, device=dev)
            run(form, st)
            torch.cuda.synchronize()
            ss = st[waves * 4:].view(waves, 8).cpu().long() & 0xffffffff
            t0 = ss[:, 0].min()
            s0 = (ss[:, 0] - t0).float() * 0.01
            xcc = ss[:, 7] & 0xf
            per = " ".join(f"{torch.quantile(s0[xcc == x], 0.5).item():.2f}/{s0[xcc == x].max().item():.2f}"
                           for x in range(8) if bool((xcc == x).any()))
            span = ((ss[:, 5] - t0).float() * 0.01).max().item()
            print(f"round {rnd} {form:9s}: start median/max by xcc {per}; search span {span:.1f} us", flush=True)
    # whole-form device time (no sync form: eager, 20 calls between two events)
    for form in ("direct", "stamp1", "occupy256"):
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run(form)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0 / 20)
        print(f"{form:9s}: {statistics.median(ts):.1f} us per forward (eager, 20 calls)", flush=True)


if __name__ == "__main__":
    main()
