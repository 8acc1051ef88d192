#!/usr/bin/env python3
"""A/B of the one-launch step on the training call's layouts (cloud 1 as
channel planes, cloud 2 rows: train.py:163's fake.transpose(2, 1) against the
GT), BASELINE config 2, through the tuning build's
pcm_tune_chamfer_loss_grad_layout: form 0 (the product: the two directions as
separate inlined forwards, compile-time strides) against form 1 (one inlined
forward, strides in registers), with the rows/rows step beside them.  Device
time per launch from 50-launch graph replays, interleaved rounds; outputs
compared bit for bit (gradients in each cloud's layout).

    python tools/ab_layout_forms.py
"""
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402
from tune_chamfer import graph_of, time_graph_us  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, n, m, reps, rounds = 32, 1024, 1024, 50, 7
    g = torch.Generator(device="cpu").manual_seed(11)
    planes = torch.rand(b, 3, n, generator=g).to(dev)
    pts = torch.rand(b, m, 3, generator=g).to(dev)
    rows = planes.transpose(1, 2).contiguous()
    L = pcm_hip.load_tune_library()
    P = pcm_hip._ptr
    vp, ci, cf, cs = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    f = L.pcm_tune_chamfer_loss_grad_layout
    f.restype = ci
    f.argtypes = [ci, vp, vp, ci, ci, ci, ci, ci, cf, cf, vp, vp, vp, vp, vp, vp, vp, vp, vp, cs, vp]
    w = pcm_hip.mean_weight(b * n)
    lam = torch.full((1,), 100.0, device=dev)
    need = int(L.pcm_chamfer_workspace_bytes(b, n, m))
    cases = {"rows/rows": (0, (0, 0)), "planes/rows form 0 (product)": (0, (1, 0)),
             "planes/rows form 1 (one forward)": (1, (1, 0))}
    outs, runs = {}, {}
    for name, (form, lay) in cases.items():
        ws = torch.zeros(need, dtype=torch.uint8, device=dev)
        o = dict(d1=torch.empty(b, n, device=dev), d2=torch.empty(b, m, device=dev),
                 i1=torch.empty(b, n, dtype=torch.int32, device=dev), i2=torch.empty(b, m, dtype=torch.int32, device=dev),
                 mo=torch.empty(4, device=dev),
                 g1=(torch.empty(b, 3, n, device=dev) if lay[0] else torch.empty(b, n, 3, device=dev)),
                 g2=torch.empty(b, m, 3, device=dev))
        x1 = planes.transpose(1, 2) if lay[0] else rows

        def run(form=form, lay=lay, o=o, ws=ws, x1=x1):
            st = pcm_hip._stream(dev)  # the capturing stream inside graph_of
            r = f(form, P(x1), P(pts), b, n, m, lay[0], lay[1], w, w, P(lam), P(o["d1"]), P(o["d2"]), P(o["i1"]),
                  P(o["i2"]), P(o["mo"]), P(o["g1"]), P(o["g2"]), P(ws), ws.numel(), st)
            if r:
                raise RuntimeError(f"status {r}")
        run()
        torch.cuda.synchronize()
        g1 = o["g1"].transpose(1, 2).contiguous() if lay[0] else o["g1"].clone()
        outs[name] = [o[k].clone() for k in ("d1", "d2", "i1", "i2", "mo", "g2")] + [g1]
        runs[name] = run
    for name in cases:  # every case's first-call outputs are taken before any graph is captured
        runs[name] = graph_of(runs[name], reps)
    ref = outs["rows/rows"]
    res = {k: [] for k in cases}
    for _ in range(rounds):
        for k in cases:
            res[k].append(time_graph_us(runs[k], reps))
    names = ("d1", "d2", "i1", "i2", "mo", "g2", "g1")
    for k in cases:
        diff = [nm for nm, a, r in zip(names, outs[k], ref) if not torch.equal(a, r)]
        print(f"{k:34s} {statistics.median(res[k]):6.2f} us (min {min(res[k]):6.2f})  outputs differing from "
              f"rows/rows: {diff or 'none'}", flush=True)
        for nm, a, r in zip(names, outs[k], ref):
            if nm in diff:
                bad = (a != r).nonzero()
                print(f"    {nm}: {bad.shape[0]} elements differ, first at {bad[0].tolist()}: {a[tuple(bad[0])].item()} "
                      f"vs {r[tuple(bad[0])].item()}", flush=True)


if __name__ == "__main__":
    main()
