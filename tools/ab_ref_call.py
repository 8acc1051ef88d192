#!/usr/bin/env python3
"""A/B of the pieces of the UNCHANGED caller's path (bench.py reference_call:
chamfer_3DDist on fake.transpose(2, 1) and points, torch means, .backward())
at BASELINE config 2, on that leg's own clouds: the plain filtered forward in
its two geometries (rows, and channel planes read in place), the backward with
a materialised against an expanded (stride-0) graddist, and the whole captured
call.  Device time per launch from graph replays, interleaved rounds; each
variant's outputs are compared bit for bit with variant 0's.

    python tools/ab_ref_call.py
"""
import ctypes
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import bench  # noqa: E402
from tune_chamfer import graph_of, time_graph_us  # noqa: E402

pcm_hip = bench.pcm_hip


def main():
    dev = torch.device("cuda:0")
    b, n, m, reps, rounds = bench.B, bench.N, bench.M, 50, 7
    g = torch.Generator(device="cpu").manual_seed(11)  # bench.reference_call_leg's clouds
    planes = torch.rand(b, 3, n, generator=g).to(dev)
    points = torch.rand(b, m, 3, generator=g).to(dev)
    fake = planes.transpose(1, 2)
    rows = fake.contiguous()
    L = pcm_hip.load_library()
    P = pcm_hip._ptr
    L.pcm_tune_chamfer_forward_layout.restype = ctypes.c_int
    L.pcm_tune_chamfer_forward_layout.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + \
        [ctypes.c_int] * 5 + [ctypes.c_void_p] * 5
    base = pcm_hip.tune_num_chamfer_variants() - 9  # kNumBaseFwdVariants: the filtered table starts there

    def outs():
        return (torch.empty(b, n, device=dev), torch.empty(b, m, device=dev),
                torch.empty(b, n, dtype=torch.int32, device=dev), torch.empty(b, m, dtype=torch.int32, device=dev))

    fw = {}
    for name, var in (("rows C32/T2048", base + 3), ("rows C16/T1024 (default)", base + 8)):
        o = outs()
        fw[name] = (o, (lambda v=var, o=o: pcm_hip.tune_chamfer_forward(v, rows, points, *o)))
    for name, var in (("planes C32/T2048", 0), ("planes C16/T1024 (default)", 1)):
        o = outs()
        fw[name] = (o, (lambda v=var, o=o: L.pcm_tune_chamfer_forward_layout(
            v, P(fake), P(points), b, n, m, 1, 0, P(o[0]), P(o[1]), P(o[2]), P(o[3]), pcm_hip._stream(dev))))
    ref = None
    for name, (o, fn) in fw.items():
        fn()
        torch.cuda.synchronize()
        if ref is None:
            ref = [t.clone() for t in o]
        same = all(torch.equal(x.view(torch.int32) if x.dtype == torch.float32 else x,
                               y.view(torch.int32) if y.dtype == torch.float32 else y) for x, y in zip(o, ref))
        print(f"{name:28s} bit-identical to the first: {same}", flush=True)
        assert same
    d1, d2, i1, i2 = ref
    g1c = torch.full((b, n), 1.0 / (b * n), device=dev)
    g2c = torch.full((b, m), 1.0 / (b * m), device=dev)
    g1e = torch.full((), 1.0 / (b * n), device=dev).expand(b, n)
    g2e = torch.full((), 1.0 / (b * m), device=dev).expand(b, m)
    gx = {k: (torch.empty(b, 3, n, device=dev), torch.empty(b, m, 3, device=dev)) for k in ("c", "e")}
    bw = {
        "bwd graddist materialised": lambda: pcm_hip.chamfer_backward_layout(
            fake, points, 1, 0, g1c, g2c, i1, i2, gx["c"][0].transpose(1, 2), gx["c"][1]),
        "bwd graddist expanded": lambda: pcm_hip.chamfer_backward_strided(
            fake, points, 1, 0, g1e, g2e, i1, i2, gx["e"][0].transpose(1, 2), gx["e"][1]),
    }
    gr = {v: (torch.empty(b, n, 3, device=dev), torch.empty(b, m, 3, device=dev)) for v in (0, 4)}
    bw["bwd rows slot buckets (default)"] = lambda: pcm_hip.tune_chamfer_backward(0, rows, points, g1c, g2c, i1, i2,
                                                                                 *gr[0])
    bw["bwd rows staged passes (r04)"] = lambda: pcm_hip.tune_chamfer_backward(4, rows, points, g1c, g2c, i1, i2,
                                                                              *gr[4])
    for fn in bw.values():
        fn()
    torch.cuda.synchronize()
    same = all(torch.equal(x.view(torch.int32), y.view(torch.int32)) for x, y in zip(gx["c"], gx["e"]))
    print(f"backward expanded vs materialised bit-identical: {same}", flush=True)
    assert same
    same = all(torch.equal(x.view(torch.int32), y.view(torch.int32)) for x, y in zip(gr[0], gr[4]))
    same &= torch.equal(gr[0][0].view(torch.int32), gx["c"][0].transpose(1, 2).contiguous().view(torch.int32))
    print(f"backward slot buckets vs staged passes (and vs the planes form) bit-identical: {same}", flush=True)
    assert same
    forms = {k: v[1] for k, v in fw.items()}
    forms.update(bw)
    graphs = {k: graph_of(fn, reps) for k, fn in forms.items()}
    res = {k: [] for k in graphs}
    for _ in range(rounds):
        for k, gr in graphs.items():
            res[k].append(time_graph_us(gr, reps))
    for k, v in res.items():
        print(f"{k:28s} median {statistics.median(v):7.2f} us  min {min(v):7.2f}  "
              f"[{' '.join(f'{x:.2f}' for x in v)}]", flush=True)
    rc = bench.reference_call_leg(dev)
    print(f"reference_call graph {rc['graph_us_per_step']:.2f} us/step, eager {rc['eager_us_per_step']:.1f} us/step",
          flush=True)


if __name__ == "__main__":
    main()
