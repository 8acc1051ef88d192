#!/usr/bin/env python3
"""Grid forward (csrc/chamfer_grid.hip) against the dense forward at the large
cloud sizes: HIP-event timing of a captured graph of 20 calls (median of 5)
and a bit-equality check of the two paths' outputs."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    cs = torch.cuda.Stream()
    cs.wait_stream(s)
    with torch.cuda.stream(cs):
        fn()
    s.wait_stream(cs)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
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
    L = pcm_hip.load_library()
    P = pcm_hip._ptr
    for (b, n, m, dt) in [(8, 16384, 16384, torch.float16), (8, 16384, 16384, torch.float32),
                          (2, 4096, 4096, torch.float32), (32, 4096, 4096, torch.float32),
                          (4, 65536, 65536, torch.float32)]:
        g = torch.Generator().manual_seed(5)
        x1 = torch.rand(b, n, 3, generator=g).to(dt).to(dev)
        x2 = torch.rand(b, m, 3, generator=g).to(dt).to(dev)
        outs = {}
        res = {}
        for path in ("dense", "grid_screened", "grid"):
            d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, m, device=dev)
            i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
            i2 = torch.empty(b, m, dtype=torch.int32, device=dev)
            if path == "dense":
                fn16 = dt == torch.float16
                f = L.pcm_chamfer_forward_f16 if fn16 else L.pcm_chamfer_forward

                def call():
                    assert f(P(x1), P(x2), b, n, m, P(d1), P(d2), P(i1), P(i2), pcm_hip._stream(dev)) == 0
            else:
                sc = "screened" if path == "grid_screened" else "filter"

                def call():
                    pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, scan=sc)
            if path == "dense" and n >= 65536:
                reps = 2
            else:
                reps = 20
            res[path] = timed(call, reps)
            torch.cuda.synchronize()
            outs[path] = (d1.clone(), d2.clone(), i1.clone(), i2.clone())
        same = all(torch.equal(a.view(torch.int32), c.view(torch.int32)) and torch.equal(a.view(torch.int32), e.view(torch.int32))
                   for a, c, e in zip(outs["dense"], outs["grid"], outs["grid_screened"]))
        pairs = 2.0 * b * n * m
        print(f"B={b} N={n} M={m} {str(dt)[6:]}: dense {res['dense']:9.1f} us  grid(screened scan) {res['grid_screened']:8.1f} us  "
              f"grid {res['grid']:8.1f} us  "
              f"x{res['dense'] / res['grid']:5.2f}  dense-equivalent {pairs / res['grid'] * 1e-6:.3e} pairs/s  "
              f"identical={same}", flush=True)


def backward_f16(dev):
    """Config-5 fp16 backward: 256- against 1024-target workgroups."""
    b, n = 8, 16384
    g = torch.Generator().manual_seed(5)
    x1 = torch.rand(b, n, 3, generator=g).half().to(dev)
    x2 = torch.rand(b, n, 3, generator=g).half().to(dev)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, n, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, n, dtype=torch.int32, device=dev)
    pcm_hip.chamfer_forward(x1, x2, d1, d2, i1, i2)
    g1 = torch.full((b, n), 1.0 / (b * n), device=dev)
    g2 = torch.full((b, n), 1.0 / (b * n), device=dev)
    res, outs = {}, {}
    for v in (1, 3):
        gx1, gx2 = torch.empty_like(x1), torch.empty_like(x2)

        def call():
            pcm_hip.tune_chamfer_backward_f16(v, x1, x2, g1, g2, i1, i2, gx1, gx2)
        res[v] = timed(call)
        torch.cuda.synchronize()
        outs[v] = (gx1.clone(), gx2.clone())
    same = all(torch.equal(a.view(torch.int16), c.view(torch.int16)) for a, c in zip(outs[1], outs[3]))
    print(f"config-5 fp16 backward: 256-target workgroups {res[1]:.1f} us, 1024-target {res[3]:.1f} us, "
          f"identical={same}", flush=True)


if __name__ == "__main__":
    backward_f16(torch.device("cuda:0"))
    main()
