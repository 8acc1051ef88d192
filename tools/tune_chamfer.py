#!/usr/bin/env python3
"""A/B the Chamfer kernels inside ONE process (interleaved rounds,
cdna_hip_programming.md section 5.4 rule 24) on BASELINE config 2 (B=32,
N=M=1024) and config 5's shape (B=8, N=M=16384, fp32 here).

Each measurement captures `reps` back-to-back launches into a hipGraph and
times graph replays with HIP events, so the numbers are device time per
launch (incl. the inter-kernel gap), not Python/ctypes launch overhead.
Every forward variant is checked bit-for-bit against variant 0 first."""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def bufs(b, n, m, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    x1 = torch.rand(b, n, 3, generator=g).to(dev)
    x2 = torch.rand(b, m, 3, generator=g).to(dev)
    return (x1, x2, torch.empty(b, n, device=dev), torch.empty(b, m, device=dev),
            torch.empty(b, n, dtype=torch.int32, device=dev), torch.empty(b, m, dtype=torch.int32, device=dev))


def graph_of(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    return g


def time_graph_us(g, reps, replays=5):
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000 / (reps * replays)


def main():
    dev = torch.device("cuda:0")
    nv = pcm_hip.tune_num_chamfer_variants()
    for (b, n, m, reps, rounds) in [(32, 1024, 1024, 50, 5), (8, 16384, 16384, 2, 3)]:
        bf = bufs(b, n, m, dev)
        pcm_hip.tune_chamfer_forward(0, *bf)
        ref = [t.clone() for t in bf[2:]]
        ok = []
        for v in range(nv):
            pcm_hip.tune_chamfer_forward(v, *bf)
            torch.cuda.synchronize()
            ok.append(all(torch.equal(a, r) for a, r in zip(bf[2:], ref)))
        graphs = {v: graph_of(lambda v=v: pcm_hip.tune_chamfer_forward(v, *bf), reps) for v in range(nv)}
        res = {v: [] for v in range(nv)}
        for _ in range(rounds):
            for v in range(nv):
                res[v].append(time_graph_us(graphs[v], reps))
        pairs = 2 * b * n * m
        print(f"config B={b} N={n} M={m}  (device us per launch, graph replay)")
        for v in range(nv):
            med = statistics.median(res[v])
            print(f"  fwd variant {v}: median {med:9.2f} us  min {min(res[v]):9.2f}  "
                  f"{pairs / med / 1e6:8.3f} Tpairs/s  exact={ok[v]}")
        x1, x2, d1, d2, i1, i2 = bf
        g1 = torch.full((b, n), 1.0 / (b * n), device=dev)
        g2 = torch.full((b, m), 1.0 / (b * m), device=dev)
        gx1 = torch.empty(b, n, 3, device=dev)
        gx2 = torch.empty(b, m, 3, device=dev)
        out = {}
        for v in (0, 1, 2):
            gr = graph_of(lambda v=v: pcm_hip.tune_chamfer_backward(v, x1, x2, g1, g2, i1, i2, gx1, gx2), reps)
            out[v] = statistics.median([time_graph_us(gr, reps) for _ in range(rounds)])
        mo = torch.empty(2, device=dev)
        ws = pcm_hip.chamfer_workspace(dev, b, n, m)
        gl = graph_of(lambda: pcm_hip.chamfer_forward_loss(x1, x2, d1, d2, i1, i2, mo, ws), reps)
        fl = statistics.median([time_graph_us(gl, reps) for _ in range(rounds)])
        torch.cuda.synchronize()
        print(f"  bwd staged {out[0]:9.2f} us  global {out[1]:9.2f} us  per-batch-lds {out[2]:9.2f} us  "
              f"fused-loss fwd (default variant) {fl:9.2f} us")
        print(f"  mean=({mo[0].item():.7g},{mo[1].item():.7g}) torch=({d1.mean().item():.7g},{d2.mean().item():.7g})")
        for mode in (1, 2, 3):
            mo2 = torch.empty(2, device=dev)
            gm = graph_of(lambda mode=mode: pcm_hip.tune_chamfer_forward_loss(-1, mode, x1, x2, d1, d2, i1, i2,
                                                                            mo2, ws), reps)
            tm = statistics.median([time_graph_us(gm, reps) for _ in range(rounds)])
            torch.cuda.synchronize()
            print(f"  fused-loss mode {mode}: {tm:9.2f} us  mean=({mo2[0].item():.7g},{mo2[1].item():.7g})")
        if pcm_hip.loss_grad_supported(x1, x2):
            # fused loss + gradient (one launch) vs fused-loss forward + backward (two)
            mo3 = torch.empty(3, device=dev)
            w1, w2 = 1.0 / (b * n), 1.0 / (b * m)
            gsep = graph_of(lambda: (pcm_hip.chamfer_forward_loss(x1, x2, d1, d2, i1, i2, mo, ws),
                                     pcm_hip.chamfer_backward(x1, x2, g1, g2, i1, i2, gx1, gx2)), reps)
            tsep = statistics.median([time_graph_us(gsep, reps) for _ in range(rounds)])
            print(f"  step as two launches (fused-loss fwd + bwd): {tsep:9.2f} us")
            pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo3, gx1, gx2, ws)
            torch.cuda.synchronize()
            gref = [t.clone() for t in (d1, d2, i1, i2, gx1, gx2, mo3)]
            for v in range(pcm_hip.tune_num_chamfer_loss_grad_variants()):
                pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo3, gx1, gx2, ws, variant=v)
                torch.cuda.synchronize()
                same = all(torch.equal(a, r) for a, r in zip((d1, d2, i1, i2, gx1, gx2, mo3), gref))
                print(f"  loss+grad fused variant {v}: bit-identical to the default: {same}")
                gv = graph_of(lambda v=v: pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo3, gx1, gx2,
                                                                    ws, variant=v), reps)
                tv = statistics.median([time_graph_us(gv, reps) for _ in range(rounds)])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(reps):
                    pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo3, gx1, gx2, ws, variant=v)
                e1.record()
                e1.synchronize()
                te = e0.elapsed_time(e1) * 1000 / reps
                print(f"  loss+grad fused variant {v}: {tv:9.2f} us (graph)  {te:9.2f} us (eager)  "
                      f"{2 * b * n * m / tv / 1e6:8.3f} Tpairs/s  mean={mo3.tolist()}")
        # eager per-call cost through the Python API, for reference
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            pcm_hip.chamfer_backward(x1, x2, g1, g2, i1, i2, gx1, gx2)
        e1.record()
        e1.synchronize()
        print(f"  eager python-API bwd call: {e0.elapsed_time(e1) * 1000 / reps:9.2f} us/call")


def main_f16():
    """fp16-cloud forward variants (BASELINE config 5) and the fp16 backward."""
    dev = torch.device("cuda:0")
    nv = pcm_hip.tune_num_chamfer_f16_variants()
    for (b, n, m, reps, rounds) in [(32, 1024, 1024, 50, 5), (8, 16384, 16384, 2, 3)]:
        x1, x2, d1, d2, i1, i2 = bufs(b, n, m, dev)
        x1, x2 = x1.half(), x2.half()
        graphs = {v: graph_of(lambda v=v: pcm_hip.tune_chamfer_forward_f16(v, x1, x2, d1, d2, i1, i2), reps)
                  for v in range(nv)}
        res = {v: [] for v in range(nv)}
        for _ in range(rounds):
            for v in range(nv):
                res[v].append(time_graph_us(graphs[v], reps))
        pairs = 2 * b * n * m
        print(f"fp16 config B={b} N={n} M={m}")
        for v in range(nv):
            med = statistics.median(res[v])
            print(f"  f16 fwd variant {v}: median {med:9.2f} us  {pairs / med / 1e6:8.3f} Tpairs/s")
        g1 = torch.full((b, n), 1.0 / (b * n), device=dev)
        g2 = torch.full((b, m), 1.0 / (b * m), device=dev)
        gx1, gx2 = torch.empty_like(x1), torch.empty_like(x2)
        gr = graph_of(lambda: pcm_hip.chamfer_backward(x1, x2, g1, g2, i1, i2, gx1, gx2), reps)
        print(f"  f16 bwd: {statistics.median([time_graph_us(gr, reps) for _ in range(rounds)]):9.2f} us")


if __name__ == "__main__":
    main()
    main_f16()
