#!/usr/bin/env python3
"""A/B of the one-launch Chamfer step (pcm_chamfer_loss_grad) for one build
(PCM_HIP_LIB=...): every fused variant from 7 up, at BASELINE config 2 (B=32,
N=M=1024), device time per launch from graph replays, interleaved rounds; each
variant's outputs are compared bit for bit with variant 7's.  Run once per
library in the same GPU session (tools/ab_chamfer.sh)."""
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402
from tune_chamfer import graph_of, time_graph_us  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, n, m, reps = 32, 1024, 1024, 50
    rounds = int(os.environ.get("AB_ROUNDS", "7"))
    # the bench's own clouds (bench.py ChamferStep, rank 0: seed BENCH_SEED = 1234)
    g = torch.Generator(device="cpu").manual_seed(1234)
    x1 = torch.rand(b, n, 3, generator=g).to(dev)
    x2 = torch.rand(b, m, 3, generator=g).to(dev)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, m, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, m, dtype=torch.int32, device=dev)
    gx1, gx2 = torch.empty(b, n, 3, device=dev), torch.empty(b, m, 3, device=dev)
    mo = torch.empty(3, device=dev)
    w1, w2 = 1.0 / (b * n), 1.0 / (b * m)
    vs = list(range(7, pcm_hip.tune_num_chamfer_loss_grad_variants()))  # (loads the tuning build first)
    ws = pcm_hip.chamfer_workspace(dev, b, n, m)  # sized for every variant of the tuning build
    if os.environ.get("AB_VARIANTS"):  # e.g. AB_VARIANTS=11,15; P = the product library's default entry
        vs = [v if v == "P" else int(v) for v in os.environ["AB_VARIANTS"].split(",")]
    out = {}

    def pv(v):
        return None if v == "P" else v
    # a zero-filled workspace per variant: variants of different granule formats
    # sharing one would make each switch's first call recompute every argmin
    wss = {v: torch.zeros_like(ws) for v in vs}
    for v in vs:
        pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo, gx1, gx2, wss[v], variant=pv(v))
        torch.cuda.synchronize()
        out[v] = [t.clone() for t in (d1, d2, i1, i2, gx1, gx2, mo)]
    same = {v: all(torch.equal(a, r) for a, r in zip(out[v], out[vs[0]])) for v in vs}
    graphs = {v: graph_of(lambda v=v: pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo, gx1, gx2, wss[v],
                                                                variant=pv(v)), reps) for v in vs}
    res = {v: [] for v in vs}
    cold = float(os.environ.get("AB_COLD", "0"))
    if cold:
        # the driver's state ("The GPU's busy state"): each
        # measurement is ONE replay of a 20-launch graph (the bench's form) after
        # the GPU sat idle for AB_COLD seconds
        graphs = {v: graph_of(lambda v=v: pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo, gx1, gx2,
                                                                    wss[v], variant=pv(v)), 20) for v in vs}
        for g in graphs.values():
            g.replay()
        torch.cuda.synchronize()
        for _ in range(rounds + 2):
            for v in vs:
                time.sleep(cold)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                graphs[v].replay()
                e1.record()
                e1.synchronize()
                res[v].append(e0.elapsed_time(e1) * 1000.0 / 20)
    else:
        for _ in range(rounds):
            for v in vs:
                res[v].append(time_graph_us(graphs[v], reps))
    lib = os.path.basename(os.environ.get("PCM_HIP_TUNE_LIB", "libpcm_hip_tune.so"))
    if cold:
        lib += f" (cold: one 20-launch graph after {cold} s idle)"
    print(lib + ": " + ", ".join(f"v{v} {statistics.median(res[v]):.2f} us (min {min(res[v]):.2f}, same={same[v]})"
                                 for v in vs), flush=True)
    if cold:  # the quartiles too: the driver's state spreads widely
        print("  quartiles: " + ", ".join(
            f"v{v} " + "/".join(f"{q:.2f}" for q in statistics.quantiles(res[v], n=4)) for v in vs), flush=True)


if __name__ == "__main__":
    main()
