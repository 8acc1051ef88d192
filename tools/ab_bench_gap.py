#!/usr/bin/env python3
"""Why the bench's 200-launch graph average (14.4 us, bench.json
kernel_us_graph200) sits ~0.8 us above tools/ab_chamfer.py's (13.6 us) for the
same product entry on the same clouds (seed 1234), same box: one process, the
forms below interleaved round by round, each a graph of 50 launches replayed 5
times (tools/tune_chamfer.time_graph_us).

  ab         ab_chamfer.py's own buffers and zero-filled workspace, mean_out fixed
  bench      bench.ChamferStep's step(0): its buffers and cached workspace
  bench_wsab the bench's buffers with the ab form's workspace
  ab_wsb     the ab form's buffers with the bench's workspace
  slots      the bench's graph form: step(i % 20), the loss mean rows rotating
  after_fb   bench after one chamfer_forward_loss + chamfer_backward on its
             workspace (what bench.py runs just before its graph200)
"""
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import bench  # noqa: E402
import pcm_hip  # noqa: E402
from tune_chamfer import graph_of, time_graph_us  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    b, n, m, reps, rounds = 32, 1024, 1024, 50, 7
    step = bench.ChamferStep(dev, 1, seed=bench.BENCH_SEED, slots=20)
    g = torch.Generator(device="cpu").manual_seed(bench.BENCH_SEED)
    x1 = torch.rand(b, n, 3, generator=g).to(dev)
    x2 = torch.rand(b, m, 3, generator=g).to(dev)
    assert torch.equal(x1, step.xyz1) and torch.equal(x2, step.xyz2)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, m, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, m, dtype=torch.int32, device=dev)
    gx1, gx2 = torch.empty(b, n, 3, device=dev), torch.empty(b, m, 3, device=dev)
    mo = torch.empty(3, device=dev)
    w1, w2 = 1.0 / (b * n), 1.0 / (b * m)
    ws_ab = torch.zeros(int(pcm_hip.load_library().pcm_chamfer_workspace_bytes(b, n, m)), dtype=torch.uint8,
                        device=dev)

    def ab(ws):
        return lambda: pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, d1, d2, i1, i2, mo, gx1, gx2, ws)

    def st(ws):
        return lambda: pcm_hip.chamfer_loss_grad(step.xyz1, step.xyz2, step.w1, step.w2, step.d1, step.d2, step.i1,
                                                 step.i2, step.loss[0], step.gx1, step.gx2, ws)

    ctr = [0]

    def slots():
        step(ctr[0] % 20)
        ctr[0] += 1

    def after_fb():
        pcm_hip.chamfer_forward_loss(step.xyz1, step.xyz2, step.d1, step.d2, step.i1, step.i2, step.loss[0], step.ws)
        pcm_hip.chamfer_backward(step.xyz1, step.xyz2, step.g1, step.g2, step.i1, step.i2, step.gx1, step.gx2)
        torch.cuda.synchronize()

    forms = {"ab": ab(ws_ab), "bench": lambda: step(0), "bench_wsab": st(ws_ab), "ab_wsb": ab(step.ws),
             "slots": slots}
    print("ws bytes: ab", ws_ab.numel(), "bench", step.ws.numel(), "ptrs", hex(ws_ab.data_ptr()),
          hex(step.ws.data_ptr()), flush=True)
    for f in forms.values():
        for _ in range(5):
            f()
    torch.cuda.synchronize()
    graphs = {k: graph_of(f, reps) for k, f in forms.items()}
    res = {k: [] for k in graphs}
    res["after_fb"] = []
    for _ in range(rounds):
        for k, gr in graphs.items():
            res[k].append(time_graph_us(gr, reps))
        after_fb()
        res["after_fb"].append(time_graph_us(graphs["bench"], reps))
    print(", ".join(f"{k} {statistics.median(v):.2f} us (min {min(v):.2f})" for k, v in res.items()), flush=True)
    # the bench's own measurement, as bench.py takes it (one replay of a 200-launch graph)
    print("bench.kernel_avg_us(step(0), 200):", round(bench.kernel_avg_us(lambda: step(0), 200, dev), 2),
          " ab form:", round(bench.kernel_avg_us(ab(ws_ab), 200, dev), 2), flush=True)
    # the same measurement after the GPU sat idle (host sleep), then again at once
    for idle in (0.05, 0.2, 1.0):
        time.sleep(idle)
        cold = bench.kernel_avg_us(lambda: step(0), 200, dev)
        warm = bench.kernel_avg_us(lambda: step(0), 200, dev)
        print(f"after {idle:.2f} s idle: kernel_avg_us {cold:.2f}, at once again {warm:.2f}", flush=True)


if __name__ == "__main__":
    main()
