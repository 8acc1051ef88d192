#!/usr/bin/env python3
"""K eager repetitions of one form of train.py's Chamfer call, for a rocprofv3
kernel trace (kernels per step = the trace's calls per kernel / K):

    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- \\
        python3 tools/training_call_trace.py {after|before|reference} [K]

after      this build's Loss().get_chamfer_loss(fake.transpose(2, 1), points)
           * lambda_cd, .backward() (bench.py training_call_leg)
before     round 5's form of the same call (bench.py _Round5LossFunction)
reference  the reference's own sequence through chamfer_3DDist + torch.mean
           (bench.py reference_call_leg, here with * lambda_cd as train.py:169)

BASELINE config 2 clouds (B=32, N=M=1024, the generator's [B, 3, N] layout).
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    form = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    g = torch.Generator(device="cpu").manual_seed(11)
    fake = torch.rand(bench.B, 3, bench.N, generator=g).to(dev).requires_grad_(True)
    points = torch.rand(bench.B, bench.M, 3, generator=g).to(dev)
    if form == "after":
        sys.path.insert(0, os.path.join(bench.PKG, "loss"))
        import loss as loss_mod
        loss_fn = loss_mod.Loss()

        def call():
            fake.grad = None
            (loss_fn.get_chamfer_loss(fake.transpose(2, 1), points) * bench.LAMBDA_CD).backward()
    elif form == "before":
        def call():
            bench._round5_training_call(fake, points)
    elif form == "reference":
        sys.path.insert(0, os.path.join(bench.PKG, "metric", "chamfer3D"))
        import dist_chamfer_3D

        def call():
            fake.grad = None
            d1, d2, _, _ = dist_chamfer_3D.chamfer_3DDist()(fake.transpose(2, 1), points)
            ((torch.mean(d1) + torch.mean(d2)) * bench.LAMBDA_CD).backward()
    else:
        raise SystemExit(f"unknown form {form}")
    for _ in range(k):
        call()
    torch.cuda.synchronize(dev)
    print(f"{form}: {k} calls", flush=True)
    if os.environ.get("TCT_GRAPH"):
        # bench.py _time_call's captured form: a graph of bench.GRAPH_STEPS calls,
        # two warm replays, then TCT_GRAPH timed replays (the trace separates
        # the replays' kernels from the eager calls by time)
        out = bench._time_call(call, dev, 20)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(bench.GRAPH_STEPS):
                call()
        for _ in range(int(os.environ["TCT_GRAPH"])):
            g.replay()
        torch.cuda.synchronize(dev)
        print(f"{form}: _time_call {out}", flush=True)


if __name__ == "__main__":
    main()
