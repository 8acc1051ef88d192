#!/usr/bin/env python3
"""bench.py training_call leg's two forms (this build's call, round 5's call)
timed alternately in one process, each as bench._time_call measures it
(a captured 20-step graph, device time per step): the spread of the leg."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    sys.path.insert(0, os.path.join(bench.PKG, "loss"))
    import loss as loss_mod
    g = torch.Generator(device="cpu").manual_seed(11)
    fake = torch.rand(bench.B, 3, bench.N, generator=g).to(dev).requires_grad_(True)
    points = torch.rand(bench.B, bench.M, 3, generator=g).to(dev)
    loss_fn = loss_mod.Loss()

    def after():
        fake.grad = None
        (loss_fn.get_chamfer_loss(fake.transpose(2, 1), points) * bench.LAMBDA_CD).backward()

    def before():
        bench._round5_training_call(fake, points)

    reps = int(os.environ.get("TC_REPS", "200"))  # bench.py's leg: 50 (2 timed replays of the 20-step graph)
    for rnd in range(4):
        a = bench._time_call(after, dev, reps)["graph_us_per_step"]
        b = bench._time_call(before, dev, reps)["graph_us_per_step"]
        print(f"round {rnd}: after {a:.2f} us, before {b:.2f} us (captured, per step; reps {reps})", flush=True)


if __name__ == "__main__":
    main()
