#!/usr/bin/env python3
"""The training_call leg after different preceding legs, to show that the
leg's figure depends on the GPU state the earlier legs leave
(profiles/r06/tc_order_r06ze.txt, measured before bench._time_call warmed the
GPU ahead of its timed replays).

    python tools/tc_order_probe.py {none|ref|head|headref}

ref: bench.reference_call_leg first; head: the headline step and its ~45 ms
sustained run first; headref: both.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    mode = sys.argv[1]
    if "head" in mode:
        step = bench.ChamferStep(dev, 1, seed=bench.BENCH_SEED, slots=20)
        for _ in range(5):
            step(0)
        print("sustained", bench.sustained_kernel_us(lambda: step(0), dev), flush=True)
    if "ref" in mode:
        print("ref", bench.reference_call_leg(dev)["graph_us_per_step"], flush=True)
    for label in ("train", "train again"):
        t = bench.training_call_leg(dev)
        print(label, t["graph_us_per_step"], t["before"]["graph_us_per_step"], flush=True)


if __name__ == "__main__":
    main()
