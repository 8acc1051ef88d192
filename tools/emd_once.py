#!/usr/bin/env python3
"""Runs the EMD forward at BASELINE config 3 (or the training call with
--train) a few times: a short target for rocprofv3 counter passes."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def main():
    train = "--train" in sys.argv
    eps, iters = (0.05, 3000) if train else (0.005, 50)
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(3)
    x1 = torch.rand(16, 1024, 3, generator=g).to(dev)
    x2 = torch.rand(16, 1024, 3, generator=g).to(dev)
    d = torch.empty(16, 1024, device=dev)
    a = torch.empty(16, 1024, dtype=torch.int32, device=dev)
    for _ in range(5):
        pcm_hip.emd_forward(x1, x2, eps, iters, d, a)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
