#!/usr/bin/env python3
"""Writes bench_data/emd_training_call.npz: the inputs of bench.py's EMD
training-call leg (loss/loss.py:23, eps 0.05, 3000 iterations).

pred   [16, 1024, 3] float32 -- the clouds a seeded random-init 3D-FENet
       generator (train/fenet.py, seed 0; the RepVGG checkpoint is absent)
       predicts for train_step.synthetic_batch(16, seed=0)'s images, computed
       on the CPU here (train.py:160's model, train/fenet.py's CPU forward is
       bit-identical to the reference generator: tests/test_train_cpu.py)
points [16, 1024, 3] float32 -- that batch's uniform [0,1) ground truth

Until round 4 bench.py ran the generator on the GPU, where the MIOpen /
hipBLASLt algorithm choice differs by box and a 1-ulp change moves the
auction: the leg was a different workload on every box.
Loading the committed clouds makes it the same everywhere.

    python tools/make_emd_train_clouds.py
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "train"))
OUT = os.path.join(REPO, "bench_data", "emd_training_call.npz")


def main():
    import fenet
    import train_step as T
    torch.manual_seed(0)
    b, n = 16, 1024
    gen = fenet.seeded_init(fenet.Generator(n), 0).train()
    images, points = T.synthetic_batch(b, n, "cpu", seed=0)
    with torch.no_grad():
        pred = gen(images)[2].transpose(2, 1).contiguous()
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, pred=pred.numpy().astype(np.float32), points=points.numpy().astype(np.float32))
    print(f"wrote {OUT}: pred {tuple(pred.shape)} range [{pred.min().item():.4f}, {pred.max().item():.4f}]")


if __name__ == "__main__":
    main()
