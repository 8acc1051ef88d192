#!/usr/bin/env python3
"""A/B timing of EMD forward builds: config 3 (uniform, eps 0.005, 50
iterations) and the training call (generator predictions, eps 0.05, 3000
iterations), defaults only.  Run once per library (PCM_HIP_LIB=...) in the
same GPU session, alternating, so box-to-box clock differences cancel."""
import hashlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import tune_emd_train as T  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    pred, points = T.generator_clouds(16, dev)
    g = torch.Generator().manual_seed(3)
    u1 = torch.rand(16, 1024, 3, generator=g).to(dev)
    u2 = torch.rand(16, 1024, 3, generator=g).to(dev)
    out = []
    for name, x1, x2, eps, iters, reps in (("config3", u1, u2, 0.005, 50, 50),
                                           ("train", pred, points, 0.05, 3000, 5)):
        d = torch.empty(16, 1024, device=dev)
        a = torch.empty(16, 1024, dtype=torch.int32, device=dev)
        t = T.timed(x1, x2, eps, iters, d, a, None, None, reps=reps)
        h = hashlib.md5(a.cpu().numpy().tobytes() + d.cpu().numpy().tobytes()).hexdigest()[:8]
        out.append(f"{name} {t:.1f} us [{h}]")  # the hash: same results across builds
    print(os.path.basename(os.environ.get("PCM_HIP_LIB", "libpcm_hip.so")) + ": " + ", ".join(out), flush=True)


if __name__ == "__main__":
    main()
