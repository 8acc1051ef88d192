#!/usr/bin/env python3
"""Counter-pass driver: BASELINE config 3 EMD forwards (B=16, N=1024, eps
0.005, 50 iterations, uniform clouds), helpers off so the auction kernel's
counters are the 16 masters' alone.  For rocprofv3 --pmc passes."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(3)
u1 = torch.rand(16, 1024, 3, generator=g).to(dev)
u2 = torch.rand(16, 1024, 3, generator=g).to(dev)
d = torch.empty(16, 1024, device=dev)
a = torch.empty(16, 1024, dtype=torch.int32, device=dev)
for _ in range(int(os.environ.get("REPS", "10"))):
    pcm_hip.emd_forward(u1, u2, 0.005, 50, d, a, helpers=0, offload_min=0)
torch.cuda.synchronize()
print("ok")
