#!/usr/bin/env python3
"""Generate the committed Chamfer golden fixtures from the REFERENCE's own CPU code.

Runs only in the build container (the reference does not exist on the GPU
box).  It imports the reference's importable pure-torch Chamfer,
``utils/utils.py:246-290`` (``array2samples_distance`` /
``chamfer_distance_numpy_test``), evaluates it on seeded ``torch.rand`` clouds
(the same kind of input as metric/chamfer3D/test.py:4-5 and loss/loss.py:41-42),
and records inputs + reference outputs:

  cd_all, cd1, cd2   reference scalars (cd_all = mean(dist1)+mean(dist2) summed
                     over the batch / B, the loss/loss.py:36 quantity)
  grad1, grad2       autograd gradients of cd_all w.r.t. both clouds
  nn1_f64, nn2_f64   float64 brute-force argmins (independent of the reference,
                     for pinning per-point indices away from float32 near-ties)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
(PYTHONDONTWRITEBYTECODE keeps __pycache__ out of the read-only reference.)
"""
import os
import sys

import numpy as np
import torch

REF = os.environ.get("PCM_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "chamfer_golden.npz")

CASES = [  # (name, seed, B, N, M)
    ("cfg1_s0", 0, 4, 256, 256),   # BASELINE config 1
    ("cfg1_s1", 1, 4, 256, 256),
    ("cfg1_s2", 2, 4, 256, 256),
    ("cfg1_s3", 3, 4, 256, 256),
    ("ragged", 4, 2, 200, 300),
    ("test_py_shape", 5, 1, 1000, 2000),  # metric/chamfer3D/test.py:4-5 (N=1000, M=2000)
]


def nn_f64(p, q):
    d = ((p[:, :, None, :].astype(np.float64) - q[:, None, :, :].astype(np.float64)) ** 2).sum(-1)
    return d.argmin(-1).astype(np.int32)


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REF, "utils"))
    sys.path.insert(0, os.path.join(REF, "loss"))
    import utils as ref_utils  # reference utils/utils.py

    out = {}
    for name, seed, b, n, m in CASES:
        torch.manual_seed(seed)
        a = torch.rand(b, n, 3)
        c = torch.rand(b, m, 3)
        x1 = a.clone().requires_grad_(True)
        x2 = c.clone().requires_grad_(True)
        cd_all, cd_b, cd_a = ref_utils.chamfer_distance_numpy_test(x1, x2)
        # reference naming: av_dist1 = samples of array2 -> array1 = mean(dist2)
        cd_all.backward()
        out[f"{name}/xyz1"] = a.numpy()
        out[f"{name}/xyz2"] = c.numpy()
        out[f"{name}/cd_all"] = np.float32(cd_all.item())
        out[f"{name}/cd_mean_dist2"] = np.float32(cd_b.item())
        out[f"{name}/cd_mean_dist1"] = np.float32(cd_a.item())
        out[f"{name}/grad1"] = x1.grad.numpy()
        out[f"{name}/grad2"] = x2.grad.numpy()
        out[f"{name}/nn1_f64"] = nn_f64(a.numpy(), c.numpy())
        out[f"{name}/nn2_f64"] = nn_f64(c.numpy(), a.numpy())
        print(f"{name}: B={b} N={n} M={m} cd_all={cd_all.item():.7f}")
    out["cases"] = np.array([c[0] for c in CASES])
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
