#!/usr/bin/env python3
"""Generate the committed ICP golden fixtures from the REFERENCE's own code.

Runs only in the build container (the reference does not exist on the GPU
box).  It imports the reference's utils/icp.py (numpy + sklearn
NearestNeighbors; sklearn 1.7.2 here) and records, on seeded clouds:

  icp/<case>/{A, B, init_pose?, T, distances, i}   icp(A, B, ...) as called by
        testnet.py:63 (tolerance=1e-10, max_iterations=1024) and with the
        function's defaults / other arguments
  nn/{src, dst, distances, indices}                nearest_neighbor(src, dst)
  bft/<case>/{A, B, T}                             best_fit_transform(A, B),
        including a mirrored cloud (the det(R) < 0 branch, utils/icp.py:34-36)
  align/{points, fake, out}                        testnet.py:57-66 on a batch

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_icp_golden.py
"""
import os
import sys

import numpy as np

REF = os.environ.get("PCM_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "icp_golden.npz")


def rot(axis, deg):
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    i, j = [(1, 2), (2, 0), (0, 1)][axis]
    R = np.eye(3)
    R[i, i] = c
    R[j, j] = c
    R[i, j] = -s
    R[j, i] = s
    return R


def shape_cloud(rng, n):
    """A non-symmetric blob (anisotropic Gaussian + a lobe): a well-posed ICP target."""
    p = rng.standard_normal((n, 3)) * np.array([0.30, 0.18, 0.10])
    lobe = rng.random(n) < 0.25
    p[lobe] += np.array([0.35, 0.10, -0.05])
    return p.astype(np.float32)


def moved(rng, A, R, t, noise):
    B = A.astype(np.float64) @ R.T + t + noise * rng.standard_normal(A.shape)
    return B[rng.permutation(A.shape[0])].astype(np.float32)


# (name, seed, n, rotation (axis, deg), translation, noise, kwargs)
ICP_CASES = [
    ("testnet_rot10", 0, 1024, (2, 10.0), (0.05, -0.02, 0.03), 1e-3, dict(tolerance=1e-10, max_iterations=1024)),
    ("testnet_rot4_noisy", 1, 1024, (0, 4.0), (0.0, 0.02, 0.0), 2e-2, dict(tolerance=1e-10, max_iterations=1024)),
    ("defaults", 2, 1024, (1, 6.0), (0.01, 0.0, -0.02), 5e-3, dict()),
    ("max_iter_1", 3, 1024, (2, 8.0), (0.0, 0.0, 0.0), 0.0, dict(max_iterations=1)),
    ("small_n", 4, 100, (1, 3.0), (0.02, 0.01, 0.0), 1e-3, dict(tolerance=1e-10, max_iterations=200)),
    ("ragged_n", 5, 1500, (0, 7.0), (-0.03, 0.0, 0.01), 1e-3, dict(tolerance=1e-9, max_iterations=300)),
]


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REF, "utils"))
    import icp as ref_icp  # reference utils/icp.py

    out = {}
    names = []
    for name, seed, n, (ax, deg), t, noise, kw in ICP_CASES:
        rng = np.random.default_rng(seed)
        A = shape_cloud(rng, n)
        B = moved(rng, A, rot(ax, deg), np.array(t), noise)
        T, dist, i = ref_icp.icp(A, B, **kw)
        out[f"icp/{name}/A"] = A
        out[f"icp/{name}/B"] = B
        out[f"icp/{name}/T"] = T
        out[f"icp/{name}/distances"] = dist
        out[f"icp/{name}/i"] = np.int64(i)
        out[f"icp/{name}/max_iterations"] = np.int64(kw.get("max_iterations", 20))
        out[f"icp/{name}/tolerance"] = np.float64(kw.get("tolerance", 0.001))
        names.append(name)
        print(f"icp {name}: n={n} i={i} mean_err={dist.mean():.3e}")

    # init_pose (utils/icp.py:95-96): start from a rough pose
    rng = np.random.default_rng(6)
    A = shape_cloud(rng, 1024)
    B = moved(rng, A, rot(2, 20.0), np.array([0.1, 0.0, 0.0]), 1e-3)
    P = np.identity(4)
    P[:3, :3] = rot(2, 15.0)
    P[:3, 3] = (0.08, 0.0, 0.0)
    T, dist, i = ref_icp.icp(A, B, init_pose=P, tolerance=1e-10, max_iterations=1024)
    for k, v in dict(A=A, B=B, init_pose=P, T=T, distances=dist, i=np.int64(i), max_iterations=np.int64(1024),
                     tolerance=np.float64(1e-10)).items():
        out[f"icp/init_pose/{k}"] = v
    names.append("init_pose")
    print(f"icp init_pose: i={i}")
    out["icp_cases"] = np.array(names)

    rng = np.random.default_rng(7)
    src = rng.random((1000, 3))
    dst = rng.random((1000, 3))
    d, k = ref_icp.nearest_neighbor(src, dst)
    out["nn/src"], out["nn/dst"], out["nn/distances"], out["nn/indices"] = src, dst, d, k

    rng = np.random.default_rng(8)
    A = rng.random((500, 3))
    Rm = rot(0, 30.0) @ rot(2, -40.0)
    bft = {"rigid": A @ Rm.T + np.array([1.0, -2.0, 0.5]),
           "mirror": A * np.array([-1.0, 1.0, 1.0]) + 0.01 * rng.standard_normal(A.shape)}
    for name, Bm in bft.items():
        T, _, _ = ref_icp.best_fit_transform(A, Bm)
        out[f"bft/{name}/A"], out[f"bft/{name}/B"], out[f"bft/{name}/T"] = A, Bm, T
    out["bft_cases"] = np.array(list(bft))

    # testnet.py:57-66 on a batch of 3
    rng = np.random.default_rng(9)
    pts = np.stack([shape_cloud(rng, 1024) for _ in range(3)])
    fake = np.stack([moved(rng, pts[j], rot(j, 3.0 + j), np.array([0.01 * j, 0.0, 0.0]), 5e-3) for j in range(3)])
    res = []
    for j in range(3):
        T, _, _ = ref_icp.icp(pts[j], fake[j], tolerance=1e-10, max_iterations=1024)
        res.append(np.matmul(fake[j], T[:3, :3]) - T[:3, 3])
    out["align/points"], out["align/fake"] = pts, fake
    out["align/out"] = np.array(res).astype("float32")

    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
