"""CPU ORACLE for ICP alignment (test infrastructure only).

A numpy restatement of the reference's utils/icp.py, which SURVEY.md §8f row 3
names as the next caller of the nearest-neighbour kernel:
  best_fit_transform  utils/icp.py:4-46   (Kabsch: centroids, H = AA^T BB, SVD,
                                           reflection fix, t = cB - R cA)
  nearest_neighbor    utils/icp.py:49-65  (sklearn NearestNeighbors(n_neighbors=1);
                                           here brute force in float64)
  icp                 utils/icp.py:68-118 (homogeneous src/dst, NN, best fit,
                                           src = T src, |prev - mean| < tol stop,
                                           final best_fit_transform(A, src))
The caller is testnet.py:62-64 (tolerance=1e-10, max_iterations=1024, A = the
ground-truth cloud, B = the prediction).

nearest_neighbor evaluates the squared distance as sklearn's Euclidean rdist
does, ((dx*dx + dy*dy) + dz*dz) in float64 with dx = src - dst, takes sqrt, and
breaks exact ties toward the lowest index (sklearn leaves ties unspecified).

Parity: pinned against the reference itself through tests/golden/icp_golden.npz
(tests/golden/make_icp_golden.py runs the reference's utils/icp.py with sklearn
1.7.2 in the build container).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import numpy as np


def best_fit_transform(A, B):
    """utils/icp.py:4-46.  Returns (T, R, t)."""
    assert A.shape == B.shape
    m = A.shape[1]
    centroid_A = np.mean(A, axis=0)
    centroid_B = np.mean(B, axis=0)
    AA = A - centroid_A
    BB = B - centroid_B
    H = AA.T @ BB
    U, _, Vt = np.linalg.svd(H)
    R = Vt.T @ U.T
    if np.linalg.det(R) < 0:  # reflection: flip the smallest singular direction
        Vt[m - 1, :] *= -1
        R = Vt.T @ U.T
    t = centroid_B.T - R @ centroid_A.T
    T = np.identity(m + 1)
    T[:m, :m] = R
    T[:m, m] = t
    return T, R, t


def sqdist_matrix(src, dst):
    """[n, m] float64 squared distances in sklearn's rdist order."""
    src = np.asarray(src, np.float64)
    dst = np.asarray(dst, np.float64)
    acc = None
    for c in range(src.shape[1]):
        d = src[:, None, c] - dst[None, :, c]
        acc = d * d if acc is None else acc + d * d
    return acc


def nearest_neighbor(src, dst, block: int = 2048):
    """utils/icp.py:49-65 by brute force: (distances, indices), lowest index on ties."""
    src = np.asarray(src, np.float64)
    dst = np.asarray(dst, np.float64)
    n = src.shape[0]
    dist = np.empty(n, np.float64)
    idx = np.empty(n, np.int64)
    for s in range(0, n, block):
        d2 = sqdist_matrix(src[s:s + block], dst)
        k = d2.argmin(axis=1)  # first occurrence = lowest index
        idx[s:s + block] = k
        dist[s:s + block] = np.sqrt(d2[np.arange(k.size), k])
    return dist, idx


def nearest_neighbor_sklearn(src, dst):
    """utils/icp.py:49-65 verbatim in algorithm: sklearn's kd-tree (the CPU
    baseline's timing of the reference's own NN search)."""
    from sklearn.neighbors import NearestNeighbors
    neigh = NearestNeighbors(n_neighbors=1)
    neigh.fit(dst)
    distances, indices = neigh.kneighbors(src, return_distance=True)
    return distances.ravel(), indices.ravel()


def icp(A, B, init_pose=None, max_iterations=20, tolerance=0.001, nn=None):
    """utils/icp.py:68-118.  Returns (T, distances, i).  nn: the NN search
    (default: the float64 brute force)."""
    nn = nn or nearest_neighbor
    assert A.shape == B.shape
    m = A.shape[1]
    src = np.ones((m + 1, A.shape[0]))
    dst = np.ones((m + 1, B.shape[0]))
    src[:m, :] = np.copy(A.T)
    dst[:m, :] = np.copy(B.T)
    if init_pose is not None:
        src = init_pose @ src
    prev_error = 0
    for i in range(max_iterations):
        distances, indices = nn(src[:m, :].T, dst[:m, :].T)
        T, _, _ = best_fit_transform(src[:m, :].T, dst[:m, indices].T)
        src = T @ src
        mean_error = np.mean(distances)
        if np.abs(prev_error - mean_error) < tolerance:
            break
        prev_error = mean_error
    T, _, _ = best_fit_transform(A, src[:m, :].T)
    return T, distances, i


def align(points, fake, tolerance=1e-10, max_iterations=1024):
    """testnet.py:57-66: per sample T = icp(points, fake), fake @ T[:3,:3] - T[:3,3]."""
    out = []
    for k in range(fake.shape[0]):
        T, _, _ = icp(points[k], fake[k], tolerance=tolerance, max_iterations=max_iterations)
        out.append(np.matmul(fake[k], T[:3, :3]) - T[:3, 3])
    return np.array(out).astype("float32")
