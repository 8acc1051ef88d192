"""ICP alignment -- MI355X counterpart of the reference's utils/icp.py.

Same functions, signatures and return values as the reference
(utils/icp.py:4, :49, :68), numpy in and numpy out, float64:
  best_fit_transform(A, B)                     -> (T, R, t)
  nearest_neighbor(src, dst)                   -> (distances, indices)
  icp(A, B, init_pose=None, max_iterations=20, tolerance=0.001)
                                               -> (T, distances, i)
The compute runs in libpcm_hip.so (csrc/icp.hip: the whole ICP loop is one
launch, one workgroup per cloud pair) on the current HIP device; there is no
CPU path, so without a GPU or the library these raise.

Batched forms for the evaluation loop:
  icp_batch(A, B, ...)          many pairs in one launch, device tensors
  align_predictions(fake, points, tolerance=1e-10, max_iterations=1024)
      testnet.py:57-67 -- per sample T = icp(points, fake), then
      fake @ T[:3,:3] - T[:3,3] as float32 -- in one launch for the batch.

Differences from the reference: the spatial dimension must be 3 (the
reference accepts any m); max_iterations must be >= 1 (the reference fails
with UnboundLocalError); exact nearest-neighbour ties resolve to the lowest
index (sklearn leaves them unspecified); icp clouds are limited to
pcm_hip.ICP_MAX_POINTS points.
Non-finite inputs raise ValueError, as sklearn's input check does.
"""
import os
import sys

import numpy as np
import torch

_METRIC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "metric")
if _METRIC not in sys.path:
    sys.path.append(_METRIC)
import pcm_hip  # noqa: E402


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("ICP runs on the HIP device (libpcm_hip.so); no GPU is visible and there is no CPU path")
    return torch.device("cuda", torch.cuda.current_device())


def _cloud(X, name):
    X = np.asarray(X, dtype=np.float64)
    if X.ndim != 2 or X.shape[1] != 3:
        raise ValueError(f"{name} must be an N x 3 array (got shape {X.shape}); only 3-D clouds are supported")
    if X.shape[0] == 0:
        raise ValueError(f"{name} has 0 points")
    if not np.isfinite(X).all():
        raise ValueError(f"Input {name} contains NaN or infinity.")
    return X


def _to_dev(X, dev):
    return torch.from_numpy(np.ascontiguousarray(X, dtype=np.float64)).to(dev)


def best_fit_transform(A, B):
    """utils/icp.py:4-46: least-squares rigid transform mapping A onto B -> (T, R, t)."""
    assert A.shape == B.shape
    A, B = _cloud(A, "A"), _cloud(B, "B")
    dev = _device()
    T = torch.empty(1, 4, 4, dtype=torch.float64, device=dev)
    pcm_hip.best_fit_transform(_to_dev(A, dev)[None], _to_dev(B, dev)[None], T)
    T = T[0].cpu().numpy()
    return T, T[:3, :3].copy(), T[:3, 3].copy()


def nearest_neighbor(src, dst):
    """utils/icp.py:49-65: Euclidean nearest neighbour in dst of each src point
    -> (distances float64 [N], indices int64 [N])."""
    assert src.shape == dst.shape
    src, dst = _cloud(src, "src"), _cloud(dst, "dst")
    dev = _device()
    n = src.shape[0]
    dist = torch.empty(1, n, dtype=torch.float64, device=dev)
    idx = torch.empty(1, n, dtype=torch.int32, device=dev)
    pcm_hip.nearest_neighbor(_to_dev(src, dev)[None], _to_dev(dst, dev)[None], dist, idx)
    return dist[0].cpu().numpy(), idx[0].cpu().numpy().astype(np.int64)


def icp_batch(A, B, init_pose=None, max_iterations=20, tolerance=0.001):
    """icp on b pairs at once: A, B device tensors [b, n, 3] (any float dtype;
    computed in float64), init_pose None or [b, 4, 4].  Returns device tensors
    (T [b,4,4] float64, distances [b,n] float64, iterations [b] int32)."""
    if A.shape != B.shape or A.dim() != 3 or A.shape[2] != 3:
        raise ValueError(f"A and B must both be [b, n, 3] (got {tuple(A.shape)} and {tuple(B.shape)})")
    if int(max_iterations) < 1:
        raise ValueError("max_iterations must be >= 1")
    b, n, _ = A.shape
    if n == 0:
        raise ValueError("clouds have 0 points")
    if n > pcm_hip.ICP_MAX_POINTS:
        raise ValueError(f"icp supports clouds of up to {pcm_hip.ICP_MAX_POINTS} points (got {n})")
    A = A.to(torch.float64).contiguous()
    B = B.to(torch.float64).contiguous()
    if not (torch.isfinite(A).all() and torch.isfinite(B).all()):
        raise ValueError("Input contains NaN or infinity.")
    P = None
    if init_pose is not None:
        P = torch.as_tensor(init_pose, dtype=torch.float64, device=A.device).expand(b, 4, 4).contiguous()
    T = torch.empty(b, 4, 4, dtype=torch.float64, device=A.device)
    dist = torch.empty(b, n, dtype=torch.float64, device=A.device)
    iters = torch.empty(b, dtype=torch.int32, device=A.device)
    pcm_hip.icp(A, B, P, int(max_iterations), float(tolerance), T, dist, iters)
    return T, dist, iters


def icp(A, B, init_pose=None, max_iterations=20, tolerance=0.001):
    """utils/icp.py:68-118: the transform mapping A onto B -> (T, distances, i)."""
    assert A.shape == B.shape
    A, B = _cloud(A, "A"), _cloud(B, "B")
    dev = _device()
    P = None if init_pose is None else np.asarray(init_pose, dtype=np.float64).reshape(1, 4, 4)
    T, dist, iters = icp_batch(_to_dev(A, dev)[None], _to_dev(B, dev)[None],
                               None if P is None else _to_dev(P, dev), max_iterations, tolerance)
    return T[0].cpu().numpy(), dist[0].cpu().numpy(), int(iters[0].item())


def align_predictions(fake, points, tolerance=1e-10, max_iterations=1024):
    """testnet.py:57-67 for a batch: align each predicted cloud to its ground
    truth (T = icp(points[k], fake[k])) and return fake @ T[:3,:3] - T[:3,3]
    as a float32 device tensor [b, n, 3]."""
    T, _, _ = icp_batch(points, fake, None, max_iterations, tolerance)
    out = torch.matmul(fake.to(torch.float64), T[:, :3, :3]) - T[:, None, :3, 3]
    return out.to(torch.float32)
