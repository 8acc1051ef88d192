"""Config-4 training step: 3D-FENet generator + Chamfer/EMD loss, one process per GPU.

Counterpart of the reference's training loop body (train.py:148-177) with the
loss path on this build's HIP kernels (loss/loss.py -> chamfer_3DLoss, emdModule):

  fake = gen(images)[2]                       # [B, 3, P]          train.py:160
  cd   = Loss.get_chamfer_loss(fake^T, gt)    # mean d1 + mean d2  train.py:163,167
  emd  = Loss.get_emd_loss(fake^T, gt)        # eps .05, 3000 it   train.py:164,168; loss/loss.py:23
  total = lambda_emd*emd            (30 < epoch <= 50)              train.py:162-165
        = lambda_cd*cd + lambda_emd*emd  (0 < epoch <= 30)          train.py:166-169
  zero_grad; total.backward(); Adam step (lr 5e-4, betas (.9,.999), wd 1e-4)   train.py:113,175-177

Differences from the reference, all deliberate:
  * no ``.item()`` inside the step (train.py:173 synchronised every step):
    the step returns device tensors and the caller reads them when it logs;
  * multi-GPU: the reference is single-GPU (train.py:5).  Here each rank owns
    a contiguous slice of the global batch and the generator is wrapped in
    DistributedDataParallel (RCCL over xGMI).  DDP's bucketed gradient
    all-reduce (177 M fp32 parameters, 709 MB) starts while backward is still
    running: the decoder's fc1_1 (134 M parameters, 537 MB) is the first large
    gradient produced, so its buckets travel while the encoder's backward runs.
    Buckets are large (``bucket_cap_mb``, default 100 MB) because xGMI is
    point-to-point and per-link bound: few large rings beat many small ones.
    The loss itself needs no collective (each rank's mean loss gives, after
    DDP's averaging, the gradient of the global mean over equal shards);
    the logged values are averaged over ranks with one 3-float all-reduce;
  * BatchNorm statistics are per rank (as DDP does by default); with one
    rank the step is the reference's step.
"""
from __future__ import annotations

import os
import sys

import torch
import torch.distributed as dist

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(_PKG, "loss"), os.path.join(_PKG, "train")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from fenet import Generator, seeded_init  # noqa: E402


def lr_at_epoch(epoch: int, base_lr: float = 5e-4) -> float:
    """Learning rate in force during `epoch` (train.py:191-199: after every
    10th epoch lr *= 0.1 below 30, 0.01 in [30, 40), 0.001 from 40)."""
    lr = base_lr
    for e in range(10, epoch, 10):
        lr *= 0.1 if e < 30 else (0.01 if e < 40 else 0.001)
    return lr


def loss_weights(epoch: int, lambda_cd: float, lambda_emd: float):
    """(w_cd, w_emd) for `epoch` (train.py:162-171); None = the reference skips the batch."""
    if 0 < epoch <= 30:
        return lambda_cd, lambda_emd
    if 30 < epoch <= 50:
        return 0.0, lambda_emd
    return None


class TrainStep:
    """One optimisation step of the generator on one rank.

    ``loss_fn`` must provide ``get_chamfer_loss(pred, gt)`` and
    ``get_emd_loss(pred, gt, eps=..., iters=...)`` on [B, P, 3] clouds; the
    default is this build's ``loss.Loss`` (HIP kernels)."""

    def __init__(self, gen: torch.nn.Module | None = None, *, device=None, loss_fn=None, lr: float = 5e-4,
                 lambda_cd: float = 100.0, lambda_emd: float = 100.0, emd_eps: float = 0.05,
                 emd_iters: int = 3000, bucket_cap_mb: float = 100.0, seed: int = 0,
                 channels_last: bool = False):
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        gen = gen if gen is not None else seeded_init(Generator(1024), seed)
        gen = gen.to(self.device).train()
        self.channels_last = channels_last
        if channels_last:  # NHWC activations for the encoder's convolutions (same fp32 math)
            gen = gen.to(memory_format=torch.channels_last)
        self.world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
        if self.world > 1:
            ids = [self.device.index] if self.device.type == "cuda" else None
            gen = torch.nn.parallel.DistributedDataParallel(
                gen, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)
        self.gen = gen
        if loss_fn is None:
            from loss import Loss
            loss_fn = Loss()
        self.loss_fn = loss_fn
        self.lambda_cd, self.lambda_emd = lambda_cd, lambda_emd
        self.emd_eps, self.emd_iters = emd_eps, emd_iters
        params = [p for p in gen.parameters() if p.requires_grad]
        kw = dict(lr=lr, betas=(0.9, 0.999), weight_decay=1e-4)
        if self.device.type == "cuda":
            kw["fused"] = True  # one multi-tensor launch over 177 M parameters
        self.opt = torch.optim.Adam(params, **kw)
        self.base_lr = lr

    def set_epoch(self, epoch: int):
        for g in self.opt.param_groups:
            g["lr"] = lr_at_epoch(epoch, self.base_lr)

    def losses(self, images, points, epoch: int):
        """Forward and loss only: (total, chamfer, emd) as device scalars."""
        w = loss_weights(epoch, self.lambda_cd, self.lambda_emd)
        if w is None:
            raise ValueError(f"epoch {epoch}: the reference trains epochs 1..50 only (train.py:170-171)")
        if self.channels_last:
            images = images.contiguous(memory_format=torch.channels_last)
        _, _, fake = self.gen(images)
        pred = fake.transpose(2, 1)
        cd = self.loss_fn.get_chamfer_loss(pred, points)
        emd = self.loss_fn.get_emd_loss(pred, points, eps=self.emd_eps, iters=self.emd_iters)
        total = emd * w[1] if w[0] == 0.0 else cd * w[0] + emd * w[1]
        return total, cd, emd

    def __call__(self, images, points, epoch: int = 1, reduce_logged: bool = False):
        """Forward, loss, backward, Adam step.  Returns device tensor [total, cd, emd]
        (averaged over ranks when `reduce_logged`); nothing here synchronises the host."""
        total, cd, emd = self.losses(images, points, epoch)
        self.opt.zero_grad(set_to_none=True)
        total.backward()
        self.opt.step()
        logged = torch.stack([total.detach(), cd.detach(), emd.detach()])
        if reduce_logged and self.world > 1:
            dist.all_reduce(logged, op=dist.ReduceOp.SUM)
            logged /= self.world
        return logged


def synthetic_batch(batch: int, num_points: int = 1024, device="cpu", seed: int = 0):
    """Images of train.py's input shape and range ([B,3,128,128], Normalize(.5,.5) -> [-1,1])
    and ground-truth clouds in [0,1) (the range the EMD kernel assumes, emd_module.py:9)."""
    g = torch.Generator().manual_seed(seed)
    images = torch.rand(batch, 3, 128, 128, generator=g) * 2 - 1
    points = torch.rand(batch, num_points, 3, generator=g)
    return images.to(device), points.to(device)
