"""EMD autograd wrapper -- drop-in for metric/emd/emd_module.py.

Same classes and signatures as the reference (emd_module.py:29-95):
``emdFunction.forward(ctx, xyz1, xyz2, eps, iters) -> (dist, assignment)``,
``.backward(ctx, graddist, gradidx) -> (gradxyz1, zeros, None, None)`` and
``emdModule()(input1, input2, eps, iters)``.

Input contract as the reference (emd_module.py:1-17, :36-39): xyz1 is the
prediction, xyz2 the ground truth, both [B, N, 3] with equal N, N % 1024 == 0,
B <= 512, coordinates normalised to [0, 1]; only xyz1 gets a gradient; the
assignment is an approximation and not guaranteed to be a bijection.

The auction runs entirely in libpcm_hip.so (one persistent master workgroup per
cloud runs all iterations in-kernel; helper workgroups take the full scans of
heavy iterations).  Any N % 1024 == 0 is accepted, as by the reference's
kernel (emd_cuda.cu:236-249).  Unlike the reference (racy GetMax,
emd_cuda.cu:188-190) the result is deterministic: bidders tying inside the
1e-6 window resolve to the lowest point index.
"""
import os
import sys

import torch
from torch import nn
from torch.autograd import Function

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcm_hip  # noqa: E402


class emdFunction(Function):
    @staticmethod
    def forward(ctx, xyz1, xyz2, eps, iters):
        batchsize, n, _ = xyz1.size()
        _, m, _ = xyz2.size()

        assert n == m
        assert xyz1.size()[0] == xyz2.size()[0]
        assert n % 1024 == 0
        assert batchsize <= 512

        # emd_module.py:41-42 moves both clouds to the GPU itself
        # (`.contiguous().float().cuda()`); so does this wrapper: to the device
        # of whichever cloud is already on one, else the current HIP device.
        # Compute never happens on the host.
        if xyz1.is_cuda:
            device = xyz1.device
        elif xyz2.is_cuda:
            device = xyz2.device
        elif torch.cuda.is_available():
            device = torch.device("cuda", torch.cuda.current_device())
        else:
            raise RuntimeError("emdFunction needs a HIP device (none is visible); there is no CPU path")
        ctx.in_devices = (xyz1.device, xyz2.device)
        xyz1 = xyz1.contiguous().float().to(device)
        xyz2 = xyz2.contiguous().float().to(device)
        dist = torch.empty(batchsize, n, device=device)
        assignment = torch.empty(batchsize, n, device=device, dtype=torch.int32)
        pcm_hip.emd_forward(xyz1, xyz2, float(eps), int(iters), dist, assignment)
        ctx.save_for_backward(xyz1, xyz2, assignment)
        ctx.mark_non_differentiable(assignment)
        ctx.set_materialize_grads(False)  # no zero-fill kernel for the int32 assignment's gradient
        return dist, assignment

    @staticmethod
    def backward(ctx, graddist, gradidx):
        xyz1, xyz2, assignment = ctx.saved_tensors
        if graddist is None:  # dist unused by the loss
            graddist = torch.zeros(assignment.shape, device=xyz1.device)
        graddist = graddist.contiguous().float().to(xyz1.device)
        gradxyz1 = torch.empty_like(xyz1)
        pcm_hip.emd_backward(xyz1, xyz2, graddist, assignment, gradxyz1)
        # gradients go back to where the inputs came from (autograd requires it)
        dev1, dev2 = ctx.in_devices
        return gradxyz1.to(dev1), torch.zeros(xyz2.shape, device=dev2), None, None


class emdModule(nn.Module):
    def __init__(self):
        super(emdModule, self).__init__()

    def forward(self, input1, input2, eps, iters):
        return emdFunction.apply(input1, input2, eps, iters)
