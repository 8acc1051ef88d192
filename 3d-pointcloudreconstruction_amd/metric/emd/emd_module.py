"""EMD autograd wrapper -- drop-in for metric/emd/emd_module.py.

Same classes and signatures as the reference (emd_module.py:29-95):
``emdFunction.forward(ctx, xyz1, xyz2, eps, iters) -> (dist, assignment)``,
``.backward(ctx, graddist, gradidx) -> (gradxyz1, zeros, None, None)`` and
``emdModule()(input1, input2, eps, iters)``.

Input contract as the reference (emd_module.py:1-17, :36-39): xyz1 is the
prediction, xyz2 the ground truth, both [B, N, 3] with equal N, N % 1024 == 0,
B <= 512, coordinates normalised to [0, 1]; only xyz1 gets a gradient; the
assignment is an approximation and not guaranteed to be a bijection.

The auction runs entirely in libpcm_hip.so (one persistent workgroup per cloud,
all iterations in-kernel).  Unlike the reference (racy GetMax,
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

        if xyz1.device.type != "cuda":
            raise RuntimeError("emdFunction needs HIP device tensors; there is no CPU path")
        device = xyz1.device
        xyz1 = xyz1.contiguous().float()
        xyz2 = xyz2.contiguous().float().to(device)
        dist = torch.empty(batchsize, n, device=device)
        assignment = torch.empty(batchsize, n, device=device, dtype=torch.int32)
        pcm_hip.emd_forward(xyz1, xyz2, float(eps), int(iters), dist, assignment)
        ctx.save_for_backward(xyz1, xyz2, assignment)
        ctx.mark_non_differentiable(assignment)
        return dist, assignment

    @staticmethod
    def backward(ctx, graddist, gradidx):
        xyz1, xyz2, assignment = ctx.saved_tensors
        graddist = graddist.contiguous().float()
        gradxyz1 = torch.empty_like(xyz1)
        gradxyz2 = torch.zeros_like(xyz2)
        pcm_hip.emd_backward(xyz1, xyz2, graddist, assignment, gradxyz1)
        return gradxyz1, gradxyz2, None, None


class emdModule(nn.Module):
    def __init__(self):
        super(emdModule, self).__init__()

    def forward(self, input1, input2, eps, iters):
        return emdFunction.apply(input1, input2, eps, iters)
