"""world_size-2 gloo test of the batch-sharded loss path (CPU, no GPU).

Each rank takes its shard of a global batch (dist_loss.shard_range), evaluates
per-point distances (here with the CPU oracle standing in for the HIP kernel:
this test covers the host-side sharding and the single all-reduce), and
global_chamfer_loss / global_emd_loss must equal the single-process value over
the whole batch, with gradients equal to the global loss's gradients.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _paths():
    repo = os.path.dirname(HERE)
    for p in (os.path.join(repo, "oracle"), os.path.join(repo, "3d-pointcloudreconstruction_amd", "loss")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _global_batch():
    g = torch.Generator().manual_seed(42)
    return torch.rand(6, 256, 3, generator=g), torch.rand(6, 256, 3, generator=g)


def _worker(rank, world, port, q):
    _paths()
    import oracle as O
    import dist_loss
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, c = _global_batch()
        s, e = dist_loss.shard_range(a.shape[0], world, rank)
        la, lc = a[s:e], c[s:e]
        d1, d2, _, _ = O.chamfer_forward(la.numpy(), lc.numpy())
        t1 = torch.from_numpy(d1).requires_grad_(True)
        t2 = torch.from_numpy(d2).requires_grad_(True)
        loss = dist_loss.global_chamfer_loss(t1, t2)
        loss.backward()
        ed, _ = O.emd_forward(np.ascontiguousarray(np.repeat(la.numpy(), 4, 1)),
                              np.ascontiguousarray(np.repeat(lc.numpy(), 4, 1)), 0.005, 5)
        emd = dist_loss.global_emd_loss(torch.from_numpy(ed))
        q.put((rank, float(loss), t1.grad.numpy(), float(emd), s, e))
    finally:
        dist.destroy_process_group()


def test_sharding_ranges():
    _paths()
    import dist_loss
    for total in (0, 1, 5, 32, 33):
        for world in (1, 2, 3, 8):
            spans = [dist_loss.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_global_loss_matches_single_process():
    _paths()
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    a, c = _global_batch()
    d1, d2, _, _ = O.chamfer_forward(a.numpy(), c.numpy())
    ref = d1.mean() + d2.mean()
    ed, _ = O.emd_forward(np.repeat(a.numpy(), 4, 1), np.repeat(c.numpy(), 4, 1), 0.005, 5)
    ref_emd = np.sqrt(ed).mean(1).mean()
    for rank, loss, g1, emd, s, e in res:
        assert abs(loss - ref) < 1e-6
        assert abs(emd - ref_emd) < 1e-6
        # d(global loss)/d(local dist1) = 1 / (global B * N)
        np.testing.assert_allclose(g1, np.full_like(g1, 1.0 / d1.size), rtol=1e-6)
