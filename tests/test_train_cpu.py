"""Config-4 training harness on the CPU: generator architecture pinned to the
reference, the reference's epoch schedule, and a world_size-2 gloo DDP step.

The generator's forward is compared with the REFERENCE generator's output on
the same seeded weights and image (tests/golden/fenet_golden.npz, made by
tests/golden/make_fenet_golden.py from models/repvgg_edge_nose_NEW_cmlp.py).
The DDP test uses a small torch stand-in for the loss (the HIP loss needs a
GPU; tests/test_train_gpu.py runs the real one): it covers the harness's
sharding, DDP wrapping and logged-loss reduction.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
TRAIN = os.path.join(os.path.dirname(HERE), "3d-pointcloudreconstruction_amd", "train")
if TRAIN not in sys.path:
    sys.path.insert(0, TRAIN)

import fenet  # noqa: E402
import train_step as T  # noqa: E402


def test_generator_matches_reference_golden():
    z = np.load(os.path.join(HERE, "golden", "fenet_golden.npz"))
    g = fenet.seeded_init(fenet.Generator(1024), int(z["seed"])).train()
    assert sum(p.numel() for p in g.parameters()) == int(z["n_params"]) == 177_276_968
    with torch.no_grad():
        out = g(torch.from_numpy(z["img"]))
    for name, t in zip(("pc1", "pc2", "pc3"), out):
        ref = z[name]
        assert t.shape == ref.shape
        # same torch CPU kernels in the same order: expected bit-exact; 1e-6 rel. leaves room for BLAS builds
        np.testing.assert_allclose(t.numpy(), ref, rtol=1e-6, atol=1e-6)


def test_epoch_schedule():
    # train.py:162-171 and :191-199
    assert T.loss_weights(1, 100, 100) == (100, 100)
    assert T.loss_weights(30, 100, 100) == (100, 100)
    assert T.loss_weights(31, 100, 100) == (0.0, 100)
    assert T.loss_weights(50, 100, 100) == (0.0, 100)
    assert T.loss_weights(0, 100, 100) is None and T.loss_weights(51, 100, 100) is None
    lr = 5e-4
    assert T.lr_at_epoch(1, lr) == lr and T.lr_at_epoch(10, lr) == lr
    assert T.lr_at_epoch(11, lr) == pytest.approx(lr * 0.1)
    assert T.lr_at_epoch(21, lr) == pytest.approx(lr * 0.01)
    assert T.lr_at_epoch(31, lr) == pytest.approx(lr * 1e-4)
    assert T.lr_at_epoch(41, lr) == pytest.approx(lr * 1e-7)


def test_generator_rejects_bad_point_count():
    with pytest.raises(ValueError):
        fenet.Generator(1000)


class _StandInLoss:
    """Torch-only stand-in for the CPU test (the product loss is HIP-only)."""

    def get_chamfer_loss(self, pred, gt):
        d = torch.cdist(pred, gt) ** 2
        return d.min(2).values.mean() + d.min(1).values.mean()

    def get_emd_loss(self, pred, gt, eps=0.05, iters=3000):
        return ((pred - gt) ** 2).sum(-1).clamp_min(1e-12).sqrt().mean(1).mean()


def _ddp_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        step = T.TrainStep(device="cpu", loss_fn=_StandInLoss(), seed=3)
        images, points = T.synthetic_batch(2, 1024, "cpu", seed=rank)
        before = step.gen.module.fc3_1.weight.detach().clone()
        logged = step(images, points, epoch=1, reduce_logged=True)
        w = step.gen.module.fc3_1.weight.detach()
        enc = step.gen.module.encoder.stage0.dense[0].weight.detach()
        frozen = all(p.grad is None for p in step.gen.module.edge1.parameters())
        q.put((rank, logged.tolist(), float((w - before).abs().max()), w.sum().item(), enc.sum().item(), frozen))
    finally:
        dist.destroy_process_group()


def test_ddp_step_gloo_world2():
    world, port = 2, 29000 + (os.getpid() % 500)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, l0, moved0, w0, e0, f0), (_, l1, moved1, w1, e1, f1) = res
    assert l0 == l1  # logged losses averaged over ranks
    assert all(np.isfinite(l0))
    assert moved0 > 0 and moved1 > 0  # Adam moved the weights
    assert w0 == w1 and e0 == e1  # DDP kept the replicas identical (decoder and encoder)
    assert f0 and f1  # the unused edge1 branch stays frozen
