"""The one-launch Chamfer step next to another kernel on the same GPU.

At N > 1 the bench captures every step's RCCL all-reduce on a side stream
that overlaps the next step's pcm_chamfer_loss_grad (bench.py capture_steps),
and that kernel's workgroups wait on each other's argmin granules (bounded:
2^16 polls, then the missing argmins are computed locally -- DESIGN.md 6).
These tests stand a kernel in for RCCL's share of the CUs (pcm_tune_occupy:
resident workgroups that only s_sleep; and a real GEMM on a side stream) and
check, at BASELINE config 2 (B=32, N=M=1024):
  * outputs bit-identical to the step run alone, and to the oracle;
  * no gradient-phase wait timed out (slow-path count unchanged);
  * the step's time, recorded (gpurun_out/test_records/coresidency.json).
Case "block_half" takes every CU of half the chip (LDS) for 1 ms: one of the
step's 257 workgroups cannot be resident until the occupier leaves, so its
batch element's other workgroups wait that long -- the step takes about the
occupier's remaining time, and is still exact without a timeout.
"""
import json
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, N, M = 32, 1024, 1024


def _record(name, value):
    d = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.getcwd()), "gpurun_out", "test_records")
    try:
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, "coresidency.json")
        rec = {}
        if os.path.exists(p):
            with open(p) as fh:
                rec = json.load(fh)
        rec[name] = value
        with open(p, "w") as fh:
            json.dump(rec, fh, indent=1)
    except OSError:
        pass


@pytest.fixture(scope="module")
def step(cuda):
    import pcm_hip
    g = torch.Generator(device="cpu").manual_seed(1234)  # the bench's clouds
    a = torch.rand(B, N, 3, generator=g)
    c = torch.rand(B, M, 3, generator=g)
    dev = cuda
    bufs = dict(x1=a.to(dev), x2=c.to(dev), d1=torch.empty(B, N, device=dev), d2=torch.empty(B, M, device=dev),
                i1=torch.empty(B, N, dtype=torch.int32, device=dev),
                i2=torch.empty(B, M, dtype=torch.int32, device=dev),
                mo=torch.empty(3, device=dev), gx1=torch.empty(B, N, 3, device=dev),
                gx2=torch.empty(B, M, 3, device=dev))
    ws = torch.zeros(pcm_hip.load_library().pcm_chamfer_workspace_bytes(B, N, M), dtype=torch.uint8, device=dev)
    w1, w2 = 1.0 / (B * N), 1.0 / (B * M)

    def run():
        pcm_hip.chamfer_loss_grad(bufs["x1"], bufs["x2"], w1, w2, bufs["d1"], bufs["d2"], bufs["i1"], bufs["i2"],
                                  bufs["mo"], bufs["gx1"], bufs["gx2"], ws)

    def outputs():
        return [bufs[k].clone() for k in ("d1", "d2", "i1", "i2", "mo", "gx1", "gx2")]

    run()
    torch.cuda.synchronize()
    return dict(a=a, c=c, run=run, outputs=outputs, ref=outputs(), ws=ws, w=(w1, w2), bufs=bufs)


def _alone_us(step, dev, reps=20):
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        step["run"]()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def _beside(step, dev, start_other):
    """start the other kernel on a side stream, give it time to become
    resident, then the step on the current stream; the step's event time"""
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        start_other()
    time.sleep(2e-4)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    step["run"]()
    e1.record(s)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) * 1000.0


# (blocks, threads, LDS bytes, microseconds) of the occupier
OCCUPIERS = {
    # a few waves on every CU, no LDS: an RCCL-like share that leaves room
    "light": (256, 256, 0, 1000),
    # 16 waves and 32 KB LDS on every CU: the step's 8-wave workgroups still fit beside it
    "heavy_waves": (256, 1024, 32 * 1024, 1000),
    # 128 KB LDS on 128 CUs (half of every XCD): the step's ~55 KB workgroups fit only
    # on the other half, two per CU -- 256 slots for 257 workgroups
    "block_half": (128, 1024, 128 * 1024, 1000),
}


@pytest.mark.parametrize("case", sorted(OCCUPIERS))
def test_loss_grad_beside_occupier(cuda, oracle, step, case):
    import pcm_hip
    blocks, threads, lds, usec = OCCUPIERS[case]
    slow0 = pcm_hip.chamfer_slow_paths(step["ws"], B, N, M)
    alone = _alone_us(step, cuda)
    for k in ("d1", "d2", "i1", "i2", "mo", "gx1", "gx2"):  # poison: the step must rewrite them
        step["bufs"][k].fill_(-7)
    us = _beside(step, cuda, lambda: pcm_hip.tune_occupy(cuda, blocks, threads, lds, usec))
    got = step["outputs"]()
    for g, r in zip(got, step["ref"]):
        assert torch.equal(g, r), case
    pcm_hip.chamfer_workspace_status(step["ws"], B, N, M)
    slow = pcm_hip.chamfer_slow_paths(step["ws"], B, N, M) - slow0
    assert slow == 0, f"{case}: {slow} gradient-phase waits timed out"
    _record(case, {"occupier": {"blocks": blocks, "threads": threads, "lds_bytes": lds, "usec": usec},
                   "step_us_beside": us, "step_us_alone": alone, "slow_paths": slow})


def test_loss_grad_beside_gemm(cuda, oracle, step):
    # a real library kernel on a side stream (hipBLASLt GEMM, ~1 ms, every CU)
    import pcm_hip
    a = torch.rand(4096, 4096, device=cuda)
    bm = torch.rand(4096, 4096, device=cuda)
    torch.mm(a, bm)
    torch.cuda.synchronize()
    slow0 = pcm_hip.chamfer_slow_paths(step["ws"], B, N, M)
    us = _beside(step, cuda, lambda: torch.mm(a, bm))
    for g, r in zip(step["outputs"](), step["ref"]):
        assert torch.equal(g, r)
    assert pcm_hip.chamfer_slow_paths(step["ws"], B, N, M) - slow0 == 0
    _record("gemm_4096", {"step_us_beside": us})


def test_reference_outputs_match_oracle(cuda, oracle, step):
    # the outputs the cases compare against are the oracle's
    d1, d2, i1, i2, mo, gx1, gx2 = [t.cpu().numpy() for t in step["ref"]]
    r1, r2, j1, j2 = oracle.chamfer_forward(step["a"].numpy(), step["c"].numpy())
    np.testing.assert_array_equal(i1, j1)
    np.testing.assert_array_equal(i2, j2)
    np.testing.assert_array_equal(d1.view(np.int32), r1.view(np.int32))
    w1, w2 = step["w"]
    g1, g2 = oracle.chamfer_backward(step["a"].numpy(), step["c"].numpy(), np.full((B, N), w1, np.float32),
                                     np.full((B, M), w2, np.float32), j1, j2)
    np.testing.assert_array_equal(gx1.view(np.int32), g1.view(np.int32))
    np.testing.assert_array_equal(gx2.view(np.int32), g2.view(np.int32))
