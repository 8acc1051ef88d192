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
Every case proves the overlap it claims: the occupier's workgroups stamp
their first start and last end (s_memrealtime) and count themselves in; the
host launches the step only once all of them have started (read on a stream
of its own while they run), and one-thread clock-stamp kernels before and
after the step on its stream bracket its run.  The step must start inside the
occupier's interval, and where it fits beside the occupier, end there too.
Case "block_half" takes every CU of half the chip's LDS for 4 ms; whether the
step also ends inside it is recorded, not asserted.
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
    # first launches of the helper kernels load their code (milliseconds):
    # paid here, not between a case's occupier and its step
    scratch = torch.tensor([-1, 0, 0], dtype=torch.int64, device=dev)
    pcm_hip.tune_occupy(dev, 1, 64, 0, 1, scratch)
    pcm_hip.tune_occupy(dev, 1, 64, 128 * 1024, 1, scratch)
    pcm_hip.tune_clock_stamp(scratch[0])
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


class _Poller:
    """Reads a device tensor's current content while other streams' kernels
    still run: a copy on a stream of its own into pinned memory, both made
    before the kernels start (allocating pinned memory takes milliseconds)."""

    def __init__(self, t, dev):
        self.t = t
        # from the high-priority pool: never the same HIP stream as a side
        # stream of the default pool (torch hands those out round-robin), or
        # the copy would queue behind the kernel it is meant to watch
        self.stream = torch.cuda.Stream(dev, priority=-1)
        self.host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)

    def read(self):
        with torch.cuda.stream(self.stream):
            self.host.copy_(self.t, non_blocking=True)
        self.stream.synchronize()
        return self.host.clone()

    def wait_for(self, ready, what, limit_s=0.5):
        t0 = time.perf_counter()
        while True:
            v = self.read()
            if ready(v):
                return v
            assert time.perf_counter() - t0 < limit_s, f"{what} not reached within {limit_s} s: {v.tolist()}"


def _step_bracketed(step, dev):
    """The step on the current stream between two one-thread clock-stamp
    kernels: [m0, m1] (s_memrealtime ticks, 100 MHz) contains its whole run."""
    import pcm_hip
    marks = torch.zeros(2, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pcm_hip.tune_clock_stamp(marks[0])
    e0.record(s)
    step["run"]()
    e1.record(s)
    pcm_hip.tune_clock_stamp(marks[1])
    torch.cuda.synchronize(dev)
    m0, m1 = (int(x) for x in marks.cpu())
    return e0.elapsed_time(e1) * 1000.0, m0, m1


# (blocks, threads, LDS bytes, microseconds) of the occupier
OCCUPIERS = {
    # a few waves on every CU, no LDS: an RCCL-like share that leaves room
    "light": (256, 256, 0, 4000),
    # 16 waves and 32 KB LDS on every CU: the step's 8-wave workgroups still fit beside it
    "heavy_waves": (256, 1024, 32 * 1024, 4000),
    # 128 KB LDS on 128 CUs (half of every XCD): the step's workgroups fit only
    # on the other half
    "block_half": (128, 1024, 128 * 1024, 4000),
}


@pytest.mark.parametrize("case", sorted(OCCUPIERS))
def test_loss_grad_beside_occupier(cuda, oracle, step, case):
    # the occupier is RESIDENT (every workgroup started: its own count, read
    # while it runs) before the step is launched, and the step's bracketing
    # clock stamps prove it started inside the occupier's [first start, last
    # end]; where the step fits beside the occupier it must also END inside it
    import pcm_hip
    blocks, threads, lds, usec = OCCUPIERS[case]
    slow0 = pcm_hip.chamfer_slow_paths(step["ws"], B, N, M)
    alone = _alone_us(step, cuda)
    for k in ("d1", "d2", "i1", "i2", "mo", "gx1", "gx2"):  # poison: the step must rewrite them
        step["bufs"][k].fill_(-7)
    stamps = torch.tensor([-1, 0, 0], dtype=torch.int64, device=cuda)  # (-1: the largest unsigned start)
    poller = _Poller(stamps, cuda)
    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    torch.cuda.synchronize(cuda)
    with torch.cuda.stream(side):
        pcm_hip.tune_occupy(cuda, blocks, threads, lds, usec, stamps)
    poller.wait_for(lambda v: int(v[2]) == blocks, f"{case}: all {blocks} occupier workgroups resident")
    us, m0, m1 = _step_bracketed(step, cuda)
    torch.cuda.synchronize(cuda)
    o0, o1, started = (int(x) for x in stamps.cpu())
    got = step["outputs"]()
    for g, r in zip(got, step["ref"]):
        assert torch.equal(g, r), case
    pcm_hip.chamfer_workspace_status(step["ws"], B, N, M)
    slow = pcm_hip.chamfer_slow_paths(step["ws"], B, N, M) - slow0
    assert slow == 0, f"{case}: {slow} gradient-phase waits timed out"
    assert started == blocks
    assert o0 < m0 < o1, f"{case}: the step did not start while the occupier ran ({o0}, {m0}, {o1})"
    fits = case != "block_half"
    if fits:
        assert m1 < o1, f"{case}: the step did not finish beside the occupier ({m1} >= {o1})"
    _record(case, {"occupier": {"blocks": blocks, "threads": threads, "lds_bytes": lds, "usec": usec},
                   "step_us_beside": us, "step_us_alone": alone, "slow_paths": slow,
                   "ticks_100mhz": {"occupier_first_start": 0, "step_start_mark": m0 - o0,
                                    "step_end_mark": m1 - o0, "occupier_last_end": o1 - o0},
                   "step_inside_occupier": m1 < o1})


def test_loss_grad_beside_gemm(cuda, oracle, step):
    # real library kernels on a side stream (four 4096^3 fp32 GEMMs on every
    # CU, ~1 ms each) bracketed by clock stamps; the step is launched only once the
    # GEMM's leading stamp has landed (the GEMM is then executing), and must
    # start before its trailing stamp: launched while the GEMM held the CUs
    import pcm_hip
    a = torch.rand(4096, 4096, device=cuda)
    bm = torch.rand(4096, 4096, device=cuda)
    torch.mm(a, bm)
    torch.cuda.synchronize()
    slow0 = pcm_hip.chamfer_slow_paths(step["ws"], B, N, M)
    gm = torch.zeros(2, dtype=torch.int64, device=cuda)
    poller = _Poller(gm, cuda)
    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    torch.cuda.synchronize(cuda)
    with torch.cuda.stream(side):
        pcm_hip.tune_clock_stamp(gm[0])
        for _ in range(4):  # ~4 ms of GEMMs on every CU
            torch.mm(a, bm)
        pcm_hip.tune_clock_stamp(gm[1])
    poller.wait_for(lambda v: int(v[0]) != 0, "the GEMM's leading stamp")
    us, m0, m1 = _step_bracketed(step, cuda)
    torch.cuda.synchronize(cuda)
    g0, g1 = (int(x) for x in gm.cpu())
    for g, r in zip(step["outputs"](), step["ref"]):
        assert torch.equal(g, r)
    assert pcm_hip.chamfer_slow_paths(step["ws"], B, N, M) - slow0 == 0
    assert g0 < m0 < g1, f"the step did not start while the GEMM ran ({g0}, {m0}, {g1})"
    _record("gemm_4096", {"step_us_beside": us,
                          "ticks_100mhz": {"gemm_start_mark": 0, "step_start_mark": m0 - g0,
                                           "step_end_mark": m1 - g0, "gemm_end_mark": g1 - g0},
                          "step_inside_gemm": m1 < g1})


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
