"""The one-launch Chamfer step next to another kernel on the same GPU.

At N > 1 the bench captures every step's RCCL all-reduce on a side stream
that overlaps the next step's pcm_chamfer_loss_grad (bench.py capture_steps),
and that kernel's workgroups wait on each other's argmin granules (bounded:
2^16 polls, then the missing argmins are computed locally -- DESIGN.md 6).
These tests stand a kernel in for RCCL's share of the CUs (pcm_tune_occupy:
resident workgroups that only s_sleep; and real GEMMs on a side stream) and
check, at BASELINE config 2 (B=32, N=M=1024), through tools/coresidency_probe.py
(one process per case, see there):
  * outputs bit-identical to the step run alone (which is the oracle's,
    test_reference_outputs_match_oracle);
  * no gradient-phase wait timed out (slow-path count unchanged);
  * OVERLAP, proven with the GPU's real-time clock: the other kernel tells the
    host through pinned memory that it is running, the step is launched only
    then, and one-thread clock-stamp kernels before and after the step must
    fall inside the other kernel's [first start, last end] -- the step's start
    always, its end where its workgroups fit beside the occupier;
  * the times and clock stamps, recorded (gpurun_out/test_records/coresidency.json).
"""
import json
import os

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


CASES = ("block_half", "gemm", "heavy_waves", "light")


@pytest.mark.parametrize("case", CASES)
def test_loss_grad_beside_other_kernel(cuda, case):
    # tools/coresidency_probe.py in a process of its own (two fresh streams:
    # in this long-lived process torch's stream pool may hand out two streams
    # that share a hardware queue, which would run them one after the other).
    # The other kernel signals through pinned host memory that it is running
    # (every occupier workgroup started; the GEMMs' leading clock stamp); the
    # step is launched only then, and its bracketing clock stamps must fall
    # inside the other kernel's run: started inside always; ended inside where
    # the step fits beside it.  Outputs bit-identical to the step alone, and no
    # gradient-phase wait timed out.
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "coresidency_probe.py"), case],
                       capture_output=True, text=True, timeout=110)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and lines, f"{case}: rc {r.returncode}\n{r.stdout}\n{r.stderr[-2000:]}"
    out = json.loads(lines[-1])
    _record(case, out)
    assert out["outputs_bit_identical"], case
    assert out["slow_paths"] == 0, f"{case}: {out['slow_paths']} gradient-phase waits timed out"
    assert out["step_started_inside"], f"{case}: the step did not start while the other kernel ran: {out}"
    if case in ("light", "heavy_waves"):  # the step's workgroups fit beside the occupier
        assert out["step_ended_inside"], f"{case}: the step did not finish beside the occupier: {out}"


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
