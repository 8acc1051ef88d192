#!/usr/bin/env python3
"""One co-residency case of the one-launch Chamfer step, in a process of its
own (tests/test_coresidency_gpu.py runs it as a subprocess):

    python tools/coresidency_probe.py CASE

A fresh process creates exactly two streams, one after the other, for the
other kernel and the step: HIP maps streams onto a few hardware queues
(GPU_MAX_HW_QUEUES) in creation order, and two streams on one queue run one
after the other -- in a long-lived process two streams chosen by torch's
round-robin pool can share a queue.  The host learns that the other kernel
is running from pinned host memory the kernel itself writes (the occupier's
last workgroup to start; a clock stamp in front of the GEMMs), not from a
copy on a third stream.  Prints one JSON line: the step's outputs against
the step alone (bit for bit), its slow-path count, its time beside and alone,
and the s_memrealtime ticks (100 MHz) of the other kernel's start and end and
of the clock stamps bracketing the step.
"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402

B, N, M = 32, 1024, 1024
# (blocks, threads, LDS bytes, microseconds) of the occupier
OCCUPIERS = {
    "light": (256, 256, 0, 4000),                     # a few waves on every CU, no LDS (an RCCL-like share)
    "heavy_waves": (256, 1024, 32 * 1024, 4000),      # 16 waves and 32 KB LDS on every CU
    "block_half": (128, 1024, 128 * 1024, 4000),      # 128 KB LDS on half the CUs
}


def main():
    case = sys.argv[1]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    s_other = torch.cuda.Stream(dev)
    s_step = torch.cuda.Stream(dev)
    assert s_other.cuda_stream != s_step.cuda_stream
    g = torch.Generator(device="cpu").manual_seed(1234)  # the bench's clouds
    x1 = torch.rand(B, N, 3, generator=g).to(dev)
    x2 = torch.rand(B, M, 3, generator=g).to(dev)
    bufs = dict(d1=torch.empty(B, N, device=dev), d2=torch.empty(B, M, device=dev),
                i1=torch.empty(B, N, dtype=torch.int32, device=dev),
                i2=torch.empty(B, M, dtype=torch.int32, device=dev), mo=torch.empty(3, device=dev),
                gx1=torch.empty(B, N, 3, device=dev), gx2=torch.empty(B, M, 3, device=dev))
    ws = torch.zeros(pcm_hip.load_library().pcm_chamfer_workspace_bytes(B, N, M), dtype=torch.uint8, device=dev)
    w1, w2 = 1.0 / (B * N), 1.0 / (B * M)
    keys = ("d1", "d2", "i1", "i2", "mo", "gx1", "gx2")

    def run():
        pcm_hip.chamfer_loss_grad(x1, x2, w1, w2, bufs["d1"], bufs["d2"], bufs["i1"], bufs["i2"], bufs["mo"],
                                  bufs["gx1"], bufs["gx2"], ws)

    marks = torch.zeros(2, dtype=torch.int64, device=dev)
    stamps = torch.tensor([-1, 0, 0], dtype=torch.int64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    hstamp = torch.zeros(1, dtype=torch.int64, pin_memory=True)
    a = torch.rand(4096, 4096, device=dev)
    bm = torch.rand(4096, 4096, device=dev)
    with torch.cuda.stream(s_step):  # first launches (code loading) and the reference outputs
        for _ in range(3):
            run()
        pcm_hip.tune_clock_stamp(marks[0])
    with torch.cuda.stream(s_other):
        pcm_hip.tune_occupy(dev, 1, 64, 128 * 1024, 1, stamps)
        torch.mm(a, bm)
    torch.cuda.synchronize()
    ref = [bufs[k].clone() for k in keys]
    alones = []
    for _ in range(7):  # one launch between two events, as the step beside is timed
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s_step):
            e0.record()
            run()
            e1.record()
        e1.synchronize()
        alones.append(e0.elapsed_time(e1) * 1000.0)
    alone = sorted(alones)[len(alones) // 2]
    slow0 = pcm_hip.chamfer_slow_paths(ws, B, N, M)
    for k in keys:  # poison: the step must rewrite them
        bufs[k].fill_(-7)
    stamps.copy_(torch.tensor([-1, 0, 0], dtype=torch.int64))
    marks.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s_other):
        if case == "gemm":
            pcm_hip.tune_clock_stamp(hstamp)  # pinned host memory: the host sees it land
            for _ in range(4):
                torch.mm(a, bm)
            pcm_hip.tune_clock_stamp(stamps[1:2])
        else:
            blocks, threads, lds, usec = OCCUPIERS[case]
            pcm_hip.tune_occupy(dev, blocks, threads, lds, usec, stamps, flag)
    seen = flag if case != "gemm" else hstamp
    while int(seen[0]) == 0:
        if time.perf_counter() - t0 > 0.5:
            torch.cuda.synchronize()
            print(json.dumps({"case": case, "error": "the other kernel never signalled", "stamps": stamps.tolist()}))
            return 1
    waited_us = (time.perf_counter() - t0) * 1e6
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s_step):
        pcm_hip.tune_clock_stamp(marks[0])
        e0.record()
        run()
        e1.record()
        pcm_hip.tune_clock_stamp(marks[1])
    torch.cuda.synchronize()
    beside = e0.elapsed_time(e1) * 1000.0
    st = [int(v) for v in stamps.cpu()]
    o0 = int(hstamp[0]) if case == "gemm" else st[0]
    o1 = st[1]
    m0, m1 = (int(v) for v in marks.cpu())
    same = all(torch.equal(bufs[k], r) for k, r in zip(keys, ref))
    slow = pcm_hip.chamfer_slow_paths(ws, B, N, M) - slow0
    out = {"case": case, "outputs_bit_identical": same, "slow_paths": slow, "step_us_beside": beside,
           "step_us_alone": alone, "host_wait_us": waited_us,
           "other": ({"kernel": "4 x torch.mm 4096^3 fp32"} if case == "gemm" else
                     dict(zip(("blocks", "threads", "lds_bytes", "usec"), OCCUPIERS[case]), started=st[2])),
           "ticks_100mhz": {"other_start": 0, "step_start_mark": m0 - o0, "step_end_mark": m1 - o0,
                            "other_end": o1 - o0},
           "step_started_inside": o0 < m0 < o1, "step_ended_inside": m1 < o1}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
