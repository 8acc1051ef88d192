#!/usr/bin/env python3
"""Where the bench's timed region loses time outside the kernel: the one-launch
Chamfer step (BASELINE config 2, the bench's clouds) timed by wall clock around
K = 20 steps in several launch forms, beside the GPU-side (HIP event) time of
the same work and the wall cost of an empty synchronised region.

    python tools/probe_replay.py
"""
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def wall(fn, dev, reps=15):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        out.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(out), min(out)


def events(fn, dev, reps=15):
    s = torch.cuda.current_stream(dev)
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        e0.record(s)
        fn()
        e1.record(s)
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1000.0)
    return statistics.median(out)


def main():
    dev = torch.device("cuda:0")
    K = 20
    step = bench.ChamferStep(dev, 1, seed=bench.BENCH_SEED, slots=K)
    for _ in range(3):
        step(0)
    torch.cuda.synchronize(dev)
    forms = {}
    for per in (20, 10, 5, 1):
        g = bench.capture_steps(step, per, dev, 1, False)
        g.replay()
        torch.cuda.synchronize(dev)
        forms[f"graph{per}x{K // per}"] = (lambda g=g, r=K // per: [g.replay() for _ in range(r)])
    forms["eager_python"] = lambda: [step(0) for _ in range(K)]
    import ctypes
    L = bench.pcm_hip.load_library()
    P = bench.pcm_hip._ptr
    L.pcm_tune_chamfer_loss_grad_repeat.restype = ctypes.c_int
    args = (P(step.xyz1), P(step.xyz2), bench.B, bench.N, bench.M, ctypes.c_float(step.w1), ctypes.c_float(step.w2),
            P(step.d1), P(step.d2), P(step.i1), P(step.i2), P(step.loss[0]), P(step.gx1), P(step.gx2), P(step.ws),
            ctypes.c_size_t(step.ws.numel()), bench.pcm_hip._stream(dev))
    forms["eager_c_loop"] = lambda: L.pcm_tune_chamfer_loss_grad_repeat(K, *args)
    for name, fn in forms.items():
        fn()
        w_med, w_min = wall(fn, dev)
        ev = events(fn, dev)
        print(f"{name:14s} wall median {w_med:8.1f} us (min {w_min:8.1f}) = {w_med / K:6.2f} us/step; "
              f"events {ev:8.1f} us = {ev / K:6.2f} us/step; wall - events {w_med - ev:6.1f} us", flush=True)
    e_med, e_min = wall(lambda: None, dev)
    print(f"empty region   wall median {e_med:8.1f} us (min {e_min:8.1f})", flush=True)
    k_us = bench.kernel_avg_us(lambda: step(0), 200, dev)
    print(f"kernel_avg_us (200-launch graph, events): {k_us:.2f} us", flush=True)


if __name__ == "__main__":
    main()
