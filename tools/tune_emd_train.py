#!/usr/bin/env python3
"""EMD diagnostics at the TRAINING call (loss/loss.py:23: eps=0.05, iters=3000)
on the clouds a seeded random-init generator predicts (train/fenet.py), and at
the other documented call settings: iterations that ran, bids / full scans,
offloaded jobs, per-phase wall time of batch 0, device time per forward for a
sweep of helper counts / offload thresholds."""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "train"))
import pcm_hip  # noqa: E402

DIAG_WSPLIT = False
TIMERS = ["bids", "full-scans", "claim", "assign", "scan/publish", "exchange/own-items", "keys|merge",
          "proof|finish", "chain-entry", "chain-scan", "chain-resolve", "exact"]


def timed(x1, x2, eps, iters, d, a, helpers, offload, wsplit=None, reps=5, tail_max=None):
    kw = {} if helpers is None else {"helpers": helpers, "offload_min": offload}
    if wsplit is not None:
        kw["wsplit"] = wsplit
    if tail_max is not None:
        kw["tail_max"] = tail_max
    pcm_hip.emd_forward(x1, x2, eps, iters, d, a, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pcm_hip.emd_forward(x1, x2, eps, iters, d, a, **kw)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def run(name, x1, x2, eps, iters, sweep):
    b, n, _ = x1.shape
    dev = x1.device
    d = torch.empty(b, n, device=dev)
    a = torch.empty(b, n, dtype=torch.int32, device=dev)
    st = torch.zeros(3 * iters + 16 + b, dtype=torch.int32, device=dev)
    pcm_hip.emd_forward(x1, x2, eps, iters, d, a, stats=st)
    torch.cuda.synchronize()
    st = st.cpu()
    misc = st[2 * iters:2 * iters + 16].tolist()
    wall = st[3 * iters + 16:3 * iters + 16 + b].tolist()
    per = st[:2 * iters].view(iters, 2)
    active = int((per[:, 0] > 0).sum())
    print(f"[{name}] B={b} N={n} eps={eps} iters={iters}: iterations with bidders {active}; "
          f"bids {int(per[:, 0].sum())}, full scans {int(per[:, 1].sum())}; offloaded jobs {misc[10]}, "
          f"items {misc[11]}, helper wake-ups {misc[12]}, exact fallbacks {misc[15]}")
    marks = [0, 1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, 2000, 5000, iters - 1]
    print("  unassigned (sum over batch) at iter:", " ".join(f"{i}:{int(per[i, 0])}" for i in marks if i < iters))
    print("  full scans (sum over batch) at iter:", " ".join(f"{i}:{int(per[i, 1])}" for i in marks if i < iters))
    print("  auction wall per batch element (us): min %.1f max %.1f" % (min(wall) / 100.0, max(wall) / 100.0))
    st.zero_()
    slow = max(range(b), key=lambda i: wall[i])
    for ws in ((None, 4) if DIAG_WSPLIT else (None,)):
        st = torch.zeros(3 * iters + 16 + b, dtype=torch.int32, device=dev)
        kw = {} if ws is None else {"wsplit": ws}
        pcm_hip.emd_forward(x1, x2, eps, iters, d, a, stats=st, diag=2 + slow, **kw)
        torch.cuda.synchronize()
        tm = st.cpu()[2 * iters:2 * iters + 15].tolist()
        act = max(tm[12], 1)
        print(f"  slowest batch element {slow}{'' if ws is None else f' (wsplit={ws})'}: {act} iterations "
              f"({tm[13]} tail mode, {tm[14]} chain mode); phase cycles per iteration: "
              + ", ".join(f"{nm}={16.0 * v / act:.0f}" for nm, v in zip(TIMERS, tm[:12])))
        print("  phase cycles total (M): " + ", ".join(f"{nm}={16.0 * v / 1e6:.2f}" for nm, v in zip(TIMERS, tm[:12])))
    print(f"  forward (defaults): {timed(x1, x2, eps, iters, d, a, None, None):.1f} us/call")
    for h, o in sweep:
        print(f"  forward helpers={h} offload_min={o}: {timed(x1, x2, eps, iters, d, a, h, o):.1f} us/call")
    for t in (0, 8, 32, 64, 128):
        print(f"  forward tail_max={t}: {timed(x1, x2, eps, iters, d, a, -1, -1, tail_max=t):.1f} us/call")
    for w in (2, 4):
        print(f"  forward wsplit={w}: {timed(x1, x2, eps, iters, d, a, -1, -1, w):.1f} us/call")


def generator_clouds(b, dev):
    import fenet
    import train_step as T
    # forward on the CPU: the same clouds in every process and on every box
    # (MIOpen's convolutions are not bitwise reproducible across processes)
    gen = fenet.seeded_init(fenet.Generator(1024), 0).train()
    images, points = T.synthetic_batch(b, 1024, torch.device("cpu"), seed=0)
    with torch.no_grad():
        pred = gen(images)[2].transpose(2, 1).contiguous()
    return pred.to(dev), points.to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--quick", action="store_true", help="training call + config 3 only")
    ap.add_argument("--diag-wsplit", action="store_true", help="phase timers with wsplit=4 as well")
    args = ap.parse_args()
    global DIAG_WSPLIT
    DIAG_WSPLIT = args.diag_wsplit
    dev = torch.device("cuda:0")
    sweep = [(0, 0), (15, 8), (15, 16), (15, 24), (15, 48), (7, 24)]
    pred, points = generator_clouds(args.b, dev)
    run("generator prediction vs uniform GT", pred, points, 0.05, 3000, sweep)
    g = torch.Generator().manual_seed(3)
    u1 = torch.rand(args.b, 1024, 3, generator=g).to(dev)
    u2 = torch.rand(args.b, 1024, 3, generator=g).to(dev)
    run("uniform vs uniform, config 3", u1, u2, 0.005, 50, sweep)
    if args.quick:
        return
    run("uniform vs uniform, training call", u1, u2, 0.05, 3000, sweep[:2])
    run("uniform vs uniform, README test-time setting", u1, u2, 0.002, 10000, sweep[:2])
    g = torch.Generator().manual_seed(4)
    w1 = torch.rand(20, 2048, 3, generator=g).to(dev)
    w2 = torch.rand(20, 2048, 3, generator=g).to(dev)
    run("metric/emd/test.py: B=20 N=2048", w1, w2, 0.05, 3000, sweep[:2])
    g = torch.Generator().manual_seed(5)
    v1 = torch.rand(2, 8192, 3, generator=g).to(dev)
    v2 = torch.rand(2, 8192, 3, generator=g).to(dev)
    run("large cloud B=2 N=8192", v1, v2, 0.005, 50, sweep[:2])
    v1 = torch.rand(2, 16384, 3, generator=g).to(dev)
    v2 = torch.rand(2, 16384, 3, generator=g).to(dev)
    run("large cloud B=2 N=16384", v1, v2, 0.005, 50, sweep[:2])


if __name__ == "__main__":
    main()
