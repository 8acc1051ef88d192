#!/usr/bin/env python3
"""EMD config-3 diagnostics for one build (PCM_HIP_LIB=...): counts (misses,
reserve bids, full scans), per-element auction wall times and the phase
timers of the slowest element, plus the forward time."""
import os
import sys

import numpy as np

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import tune_emd_train as T  # noqa: E402

pcm_hip = T.pcm_hip


def main():
    dev = torch.device("cuda:0")
    train = "--train" in sys.argv
    if train:
        x1, x2 = T.generator_clouds(16, dev)
        eps, iters = 0.05, 3000
    else:
        g = torch.Generator().manual_seed(3)
        x1 = torch.rand(16, 1024, 3, generator=g).to(dev)
        x2 = torch.rand(16, 1024, 3, generator=g).to(dev)
        eps, iters = 0.005, 50
    b, n = 16, 1024
    d = torch.empty(b, n, device=dev)
    a = torch.empty(b, n, dtype=torch.int32, device=dev)
    st = torch.zeros(3 * iters + 16 + b, dtype=torch.int32, device=dev)
    pcm_hip.emd_forward(x1, x2, eps, iters, d, a, stats=st)
    torch.cuda.synchronize()
    st = st.cpu()
    per = st[:2 * iters].view(iters, 2)
    misc = st[2 * iters:2 * iters + 16].tolist()
    wall = [w / 100.0 for w in st[3 * iters + 16:3 * iters + 16 + b].tolist()]
    lib = os.path.basename(os.environ.get("PCM_HIP_LIB", "libpcm_hip.so"))
    print(f"{lib}: bids {int(per[:, 0].sum())} misses {int(per[:, 1].sum())} reserve bids {misc[13]} "
          f"jobs {misc[10]}; wall us min {min(wall):.1f} med {sorted(wall)[b // 2]:.1f} max {max(wall):.1f}")
    if "--hist" in sys.argv:  # bids / misses per iteration, summed over the batch, in bins
        pr = per.numpy()
        last = int(np.nonzero(pr[:, 0])[0].max()) + 1 if pr[:, 0].any() else 0
        step = 25 if last > 200 else 1
        for i0 in range(0, last, step):
            seg = pr[i0:i0 + step]
            print(f"    it {i0:5d}-{min(i0 + step, last) - 1:5d}: bids {int(seg[:, 0].sum()):7d} misses {int(seg[:, 1].sum()):7d}")
    slow = max(range(b), key=lambda i: wall[i])
    st = torch.zeros(3 * iters + 16 + b, dtype=torch.int32, device=dev)
    pcm_hip.emd_forward(x1, x2, eps, iters, d, a, stats=st, diag=2 + slow)
    torch.cuda.synchronize()
    stc = st.cpu()
    tm = stc[2 * iters:2 * iters + 15].tolist()
    act = max(tm[12], 1)
    if "--per-iter" in sys.argv:  # cycles per iteration of the slowest element (x16 units)
        for it in range(iters):
            nu = int(stc[2 * iters + 16 + it])
            if nu == 0 and int(stc[2 * it]) == 0:
                continue
            print(f"    it {it:4d} bidders {nu:5d} cycles {16 * int(stc[2 * it]):7d} bids(B1) {16 * int(stc[2 * it + 1]):7d}")
    if "--by-nu" in sys.argv:  # the slowest element's iteration cycles by bidder count
        bins = [(1, 1), (2, 4), (5, 16), (17, 64), (65, 256), (257, 1 << 30)]
        acc = {bn: [0, 0] for bn in bins}
        for it in range(iters):
            nu = int(stc[2 * iters + 16 + it])
            cyc = 16 * int(stc[2 * it])
            for bn in bins:
                if bn[0] <= nu <= bn[1]:
                    acc[bn][0] += 1
                    acc[bn][1] += cyc
        tot = sum(v[1] for v in acc.values())
        for bn, (cnt, cyc) in acc.items():
            if cnt:
                print(f"    bidders {bn[0]:4d}-{min(bn[1], 99999):5d}: {cnt:5d} iterations, {cyc / 1e6:7.2f} M cycles "
                      f"({100.0 * cyc / max(tot, 1):4.1f} %), {cyc / cnt:8.0f} per iteration")
    print(f"  slowest element {slow}: {act} iterations; cycles/iteration "
          + ", ".join(f"{nm}={16.0 * v / act:.0f}" for nm, v in zip(T.TIMERS, tm[:12])))
    print(f"  forward {T.timed(x1, x2, eps, iters, d, a, None, None, reps=20):.1f} us", flush=True)


if __name__ == "__main__":
    main()
