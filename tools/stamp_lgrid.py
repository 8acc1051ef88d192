#!/usr/bin/env python3
"""Phase stamps of the one-launch Chamfer step's LDS-grid variant (13,
csrc/chamfer_lgrid.h) at BASELINE config 2 on the bench's clouds.  Needs the
profiling build (make -C 3d-pointcloudreconstruction_amd/csrc stamps).
Upper-half stamps per workgroup: 0 start, 1 loads + box, 2 sorts done,
3 screen done, 4 proofs / rescans done, 5 listed queries done, 6 argmin
granules in, 7 end; lower half: 0 listed queries, 2..5 window size per group.

    python tools/stamp_lgrid.py [VARIANT]
"""
import ctypes
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PCM_HIP_LIB"] = os.environ.get(
    "PCM_STAMPS_LIB", os.path.join(REPO, "3d-pointcloudreconstruction_amd", "lib", "libpcm_hip_stamps.so"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import torch  # noqa: E402
import pcm_hip  # noqa: E402

TICK_US = 0.01


def main():
    v = int(sys.argv[1]) if len(sys.argv) > 1 else 13
    dev = torch.device("cuda:0")
    b, n, m = 32, 1024, 1024
    g = torch.Generator(device="cpu").manual_seed(1234)
    x1 = torch.rand(b, n, 3, generator=g).to(dev)
    x2 = torch.rand(b, m, 3, generator=g).to(dev)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, m, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, m, dtype=torch.int32, device=dev)
    g1, g2 = torch.empty(b, n, 3, device=dev), torch.empty(b, m, 3, device=dev)
    mo = torch.empty(3, device=dev)
    for _ in range(5):
        pcm_hip.chamfer_loss_grad(x1, x2, 1.0 / (b * n), 1.0 / (b * m), d1, d2, i1, i2, mo, g1, g2, variant=v)
    torch.cuda.synchronize()
    nblk = b * 8 + 1
    L = pcm_hip.load_library()
    L.pcm_tune_read_stamps.restype = ctypes.c_int
    L.pcm_tune_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    half = 1 << 15
    buf = (ctypes.c_ulonglong * ((half + nblk) * 8))()
    L.pcm_tune_read_stamps(buf, half + nblk)
    rows = [[buf[(half + i) * 8 + k] for k in range(8)] for i in range(nblk)]
    lo = [[buf[i * 8 + k] for k in range(8)] for i in range(nblk)]
    poll = rows.pop()
    lo.pop()
    t0 = min(r[0] for r in rows)
    end = max(r[7] for r in rows)
    print(f"variant {v}: {nblk} workgroups, span {(end - t0) * TICK_US:.2f} us, starts spread "
          f"{(max(r[0] for r in rows) - t0) * TICK_US:.2f} us; poller starts {(poll[5] - t0) * TICK_US:.2f}, "
          f"done {(poll[6] - t0) * TICK_US:.2f} us")
    names = ["loads+box", "sorts", "screen", "proof", "listed", "sweep", "grads"]
    for k, nm in enumerate(names):
        dur = sorted((r[k + 1] - r[k]) * TICK_US for r in rows)
        print(f"  {nm:9s} median {statistics.median(dur):6.2f} us  p90 {dur[int(0.9 * len(dur))]:6.2f}  "
              f"max {dur[-1]:6.2f}")
    for k in range(1, 8):
        at = sorted((r[k] - t0) * TICK_US for r in rows)
        print(f"  stamp {k} reached: median {statistics.median(at):6.2f}  max {at[-1]:6.2f} us")
    if v == 13:
        buf2 = (ctypes.c_ulonglong * ((3 * 4096) * 8))()
        L.pcm_tune_read_stamps(buf2, 3 * 4096)
        f1 = [[buf2[(4096 + i) * 8 + k] for k in range(8)] for i in range(nblk - 1)]
        f2 = [[buf2[(8192 + i) * 8 + k] for k in range(8)] for i in range(nblk - 1)]
        seq = [("atomics", None, (1, 0)), ("B2", (1, 0), (1, 1)), ("scan+B3", (1, 1), (1, 2)),
               ("starts+B4", (1, 2), (1, 3)), ("scatter", (1, 3), (1, 4)), ("B5", (1, 4), (1, 5)),
               ("ranks", (1, 5), (1, 6)), ("B6", (1, 6), None), ("gather0", None, (1, 7)),
               ("scan", (1, 7), None), ("B7", None, (2, 0)), ("merge", (2, 0), (2, 1)), ("rescan", (2, 1), (2, 2)),
               ("region+out", (2, 2), (2, 3)), ("B8", (2, 3), None)]
        up = {1: rows}
        tabs = {1: f1, 2: f2}

        def at(i, key, default_up):
            if key is None:
                return up[1][i][default_up]
            return tabs[key[0]][i][key[1]]
        defaults = {"atomics": (1, None), "B6": (None, 2), "gather0": (2, None), "scan": (None, 3), "B7": (3, None),
                    "B8": (None, 4)}
        for nm, k0, k1 in seq:
            d0, d1 = defaults.get(nm, (None, None))
            dur = sorted((at(i, k1, d1) - at(i, k0, d0)) * TICK_US for i in range(nblk - 1))
            print(f"    {nm:10s} median {statistics.median(dur):6.2f} us  p90 {dur[int(0.9 * len(dur))]:6.2f}  "
                  f"max {dur[-1]:6.2f}")
        nl = [r[0] for r in lo]
        wins = [r[k] for r in lo for k in range(2, 6)]
        print(f"  listed queries per workgroup: mean {statistics.mean(nl):.2f} max {max(nl)} total {sum(nl)}; "
              f"window per group: mean {statistics.mean(wins):.0f} median {statistics.median(wins)} "
              f"max {max(wins)}")


if __name__ == "__main__":
    main()
