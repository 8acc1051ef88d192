#!/usr/bin/env python3
"""Phase breakdown of the filtered Chamfer forward from in-kernel stamps.

Needs the profiling build (make -C 3d-pointcloudreconstruction_amd/csrc stamps),
loaded through PCM_HIP_LIB.  Thread 0 of every workgroup records
s_memrealtime (100 MHz) at: 0 start, 1 centre barrier, 2 first tile staged,
3 scan done, 4 merge/proof done, 5 rescan done, 6 near-tie scans done,
7 end.

    python tools/stamp_filt.py VARIANT [VARIANT ...]
    python tools/stamp_filt.py fused [VARIANT ...]     (pcm_chamfer_loss_grad)
"""
import ctypes
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PCM_HIP_LIB"] = os.environ.get(
    "PCM_STAMPS_LIB", os.path.join(REPO, "3d-pointcloudreconstruction_amd", "lib", "libpcm_hip_stamps.so"))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import torch  # noqa: E402
import pcm_hip  # noqa: E402

NBASE = 10                                  # csrc/chamfer.hip kNumBaseFwdVariants
FILT_QPT = [2, 4, 4, 4, 4, 2, 4, 8]         # csrc/chamfer_filt.hip kPcmFiltVariants
TICK_US = 0.01                              # s_memrealtime: 100 MHz


def run(v, b, n, m, dev):
    g = torch.Generator().manual_seed(0)
    x1 = torch.rand(b, n, 3, generator=g).to(dev)
    x2 = torch.rand(b, m, 3, generator=g).to(dev)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, m, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, m, dtype=torch.int32, device=dev)
    for _ in range(5):
        pcm_hip.tune_chamfer_forward(v, x1, x2, d1, d2, i1, i2)
    torch.cuda.synchronize()
    qw = 64 * FILT_QPT[v - NBASE]
    nblk = b * ((n + qw - 1) // qw + (m + qw - 1) // qw)
    L = pcm_hip.load_library()
    L.pcm_tune_read_stamps.restype = ctypes.c_int
    L.pcm_tune_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (nblk * 8))()
    got = L.pcm_tune_read_stamps(buf, nblk)
    rows = [[buf[i * 8 + k] for k in range(8)] for i in range(got)]
    t0 = min(r[0] for r in rows)
    ends = [r[7] for r in rows]
    names = ["centre", "stage", "scan", "proof", "rescan", "ties"]
    print(f"variant {v} B={b} N={n} M={m}: {got} workgroups, kernel span "
          f"{(max(ends) - t0) * TICK_US:.2f} us, start spread {(max(r[0] for r in rows) - t0) * TICK_US:.2f} us")
    for k, nm in enumerate(names):
        dur = [(r[k + 1] - r[k]) * TICK_US for r in rows]
        print(f"  {nm:7s} median {statistics.median(dur):7.2f} us  mean {statistics.mean(dur):7.2f}  "
              f"max {max(dur):7.2f}")
    tail = [(e - r[6]) * TICK_US for e, r in zip(ends, rows)]
    tot = [(e - r[0]) * TICK_US for e, r in zip(ends, rows)]
    print(f"  tail    median {statistics.median(tail):7.2f} us;  per-WG total median "
          f"{statistics.median(tot):7.2f} max {max(tot):7.2f}")


def run_fused(v, b, n, m, dev):
    """pcm_chamfer_loss_grad variant v: stamps in the table's upper half
    (0 start, 1 forward done, 2 every workgroup of the batch element arrived,
    3 argmins loaded, 4 buckets filled, 7 this range's gradients stored)."""
    g = torch.Generator().manual_seed(0)
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
    warm = int(os.environ.get("STAMP_WARM", "0"))
    if warm:
        # STAMP_WARM=K: K replays of a 200-launch graph (~3 ms each) right
        # before the stamped launch, so it runs on a GPU that has been busy
        # (tools/clock_state.py); default: a GPU idle but for the 5 launches
        from tune_chamfer import graph_of
        gr = graph_of(lambda: pcm_hip.chamfer_loss_grad(x1, x2, 1.0 / (b * n), 1.0 / (b * m), d1, d2, i1, i2, mo,
                                                        g1, g2, variant=v), 200)
        torch.cuda.synchronize()
        time.sleep(0.5)
        for _ in range(warm):
            gr.replay()
        pcm_hip.chamfer_loss_grad(x1, x2, 1.0 / (b * n), 1.0 / (b * m), d1, d2, i1, i2, mo, g1, g2, variant=v)
        torch.cuda.synchronize()
        print(f"(stamped launch after {warm} back-to-back 200-launch graphs)")
    qw = 64 * FUSED_QPT[v]
    nblk = b * ((n + qw - 1) // qw + (m + qw - 1) // qw) + 1  # + the polling workgroup
    L = pcm_hip.load_library()
    L.pcm_tune_read_stamps.restype = ctypes.c_int
    L.pcm_tune_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    half = 1 << 15
    buf = (ctypes.c_ulonglong * ((half + nblk) * 8))()
    L.pcm_tune_read_stamps(buf, half + nblk)
    rows = [[buf[(half + i) * 8 + k] for k in range(8)] for i in range(nblk)]
    poll = rows.pop()
    t0 = min(r[0] for r in rows)
    end = max(r[7] for r in rows)
    print(f"fused variant {v} B={b} N={n} M={m}: {nblk} workgroups, span {(end - t0) * TICK_US:.2f} us, "
          f"forwards done by {(max(r[1] for r in rows) - t0) * TICK_US:.2f} us")
    for nm, k0, k1 in [("forward", 0, 1), ("wait", 1, 2), ("loads", 2, 3), ("buckets", 3, 4), ("grads", 4, 7)]:
        dur = [(r[k1] - r[k0]) * TICK_US for r in rows]
        print(f"  {nm:7s} median {statistics.median(dur):7.2f} us  max {max(dur):7.2f}")
    print(f"  starts: {(max(r[0] for r in rows) - t0) * TICK_US:.2f} us spread; waits end "
          f"{(min(r[2] for r in rows) - t0) * TICK_US:.2f} .. {(max(r[2] for r in rows) - t0) * TICK_US:.2f} us")
    print(f"  poller: starts {(poll[5] - t0) * TICK_US:.2f} us, done {(poll[6] - t0) * TICK_US:.2f} us")
    # per batch element: its last forward -> its waits' end (arrival
    # propagation), using the kernel's workgroup -> (batch element) mapping
    g = nblk - 1
    per_el = (n + qw - 1) // qw + (m + qw - 1) // qw
    pr, rem = g // 8, g % 8
    el = {}
    for i, r in enumerate(rows):
        x, s_ = i % 8, i // 8
        bid = (x * (pr + 1) if x < rem else rem * (pr + 1) + (x - rem) * pr) + s_
        el.setdefault(bid // per_el, []).append(r)
    lags = sorted(((max(r[2] for r in rs) - max(r[1] for r in rs)) * TICK_US, k) for k, rs in el.items())
    spread = [((max(r[2] for r in rs) - min(r[2] for r in rs)) * TICK_US) for rs in el.values()]
    print(f"  per element: last forward -> last wait end median {statistics.median([l for l, _ in lags]):.2f} us, "
          f"max {lags[-1][0]:.2f} us (element {lags[-1][1]}); wait-end spread inside an element median "
          f"{statistics.median(spread):.2f} max {max(spread):.2f} us")
    # the forward's own stamps (table's lower half, same workgroup numbering)
    lo = [[buf[i * 8 + k] for k in range(8)] for i in range(nblk - 1)]
    if v == 6:  # the matrix-core forward stores its near-tie census in slot 0
        nl = [r[0] & 0xffff for r in lo]
        full = sum((r[0] >> 16) & 0xffffff for r in lo)
        single = sum(r[0] >> 40 for r in lo)
        print(f"  near-ties per workgroup: median {statistics.median(nl)} max {max(nl)} total {sum(nl)} "
              f"({100.0 * sum(nl) / (64 * FUSED_QPT[v] * len(lo)):.2f}% of queries); whole quarters {full}, "
              f"single chunks {single}")
        cyc = [[buf[(8192 + i) * 8 + k] for k in range(8)] for i in range(nblk - 1)]
        ghz = [(c[6] - c[1]) / ((r[6] - r[1]) * 10.0) for c, r in zip(cyc, lo) if r[6] > r[1]]
        print(f"  shader clock over stamps 1..6: median {statistics.median(ghz):.2f} GHz, "
              f"min {min(ghz):.2f}, max {max(ghz):.2f}")
        for r in lo:
            r[0] = r[1]
    else:
        # the fused kernel's forward writes no stamp 0 of its own: its
        # centre phase starts at the workgroup's entry (upper-half stamp 0)
        for r, u in zip(lo, rows):
            r[0] = u[0]
    for nm, k0, k1 in [("centre", 0, 1), ("stage", 1, 2), ("scan", 2, 3), ("proof", 3, 4), ("rescan", 4, 5),
                       ("ties", 5, 6)]:
        dur = [(r[k1] - r[k0]) * TICK_US for r in lo]
        srt = sorted(dur)
        print(f"  fwd {nm:7s} median {statistics.median(dur):7.2f} us  p90 {srt[int(0.9 * len(srt))]:7.2f}  "
              f"max {max(dur):7.2f}  (>1 us: {sum(d > 1.0 for d in dur)} workgroups)")


FUSED_QPT = [2, 4, 2, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4]          # csrc/chamfer_filt.hip kGradVariants


def main():
    dev = torch.device("cuda:0")
    if sys.argv[1:2] == ["fused"]:
        for v in [int(a) for a in sys.argv[2:]] or [0]:
            run_fused(v, 32, 1024, 1024, dev)
        return
    vs = [int(a) for a in sys.argv[1:]] or [NBASE, NBASE + 1]
    for v in vs:
        run(v, 32, 1024, 1024, dev)
    for v in vs:
        run(v, 8, 16384, 16384, dev)


if __name__ == "__main__":
    main()
