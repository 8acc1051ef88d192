#!/usr/bin/env python3
"""Grid forward diagnostics at BASELINE config 5 (B=8, N=M=16384 fp16) and a
few other sizes: the build and search kernels timed apart (graph of 20 calls,
HIP events), and per search wave the rounds it ran and the candidates it
gathered (csrc/chamfer_grid.hip stats)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pcm_hip  # noqa: E402
from ab_grid import timed  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for (b, n, m, dt) in [(8, 16384, 16384, torch.float16), (2, 4096, 4096, torch.float32),
                          (4, 65536, 65536, torch.float32)]:
        g = torch.Generator().manual_seed(5)
        x1 = torch.rand(b, n, 3, generator=g).to(dt).to(dev)
        x2 = torch.rand(b, m, 3, generator=g).to(dt).to(dev)
        d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, m, device=dev)
        i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
        i2 = torch.empty(b, m, dtype=torch.int32, device=dev)
        ws = pcm_hip.forward_workspace(dev, b, n, m, force_grid=True)
        waves = b * ((n + 63) // 64 + (m + 63) // 64)
        st_all = torch.zeros(waves * 4 + waves * 8, dtype=torch.int32, device=dev)
        pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, stats=st_all, workspace=ws)
        torch.cuda.synchronize()
        st = st_all[: waves * 4].view(waves, 4)
        ss = st_all[waves * 4:].view(waves, 8).cpu().long() & 0xffffffff
        t_all = timed(lambda: pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, workspace=ws))
        t_b = timed(lambda: pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="build", workspace=ws))
        t_s = timed(lambda: pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="search", workspace=ws))
        t_sr = timed(lambda: pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="search", workspace=ws,
                                                               reg_gather=True))
        t_sf = timed(lambda: pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="search", workspace=ws,
                                                               scan="screened"))
        t_s4 = timed(lambda: pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="search", workspace=ws,
                                                               small_wg=True))
        s = st.cpu()
        r, c0, ca = s[:, 0].float(), s[:, 1].float(), s[:, 2].float()
        q = torch.tensor([0.5, 0.9, 0.99, 1.0])
        print(f"B={b} N={n} M={m} {str(dt)[6:]}: both {t_all:.1f} us, build {t_b:.1f} us, search {t_s:.1f} us (256-thread workgroups {t_s4:.1f}, register gather {t_sr:.1f}, screened scan {t_sf:.1f}); "
              f"{waves} waves", flush=True)
        print(f"  rounds: 1: {(r == 1).sum().item()}, 2: {(r == 2).sum().item()}, 3: {(r == 3).sum().item()}", flush=True)
        t0 = ss[:, 0].min()
        sd = (ss[:, 1:6] - ss[:, 0:5]).float() * 0.01
        names = ["prologue", "box+rows", "gather", "scan", "proof+out"]
        print("  search phases per wave (median / p90, us): " +
              ", ".join(f"{nm} {sd[:, i].median().item():.2f}/{torch.quantile(sd[:, i], 0.9).item():.2f}"
                        for i, nm in enumerate(names)) +
              f"; wave total {((ss[:, 5] - ss[:, 0]).float() * 0.01).median().item():.2f}; starts spread "
              f"{((ss[:, 0] - t0).float() * 0.01).max().item():.2f}, last end {((ss[:, 5] - t0).float() * 0.01).max().item():.2f}",
              flush=True)
        st0 = ((ss[:, 0] - t0).float() * 0.01)
        print("  wave start offsets p10/p50/p90/max (us): " +
              "/".join(f"{torch.quantile(st0, qq).item():.2f}" for qq in (0.1, 0.5, 0.9, 1.0)), flush=True)
        hw, xcc = ss[:, 6], ss[:, 7] & 0xf
        cu = (hw >> 8) & 0xf
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        unit = ((xcc * 8 + se) * 2 + sh) * 16 + cu
        ucnt = torch.bincount(unit, minlength=int(unit.max().item()) + 1)
        print(f"  placement: {int((ucnt > 0).sum().item())} distinct (xcc, se, sh, cu) units, waves per unit "
              f"min {int(ucnt[ucnt > 0].min().item())} max {int(ucnt.max().item())}; xcc counts "
              f"{torch.bincount(xcc, minlength=8).tolist()}", flush=True)
        # where the late starts are: by XCD, and by the wave's slot inside its
        # workgroup (stamps are indexed by workgroup * waves + slot)
        full = 16 * 256  # launch_grid's rule (csrc/chamfer_grid.hip): 16-wave workgroups iff 3/4 full <= waves <= full
        kw = 16 if full * 3 // 4 <= len(st0) <= full else 4
        slot = torch.arange(len(st0), device=st0.device) % kw
        print("  start median/max by xcc (us): " + " ".join(
            f"{torch.quantile(st0[xcc == x], 0.5).item():.2f}/{st0[xcc == x].max().item():.2f}"
            for x in range(8) if bool((xcc == x).any())), flush=True)
        print(f"  start median by wave slot (of {kw}): " + " ".join(
            f"{torch.quantile(st0[slot == j], 0.5).item():.2f}" for j in range(kw)), flush=True)
        # the search alone (after a synchronize): its XCDs' start skew without the build before it
        st_s = torch.zeros_like(st_all)
        torch.cuda.synchronize()
        pcm_hip.tune_chamfer_forward_grid(x1, x2, d1, d2, i1, i2, only="search", stats=st_s, workspace=ws)
        torch.cuda.synchronize()
        s2 = st_s[waves * 4:].view(waves, 8).cpu().long() & 0xffffffff
        a0 = (s2[:, 0] - s2[:, 0].min()).float() * 0.01
        x2c = s2[:, 7] & 0xf
        print("  search alone: start median/max by xcc (us): " + " ".join(
            f"{torch.quantile(a0[x2c == x], 0.5).item():.2f}/{a0[x2c == x].max().item():.2f}"
            for x in range(8) if bool((x2c == x).any())) +
            f"; last end {((s2[:, 5] - s2[:, 0].min()).float() * 0.01).max().item():.2f}", flush=True)
        print(f"  candidates round 0 p50/p90/p99/max {[round(v) for v in torch.quantile(c0, q).tolist()]}, "
              f"all rounds {[round(v) for v in torch.quantile(ca, q).tolist()]}, mean {ca.mean().item():.0f}",
              flush=True)


if __name__ == "__main__":
    main()
