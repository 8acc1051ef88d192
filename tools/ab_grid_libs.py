#!/usr/bin/env python3
"""Config-5 grid forward (B=8, N=M=16384, fp16 and fp32) for the library in
PCM_HIP_LIB: median of 5 replays of a 20-call graph, per call, and a hash of
the outputs (equal hashes across libraries = identical results).  Run once per
library, alternating, in one GPU session (tools/gpu_run.sh abgl)."""
import hashlib
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import pcm_hip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, n = 8, 16384
    g = torch.Generator().manual_seed(5)
    x = torch.rand(b, n, 3, generator=g).to(dev)
    y = torch.rand(b, n, 3, generator=g).to(dev)
    d1, d2 = torch.empty(b, n, device=dev), torch.empty(b, n, device=dev)
    i1 = torch.empty(b, n, dtype=torch.int32, device=dev)
    i2 = torch.empty(b, n, dtype=torch.int32, device=dev)
    out = []
    for name, (a, c) in (("fp16", (x.half(), y.half())), ("fp32", (x, y))):
        fn = lambda: pcm_hip.chamfer_forward(a, c, d1, d2, i1, i2)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        h = hashlib.sha1(b"".join(t.cpu().numpy().tobytes() for t in (d1, d2, i1, i2))).hexdigest()[:12]
        s = torch.cuda.current_stream()
        cs = torch.cuda.Stream()
        cs.wait_stream(s)
        with torch.cuda.stream(cs):
            fn()
        s.wait_stream(cs)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(20):
                fn()
        gr.replay()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            gr.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0 / 20)
        out.append(f"{name} {statistics.median(ts):.1f} us (hash {h})")
    print(os.path.basename(os.environ.get("PCM_HIP_LIB", "libpcm_hip.so")) + ": " + ", ".join(out), flush=True)


if __name__ == "__main__":
    main()
