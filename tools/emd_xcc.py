#!/usr/bin/env python3
"""Profiling build only (libpcm_hip_stamps.so): on which XCD the seed kernel's
first workgroup of each batch element ran, against the XCD of that element's
auction master -- the seed writes the element's caches into its XCD's L2, so
a mismatch turns every cache read of the auction into a cross-XCD miss."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PCM_HIP_LIB"] = os.path.join(REPO, "3d-pointcloudreconstruction_amd", "lib", "libpcm_hip_stamps.so")
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import torch  # noqa: E402
import pcm_hip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, n = 16, 1024
    g = torch.Generator().manual_seed(3)
    x1 = torch.rand(b, n, 3, generator=g).to(dev)
    x2 = torch.rand(b, n, 3, generator=g).to(dev)
    d = torch.empty(b, n, device=dev)
    a = torch.empty(b, n, dtype=torch.int32, device=dev)
    L = pcm_hip.load_library()
    L.pcm_tune_emd_xcc.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_int * 1024)()
    for rep in range(6):
        pcm_hip.emd_forward(x1, x2, 0.005, 50, d, a)
        torch.cuda.synchronize()
        L.pcm_tune_emd_xcc(buf)
        seed = [buf[i] for i in range(b)]
        mast = [buf[512 + i] for i in range(b)]
        same = sum(s == m for s, m in zip(seed, mast))
        print(f"run {rep}: seed xcc {seed}\n       master xcc {mast}  same XCD: {same}/{b}", flush=True)


if __name__ == "__main__":
    main()
