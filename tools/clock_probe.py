#!/usr/bin/env python3
"""Core clock under load (profiling build): s_memtime ticks per s_memrealtime
(100 MHz) tick over a ~dependent-FMA spin, one workgroup per CU and 4 per CU."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PCM_HIP_LIB"] = os.path.join(REPO, "3d-pointcloudreconstruction_amd", "lib", "libpcm_hip_stamps.so")
sys.path.insert(0, os.path.join(REPO, "3d-pointcloudreconstruction_amd", "metric"))
import torch  # noqa: E402
import pcm_hip  # noqa: E402


def main():
    L = pcm_hip.load_library()
    L.pcm_tune_clock.restype = ctypes.c_int
    L.pcm_tune_clock.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    for blocks, iters in [(256, 2000), (256, 20000), (1024, 20000), (1024, 200000)]:
        out = torch.zeros(blocks * 4, dtype=torch.int64, device="cuda")
        for _ in range(3):
            L.pcm_tune_clock(out.data_ptr(), blocks, iters, None)
        torch.cuda.synchronize()
        o = out.view(blocks, 4).cpu()
        mhz = (o[:, 0].double() / o[:, 1].double() * 100.0)
        print(f"blocks={blocks} iters={iters}: core clock {mhz.median().item():.0f} MHz "
              f"(min {mhz.min().item():.0f}, max {mhz.max().item():.0f}), spin {o[:, 1].double().median().item() / 100:.1f} us")


if __name__ == "__main__":
    main()
