"""Build checks that need no GPU: the profiling-only code paths keep compiling.

`make stamps` builds every source with -DPCM_STAMPS (tools/stamp_filt.py and
the EMD phase tools load that library); a stamp naming a variable that a later
change removed breaks only that build.  Device-side syntax
check of the sources that carry stamps, with the library's own flags.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "3d-pointcloudreconstruction_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src", ["chamfer_filt.hip", "emd.hip"])
def test_stamps_build_compiles(src):
    cmd = [HIPCC, "-O1", "--offload-arch=gfx950", "-ffp-contract=off", "-std=c++17", "-fsyntax-only",
           "--cuda-device-only", "-DPCM_STAMPS", "-I" + os.path.join(REPO, "include"), "-I" + CSRC,
           os.path.join(CSRC, src)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
