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


# Hidden LDS round trips on the kernels' critical paths (round 4: the one-launch
# Chamfer step 13.6-13.8 -> 12.7-12.9 us once they were removed).  HIP's
# __syncthreads_or re-reads the workgroup size from the dispatch packet and
# takes three barriers (pcm_wg_or takes one); __shfl_xor reductions lower to six
# dependent ds_bpermute round trips (PCM_DPP_WAVE_STEPS / pcm_wave_lexmin do
# not).  Allowed: the rare near-tie / MFMA-variant / fallback paths listed.
_SHFL_ALLOWED = {
    # non-resident near-tie pass (3 coordinate broadcasts); the 16-byte granule
    # store's gather (4 independent ds_bpermute behind one wait, no chain)
    "chamfer_filt.hip": 7,
}
_XOR_ALLOWED = {
    # non-resident near-tie pass (2 lines), the MFMA variant's lane merge (2)
    # and its near-tie pass (1): none on the default variant's path
    "chamfer_filt.hip": 5,
}


def _code_lines(path):
    out = []
    for ln in open(path):
        code = ln.split("//", 1)[0]
        if code.strip():
            out.append(code)
    return out


@pytest.mark.parametrize("src", ["chamfer_filt.hip", "chamfer.hip", "chamfer_grid.hip", "emd.hip", "icp.hip"])
def test_no_generic_workgroup_votes(src):
    lines = _code_lines(os.path.join(CSRC, src))
    assert not [ln for ln in lines if "__syncthreads_or" in ln or "__syncthreads_and" in ln or
                "__syncthreads_count" in ln], "use pcm_wg_or (pcm_common.h): one barrier"


def test_no_shuffle_reductions_on_hot_paths():
    for src in ("chamfer_filt.hip", "chamfer.hip", "chamfer_grid.hip", "emd.hip", "icp.hip", "chamfer_loss.h"):
        lines = _code_lines(os.path.join(CSRC, src))
        xor = [ln for ln in lines if "__shfl_xor" in ln]
        shfl = [ln for ln in lines if "__shfl" in ln and "__shfl_xor" not in ln]
        assert len(xor) <= _XOR_ALLOWED.get(src, 0), (src, xor)
        assert len(shfl) <= _SHFL_ALLOWED.get(src, 0), (src, shfl)
