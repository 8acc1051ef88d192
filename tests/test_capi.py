"""C-ABI checks that need no GPU: libpcm_hip.so loads, exports every function
include/pcm.h declares, and rejects bad arguments before touching the device."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "pcm.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pcm_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import pcm_hip
    return pcm_hip.load_library()


def test_header_declares_expected_api():
    import pcm_hip
    assert set(_declared()) == set(pcm_hip.EXPORTED)


def test_library_exports_every_declared_symbol(lib):
    for name in _declared():
        assert hasattr(lib, name), name


def test_version_and_strerror(lib):
    assert lib.pcm_version() >= 100
    for code in (0, -1, -2, -3, -4, 7):
        assert lib.pcm_strerror(code)


def test_invalid_arguments_rejected_without_device(lib):
    import pcm_hip
    L = lib
    null = None
    # negative sizes
    assert L.pcm_chamfer_forward(null, null, -1, 4, 4, null, null, null, null, null) == -1
    assert L.pcm_chamfer_backward(null, null, 2, -3, 4, null, null, null, null, null, null, null) == -1
    # null pointers with non-empty shapes
    assert L.pcm_chamfer_forward(null, null, 2, 4, 4, null, null, null, null, null) == -1
    # backward needs both clouds non-empty
    assert L.pcm_chamfer_backward(null, null, 2, 0, 4, null, null, null, null, null, null, null) == -1
    # EMD contract of emd_cuda.cu:236-249
    assert L.pcm_emd_forward(null, null, 2, 1000, 0.005, 50, null, null, null, null, 0, null) == -1
    assert L.pcm_emd_forward(null, null, 513, 1024, 0.005, 50, null, null, null, null, 0, null) == -1
    assert L.pcm_emd_forward(null, null, 2, 1024, 0.005, 0, null, null, null, null, 0, null) == -1
    # fp16 entry points validate the same way
    assert L.pcm_chamfer_forward_f16(null, null, -1, 4, 4, null, null, null, null, null) == -1
    assert L.pcm_chamfer_forward_f16(null, null, 2, 4, 4, null, null, null, null, null) == -1
    assert L.pcm_chamfer_backward_f16(null, null, 2, 0, 4, null, null, null, null, null, null, null) == -1
    assert L.pcm_chamfer_forward_f16(null, null, 0, 4, 4, null, null, null, null, null) == 0
    # empty problems are no-ops
    assert L.pcm_chamfer_forward(null, null, 0, 4, 4, null, null, null, null, null) == 0
    assert L.pcm_emd_forward(null, null, 0, 1024, 0.005, 50, null, null, null, null, 0, null) == 0
    assert pcm_hip.emd_workspace_bytes(16, 1024) >= 0


def test_layout_and_strided_entries_reject_bad_arguments(lib):
    # pcm_chamfer_forward_layout / _backward_layout / _backward_strided check
    # layouts, sizes, strides and pointers before any device call
    L = lib
    null = None
    # layouts are 0 (rows) or 1 (channel planes)
    assert L.pcm_chamfer_forward_layout(null, null, 2, 4, 4, 2, 0, null, null, null, null, null) == -1
    assert L.pcm_chamfer_forward_layout(null, null, 2, 4, 4, 0, -1, null, null, null, null, null) == -1
    assert L.pcm_chamfer_backward_layout(null, null, 2, 4, 4, 0, 3, null, null, null, null, null, null, null) == -1
    assert L.pcm_chamfer_backward_strided(null, null, 2, 4, 4, 5, 0, null, 4, 1, null, 4, 1, null, null, null, null,
                                          null) == -1
    # negative sizes, null pointers with non-empty shapes
    assert L.pcm_chamfer_forward_layout(null, null, -1, 4, 4, 1, 0, null, null, null, null, null) == -1
    assert L.pcm_chamfer_forward_layout(null, null, 2, 4, 4, 1, 0, null, null, null, null, null) == -1
    # graddist strides must be >= 0 and fit an int
    assert L.pcm_chamfer_backward_strided(null, null, 2, 4, 4, 0, 0, null, -1, 1, null, 4, 1, null, null, null, null,
                                          null) == -1
    assert L.pcm_chamfer_backward_strided(null, null, 2, 4, 4, 0, 0, null, 4, 1 << 31, null, 4, 1, null, null, null,
                                          null, null) == -1
    # the backward needs both clouds non-empty, and its pointers
    assert L.pcm_chamfer_backward_strided(null, null, 2, 0, 4, 0, 0, null, 0, 0, null, 0, 0, null, null, null, null,
                                          null) == -1
    assert L.pcm_chamfer_backward_strided(null, null, 2, 4, 4, 0, 0, null, 0, 0, null, 0, 0, null, null, null, null,
                                          null) == -1
    # empty problems are no-ops
    assert L.pcm_chamfer_forward_layout(null, null, 0, 4, 4, 1, 1, null, null, null, null, null) == 0
    assert L.pcm_chamfer_backward_strided(null, null, 0, 4, 4, 1, 0, null, 0, 0, null, 0, 0, null, null, null, null,
                                          null) == 0
