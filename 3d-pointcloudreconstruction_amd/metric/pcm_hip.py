"""ctypes binding of libpcm_hip.so (the gfx950 HIP kernels behind include/pcm.h).

This is the product path's only route to compute: there is no CPU fallback.
If the library is missing, or a tensor is not on a HIP device, every entry
point raises.  Kernels are enqueued on PyTorch's *current* stream of the
tensors' device (the reference launched on the legacy default stream,
chamfer3D.cu:142-143 -- SURVEY.md appendix A.5).
"""
from __future__ import annotations

import collections
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "PCM_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libpcm_hip.so"))
# the tuning build (make -C csrc tune): the product library plus the measured
# alternatives of the one-launch Chamfer step (fused variants 0-18 beside the default 7), which
# tools/ and the variant tests select by number; never on the product path
TUNE_LIB_PATH = os.environ.get(
    "PCM_HIP_TUNE_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libpcm_hip_tune.so"))

_lib = None
_tune_lib = None

# every symbol include/pcm.h declares (checked by tests/test_capi.py)
EXPORTED = (
    "pcm_version", "pcm_strerror",
    "pcm_chamfer_forward", "pcm_chamfer_backward",
    "pcm_chamfer_workspace_bytes", "pcm_chamfer_forward_loss", "pcm_chamfer_workspace_status",
    "pcm_emd_workspace_bytes", "pcm_emd_forward", "pcm_emd_backward", "pcm_emd_workspace_status",
    "pcm_chamfer_forward_f16", "pcm_chamfer_backward_f16",
    "pcm_chamfer_forward_ws_bytes", "pcm_chamfer_forward_ws", "pcm_chamfer_forward_ws_f16",
    "pcm_chamfer_loss_grad", "pcm_chamfer_forward_layout", "pcm_chamfer_backward_layout",
    "pcm_chamfer_backward_strided", "pcm_chamfer_loss_grad_layout", "pcm_chamfer_loss_grad_rescale",
    "pcm_chamfer_loss_grad_steps",
    "pcm_icp_workspace_bytes", "pcm_icp", "pcm_icp_workspace_status", "pcm_nearest_neighbor",
    "pcm_best_fit_transform",
    "pcm_npy_cloud_points", "pcm_npy_load_clouds",
)

# largest cloud pcm_icp takes (csrc/icp.hip kIcpMaxN: 16 slices of 1024 points)
ICP_MAX_POINTS = 16384

# largest cloud (points per batch element) pcm_chamfer_loss_grad runs as one
# launch (csrc/chamfer_filt.hip kGradCap); larger clouds take forward + backward
LOSS_GRAD_MAX_POINTS = 1024


class PcmError(RuntimeError):
    """A libpcm_hip call returned a non-zero pcm_status."""


def load_library():
    """Load libpcm_hip.so (raises OSError with the path if it is missing)."""
    global _lib
    if _lib is None:
        _lib = _open(LIB_PATH)
    return _lib


def load_tune_library():
    """Load libpcm_hip_tune.so, the tuning build (fused variants 0-18 beside
    the default); raises OSError if it is missing."""
    global _tune_lib
    if _tune_lib is None:
        _tune_lib = _open(TUNE_LIB_PATH)
    return _tune_lib


def _open(path):
    if not os.path.exists(path):
        raise OSError(
            f"{os.path.basename(path)} not found at {path}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C "
            "3d-pointcloudreconstruction_amd/csrc`")
    L = ctypes.CDLL(path)
    vp, ci, cf, cs = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    L.pcm_version.restype = ci
    L.pcm_version.argtypes = []
    L.pcm_strerror.restype = ctypes.c_char_p
    L.pcm_strerror.argtypes = [ci]
    L.pcm_chamfer_forward.restype = ci
    L.pcm_chamfer_forward.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp]
    L.pcm_chamfer_backward.restype = ci
    L.pcm_chamfer_backward.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp]
    L.pcm_chamfer_workspace_bytes.restype = cs
    L.pcm_chamfer_workspace_bytes.argtypes = [ci, ci, ci]
    L.pcm_chamfer_workspace_status.restype = ci
    L.pcm_chamfer_workspace_status.argtypes = [vp, cs, ci, ci, ci, vp]
    L.pcm_tune_chamfer_loss_grad_spins.restype = ci
    L.pcm_tune_chamfer_loss_grad_spins.argtypes = [ctypes.c_uint, ctypes.c_uint, vp, vp, ci, ci, ci, cf, cf, vp, vp,
                                                   vp, vp, vp, vp, vp, vp, cs, vp]
    L.pcm_tune_chamfer_slow_paths.restype = ci
    L.pcm_tune_chamfer_slow_paths.argtypes = [vp, cs, ci, ci, ci, vp]
    L.pcm_tune_chamfer_err_offset.restype = cs
    L.pcm_tune_chamfer_err_offset.argtypes = [ci, ci, ci, ci]
    L.pcm_chamfer_forward_loss.restype = ci
    L.pcm_chamfer_forward_loss.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, cs, vp]
    L.pcm_tune_num_chamfer_variants.restype = ci
    L.pcm_tune_num_chamfer_variants.argtypes = []
    L.pcm_tune_chamfer_forward.restype = ci
    L.pcm_tune_chamfer_forward.argtypes = [ci, vp, vp, ci, ci, ci, vp, vp, vp, vp, vp]
    L.pcm_tune_chamfer_backward.restype = ci
    L.pcm_tune_chamfer_backward.argtypes = [ci, vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp]
    L.pcm_tune_chamfer_forward_loss.restype = ci
    L.pcm_tune_chamfer_forward_loss.argtypes = [ci, ci, vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, cs, vp]
    if hasattr(L, "pcm_chamfer_forward_layout"):  # absent from A/B builds of older sources
        L.pcm_chamfer_forward_layout.restype = ci
        L.pcm_chamfer_forward_layout.argtypes = [vp, vp, ci, ci, ci, ci, ci, vp, vp, vp, vp, vp]
        L.pcm_chamfer_backward_layout.restype = ci
        L.pcm_chamfer_backward_layout.argtypes = [vp, vp, ci, ci, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp]
    if hasattr(L, "pcm_chamfer_backward_strided"):
        ll = ctypes.c_longlong
        L.pcm_chamfer_backward_strided.restype = ci
        L.pcm_chamfer_backward_strided.argtypes = [vp, vp, ci, ci, ci, ci, ci, vp, ll, ll, vp, ll, ll, vp, vp, vp,
                                                   vp, vp]
    L.pcm_chamfer_forward_f16.restype = ci
    L.pcm_chamfer_forward_f16.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp]
    L.pcm_chamfer_backward_f16.restype = ci
    L.pcm_chamfer_backward_f16.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp]
    if hasattr(L, "pcm_chamfer_forward_ws"):  # absent from A/B builds of older sources
        L.pcm_chamfer_forward_ws_bytes.restype = cs
        L.pcm_chamfer_forward_ws_bytes.argtypes = [ci, ci, ci]
        L.pcm_chamfer_forward_ws.restype = ci
        L.pcm_chamfer_forward_ws.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, cs, vp]
        L.pcm_chamfer_forward_ws_f16.restype = ci
        L.pcm_chamfer_forward_ws_f16.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, cs, vp]
        L.pcm_tune_chamfer_forward_grid_ws_bytes.restype = cs
        L.pcm_tune_chamfer_forward_grid_ws_bytes.argtypes = [ci, ci, ci]
        L.pcm_tune_chamfer_forward_grid.restype = ci
        L.pcm_tune_chamfer_forward_grid.argtypes = [ci, vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, cs, vp, vp]
        L.pcm_tune_chamfer_backward_f16.restype = ci
        L.pcm_tune_chamfer_backward_f16.argtypes = [ci, vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp]
    L.pcm_tune_num_chamfer_f16_variants.restype = ci
    L.pcm_tune_num_chamfer_f16_variants.argtypes = []
    L.pcm_tune_chamfer_forward_f16.restype = ci
    L.pcm_tune_chamfer_forward_f16.argtypes = [ci, vp, vp, ci, ci, ci, vp, vp, vp, vp, vp]
    L.pcm_emd_workspace_bytes.restype = cs
    L.pcm_emd_workspace_bytes.argtypes = [ci, ci]
    L.pcm_emd_forward.restype = ci
    L.pcm_emd_forward.argtypes = [vp, vp, ci, ci, cf, ci, vp, vp, vp, vp, cs, vp]
    L.pcm_emd_backward.restype = ci
    L.pcm_emd_backward.argtypes = [vp, vp, ci, ci, vp, vp, vp, vp]
    L.pcm_emd_workspace_status.restype = ci
    L.pcm_emd_workspace_status.argtypes = [vp, cs, ci, ci, vp]
    L.pcm_tune_emd_forward_cfg.restype = ci
    L.pcm_tune_emd_forward_cfg.argtypes = [vp, vp, ci, ci, cf, ci, vp, vp, vp, vp, cs, ci, ci, ci, ci, ci, ci, vp,
                                           vp]
    L.pcm_tune_emd_timeouts.restype = ci
    L.pcm_tune_emd_timeouts.argtypes = [vp, cs, ci, ci, vp]
    L.pcm_chamfer_loss_grad.restype = ci
    L.pcm_chamfer_loss_grad.argtypes = [vp, vp, ci, ci, ci, cf, cf, vp, vp, vp, vp, vp, vp, vp, vp, cs, vp]
    L.pcm_tune_chamfer_loss_grad.restype = ci
    L.pcm_tune_chamfer_loss_grad.argtypes = [ci, vp, vp, ci, ci, ci, cf, cf, vp, vp, vp, vp, vp, vp, vp, vp, cs,
                                             vp]
    L.pcm_tune_num_chamfer_loss_grad_variants.restype = ci
    L.pcm_tune_num_chamfer_loss_grad_variants.argtypes = []
    if hasattr(L, "pcm_chamfer_loss_grad_layout"):  # absent from A/B builds of older sources
        L.pcm_chamfer_loss_grad_layout.restype = ci
        L.pcm_chamfer_loss_grad_layout.argtypes = [vp, vp, ci, ci, ci, ci, ci, cf, cf, vp, vp, vp, vp, vp, vp, vp,
                                                   vp, vp, cs, vp]
        L.pcm_chamfer_loss_grad_rescale.restype = ci
        L.pcm_chamfer_loss_grad_rescale.argtypes = [vp, vp, ci, ci, ci, ci, ci, cf, cf, vp, vp, vp, vp, vp, vp, vp,
                                                    vp]
        L.pcm_chamfer_loss_grad_steps.restype = ci
        L.pcm_chamfer_loss_grad_steps.argtypes = [ci, vp, vp, ci, ci, ci, cf, cf, vp, vp, vp, vp, vp, vp, vp, vp,
                                                  cs, vp]
    if hasattr(L, "pcm_tune_occupy"):  # absent from A/B builds of older sources
        L.pcm_tune_occupy.restype = ci
        L.pcm_tune_occupy.argtypes = [ci, ci, ci, ctypes.c_uint, vp]
    if hasattr(L, "pcm_tune_occupy_stamped"):
        L.pcm_tune_occupy_stamped.restype = ci
        L.pcm_tune_occupy_stamped.argtypes = [ci, ci, ci, ctypes.c_uint, vp, vp]
        L.pcm_tune_clock_stamp.restype = ci
        L.pcm_tune_clock_stamp.argtypes = [vp, vp]
    if hasattr(L, "pcm_tune_clock_rate"):
        L.pcm_tune_clock_rate.restype = ci
        L.pcm_tune_clock_rate.argtypes = [vp, ci, vp]
    if hasattr(L, "pcm_tune_occupy_flagged"):
        L.pcm_tune_occupy_flagged.restype = ci
        L.pcm_tune_occupy_flagged.argtypes = [ci, ci, ci, ctypes.c_uint, vp, vp, vp]
    cd = ctypes.c_double
    L.pcm_icp.restype = ci
    L.pcm_icp.argtypes = [vp, vp, ci, ci, vp, ci, cd, vp, vp, vp, vp, cs, vp]
    L.pcm_icp_workspace_status.restype = ci
    L.pcm_icp_workspace_status.argtypes = [vp, cs, ci, ci, vp]
    L.pcm_icp_workspace_bytes.restype = cs
    L.pcm_icp_workspace_bytes.argtypes = [ci, ci]
    L.pcm_nearest_neighbor.restype = ci
    L.pcm_nearest_neighbor.argtypes = [vp, vp, ci, ci, ci, vp, vp, vp, cs, vp]
    L.pcm_best_fit_transform.restype = ci
    L.pcm_best_fit_transform.argtypes = [vp, vp, ci, ci, vp, vp]
    return L


def strerror(status: int) -> str:
    return load_library().pcm_strerror(int(status)).decode()


def _check(status: int, what: str) -> None:
    if status != 0:
        raise PcmError(f"{what} failed: {strerror(status)} (status {status})")


def _require_device(*tensors: torch.Tensor) -> torch.device:
    dev = tensors[0].device
    for t in tensors:
        if t.device.type != "cuda":
            raise RuntimeError(
                "pcm_hip kernels need HIP device tensors (got a tensor on "
                f"{t.device}); there is no CPU path")
        if t.device != dev:
            raise RuntimeError(f"tensors on different devices: {dev} vs {t.device}")
    return dev


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _cloud_kind(xyz1, xyz2) -> str:
    if xyz1.dtype != xyz2.dtype or xyz1.dtype not in (torch.float32, torch.float16):
        raise TypeError(f"Chamfer clouds must both be float32 or both float16 (got {xyz1.dtype}, {xyz2.dtype})")
    return "f16" if xyz1.dtype == torch.float16 else "f32"


# clouds at least this large (both) take the grid forward (csrc/chamfer_grid.hip
# kGridMinPoints), which needs pcm_chamfer_forward_ws_bytes of workspace
GRID_MIN_POINTS = 4096


def forward_workspace(dev: torch.device, b: int, n: int, m: int, force_grid: bool = False):
    """Scratch for the grid forward (no state between calls, no zero-fill):
    None when the problem takes the dense kernels (pcm_chamfer_forward_ws_bytes
    is 0), else ONE buffer per (device, current stream), grown when a larger
    problem needs more (it holds nothing between calls).  force_grid: the
    size the grid path needs at any problem size (tune_chamfer_forward_grid)."""
    L = load_library()
    need = int(L.pcm_tune_chamfer_forward_grid_ws_bytes(b, n, m) if force_grid
               else L.pcm_chamfer_forward_ws_bytes(b, n, m))
    if need == 0:
        return None
    key = ("forward", dev, _stream_id(dev))
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        _cache_put(key, ws)
    return _hand_out(ws)


def cloud_layout(t: torch.Tensor):
    """0 for a contiguous [B, N, 3] cloud (rows), 1 for a [B, N, 3] view of a
    contiguous [B, 3, N] tensor (channel planes: the generator output
    train.py:163 passes as fake.transpose(2, 1)), None for anything else."""
    if t.dim() != 3 or t.shape[2] != 3:
        return None
    b, n, _ = t.shape
    if t.is_contiguous():
        return 0
    st = t.stride()
    if (st[1] == 1 or n == 1) and st[2] == n and (st[0] == 3 * n or b == 1):
        return 1
    return None


def chamfer_forward_layout(xyz1, xyz2, lay1, lay2, dist1, dist2, idx1, idx2) -> None:
    """pcm_chamfer_forward_layout: float32 clouds each in rows (0) or channel
    planes (1, see cloud_layout); results identical to chamfer_forward on rows."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    if xyz1.dtype != torch.float32 or xyz2.dtype != torch.float32:
        raise TypeError("chamfer_forward_layout takes float32 clouds")
    with torch.cuda.device(dev):
        _check(load_library().pcm_chamfer_forward_layout(
            _ptr(xyz1), _ptr(xyz2), b, n, m, int(lay1), int(lay2), _ptr(dist1), _ptr(dist2), _ptr(idx1),
            _ptr(idx2), _stream(dev)), "pcm_chamfer_forward_layout")


def chamfer_backward_layout(xyz1, xyz2, lay1, lay2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2) -> None:
    """pcm_chamfer_backward_layout: gradxyz1/2 written in their cloud's layout."""
    dev = _require_device(xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    with torch.cuda.device(dev):
        _check(load_library().pcm_chamfer_backward_layout(
            _ptr(xyz1), _ptr(xyz2), b, n, m, int(lay1), int(lay2), _ptr(graddist1), _ptr(graddist2), _ptr(idx1),
            _ptr(idx2), _ptr(gradxyz1), _ptr(gradxyz2), _stream(dev)), "pcm_chamfer_backward_layout")


def chamfer_backward_strided(xyz1, xyz2, lay1, lay2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2) -> None:
    """pcm_chamfer_backward_strided: float32 [B, N] graddists read in place at
    their own strides (an expanded scalar included); gradients in their cloud's
    layout (lay 0 rows, 1 channel planes)."""
    dev = _require_device(xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    for g, k in ((graddist1, n), (graddist2, m)):
        if g.dtype != torch.float32 or tuple(g.shape) != (b, k):
            raise ValueError("chamfer_backward_strided takes float32 graddists of shape [B, N] and [B, M]")
    with torch.cuda.device(dev):
        _check(load_library().pcm_chamfer_backward_strided(
            _ptr(xyz1), _ptr(xyz2), b, n, m, int(lay1), int(lay2), _ptr(graddist1), graddist1.stride(0),
            graddist1.stride(1), _ptr(graddist2), graddist2.stride(0), graddist2.stride(1), _ptr(idx1), _ptr(idx2),
            _ptr(gradxyz1), _ptr(gradxyz2), _stream(dev)), "pcm_chamfer_backward_strided")


def chamfer_forward(xyz1, xyz2, dist1, dist2, idx1, idx2) -> None:
    """pcm_chamfer_forward (float32 clouds) or pcm_chamfer_forward_f16 (float16
    clouds) on contiguous [B,N,3]/[B,M,3] device tensors; dist is float32.
    Clouds of >= GRID_MIN_POINTS points go through pcm_chamfer_forward_ws[_f16]
    (the grid forward; same outputs bit for bit)."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    f16 = _cloud_kind(xyz1, xyz2) == "f16"
    L = load_library()
    with torch.cuda.device(dev):
        ws = forward_workspace(dev, b, n, m) if (n >= GRID_MIN_POINTS and m >= GRID_MIN_POINTS and b > 0) else None
        if ws is not None:  # the grid forward pays at this size (csrc/chamfer_grid.hip grid_pays)
            fn = "pcm_chamfer_forward_ws_f16" if f16 else "pcm_chamfer_forward_ws"
            _check(getattr(L, fn)(
                _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2), _ptr(idx1), _ptr(idx2),
                _ptr(ws), ws.numel(), _stream(dev)), fn)
            return
        fn = "pcm_chamfer_forward_f16" if f16 else "pcm_chamfer_forward"
        _check(getattr(L, fn)(
            _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2), _ptr(idx1), _ptr(idx2),
            _stream(dev)), fn)


def tune_chamfer_forward_grid(xyz1, xyz2, dist1, dist2, idx1, idx2, scan="filter", only=None,
                              stats=None, workspace=None, small_wg=False, reg_gather=False) -> None:
    """Internal: the grid forward at any size (float32 or float16 clouds).
    scan: "filter" (default: packed (u, w) screen + proof), "screened" (exact
    distances, chunk minima) or "exact" (every candidate's key); only =
    "build" / "search" runs one of its two kernels (search reuses the
    workspace of a previous call with the same clouds); stats: int32 device
    tensor, 12 ints per search wave (csrc/chamfer_grid.hip)."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    f16 = _cloud_kind(xyz1, xyz2) == "f16"
    mode = int(f16) | {"filter": 0, "screened": 64, "exact": 2}[scan] | {None: 0, "build": 4, "search": 8}[only]
    mode |= (16 if small_wg else 0) | (32 if reg_gather else 0)
    with torch.cuda.device(dev):
        ws = workspace if workspace is not None else forward_workspace(dev, b, n, m, force_grid=True)
        _check(load_library().pcm_tune_chamfer_forward_grid(
            mode, _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2), _ptr(idx1), _ptr(idx2),
            _ptr(ws), ws.numel(), _stream(dev), _ptr(stats)), "pcm_tune_chamfer_forward_grid")


def tune_chamfer_forward_f16(variant, xyz1, xyz2, dist1, dist2, idx1, idx2) -> None:
    """Internal: fp16 forward variant `variant` (-1 = default)."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_chamfer_forward_f16(
            int(variant), _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2), _ptr(idx1),
            _ptr(idx2), _stream(dev)), "pcm_tune_chamfer_forward_f16")


def tune_num_chamfer_f16_variants() -> int:
    return int(load_library().pcm_tune_num_chamfer_f16_variants())


# cached device workspaces: an LRU of at most _WS_CACHE_MAX buffers (the
# fused-loss workspaces are per shape; the grid forward's one per stream)
_ws_cache = collections.OrderedDict()
_WS_CACHE_MAX = 16
# every cached buffer handed out while a graph was being captured: the graph
# keeps its raw pointer, so the buffer must outlive any eviction or growth of
# the cache (else a replay would write into freed, possibly reused memory)
_graph_pinned = {}


def _cache_put(key, ws):
    _ws_cache[key] = ws
    _ws_cache.move_to_end(key)
    while len(_ws_cache) > _WS_CACHE_MAX:
        old_key, _ = _ws_cache.popitem(last=False)
        _watches.pop(old_key, None)


def _hand_out(ws):
    """A cached buffer about to be passed to a kernel: pinned for the life of
    the process if the current stream is capturing a graph."""
    if ws is not None and torch.cuda.is_current_stream_capturing():
        _graph_pinned.setdefault(ws.data_ptr(), ws)
    return ws


def _stream_id(dev: torch.device) -> int:
    return int(torch.cuda.current_stream(dev).cuda_stream)


def chamfer_workspace(dev: torch.device, b: int, n: int, m: int) -> torch.Tensor:
    """Zero-filled workspace for the fused-loss kernels, cached per (device,
    current stream, shape): the kernels keep cross-launch state in it (epoch,
    arrival counters, argmin granules), so only stream-ordered calls may share
    one; one per shape keeps every call's granules trusted (a workspace last
    used by another shape makes the next call recompute its argmins,
    csrc/chamfer_filt.hip kGradShapeWord)."""
    need = int(load_library().pcm_chamfer_workspace_bytes(b, n, m))
    if _tune_lib is not None:  # the tuning build's variants need more (all of them fit)
        need = max(need, int(_tune_lib.pcm_chamfer_workspace_bytes(b, n, m)))
    key = ("chamfer", dev, _stream_id(dev), b, n, m)
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.zeros(need, dtype=torch.uint8, device=dev)
        _cache_put(key, ws)
    else:
        _ws_cache.move_to_end(key)
    return _hand_out(ws)


_scale_hints = {}


def grad_scale_hint(dev: torch.device) -> torch.Tensor:
    """The upstream gradient the next one-launch Chamfer loss on (device,
    current stream) expects (a device float, 1.0 at first):
    chamfer_3DLossFunction's forward computes its gradient for this scale and
    its backward (pcm_chamfer_loss_grad_rescale) stores the real one here, so
    a training loop with a constant loss weight computes it right from its
    second step on.  Never freed (graphs keep its pointer)."""
    key = (dev, _stream_id(dev))
    t = _scale_hints.get(key)
    if t is None:
        last = _scale_hints.get(("last", dev))
        if last is not None and torch.cuda.is_current_stream_capturing():
            # a capture stream takes the device's last-used hint (the scale the
            # eager warm-up learned): a new tensor's fill would be captured and
            # reset the scale at every replay
            t = last
        else:
            t = torch.ones(1, dtype=torch.float32, device=dev)
        _scale_hints[key] = t
    _scale_hints[("last", dev)] = t
    return t


class _StickyWatch:
    """Lagged, sync-free check of a cached fused-loss workspace's sticky error
    words (a loss poll that timed out: NaN means from then on).  After every
    call the two words are copied asynchronously to pinned host memory behind
    an event, into a small ring of such copies; each call first reads the
    copies whose events have completed, oldest first, and, if a word is set,
    re-zeroes the workspace and raises PcmError, so a timeout is reported
    instead of silently persisting.  No copy is ever dropped: a host that
    runs ahead of the GPU fills the ring, and a full ring waits for its
    oldest copy, which bounds the calls between a timeout and its report.
    The words are copied after the first and then every `every`-th call (a copy is a
    kernel on the stream: two per call had cost ~9 us of GPU time per step
    of a ~17 us training call), so a timeout is reported within
    every * (depth + 1) calls; its NaN means are visible at once anyway."""

    depth = 4
    every = 32

    def __init__(self, ws, b, n, m):
        L = load_library()
        self.ws = ws
        self.offs = [int(L.pcm_tune_chamfer_err_offset(w, b, n, m)) for w in (0, 1)]
        self.bufs = [torch.zeros(2, dtype=torch.int32, pin_memory=True) for _ in range(self.depth)]
        self.ring = collections.deque()  # (buffer index, event), oldest first
        self.next = 0
        self.calls = 0

    def _read(self, k):
        if bool(self.bufs[k].any()):
            for kk, ev in self.ring:  # pending copies hold the same sticky words
                ev.synchronize()
            self.ring.clear()
            for buf in self.bufs:
                buf.zero_()
            self.ws.zero_()
            raise PcmError("a fused Chamfer loss kernel timed out waiting on its other workgroups "
                           "(NaN means); its workspace has been reset -- repeat the step")

    def check(self):
        while self.ring and self.ring[0][1].query():
            self._read(self.ring.popleft()[0])
        if len(self.ring) >= self.depth:
            k, ev = self.ring.popleft()
            ev.synchronize()
            self._read(k)

    def record(self):
        self.calls += 1
        if self.calls % self.every != 1 and self.every > 1:  # the first call, then every `every`-th
            return
        k = self.next
        self.next = (k + 1) % self.depth
        for i, o in enumerate(self.offs):
            self.bufs[k][i:i + 1].copy_(self.ws[o:o + 4].view(torch.int32), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.ring.append((k, ev))


_watches = {}


def _watched_workspace(dev, b, n, m):
    """The cached workspace plus its sticky-error watch (None under graph
    capture, where host reads and events are not part of the graph)."""
    ws = chamfer_workspace(dev, b, n, m)
    if torch.cuda.is_current_stream_capturing():
        return ws, None
    key = ("chamfer", dev, _stream_id(dev), b, n, m)
    w = _watches.get(key)
    if w is None or w.ws is not ws:
        w = _watches[key] = _StickyWatch(ws, b, n, m)
    w.check()
    return ws, w


def chamfer_forward_loss(xyz1, xyz2, dist1, dist2, idx1, idx2, mean_out, workspace=None) -> None:
    """pcm_chamfer_forward_loss: forward + mean_out[0:2] = (mean(dist1), mean(dist2))."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2, mean_out)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    watch = None
    with torch.cuda.device(dev):
        if workspace is None:
            workspace, watch = _watched_workspace(dev, b, n, m)
        _check(load_library().pcm_chamfer_forward_loss(
            _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2), _ptr(idx1), _ptr(idx2),
            _ptr(mean_out), _ptr(workspace), workspace.numel(), _stream(dev)),
            "pcm_chamfer_forward_loss")
        if watch is not None:
            watch.record()


def loss_grad_supported(xyz1, xyz2) -> bool:
    """Whether pcm_chamfer_loss_grad takes these clouds in one launch."""
    return (xyz1.dtype == torch.float32 and xyz2.dtype == torch.float32 and xyz1.shape[0] > 0
            and 0 < xyz1.shape[1] <= LOSS_GRAD_MAX_POINTS and 0 < xyz2.shape[1] <= LOSS_GRAD_MAX_POINTS)


def chamfer_loss_grad(xyz1, xyz2, w1, w2, dist1, dist2, idx1, idx2, mean_out, gradxyz1, gradxyz2,
                      workspace=None, variant=None, layouts=(0, 0), grad_scale=None) -> None:
    """pcm_chamfer_loss_grad: the forward (dist/idx), mean_out[0:3] = (mean(dist1),
    mean(dist2), their sum), and the gradients of w1*sum(dist1) + w2*sum(dist2)
    w.r.t. both clouds, in one launch (float32, n, m <= LOSS_GRAD_MAX_POINTS).
    layouts / grad_scale: pcm_chamfer_loss_grad_layout (clouds and gradients
    in channel planes where layout is 1; the gradients for the expected
    upstream scale in the device float grad_scale, recorded in mean_out[3]).
    variant: a fused variant of the tuning build (libpcm_hip_tune.so)."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2, mean_out, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    lay = (int(layouts[0]), int(layouts[1]))
    if mean_out.numel() < (3 if grad_scale is None else 4):
        raise ValueError("mean_out needs 3 floats (4 with grad_scale)")
    if variant is not None and (lay != (0, 0) or grad_scale is not None):
        raise ValueError("tuning variants take row clouds and no grad_scale")
    L = load_library() if variant is None else load_tune_library()
    watch = None
    with torch.cuda.device(dev):
        if workspace is None:
            workspace, watch = _watched_workspace(dev, b, n, m)
        tail = (_ptr(dist1), _ptr(dist2), _ptr(idx1), _ptr(idx2), _ptr(mean_out), _ptr(gradxyz1), _ptr(gradxyz2),
                _ptr(workspace), workspace.numel(), _stream(dev))
        if variant is not None:
            _check(L.pcm_tune_chamfer_loss_grad(int(variant), _ptr(xyz1), _ptr(xyz2), b, n, m, float(w1), float(w2),
                                                *tail), "pcm_tune_chamfer_loss_grad")
        elif lay == (0, 0) and grad_scale is None:
            _check(L.pcm_chamfer_loss_grad(_ptr(xyz1), _ptr(xyz2), b, n, m, float(w1), float(w2), *tail),
                   "pcm_chamfer_loss_grad")
        else:
            if grad_scale is not None and (grad_scale.dtype != torch.float32 or grad_scale.device != dev):
                raise ValueError("grad_scale must be a float32 tensor on the clouds' device")
            _check(L.pcm_chamfer_loss_grad_layout(_ptr(xyz1), _ptr(xyz2), b, n, m, lay[0], lay[1], float(w1),
                                                  float(w2), _ptr(grad_scale), *tail),
                   "pcm_chamfer_loss_grad_layout")
        if watch is not None:
            watch.record()


def chamfer_loss_grad_rescale(xyz1, xyz2, layouts, w1, w2, grad_loss, scale_used, scale_next, idx1, idx2,
                              gradxyz1, gradxyz2) -> None:
    """pcm_chamfer_loss_grad_rescale: the backward of a chamfer_loss_grad call
    made with grad_scale, now that the upstream gradient grad_loss (a device
    float) is known -- nothing when it equals scale_used bit for bit, else the
    exact gradients for it, in place; scale_next (nullable) receives it.
    scale_used None: always recompute."""
    dev = _require_device(xyz1, xyz2, grad_loss, idx1, idx2, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    with torch.cuda.device(dev):
        _check(load_library().pcm_chamfer_loss_grad_rescale(
            _ptr(xyz1), _ptr(xyz2), b, n, m, int(layouts[0]), int(layouts[1]), float(w1), float(w2),
            _ptr(grad_loss), _ptr(scale_used), _ptr(scale_next), _ptr(idx1), _ptr(idx2), _ptr(gradxyz1),
            _ptr(gradxyz2), _stream(dev)), "pcm_chamfer_loss_grad_rescale")


def chamfer_workspace_status(workspace, b: int, n: int, m: int) -> None:
    """Raise PcmError if a fused-loss kernel on `workspace` hit a device-side
    timeout (sticky until the workspace is zero-filled again; synchronises the
    current stream)."""
    dev = workspace.device
    with torch.cuda.device(dev):
        _check(load_library().pcm_chamfer_workspace_status(_ptr(workspace), workspace.numel(), b, n, m, _stream(dev)),
               "pcm_chamfer_workspace_status")


def tune_chamfer_loss_grad_spins(wait_spins, poll_spins, xyz1, xyz2, w1, w2, dist1, dist2, idx1, idx2, mean_out,
                                 gradxyz1, gradxyz2, workspace) -> None:
    """Internal: pcm_chamfer_loss_grad with the gradient-phase waits bounded by
    wait_spins polls (0: every argmin recomputed locally -- exact results) and
    the loss poll by poll_spins (0 forces its timeout: sticky error, NaN means)."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2, mean_out, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_chamfer_loss_grad_spins(
            int(wait_spins), int(poll_spins), _ptr(xyz1), _ptr(xyz2), b, n, m, float(w1), float(w2), _ptr(dist1),
            _ptr(dist2), _ptr(idx1), _ptr(idx2), _ptr(mean_out), _ptr(gradxyz1), _ptr(gradxyz2), _ptr(workspace),
            workspace.numel(), _stream(dev)), "pcm_tune_chamfer_loss_grad_spins")


def chamfer_slow_paths(workspace, b: int, n: int, m: int) -> int:
    """Internal: gradient-phase waits on `workspace` that timed out and computed
    the missing argmins locally (since the workspace was zero-filled)."""
    dev = workspace.device
    with torch.cuda.device(dev):
        r = int(load_library().pcm_tune_chamfer_slow_paths(_ptr(workspace), workspace.numel(), b, n, m,
                                                           _stream(dev)))
    if r < 0:
        _check(r, "pcm_tune_chamfer_slow_paths")
    return r


def tune_occupy(dev: torch.device, blocks: int, threads: int, lds_bytes: int, usec: int, stamps=None,
                host_flag=None) -> None:
    """Internal (tests): hold `blocks` workgroups of `threads` threads and
    `lds_bytes` of LDS resident for `usec` microseconds on the current stream,
    issuing only s_sleep -- another kernel sharing the CUs.  stamps: an int64
    device tensor of 3, initialised to (-1, 0, 0): the earliest workgroup
    start, the latest end (s_memrealtime ticks, 100 MHz) and the count of
    workgroups that started.  host_flag: a pinned host int32 tensor the last
    workgroup to start sets to 1 (the host sees residency without a copy)."""
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_occupy_flagged(int(blocks), int(threads), int(lds_bytes), int(usec),
                                                      _ptr(stamps), _ptr(host_flag), _stream(dev)),
               "pcm_tune_occupy_flagged")


def tune_clock_stamp(out) -> None:
    """Internal (tests): a one-thread kernel on the current stream writes the
    GPU real-time clock (s_memrealtime, 100 MHz ticks) to the int64 device
    scalar `out`, or to pinned host memory (a store the host can poll; the
    current device's kernel)."""
    dev = out.device if out.is_cuda else torch.device("cuda", torch.cuda.current_device())
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_clock_stamp(_ptr(out), _stream(dev)), "pcm_tune_clock_stamp")


def tune_clock_rate(out, iters: int = 20000) -> None:
    """Internal (tools/clock_state.py): one wave runs `iters` dependent FMAs on
    the current stream and writes (s_memrealtime ticks, s_memtime ticks) over
    them to out[0:2] (int64, device); the ratio x 0.1 is the shader clock in
    GHz while it ran."""
    with torch.cuda.device(out.device):
        _check(load_library().pcm_tune_clock_rate(_ptr(out), int(iters), _stream(out.device)), "pcm_tune_clock_rate")


def tune_num_chamfer_loss_grad_variants() -> int:
    """Fused variants of the tuning build (numbered 0 .. count - 1; the product
    library holds only the default, DEFAULT_LOSS_GRAD_VARIANT)."""
    return int(load_tune_library().pcm_tune_num_chamfer_loss_grad_variants())


# the product library's one-launch step (csrc/chamfer_filt.hip kDefaultGradVariant)
DEFAULT_LOSS_GRAD_VARIANT = 7


def mean_weight(count: int) -> float:
    """The per-element weight torch's mean backward multiplies the upstream
    gradient by: fl32(1 / count), as its device kernel forms it (a reciprocal
    then a multiply for a CPU-scalar divisor)."""
    import numpy as np
    return float(np.float32(1.0) / np.float32(count))


def tune_chamfer_forward(variant, xyz1, xyz2, dist1, dist2, idx1, idx2) -> None:
    """Internal: launch forward kernel variant `variant` (tools/tune_chamfer.py)."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_chamfer_forward(
            int(variant), _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2), _ptr(idx1),
            _ptr(idx2), _stream(dev)), "pcm_tune_chamfer_forward")


def tune_chamfer_backward_f16(variant, xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1,
                              gradxyz2) -> None:
    """Internal: fp16 backward `variant` (0 = automatic, 1 = 256-target workgroups, 3 = 1024-target)."""
    dev = _require_device(xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_chamfer_backward_f16(
            int(variant), _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(graddist1), _ptr(graddist2),
            _ptr(idx1), _ptr(idx2), _ptr(gradxyz1), _ptr(gradxyz2), _stream(dev)),
            "pcm_tune_chamfer_backward_f16")


def tune_chamfer_backward(variant, xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1,
                          gradxyz2) -> None:
    """Internal: backward path `variant` (0 = automatic: staged, 1 = global-memory kernel, 2 = per-batch LDS
    kernel, 3 = global-memory kernel with 1024-target workgroups)."""
    dev = _require_device(xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_chamfer_backward(
            int(variant), _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(graddist1), _ptr(graddist2),
            _ptr(idx1), _ptr(idx2), _ptr(gradxyz1), _ptr(gradxyz2), _stream(dev)),
            "pcm_tune_chamfer_backward")


def tune_chamfer_forward_loss(variant, loss_mode, xyz1, xyz2, dist1, dist2, idx1, idx2, mean_out,
                              workspace=None) -> None:
    """Internal: fused-loss forward with an explicit variant (-1 = default) and
    loss mode (1 = in-kernel ticket, 2 = partials + finalize kernel)."""
    dev = _require_device(xyz1, xyz2, dist1, dist2, idx1, idx2, mean_out)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    if workspace is None:
        workspace = chamfer_workspace(dev, b, n, m)
    with torch.cuda.device(dev):
        _check(load_library().pcm_tune_chamfer_forward_loss(
            int(variant), int(loss_mode), _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(dist1), _ptr(dist2),
            _ptr(idx1), _ptr(idx2), _ptr(mean_out), _ptr(workspace), workspace.numel(), _stream(dev)),
            "pcm_tune_chamfer_forward_loss")


def tune_num_chamfer_variants() -> int:
    return int(load_library().pcm_tune_num_chamfer_variants())


def chamfer_backward(xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2) -> None:
    """pcm_chamfer_backward (float32 clouds and gradients) or pcm_chamfer_backward_f16
    (float16 clouds and gradients); graddist is float32 in both."""
    dev = _require_device(xyz1, xyz2, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2)
    b, n, _ = xyz1.shape
    m = xyz2.shape[1]
    kind = _cloud_kind(xyz1, xyz2)
    if gradxyz1.dtype != xyz1.dtype or gradxyz2.dtype != xyz2.dtype:
        raise TypeError("gradients must have the clouds' dtype")
    fn = "pcm_chamfer_backward_f16" if kind == "f16" else "pcm_chamfer_backward"
    with torch.cuda.device(dev):
        _check(getattr(load_library(), fn)(
            _ptr(xyz1), _ptr(xyz2), b, n, m, _ptr(graddist1), _ptr(graddist2), _ptr(idx1),
            _ptr(idx2), _ptr(gradxyz1), _ptr(gradxyz2), _stream(dev)), fn)


def emd_workspace_bytes(b: int, n: int) -> int:
    return int(load_library().pcm_emd_workspace_bytes(b, n))


def emd_workspace(dev: torch.device, b: int, n: int) -> torch.Tensor:
    """EMD workspace cached per (device, current stream, size); its content on
    entry is irrelevant, but a call's auction state lives in it until the call
    ends, so concurrent calls on different streams get different buffers."""
    ws_bytes = max(emd_workspace_bytes(b, n), 1)
    key = ("emd", dev, _stream_id(dev))
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < ws_bytes:  # one per (device, stream), grown when needed
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        _cache_put(key, ws)
    return _hand_out(ws)


def emd_forward(xyz1, xyz2, eps: float, iters: int, dist, assignment, price=None,
                workspace=None, helpers=None, offload_min=None, stats=None, diag=1, wsplit=None,
                tail_max=None, spin_limit=None) -> None:
    """pcm_emd_forward; helpers / offload_min / stats select the tuning entry
    (helper workgroups per cloud, the miss count above which an iteration's
    full scans are offloaded, diagnostics of kind `diag`: 1 counts, 2 + i phase
    timers of batch element i; wsplit: waves per few-miss full scan; tail_max:
    bidders at or below which an iteration runs in tail mode, 0 = never;
    spin_limit: bound of the waits between workgroups, 0 forces the timeout
    path -- csrc/emd.hip pcm_tune_emd_forward_cfg) -- None = the defaults."""
    dev = _require_device(xyz1, xyz2, dist, assignment)
    b, n, _ = xyz1.shape
    ws_bytes = emd_workspace_bytes(b, n)
    if ws_bytes and (workspace is None or workspace.numel() * workspace.element_size() < ws_bytes):
        workspace = emd_workspace(dev, b, n)
    with torch.cuda.device(dev):
        if (helpers is None and offload_min is None and stats is None and wsplit is None and tail_max is None
                and spin_limit is None):
            _check(load_library().pcm_emd_forward(
                _ptr(xyz1), _ptr(xyz2), b, n, float(eps), int(iters), _ptr(dist), _ptr(assignment),
                _ptr(price), _ptr(workspace), ws_bytes, _stream(dev)), "pcm_emd_forward")
        else:
            if stats is not None and stats.numel() < 3 * int(iters) + 16 + b:
                raise ValueError("stats needs 3*iters + 16 + B int32 entries")
            _check(load_library().pcm_tune_emd_forward_cfg(
                _ptr(xyz1), _ptr(xyz2), b, n, float(eps), int(iters), _ptr(dist), _ptr(assignment),
                _ptr(price), _ptr(workspace), ws_bytes, -1 if helpers is None else int(helpers),
                -1 if offload_min is None else int(offload_min), int(diag), 0 if wsplit is None else int(wsplit),
                -1 if tail_max is None else int(tail_max), -1 if spin_limit is None else int(spin_limit),
                _ptr(stats), _stream(dev)),
                "pcm_tune_emd_forward_cfg")


def emd_workspace_status(workspace, b: int, n: int) -> None:
    """Raise PcmError if reading the last EMD forward's status fails
    (synchronises the current stream).  A helper job that timed out is not an
    error: the master scanned those items itself (emd_timeouts counts them)."""
    dev = workspace.device
    with torch.cuda.device(dev):
        _check(load_library().pcm_emd_workspace_status(_ptr(workspace), workspace.numel(), b, n, _stream(dev)),
               "pcm_emd_workspace_status")


def emd_timeouts(workspace, b: int, n: int) -> int:
    """Internal: batch elements of the last EMD forward on `workspace` whose
    master timed out on a helper job and scanned the items itself."""
    dev = workspace.device
    with torch.cuda.device(dev):
        r = int(load_library().pcm_tune_emd_timeouts(_ptr(workspace), workspace.numel(), b, n, _stream(dev)))
    if r < 0:
        _check(r, "pcm_tune_emd_timeouts")
    return r


def emd_backward(xyz1, xyz2, graddist, assignment, gradxyz1) -> None:
    dev = _require_device(xyz1, xyz2, graddist, assignment, gradxyz1)
    b, n, _ = xyz1.shape
    with torch.cuda.device(dev):
        _check(load_library().pcm_emd_backward(
            _ptr(xyz1), _ptr(xyz2), b, n, _ptr(graddist), _ptr(assignment), _ptr(gradxyz1),
            _stream(dev)), "pcm_emd_backward")


def _nn_workspace(dev, b: int, m: int):
    """Cached workspace for the screening rows (content on entry irrelevant)."""
    need = max(int(load_library().pcm_icp_workspace_bytes(b, m)), 1)
    key = ("nn", dev, _stream_id(dev))
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        _cache_put(key, ws)
    return _hand_out(ws)


def icp(A, B, init_pose, max_iterations: int, tolerance: float, T_out, distances, iterations,
        workspace=None) -> None:
    """pcm_icp on float64 device tensors A, B [b,n,3], init_pose None or [b,4,4];
    outputs T_out [b,4,4] float64, distances [b,n] float64, iterations [b] int32."""
    dev = _require_device(A, B, T_out, distances, iterations)
    b, n, _ = A.shape
    if workspace is None:
        workspace = _nn_workspace(dev, b, n)
    with torch.cuda.device(dev):
        _check(load_library().pcm_icp(
            _ptr(A), _ptr(B), b, n, _ptr(init_pose), int(max_iterations), float(tolerance), _ptr(T_out),
            _ptr(distances), _ptr(iterations), _ptr(workspace), workspace.numel(), _stream(dev)), "pcm_icp")


def icp_workspace_status(workspace, b: int, n: int) -> None:
    """Raise PcmError if the last pcm_icp on `workspace` hit a device-side
    timeout between the workgroups of a pair (synchronises the current stream)."""
    dev = workspace.device
    with torch.cuda.device(dev):
        _check(load_library().pcm_icp_workspace_status(_ptr(workspace), workspace.numel(), b, n, _stream(dev)),
               "pcm_icp_workspace_status")


def nearest_neighbor(src, dst, distances, indices, workspace=None) -> None:
    """pcm_nearest_neighbor on float64 device tensors src [b,n,3], dst [b,m,3]."""
    dev = _require_device(src, dst, distances, indices)
    b, n, _ = src.shape
    m = dst.shape[1]
    if workspace is None:
        workspace = _nn_workspace(dev, b, m)
    with torch.cuda.device(dev):
        _check(load_library().pcm_nearest_neighbor(
            _ptr(src), _ptr(dst), b, n, m, _ptr(distances), _ptr(indices), _ptr(workspace), workspace.numel(),
            _stream(dev)), "pcm_nearest_neighbor")


def best_fit_transform(A, B, T_out) -> None:
    """pcm_best_fit_transform on float64 device tensors A, B [b,n,3] -> T_out [b,4,4]."""
    dev = _require_device(A, B, T_out)
    b, n, _ = A.shape
    with torch.cuda.device(dev):
        _check(load_library().pcm_best_fit_transform(_ptr(A), _ptr(B), b, n, _ptr(T_out), _stream(dev)),
               "pcm_best_fit_transform")
