"""GPU parity of the grid forward (csrc/chamfer_grid.hip) against the CPU oracle.

The grid path must return exactly what the dense forward returns (and the
oracle, oracle/pcm_oracle.c chamfer_forward), bit for bit: it only narrows
the candidates each query evaluates and proves that nothing outside can win.
These tests force the grid path at every size (pcm_tune_chamfer_forward_grid)
and cover the cases where the proof fails (separated clouds, outliers) and
the degenerate grids (one point, coincident points, huge and tiny extents).
"""
import numpy as np
import pytest
import torch

from test_chamfer_gpu import _assert_fwd_equal, _clouds, _stress_clouds

pytestmark = pytest.mark.gpu


def _grid_fwd(a, c, dev, scan="filter"):
    import pcm_hip
    b, n, m = a.shape[0], a.shape[1], c.shape[1]
    d1 = torch.full((b, n), -1.0, device=dev)
    d2 = torch.full((b, m), -1.0, device=dev)
    i1 = torch.full((b, n), -1, dtype=torch.int32, device=dev)
    i2 = torch.full((b, m), -1, dtype=torch.int32, device=dev)
    pcm_hip.tune_chamfer_forward_grid(a.to(dev), c.to(dev), d1, d2, i1, i2, scan=scan)
    torch.cuda.synchronize()
    return d1.cpu().numpy(), d2.cpu().numpy(), i1.cpu().numpy(), i2.cpu().numpy()


def _ref(oracle, a, c):
    return oracle.chamfer_forward(a.float().numpy(), c.float().numpy())


@pytest.mark.parametrize("b,n,m,seed,dist", [
    (3, 1, 1, 0, "uniform"),
    (2, 5, 3, 1, "normal"),
    (2, 33, 31, 2, "normal"),
    (4, 256, 256, 3, "uniform"),
    (3, 700, 1900, 4, "uniform"),
    (2, 5000, 300, 5, "normal"),
    (2, 4096, 4096, 6, "uniform"),
    (1, 16384, 16384, 7, "uniform"),
])
def test_grid_forward_matches_oracle(cuda, oracle, b, n, m, seed, dist):
    a, c = _clouds(seed, b, n, m, dist)
    _assert_fwd_equal(_grid_fwd(a, c, cuda), _ref(oracle, a, c))


@pytest.mark.parametrize("kind", ["grid", "near_ties", "offset", "tiny", "huge", "dup_queries"])
@pytest.mark.parametrize("scan", ["screened", "exact", "filter"])
def test_grid_forward_stress(cuda, oracle, kind, scan):
    # "grid" puts every coordinate on a 1/8 lattice: exact distance ties
    # across chunks (the screened scan's exact-rescan path, the filter's
    # near-tie path); "offset" / "huge" stretch the filter's error bound
    a, c = _stress_clouds(kind, b=2, n=3000, m=2500)
    _assert_fwd_equal(_grid_fwd(a, c, cuda, scan), _ref(oracle, a, c))


@pytest.mark.parametrize("b,n,m,seed,dist,f16", [
    (2, 33, 31, 2, "normal", False),
    (3, 700, 1900, 4, "uniform", False),
    (1, 16384, 16384, 7, "uniform", False),
    (2, 8192, 8192, 31, "uniform", True),
])
def test_grid_forward_screened_scan(cuda, oracle, b, n, m, seed, dist, f16):
    # the non-default screened exact-distance scan (the filtered scan is the
    # default and runs in every other test)
    a, c = _clouds(seed, b, n, m, dist)
    if f16:
        a, c = a.half(), c.half()
    _assert_fwd_equal(_grid_fwd(a, c, cuda, "screened"), _ref(oracle, a, c))


@pytest.mark.parametrize("kind", ["separated", "outliers", "unsampled_outliers", "clustered", "collapsed", "one_target",
                                  "plane"])
def test_grid_forward_unproven_and_degenerate(cuda, oracle, kind):
    g = torch.Generator().manual_seed(21)
    a = torch.rand(2, 3000, 3, generator=g)
    c = torch.rand(2, 2000, 3, generator=g)
    if kind == "separated":      # no query's region holds its nearest target: every proof fails
        c = c + torch.tensor([10.0, 0.0, 0.0])
    elif kind == "outliers":     # a few far points stretch the grid: most cells empty
        a[:, :5] *= 1000.0
        c[:, :3] *= -1000.0
    elif kind == "unsampled_outliers":  # far points the grid's box sample skips: clamped into boundary cells
        a[:, 1] = torch.tensor([50.0, -40.0, 30.0])
        a[:, 3] = torch.tensor([-60.0, 20.0, 90.0])
        c[:, 1] = torch.tensor([-70.0, 80.0, -10.0])
    elif kind == "clustered":    # all points in a few tight blobs
        a = torch.floor(a * 3) / 3 + a * 1e-3
        c = torch.floor(c * 3) / 3 + c * 1e-3
    elif kind == "collapsed":    # one coincident cloud: zero extent
        a = torch.full_like(a, 0.25)
    elif kind == "one_target":
        c = c[:, :1]
    else:                        # all points on the plane z = 0.5
        a[..., 2] = 0.5
        c[..., 2] = 0.5
    _assert_fwd_equal(_grid_fwd(a, c, cuda), _ref(oracle, a, c))


@pytest.mark.parametrize("kind", ["nan_first", "nan_tile_start", "inf", "nan_query"])
def test_grid_forward_nonfinite(cuda, oracle, kind):
    a, c = _clouds(14, 2, 700, 1300)
    if kind == "nan_first":
        c[0, 0, 1] = float("nan")
    elif kind == "nan_tile_start":
        c[1, 512, 0] = float("nan")
    elif kind == "inf":
        c[0, 5, 0] = float("inf")
        a[1, 3, 1] = float("-inf")
    else:
        a[1, 100, 0] = float("nan")
    got = _grid_fwd(a, c, cuda)
    ref = _ref(oracle, a, c)
    for g_, r in zip(got[2:], ref[2:]):
        np.testing.assert_array_equal(g_, r)
    for g_, r in zip(got[:2], ref[:2]):
        np.testing.assert_array_equal(np.isnan(g_), np.isnan(r))
        fin = ~np.isnan(r)
        np.testing.assert_array_equal(g_[fin].view(np.int32), r[fin].view(np.int32))


@pytest.mark.parametrize("b,n,m,seed", [(2, 300, 5000, 30), (2, 8192, 8192, 31)])
def test_grid_forward_f16(cuda, oracle, b, n, m, seed):
    a, c = _clouds(seed, b, n, m)
    ah, ch = a.half(), c.half()  # fp16 rounding makes many exact ties
    _assert_fwd_equal(_grid_fwd(ah, ch, cuda), _ref(oracle, ah, ch))


def test_grid_forward_empty_sides_untouched(cuda):
    import pcm_hip
    d1 = torch.full((2, 0), -1.0, device=cuda)
    d2 = torch.full((2, 7), -1.0, device=cuda)
    i1 = torch.full((2, 0), -1, dtype=torch.int32, device=cuda)
    i2 = torch.full((2, 7), -1, dtype=torch.int32, device=cuda)
    pcm_hip.tune_chamfer_forward_grid(torch.rand(2, 0, 3, device=cuda), torch.rand(2, 7, 3, device=cuda),
                                      d1, d2, i1, i2)
    torch.cuda.synchronize()
    assert (d2.cpu() == -1).all() and (i2.cpu() == -1).all()


def test_public_entry_routes_large_clouds_to_grid(cuda, oracle):
    # pcm_chamfer_forward_ws at >= 4096 points and b n m >= 2^28 is the grid
    # path (here 11 * 4100 * 6000); equal to the dense entry
    import pcm_hip
    a, c = _clouds(40, 11, 4100, 6000)
    x1, x2 = a.to(cuda), c.to(cuda)
    outs = []
    for fn in ("chamfer_forward", "dense"):
        d1 = torch.empty(11, 4100, device=cuda)
        d2 = torch.empty(11, 6000, device=cuda)
        i1 = torch.empty(11, 4100, dtype=torch.int32, device=cuda)
        i2 = torch.empty(11, 6000, dtype=torch.int32, device=cuda)
        if fn == "dense":
            P = pcm_hip._ptr
            assert pcm_hip.load_library().pcm_chamfer_forward(
                P(x1), P(x2), 11, 4100, 6000, P(d1), P(d2), P(i1), P(i2), pcm_hip._stream(cuda)) == 0
        else:
            pcm_hip.chamfer_forward(x1, x2, d1, d2, i1, i2)
        torch.cuda.synchronize()
        outs.append((d1.cpu().numpy(), d2.cpu().numpy(), i1.cpu().numpy(), i2.cpu().numpy()))
    ref = _ref(oracle, a, c)
    _assert_fwd_equal(outs[0], ref)
    _assert_fwd_equal(outs[1], ref)
