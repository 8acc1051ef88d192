"""Oracle self-consistency on the reference's semantics (CPU only).

These pin the edge-case behaviour the HIP kernels are later compared against:
512-point tile NaN rules (chamfer3D.cu:36/:79/:121/:126), lowest-index ties,
untouched outputs for empty targets, EMD's "Verified EMD" invariant
(metric/emd/test.py:24-28) and its determinism.
"""
import numpy as np
import pytest


def _rand(seed, *shape):
    return np.random.default_rng(seed).random(shape, dtype=np.float32)


def test_chamfer_direction_swap(oracle):
    a, q = _rand(0, 3, 100, 3), _rand(1, 3, 150, 3)
    d1, d2, i1, i2 = oracle.chamfer_forward(a, q)
    e1, e2, j1, j2 = oracle.chamfer_forward(q, a)
    assert np.array_equal(d1, e2) and np.array_equal(i1, j2)
    assert np.array_equal(d2, e1) and np.array_equal(i2, j1)


def test_chamfer_dist_is_min_over_targets(oracle):
    a, q = _rand(2, 2, 64, 3), _rand(3, 2, 80, 3)
    d, i = oracle.chamfer_nn(a, q)
    full = ((q[:, None, :, :] - a[:, :, None, :]) ** 2).sum(-1)
    assert np.allclose(d, full.min(-1), rtol=1e-6, atol=1e-9)
    assert (np.take_along_axis(full, i[..., None].astype(np.int64), -1)[..., 0] <= full.min(-1) + 1e-6).all()


def test_chamfer_ties_lowest_index(oracle):
    q = _rand(4, 1, 10, 3)
    q = np.concatenate([q, q], axis=1)  # duplicates at k and k+10
    d, i = oracle.chamfer_nn(q[:, :10].copy(), q)
    assert np.array_equal(i[0], np.arange(10))
    assert (d == 0).all()


def test_chamfer_nan_tile_rules(oracle):
    a = _rand(5, 1, 4, 3)
    q = _rand(6, 1, 1100, 3)
    # NaN at the very first target: tile 0 result is (NaN, 0) and sticks
    q0 = q.copy(); q0[0, 0, 0] = np.nan
    d, i = oracle.chamfer_nn(a, q0)
    assert np.isnan(d).all() and (i == 0).all()
    # NaN at a later tile's first point: that whole 512-tile is ignored
    a1 = q[:, 600:604].copy()          # exact matches inside tile 1 (512..1023)
    q1 = q.copy(); q1[0, 512, 1] = np.nan
    d, i = oracle.chamfer_nn(a1, q1)
    assert not np.isnan(d).any()
    assert ((i < 512) | (i >= 1024)).all()  # tile 1 skipped despite exact matches
    # NaN elsewhere: just skipped
    q2 = q.copy(); q2[0, 700, 2] = np.nan
    d, i = oracle.chamfer_nn(a1, q2)
    assert np.array_equal(i[0], np.arange(600, 604)) and (d == 0).all()


def test_chamfer_empty_targets_untouched(oracle):
    a = _rand(7, 2, 5, 3)
    q = np.zeros((2, 0, 3), np.float32)
    d, i = oracle.chamfer_nn(a, q)
    assert (d == 0).all() and (i == 0).all()  # buffers as allocated (zeros)


@pytest.mark.parametrize("eps,iters", [(0.005, 50), (0.05, 200), (0.005, 1)])
def test_emd_invariants(oracle, eps, iters):
    a, q = _rand(8, 2, 1024, 3), _rand(9, 2, 1024, 3)
    d, ass, price, hist = oracle.emd_forward(a, q, eps, iters, with_stats=True)
    assert ((ass >= 0) & (ass < 1024)).all()
    g = np.take_along_axis(q, ass[..., None].astype(np.int64), axis=1)
    np.testing.assert_allclose(d, ((a - g) ** 2).sum(-1), rtol=1e-6, atol=1e-8)
    assert hist[0] == 2 * 1024 and (np.diff(hist) <= 1024).all()
    assert (price >= 0).all()
    d2, ass2 = oracle.emd_forward(a, q, eps, iters)
    assert np.array_equal(ass, ass2) and np.array_equal(d, d2)  # deterministic


def test_emd_more_iterations_approach_bijection(oracle):
    a, q = _rand(10, 1, 1024, 3), _rand(11, 1, 1024, 3)
    _, a50 = oracle.emd_forward(a, q, 0.005, 50)
    _, a500 = oracle.emd_forward(a, q, 0.005, 500)
    assert len(np.unique(a500)) >= len(np.unique(a50))
    assert len(np.unique(a500)) > 1000


def test_emd_backward_formula(oracle):
    a, q = _rand(12, 2, 1024, 3), _rand(13, 2, 1024, 3)
    _, ass = oracle.emd_forward(a, q, 0.005, 20)
    gd = _rand(14, 2, 1024)
    g = oracle.emd_backward(a, q, gd, ass)
    ref = 2 * gd[..., None] * (a - np.take_along_axis(q, ass[..., None].astype(np.int64), axis=1))
    np.testing.assert_allclose(g, ref, rtol=1e-6, atol=1e-9)


def _reference_bid(v, nu):
    """emd_cuda.cu:103-176 for ONE bidder, literally: tpu threads, each scans
    its [l, r) range of every 2048-object tile with the strict '>' top-2
    update (:136-155), then thread 0 merges the others in thread order
    (:165-173).  v: the bidder's values (the oracle's, emd_cuda.cu:146)."""
    n = v.shape[0]
    block_cnt = n // 1024
    upb = (nu + block_cnt - 1) // block_cnt
    tpu = 1024 // upb
    best = [np.float32(-1e9)] * tpu
    better = [np.float32(-1e9)] * tpu
    best_i = [-1] * tpu
    for k2 in range(0, n, 2048):
        end_k = min(n, k2 + 2048) - k2
        delta = (end_k + tpu - 1) // tpu
        for t in range(tpu):
            for k in range(t * delta, min((t + 1) * delta, end_k)):
                d = v[k + k2]
                if d > best[t]:
                    better[t], best[t], best_i[t] = best[t], d, k + k2
                elif d > better[t]:
                    better[t] = d
    b, bb, bi = best[0], better[0], best_i[0]
    for t in range(1, tpu):
        if best[t] > b:
            bb = max(b, better[t])
            b, bi = best[t], best_i[t]
        else:
            bb = max(bb, best[t])
    return bi, b, bb


@pytest.mark.parametrize("n,nu", [(4096, 1), (4096, 5), (4096, 700), (4096, 2049), (4096, 4096), (3072, 3),
                                  (3072, 900), (8192, 17), (2048, 1), (1024, 1)])
def test_emd_bid_tie_order_matches_reference_threads(oracle, n, nu):
    # duplicated targets give exact value ties between objects in different
    # tiles and thread ranges: the oracle's winner must be the reference's
    # (lowest (thread, tile, k)), and the values its top two
    rng = np.random.default_rng(n + nu)
    q = rng.random((n, 3), dtype=np.float32)
    src = rng.permutation(n)[:64]
    q[rng.permutation(n)[:64]] = q[src]          # twins at random offsets
    q[rng.permutation(n)[:n // 8]] = q[7]        # and a crowd of copies of object 7
    price = np.zeros(n, np.float32)
    price[rng.permutation(n)[:n // 4]] = np.float32(0.01)
    for trial in range(24):
        p = (q[7] if trial % 4 == 3 else q[src[trial]]) if trial % 2 else rng.random(3, dtype=np.float32)
        v = oracle.emd_values(p, q, price)
        ref = _reference_bid(v, nu)
        got = oracle.emd_bid(p, q, price, nu)
        assert got[0] == ref[0], (trial, got, ref)
        assert got[1] == ref[1] and got[2] == ref[2]
